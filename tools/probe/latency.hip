// Host round-trip floor of a synchronous call on one MI355X: the primitives a host-form matcher
// call is made of (pinned H2D copy, a kernel launch, a D2H copy, stream synchronisation), each
// alone and chained, in microseconds per call (median of 2000).  Build: see tools/probe/README.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <vector>

__global__ void touch(int* p) {
    if (threadIdx.x == 0) p[blockIdx.x] += 1;
}
__global__ void touch_host(int* p, int* h) {
    if (threadIdx.x == 0) {
        p[0] += 1;
        h[0] = p[0];
    }
}

template <class F>
double med_us(F&& f, int n = 2000) {
    std::vector<double> t(n);
    for (int i = 0; i < 50; ++i) f();
    for (int i = 0; i < n; ++i) {
        auto t0 = std::chrono::steady_clock::now();
        f();
        t[i] = std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count();
    }
    std::sort(t.begin(), t.end());
    return t[n / 2];
}

int main() {
    hipStream_t s;
    hipStreamCreateWithFlags(&s, hipStreamNonBlocking);
    const size_t B = 80 << 10;
    void *h, *d, *hh;
    hipHostMalloc(&h, B, hipHostMallocDefault);
    hipHostMalloc(&hh, 4096, hipHostMallocDefault);
    hipMalloc(&d, B);
    int* di = static_cast<int*>(d);
    printf("{\"sync_only\": %.1f", med_us([&] { hipStreamSynchronize(s); }));
    printf(", \"launch_sync\": %.1f", med_us([&] {
               touch<<<1, 64, 0, s>>>(di);
               hipStreamSynchronize(s);
           }));
    printf(", \"launch2_sync\": %.1f", med_us([&] {
               touch<<<1, 64, 0, s>>>(di);
               touch<<<1, 64, 0, s>>>(di);
               hipStreamSynchronize(s);
           }));
    printf(", \"h2d80k_sync\": %.1f", med_us([&] {
               hipMemcpyAsync(d, h, B, hipMemcpyHostToDevice, s);
               hipStreamSynchronize(s);
           }));
    printf(", \"d2h4k_sync\": %.1f", med_us([&] {
               hipMemcpyAsync(h, d, 4096, hipMemcpyDeviceToHost, s);
               hipStreamSynchronize(s);
           }));
    printf(", \"h2d_launch_d2h_sync\": %.1f", med_us([&] {
               hipMemcpyAsync(d, h, B, hipMemcpyHostToDevice, s);
               touch<<<1, 64, 0, s>>>(di);
               hipMemcpyAsync(h, d, 4096, hipMemcpyDeviceToHost, s);
               hipStreamSynchronize(s);
           }));
    printf(", \"h2d_launch_hostwrite_sync\": %.1f", med_us([&] {
               hipMemcpyAsync(d, h, B, hipMemcpyHostToDevice, s);
               touch_host<<<1, 64, 0, s>>>(di, static_cast<int*>(hh));
               hipStreamSynchronize(s);
           }));
    printf(", \"launch_hostwrite_sync\": %.1f", med_us([&] {
               touch_host<<<1, 64, 0, s>>>(di, static_cast<int*>(hh));
               hipStreamSynchronize(s);
           }));
    printf("}\n");
    return 0;
}
