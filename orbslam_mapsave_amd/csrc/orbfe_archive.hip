// orbfe_archive.hip — the on-disk record formats of the extractor's outputs in the reference's
// map archive (MapPoint.h:196-247, used by KeyFrame::serialize / MapPoint::serialize through
// Boost binary archives, KeyFrame.cc:133-134, 354-355, MapPoint.cc:121, 194), written from and
// read into HBM-resident extractor / map-point buffers without a host round trip.
//
//   keypoint record (MapPoint.h:196-209): angle f32, class_id i32, octave i32, response f32,
//       response f32 (written twice), pt.x f32, pt.y f32 — 28 bytes; `size` is not stored, so a
//       loaded cv::KeyPoint keeps its default-constructed size 0
//   cv::Mat record (MapPoint.h:215-247): cols i32, rows i32, elemSize u64, type u64, then
//       rows*cols*elemSize raw bytes (a binary archive writes primitives and primitive arrays
//       as their native little-endian bytes)
//
// Descriptors are CV_8UC1 Mats of 32 columns (type 0, elemSize 1): a keyframe's mDescriptors
// (N x 32) or a map point's mDescriptor (1 x 32).  Boost's own framing around these bodies
// (class-info preamble of the first cv::Mat, the collection count of std::vector<KeyPoint>)
// belongs to the archive writer and is not produced here.
//
// Both directions are byte streaming (HBM-bound): one thread per keypoint record, one thread
// per 8 descriptor bytes.
#include <hip/hip_runtime.h>

#include "../../include/orbfe.h"

namespace orbfe {

constexpr int kArcBlock = 256;
constexpr int kMatHeader = 24;  // cols, rows (i32), elemSize, type (u64)

struct KpRecord {  // MapPoint.h:199-205, in archive order
    float angle;
    int32_t class_id, octave;
    float response0, response1, x, y;
};
static_assert(sizeof(KpRecord) == 28, "keypoint record is 28 bytes");

__device__ __forceinline__ int rows_of(const int32_t* d_n, int rows_fixed, int f) {
    return d_n ? d_n[f] : rows_fixed;
}

// grid (ceil(cap / 256), frames)
__global__ __launch_bounds__(kArcBlock) void archive_write_keys_kernel(
    const orbfe_keypoint* keys, size_t keys_pitch, const int32_t* n, int cap, uint8_t* out,
    size_t out_pitch) {
    const int f = blockIdx.y, i = blockIdx.x * kArcBlock + threadIdx.x;
    if (i >= min(n[f], cap)) return;
    const orbfe_keypoint k = keys[(size_t)f * keys_pitch + i];
    KpRecord r{k.angle, k.class_id, k.octave, k.response, k.response, k.x, k.y};
    uint32_t w[7];
    __builtin_memcpy(w, &r, 28);
    uint32_t* o = reinterpret_cast<uint32_t*>(out + (size_t)f * out_pitch + (size_t)i * 28);
#pragma unroll
    for (int j = 0; j < 7; ++j) o[j] = w[j];
}

__global__ __launch_bounds__(kArcBlock) void archive_read_keys_kernel(
    const uint8_t* in, size_t in_pitch, const int32_t* n, int cap, orbfe_keypoint* keys,
    size_t keys_pitch) {
    const int f = blockIdx.y, i = blockIdx.x * kArcBlock + threadIdx.x;
    if (i >= min(n[f], cap)) return;
    const uint32_t* src = reinterpret_cast<const uint32_t*>(in + (size_t)f * in_pitch + (size_t)i * 28);
    uint32_t w[7];
#pragma unroll
    for (int j = 0; j < 7; ++j) w[j] = src[j];
    KpRecord r;
    __builtin_memcpy(&r, w, 28);
    // the second response read overwrites the first; size keeps cv::KeyPoint()'s 0
    keys[(size_t)f * keys_pitch + i] = orbfe_keypoint{r.x, r.y, 0.0f, r.angle, r.response1,
                                                      r.octave, r.class_id};
}

// Mat records of rows x 32 CV_8UC1 descriptors.  Thread t of a frame writes bytes
// [8 t, 8 t + 8) of the record (header = the first 3 threads).  grid (ceil(chunks/256), frames)
__global__ __launch_bounds__(kArcBlock) void archive_write_desc_kernel(
    const uint8_t* desc, size_t desc_pitch, const int32_t* n, int rows_fixed, int cap,
    uint8_t* out, size_t out_pitch, int64_t* len) {
    const int f = blockIdx.y, t = blockIdx.x * kArcBlock + threadIdx.x;
    const int rows = min(rows_of(n, rows_fixed, f), cap);
    const int chunks = kMatHeader / 8 + rows * 4;
    if (t >= chunks) return;
    uint2* o = reinterpret_cast<uint2*>(out + (size_t)f * out_pitch);
    if (t == 0) {
        o[0] = make_uint2(32u, (uint32_t)rows);  // cols, rows
        o[1] = make_uint2(1u, 0u);                // elemSize
        o[2] = make_uint2(0u, 0u);                // type CV_8UC1
        if (len) len[f] = kMatHeader + 32ll * rows;
    } else if (t >= kMatHeader / 8) {
        const int b = t - kMatHeader / 8;
        o[t] = reinterpret_cast<const uint2*>(desc + (size_t)f * desc_pitch)[b];
    }
}

// Reads rows x 32 CV_8UC1 records; a header that is not (32, rows <= cap, 1, 0) sets *status
// and leaves that frame's descriptors untouched (rows_out = -1).
__global__ __launch_bounds__(kArcBlock) void archive_read_desc_kernel(
    const uint8_t* in, size_t in_pitch, int cap, uint8_t* desc, size_t desc_pitch,
    int32_t* rows_out, int32_t* status) {
    const int f = blockIdx.y, t = blockIdx.x * kArcBlock + threadIdx.x;
    const uint2* src = reinterpret_cast<const uint2*>(in + (size_t)f * in_pitch);
    const uint2 h0 = src[0], h1 = src[1], h2 = src[2];
    const int cols = (int)h0.x, rows = (int)h0.y;
    const bool ok = cols == 32 && rows >= 0 && rows <= cap && h1.x == 1u && h1.y == 0u &&
                    h2.x == 0u && h2.y == 0u;
    if (!ok) {
        if (t == 0) {
            if (rows_out) rows_out[f] = -1;
            atomicExch(status, ORBFE_ERR_ARG);
        }
        return;
    }
    if (t == 0 && rows_out) rows_out[f] = rows;
    if (t < rows * 4)
        reinterpret_cast<uint2*>(desc + (size_t)f * desc_pitch)[t] = src[kMatHeader / 8 + t];
}

}  // namespace orbfe

using namespace orbfe;

extern "C" {

int64_t orbfe_archive_mat_bytes(int rows, int cols, int elem_size) {
    if (rows < 0 || cols < 0 || elem_size < 0) return -1;
    return kMatHeader + (int64_t)rows * cols * elem_size;
}

int orbfe_archive_write_keypoints_device(int n_frames, const orbfe_keypoint* d_keys,
                                         size_t keys_pitch, const int32_t* d_n, int cap,
                                         uint8_t* d_out, size_t out_pitch, void* hip_stream) {
    if (n_frames < 0 || n_frames > 65535 || cap < 0 || (n_frames && (!d_keys || !d_n || !d_out)) ||
        keys_pitch < (size_t)cap || out_pitch < (size_t)cap * 28 || (out_pitch & 3))
        return ORBFE_ERR_ARG;
    if (!n_frames || !cap) return ORBFE_OK;
    hipLaunchKernelGGL(archive_write_keys_kernel, dim3((cap + kArcBlock - 1) / kArcBlock, n_frames),
                       dim3(kArcBlock), 0, static_cast<hipStream_t>(hip_stream), d_keys,
                       keys_pitch, d_n, cap, d_out, out_pitch);
    return hipGetLastError() == hipSuccess ? ORBFE_OK : ORBFE_ERR_HIP;
}

int orbfe_archive_read_keypoints_device(int n_frames, const uint8_t* d_in, size_t in_pitch,
                                        const int32_t* d_n, int cap, orbfe_keypoint* d_keys,
                                        size_t keys_pitch, void* hip_stream) {
    if (n_frames < 0 || n_frames > 65535 || cap < 0 || (n_frames && (!d_keys || !d_n || !d_in)) ||
        keys_pitch < (size_t)cap || in_pitch < (size_t)cap * 28 || (in_pitch & 3))
        return ORBFE_ERR_ARG;
    if (!n_frames || !cap) return ORBFE_OK;
    hipLaunchKernelGGL(archive_read_keys_kernel, dim3((cap + kArcBlock - 1) / kArcBlock, n_frames),
                       dim3(kArcBlock), 0, static_cast<hipStream_t>(hip_stream), d_in, in_pitch,
                       d_n, cap, d_keys, keys_pitch);
    return hipGetLastError() == hipSuccess ? ORBFE_OK : ORBFE_ERR_HIP;
}

int orbfe_archive_write_descriptors_device(int n_mats, const uint8_t* d_desc, size_t desc_pitch,
                                           const int32_t* d_rows, int rows_fixed, int cap,
                                           uint8_t* d_out, size_t out_pitch, int64_t* d_len,
                                           void* hip_stream) {
    if (n_mats < 0 || n_mats > 65535 || cap < 0 || (n_mats && (!d_desc || !d_out)) ||
        (!d_rows && (rows_fixed < 0 || rows_fixed > cap)) || desc_pitch < (size_t)cap * 32 ||
        (desc_pitch & 7) || out_pitch < (size_t)orbfe_archive_mat_bytes(cap, 32, 1) ||
        (out_pitch & 7))
        return ORBFE_ERR_ARG;
    if (!n_mats) return ORBFE_OK;
    const int chunks = kMatHeader / 8 + cap * 4;
    hipLaunchKernelGGL(archive_write_desc_kernel, dim3((chunks + kArcBlock - 1) / kArcBlock, n_mats),
                       dim3(kArcBlock), 0, static_cast<hipStream_t>(hip_stream), d_desc,
                       desc_pitch, d_rows, rows_fixed, cap, d_out, out_pitch, d_len);
    return hipGetLastError() == hipSuccess ? ORBFE_OK : ORBFE_ERR_HIP;
}

int orbfe_archive_read_descriptors_device(int n_mats, const uint8_t* d_in, size_t in_pitch,
                                          int cap, uint8_t* d_desc, size_t desc_pitch,
                                          int32_t* d_rows, int32_t* d_status, void* hip_stream) {
    if (n_mats < 0 || n_mats > 65535 || cap < 0 || !d_status || (n_mats && (!d_in || !d_desc)) ||
        desc_pitch < (size_t)cap * 32 || (desc_pitch & 7) || in_pitch < (size_t)kMatHeader ||
        (in_pitch & 7))
        return ORBFE_ERR_ARG;
    const hipStream_t s = static_cast<hipStream_t>(hip_stream);
    if (hipMemsetAsync(d_status, 0, sizeof(int32_t), s) != hipSuccess) return ORBFE_ERR_HIP;
    if (!n_mats) return ORBFE_OK;
    // records are read up to their own rows; in_pitch must hold a full cap-row record
    if (in_pitch < (size_t)orbfe_archive_mat_bytes(cap, 32, 1)) return ORBFE_ERR_ARG;
    hipLaunchKernelGGL(archive_read_desc_kernel,
                       dim3((cap * 4 + kArcBlock - 1) / kArcBlock > 0 ? (cap * 4 + kArcBlock - 1) / kArcBlock : 1, n_mats),
                       dim3(kArcBlock), 0, s, d_in, in_pitch, cap, d_desc, desc_pitch, d_rows,
                       d_status);
    return hipGetLastError() == hipSuccess ? ORBFE_OK : ORBFE_ERR_HIP;
}

}  // extern "C"
