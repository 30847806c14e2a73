// variant_rot.cpp — TEST INFRASTRUCTURE ONLY: the rBRIEF sample offsets of
// computeOrbDescriptor (skaegy/ORBSLAM_MapSave src/ORBextractor.cc:107-119) evaluated the way a
// real build of the reference evaluates them, for the H4 residual study (oracle/residuals.py).
//
// The reference writes `float a = (float)cos(angle), b = (float)sin(angle)` with a float
// `angle` under `using namespace std` (66, 111), i.e. glibc cosf / sinf, and samples
// center[cvRound(x*b + y*a)*step + cvRound(x*a - y*b)].  Its Release build is
// `-O3 -march=native` in C++ mode (CMakeLists.txt:10-11 + CMAKE_BUILD_TYPE=Release, build.sh),
// where GCC contracts those expressions into FMAs on an FMA-capable host.  oracle/Makefile
// compiles this file twice: ROT_NAME=oracle_rot_fma with -ffp-contract=fast on x86-64-v3 (GCC
// picks the contraction, as it would in the reference), and ROT_NAME=oracle_rot_plain with
// -ffp-contract=off.  -fno-tree-vectorize keeps the scalar form the reference's macro loop has.
#include <cmath>

extern "C" void ROT_NAME(float kpt_angle, int glibc_trig, const int* pattern, int npoints,
                         int* iy, int* ix) {
    const float factor_pi = (float)(3.14159265358979323846 / 180.f);  // factorPI (106)
    const float angle = kpt_angle * factor_pi;
    float a, b;
    if (glibc_trig) {
        a = (float)std::cos(angle);  // cosf
        b = (float)std::sin(angle);
    } else {
        a = (float)std::cos((double)angle);  // the pinned oracle's correctly rounded choice
        b = (float)std::sin((double)angle);
    }
    for (int i = 0; i < npoints; ++i) {
        const int x = pattern[2 * i], y = pattern[2 * i + 1];
        iy[i] = (int)std::lrintf(x * b + y * a);  // cvRound: round half to even
        ix[i] = (int)std::lrintf(x * a - y * b);
    }
}
