// hsflow_pyramid.hip -- config 5: the coarse-to-fine
// warm start around the Horn-Schunck hot loop.
//
// HornSchunckOF has no pyramid; the design precedent is the repository's BM
// module (BMOpticalFlow/.../OpticalFlow/MultiResolution.cpp:9-97 Pyramider,
// OpticalFlow.cpp:197-210 Add_VectorOffset):
//
//  K0 hs_pyrdown_kernel   one level down: 5-tap kernel (a/2, 1/2, a, 1/2, a/2)
//     normalised, a = 0.4, i.e. (2, 5, 4, 5, 2) / 18 per axis, stride 2,
//     reflect-101 border, level size ceil(n / 2).  For integer-valued pairs
//     (K1's per-pair flag is 0) the weighted sum S is an exact integer in
//     fp32 (<= 255 * 324) and the level is rounded half-up, floor((S + 162) /
//     324), in integer arithmetic -- bit-exact with the fp64 oracle and still
//     integer-valued, so every level keeps K2's packed exact gradients.
//     Other pairs keep S / 324.
//  KU hs_upflow_kernel    warm start of the finer level: u = 2 u_c(y/2, x/2).
//
// Both are one-off per level (HBM-bound, a few bytes per pixel) next to the
// `iters` Jacobi iterations that follow; a plain one-pixel-per-thread map
// with the 5x5 neighbourhood served from L1/L2 is enough.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "hsflow_internal.h"

namespace hsflow {
namespace {

__device__ __forceinline__ int refl101(int p, int len) {
    // |overshoot| <= 3 here (2y + 4 <= len + 2 for len >= 1)
    if (len == 1) return 0;
    p = p < 0 ? -p : p;
    p = p >= len ? 2 * (len - 1) - p : p;
    return p < 0 ? -p : p;  // len == 2 can bounce twice
}

template <typename T> __device__ __forceinline__ float ldf(const T *p) {
    return (float)*p;
}

// block 64 x 4, one output pixel per thread; grid (ceil(c2/64), ceil(r2/4), batch)
template <typename T>
__global__ __launch_bounds__(256) void hs_pyrdown_kernel(const T *__restrict__ src,
                                                         int rows, int cols,
                                                         float *__restrict__ dst, int r2,
                                                         int c2,
                                                         const uint32_t *__restrict__ flags) {
    const int x = blockIdx.x * 64 + threadIdx.x;
    const int y = blockIdx.y * 4 + threadIdx.y;
    if (x >= c2 || y >= r2) return;
    const T *s = src + (size_t)blockIdx.z * rows * cols;
    const float w[5] = {2.f, 5.f, 4.f, 5.f, 2.f};
    int cx[5];
#pragma unroll
    for (int n = 0; n < 5; ++n) cx[n] = refl101(2 * x + n - 2, cols);
    float S = 0.f;
#pragma unroll
    for (int m = 0; m < 5; ++m) {
        const T *row = s + (size_t)refl101(2 * y + m - 2, rows) * cols;
        float h = 0.f;
#pragma unroll
        for (int n = 0; n < 5; ++n) h += w[n] * ldf(row + cx[n]);
        S += w[m] * h;
    }
    float out;
    if (flags[blockIdx.z] == 0u)
        out = (float)(((int)S + 162) / 324);  // exact: S is an integer <= 82620
    else
        out = S / 324.0f;
    dst[(size_t)blockIdx.z * r2 * c2 + (size_t)y * c2 + x] = out;
}

__global__ __launch_bounds__(256) void hs_upflow_kernel(const float *__restrict__ uc,
                                                        const float *__restrict__ vc,
                                                        int rc, int cc,
                                                        float *__restrict__ u,
                                                        float *__restrict__ v, int rows,
                                                        int cols) {
    const int x = blockIdx.x * 64 + threadIdx.x;
    const int y = blockIdx.y * 4 + threadIdx.y;
    if (x >= cols || y >= rows) return;
    const size_t ic = (size_t)blockIdx.z * rc * cc + (size_t)(y >> 1) * cc + (x >> 1);
    const size_t o = (size_t)blockIdx.z * rows * cols + (size_t)y * cols + x;
    u[o] = 2.0f * uc[ic];  // OpticalFlow.cpp:205-206
    v[o] = 2.0f * vc[ic];
}

}  // namespace

hipError_t launch_pyrdown(const void *src, int dtype, int rows, int cols, int batch,
                          float *dst, const uint32_t *flags, hipStream_t s) {
    const int r2 = (rows + 1) / 2, c2 = (cols + 1) / 2;
    dim3 blk(64, 4, 1), grd((c2 + 63) / 64, (r2 + 3) / 4, batch);
    switch (dtype) {
    case 0:
        hipLaunchKernelGGL(hs_pyrdown_kernel<uint8_t>, grd, blk, 0, s,
                           (const uint8_t *)src, rows, cols, dst, r2, c2, flags);
        break;
    case 1:
        hipLaunchKernelGGL(hs_pyrdown_kernel<float>, grd, blk, 0, s, (const float *)src,
                           rows, cols, dst, r2, c2, flags);
        break;
    case 2:  // HSFLOW_F64
        hipLaunchKernelGGL(hs_pyrdown_kernel<double>, grd, blk, 0, s, (const double *)src,
                           rows, cols, dst, r2, c2, flags);
        break;
    case 3:
        hipLaunchKernelGGL(hs_pyrdown_kernel<_Float16>, grd, blk, 0, s,
                           (const _Float16 *)src, rows, cols, dst, r2, c2, flags);
        break;
    default: return hipErrorInvalidValue;
    }
    return hipGetLastError();
}

hipError_t launch_upflow(const float *uc, const float *vc, int rc, int cc, float *u,
                         float *v, int rows, int cols, int batch, hipStream_t s) {
    dim3 blk(64, 4, 1), grd((cols + 63) / 64, (rows + 3) / 4, batch);
    hipLaunchKernelGGL(hs_upflow_kernel, grd, blk, 0, s, uc, vc, rc, cc, u, v, rows, cols);
    return hipGetLastError();
}

}  // namespace hsflow
