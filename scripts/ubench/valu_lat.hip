// Issue rate of dependent VALU chains on gfx950 at low occupancy: C
// independent chains per wave (ILP), 1 or 2 waves per SIMD (forced by
// dynamic LDS).  Prints shader cycles per instruction per wave.
#include <hip/hip_runtime.h>
#include <cstdio>
typedef float f2 __attribute__((ext_vector_type(2)));
#define N 2048

template <int C, int OP>
__global__ __launch_bounds__(1024) void k(float *o, long long *cyc, float s) {
    extern __shared__ float pad[];
    float a[8];
    f2 b[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) { a[j] = threadIdx.x + j; b[j] = f2{a[j], a[j] + 1}; }
    const f2 sv = {s, s};
    const long long t0 = clock64();
    for (int i = 0; i < N; ++i) {
#pragma unroll
        for (int r = 0; r < 8 / C; ++r)
#pragma unroll
            for (int j = 0; j < C; ++j) {
                if constexpr (OP == 0)
                    asm volatile("v_add_f32 %0, %0, %1" : "+v"(a[j]) : "s"(s));
                else if constexpr (OP == 1)
                    asm volatile("v_pk_fma_f32 %0, %0, %1, %1" : "+v"(b[j]) : "v"(sv));
                else if constexpr (OP == 2)
                    asm volatile("s_nop 1\n v_add_f32_dpp %0, %0, %0 wave_shr:1 row_mask:0xf bank_mask:0xf bound_ctrl:1"
                                 : "+v"(a[j]));
                else if constexpr (OP == 3)  // no hazard padding (needs >= 4 chains)
                    asm volatile("v_add_f32_dpp %0, %0, %0 wave_shr:1 row_mask:0xf bank_mask:0xf bound_ctrl:1"
                                 : "+v"(a[j]));
                else if constexpr (OP == 4)  // row_shr:1 (within 16-lane rows)
                    asm volatile("v_add_f32_dpp %0, %0, %0 row_shr:1 row_mask:0xf bank_mask:0xf bound_ctrl:1"
                                 : "+v"(a[j]));
                else  // quad_perm swizzle
                    asm volatile("v_add_f32_dpp %0, %0, %0 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf"
                                 : "+v"(a[j]));
            }
    }
    const long long t1 = clock64();
    float acc = 0;
#pragma unroll
    for (int j = 0; j < 8; ++j) acc += a[j] + b[j].x;
    o[blockIdx.x * blockDim.x + threadIdx.x] = acc;
    if ((threadIdx.x & 63) == 0) cyc[blockIdx.x * (blockDim.x / 64) + threadIdx.x / 64] = t1 - t0;
    (void)pad;
}

template <int C, int OP>
void run(int threads, float *o, long long *cyc, long long *h, int lds = 100 * 1024, int blocks = 256) {
    hipLaunchKernelGGL((k<C, OP>), dim3(blocks), dim3(threads), lds, 0, o, cyc, 1.0f);
    if (hipGetLastError() != hipSuccess) { printf("launch failed\n"); return; }
    hipDeviceSynchronize();
    const int nw = blocks * threads / 64;
    hipMemcpy(h, cyc, nw * sizeof(long long), hipMemcpyDeviceToHost);
    double m = 0;
    for (int i = 0; i < nw; ++i) m += h[i];
    m /= nw;
    printf("op %d chains %d waves/SIMD %d x blocks/CU %d: %.2f cycles/instr/wave\n", OP, C,
           threads / 256, blocks / 256, m / (N * 8.0));
}

int main() {
    float *o;
    long long *cyc; static long long h[65536];
    hipMalloc(&o, 1024 * 1024 * 4);
    hipMalloc(&cyc, 65536 * 8);
    hipFuncSetAttribute((const void *)k<1, 0>, hipFuncAttributeMaxDynamicSharedMemorySize, 100 * 1024);
    for (int t : {256, 512, 1024}) {
        run<8, 0>(t, o, cyc, h); run<8, 1>(t, o, cyc, h); run<8, 3>(t, o, cyc, h);
    }
    // 2 and 4 blocks of 1024 threads per CU: 8 and 16 waves per SIMD
    run<8, 0>(1024, o, cyc, h, 60 * 1024, 512); run<8, 1>(1024, o, cyc, h, 60 * 1024, 512);
    run<8, 0>(1024, o, cyc, h, 30 * 1024, 1024); run<8, 1>(1024, o, cyc, h, 30 * 1024, 1024);
    return 0;
}
