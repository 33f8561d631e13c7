// Per-instruction VALU throughput on gfx950: each kernel runs N iterations of
// 8 independent chains of one instruction type.  Every wave reads the shader
// clock (s_memtime: one tick per shader cycle, MI355X_MICROARCH.md constants
// table) around its loop, so the cost is in cycles, independent of the DVFS
// clock; W waves per SIMD share the SIMD, so the SIMD's cycles per
// wave-instruction = a wave's loop cycles / (N * 8 * W).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>
typedef float f2 __attribute__((ext_vector_type(2)));
#define N 4096
#define REP8(X) X X X X X X X X

__global__ __launch_bounds__(256) void k_add(float *o, float s, long long *cyc) {
    float a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;
    const long long t0 = __builtin_amdgcn_s_memtime();
    for (int i = 0; i < N; ++i) {
        asm volatile("v_add_f32 %0, %0, %8\n v_add_f32 %1, %1, %8\n v_add_f32 %2, %2, %8\n v_add_f32 %3, %3, %8\n"
                     "v_add_f32 %4, %4, %8\n v_add_f32 %5, %5, %8\n v_add_f32 %6, %6, %8\n v_add_f32 %7, %7, %8"
                     : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) : "s"(s));
    }
    const long long t1 = __builtin_amdgcn_s_memtime();
    if ((threadIdx.x & 63) == 0) cyc[blockIdx.x * 4 + (threadIdx.x >> 6)] = t1 - t0;
    o[blockIdx.x * 256 + threadIdx.x] = a0 + a1 + a2 + a3 + a4 + a5 + a6 + a7;
}
__global__ __launch_bounds__(256) void k_dpp(float *o, float s, long long *cyc) {
    float a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;
    float b = s;
    const long long t0 = __builtin_amdgcn_s_memtime();
    for (int i = 0; i < N; ++i) {
        asm volatile("v_add_f32_dpp %0, %8, %0 wave_shr:1 row_mask:0xf bank_mask:0xf bound_ctrl:1\n"
                     "v_add_f32_dpp %1, %8, %1 wave_shr:1 row_mask:0xf bank_mask:0xf bound_ctrl:1\n"
                     "v_add_f32_dpp %2, %8, %2 wave_shr:1 row_mask:0xf bank_mask:0xf bound_ctrl:1\n"
                     "v_add_f32_dpp %3, %8, %3 wave_shr:1 row_mask:0xf bank_mask:0xf bound_ctrl:1\n"
                     "v_add_f32_dpp %4, %8, %4 wave_shr:1 row_mask:0xf bank_mask:0xf bound_ctrl:1\n"
                     "v_add_f32_dpp %5, %8, %5 wave_shr:1 row_mask:0xf bank_mask:0xf bound_ctrl:1\n"
                     "v_add_f32_dpp %6, %8, %6 wave_shr:1 row_mask:0xf bank_mask:0xf bound_ctrl:1\n"
                     "v_add_f32_dpp %7, %8, %7 wave_shr:1 row_mask:0xf bank_mask:0xf bound_ctrl:1"
                     : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) : "v"(b));
    }
    const long long t1 = __builtin_amdgcn_s_memtime();
    if ((threadIdx.x & 63) == 0) cyc[blockIdx.x * 4 + (threadIdx.x >> 6)] = t1 - t0;
    o[blockIdx.x * 256 + threadIdx.x] = a0 + a1 + a2 + a3 + a4 + a5 + a6 + a7;
}
__global__ __launch_bounds__(256) void k_pk(float *o, float s, long long *cyc) {
    f2 a0 = {1.f * threadIdx.x, 2.f}, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;
    f2 b = {s, s};
    const long long t0 = __builtin_amdgcn_s_memtime();
    for (int i = 0; i < N; ++i) {
        asm volatile("v_pk_add_f32 %0, %0, %8\n v_pk_add_f32 %1, %1, %8\n v_pk_add_f32 %2, %2, %8\n v_pk_add_f32 %3, %3, %8\n"
                     "v_pk_add_f32 %4, %4, %8\n v_pk_add_f32 %5, %5, %8\n v_pk_add_f32 %6, %6, %8\n v_pk_add_f32 %7, %7, %8"
                     : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) : "v"(b));
    }
    const long long t1 = __builtin_amdgcn_s_memtime();
    if ((threadIdx.x & 63) == 0) cyc[blockIdx.x * 4 + (threadIdx.x >> 6)] = t1 - t0;
    f2 t = a0 + a1 + a2 + a3 + a4 + a5 + a6 + a7;
    o[blockIdx.x * 256 + threadIdx.x] = t.x + t.y;
}
__global__ __launch_bounds__(256) void k_rcp(float *o, float s, long long *cyc) {
    float a0 = threadIdx.x + 1, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;
    const long long t0 = __builtin_amdgcn_s_memtime();
    for (int i = 0; i < N; ++i) {
        asm volatile("v_rcp_f32 %0, %0\n v_rcp_f32 %1, %1\n v_rcp_f32 %2, %2\n v_rcp_f32 %3, %3\n"
                     "v_rcp_f32 %4, %4\n v_rcp_f32 %5, %5\n v_rcp_f32 %6, %6\n v_rcp_f32 %7, %7"
                     : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7));
    }
    const long long t1 = __builtin_amdgcn_s_memtime();
    if ((threadIdx.x & 63) == 0) cyc[blockIdx.x * 4 + (threadIdx.x >> 6)] = t1 - t0;
    o[blockIdx.x * 256 + threadIdx.x] = a0 + a1 + a2 + a3 + a4 + a5 + a6 + a7 + s;
}
__global__ __launch_bounds__(256) void k_bfecvt(float *o, float s, long long *cyc) {
    int a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;
    const long long t0 = __builtin_amdgcn_s_memtime();
    for (int i = 0; i < N; ++i) {
        asm volatile("v_bfe_i32 %0, %0, 3, 11\n v_bfe_i32 %1, %1, 3, 11\n v_bfe_i32 %2, %2, 3, 11\n v_bfe_i32 %3, %3, 3, 11\n"
                     "v_bfe_i32 %4, %4, 3, 11\n v_bfe_i32 %5, %5, 3, 11\n v_bfe_i32 %6, %6, 3, 11\n v_bfe_i32 %7, %7, 3, 11"
                     : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7));
    }
    const long long t1 = __builtin_amdgcn_s_memtime();
    if ((threadIdx.x & 63) == 0) cyc[blockIdx.x * 4 + (threadIdx.x >> 6)] = t1 - t0;
    o[blockIdx.x * 256 + threadIdx.x] = a0 + a1 + a2 + a3 + a4 + a5 + a6 + a7 + s;
}
__global__ __launch_bounds__(256) void k_fma(float *o, float s, long long *cyc) {
    float a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;
    float b = s;
    const long long t0 = __builtin_amdgcn_s_memtime();
    for (int i = 0; i < N; ++i) {
        asm volatile("v_fma_f32 %0, %0, %8, %8\n v_fma_f32 %1, %1, %8, %8\n v_fma_f32 %2, %2, %8, %8\n v_fma_f32 %3, %3, %8, %8\n"
                     "v_fma_f32 %4, %4, %8, %8\n v_fma_f32 %5, %5, %8, %8\n v_fma_f32 %6, %6, %8, %8\n v_fma_f32 %7, %7, %8, %8"
                     : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) : "v"(b));
    }
    const long long t1 = __builtin_amdgcn_s_memtime();
    if ((threadIdx.x & 63) == 0) cyc[blockIdx.x * 4 + (threadIdx.x >> 6)] = t1 - t0;
    o[blockIdx.x * 256 + threadIdx.x] = a0 + a1 + a2 + a3 + a4 + a5 + a6 + a7;
}
__global__ __launch_bounds__(256) void k_pkfma(float *o, float s, long long *cyc) {
    f2 a0 = {1.f * threadIdx.x, 2.f}, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;
    f2 b = {s, s};
    const long long t0 = __builtin_amdgcn_s_memtime();
    for (int i = 0; i < N; ++i) {
        asm volatile("v_pk_fma_f32 %0, %0, %8, %8\n v_pk_fma_f32 %1, %1, %8, %8\n v_pk_fma_f32 %2, %2, %8, %8\n v_pk_fma_f32 %3, %3, %8, %8\n"
                     "v_pk_fma_f32 %4, %4, %8, %8\n v_pk_fma_f32 %5, %5, %8, %8\n v_pk_fma_f32 %6, %6, %8, %8\n v_pk_fma_f32 %7, %7, %8, %8"
                     : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) : "v"(b));
    }
    const long long t1 = __builtin_amdgcn_s_memtime();
    if ((threadIdx.x & 63) == 0) cyc[blockIdx.x * 4 + (threadIdx.x >> 6)] = t1 - t0;
    f2 t = a0 + a1 + a2 + a3 + a4 + a5 + a6 + a7;
    o[blockIdx.x * 256 + threadIdx.x] = t.x + t.y;
}

int main() {
    struct { const char *n; void (*k)(float *, float, long long *); } ks[] = {
        {"v_add_f32", k_add}, {"v_add_f32_dpp wave_shr", k_dpp}, {"v_pk_add_f32", k_pk},
        {"v_fma_f32", k_fma}, {"v_pk_fma_f32", k_pkfma}, {"v_rcp_f32", k_rcp}, {"v_bfe_i32", k_bfecvt}};
    const int maxb = 256 * 8;
    float *o; hipMalloc(&o, maxb * 256 * 4);
    long long *cyc; hipMalloc(&cyc, maxb * 4 * 8);
    std::vector<long long> h(maxb * 4);
    printf("cycles per wave-instruction per SIMD (s_memtime shader cycles), W waves/SIMD\n");
    printf("%-26s %8s %8s %8s %8s   %s\n", "instruction", "W=1", "W=2", "W=4", "W=8", "wall ms @W=8 -> GHz");
    for (auto &k : ks) {
        printf("%-26s", k.n);
        float ms8 = 0; double c8 = 0;
        for (int W : {1, 2, 4, 8}) {
            const int blocks = 256 * W;  // 4-wave blocks, W per CU = W waves per SIMD
            hipLaunchKernelGGL(k.k, dim3(blocks), dim3(256), 0, 0, o, 1.0f, cyc);
            hipEvent_t a, b; hipEventCreate(&a); hipEventCreate(&b);
            hipEventRecord(a);
            hipLaunchKernelGGL(k.k, dim3(blocks), dim3(256), 0, 0, o, 1.0f, cyc);
            hipEventRecord(b); hipEventSynchronize(b);
            float ms; hipEventElapsedTime(&ms, a, b);
            hipMemcpy(h.data(), cyc, blocks * 4 * 8, hipMemcpyDeviceToHost);
            double sum = 0; for (int i = 0; i < blocks * 4; ++i) sum += (double)h[i];
            const double per = sum / (blocks * 4) / ((double)N * 8 * W);
            printf(" %8.2f", per);
            if (W == 8) { ms8 = ms; c8 = sum / (blocks * 4); }
        }
        // effective clock: a wave's loop cycles / wall time of the launch
        printf("   %.3f ms -> %.2f GHz\n", ms8, c8 / (ms8 * 1e-3) / 1e9);
    }
    return 0;
}
