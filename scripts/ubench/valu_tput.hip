// Per-instruction VALU throughput on gfx950: each kernel runs n iterations of
// 8 independent chains of one instruction type, W waves per SIMD on every
// SIMD of the chip.  Each wave reads the shader clock (s_memtime, one tick
// per shader cycle: MI355X_MICROARCH.md constants table) and the 100 MHz
// real-time clock (s_memrealtime) around its loop.  Printed per W:
//   cyc   shader cycles per wave-instruction per SIMD (loop cycles / (n 8 W))
//   GHz   the shader clock during the loop (cycles / real time)
//   G/s   wave-instructions per second per SIMD by the wall clock (hipEvent
//         around the launch): the issue rate a kernel can actually reach,
//         whatever the DVFS clock does
// Runs ~10 ms per launch at W = 8 so the clock settles.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>
typedef float f2 __attribute__((ext_vector_type(2)));
#define REP8(X) X X X X X X X X

__global__ __launch_bounds__(256) void k_add(float *o, float s, long long *cyc, int n) {
    float a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;
    const long long r0 = __builtin_amdgcn_s_memrealtime();
    const long long t0 = __builtin_amdgcn_s_memtime();
    for (int i = 0; i < n; ++i) {
        asm volatile("v_add_f32 %0, %0, %8\n v_add_f32 %1, %1, %8\n v_add_f32 %2, %2, %8\n v_add_f32 %3, %3, %8\n"
                     "v_add_f32 %4, %4, %8\n v_add_f32 %5, %5, %8\n v_add_f32 %6, %6, %8\n v_add_f32 %7, %7, %8"
                     : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) : "s"(s));
    }
    const long long t1 = __builtin_amdgcn_s_memtime();
    const long long r1 = __builtin_amdgcn_s_memrealtime();
    if ((threadIdx.x & 63) == 0) {
        cyc[2 * (blockIdx.x * 4 + (threadIdx.x >> 6))] = t1 - t0;
        cyc[2 * (blockIdx.x * 4 + (threadIdx.x >> 6)) + 1] = r1 - r0;
    }
    o[blockIdx.x * 256 + threadIdx.x] = a0 + a1 + a2 + a3 + a4 + a5 + a6 + a7;
}
__global__ __launch_bounds__(256) void k_dpp(float *o, float s, long long *cyc, int n) {
    float a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;
    float b = s;
    const long long r0 = __builtin_amdgcn_s_memrealtime();
    const long long t0 = __builtin_amdgcn_s_memtime();
    for (int i = 0; i < n; ++i) {
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
    const long long r1 = __builtin_amdgcn_s_memrealtime();
    if ((threadIdx.x & 63) == 0) {
        cyc[2 * (blockIdx.x * 4 + (threadIdx.x >> 6))] = t1 - t0;
        cyc[2 * (blockIdx.x * 4 + (threadIdx.x >> 6)) + 1] = r1 - r0;
    }
    o[blockIdx.x * 256 + threadIdx.x] = a0 + a1 + a2 + a3 + a4 + a5 + a6 + a7;
}
__global__ __launch_bounds__(256) void k_pk(float *o, float s, long long *cyc, int n) {
    f2 a0 = {1.f * threadIdx.x, 2.f}, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;
    f2 b = {s, s};
    const long long r0 = __builtin_amdgcn_s_memrealtime();
    const long long t0 = __builtin_amdgcn_s_memtime();
    for (int i = 0; i < n; ++i) {
        asm volatile("v_pk_add_f32 %0, %0, %8\n v_pk_add_f32 %1, %1, %8\n v_pk_add_f32 %2, %2, %8\n v_pk_add_f32 %3, %3, %8\n"
                     "v_pk_add_f32 %4, %4, %8\n v_pk_add_f32 %5, %5, %8\n v_pk_add_f32 %6, %6, %8\n v_pk_add_f32 %7, %7, %8"
                     : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) : "v"(b));
    }
    const long long t1 = __builtin_amdgcn_s_memtime();
    const long long r1 = __builtin_amdgcn_s_memrealtime();
    if ((threadIdx.x & 63) == 0) {
        cyc[2 * (blockIdx.x * 4 + (threadIdx.x >> 6))] = t1 - t0;
        cyc[2 * (blockIdx.x * 4 + (threadIdx.x >> 6)) + 1] = r1 - r0;
    }
    f2 t = a0 + a1 + a2 + a3 + a4 + a5 + a6 + a7;
    o[blockIdx.x * 256 + threadIdx.x] = t.x + t.y;
}
__global__ __launch_bounds__(256) void k_rcp(float *o, float s, long long *cyc, int n) {
    float a0 = threadIdx.x + 1, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;
    const long long r0 = __builtin_amdgcn_s_memrealtime();
    const long long t0 = __builtin_amdgcn_s_memtime();
    for (int i = 0; i < n; ++i) {
        asm volatile("v_rcp_f32 %0, %0\n v_rcp_f32 %1, %1\n v_rcp_f32 %2, %2\n v_rcp_f32 %3, %3\n"
                     "v_rcp_f32 %4, %4\n v_rcp_f32 %5, %5\n v_rcp_f32 %6, %6\n v_rcp_f32 %7, %7"
                     : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7));
    }
    const long long t1 = __builtin_amdgcn_s_memtime();
    const long long r1 = __builtin_amdgcn_s_memrealtime();
    if ((threadIdx.x & 63) == 0) {
        cyc[2 * (blockIdx.x * 4 + (threadIdx.x >> 6))] = t1 - t0;
        cyc[2 * (blockIdx.x * 4 + (threadIdx.x >> 6)) + 1] = r1 - r0;
    }
    o[blockIdx.x * 256 + threadIdx.x] = a0 + a1 + a2 + a3 + a4 + a5 + a6 + a7 + s;
}
__global__ __launch_bounds__(256) void k_bfecvt(float *o, float s, long long *cyc, int n) {
    int a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;
    const long long r0 = __builtin_amdgcn_s_memrealtime();
    const long long t0 = __builtin_amdgcn_s_memtime();
    for (int i = 0; i < n; ++i) {
        asm volatile("v_bfe_i32 %0, %0, 3, 11\n v_bfe_i32 %1, %1, 3, 11\n v_bfe_i32 %2, %2, 3, 11\n v_bfe_i32 %3, %3, 3, 11\n"
                     "v_bfe_i32 %4, %4, 3, 11\n v_bfe_i32 %5, %5, 3, 11\n v_bfe_i32 %6, %6, 3, 11\n v_bfe_i32 %7, %7, 3, 11"
                     : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7));
    }
    const long long t1 = __builtin_amdgcn_s_memtime();
    const long long r1 = __builtin_amdgcn_s_memrealtime();
    if ((threadIdx.x & 63) == 0) {
        cyc[2 * (blockIdx.x * 4 + (threadIdx.x >> 6))] = t1 - t0;
        cyc[2 * (blockIdx.x * 4 + (threadIdx.x >> 6)) + 1] = r1 - r0;
    }
    o[blockIdx.x * 256 + threadIdx.x] = a0 + a1 + a2 + a3 + a4 + a5 + a6 + a7 + s;
}
__global__ __launch_bounds__(256) void k_fma(float *o, float s, long long *cyc, int n) {
    float a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;
    float b = s;
    const long long r0 = __builtin_amdgcn_s_memrealtime();
    const long long t0 = __builtin_amdgcn_s_memtime();
    for (int i = 0; i < n; ++i) {
        asm volatile("v_fma_f32 %0, %0, %8, %8\n v_fma_f32 %1, %1, %8, %8\n v_fma_f32 %2, %2, %8, %8\n v_fma_f32 %3, %3, %8, %8\n"
                     "v_fma_f32 %4, %4, %8, %8\n v_fma_f32 %5, %5, %8, %8\n v_fma_f32 %6, %6, %8, %8\n v_fma_f32 %7, %7, %8, %8"
                     : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) : "v"(b));
    }
    const long long t1 = __builtin_amdgcn_s_memtime();
    const long long r1 = __builtin_amdgcn_s_memrealtime();
    if ((threadIdx.x & 63) == 0) {
        cyc[2 * (blockIdx.x * 4 + (threadIdx.x >> 6))] = t1 - t0;
        cyc[2 * (blockIdx.x * 4 + (threadIdx.x >> 6)) + 1] = r1 - r0;
    }
    o[blockIdx.x * 256 + threadIdx.x] = a0 + a1 + a2 + a3 + a4 + a5 + a6 + a7;
}
__global__ __launch_bounds__(256) void k_pkfma(float *o, float s, long long *cyc, int n) {
    f2 a0 = {1.f * threadIdx.x, 2.f}, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;
    f2 b = {s, s};
    const long long r0 = __builtin_amdgcn_s_memrealtime();
    const long long t0 = __builtin_amdgcn_s_memtime();
    for (int i = 0; i < n; ++i) {
        asm volatile("v_pk_fma_f32 %0, %0, %8, %8\n v_pk_fma_f32 %1, %1, %8, %8\n v_pk_fma_f32 %2, %2, %8, %8\n v_pk_fma_f32 %3, %3, %8, %8\n"
                     "v_pk_fma_f32 %4, %4, %8, %8\n v_pk_fma_f32 %5, %5, %8, %8\n v_pk_fma_f32 %6, %6, %8, %8\n v_pk_fma_f32 %7, %7, %8, %8"
                     : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) : "v"(b));
    }
    const long long t1 = __builtin_amdgcn_s_memtime();
    const long long r1 = __builtin_amdgcn_s_memrealtime();
    if ((threadIdx.x & 63) == 0) {
        cyc[2 * (blockIdx.x * 4 + (threadIdx.x >> 6))] = t1 - t0;
        cyc[2 * (blockIdx.x * 4 + (threadIdx.x >> 6)) + 1] = r1 - r0;
    }
    f2 t = a0 + a1 + a2 + a3 + a4 + a5 + a6 + a7;
    o[blockIdx.x * 256 + threadIdx.x] = t.x + t.y;
}

int main() {
    struct { const char *n; void (*k)(float *, float, long long *, int); } ks[] = {
        {"v_add_f32", k_add}, {"v_add_f32_dpp wave_shr", k_dpp}, {"v_pk_add_f32", k_pk},
        {"v_fma_f32", k_fma}, {"v_pk_fma_f32", k_pkfma}, {"v_rcp_f32", k_rcp}, {"v_bfe_i32", k_bfecvt}};
    const int maxb = 256 * 8;
    const int n = 65536;  // iterations per wave at W = 8 (scaled by 8 / W)
    float *o; hipMalloc(&o, maxb * 256 * 4);
    long long *cyc; hipMalloc(&cyc, maxb * 4 * 16);
    std::vector<long long> h(maxb * 8);
    printf("per W waves/SIMD: shader cycles per wave-instruction per SIMD | shader GHz | G wave-instr/s per SIMD (wall)\n");
    printf("%-24s", "instruction");
    for (int W : {1, 2, 4, 8}) printf(" |   W=%d cyc   GHz   G/s", W);
    printf("\n");
    for (auto &k : ks) {
        printf("%-24s", k.n);
        for (int W : {1, 2, 4, 8}) {
            const int blocks = 256 * W;  // 4-wave blocks, W per CU = W waves per SIMD
            const int nw = n * 8 / W;   // same instructions per SIMD for every W
            hipLaunchKernelGGL(k.k, dim3(blocks), dim3(256), 0, 0, o, 1.0f, cyc, nw / 16);
            hipEvent_t a, b; hipEventCreate(&a); hipEventCreate(&b);
            hipEventRecord(a);
            hipLaunchKernelGGL(k.k, dim3(blocks), dim3(256), 0, 0, o, 1.0f, cyc, nw);
            hipEventRecord(b); hipEventSynchronize(b);
            float ms; hipEventElapsedTime(&ms, a, b);
            hipMemcpy(h.data(), cyc, blocks * 4 * 16, hipMemcpyDeviceToHost);
            double sc = 0, sr = 0;
            for (int i = 0; i < blocks * 4; ++i) { sc += (double)h[2 * i]; sr += (double)h[2 * i + 1]; }
            const double per = sc / (blocks * 4) / ((double)nw * 8 * W);
            const double ghz = sc / (sr / 100e6) / 1e9;  // s_memrealtime: 100 MHz
            const double gps = (double)nw * 8 * W / (ms * 1e-3) / 1e9;  // per SIMD
            printf(" | %7.2f %5.2f %5.3f", per, ghz, gps);
        }
        printf("\n");
    }
    return 0;
}
