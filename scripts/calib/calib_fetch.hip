// FETCH_SIZE calibration for 4-byte-per-lane coalesced loads on gfx950 (the
// access width hs_jacobi_kernel uses).  Reads `n` floats exactly once, one
// dword per lane per row of 64, via raw buffer loads like K2; writes one
// float per wave.  Known byte count = 4*n; compare with FETCH_SIZE*1024.
#include <hip/hip_runtime.h>
__global__ __launch_bounds__(256) void calib_dword_read(const float *x, long n, float *out) {
    const long wave = (blockIdx.x * 256L + threadIdx.x) >> 6;
    const int lane = threadIdx.x & 63;
    const long rows = n / 64;
    const long nw = (long)gridDim.x * 4;
    float s = 0.f;
    for (long r = wave; r < rows; r += nw) {
        const auto rs = __builtin_amdgcn_make_buffer_rsrc((void *)(x + r * 64), 0, 256, 0x00020000);
        s += __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(rs, lane * 4, 0, 0));
    }
    if (lane == 0) out[wave] = s;
}
extern "C" int calib_run(const float *x, long n, float *out, int blocks) {
    hipLaunchKernelGGL(calib_dword_read, dim3(blocks), dim3(256), 0, 0, x, n, out);
    return (int)hipDeviceSynchronize();
}
