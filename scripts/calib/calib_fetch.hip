// FETCH_SIZE calibration for K2's access widths on gfx950: 4-byte-per-lane
// (dword, odd-width images) and 8-byte-per-lane (qword, the column-pair
// loads of even-width images) coalesced raw buffer loads.  Each kernel reads
// `n` floats exactly once and writes one float per wave.  Known byte count =
// 4*n; compare with FETCH_SIZE*1024.
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
__global__ __launch_bounds__(256) void calib_qword_read(const float *x, long n, float *out) {
    const long wave = (blockIdx.x * 256L + threadIdx.x) >> 6;
    const int lane = threadIdx.x & 63;
    const long rows = n / 128;
    const long nw = (long)gridDim.x * 4;
    float s = 0.f;
    for (long r = wave; r < rows; r += nw) {
        const auto rs = __builtin_amdgcn_make_buffer_rsrc((void *)(x + r * 128), 0, 512, 0x00020000);
        const auto v = __builtin_amdgcn_raw_buffer_load_b64(rs, lane * 8, 0, 0);
        s += __uint_as_float(v[0]) + __uint_as_float(v[1]);
    }
    if (lane == 0) out[wave] = s;
}
extern "C" int calib_run(const float *x, long n, float *out, int blocks) {
    hipLaunchKernelGGL(calib_dword_read, dim3(blocks), dim3(256), 0, 0, x, n, out);
    return (int)hipDeviceSynchronize();
}
extern "C" int calib_run_qword(const float *x, long n, float *out, int blocks) {
    hipLaunchKernelGGL(calib_qword_read, dim3(blocks), dim3(256), 0, 0, x, n, out);
    return (int)hipDeviceSynchronize();
}
