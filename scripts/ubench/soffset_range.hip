// Does the gfx950 raw-buffer range check include soffset?  Loads with voffset
// in range and soffset past num_records, and a "negative" soffset: all read 0
// (measured on MI355X: soffset is range-checked), which K4 relies on.
#include <hip/hip_runtime.h>
#include <cstdio>
__global__ void k(float *buf, int nbytes, float *out) {
    auto r = __builtin_amdgcn_make_buffer_rsrc(buf, 0, nbytes, 0x00020000);
    const int lane = threadIdx.x;
    out[lane] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(r, lane * 4, 0, 0));
    out[64 + lane] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(r, lane * 4, nbytes, 0));
    out[128 + lane] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(r, lane * 4, nbytes - 128, 0));
    out[192 + lane] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(r, lane * 4, -256, 0));
}
int main() {
    const int n = 1024;  // floats in the descriptor; the buffer is larger
    float *buf, *out;
    hipMalloc(&buf, 4 * n * 4);
    hipMalloc(&out, 256 * 4);
    float h[4 * 1024];
    for (int i = 0; i < 4 * n; ++i) h[i] = 1.0f + i;
    hipMemcpy(buf, h, sizeof h, hipMemcpyHostToDevice);
    hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, buf + 1024, n * 4, out);
    float o[256];
    hipMemcpy(o, out, sizeof o, hipMemcpyDeviceToHost);
    printf("soff 0:      lane0 %g lane63 %g\n", o[0], o[63]);
    printf("soff=nbytes: lane0 %g lane63 %g  (0 => soffset range-checked)\n", o[64], o[127]);
    printf("soff=nb-128: lane0 %g lane31 %g lane32 %g lane63 %g\n", o[128], o[159], o[160], o[191]);
    printf("soff=-256:   lane0 %g lane63 %g\n", o[192], o[255]);
    return 0;
}
