// FETCH_SIZE / WRITE_SIZE calibration for the access widths the Jacobi
// kernels use (MI355X_MICROARCH.md: "other access widths are uncalibrated:
// calibrate on a known byte count in your own access pattern").  Each kernel
// streams a 1 GiB buffer (4x the 256 MiB Infinity Cache) once with raw buffer
// loads or stores of 4, 8 or 16 B per lane, rows of 512 B per wave like K4's
// row loads; rocprofv3 --pmc FETCH_SIZE (or WRITE_SIZE) per dispatch divided
// by the printed byte count is the correction factor.
//
//   hipcc --offload-arch=gfx950 -O3 -o fetch_calib fetch_calib.hip
//   rocprofv3 --pmc FETCH_SIZE -d out -o run --output-format csv -- ./fetch_calib
#include <hip/hip_runtime.h>
#include <cstdio>

typedef unsigned u2v __attribute__((ext_vector_type(2)));
typedef unsigned u4v __attribute__((ext_vector_type(4)));

constexpr size_t kBytes = size_t(1) << 30;

template <int B>
__global__ void __launch_bounds__(256) rd(const unsigned *buf, unsigned *out) {
    auto r = __builtin_amdgcn_make_buffer_rsrc(const_cast<unsigned *>(buf), 0, 0x7fffffff, 0x00020000);
    const size_t per_wave = 64 * B;
    const size_t waves = kBytes / per_wave;
    const size_t gw = (blockIdx.x * blockDim.x + threadIdx.x) >> 6;
    const size_t nw = (gridDim.x * blockDim.x) >> 6;
    const int lane = threadIdx.x & 63;
    unsigned acc = 0;
    for (size_t w = gw; w < waves; w += nw) {
        const size_t off = w * per_wave + size_t(lane) * B;
        // voffset holds the low 31 bits, soffset the rest (buffer < 2 GiB)
        if constexpr (B == 4) acc ^= __builtin_amdgcn_raw_buffer_load_b32(r, (int)off, 0, 0);
        if constexpr (B == 8) {
            u2v x = __builtin_amdgcn_raw_buffer_load_b64(r, (int)off, 0, 0);
            acc ^= x.x ^ x.y;
        }
        if constexpr (B == 16) {
            u4v x = __builtin_amdgcn_raw_buffer_load_b128(r, (int)off, 0, 0);
            acc ^= x.x ^ x.y ^ x.z ^ x.w;
        }
    }
    out[blockIdx.x * blockDim.x + threadIdx.x] = acc;
}

template <int B>
__global__ void __launch_bounds__(256) wr(unsigned *buf) {
    auto r = __builtin_amdgcn_make_buffer_rsrc(buf, 0, 0x7fffffff, 0x00020000);
    const size_t per_wave = 64 * B;
    const size_t waves = kBytes / per_wave;
    const size_t gw = (blockIdx.x * blockDim.x + threadIdx.x) >> 6;
    const size_t nw = (gridDim.x * blockDim.x) >> 6;
    const int lane = threadIdx.x & 63;
    for (size_t w = gw; w < waves; w += nw) {
        const size_t off = w * per_wave + size_t(lane) * B;
        if constexpr (B == 4) __builtin_amdgcn_raw_buffer_store_b32(unsigned(w), r, (int)off, 0, 0);
        if constexpr (B == 8) __builtin_amdgcn_raw_buffer_store_b64(u2v{unsigned(w), 1u}, r, (int)off, 0, 0);
        if constexpr (B == 16)
            __builtin_amdgcn_raw_buffer_store_b128(u4v{unsigned(w), 1u, 2u, 3u}, r, (int)off, 0, 0);
    }
}

int main() {
    unsigned *buf, *out;
    const int blocks = 4096, threads = 256;
    if (hipMalloc(&buf, kBytes) != hipSuccess || hipMalloc(&out, size_t(blocks) * threads * 4) != hipSuccess) {
        printf("alloc failed\n");
        return 1;
    }
    hipMemset(buf, 1, kBytes);
    hipDeviceSynchronize();
    for (int rep = 0; rep < 2; ++rep) {
        hipLaunchKernelGGL(rd<4>, dim3(blocks), dim3(threads), 0, 0, buf, out);
        hipLaunchKernelGGL(rd<8>, dim3(blocks), dim3(threads), 0, 0, buf, out);
        hipLaunchKernelGGL(rd<16>, dim3(blocks), dim3(threads), 0, 0, buf, out);
        hipLaunchKernelGGL(wr<4>, dim3(blocks), dim3(threads), 0, 0, buf);
        hipLaunchKernelGGL(wr<8>, dim3(blocks), dim3(threads), 0, 0, buf);
        hipLaunchKernelGGL(wr<16>, dim3(blocks), dim3(threads), 0, 0, buf);
    }
    if (hipDeviceSynchronize() != hipSuccess) {
        printf("kernel failed\n");
        return 1;
    }
    printf("{\"bytes_per_dispatch\": %zu}\n", kBytes);
    hipFree(buf);
    hipFree(out);
    return 0;
}
