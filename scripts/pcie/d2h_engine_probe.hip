// Does a D2H copy overlap a chip-filling kernel (a DMA engine) or wait for
// its workgroup slots (a blit kernel)?  A filler kernel occupies every CU
// for ~13 ms on stream s2; the copy is issued on s1 right after; we time the
// copy's completion relative to the filler's end.  Variants: hipMemcpyAsync,
// hipMemcpyDtoHAsync, hipMemcpy2DAsync (row-pitched), hipMemcpyAsync with
// hipMemcpyDefault.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <chrono>
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); exit(1); } } while (0)

__global__ void spin(float *o, int n) {
    float a = threadIdx.x, b = 1.0001f;
    for (int i = 0; i < n; ++i) a = a * b + 0.5f;
    if (a == 12345.f) o[0] = a;
}

int main() {
    const char *sd = getenv("HSA_ENABLE_SDMA");
    printf("HSA_ENABLE_SDMA=%s\n", sd ? sd : "(unset)");
    const size_t bytes = 8ull * 1080 * 1920 * 4;  // one f32 plane batch, 66 MB
    void *d; CK(hipMalloc(&d, bytes)); CK(hipMemset(d, 1, bytes));
    void *h; CK(hipHostMalloc(&h, bytes, hipHostMallocDefault));
    float *o; CK(hipMalloc(&o, 4));
    hipStream_t s1, s2; CK(hipStreamCreateWithFlags(&s1, hipStreamNonBlocking)); CK(hipStreamCreateWithFlags(&s2, hipStreamNonBlocking));
    hipEvent_t f0, f1, c1; CK(hipEventCreate(&f0)); CK(hipEventCreate(&f1)); CK(hipEventCreate(&c1));
    auto copy = [&](int v) {
        switch (v) {
        case 0: CK(hipMemcpyAsync(h, d, bytes, hipMemcpyDeviceToHost, s1)); break;
        case 1: CK(hipMemcpyDtoHAsync(h, (hipDeviceptr_t)d, bytes, s1)); break;
        case 2: CK(hipMemcpy2DAsync(h, 7680, d, 7680, 7680, bytes / 7680, hipMemcpyDeviceToHost, s1)); break;
        case 3: CK(hipMemcpyAsync(h, d, bytes, hipMemcpyDefault, s1)); break;
        }
    };
    const char *names[] = {"hipMemcpyAsync D2H", "hipMemcpyDtoHAsync", "hipMemcpy2DAsync", "hipMemcpyAsync Default"};
    for (int v = 0; v < 4; ++v) {
        copy(v); CK(hipDeviceSynchronize());
        // alone
        CK(hipEventRecord(f0, s1)); copy(v); CK(hipEventRecord(c1, s1)); CK(hipEventSynchronize(c1));
        float alone; CK(hipEventElapsedTime(&alone, f0, c1));
        // behind a chip-filling kernel on another stream
        CK(hipEventRecord(f0, s2));
        hipLaunchKernelGGL(spin, dim3(256 * 8), dim3(256), 0, s2, o, 400000);
        CK(hipEventRecord(f1, s2));
        copy(v);
        CK(hipEventRecord(c1, s1));
        CK(hipDeviceSynchronize());
        float fill, done; CK(hipEventElapsedTime(&fill, f0, f1)); CK(hipEventElapsedTime(&done, f0, c1));
        printf("%-24s alone %6.3f ms (%5.1f GB/s) | filler %6.3f ms, copy done at %6.3f ms -> %s\n",
               names[v], alone, bytes / alone / 1e6, fill, done,
               done < fill * 0.9 ? "overlapped (DMA engine)" : "after the filler (blit kernel)");
    }
    return 0;
}
