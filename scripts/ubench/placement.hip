// placement.hip -- where does the dispatcher put the waves of a launch that
// has fewer single-wave workgroups than the chip has SIMDs (a single 4K
// pair's K4 pass: 962 waves, 247 VGPRs, two waves per SIMD allowed)?
// Each wave records its XCC / SE / CU / SIMD (hardware id registers) and
// stays resident ~40 us, so every wave of the grid is in flight together;
// the host counts the SIMDs that hold two of them.
//   usage: placement [waves] [lds_bytes]
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <map>
#include <vector>

__global__ __launch_bounds__(64, 2) void place_kernel(unsigned *out, long spin) {
    // hold 247 VGPRs, as K4 at KB 6 does (the allocation sets the occupancy)
    asm volatile("" ::: "v246");
    unsigned hw = 0, xcc = 0;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hw));
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
    const long t0 = wall_clock64();
    while (wall_clock64() - t0 < spin) __builtin_amdgcn_s_sleep(10);
    if (threadIdx.x == 0) {
        out[2 * blockIdx.x] = hw;
        out[2 * blockIdx.x + 1] = xcc;
    }
}

int main(int argc, char **argv) {
    const int waves = argc > 1 ? atoi(argv[1]) : 962;
    const int lds = argc > 2 ? atoi(argv[2]) : 0;
    unsigned *d = nullptr;
    if (hipMalloc(&d, 8u * waves) != hipSuccess) return 1;
    // wall_clock64 runs at 100 MHz: 4000 ticks = 40 us
    hipLaunchKernelGGL(place_kernel, dim3(waves), dim3(64), lds, 0, d, 4000L);
    if (hipDeviceSynchronize() != hipSuccess) return 2;
    std::vector<unsigned> h(2 * waves);
    hipMemcpy(h.data(), d, 8u * waves, hipMemcpyDeviceToHost);
    std::map<unsigned long, int> per_simd, per_cu;
    for (int i = 0; i < waves; ++i) {
        const unsigned hw = h[2 * i], xcc = h[2 * i + 1] & 0xF;
        const unsigned simd = (hw >> 4) & 3, cu = (hw >> 8) & 15, sh = (hw >> 12) & 1,
                       se = (hw >> 13) & 7;
        const unsigned long cu_key = ((unsigned long)xcc << 16) | (se << 8) | (sh << 4) | cu;
        per_cu[cu_key]++;
        per_simd[(cu_key << 2) | simd]++;
    }
    std::map<int, int> hist_simd, hist_cu;
    for (auto &kv : per_simd) hist_simd[kv.second]++;
    for (auto &kv : per_cu) hist_cu[kv.second]++;
    printf("{\"waves\": %d, \"lds\": %d, \"simds_used\": %zu, \"cus_used\": %zu, \"waves_per_simd\": {",
           waves, lds, per_simd.size(), per_cu.size());
    bool first = true;
    for (auto &kv : hist_simd) {
        printf("%s\"%d\": %d", first ? "" : ", ", kv.first, kv.second);
        first = false;
    }
    printf("}, \"waves_per_cu\": {");
    first = true;
    for (auto &kv : hist_cu) {
        printf("%s\"%d\": %d", first ? "" : ", ", kv.first, kv.second);
        first = false;
    }
    printf("}}\n");
    hipFree(d);
    return 0;
}
