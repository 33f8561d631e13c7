// First-touch cost of a caller's fresh output planes (main.cpp:93 declares
// `cv::Mat u, v;` anew per call): time to fault in 2 planes of rows x cols
// doubles from fresh anonymous pages, by strategy and thread count.
//   hipcc -O2 -std=c++17 -pthread scripts/pcie/fault_probe.cpp -o scripts/pcie/fault_probe
//   scripts/pcie/fault_probe 2160 3840 [gpu]
// `gpu`: the HIP runtime initialised first, with a device allocation and a
// pinned stage, as in a process that calls the library.
#include <hip/hip_runtime.h>
#include <sys/mman.h>
#include <sys/utsname.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <thread>
#include <vector>

#ifndef MADV_POPULATE_WRITE
#define MADV_POPULATE_WRITE 23
#endif

static double now() {
    return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

int main(int argc, char **argv) {
    const size_t rows = argc > 1 ? atol(argv[1]) : 2160, cols = argc > 2 ? atol(argv[2]) : 3840;
    const size_t bytes = 2 * rows * cols * 8;
    const bool gpu = argc > 3 && strcmp(argv[3], "gpu") == 0;
    if (gpu) {
        void *d = nullptr, *h = nullptr;
        if (hipMalloc(&d, bytes) != hipSuccess || hipHostMalloc(&h, bytes / 2, 0) != hipSuccess)
            return 2;
        hipMemset(d, 0, bytes);
        hipDeviceSynchronize();
    }
    utsname u;
    uname(&u);
    char thp[256] = "?";
    if (FILE *f = fopen("/sys/kernel/mm/transparent_hugepage/enabled", "r")) {
        if (!fgets(thp, sizeof thp, f)) thp[0] = 0;
        fclose(f);
        thp[strcspn(thp, "\n")] = 0;
    }
    printf("{\"kernel\": \"%s\", \"thp\": \"%s\", \"MB\": %.1f, \"hip\": %d}\n", u.release, thp,
           bytes / 1e6, (int)gpu);
    const char *names[] = {"touch", "populate_write", "hugepage_touch", "hugepage_populate", "memset"};
    for (int strat = 0; strat < 5; ++strat) {
        for (int nt : {1, 4, 8, 16}) {
            double best = 1e9;
            int ok = 1;
            for (int rep = 0; rep < 3; ++rep) {
                char *p = (char *)mmap(nullptr, bytes, PROT_READ | PROT_WRITE,
                                       MAP_PRIVATE | MAP_ANONYMOUS, -1, 0);
                if (p == MAP_FAILED) return 1;
                const double t0 = now();
                if (strat == 2 || strat == 3) madvise(p, bytes, MADV_HUGEPAGE);
                std::vector<std::thread> th;
                for (int t = 0; t < nt; ++t)
                    th.emplace_back([&, t] {
                        const size_t a = bytes * t / nt & ~(size_t)4095, b = bytes * (t + 1) / nt & ~(size_t)4095;
                        const size_t e = t == nt - 1 ? bytes : b;
                        if (strat == 1 || strat == 3) {
                            if (madvise(p + a, e - a, MADV_POPULATE_WRITE) != 0) ok = 0;
                        } else if (strat == 4) {
                            memset(p + a, 0, e - a);
                        } else {
                            for (size_t o = a; o < e; o += 4096) *(volatile char *)(p + o) = 0;
                        }
                    });
                for (auto &x : th) x.join();
                const double dt = now() - t0;
                if (dt < best) best = dt;
                munmap(p, bytes);
            }
            printf("{\"strategy\": \"%s\", \"threads\": %d, \"ms\": %.3f, \"ok\": %d}\n", names[strat],
                   nt, best * 1e3, ok);
            fflush(stdout);
        }
    }
    return 0;
}
