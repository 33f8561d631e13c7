// ThreadSanitizer hammer of the host copy pool (cpp-optical-flow_amd/csrc/
// hsflow_pool.h), built and run by tests/test_sanitizers.py on the CPU:
// several host threads submit jobs at once, as hsflow_flow_multi's
// per-device workers do (one job runs on the pool, the others inline), and
// every item of every job must run exactly once.
#include <cstdio>
#include <cstdlib>
#include <thread>
#include <vector>

#include "hsflow_pool.h"

int main(int argc, char **argv) {
    const int callers = argc > 1 ? std::atoi(argv[1]) : 4;
    const int rounds = argc > 2 ? std::atoi(argv[2]) : 300;
    hsflow::Pool pool(6);
    std::vector<std::thread> th;
    std::vector<int> bad(callers, 0);
    for (int c = 0; c < callers; ++c) {
        th.emplace_back([&, c] {
            for (int r = 0; r < rounds; ++r) {
                const int n = 1 + (r * 7 + c) % 24;
                std::vector<int> hit(n, 0);  // each item writes only its own slot
                pool.run(n, [&](int i) { hit[i] += 1 + i; });
                for (int i = 0; i < n; ++i) bad[c] += hit[i] != 1 + i;
                // the process-wide singleton too (what the library uses)
                std::vector<long> sum(3, 0);
                hsflow::Pool::get().run(3, [&](int i) { sum[i] = (long)i * r; });
                bad[c] += sum[2] != 2L * r;
            }
        });
    }
    for (auto &t : th) t.join();
    int nbad = 0;
    for (int b : bad) nbad += b;
    std::printf("pool_tsan: %d callers x %d rounds, %d wrong items\n", callers, rounds, nbad);
    return nbad == 0 ? 0 : 1;
}
