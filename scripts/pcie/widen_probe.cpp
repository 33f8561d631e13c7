// Host-side f32 -> f64 widening throughput of the getFlow download (the
// pool of hsflow_hostio.cpp) against thread count, thread placement over the
// box's L3 domains and store type.  One 1080p pair: 2 x 2 Mpx of f32 from a
// pinned stage into warm pageable f64 rows.  Median of 15 per variant.
//   hipcc -O2 -o widen_probe scripts/pcie/widen_probe.cpp -lpthread
#include <hip/hip_runtime.h>
#include <immintrin.h>
#include <pthread.h>
#include <sched.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <map>
#include <string>
#include <thread>
#include <vector>

static double now_ms() {
    return std::chrono::duration<double, std::milli>(
               std::chrono::steady_clock::now().time_since_epoch())
        .count();
}

__attribute__((target("avx2"))) static void widen_nt(const float *s, double *d, size_t n) {
    size_t x = 0;
    for (; x < n && (reinterpret_cast<uintptr_t>(d + x) & 31) != 0; ++x) d[x] = s[x];
    for (; x + 8 <= n; x += 8) {
        _mm256_stream_pd(d + x, _mm256_cvtps_pd(_mm_loadu_ps(s + x)));
        _mm256_stream_pd(d + x + 4, _mm256_cvtps_pd(_mm_loadu_ps(s + x + 4)));
    }
    for (; x < n; ++x) d[x] = s[x];
    _mm_sfence();
}
__attribute__((target("avx2"))) static void widen_cached(const float *s, double *d, size_t n) {
    size_t x = 0;
    for (; x + 8 <= n; x += 8) {
        _mm256_storeu_pd(d + x, _mm256_cvtps_pd(_mm_loadu_ps(s + x)));
        _mm256_storeu_pd(d + x + 4, _mm256_cvtps_pd(_mm_loadu_ps(s + x + 4)));
    }
    for (; x < n; ++x) d[x] = s[x];
}

// persistent spinning workers: start flag per round, done counter
struct Team {
    std::vector<std::thread> th;
    std::atomic<int> round{0}, done{0};
    std::atomic<bool> quit{false};
    int nt = 0;
    bool nt_store = true;
    const float *src = nullptr;
    double *dst = nullptr;
    size_t n = 0;
    void slice(int t) {
        const size_t a = n * t / nt, b = n * (t + 1) / nt;
        if (nt_store)
            widen_nt(src + a, dst + a, b - a);
        else
            widen_cached(src + a, dst + a, b - a);
    }
    Team(int nthreads, const std::vector<int> &cpus) : nt(nthreads) {
        for (int t = 1; t < nt; ++t)
            th.emplace_back([this, t, cpus] {
                if (!cpus.empty()) {
                    cpu_set_t cs;
                    CPU_ZERO(&cs);
                    CPU_SET(cpus[t % cpus.size()], &cs);
                    pthread_setaffinity_np(pthread_self(), sizeof(cs), &cs);
                }
                int seen = 0;
                for (;;) {
                    int r;
                    while ((r = round.load(std::memory_order_acquire)) == seen) {
                        if (quit.load()) return;
                        _mm_pause();
                    }
                    seen = r;
                    slice(t);
                    done.fetch_add(1, std::memory_order_acq_rel);
                }
            });
        if (!cpus.empty()) {
            cpu_set_t cs;
            CPU_ZERO(&cs);
            CPU_SET(cpus[0], &cs);
            pthread_setaffinity_np(pthread_self(), sizeof(cs), &cs);
        }
    }
    void run() {
        done.store(0);
        round.fetch_add(1, std::memory_order_acq_rel);
        slice(0);
        while (done.load(std::memory_order_acquire) < nt - 1) _mm_pause();
    }
    ~Team() {
        quit = true;
        for (auto &t : th) t.join();
    }
};

static std::string read_line(const std::string &p) {
    std::ifstream f(p);
    std::string s;
    std::getline(f, s);
    return s;
}

int main() {
    setvbuf(stdout, nullptr, _IOLBF, 0);
    cpu_set_t all;
    sched_getaffinity(0, sizeof(all), &all);
    std::vector<int> allowed;
    for (int c = 0; c < CPU_SETSIZE; ++c)
        if (CPU_ISSET(c, &all)) allowed.push_back(c);
    // L3 domain and physical core of every allowed cpu
    std::map<std::string, std::vector<int>> l3;
    std::map<std::string, int> core_seen;
    std::vector<int> first_thread;  // one hardware thread per physical core
    for (int c : allowed) {
        const std::string base = "/sys/devices/system/cpu/cpu" + std::to_string(c);
        const std::string sib = read_line(base + "/topology/thread_siblings_list");
        if (core_seen.count(sib)) continue;
        core_seen[sib] = c;
        first_thread.push_back(c);
        l3[read_line(base + "/cache/index3/shared_cpu_list")].push_back(c);
    }
    std::printf("allowed cpus %zu, physical cores %zu, L3 domains %zu (cores per domain:",
                allowed.size(), first_thread.size(), l3.size());
    for (auto &kv : l3) std::printf(" %zu", kv.second.size());
    std::printf(")\n");
    // spread: round robin over the L3 domains; packed: fill one domain first
    std::vector<int> spread, packed;
    for (size_t i = 0;; ++i) {
        bool any = false;
        for (auto &kv : l3)
            if (i < kv.second.size()) {
                spread.push_back(kv.second[i]);
                any = true;
            }
        if (!any) break;
    }
    for (auto &kv : l3)
        for (int c : kv.second) packed.push_back(c);

    const size_t n = 2ull * 1080 * 1920;
    float *src;
    bool pinned = hipHostMalloc((void **)&src, n * 4, hipHostMallocDefault) == hipSuccess;
    if (!pinned) src = (float *)aligned_alloc(4096, n * 4);  // no GPU: pageable stage
    std::printf("stage: %s\n", pinned ? "pinned (hipHostMalloc)" : "pageable (no GPU)");
    for (size_t i = 0; i < n; ++i) src[i] = (float)(i % 977) * 0.25f;
    std::vector<double> dst(n, 0.0);
    const double mb = (n * 4 + n * 8) / 1e6;

    struct Placement {
        const char *name;
        const std::vector<int> *cpus;
    } places[] = {{"unpinned", nullptr}, {"spread over L3", &spread}, {"packed in L3", &packed}};
    for (bool nt_store : {true, false})
        for (auto &pl : places)
            for (int nt : {4, 8, 12, 16, 24}) {
                if (pl.cpus && (size_t)nt > pl.cpus->size()) continue;
                sched_setaffinity(0, sizeof(all), &all);
                Team team(nt, pl.cpus ? *pl.cpus : std::vector<int>{});
                team.nt_store = nt_store;
                team.src = src;
                team.dst = dst.data();
                team.n = n;
                team.run();
                std::vector<double> t;
                for (int i = 0; i < 15; ++i) {
                    double a = now_ms();
                    team.run();
                    t.push_back(now_ms() - a);
                }
                std::sort(t.begin(), t.end());
                std::printf("%-7s %-15s %2d threads  %.3f ms  %.1f GB/s\n",
                            nt_store ? "nt" : "cached", pl.name, nt, t[7], mb / t[7]);
            }
    if (pinned) (void)hipHostFree(src);
    return 0;
}
