// The f64 download of the getFlow path (hsflow_hostio.cpp
// download_planes_pipelined) in variants: how the host threads learn that a
// chunk has landed (hipEventSynchronize / polling hipEventQuery), how they
// are woken (condition variable per call / spinning for the call), chunks per
// plane, store type.  One pair of f32 planes on the device -> pageable f64
// rows (warm, reused as cv::Mat::create keeps them).  Median of 21.
//   hipcc -O2 -o dl_probe scripts/pcie/dl_probe.cpp -lpthread
//   ./dl_probe [rows cols]
#include <hip/hip_runtime.h>
#include <immintrin.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <cstdio>
#include <cstdlib>
#include <functional>
#include <mutex>
#include <thread>
#include <vector>

#define CK(x)                                                               \
    do {                                                                    \
        hipError_t e_ = (x);                                                \
        if (e_ != hipSuccess) {                                             \
            std::printf("%s: %s\n", #x, hipGetErrorString(e_));             \
            std::exit(1);                                                   \
        }                                                                   \
    } while (0)

static double now_ms() {
    return std::chrono::duration<double, std::milli>(
               std::chrono::steady_clock::now().time_since_epoch())
        .count();
}

__attribute__((target("avx2"))) static void widen(const float *s, double *d, size_t n, bool nt) {
    size_t x = 0;
    if (nt) {
        for (; x < n && (reinterpret_cast<uintptr_t>(d + x) & 31) != 0; ++x) d[x] = s[x];
        for (; x + 8 <= n; x += 8) {
            _mm256_stream_pd(d + x, _mm256_cvtps_pd(_mm_loadu_ps(s + x)));
            _mm256_stream_pd(d + x + 4, _mm256_cvtps_pd(_mm_loadu_ps(s + x + 4)));
        }
        for (; x < n; ++x) d[x] = s[x];
        _mm_sfence();
    } else {
        for (; x + 8 <= n; x += 8) {
            _mm256_storeu_pd(d + x, _mm256_cvtps_pd(_mm_loadu_ps(s + x)));
            _mm256_storeu_pd(d + x + 4, _mm256_cvtps_pd(_mm_loadu_ps(s + x + 4)));
        }
        for (; x < n; ++x) d[x] = s[x];
    }
}

// Workers: sleep on a condition variable between calls; `spin` keeps them
// polling an atomic job counter for the call instead (woken at the call's
// start, before the copies are enqueued).
struct Pool {
    std::vector<std::thread> th;
    std::mutex mu;
    std::condition_variable cv;
    std::atomic<unsigned> gen{0};
    std::atomic<int> next{0}, done{0}, active{0};
    const std::function<void(int)> *fn = nullptr;
    std::atomic<int> n{0};
    std::atomic<bool> armed{false};
    explicit Pool(int nt) {
        for (int t = 1; t < nt; ++t)
            th.emplace_back([this] {
                unsigned seen = 0;
                for (;;) {
                    {
                        std::unique_lock<std::mutex> g(mu);
                        cv.wait(g, [&] { return gen.load() != seen; });
                        seen = gen.load();
                    }
                    // wait (spinning) until the job is published, then work
                    while (!armed.load(std::memory_order_acquire)) _mm_pause();
                    active.fetch_add(1);
                    work();
                    active.fetch_sub(1);
                }
            });
        for (auto &t : th) t.detach();
    }
    void wake() {  // the call starts: workers leave their sleep now
        {
            std::lock_guard<std::mutex> g(mu);
            gen.fetch_add(1);
        }
        cv.notify_all();
    }
    void work() {
        for (int i = next.fetch_add(1); i < n.load(); i = next.fetch_add(1)) {
            (*fn)(i);
            done.fetch_add(1);
        }
    }
    void run(int items, const std::function<void(int)> &f) {
        fn = &f;
        next = 0;
        done = 0;
        n = items;
        armed.store(true, std::memory_order_release);
        work();
        while (done.load() < items) _mm_pause();
        armed.store(false, std::memory_order_release);
        while (active.load() != 0) _mm_pause();
    }
};

int main(int argc, char **argv) {
    setvbuf(stdout, nullptr, _IOLBF, 0);
    const int rows = argc > 1 ? atoi(argv[1]) : 1080, cols = argc > 2 ? atoi(argv[2]) : 1920;
    const size_t plane = (size_t)rows * cols, rb = (size_t)cols * 4;
    hipStream_t s;
    CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    float *dU;
    CK(hipMalloc(&dU, 2 * plane * 4));
    CK(hipMemset(dU, 0, 2 * plane * 4));
    float *stage;
    CK(hipHostMalloc((void **)&stage, 2 * plane * 4, hipHostMallocDefault));
    std::vector<double> u(plane, 1.0), v(plane, 1.0);
    double *dst[2] = {u.data(), v.data()};
    std::vector<hipEvent_t> ev(64);
    for (auto &e : ev) CK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
    Pool &pool = *new Pool(8);  // leaked: its detached workers sleep on its
                                // condition variable until the process ends

    auto med = [](const std::function<void()> &f) {
        f();
        f();
        std::vector<double> t;
        for (int i = 0; i < 21; ++i) {
            double a = now_ms();
            f();
            t.push_back(now_ms() - a);
        }
        std::sort(t.begin(), t.end());
        return t[10];
    };
    std::printf("%dx%d, f64 outputs of two f32 planes\n", cols, rows);
    std::printf("D2H f32 only, 1 copy per plane                     %.3f ms\n", med([&] {
        for (int k = 0; k < 2; ++k)
            CK(hipMemcpy2DAsync(stage + k * plane, rb, dU + k * plane, rb, rb, rows,
                                hipMemcpyDeviceToHost, s));
        CK(hipStreamSynchronize(s));
    }));
    // the widening alone, from a stage the DMA has just written (cold in the
    // host caches), all 8 threads
    for (bool nt : {true, false}) {
        std::vector<double> t;
        for (int i = 0; i < 21; ++i) {
            for (int k = 0; k < 2; ++k)
                CK(hipMemcpy2DAsync(stage + k * plane, rb, dU + k * plane, rb, rb, rows,
                                    hipMemcpyDeviceToHost, s));
            CK(hipStreamSynchronize(s));
            pool.wake();
            for (double w = now_ms(); now_ms() - w < 0.3;) _mm_pause();  // workers up
            double a = now_ms();
            pool.run(16, [&](int item) {
                const int k = item / 8, sl = item % 8;
                const size_t q0 = plane * sl / 8, q1 = plane * (sl + 1) / 8;
                widen(stage + k * plane + q0, dst[k] + q0, q1 - q0, nt);
            });
            t.push_back(now_ms() - a);
        }
        std::sort(t.begin(), t.end());
        std::printf("widen alone after the DMA, 8 threads, %-6s          %.3f ms\n",
                    nt ? "nt" : "cached", t[10]);
    }
    // the D2H while the 8 threads widen a second (host) copy of the planes
    {
        std::vector<float> other(2 * plane, 0.5f);
        std::vector<double> t;
        for (int i = 0; i < 21; ++i) {
            pool.wake();
            double a = now_ms(), d2h = 0;
            for (int k = 0; k < 2; ++k)
                CK(hipMemcpy2DAsync(stage + k * plane, rb, dU + k * plane, rb, rb, rows,
                                    hipMemcpyDeviceToHost, s));
            CK(hipEventRecord(ev[0], s));
            std::atomic<bool> landed{false};
            pool.run(16, [&](int item) {
                if (item == 0) {  // one thread times the copy and then widens too
                    CK(hipEventSynchronize(ev[0]));
                    d2h = now_ms() - a;
                    landed = true;
                }
                const int k = item / 8, sl = item % 8;
                const size_t q0 = plane * sl / 8, q1 = plane * (sl + 1) / 8;
                for (int rep = 0; rep < 3 && !landed.load(); ++rep)
                    widen(other.data() + k * plane + q0, dst[k] + q0, q1 - q0, true);
            });
            t.push_back(d2h);
        }
        std::sort(t.begin(), t.end());
        std::printf("D2H f32 while the threads widen other host data        %.3f ms\n", t[10]);
    }
    // timeline of one variant (2 chunks per plane, polling, nt): when each
    // chunk is seen landed and when its last slice is widened, from the
    // call's start; the run with the median total
    {
        const int chunks = 2, slices = 8, cr = (rows + chunks - 1) / chunks;
        const int per = (rows + cr - 1) / cr, total = 2 * per;
        std::vector<std::vector<double>> runs;
        for (int it = 0; it < 23; ++it) {
            std::vector<std::atomic<double>> seen(total), wdone(total);
            std::vector<std::atomic<int>> left(total);
            for (int i = 0; i < total; ++i) {
                seen[i] = 0;
                left[i] = slices;
            }
            pool.wake();
            const double a = now_ms();
            for (int i = 0; i < total; ++i) {
                const int k = i / per, c = i % per;
                const int r0 = c * cr, r1 = std::min(rows, r0 + cr);
                CK(hipMemcpy2DAsync(stage + k * plane + (size_t)r0 * cols, rb,
                                    dU + k * plane + (size_t)r0 * cols, rb, rb, r1 - r0,
                                    hipMemcpyDeviceToHost, s));
                CK(hipEventRecord(ev[i], s));
            }
            const double issued = now_ms() - a;
            pool.run(total * slices, [&](int item) {
                const int i = item / slices, sl = item % slices;
                hipError_t q;
                while ((q = hipEventQuery(ev[i])) == hipErrorNotReady) _mm_pause();
                CK(q);
                double z = 0;
                seen[i].compare_exchange_strong(z, now_ms() - a);
                const int k = i / per, c = i % per;
                const int r0 = c * cr, r1 = std::min(rows, r0 + cr), h = r1 - r0;
                const int q0 = r0 + h * sl / slices, q1 = r0 + h * (sl + 1) / slices;
                widen(stage + k * plane + (size_t)q0 * cols, dst[k] + (size_t)q0 * cols,
                      (size_t)(q1 - q0) * cols, true);
                if (left[i].fetch_sub(1) == 1) wdone[i] = now_ms() - a;
            });
            std::vector<double> r{now_ms() - a, issued};
            for (int i = 0; i < total; ++i) {
                r.push_back(seen[i]);
                r.push_back(wdone[i]);
            }
            runs.push_back(r);
        }
        std::sort(runs.begin(), runs.end());
        const auto &r = runs[11];
        std::printf("timeline (2 chunks/plane, poll, nt): total %.3f ms, copies issued by %.3f\n",
                    r[0], r[1]);
        for (int i = 0; i < total; ++i)
            std::printf("  chunk %d: landed %.3f  widened %.3f\n", i, r[2 + 2 * i], r[3 + 2 * i]);
    }
    // uneven chunks: fractions of each plane's rows, largest first (the
    // threads widen ~1.3x faster than the copies land, so a chunk may be
    // 0.75x its predecessor and the exposed tail is the last chunk's
    // widening); 1-D copies (the stage rows are contiguous) or pitched ones
    {
        struct Split {
            const char *name;
            std::vector<double> fu, fv;
        } splits[] = {{"u 1 | v .6 .4", {1.0}, {0.6, 0.4}},
                      {"u 1 | v .75 .25", {1.0}, {0.75, 0.25}},
                      {"u 1 | v .5 .3 .2", {1.0}, {0.5, 0.3, 0.2}},
                      {"u .5 .5 | v .5 .3 .2", {0.5, 0.5}, {0.5, 0.3, 0.2}},
                      {"u .6 .4 | v .55 .3 .15", {0.6, 0.4}, {0.55, 0.3, 0.15}},
                      {"u .5 .5 | v .5 .5 (even)", {0.5, 0.5}, {0.5, 0.5}}};
        for (auto &sp : splits)
            for (bool one_d : {true, false}) {
                struct Chunk {
                    int k, r0, r1, slices;
                };
                std::vector<Chunk> ch;
                for (int k = 0; k < 2; ++k) {
                    const auto &f = k ? sp.fv : sp.fu;
                    double acc = 0;
                    int r0 = 0;
                    for (size_t j = 0; j < f.size(); ++j) {
                        acc += f[j];
                        const int r1 = j + 1 == f.size() ? rows : (int)(rows * acc + 0.5);
                        ch.push_back({k, r0, r1, std::max(2, (int)(16 * f[j] + 0.5))});
                        r0 = r1;
                    }
                }
                std::vector<int> first(ch.size() + 1, 0);
                for (size_t i = 0; i < ch.size(); ++i) first[i + 1] = first[i] + ch[i].slices;
                const double ms = med([&] {
                    pool.wake();
                    for (size_t i = 0; i < ch.size(); ++i) {
                        const auto &c = ch[i];
                        float *d = stage + c.k * plane + (size_t)c.r0 * cols;
                        const float *sp_ = dU + c.k * plane + (size_t)c.r0 * cols;
                        if (one_d)
                            CK(hipMemcpyAsync(d, sp_, (size_t)(c.r1 - c.r0) * rb,
                                              hipMemcpyDeviceToHost, s));
                        else
                            CK(hipMemcpy2DAsync(d, rb, sp_, rb, rb, c.r1 - c.r0,
                                                hipMemcpyDeviceToHost, s));
                        CK(hipEventRecord(ev[i], s));
                    }
                    pool.run(first.back(), [&](int item) {
                        const int i = (int)(std::upper_bound(first.begin(), first.end(), item) -
                                            first.begin()) - 1;
                        const int sl = item - first[i];
                        const auto &c = ch[i];
                        hipError_t q;
                        while ((q = hipEventQuery(ev[i])) == hipErrorNotReady) _mm_pause();
                        CK(q);
                        const int h = c.r1 - c.r0;
                        const int q0 = c.r0 + h * sl / c.slices, q1 = c.r0 + h * (sl + 1) / c.slices;
                        widen(stage + c.k * plane + (size_t)q0 * cols,
                              dst[c.k] + (size_t)q0 * cols, (size_t)(q1 - q0) * cols, true);
                    });
                });
                std::printf("split %-26s %s copies, poll, nt  %.3f ms\n", sp.name,
                            one_d ? "1-D" : "2-D", ms);
            }
    }
    for (int chunks : {2, 3, 4, 6})
        for (int wait_mode = 0; wait_mode < 2; ++wait_mode)
            for (int slices : {8, 16})
                for (bool nt : {true, false}) {
                    if (slices == 16 && (wait_mode == 0 || !nt)) continue;
                    const int cr = (rows + chunks - 1) / chunks;
                    const int per = (rows + cr - 1) / cr, total = 2 * per;
                    const double ms = med([&] {
                        pool.wake();
                        for (int i = 0; i < total; ++i) {
                            const int k = i / per, c = i % per;
                            const int r0 = c * cr, r1 = std::min(rows, r0 + cr);
                            CK(hipMemcpy2DAsync(stage + k * plane + (size_t)r0 * cols, rb,
                                                dU + k * plane + (size_t)r0 * cols, rb, rb,
                                                r1 - r0, hipMemcpyDeviceToHost, s));
                            CK(hipEventRecord(ev[i], s));
                        }
                        pool.run(total * slices, [&](int item) {
                            const int i = item / slices, sl = item % slices;
                            if (wait_mode == 0) {
                                CK(hipEventSynchronize(ev[i]));
                            } else {
                                hipError_t q;
                                while ((q = hipEventQuery(ev[i])) == hipErrorNotReady) _mm_pause();
                                CK(q);
                            }
                            const int k = i / per, c = i % per;
                            const int r0 = c * cr, r1 = std::min(rows, r0 + cr), h = r1 - r0;
                            const int q0 = r0 + h * sl / slices, q1 = r0 + h * (sl + 1) / slices;
                            widen(stage + k * plane + (size_t)q0 * cols,
                                  dst[k] + (size_t)q0 * cols, (size_t)(q1 - q0) * cols, nt);
                        });
                    });
                    std::printf("%d chunks/plane, %-19s %2d slices, %-6s  %.3f ms\n", chunks,
                                wait_mode ? "poll hipEventQuery" : "hipEventSynchronize", slices,
                                nt ? "nt" : "cached", ms);
                }
    return 0;
}
