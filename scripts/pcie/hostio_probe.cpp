// Phase costs of the host-buffer path (hsflow_flow) for one 1080p pair:
// upload of two u8 frames, download of two f32 planes, f32 -> f64 widening,
// each in the variants the library could use.  Median of 15 per variant.
//   hipcc -O2 -o hostio_probe scripts/pcie/hostio_probe.cpp -lpthread
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <atomic>
#include <condition_variable>
#include <functional>
#include <immintrin.h>
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

static double med(const std::function<void()> &f, int n = 15) {
    f();
    std::vector<double> t;
    for (int i = 0; i < n; ++i) {
        double a = now_ms();
        f();
        t.push_back(now_ms() - a);
    }
    std::sort(t.begin(), t.end());
    return t[n / 2];
}

static void par(int nt, int n, const std::function<void(int)> &fn) {
    std::vector<std::thread> th;
    for (int t = 0; t < nt; ++t)
        th.emplace_back([&, t] {
            for (int i = t; i < n; i += nt) fn(i);
        });
    for (auto &x : th) x.join();
}

// persistent workers (the library's pool has the same shape): run(n, fn)
// hands items 0..n-1 to the 7 workers and the caller
struct Pool {
    std::vector<std::thread> th;
    std::mutex mu;
    std::condition_variable cv, dcv;
    const std::function<void(int)> *fn = nullptr;
    int n = 0, busy = 0;
    std::atomic<int> next{0}, done{0};
    unsigned long gen = 0;
    explicit Pool(int nt) {
        for (int t = 1; t < nt; ++t)
            th.emplace_back([this] {
                unsigned long seen = 0;
                for (;;) {
                    {
                        std::unique_lock<std::mutex> g(mu);
                        cv.wait(g, [&] { return gen != seen; });
                        seen = gen;
                        ++busy;
                    }
                    work();
                    {
                        std::lock_guard<std::mutex> g(mu);
                        --busy;
                    }
                    dcv.notify_all();
                }
            });
        for (auto &t : th) t.detach();
    }
    void work() {
        for (int i = next.fetch_add(1); i < n; i = next.fetch_add(1)) {
            (*fn)(i);
            done.fetch_add(1);
        }
    }
    void run(int items, const std::function<void(int)> &f) {
        {
            std::lock_guard<std::mutex> g(mu);
            fn = &f;
            n = items;
            next = 0;
            done = 0;
            ++gen;
        }
        cv.notify_all();
        work();
        std::unique_lock<std::mutex> g(mu);
        dcv.wait(g, [&] { return done.load() == n && busy == 0; });
    }
};

__attribute__((target("avx2"))) static void widen_row(const float *s, double *d, int n) {
    int x = 0;
    for (; x < n && (reinterpret_cast<uintptr_t>(d + x) & 31) != 0; ++x) d[x] = s[x];
    for (; x + 8 <= n; x += 8) {
        _mm256_stream_pd(d + x, _mm256_cvtps_pd(_mm_loadu_ps(s + x)));
        _mm256_stream_pd(d + x + 4, _mm256_cvtps_pd(_mm_loadu_ps(s + x + 4)));
    }
    for (; x < n; ++x) d[x] = s[x];
}

int main(int argc, char **argv) {
    setvbuf(stdout, nullptr, _IOLBF, 0);
    const int rows = argc > 1 ? atoi(argv[1]) : 1080, cols = argc > 2 ? atoi(argv[2]) : 1920;
    const size_t n = (size_t)rows * cols;
    hipStream_t s;
    CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    std::vector<uint8_t> f0(n, 1), f1(n, 2);  // pageable frames
    std::vector<double> u(n), v(n);            // pageable outputs (warm)
    std::memset(u.data(), 0, n * 8);
    std::memset(v.data(), 0, n * 8);
    uint8_t *dI;
    float *dU;
    CK(hipMalloc(&dI, 2 * n));
    CK(hipMalloc(&dU, 2 * n * 4));
    CK(hipMemset(dU, 0, 2 * n * 4));
    char *pin;
    CK(hipHostMalloc((void **)&pin, 2 * n + 2 * n * 4 + 4096, hipHostMallocDefault));
    float *pst = (float *)(pin + ((2 * n + 4095) / 4096) * 4096);
    std::vector<float> pagef(2 * n);
    std::vector<hipEvent_t> ev(64);
    for (auto &e : ev) CK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
    hipEvent_t evb;
    CK(hipEventCreateWithFlags(&evb, hipEventDisableTiming | hipEventBlockingSync));

    std::printf("%dx%d\n", cols, rows);
    // ---- uploads
    std::printf("up pageable 2x hipMemcpyAsync        %.3f ms\n", med([&] {
        CK(hipMemcpyAsync(dI, f0.data(), n, hipMemcpyHostToDevice, s));
        CK(hipMemcpyAsync(dI + n, f1.data(), n, hipMemcpyHostToDevice, s));
        CK(hipStreamSynchronize(s));
    }));
    std::printf("up memcpy->pinned (1 thr) + 1 H2D      %.3f ms\n", med([&] {
        std::memcpy(pin, f0.data(), n);
        std::memcpy(pin + n, f1.data(), n);
        CK(hipMemcpyAsync(dI, pin, 2 * n, hipMemcpyHostToDevice, s));
        CK(hipStreamSynchronize(s));
    }));
    std::printf("up memcpy->pinned (8 thr) + 1 H2D      %.3f ms\n", med([&] {
        par(8, 16, [&](int i) {
            size_t c = 2 * n / 16;
            std::memcpy(pin + i * c, (i < 8 ? f0.data() : f1.data()) + (i % 8) * c, c);
        });
        CK(hipMemcpyAsync(dI, pin, 2 * n, hipMemcpyHostToDevice, s));
        CK(hipStreamSynchronize(s));
    }));
    std::printf("up pinned H2D only (1 call)            %.3f ms\n", med([&] {
        CK(hipMemcpyAsync(dI, pin, 2 * n, hipMemcpyHostToDevice, s));
        CK(hipStreamSynchronize(s));
    }));
    std::printf("up pinned H2D 16 chunks                %.3f ms\n", med([&] {
        size_t c = 2 * n / 16;
        for (int i = 0; i < 16; ++i)
            CK(hipMemcpyAsync(dI + i * c, pin + i * c, c, hipMemcpyHostToDevice, s));
        CK(hipStreamSynchronize(s));
    }));
    // ---- downloads (2 planes, f32)
    const size_t rb = (size_t)cols * 4;
    std::printf("down flat 2x hipMemcpyAsync -> pinned  %.3f ms\n", med([&] {
        CK(hipMemcpyAsync(pst, dU, n * 4, hipMemcpyDeviceToHost, s));
        CK(hipMemcpyAsync(pst + n, dU + n, n * 4, hipMemcpyDeviceToHost, s));
        CK(hipStreamSynchronize(s));
    }));
    std::printf("down pitched 2x 2D -> pinned           %.3f ms\n", med([&] {
        CK(hipMemcpy2DAsync(pst, rb, dU, rb, rb, rows, hipMemcpyDeviceToHost, s));
        CK(hipMemcpy2DAsync(pst + n, rb, dU + n, rb, rb, rows, hipMemcpyDeviceToHost, s));
        CK(hipStreamSynchronize(s));
    }));
    std::printf("down pitched 1x 2D both planes         %.3f ms\n", med([&] {
        CK(hipMemcpy2DAsync(pst, rb, dU, rb, rb, 2 * rows, hipMemcpyDeviceToHost, s));
        CK(hipStreamSynchronize(s));
    }));
    for (int per : {2, 4, 8, 16}) {
        int cr = (rows + per - 1) / per;
        std::printf("down pitched %2d chunks/plane + events  %.3f ms\n", per, med([&] {
            int k = 0;
            for (int p = 0; p < 2; ++p)
                for (int r0 = 0; r0 < rows; r0 += cr, ++k) {
                    int h = std::min(cr, rows - r0);
                    CK(hipMemcpy2DAsync(pst + p * n + (size_t)r0 * cols, rb,
                                        dU + p * n + (size_t)r0 * cols, rb, rb, h,
                                        hipMemcpyDeviceToHost, s));
                    CK(hipEventRecord(ev[k], s));
                }
            CK(hipEventSynchronize(ev[k - 1]));
        }));
    }
    hipStream_t s2;
    CK(hipStreamCreateWithFlags(&s2, hipStreamNonBlocking));
    std::printf("down 2 planes on 2 streams -> pinned   %.3f ms\n", med([&] {
        CK(hipMemcpy2DAsync(pst, rb, dU, rb, rb, rows, hipMemcpyDeviceToHost, s));
        CK(hipMemcpy2DAsync(pst + n, rb, dU + n, rb, rb, rows, hipMemcpyDeviceToHost, s2));
        CK(hipStreamSynchronize(s));
        CK(hipStreamSynchronize(s2));
    }));
    std::printf("down 2 planes on 2 streams -> pageable %.3f ms\n", med([&] {
        CK(hipMemcpy2DAsync(pagef.data(), rb, dU, rb, rb, rows, hipMemcpyDeviceToHost, s));
        CK(hipMemcpy2DAsync(pagef.data() + n, rb, dU + n, rb, rb, rows, hipMemcpyDeviceToHost,
                            s2));
        CK(hipStreamSynchronize(s));
        CK(hipStreamSynchronize(s2));
    }));
    std::printf("up pageable 2 frames on 2 streams      %.3f ms\n", med([&] {
        CK(hipMemcpyAsync(dI, f0.data(), n, hipMemcpyHostToDevice, s));
        CK(hipMemcpyAsync(dI + n, f1.data(), n, hipMemcpyHostToDevice, s2));
        CK(hipStreamSynchronize(s));
        CK(hipStreamSynchronize(s2));
    }));
    std::printf("down flat 2x -> pageable f32           %.3f ms\n", med([&] {
        CK(hipMemcpyAsync(pagef.data(), dU, n * 4, hipMemcpyDeviceToHost, s));
        CK(hipMemcpyAsync(pagef.data() + n, dU + n, n * 4, hipMemcpyDeviceToHost, s));
        CK(hipStreamSynchronize(s));
    }));
    // ---- sync latency
    std::printf("event sync (empty stream, default)     %.3f ms\n", med([&] {
        CK(hipEventRecord(ev[0], s));
        CK(hipEventSynchronize(ev[0]));
    }));
    std::printf("event sync (empty stream, blocking)    %.3f ms\n", med([&] {
        CK(hipEventRecord(evb, s));
        CK(hipEventSynchronize(evb));
    }));
    std::printf("stream sync (empty)                    %.3f ms\n",
                med([&] { CK(hipStreamSynchronize(s)); }));
    // ---- widening (warm output pages)
    for (int nt : {1, 2, 4, 8, 16}) {
        std::printf("widen f32->f64 2 planes, %2d threads    %.3f ms\n", nt, med([&] {
            par(nt, 64, [&](int i) {
                size_t c = 2 * n / 64, a = i * c;
                for (size_t x = a; x < a + c; ++x) {
                    if (x < n)
                        u[x] = pst[x];
                    else
                        v[x - n] = pst[x];
                }
            });
        }));
    }
    // ---- f64 outputs: CPU-widened f32 head rows + GPU-widened f64 tail rows
    // (the f64 tail comes from a device buffer; its widening kernel is a few
    // microseconds and not timed here)
    double *dD;
    CK(hipMalloc(&dD, 2 * n * 8));
    CK(hipMemset(dD, 0, 2 * n * 8));
    Pool &pool = *new Pool(8);  // leaked: destroying a condition variable
                                // its detached waiters sleep on blocks
    for (int pct : {0, 30, 40, 50, 60, 100}) {
        const int tail = rows * pct / 100, head = rows - tail, cr = (head + 1) / 2;
        std::printf("down f64 %3d%% rows GPU-widened, rest 2 chunks + pool  %.3f ms\n", pct,
                    med([&] {
            int k = 0;
            for (int p = 0; p < 2; ++p)
                for (int r0 = 0; r0 < head; r0 += cr, ++k) {
                    int h = std::min(cr, head - r0);
                    CK(hipMemcpyAsync(pst + p * n + (size_t)r0 * cols, dU + p * n + (size_t)r0 * cols,
                                      (size_t)h * rb, hipMemcpyDeviceToHost, s));
                    CK(hipEventRecord(ev[k], s));
                }
            for (int p = 0; p < 2 && tail > 0; ++p)
                CK(hipMemcpyAsync((p ? v.data() : u.data()) + (size_t)head * cols,
                                  dD + p * n + (size_t)head * cols, (size_t)tail * cols * 8,
                                  hipMemcpyDeviceToHost, s));
            CK(hipEventRecord(ev[k], s));
            const int nk = k;
            if (nk > 0)
                pool.run(nk * 8, [&](int item) {
                    const int i = item / 8, sl = item % 8, p = i / ((head + cr - 1) / cr),
                              c = i % ((head + cr - 1) / cr);
                    const int r0 = c * cr, r1 = std::min(head, r0 + cr), hh = r1 - r0;
                    CK(hipEventSynchronize(ev[i]));
                    for (int r = r0 + hh * sl / 8; r < r0 + hh * (sl + 1) / 8; ++r)
                        widen_row(pst + p * n + (size_t)r * cols,
                                  (p ? v.data() : u.data()) + (size_t)r * cols, cols);
                });
            _mm_sfence();
            CK(hipEventSynchronize(ev[nk]));
        }));
    }
    std::printf("thread spawn+join x7                   %.3f ms\n",
                med([&] { par(7, 7, [](int) {}); }));
    return 0;
}
