// hsflow_hostio.cpp -- host side of the host-buffer entry points (hsflow_flow,
// hsflow_gradients, hsflow_flow_bgr, hsflow_flow_pyramid): the path the
// cv::Mat drop-in takes for main.cpp:97-98 (frames in pageable host memory,
// u and v back as CV_64FC1, hornSchunck.cpp:49-50, 72-73).
//
// Both directions go through the context's pinned stage in row chunks, so
// the DMA engines and the host threads work at the same time:
//   upload    pool threads copy the caller's rows into the stage chunk by
//             chunk; each chunk's H2D copy is queued as soon as its rows
//             are staged (the runtime's own pageable path stages through a
//             single thread);
//   download  every chunk of every plane is queued at once as a pitched DMA
//             copy (the runtime gives pitched device -> pinned copies its
//             DMA engines: ~46 GB/s against ~29 GB/s flat,
//             scripts/pcie/d2h_engine_probe.hip) with an event behind it;
//             pool threads widen f32 -> f64 (or copy f32) chunk k into the
//             caller's rows as soon as its event has fired, while later
//             chunks are still in flight.
// Only the last chunk's widening is left after the last DMA copy.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <condition_variable>
#include <cstring>
#include <functional>
#include <mutex>
#include <thread>
#include <vector>

#include "hsflow_internal.h"

namespace hsflow {

namespace {

// A fixed set of worker threads for the host-side copies, created on first
// use and never destroyed (they sleep on a condition variable between
// jobs; a leaked singleton has no static-destruction hazards at exit).  One
// job at a time: a call that finds the pool busy (another host thread's
// solve, e.g. hsflow_flow_multi's per-device workers) runs its job inline.
class Pool {
public:
    static Pool &get() {
        static Pool *p = new Pool();
        return *p;
    }
    int width() const { return (int)workers_.size() + 1; }

    // fn(i) for i in [0, n), on the workers and the calling thread
    void run(int n, const std::function<void(int)> &fn) {
        if (n <= 0) return;
        std::unique_lock<std::mutex> busy(job_mu_, std::try_to_lock);
        if (!busy.owns_lock() || workers_.empty() || n == 1) {
            for (int i = 0; i < n; ++i) fn(i);
            return;
        }
        Job job{&fn, n};
        {
            std::lock_guard<std::mutex> g(mu_);
            job_ = &job;
            ++gen_;
        }
        cv_.notify_all();
        work(job);
        // every item claimed: wait for the ones still running and for every
        // worker to let go of the job before it leaves this frame
        std::unique_lock<std::mutex> g(mu_);
        done_cv_.wait(g, [&] { return job.done.load() == n && job.refs == 0; });
        job_ = nullptr;
    }

private:
    struct Job {
        const std::function<void(int)> *fn;
        int n;
        std::atomic<int> next{0}, done{0};
        int refs = 0;  // workers holding the job (guarded by mu_)
    };
    Pool() {
        unsigned hw = std::thread::hardware_concurrency();
        // the GPU boxes give each GPU a 16-core share; 8 threads saturate the
        // page-fault and memory-write rate of the widening
        const int nt = (int)std::min<unsigned>(8u, hw ? hw : 1u);
        for (int t = 1; t < nt; ++t) workers_.emplace_back([this] { loop(); });
        for (auto &w : workers_) w.detach();
    }
    static void work(Job &j) {
        for (int i = j.next.fetch_add(1); i < j.n; i = j.next.fetch_add(1)) {
            (*j.fn)(i);
            j.done.fetch_add(1);
        }
    }
    void loop() {
        unsigned long seen = 0;
        for (;;) {
            Job *j = nullptr;
            {
                std::unique_lock<std::mutex> g(mu_);
                cv_.wait(g, [&] { return gen_ != seen; });
                seen = gen_;
                j = job_;
                if (!j) continue;
                ++j->refs;
            }
            work(*j);
            {
                std::lock_guard<std::mutex> g(mu_);
                --j->refs;
            }
            done_cv_.notify_all();
        }
    }

    std::vector<std::thread> workers_;
    std::mutex job_mu_;  // one job at a time
    std::mutex mu_;
    std::condition_variable cv_, done_cv_;
    Job *job_ = nullptr;
    unsigned long gen_ = 0;
};

// rows per chunk: ~256 K pixels (1 MB of f32), at most 32 chunks per plane
int chunk_rows(int rows, int cols) {
    const long px = 256L * 1024;
    int r = (int)std::max<long>(1, px / std::max(1, cols));
    r = std::max(r, (rows + 31) / 32);
    return std::min(r, rows);
}

}  // namespace

int host_pool_width() { return Pool::get().width(); }

hipError_t upload_frames(const void *const *src, const size_t *step, int n, int rows, int cols,
                         int elem, void *const *dst, char *stage, hipStream_t s) {
    const size_t row_bytes = (size_t)cols * elem;
    const int cr = chunk_rows(rows, cols);
    const int per = (rows + cr - 1) / cr;
    std::atomic<int> err{(int)hipSuccess};
    Pool::get().run(n * per, [&](int i) {
        const int k = i / per, c = i % per;
        const int r0 = c * cr, r1 = std::min(rows, r0 + cr);
        char *st = stage + (size_t)k * rows * row_bytes + (size_t)r0 * row_bytes;
        const char *sp = (const char *)src[k] + (size_t)r0 * step[k];
        if (step[k] == row_bytes) {
            std::memcpy(st, sp, (size_t)(r1 - r0) * row_bytes);
        } else {
            for (int r = r0; r < r1; ++r)
                std::memcpy(st + (size_t)(r - r0) * row_bytes, sp + (size_t)(r - r0) * step[k],
                            row_bytes);
        }
        hipError_t e = hipMemcpyAsync((char *)dst[k] + (size_t)r0 * row_bytes, st,
                                      (size_t)(r1 - r0) * row_bytes, hipMemcpyHostToDevice, s);
        if (e != hipSuccess) err.store((int)e);
    });
    return (hipError_t)err.load();
}

hipError_t download_planes_pipelined(const float *const *src, void *const *dst, int n, int rows,
                                     int cols, bool f64, size_t step, float *stage,
                                     std::vector<hipEvent_t> &events, hipStream_t s) {
    const int cr = chunk_rows(rows, cols);
    const int per = (rows + cr - 1) / cr;
    const int total = n * per;
    while ((int)events.size() < total) {
        hipEvent_t ev;
        hipError_t e = hipEventCreateWithFlags(&ev, hipEventDisableTiming);
        if (e != hipSuccess) return e;
        events.push_back(ev);
    }
    const size_t plane = (size_t)rows * cols;
    const size_t row_bytes = (size_t)cols * 4;
    // every chunk's DMA copy first, in plane-major order (the order the
    // widening consumes them)
    for (int i = 0; i < total; ++i) {
        const int k = i / per, c = i % per;
        const int r0 = c * cr, r1 = std::min(rows, r0 + cr);
        hipError_t e = hipMemcpy2DAsync(stage + k * plane + (size_t)r0 * cols, row_bytes,
                                        src[k] + (size_t)r0 * cols, row_bytes, row_bytes,
                                        (size_t)(r1 - r0), hipMemcpyDeviceToHost, s);
        if (e == hipSuccess) e = hipEventRecord(events[i], s);
        if (e != hipSuccess) return e;
    }
    std::atomic<int> err{(int)hipSuccess};
    Pool::get().run(total, [&](int i) {
        hipError_t e = hipEventSynchronize(events[i]);
        if (e != hipSuccess) {
            err.store((int)e);
            return;
        }
        const int k = i / per, c = i % per;
        const int r0 = c * cr, r1 = std::min(rows, r0 + cr);
        const float *sp = stage + k * plane;
        for (int r = r0; r < r1; ++r) {
            const float *row = sp + (size_t)r * cols;
            char *d = (char *)dst[k] + (size_t)r * step;
            if (f64) {
                double *dd = (double *)d;
                for (int x = 0; x < cols; ++x) dd[x] = (double)row[x];
            } else {
                std::memcpy(d, row, row_bytes);
            }
        }
    });
    if (err.load() != (int)hipSuccess) return (hipError_t)err.load();
    // the stream is idle now (the last event fired): later work may reuse the stage
    return hipSuccess;
}

}  // namespace hsflow
