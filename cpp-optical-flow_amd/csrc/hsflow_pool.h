// hsflow_pool.h -- the host copy pool of the host-buffer entry points
// (hsflow_hostio.cpp): plain C++ with no HIP types, so a CPU-only
// ThreadSanitizer test (tests/cpp/pool_tsan.cpp) hammers the same class.
#pragma once
#include <algorithm>
#include <atomic>
#include <condition_variable>
#include <functional>
#include <mutex>
#include <thread>
#include <vector>

namespace hsflow {

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
    // nt threads in all (the caller included); the singleton takes
    // min(8, hardware threads)
    explicit Pool(int nt) {
        for (int t = 1; t < nt; ++t) workers_.emplace_back([this] { loop(); });
    }
    // a pool other than the (leaked) singleton stops and joins its workers;
    // no job may be running
    ~Pool() {
        {
            std::lock_guard<std::mutex> g(mu_);
            stop_ = true;
        }
        cv_.notify_all();
        for (auto &w : workers_) w.join();
    }
    Pool(const Pool &) = delete;
    Pool &operator=(const Pool &) = delete;
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
    // the GPU boxes give each GPU a 16-core share; 8 threads saturate the
    // page-fault and memory-write rate of the widening
    Pool() : Pool(default_width()) {}
    static int default_width() {
        unsigned hw = std::thread::hardware_concurrency();
        return (int)std::min<unsigned>(8u, hw ? hw : 1u);
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
                cv_.wait(g, [&] { return gen_ != seen || stop_; });
                if (stop_) return;
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
    bool stop_ = false;
};

}  // namespace hsflow
