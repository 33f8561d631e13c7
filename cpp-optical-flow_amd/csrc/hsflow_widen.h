// hsflow_widen.h -- host-side f32 -> f64 widening of downloaded (u, v) rows
// into the caller's CV_64FC1 planes (hornSchunck.cpp:49-50, 72-73 hand back
// f64), with the first-touch page faults of a fresh output taken beforehand.
// Plain C++ with no HIP types: hsflow_hostio.cpp drives it with an event
// wait per row chunk, and a CPU-only ThreadSanitizer test
// (tests/cpp/widen_tsan.cpp) drives the same code with a fake wait.
#pragma once
#include <algorithm>
#include <atomic>
#include <cstddef>
#include <cstdint>
#include <functional>

#include <sys/mman.h>

#if defined(__x86_64__)
#include <immintrin.h>
#endif

#include "hsflow_pool.h"

namespace hsflow {

// f32 -> f64 of one row.  x86-64 with AVX2: 4 floats widened per instruction
// and written with non-temporal stores (the destination is written once and
// not read back here, so the stores skip the read-for-ownership of each
// line).  Elsewhere a plain loop.
#if defined(__x86_64__)
__attribute__((target("avx2"))) inline void widen_row_avx2(const float *src, double *dst, int n) {
    int x = 0;
    for (; x < n && (reinterpret_cast<uintptr_t>(dst + x) & 31) != 0; ++x)
        dst[x] = (double)src[x];
    for (; x + 8 <= n; x += 8) {
        const __m256d a = _mm256_cvtps_pd(_mm_loadu_ps(src + x));
        const __m256d b = _mm256_cvtps_pd(_mm_loadu_ps(src + x + 4));
        _mm256_stream_pd(dst + x, a);
        _mm256_stream_pd(dst + x + 4, b);
    }
    for (; x < n; ++x) dst[x] = (double)src[x];
}
#endif

// rows [r0, r1); ends with a store fence, so the rows are visible to the
// thread that waits for the pool
inline void widen_rows(const float *src, size_t src_pitch, char *dst, size_t step, int r0, int r1,
                       int cols) {
#if defined(__x86_64__) && !defined(HSFLOW_PLAIN_WIDEN)
    static const bool avx2 = __builtin_cpu_supports("avx2");
    if (avx2) {
        for (int r = r0; r < r1; ++r)
            widen_row_avx2(src + (size_t)r * src_pitch, (double *)(dst + (size_t)r * step), cols);
        _mm_sfence();
        return;
    }
#endif
    for (int r = r0; r < r1; ++r) {
        const float *row = src + (size_t)r * src_pitch;
        double *d = (double *)(dst + (size_t)r * step);
        for (int x = 0; x < cols; ++x) d[x] = (double)row[x];
    }
}

// Fresh output planes (main.cpp:93 declares `cv::Mat u, v;` anew for every
// getFlow) take a first-touch page fault per 4 KB page.  Measured on the GPU
// box (scripts/pcie/fault_probe.cpp, profiles/r05_fault_probe.txt), for the
// 132 MB of a 4K pair's two f64 planes: touching every page 18.5 ms on one
// thread, 8-10 ms on 4-16 (the faults contend); MADV_POPULATE_WRITE 3.3 ms
// on 4 threads, 6.2 on 8; with MADV_HUGEPAGE first (THP is in `madvise`
// mode there) the same touches fault 2 MB pages: 1.1-1.4 ms on 8-16 threads.
// So huge pages are advised over the whole 2 MB extents inside each plane's
// row span.  The advice stays on the caller's allocation after the call
// (hsflow.h): it changes no byte, memory already resident
// keeps its pages, and hsflow_set_output_hugepages(0) turns it off.
inline void advise_hugepages(char *base, size_t step, size_t row_bytes, int rows) {
    if (rows <= 0) return;
    const uintptr_t hp = (uintptr_t)2 << 20;
    const uintptr_t a = ((uintptr_t)base + hp - 1) & ~(hp - 1);
    const uintptr_t e = ((uintptr_t)(base + (size_t)(rows - 1) * step + row_bytes)) & ~(hp - 1);
    if (e > a) (void)madvise((void *)a, e - a, MADV_HUGEPAGE);
}

// one byte per 4 KB page inside rows [r0, r1) set to 0 (bytes the call
// overwrites later): the page is faulted in writable
inline void prefault_rows(char *base, size_t step, size_t row_bytes, int r0, int r1) {
    const uintptr_t pg = 4096;
    for (int r = r0; r < r1; ++r) {
        char *row = base + (size_t)r * step;
        for (size_t o = 0; o < row_bytes;) {
            *(volatile char *)(row + o) = 0;
            o = (((uintptr_t)(row + o)) | (pg - 1)) + 1 - (uintptr_t)row;
        }
    }
}

// The host half of an f64 download: n planes of rows x cols f32 in `stage`
// (plane k at stage + k rows cols), landing in `per` row chunks of `cr` rows
// each; wait(i) returns 0 once chunk i (plane i / per, chunk i % per) has
// landed, else an error code that the call returns.  Two pool jobs, in
// order: (1) the destination's pages, faulted in while the device work is
// still running; (2) the chunks in order, kSlices row slices each, every
// thread widening the chunk that has landed.  The fault job ends before the
// widening starts: a fault slice zeroes one byte per page of rows that a
// widening slice writes, so the two must never overlap in time (within one
// job items are claimed in order but finish in any order).  before_fault
// (tests only) runs ahead of each fault slice.
inline int fault_then_widen(Pool &pool, const float *stage, void *const *dst, int n, int rows,
                            int cols, size_t step, int cr, int per,
                            const std::function<int(int)> &wait, bool prefault = true,
                            bool advise = true,
                            const std::function<void(int)> &before_fault = nullptr) {
    constexpr int kSlices = 8, kFault = 8;
    const size_t plane = (size_t)rows * cols;
    const int total = n * per;
    if (prefault) {
        if (advise)
            for (int k = 0; k < n; ++k)
                advise_hugepages((char *)dst[k], step, (size_t)cols * 8, rows);
        pool.run(n * kFault, [&](int item) {
            const int k = item / kFault, sl = item % kFault;
            if (before_fault) before_fault(item);  // tests: a slow pre-touch
            prefault_rows((char *)dst[k], step, (size_t)cols * 8, rows * sl / kFault,
                          rows * (sl + 1) / kFault);
        });
    }
    std::atomic<int> err{0};
    pool.run(total * kSlices, [&](int item) {
        const int i = item / kSlices, sl = item % kSlices;
        const int e = wait(i);
        if (e != 0) {
            err.store(e);
            return;
        }
        const int k = i / per, c = i % per;
        const int r0 = c * cr, r1 = std::min(rows, r0 + cr);
        const int h = r1 - r0, q0 = r0 + h * sl / kSlices, q1 = r0 + h * (sl + 1) / kSlices;
        widen_rows(stage + k * plane, (size_t)cols, (char *)dst[k], step, q0, q1, cols);
    });
    return err.load();
}

}  // namespace hsflow
