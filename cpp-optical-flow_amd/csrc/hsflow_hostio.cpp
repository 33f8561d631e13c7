// hsflow_hostio.cpp -- host side of the host-buffer entry points (hsflow_flow,
// hsflow_gradients, hsflow_flow_bgr, hsflow_flow_pyramid): the path the
// cv::Mat drop-in takes for main.cpp:97-98 (frames in pageable host memory,
// u and v back as CV_64FC1, hornSchunck.cpp:49-50, 72-73).
//
// Measured phase costs of a 1080p pair (profiles/r04_hostio_probe.txt,
// scripts/pcie/hostio_probe.cpp): the runtime's own pageable H2D of the two
// u8 frames 0.09 ms (staging them through a pinned buffer first: 0.16 ms);
// the D2H of the two f32 planes 0.31 ms, pageable or pinned alike; widening
// them to f64 on the host 1.73 ms on one thread, 0.44 ms on eight.  So the
// frames go up as they are, f32 results come down straight into the
// caller's rows, and only f64 (CV_64FC1, the reference's output type) goes
// through the pinned stage: the planes come down in row chunks with an event
// behind each, and the whole pool widens chunk k while chunks k+1.. are
// still in flight; only the last chunk's widening follows the last copy.
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
#include "hsflow_pool.h"

#include <sys/mman.h>

#if defined(__x86_64__)
#include <immintrin.h>
#endif



namespace hsflow {

namespace {

// f32 -> f64 of one row.  x86-64 with AVX2: 4 floats widened per instruction
// and written with non-temporal stores (the destination is written once and
// not read back here, so the stores skip the read-for-ownership of each
// line); ends with a store fence, so the rows are visible to the thread that
// waits for the pool.  Elsewhere a plain loop.
#if defined(__x86_64__)
__attribute__((target("avx2"))) void widen_row_avx2(const float *src, double *dst, int n) {
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

void widen_rows(const float *src, size_t src_pitch, char *dst, size_t step, int r0, int r1,
                int cols) {
#if defined(__x86_64__)
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
// So: advise huge pages over the whole 2 MB extents of each plane's row
// span (advice only: no byte changes, and memory already resident keeps its
// pages), then let the pool touch one byte per page inside the rows (bytes
// the call overwrites) while the device solve runs.
void advise_hugepages(char *base, size_t step, size_t row_bytes, int rows) {
    if (rows <= 0) return;
    const uintptr_t hp = (uintptr_t)2 << 20;
    const uintptr_t a = ((uintptr_t)base + hp - 1) & ~(hp - 1);
    const uintptr_t e = ((uintptr_t)(base + (size_t)(rows - 1) * step + row_bytes)) & ~(hp - 1);
    if (e > a) (void)madvise((void *)a, e - a, MADV_HUGEPAGE);
}

void prefault_rows(char *base, size_t step, size_t row_bytes, int r0, int r1) {
    const uintptr_t pg = 4096;
    for (int r = r0; r < r1; ++r) {
        char *row = base + (size_t)r * step;
        for (size_t o = 0; o < row_bytes;) {
            *(volatile char *)(row + o) = 0;
            o = (((uintptr_t)(row + o)) | (pg - 1)) + 1 - (uintptr_t)row;
        }
    }
}

}  // namespace

int host_pool_width() { return Pool::get().width(); }

hipError_t download_planes_pipelined(const float *const *src, void *const *dst, int n, int rows,
                                     int cols, bool f64, size_t step, float *stage,
                                     std::vector<hipEvent_t> &events, hipStream_t s) {
    const size_t row_bytes = (size_t)cols * 4;
    if (!f64) {
        // f32 rows need no host work: one pitched DMA copy per plane straight
        // into the caller's rows (pageable memory downloads as fast as pinned
        // here: 0.314 vs 0.311 ms for a 1080p pair, profiles/r04_hostio_probe.txt)
        for (int k = 0; k < n; ++k) {
            hipError_t e = hipMemcpy2DAsync(dst[k], step, src[k], row_bytes, row_bytes,
                                            (size_t)rows, hipMemcpyDeviceToHost, s);
            if (e != hipSuccess) return e;
        }
        return hipStreamSynchronize(s);
    }
    // f64: each plane in kChunks row chunks (more chunks cost more DMA setup
    // than they hide: 2 / 4 / 8 / 16 chunks per plane 0.354 / 0.407 / 0.522 /
    // 0.767 ms against 0.311 ms in one copy, same probe), every chunk widened
    // by ALL pool threads as soon as it has landed (cached stores: one thread
    // widens a 1080p pair at ~19 GB/s of writes, eight at ~110 GB/s; the
    // non-temporal stores of widen_rows skip the destination's line reads)
    constexpr int kChunks = 2, kSlices = 8;
    const int cr = (rows + kChunks - 1) / kChunks;
    const int per = (rows + cr - 1) / cr;
    const int total = n * per;
    while ((int)events.size() < total) {
        hipEvent_t ev;
        hipError_t e = hipEventCreateWithFlags(&ev, hipEventDisableTiming);
        if (e != hipSuccess) return e;
        events.push_back(ev);
    }
    const size_t plane = (size_t)rows * cols;
    for (int i = 0; i < total; ++i) {
        const int k = i / per, c = i % per;
        const int r0 = c * cr, r1 = std::min(rows, r0 + cr);
        hipError_t e = hipMemcpy2DAsync(stage + k * plane + (size_t)r0 * cols, row_bytes,
                                        src[k] + (size_t)r0 * cols, row_bytes, row_bytes,
                                        (size_t)(r1 - r0), hipMemcpyDeviceToHost, s);
        if (e == hipSuccess) e = hipEventRecord(events[i], s);
        if (e != hipSuccess) return e;
    }
    // work items: first the destination's pages, faulted in while the
    // solve still runs (a caller's fresh output -- main.cpp:93 declares
    // `cv::Mat u, v;` anew for every getFlow -- would otherwise take its
    // first-touch faults in the widening after the last copy: 6 ms of a
    // 4K call), then the chunks in order, kSlices row slices each: the
    // pool's threads all wait for chunk 0, widen it together, then chunk 1
    std::atomic<int> err{(int)hipSuccess};
    for (int k = 0; k < n; ++k) advise_hugepages((char *)dst[k], step, (size_t)cols * 8, rows);
    constexpr int kFault = 8;  // slices per plane
    const int nfault = n * kFault;
    Pool::get().run(nfault + total * kSlices, [&](int item) {
        if (item < nfault) {
            const int k = item / kFault, sl = item % kFault;
            prefault_rows((char *)dst[k], step, (size_t)cols * 8, rows * sl / kFault,
                          rows * (sl + 1) / kFault);
            return;
        }
        item -= nfault;
        const int i = item / kSlices, sl = item % kSlices;
        hipError_t e = hipEventSynchronize(events[i]);
        if (e != hipSuccess) {
            err.store((int)e);
            return;
        }
        const int k = i / per, c = i % per;
        const int r0 = c * cr, r1 = std::min(rows, r0 + cr);
        const int h = r1 - r0, q0 = r0 + h * sl / kSlices, q1 = r0 + h * (sl + 1) / kSlices;
        widen_rows(stage + k * plane, (size_t)cols, (char *)dst[k], step, q0, q1, cols);
    });
    return (hipError_t)err.load();
}

}  // namespace hsflow
