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

#include <atomic>
#include <vector>

#include "hsflow_internal.h"
#include "hsflow_pool.h"
#include "hsflow_widen.h"

namespace hsflow {

std::atomic<int> g_output_hugepages{1};  // hsflow_set_output_hugepages

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
    constexpr int kChunks = 2;
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
    // the host half (hsflow_widen.h): the destination's pages faulted in
    // while the solve still runs (a caller's fresh output -- main.cpp:93
    // declares `cv::Mat u, v;` anew for every getFlow -- would otherwise
    // take its first-touch faults in the widening after the last copy: 6 ms
    // of a 4K call), then every chunk widened by the whole pool as soon as
    // its copy has landed
    const int e = fault_then_widen(
        Pool::get(), stage, dst, n, rows, cols, step, cr, per,
        [&](int i) { return (int)hipEventSynchronize(events[i]); }, true,
        g_output_hugepages.load(std::memory_order_relaxed) != 0);
    return (hipError_t)e;
}

}  // namespace hsflow
