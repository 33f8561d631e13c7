// hsflow_api.cpp -- the C ABI declared in include/hsflow.h.
//
// Host side of the drop-in boundary for HornSchunckOF/hornSchunck.cpp:
//   getFlow      (hornSchunck.cpp:43-75) -> hsflow_flow / hsflow_flow_device
//   getGradients (hornSchunck.cpp:19-41) -> hsflow_gradients / *_device
// Context = device + stream + grow-only device buffers, so repeated getFlow
// calls on same-size frames (main.cpp:97-98 in a loop) never reallocate.

#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "../../include/hsflow.h"
#include "hsflow_internal.h"

using hsflow::JacobiArgs;

struct hsflow_ctx {
    int device = 0;
    hipStream_t stream = nullptr;
    std::string err;
    // device buffers (grow-only)
    void *d_in = nullptr;
    size_t d_in_bytes = 0;  // holds I0 and I1
    void *d_out = nullptr;
    size_t d_out_bytes = 0;  // holds u, v (or gx, gy, gt)
    void *d_ws = nullptr;
    size_t d_ws_bytes = 0;
    // pinned host staging of f32 planes on their way to f64 rows
    char *h_stage = nullptr;
    size_t h_stage_bytes = 0;
    // one event per downloaded row chunk (created on first use)
    std::vector<hipEvent_t> dl_ev;
};

namespace {

thread_local std::string g_err;  // errors from calls without a context
int g_kb_override = 0;
// Jacobi pass kernel (hsflow_set_jacobi_kernel): 0 = automatic (K4 strips
// where built, else K2), 2 = K2 tiles everywhere, 4 = K4 where built
int g_kernel_override = 0;
// K4 rows per segment (hsflow_set_strip_rows): 0 = automatic
int g_strip_rows = 0;


// Kernel and blocking depth of a launch's passes.  K4 (streaming strips)
// runs the full-depth passes when it is built for the window's default
// depth and -- automatic choice -- its waves fill the chip (launches too
// small for it keep K2's tiles, whose depth adapts to the fill);
// hsflow_set_jacobi_kernel(4) forces it wherever it is built.
struct PassPlan {
    int kb;
    bool strip;
};

// K4's depth: the caller's (hsflow_set_iters_per_launch) or the window's default
int strip_kb(int window) {
    return g_kb_override > 0 ? g_kb_override : hsflow::default_kb(window);
}

bool strip_use(int window, int rows, int cols, int batch) {
    const int kb = strip_kb(window);
    if (g_kernel_override == 2 || window > 9 || !hsflow::strip_supported(window, kb)) return false;
    if (g_kernel_override == 4) return true;
    return rows > 0 && cols > 0 && batch > 0 &&
           hsflow::strip_fills(window, kb, rows, cols, batch, 8 * hsflow::device_cus());
}

int fail(hsflow_ctx *ctx, int code, const char *fmt, ...) {
    char buf[512];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof buf, fmt, ap);
    va_end(ap);
    if (ctx)
        ctx->err = buf;
    else
        g_err = buf;
    return code;
}

int hip_fail(hsflow_ctx *ctx, hipError_t e, const char *what) {
    return fail(ctx, e == hipErrorOutOfMemory ? HSFLOW_ERR_OOM : HSFLOW_ERR_HIP,
                "%s: %s (%d)", what, hipGetErrorString(e), (int)e);
}

#define HIP_TRY(ctx, expr)                                    \
    do {                                                      \
        hipError_t e_ = (expr);                               \
        if (e_ != hipSuccess) return hip_fail(ctx, e_, #expr); \
    } while (0)

constexpr size_t kAlign = 256;
size_t align_up(size_t x) { return (x + kAlign - 1) / kAlign * kAlign; }

// Largest frame: plane bytes must fit the 31-bit buffer offsets of K2.
constexpr long long kMaxPlanePixels = (1ll << 29) - 1;

// Largest batch: pairs index gridDim.y / gridDim.z of the kernels (65535);
// tallest plane: the 64 x 4 per-pixel kernels put rows / 4 in gridDim.y.
constexpr int kMaxBatch = 65535;
constexpr int kMaxRows = 4 * 65535;

bool sizes_ok(int rows, int cols, int batch) {
    return rows >= 1 && rows <= kMaxRows && cols >= 1 && batch >= 1 &&
           batch <= kMaxBatch && (long long)rows * cols <= kMaxPlanePixels;
}

struct Workspace {
    uint32_t *gpack;
    float *gx, *gy, *gt, *u2, *v2;
    uint32_t *flags;
    size_t bytes;
};

Workspace carve(void *base, int rows, int cols, int batch) {
    const size_t n = (size_t)rows * cols * batch;
    Workspace w{};
    size_t off = 0;
    auto take = [&](size_t bytes) {
        size_t o = off;
        off = align_up(off + bytes);
        return (char *)base + o;
    };
    w.gpack = (uint32_t *)take(n * 4);
    w.gx = (float *)take(n * 4);
    w.gy = (float *)take(n * 4);
    w.gt = (float *)take(n * 4);
    w.u2 = (float *)take(n * 4);
    w.v2 = (float *)take(n * 4);
    w.flags = (uint32_t *)take((size_t)batch * 4);
    w.bytes = off;
    return w;
}

int elem_size(int dtype) {
    switch (dtype) {
    case HSFLOW_U8: return 1;
    case HSFLOW_F32: return 4;
    case HSFLOW_F64: return 8;
    case HSFLOW_F16: return 2;
    default: return 0;
    }
}

// element size of the device copy of a host input (every input type is
// uploaded as it is: K1 reads u8, f16, f32 and f64 frames)
int dev_elem_size(int dtype) { return elem_size(dtype); }

bool device_dtype_ok(int dtype) {
    return dtype == HSFLOW_U8 || dtype == HSFLOW_F32 || dtype == HSFLOW_F16 ||
           dtype == HSFLOW_F64;
}

// `batch`: every pair in flight at once (the whole batch, also when it is
// split over side streams); 0 = shape unknown (no fill adjustment)
PassPlan plan_passes(int window, bool need_f32, int rows = 0, int cols = 0, int batch = 0) {
    if (window > 9) return {1, false};
    if (strip_use(window, rows, cols, batch)) return {strip_kb(window), true};
    if (g_kb_override > 0 && hsflow::kb_supported(window, g_kb_override, need_f32))
        return {g_kb_override, false};
    int kb = hsflow::fill_kb(window, hsflow::default_kb(window), rows, cols, batch);
    while (kb > 1 && !hsflow::kb_supported(window, kb, need_f32)) kb /= 2;
    return {kb, false};
}

int pick_kb(int window, bool need_f32, int rows = 0, int cols = 0, int batch = 0) {
    return plan_passes(window, need_f32, rows, cols, batch).kb;
}

// Per-thread, per-device side streams for splitting a batch: each sub-batch
// runs its Jacobi passes on its own stream, so the launches of the two halves
// overlap (one's tail and boundary with the other's work).  Default 2 halves:
// same-box bench, 1080p x 8 / 4K x 2 Mpix*iter/s: 1 stream 905k / 960k,
// 2 streams 967k / 1034k, 4 streams 901k / 1033k, 8 streams 865k / 1032k
// (scripts/streams_ab.sh).  Fork and join are event based (capturable into a
// hipGraph).  Never destroyed: they live until the process exits (no
// static-destruction-order hazards).
// The *_device entry points run on the device their stream belongs to
// (the current device for the null stream), whatever device the calling
// thread has current: side streams, the CU count and the launches all follow
// the caller's stream.
struct DeviceGuard {
    int prev = -1;
    explicit DeviceGuard(hipStream_t s) {
        int cur = 0;
        hipDevice_t d = 0;
        if (!s || hipGetDevice(&cur) != hipSuccess || hipStreamGetDevice(s, &d) != hipSuccess)
            return;
        if (d != cur && hipSetDevice(d) == hipSuccess) prev = cur;
    }
    ~DeviceGuard() {
        if (prev >= 0) (void)hipSetDevice(prev);
    }
    DeviceGuard(const DeviceGuard &) = delete;
    DeviceGuard &operator=(const DeviceGuard &) = delete;
};

struct SidePool {
    int device = -1;
    std::vector<hipStream_t> streams;
    std::vector<hipEvent_t> events;  // [0] fork, [1..] joins
};

// hsflow_set_max_streams: 0 = automatic (split in 2 eagerly, not at all
// while the caller's stream is capturing), n >= 1 = up to n streams always
int g_split_override = 0;

// Streams a batch of `batch` pairs on `s` is split over.  Under stream
// capture the automatic choice does not split: a stream forked inside a
// capture from a capturing stream that is not the capture's origin crashes
// hipStreamEndCapture on ROCm 7.2 (profiles/r04_capture_crash.txt; legal in
// CUDA), and the library cannot tell an origin from a forked stream.  A
// caller that captures on the origin itself may ask for the split with
// hsflow_set_max_streams(n >= 2) (the bench's timed graphs do).
int split_for(int batch, hipStream_t s) {
    if (g_split_override > 0) return std::min(batch, g_split_override);
    if (batch < 2) return 1;
    hipStreamCaptureStatus st = hipStreamCaptureStatusNone;
    if (hipStreamIsCapturing(s, &st) != hipSuccess || st != hipStreamCaptureStatusNone) return 1;
    return 2;
}

SidePool *side_pool(int need) {
    // one pool per device and thread: a thread that alternates devices keeps
    // each device's streams (re-creating them per switch would leak them)
    thread_local std::vector<SidePool> pools;
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || dev < 0) return nullptr;
    if ((int)pools.size() <= dev) pools.resize(dev + 1);
    SidePool &pool = pools[dev];
    pool.device = dev;
    while ((int)pool.streams.size() < need) {
        hipStream_t st;
        if (hipStreamCreateWithFlags(&st, hipStreamNonBlocking) != hipSuccess) return nullptr;
        pool.streams.push_back(st);
    }
    while ((int)pool.events.size() < need + 1) {
        hipEvent_t ev;
        if (hipEventCreateWithFlags(&ev, hipEventDisableTiming) != hipSuccess) return nullptr;
        pool.events.push_back(ev);
    }
    return &pool;
}

int jacobi_one(hsflow_ctx *ctx, int rows, int cols, int batch, int window, int iters,
               float alpha, bool warm, bool maybe_f32, float *u, float *v,
               void *workspace, size_t ws_bytes, hipStream_t s);
int check_jacobi_args(hsflow_ctx *ctx, int rows, int cols, int batch, int window,
                      int iters, const float *u, const float *v, void *workspace,
                      size_t ws_bytes);
int jacobi_sub(hsflow_ctx *ctx, int rows, int cols, int nb, int first, int batch,
               int window, int iters, float alpha, bool warm, bool maybe_f32, float *u,
               float *v, const Workspace &w, hipStream_t s);

int jacobi_impl(hsflow_ctx *ctx, int rows, int cols, int batch, int window, int iters,
                float alpha, bool warm, bool maybe_f32, float *u, float *v,
                void *workspace, size_t ws_bytes, hipStream_t s) {
    int rc0 = check_jacobi_args(ctx, rows, cols, batch, window, iters, u, v, workspace,
                                ws_bytes);
    if (rc0) return rc0;
    const int split = split_for(batch, s);
    if (split <= 1 || iters == 0)
        return jacobi_one(ctx, rows, cols, batch, window, iters, alpha, warm, maybe_f32, u,
                          v, workspace, ws_bytes, s);
    Workspace w = carve(workspace, rows, cols, batch);
    SidePool *pool = side_pool(split);
    if (!pool)
        return jacobi_one(ctx, rows, cols, batch, window, iters, alpha, warm, maybe_f32, u,
                          v, workspace, ws_bytes, s);
    const size_t plane = (size_t)rows * cols;
    HIP_TRY(ctx, hipEventRecord(pool->events[0], s));
    int first = 0, forked = 0, rc = HSFLOW_OK;
    for (int k = 0; k < split && rc == HSFLOW_OK; ++k) {
        const int nb = batch / split + (k < batch % split ? 1 : 0);
        hipStream_t sk = pool->streams[k];
        hipError_t e = hipStreamWaitEvent(sk, pool->events[0], 0);
        if (e != hipSuccess) {
            rc = hip_fail(ctx, e, "hipStreamWaitEvent (fork)");
            break;
        }
        ++forked;
        // the sub-batch's slice of every workspace plane, as its own workspace
        rc = jacobi_sub(ctx, rows, cols, nb, first, batch, window, iters, alpha, warm,
                        maybe_f32, u + first * plane, v + first * plane, w, sk);
        first += nb;
    }
    // join every forked stream back, the error path included (a capture
    // must not be left with streams that never rejoin its origin)
    for (int k = 0; k < forked; ++k) {
        hipError_t e = hipEventRecord(pool->events[1 + k], pool->streams[k]);
        if (e == hipSuccess) e = hipStreamWaitEvent(s, pool->events[1 + k], 0);
        if (e != hipSuccess && rc == HSFLOW_OK) rc = hip_fail(ctx, e, "stream join");
    }
    return rc;
}

// The Jacobi passes of `batch` pairs whose workspace planes are `w` (a view
// that may start at any pair of a larger workspace).
int run_passes(hsflow_ctx *ctx, int rows, int cols, int batch, int window, int iters,
               float alpha, bool warm, bool maybe_f32, float *u, float *v,
               const Workspace &w, hipStream_t s, int fill_batch) {
    const size_t n = (size_t)rows * cols * batch;
    if (iters == 0) {
        // hornSchunck.cpp:49-50: the loop does not run, u = v = 0
        if (!warm) {
            HIP_TRY(ctx, hipMemsetAsync(u, 0, n * 4, s));
            HIP_TRY(ctx, hipMemsetAsync(v, 0, n * 4, s));
        }
        return HSFLOW_OK;
    }
    const PassPlan plan = plan_passes(window, maybe_f32, rows, cols, fill_batch);
    const int kb = plan.kb;
    const int passes = (iters + kb - 1) / kb;
    // K4 for the full-depth passes (two waves per SIMD: 8 per CU), K2 for a
    // shorter last pass -- identical bits either way
    const bool strip = plan.strip;
    // K4 segment height from every pair in flight (the halves of a split
    // batch run concurrently and share the chip's slots)
    int strip_rows = g_strip_rows;
    if (strip && strip_rows <= 0) {
        int nseg = 0, nstrips = 0;
        strip_rows = hsflow::strip_seg_rows(window, kb, rows, cols, fill_batch,
                                            8 * hsflow::device_cus(), &nseg, &nstrips, 0);
    }
    JacobiArgs a{};
    a.rows = rows;
    a.cols = cols;
    a.batch = batch;
    a.alpha2 = (float)((double)alpha * (double)alpha);  // pow(alpha, 2)
    a.inv_w2 = (float)(1.0 / ((double)window * (double)window));
    a.gpack = w.gpack;
    a.gx = w.gx;
    a.gy = w.gy;
    a.gt = w.gt;
    a.flags = w.flags;
    a.write_through =
        hsflow::fill_limited(window, kb, strip, rows, cols, fill_batch, strip_rows) ? 1 : 0;

    // pass p writes the caller's buffers iff (passes-1-p) is even, so the
    // last pass always lands in (u, v)
    auto dst_is_user = [&](int pass) { return ((passes - 1 - pass) & 1) == 0; };
    const float *src_u = nullptr, *src_v = nullptr;
    if (warm) {
        if (dst_is_user(0)) {  // would read and write (u, v) in one pass
            HIP_TRY(ctx, hipMemcpyAsync(w.u2, u, n * 4, hipMemcpyDeviceToDevice, s));
            HIP_TRY(ctx, hipMemcpyAsync(w.v2, v, n * 4, hipMemcpyDeviceToDevice, s));
            src_u = w.u2;
            src_v = w.v2;
        } else {
            src_u = u;
            src_v = v;
        }
    }
    int done = 0;
    for (int pass = 0; pass < passes; ++pass) {
        a.iters = std::min(kb, iters - done);
        a.u_in = src_u;
        a.v_in = src_v;
        a.u_out = dst_is_user(pass) ? u : w.u2;
        a.v_out = dst_is_user(pass) ? v : w.v2;
        // a K2 pass (a shorter last pass of a K4 solve) takes a depth K2 is
        // built for: any depth >= its iterations gives the same bits
        int kb2 = kb;
        if (!hsflow::kb_supported(window, kb2, maybe_f32)) {
            kb2 = a.iters;
            while (kb2 < 8 && !hsflow::kb_supported(window, kb2, maybe_f32)) ++kb2;
            if (!hsflow::kb_supported(window, kb2, maybe_f32))
                return fail(ctx, HSFLOW_ERR_ARG, "no K2 depth >= %d for window %d", a.iters,
                            window);
        }
        hipError_t e = (strip && a.iters == kb)
                           ? hsflow::launch_jacobi_strip(a, window, kb, strip_rows, s)
                           : hsflow::launch_jacobi(a, window, kb2, s);
        if (e != hipSuccess) return hip_fail(ctx, e, "jacobi launch");
        src_u = a.u_out;
        src_v = a.v_out;
        done += a.iters;
    }
    return HSFLOW_OK;
}

int check_jacobi_args(hsflow_ctx *ctx, int rows, int cols, int batch, int window,
                      int iters, const float *u, const float *v, void *workspace,
                      size_t ws_bytes) {
    if (!sizes_ok(rows, cols, batch))
        return fail(ctx, HSFLOW_ERR_ARG, "bad size %dx%d batch %d", rows, cols, batch);
    if (window < 1 || window > HSFLOW_MAX_WINDOW)
        return fail(ctx, HSFLOW_ERR_ARG, "windowSize %d outside [1, %d]", window,
                    HSFLOW_MAX_WINDOW);
    if (iters < 0) return fail(ctx, HSFLOW_ERR_ARG, "maxIterations %d < 0", iters);
    if (!u || !v || !workspace) return fail(ctx, HSFLOW_ERR_ARG, "null device pointer");
    if (ws_bytes < carve(workspace, rows, cols, batch).bytes)
        return fail(ctx, HSFLOW_ERR_ARG, "workspace %zu < %zu bytes", ws_bytes,
                    carve(workspace, rows, cols, batch).bytes);
    return HSFLOW_OK;
}

int jacobi_one(hsflow_ctx *ctx, int rows, int cols, int batch, int window, int iters,
               float alpha, bool warm, bool maybe_f32, float *u, float *v,
               void *workspace, size_t ws_bytes, hipStream_t s) {
    int rc = check_jacobi_args(ctx, rows, cols, batch, window, iters, u, v, workspace,
                               ws_bytes);
    if (rc) return rc;
    return run_passes(ctx, rows, cols, batch, window, iters, alpha, warm, maybe_f32, u, v,
                      carve(workspace, rows, cols, batch), s, batch);
}

// pairs [first, first + nb) of a `batch`-pair workspace w
int jacobi_sub(hsflow_ctx *ctx, int rows, int cols, int nb, int first, int batch,
               int window, int iters, float alpha, bool warm, bool maybe_f32, float *u,
               float *v, const Workspace &w, hipStream_t s) {
    const size_t off = (size_t)first * rows * cols;
    Workspace sub = w;
    sub.gpack = w.gpack + off;
    sub.gx = w.gx + off;
    sub.gy = w.gy + off;
    sub.gt = w.gt + off;
    sub.u2 = w.u2 + off;
    sub.v2 = w.v2 + off;
    sub.flags = w.flags + first;
    // the split's halves run concurrently: the depth is chosen for the batch
    return run_passes(ctx, rows, cols, nb, window, iters, alpha, warm, maybe_f32, u, v, sub,
                      s, batch);
}

int gradients_impl(hsflow_ctx *ctx, const void *I0, const void *I1, int dtype_in,
                   int rows, int cols, int batch, float *gx, float *gy, float *gt,
                   void *workspace, size_t ws_bytes, hipStream_t s) {
    if (!sizes_ok(rows, cols, batch))
        return fail(ctx, HSFLOW_ERR_ARG, "bad size %dx%d batch %d", rows, cols, batch);
    if (!device_dtype_ok(dtype_in))
        return fail(ctx, HSFLOW_ERR_ARG, "device input dtype must be U8, F16, F32 or F64");
    if (!I0 || !I1 || !workspace) return fail(ctx, HSFLOW_ERR_ARG, "null device pointer");
    Workspace w = carve(workspace, rows, cols, batch);
    if (ws_bytes < w.bytes)
        return fail(ctx, HSFLOW_ERR_ARG, "workspace %zu < %zu bytes", ws_bytes, w.bytes);
    // K1 stores 8-bit frames' flags itself (always 0); the others OR into zeros
    if (dtype_in != HSFLOW_U8) HIP_TRY(ctx, hipMemsetAsync(w.flags, 0, (size_t)batch * 4, s));
    // the f32 planes for every pair only when the caller takes them
    hipError_t e = hsflow::launch_gradients(I0, I1, dtype_in, rows, cols, batch, w.gpack,
                                            w.gx, w.gy, w.gt, w.flags, gx || gy || gt, s);
    if (e != hipSuccess) return hip_fail(ctx, e, "gradients launch");
    const size_t n = (size_t)rows * cols * batch;
    if (gx) HIP_TRY(ctx, hipMemcpyAsync(gx, w.gx, n * 4, hipMemcpyDeviceToDevice, s));
    if (gy) HIP_TRY(ctx, hipMemcpyAsync(gy, w.gy, n * 4, hipMemcpyDeviceToDevice, s));
    if (gt) HIP_TRY(ctx, hipMemcpyAsync(gt, w.gt, n * 4, hipMemcpyDeviceToDevice, s));
    return HSFLOW_OK;
}

int grow(hsflow_ctx *ctx, void **p, size_t *have, size_t need) {
    if (*have >= need) return HSFLOW_OK;
    if (*p) {
        HIP_TRY(ctx, hipStreamSynchronize(ctx->stream));
        HIP_TRY(ctx, hipFree(*p));
        *p = nullptr;
        *have = 0;
    }
    HIP_TRY(ctx, hipMalloc(p, need));
    *have = need;
    return HSFLOW_OK;
}

int grow_host(hsflow_ctx *ctx, size_t need) {
    if (ctx->h_stage_bytes >= need) return HSFLOW_OK;
    if (ctx->h_stage) {
        HIP_TRY(ctx, hipHostFree(ctx->h_stage));
        ctx->h_stage = nullptr;
        ctx->h_stage_bytes = 0;
    }
    HIP_TRY(ctx, hipHostMalloc((void **)&ctx->h_stage, need, hipHostMallocDefault));
    ctx->h_stage_bytes = need;
    return HSFLOW_OK;
}

// Two host frames (any supported dtype, any row steps) -> dense device rows
// of the same type (K1 takes the Sobel sums of CV_64FC1 frames in float64,
// as hornSchunck.cpp:23-28 do, and rounds each gradient to f32 once).  The
// runtime's own pageable upload is the fastest route measured
// (hsflow_hostio.cpp).
int upload_pair(hsflow_ctx *ctx, const void *I0, const void *I1, int elem, int rows, int cols,
                size_t step0, size_t step1, void *dst0, void *dst1) {
    const size_t rb = (size_t)cols * elem;
    HIP_TRY(ctx, hipMemcpy2DAsync(dst0, rb, I0, step0, rb, rows, hipMemcpyHostToDevice,
                                  ctx->stream));
    HIP_TRY(ctx, hipMemcpy2DAsync(dst1, rb, I1, step1, rb, rows, hipMemcpyHostToDevice,
                                  ctx->stream));
    return HSFLOW_OK;
}

// n dense device f32 planes -> host rows of dtype_out with step `step`
// (hsflow_hostio.cpp: f32 straight down, f64 through the pinned stage,
// widened by the host pool chunk by chunk as the copies land).
int download_planes(hsflow_ctx *ctx, const float *const *src, void *const *dst, int n,
                    int rows, int cols, int dtype_out, size_t step) {
    const bool f64 = dtype_out == HSFLOW_F64;
    if (f64) {
        int rc = grow_host(ctx, (size_t)n * rows * cols * 4);
        if (rc) return rc;
    }
    HIP_TRY(ctx, hsflow::download_planes_pipelined(src, dst, n, rows, cols, f64, step,
                                                   (float *)ctx->h_stage, ctx->dl_ev,
                                                   ctx->stream));
    return HSFLOW_OK;
}

int check_host_args(hsflow_ctx *ctx, const void *I0, const void *I1, int dtype_in,
                    int rows, int cols, size_t step0, size_t step1, int dtype_out,
                    size_t out_step) {
    if (!ctx) return HSFLOW_ERR_ARG;
    if (!I0 || !I1) return fail(ctx, HSFLOW_ERR_ARG, "null image");
    if (!sizes_ok(rows, cols, 1))
        return fail(ctx, HSFLOW_ERR_ARG, "bad size %dx%d", rows, cols);
    const int es = elem_size(dtype_in);
    if (!es) return fail(ctx, HSFLOW_ERR_ARG, "unsupported input dtype %d", dtype_in);
    if (step0 < (size_t)cols * es || step1 < (size_t)cols * es)
        return fail(ctx, HSFLOW_ERR_ARG, "input steps %zu, %zu < row bytes %zu", step0, step1,
                    (size_t)cols * es);
    if (dtype_out != HSFLOW_F32 && dtype_out != HSFLOW_F64)
        return fail(ctx, HSFLOW_ERR_ARG, "output dtype must be F32 or F64");
    if (out_step < (size_t)cols * elem_size(dtype_out))
        return fail(ctx, HSFLOW_ERR_ARG, "output step %zu < row bytes", out_step);
    return HSFLOW_OK;
}

// ---- config 5 pyramid ----------------------------------------------------
// Workspace: [Jacobi workspace of level 0][integrality flags][per level
// l >= 1: I0_l, I1_l, u_l, v_l (batch x level plane, f32)].  Coarser levels
// reuse the front of the level-0 Jacobi workspace.
struct PyrLayout {
    int levels;
    int R[HSFLOW_MAX_LEVELS], C[HSFLOW_MAX_LEVELS];
    size_t jac_bytes, flags_off;
    size_t off[HSFLOW_MAX_LEVELS][4];  // I0, I1, u, v of level l >= 1
    size_t bytes;
};

PyrLayout pyr_layout(int rows, int cols, int batch, int levels) {
    PyrLayout L{};
    L.levels = levels;
    L.R[0] = rows;
    L.C[0] = cols;
    for (int l = 1; l < levels; ++l) {
        L.R[l] = (L.R[l - 1] + 1) / 2;
        L.C[l] = (L.C[l - 1] + 1) / 2;
    }
    L.jac_bytes = carve(nullptr, rows, cols, batch).bytes;
    L.flags_off = L.jac_bytes;
    size_t off = align_up(L.flags_off + (size_t)batch * 4);
    for (int l = 1; l < levels; ++l) {
        const size_t plane = align_up((size_t)L.R[l] * L.C[l] * batch * 4);
        for (int k = 0; k < 4; ++k) {
            L.off[l][k] = off;
            off += plane;
        }
    }
    L.bytes = off;
    return L;
}

int pyramid_impl(hsflow_ctx *ctx, const void *I0, const void *I1, int dtype_in, int rows,
                 int cols, int batch, int levels, int window, int iters, float alpha,
                 float *u, float *v, void *ws, size_t ws_bytes, hipStream_t s) {
    if (levels < 1 || levels > HSFLOW_MAX_LEVELS)
        return fail(ctx, HSFLOW_ERR_ARG, "levels %d outside [1, %d]", levels,
                    HSFLOW_MAX_LEVELS);
    if (!sizes_ok(rows, cols, batch))
        return fail(ctx, HSFLOW_ERR_ARG, "bad size %dx%d batch %d", rows, cols, batch);
    if (!device_dtype_ok(dtype_in))
        return fail(ctx, HSFLOW_ERR_ARG, "device input dtype must be U8, F16, F32 or F64");
    if (!I0 || !I1 || !u || !v || !ws)
        return fail(ctx, HSFLOW_ERR_ARG, "null device pointer");
    const PyrLayout L = pyr_layout(rows, cols, batch, levels);
    if (ws_bytes < L.bytes)
        return fail(ctx, HSFLOW_ERR_ARG, "workspace %zu < %zu bytes", ws_bytes, L.bytes);
    const bool maybe_f32 = dtype_in != HSFLOW_U8;
    char *base = (char *)ws;
    int rc;
    if (levels > 1) {
        // integrality of each pair (K1's flag at level 0) decides the rounding
        // of every level; saved because each level's K1 rewrites the flags
        rc = gradients_impl(ctx, I0, I1, dtype_in, rows, cols, batch, nullptr, nullptr,
                            nullptr, ws, L.jac_bytes, s);
        if (rc) return rc;
        uint32_t *intf = (uint32_t *)(base + L.flags_off);
        HIP_TRY(ctx, hipMemcpyAsync(intf, carve(ws, rows, cols, batch).flags,
                                    (size_t)batch * 4, hipMemcpyDeviceToDevice, s));
        for (int l = 1; l < levels; ++l)
            for (int k = 0; k < 2; ++k) {
                const void *src = l == 1 ? (k ? I1 : I0) : base + L.off[l - 1][k];
                hipError_t e = hsflow::launch_pyrdown(
                    src, l == 1 ? dtype_in : HSFLOW_F32, L.R[l - 1], L.C[l - 1], batch,
                    (float *)(base + L.off[l][k]), intf, s);
                if (e != hipSuccess) return hip_fail(ctx, e, "pyrdown launch");
            }
    }
    for (int l = levels - 1; l >= 0; --l) {
        float *ul = l ? (float *)(base + L.off[l][2]) : u;
        float *vl = l ? (float *)(base + L.off[l][3]) : v;
        const bool warm = l < levels - 1;
        if (warm) {
            hipError_t e = hsflow::launch_upflow(
                (const float *)(base + L.off[l + 1][2]), (const float *)(base + L.off[l + 1][3]),
                L.R[l + 1], L.C[l + 1], ul, vl, L.R[l], L.C[l], batch, s);
            if (e != hipSuccess) return hip_fail(ctx, e, "upflow launch");
        }
        rc = gradients_impl(ctx, l ? (const void *)(base + L.off[l][0]) : I0,
                            l ? (const void *)(base + L.off[l][1]) : I1,
                            l ? HSFLOW_F32 : dtype_in, L.R[l], L.C[l], batch, nullptr,
                            nullptr, nullptr, ws, L.jac_bytes, s);
        if (rc) return rc;
        rc = jacobi_impl(ctx, L.R[l], L.C[l], batch, window, iters, alpha, warm, maybe_f32,
                         ul, vl, ws, L.jac_bytes, s);
        if (rc) return rc;
    }
    return HSFLOW_OK;
}

// hsflow_flow_multi's kept contexts: one per (device, slot), each behind its
// own lock (calls that list disjoint devices run concurrently); the registry
// lock only guards the table's shape.  Slots are never freed (stable
// pointers); hsflow_flow_multi_release destroys their contexts.
struct MultiSlot {
    std::mutex mu;
    hsflow_ctx *ctx = nullptr;
};
std::mutex g_multi_mu;
std::vector<std::vector<std::unique_ptr<MultiSlot>>> g_multi;  // [device][slot]

std::vector<MultiSlot *> multi_slots(const int *devices, int nw) {
    std::lock_guard<std::mutex> reg(g_multi_mu);
    std::vector<MultiSlot *> out(nw);
    for (int k = 0; k < nw; ++k) {
        int dup = 0;  // earlier workers on the same device
        for (int i = 0; i < k; ++i) dup += devices[i] == devices[k];
        if ((int)g_multi.size() <= devices[k]) g_multi.resize(devices[k] + 1);
        auto &dv = g_multi[devices[k]];
        while ((int)dv.size() <= dup) dv.push_back(std::make_unique<MultiSlot>());
        out[k] = dv[dup].get();
    }
    return out;
}

}  // namespace

extern "C" {

int hsflow_version(void) { return HSFLOW_VERSION; }

// No diagnostic build exists any more (the environment-honouring probe build
// of round 2 was retired with its switches); kept for ABI stability.
int hsflow_build_flags(void) { return 0; }

const char *hsflow_status_string(int status) {
    switch (status) {
    case HSFLOW_OK: return "ok";
    case HSFLOW_ERR_ARG: return "invalid argument";
    case HSFLOW_ERR_HIP: return "HIP runtime error";
    case HSFLOW_ERR_OOM: return "device out of memory";
    case HSFLOW_ERR_NODEV: return "no usable HIP device";
    case HSFLOW_ERR_SIZE: return "image sizes differ";
    default: return "unknown status";
    }
}

int hsflow_create(hsflow_ctx **out, int device) {
    if (!out) return fail(nullptr, HSFLOW_ERR_ARG, "null ctx pointer");
    *out = nullptr;
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess || n <= 0)
        return fail(nullptr, HSFLOW_ERR_NODEV, "no HIP device");
    if (device < 0 || device >= n)
        return fail(nullptr, HSFLOW_ERR_NODEV, "device %d of %d", device, n);
    hipDeviceProp_t prop;
    if (hipGetDeviceProperties(&prop, device) != hipSuccess)
        return fail(nullptr, HSFLOW_ERR_NODEV, "hipGetDeviceProperties failed");
    if (std::strncmp(prop.gcnArchName, "gfx950", 6) != 0)
        return fail(nullptr, HSFLOW_ERR_NODEV, "device %d is %s, libhsflow is built for gfx950",
                    device, prop.gcnArchName);
    hsflow_ctx *ctx = new hsflow_ctx();
    ctx->device = device;
    if (hipSetDevice(device) != hipSuccess ||
        hipStreamCreateWithFlags(&ctx->stream, hipStreamNonBlocking) != hipSuccess) {
        delete ctx;
        return fail(nullptr, HSFLOW_ERR_HIP, "stream creation failed");
    }
    *out = ctx;
    return HSFLOW_OK;
}

void hsflow_destroy(hsflow_ctx *ctx) {
    if (!ctx) return;
    (void)hipSetDevice(ctx->device);
    if (ctx->stream) (void)hipStreamSynchronize(ctx->stream);
    if (ctx->d_in) (void)hipFree(ctx->d_in);
    if (ctx->d_out) (void)hipFree(ctx->d_out);
    if (ctx->d_ws) (void)hipFree(ctx->d_ws);
    if (ctx->h_stage) (void)hipHostFree(ctx->h_stage);
    for (hipEvent_t e : ctx->dl_ev) (void)hipEventDestroy(e);
    if (ctx->stream) (void)hipStreamDestroy(ctx->stream);
    delete ctx;
}

const char *hsflow_last_error(const hsflow_ctx *ctx) {
    return ctx ? ctx->err.c_str() : g_err.c_str();
}

void *hsflow_stream(hsflow_ctx *ctx) { return ctx ? (void *)ctx->stream : nullptr; }

size_t hsflow_workspace_bytes(int rows, int cols, int batch) {
    if (!sizes_ok(rows, cols, batch)) return 0;
    return carve(nullptr, rows, cols, batch).bytes;
}

int hsflow_set_iters_per_launch(int k) {
    if (k < 0) return HSFLOW_ERR_ARG;
    g_kb_override = k;
    return HSFLOW_OK;
}

int hsflow_set_jacobi_kernel(int k) {
    if (k != 0 && k != 2 && k != 4) return HSFLOW_ERR_ARG;
    g_kernel_override = k;
    return HSFLOW_OK;
}

int hsflow_set_strip_rows(int seg_rows) {
    if (seg_rows < 0 || seg_rows > kMaxRows) return HSFLOW_ERR_ARG;
    g_strip_rows = seg_rows;
    return HSFLOW_OK;
}

const char *hsflow_jacobi_kernel_name(int rows, int cols, int batch, int window) {
    if (window < 1 || window > HSFLOW_MAX_WINDOW || !sizes_ok(rows, cols, batch)) return "";
    if (window > 9) return "hs_jacobi_generic_kernel";
    if (plan_passes(window, true, rows, cols, batch).strip) return "hs_jacobi_strip_kernel";
    return window >= 3 ? "hs_jacobi_wg_kernel" : "hs_jacobi_kernel";
}

int hsflow_strip_seg_rows(int rows, int cols, int batch, int window) {
    if (window < 1 || window > HSFLOW_MAX_WINDOW || !sizes_ok(rows, cols, batch)) return 0;
    if (!plan_passes(window, true, rows, cols, batch).strip) return 0;
    if (g_strip_rows > 0) {
        int nseg = 0, nstrips = 0;
        return hsflow::strip_seg_rows(window, strip_kb(window), rows, cols, batch, 1, &nseg,
                                      &nstrips, g_strip_rows);
    }
    int nseg = 0, nstrips = 0;
    return hsflow::strip_seg_rows(window, strip_kb(window), rows, cols, batch,
                                  8 * hsflow::device_cus(), &nseg, &nstrips, 0);
}

int hsflow_set_max_streams(int n) {
    if (n < 0 || n > 16) return HSFLOW_ERR_ARG;
    g_split_override = n;
    return HSFLOW_OK;
}

int hsflow_max_streams(void) { return g_split_override; }

int hsflow_set_output_hugepages(int on) {
    return hsflow::g_output_hugepages.exchange(on ? 1 : 0);
}

int hsflow_iters_per_launch(int rows, int cols, int batch, int window) {
    if (window < 1 || window > HSFLOW_MAX_WINDOW) return HSFLOW_ERR_ARG;
    if (!sizes_ok(rows, cols, batch)) return HSFLOW_ERR_ARG;
    return pick_kb(window, true, rows, cols, batch);
}

int hsflow_gradients_device(const void *I0, const void *I1, int dtype_in, int rows,
                            int cols, int batch, float *gx, float *gy, float *gt,
                            void *workspace, size_t workspace_bytes, void *stream) {
    DeviceGuard g((hipStream_t)stream);
    return gradients_impl(nullptr, I0, I1, dtype_in, rows, cols, batch, gx, gy, gt,
                          workspace, workspace_bytes, (hipStream_t)stream);
}

int hsflow_jacobi_device(int rows, int cols, int batch, int window, int iters,
                         float alpha, int warm_start, float *u, float *v, void *workspace,
                         size_t workspace_bytes, void *stream) {
    DeviceGuard g((hipStream_t)stream);
    // the workspace flags say per pair which gradient format is valid; the
    // f32 variant is launched too unless we know every pair is packed
    return jacobi_impl(nullptr, rows, cols, batch, window, iters, alpha, warm_start != 0,
                       true, u, v, workspace, workspace_bytes, (hipStream_t)stream);
}

int hsflow_flow_device(const void *I0, const void *I1, int dtype_in, int rows, int cols,
                       int batch, int window, int iters, float alpha, float *u, float *v,
                       void *workspace, size_t workspace_bytes, void *stream) {
    DeviceGuard g((hipStream_t)stream);
    // K1 for the whole batch, then the passes (split over the side streams).
    // Running each half's K1 on its side stream instead measured 0.6 % slower
    // (the halves' first passes start out of step; profiles/r05_k1_ab.txt)
    int rc = gradients_impl(nullptr, I0, I1, dtype_in, rows, cols, batch, nullptr,
                            nullptr, nullptr, workspace, workspace_bytes,
                            (hipStream_t)stream);
    if (rc) return rc;
    // 8-bit inputs always give exact packed gradients: skip the f32 variant
    return jacobi_impl(nullptr, rows, cols, batch, window, iters, alpha, false,
                       dtype_in != HSFLOW_U8, u, v, workspace, workspace_bytes,
                       (hipStream_t)stream);
}

int hsflow_flow(hsflow_ctx *ctx, const void *I0, const void *I1, int dtype_in, int rows,
                int cols, size_t in_step0, size_t in_step1, int window, int iters,
                double alpha, void *u, void *v, int dtype_out, size_t out_step) {
    int rc = check_host_args(ctx, I0, I1, dtype_in, rows, cols, in_step0, in_step1,
                             dtype_out, out_step);
    if (rc) return rc;
    if (!u || !v) return fail(ctx, HSFLOW_ERR_ARG, "null output");
    if (window < 1 || window > HSFLOW_MAX_WINDOW)
        return fail(ctx, HSFLOW_ERR_ARG, "windowSize %d outside [1, %d]", window,
                    HSFLOW_MAX_WINDOW);
    if (iters < 0) return fail(ctx, HSFLOW_ERR_ARG, "maxIterations %d < 0", iters);
    HIP_TRY(ctx, hipSetDevice(ctx->device));
    const size_t n = (size_t)rows * cols;
    const size_t in_es = (size_t)dev_elem_size(dtype_in);
    if ((rc = grow(ctx, &ctx->d_in, &ctx->d_in_bytes, align_up(n * in_es) * 2))) return rc;
    if ((rc = grow(ctx, &ctx->d_out, &ctx->d_out_bytes, align_up(n * 4) * 3))) return rc;
    const size_t wsb = hsflow_workspace_bytes(rows, cols, 1);
    if ((rc = grow(ctx, &ctx->d_ws, &ctx->d_ws_bytes, wsb))) return rc;
    char *in0 = (char *)ctx->d_in, *in1 = in0 + align_up(n * in_es);
    float *du = (float *)ctx->d_out, *dv = (float *)((char *)du + align_up(n * 4));
    if ((rc = upload_pair(ctx, I0, I1, (int)in_es, rows, cols, in_step0, in_step1, in0, in1)))
        return rc;
    const int dt0 = dtype_in;
    rc = gradients_impl(ctx, in0, in1, dt0, rows, cols, 1, nullptr, nullptr, nullptr,
                        ctx->d_ws, ctx->d_ws_bytes, ctx->stream);
    if (rc) return rc;
    rc = jacobi_impl(ctx, rows, cols, 1, window, iters, (float)alpha, false,
                     dt0 != HSFLOW_U8, du, dv, ctx->d_ws, ctx->d_ws_bytes, ctx->stream);
    if (rc) return rc;
    {
        const float *srcs[2] = {du, dv};
        void *dsts[2] = {u, v};
        if ((rc = download_planes(ctx, srcs, dsts, 2, rows, cols, dtype_out, out_step)))
            return rc;
    }
    return HSFLOW_OK;
}

// Frame-parallel host API over several GPUs of the node from ONE process
// (include/hsflow.h): one host thread, context and stream per listed device,
// pair j on devices[j % n].  The per-pair work is exactly hsflow_flow.
int hsflow_flow_multi(const int *devices, int n_devices, int batch,
                      const void *const *I0, const void *const *I1, int dtype_in, int rows,
                      int cols, size_t in_step0, size_t in_step1, int window, int iters,
                      double alpha, void *const *u, void *const *v, int dtype_out,
                      size_t out_step) {
    if (!devices || n_devices < 1 || n_devices > 64)
        return fail(nullptr, HSFLOW_ERR_ARG, "need 1..64 devices, got %d", n_devices);
    if (batch < 0) return fail(nullptr, HSFLOW_ERR_ARG, "batch %d < 0", batch);
    if (batch == 0) return HSFLOW_OK;
    if (!I0 || !I1 || !u || !v) return fail(nullptr, HSFLOW_ERR_ARG, "null pair array");
    for (int j = 0; j < batch; ++j)
        if (!I0[j] || !I1[j] || !u[j] || !v[j])
            return fail(nullptr, HSFLOW_ERR_ARG, "null buffer in pair %d", j);
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= 0)
        return fail(nullptr, HSFLOW_ERR_NODEV, "no HIP device");
    for (int k = 0; k < n_devices; ++k)
        if (devices[k] < 0 || devices[k] >= ndev)
            return fail(nullptr, HSFLOW_ERR_NODEV, "device %d of %d", devices[k], ndev);
    const int nw = std::min(n_devices, batch);
    std::vector<MultiSlot *> slot = multi_slots(devices, nw);
    std::vector<int> rc(nw, HSFLOW_OK);
    std::vector<std::string> msg(nw);
    std::vector<std::thread> pool;
    pool.reserve(nw);
    for (int k = 0; k < nw; ++k) {
        pool.emplace_back([&, k] {
            std::lock_guard<std::mutex> hold(slot[k]->mu);
            int r = HSFLOW_OK;
            if (!slot[k]->ctx) {
                r = hsflow_create(&slot[k]->ctx, devices[k]);
                if (r) {
                    rc[k] = r;
                    msg[k] = hsflow_last_error(nullptr);  // this worker's message
                    return;
                }
            }
            hsflow_ctx *ctx = slot[k]->ctx;
            for (int j = k; j < batch && r == HSFLOW_OK; j += nw)
                r = hsflow_flow(ctx, I0[j], I1[j], dtype_in, rows, cols, in_step0, in_step1,
                                window, iters, alpha, u[j], v[j], dtype_out, out_step);
            if (r) {
                msg[k] = hsflow_last_error(ctx);
                // a context that hit a runtime error is not trusted with the
                // next call; argument and size errors leave it as it was
                if (r != HSFLOW_ERR_ARG && r != HSFLOW_ERR_SIZE) {
                    hsflow_destroy(ctx);
                    slot[k]->ctx = nullptr;
                }
            }
            rc[k] = r;
        });
    }
    for (auto &t : pool) t.join();
    for (int k = 0; k < nw; ++k)
        if (rc[k]) return fail(nullptr, rc[k], "device %d: %s", devices[k], msg[k].c_str());
    return HSFLOW_OK;
}

void hsflow_flow_multi_release(void) {
    std::lock_guard<std::mutex> reg(g_multi_mu);
    for (auto &dv : g_multi)
        for (auto &sl : dv) {
            std::lock_guard<std::mutex> hold(sl->mu);
            if (sl->ctx) hsflow_destroy(sl->ctx);
            sl->ctx = nullptr;
        }
}

int hsflow_pyramid_level_size(int rows, int cols, int level, int *level_rows,
                              int *level_cols) {
    if (rows < 1 || cols < 1 || level < 0 || level >= HSFLOW_MAX_LEVELS) return HSFLOW_ERR_ARG;
    for (int l = 0; l < level; ++l) {
        rows = (rows + 1) / 2;
        cols = (cols + 1) / 2;
    }
    if (level_rows) *level_rows = rows;
    if (level_cols) *level_cols = cols;
    return HSFLOW_OK;
}

size_t hsflow_pyramid_workspace_bytes(int rows, int cols, int batch, int levels) {
    if (!sizes_ok(rows, cols, batch) || levels < 1 || levels > HSFLOW_MAX_LEVELS) return 0;
    return pyr_layout(rows, cols, batch, levels).bytes;
}

int hsflow_pyramid_build_device(const void *I0, const void *I1, int dtype_in, int rows,
                                int cols, int batch, int levels, float *const *I0_levels,
                                float *const *I1_levels, void *workspace,
                                size_t workspace_bytes, void *stream) {
    if (levels < 1 || levels > HSFLOW_MAX_LEVELS)
        return fail(nullptr, HSFLOW_ERR_ARG, "levels %d outside [1, %d]", levels,
                    HSFLOW_MAX_LEVELS);
    if (levels > 1 && (!I0_levels || !I1_levels))
        return fail(nullptr, HSFLOW_ERR_ARG, "null level array");
    for (int l = 1; l < levels; ++l)
        if (!I0_levels[l - 1] || !I1_levels[l - 1])
            return fail(nullptr, HSFLOW_ERR_ARG, "null level plane %d", l);
    hipStream_t s = (hipStream_t)stream;
    DeviceGuard g(s);
    // K1 at level 0 decides each pair's rounding (flags in the workspace)
    int rc = gradients_impl(nullptr, I0, I1, dtype_in, rows, cols, batch, nullptr, nullptr,
                            nullptr, workspace, workspace_bytes, s);
    if (rc || levels == 1) return rc;
    const uint32_t *flags = carve(workspace, rows, cols, batch).flags;
    int r = rows, c = cols;
    for (int l = 1; l < levels; ++l) {
        for (int k = 0; k < 2; ++k) {
            const void *src = l == 1 ? (k ? I1 : I0)
                                     : (const void *)(k ? I1_levels[l - 2] : I0_levels[l - 2]);
            hipError_t e = hsflow::launch_pyrdown(src, l == 1 ? dtype_in : HSFLOW_F32, r, c,
                                                  batch, k ? I1_levels[l - 1] : I0_levels[l - 1],
                                                  flags, s);
            if (e != hipSuccess) return hip_fail(nullptr, e, "pyrdown launch");
        }
        r = (r + 1) / 2;
        c = (c + 1) / 2;
    }
    return HSFLOW_OK;
}

int hsflow_upflow_device(const float *uc, const float *vc, int rc, int cc, float *u,
                         float *v, int rows, int cols, int batch, void *stream) {
    DeviceGuard g((hipStream_t)stream);
    if (!uc || !vc || !u || !v) return fail(nullptr, HSFLOW_ERR_ARG, "null device pointer");
    if (!sizes_ok(rows, cols, batch) || rc < (rows + 1) / 2 || cc < (cols + 1) / 2)
        return fail(nullptr, HSFLOW_ERR_ARG, "bad sizes %dx%d from %dx%d", rows, cols, rc, cc);
    hipError_t e = hsflow::launch_upflow(uc, vc, rc, cc, u, v, rows, cols, batch,
                                         (hipStream_t)stream);
    if (e != hipSuccess) return hip_fail(nullptr, e, "upflow launch");
    return HSFLOW_OK;
}

int hsflow_flow_pyramid_device(const void *I0, const void *I1, int dtype_in, int rows,
                               int cols, int batch, int levels, int window, int iters,
                               float alpha, float *u, float *v, void *workspace,
                               size_t workspace_bytes, void *stream) {
    DeviceGuard g((hipStream_t)stream);
    return pyramid_impl(nullptr, I0, I1, dtype_in, rows, cols, batch, levels, window, iters,
                        alpha, u, v, workspace, workspace_bytes, (hipStream_t)stream);
}

int hsflow_flow_pyramid(hsflow_ctx *ctx, const void *I0, const void *I1, int dtype_in,
                        int rows, int cols, size_t in_step0, size_t in_step1, int levels,
                        int window, int iters, double alpha, void *u, void *v,
                        int dtype_out, size_t out_step) {
    int rc = check_host_args(ctx, I0, I1, dtype_in, rows, cols, in_step0, in_step1,
                             dtype_out, out_step);
    if (rc) return rc;
    if (!u || !v) return fail(ctx, HSFLOW_ERR_ARG, "null output");
    if (levels < 1 || levels > HSFLOW_MAX_LEVELS)
        return fail(ctx, HSFLOW_ERR_ARG, "levels %d outside [1, %d]", levels,
                    HSFLOW_MAX_LEVELS);
    HIP_TRY(ctx, hipSetDevice(ctx->device));
    const size_t n = (size_t)rows * cols;
    const size_t in_es = (size_t)dev_elem_size(dtype_in);
    if ((rc = grow(ctx, &ctx->d_in, &ctx->d_in_bytes, align_up(n * in_es) * 2))) return rc;
    if ((rc = grow(ctx, &ctx->d_out, &ctx->d_out_bytes, align_up(n * 4) * 3))) return rc;
    const size_t wsb = hsflow_pyramid_workspace_bytes(rows, cols, 1, levels);
    if ((rc = grow(ctx, &ctx->d_ws, &ctx->d_ws_bytes, wsb))) return rc;
    char *in0 = (char *)ctx->d_in, *in1 = in0 + align_up(n * in_es);
    float *du = (float *)ctx->d_out, *dv = (float *)((char *)du + align_up(n * 4));
    if ((rc = upload_pair(ctx, I0, I1, (int)in_es, rows, cols, in_step0, in_step1, in0, in1)))
        return rc;
    const int dt0 = dtype_in;
    rc = pyramid_impl(ctx, in0, in1, dt0, rows, cols, 1, levels, window, iters,
                      (float)alpha, du, dv, ctx->d_ws, ctx->d_ws_bytes, ctx->stream);
    if (rc) return rc;
    {
        const float *srcs[2] = {du, dv};
        void *dsts[2] = {u, v};
        if ((rc = download_planes(ctx, srcs, dsts, 2, rows, cols, dtype_out, out_step)))
            return rc;
    }
    return HSFLOW_OK;
}

int hsflow_bgr_to_gray_device(const uint8_t *bgr, int rows, int cols, int batch,
                              uint8_t *gray, void *stream) {
    DeviceGuard g((hipStream_t)stream);
    if (!bgr || !gray) return fail(nullptr, HSFLOW_ERR_ARG, "null device pointer");
    if (!sizes_ok(rows, cols, batch))
        return fail(nullptr, HSFLOW_ERR_ARG, "bad size %dx%d batch %d", rows, cols, batch);
    hipError_t e = hsflow::launch_bgr2gray(bgr, rows, cols, batch, gray, (hipStream_t)stream);
    if (e != hipSuccess) return hip_fail(nullptr, e, "bgr2gray launch");
    return HSFLOW_OK;
}

int hsflow_download_device(void *dst, const void *src, size_t bytes, void *stream) {
    if (bytes == 0) return HSFLOW_OK;
    if (!dst || !src) return fail(nullptr, HSFLOW_ERR_ARG, "null pointer");
    DeviceGuard g((hipStream_t)stream);
    // As a pitched copy the runtime moves a device -> pinned host download
    // with its DMA engines at ~46 GB/s (a flat hipMemcpyAsync: ~29 GB/s;
    // torch's copy_ of pinned memory: a blit kernel that takes the Jacobi
    // passes' workgroup slots; scripts/pcie/d2h_engine_probe.hip).
    constexpr size_t kRow = 7680;  // bytes per pitched row
    const size_t rows = bytes / kRow, tail = bytes - rows * kRow;
    hipStream_t s = (hipStream_t)stream;
    if (rows > 0)
        HIP_TRY(nullptr, hipMemcpy2DAsync(dst, kRow, src, kRow, kRow, rows,
                                          hipMemcpyDeviceToHost, s));
    if (tail > 0)
        HIP_TRY(nullptr, hipMemcpyAsync((char *)dst + rows * kRow,
                                        (const char *)src + rows * kRow, tail,
                                        hipMemcpyDeviceToHost, s));
    return HSFLOW_OK;
}

int hsflow_flow_bgr(hsflow_ctx *ctx, const uint8_t *bgr0, const uint8_t *bgr1, int rows,
                    int cols, size_t bgr_step0, size_t bgr_step1, int window, int iters,
                    double alpha, void *u, void *v, int dtype_out, size_t out_step) {
    if (!ctx) return HSFLOW_ERR_ARG;
    if (!bgr0 || !bgr1 || !u || !v) return fail(ctx, HSFLOW_ERR_ARG, "null pointer");
    if (!sizes_ok(rows, cols, 1)) return fail(ctx, HSFLOW_ERR_ARG, "bad size %dx%d", rows, cols);
    if (bgr_step0 < (size_t)cols * 3 || bgr_step1 < (size_t)cols * 3)
        return fail(ctx, HSFLOW_ERR_ARG, "BGR steps %zu, %zu < row bytes", bgr_step0,
                    bgr_step1);
    if (dtype_out != HSFLOW_F32 && dtype_out != HSFLOW_F64)
        return fail(ctx, HSFLOW_ERR_ARG, "output dtype must be F32 or F64");
    if (out_step < (size_t)cols * elem_size(dtype_out))
        return fail(ctx, HSFLOW_ERR_ARG, "output step %zu < row bytes", out_step);
    if (window < 1 || window > HSFLOW_MAX_WINDOW)
        return fail(ctx, HSFLOW_ERR_ARG, "windowSize %d outside [1, %d]", window,
                    HSFLOW_MAX_WINDOW);
    if (iters < 0) return fail(ctx, HSFLOW_ERR_ARG, "maxIterations %d < 0", iters);
    HIP_TRY(ctx, hipSetDevice(ctx->device));
    const size_t n = (size_t)rows * cols;
    // [bgr0 bgr1] back to back (one batch-2 launch), then [gray0 gray1]
    const size_t gray_off = align_up(6 * n);
    int rc;
    if ((rc = grow(ctx, &ctx->d_in, &ctx->d_in_bytes, gray_off + align_up(2 * n)))) return rc;
    if ((rc = grow(ctx, &ctx->d_out, &ctx->d_out_bytes, align_up(n * 4) * 3))) return rc;
    if ((rc = grow(ctx, &ctx->d_ws, &ctx->d_ws_bytes, hsflow_workspace_bytes(rows, cols, 1))))
        return rc;
    uint8_t *db = (uint8_t *)ctx->d_in, *dg = db + gray_off;
    if ((rc = upload_pair(ctx, bgr0, bgr1, 3, rows, cols, bgr_step0, bgr_step1, db, db + 3 * n)))
        return rc;
    hipError_t e = hsflow::launch_bgr2gray(db, rows, cols, 2, dg, ctx->stream);
    if (e != hipSuccess) return hip_fail(ctx, e, "bgr2gray launch");
    float *du = (float *)ctx->d_out, *dv = (float *)((char *)du + align_up(n * 4));
    rc = gradients_impl(ctx, dg, dg + n, HSFLOW_U8, rows, cols, 1, nullptr, nullptr, nullptr,
                        ctx->d_ws, ctx->d_ws_bytes, ctx->stream);
    if (rc) return rc;
    rc = jacobi_impl(ctx, rows, cols, 1, window, iters, (float)alpha, false, false, du, dv,
                     ctx->d_ws, ctx->d_ws_bytes, ctx->stream);
    if (rc) return rc;
    {
        const float *srcs[2] = {du, dv};
        void *dsts[2] = {u, v};
        if ((rc = download_planes(ctx, srcs, dsts, 2, rows, cols, dtype_out, out_step)))
            return rc;
    }
    return HSFLOW_OK;
}

int hsflow_gradients(hsflow_ctx *ctx, const void *I0, const void *I1, int dtype_in,
                     int rows, int cols, size_t in_step0, size_t in_step1, void *gx,
                     void *gy, void *gt, int dtype_out, size_t out_step) {
    int rc = check_host_args(ctx, I0, I1, dtype_in, rows, cols, in_step0, in_step1,
                             dtype_out, out_step);
    if (rc) return rc;
    if (!gx || !gy || !gt) return fail(ctx, HSFLOW_ERR_ARG, "null output");
    HIP_TRY(ctx, hipSetDevice(ctx->device));
    const size_t n = (size_t)rows * cols;
    const size_t in_es = (size_t)dev_elem_size(dtype_in);
    if ((rc = grow(ctx, &ctx->d_in, &ctx->d_in_bytes, align_up(n * in_es) * 2))) return rc;
    if ((rc = grow(ctx, &ctx->d_out, &ctx->d_out_bytes, align_up(n * 4) * 3))) return rc;
    const size_t wsb = hsflow_workspace_bytes(rows, cols, 1);
    if ((rc = grow(ctx, &ctx->d_ws, &ctx->d_ws_bytes, wsb))) return rc;
    char *in0 = (char *)ctx->d_in, *in1 = in0 + align_up(n * in_es);
    float *dx = (float *)ctx->d_out;
    float *dy = (float *)((char *)dx + align_up(n * 4));
    float *dt = (float *)((char *)dy + align_up(n * 4));
    if ((rc = upload_pair(ctx, I0, I1, (int)in_es, rows, cols, in_step0, in_step1, in0, in1)))
        return rc;
    const int dt0 = dtype_in;
    rc = gradients_impl(ctx, in0, in1, dt0, rows, cols, 1, dx, dy, dt, ctx->d_ws,
                        ctx->d_ws_bytes, ctx->stream);
    if (rc) return rc;
    {
        const float *srcs[3] = {dx, dy, dt};
        void *dsts[3] = {gx, gy, gt};
        if ((rc = download_planes(ctx, srcs, dsts, 3, rows, cols, dtype_out, out_step)))
            return rc;
    }
    return HSFLOW_OK;
}

}  // extern "C"
