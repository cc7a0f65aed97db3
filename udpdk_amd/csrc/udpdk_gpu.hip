// udpdk_gpu.hip — host side of the C ABI declared in include/udpdk_gpu.h.
//
// Owns the per-device context (stream, bind snapshot, workspace, pinned readback) and enqueues
// the RX and TX kernels. No hidden synchronisation on the RX/TX enqueue path: everything stays
// on the context stream, so a caller may capture udpdk_gpu_rx into a hipGraph.
#include <hip/hip_runtime.h>
#include <hip/hip_ext.h>

#include <errno.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <new>
#include <vector>

#include "udpdk_gpu.h"
#include "rx_common.h"

using namespace udpdk;

namespace {

constexpr int EVENT_SETS = 256;   // timed calls buffered between two timing reads

struct DevResult {
    unsigned long long counters[UDPDK_N_COUNTERS];
    uint32_t total;
    uint32_t pad;
    // speculative single-lane compaction: word k = max of (call epoch << 32 | ~tile) over the
    // tiles t = k mod 64 that did not deliver all their frames (rx_classify); the smallest tile
    // over the 64 words is the call's first such tile (64 words: a batch with many short tiles
    // does not serialise on one address)
    unsigned long long nonfull[UDPDK_SPEC_WORDS];
};

// Per-call kernel timing: start/stop events carried by the kernel dispatches themselves
// (hipExtLaunchKernelGGL), so timing adds no marker packets between back-to-back kernels.
constexpr int TIMED_KERNELS = 3;  // classify, scan, scatter (single-lane path: compact)
struct TimingSet {
    hipEvent_t ev[2 * TIMED_KERNELS];
    bool used[TIMED_KERNELS];
};

// One RX pipe = a stream and the per-call workspace. With pipelining depth d > 1, consecutive
// udpdk_gpu_rx calls rotate over d pipes, so one batch's prologue, tail and compaction overlap
// the other batches' streaming phases (the calls are independent: distinct batches and output
// buffers). Depth 3 is the measured optimum for 1 M x 64 B (tools/probe/classify_probe: classify
// + compaction 22.2 / 19.0 / 15.5 / 17.4 us per batch at 1 / 2 / 3 / 4 streams; 4 streams exceed
// the box's 4 hardware queues with the context stream's own traffic).
struct Pipe {
    hipStream_t stream = nullptr;
    uint32_t *hist = nullptr;
    uint32_t *partial = nullptr;
    uint32_t *base = nullptr;                 // [tiles][lanes] absolute positions (rx_scan_cols)
    unsigned long long *agg = nullptr;        // rx_scan_cols look-back words, one per lane block
    uint32_t *ticket = nullptr;               // rx_scan_cols lane-block tickets
    uint32_t epoch = 0;                       // rx_scan_cols calls on this pipe (look-back tag)
    uint32_t spec_epoch = 0;                  // speculative compaction calls (DevResult::nonfull tag)
    unsigned long long *fuse = nullptr;       // rx_classify fused-completion fan-in words (zeroed)
    uint32_t *tile_cnt = nullptr;
    DevResult *res = nullptr;                 // counters, total (device)
    DevResult *h_res = nullptr;               // pinned mirror, filled by udpdk_gpu_rx_stats
    hipEvent_t tail = nullptr;                // join point for udpdk_gpu_join
    bool dirty = false;                       // work enqueued since the last join
    uint32_t last_tiles = 0;                  // tiles of this pipe's last call (counter rows)
    uint32_t last_lane_cap = 0;
    // host-resident batches (udpdk_gpu_rx_host[_async]): staging, lazily sized
    uint8_t *st_frames_d = nullptr; size_t st_frames_dcap = 0;
    uint8_t *st_frames_h = nullptr; size_t st_frames_hcap = 0;
    uint8_t *st_desc_d = nullptr; size_t st_desc_dcap = 0;
    uint8_t *st_desc_h = nullptr; size_t st_desc_hcap = 0;
    uint8_t *st_out_d = nullptr; size_t st_out_cap = 0;
    udpdk_rx_stats_t *host_stats = nullptr;   // outstanding async host call: where its stats go
    udpdk_rx_batch_t staged{};                // device view of the last host batch staged here
    const uint32_t *staged_meta = nullptr;    // and its verdict words
};
constexpr int MAX_PIPES = 4;
constexpr size_t FUSE_BYTES = 128u * UDPDK_FUSE_LINES;   // one 128-B line per fan-in / repair word
constexpr size_t HINT_BYTES = 192u;
constexpr uint32_t RSS_FUSE_MAX_ENTRIES = 8192u;   // rss_hash's last workgroup scans <= this many
#ifndef UDPDK_HINT_WINDOW
#define UDPDK_HINT_WINDOW 8u       // calls (as far as the GPU got) a tail pass / a not-full tile
                                   // keeps the other form on
#endif

} // namespace

struct udpdk_gpu_ctx {
    int device = 0;
    hipStream_t stream = nullptr;             // = pipes[0].stream: the context stream
    int last_err = 0;
    uint32_t max_frames = 0, max_lanes = 0;

    // bind snapshot (device)
    uint4 *port_tab = nullptr;          // [65536]
    uint2 *binds = nullptr;
    uint32_t binds_cap = 0;
    uint4 *slots = nullptr;
    uint32_t slots_cap = 0, n_slots = 0;
    uint32_t n_lanes = 1, lane_mask = 0xFFFFFFFFu, key_bits = 0, max_fanout = 0;
    // the bound ports when there are at most UDPDK_INLINE_PORTS (RxArgs::inl)
    uint32_t inl = 0, n_inl = 0, inl_port[UDPDK_INLINE_PORTS] = {};
    uint4 inl_ent[UDPDK_INLINE_PORTS] = {};
    uint32_t one_lane_tile = 0;    // UDPDK_ONE_LANE_TILE (diagnostic): single-lane tile override
    uint64_t geo_cap = RX_HIST_CAP; // UDPDK_RX_HIST_CAP (diagnostic): lanes x tiles bound of the geometry
    // Kernel hints (pinned host memory the kernels write, RxArgs::hint): the call sequence number
    // of the last call that ran a tail pass / had a tile before the last not full. The single-lane
    // path takes rx_classify<1> and the fused completion while neither was seen in the last
    // UDPDK_HINT_WINDOW calls; both forms are exact for any batch, the hint only picks the faster.
    uint32_t *hint = nullptr;
    uint32_t rx_seq = 0;
    int force_fuse = -1;           // UDPDK_RX_FUSE=0/1 (tests, A/B): fused completion off / always
    int force_tailg = 0;           // UDPDK_RX_TAILG=1/2 (tests, A/B): rx_classify<G> always
    int force_mr = -1;             // UDPDK_RX_MR=0/1 (tests, A/B): the round-ahead descriptor form
    bool no_span = false;          // UDPDK_RX_SPAN=0 (tests, A/B): no span sweep (RxArgs::span)
    bool trace = false;            // UDPDK_RX_TRACE (diagnostic): the form of every call on stderr
    bool no_inline = false;        // UDPDK_RX_NO_INLINE (tests, A/B): always the port-table loads
    uint32_t scatter_group_frames = UDPDK_SCATTER_GROUP_FRAMES;   // UDPDK_SCATTER_GROUP_FRAMES (tests, A/B)
    uint32_t scatter_min_wg = UDPDK_SCATTER_MIN_WG;               // UDPDK_SCATTER_MIN_WG (tests, A/B)
    bool have_snapshot = false;

    // RX workspace, one set per pipe
    Pipe pipes[MAX_PIPES];
    int depth = 1;                            // udpdk_gpu_pipeline_depth
    uint64_t rx_calls = 0;
    int last_pipe = -1;                       // pipe of the last udpdk_gpu_rx (-1: none yet)
    size_t hist_cap = 0;
    size_t partial_cap = 0;
    size_t tiles_cap = 0;

    uint64_t host_calls = 0;                  // udpdk_gpu_rx_host_async calls (pipe choice)

    unsigned long long *dbg = nullptr;        // diagnostic stamp buffer (UDPDK_STAMPS builds)
    Reasm *reasm = nullptr;                   // udpdk_gpu_frag_table_create
    // receive-side scaling (udpdk_gpu_rss_config)
    bool rss_ready = false;
    RssArgs rss{};
    uint16_t *rss_reta = nullptr;
    uint32_t *rss_ktab = nullptr;             // [12][256] key windows
    uint8_t *rss_qid = nullptr;
    uint32_t *rss_hist = nullptr, *rss_partial = nullptr, *rss_total = nullptr;
    unsigned long long *rss_fuse = nullptr;   // rss_hash fan-in words (fused queue bases)
    bool rss_no_fuse = false;                 // UDPDK_RSS_FUSE=0 (tests, A/B): the rss_base launch

    // timing
    uint32_t timing_every = 0;                // 0 off, N: events on every Nth call
    uint64_t timing_calls = 0;
    TimingSet *sets = nullptr;
    int n_sets_used = 0;
    double ms[UDPDK_N_KERNEL_IDS] = {};
    uint32_t launches[UDPDK_N_KERNEL_IDS] = {};
};

#define HIPC(ctx, expr)                                                      \
    do {                                                                     \
        hipError_t e_ = (expr);                                              \
        if (e_ != hipSuccess) {                                              \
            if (ctx) (ctx)->last_err = (int)e_;                              \
            return -EIO;                                                     \
        }                                                                    \
    } while (0)

namespace {

uint32_t ceil_div(uint64_t a, uint64_t b) { return (uint32_t)((a + b - 1) / b); }

// Range of the frames buffer resource. Buffer loads are range-checked per dword (a dword is
// returned only if it ends within the range, zero otherwise, with no memory access:
// tools/probe/range_probe.hip) and the RX kernels load at byte-aligned frame offsets, so a
// dword holding the last frame bytes may end up to 3 bytes past frames_bytes: the range is
// frames_bytes + 3 rounded up to a dword, inside the UDPDK_GPU_FRAMES_TAILROOM bytes the frames
// buffer must keep readable after frames_bytes (udpdk_gpu.h).
uint32_t frames_rsrc_bytes(uint64_t frames_bytes)
{
    return (uint32_t)std::min<uint64_t>((frames_bytes + 3 + 3) & ~3ull, 0xFFFFFFFCull);
}

void geometry(uint32_t n, uint32_t lanes, uint32_t *T, uint32_t *tiles, uint64_t cap = RX_HIST_CAP)
{
    uint32_t t = RX_TILE_MIN;
    while (t < RX_TILE_MAX && (uint64_t)ceil_div(n, t) * lanes > cap) t *= 2;
    *T = t;
    *tiles = std::max<uint32_t>(1u, ceil_div(n, t));
}

int fold_timing(udpdk_gpu_ctx *c)
{
    if (!c->n_sets_used) return 0;
    for (Pipe &P : c->pipes) HIPC(c, hipStreamSynchronize(P.stream));
    static const int kid[TIMED_KERNELS] = {UDPDK_K_RX_CLASSIFY, UDPDK_K_RX_SCAN, UDPDK_K_RX_SCATTER};
    for (int i = 0; i < c->n_sets_used; ++i) {
        for (int k = 0; k < TIMED_KERNELS; ++k) {
            if (!c->sets[i].used[k]) continue;
            float ms = 0;
            HIPC(c, hipEventElapsedTime(&ms, c->sets[i].ev[2 * k], c->sets[i].ev[2 * k + 1]));
            c->ms[kid[k]] += ms;
            c->launches[kid[k]]++;
        }
    }
    c->n_sets_used = 0;
    return 0;
}

// Launch on the context stream; with a timing set, kernel k's dispatch carries the set's start
// event (first=true) and/or stop event (last=true).
template <typename K, typename... A>
hipError_t launch(hipStream_t st, TimingSet *ts, int k, bool first, bool last, K kern, dim3 grid,
                  dim3 block, uint32_t lds, A... args)
{
    if (ts) {
        ts->used[k] = true;
        hipExtLaunchKernelGGL(kern, grid, block, lds, st, first ? ts->ev[2 * k] : nullptr,
                              last ? ts->ev[2 * k + 1] : nullptr, 0u, args...);
    } else {
        hipLaunchKernelGGL(kern, grid, block, lds, st, args...);
    }
    return hipGetLastError();
}

// Order everything enqueued on the other pipes before what comes next on the context stream.
int join_pipes(udpdk_gpu_ctx *c)
{
    for (int i = 1; i < MAX_PIPES; ++i) {
        Pipe &P = c->pipes[i];
        // an event record + stream wait costs host and GPU time even on an idle stream: only
        // pipes with work since their last join
        if (!P.stream || !P.dirty) continue;
        HIPC(c, hipEventRecord(P.tail, P.stream));
        HIPC(c, hipStreamWaitEvent(c->stream, P.tail, 0));
        P.dirty = false;
    }
    return 0;
}

int sync_all(udpdk_gpu_ctx *c)
{
    for (Pipe &P : c->pipes)
        if (P.stream) HIPC(c, hipStreamSynchronize(P.stream));
    return 0;
}

int ensure_dev(udpdk_gpu_ctx *c, void **p, size_t *cap, size_t need)
{
    if (*cap >= need) return 0;
    if (*p) HIPC(c, hipFree(*p));
    *p = nullptr;
    *cap = 0;
    HIPC(c, hipMalloc(p, need));
    *cap = need;
    return 0;
}

int ensure_host(udpdk_gpu_ctx *c, void **p, size_t *cap, size_t need)
{
    if (*cap >= need) return 0;
    if (*p) HIPC(c, hipHostFree(*p));
    *p = nullptr;
    *cap = 0;
    HIPC(c, hipHostMalloc(p, need, hipHostMallocDefault));
    *cap = need;
    return 0;
}

} // namespace

extern "C" {

int udpdk_gpu_abi_version(void) { return UDPDK_GPU_ABI_VERSION; }

int udpdk_gpu_device_count(int *count)
{
    if (!count) return -EINVAL;
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess) n = 0;
    *count = n;
    return 0;
}

int udpdk_gpu_rx_geometry(uint32_t n, uint32_t n_lanes, uint32_t *tile_frames, uint32_t *n_tiles)
{
    if (!tile_frames || !n_tiles || n_lanes == 0) return -EINVAL;
    geometry(n, n_lanes, tile_frames, n_tiles);
    return 0;
}

int udpdk_gpu_ctx_create(int device, uint32_t max_frames, uint32_t max_lanes, udpdk_gpu_ctx **out)
{
    if (!out || max_lanes == 0 || max_lanes > UDPDK_GPU_MAX_LANES || max_frames == 0) return -EINVAL;
    *out = nullptr;
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || device < 0 || device >= ndev) return -ENODEV;
    udpdk_gpu_ctx *c = new (std::nothrow) udpdk_gpu_ctx();
    if (!c) return -ENOMEM;
    c->device = device;
    c->max_frames = max_frames;
    c->max_lanes = max_lanes;
    if (const char *e = getenv("UDPDK_ONE_LANE_TILE")) {
        const uint32_t t = (uint32_t)atoi(e);
        if (t >= RX_TILE_MIN && t <= RX_TILE_MAX && (t & (t - 1)) == 0) c->one_lane_tile = t;
    }
    if (const char *e = getenv("UDPDK_RX_HIST_CAP")) {
        const uint64_t v = strtoull(e, nullptr, 0);
        if (v >= (1u << 16) && v <= (1u << 26)) c->geo_cap = v;
    }
    if (const char *e = getenv("UDPDK_RX_FUSE")) c->force_fuse = atoi(e) ? 1 : 0;
    c->trace = getenv("UDPDK_RX_TRACE") != nullptr;
    c->no_inline = getenv("UDPDK_RX_NO_INLINE") != nullptr;
    if (const char *e = getenv("UDPDK_RX_MR")) c->force_mr = atoi(e) ? 1 : 0;
    if (const char *e = getenv("UDPDK_RX_SPAN")) c->no_span = atoi(e) == 0;
    if (const char *e = getenv("UDPDK_SCATTER_GROUP_FRAMES")) c->scatter_group_frames = (uint32_t)atoi(e);
    if (const char *e = getenv("UDPDK_SCATTER_MIN_WG")) c->scatter_min_wg = (uint32_t)atoi(e);
    if (const char *e = getenv("UDPDK_RX_TAILG")) {
        const int g = atoi(e);
        if (g == 1 || g == 2) c->force_tailg = g;
    }
    int rc = -EIO;
    do {
        if (hipSetDevice(device) != hipSuccess) break;
        bool ok = true;
        for (Pipe &P : c->pipes) {
            ok = ok && hipStreamCreateWithFlags(&P.stream, hipStreamNonBlocking) == hipSuccess;
            ok = ok && hipEventCreateWithFlags(&P.tail, hipEventDisableTiming) == hipSuccess;
        }
        if (!ok) break;
        c->stream = c->pipes[0].stream;
        if (hipMalloc((void **)&c->port_tab, UDPDK_UDP_PORTS * sizeof(uint4)) != hipSuccess) break;
        if (hipMemset(c->port_tab, 0, UDPDK_UDP_PORTS * sizeof(uint4)) != hipSuccess) break;
        const uint64_t e_cap = std::max<uint64_t>(std::max<uint64_t>(RX_HIST_CAP, c->geo_cap) + max_lanes,
                                                  (uint64_t)ceil_div(max_frames, RX_TILE_MAX) * max_lanes);
        c->hist_cap = e_cap;
        c->partial_cap = e_cap / SCAN_COL_CHUNK + max_lanes + 1;   // chunks x lanes
        c->tiles_cap = ceil_div(max_frames, RX_TILE_MIN) + 1;
        for (Pipe &P : c->pipes) {
            ok = ok && hipMalloc((void **)&P.hist, e_cap * 4) == hipSuccess;
            ok = ok && hipMalloc((void **)&P.partial, c->partial_cap * 4) == hipSuccess;
            ok = ok && hipMalloc((void **)&P.base, e_cap * 4) == hipSuccess;
            // one look-back word per lane block: down to one lane per block when a batch has so
            // many tiles that a column chunk holds a single lane (rx_scan_cols' lb = 0)
            ok = ok && hipMalloc((void **)&P.agg, ((size_t)max_lanes + 1) * 8) == hipSuccess;
            ok = ok && hipMemset(P.agg, 0, ((size_t)max_lanes + 1) * 8) == hipSuccess;
            ok = ok && hipMalloc((void **)&P.ticket, 64) == hipSuccess;
            ok = ok && hipMemset(P.ticket, 0, 64) == hipSuccess;
            ok = ok && hipMalloc((void **)&P.tile_cnt, c->tiles_cap * UDPDK_N_COUNTERS * 4) == hipSuccess;
            ok = ok && hipMalloc((void **)&P.res, sizeof(DevResult)) == hipSuccess;
            ok = ok && hipMemset(P.res, 0, sizeof(DevResult)) == hipSuccess;
            ok = ok && hipHostMalloc((void **)&P.h_res, sizeof(DevResult), hipHostMallocDefault) == hipSuccess;
            ok = ok && hipMalloc((void **)&P.fuse, FUSE_BYTES) == hipSuccess;
            ok = ok && hipMemset(P.fuse, 0, FUSE_BYTES) == hipSuccess;
        }
        // fine-grained (coherent) host memory: the kernels' hint stores go straight to it
        ok = ok && hipHostMalloc((void **)&c->hint, HINT_BYTES, hipHostMallocCoherent | hipHostMallocMapped) == hipSuccess;
        if (ok) {
            // a fresh context starts on the two-launch form (as if call 1 had a tile not full):
            // the fused completion's rewrite of a not-full call is one workgroup's work
            memset(c->hint, 0, HINT_BYTES);
            c->hint[UDPDK_HINT_NONFULL] = 1u;
        }
        if (!ok) break;
        // rx_classify needs up to 141 KiB of dynamic LDS (16384 lanes, 8192-frame tiles)
        // (+ the span sweep's ring, one-round tiles only)
        const int cls_lds = (int)std::min<uint32_t>(
            std::max(classify_lds_bytes(UDPDK_GPU_MAX_LANES, RX_TILE_MAX),
                     classify_lds_bytes(UDPDK_GPU_MAX_LANES, RX_ROUND) + SPAN_LDS_BYTES),
            160u * 1024u - 1024u);   // static LDS besides
        if (hipFuncSetAttribute((const void *)rx_classify<2, 0>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                cls_lds) != hipSuccess) break;
        if (hipFuncSetAttribute((const void *)rx_classify<1, 0>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                cls_lds) != hipSuccess) break;
        if (hipFuncSetAttribute((const void *)rx_classify<2, 1>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                cls_lds) != hipSuccess) break;
        if (hipFuncSetAttribute((const void *)rx_classify<1, 1>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                cls_lds) != hipSuccess) break;
        if (hipFuncSetAttribute((const void *)rx_scatter, hipFuncAttributeMaxDynamicSharedMemorySize,
                                (int)scatter1_lds_bytes(UDPDK_GPU_MAX_LANES)) != hipSuccess) break;
        if (hipFuncSetAttribute((const void *)rx_scatterw<SCATTER_WAVES>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                scatterw_lds_bytes(SCATTERW_MAX_LANES)) != hipSuccess) break;
        if (hipFuncSetAttribute((const void *)rx_scatterw<2 * SCATTER_WAVES>,
                                hipFuncAttributeMaxDynamicSharedMemorySize,
                                scatterw_lds_bytes(SCATTERW_MAX_LANES, 2 * SCATTER_WAVES)) != hipSuccess) break;
        // rx_scan_top's lane totals: 4 B per lane, up to UDPDK_GPU_MAX_LANES (64 KiB)
        if (hipFuncSetAttribute((const void *)rx_scan_top, hipFuncAttributeMaxDynamicSharedMemorySize,
                                4 * UDPDK_GPU_MAX_LANES) != hipSuccess) break;
        rc = 0;
    } while (0);
    if (rc) {
        (void)hipGetLastError();
        udpdk_gpu_ctx_destroy(c);
        return rc;
    }
    *out = c;
    return 0;
}

int udpdk_gpu_ctx_destroy(udpdk_gpu_ctx *c)
{
    if (!c) return 0;
    (void)hipSetDevice(c->device);
    for (Pipe &P : c->pipes)
        if (P.stream) (void)hipStreamSynchronize(P.stream);
    reasm_destroy(c->reasm);
    c->reasm = nullptr;
    for (void *p : {(void *)c->rss_reta, (void *)c->rss_ktab, (void *)c->rss_qid, (void *)c->rss_hist,
                    (void *)c->rss_partial, (void *)c->rss_total, (void *)c->rss_fuse})
        if (p) (void)hipFree(p);
    void *dev[] = {c->port_tab, c->binds, c->slots};
    for (void *p : dev) if (p) (void)hipFree(p);
    for (Pipe &P : c->pipes) {
        void *ph[] = {P.st_frames_h, P.st_desc_h};
        for (void *p : ph) if (p) (void)hipHostFree(p);
        void *pd[] = {P.hist, P.partial, P.base, P.agg, P.ticket, P.tile_cnt, P.res, P.st_frames_d,
                      P.st_desc_d, P.st_out_d, P.fuse};
        for (void *p : pd) if (p) (void)hipFree(p);
        if (P.h_res) (void)hipHostFree(P.h_res);
        if (P.tail) (void)hipEventDestroy(P.tail);
    }
    if (c->sets) {
        for (int i = 0; i < EVENT_SETS; ++i)
            for (int k = 0; k < 2 * TIMED_KERNELS; ++k) (void)hipEventDestroy(c->sets[i].ev[k]);
        delete[] c->sets;
    }
    if (c->hint) (void)hipHostFree(c->hint);
    for (Pipe &P : c->pipes)
        if (P.stream) (void)hipStreamDestroy(P.stream);
    delete c;
    return 0;
}

int udpdk_gpu_sync(udpdk_gpu_ctx *c)
{
    if (!c) return -EINVAL;
    return sync_all(c);
}

int udpdk_gpu_join(udpdk_gpu_ctx *c)
{
    if (!c) return -EINVAL;
    HIPC(c, hipSetDevice(c->device));
    return join_pipes(c);
}

int udpdk_gpu_pipeline_depth(udpdk_gpu_ctx *c, int depth)
{
    if (!c || depth < 1 || depth > MAX_PIPES) return -EINVAL;
    int rc = sync_all(c);
    if (rc) return rc;
    c->depth = depth;
    return 0;
}

int udpdk_gpu_last_hip_error(const udpdk_gpu_ctx *c) { return c ? c->last_err : 0; }

void *udpdk_gpu_stream(udpdk_gpu_ctx *c) { return c ? (void *)c->stream : nullptr; }

int udpdk_gpu_alloc(udpdk_gpu_ctx *c, size_t bytes, void **dev)
{
    if (!c || !dev) return -EINVAL;
    HIPC(c, hipSetDevice(c->device));
    // round up so 16-byte chunk loads past the last frame stay inside the allocation
    const size_t b = ((bytes ? bytes : 1) + 255) & ~(size_t)255;
    if (hipMalloc(dev, b) != hipSuccess) { (void)hipGetLastError(); *dev = nullptr; return -ENOMEM; }
    return 0;
}

int udpdk_gpu_free(udpdk_gpu_ctx *c, void *dev)
{
    if (!c) return -EINVAL;
    if (dev) HIPC(c, hipFree(dev));
    return 0;
}

int udpdk_gpu_host_alloc(udpdk_gpu_ctx *c, size_t bytes, void **host)
{
    if (!c || !host) return -EINVAL;
    if (hipHostMalloc(host, bytes ? bytes : 1, hipHostMallocDefault) != hipSuccess) {
        (void)hipGetLastError();
        *host = nullptr;
        return -ENOMEM;
    }
    return 0;
}

int udpdk_gpu_host_free(udpdk_gpu_ctx *c, void *host)
{
    if (!c) return -EINVAL;
    if (host) HIPC(c, hipHostFree(host));
    return 0;
}

int udpdk_gpu_memset(udpdk_gpu_ctx *c, void *dev, int value, size_t bytes)
{
    if (!c || (!dev && bytes)) return -EINVAL;
    if (c->depth > 1) { int rc = join_pipes(c); if (rc) return rc; }
    if (bytes) HIPC(c, hipMemsetAsync(dev, value, bytes, c->stream));
    return 0;
}

int udpdk_gpu_h2d(udpdk_gpu_ctx *c, void *dev, const void *host, size_t bytes)
{
    if (!c || ((!dev || !host) && bytes)) return -EINVAL;
    if (c->depth > 1) { int rc = join_pipes(c); if (rc) return rc; }
    if (bytes) HIPC(c, hipMemcpyAsync(dev, host, bytes, hipMemcpyHostToDevice, c->stream));
    return 0;
}

int udpdk_gpu_d2h(udpdk_gpu_ctx *c, void *host, const void *dev, size_t bytes)
{
    if (!c || ((!dev || !host) && bytes)) return -EINVAL;
    if (c->depth > 1) { int rc = join_pipes(c); if (rc) return rc; }
    if (bytes) HIPC(c, hipMemcpyAsync(host, dev, bytes, hipMemcpyDeviceToHost, c->stream));
    return 0;
}

int udpdk_gpu_bind_snapshot_upload(udpdk_gpu_ctx *c, const udpdk_bind_snapshot_t *s)
{
    if (!c || !s || !s->port_first || !s->port_count || (s->n_binds && !s->binds)) return -EINVAL;
    if (s->n_lanes == 0 || s->n_lanes > c->max_lanes || s->n_binds > UDPDK_GPU_MAX_BINDS) return -EINVAL;
    if (s->n_slots && !s->slots) return -EINVAL;
    std::vector<uint4> tab(UDPDK_UDP_PORTS, make_uint4(0, 0, 0, 0));
    uint32_t maxfan = 0, nports = 0, iport[UDPDK_INLINE_PORTS] = {};
    uint4 ient[UDPDK_INLINE_PORTS] = {};
    for (uint32_t p = 0; p < UDPDK_UDP_PORTS; ++p) {
        const uint32_t cnt = s->port_count[p];
        if (!cnt) continue;
        const uint32_t first = s->port_first[p];
        if (cnt > UDPDK_GPU_MAX_PORT_BINDS || (uint64_t)first + cnt > s->n_binds) return -EINVAL;
        const udpdk_binding_t &b0 = s->binds[first];
        tab[p] = make_uint4(cnt, first, b0.ip, (uint32_t)b0.sockfd | (b0.reuse ? 0x80000000u : 0u));
        maxfan = std::max(maxfan, cnt);
        if (nports < UDPDK_INLINE_PORTS) {
            iport[nports] = p;
            ient[nports] = tab[p];
        }
        ++nports;
    }
    std::vector<uint2> b(s->n_binds ? s->n_binds : 1);
    for (uint32_t i = 0; i < s->n_binds; ++i) {
        const udpdk_binding_t &x = s->binds[i];
        if (x.sockfd < 0 || x.sockfd > 0xFFFF) return -EINVAL;
        if (((uint32_t)x.sockfd & s->lane_mask) >= s->n_lanes) return -EINVAL;
        b[i] = make_uint2(x.ip, (uint32_t)x.sockfd | (x.reuse ? 0x80000000u : 0u));
    }
    HIPC(c, hipSetDevice(c->device));
    { int rc = sync_all(c); if (rc) return rc; }
    if (s->n_binds > c->binds_cap) {
        if (c->binds) HIPC(c, hipFree(c->binds));
        c->binds = nullptr;
        c->binds_cap = 0;
        HIPC(c, hipMalloc((void **)&c->binds, (size_t)s->n_binds * sizeof(uint2)));
        c->binds_cap = s->n_binds;
    }
    if (!c->binds) {
        HIPC(c, hipMalloc((void **)&c->binds, sizeof(uint2)));
        c->binds_cap = 1;
    }
    HIPC(c, hipMemcpy(c->port_tab, tab.data(), UDPDK_UDP_PORTS * sizeof(uint4), hipMemcpyHostToDevice));
    if (s->n_binds)
        HIPC(c, hipMemcpy(c->binds, b.data(), (size_t)s->n_binds * sizeof(uint2), hipMemcpyHostToDevice));
    if (s->n_slots) {
        if (s->n_slots > c->slots_cap) {
            if (c->slots) HIPC(c, hipFree(c->slots));
            c->slots = nullptr;
            HIPC(c, hipMalloc((void **)&c->slots, (size_t)s->n_slots * sizeof(uint4)));
            c->slots_cap = s->n_slots;
        }
        std::vector<uint4> sl(s->n_slots);
        for (uint32_t i = 0; i < s->n_slots; ++i)
            sl[i] = make_uint4(s->slots[i].ip, s->slots[i].udp_port & 0xFFFFu, s->slots[i].bound ? 1u : 0u, 0u);
        HIPC(c, hipMemcpy(c->slots, sl.data(), (size_t)s->n_slots * sizeof(uint4), hipMemcpyHostToDevice));
    }
    c->n_slots = s->n_slots;
    c->n_lanes = s->n_lanes;
    c->lane_mask = s->lane_mask;
    uint32_t kb = 0;
    while ((1u << kb) < s->n_lanes) ++kb;
    c->key_bits = kb;
    c->max_fanout = maxfan;
    c->inl = nports <= UDPDK_INLINE_PORTS && !c->no_inline ? 1u : 0u;
    c->n_inl = c->inl ? nports : 0u;
    for (uint32_t k = 0; k < UDPDK_INLINE_PORTS; ++k) {
        c->inl_port[k] = iport[k];
        c->inl_ent[k] = ient[k];
    }
    c->have_snapshot = true;
    return 0;
}

int udpdk_gpu_timing_enable(udpdk_gpu_ctx *c, int enable)
{
    if (!c) return -EINVAL;
    if (enable && !c->sets) {
        c->sets = new (std::nothrow) TimingSet[EVENT_SETS];
        if (!c->sets) return -ENOMEM;
        for (int i = 0; i < EVENT_SETS; ++i)
            for (int k = 0; k < 2 * TIMED_KERNELS; ++k) HIPC(c, hipEventCreate(&c->sets[i].ev[k]));
    }
    c->timing_every = enable > 0 ? (uint32_t)enable : 0u;
    c->timing_calls = 0;
    return 0;
}

int udpdk_gpu_timing_read(udpdk_gpu_ctx *c, double ms[UDPDK_N_KERNEL_IDS],
                          uint32_t launches[UDPDK_N_KERNEL_IDS])
{
    if (!c) return -EINVAL;
    int rc = fold_timing(c);
    if (rc) return rc;
    for (int k = 0; k < UDPDK_N_KERNEL_IDS; ++k) {
        if (ms) ms[k] = c->ms[k];
        if (launches) launches[k] = c->launches[k];
        c->ms[k] = 0;
        c->launches[k] = 0;
    }
    return 0;
}

namespace {

int rx_on_pipe(udpdk_gpu_ctx *c, int pipe, const udpdk_rx_batch_t *bt, const udpdk_rx_out_t *o)
{
    if (!c || !bt || !o || !c->have_snapshot) return -EINVAL;
    if (bt->n > c->max_frames || bt->frames_bytes >= (1ull << 32)) return -EINVAL;
    if (bt->n && (!bt->frames_dev || !bt->offset_dev || !bt->length_dev)) return -EINVAL;
    if (((uintptr_t)bt->frames_dev & 15u) != 0) return -EINVAL;
    if (!o->meta_dev && bt->n) return -EINVAL;
    if (!o->lane_off_dev || (!o->lane_pkt_dev && o->lane_cap)) return -EINVAL;
    HIPC(c, hipSetDevice(c->device));
    Pipe &P = c->pipes[pipe];
    const hipStream_t st = P.stream;
    P.dirty = true;
    c->last_pipe = pipe;
    const uint32_t S = c->n_lanes;
    TimingSet *ts = nullptr;
    if (c->timing_every && (c->timing_calls++ % c->timing_every) == 0) {
        if (c->n_sets_used == EVENT_SETS) { int rc = fold_timing(c); if (rc) return rc; }
        ts = &c->sets[c->n_sets_used++];
    }
    P.last_lane_cap = o->lane_cap;
    if (bt->n == 0) {
        HIPC(c, hipMemsetAsync(o->lane_off_dev, 0, (size_t)(S + 1) * 4, st));
        HIPC(c, hipMemsetAsync(P.res, 0, sizeof(DevResult), st));
        P.last_tiles = 0;
        if (ts) c->n_sets_used--;                         // nothing was launched
        return 0;
    }
    uint32_t T, tiles;
    geometry(bt->n, S, &T, &tiles, c->geo_cap);
    if (S == 1 && c->max_fanout <= 1 && c->one_lane_tile) {   // diagnostic override
        T = c->one_lane_tile;
        tiles = std::max<uint32_t>(1u, ceil_div(bt->n, T));
    }
    const uint64_t E = (uint64_t)S * tiles;
    if (E > c->hist_cap || tiles > c->tiles_cap) return -EINVAL;
    // single lane, no fan-out: classify + rx_compact1; otherwise classify + scan + scatter
    const bool one_lane = S == 1 && c->max_fanout <= 1;
    P.last_tiles = tiles;

    // the one-launch column scan while each thread's tile chunk fits its registers; beyond (very
    // large batches over few lanes) the reduce / top / down chain over u32 counts
    const bool cols = !one_lane && tiles <= SCAN_COLS_MAX_TILES;
    // u16 tile histograms where a lane's count per tile cannot pass 2^16 (no fan-out): half the
    // bytes classify stores at its tile ends and the scan reads
    const bool hist16 = cols && c->max_fanout <= 1;
    RxArgs ra;
    memset(&ra, 0, sizeof(ra));
    ra.hist16 = hist16 ? 1u : 0u;
    ra.frames = bt->frames_dev;
    ra.offset = bt->offset_dev;
    ra.length = bt->length_dev;
    ra.ptype = bt->ptype_dev;
    ra.port_tab = c->port_tab;
    ra.binds = c->binds;
    ra.meta = o->meta_dev;
    ra.hist = P.hist;
    ra.tile_cnt = P.tile_cnt;
    ra.dbg = c->dbg;
    ra.key_bits = c->key_bits;
    ra.frames_bytes = (uint32_t)bt->frames_bytes;
    ra.rsrc_bytes = frames_rsrc_bytes(bt->frames_bytes);
    ra.n = bt->n;
    ra.tile_frames = T;
    ra.n_tiles = tiles;
    ra.lane_mask = c->lane_mask;
    ra.n_lanes = S;
    ra.inl = c->inl;
    ra.n_inl = c->n_inl;
    for (uint32_t k = 0; k < UDPDK_INLINE_PORTS; ++k) {
        ra.inl_port[k] = c->inl_port[k];
        ra.inl_ent[k] = c->inl_ent[k];
    }
    // speculative single-lane entries from classify (see RxArgs::spec_pkt)
    const bool spec = UDPDK_SPEC_COMPACT && one_lane && T == (uint32_t)RX_ROUND && CLS_BLOCK * 4 == RX_ROUND;
    ra.spec_pkt = spec ? o->lane_pkt_dev : nullptr;
    ra.spec_cap = spec ? o->lane_cap : 0u;
    if (spec && ++P.spec_epoch == 0) P.spec_epoch = 1;       // 0: the zeroed word's tag
    ra.spec_nonfull = spec ? P.res->nonfull : nullptr;
    ra.spec_epoch = P.spec_epoch;
    // kernel form from the hints of the recent calls (RxArgs::hint)
    if (++c->rx_seq == 0) c->rx_seq = 1;
    const uint32_t seq = c->rx_seq;
    // measured against the latest call the GPU has reached (the host may run tens of calls ahead)
    const uint32_t done = __atomic_load_n(&c->hint[UDPDK_HINT_DONE], __ATOMIC_RELAXED);
    auto recent = [&](int k) {
        const uint32_t v = __atomic_load_n(&c->hint[k], __ATOMIC_RELAXED);
        return v != 0u && (int32_t)(done - v) <= (int32_t)UDPDK_HINT_WINDOW;
    };
    ra.hint = c->hint;
    ra.seq = seq;
    // fused completion whenever it applies: a call with a short tile repairs its lane inside the
    // same launch (classify_complete), so no form switching follows a stray frame
    const bool fuse = spec && tiles <= UDPDK_FUSE_MAX_TILES && c->force_fuse != 0;
    const int tailg = c->force_tailg ? c->force_tailg : (one_lane && !recent(UDPDK_HINT_TAIL)) ? 1 : 2;
    if (c->trace)
        fprintf(stderr, "udpdk_gpu_rx seq %u done %u hint tail %u nonfull %u -> classify<%d>%s\n", seq,
                done, c->hint[UDPDK_HINT_TAIL], c->hint[UDPDK_HINT_NONFULL], tailg, fuse ? " fused" : "");
    ra.fuse = fuse ? P.fuse : nullptr;
    ra.lane_off = o->lane_off_dev;
    ra.total = &P.res->total;

    if (ts) for (int k = 0; k < TIMED_KERNELS; ++k) ts->used[k] = false;
    // tiles of several rounds (many lanes: config 5's 8192-frame tiles) take the form that loads
    // each next round's descriptors a round ahead
    const bool mr = c->force_mr >= 0 ? c->force_mr == 1 : T > (uint32_t)RX_ROUND;
    auto cls = tailg == 1 ? (mr ? rx_classify<1, 1> : rx_classify<1, 0>) : (mr ? rx_classify<2, 1> : rx_classify<2, 0>);
    // the span sweep: the long-frame form of one-round tiles (its LDS ring after the carve)
    const uint32_t cls_lds = classify_lds_bytes(S, T, hist16);
    ra.span = tailg == 2 && !mr && T == (uint32_t)RX_ROUND && !c->no_span &&
              cls_lds + SPAN_LDS_BYTES <= 160u * 1024u - 1024u ? 1u : 0u;
    HIPC(c, launch(st, ts, 0, true, true, cls, dim3(tiles),
                   dim3(CLS_BLOCK), cls_lds + (ra.span ? SPAN_LDS_BYTES : 0u), ra));
    if (fuse) return 0;                        // the last workgroup completed the lane
    if (one_lane) {
        Compact1Args ca;
        ca.meta = o->meta_dev;
        ca.tile_count = P.hist;
        ca.lane_pkt = o->lane_pkt_dev;
        ca.lane_off = o->lane_off_dev;
        ca.total = &P.res->total;
        ca.n = bt->n;
        ca.tile_frames = T;
        ca.n_tiles = tiles;
        ca.lane_cap = o->lane_cap;
        ca.base = nullptr;
        ca.spec = spec ? 1u : 0u;
        ca.spec_nonfull = P.res->nonfull;
        ca.spec_epoch = P.spec_epoch;
        ca.hint = c->hint;
        ca.seq = seq;
        if (tiles > COMPACT1_DIRECT_TILES && tiles <= c->partial_cap) {
            // past a few thousand tiles each workgroup's sum over its predecessors costs more
            // than one extra launch scanning the counts once
            hipLaunchKernelGGL(rx_tile_base, dim3(1), dim3(1024), 0, st, (const uint32_t *)P.hist,
                               P.partial, tiles);
            HIPC(c, hipGetLastError());
            ca.base = P.partial;
        }
        // speculative: grid-stride over the tiles after the call's first flagged one (usually
        // none); the grid size does not change the all-full call's cost (same-box A/B: 32, 128
        // and 1024 workgroups all 4.8-5.0 us), 256 keeps a flagged call's rewrite wide
        const uint32_t cgrid = spec ? std::min<uint32_t>(tiles, UDPDK_COMPACT1_SPEC_GRID) : tiles;
        HIPC(c, launch(st, ts, 2, true, true, rx_compact1, dim3(cgrid), dim3(RX_BLOCK), 0u, ca));
        return 0;
    }

    // rx_scatterw: G classify tiles per scatter workgroup while the scatter tile stays within
    // UDPDK_SCATTER_GROUP_FRAMES, its (frame, position) pairs fit the LDS counter region (8 B each
    // in 2 W S bytes) and the grid keeps UDPDK_SCATTER_MIN_WG workgroups; the column scan then
    // writes only the base rows of each group's first tile
    const bool scatterw = c->max_fanout <= 1 && S <= SCATTERW_MAX_LANES;
    uint32_t G = 1, W = SCATTER_WAVES;
    while (scatterw && G < tiles) {
        const uint32_t g2 = 2 * G, f2 = g2 * T;
        const uint32_t w2 = f2 > 64u * SCATTER_WAVES * SCATTERW_MV ? 2 * SCATTER_WAVES : SCATTER_WAVES;
        if (f2 > c->scatter_group_frames || f2 > 64u * w2 * SCATTERW_MV || 8ull * f2 > 2ull * w2 * S ||
            (S & 1u) || ceil_div(tiles, g2) < c->scatter_min_wg)
            break;
        G = g2;
        W = w2;
    }

    ScanArgs sa;
    memset(&sa, 0, sizeof(sa));
    sa.row_mask = cols ? G - 1u : 0u;
    sa.dbg = c->dbg;
    sa.hist = P.hist;
    sa.partial = P.partial;
    sa.lane_off = o->lane_off_dev;
    sa.total = &P.res->total;
    sa.n_elems = (uint32_t)E;
    sa.n_tiles = tiles;
    sa.n_lanes = S;
    sa.base = P.base;
    sa.agg = P.agg;
    sa.ticket = P.ticket;
    sa.epoch = ++P.epoch ? P.epoch : ++P.epoch;        // 0 marks a never-written look-back word
    sa.hist16 = ra.hist16;
    if (cols) {
        // lanes per workgroup: as many as the chunking allows (<= 64, 256 B rows), then fewer
        // until the grid has >= UDPDK_SCAN_MIN_WG workgroups, never under 8 lanes (32 B row
        // segments). Wider rows beat more workgroups: at 1024 lanes x 1024 tiles, 16-lane
        // columns (64 workgroups) take 8.0 us, 8-lane (128) 11.9 us, 4-lane (256) 13.0 us.
        // Workgroups of 1024 threads when that still leaves >= 16-lane columns (config 5: 11.2-11.8
        // -> 7.3-7.7 us against 256 threads; more waves per CU for the column loads' latency),
        // else 512 (config 4's 1024 lanes x 1024 tiles: 10.3-10.4 -> 8.9-9.1 us)
        auto pick_lb = [&](uint32_t block) {
            const uint32_t cmin = ceil_div(tiles, scan_cols_tpt(block));
            uint32_t lb = 0;
            while ((2u << lb) <= std::min<uint32_t>(64u, block / cmin)) ++lb;
            while (lb > 3 && ceil_div(S, 1u << lb) < UDPDK_SCAN_MIN_WG) --lb;
            return lb;
        };
        const uint32_t lb1 = pick_lb(1024u);
        if (lb1 >= 4) {
            HIPC(c, launch(st, ts, 1, true, true, rx_scan_cols<1024>, dim3(ceil_div(S, 1u << lb1)),
                           dim3(1024), 0u, sa, lb1));
        } else {
            const uint32_t lb = pick_lb(512u);
            HIPC(c, launch(st, ts, 1, true, true, rx_scan_cols<512>, dim3(ceil_div(S, 1u << lb)),
                           dim3(512), 0u, sa, lb));
        }
    } else {
        const uint32_t nc = ceil_div(tiles, SCAN_COL_CHUNK);
        if ((uint64_t)nc * S > c->partial_cap) return -EINVAL;
        const dim3 grid(nc, ceil_div(S, (uint32_t)SCAN_BLOCK));
        HIPC(c, launch(st, ts, 1, true, false, rx_scan_reduce, grid, dim3(SCAN_BLOCK), 0u, sa));
        HIPC(c, launch(st, ts, 1, false, false, rx_scan_top, dim3(1), dim3(SCAN_TOP_BLOCK), 4u * S, sa, nc));
        HIPC(c, launch(st, ts, 1, false, true, rx_scan_down, grid, dim3(SCAN_BLOCK), 0u, sa));
    }

    ScatterArgs xa;
    xa.meta = o->meta_dev;
    xa.base = cols ? P.base : P.hist;
    xa.total = &P.res->total;
    xa.frames = bt->frames_dev;
    xa.offset = bt->offset_dev;
    xa.port_tab = c->port_tab;
    xa.binds = c->binds;
    xa.lane_pkt = o->lane_pkt_dev;
    xa.n = bt->n;
    xa.tile_frames = T;
    xa.n_tiles = tiles;
    xa.n_lanes = S;
    xa.lane_mask = c->lane_mask;
    xa.key_bits = c->key_bits;
    xa.lane_cap = o->lane_cap;
    xa.row_step = 1;
    xa.dbg = c->dbg;
    if (scatterw) {
        xa.tile_frames = G * T;
        xa.n_tiles = ceil_div(tiles, G);
        xa.row_step = G;
        if (W == SCATTER_WAVES)
            HIPC(c, launch(st, ts, 2, true, true, rx_scatterw<SCATTER_WAVES>, dim3(xa.n_tiles),
                           dim3(64 * SCATTER_WAVES), scatterw_lds_bytes(S), xa));
        else
            HIPC(c, launch(st, ts, 2, true, true, rx_scatterw<2 * SCATTER_WAVES>, dim3(xa.n_tiles),
                           dim3(128 * SCATTER_WAVES), scatterw_lds_bytes(S, 2 * SCATTER_WAVES), xa));
    } else
        HIPC(c, launch(st, ts, 2, true, true, rx_scatter, dim3(tiles), dim3(SCATTER1_BLOCK),
                       scatter1_lds_bytes(S), xa));
    return 0;
}

} // namespace

int udpdk_gpu_rx(udpdk_gpu_ctx *c, const udpdk_rx_batch_t *bt, const udpdk_rx_out_t *o)
{
    if (!c) return -EINVAL;
    const int pipe = c->depth > 1 ? (int)(c->rx_calls % (uint64_t)c->depth) : 0;
    const int rc = rx_on_pipe(c, pipe, bt, o);
    if (rc == 0) ++c->rx_calls;
    return rc;
}

namespace {
int enqueue_result(udpdk_gpu_ctx *c, Pipe &P);
int read_result(Pipe &P, udpdk_rx_stats_t *st);
} // namespace

int udpdk_gpu_rx_stats(udpdk_gpu_ctx *c, udpdk_rx_stats_t *st)
{
    if (!c || !st) return -EINVAL;
    if (c->last_pipe < 0) return -EINVAL;
    HIPC(c, hipSetDevice(c->device));
    Pipe &P = c->pipes[c->last_pipe];
    int rc = enqueue_result(c, P);
    if (rc) return rc;
    HIPC(c, hipStreamSynchronize(P.stream));
    return read_result(P, st);
}

namespace {

// The counter reduction and the result row (counters, delivery total) of pipe p's last call
// into its pinned mirror, on the pipe's stream.
int enqueue_result(udpdk_gpu_ctx *c, Pipe &P)
{
    P.dirty = true;
    if (P.last_tiles) {
        hipLaunchKernelGGL(rx_counters, dim3(1), dim3(256), 0, P.stream, (const uint32_t *)P.tile_cnt,
                           P.last_tiles, P.res->counters);
        HIPC(c, hipGetLastError());
    }
    HIPC(c, hipMemcpyAsync(P.h_res, P.res, sizeof(DevResult), hipMemcpyDeviceToHost, P.stream));
    return 0;
}

int read_result(Pipe &P, udpdk_rx_stats_t *st)
{
    for (int k = 0; k < UDPDK_N_COUNTERS; ++k) st->counters[k] = P.h_res->counters[k];
    st->deliveries = P.h_res->total;
    st->overflow = st->deliveries > P.last_lane_cap ? 1u : 0u;
    return st->overflow ? -ENOSPC : 0;
}

// Wait for pipe p's outstanding host call, if any, and fill its stats.
int finish_host(udpdk_gpu_ctx *c, Pipe &P)
{
    if (!P.host_stats) return 0;
    udpdk_rx_stats_t *st = P.host_stats;
    P.host_stats = nullptr;
    HIPC(c, hipStreamSynchronize(P.stream));
    return read_result(P, st);
}

// One host-resident batch on pipe p, all on the pipe's stream: (pageable input: a host copy
// into pinned staging first) H2D of frames + descriptors, the RX pipeline, the counter
// reduction, D2H of the result row, meta, lane_off and lane_pkt[0, lane_cap).
int enqueue_host(udpdk_gpu_ctx *c, int pipe, const uint8_t *frames_host, uint64_t frames_bytes,
                 const uint32_t *offset_host, const uint16_t *length_host,
                 const uint32_t *ptype_host, uint32_t n, uint32_t *meta_host,
                 uint32_t *lane_off_host, uint32_t *lane_pkt_host, uint32_t lane_cap,
                 udpdk_rx_stats_t *stats, bool copy_lanes = true, uint32_t offset_base = 0)
{
    if (!stats || !lane_off_host || n > c->max_frames) return -EINVAL;
    if (n && (!frames_host || !offset_host || !length_host || !meta_host)) return -EINVAL;
    if (lane_cap && !lane_pkt_host) return -EINVAL;
    if (frames_bytes >= (1ull << 32)) return -EINVAL;
    Pipe &P = c->pipes[pipe];
    const hipStream_t s = P.stream;
    P.dirty = true;
    // frames + the tailroom the kernels may read past them (UDPDK_GPU_FRAMES_TAILROOM)
    const size_t fb = (((size_t)frames_bytes + 255) & ~(size_t)255) + UDPDK_GPU_FRAMES_TAILROOM;
    const size_t desc = (size_t)n * 10 + 64;
    const size_t outb = (size_t)n * 4 + (size_t)(c->n_lanes + 1) * 4 + (size_t)lane_cap * 4 + 64;
    int rc;
    // The frames are expected in pinned memory (DPDK hugepage mbufs registered with the
    // runtime); pageable input is copied into a pinned staging buffer first.
    // (a chunk of a larger buffer: the allocation is looked up by the buffer's own start)
    hipPointerAttribute_t attr;
    const bool pinned = n && hipPointerGetAttributes(&attr, frames_host - offset_base) == hipSuccess &&
                        attr.type == hipMemoryTypeHost;
    (void)hipGetLastError();
    if ((rc = ensure_dev(c, (void **)&P.st_frames_d, &P.st_frames_dcap, fb))) return rc;
    if (n && !pinned &&
        (rc = ensure_host(c, (void **)&P.st_frames_h, &P.st_frames_hcap, fb))) return rc;
    if ((rc = ensure_dev(c, (void **)&P.st_desc_d, &P.st_desc_dcap, desc))) return rc;
    if ((rc = ensure_host(c, (void **)&P.st_desc_h, &P.st_desc_hcap, desc))) return rc;
    if ((rc = ensure_dev(c, (void **)&P.st_out_d, &P.st_out_cap, outb))) return rc;
    const uint8_t *src = frames_host;
    if (n && !pinned) {
        memcpy(P.st_frames_h, frames_host, frames_bytes);
        src = P.st_frames_h;
    }
    uint8_t *dh = P.st_desc_h;
    if (offset_base) {                          // a chunk of a larger batch: offsets rebased
        uint32_t *o = (uint32_t *)dh;
        for (uint32_t i = 0; i < n; ++i) o[i] = offset_host[i] - offset_base;
    } else {
        memcpy(dh, offset_host, (size_t)n * 4);
    }
    memcpy(dh + (size_t)n * 4, length_host, (size_t)n * 2);
    const size_t pt_off = ((size_t)n * 6 + 15) & ~(size_t)15;
    if (ptype_host) memcpy(dh + pt_off, ptype_host, (size_t)n * 4);
    if (n) HIPC(c, hipMemcpyAsync(P.st_frames_d, src, frames_bytes, hipMemcpyHostToDevice, s));
    HIPC(c, hipMemcpyAsync(P.st_desc_d, dh, pt_off + (ptype_host ? (size_t)n * 4 : 0),
                           hipMemcpyHostToDevice, s));
    uint32_t *meta_d = (uint32_t *)P.st_out_d;
    uint32_t *off_d = meta_d + n;
    uint32_t *pkt_d = off_d + c->n_lanes + 1;
    udpdk_rx_batch_t b = {P.st_frames_d, frames_bytes, (const uint32_t *)P.st_desc_d,
                          (const uint16_t *)(P.st_desc_d + (size_t)n * 4),
                          ptype_host ? (const uint32_t *)(P.st_desc_d + pt_off) : nullptr, n};
    udpdk_rx_out_t o = {meta_d, off_d, pkt_d, lane_cap};
    if ((rc = rx_on_pipe(c, pipe, &b, &o))) return rc;
    if ((rc = enqueue_result(c, P))) return rc;
    if (n) HIPC(c, hipMemcpyAsync(meta_host, meta_d, (size_t)n * 4, hipMemcpyDeviceToHost, s));
    HIPC(c, hipMemcpyAsync(lane_off_host, off_d, (size_t)(c->n_lanes + 1) * 4, hipMemcpyDeviceToHost, s));
    if (lane_cap && copy_lanes)
        HIPC(c, hipMemcpyAsync(lane_pkt_host, pkt_d, (size_t)lane_cap * 4, hipMemcpyDeviceToHost, s));
    P.host_stats = stats;
    P.staged = b;
    P.staged_meta = meta_d;
    return 0;
}

int finish_all_host(udpdk_gpu_ctx *c)
{
    int rc = 0;
    const int d = std::max(1, c->depth);
    for (int k = 0; k < d; ++k) {          // oldest first
        Pipe &P = c->pipes[(c->host_calls + (uint64_t)k) % (uint64_t)d];
        const int r = finish_host(c, P);
        if (r && !rc) rc = r;
    }
    return rc;
}

} // namespace

int udpdk_gpu_rx_host(udpdk_gpu_ctx *c, const uint8_t *frames_host, uint64_t frames_bytes,
                      const uint32_t *offset_host, const uint16_t *length_host,
                      const uint32_t *ptype_host, uint32_t n, uint32_t *meta_host,
                      uint32_t *lane_off_host, uint32_t *lane_pkt_host, uint32_t lane_cap,
                      udpdk_rx_stats_t *stats)
{
    if (!c) return -EINVAL;
    HIPC(c, hipSetDevice(c->device));
    int rc = finish_all_host(c);
    if (rc && rc != -ENOSPC) return rc;
    if (c->depth > 1) { int r = join_pipes(c); if (r) return r; }
    // synchronous: the lane entries come back after the counters, only as many as were made
    if ((rc = enqueue_host(c, 0, frames_host, frames_bytes, offset_host, length_host, ptype_host, n,
                           meta_host, lane_off_host, lane_pkt_host, lane_cap, stats, false))) return rc;
    Pipe &P = c->pipes[0];
    rc = finish_host(c, P);
    if (rc && rc != -ENOSPC) return rc;
    const uint32_t d = std::min(stats->deliveries, lane_cap);
    if (d) {
        const uint32_t *pkt_d = P.staged_meta + n + c->n_lanes + 1;
        HIPC(c, hipMemcpyAsync(lane_pkt_host, pkt_d, (size_t)d * 4, hipMemcpyDeviceToHost, P.stream));
        HIPC(c, hipStreamSynchronize(P.stream));
    }
    return rc;
}

int udpdk_gpu_rx_host_batch(udpdk_gpu_ctx *c, udpdk_rx_batch_t *batch, const uint32_t **meta_dev)
{
    if (!c || !batch) return -EINVAL;
    const Pipe &P = c->pipes[0];
    if (!P.staged_meta) return -ENOENT;
    *batch = P.staged;
    if (meta_dev) *meta_dev = P.staged_meta;
    return 0;
}

int udpdk_gpu_rx_host_async(udpdk_gpu_ctx *c, const uint8_t *frames_host, uint64_t frames_bytes,
                            const uint32_t *offset_host, const uint16_t *length_host,
                            const uint32_t *ptype_host, uint32_t n, uint32_t *meta_host,
                            uint32_t *lane_off_host, uint32_t *lane_pkt_host, uint32_t lane_cap,
                            udpdk_rx_stats_t *stats)
{
    if (!c) return -EINVAL;
    HIPC(c, hipSetDevice(c->device));
    const int pipe = (int)(c->host_calls % (uint64_t)std::max(1, c->depth));
    Pipe &P = c->pipes[pipe];
    int rc = finish_host(c, P);                 // at most `depth` calls outstanding
    if (rc && rc != -ENOSPC) return rc;
    if ((rc = enqueue_host(c, pipe, frames_host, frames_bytes, offset_host, length_host, ptype_host,
                           n, meta_host, lane_off_host, lane_pkt_host, lane_cap, stats))) return rc;
    ++c->host_calls;
    return 0;
}

int udpdk_gpu_rx_host_wait(udpdk_gpu_ctx *c)
{
    if (!c) return -EINVAL;
    HIPC(c, hipSetDevice(c->device));
    return finish_all_host(c);
}

namespace {

static int rx_gather_launch(udpdk_gpu_ctx *c, const udpdk_rx_batch_t *bt, const uint32_t *lane_pkt_dev,
                     uint32_t first, uint32_t count, const uint32_t *slot_off_dev,
                     const udpdk_rx_gather_t *o, int pipe = -1)
{
    if (!c || !bt || !o) return -EINVAL;
    if (!count) return 0;
    if (!bt->n || !bt->frames_dev || !bt->offset_dev || !bt->length_dev || !lane_pkt_dev ||
        !o->payload_dev || !o->len_dev || !o->src_ip_dev || !o->src_port_dev) return -EINVAL;
    if (!slot_off_dev && (o->slot_bytes < 16u || (o->slot_bytes & 15u))) return -EINVAL;
    if ((uintptr_t)o->payload_dev & 15u) return -EINVAL;
    if (bt->frames_bytes >= (1ull << 32) || (uint64_t)first + count > 0xFFFFFFFFull) return -EINVAL;
    HIPC(c, hipSetDevice(c->device));
    // pipe >= 0: on that pipe's stream, after its own work only (udpdk_gpu_pipe_gather_packed)
    if (pipe < 0 && c->depth > 1) { int r = join_pipes(c); if (r) return r; }
    const hipStream_t gst = pipe < 0 ? c->stream : c->pipes[pipe].stream;
    if (pipe >= 0) c->pipes[pipe].dirty = true;
    GatherArgs ga;
    ga.frames = bt->frames_dev;
    ga.offset = bt->offset_dev;
    ga.length = bt->length_dev;
    ga.lane_pkt = lane_pkt_dev;
    ga.payload = o->payload_dev;
    ga.len_out = o->len_dev;
    ga.src_ip = o->src_ip_dev;
    ga.src_port = o->src_port_dev;
    ga.first = first;
    ga.count = count;
    ga.slot_bytes = o->slot_bytes;
    ga.rsrc_bytes = frames_rsrc_bytes(bt->frames_bytes);
    ga.n = bt->n;
    ga.slot_off = slot_off_dev;
    const uint32_t grid = std::min<uint32_t>(ceil_div(count, GATHER_BLOCK), 16384);
    hipEvent_t e0 = nullptr, e1 = nullptr;
    if (c->timing_every) {
        HIPC(c, hipEventCreate(&e0));
        HIPC(c, hipEventCreate(&e1));
        HIPC(c, hipEventRecord(e0, gst));
    }
    hipLaunchKernelGGL(rx_gather, dim3(grid), dim3(GATHER_BLOCK), 0, gst, ga);
    HIPC(c, hipGetLastError());
    if (c->timing_every) {
        HIPC(c, hipEventRecord(e1, gst));
        HIPC(c, hipEventSynchronize(e1));
        float ms = 0;
        HIPC(c, hipEventElapsedTime(&ms, e0, e1));
        c->ms[UDPDK_K_RX_GATHER] += ms;
        c->launches[UDPDK_K_RX_GATHER]++;
        (void)hipEventDestroy(e0);
        (void)hipEventDestroy(e1);
    }
    return 0;
}

} // namespace

int udpdk_gpu_rx_gather(udpdk_gpu_ctx *c, const udpdk_rx_batch_t *bt, const uint32_t *lane_pkt_dev,
                        uint32_t first, uint32_t count, const udpdk_rx_gather_t *o)
{
    return rx_gather_launch(c, bt, lane_pkt_dev, first, count, nullptr, o);
}

int udpdk_gpu_rx_gather_packed(udpdk_gpu_ctx *c, const udpdk_rx_batch_t *bt, const uint32_t *lane_pkt_dev,
                               uint32_t first, uint32_t count, const uint32_t *slot_off_dev,
                               const udpdk_rx_gather_t *o)
{
    if (count && !slot_off_dev) return -EINVAL;
    return rx_gather_launch(c, bt, lane_pkt_dev, first, count, slot_off_dev, o);
}

// ---- poller internals: udpdk_poll_rx's pipelined form (explicit pipes, no cross-pipe joins) ----
int udpdk_gpu_pipe_rx_host(udpdk_gpu_ctx *c, int pipe, const uint8_t *frames_host, uint64_t frames_bytes,
                           const uint32_t *offset_host, uint32_t offset_base, const uint16_t *length_host,
                           const uint32_t *ptype_host, uint32_t n, uint32_t *meta_host,
                           uint32_t *lane_off_host, uint32_t *lane_pkt_host, uint32_t lane_cap,
                           udpdk_rx_stats_t *stats)
{
    if (!c || pipe < 1 || pipe >= MAX_PIPES) return -EINVAL;
    HIPC(c, hipSetDevice(c->device));
    int rc = finish_host(c, c->pipes[pipe]);
    if (rc && rc != -ENOSPC) return rc;
    return enqueue_host(c, pipe, frames_host, frames_bytes, offset_host, length_host, ptype_host, n,
                        meta_host, lane_off_host, lane_pkt_host, lane_cap, stats, true, offset_base);
}

int udpdk_gpu_pipe_wait(udpdk_gpu_ctx *c, int pipe)
{
    if (!c || pipe < 1 || pipe >= MAX_PIPES) return -EINVAL;
    HIPC(c, hipSetDevice(c->device));
    Pipe &P = c->pipes[pipe];
    const int rc = finish_host(c, P);
    HIPC(c, hipStreamSynchronize(P.stream));
    return rc;
}

int udpdk_gpu_pipe_batch(udpdk_gpu_ctx *c, int pipe, udpdk_rx_batch_t *batch, const uint32_t **meta_dev)
{
    if (!c || !batch || pipe < 1 || pipe >= MAX_PIPES) return -EINVAL;
    const Pipe &P = c->pipes[pipe];
    if (!P.staged_meta) return -ENOENT;
    *batch = P.staged;
    if (meta_dev) *meta_dev = P.staged_meta;
    return 0;
}

// (explicit directions: hipMemcpyDefault made the runtime block the caller on these D2H copies
// into pinned slabs, 8-10 ms of a pipelined poll's issue time)
static int pipe_copy(udpdk_gpu_ctx *c, int pipe, void *dst, const void *src, size_t bytes, hipMemcpyKind kind)
{
    if (!c || pipe < 1 || pipe >= MAX_PIPES || ((!dst || !src) && bytes)) return -EINVAL;
    HIPC(c, hipSetDevice(c->device));
    c->pipes[pipe].dirty = true;
    if (bytes) HIPC(c, hipMemcpyAsync(dst, src, bytes, kind, c->pipes[pipe].stream));
    return 0;
}

int udpdk_gpu_pipe_h2d(udpdk_gpu_ctx *c, int pipe, void *dev, const void *host, size_t bytes)
{
    return pipe_copy(c, pipe, dev, host, bytes, hipMemcpyHostToDevice);
}

int udpdk_gpu_pipe_d2h(udpdk_gpu_ctx *c, int pipe, void *host, const void *dev, size_t bytes)
{
    return pipe_copy(c, pipe, host, dev, bytes, hipMemcpyDeviceToHost);
}

int udpdk_gpu_pipe_gather_packed(udpdk_gpu_ctx *c, int pipe, const udpdk_rx_batch_t *bt,
                                 const uint32_t *lane_pkt_dev, uint32_t first, uint32_t count,
                                 const uint32_t *slot_off_dev, const udpdk_rx_gather_t *o)
{
    if (!c || pipe < 1 || pipe >= MAX_PIPES || (count && !slot_off_dev)) return -EINVAL;
    return rx_gather_launch(c, bt, lane_pkt_dev, first, count, slot_off_dev, o, pipe);
}

int udpdk_gpu_rss_default_conf(udpdk_rss_conf_t *conf, uint32_t n_queues)
{
    static const uint8_t key[UDPDK_RSS_KEY_BYTES] = {
        0x6d, 0x5a, 0x56, 0xda, 0x25, 0x5b, 0x0e, 0xc2, 0x41, 0x67, 0x25, 0x3d, 0x43, 0xa3,
        0x8f, 0xb0, 0xd0, 0xca, 0x2b, 0xcb, 0xae, 0x7b, 0x30, 0xb4, 0x77, 0xcb, 0x2d, 0xa3,
        0x80, 0x30, 0xf2, 0x0c, 0x6a, 0x42, 0xb7, 0x3b, 0xbe, 0xac, 0x01, 0xfa};
    if (!conf || !n_queues || n_queues > UDPDK_RSS_MAX_QUEUES) return -EINVAL;
    memset(conf, 0, sizeof(*conf));
    memcpy(conf->key, key, sizeof(key));
    conf->hash_types = UDPDK_RSS_IPV4 | UDPDK_RSS_NONFRAG_IPV4_UDP;
    conf->n_queues = n_queues;
    conf->reta_size = 128;
    for (uint32_t i = 0; i < conf->reta_size; ++i) conf->reta[i] = (uint16_t)(i % n_queues);
    return 0;
}

int udpdk_gpu_rss_config(udpdk_gpu_ctx *c, const udpdk_rss_conf_t *conf)
{
    if (!c || !conf) return -EINVAL;
    if (!conf->n_queues || conf->n_queues > UDPDK_RSS_MAX_QUEUES || !conf->reta_size ||
        conf->reta_size > UDPDK_RSS_RETA_MAX || (conf->reta_size & (conf->reta_size - 1)) ||
        (conf->hash_types & ~3u))
        return -EINVAL;
    for (uint32_t i = 0; i < conf->reta_size; ++i)
        if (conf->reta[i] >= conf->n_queues) return -EINVAL;
    HIPC(c, hipSetDevice(c->device));
    { int r = join_pipes(c); if (r) return r; }
    HIPC(c, hipStreamSynchronize(c->stream));
    const uint32_t tiles = ceil_div(std::max<uint32_t>(c->max_frames, 1), RSS_TILE);
    if (!c->rss_reta) {
        HIPC(c, hipMalloc((void **)&c->rss_reta, RSS_RETA_MAX * sizeof(uint16_t)));
        HIPC(c, hipMalloc((void **)&c->rss_ktab, 12 * 256 * sizeof(uint32_t)));
        HIPC(c, hipMalloc((void **)&c->rss_qid, std::max<uint32_t>(c->max_frames, 1)));
        HIPC(c, hipMalloc((void **)&c->rss_hist, (size_t)tiles * RSS_MAX_QUEUES * 4));
        HIPC(c, hipMalloc((void **)&c->rss_partial, (size_t)ceil_div(tiles, SCAN_COL_CHUNK) * RSS_MAX_QUEUES * 4));
        HIPC(c, hipMalloc((void **)&c->rss_total, 64));
        HIPC(c, hipMalloc((void **)&c->rss_fuse, FUSE_BYTES));
        HIPC(c, hipMemset(c->rss_fuse, 0, FUSE_BYTES));
    }
    {
        const char *e = getenv("UDPDK_RSS_FUSE");
        c->rss_no_fuse = e && atoi(e) == 0;
    }
    HIPC(c, hipMemcpy(c->rss_reta, conf->reta, conf->reta_size * sizeof(uint16_t), hipMemcpyHostToDevice));
    // Toeplitz key windows per (input byte position, byte value): win(b) = key bits [b, b + 32)
    // MSB first; the hash of a 12-byte input is the XOR of 12 table entries
    {
        std::vector<uint32_t> tab(12 * 256);
        auto win = [&](uint32_t b) {
            uint64_t w = 0;
            for (uint32_t k = 0; k < 5; ++k) w = (w << 8) | conf->key[(b >> 3) + k];
            return (uint32_t)(w >> (8u - (b & 7u)));
        };
        for (uint32_t p = 0; p < 12; ++p)
            for (uint32_t v = 0; v < 256; ++v) {
                uint32_t h = 0;
                for (uint32_t j = 0; j < 8; ++j)
                    if ((v >> (7u - j)) & 1u) h ^= win(8u * p + j);
                tab[p * 256 + v] = h;
            }
        HIPC(c, hipMemcpy(c->rss_ktab, tab.data(), tab.size() * sizeof(uint32_t), hipMemcpyHostToDevice));
    }
    RssArgs &r = c->rss;
    memset(&r, 0, sizeof(r));
    r.reta = c->rss_reta;
    r.ktab = c->rss_ktab;
    r.qid = c->rss_qid;
    r.hist = c->rss_hist;
    r.reta_size = conf->reta_size;
    r.n_queues = conf->n_queues;
    uint32_t qb = 0;
    while ((1u << qb) < conf->n_queues) ++qb;
    r.q_bits = qb;
    r.hash_types = conf->hash_types;
    c->rss_ready = true;
    return 0;
}

int udpdk_gpu_rss(udpdk_gpu_ctx *c, const udpdk_rx_batch_t *bt, const udpdk_rss_out_t *o)
{
    if (!c || !bt || !o || !c->rss_ready) return -EINVAL;
    if (bt->n > c->max_frames || bt->frames_bytes >= (1ull << 32)) return -EINVAL;
    if (bt->n && (!bt->frames_dev || !bt->offset_dev || !bt->length_dev || !o->hash_dev ||
                  !o->queue_off_dev || !o->queue_pkt_dev))
        return -EINVAL;
    if (!o->queue_off_dev) return -EINVAL;
    HIPC(c, hipSetDevice(c->device));
    { int r = join_pipes(c); if (r) return r; }
    hipStream_t st = c->stream;
    RssArgs a = c->rss;
    const uint32_t S = a.n_queues;
    if (!bt->n) {
        HIPC(c, hipMemsetAsync(o->queue_off_dev, 0, (S + 1) * sizeof(uint32_t), st));
        return 0;
    }
    a.frames = bt->frames_dev;
    a.offset = bt->offset_dev;
    a.length = bt->length_dev;
    a.ptype = bt->ptype_dev;
    a.hash = o->hash_dev;
    a.queue_pkt = o->queue_pkt_dev;
    a.frames_bytes = bt->frames_bytes;
    a.rsrc_bytes = frames_rsrc_bytes(bt->frames_bytes);
    a.n = bt->n;
    const uint32_t tiles = ceil_div(bt->n, RSS_TILE);
    a.n_tiles = tiles;
    a.qmajor = tiles * S <= RSS_BASE_MAX ? 1u : 0u;
    // queue-major histogram: the last rss_hash workgroup scans it (no rss_base launch)
    // (only for small histograms: at 4 M frames x 8 queues the one-workgroup tail scan of 32 K
    // entries cost more than the 1024-thread rss_base launch, 90.7 vs 84.7 us per call; at 1 M
    // frames 25.5 vs 26.0, same-box A/B)
    const bool fuse = a.qmajor && !c->rss_no_fuse && tiles * S <= RSS_FUSE_MAX_ENTRIES;
    a.fuse = fuse ? c->rss_fuse : nullptr;
    a.queue_off = o->queue_off_dev;
    a.total = c->rss_total;
    hipLaunchKernelGGL(rss_hash, dim3(tiles), dim3(RSS_BLOCK), 0, st, a);
    HIPC(c, hipGetLastError());
    ScanArgs sa;
    sa.hist = c->rss_hist;
    sa.partial = c->rss_partial;
    sa.lane_off = o->queue_off_dev;
    sa.total = c->rss_total;
    sa.tot = nullptr;
    sa.n_elems = tiles * S;
    sa.n_tiles = tiles;
    sa.n_lanes = S;
    if (fuse) {
        // (the bases were written by rss_hash's last workgroup)
    } else if (a.qmajor) {
        hipLaunchKernelGGL(rss_base, dim3(1), dim3(1024), 0, st, c->rss_hist, tiles * S, tiles,
                           o->queue_off_dev, c->rss_total);
    } else {
        const uint32_t nc = ceil_div(tiles, SCAN_COL_CHUNK);
        const dim3 grid(nc, ceil_div(S, (uint32_t)SCAN_BLOCK));
        hipLaunchKernelGGL(rx_scan_reduce, grid, dim3(SCAN_BLOCK), 0, st, sa);
        hipLaunchKernelGGL(rx_scan_top, dim3(1), dim3(SCAN_TOP_BLOCK), 4u * S, st, sa, nc);
        hipLaunchKernelGGL(rx_scan_down, grid, dim3(SCAN_BLOCK), 0, st, sa);
    }
    HIPC(c, hipGetLastError());
    hipLaunchKernelGGL(rss_scatter, dim3(tiles), dim3(RSS_BLOCK), 0, st, a);
    HIPC(c, hipGetLastError());
    return 0;
}

int udpdk_gpu_frag_table_create(udpdk_gpu_ctx *c, const udpdk_frag_table_cfg_t *cfg)
{
    if (!c || !cfg) return -EINVAL;
    HIPC(c, hipSetDevice(c->device));
    { int r = join_pipes(c); if (r) return r; }
    HIPC(c, hipStreamSynchronize(c->stream));
    reasm_destroy(c->reasm);
    c->reasm = nullptr;
    return reasm_create(&c->reasm, c->device, c->max_frames, cfg, &c->last_err);
}

int udpdk_gpu_rx_reassemble(udpdk_gpu_ctx *c, const udpdk_rx_batch_t *bt, const uint32_t *meta_dev,
                            uint64_t tms, udpdk_reasm_out_t *o)
{
    if (!c || !bt || !o) return -EINVAL;
    if (!c->reasm) return -EINVAL;
    if (bt->n && (!bt->frames_dev || !bt->offset_dev || !bt->length_dev || !meta_dev)) return -EINVAL;
    if (bt->frames_bytes >= (1ull << 32) || bt->n > c->max_frames) return -EINVAL;
    HIPC(c, hipSetDevice(c->device));
    { int r = join_pipes(c); if (r) return r; }
    return reasm_run(c->reasm, c->stream, bt, meta_dev, tms, o, &c->last_err, false);
}

int udpdk_gpu_rx_reassemble_inplace(udpdk_gpu_ctx *c, udpdk_rx_batch_t *bt, const uint32_t *meta_dev,
                                    uint64_t tms, udpdk_reasm_out_t *o)
{
    if (!c || !bt || !o) return -EINVAL;
    if (!c->reasm) return -EINVAL;
    if (bt->n && (!bt->frames_dev || !bt->offset_dev || !bt->length_dev || !meta_dev)) return -EINVAL;
    if (bt->frames_bytes >= (1ull << 32) || bt->n > c->max_frames) return -EINVAL;
    HIPC(c, hipSetDevice(c->device));
    { int r = join_pipes(c); if (r) return r; }
    return reasm_run(c->reasm, c->stream, bt, meta_dev, tms, o, &c->last_err, true);
}

uint64_t udpdk_gpu_tx_span(uint32_t len, uint32_t mtu, uint32_t *n_frames)
{
    uint32_t nf = 1;
    uint64_t span = (uint64_t)len + 42u;
    if (mtu >= 68u && (mtu - 20u) % 8u == 0 && (uint64_t)len + 42u > mtu) {
        nf = (uint32_t)(((uint64_t)len + 8u + (mtu - 20u) - 1u) / (mtu - 20u));
        span = (uint64_t)len + 8u + 34ull * nf;
    }
    if (n_frames) *n_frames = nf;
    return span;
}

int udpdk_gpu_tx_build(udpdk_gpu_ctx *c, const udpdk_tx_config_t *cfg, const udpdk_tx_batch_t *bt,
                       const udpdk_tx_out_t *o)
{
    return udpdk_gpu_tx_build_mtu(c, cfg, bt, o, 0);
}

int udpdk_gpu_tx_build_mtu(udpdk_gpu_ctx *c, const udpdk_tx_config_t *cfg,
                           const udpdk_tx_batch_t *bt, const udpdk_tx_out_t *o, uint32_t mtu)
{
    if (!c || !cfg || !bt || !o) return -EINVAL;
    if (mtu && (mtu < 68u || mtu > 65535u || (mtu - 20u) % 8u)) return -EINVAL;
    if (!bt->n) return 0;
    if (!bt->payload_dev || !bt->payload_off_dev || !bt->payload_len_dev || !bt->sockfd_dev ||
        !bt->dst_ip_dev || !bt->dst_port_dev || !o->frames_dev || !o->frame_off_dev) return -EINVAL;
    if (!c->slots || !c->n_slots) return -EINVAL;
    if (bt->payload_bytes >= (1ull << 32) || o->frames_bytes >= (1ull << 32)) return -EINVAL;
    if (((uintptr_t)o->frames_dev & 15u) || ((uintptr_t)bt->payload_dev & 15u)) return -EINVAL;
    HIPC(c, hipSetDevice(c->device));
    if (c->depth > 1) { int r = join_pipes(c); if (r) return r; }
    TxArgs ta;
    ta.payload = bt->payload_dev;
    ta.payload_off = bt->payload_off_dev;
    ta.payload_len = bt->payload_len_dev;
    ta.sockfd = bt->sockfd_dev;
    ta.dst_ip = bt->dst_ip_dev;
    ta.dst_port = bt->dst_port_dev;
    ta.frame_off = o->frame_off_dev;
    ta.slots = c->slots;
    ta.frames = o->frames_dev;
    ta.n = bt->n;
    ta.n_slots = c->n_slots;
    ta.payload_bytes = (uint32_t)bt->payload_bytes;
    // a dword comes back from a buffer load only if it ends inside the range: a
    // payload's last bytes are read by a byte-aligned load whose last dword may end up to 3
    // bytes past payload_bytes, inside the caller's UDPDK_GPU_FRAMES_TAILROOM
    ta.payload_rsrc = (uint32_t)std::min<uint64_t>((bt->payload_bytes + 3 + 3) & ~3ull, 0xFFFFFFFCull);
    ta.frames_bytes = (uint32_t)o->frames_bytes;
    ta.src_ip = cfg->src_ip;
    ta.mtu = mtu;
    uint8_t mac[12];
    memcpy(mac, cfg->dst_mac, 6);   // Ethernet d_addr first (udpdk_syscall.c:317)
    memcpy(mac + 6, cfg->src_mac, 6);
    memcpy(ta.mac_lo, mac, 12);
    const uint32_t groups = ceil_div(bt->n, 64);
    // waves per group of 64 datagrams: up to 4 while groups alone would leave the chip under
    // ~16 K waves (their chunk sweeps split between them)
    ta.parts = std::max<uint32_t>(1u, std::min<uint32_t>(4u, 16384u / std::max<uint32_t>(groups, 1u)));
    const uint32_t grid = std::min<uint32_t>(ceil_div(groups * ta.parts, TX_BLOCK / 64), 4096);
    hipEvent_t e0 = nullptr, e1 = nullptr;
    if (c->timing_every) {
        HIPC(c, hipEventCreate(&e0));
        HIPC(c, hipEventCreate(&e1));
        HIPC(c, hipEventRecord(e0, c->stream));
    }
    hipLaunchKernelGGL(tx_build, dim3(grid), dim3(TX_BLOCK), 0, c->stream, ta);
    HIPC(c, hipGetLastError());
    if (c->timing_every) {
        HIPC(c, hipEventRecord(e1, c->stream));
        HIPC(c, hipEventSynchronize(e1));
        float ms = 0;
        HIPC(c, hipEventElapsedTime(&ms, e0, e1));
        c->ms[UDPDK_K_TX_BUILD] += ms;
        c->launches[UDPDK_K_TX_BUILD]++;
        (void)hipEventDestroy(e0);
        (void)hipEventDestroy(e1);
    }
    return 0;
}

#ifdef UDPDK_STAMPS
// Diagnostic builds only (not part of the ABI headers): per-workgroup phase stamps.
int udpdk_gpu_debug_buffer(udpdk_gpu_ctx *c, void *dev)
{
    if (!c) return -EINVAL;
    c->dbg = (unsigned long long *)dev;
    return 0;
}
#endif

} // extern "C"
