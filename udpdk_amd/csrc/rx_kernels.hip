// rx_kernels.hip — gfx950 RX datapath: parse + validate + checksums + port demux + lanes.
//
// Replaces, for a batch of N frames, N calls of reassemble() (udpdk_poller.c:316-413) from the
// burst loop (udpdk_poller.c:516-545) plus the per-socket rx_buffer appends and ring flushes
// (udpdk_poller.c:274-298). All integer/byte work, bound by HBM:
//
//   rx_classify<G, MR>  one workgroup (4 waves) per tile of T frames, lane = frame, each wave
//       walking 64-frame steps in rounds of 1024 frames. The round's descriptors are staged in
//       LDS; the header window (frame bytes [12, 64), 3 x 16 B + 8 B dword-aligned loads
//       funnelled to frame-relative words) of the next step is in flight while the current one
//       is parsed. Per step: IPv4 gate, fragment / protocol tests, IPv4 header checksum, the UDP
//       checksum of datagrams that end within the window, and, with at most 8 bound ports in
//       the kernel arguments and one-round tiles, the demux (else a demux pass per round: all
//       the round's 16-byte port-table entries in flight at once). Longer datagrams: the step's
//       tail pass (frame bytes >= 64 as 64-byte chunks swept across the wave's lanes, per-frame
//       sums from a DPP prefix scan) or, for steps of back-to-back frames in the long-frame form
//       <2, 0>, the span sweep (the step's bytes read once on a line grid, windows taken from an
//       LDS ring, checksums from prefix sums over the span). Writes the verdict words, the
//       tile's per-lane delivery histogram (tile-major row hist[tile][lane]) and counter row;
//       single-lane calls also write speculative lane entries and, fused, complete the lane in
//       the last workgroup (repairing tiles that were not full). MR = 1: multi-round tiles with
//       the next round's descriptors loaded a round ahead.
//   rx_compact1  the single-lane completion as a second launch (fused form not taken): keeps the
//       speculative entries up to the first tile that was not full, rewrites the rest.
//   rx_scan_cols + rx_scatterw  general case: per-lane column scan of the tile-major histogram
//       (decoupled look-back over lane blocks, base rows out), then a stable per-lane scatter
//       (LDS atomic ranks, key-ordered staging, linear stores). rx_scan_reduce/top/down and
//       rx_scatter: the same past their limits (more tiles, more lanes, fan-out).
//   rx_counters  on demand (udpdk_gpu_rx_stats): sum of the per-tile counter rows.
//
// Algorithmic bytes per frame in rx_classify: frame_len + 6 (u32 offset + u16 length) + 4
// (verdict word), + 4 per (lane, tile) histogram entry.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <type_traits>

#include "udpdk_gpu.h"
#include "rx_common.h"

namespace udpdk {

// ------------------------------------------------------------------------------------------
// wave helpers (wave64)
// ------------------------------------------------------------------------------------------
__device__ __forceinline__ uint32_t lane_id() { return __lane_id(); }

// Orders LDS accesses of one wave across lanes. The hardware executes a wave's DS instructions
// in order, so only the compiler must be kept from reordering them; a wavefront-scope fence
// would also emit vmcnt(0) and drain every prefetch in flight.
__device__ __forceinline__ void wave_sync()
{
    asm volatile("" ::: "memory");
    __builtin_amdgcn_wave_barrier();
}

// Inclusive prefix sum across the wave, on the DPP network (row shifts + row broadcasts: six
// VALU ops; the __shfl_up form was six ds_bpermute round trips through the LDS pipeline, which
// the LDS-bound scatter paid for in every scan). Every lane must be active.
__device__ __forceinline__ uint32_t wave_incl_scan(uint32_t v)
{
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x111, 0xF, 0xF, false);   // row_shr:1
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x112, 0xF, 0xF, false);   // row_shr:2
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x114, 0xF, 0xF, false);   // row_shr:4
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x118, 0xF, 0xF, false);   // row_shr:8
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x142, 0xA, 0xF, false);   // row_bcast:15
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x143, 0xC, 0xF, false);   // row_bcast:31
    return v;
}

__device__ __forceinline__ uint32_t wave_sum(uint32_t v)
{
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) v += __shfl_xor(v, d, 64);
    return v;
}

// Bytes [a, e) of a 16-byte chunk as a dword mask for dword i (a, e clamped to [0, 16]).
__device__ __forceinline__ uint32_t dword_window(int a, int e, int i)
{
    const int la = min(max(a - 4 * i, 0), 4);
    const int le = min(max(e - 4 * i, 0), 4);
    const uint32_t hm = le >= 4 ? 0xFFFFFFFFu : ((1u << (8 * le)) - 1u);
    const uint32_t lm = la >= 4 ? 0xFFFFFFFFu : ((1u << (8 * la)) - 1u);
    return hm & ~lm;
}

__device__ __forceinline__ uint32_t sum16(uint32_t v) { return (v & 0xFFFFu) + (v >> 16); }

// acc + both 16-bit halves of v in ONE instruction: v_sad_u16(v, 0, acc) = |v.lo - 0| + |v.hi - 0|
// + acc. The RFC 1071 sums below are chains of these (the and/shift/add3 form of sum16 is three).
__device__ __forceinline__ uint32_t sad16(uint32_t v, uint32_t acc)
{
    return __builtin_amdgcn_sad_u16(v, 0u, acc);
}

// One's-complement fold of a 32-bit sum of 16-bit words to [0, 0xffff] (0xffff is -0: a valid
// RFC 1071 sum folds to 0xffff; only an all-zero input folds to 0).
__device__ __forceinline__ uint32_t fold32(uint32_t x)
{
    x = (x & 0xFFFFu) + (x >> 16);
    return (x & 0xFFFFu) + (x >> 16);
}

// Sum of the 16-bit halves of the bytes [a, e) of the chunk: <= 8 * 0xFFFF.
__device__ __forceinline__ uint32_t chunk_sum(const uint4 d, int a, int e)
{
    if (e <= a) return 0u;
    if (a <= 0 && e >= 16) return sum16(d.x) + sum16(d.y) + sum16(d.z) + sum16(d.w);
    return sum16(d.x & dword_window(a, e, 0)) + sum16(d.y & dword_window(a, e, 1)) +
           sum16(d.z & dword_window(a, e, 2)) + sum16(d.w & dword_window(a, e, 3));
}

__device__ __forceinline__ __amdgpu_buffer_rsrc_t make_rsrc(const void *p, uint32_t bytes)
{
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<void *>(p), (short)0, (int)bytes,
                                             0x00020000);
}

__device__ __forceinline__ uint4 load16(__amdgpu_buffer_rsrc_t r, uint32_t off)
{
    const auto v = __builtin_amdgcn_raw_buffer_load_b128(r, (int)off, 0, 0);
    return make_uint4(v[0], v[1], v[2], v[3]);
}

// Diagnostic build (-DUDPDK_STAMPS): wave 0 of every workgroup accumulates s_memtime cycles per
// phase into a.dbg[block][16]. Stamps never feed an output (cdna_hip_programming.md §7).
// -DUDPDK_STAMPS_LIGHT keeps only the entry/exit realtime stamps (dispatch timeline).
#if defined(UDPDK_STAMPS) && !defined(UDPDK_STAMPS_LIGHT)
#define STAMP(k)                                                                 \
    do {                                                                         \
        if (w == 0) {                                                            \
            const unsigned long long t_ = __builtin_amdgcn_s_memtime();          \
            if (lane == 0) st_acc[k] += t_ - st_last;                            \
            st_last = t_;                                                        \
        }                                                                        \
    } while (0)
// slots 12-15: realtime (100 MHz, chip-synchronous) at entry and exit, HW_ID | XCC_ID << 32, tile
#else
#define STAMP(k) do {} while (0)
#endif
#ifdef UDPDK_STAMPS
#define STAMP_END()                                                                   \
    do {                                                                              \
        if (tid != 0) break;                                                          \
        st_acc[13] = __builtin_amdgcn_s_memrealtime();                                \
        st_acc[14] = (unsigned long long)__builtin_amdgcn_s_getreg(4 | (31 << 11)) |  \
                     ((unsigned long long)__builtin_amdgcn_s_getreg(20 | (31 << 11)) << 32); \
        st_acc[15] = tile;                                                            \
    } while (0)
#endif


// counters[c] = sum over tiles of tile_cnt[t][c] (64-bit). Thread (g, c) = (tid / 16, tid % 16)
// sums counter c of rows g, g + G, ... (each pass of the block reads 16 whole rows, coalesced);
// two xor-shuffles fold the 4 row groups of a wave, LDS the waves. lds: >= 16 * waves u64.
__device__ unsigned long long reduce_counters(const uint32_t *tile_cnt, uint32_t n_tiles,
                                              unsigned long long *counters, unsigned long long *lds)
{
    const uint32_t tid = threadIdx.x, lane = lane_id(), w = tid >> 6, nw = blockDim.x >> 6;
    const uint32_t c = tid & 15u, G = blockDim.x >> 4;
    unsigned long long s = 0;
    uint32_t t = tid >> 4;
    auto ld = [&](uint32_t row) -> uint32_t {
        const uint32_t *p = &tile_cnt[(size_t)row * UDPDK_N_COUNTERS + c];
        return *p;
    };
    for (; t + 3u * G < n_tiles; t += 4u * G) {
        const uint32_t v0 = ld(t), v1 = ld(t + G), v2 = ld(t + 2u * G), v3 = ld(t + 3u * G);
        s += (unsigned long long)v0 + v1 + v2 + v3;
    }
    for (; t < n_tiles; t += G) s += ld(t);
    s += __shfl_xor(s, 16, 64);
    s += __shfl_xor(s, 32, 64);
    if (lane < 16) lds[w * 16 + lane] = s;
    __syncthreads();
    unsigned long long r = 0;
    if (tid < UDPDK_N_COUNTERS) {
        for (uint32_t i = 0; i < nw; ++i) r += lds[i * 16 + tid];
        counters[tid] = r;
    }
    return r;                                               // counter tid, for tid < 16
}

// ------------------------------------------------------------------------------------------
// rx_classify
// ------------------------------------------------------------------------------------------
// Bytes [lo, hi) of the little-endian dword holding frame bytes [base, base + 4), as a mask.
__device__ __forceinline__ uint32_t byte_mask(int lo, int hi, int base)
{
    const int la = min(max(lo - base, 0), 4);
    const int le = min(max(hi - base, 0), 4);
    const uint32_t hm = le >= 4 ? 0xFFFFFFFFu : ((1u << (8 * le)) - 1u);
    const uint32_t lm = la >= 4 ? 0xFFFFFFFFu : ((1u << (8 * la)) - 1u);
    return hm & ~lm;
}

// Inclusive wave64 prefix sum on the DPP network (no LDS traffic).
__device__ __forceinline__ uint32_t scan_dpp(uint32_t v) { return wave_incl_scan(v); }

// Inclusive wave64 prefix maximum on the DPP network (same shifts as scan_dpp).
__device__ __forceinline__ uint32_t max_scan_dpp(uint32_t v)
{
    v = max(v, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x111, 0xF, 0xF, false));
    v = max(v, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x112, 0xF, 0xF, false));
    v = max(v, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x114, 0xF, 0xF, false));
    v = max(v, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x118, 0xF, 0xF, false));
    v = max(v, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x142, 0xA, 0xF, false));
    v = max(v, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x143, 0xC, 0xF, false));
    return v;
}

// ------------------------------------------------------------------------------------------
// Fused single-lane completion (rx_classify with a.fuse): what rx_compact1 does in a second
// launch, done by the last workgroup to finish. Each workgroup, once its written-through stores
// are drained, adds {1 arrival, not-full flag, its deliveries} to its shard's fan-in word
// (a.fuse[16 s], s = tile mod 8, 128 B apart: one word for 1024 arrivals serialises them,
// tools/probe/ticket_probe.hip); the shard's last arrival adds the shard's sums to the top word
// (a.fuse[128]) and the top's last arrival completes the call. Every word is reset by its last
// arrival, so the pipe's next call starts from zeros. When every tile before the last delivered
// all its frames (the common case of a port-bound stream) the speculative entries are the lane
// already and the completion writes lane_off and the total only.
//
// Repair (a tile before the last not full: a stray frame, a drop): every later tile's entries sit
// at tile x T + rank instead of their base + rank. A short tile raises the call's FLAG word
// (before its arrival); every workgroup loads FLAG beside its store drain, so the value costs no
// round trip. The last UDPDK_FIX_HELPERS arrivals of each shard that saw FLAG wait for the call's
// last arrival, which opens the repair (WORK = epoch << 32, then DONE = epoch) and joins it. Each
// participant takes every tile's delivery count (sc1 loads behind an agent acquire), their
// exclusive prefix in LDS, and then chunks of UDPDK_FIX_CHUNK tiles after the first short tile
// from WORK: a full tile's entries are its frame indices in order (stores only), a short tile's
// come from its verdict words. Helpers are optional (a helper that waits past UDPDK_FIX_SPIN
// leaves; the last arrival works through every chunk itself if it must), so the repair is exact
// whoever joins; with helpers it costs a few microseconds instead of a one-workgroup rewrite.
// No workgroup waits unless a tile of its call was short, and at most UDPDK_FIX_HELPERS x 8 wait,
// far fewer than the workgroups resident at once, so no workgroup waits on one that cannot start.
// ------------------------------------------------------------------------------------------
__device__ __forceinline__ uint32_t block_scan4(uint32_t v, uint32_t *ws, uint32_t lane, uint32_t w,
                                                uint32_t *total)
{
    // exclusive scan over the CLS_WAVES x 64 threads (ws: CLS_WAVES words of LDS)
    const uint32_t incl = scan_dpp(v);
    if (lane == 63) ws[w] = incl;
    __syncthreads();
    uint32_t pre = incl - v, tot = 0;
#pragma unroll
    for (uint32_t i = 0; i < CLS_WAVES; ++i) {
        pre += i < w ? ws[i] : 0u;
        tot += ws[i];
    }
    __syncthreads();
    *total = tot;
    return pre;
}

__device__ __forceinline__ void classify_complete(const RxArgs &a, uint32_t tile, uint32_t tcount,
                                                  uint32_t tid, uint32_t lane, uint32_t w, uint8_t *smem)
{
    __shared__ uint32_t fz[8 + CLS_WAVES];
    const uint32_t T = a.tile_frames;
    const bool nonfull = tile + 1u < a.n_tiles && tcount != T;
    unsigned long long flag = 0;
    if (tid == 0) {
        if (nonfull) atomicMax(&a.fuse[UDPDK_FUSE_FLAG], (unsigned long long)a.spec_epoch);
        flag = __hip_atomic_load(&a.fuse[UDPDK_FUSE_FLAG], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");      // every wave: its stores written through
    __syncthreads();
    if (tid == 0) {
        // payload: {tiles before the last that were not full << 32 | deliveries}
        unsigned long long fin = 0;
        uint32_t left = 0;
        const bool last = fanin_arrive(a.fuse, tile, a.n_tiles, (nonfull ? 1ull << 32 : 0ull) | tcount, &fin, &left);
        fz[0] = last ? 1u : 0u;
        fz[1] = (uint32_t)fin;                              // deliveries of the call
        fz[2] = (uint32_t)(fin >> 32) & 0xFFFFu;            // tiles (not the last) not full
        fz[3] = !last && (uint32_t)flag == a.spec_epoch && left < UDPDK_FIX_HELPERS ? 1u : 0u;
    }
    __syncthreads();
    const bool last = fz[0] != 0u;
    if (last) {
        if (tid == 0) {
            a.lane_off[0] = 0u;
            a.lane_off[1] = fz[1];
            *a.total = fz[1];
            if (fz[2] != 0u) {                             // open the repair
                __hip_atomic_store(&a.fuse[UDPDK_FUSE_WORK], (unsigned long long)a.spec_epoch << 32,
                                   __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                __hip_atomic_store(&a.fuse[UDPDK_FUSE_DONE], (unsigned long long)a.spec_epoch,
                                   __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
            }
        }
        if (fz[2] == 0u) return;
    } else {
        if (fz[3] == 0u) return;
        if (tid == 0) {
            uint32_t ok = 0;
            for (uint32_t it = 0; it < UDPDK_FIX_SPIN; ++it) {
                if (__hip_atomic_load(&a.fuse[UDPDK_FUSE_DONE], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) ==
                    (unsigned long long)a.spec_epoch) {
                    ok = 1u;
                    break;
                }
                __builtin_amdgcn_s_sleep(4);
            }
            fz[4] = ok;
        }
        __syncthreads();
        if (fz[4] == 0u) return;
    }
    // the other workgroups' tile counts and verdict words: one acquire, then sc1 loads
    if (tid == 0) __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    const uint32_t nt = a.n_tiles;
    uint32_t *base = reinterpret_cast<uint32_t *>(smem + DSC_OFF);   // [nt + 1] tile bases
    uint32_t *ws = fz + 8;
    {
        // thread tid holds tiles [k0, k0 + per): counts, their exclusive prefix, the first
        // short tile (not the last)
        const __amdgpu_buffer_rsrc_t hr = make_rsrc(a.hist, nt * 4u);
        const uint32_t per = (nt + CLS_BLOCK - 1u) / CLS_BLOCK, k0 = tid * per;
        uint32_t sum = 0, f = 0xFFFFFFFFu;
        for (uint32_t k = 0; k < per; ++k) {
            const uint32_t t = k0 + k;
            const uint32_t c = t < nt ? __builtin_amdgcn_raw_buffer_load_b32(hr, (int)(4u * t), 0, 16) : 0u;
            if (t < nt) base[t] = c;                        // counts first, prefix below
            if (t + 1u < nt && c != T) f = min(f, t);
            sum += c;
        }
        uint32_t tot;
        uint32_t run = block_scan4(sum, ws, lane, w, &tot);
        for (uint32_t k = 0; k < per; ++k) {
            const uint32_t t = k0 + k;
            if (t < nt) {
                const uint32_t c = base[t];
                base[t] = run;
                run += c;
            }
        }
        if (tid == 0) base[nt] = tot;
#pragma unroll
        for (int d = 32; d >= 1; d >>= 1) f = min(f, (uint32_t)__shfl_xor((int)f, d, 64));
        if (lane == 0) ws[w] = f;
        __syncthreads();
        f = ws[0];
#pragma unroll
        for (uint32_t i = 1; i < CLS_WAVES; ++i) f = min(f, ws[i]);
        __syncthreads();
        if (tid == 0) fz[6] = f;
        __syncthreads();
    }
    const uint32_t first = fz[6];                           // tiles up to it hold their entries
    const __amdgpu_buffer_rsrc_t sr =
        make_rsrc(a.spec_pkt, a.spec_cap >= 0x40000000u ? 0xFFFFFFFCu : a.spec_cap * 4u);
    const __amdgpu_buffer_rsrc_t mr = make_rsrc(a.meta, a.n * 4u);
    for (;;) {
        __syncthreads();                                    // fz[5] of the previous chunk read
        if (tid == 0) {
            const unsigned long long k = __hip_atomic_fetch_add(&a.fuse[UDPDK_FUSE_WORK], 1ull,
                                                                __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            fz[5] = (uint32_t)(k >> 32) == a.spec_epoch ? (uint32_t)k : 0xFFFFFFFFu;
        }
        __syncthreads();
        const uint32_t k = fz[5];
        if (first == 0xFFFFFFFFu || k == 0xFFFFFFFFu || k >= nt) break;
        const uint32_t ta = first + 1u + k * UDPDK_FIX_CHUNK;
        if (ta >= nt) break;
        const uint32_t tb = min(nt, ta + UDPDK_FIX_CHUNK);
        for (uint32_t t = ta; t < tb; ++t) {
            const uint32_t b = base[t], c = base[t + 1u] - b, f0 = t * T;
            if (c == T) {
                // a full tile: its frames in order (stores only)
                const uint32_t j = 4u * tid, pos = b + j;
                const __attribute__((ext_vector_type(4))) uint32_t x = {f0 + j, f0 + j + 1u, f0 + j + 2u, f0 + j + 3u};
                if ((pos & 3u) == 0u) {
                    __builtin_amdgcn_raw_buffer_store_b128(x, sr, (int)(4u * pos), 0, 0);
                } else {
#pragma unroll
                    for (uint32_t i = 0; i < 4; ++i)
                        __builtin_amdgcn_raw_buffer_store_b32(f0 + j + i, sr, (int)(4u * (pos + i)), 0, 0);
                }
            } else {
                // a short (or the last) tile: its delivered frames from its verdict words
                const uint32_t fb = f0 + 4u * tid;
                const auto v = __builtin_amdgcn_raw_buffer_load_b128(mr, (int)(4u * fb), 0, 16);
                uint32_t bits = 0;
#pragma unroll
                for (uint32_t i = 0; i < 4; ++i)
                    if ((v[i] & 0xFu) == UDPDK_V_DELIVERED && fb + i < a.n && 4u * tid + i < T) bits |= 1u << i;
                const uint32_t cnt = (uint32_t)__builtin_popcount(bits);
                uint32_t tot;
                uint32_t pos = b + block_scan4(cnt, ws, lane, w, &tot);
#pragma unroll
                for (uint32_t i = 0; i < 4; ++i)
                    if ((bits >> i) & 1u) {
                        __builtin_amdgcn_raw_buffer_store_b32(fb + i, sr, (int)(4u * pos), 0, 0);
                        ++pos;
                    }
            }
        }
    }
}

// Frame bytes [12, 64) of one frame: 14 dwords from the dword at or below frame byte 12 (3 x 16 B
// + 8 B; at 64 B frame strides a dword-aligned start costs the same as an aligned one, a byte-
// aligned one ~25 % more, tools/probe/align_probe.hip), funnelled to g[i] = frame bytes 12 + 4i ..
struct Win {
    uint4 a, b, c;
    uint2 d;
};

// 4 waves per SIMD (<= 128 VGPRs, the tail pass's two groups in flight): one tile of 1024 frames
// per workgroup puts 4 workgroups on each CU at 1 M frames. (Round 1: a 96-VGPR budget spilled
// and ran 19 % slower at 64 B; four tail groups in flight at 148 VGPRs and 3 waves per SIMD were
// no faster at 1500 B and slower at IMIX and 106 B. Round 2: three groups at 127 VGPRs, DESIGN.md
// §4.) Round 4: G = tail-pass chunk groups in flight per wave. G = 2 (122 VGPRs, 4 waves per
// SIMD) for batches with long datagrams; G = 1 (92 VGPRs, 5 waves per SIMD, the LDS limit of a
// one-round tile) lets a fifth workgroup per CU in, which is what consecutive short-frame
// batches overlapping on several streams want (config 2, --steps 20, same-box A/B with the
// compaction launch gone: 57.1 -> 63.0 Gpkt/s; config 1 (106 B, one tail chunk per frame) is
// 8 % slower at G = 1, so the host picks G by whether recent calls had tail passes).
template <int G, int MR>
__global__ void __launch_bounds__(CLS_BLOCK)
__attribute__((amdgpu_waves_per_eu(MR ? 2 : G == 1 ? 5 : UDPDK_CLS_WPE, 8)))
rx_classify(RxArgs a)
{
    static_assert(G == 1 || G == 2, "one or two tail chunk groups in flight");
    // the span sweep (RxArgs::span) is compiled into the long-frame form of one-round tiles only
    constexpr bool SPAN = G == 2 && MR == 0;
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    const uint32_t tid = threadIdx.x, lane = lane_id(), w = tid >> 6;
    const uint32_t steps = a.tile_frames / 64;
    constexpr uint32_t RSTEPS = RX_ROUND / 64;              // steps per staging round
    constexpr uint32_t SPR = RSTEPS / CLS_WAVES;            // steps per wave per staging round
    static_assert(SPR >= 2, "round staging needs two steps per wave per round");
#ifdef UDPDK_STAMPS
    // (in LDS: a register array indexed by lane at the end went to scratch, and the scratch
    // allocation held workgroups back from starting)
    __shared__ unsigned long long st_acc[16];
    unsigned long long st_last = __builtin_amdgcn_s_memtime();
    if (tid < 16) st_acc[tid] = 0;
    if (tid == 0) st_acc[12] = __builtin_amdgcn_s_memrealtime();
#endif

    uint32_t *cntw = reinterpret_cast<uint32_t *>(smem + CNT_OFF);    // [wave][counter]
    // descriptors of the current (and, double-buffered, the next) round of RX_ROUND frames:
    // staged with coalesced loads by the whole workgroup, so the per-step reads are LDS reads
    // (lgkmcnt) and never make a step wait on vector-memory loads it issued for a later step
    const uint32_t nbuf = classify_dsc_bufs(a.tile_frames);
    uint32_t *d_off = reinterpret_cast<uint32_t *>(smem + DSC_OFF);  // [nbuf][RX_ROUND]
    uint32_t *d_lp = d_off + nbuf * RX_ROUND;                        // length | ptype-IPv4 << 16
    uint32_t *hist = d_lp + nbuf * RX_ROUND;                         // [n_lanes] this tile
    // The tile's verdict words are staged in LDS and stored once per tile (16 B per lane): no
    // global store inside the step loop, so no s_waitcnt there ever waits for a store (on gfx9
    // stores count in vmcnt, in order with the loads).
    uint32_t *mstage = hist + classify_hist_words(a.n_lanes, a.hist16 != 0u);   // [stage frames]
    // datagram end (34 + UDP length) of the frames whose checksum the tail pass completes
    // pending frames' datagram end | folded window part of the UDP sum << 16
    uint32_t *dgl = mstage + classify_stage_frames(a.tile_frames);   // [RX_ROUND]
    // the round's port-table lookups: raw dst port | is-UDP << 16, raw dst IPv4
    uint2 *dstash = reinterpret_cast<uint2 *>(dgl + RX_ROUND);       // [RX_ROUND]

    // (hist is only used with several lanes; its zeroing is ordered by the staging barrier)
    // hist16: two lanes per LDS word (lane k in the half k & 1), counts < 2^16 (a tile's
    // deliveries per lane, <= 8192 without fan-out), stored as a u16 row
    const uint32_t hsh = a.hist16 ? 1u : 0u;
    auto hist_add = [&](uint32_t k, uint32_t v) { atomicAdd(&hist[k >> hsh], v << ((k & hsh) << 4)); };
    // Tiles in dispatch order (consecutive tiles on different XCDs). An XCD-contiguous remap
    // (each XCD's L2 streaming one contiguous eighth of the batch) measured 1.7 us slower per
    // 1 M x 64 B launch (tools/probe/stream_probe.hip, feat4).
    const uint32_t tile = blockIdx.x;

    const __amdgpu_buffer_rsrc_t fr = make_rsrc(a.frames, a.rsrc_bytes);
    const uint32_t t0 = tile * a.tile_frames;
    const uint32_t t1 = min(a.n, t0 + a.tile_frames);

    // counters: per-lane packed 8-bit fields (verdicts 0-3 / 4-7, flag counters), deliveries
    // and bytes; reduced across the wave once per tile
    uint32_t acc_v0 = 0, acc_v1 = 0, acc_f0 = 0, acc_f1 = 0, acc_fan = 0, lane_bytes = 0;

    // Loads are unconditional (clamped index / range-checked buffer offsets): a load under a
    // lane condition makes the compiler wait for it at the end of the branch, which would drain
    // the prefetch pipeline every step.
    const uint32_t plast = a.n - 1u;
    // round r's descriptors (frames t0 + RX_ROUND r + [0, RX_ROUND)) into buffer r & 1; the
    // ptype array, when given, only contributes its L3_IPV4 bit (udpdk_poller.c:334)
    // (the ptype word is loaded unconditionally, from the offset array when there is no ptype
    // array, and masked: a load under a condition makes the compiler wait for it in the branch)
    const bool has_ptype = a.ptype != nullptr;
    const uint32_t *ptw = has_ptype ? a.ptype : a.offset;
    constexpr uint32_t SPT = RX_ROUND / CLS_BLOCK;          // descriptors staged per thread
    auto stage_load = [&](uint32_t r, uint32_t (&o)[SPT], uint32_t (&l)[SPT], uint32_t (&t)[SPT]) {
#pragma unroll
        for (uint32_t i = 0; i < SPT; ++i) {
            const uint32_t pc = min(t0 + r * RX_ROUND + i * CLS_BLOCK + tid, plast);
            o[i] = a.offset[pc];
            l[i] = a.length[pc];
            t[i] = ptw[pc];
        }
    };
    auto stage_store = [&](uint32_t r, const uint32_t (&o)[SPT], const uint32_t (&l)[SPT], const uint32_t (&t)[SPT]) {
        const uint32_t b = (r & (nbuf - 1u)) * RX_ROUND;
#pragma unroll
        for (uint32_t i = 0; i < SPT; ++i) {
            d_off[b + i * CLS_BLOCK + tid] = o[i];
            d_lp[b + i * CLS_BLOCK + tid] = l[i] | (has_ptype ? (t[i] & 0x10u) << 12 : 0u);
        }
    };
    auto stage = [&](uint32_t r) {
        uint32_t o[SPT], l[SPT], t[SPT];
        stage_load(r, o, l, t);
        stage_store(r, o, l, t);
    };
    // step s's descriptor for this lane (the index wraps inside the buffers for s >= steps)
    auto read_desc = [&](uint32_t s, uint32_t &o, uint32_t &lp) {
        const uint32_t i = s * 64 + lane;
        const uint32_t b = (((i / RX_ROUND) & (nbuf - 1u)) * RX_ROUND) + (i % RX_ROUND);
        o = d_off[b];
        lp = d_lp[b];
    };
    // The frame's header window, frame bytes [12, 64) (bytes 0-11, the MAC addresses, are never
    // read). One lane per frame, 14 dwords from the dword-aligned buffer offset at or below
    // offset + 12 (byte-aligned 16-byte loads cost the vector memory path ~25 %); the step
    // funnels them to frame-relative words by offset & 3. Bytes past the frame are never used
    // (parse and sums mask by length); lanes without a frame read the buffer's first bytes
    // (cached, never used).
    // (a step that sweeps its span takes its windows from the sweep: nothing loaded here)
    constexpr uint32_t OOR = 0xFFFFFFF0u;   // past any batch's range (< 4 GiB - 16)
    auto load_win = [&](uint32_t s, uint32_t o, uint32_t l, bool swept = false) -> Win {
        const uint32_t p = t0 + s * 64 + lane;
        const bool ok = s < steps && p < t1 && l >= 14u && l <= a.frames_bytes && o <= a.frames_bytes - l;
        const uint32_t b = swept ? OOR : ok ? (o + 12u) & ~3u : 0u;
        Win r;
        r.a = load16(fr, b);
        r.b = load16(fr, b + 16u);
        r.c = load16(fr, b + 32u);
        const auto d = __builtin_amdgcn_raw_buffer_load_b64(fr, (int)(b + 48u), 0, 0);
        r.d = make_uint2(d[0], d[1]);
        return r;
    };

    // Prologue, shortest chain first: the round's descriptor loads go out before anything else,
    // and the first window (step w: frames t0 + tid, this thread's own first descriptor) before
    // the descriptors are staged and the workgroup waits at the barrier. The argument-borne bind
    // table (a vector load from the kernel-argument segment) and the LDS initialisation follow,
    // off that chain (each used to cost a dependent round trip ahead of the descriptor loads).
    __shared__ uint32_t tail_any;           // some wave of the tile ran a tail pass (kernel hint)
    __shared__ uint4 inl_tab[UDPDK_INLINE_PORTS + 1];   // RxArgs::inl entries + a zero slot
    uint32_t st = __builtin_amdgcn_readfirstlane(w);             // wave-uniform step (SGPR)
    uint32_t c_off, c_lp;
    Win W;

    // ---- span sweep (SPAN forms, a.span): is step s's span [A, Ep) sweepable? ----
    // Every frame of the step in range, each starting within SPAN_MAX_GAP bytes after the previous
    // one's end (ascending, disjoint: what a NIC's back-to-back mbuf images are), and on average
    // at least SPAN_MIN_AVG bytes long (shorter frames are all window: the per-frame windows read
    // the same lines). A = the 128-byte line holding the first frame, Ep = the end of the last
    // frame or of the furthest window (windows read 56 bytes from the dword at or below offset +
    // 12). Wave-uniform.
    auto span_check = [&](uint32_t s, uint32_t o, uint32_t l, uint32_t &A, uint32_t &Ep) -> bool {
        if (!SPAN || !a.span || s >= steps) return false;
        const uint32_t p = t0 + s * 64u + lane;
        const bool v = p < t1;
        const unsigned long long vm = __ballot(v);
        if (vm == 0ull) return false;
        const uint32_t on = (uint32_t)__shfl_down((int)o, 1, 64);    // the next frame's offset
        const bool nv = lane < 63u && p + 1u < t1;
        const bool good = l <= a.frames_bytes && o <= a.frames_bytes - l;
        const bool bad = v && (!good || (nv && on - (o + l) >= SPAN_MAX_GAP));
        if (__ballot(bad)) return false;
        const uint32_t ee = v ? max(o + l, ((o + 12u) & ~3u) + 56u) : 0u;
        const uint32_t em = (uint32_t)__builtin_amdgcn_readlane((int)max_scan_dpp(ee), 63);
        const uint32_t a0 = (uint32_t)__builtin_amdgcn_readfirstlane((int)o) & ~127u;
        if (em - a0 < SPAN_MIN_AVG * (uint32_t)__popcll(vm)) return false;
        A = a0;
        Ep = em;
        return true;
    };
    bool span_cur = false;                  // the current step sweeps its span (wave-uniform)
    uint32_t span_A = 0, span_E = 0;
    {
        uint32_t o[SPT], l[SPT], t[SPT];
        stage_load(0, o, l, t);
        // (issued before the window: its wait then leaves the window loads in flight)
        const uint4 ie = a.inl_ent[min(tid, UDPDK_INLINE_PORTS - 1u)];
        c_off = o[0];
        c_lp = l[0] | (has_ptype ? (t[0] & 0x10u) << 12 : 0u);
        span_cur = span_check(st, c_off, c_lp & 0xFFFFu, span_A, span_E);
        W = load_win(st, c_off, c_lp & 0xFFFFu, span_cur);
        __builtin_amdgcn_sched_barrier(0);
        const bool inl = a.inl && tid <= UDPDK_INLINE_PORTS;
        if (tid == 0) tail_any = 0u;        // (ordered by the staging barrier)
        if (a.n_lanes > 1u)
            for (uint32_t s = tid; s < ((a.n_lanes + hsh) >> hsh); s += CLS_BLOCK) hist[s] = 0;
        stage_store(0, o, l, t);
        if (inl) inl_tab[tid] = tid < a.n_inl ? ie : make_uint4(0, 0, 0, 0);
    }
    __syncthreads();
    STAMP(0);

    // ---- tail pass: UDP checksums of the datagrams that extend past the header window ----
    // Run for each step right after it (while the frames' first lines are still in L2: a pass
    // per round of four steps re-fetched the line shared by a frame's header window and its
    // first tail chunk from HBM). The step's pending frames (state 3): the tail's bytes, frame
    // bytes [64, dge) at buffer offsets [S, E) = [offset + 64, offset + dge), as 64-byte
    // super-chunks from the dword-aligned Sa = S & ~3 (chunk j = [Sa + 64 j, Sa + 64 j + 64), 4
    // dword-aligned 16-byte pieces; byte-aligned pieces ran the vector memory path at 4.45
    // instead of 5.9 TB/s, tools/probe/align_probe.hip). The words are then buffer-aligned, not
    // frame-aligned: a frame at an odd offset has its tail sum byte-swapped (RFC 1071 sums are
    // byte-order independent up to that swap), and the first chunk's S - Sa lead bytes (the
    // window's) come off again. The chunks are swept across the wave's lanes: lane i of a group
    // takes chunk k0 + i of the step's chunk space, so a group is 4 KiB of dense frame bytes. A chunk's frame comes from a prefix
    // maximum over the group's lanes of the marks the frames starting inside the group leave in
    // LDS (one LDS round trip; a binary search over the chunk starts took six). Pieces at or past
    // the datagram end are addressed out of the buffer's range (no memory access, zeros); the
    // piece holding the end, when it ends inside it, has its bytes past the end subtracted from
    // the chunk sum, so every chunk is summed the same way (v_sad_u16 chains, no masked re-sum).
    // Per-frame sums are segment sums of a DPP prefix scan; two groups in flight.
    // per frame q of the step: chunk k of q starts at buffer offset B_q + 64 k and holds D_q - 64 k
    // bytes up to the datagram end (B_q = Sa - 64 cs_q, D_q = E - Sa + 64 cs_q, cs_q = the frame's
    // first chunk index in the step), so a chunk needs two LDS words of its frame (B_q's low two
    // bits carry the lead S - Sa)
    uint32_t *l_B = reinterpret_cast<uint32_t *>(smem + TP_OFF) + w * 192;   // [64]
    uint32_t *l_D = l_B + 64;                                               // [64]
    uint32_t *l_own = l_B + 128;            // [64] frame + 1 whose chunks start at k0 + slot, else 0
    l_own[lane] = 0;
    bool tailed = false;                    // this wave ran a tail pass (the host's kernel hint)
    auto tail_step = [&](uint32_t s2) {
            const uint32_t i = s2 * 64 + lane;
            const uint32_t m = mstage[i & (RX_ROUND - 1u)];
            const bool pd = t0 + i < t1 && ((m >> 5) & 3u) == 3u;
            if (!__ballot(pd)) return;
            // the frame's offset: the staged descriptor of a single-round tile, else global
            const uint32_t fo = nbuf == 1u ? d_off[i] : a.offset[min(t0 + i, plast)];
            const uint32_t dw = dgl[i & (RX_ROUND - 1u)];
            const uint32_t de = pd ? dw & 0xFFFFu : 64u;
            const uint32_t lead = (fo + 64u) & 3u;
            const uint32_t my_nt = pd ? (de - 64u + lead + 63u) >> 6 : 0u;
            const uint32_t inc = scan_dpp(my_nt);
            const uint32_t my_cs = inc - my_nt;
            const uint32_t total = (uint32_t)__builtin_amdgcn_readlane((int)inc, 63);
            l_B[lane] = (fo + 64u - lead - 64u * my_cs) | lead;
            l_D[lane] = de - 64u + lead + 64u * my_cs;
            uint32_t tsum = 0, carry = 0;
            // group k0: each lane's frame (q), the chunk's bytes in the datagram (left) and its
            // four pieces in flight
            auto issue = [&](uint32_t k0, uint32_t &q, int &left, uint32_t &lead_b, uint4 (&R)[4]) {
                const uint32_t k = k0 + lane;
                if (my_nt != 0u && my_cs >= k0 && my_cs < k0 + 64u) l_own[my_cs - k0] = lane + 1u;
                wave_sync();
                const uint32_t mark = l_own[lane];
                l_own[lane] = 0u;                       // cleared for the next group (in order)
                const uint32_t own = max(max_scan_dpp(mark), carry);
                carry = (uint32_t)__builtin_amdgcn_readlane((int)own, 63);
                q = (own - 1u) & 63u;
                left = k < total ? (int)(l_D[q] - 64u * k) : 0;
                const uint32_t bq = l_B[q];
                lead_b = mark != 0u ? bq & 3u : 0u;     // a frame's first chunk: its lead bytes
                const uint32_t base = (bq & ~3u) + 64u * k;
#pragma unroll
                for (int c = 0; c < 4; ++c) R[c] = load16(fr, 16 * c < left ? base + 16u * c : OOR);
            };
            // The full-chunk sum reads every loaded register unconditionally, so the compiler's
            // wait for this group is placed here on every path.
            auto consume = [&](uint32_t k0, int left, uint32_t lead_b, const uint4 (&R)[4]) {
                uint32_t pa = 0, pb = 0;
#pragma unroll
                for (int c = 0; c < 4; ++c) {
                    pa = sad16(R[c].x, pa);
                    pb = sad16(R[c].y, pb);
                    pa = sad16(R[c].z, pa);
                    pb = sad16(R[c].w, pb);
                }
                // the piece holding the datagram end, if the end falls inside it: its bytes
                // [r, 16) are the next frame's (or padding) and come off again
                const int r = left & 15;
                const uint32_t pc = (uint32_t)left >> 4;
                const uint4 P = pc == 0u ? R[0] : pc == 1u ? R[1] : pc == 2u ? R[2] : R[3];
                const uint32_t pv[4] = {P.x, P.y, P.z, P.w};
                uint32_t ex = 0;
#pragma unroll
                for (int d = 0; d < 4; ++d) {
                    const int keep = min(max(r - 4 * d, 0), 4);
                    ex = sad16(pv[d] & (keep >= 4 ? 0u : 0xFFFFFFFFu << (8 * keep)), ex);
                }
                // and the first chunk's lead bytes [0, lead_b) (<= 3: in the first dword)
                ex = sad16(R[0].x & ((1u << (8u * lead_b)) - 1u), ex & (left > 0 && left < 64 && r != 0 ? ~0u : 0u));
                const uint32_t part = pa + pb - ex;
                const uint32_t Pp = scan_dpp(part);
                const uint32_t lo = max(my_cs, k0), hi = min(my_cs + my_nt, k0 + 64u);
                const uint32_t ph = __shfl(Pp, (int)((hi > k0 ? hi - 1u - k0 : 0u) & 63u), 64);
                const uint32_t pl = __shfl(Pp, (int)((lo > k0 ? lo - 1u - k0 : 0u) & 63u), 64);
                if (lo < hi) tsum += ph - (lo > k0 ? pl : 0u);
            };
            // Two groups in flight; one back edge, after the second group is consumed (a loop
            // exit between the two halves leaves the second group's loads pending at the
            // header, which then waits for everything). Groups past the end load nothing.
            uint32_t qa, qb, ea, eb;
            int la, lb;
            uint4 Ra[4], Rb[4];
            issue(0, qa, la, ea, Ra);
            tailed = true;
            if constexpr (G == 1) {
                // one group in flight: the next group's loads are issued after this one is summed
                for (uint32_t k0 = 0;; k0 += 64) {
                    consume(k0, la, ea, Ra);
                    if (k0 + 64 >= total) break;
                    issue(k0 + 64, qa, la, ea, Ra);
                }
                (void)qb; (void)lb; (void)eb; (void)Rb;
            } else if (total <= 64u) {
                // one group (e.g. every frame's tail one chunk): no groups issued past the end
                consume(0, la, ea, Ra);
            } else {
                for (uint32_t k0 = 0;; k0 += 128) {
                    issue(k0 + 64, qb, lb, eb, Rb);
                    consume(k0, la, ea, Ra);
                    issue(k0 + 128, qa, la, ea, Ra);
                    consume(k0 + 64, lb, eb, Rb);
                    if (k0 + 128 >= total) break;
                }
            }
            wave_sync();
            if (pd) {
                uint32_t t = fold32(tsum);
                if (fo & 1u) t = ((t & 0xFFu) << 8) | (t >> 8);   // buffer-aligned words: swap back
                const bool ok = fold32(t + (dw >> 16)) == 0xFFFFu;
                mstage[i & (RX_ROUND - 1u)] = (m & ~0x60u) | ((ok ? UDPDK_UDP_CSUM_OK : UDPDK_UDP_CSUM_BAD) << 5);
                acc_f0 += ok ? 0x10000u : 0x1000000u;
            }
    };

    // ---- span sweep: the step's bytes [A, Ep) read once, each 128-byte line by one load ----
    // (tools/probe/sweep_probe.hip: loads that each cover 1 KiB of consecutive 16-byte pieces read
    // 1.004x the span's bytes from HBM; one 64-byte chunk per lane, 1.030x; the per-frame windows
    // and tail chunks, 1.13x.) Blocks of 64 pieces, four per group, two groups in flight. Per
    // block: the pieces' RFC 1071 sums (buffer-aligned words, whole pieces) and their prefix sum
    // on the DPP network give Q(k), the sum of pieces [0, k) of the span, at each frame's two
    // piece indices (the piece holding its tail start, offset + 64, and the first piece past its
    // end); the block goes to a two-block LDS ring, from which a frame takes its header window
    // (the same 14 dwords load_win reads) when the block holding its last window byte arrives,
    // and the piece holding its end. Then a frame's tail sum over [offset + 64, offset + length)
    // = Q(end) - Q(start) - the lead bytes of the start piece (in its window) - the bytes of the
    // end piece past the frame (span_tail). Sums of 16-bit words up to 65535 bytes stay below
    // 2^32, so the differences of the wrapping prefix sums are exact.
    uint32_t *ring = reinterpret_cast<uint32_t *>(
        smem + classify_lds_bytes(a.n_lanes, a.tile_frames, a.hist16 != 0u)) + w * SPAN_RING_DW;
    uint32_t sp_Qs = 0, sp_Qe = 0;          // Q at the frame's tail-start piece and past its end
    uint4 sp_EP = make_uint4(0, 0, 0, 0);   // the piece holding the frame's end
    auto span_sweep = [&](uint32_t s, uint32_t A, uint32_t Ep, uint32_t o, uint32_t l) -> Win {
        const bool v = t0 + s * 64u + lane < t1;
        const uint32_t w0 = (o + 12u) & ~3u;
        const uint32_t s_idx = v ? (o + 64u - A) >> 4 : 0u;
        const uint32_t e_idx = v ? (o + l - A + 15u) >> 4 : 0u;
        const uint32_t wblk = v ? (w0 + 52u - A) >> 10 : 0xFFFFFFFFu;
        const uint32_t eblk = v && l > 64u && ((o + l) & 15u) != 0u ? (o + l - A) >> 10 : 0xFFFFFFFFu;
        const uint32_t ep = ((o + l - A) >> 4) & 127u;     // ring piece of the frame's end
        const uint32_t rb = ((w0 - A) >> 2) & 511u;         // ring dword of the window's first
        const uint32_t nb = (Ep - A + 1023u) >> 10;          // blocks
        const uint32_t ng = (nb + 3u) >> 2;                  // groups
        uint32_t C = 0, Qs = 0, Qe = 0;
        uint32_t Dw[14];
#pragma unroll
        for (int k = 0; k < 14; ++k) Dw[k] = 0;
        uint4 EP = make_uint4(0, 0, 0, 0);
        uint4 *rq = reinterpret_cast<uint4 *>(ring);
        auto block = [&](uint32_t b, const uint4 &R) {
            const uint32_t ps = sad16(R.x, sad16(R.z, 0u)) + sad16(R.y, sad16(R.w, 0u));
            const uint32_t P = scan_dpp(ps);
            const uint32_t ds = s_idx - 64u * b - 1u, de = e_idx - 64u * b - 1u;
            const uint32_t Ps = (uint32_t)__shfl((int)P, (int)(ds & 63u), 64);
            const uint32_t Pe = (uint32_t)__shfl((int)P, (int)(de & 63u), 64);
            Qs = ds < 64u ? C + Ps : Qs;
            Qe = de < 64u ? C + Pe : Qe;
            C += (uint32_t)__builtin_amdgcn_readlane((int)P, 63);
            wave_sync();                                     // the previous block's ring reads first
            rq[(b & 1u) * 64u + lane] = R;
            if ((b & 1u) == 0u && lane < 4u) rq[128u + lane] = R;
            wave_sync();
            if (__ballot(wblk == b)) {
                if (wblk == b) {
#pragma unroll
                    for (int k = 0; k < 14; ++k) Dw[k] = ring[rb + k];
                }
            }
            if (__ballot(eblk == b)) {
                if (eblk == b) EP = rq[ep];
            }
        };
        auto issue = [&](uint32_t g, uint4 (&R)[4]) {
#pragma unroll
            for (uint32_t c = 0; c < 4; ++c) {
                const uint32_t x = A + 4096u * g + 1024u * c + 16u * lane;
                R[c] = load16(fr, x < Ep ? x : OOR);
            }
        };
        auto consume = [&](uint32_t g, const uint4 (&R)[4]) {
#pragma unroll
            for (uint32_t c = 0; c < 4; ++c)
                if (4u * g + c < nb) block(4u * g + c, R[c]);
        };
        uint4 Ra[4], Rb[4];
        issue(0, Ra);
        for (uint32_t g = 0;; g += 2) {
            issue(g + 1u, Rb);
            consume(g, Ra);
            issue(g + 2u, Ra);
            consume(g + 1u, Rb);
            if (g + 2u >= ng) break;
        }
        sp_Qs = Qs;
        sp_Qe = Qe;
        sp_EP = EP;
        Win r;
        r.a = make_uint4(Dw[0], Dw[1], Dw[2], Dw[3]);
        r.b = make_uint4(Dw[4], Dw[5], Dw[6], Dw[7]);
        r.c = make_uint4(Dw[8], Dw[9], Dw[10], Dw[11]);
        r.d = make_uint2(Dw[12], Dw[13]);
        return r;
    };
    // the swept frame's tail sum over buffer bytes [o + 64, o + l) (buffer-aligned 16-bit words):
    // D = the window's raw dwords (buffer dwords from w0 = (o + 12) & ~3)
    auto span_tail = [&](uint32_t o, uint32_t l, const uint32_t (&D)[14]) -> uint32_t {
        const int hi = (int)(o + 64u - ((o + 12u) & ~3u)), lo = hi - (int)((o + 64u) & 15u);
        uint32_t lead = 0;
#pragma unroll
        for (int k = 9; k < 14; ++k) lead = sad16(D[k] & byte_mask(lo, hi, 4 * k), lead);
        const int r = (int)((o + l) & 15u);
        const uint32_t ev[4] = {sp_EP.x, sp_EP.y, sp_EP.z, sp_EP.w};
        uint32_t over = 0;
#pragma unroll
        for (int d = 0; d < 4; ++d) over = sad16(ev[d] & byte_mask(r, 16, 4 * d), over);
        return sp_Qe - sp_Qs - lead - (r != 0 ? over : 0u);
    };

    // ---- demux of one frame: btable_get_bindings + list walk, udpdk_poller.c:376-405 ----
    // i: the frame's index in the tile, m: its verdict word so far (verdict field 0xF: UDP, port
    // lookup pending), Sv: {raw dst port | is-UDP << 16, raw dst IPv4}, Ev: the port's 16-byte
    // entry (first binding inline; the binding list is walked only for ports with several).
    // Returns the final verdict word; counts the frame and adds it to the tile histogram.
    auto demux_frame = [&](uint32_t i, uint32_t m, uint2 Sv, uint4 Ev) -> uint32_t {
        const bool valid = t0 + i < t1;
        const uint4 e = (Sv.x >> 16) ? Ev : make_uint4(0, 0, 0, 0);
        const uint32_t dip = Sv.y;
        const bool match0 = e.x != 0u && (dip == e.z || e.z == 0u);     // poller.c:391
        uint32_t fan = match0 ? 1u : 0u;
        uint32_t first = match0 ? (e.w & 0x7FFFFFFFu) : 0u;
        const bool walk = e.x > 1u && !(match0 && !(e.w >> 31));        // poller.c:396-403
        if (__ballot(walk)) {
            if (walk) {
                for (uint32_t b = 1; b < e.x; ++b) {
                    const uint2 bd = a.binds[e.y + b];
                    if (dip == bd.x || bd.x == 0u) {
                        const uint32_t sock = bd.y & 0x7FFFFFFFu;
                        if (fan > 0 && a.n_lanes > 1u)
                            hist_add(sock & a.lane_mask, 1u);           // clones (rare)
                        if (fan == 0) first = sock;
                        ++fan;
                        if (!(bd.y >> 31)) break;
                    }
                }
            }
        }
        const uint32_t pre = m & 0xFu;
        const uint32_t verdict = pre != 0xFu ? pre
                               : e.x == 0u ? UDPDK_V_NO_BIND
                               : fan ? UDPDK_V_DELIVERED : UDPDK_V_NO_MATCH;
        const uint32_t fin = (m & ~0xFu) | verdict | (min(fan, 127u) << 9) | ((first & 0xFFFFu) << 16);
        // per-lane packed counters (8-bit fields; a lane sees <= 64 frames per tile)
        const uint32_t vinc = valid ? 1u << (8u * (verdict & 3u)) : 0u;
        acc_v0 += verdict < 4u ? vinc : 0u;
        acc_v1 += verdict < 4u ? 0u : vinc;
        acc_fan += fan;
        const bool delivered = valid && fan > 0u;
        // first delivery of every frame into the tile histogram; small key spaces are
        // aggregated with a wave multi-split first (all 64 lanes may share one lane)
        // (one lane: the tile's count is its delivery counter, written at the tile end)
        const uint32_t key = first & a.lane_mask;
        if (a.n_lanes == 1u) {
        } else if (a.key_bits <= 4u) {
            unsigned long long peers = __ballot(delivered);
            for (uint32_t bit = 0; bit < a.key_bits; ++bit) {
                const bool kb = (key >> bit) & 1u;
                const unsigned long long bal = __ballot(kb);
                peers &= kb ? bal : ~bal;
            }
            if (delivered && lane == (uint32_t)__ffsll((long long)peers) - 1u)
                hist_add(key, (uint32_t)__popcll(peers));
        } else if (delivered) {
            hist_add(key, 1u);
        }
        return fin;
    };
    // the argument-borne bind table (few bound ports): the port's entry from LDS (slot n_inl is
    // zero: an unbound port); one bound port, the pktgen case, is one compare
    auto inl_entry = [&](uint32_t pt) -> uint4 {
        uint32_t k = a.n_inl;
        if (a.n_inl == 1u) {
            k = pt == a.inl_port[0] ? 0u : 1u;
        } else {
#pragma unroll
            for (uint32_t q = 0; q < UDPDK_INLINE_PORTS; ++q)
                k = q < a.n_inl && pt == a.inl_port[q] ? q : k;
        }
        return inl_tab[k];
    };
    // One-round tiles with the argument-borne table demux each frame in its step (an LDS lookup,
    // no global load to batch): the tile's end no longer waits for a demux pass over the round.
    // Several rounds keep the round's pass (their verdict words are stored by it, after the
    // round's tail passes).
    const bool step_demux = a.inl && nbuf == 1u;
    uint32_t pf_o[SPT], pf_l[SPT], pf_t[SPT];             // MR: the next round's descriptors
    // rounds of RX_ROUND frames: SPR steps per wave (each followed by its tail pass when a frame
    // of the step is pending), then the round's demux pass
    for (uint32_t rnd = 0; rnd < steps / RSTEPS; ++rnd) {
#pragma unroll 1
        for (uint32_t jstep = 0; jstep < SPR; ++jstep) {
            const uint32_t p = t0 + st * 64 + lane;
            const bool valid = p < t1;
            const uint32_t off = c_off, len = c_lp & 0xFFFFu;
            const bool good = valid && len <= a.frames_bytes && off <= a.frames_bytes - len;
            // MR: the next round's descriptors go out at the round's first step, into registers,
            // and are stored to LDS at its staging step: the staging no longer waits a round trip
            // (config 5: a descriptor round trip per round was a fifth of each workgroup's time)
            if (MR && jstep == 0u && rnd + 1u < steps / RSTEPS) {
                stage_load(rnd + 1u, pf_o, pf_l, pf_t);
                __builtin_amdgcn_sched_barrier(0);
            }
            const uint32_t nst = st + CLS_WAVES;
            uint32_t n_off, n_lp;
            Win NW;
            // Fairness between the workgroups sharing a CU: the instruction arbiter favours higher
            // priority, then age, so the workgroups dispatched first kept winning the memory
            // pipeline and the launch waited for the last ones (config 3 stamps: workgroup
            // durations 168 / 227 / 299 us at p0 / p50 / p100, all resident from the start). A wave
            // drops a priority level each quarter of its steps, so the ones behind catch up.
            // (Long-frame forms only: config 2's G = 1 form measured even to slightly slower.)
            if constexpr (G == 2) {
                const uint32_t lv = (4u * (st / CLS_WAVES)) / (steps / CLS_WAVES);
                if (lv == 0u) __builtin_amdgcn_s_setprio(3);
                else if (lv == 1u) __builtin_amdgcn_s_setprio(2);
                else if (lv == 2u) __builtin_amdgcn_s_setprio(1);
                else __builtin_amdgcn_s_setprio(0);
            }
            // a step that sweeps its span reads its window from the sweep (no window was loaded)
            if (SPAN && span_cur) {
                W = span_sweep(st, span_A, span_E, off, len);
                tailed = true;
            }

            // ---- header fields from the window registers (lane = frame) ----
            const uint32_t D[14] = {W.a.x, W.a.y, W.a.z, W.a.w, W.b.x, W.b.y, W.b.z, W.b.w,
                                    W.c.x, W.c.y, W.c.z, W.c.w, W.d.x, W.d.y};
            const uint32_t sh = off & 3u;     // lanes whose window was not loaded: unused words
            uint32_t g[13];                   // g[i] = frame bytes 12+4i ..
#pragma unroll
            for (int i = 0; i < 13; ++i) g[i] = __builtin_amdgcn_alignbyte(D[i + 1], D[i], sh);
            // IPv4 gate (udpdk_poller.c:334): the ptype array's L3_IPV4 bit when given, else derived
            // from ether_type (frames shorter than an Ethernet header are not IPv4)
            const uint32_t eth_ip = (len >= 14u && (g[0] & 0xFFFFu) == 0x0008u) ? 0x10u : 0u;
            const bool ipv4 = good && ((has_ptype ? (c_lp >> 12) : eth_ip) & 0x10u);
            const uint32_t frag = ((g[2] & 0xFFu) << 8) | ((g[2] >> 8) & 0xFFu);
            const bool l3 = ipv4 && len >= 42u;
            const bool fragd = (frag & 0x3FFFu) != 0u;                // udpdk_poller.c:338
            // a fragment needs only its IPv4 header (poller.c:338-361): 34-41 B fragments reassemble
            const bool l3h = ipv4 && len >= 34u;
            const bool hdr = l3 || (l3h && fragd);                    // IPv4 flags and counters
            const bool not_udp = (g[2] >> 24) != 17u;                 // udpdk_poller.c:368-371
            const bool is_udp = l3 && !fragd && !not_udp;
            const uint32_t dport = g[6] & 0xFFFFu;                   // poller.c:372
            STAMP(1);

            // ---- everything the header window gives ----
            // IPv4 header checksum over the fixed 20 bytes at offset 14 (RFC 1071)
            const uint32_t ipraw = sad16(g[4], sad16(g[3], sad16(g[2], sad16(g[1],
                                   (g[0] >> 16) + (g[5] & 0xFFFFu)))));
            const bool ip_ok = fold32(ipraw) == 0xFFFFu;
            const bool ihl_ne5 = ((g[0] >> 16) & 0x0Fu) != 5u;
            const uint32_t dip = (g[4] >> 16) | (g[5] << 16);         // poller.c:373
            const uint32_t ulen_raw = g[6] >> 16;
            const uint32_t ulen = ((ulen_raw & 0xFFu) << 8) | (ulen_raw >> 8);
            const uint32_t ucks = g[7] & 0xFFFFu;
            const bool len_bad = ulen < 8u || 34u + ulen > len;
            // UDP checksum (RFC 768 over the datagram, frame bytes [34, 34 + ulen), plus the pseudo-
            // header {src, dst, proto 17, udp length}), computed only where it decides the state:
            // a frame whose datagram ends within the window is summed here; a longer one is left to
            // the tile's tail pass (state 3 = pending until then). Ethernet padding after the
            // datagram is never summed.
            const bool need_cs = is_udp && ucks != 0u && !len_bad;
            const uint32_t dge = 34u + ulen;                          // datagram end (<= len)
            // a swept step has every frame's tail sum over [64, len): a datagram that ends there
            // (no padding) is complete now, any other pending one goes to the tail pass
            const bool swept = SPAN && span_cur && dge == len;
            const bool pend = need_cs && dge > 64u && !swept;
            const bool pend_sw = need_cs && dge > 64u && swept;
            uint32_t ws = 0, ws2 = 0;
#pragma unroll
            for (int i = 6; i < 13; i += 2) ws = sad16(g[i], ws);
#pragma unroll
            for (int i = 7; i < 13; i += 2) ws2 = sad16(g[i], ws2);
            ws += ws2;
            if (__ballot(need_cs && dge < 64u)) {                     // short or padded frames
                uint32_t wm = 0;
#pragma unroll
                for (int i = 6; i < 13; ++i) wm = sad16(g[i] & byte_mask(34, (int)dge, 12 + 4 * i), wm);
                ws = dge < 64u ? wm : ws;
            }
            const uint32_t us = ws + (g[5] >> 16) + (g[3] >> 16) + (g[4] & 0xFFFFu) + (dip & 0xFFFFu) +
                                (dip >> 16) + 0x1100u + ulen_raw;
            dgl[(st * 64 + lane) & (RX_ROUND - 1u)] = dge | fold32(us) << 16;
            // the swept datagrams' checksums (buffer-aligned tail words: swapped back at odd offsets)
            bool sw_ok = false;
            if (SPAN && __ballot(pend_sw)) {
                uint32_t t = fold32(span_tail(off, len, D));
                if (off & 1u) t = ((t & 0xFFu) << 8) | (t >> 8);
                sw_ok = fold32(t + fold32(us)) == 0xFFFFu;
            }
            STAMP(2);

            // ---- next step of this wave: window loads stay in flight across the rest of this step.
            // A step with pending frames issues them after its tail pass instead: a window's lines
            // (the one it shares with the frame's first tail chunk, and the one the previous
            // frame's tail ends in) are then still in L2 when that step's tail reads them, where a
            // window loaded a whole step earlier had left L2 by then (IMIX fetched 1.29x its bytes).
            // A next step that sweeps its span loads no window.
            read_desc(nst, n_off, n_lp);      // in range of the buffers for any s (unused past the tile)
            uint32_t n_A = 0, n_E = 0;
            const bool span_n = span_check(nst, n_off, n_lp & 0xFFFFu, n_A, n_E);
            const bool tail_now = __ballot(pend) != 0ull;
            if (!tail_now) NW = load_win(nst, n_off, n_lp & 0xFFFFu, span_n);

            // ---- what does not need the port entry: UDP state, flags, flag counters ----
            const uint32_t state = ucks == 0u ? UDPDK_UDP_CSUM_NONE
                                 : pend ? 3u
                                 : pend_sw ? (sw_ok ? UDPDK_UDP_CSUM_OK : UDPDK_UDP_CSUM_BAD)
                                 : (len_bad || fold32(us) != 0xFFFFu) ? UDPDK_UDP_CSUM_BAD
                                                                       : UDPDK_UDP_CSUM_OK;
            const uint32_t pre = !good ? UDPDK_V_BAD_DESC
                               : !ipv4 ? UDPDK_V_NOT_IPV4
                               : !l3h ? UDPDK_V_TRUNC
                               : fragd ? UDPDK_V_FRAG
                               : !l3 ? UDPDK_V_TRUNC
                               : not_udp ? UDPDK_V_NOT_UDP : 0xFFu;       // 0xFF: UDP, demux pending
            const uint32_t l3f = hdr ? ((ip_ok ? 1u : 0u) << 4 | (ihl_ne5 ? 1u : 0u) << 8) : 0u;
            const uint32_t udpf = is_udp ? (state << 5 | (len_bad ? 1u : 0u) << 7) : 0u;
            // (pending frames count their UDP state in the tail pass)
            acc_f0 += (hdr && !ip_ok ? 1u : 0u) | (hdr && ihl_ne5 ? 0x100u : 0u) |
                      (is_udp && state == UDPDK_UDP_CSUM_OK ? 0x10000u : 0u) |
                      (is_udp && state == UDPDK_UDP_CSUM_BAD ? 0x1000000u : 0u);
            acc_f1 += (is_udp && state == UDPDK_UDP_CSUM_NONE ? 1u : 0u) | (is_udp && len_bad ? 0x100u : 0u);
            if (good) lane_bytes += len;

            // the port-table lookup: now (step_demux), else in the round's demux pass (verdict
            // field 0xF until then)
            {
                const uint32_t w0 = (pre == 0xFFu ? 0xFu : pre) | l3f | udpf;
                const uint2 sv = make_uint2(dport | (is_udp ? 0x10000u : 0u), dip);
                const uint32_t si = (st * 64 + lane) & (RX_ROUND - 1u);
                if (step_demux) {
                    mstage[si] = demux_frame(st * 64 + lane, w0, sv, inl_entry(dport));
                } else {
                    mstage[si] = w0;
                    dstash[si] = sv;
                }
            }
            if (tail_now) {
                tail_step(st);
                NW = load_win(nst, n_off, n_lp & 0xFFFFu, span_n);
            }
            STAMP(6);
            // next round's descriptors into the other buffer at the wave's next-to-last step of a
            // round (its steps of round r are 16 r + w + CLS_WAVES j, j < SPR): the last reads of that
            // buffer were before the previous round's barrier, and the next round is first read at
            // j = SPR - 1.
            // Uniform across the workgroup (every wave has steps / 4 steps).
            if ((st / CLS_WAVES) % SPR == SPR - 2u && st / RSTEPS + 1u < steps / RSTEPS) {
                if constexpr (MR != 0)
                    stage_store(st / RSTEPS + 1u, pf_o, pf_l, pf_t);
                else
                    stage(st / RSTEPS + 1u);
                __syncthreads();
                STAMP(5);
            }
            W = NW;
            c_off = n_off;
            c_lp = n_lp;
            span_cur = span_n;
            span_A = n_A;
            span_E = n_E;
            st = nst;
        }
        // ---- demux pass (not step_demux): the round's port-table lookups of this wave, all SPR
        // steps' 16-byte entries in flight at once (one round trip per round instead of one
        // exposed per step) ----
        if (!step_demux) {
            uint4 E[SPR];
            uint2 S[SPR];
#pragma unroll
            for (uint32_t j = 0; j < SPR; ++j) S[j] = dstash[((st - RSTEPS + CLS_WAVES * j) * 64 + lane) & (RX_ROUND - 1u)];
            if (a.inl) {
#pragma unroll
                for (uint32_t j = 0; j < SPR; ++j) E[j] = inl_entry(S[j].x & 0xFFFFu);
            } else {
#pragma unroll
                for (uint32_t j = 0; j < SPR; ++j) E[j] = a.port_tab[S[j].x & 0xFFFFu];
            }
#pragma unroll
            for (uint32_t j = 0; j < SPR; ++j) {
                const uint32_t i = (st - RSTEPS + CLS_WAVES * j) * 64 + lane;
                const uint32_t fin = demux_frame(i, mstage[i & (RX_ROUND - 1u)], S[j], E[j]);
                mstage[i & (RX_ROUND - 1u)] = fin;
                // a tile of several rounds stores each round's verdict words here (its LDS holds
                // one round, so three workgroups fit a CU at 4096 lanes instead of two)
                if (nbuf > 1u && t0 + i < t1) a.meta[t0 + i] = fin;
            }
        }
        STAMP(3);
    }

    // The tile's stores go out first (its verdict words are all in LDS after this barrier), the
    // counter reduction after them: the fused completion's drain then finds them written.
    __syncthreads();
    auto tile_counter = [&](uint32_t c) -> uint32_t {
        uint32_t v = 0;
#pragma unroll
        for (int i = 0; i < CLS_WAVES; ++i) v += cntw[i * 16 + c];
        return v;
    };
    // Fused completion (a.fuse, single lane, one-round tiles): every store another workgroup may
    // read in this launch is written through (sc1) and drained before the workgroup's arrival,
    // as cdna_hip_programming.md Guideline 16 / MI355X_MICROARCH.md "Valid forms" require.
    const bool fuse = a.fuse != nullptr;
    uint32_t tcount = 0;                                   // the tile's deliveries (spec / fuse)
    if (a.spec_pkt) {
        // Speculative lane entries (single lane, 1024-frame one-round tile, 4 frames per
        // thread): the tile's delivered frames in order at t0 + rank, which is where they belong
        // when every earlier tile delivered all its frames. rx_compact1 (or the fused completion
        // below) keeps them then and rewrites the later tiles otherwise.
        __shared__ uint32_t spec_ws[CLS_WAVES];
        const uint32_t nv = t1 - t0, j0 = 4u * tid;
        uint32_t d = 0;
        if (j0 < nv) {
            const uint4 v = reinterpret_cast<const uint4 *>(mstage)[tid];
            d = ((v.x & 0xFu) == UDPDK_V_DELIVERED ? 1u : 0u) |
                ((v.y & 0xFu) == UDPDK_V_DELIVERED && j0 + 1u < nv ? 2u : 0u) |
                ((v.z & 0xFu) == UDPDK_V_DELIVERED && j0 + 2u < nv ? 4u : 0u) |
                ((v.w & 0xFu) == UDPDK_V_DELIVERED && j0 + 3u < nv ? 8u : 0u);
        }
        const uint32_t cnt = (uint32_t)__builtin_popcount(d);
        const uint32_t incl = scan_dpp(cnt);
        if (lane == 63) spec_ws[w] = incl;
        __syncthreads();
        uint32_t pos = t0 + incl - cnt;
#pragma unroll
        for (uint32_t i = 0; i < CLS_WAVES; ++i) {
            pos += i < w ? spec_ws[i] : 0u;
            tcount += spec_ws[i];
        }
        // a tile short of a full tile's deliveries (the last tile never counts: nothing follows
        // it) marks its successors' entries wrong; every other word of the flag stays untouched
        if (tid == 0 && tile + 1u < a.n_tiles && tcount != a.tile_frames)
            atomicMax(&a.spec_nonfull[tile % UDPDK_SPEC_WORDS],
                      ((unsigned long long)a.spec_epoch << 32) | (0xFFFFFFFFu - tile));
        const uint32_t f = t0 + j0;
        if (fuse) {
            // written through: the completing workgroup may rewrite these words (no stale dirty
            // copy may stay behind in this XCD's L2) -- range-checked by the resource
            const __amdgpu_buffer_rsrc_t sr =
                make_rsrc(a.spec_pkt, a.spec_cap >= 0x40000000u ? 0xFFFFFFFCu : a.spec_cap * 4u);
            if (d == 0xFu && (pos & 3u) == 0u) {
                const __attribute__((ext_vector_type(4))) uint32_t x = {f, f + 1u, f + 2u, f + 3u};
                __builtin_amdgcn_raw_buffer_store_b128(x, sr, (int)(4u * pos), 0, 16);
            } else {
#pragma unroll
                for (uint32_t j = 0; j < 4; ++j)
                    if ((d >> j) & 1u) {
                        __builtin_amdgcn_raw_buffer_store_b32(f + j, sr, (int)(4u * pos), 0, 16);
                        ++pos;
                    }
            }
        } else if (d == 0xFu && (pos & 3u) == 0u && pos + 4u <= a.spec_cap) {
            *reinterpret_cast<uint4 *>(a.spec_pkt + pos) = make_uint4(f, f + 1u, f + 2u, f + 3u);
        } else {
#pragma unroll
            for (uint32_t j = 0; j < 4; ++j)
                if ((d >> j) & 1u) {
                    if (pos < a.spec_cap) a.spec_pkt[pos] = f + j;
                    ++pos;
                }
        }
    }
    if (nbuf == 1u) {
        const uint32_t nv = t1 - t0;
        uint32_t *dst = a.meta + t0;
        if (fuse) {
            // verdict words written through (the completing workgroup reads them back when a
            // tile was not full)
            const __amdgpu_buffer_rsrc_t mr = make_rsrc(dst, nv * 4u);
            if (((uintptr_t)dst & 15u) == 0) {
                const uint4 *s4 = reinterpret_cast<const uint4 *>(mstage);
                for (uint32_t i = tid; i < (nv + 3u) / 4u; i += CLS_BLOCK) {
                    const uint4 v = s4[i];
                    const __attribute__((ext_vector_type(4))) uint32_t x = {v.x, v.y, v.z, v.w};
                    if (4u * i + 4u <= nv)
                        __builtin_amdgcn_raw_buffer_store_b128(x, mr, (int)(16u * i), 0, 16);
                    else
                        for (uint32_t j = 4u * i; j < nv; ++j)
                            __builtin_amdgcn_raw_buffer_store_b32(mstage[j], mr, (int)(4u * j), 0, 16);
                }
            } else {
                for (uint32_t i = tid; i < nv; i += CLS_BLOCK)
                    __builtin_amdgcn_raw_buffer_store_b32(mstage[i], mr, (int)(4u * i), 0, 16);
            }
        } else if (nv == a.tile_frames && ((uintptr_t)dst & 15u) == 0) {
            uint4 *d4 = reinterpret_cast<uint4 *>(dst);
            const uint4 *s4 = reinterpret_cast<const uint4 *>(mstage);
            for (uint32_t i = tid; i < nv / 4; i += CLS_BLOCK) d4[i] = s4[i];
        } else {
            for (uint32_t i = tid; i < nv; i += CLS_BLOCK) dst[i] = mstage[i];
        }
    }
    // ---- tile counters: one row per wave (lanes 0-15), summed by the readers ----
    uint32_t sc[UDPDK_N_COUNTERS];
    {
        auto wsum = [](uint32_t v) { return (uint32_t)__builtin_amdgcn_readlane((int)scan_dpp(v), 63); };
        const uint32_t packed[4] = {acc_v0, acc_v1, acc_f0, acc_f1};
        const int field[4][4] = {{0, 1, 2, 3}, {4, 5, 6, 7},
                                 {UDPDK_C_IP_BAD, UDPDK_C_IHL_NE5, UDPDK_C_UDP_OK, UDPDK_C_UDP_BAD},
                                 {UDPDK_C_UDP_NONE, UDPDK_C_LEN_BAD, -1, -1}};
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const uint32_t ev = wsum(packed[k] & 0x00FF00FFu);        // 16-bit sums: no carry
            const uint32_t od = wsum((packed[k] >> 8) & 0x00FF00FFu);
            if (field[k][0] >= 0) sc[field[k][0]] = ev & 0xFFFFu;
            if (field[k][1] >= 0) sc[field[k][1]] = od & 0xFFFFu;
            if (field[k][2] >= 0) sc[field[k][2]] = ev >> 16;
            if (field[k][3] >= 0) sc[field[k][3]] = od >> 16;
        }
        sc[UDPDK_C_DELIVERIES] = wsum(acc_fan);
        sc[UDPDK_C_BYTES] = wsum(lane_bytes);
    }
    {
        uint32_t row = 0;
#pragma unroll
        for (int c = 0; c < UDPDK_N_COUNTERS; ++c) row = lane == (uint32_t)c ? sc[c] : row;
        if (lane < UDPDK_N_COUNTERS) cntw[w * 16 + lane] = row;
        if (tailed && lane == 0) tail_any = 1u;
    }
    __syncthreads();
    STAMP(7);
    if (a.n_lanes == 1u) {
        if (tid == 0) {
            if (fuse)
                __hip_atomic_store(&a.hist[tile], tcount, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            else
                a.hist[tile] = tile_counter(UDPDK_C_DELIVERIES);
        }
    } else {
        if (a.hist16) {           // u16 row of n_lanes (rounded up to even) counts
            const uint32_t hw = (a.n_lanes + 1u) >> 1;
            for (uint32_t s = tid; s < hw; s += CLS_BLOCK) a.hist[(size_t)tile * hw + s] = hist[s];
        } else {
            for (uint32_t s = tid; s < a.n_lanes; s += CLS_BLOCK)
                a.hist[(size_t)tile * a.n_lanes + s] = hist[s];
        }
    }
    if (tid < UDPDK_N_COUNTERS) a.tile_cnt[(size_t)tile * UDPDK_N_COUNTERS + tid] = tile_counter(tid);
    // the host's kernel choice for its next calls: this call needed tail passes. Sampled (every
    // 64th tile, one lane): a store to host memory per wave cost IMIX classify 91 -> 544 us. After
    // the fused completion: its drain would otherwise wait for these stores to cross PCIe.
    const bool hint = a.hint && (tile & 63u) == 0u && tid == 0;
    const bool tail_seen = tail_any != 0u;
    if (fuse) classify_complete(a, tile, tcount, tid, lane, w, smem);
    if (hint) {
        if (tail_seen)
            __hip_atomic_store(&a.hint[UDPDK_HINT_TAIL], a.seq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        if (tile == 0u)
            __hip_atomic_store(&a.hint[UDPDK_HINT_DONE], a.seq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    }
#ifdef UDPDK_STAMPS
    STAMP(4);                                              // slot 4: fused completion
    STAMP_END();
    __syncthreads();
    if (a.dbg && w == 0 && lane < 16) a.dbg[blockIdx.x * 16 + lane] = st_acc[lane];
#endif
}
template __global__ void rx_classify<1, 0>(RxArgs a);
template __global__ void rx_classify<2, 0>(RxArgs a);
template __global__ void rx_classify<1, 1>(RxArgs a);
template __global__ void rx_classify<2, 1>(RxArgs a);


// ------------------------------------------------------------------------------------------
// rx_compact1: the single-lane batch's lane (no fan-out: every delivery is a whole frame).
// Workgroup = tile (grid-stride over the tiles after the first flagged one when rx_classify
// wrote speculative entries). Each wave ballots its quarter of the tile's verdict words (delivered =
// verdict 0) into LDS masks, the tile's base is the sum of the predecessors' delivery counts
// (<= n_tiles words, read straight from the classify kernel's per-tile histogram: no scan
// kernel and no cross-workgroup waits), then every delivered frame writes its index.
// The last tile's workgroup writes lane_off[1] = total.
// ------------------------------------------------------------------------------------------
__device__ __forceinline__ void compact1_tile(const Compact1Args &a, uint32_t tile, uint32_t steps,
                                              uint32_t tid, uint32_t lane, uint32_t w)
{
    constexpr uint32_t MAXS = RX_TILE_MAX / RX_BLOCK;      // steps per wave, <= 64
    __shared__ unsigned long long msk[RX_WAVES][MAXS];
    __shared__ uint32_t red[2 * RX_WAVES];
    const uint32_t t1 = min(a.n, (tile + 1) * a.tile_frames);
    const uint32_t wb = tile * a.tile_frames + w * steps * 64;
    const uint32_t plast = a.n - 1u;
    // predecessors' counts first (the first two per thread unconditionally, clamped), so they
    // are in flight together with the verdict words: one memory round trip for both
    const uint32_t tl = a.n_tiles - 1u;
    const uint32_t c0 = a.tile_count[min(tid, tl)], c1 = a.tile_count[min(tid + RX_BLOCK, tl)];
    uint32_t wcount = 0;
    for (uint32_t s0 = 0; s0 < steps; s0 += 4) {
        uint32_t mv[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) mv[u] = a.meta[min(wb + (s0 + u) * 64 + lane, plast)];
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            if (s0 + u >= steps) break;                     // fewer than 4 steps per wave
            const uint32_t p = wb + (s0 + u) * 64 + lane;
            const unsigned long long m = __ballot(p < t1 && (mv[u] & 0xFu) == UDPDK_V_DELIVERED);
            if (lane == 0) msk[w][s0 + u] = m;
            wcount += (uint32_t)__popcll(m);
        }
    }
    uint32_t pre = 0;
    if (!a.base) {
        pre = (tid < tile ? c0 : 0u) + (tid + RX_BLOCK < tile ? c1 : 0u);
        for (uint32_t t = tid + 2 * RX_BLOCK; t < tile; t += RX_BLOCK) pre += a.tile_count[t];
        pre = wave_sum(pre);
    }
    if (lane == 0) { red[w] = pre; red[RX_WAVES + w] = wcount; }
    __syncthreads();
    // many tiles: the base comes from rx_tile_base (the all-predecessor sum grows with tiles^2)
    uint32_t base = a.base ? a.base[tile] : 0u, tcount = 0, before = 0;
#pragma unroll
    for (int i = 0; i < RX_WAVES; ++i) {
        base += red[i];
        tcount += red[RX_WAVES + i];
        before += (uint32_t)i < w ? red[RX_WAVES + i] : 0u;
    }
    uint32_t run = base + before;
    const uint32_t total = base + tcount;
    if (tile == a.n_tiles - 1u && tid == 0) {
        a.lane_off[0] = 0u;
        a.lane_off[1] = total;
        *a.total = total;
    }
    const unsigned long long lt = (1ull << lane) - 1ull;
    for (uint32_t s = 0; s < steps; ++s) {
        const unsigned long long m = msk[w][s];
        if ((m >> lane) & 1ull) {
            const uint32_t pos = run + (uint32_t)__popcll(m & lt);
            if (pos < a.lane_cap) a.lane_pkt[pos] = wb + s * 64 + lane;
        }
        run += (uint32_t)__popcll(m);
    }
}

__global__ void __launch_bounds__(RX_BLOCK)
rx_compact1(Compact1Args a)
{
    const uint32_t tid = threadIdx.x, lane = lane_id(), w = tid >> 6;
    const uint32_t steps = a.tile_frames / RX_BLOCK;
    const uint32_t tl = a.n_tiles - 1u;
    // speculative entries: rx_classify placed every tile's entries at tile x tile_frames + rank,
    // right when every earlier tile delivered all its frames, i.e. up to and including the call's
    // first flagged tile. Every wave reads the 64 flag words (one load per lane) and takes the
    // smallest flagged tile; only the tiles after it are rewritten (grid-stride: the launch is
    // small, so the common all-full call costs one flag read and the total's store).
    uint32_t t_first = blockIdx.x;
    if (a.spec) {
        const unsigned long long nf = __hip_atomic_load(&a.spec_nonfull[lane % UDPDK_SPEC_WORDS], __ATOMIC_RELAXED,
                                                        __HIP_MEMORY_SCOPE_AGENT);
        uint32_t first = (uint32_t)(nf >> 32) == a.spec_epoch ? 0xFFFFFFFFu - (uint32_t)nf : 0xFFFFFFFFu;
#pragma unroll
        for (int d = 32; d >= 1; d >>= 1) first = min(first, (uint32_t)__shfl_xor((int)first, d, 64));
        if (first < tl && blockIdx.x == 0 && tid == 0 && a.hint)
            __hip_atomic_store(&a.hint[UDPDK_HINT_NONFULL], a.seq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        if (first >= tl) {
            if (blockIdx.x == 0 && tid == 0) {
                const uint32_t total = tl * a.tile_frames + a.tile_count[tl];
                a.lane_off[0] = 0u;
                a.lane_off[1] = total;
                *a.total = total;
            }
            return;
        }
        t_first = first + 1u + blockIdx.x;
    }
    for (uint32_t tile = t_first; tile < a.n_tiles; tile += gridDim.x) {
        compact1_tile(a, tile, steps, tid, lane, w);
        __syncthreads();                       // msk / red reused by the next tile
    }
}

// ------------------------------------------------------------------------------------------
// rx_tile_base: exclusive prefix of the per-tile delivery counts for rx_compact1 when a batch
// has many tiles (one workgroup: a contiguous block of tiles per thread + a block scan).
// ------------------------------------------------------------------------------------------
__global__ void __launch_bounds__(1024)
rx_tile_base(const uint32_t *cnt, uint32_t *base, uint32_t n)
{
    __shared__ uint32_t wsum[16];
    const uint32_t tid = threadIdx.x, lane = lane_id(), w = tid >> 6;
    const uint32_t per = (n + 1023u) / 1024u, b0 = min(n, tid * per), b1 = min(n, b0 + per);
    uint32_t s = 0;
    for (uint32_t i = b0; i < b1; ++i) s += cnt[i];
    const uint32_t incl = wave_incl_scan(s);
    if (lane == 63) wsum[w] = incl;
    __syncthreads();
    uint32_t before = incl - s;
    for (uint32_t i = 0; i < w; ++i) before += wsum[i];
    for (uint32_t i = b0; i < b1; ++i) {
        base[i] = before;
        before += cnt[i];
    }
}

// ------------------------------------------------------------------------------------------
// rx_counters: counters[c] = sum over the last call's tiles of tile_cnt[t][c] (one workgroup,
// launched by udpdk_gpu_rx_stats only, so a batch that nobody asks statistics for pays nothing)
// ------------------------------------------------------------------------------------------
__global__ void __launch_bounds__(256)
rx_counters(const uint32_t *tile_cnt, uint32_t n_tiles, unsigned long long *counters)
{
    __shared__ unsigned long long lcnt[16 * 4];
    reduce_counters(tile_cnt, n_tiles, counters, lcnt);
}

// ------------------------------------------------------------------------------------------
// rx_scan: the tile-major histogram hist[tile][lane] becomes each (tile, lane)'s start position
// in the lane array: pos(t, l) = lane_off[l] + sum_{t' < t} hist[t'][l], with lane_off the
// exclusive scan of the lane totals. Every access is row-contiguous (threads = lanes).
//   small (one launch):  lanes x tiles <= SCAN_SMALL_MAX and tiles <= SCAN_SMALL_TILES
//   reduce / top / down: per-chunk column sums (chunks of SCAN_COL_CHUNK tiles), one workgroup
//                        scanning chunks and lanes, then the in-place rescan of every chunk.
// ------------------------------------------------------------------------------------------
// exclusive scan over a block of any wave count; lds16 >= waves words
__device__ __forceinline__ uint32_t block_excl_scan(uint32_t v, uint32_t *lds16, uint32_t *total)
{
    const uint32_t lane = lane_id(), w = threadIdx.x >> 6, nw = blockDim.x >> 6;
    const uint32_t inc = wave_incl_scan(v);
    if (lane == 63) lds16[w] = inc;
    __syncthreads();
    uint32_t pre = 0, tot = 0;
    for (uint32_t i = 0; i < nw; ++i) {
        const uint32_t t = lds16[i];
        if (i < w) pre += t;
        tot += t;
    }
    __syncthreads();
    *total = tot;
    return pre + inc - v;
}

// Lane totals tot[] (LDS, n_lanes words) -> lane_off[] exclusive scan + total. Thread j takes the
// contiguous lanes [j * L, (j + 1) * L).
__device__ __forceinline__ void scan_lane_totals(const uint32_t *tot, uint32_t n_lanes, uint32_t *lane_off,
                                 uint32_t *total_out, uint32_t *lds16)
{
    const uint32_t tid = threadIdx.x, L = (n_lanes + blockDim.x - 1) / blockDim.x;
    const uint32_t l0 = min(n_lanes, tid * L), l1 = min(n_lanes, l0 + L);
    // the thread's lanes in registers, loaded at once with clamped indices (a loop with a
    // data-dependent trip count waited for every load in turn); LR = 4, 8 or 16 lanes per thread
    // covers UDPDK_GPU_MAX_LANES at 1024 threads
    auto regs = [&](auto lr) {
        constexpr uint32_t LR = decltype(lr)::value;
        uint32_t v[LR], s = 0;
#pragma unroll
        for (uint32_t i = 0; i < LR; ++i) {
            const uint32_t x = tot[min(l0 + i, n_lanes - 1u)];
            v[i] = l0 + i < l1 ? x : 0u;
            s += v[i];
        }
        uint32_t total;
        uint32_t run = block_excl_scan(s, lds16, &total);
#pragma unroll
        for (uint32_t i = 0; i < LR; ++i) {
            if (l0 + i < l1) lane_off[l0 + i] = run;
            run += v[i];
        }
        if (tid == 0) { lane_off[n_lanes] = total; *total_out = total; }
    };
    if (L <= 4u) return regs(std::integral_constant<uint32_t, 4>{});
    if (L <= 8u) return regs(std::integral_constant<uint32_t, 8>{});
    if (L <= 16u) return regs(std::integral_constant<uint32_t, 16>{});
    uint32_t s = 0;
    for (uint32_t l = l0; l < l1; ++l) s += tot[l];
    uint32_t total;
    uint32_t run = block_excl_scan(s, lds16, &total);
    for (uint32_t l = l0; l < l1; ++l) {
        lane_off[l] = run;
        run += tot[l];
    }
    if (tid == 0) { lane_off[n_lanes] = total; *total_out = total; }
}

// rx_scan_cols: the whole scan in one launch. Workgroup = a block of LB = 2^lb lanes x every
// tile; thread (c, l) holds lane l's counts of the c-th of B / LB contiguous tile chunks
// (<= scan_cols_tpt(B) tiles) in registers, all loaded at once (LB lanes x 2 or 4 B contiguous per
// tile row). The chunk sums meet in LDS and give the lane totals; the lane offsets (the exclusive
// scan of the totals over ALL lanes, which other workgroups hold) come from a decoupled look-back
// over the lane blocks: blocks take tickets in dispatch order, publish their total (A) at once
// and their inclusive prefix (P) once they know it, and a block sums its predecessors' words back
// to the nearest P, one 64-word window per wave load. Each thread then writes its tiles' absolute
// positions base[t][l] = lane_off[l] + sum over t' < t of hist[t'][l], so the scatter reads one
// row per tile and no launch runs between this one and it (the former rx_lane_off).
// Look-back words: epoch << 32 | flag << 30 | value, flag 1 = A, 2 = P; a word from an earlier
// call (older epoch) is not ready. Value < 2^30: deliveries <= max_frames x fan-out.
__device__ __forceinline__ unsigned long long lb_poll(unsigned long long *p, uint32_t epoch)
{
    unsigned long long v;
    for (;;) {
        v = __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if ((uint32_t)(v >> 32) == epoch && ((v >> 30) & 3u)) return v;
        __builtin_amdgcn_s_sleep(1);
    }
}

template <uint32_t B>
__global__ void __launch_bounds__(B)
rx_scan_cols(ScanArgs a, uint32_t lb)
{
    constexpr uint32_t TPT = scan_cols_tpt(B);
#ifdef UDPDK_STAMPS
    // diagnostic: memtime at start, loads summed, look-back done, stores issued; memrealtime at
    // start and end (rows RX_TILE_MAX * 3 + ticket of a.dbg)
    unsigned long long sst[6];
    sst[0] = __builtin_amdgcn_s_memtime();
    sst[4] = __builtin_amdgcn_s_memrealtime();
#endif
    __shared__ uint32_t part[B];
    __shared__ uint32_t loff_sh[64];
    __shared__ uint32_t jb;
    const uint32_t LB = 1u << lb, C = B >> lb;
    const uint32_t l = threadIdx.x & (LB - 1u), c = threadIdx.x >> lb;
    if (threadIdx.x == 0) {
        const uint32_t j = atomicAdd(a.ticket, 1u);
        if (j == gridDim.x - 1u) atomicExch(a.ticket, 0u); // every ticket taken: reset for the next call
        jb = j;
    }
    __syncthreads();
    const uint32_t j = jb;
    const uint32_t S = a.n_lanes, lanei = j * LB + l;
    const uint32_t tpc = (a.n_tiles + C - 1u) / C;
    const uint32_t t0 = min(a.n_tiles, c * tpc), t1 = min(a.n_tiles, t0 + tpc);
    const bool ok = lanei < S;
    const uint32_t hs = a.hist16 ? ((S + 1u) & ~1u) : S;   // row stride in counts
    const uint16_t *col16 = reinterpret_cast<const uint16_t *>(a.hist) + lanei;
    const uint32_t *col32 = a.hist + lanei;
    uint32_t v[TPT];
#pragma unroll
    for (uint32_t k = 0; k < TPT; ++k) {
        const bool in = ok && t0 + k < t1;
        const size_t o = (size_t)(in ? t0 + k : 0u) * hs;
        v[k] = !in ? 0u : a.hist16 ? (uint32_t)col16[o] : col32[o];
    }
    uint32_t sum = 0;
#pragma unroll
    for (uint32_t k = 0; k < TPT; ++k) sum += v[k];
    part[c * LB + l] = sum;
    __syncthreads();
#ifdef UDPDK_STAMPS
    sst[1] = __builtin_amdgcn_s_memtime();
#endif
    uint32_t run = 0, tot = 0;
    for (uint32_t i = 0; i < C; ++i) {
        const uint32_t x = part[i * LB + l];
        run += i < c ? x : 0u;
        tot += x;
    }
    if (threadIdx.x < 64) {                                  // wave 0: threads (0, l), l < LB <= 64
        const uint32_t lane = lane_id();
        const uint32_t mine = lane < LB && ok ? tot : 0u;
        const uint32_t incl = wave_incl_scan(mine);
        const uint32_t btot = (uint32_t)__builtin_amdgcn_readlane((int)incl, 63);
        const unsigned long long tag = (unsigned long long)a.epoch << 32;
        if (lane == 0)
            __hip_atomic_store(&a.agg[j], tag | (1ull << 30) | btot,
                               __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        // look-back: the predecessors' words, 64 at a time, down to the nearest inclusive one
        uint32_t pre = 0;
        for (uint32_t k = j; k > 0;) {
            const uint32_t idx = k - 1u - lane;                 // lane 0 = nearest predecessor
            const bool in = lane < k;
            const unsigned long long wv = in ? lb_poll(&a.agg[idx], a.epoch) : (tag | (2ull << 30));
            const unsigned long long pm = __ballot(((wv >> 30) & 3u) == 2u);
            const uint32_t stop = pm ? (uint32_t)__ffsll((long long)pm) - 1u : 64u;
            const uint32_t val = in && lane <= stop ? (uint32_t)(wv & 0x3FFFFFFFu) : 0u;
            pre += wave_sum(val);
            if (pm) break;
            k = k > 64u ? k - 64u : 0u;
        }
        if (lane == 0)
            __hip_atomic_store(&a.agg[j], tag | (2ull << 30) | (pre + btot),
                               __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (lane < LB) {
            const uint32_t lo = pre + incl - mine;
            loff_sh[lane] = lo;
            if (ok) a.lane_off[lanei] = lo;
        }
        if (lane == 0 && (j + 1u) * LB >= S) {             // the last block: the grand total
            a.lane_off[S] = pre + btot;
            *a.total = pre + btot;
        }
    }
    __syncthreads();
#ifdef UDPDK_STAMPS
    sst[2] = __builtin_amdgcn_s_memtime();
#endif
    run += loff_sh[l];
    uint32_t *out = a.base + lanei;
#pragma unroll
    for (uint32_t k = 0; k < TPT; ++k) {
        if (ok && t0 + k < t1 && ((t0 + k) & a.row_mask) == 0u) out[(size_t)(t0 + k) * S] = run;
        run += v[k];
    }
#ifdef UDPDK_STAMPS
    sst[3] = __builtin_amdgcn_s_memtime();
    sst[5] = __builtin_amdgcn_s_memrealtime();
    if (a.dbg && threadIdx.x == 0 && j < RX_TILE_MAX) {
        unsigned long long *d = a.dbg + (size_t)(RX_TILE_MAX * 3 + j) * 16;
        d[0] = sst[1] - sst[0];
        d[1] = sst[2] - sst[1];
        d[2] = sst[3] - sst[2];
        d[3] = sst[4];
        d[4] = sst[5];
        d[5] = j;
    }
#endif
}

template __global__ void rx_scan_cols<512>(ScanArgs a, uint32_t lb);
template __global__ void rx_scan_cols<1024>(ScanArgs a, uint32_t lb);

// Pass 1, grid (chunks, ceil(lanes / SCAN_BLOCK)): partial[c][l] = column sum of chunk c.
__global__ void __launch_bounds__(SCAN_BLOCK)
rx_scan_reduce(ScanArgs a)
{
    const uint32_t S = a.n_lanes, l = blockIdx.y * SCAN_BLOCK + threadIdx.x;
    if (l >= S) return;
    const uint32_t t0 = blockIdx.x * SCAN_COL_CHUNK, t1 = min(a.n_tiles, t0 + SCAN_COL_CHUNK);
    uint32_t v[SCAN_COL_CHUNK];                            // all loads in flight at once
#pragma unroll
    for (uint32_t k = 0; k < SCAN_COL_CHUNK; ++k)
        v[k] = t0 + k < t1 ? a.hist[(size_t)(t0 + k) * S + l] : 0u;
    uint32_t s = 0;
#pragma unroll
    for (uint32_t k = 0; k < SCAN_COL_CHUNK; ++k) s += v[k];
    a.partial[(size_t)blockIdx.x * S + l] = s;
}

// Pass 2, one workgroup: per lane, exclusive scan of its chunk sums (in place) and its total;
// then lane_off = exclusive scan of the totals.
__global__ void __launch_bounds__(SCAN_TOP_BLOCK)
rx_scan_top(ScanArgs a, uint32_t n_chunks)
{
    extern __shared__ uint32_t tot[];                       // [n_lanes]
    __shared__ uint32_t lds16[SCAN_TOP_BLOCK / 64];
    const uint32_t S = a.n_lanes;
    for (uint32_t l = threadIdx.x; l < S; l += SCAN_TOP_BLOCK) {
        uint32_t run = 0;
        for (uint32_t c0 = 0; c0 < n_chunks; c0 += 32) {   // 32 loads in flight per batch
            uint32_t v[32];
#pragma unroll
            for (uint32_t k = 0; k < 32; ++k)
                v[k] = c0 + k < n_chunks ? a.partial[(size_t)(c0 + k) * S + l] : 0u;
#pragma unroll
            for (uint32_t k = 0; k < 32; ++k) {
                if (c0 + k < n_chunks) a.partial[(size_t)(c0 + k) * S + l] = run;
                run += v[k];
            }
        }
        tot[l] = run;
    }
    __syncthreads();
    scan_lane_totals(tot, S, a.lane_off, a.total, lds16);
}

// Pass 3, grid (chunks, ceil(lanes / SCAN_BLOCK)): rescan chunk c from lane_off + its prefix.
__global__ void __launch_bounds__(SCAN_BLOCK)
rx_scan_down(ScanArgs a)
{
    const uint32_t S = a.n_lanes, l = blockIdx.y * SCAN_BLOCK + threadIdx.x;
    if (l >= S) return;
    const uint32_t t0 = blockIdx.x * SCAN_COL_CHUNK, t1 = min(a.n_tiles, t0 + SCAN_COL_CHUNK);
    uint32_t v[SCAN_COL_CHUNK];
#pragma unroll
    for (uint32_t k = 0; k < SCAN_COL_CHUNK; ++k)
        v[k] = t0 + k < t1 ? a.hist[(size_t)(t0 + k) * S + l] : 0u;
    uint32_t run = a.lane_off[l] + a.partial[(size_t)blockIdx.x * S + l];
#pragma unroll
    for (uint32_t k = 0; k < SCAN_COL_CHUNK; ++k) {
        if (t0 + k < t1) a.hist[(size_t)(t0 + k) * S + l] = run;
        run += v[k];
    }
}

// Tile of workgroup b out of n so that each XCD walks a contiguous run of tiles (blocks are dealt
// round-robin over the 8 XCDs, MI355X_MICROARCH.md §Workgroup dispatch; b % 8 labels the blocks
// sharing one). Bijective for any n. A lane's entries from consecutive tiles are adjacent in
// lane_pkt, so with this order the partial lines one tile leaves in a lane are completed by the
// next tiles in the SAME L2 and written back once, instead of once per XCD that touched them.
// Placement is a speed choice only: any order gives the same output.
__device__ __forceinline__ uint32_t xcd_tile(uint32_t b, uint32_t n)
{
    const uint32_t x = b & 7u, q = n >> 3, r = n & 7u;
    return (x < r ? x * (q + 1u) : r * (q + 1u) + (x - r) * q) + (b >> 3);
}

// Scatter prologue: cur[k] = base[tile][k], the absolute start of the tile's deliveries in lane k
// (rx_scan_cols / rx_scan_down fold lane_off in), for the S lanes, CU loads per thread in flight at
// once (clamped indices, stores guarded): a plain strided loop waited for each iteration's loads,
// one L2 / HBM round trip per NT lanes (8 at 4096 lanes and 512 threads).
__device__ __forceinline__ void lane_cursors(const ScatterArgs &a, uint32_t tile, uint32_t *cur)
{
    const uint32_t tid = threadIdx.x, NT = blockDim.x, S = a.n_lanes;
    const uint32_t *base = a.base + (size_t)tile * a.row_step * S;
    constexpr uint32_t CU = 8;
    for (uint32_t k0 = tid; k0 < S; k0 += NT * CU) {
        uint32_t vy[CU];
#pragma unroll
        for (uint32_t u = 0; u < CU; ++u) vy[u] = base[min(k0 + u * NT, S - 1u)];
#pragma unroll
        for (uint32_t u = 0; u < CU; ++u)
            if (k0 + u * NT < S) cur[k0 + u * NT] = vy[u];
    }
    __syncthreads();
}

// ------------------------------------------------------------------------------------------
// rx_scatterw: stable per-lane compaction without fan-out, W waves per scatter tile (one or
// several consecutive classify tiles, ScatterArgs::row_step). Wave w owns the w-th contiguous
// slice of the tile. Pass 1 counts each wave's deliveries per lane key with LDS atomics, whose
// returns are each delivery's rank within its key in the slice; each key's wave offsets then
// become the exclusive prefix over the earlier slices (and the keys' starts in the tile, for
// the staged write-out); the placement puts every delivery at cursor + slice offset + rank.
//
// Stability comes from the order in which a ds_add_rtn_u32 resolves lanes of one instruction
// that hit the same word: lane order on gfx950 (tools/probe/lds_order_probe.hip: 1.3e10 same-key
// lane pairs over 1-4096 keys, none out of order), and one wave's instructions execute in
// program order, so the returns number a key's frames of the slice in arrival order. (The first
// form ranked lanes by a wave multi-split over the key bits, 12 ballots per 64 frames at 4096
// lanes: 11 us per pass at config 5, instruction-bound; the atomics make a pass a few
// instructions per 64 frames.) Counters hold two waves each, 16 bits per wave (a scatter tile
// has <= 16384 frames, so neither half can carry into the other).
// LDS: 4 x max(n_lanes, W) (cursors) + 2 x W x n_lanes bytes (scatterw_lds_bytes).
// ------------------------------------------------------------------------------------------
template <uint32_t W>
__global__ void __launch_bounds__(64 * W)
rx_scatterw(ScatterArgs a)
{
    extern __shared__ __attribute__((aligned(16))) uint32_t smw[];
    const uint32_t S = a.n_lanes;
    // cursors [max(S, W)]: the first W words carry the key scan's wave totals until pass 2 (their
    // cursors wait in registers), so the LDS stays at 80 KiB for 8 waves at 4096 lanes (two
    // workgroups per CU)
    const uint32_t SC = S > W ? S : W;
    uint32_t *cur = smw;
    uint32_t *cnt = smw + SC;                                          // [W / 2][S] packed pairs
    const uint32_t tid = threadIdx.x, lane = lane_id(), w = tid >> 6;
    const uint32_t tile = xcd_tile(blockIdx.x, a.n_tiles);
    const uint32_t t1 = min(a.n, (tile + 1) * a.tile_frames);
    const uint32_t q = a.tile_frames / W;
    const uint32_t wb = tile * a.tile_frames + w * q, we = min(t1, wb + q);
    const uint32_t plast = a.n - 1u;
    uint32_t *mine = cnt + (w >> 1) * S;
    const uint32_t inc = (w & 1u) ? 0x10000u : 1u, sh = (w & 1u) * 16u;
    // the wave's whole slice of verdict words in registers (<= 16 per lane: tile_frames <=
    // 64 W SCATTERW_MV, checked by the host), loaded once for both passes (no load in the
    // counting or the placing loop) and issued first, so they are in flight during the cursor
    // prologue
    constexpr uint32_t MV = SCATTERW_MV;
    uint32_t mv[MV];
#pragma unroll
    for (uint32_t i = 0; i < MV; ++i) {
        const uint32_t p = wb + i * 64 + lane;
        mv[i] = (i * 64 < q) ? a.meta[min(p, plast)] : 0u;
    }
#ifdef UDPDK_STAMPS
    unsigned long long sacc[16] = {0}, slast = __builtin_amdgcn_s_memtime();
    sacc[12] = __builtin_amdgcn_s_memrealtime();
#define SSTAMP(k)                                                         \
    do {                                                                  \
        if (w == 0) {                                                     \
            const unsigned long long t_ = __builtin_amdgcn_s_memtime();   \
            sacc[k] += t_ - slast;                                        \
            slast = t_;                                                   \
        }                                                                 \
    } while (0)
#else
#define SSTAMP(k) do {} while (0)
#endif
    // the cursors' loads (up to 8 per thread) in flight while the counters are zeroed (16-byte
    // LDS stores), then one barrier (the zeroing waited behind the cursor round trip before)
    uint32_t cur_lo;
    {
        const uint32_t *brow = a.base + (size_t)tile * a.row_step * S;
        constexpr uint32_t CU = 8;
        const uint32_t NT = 64 * W;
        uint32_t vy[CU];
#pragma unroll
        for (uint32_t u = 0; u < CU; ++u) vy[u] = brow[min(tid + u * NT, S - 1u)];
        if ((SC & 3u) == 0u) {                    // cnt = smw + SC is 16-byte aligned
            uint4 *c4 = reinterpret_cast<uint4 *>(cnt);
            for (uint32_t k = tid; k < (W / 2) * S / 4; k += NT) c4[k] = make_uint4(0, 0, 0, 0);
        } else {
            for (uint32_t k = tid; k < (W / 2) * S; k += NT) cnt[k] = 0;
        }
#pragma unroll
        for (uint32_t u = 0; u < CU; ++u)
            if (tid + u * NT < S && (u > 0 || tid >= W)) cur[tid + u * NT] = vy[u];
        cur_lo = vy[0];
        for (uint32_t k0 = tid + NT * CU; k0 < S; k0 += NT) cur[k0] = brow[k0];   // S > 4096: none
    }
    SSTAMP(0);
    __syncthreads();
    SSTAMP(1);
    // pass 1: per-wave counts; each atomic's return is the delivery's rank within its key in the
    // wave's slice (kept with the key: the placement adds the slice's offset, a plain LDS read,
    // where it made a second atomic per delivery)
    uint32_t kr[MV];                                                   // rank | key << 16
#pragma unroll
    for (uint32_t i = 0; i < MV; ++i) {
        kr[i] = 0xFFFFFFFFu;
        if (i * 64 >= q) break;                                        // uniform
        const uint32_t p = wb + i * 64 + lane;
        if (p < we && UDPDK_META_VERDICT(mv[i]) == UDPDK_V_DELIVERED) {
            const uint32_t key = UDPDK_META_SOCKFD(mv[i]) & a.lane_mask;
            const uint32_t o = atomicAdd(&mine[key], inc);
            kr[i] = ((o >> sh) & 0xFFFFu) | key << 16;
        }
    }
    __syncthreads();
    SSTAMP(2);
    // slice offsets: each wave's counts become the sum of the earlier slices' counts. Wave w
    // takes the contiguous keys [w KW, (w + 1) KW), lane l the keys w KW + 64 j + l (conflict-
    // free LDS rows), and keeps each key's tile total: their exclusive scan in key order (a wave
    // scan per j plus the earlier waves' totals) is each key's start in the tile's key-ordered
    // staging, held in registers until pass 2 has released the counter region. (The former
    // separate pass re-read the last pair's totals with 8 consecutive keys per thread: 8-way bank
    // conflicts and two more barriers, 6000 cycles of a 16-wave workgroup at config 5.)
    constexpr uint32_t KPT = SCATTERW_MAX_LANES / (64 * W);           // keys per lane
    const uint32_t KW = (S + 64 * W - 1) / (64 * W) * 64;               // keys per wave
    uint32_t *wtot = cur;                                               // [W] wave totals
    uint32_t kt[KPT] = {};
    {
        // every count the lane needs in flight at once (clamped addresses, masked values): one
        // LDS round trip instead of one per (key, wave pair). The j loops end at the wave's keys
        // (uniform), so the reads of one j are straight-line code.
        uint32_t cv[KPT][W / 2];
#pragma unroll
        for (uint32_t j = 0; j < KPT; ++j) {
            if (j * 64 >= KW) break;
            const uint32_t k = min(w * KW + j * 64 + lane, S - 1u);
#pragma unroll
            for (uint32_t jj = 0; jj < W / 2; ++jj) cv[j][jj] = cnt[jj * S + k];
        }
        __builtin_amdgcn_sched_barrier(0);         // all reads issued before the first use
        uint32_t run = 0;
#pragma unroll
        for (uint32_t j = 0; j < KPT; ++j) {
            if (j * 64 >= KW) break;
            const uint32_t k = w * KW + j * 64 + lane;
            const bool in = k < S;
            uint32_t c = 0;
#pragma unroll
            for (uint32_t jj = 0; jj < W / 2; ++jj) {
                const uint32_t v = in ? cv[j][jj] : 0u;
                const uint32_t lo = c, hi = c + (v & 0xFFFFu);
                cv[j][jj] = lo | (hi << 16);
                c = hi + (v >> 16);
            }
            if (in) {
#pragma unroll
                for (uint32_t jj = 0; jj < W / 2; ++jj) cnt[jj * S + k] = cv[j][jj];
            }
            const uint32_t incl = wave_incl_scan(c);
            kt[j] = run + incl - c;
            run += (uint32_t)__builtin_amdgcn_readlane((int)incl, 63);
        }
        if (lane == 0) wtot[w] = run;
    }
    __syncthreads();
    uint32_t nd = 0;                                                    // the tile's deliveries
    {
        uint32_t before = 0;
#pragma unroll
        for (uint32_t j = 0; j < W; ++j) {
            const uint32_t t = wtot[j];
            before += j < w ? t : 0u;
            nd += t;
        }
#pragma unroll
        for (uint32_t j = 0; j < KPT; ++j) kt[j] += before;
    }
    SSTAMP(3);
    // pass 2: placement. Staged when the tile's (frame, position) pairs fit the counter region:
    // every delivery's rank within its key comes from the atomics; the tile's deliveries are then
    // laid out in LDS in key order (each key's start from the scan above) and written out
    // linearly, so a wave's 64 stores fill runs of consecutive lane_pkt words (one run per key of
    // the tile) instead of 64 scattered words (config 5: rx_scatterw 24.5 -> 22.5 us). Otherwise
    // each delivery stores its own word (and needs every cursor now).
    const uint32_t T = a.tile_frames;
    const bool staged = (S & 1u) == 0u && 8u * T <= 4u * (W / 2) * S;   // 8-byte pairs in cnt
    if (!staged) {
        __syncthreads();                                               // wave totals read
        if (tid < W && tid < S) cur[tid] = cur_lo;
        __syncthreads();
    }
#pragma unroll
    for (uint32_t i = 0; i < MV; ++i) {
        if (i * 64 >= q) break;                                        // uniform
        if (kr[i] != 0xFFFFFFFFu) {
            const uint32_t key = kr[i] >> 16;
            const uint32_t rank = (kr[i] & 0xFFFFu) + ((mine[key] >> sh) & 0xFFFFu);
            if (staged) {
                kr[i] = rank | key << 16;
            } else {
                const uint32_t pos = cur[key] + rank;
                if (pos < a.lane_cap) a.lane_pkt[pos] = wb + i * 64 + lane;
            }
        }
    }
    SSTAMP(4);
    if (staged) {
        // every wave's pass 2 is done with the counters: the key starts go where they were
        __syncthreads();
        uint32_t *lex = cnt;                                           // [S] key start in the tile
#pragma unroll
        for (uint32_t j = 0; j < KPT; ++j) {
            const uint32_t k = w * KW + j * 64 + lane;
            if (j * 64 < KW && k < S) lex[k] = kt[j];
        }
        if (tid < W && tid < S) cur[tid] = cur_lo;                     // wave totals read long ago
        __syncthreads();
        SSTAMP(6);
        // each delivery's place in key order and its lane position into registers first (lex
        // is read), then (frame, position) pairs into LDS over the whole counter region
        uint32_t li[MV], ps[MV];
#pragma unroll
        for (uint32_t i = 0; i < MV; ++i) {
            li[i] = 0xFFFFFFFFu;
            if (i * 64 >= q) break;
            if (kr[i] != 0xFFFFFFFFu) {
                const uint32_t key = kr[i] >> 16, rank = kr[i] & 0xFFFFu;
                li[i] = lex[key] + rank;
                ps[i] = cur[key] + rank;
            }
        }
        __syncthreads();
        SSTAMP(7);
        uint2 *pp = reinterpret_cast<uint2 *>(cnt);                    // [T] (frame, position)
#pragma unroll
        for (uint32_t i = 0; i < MV; ++i) {
            if (i * 64 >= q) break;
            if (li[i] != 0xFFFFFFFFu) pp[li[i]] = make_uint2(wb + i * 64 + lane, ps[i]);
        }
        __syncthreads();
        SSTAMP(8);
        for (uint32_t i = tid; i < nd; i += 64 * W) {
            const uint2 e = pp[i];
            if (e.y < a.lane_cap) a.lane_pkt[e.y] = e.x;
        }
    }
    SSTAMP(5);
#ifdef UDPDK_STAMPS
    sacc[13] = __builtin_amdgcn_s_memrealtime();
    sacc[14] = (unsigned long long)__builtin_amdgcn_s_getreg(4 | (31 << 11)) |
               ((unsigned long long)__builtin_amdgcn_s_getreg(20 | (31 << 11)) << 32);
    sacc[15] = tile;
    if (a.dbg && w == 0 && lane < 16 && tile < RX_TILE_MAX) a.dbg[(size_t)(RX_TILE_MAX * 2 + tile) * 16 + lane] = sacc[lane];
#endif
#undef SSTAMP
}

template __global__ void rx_scatterw<SCATTER_WAVES>(ScatterArgs a);
template __global__ void rx_scatterw<2 * SCATTER_WAVES>(ScatterArgs a);

// ------------------------------------------------------------------------------------------
// rx_scatter: stable per-lane compaction, one wave per tile
// ------------------------------------------------------------------------------------------
__global__ void __launch_bounds__(SCATTER1_BLOCK)
rx_scatter(ScatterArgs a)
{
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    uint32_t *cur = reinterpret_cast<uint32_t *>(smem);   // running position per lane
    const uint32_t lane = lane_id();
    const uint32_t tile = xcd_tile(blockIdx.x, a.n_tiles);
    // cursor of every lane for this tile: the whole workgroup runs the prologue, wave 0 the walk
    lane_cursors(a, tile, cur);
    if (threadIdx.x >= 64) return;
    const uint32_t t0 = tile * a.tile_frames;
    const uint32_t t1 = min(a.n, t0 + a.tile_frames);

    constexpr int PF = 8;                                 // verdict words prefetched per lane
    for (uint32_t g0 = t0; g0 < t1; g0 += 64 * PF) {
        uint32_t mv[PF];
#pragma unroll
        for (int i = 0; i < PF; ++i) {
            const uint32_t p = g0 + i * 64 + lane;
            mv[i] = p < t1 ? a.meta[p] : 0u;
        }
#pragma unroll
        for (int i = 0; i < PF; ++i) {
            const uint32_t f0 = g0 + i * 64;
            if (f0 >= t1) break;
            const uint32_t p = f0 + lane;
            const bool valid = p < t1;
            const uint32_t m = mv[i];
            const bool deliver = valid && UDPDK_META_VERDICT(m) == UDPDK_V_DELIVERED;
            const uint32_t fan = UDPDK_META_FANOUT(m);
            const unsigned long long multi = __ballot(deliver && fan > 1u);
            if (multi == 0ull) {
                // one delivery per frame: the LDS atomic on the lane's cursor returns the
                // position, lanes of one key numbered in lane order (see rx_scatterw)
                if (deliver) {
                    const uint32_t pos = atomicAdd(&cur[UDPDK_META_SOCKFD(m) & a.lane_mask], 1u);
                    if (pos < a.lane_cap) a.lane_pkt[pos] = p;
                }
            } else if (lane == 0) {
                // fan-out (SO_REUSEADDR/SO_REUSEPORT clones, poller.c:396-399): deliveries in
                // frame order then list order, re-derived from the frame header. Serial.
                for (uint32_t q = 0; q < 64 && f0 + q < t1; ++q) {
                    const uint32_t fp = f0 + q;
                    const uint32_t mi = a.meta[fp];
                    if (UDPDK_META_VERDICT(mi) != UDPDK_V_DELIVERED) continue;
                    const uint8_t *f = a.frames + a.offset[fp];
                    const uint32_t dport = (uint32_t)f[36] | ((uint32_t)f[37] << 8);
                    const uint32_t dip = (uint32_t)f[30] | ((uint32_t)f[31] << 8) |
                                         ((uint32_t)f[32] << 16) | ((uint32_t)f[33] << 24);
                    const uint4 e = a.port_tab[dport];
                    uint32_t bip = e.z, bsr = e.w;
                    for (uint32_t k = 0;;) {
                        if (dip == bip || bip == 0u) {
                            const uint32_t key = (bsr & 0x7FFFFFFFu) & a.lane_mask;
                            const uint32_t c = cur[key];
                            cur[key] = c + 1u;
                            if (c < a.lane_cap) a.lane_pkt[c] = fp;
                            if (!(bsr >> 31)) break;
                        }
                        if (++k >= e.x) break;
                        const uint2 b = a.binds[e.y + k];
                        bip = b.x;
                        bsr = b.y;
                    }
                }
            }
            wave_sync();
        }
    }
}

} // namespace udpdk
