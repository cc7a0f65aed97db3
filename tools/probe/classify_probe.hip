// The real rx_classify in the streaming-probe harness (back-to-back launches over 10 rotated
// device copies of 1 M x 64 B valid UDP frames, one bound port, ptype derived), timed with the
// same events as tools/probe/stream_probe.hip, to separate kernel cost from harness cost.
// Build: hipcc -O3 --offload-arch=gfx950 -Iinclude -Iudpdk_amd/csrc [-DUDPDK_EXP_...]
//        -o tools/probe/classify_probe tools/probe/classify_probe.hip
#include "../../udpdk_amd/csrc/rx_kernels.hip"
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>
#include <chrono>

using namespace udpdk;

namespace udpdk {
// ------------------------------------------------------------------------------------------
// rx_compact1w (probe only; measured no faster than rx_compact1 under two streams): rx_compact1 with each workgroup taking `tpb` consecutive tiles (fewer, longer
// workgroups): the base of its first tile is read once, the next tile's verdict words are in
// flight while the current tile's entries are written.
// ------------------------------------------------------------------------------------------
__global__ void __launch_bounds__(RX_BLOCK)
rx_compact1w(Compact1Args a, uint32_t tpb)
{
    __shared__ uint32_t red[2][RX_WAVES];
    const uint32_t tid = threadIdx.x, lane = lane_id(), w = tid >> 6;
    const uint32_t tb = blockIdx.x * tpb, te = min(a.n_tiles, tb + tpb);
    const uint32_t steps = a.tile_frames / RX_BLOCK;        // 64-frame steps per wave per tile
    const uint32_t plast = a.n - 1u;
    uint32_t pre = 0;
    for (uint32_t t = tid; t < tb; t += RX_BLOCK) pre += a.tile_count[t];
    pre = wave_sum(pre);
    if (lane == 0) red[0][w] = pre;
    __syncthreads();
    uint32_t run_base = 0;
#pragma unroll
    for (int i = 0; i < RX_WAVES; ++i) run_base += red[0][i];
    const unsigned long long lt = (1ull << lane) - 1ull;
    constexpr uint32_t MAXU = 8;                            // steps held in registers
    uint32_t mv[MAXU];
    auto load_tile = [&](uint32_t t) {
        const uint32_t wb = t * a.tile_frames + w * steps * 64;
#pragma unroll
        for (uint32_t u = 0; u < MAXU; ++u)
            if (u < steps) mv[u] = a.meta[min(wb + u * 64 + lane, plast)];
    };
    if (tb < te) load_tile(tb);
    for (uint32_t t = tb; t < te; ++t) {
        const uint32_t t1 = min(a.n, (t + 1) * a.tile_frames);
        const uint32_t wb = t * a.tile_frames + w * steps * 64;
        unsigned long long m[MAXU];
        uint32_t wcount = 0;
#pragma unroll
        for (uint32_t u = 0; u < MAXU; ++u) {
            m[u] = 0;
            if (u < steps) {
                const uint32_t p = wb + u * 64 + lane;
                m[u] = __ballot(p < t1 && (mv[u] & 0xFu) == UDPDK_V_DELIVERED);
                wcount += (uint32_t)__popcll(m[u]);
            }
        }
        if (t + 1 < te) load_tile(t + 1);                   // next tile's words in flight
        const uint32_t buf = (t - tb) & 1u;
        if (lane == 0) red[buf][w] = wcount;
        __syncthreads();
        uint32_t before = 0, tcount = 0;
#pragma unroll
        for (int i = 0; i < RX_WAVES; ++i) {
            tcount += red[buf][i];
            before += (uint32_t)i < w ? red[buf][i] : 0u;
        }
        uint32_t run = run_base + before;
#pragma unroll
        for (uint32_t u = 0; u < MAXU; ++u) {
            if (u < steps) {
                if ((m[u] >> lane) & 1ull) {
                    const uint32_t pos = run + (uint32_t)__popcll(m[u] & lt);
                    if (pos < a.lane_cap) a.lane_pkt[pos] = wb + u * 64 + lane;
                }
                run += (uint32_t)__popcll(m[u]);
            }
        }
        run_base += tcount;
        if (t == a.n_tiles - 1u && tid == 0) {
            a.lane_off[0] = 0u;
            a.lane_off[1] = run_base;
            *a.total = run_base;
        }
    }
}

} // namespace udpdk

int main()
{
    const uint32_t N = 1u << 20, COPIES = 10, FL = 64;
    // one valid Eth/IPv4/UDP frame, dst port 10001, 30-byte datagram (frame ends at the datagram)
    uint8_t t[64] = {0};
    const uint8_t hdr[42] = {0x68, 0x05, 0xca, 0x95, 0xf8, 0xec, 0x68, 0x05, 0xca, 0x95, 0xfa, 0x64, 0x08, 0x00,
                             0x45, 0x00, 0x00, 0x32, 0x12, 0x34, 0x00, 0x00, 0x40, 0x11, 0x00, 0x00,
                             0xac, 0x1f, 0x64, 0x02, 0xac, 0x1f, 0x64, 0x01,
                             0x27, 0x10, 0x27, 0x11, 0x00, 0x1e, 0xab, 0xcd};
    memcpy(t, hdr, 42);
    for (int i = 42; i < 64; ++i) t[i] = (uint8_t)(i * 7);
    std::vector<uint8_t> hf((size_t)N * FL);
    for (uint32_t i = 0; i < N; ++i) memcpy(&hf[(size_t)i * FL], t, FL);
    std::vector<uint32_t> ho(N);
    std::vector<uint16_t> hl(N, FL);
    for (uint32_t i = 0; i < N; ++i) ho[i] = i * FL;

    uint8_t *fr; uint32_t *off; uint16_t *len;
    (void)hipMalloc(&fr, (size_t)N * FL * COPIES);
    (void)hipMalloc(&off, (size_t)N * 4 * COPIES);
    (void)hipMalloc(&len, (size_t)N * 2 * COPIES);
    for (uint32_t c = 0; c < COPIES; ++c) {
        (void)hipMemcpy(fr + (size_t)c * N * FL, hf.data(), (size_t)N * FL, hipMemcpyHostToDevice);
        (void)hipMemcpy(off + (size_t)c * N, ho.data(), (size_t)N * 4, hipMemcpyHostToDevice);
        (void)hipMemcpy(len + (size_t)c * N, hl.data(), (size_t)N * 2, hipMemcpyHostToDevice);
    }
    std::vector<uint4> pt(65536, make_uint4(0, 0, 0, 0));
    const uint32_t rp = (10001 >> 8) | ((10001 & 0xFF) << 8);
    pt[rp] = make_uint4(1, 0, 0, 0);
    uint4 *port_tab; uint2 *binds;
    (void)hipMalloc(&port_tab, 65536 * 16);
    (void)hipMemcpy(port_tab, pt.data(), 65536 * 16, hipMemcpyHostToDevice);
    (void)hipMalloc(&binds, 8);
    (void)hipMemset(binds, 0, 8);
    const uint32_t T = getenv("TILE") ? (uint32_t)atoi(getenv("TILE")) : 1024u, tiles = N / T;
    uint32_t *meta, *hist, *tcnt;
    (void)hipMalloc(&meta, (size_t)N * 4);
    (void)hipMalloc(&hist, tiles * 4);
    (void)hipMalloc(&tcnt, tiles * 64);

    RxArgs a;
    memset(&a, 0, sizeof(a));
    a.port_tab = port_tab; a.binds = binds; a.meta = meta; a.hist = hist; a.tile_cnt = tcnt;
    a.frames_bytes = N * FL; a.rsrc_bytes = N * FL; a.n = N; a.tile_frames = T; a.n_tiles = tiles;
    a.lane_mask = 0; a.n_lanes = 1; a.key_bits = 0;
    const uint32_t lds = classify_lds_bytes(1, T);
    // STREAMS=2: consecutive launches alternate between two streams with their own outputs,
    // so two launches may run concurrently
    const int NS = getenv("STREAMS") ? atoi(getenv("STREAMS")) : 1;
    hipStream_t ss[4];
    uint32_t *metak[4], *histk[4], *tcntk[4], *lpk[4], *lok[4], *totk[4];
    for (int k = 0; k < 4; ++k) {
        (void)hipStreamCreateWithFlags(&ss[k], hipStreamNonBlocking);
        if (k == 0) { metak[0] = meta; histk[0] = hist; tcntk[0] = tcnt; }
        else {
            (void)hipMalloc(&metak[k], (size_t)N * 4);
            (void)hipMalloc(&histk[k], tiles * 4);
            (void)hipMalloc(&tcntk[k], tiles * 64);
        }
        (void)hipMalloc(&lpk[k], (size_t)N * 4);
        (void)hipMalloc(&lok[k], 64);
        (void)hipMalloc(&totk[k], 64);
    }
    uint32_t *lp1 = lpk[0], *tot1 = totk[0];
    auto launch = [&](int i) {
        RxArgs b = a;
        b.frames = fr + (size_t)(i % COPIES) * N * FL;
        b.offset = off + (size_t)(i % COPIES) * N;
        b.length = len + (size_t)(i % COPIES) * N;
        const int k = i % NS;
        b.meta = metak[k]; b.hist = histk[k]; b.tile_cnt = tcntk[k];
        hipLaunchKernelGGL(rx_classify, dim3(tiles), dim3(CLS_BLOCK), lds, ss[k], b);
        if (getenv("COMPACT")) {              // the single-lane compaction after it, same stream
            Compact1Args ca;
            ca.meta = b.meta; ca.tile_count = b.hist; ca.lane_pkt = lpk[k];
            ca.lane_off = lok[k]; ca.total = totk[k]; ca.n = N; ca.tile_frames = T;
            ca.n_tiles = tiles; ca.lane_cap = N; ca.base = nullptr;
            const int tpb = getenv("TPB") ? atoi(getenv("TPB")) : 0;
            if (tpb > 0)
                hipLaunchKernelGGL(rx_compact1w, dim3((tiles + tpb - 1) / tpb), dim3(RX_BLOCK), 0, ss[k], ca,
                                   (uint32_t)tpb);
            else
                hipLaunchKernelGGL(rx_compact1, dim3(tiles), dim3(RX_BLOCK), 0, ss[k], ca);
        }
    };
    hipEvent_t e0, e1; (void)hipEventCreate(&e0); (void)hipEventCreate(&e1);
    for (int i = 0; i < 10; ++i) launch(i);
    (void)hipDeviceSynchronize();
    const int R = 200;
    const auto t0 = std::chrono::steady_clock::now();
    for (int i = 0; i < R; ++i) launch(i);
    (void)hipDeviceSynchronize();
    const double us = std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count();
    (void)hipEventRecord(e0, 0);
    (void)hipEventRecord(e1, 0);
    (void)hipEventSynchronize(e1);
    float ms; (void)hipEventElapsedTime(&ms, e0, e1);
    std::vector<uint32_t> hm(16);
    (void)hipMemcpy(hm.data(), meta, 64, hipMemcpyDeviceToHost);
    (void)ms;
    uint32_t lp[4] = {0, 0, 0, 0}, tot = 0;
    if (getenv("COMPACT")) {
        (void)hipMemcpy(lp, lp1 + (N - 4), 16, hipMemcpyDeviceToHost);
        (void)hipMemcpy(&tot, tot1, 4, hipMemcpyDeviceToHost);
    }
    printf("rx_classify%s %7.2f us per launch, %d stream(s) (meta[0] = %08x, total %u, last %u)\n",
           getenv("COMPACT") ? (getenv("TPB") ? "+compact1w" : "+compact1") : "", us / R, NS, hm[0],
           tot, lp[3]);
    return 0;
}
