// k_kahan.hip -- the reference's Kahan centroids (sumInArea, src/Quantizer.cpp:59-87) on the
// device, exactly, for the byte engine's SCALED values (kahan_par.hpp has the arithmetic).
// Used on the levels whose tie band is not empty.
//
// Pipeline (one stream):
//   1. stable counting sort of the rows by cell: per-4096-row histograms, a scan per cell, cell
//      offsets, then a wave per 4096 rows writes each row's bytes at its sorted position into
//      the component planes (planes[d][p] = component d of the p-th row in cell order);
//   3. meta: a wave per block of 64 segments (64 steps each) of one chain and component:
//      each lane's SegMeta, the block's total;
//   4. block prefix: per chain and component, the exact sums before each block;
//   5. build: a wave per block: each lane builds its segment's function (estimate D = 0), the
//      wave composes the 64 into the block's function;
//   6. eval: a wave per chain and component: the transient, block functions checked, blocks
//      whose function does not answer re-walked segment by segment with the exact state
//      (segments that do not answer replayed step by step); C = sum * fl(1/n), and the split.
#include <hip/hip_runtime.h>

#include "common.hpp"
#include "kahan_par.hpp"

#define QVQ_FOR_EACH_DP(X) X(4) X(8) X(12) X(16) X(20) X(24) X(28) X(32) X(36) X(40) X(44) X(48) X(52) X(56) X(60) X(64)

// QVQ_KDEBUG builds (tools: a debug libqvq): bounds checks on the chains' global accesses, a
// failed one printed and the access skipped
#ifdef QVQ_KDEBUG
#define KCHK(cond)                                                                                          \
    do {                                                                                                    \
        if (!(cond)) {                                                                                      \
            printf("KCHK line %d: %s (block %u thread %u)\n", __LINE__, #cond, blockIdx.x, threadIdx.x);     \
            return;                                                                                         \
        }                                                                                                   \
    } while (0)
#else
#define KCHK(cond) \
    do {           \
    } while (0)
#endif

namespace qvq {

using kahan::ByteTab;
using kahan::Fn;
using kahan::i128;
using kahan::SegMeta;
using kahan::u128;
using kahan::L;
using kahan::SPB;

namespace {

constexpr uint32_t SROWS = 1024;   // rows per sort block (one wave)
constexpr uint32_t BLK_STEPS = L * SPB;

__device__ inline uint32_t lane_id() { return threadIdx.x & 63; }
// LDS written by other lanes of the same wave becomes visible to this lane (waves of one
// workgroup work on independent chains here, so no workgroup barrier after the table staging)
__device__ inline void wave_sync() {
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "workgroup");
    __builtin_amdgcn_wave_barrier();
}

// ---- 1. stable counting sort, writing the planes ----------------------------------------------
// hist[k][g]: rows of 4096-row block g with index k (transposed: a key's column is contiguous)
// a row's key: its cell, or with sel its cell's slot; ~0u for a row not summed
__device__ inline uint32_t ks_key(uint32_t a, uint32_t K, const uint32_t *__restrict__ sel, uint32_t n_sel) {
    if (!sel) return a < K ? a : ~0u;
    const uint32_t s = a < n_sel ? sel[a] : 0u;
    return s ? s - 1 : ~0u;
}

__global__ __launch_bounds__(64) void ks_hist_kernel(const uint32_t *__restrict__ A, uint64_t N, uint32_t K,
                                                    uint32_t G, uint32_t *__restrict__ hist,
                                                    const uint32_t *__restrict__ sel, uint32_t n_sel) {
    extern __shared__ uint32_t h[];
    for (uint32_t i = threadIdx.x; i < K; i += 64) h[i] = 0;
    __syncthreads();
    // the block's 1024 indices in four 16-byte loads per lane, all in flight before the first
    // use (a load per row and loop trip waited for each: 12.8 us for C3's 16.8 MB)
    const uint64_t r0 = (uint64_t)blockIdx.x * SROWS, r1 = min(N, r0 + SROWS);
    uint4 q[SROWS / 256];
    const bool full = r1 - r0 == SROWS && ((uintptr_t)A & 15) == 0;
#pragma unroll
    for (int i = 0; i < (int)(SROWS / 256); i++) {
        const uint64_t r = r0 + 256 * i + 4 * threadIdx.x;
        if (full) q[i] = *reinterpret_cast<const uint4 *>(A + r);   // (N % 4 != 0: the last block is partial)
        else {
            q[i].x = r < r1 ? A[r] : ~0u;
            q[i].y = r + 1 < r1 ? A[r + 1] : ~0u;
            q[i].z = r + 2 < r1 ? A[r + 2] : ~0u;
            q[i].w = r + 3 < r1 ? A[r + 3] : ~0u;
        }
    }
#pragma unroll
    for (int i = 0; i < (int)(SROWS / 256); i++)
#pragma unroll
        for (int j = 0; j < 4; j++) {
            const uint32_t a = ks_key(j == 0 ? q[i].x : j == 1 ? q[i].y : j == 2 ? q[i].z : q[i].w, K, sel, n_sel);
            if (a != ~0u) atomicAdd(&h[a], 1u);
        }
    __syncthreads();
    for (uint32_t i = threadIdx.x; i < K; i += 64) hist[(uint64_t)i * G + blockIdx.x] = h[i];
}

// Per key (a block each): hist[k][g] <- rows of blocks before g with index k; tot[k].
__global__ __launch_bounds__(256) void ks_colscan_kernel(uint32_t *__restrict__ hist, uint32_t G,
                                                        uint32_t *__restrict__ tot) {
    __shared__ uint32_t wsum[4];
    uint32_t *col = hist + (uint64_t)blockIdx.x * G;
    const uint32_t per = (G + 255) / 256, g0 = min(G, threadIdx.x * per), g1 = min(G, g0 + per);
    uint32_t s = 0;
    for (uint32_t g = g0; g < g1; g++) s += col[g];
    // block exclusive scan of the threads' sums
    const uint32_t lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    uint32_t inc = s;
    for (int o = 1; o < 64; o <<= 1) {
        const uint32_t v = __shfl_up(inc, o, 64);
        if (lane >= (uint32_t)o) inc += v;
    }
    if (lane == 63) wsum[w] = inc;
    __syncthreads();
    uint32_t base = inc - s;
    for (uint32_t i = 0; i < w; i++) base += wsum[i];
    for (uint32_t g = g0; g < g1; g++) {
        const uint32_t v = col[g];
        col[g] = base;
        base += v;
    }
    if (threadIdx.x == 255) tot[blockIdx.x] = base;
}

// koff[k] = rows with index < k, koff[K] = N; seg/blk offsets of the chains (64-step segments,
// 64-segment blocks).  One block of 1024 threads.
__global__ __launch_bounds__(1024) void ks_offsets_kernel(const uint32_t *__restrict__ tot, uint32_t K,
                                                         uint32_t *__restrict__ koff, uint32_t *__restrict__ segoff,
                                                         uint32_t *__restrict__ blkoff) {
    __shared__ uint32_t part[3][1024];
    const uint32_t per = (K + 1023) / 1024, b = min(K, threadIdx.x * per), e = min(K, b + per);
    uint32_t s[3] = {0, 0, 0};
    for (uint32_t i = b; i < e; i++) {
        const uint32_t n = tot[i], ns = (n + L - 1) / L;
        s[0] += n;
        s[1] += ns;
        s[2] += (ns + SPB - 1) / SPB;
    }
    for (int l = 0; l < 3; l++) part[l][threadIdx.x] = s[l];
    __syncthreads();
    for (uint32_t o = 1; o < 1024; o <<= 1) {
        uint32_t v[3];
        for (int l = 0; l < 3; l++) v[l] = threadIdx.x >= o ? part[l][threadIdx.x - o] : 0u;
        __syncthreads();
        for (int l = 0; l < 3; l++) part[l][threadIdx.x] += v[l];
        __syncthreads();
    }
    uint32_t base[3];
    for (int l = 0; l < 3; l++) base[l] = part[l][threadIdx.x] - s[l];
    for (uint32_t i = b; i < e; i++) {
        const uint32_t n = tot[i], ns = (n + L - 1) / L;
        koff[i] = base[0];
        segoff[i] = base[1];
        blkoff[i] = base[2];
        base[0] += n;
        base[1] += ns;
        base[2] += (ns + SPB - 1) / SPB;
    }
    if (threadIdx.x == 1023) {
        koff[K] = part[0][1023];
        segoff[K] = part[1][1023];
        blkoff[K] = part[2][1023];
    }
}

// planes[d][p] = component d of the p-th row in (cell, row) order: a wave per 4096 rows, 64-row
// chunks in order.  Each chunk's (cell, lane) pairs are sorted across the wave (bitonic, by
// shuffles), so a row's rank among the chunk's rows of its cell is its distance from its run's
// start; the sorted lanes write the rows (each run's bytes contiguous) and each run's last lane
// advances its cell's position.
template <int DP>
__global__ __launch_bounds__(64) void ks_scatter_kernel(const uint8_t *__restrict__ codes, const uint32_t *__restrict__ A,
                                                       uint64_t N, uint32_t K, uint32_t D, uint32_t G,
                                                       const uint32_t *__restrict__ hist,
                                                       const uint32_t *__restrict__ koff, uint64_t PL,
                                                       uint8_t *__restrict__ planes, const uint32_t *__restrict__ sel,
                                                       uint32_t n_sel) {
    constexpr int W = DP / 4;
    extern __shared__ uint32_t cur[];
    for (uint32_t i = threadIdx.x; i < K; i += 64) cur[i] = koff[i] + hist[(uint64_t)i * G + blockIdx.x];
    __syncthreads();
    const uint32_t lane = lane_id();
    constexpr uint32_t NOKEY = (1u << 26) - 1;
    const uint64_t r0 = (uint64_t)blockIdx.x * SROWS, r1 = min(N, r0 + SROWS);
    // the block's indices, all loads in flight before the first chunk (with few cells selected
    // most chunks have no row to move, and the index loads were the kernel's time)
    uint32_t ak[SROWS / 64];
#pragma unroll
    for (int i = 0; i < (int)(SROWS / 64); i++) {
        const uint64_t r = r0 + 64 * i + lane;
        ak[i] = r < r1 ? A[r] : ~0u;
    }
#pragma unroll
    for (int i = 0; i < (int)(SROWS / 64); i++) {
        const uint64_t base = r0 + 64 * i;
        if (base >= r1) break;
        const uint64_t r = base + lane;
        uint32_t a = r < r1 ? ks_key(ak[i], K, sel, n_sel) : ~0u;
        if (a == ~0u) a = NOKEY;   // a row of a cell not asked for
        if (__ballot(a != NOKEY) == 0) continue;      // (wave-uniform)
        uint32_t w[W];
        const uint32_t *src = reinterpret_cast<const uint32_t *>(codes + (a != NOKEY ? r : r0) * DP);
#pragma unroll
        for (int u = 0; u < W; u++) w[u] = a != NOKEY ? src[u] : 0u;
        uint32_t v = (a << 6) | lane;
        for (uint32_t k = 2; k <= 64; k <<= 1)
            for (uint32_t j = k >> 1; j > 0; j >>= 1) {
                const uint32_t o = __shfl_xor(v, j, 64);
                const bool lo_half = (lane & j) == 0, up = (lane & k) == 0;
                v = (lo_half == up) ? min(v, o) : max(v, o);
            }
        const uint32_t key = v >> 6, from = v & 63;
        const uint32_t kprev = __shfl_up(key, 1, 64), knext = __shfl_down(key, 1, 64);
        const bool start = lane == 0 || kprev != key, end = lane == 63 || knext != key;
        uint32_t rs = start ? lane : 0;
        for (int o = 1; o < 64; o <<= 1) {
            const uint32_t t = __shfl_up(rs, o, 64);
            if (lane >= (uint32_t)o) rs = max(rs, t);
        }
        uint32_t row[W];
#pragma unroll
        for (int u = 0; u < W; u++) row[u] = __shfl(w[u], from, 64);
        if (key != NOKEY) {
            const uint32_t dst = cur[key] + (lane - rs);
            KCHK(key < K && dst < PL && (uint64_t)(D - 1) * PL + dst < (uint64_t)PL * D + 64);
#pragma unroll
            for (int d = 0; d < DP; d++)
                if ((uint32_t)d < D) planes[(uint64_t)d * PL + dst] = (uint8_t)(row[d >> 2] >> (8 * (d & 3)));
            if (end) cur[key] = dst + 1;
        }
        wave_sync();
    }
}

// The mean's single cell (no sort): planes[d][p] = component d of row p.
template <int DP>
__global__ __launch_bounds__(256) void ks_transpose_kernel(const uint8_t *__restrict__ codes, uint64_t N, uint32_t D,
                                                          uint64_t PL, uint8_t *__restrict__ planes) {
    constexpr int W = DP / 4;
    const uint64_t p0 = ((uint64_t)blockIdx.x * 256 + threadIdx.x) * 4;
    if (p0 >= N) return;
    uint32_t w[4][W];
#pragma unroll
    for (int i = 0; i < 4; i++) {
        const uint32_t *src = reinterpret_cast<const uint32_t *>(codes + min(p0 + i, N - 1) * DP);
#pragma unroll
        for (int u = 0; u < W; u++) w[i][u] = src[u];
    }
#pragma unroll
    for (int d = 0; d < DP; d++)
        if ((uint32_t)d < D) {
            uint32_t v = 0;
#pragma unroll
            for (int t = 0; t < 4; t++) v |= ((w[t][d >> 2] >> (8 * (d & 3))) & 0xFFu) << (8 * t);
            *reinterpret_cast<uint32_t *>(planes + (uint64_t)d * PL + p0) = v;
        }
}

// ---- shared: blocks of a chain ---------------------------------------------------------------
struct Geo {
    const uint8_t *planes;
    uint64_t PL;                              // plane stride (N rounded up, plus padding)
    const uint32_t *koff, *segoff, *blkoff;   // [K + 1] each
    uint32_t K, D;
    SegMeta *meta;                            // [D][segoff[K]]
    u128 *bsum;                               // [D][blkoff[K]]: block totals, then (scan) block prefixes
    Fn *bfn;                                  // [D][blkoff[K]]
    kahan::SegFn *sfn;                        // [D][segoff[K]]: the segment functions (estimates 0)
    Fn *bfn8;                                 // [D][blkoff[K]][8]: 8-segment sub-block functions
    unsigned *stats;                          // [4]: blocks not composable, block misses, segment replays, chains
    uint64_t plane_bytes, seg_cap, blk_cap;   // capacities (QVQ_KDEBUG checks)
};

__device__ inline void stage_tab(const ByteTab *__restrict__ g, ByteTab *t) {
    const uint32_t *src = reinterpret_cast<const uint32_t *>(g);
    uint32_t *dst = reinterpret_cast<uint32_t *>(t);
    for (uint32_t i = threadIdx.x; i < sizeof(ByteTab) / 4; i += blockDim.x) dst[i] = src[i];
}

// cell of flat block index fb (blkoff in LDS)
__device__ inline uint32_t find_cell(const uint32_t *off, uint32_t K, uint32_t v) {   // off[k] <= v < off[k+1]
    uint32_t lo = 0, hi = K;
    while (hi - lo > 1) {
        const uint32_t mid = (lo + hi) / 2;
        if (off[mid] <= v) lo = mid;
        else hi = mid;
    }
    return lo;
}

// The wave stages the bytes [src, src + n) (n <= BLK_STEPS) into dst (4-byte aligned).
__device__ inline void stage_bytes(const uint8_t *__restrict__ src, uint32_t n, uint8_t *dst) {
    const uint32_t lane = lane_id();
    const uintptr_t a = (uintptr_t)src, a0 = a & ~(uintptr_t)3;
    const uint32_t m = (uint32_t)(a - a0);
    const uint32_t *s32 = reinterpret_cast<const uint32_t *>(a0);
    uint32_t *d32 = reinterpret_cast<uint32_t *>(dst);
    const uint32_t nw = (n + 3) / 4;
    for (uint32_t i = lane; i < nw; i += 64) {
        const uint32_t lo = s32[i], hi = m ? s32[i + 1] : 0u;   // planes are padded past the end
        d32[i] = m ? (uint32_t)(((uint64_t)hi << 32 | lo) >> (8 * m)) : lo;
    }
}

// ---- 3. meta ---------------------------------------------------------------------------------
constexpr int WPB = 4;   // waves per workgroup (meta, build)

__device__ inline void meta_block(const Geo &g, const ByteTab &tab, uint8_t *bytes_w, uint32_t TB, uint64_t fb,
                                  uint32_t lane) {
    const uint32_t d = (uint32_t)(fb / TB), bb = (uint32_t)(fb - (uint64_t)d * TB);
    const uint32_t k = find_cell(g.blkoff, g.K, bb), b = bb - g.blkoff[k];
    const uint32_t n = g.koff[k + 1] - g.koff[k];
    const uint32_t s0 = b * SPB, first = s0 * L, nb = min(BLK_STEPS, n - first);
    KCHK(TB <= g.blk_cap && g.segoff[g.K] <= g.seg_cap && first < n && k < g.K);
    KCHK((uint64_t)d * g.PL + g.koff[k] + first + nb + 8 <= g.plane_bytes);
    stage_bytes(g.planes + (uint64_t)d * g.PL + g.koff[k] + first, nb, bytes_w);
    wave_sync();
    const uint32_t s = s0 + lane, nseg = (n + L - 1) / L;
    u128 tot = 0;
    if (s < nseg) {
        const uint32_t len = min(L, n - s * L);
        const SegMeta m = kahan::seg_meta(tab, bytes_w + lane * L, len);
        g.meta[(uint64_t)d * g.segoff[g.K] + g.segoff[k] + s] = m;
        tot = kahan::meta_sum(m);
    }
    uint64_t lo = (uint64_t)tot, hi = (uint64_t)(tot >> 64);
    for (int o = 32; o >= 1; o >>= 1) {   // wave sum of the block's segments (128-bit)
        const uint64_t l2 = __shfl_xor((unsigned long long)lo, o, 64), h2 = __shfl_xor((unsigned long long)hi, o, 64);
        const uint64_t t = lo + l2;
        hi = hi + h2 + (t < lo);
        lo = t;
    }
    if (lane == 0) g.bsum[(uint64_t)d * TB + bb] = ((u128)hi << 64) | lo;
}

// Grid-stride over the (component, block) pairs: the grid is sized by the capacity (the host
// does not know the block count), and a workgroup without a pair leaves before staging the
// 6.5 KB byte table (28k empty workgroups staged it at C4: ~180 MB of L2 reads per launch).
__global__ __launch_bounds__(64 * WPB) void ks_meta_kernel(Geo g, const ByteTab *__restrict__ gtab) {
    __shared__ ByteTab tab;
    __shared__ __attribute__((aligned(16))) uint8_t bytes[WPB][BLK_STEPS];
    const uint32_t TB = g.blkoff[g.K];
    const uint64_t total = (uint64_t)TB * g.D;
    if ((uint64_t)blockIdx.x * WPB >= total) return;
    stage_tab(gtab, &tab);
    __syncthreads();
    const uint32_t w = threadIdx.x >> 6, lane = lane_id();
    for (uint64_t fb = (uint64_t)blockIdx.x * WPB + w; fb < total; fb += (uint64_t)gridDim.x * WPB)
        meta_block(g, tab, bytes[w], TB, fb, lane);
}

// ---- 3b. chained: this rank's chain totals and row counts into its slice of gather ----------
__global__ __launch_bounds__(256) void ks_totals_kernel(Geo g, uint64_t *__restrict__ gather, uint32_t rank,
                                                       uint32_t nranks) {
    const uint32_t lane = lane_id();
    const uint64_t wv = ((uint64_t)blockIdx.x * 256 + threadIdx.x) >> 6;
    if (wv >= (uint64_t)g.K * g.D) return;
    const uint32_t k = (uint32_t)(wv / g.D), d = (uint32_t)(wv - (uint64_t)k * g.D);
    const uint32_t TB = g.blkoff[g.K];
    KCHK(TB <= g.blk_cap && g.blkoff[k + 1] <= TB && g.blkoff[k] <= g.blkoff[k + 1]);
    const u128 *p = g.bsum + (uint64_t)d * TB;
    uint64_t lo = 0, hi = 0;
    for (uint32_t i = g.blkoff[k] + lane; i < g.blkoff[k + 1]; i += 64) {
        const u128 v = p[i];
        const uint64_t t = lo + (uint64_t)v;
        hi += (uint64_t)(v >> 64) + (t < lo);
        lo = t;
    }
    for (int o = 32; o >= 1; o >>= 1) {
        const uint64_t l2 = __shfl_xor((unsigned long long)lo, o, 64), h2 = __shfl_xor((unsigned long long)hi, o, 64);
        const uint64_t t = lo + l2;
        hi = hi + h2 + (t < lo);
        lo = t;
    }
    if (lane == 0) {
        const uint64_t KD = (uint64_t)g.K * g.D;
        uint64_t *e = gather + 2 * (rank * KD + (uint64_t)k * g.D + d);
        e[0] = lo;
        e[1] = hi;
        if (d == 0) gather[2 * nranks * KD + (uint64_t)rank * g.K + k] = g.koff[k + 1] - g.koff[k];
    }
}

// ---- 4. block prefixes: exclusive scan of the block totals along every chain --------------------
// Chained chains (a cell's rows split over ranks): gather (u64) holds every rank's
// chain totals [nranks][K * D][lo, hi] and row counts [nranks][K]; a rank's chains start at
// the exact sum of the lower ranks' rows.
__device__ inline u128 chain_prefix(const uint64_t *gather, uint32_t rank, uint64_t KD, uint64_t t) {
    u128 p = 0;
    for (uint32_t q = 0; q < rank; q++) {
        const uint64_t *e = gather + 2 * (q * KD + t);
        p += ((u128)e[1] << 64) | e[0];
    }
    return p;
}

__global__ __launch_bounds__(256) void ks_bscan_kernel(Geo g, const uint64_t *__restrict__ gather, uint32_t rank) {
    const uint32_t lane = lane_id();
    const uint64_t wv = ((uint64_t)blockIdx.x * 256 + threadIdx.x) >> 6;
    if (wv >= (uint64_t)g.K * g.D) return;
    const uint32_t k = (uint32_t)(wv / g.D), d = (uint32_t)(wv - (uint64_t)k * g.D);
    const uint32_t TB = g.blkoff[g.K];
    u128 *p = g.bsum + (uint64_t)d * TB;
    const uint32_t b0 = g.blkoff[k], b1 = g.blkoff[k + 1];
    u128 carry = gather ? chain_prefix(gather, rank, (uint64_t)g.K * g.D, (uint64_t)k * g.D + d) : (u128)0;
    for (uint32_t base = b0; base < b1; base += 64) {
        const uint32_t i = base + lane;
        const u128 v = i < b1 ? p[i] : 0;
        u128 inc = v;
        for (int o = 1; o < 64; o <<= 1) {
            const uint64_t l = __shfl_up((unsigned long long)(uint64_t)inc, o, 64);
            const uint64_t h = __shfl_up((unsigned long long)(uint64_t)(inc >> 64), o, 64);
            if (lane >= (uint32_t)o) inc += ((u128)h << 64) | l;
        }
        if (i < b1) p[i] = carry + inc - v;
        const uint64_t tl = __shfl((unsigned long long)(uint64_t)inc, 63, 64);
        const uint64_t th = __shfl((unsigned long long)(uint64_t)(inc >> 64), 63, 64);
        carry += ((u128)th << 64) | tl;
    }
}

// Exclusive wave scan of 128-bit values.
__device__ inline u128 wave_excl_scan(u128 v) {
    const uint32_t lane = lane_id();
    u128 inc = v;
    for (int o = 1; o < 64; o <<= 1) {
        const uint64_t l = __shfl_up((unsigned long long)(uint64_t)inc, o, 64);
        const uint64_t h = __shfl_up((unsigned long long)(uint64_t)(inc >> 64), o, 64);
        if (lane >= (uint32_t)o) inc += ((u128)h << 64) | l;
    }
    return inc - v;
}

// Each lane's function for segment b * SPB + lane of chain (k, d) (the block's bytes already in
// `bytes`), estimate D_est, into fns[lane]; returns the exact prefix sum at the segment's start.
// Lanes past the chain's end get an empty translation.
__device__ inline u128 build_block_fns(const Geo &g, const ByteTab &tab, const uint8_t *bytes, uint32_t k, uint32_t d,
                                       uint32_t b, int64_t D_est, Fn *fns) {
    const uint32_t lane = lane_id();
    const uint32_t n = g.koff[k + 1] - g.koff[k], nseg = (n + L - 1) / L;
    const uint32_t s = b * SPB + lane;
    const uint64_t mbase = (uint64_t)d * g.segoff[g.K] + g.segoff[k];
    SegMeta self{};
    if (s < nseg) self = g.meta[mbase + s];
    const u128 P = g.bsum[(uint64_t)d * g.blkoff[g.K] + g.blkoff[k] + b] +
                   wave_excl_scan(s < nseg ? kahan::meta_sum(self) : (u128)0);
    Fn f;
    int ne = 0, bl0 = 0;
    const uint8_t *bs = bytes + lane * L;
    const uint32_t len = s < nseg ? min(L, n - s * L) : L;
    if (s < nseg) {
        int c_in;
        uint32_t off_in;
        kahan::input_structure([&](int i) { return g.meta[mbase + s - i]; }, (int)min(8u, s), c_in, off_in);
        ne = kahan::build_header(bs, len, P, self, c_in, off_in, s + 1 == nseg, f, bl0);
    } else {
        f.kind = kahan::FK_TRANS;
        f.c_in = f.lne = f.c_out = 0;
        f.off_in = f.off_out = f.sx9 = f.pad = 0;
        f.lo = f.hi = 0;
        for (int e = 0; e < kahan::NE; e++) f.dlt[e] = 0;
    }
    // the entries, wave-uniform (lanes of one wave otherwise run every template variant in turn)
    const bool fast = ne && bl0, slow = ne && !bl0;
    int nf = fast ? ne : 0, nx = slow ? ne : 0;
    for (int o = 32; o >= 1; o >>= 1) {
        nf = max(nf, __shfl_xor(nf, o, 64));
        nx = max(nx, __shfl_xor(nx, o, 64));
    }
    if (nf == 1 || nf == 2) kahan::build_entries<2, false>(tab, bs, len, P, bl0, D_est, 0, f, fast);
    else
        for (int e0 = 0; e0 < nf; e0 += 4) kahan::build_entries<4, false>(tab, bs, len, P, bl0, D_est, e0, f, fast && e0 < ne);
    for (int e0 = 0; e0 < nx; e0++) kahan::build_entries<1, true>(tab, bs, len, P, 0, D_est, e0, f, slow && e0 < ne);
    fns[lane] = f;
    return P;
}

// ---- 5. build: block functions ------------------------------------------------------------------
__device__ inline void build_block(const Geo &g, const ByteTab &tab, uint8_t *bytes_w, Fn *fns_w, uint8_t *ok_w,
                                   uint32_t TB, uint64_t fb, uint32_t lane) {
    const uint32_t d = (uint32_t)(fb / TB), bb = (uint32_t)(fb - (uint64_t)d * TB);
    const uint32_t k = find_cell(g.blkoff, g.K, bb), b = bb - g.blkoff[k];
    const uint32_t n = g.koff[k + 1] - g.koff[k];
    const uint32_t first = b * BLK_STEPS;
    stage_bytes(g.planes + (uint64_t)d * g.PL + g.koff[k] + first, min(BLK_STEPS, n - first), bytes_w);
    wave_sync();
    build_block_fns(g, tab, bytes_w, k, d, b, 0, fns_w);
    const uint32_t nseg = (n + L - 1) / L, cnt = min(SPB, nseg - b * SPB);
    if (lane < cnt) {   // for the evaluation's re-walks of blocks that do not answer
        kahan::SegFn sf;
        kahan::pack_seg(fns_w[lane], sf);
        g.sfn[(uint64_t)d * g.segoff[g.K] + g.segoff[k] + b * SPB + lane] = sf;
    }
    ok_w[lane] = kahan::fkind(fns_w[lane]) != kahan::FK_RAW;
    wave_sync();
    for (uint32_t st = 1; st < SPB; st <<= 1) {   // tree: fns[i] <- fns[i] then fns[i + st]
        if ((lane & (2 * st - 1)) == 0 && lane + st < cnt) {
            Fn h;
            const bool c = ok_w[lane] && ok_w[lane + st] && kahan::compose(fns_w[lane], fns_w[lane + st], h);
            ok_w[lane] = c;
            if (c) fns_w[lane] = h;
        }
        wave_sync();
        if (st == 4 && (lane & 7) == 0 && lane < cnt) {   // the 8-segment sub-blocks, for the evaluation
            Fn r = fns_w[lane];
            if (!ok_w[lane]) kahan::set_raw(r);
            g.bfn8[((uint64_t)d * TB + bb) * 8 + lane / 8] = r;
        }
    }
    if (lane == 0) {
        Fn r = fns_w[0];
        if (!ok_w[0]) {
            kahan::set_raw(r);
            if (g.stats) atomicAdd(&g.stats[0], 1u);
        }
        g.bfn[(uint64_t)d * TB + bb] = r;
    }
}

__global__ __launch_bounds__(64 * WPB) void ks_build_kernel(Geo g, const ByteTab *__restrict__ gtab) {
    __shared__ ByteTab tab;
    __shared__ __attribute__((aligned(16))) uint8_t bytes[WPB][BLK_STEPS];
    __shared__ Fn fns[WPB][SPB];
    __shared__ uint8_t ok[WPB][SPB];
    const uint32_t TB = g.blkoff[g.K];
    const uint64_t total = (uint64_t)TB * g.D;
    if ((uint64_t)blockIdx.x * WPB >= total) return;   // (ks_meta_kernel's note)
    stage_tab(gtab, &tab);
    __syncthreads();
    const uint32_t w = threadIdx.x >> 6, lane = lane_id();
    for (uint64_t fb = (uint64_t)blockIdx.x * WPB + w; fb < total; fb += (uint64_t)gridDim.x * WPB)
        build_block(g, tab, bytes[w], fns[w], ok[w], TB, fb, lane);
}

// ---- 6. eval ----------------------------------------------------------------------------------
constexpr int EPB = 4;   // chains per workgroup (a wave each)

__device__ inline u128 bcast_u128(u128 v) {
    return ((u128)(uint64_t)__shfl((unsigned long long)(uint64_t)(v >> 64), 0, 64) << 64) |
           (uint64_t)__shfl((unsigned long long)(uint64_t)v, 0, 64);
}

// state (chained, nullptr: one rank): per chain the reference's state (sum, c) as two doubles'
// bits, read as the chain's input (the lower ranks' rows summed) and overwritten by its state
// after this rank's rows; C and split_out are then not written (ks_finish_kernel divides).
// gather / rank: the chains' exact prefix at this rank's first row (chain_prefix).
__global__ __launch_bounds__(64 * EPB) void ks_eval_kernel(Geo g, const ByteTab *__restrict__ gtab,
                                                          double *__restrict__ C, double *__restrict__ split_out,
                                                          uint64_t *__restrict__ state,
                                                          const uint64_t *__restrict__ gather, uint32_t rank) {
    __shared__ ByteTab tab;
    __shared__ __attribute__((aligned(16))) uint8_t bytes[EPB][BLK_STEPS];
    __shared__ Fn fns[EPB][SPB];
    __shared__ u128 pseg[EPB][SPB];
    stage_tab(gtab, &tab);
    __syncthreads();
    const uint32_t w = threadIdx.x >> 6, lane = lane_id();
    const uint64_t wv = (uint64_t)blockIdx.x * EPB + w;
    if (wv >= (uint64_t)g.K * g.D) return;
    const uint32_t k = (uint32_t)(wv / g.D), d = (uint32_t)(wv - (uint64_t)k * g.D);
    const uint32_t n = g.koff[k + 1] - g.koff[k], nseg = (n + L - 1) / L;
    const uint8_t *src = g.planes + (uint64_t)d * g.PL + g.koff[k];
    const uint32_t TB = g.blkoff[g.K];
    const u128 *bpre = g.bsum + (uint64_t)d * TB + g.blkoff[k];
    const uint64_t mbase = (uint64_t)d * g.segoff[g.K] + g.segoff[k];
    const uint64_t t_out = (uint64_t)k * g.D + d;
    KCHK(TB <= g.blk_cap && g.segoff[g.K] <= g.seg_cap && g.blkoff[k + 1] <= TB && g.koff[k + 1] <= g.koff[g.K]);
    KCHK((uint64_t)d * g.PL + g.koff[g.K] + 64 <= g.plane_bytes);
    KCHK(g.segoff[k] + nseg <= g.segoff[g.K] && g.blkoff[k] + (nseg + SPB - 1) / SPB <= g.blkoff[k + 1]);
    // the state entering this rank's rows, and their exact prefix (one rank: the chain's start)
    double sum = 0, c = 0;
    u128 P0 = 0;
    if (state) {
        sum = __longlong_as_double((long long)state[2 * t_out]);
        c = __longlong_as_double((long long)state[2 * t_out + 1]);
        if (gather) P0 = chain_prefix(gather, rank, (uint64_t)g.K * g.D, t_out);
    }
    // the exact total after this rank's rows: the last block's prefix and its segments' sums
    u128 Pn = P0;
    if (n) {
        const uint32_t lb = (nseg - 1) / SPB, s = lb * SPB + lane;
        const u128 v = s < nseg ? kahan::meta_sum(g.meta[mbase + s]) : (u128)0;
        uint64_t lo = (uint64_t)v, hi = (uint64_t)(v >> 64);
        for (int o = 32; o >= 1; o >>= 1) {
            const uint64_t l2 = __shfl_xor((unsigned long long)lo, o, 64), h2 = __shfl_xor((unsigned long long)hi, o, 64);
            const uint64_t t = lo + l2;
            hi = hi + h2 + (t < lo);
            lo = t;
        }
        Pn = bpre[lb] + (((u128)hi << 64) | lo);
    }
    // nothing to add: no rows, or every value 0 while c = 0 (a zero step then changes nothing;
    // with sum >= 2 a zero step is exact for any c)
    if (n && (Pn != P0 || (c != 0.0 && !(sum >= 2.0)))) {
        // the transient: the reference's doubles until sum >= 2 (lane 0; bytes staged per block;
        // segments of zeros skipped while c = 0, where a zero step changes nothing)
        uint32_t i = 0, staged = 0xFFFFFFFFu;
        u128 P = P0;
        while (i < n && !(sum >= 2.0)) {
            const uint32_t b = i / BLK_STEPS;
            if (c == 0 && i % L == 0) {
                const uint32_t s = b * SPB + lane;
                const bool nz = s >= i / L && s < nseg && kahan::meta_sum(g.meta[mbase + s]) != 0;
                const uint64_t mask = __ballot(nz);
                if (!mask) {
                    i = min(n, (b + 1) * BLK_STEPS);
                    continue;
                }
                i = max(i, (b * SPB + (uint32_t)(__ffsll((long long)mask) - 1)) * L);
            }
            if (b != staged) {
                stage_bytes(src + b * BLK_STEPS, min(BLK_STEPS, n - b * BLK_STEPS), bytes[w]);
                wave_sync();
                staged = b;
            }
            const uint32_t e = min(n, (i / L + 1) * L);   // to the end of the segment
            if (lane == 0)
                while (i < e && !(sum >= 2.0)) {
                    const uint64_t X = tab.X[bytes[w][i - b * BLK_STEPS]];
                    kahan::fstep(sum, c, ldexp((double)X, -60));
                    P += X;
                    i++;
                }
            i = __shfl(i, 0, 64);
            sum = __shfl(sum, 0, 64);
            c = __shfl(c, 0, 64);
            P = bcast_u128(P);
        }
        if (sum >= 2.0) {
            const u128 E = (u128)(kahan::to_units(sum) - kahan::to_units(c));
            int64_t D = (int64_t)(E - P);
            uint32_t F = (uint32_t)E & 511;
            uint32_t j = (i + L - 1) / L;
            if (i % L) {   // exactly to the next segment boundary (inside the staged block)
                const uint32_t e = min(n, j * L);
                if (lane == 0) D += kahan::replay(tab, bytes[w] + (i - staged * BLK_STEPS), e - i, P, F, D);
                D = __shfl((long long)D, 0, 64);
                F = __shfl(F, 0, 64);
            }
            unsigned nmiss = 0, nrep = 0;
            const Fn *bf = g.bfn + (uint64_t)d * TB + g.blkoff[k];
            const Fn *bf8 = g.bfn8 + ((uint64_t)d * TB + g.blkoff[k]) * 8;
            const uint32_t nblk = (nseg + SPB - 1) / SPB;
            uint32_t loaded = 0xFFFFFFFFu;   // the block whose segment functions sit in fns[w]
            Fn fnext;
            if (j % SPB == 0 && j < nseg) fnext = bf[j / SPB];
            while (j < nseg) {
                const uint32_t b = j / SPB;
                if (j % SPB == 0) {
                    const Fn f = fnext;   // every lane: uniform
                    if (b + 1 < nblk) fnext = bf[b + 1];
                    if (kahan::apply(f, F, D)) {
                        j = min(nseg, j + SPB);
                        continue;
                    }
                    nmiss++;
                }
                if (j % 8 == 0) {   // the 8-segment sub-block
                    const Fn f = bf8[j / 8];
                    if (kahan::apply(f, F, D)) {
                        j = min(nseg, j + 8);
                        if (j % SPB == 0 && j < nseg) fnext = bf[j / SPB];
                        continue;
                    }
                }
                // segment by segment: the block's stored segment functions, each checked
                if (loaded != b) {
                    if (staged != b) {
                        stage_bytes(src + b * BLK_STEPS, min(BLK_STEPS, n - b * BLK_STEPS), bytes[w]);
                        staged = b;
                    }
                    const uint32_t s = b * SPB + lane;
                    const u128 v = s < nseg ? kahan::meta_sum(g.meta[mbase + s]) : (u128)0;
                    pseg[w][lane] = bpre[b] + wave_excl_scan(v);
                    if (s < nseg) kahan::unpack_seg(g.sfn[mbase + s], fns[w][lane]);
                    loaded = b;
                    wave_sync();
                }
                const uint32_t end = min(nseg, (j / 8 + 1) * 8);
                for (; j < end; j++) {
                    if (kahan::apply(fns[w][j - b * SPB], F, D)) continue;
                    nrep++;
                    if (lane == 0)
                        D += kahan::replay(tab, bytes[w] + (j - b * SPB) * L, min(L, n - j * L), pseg[w][j - b * SPB],
                                           F, D);
                    D = __shfl((long long)D, 0, 64);
                    F = __shfl(F, 0, 64);
                }
                if (j % SPB == 0 && j < nseg) fnext = bf[j / SPB];
            }
            // the state is E = Pn + D exactly: sum = RN(E), c = sum - E (kahan_par.hpp)
            const u128 Ef = Pn + (u128)(i128)D;
            sum = kahan::to_double(Ef);
            c = ldexp((double)(int64_t)(kahan::to_units(sum) - (i128)Ef), -60);
            if (g.stats && lane == 0 && (nmiss | nrep)) {
                atomicAdd(&g.stats[1], nmiss);
                atomicAdd(&g.stats[2], nrep);
            }
        }
    }
    if (lane == 0) {
        if (state) {
            state[2 * t_out] = (uint64_t)__double_as_longlong(sum);
            state[2 * t_out + 1] = (uint64_t)__double_as_longlong(c);
        } else {
            // operator/= by a scalar under -freciprocal-math; an empty cell stays 0 (no divide)
            const double result = n ? __dmul_rn(sum, 1.0 / (double)n) : 0.0;
            C[t_out] = result;
            if (split_out) {   // src/Quantizer.cpp:134-138: C * (1 + 0.2), then C * (1 - 0.2)
                split_out[t_out] = __dmul_rn(result, (double)(1 + 0.2));
                split_out[(uint64_t)g.K * g.D + t_out] = __dmul_rn(result, (double)(1 - 0.2));
            }
        }
    }
}

// Chained: C = sum * fl(1/n) with n the cell's rows on every rank (an empty cell stays 0), and
// the split, from the state after the last rank's rows.
__global__ __launch_bounds__(256) void ks_finish_kernel(uint32_t K, uint32_t D, const uint64_t *__restrict__ state,
                                                       const uint64_t *__restrict__ gather, uint32_t nranks,
                                                       double *__restrict__ C, double *__restrict__ split_out) {
    const uint64_t t = (uint64_t)blockIdx.x * 256 + threadIdx.x;
    const uint64_t KD = (uint64_t)K * D;
    if (t >= KD) return;
    const uint32_t k = (uint32_t)(t / D);
    uint64_t n = 0;
    for (uint32_t q = 0; q < nranks; q++) n += gather[2 * nranks * KD + (uint64_t)q * K + k];
    const double sum = __longlong_as_double((long long)state[2 * t]);
    const double result = n ? __dmul_rn(sum, 1.0 / (double)n) : 0.0;
    C[t] = result;
    if (split_out) {
        split_out[t] = __dmul_rn(result, (double)(1 + 0.2));
        split_out[KD + t] = __dmul_rn(result, (double)(1 - 0.2));
    }
}

__global__ void ks_set_u32_kernel(uint32_t *p, uint32_t v) { *p = v; }

// Short chains: the reference's chain (src/Quantizer.cpp:59-70) step by step, one lane per
// (cell, component), bytes from the sorted planes, values from the byte table; then fl(1/n) and
// the split as ks_eval_kernel.  For cells of a few thousand rows this beats the segment
// functions' meta / scan / build / eval (~200 us for C4's 20 checked cells, profiles/r05h: the
// build of 64 functions per wave is the pole) at ~25 ns per step.
__global__ __launch_bounds__(256) void ks_direct_kernel(const uint8_t *__restrict__ planes, uint64_t PL,
                                                       const uint32_t *__restrict__ koff, uint32_t K, uint32_t D,
                                                       const ByteTab *__restrict__ gtab, double *__restrict__ C,
                                                       double *__restrict__ split_out) {
    __shared__ double xv[256];
    xv[threadIdx.x] = ldexp((double)gtab->X[threadIdx.x], -60);   // the byte's value, exactly
    __syncthreads();
    const uint64_t t = (uint64_t)blockIdx.x * 256 + threadIdx.x;
    if (t >= (uint64_t)K * D) return;
    const uint32_t k = (uint32_t)(t / D), d = (uint32_t)(t - (uint64_t)k * D);
    const uint32_t n = koff[k + 1] - koff[k];
    const uint8_t *src = planes + (uint64_t)d * PL + koff[k];
    double sum = 0, c = 0;
    uint32_t i = 0;
    for (; i + 16 <= n; i += 16) {   // the loads of 16 steps issued together
        uint8_t b[16];
#pragma unroll
        for (int j = 0; j < 16; j++) b[j] = src[i + j];
#pragma unroll
        for (int j = 0; j < 16; j++) kahan::fstep(sum, c, xv[b[j]]);
    }
    for (; i < n; i++) kahan::fstep(sum, c, xv[src[i]]);
    const double result = n ? __dmul_rn(sum, 1.0 / (double)n) : 0.0;
    C[t] = result;
    if (split_out) {   // src/Quantizer.cpp:134-138
        split_out[t] = __dmul_rn(result, (double)(1 + 0.2));
        split_out[(uint64_t)K * D + t] = __dmul_rn(result, (double)(1 - 0.2));
    }
}

}  // namespace

// ---- host side -------------------------------------------------------------------------------
size_t KahanWork::tab_bytes() { return sizeof(ByteTab); }

void KahanWork::make_tab(const uint64_t *X, void *out) { kahan::make_tab(X, *reinterpret_cast<ByteTab *>(out)); }

void KahanWork::caps(uint64_t N, uint32_t K, uint64_t &segs, uint64_t &blks) {
    segs = (N + L - 1) / L + K;
    blks = segs / SPB + K + 1;
}
uint64_t KahanWork::plane_len(uint64_t N) { return (N + 63) / 64 * 64 + 64; }
size_t KahanWork::meta_bytes() { return sizeof(SegMeta); }
size_t KahanWork::fn_bytes() { return sizeof(Fn); }
size_t KahanWork::segfn_bytes() { return sizeof(kahan::SegFn); }
uint32_t KahanWork::sort_blocks(uint64_t N) { return (uint32_t)((N + SROWS - 1) / SROWS); }

namespace {

// The sort into component planes (the selected cells' rows, or every row for the mean).
hipError_t kahan_sort(hipStream_t s, const KahanWork &w, const uint8_t *codes, uint32_t Dp, uint32_t D, uint64_t N,
                      const uint32_t *A, uint32_t K, const uint32_t *sel, uint32_t n_sel) {
    if (N == 0 || N > 0xFFFFFFFFull || D == 0 || K == 0 || D > Dp || Dp > 64 || (Dp & 3) || N > w.n_cap ||
        K > w.k_cap || D > w.d_cap)
        return hipErrorInvalidValue;
    const uint32_t G = KahanWork::sort_blocks(N);
    const uint64_t PL = KahanWork::plane_len(N);
    if (A) {
        hipLaunchKernelGGL(ks_hist_kernel, dim3(G), dim3(64), K * 4, s, A, N, K, G, w.hist, sel, n_sel);
        hipLaunchKernelGGL(ks_colscan_kernel, dim3(K), dim3(256), 0, s, w.hist, G, w.tot);
    } else {
        if (K != 1) return hipErrorInvalidValue;
        hipLaunchKernelGGL(ks_set_u32_kernel, dim3(1), dim3(1), 0, s, w.tot, (uint32_t)N);
    }
    hipLaunchKernelGGL(ks_offsets_kernel, dim3(1), dim3(1024), 0, s, w.tot, K, w.koff, w.segoff, w.blkoff);
    switch (Dp) {
#define X(DPV)                                                                                                     \
    case DPV:                                                                                                      \
        if (A)                                                                                                     \
            hipLaunchKernelGGL(ks_scatter_kernel<DPV>, dim3(G), dim3(64), K * 4, s, codes, A, N, K, D, G, w.hist,  \
                               w.koff, PL, w.planes, sel, n_sel);                                                  \
        else                                                                                                       \
            hipLaunchKernelGGL(ks_transpose_kernel<DPV>, dim3((uint32_t)((N + 1023) / 1024)), dim3(256), 0, s,     \
                               codes, N, D, PL, w.planes);                                                         \
        break;
        QVQ_FOR_EACH_DP(X)
#undef X
    default:
        return hipErrorInvalidValue;
    }
    return hipSuccess;
}

Geo make_geo(const KahanWork &w, uint64_t N, uint32_t K, uint32_t D) {
    Geo g{};
    g.planes = w.planes;
    g.PL = KahanWork::plane_len(N);
    g.koff = w.koff;
    g.segoff = w.segoff;
    g.blkoff = w.blkoff;
    g.K = K;
    g.D = D;
    g.meta = reinterpret_cast<SegMeta *>(w.meta);
    g.bsum = reinterpret_cast<u128 *>(w.bsum);
    g.bfn = reinterpret_cast<Fn *>(w.bfn);
    g.sfn = reinterpret_cast<kahan::SegFn *>(w.sfn);
    g.bfn8 = reinterpret_cast<Fn *>(w.bfn8);
    g.stats = w.stats;
    g.plane_bytes = (uint64_t)w.d_cap * KahanWork::plane_len(w.n_cap);
    g.seg_cap = w.seg_cap;
    g.blk_cap = w.blk_cap;
    return g;
}

// grids sized by the capacities; waves past the actual block count return at once
// (grid-stride kernels: at most 8 workgroups per CU)
uint32_t blk_grid(const KahanWork &w, uint32_t D) {
    return (uint32_t)std::min<uint64_t>(((uint64_t)w.blk_cap * D + WPB - 1) / WPB, 2048);
}
uint32_t chain_grid(uint32_t K, uint32_t D) { return (uint32_t)(((uint64_t)K * D * 64 + 255) / 256); }

}  // namespace

uint64_t kahan_direct_max() {
    static const uint64_t v = std::getenv("QVQ_KAHAN_DIRECT_MAX") ? std::strtoull(std::getenv("QVQ_KAHAN_DIRECT_MAX"), nullptr, 10)
                                                                   : 4096;
    return v;
}

hipError_t launch_kahan_centroids(hipStream_t s, const KahanWork &w, const uint8_t *codes, uint32_t Dp, uint32_t D,
                                  uint64_t N, const uint32_t *A, uint32_t K, double *C, double *split_out,
                                  const uint32_t *sel, uint32_t n_sel, uint64_t max_rows) {
    hipError_t e = kahan_sort(s, w, codes, Dp, D, N, A, K, sel, n_sel);
    if (e != hipSuccess) return e;
    const Geo g = make_geo(w, N, K, D);
    const ByteTab *tab = reinterpret_cast<const ByteTab *>(w.tab);
    if (max_rows && max_rows <= kahan_direct_max()) {
        hipLaunchKernelGGL(ks_direct_kernel, dim3((uint32_t)(((uint64_t)K * D + 255) / 256)), dim3(256), 0, s,
                           w.planes, KahanWork::plane_len(N), w.koff, K, D, tab, C, split_out);
        return hipGetLastError();
    }
    hipLaunchKernelGGL(ks_meta_kernel, dim3(blk_grid(w, D)), dim3(64 * WPB), 0, s, g, tab);
    hipLaunchKernelGGL(ks_bscan_kernel, dim3(chain_grid(K, D)), dim3(256), 0, s, g, (const uint64_t *)nullptr, 0u);
    hipLaunchKernelGGL(ks_build_kernel, dim3(blk_grid(w, D)), dim3(64 * WPB), 0, s, g, tab);
    hipLaunchKernelGGL(ks_eval_kernel, dim3((uint32_t)(((uint64_t)K * D + EPB - 1) / EPB)), dim3(64 * EPB), 0, s, g,
                       tab, C, split_out, (uint64_t *)nullptr, (const uint64_t *)nullptr, 0u);
    return hipGetLastError();
}

hipError_t launch_kahan_chain_local(hipStream_t s, const KahanWork &w, const uint8_t *codes, uint32_t Dp, uint32_t D,
                                    uint64_t N, const uint32_t *A, uint32_t K, const uint32_t *sel, uint32_t n_sel,
                                    uint64_t *gather, uint32_t rank, uint32_t nranks) {
    if (!gather || rank >= nranks) return hipErrorInvalidValue;
    hipError_t e = kahan_sort(s, w, codes, Dp, D, N, A, K, sel, n_sel);
    if (e != hipSuccess) return e;
    const Geo g = make_geo(w, N, K, D);
    hipLaunchKernelGGL(ks_meta_kernel, dim3(blk_grid(w, D)), dim3(64 * WPB), 0, s, g,
                       reinterpret_cast<const ByteTab *>(w.tab));
    hipLaunchKernelGGL(ks_totals_kernel, dim3(chain_grid(K, D)), dim3(256), 0, s, g, gather, rank, nranks);
    return hipGetLastError();
}

hipError_t launch_kahan_chain_build(hipStream_t s, const KahanWork &w, uint32_t D, uint64_t N, uint32_t K,
                                    const uint64_t *gather, uint32_t rank) {
    const Geo g = make_geo(w, N, K, D);
    hipLaunchKernelGGL(ks_bscan_kernel, dim3(chain_grid(K, D)), dim3(256), 0, s, g, gather, rank);
    hipLaunchKernelGGL(ks_build_kernel, dim3(blk_grid(w, D)), dim3(64 * WPB), 0, s, g,
                       reinterpret_cast<const ByteTab *>(w.tab));
    return hipGetLastError();
}

hipError_t launch_kahan_chain_eval(hipStream_t s, const KahanWork &w, uint32_t D, uint64_t N, uint32_t K,
                                   uint64_t *state, const uint64_t *gather, uint32_t rank) {
    if (!state) return hipErrorInvalidValue;
    const Geo g = make_geo(w, N, K, D);
    hipLaunchKernelGGL(ks_eval_kernel, dim3((uint32_t)(((uint64_t)K * D + EPB - 1) / EPB)), dim3(64 * EPB), 0, s, g,
                       reinterpret_cast<const ByteTab *>(w.tab), (double *)nullptr, (double *)nullptr, state, gather,
                       rank);
    return hipGetLastError();
}

hipError_t launch_kahan_chain_finish(hipStream_t s, uint32_t D, uint32_t K, const uint64_t *state,
                                     const uint64_t *gather, uint32_t nranks, double *C, double *split_out) {
    const uint64_t KD = (uint64_t)K * D;
    if (KD == 0) return hipSuccess;
    hipLaunchKernelGGL(ks_finish_kernel, dim3((uint32_t)((KD + 255) / 256)), dim3(256), 0, s, K, D, state, gather,
                       nranks, C, split_out);
    return hipGetLastError();
}

}  // namespace qvq
