// k_wide.hip -- MFMA nearest-code-vector search for every block dimension other than 12
// (src/Quantizer.cpp:24-32 semantics; C4's 4x4 blocks are D = 48).
//
// Scoring as in assign_mfma_kernel (k_assign.hip): per code vector c one f16 row in the wide
// layout (common.hpp) [c''_hi(DH) | c''_lo(DH) | n_hi n_lo | 0 ...] against the data column
// [w(DH) | w(DH) | 1 1 | 0 ...], KS chained v_mfma_f32_16x16x32_f16 per 16 x 16 tile, so
// score = 2^t (||x-c||^2 - ||x-mu||^2).  A wave keeps 64 rows (4 data tiles) as B fragments
// for its whole pass over the codebook, so every A fragment read from LDS feeds 4 MFMAs.
// The codebook sits in LDS whole when it fits; otherwise it streams in 128-code-vector slices
// through two LDS buffers: the next slice's global loads are issued before the current
// slice's MFMAs and written to the other buffer after them, one barrier per slice.
// Epilogue, recompute in direct fp32 and the flag rule follow the D = 12 kernel, except that
// with KS >= 2 (MFMA-bound, VALU to spare) the epilogue keeps the best two 8-code-vector
// units and the third-best score: both units are recomputed, and the MFMA error bound only
// applies against the third unit, so far fewer rows are flagged.
#include <cstdlib>

#include "common.hpp"
#include "mfma_util.hpp"

namespace qvq {

constexpr int WD_THREADS = 512;   // 8 waves, 2 per SIMD: up to 256 VGPRs each
constexpr int WD_WAVES = WD_THREADS / 64;
constexpr int WD_TILES = 4;       // 16-row data tiles per wave
constexpr int WD_ROWS = 16 * WD_TILES;
constexpr uint32_t WD_SLICE = 128;   // code vectors per streamed slice
constexpr uint32_t WD_LDS_MAX = 160 * 1024;

template <int DP>
struct WideCfg {
    static constexpr int DH = (int)wide_dh(DP);
    static constexpr int KS = (int)wide_ks(DP);
    static constexpr int GROW = 64 * KS;     // global row bytes
    static constexpr int LSTR = GROW + 16;   // LDS row stride: the 16 lanes of a k-group read
                                             // 16 consecutive rows at 4 distinct bank quads
    static constexpr int UPR = GROW / 16;    // 16-byte units per row
};

bool wide_can_search(uint32_t Dp) { return Dp >= 4 && Dp <= 64 && Dp % 4 == 0; }

template <int DP>
__host__ __device__ inline bool wide_resident(uint32_t K) {
    return (uint64_t)((K + 31) & ~31u) * WideCfg<DP>::LSTR <= WD_LDS_MAX;
}

// PRUNE (streamed codebooks; code vectors in the order of perm with tile envelopes tint,
// finalize's prune_order): the workgroup's 8 waves take 8 chunks stacked across image rows
// (chunk stride cpr, the chunks per image column of blocks) so that their rows are one compact
// image region; the workgroup searches the slice holding the tile nearest its rows' projection
// first, takes one distance bound from it (every row's best so far, max over the workgroup) and
// then streams only the slices whose tiles the projection bound cannot exclude (DESIGN.md
// 3.1.1: ||x - c||^2 >= sx^2 (sum w - q_c)^2 / D).
__host__ __device__ inline uint64_t wide_chunk(uint64_t task, uint32_t wave, uint64_t ntask, uint32_t cpr) {
    const uint64_t full = ntask / cpr * cpr;   // tasks in whole groups of cpr
    if (task < full) return task / cpr * cpr * WD_WAVES + task % cpr + (uint64_t)wave * cpr;
    return task * WD_WAVES + wave;
}

template <int DP, bool PRUNE>
__global__ __launch_bounds__(WD_THREADS) void assign_wide_kernel(
    const uint8_t *__restrict__ codes, uint64_t N, uint32_t D, const _Float16 *__restrict__ g_rows, uint32_t K,
    const float *__restrict__ g_C32, MfThresholds th, uint32_t *__restrict__ A, uint32_t *__restrict__ flags,
    unsigned *__restrict__ flag_cnt, const uint32_t *__restrict__ g_perm, const int32_t *__restrict__ g_tint,
    uint32_t cpr, unsigned *__restrict__ sched) {
    using C = WideCfg<DP>;
    constexpr int KS = C::KS, LSTR = C::LSTR, UPR = C::UPR, NH = C::DH / 8;
    constexpr bool TWO = KS >= 2;   // keep two units
    extern __shared__ __attribute__((aligned(16))) unsigned char lds[];
    const uint32_t Kp = (K + 31) & ~31u;
    const bool resident = wide_resident<DP>(K);
    const uint32_t SL = resident ? Kp : WD_SLICE;
    const uint32_t ns = (Kp + SL - 1) / SL;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int g = lane >> 4, c = lane & 15;
    const unsigned char *gsrc = reinterpret_cast<const unsigned char *>(g_rows);
    unsigned char *buf0 = lds, *buf1 = lds + (resident ? 0 : WD_SLICE * LSTR);
    // PRUNE: perm (u16 per position) and the tile envelopes after the codebook / slice buffers
    const uint32_t cb_bytes = resident ? Kp * LSTR : 2 * WD_SLICE * LSTR;
    uint16_t *perm_l = reinterpret_cast<uint16_t *>(lds + cb_bytes);
    int32_t *tint_l = reinterpret_cast<int32_t *>(lds + cb_bytes + ((2 * Kp + 15) & ~15u));
    const uint32_t ntiles = Kp / 32;

    // slice s: code vectors s*WD_SLICE.. (KS 16-byte units per thread, staged in registers)
    uint4 stage[KS];
#define WD_STAGE_LOAD(S)                                                                                         \
    _Pragma("unroll") for (int i = 0; i < KS; i++) {                                                            \
        const uint32_t u = tid + i * WD_THREADS, row = (S) * WD_SLICE + u / UPR, col = u % UPR;                  \
        const uint32_t src = PRUNE && row < Kp ? (uint32_t)perm_l[row] : row;                                    \
        stage[i] = row < Kp ? *reinterpret_cast<const uint4 *>(gsrc + (size_t)src * C::GROW + col * 16)          \
                            : make_uint4(0, 0, 0, 0);                                                             \
    }
#define WD_STAGE_STORE(S, BUF)                                                                                   \
    _Pragma("unroll") for (int i = 0; i < KS; i++) {                                                            \
        const uint32_t u = tid + i * WD_THREADS, row = u / UPR, col = u % UPR;                                   \
        if ((S) * WD_SLICE + row < Kp) *reinterpret_cast<uint4 *>((BUF) + row * LSTR + col * 16) = stage[i];      \
    }
    if (PRUNE) {
        for (uint32_t i = tid; i < Kp; i += WD_THREADS) perm_l[i] = (uint16_t)g_perm[i];
        for (uint32_t i = tid; i < 2 * ntiles; i += WD_THREADS) tint_l[i] = g_tint[i];
        __syncthreads();
    }
    if (resident) {   // (PRUNE: in the order of perm)
        for (uint32_t u = tid; u < Kp * UPR; u += WD_THREADS) {
            const uint32_t row = u / UPR, col = u % UPR;
            const uint32_t src = PRUNE ? (uint32_t)perm_l[row] : row;
            *reinterpret_cast<uint4 *>(buf0 + row * LSTR + col * 16) =
                *reinterpret_cast<const uint4 *>(gsrc + (size_t)src * C::GROW + col * 16);
        }
    } else if (!PRUNE) {
        WD_STAGE_LOAD(0u)
        WD_STAGE_STORE(0u, buf0)
    }
    __syncthreads();

    const uint64_t nchunks = (N + WD_ROWS - 1) / WD_ROWS;
    const uint64_t ntask = (nchunks + WD_WAVES - 1) / WD_WAVES;
    const f32x4 zero = {0.f, 0.f, 0.f, 0.f};
    uint32_t it = 0;   // slices consumed (buffer parity)
    __shared__ int32_t red_i[2][WD_WAVES];
    __shared__ float red_f[WD_WAVES];
    __shared__ int32_t win_lo, win_hi;
    // PRUNE: tasks from a counter (sched[0]; the windows differ per task, and a static split left
    // the busiest workgroup ~1.5x the mean), the next one fetched while this one runs
    __shared__ uint32_t sched_next;
    uint64_t task = blockIdx.x;
    if (PRUNE) {
        if (tid == 0) sched_next = atomicAdd(&sched[0], 1u);
        __syncthreads();
        task = sched_next;
    }
    while (task < ntask) {
        const uint64_t chunk = PRUNE ? wide_chunk(task, wave, ntask, cpr) : task * WD_WAVES + wave;
        const uint64_t base = chunk * WD_ROWS;
        const bool more = !PRUNE && task + gridDim.x < ntask;   // uniform over the workgroup
        if (PRUNE) {
            __syncthreads();   // (every thread has read sched_next)
            if (tid == 0) sched_next = atomicAdd(&sched[0], 1u);
        }

        // B fragments: lane (g, c) holds k-slots 32ks + 8g .. +7 of row c of each tile, i.e.
        // 8-slot group G = 4ks + g: hi components 8G.., lo components 8(G-NH).., the two ones
        // of the norm slots, or zeros.
        half8 b[WD_TILES][KS];
#pragma unroll
        for (int t = 0; t < WD_TILES; t++) {
            const uint64_t row = base + t * 16 + c;
            const bool valid = chunk < nchunks && row < N;
            const uint8_t *rp = codes + row * DP;
#pragma unroll
            for (int ks = 0; ks < KS; ks++) {
                const int G = 4 * ks + g;
                half8 h = {0, 0, 0, 0, 0, 0, 0, 0};
                if (G < 2 * NH) {
                    if (valid) {
                        const int m = G < NH ? G : G - NH;
                        const uint32_t w0 = *reinterpret_cast<const uint32_t *>(rp + 8 * m);
                        const uint32_t w1 = 8 * m + 4 < DP ? *reinterpret_cast<const uint32_t *>(rp + 8 * m + 4) : 0u;
#pragma unroll
                        for (int j = 0; j < 4; j++) {
                            h[j] = (_Float16)byte_w(w0, j);
                            h[4 + j] = (_Float16)byte_w(w1, j);
                        }
                    }
                } else if (G == 2 * NH) {
                    h[0] = (_Float16)1.f;
                    h[1] = (_Float16)1.f;
                }
                b[t][ks] = h;
            }
        }
        float b1[WD_TILES], b2[WD_TILES], b3[WD_TILES];
        uint32_t bp[WD_TILES], bq[WD_TILES];
#pragma unroll
        for (int t = 0; t < WD_TILES; t++) {
            b1[t] = INFINITY;
            b2[t] = INFINITY;
            b3[t] = INFINITY;
            bp[t] = 0;
            bq[t] = 0;
        }
        // one streamed or resident slice of code vectors (positions r0 .. r0 + np*32) against the
        // wave's 64 rows
        auto search_slice = [&](const unsigned char *cur, uint32_t r0, uint32_t np) {
            const unsigned char *abase = cur + c * LSTR + 16 * g;
#pragma unroll 2
            for (uint32_t p = 0; p < np; p++) {
                half8 a0[KS], a1[KS];
#pragma unroll
                for (int ks = 0; ks < KS; ks++) {
                    a0[ks] = *reinterpret_cast<const half8 *>(abase + (size_t)(32 * p) * LSTR + 64 * ks);
                    a1[ks] = *reinterpret_cast<const half8 *>(abase + (size_t)(32 * p + 16) * LSTR + 64 * ks);
                }
                f32x4 p0[WD_TILES], p1[WD_TILES];
#pragma unroll
                for (int t = 0; t < WD_TILES; t++) {
                    p0[t] = __builtin_amdgcn_mfma_f32_16x16x32_f16(a0[0], b[t][0], zero, 0, 0, 0);
                    p1[t] = __builtin_amdgcn_mfma_f32_16x16x32_f16(a1[0], b[t][0], zero, 0, 0, 0);
                }
#pragma unroll
                for (int ks = 1; ks < KS; ks++)
#pragma unroll
                    for (int t = 0; t < WD_TILES; t++) {
                        p0[t] = __builtin_amdgcn_mfma_f32_16x16x32_f16(a0[ks], b[t][ks], p0[t], 0, 0, 0);
                        p1[t] = __builtin_amdgcn_mfma_f32_16x16x32_f16(a1[ks], b[t][ks], p1[t], 0, 0, 0);
                    }
#pragma unroll
                for (int t = 0; t < WD_TILES; t++) {
                    if (TWO)
                        pair_update2(p0[t], p1[t], r0 / 32 + p, b1[t], b2[t], b3[t], bp[t], bq[t]);
                    else
                        pair_update(p0[t], p1[t], r0 / 32 + p, b1[t], b2[t], bp[t]);
                }
            }
        };
        if constexpr (PRUNE) {
            // the rows' sum w (exact integers) and ||x - mu||^2: lane (g, c) takes row c of each tile
            int32_t qmn = 0x7FFFFFFF, qmx = (int32_t)0x80000000;
            float xn2[WD_TILES];
            const float sx2 = th.sx * th.sx;
#pragma unroll
            for (int t = 0; t < WD_TILES; t++) {
                const uint64_t row = base + t * 16 + c;
                const bool valid = chunk < nchunks && row < N;
                const uint32_t *rw = reinterpret_cast<const uint32_t *>(codes + (valid ? row : 0) * DP);
                uint32_t su = 0, s2 = 0;
#pragma unroll
                for (int q = 0; q < DP / 4; q++) {
                    uint32_t u = rw[q] ^ 0x80808080u;
                    const int rem = (int)D - 4 * q;   // real components in this word
                    u = rem >= 4 ? u : (rem <= 0 ? 0u : u & (0xFFFFFFFFu >> (8 * (4 - rem))));
                    su = __builtin_amdgcn_sad_u8(u, 0u, su);
                    s2 = __builtin_amdgcn_udot4(u, u, s2, false);
                }
                const int32_t qw = 2 * (int32_t)su - 255 * (int32_t)D;   // sum_d (2u - 255)
                xn2[t] = valid ? (float)(4.0 * (double)s2 - 1020.0 * (double)su + 65025.0 * (double)D) * sx2 : 0.f;
                qmn = valid ? min(qmn, qw) : qmn;
                qmx = valid ? max(qmx, qw) : qmx;
            }
            qmn = (int32_t)(wave_min_u32((uint32_t)qmn ^ 0x80000000u) ^ 0x80000000u);
            qmx = (int32_t)(~wave_min_u32(~((uint32_t)qmx ^ 0x80000000u)) ^ 0x80000000u);
            // the row's best distance so far from above: its best MFMA score over the four lane
            // groups plus the score error, max over the wave's rows
            auto wave_bound = [&]() {
                float ub = 0.f;
#pragma unroll
                for (int t = 0; t < WD_TILES; t++) {
                    float v = __fmaf_rn(b1[t], th.inv_scale, xn2[t]) + th.mfma;
                    v = fminf(v, xor16_f32(v));
                    v = fminf(v, xor32_f32(v));
                    const uint64_t row = base + t * 16 + c;
                    ub = chunk < nchunks && row < N ? fmaxf(ub, v) : ub;
                }
                return __uint_as_float(~wave_min_u32(~__float_as_uint(fmaxf(ub, 0.f))));   // >= 0: bits order as values
            };
            if (resident) {   // the whole codebook in LDS: every wave its own window, no barriers
                const int32_t tlo = lane < (int)ntiles ? tint_l[2 * lane] : 0x7FFFFFFF;
                const int32_t thi = lane < (int)ntiles ? tint_l[2 * lane + 1] : (int32_t)0x80000000;
                if (qmn <= qmx) {
                    const int32_t mid = (int32_t)(((int64_t)qmn + qmx) >> 1);
                    const uint32_t t0 = min((uint32_t)__popcll(__ballot(lane < (int)ntiles && thi < mid)), ntiles - 1);
                    search_slice(buf0 + (size_t)t0 * 32 * LSTR, t0 * 32, 1);
                    const float bw = wave_bound() * ((float)D / sx2) * 1.00001f + 1.0f;
                    const float gap = (float)max(0, max(tlo - qmx, qmn - thi));
                    const uint64_t win = __ballot(lane < (int)ntiles && gap * gap <= bw);
                    const uint32_t lo = min(t0, win ? (uint32_t)(__ffsll((unsigned long long)win) - 1) : t0);
                    const uint32_t hi = max(t0, win ? (uint32_t)(63 - __clzll((long long)win)) : t0);
                    if (t0 > lo) search_slice(buf0 + (size_t)lo * 32 * LSTR, lo * 32, t0 - lo);
                    if (hi > t0) search_slice(buf0 + (size_t)(t0 + 1) * 32 * LSTR, (t0 + 1) * 32, hi - t0);
                }
            } else {
            if (lane == 0) {
                red_i[0][wave] = qmn;
                red_i[1][wave] = qmx;
            }
            __syncthreads();
            int32_t Qmn = red_i[0][0], Qmx = red_i[1][0];
#pragma unroll
            for (int w = 1; w < WD_WAVES; w++) {
                Qmn = min(Qmn, red_i[0][w]);
                Qmx = max(Qmx, red_i[1][w]);
            }
            if (Qmn <= Qmx) {   // (uniform) the workgroup has rows
                // the tile whose envelope reaches the rows' centre, and its slice first
                const int32_t mid = (int32_t)(((int64_t)Qmn + Qmx) >> 1);
                const uint32_t below = __syncthreads_count(tid < ntiles && tint_l[2 * tid + 1] < mid);
                const uint32_t t0 = min(below, ntiles - 1), s0 = t0 * 32 / WD_SLICE;
                auto stage_now = [&](uint32_t sl, unsigned char *dst) {
                    WD_STAGE_LOAD(sl)
                    WD_STAGE_STORE(sl, dst)
                };
                stage_now(s0, buf0);
                __syncthreads();
                search_slice(buf0, s0 * WD_SLICE, min(WD_SLICE, Kp - s0 * WD_SLICE) / 32);
                // one bound: every row's best distance so far from above (its best MFMA score over
                // the four lane groups, plus the score error), max over the workgroup
                const float ub = wave_bound();
                if (tid == 0) {
                    win_lo = 0x7FFFFFFF;
                    win_hi = -1;
                }
                if (lane == 0) red_f[wave] = ub;
                __syncthreads();
                float B = red_f[0];
#pragma unroll
                for (int w = 1; w < WD_WAVES; w++) B = fmaxf(B, red_f[w]);
                const float bw = B * ((float)D / sx2) * 1.00001f + 1.0f;
                if (tid < ntiles) {   // the tiles' gaps grow away from the centre: one range
                    const float gap = (float)max(0, max(tint_l[2 * tid] - Qmx, Qmn - tint_l[2 * tid + 1]));
                    if (gap * gap <= bw) {
                        atomicMin(&win_lo, (int32_t)tid);
                        atomicMax(&win_hi, (int32_t)tid);
                    }
                }
                __syncthreads();
                const uint32_t slo = min(s0, (uint32_t)(win_lo == 0x7FFFFFFF ? t0 : win_lo) * 32 / WD_SLICE);
                const uint32_t shi = max(s0, (uint32_t)(win_hi < 0 ? t0 : win_hi) * 32 / WD_SLICE);
                // the window's other slices, the next one staged under each one's MFMAs
                uint32_t sl = slo == s0 ? s0 + 1 : slo;
                if (sl <= shi) {
                    stage_now(sl, buf1);
                    __syncthreads();
                    uint32_t par = 1;
                    for (;;) {
                        const uint32_t nx = sl + 1 == s0 ? sl + 2 : sl + 1;
                        const bool pre = nx <= shi;
                        if (pre) {
                            WD_STAGE_LOAD(nx)
                        }
                        search_slice(par ? buf1 : buf0, sl * WD_SLICE, min(WD_SLICE, Kp - sl * WD_SLICE) / 32);
                        if (!pre) break;
                        WD_STAGE_STORE(nx, par ? buf0 : buf1)
                        __syncthreads();
                        par ^= 1;
                        sl = nx;
                    }
                }
                __syncthreads();   // (the buffers are free for the next task)
            }
            }   // (streamed)
        } else {
            for (uint32_t s = 0; s < ns; s++) {
                const unsigned char *cur = (it & 1) ? buf1 : buf0;
                const bool pre = !resident && (s + 1 < ns || more);
                const uint32_t snext = s + 1 < ns ? s + 1 : 0;
                if (pre) {
                    WD_STAGE_LOAD(snext)
                }
                const uint32_t r0 = resident ? 0 : s * WD_SLICE;
                const uint32_t np = min(SL, Kp - r0) / 32;
                search_slice(cur, r0, np);
                if (!resident) {
                    if (pre) {
                        unsigned char *nb = (it & 1) ? buf0 : buf1;
                        WD_STAGE_STORE(snext, nb)
                    }
                    __syncthreads();
                    it++;
                }
            }

        }

        // Combine the four lanes of each data row.  One unit: the winning 8-code-vector unit
        // (pair*4 + g) and the best MFMA score among all other units.  Two units: the best two
        // units (ordered by score, then unit) and the best score among all other units.  A
        // reduce-scatter on the VALU as in assign_mfma_kernel: v_permlane32_swap merges tiles
        // t and t + 2 across lane ^ 32, v_permlane16_swap the survivors across lane ^ 16, and
        // lane (g, c) keeps tile g, row c (its own row).  Both merges are order-free.
        struct St {
            float b1, b2, b3;
            uint32_t u, v;
        };
        auto lt = [](float x, uint32_t xu, float y, uint32_t yu) { return x < y || (x == y && xu < yu); };
        auto merge = [&](St &m, const St &o) {
            if (!TWO) {
                if (lt(o.b1, o.u, m.b1, m.u)) {
                    m.b2 = min2f(o.b2, m.b1);
                    m.b1 = o.b1;
                    m.u = o.u;
                } else {
                    m.b2 = min2f(m.b2, o.b1);
                }
                return;
            }
            // merge (b1,u) <= (b2,v) with (o1,ou) <= (o2,ov); thirds b3, o3
            float n1, n2, n3;
            uint32_t m1, m2;
            if (lt(o.b1, o.u, m.b1, m.u)) {   // partner's best first; then (b1,u) vs (o2,ov)
                n1 = o.b1;
                m1 = o.u;
                const bool mine = lt(m.b1, m.u, o.b2, o.v);
                n2 = mine ? m.b1 : o.b2;
                m2 = mine ? m.u : o.v;
                n3 = min3f(mine ? o.b2 : m.b1, m.b2, min2f(m.b3, o.b3));
            } else {
                n1 = m.b1;
                m1 = m.u;
                const bool mine = lt(m.b2, m.v, o.b1, o.u);
                n2 = mine ? m.b2 : o.b1;
                m2 = mine ? m.v : o.u;
                n3 = min3f(mine ? o.b1 : m.b2, o.b2, min2f(m.b3, o.b3));
            }
            m = {n1, n2, n3, m1, m2};
        };
        // lo / hi of a swap of every field (x: state of the lower tile, y: of the upper)
        auto swap_st = [&](const St &x, const St &y, bool by32, St &lo, St &hi) {
            auto sf = [&](float a, float b, float &l, float &h) {
                const LanePairF r = by32 ? swap32_f32(a, b) : swap16_f32(a, b);
                l = r.lo;
                h = r.hi;
            };
            auto su = [&](uint32_t a, uint32_t b, uint32_t &l, uint32_t &h) {
                const LanePair r = by32 ? swap32_u32(a, b) : swap16_u32(a, b);
                l = r.lo;
                h = r.hi;
            };
            sf(x.b1, y.b1, lo.b1, hi.b1);
            sf(x.b2, y.b2, lo.b2, hi.b2);
            su(x.u, y.u, lo.u, hi.u);
            if (TWO) {
                sf(x.b3, y.b3, lo.b3, hi.b3);
                su(x.v, y.v, lo.v, hi.v);
            } else {
                lo.b3 = hi.b3 = INFINITY;
                lo.v = hi.v = 0;
            }
        };
        St h[2];
#pragma unroll
        for (int t = 0; t < 2; t++) {   // lanes < 32 end with tile t, lanes >= 32 with tile t + 2
            const St x = {b1[t], b2[t], TWO ? b3[t] : INFINITY, bp[t] * 4 + g, TWO ? bq[t] * 4 + g : 0u};
            const St y = {b1[t + 2], b2[t + 2], TWO ? b3[t + 2] : INFINITY, bp[t + 2] * 4 + g,
                          TWO ? bq[t + 2] * 4 + g : 0u};
            St o;
            swap_st(x, y, true, h[t], o);
            merge(h[t], o);
        }
        St fin, o;   // even rows keep h[0] (tile 0 or 2), odd rows h[1] (tile 1 or 3): tile g
        swap_st(h[0], h[1], false, fin, o);
        merge(fin, o);
        const uint32_t unit = fin.u, unit2 = fin.v;
        const float sec_m = TWO ? fin.b3 : fin.b2;
        // Lane L owns row base + L: direct fp32 (x - c)^2 over the 8 code vectors of its unit.
        const uint64_t row = base + lane;
        if (chunk < nchunks && row < N) {
            float x[DP];
            float xn = 0.f;   // ||x - mu||^2 over the D real components
            const uint32_t *rw = reinterpret_cast<const uint32_t *>(codes + row * DP);
#pragma unroll
            for (int q = 0; q < DP / 4; q++) {
                const uint32_t word = rw[q];
#pragma unroll
                for (int j = 0; j < 4; j++) {
                    const int d = 4 * q + j;
                    const float e = byte_w(word, j) * th.sx;
                    const bool real = (uint32_t)d < D;
                    xn = real ? __fmaf_rn(e, e, xn) : xn;
                    x[d] = real ? e + th.mu : 0.f;   // C32 holds 0 in the padding components
                }
            }
            float r1 = INFINITY, r2 = INFINITY;
            uint32_t rk = 0;
#pragma unroll 2
            for (int j = 0; j < (TWO ? 16 : 8); j++) {
                const uint32_t un = j < 8 ? unit : unit2, jj = j & 7;
                const uint32_t pos = (2 * (un >> 2) + (jj >> 2)) * 16 + 4 * (un & 3) + (jj & 3);
                const uint32_t cv = PRUNE ? (uint32_t)perm_l[pos] : pos;   // the code vector at that position
                const float4 *c4 = reinterpret_cast<const float4 *>(g_C32 + (size_t)cv * DP);
                float dist = 0.f;
#pragma unroll
                for (int q = 0; q < DP / 4; q++) {
                    const float4 cq = c4[q];
                    float e;
                    e = x[4 * q + 0] - cq.x; dist = __fmaf_rn(e, e, dist);
                    e = x[4 * q + 1] - cq.y; dist = __fmaf_rn(e, e, dist);
                    e = x[4 * q + 2] - cq.z; dist = __fmaf_rn(e, e, dist);
                    e = x[4 * q + 3] - cq.w; dist = __fmaf_rn(e, e, dist);
                }
                dist = cv < K ? dist : INFINITY;   // padding code vectors never win
                r2 = med3f(r1, r2, dist);
                rk = dist < r1 ? cv : rk;
                r1 = min2f(r1, dist);
            }
            // best unit not recomputed; from an MFMA score it can be slightly negative (a row on a
            // code vector): clamped, so no NaN reaches the -fno-honor-nans compares (r1 >= 0
            // flags such a row anyway)
            const float rest = fmaxf(__fmaf_rn(sec_m, th.inv_scale, xn), 0.f);
            bool flag;
            if (TWO) {   // recomputed runner-up (direct fp32 error), rest (plus the MFMA error)
                const float thr2 = 2.f * (th.alpha * sqrtf(r2) + th.beta * r2) + th.gamma;
                const float thr3 = th.mfma + 2.f * (th.alpha * sqrtf(rest) + th.beta * rest) + th.gamma;
                flag = !(r2 - r1 > thr2) || !(rest - r1 > thr3);
            } else {
                const float sec = min2f(rest, r2);
                const float thr = th.mfma + 2.f * (th.alpha * sqrtf(sec) + th.beta * sec) + th.gamma;
                flag = !(sec - r1 > thr);
            }
            A[row] = rk;
            if (flag) flags[atomicAdd(flag_cnt, 1u)] = (uint32_t)row;
        }
        if (PRUNE) {
            __syncthreads();
            task = sched_next;
        } else {
            task += gridDim.x;
        }
    }
    if (PRUNE && tid == 0) {   // the last workgroup out resets the counters for the next launch
        __threadfence();
        if (atomicAdd(&sched[1], 1u) == gridDim.x - 1) {
            sched[0] = 0;
            sched[1] = 0;
        }
    }
}

#undef WD_STAGE_LOAD
#undef WD_STAGE_STORE

template <int DP>
static size_t wide_prune_lds(uint32_t K) {
    const uint32_t Kp = (K + 31) & ~31u;
    const size_t cb = wide_resident<DP>(K) ? (size_t)Kp * WideCfg<DP>::LSTR : 2 * (size_t)WD_SLICE * WideCfg<DP>::LSTR;
    return cb + ((2 * Kp + 15) & ~15u) + 8 * (size_t)(Kp / 32);
}
template <int DP>
static bool wide_prune_fits_dp(uint32_t K) {   // (resident: one envelope per lane, <= 64 tiles)
    const uint32_t Kp = (K + 31) & ~31u;
    return K <= 65536 && wide_prune_lds<DP>(K) <= WD_LDS_MAX && (!wide_resident<DP>(K) || Kp / 32 <= 64);
}

template <int DP>
static hipError_t launch_wide_dp(hipStream_t s, int num_cu, uint32_t D, const uint8_t *codes, uint64_t N,
                                 const _Float16 *cb_rows, uint32_t K, const float *C32, const MfThresholds &th,
                                 uint32_t *A, uint32_t *flags, unsigned *flag_cnt, const uint32_t *perm,
                                 const int32_t *tint, uint32_t cpr, unsigned *sched) {
    using C = WideCfg<DP>;
    const uint32_t Kp = (K + 31) & ~31u;
    const bool prune = perm && tint && sched;
    if (prune && !wide_prune_fits_dp<DP>(K)) return hipErrorInvalidValue;
    const size_t lds = prune ? wide_prune_lds<DP>(K)
                             : (wide_resident<DP>(K) ? (size_t)Kp * C::LSTR : 2 * (size_t)WD_SLICE * C::LSTR);
    const uint64_t nchunks = (N + WD_ROWS - 1) / WD_ROWS;
    const int grid = (int)std::max<uint64_t>(1, std::min<uint64_t>((nchunks + WD_WAVES - 1) / WD_WAVES, num_cu));
    if (prune)
        hipLaunchKernelGGL((assign_wide_kernel<DP, true>), dim3(grid), dim3(WD_THREADS), lds, s, codes, N, D, cb_rows, K,
                           C32, th, A, flags, flag_cnt, perm, tint, std::max(1u, cpr), sched);
    else
        hipLaunchKernelGGL((assign_wide_kernel<DP, false>), dim3(grid), dim3(WD_THREADS), lds, s, codes, N, D, cb_rows,
                           K, C32, th, A, flags, flag_cnt, nullptr, nullptr, 1u, nullptr);
    return hipGetLastError();
}

bool wide_codebook_resident(uint32_t Dp, uint32_t K) {
    switch (Dp) {
#define X(DPV) \
    case DPV: return wide_resident<DPV>(K);
        X(4) X(8) X(12) X(16) X(20) X(24) X(28) X(32) X(36) X(40) X(44) X(48) X(52) X(56) X(60) X(64)
#undef X
    }
    return false;
}

bool wide_prune_fits(uint32_t Dp, uint32_t K) {
    switch (Dp) {
#define X(DPV) \
    case DPV: return wide_prune_fits_dp<DPV>(K);
        X(4) X(8) X(12) X(16) X(20) X(24) X(28) X(32) X(36) X(40) X(44) X(48) X(52) X(56) X(60) X(64)
#undef X
    }
    return false;
}

hipError_t launch_assign_wide(hipStream_t s, int num_cu, uint32_t Dp, uint32_t D, const uint8_t *codes, uint64_t N,
                              const _Float16 *cb_rows, uint32_t K, const float *C32, const MfThresholds &th,
                              uint32_t *A, uint32_t *flags, unsigned *flag_cnt, const uint32_t *perm,
                              const int32_t *tint, uint32_t cpr, unsigned *sched) {
    if (K == 0 || !wide_can_search(Dp) || D > Dp || D + 4 <= Dp) return hipErrorInvalidValue;
    switch (Dp) {
#define X(DPV) \
    case DPV: return launch_wide_dp<DPV>(s, num_cu, D, codes, N, cb_rows, K, C32, th, A, flags, flag_cnt, perm, tint, cpr, \
                                         sched);
        X(4) X(8) X(12) X(16) X(20) X(24) X(28) X(32) X(36) X(40) X(44) X(48) X(52) X(56) X(60) X(64)
#undef X
    }
    return hipErrorInvalidValue;
}

}  // namespace qvq
