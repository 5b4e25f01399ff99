// k_mf32.hip -- D = 12 nearest-code-vector search on v_mfma_f32_32x32x16_f16
// (src/Quantizer.cpp:24-32 semantics; nanoflann's exact answer via the recheck).
//
// Same scores as assign_mfma_kernel (k_assign.hip): score = 2^t (||x-c||^2 - ||x-mu||^2) from
// f16 hi/lo code-vector terms against the exact centred byte integers w of the data row, but
// on 32 x 32 tiles: one (code tile, data tile) pair is two chained 32x32x16 MFMAs
//   MFMA 1, k-slots 0..15: A = [hi(0..7) | lo(0..7)]          B = [w(0..7) | w(0..7)]
//   MFMA 2, k-slots 0..15: A = [hi(8..11) n_hi n_lo 0 0 | lo(8..11) * * * *]
//                          B = [w(8..11) 1 1 0 0 | w(8..11) 0 0 0 0]
// (the '*' slots meet zeros in B: any finite f16 does).  Per 1024 scores that is half the
// MFMA instructions of the 16x16x32 form, so half the vector-issue cycles the matrix pipe
// holds (MI355X_MICROARCH.md, 'vector-instruction ISSUE cost': 8 per MFMA either shape), and
// a lane's 16 results all belong to one data row, so its epilogue covers 8-code-vector units
// (two per tile) or 4-code-vector units (four per tile) without lane traffic.
//
// LDS image of the codebook (staged from the 56-byte rows of common.hpp):
//   P [Kp][32 B]  [hi(0..7) | lo(0..7)], the two 16-byte halves swapped when bit 3 of the
//                 code vector's index is set: the ds_read_b128 lane groups {0-3,12-15,20-27}
//                 and {4-11,16-19,28-31} then cover the 64 banks once (MI355X_MICROARCH.md, LDS)
//   Q [Kp][24 B]  [lo(8..11) | hi(8..11) | n_hi n_lo 0 0]: half h = 0 reads bytes 8..23,
//                 h = 1 bytes 0..15 (two ds_read_b64: a 24-byte stride is bank-conflict free)
// The rest (fp32 recompute of the winning unit, rigorous near-tie flag, fused exact centroid
// sums) follows assign_mfma_kernel.
#include <cstdlib>

#include "common.hpp"
#include "mfma_util.hpp"
#include "kd_walk.hpp"   // RowN, load_row, ref_l2_n

namespace qvq {

typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef uint32_t u32x4v __attribute__((ext_vector_type(4)));
typedef uint64_t u64x2v __attribute__((ext_vector_type(2)));

constexpr int M32_THREADS = 1024;   // 16 waves, 4 per SIMD, one workgroup per CU
constexpr int M32_WAVES = M32_THREADS / 64;
constexpr int M32_ROWS = 64;        // rows per wave and chunk: two 32-row data tiles
constexpr uint32_t M32_LDS_MAX = 160 * 1024;

struct M32Lds {
    uint32_t q, c32, sums, cnt, perm, plut, total;
};
// Sums copies (fused, copies > 1): strides one u64 / u32 past K * D / K, so the copies of one
// (component, code vector) fall on different LDS banks (a 256-byte multiple put them all on
// one: K = 256 / 512 showed 3x the bank-conflict cycles of the other levels)
// component rows of the LDS sums [d][k] are K + 1 apart (QVQ_SUMS_KPAD builds: A/B)
#ifndef QVQ_SUMS_KPAD
#define QVQ_SUMS_KPAD 1
#endif
__host__ __device__ inline uint32_t m32_kstride(uint32_t K) { return K + QVQ_SUMS_KPAD; }
__host__ __device__ inline uint32_t m32_sum_stride(uint32_t K, uint32_t copies) { return m32_kstride(K) * MF_D + (copies > 1 ? 1 : 0); }
__host__ __device__ inline uint32_t m32_cnt_stride(uint32_t K, uint32_t copies) { return K + (copies > 1 ? 1 : 0); }
__host__ __device__ inline M32Lds m32_lds_layout(uint32_t K, bool fuse, bool staged, uint32_t copies = 1,
                                                  bool prune = false) {
    const uint32_t Kp = (K + 31) & ~31u;
    M32Lds L;
    // fused: the byte LUT first (LDS address 0: a lookup's address is the byte itself, no
    // base add per byte), the code-vector rows after it (ROWS0 in the kernel)
    uint32_t o = fuse ? 256 : 0;
    o += Kp * 32;
    L.q = o;
    o += Kp * 24;
    L.c32 = o;
    if (staged) o += Kp * MF_D * 4;
    L.sums = o;
    if (fuse) o += copies * m32_sum_stride(K, copies) * 8;
    L.cnt = o;
    if (fuse) o += copies * ((m32_cnt_stride(K, copies) + 1) & ~1u) * 4;
    L.perm = o;   // pruned searches: the code vector at each tile position (u16)
    if (prune) o += ((Kp * 2 + 7) & ~7u);
    L.plut = 0;
    L.total = o;
    return L;
}

// Per-run sums over consecutive lanes with equal key (as in k_assign.hip): returns true on the
// last lane of each run, which then holds the run's sums.
__device__ inline bool m32_runs_reduce(uint32_t key, uint32_t (&v)[MF_D + 1], int lane) {
    const uint32_t prev = wave_prev_u32(key);
    const uint32_t next = wave_next_u32(key);
    const bool head = lane == 0 || prev != key;
    const uint32_t h = wave_scan_max(head ? (uint32_t)lane : 0u);
    const int src = h == 0 ? 0 : (int)h - 1;
#pragma unroll
    for (int i = 0; i <= MF_D; i++) {
        const uint32_t pre = wave_scan_add(v[i]);
        const uint32_t before = __shfl(pre, src);
        v[i] = pre - (h == 0 ? 0u : before);
    }
    return lane == 63 || next != key;
}

// P / Q (LDS, layout above) from the 56-byte rows [hi0..3 lo0..3 | hi4..7 lo4..7 | hi8..11
// lo8..11 | n] of Kp code vectors.
__device__ inline void m32_stage_pq(unsigned char *lds, uint32_t qoff, const _Float16 *g_rows, uint32_t Kp, int tid,
                                    uint32_t rows0 = 0, const uint32_t *perm = nullptr) {
    const uint64_t *src = reinterpret_cast<const uint64_t *>(g_rows);
    for (uint32_t i = tid; i < Kp; i += M32_THREADS) {
        const uint64_t *r = src + (size_t)(perm ? perm[i] : i) * 7;   // position i holds code vector perm[i]
        const uint64_t w0 = r[0], w1 = r[1], w2 = r[2], w3 = r[3], w4 = r[4], w5 = r[5], w6 = r[6];
        const bool sw = (i >> 3) & 1;
        u64x2v *p = reinterpret_cast<u64x2v *>(lds + rows0 + (size_t)i * 32);
        const u64x2v hi = {w0, w2}, lo = {w1, w3};
        p[0] = sw ? lo : hi;
        p[1] = sw ? hi : lo;
        uint64_t *q = reinterpret_cast<uint64_t *>(lds + qoff + (size_t)i * 24);
        q[0] = w5;
        q[1] = w4;
        q[2] = w6;
    }
}

// Running best unit / best score / second-best unit minimum of one lane and data tile.
__device__ inline void m32_track(float m, uint32_t u, float &b1, float &b2, uint32_t &bu) {
    b2 = med3f(b1, b2, m);
    bu = m < b1 ? u : bu;
    b1 = min2f(b1, m);
}
// The same with the unit index u in the low `idbits` mantissa bits of the unit minimum
// (v_and_or_b32): tracking is min + med3, and b1's low bits name its unit.  A tagged value
// differs from the score by < 2^idbits ulps, i.e. relatively by < 2^(idbits - 23); the flag
// threshold carries that (orrel, below).
__device__ inline void m32_track_tagged(float m, uint32_t keep, uint32_t u, float &b1, float &b2) {
    // one v_and_or_b32 (the compiler splits (m & keep) | u into and + or); m comes from VALU
    // min3s, never straight from an MFMA, so no hazard hides inside the asm
    uint32_t r;
    asm("v_and_or_b32 %0, %1, %2, %3" : "=v"(r) : "v"(__float_as_uint(m)), "v"(keep), "s"(u));
    const float t = __uint_as_float(r);
    b2 = med3f(b1, b2, t);
    b1 = min2f(b1, t);
}

// TAG: unit indices in the scores' low bits (idbits of them, idbits >= log2 of the units per
// lane; orrel = 2^(idbits - 22) bounds twice the relative change).
// copies > 1 (fused): every row adds its terms straight into LDS copy lane % copies of the
// sums (runs of equal indices then meet copies instead of one address); copies = 1: the
// wave run reduction first, then one atomic set per run.
// PRUNE (tiles in the order of perm, tint: finalize's prune_order): a chunk visits its code
// tiles outward from the one nearest its rows' projection and stops once the tiles left on both
// sides are provably farther than every row's current best (see the tile loop).
template <bool FUSE, bool STAGED, int U, bool TAG, bool PRUNE>
__global__ __launch_bounds__(M32_THREADS) void assign_mf32_kernel(
    const uint8_t *__restrict__ codes, uint64_t N, const _Float16 *__restrict__ g_rows, uint32_t K,
    const float *__restrict__ g_C32, const uint64_t *__restrict__ g_plut, MfThresholds th, uint32_t idbits,
    float orrel, uint32_t *__restrict__ A, uint32_t *__restrict__ flags, unsigned *__restrict__ flag_cnt,
    uint64_t *__restrict__ part, uint32_t *__restrict__ part_cnt, uint32_t copies,
    const uint32_t *__restrict__ g_perm, const int32_t *__restrict__ g_tint, uint64_t *__restrict__ z1,
    uint32_t nz1) {
    static_assert(U == 4 || U == 8, "unit of 4 or 8 code vectors");
    constexpr int NU = 16 / U;   // units per lane and code tile
    extern __shared__ __attribute__((aligned(16))) unsigned char lds[];
    const uint32_t Kp = (K + 31) & ~31u;
    const M32Lds L = m32_lds_layout(K, FUSE, STAGED, copies, PRUNE);
    uint16_t *perm_l = reinterpret_cast<uint16_t *>(lds + L.perm);
    float *c32s = reinterpret_cast<float *>(lds + L.c32);
    uint64_t *sums = reinterpret_cast<uint64_t *>(lds + L.sums);   // [d][k]
    uint32_t *cnt = reinterpret_cast<uint32_t *>(lds + L.cnt);
    uint8_t *lo8 = lds + L.plut;   // low part of each byte's exact term (high part: b ^ 0x80)
    // The same table addressed as LDS byte 0 (the kernel has no static LDS, so the dynamic
    // block starts there): lookups take the byte as their address.
    const __attribute__((address_space(3))) uint8_t *lo8_at0 =
        (const __attribute__((address_space(3))) uint8_t *)(uintptr_t)0;
    constexpr uint32_t ROWS0 = FUSE ? 256 : 0;   // m32_lds_layout
    const int tid = threadIdx.x;
    const int lane = tid & 63, wave = tid >> 6;
    const int r32 = lane & 31, h = lane >> 5;
    const uint64_t nchunks = (N + M32_ROWS - 1) / M32_ROWS;
    // lane (r32, h) loads row r32 of both data tiles (the words of data tile T in q[3T..3T+2]);
    // its own row base + lane is the one of tile h.  Branch-free: rows past N read row N - 1.
    auto load_codes = [&](uint64_t chunk, uint32_t (&q)[6]) {
#pragma unroll
        for (int T = 0; T < 2; T++) {
            uint64_t row = chunk * M32_ROWS + 32 * T + r32;
            row = row < N ? row : N - 1;
            const uint32_t *p = reinterpret_cast<const uint32_t *>(codes + row * MF_D);
            q[3 * T] = p[0];
            q[3 * T + 1] = p[1];
            q[3 * T + 2] = p[2];
        }
    };
    uint64_t chunk = (uint64_t)blockIdx.x * M32_WAVES + wave;
    const uint64_t stride = (uint64_t)gridDim.x * M32_WAVES;
    uint32_t qn[6];
    load_codes(chunk, qn);   // the first chunk's rows go out before the LDS staging, under its latency
    m32_stage_pq(lds, L.q, g_rows, Kp, tid, ROWS0, PRUNE ? g_perm : nullptr);
    if (PRUNE)
        for (uint32_t i = tid; i < Kp; i += M32_THREADS) perm_l[i] = (uint16_t)g_perm[i];
    if (STAGED) {
        const float4 *src = reinterpret_cast<const float4 *>(g_C32);
        float4 *dst = reinterpret_cast<float4 *>(c32s);
        for (uint32_t i = tid; i < Kp * (MF_D / 4); i += M32_THREADS) dst[i] = src[i];
    }
    if (FUSE) {
        for (uint32_t i = tid; i < copies * m32_sum_stride(K, copies); i += M32_THREADS) sums[i] = 0;
        for (uint32_t i = tid; i < copies * m32_cnt_stride(K, copies); i += M32_THREADS) cnt[i] = 0;
        if (tid < 256) lo8[tid] = (uint8_t)(g_plut[tid] & 0xFF);
        if (blockIdx.x == 0) {   // the correction slabs G (+) and G + 1 (-), after all G others
            for (uint32_t i = tid; i < 2 * K * MF_D; i += M32_THREADS) part[(uint64_t)gridDim.x * K * MF_D + i] = 0;
            for (uint32_t i = tid; i < 2 * K; i += M32_THREADS) part_cnt[(uint64_t)gridDim.x * K + i] = 0;
        }
        // copy 1 of the final sums (the kd ties' moves, kd_reduce_kernel), spread over the grid:
        // the finalize that added it no longer clears it in one block
        for (uint32_t i = blockIdx.x * M32_THREADS + tid; i < nz1; i += gridDim.x * M32_THREADS) z1[i] = 0;
    }
    __syncthreads();
    const float *C32 = STAGED ? c32s : g_C32;

    const uint32_t ntiles = Kp / 32;
    // A fragments of code tile t: P half h of code vector 32t + r32 (halves swapped on bit 3),
    // Q bytes 8(1-h) .. +15
    const unsigned char *pa = lds + ROWS0 + r32 * 32 + 16 * (h ^ ((r32 >> 3) & 1));
    const unsigned char *qa = lds + L.q + r32 * 24 + 8 * (1 - h);
    auto load_a = [&](uint32_t t, half8 &a1, half8 &a2) {
        const u32x4v v1 = *reinterpret_cast<const u32x4v *>(pa + (size_t)t * (32 * 32));
        const uint64_t *q = reinterpret_cast<const uint64_t *>(qa + (size_t)t * (32 * 24));
        const u64x2v v2 = {q[0], q[1]};
        a1 = __builtin_bit_cast(half8, v1);
        a2 = __builtin_bit_cast(half8, v2);
    };
    const uint32_t ones = h ? 0u : 0x3C003C00u;   // f16 (1, 1) on the n_hi n_lo slots of half 0
    // PRUNE: lane l < ntiles keeps tile l's projection envelope [tlo, thi] (row-sum units)
    const int32_t tlo = PRUNE && lane < (int)ntiles ? g_tint[2 * lane] : 0x7FFFFFFF;
    const int32_t thi = PRUNE && lane < (int)ntiles ? g_tint[2 * lane + 1] : (int32_t)0x80000000;
    const float sx2 = th.sx * th.sx, dsx = (float)MF_D / sx2;

    for (; chunk < nchunks; chunk += stride) {
        const uint64_t base = chunk * M32_ROWS;
        uint32_t q[6];
#pragma unroll
        for (int i = 0; i < 6; i++) q[i] = qn[i];
        load_codes(chunk + stride, qn);   // prefetch the next chunk under this one's search
        const uint32_t own[3] = {h ? q[3] : q[0], h ? q[4] : q[1], h ? q[5] : q[2]};
        half8 b1[2], b2[2];
#pragma unroll
        for (int T = 0; T < 2; T++) {
            uint32_t w01, w23, w45, w67, w89, wab;
            byte_quad_w(q[3 * T], w01, w23);
            byte_quad_w(q[3 * T + 1], w45, w67);
            byte_quad_w(q[3 * T + 2], w89, wab);
            const u32x4v v1 = {w01, w23, w45, w67};
            const u32x4v v2 = {w89, wab, ones, 0u};
            b1[T] = __builtin_bit_cast(half8, v1);
            b2[T] = __builtin_bit_cast(half8, v2);
        }
        float s1[2], s2[2];
        uint32_t su[2];
#pragma unroll
        for (int T = 0; T < 2; T++) {
            s1[T] = INFINITY;
            s2[T] = INFINITY;
            su[T] = 0;
        }
        half8 a1, a2;
        const f32x16 zero16 = {};
        const uint32_t idmask = (1u << idbits) - 1, keep = ~idmask;
        auto tile_step = [&](uint32_t t, const f32x16 (&c)[2]) {
#pragma unroll
            for (int T = 0; T < 2; T++) {
#pragma unroll
                for (int qq = 0; qq < NU; qq++) {
                    const int o = qq * U;
                    float m;
                    if constexpr (U == 8)
                        m = min2f(min3f(min3f(min3f(c[T][o], c[T][o + 1], c[T][o + 2]), c[T][o + 3], c[T][o + 4]),
                                        c[T][o + 5], c[T][o + 6]),
                                  c[T][o + 7]);
                    else
                        m = min2f(min3f(c[T][o], c[T][o + 1], c[T][o + 2]), c[T][o + 3]);
                    // (the id as one scalar operand: v_and_or_b32, not and + or3 of its parts)
                    if constexpr (TAG)
                        m32_track_tagged(m, keep, (uint32_t)__builtin_amdgcn_readfirstlane((int)(t * NU + qq)), s1[T],
                                         s2[T]);
                    else m32_track(m, t * NU + qq, s1[T], s2[T], su[T]);
                }
            }
        };
        auto mfma4 = [&](f32x16 (&c)[2]) {
            c[0] = __builtin_amdgcn_mfma_f32_32x32x16_f16(a1, b1[0], zero16, 0, 0, 0);
            c[1] = __builtin_amdgcn_mfma_f32_32x32x16_f16(a1, b1[1], zero16, 0, 0, 0);
            c[0] = __builtin_amdgcn_mfma_f32_32x32x16_f16(a2, b2[0], c[0], 0, 0, 0);
            c[1] = __builtin_amdgcn_mfma_f32_32x32x16_f16(a2, b2[1], c[1], 0, 0, 0);
        };
        if constexpr (PRUNE) {
            // ||x - c||^2 >= (sum_d (x_d - c_d))^2 / D = sx^2 (sum w - q_c)^2 / D: with the rows'
            // sums of w in [qmn, qmx] and a tile's q in [lo, hi], a tile whose gap g satisfies
            // sx^2 g^2 / D > every row's current best distance (plus its MFMA error) holds no
            // code vector that can be any row's answer or tie with it -- strictly farther.
            int qmn, qmx;
            float xn2[2];   // ||x - mu||^2 of this lane's two rows
            {
                int qw[2];
#pragma unroll
                for (int T = 0; T < 2; T++) {
                    const uint32_t u0 = q[3 * T] ^ 0x80808080u, u1 = q[3 * T + 1] ^ 0x80808080u,
                                   u2 = q[3 * T + 2] ^ 0x80808080u;
                    const uint32_t su =
                        __builtin_amdgcn_sad_u8(u0, 0u, __builtin_amdgcn_sad_u8(u1, 0u, __builtin_amdgcn_sad_u8(u2, 0u, 0u)));
                    const uint32_t s2q = __builtin_amdgcn_udot4(u0, u0, __builtin_amdgcn_udot4(u1, u1,
                                         __builtin_amdgcn_udot4(u2, u2, 0u, false), false), false);
                    qw[T] = 2 * (int)su - 2 * 1530;   // sum_d w_d, w = 2u - 255
                    xn2[T] = (float)(int)(4 * s2q - 1020 * su + 12 * 65025) * sx2;   // sum w^2 exact
                }
                qmn = (int)(wave_min_u32((uint32_t)min(qw[0], qw[1]) ^ 0x80000000u) ^ 0x80000000u);
                qmx = (int)(~wave_min_u32(~((uint32_t)max(qw[0], qw[1]) ^ 0x80000000u)) ^ 0x80000000u);
            }
            // The nearest tile first (the first whose envelope reaches the rows' centre), then one
            // bound from it -- every row's best distance so far, from above: the lane's two tagged
            // bests (tag error orrel relative) plus the MFMA error, max over the wave -- and the
            // window of tiles within it: the tiles' gaps grow away from the centre (monotone
            // envelopes), so the window is one contiguous range.  One decision per chunk keeps
            // the tile loop free of per-tile dependencies (a per-tile bound measured no faster).
            const int t0 = min((int)__popcll(__ballot(lane < (int)ntiles && thi < ((qmn + qmx) >> 1))), (int)ntiles - 1);
            {
                load_a((uint32_t)t0, a1, a2);
                f32x16 c[2];
                mfma4(c);
                tile_step((uint32_t)t0, c);
            }
            float ub = 0.f;
#pragma unroll
            for (int T = 0; T < 2; T++) {   // the row's bound: the better of its two halves (lane ^ 32)
                const float v = __fmaf_rn(s1[T], th.inv_scale, xn2[T]);
                const float b = __fmaf_rn(orrel * th.inv_scale, fabsf(s1[T]), v + th.mfma);
                ub = fmaxf(ub, fminf(b, xor32_f32(b)));
            }
            ub = __uint_as_float(~wave_min_u32(~__float_as_uint(fmaxf(ub, 0.f))));   // >= 0: bits order as values
            const float bw = ub * dsx * 1.00001f + 1.0f;
            const float gap = (float)max(0, max(tlo - qmx, qmn - thi));   // this lane's tile
            const uint64_t win = __ballot(lane < (int)ntiles && gap * gap <= bw);
            const int lo_t = win ? __ffsll((unsigned long long)win) - 1 : t0;
            const int hi_t = win ? 63 - __clzll((long long)win) : t0;
            // [lo_t, hi_t] without t0, in two runs, the next tile's fragments under each tile's work
            for (int seg = 0; seg < 2; seg++) {
                const int b = seg ? t0 + 1 : lo_t, e = seg ? hi_t : t0 - 1;   // inclusive
                if (b > e) continue;
                load_a((uint32_t)b, a1, a2);
                for (int t = b; t <= e; t++) {
                    f32x16 c[2];
                    mfma4(c);
                    load_a((uint32_t)(t < e ? t + 1 : t), a1, a2);
                    tile_step((uint32_t)t, c);
                }
            }
        } else {
            load_a(0, a1, a2);
            for (uint32_t t = 0; t < ntiles; t++) {
                f32x16 c[2];
                mfma4(c);
                load_a(t + 1 < ntiles ? t + 1 : t, a1, a2);   // the next tile's fragments under these
                tile_step(t, c);
            }
        }
        if constexpr (TAG) {
#pragma unroll
            for (int T = 0; T < 2; T++) su[T] = __float_as_uint(s1[T]) & idmask;
        }
        // Merge the two halves of every data row: swap32(x = tile 0, y = tile 1) leaves lanes
        // < 32 with tile 0 row r32 (lo: own half, hi: half 1 of lane + 32) and lanes >= 32
        // with tile 1 row r32 (lo: half 0 of lane - 32, hi: own half) -- the own row base +
        // lane in both.  Units carry their half: unit * 2 + h.
        float sec_m;
        uint32_t unit;
        {
            const auto p1 = swap32_f32(s1[0], s1[1]);
            const auto p2 = swap32_f32(s2[0], s2[1]);
            const auto pu = swap32_u32(su[0] * 2 + h, su[1] * 2 + h);
            float m1 = p1.lo;
            sec_m = p2.lo;
            unit = pu.lo;
            if (p1.hi < m1 || (p1.hi == m1 && pu.hi < unit)) {
                sec_m = min2f(p2.hi, m1);
                m1 = p1.hi;
                unit = pu.hi;
            } else {
                sec_m = min2f(sec_m, p1.hi);
            }
        }
        // Recompute the winning unit's code vectors in the direct fp32 form (x - c)^2.
        const uint64_t row = base + lane;
        const bool valid = row < N;
        uint32_t rk = 0;
        if (valid) {
            // x_d = mu + w_d sx = (mu - 255 sx) + u_d (2 sx) in one fma from the centred byte u,
            // and ||x - mu||^2 = sx^2 sum_d w_d^2 from the exact integer sum (v_sad_u8 / v_dot4:
            // sum w^2 = 4 sum u^2 - 1020 sum u + D 255^2): 2 VALU per component instead of 5,
            // and both within the recompute's error model (one rounding per x_d, two for xn)
            float x[MF_D];
            const uint32_t uq[3] = {own[0] ^ 0x80808080u, own[1] ^ 0x80808080u, own[2] ^ 0x80808080u};
            const uint32_t su = __builtin_amdgcn_sad_u8(uq[0], 0u, __builtin_amdgcn_sad_u8(uq[1], 0u,
                                __builtin_amdgcn_sad_u8(uq[2], 0u, 0u)));
            const uint32_t s2q = __builtin_amdgcn_udot4(uq[0], uq[0], __builtin_amdgcn_udot4(uq[1], uq[1],
                                 __builtin_amdgcn_udot4(uq[2], uq[2], 0u, false), false), false);
            const float xn = (float)(int)(4 * s2q - 1020 * su + MF_D * 65025) * (th.sx * th.sx);   // ||x - mu||^2
            {
                const float two_sx = 2.f * th.sx, x0 = __fmaf_rn(-255.f, th.sx, th.mu);
#pragma unroll
                for (int d = 0; d < MF_D; d++)
                    x[d] = __fmaf_rn((float)((uq[d / 4] >> (8 * (d % 4))) & 0xFF), two_sx, x0);
            }
            // unit = ((tile * NU + q) * 2 + hh): 8-unit q covers rows 16q + 4hh + {0..3, 8..11}
            // of the tile, 4-unit q rows 8q + 4hh + {0..3}
            const uint32_t hh = unit & 1, qq = (unit >> 1) % NU, tile = (unit >> 1) / NU;
            const uint32_t cb = tile * 32 + (U == 8 ? 16 * qq : 8 * qq) + 4 * hh;
            float r1 = INFINITY, r2 = INFINITY;
#pragma unroll
            for (int j = 0; j < U; j++) {
                const uint32_t cp = cb + (j & 3) + 8 * (j >> 2);   // tile position
                const uint32_t cv = PRUNE ? perm_l[cp] : cp;         // its code vector
                const float4 *c4 = reinterpret_cast<const float4 *>(C32 + (size_t)cv * MF_D);
                float dist = 0.f;
#pragma unroll
                for (int k4 = 0; k4 < 3; k4++) {
                    const float4 cq = c4[k4];
                    float e;
                    e = x[4 * k4 + 0] - cq.x; dist = __fmaf_rn(e, e, dist);
                    e = x[4 * k4 + 1] - cq.y; dist = __fmaf_rn(e, e, dist);
                    e = x[4 * k4 + 2] - cq.z; dist = __fmaf_rn(e, e, dist);
                    e = x[4 * k4 + 3] - cq.w; dist = __fmaf_rn(e, e, dist);
                }
                dist = cv < K ? dist : INFINITY;   // padding code vectors never win
                r2 = med3f(r1, r2, dist);
                rk = dist < r1 ? cv : rk;
                r1 = min2f(r1, dist);
            }
            const float sec = min2f(__fmaf_rn(sec_m, th.inv_scale, xn), r2);
            // per-row MFMA bound: sum_d |w_d| <= 2 sum_d |u_d - 127| + D (v_sad_u8 of the bytes)
            uint32_t sad = 0;
#pragma unroll
            for (int k4 = 0; k4 < 3; k4++) sad = __builtin_amdgcn_sad_u8(own[k4] ^ 0x80808080u, 0x7F7F7F7Fu, sad);
            const float thm = __fmaf_rn((float)(2 * sad + MF_D), th.m1, th.m0);
            // sec from an MFMA score can be slightly negative (a row on a code vector): the
            // row is flagged then anyway (r1 >= 0), and no NaN reaches the -fno-honor-nans compare
            const float sp = fmaxf(sec, 0.f);
            float thr = thm + 2.f * (th.alpha * sqrtf(sp) + th.beta * sp) + th.gamma;
            // tagged unit minima: sec_m (and the choice of the best unit) is off by at most
            // orrel / 2 relative, in distance units |sec_m| 2^-t
            if (TAG) thr = __fmaf_rn(orrel * th.inv_scale, fabsf(sec_m), thr);
            A[row] = rk;
            if (!(sec - r1 > thr)) flags[atomicAdd(flag_cnt, 1u)] = (uint32_t)row;
        }
        if (FUSE) {
            // every row at its provisional index; the recheck / kd-tree move re-assigned ones
            if (copies > 1) {
                if (valid) {
                    const uint32_t cp = (uint32_t)lane & (copies - 1);
                    uint64_t *my = sums + (size_t)cp * m32_sum_stride(K, copies);
#pragma unroll
                    for (int d = 0; d < MF_D; d++) {
                        const uint32_t b = (own[d / 4] >> (8 * (d % 4))) & 0xFF;
                        atomicAdd((unsigned long long *)&my[(uint32_t)d * m32_kstride(K) + rk],
                                  (unsigned long long)((uint64_t)(b ^ 0x80u) << 32 | lo8_at0[b]));
                    }
                    atomicAdd(&cnt[cp * m32_cnt_stride(K, copies) + rk], 1u);
                }
            } else {
                uint32_t v[MF_D + 1];
#pragma unroll
                for (int d = 0; d < MF_D; d++) {
                    const uint32_t b = (own[d / 4] >> (8 * (d % 4))) & 0xFF;
                    v[d] = valid ? ((b ^ 0x80u) << 16 | lo8_at0[b]) : 0u;   // <= 64 rows: no carry
                }
                v[MF_D] = valid ? 1u : 0u;
                const bool tail = m32_runs_reduce(valid ? rk : 0xFFFFFFFFu, v, lane);
                if (tail && valid) {
#pragma unroll
                    for (int d = 0; d < MF_D; d++)
                        atomicAdd((unsigned long long *)&sums[(uint32_t)d * m32_kstride(K) + rk],
                                  (unsigned long long)((((uint64_t)(v[d] >> 16)) << 32) | (v[d] & 0xFFFF)));
                    atomicAdd(&cnt[rk], v[MF_D]);
                }
            }
        }
    }
    if (FUSE) {
        __syncthreads();
        uint64_t *pdst = part + (uint64_t)blockIdx.x * K * MF_D;   // slab layout [d][k]
        for (uint32_t i = tid; i < K * MF_D; i += M32_THREADS) {
            const uint32_t d = i / K, j = d * m32_kstride(K) + (i - d * K);
            uint64_t v = 0;
            for (uint32_t c = 0; c < copies; c++) v += sums[(size_t)c * m32_sum_stride(K, copies) + j];
            pdst[i] = v;
        }
        uint32_t *cdst = part_cnt + (uint64_t)blockIdx.x * K;
        for (uint32_t i = tid; i < K; i += M32_THREADS) {
            uint32_t v = 0;
            for (uint32_t c = 0; c < copies; c++) v += cnt[c * m32_cnt_stride(K, copies) + i];
            cdst[i] = v;
        }
    }
}

// =======================================================================================
// Recheck of flagged rows on the same MFMA scores (D = 12).  A wave takes 32 flagged rows (one
// data tile, both lane halves) through every code tile twice: pass 1 takes each row's minimum
// score m; pass 2 lists the code vectors whose score is within m + 2E, E the row's MFMA bound
// (m0 + m1 sum|w|, scaled) -- every other code vector is farther than the best in exact
// arithmetic by more than the tie tolerance.  Those candidates (a few per row) get the fp64
// distance in the reference's order (ref_l2_hd; lut64 values, C64); the row then takes the
// lexicographic (distance, index) minimum, or goes to the kd-tree tie list when its best two
// are within tie_rel.  Replaces the fp32 pass over all K per row (a wave per row) of
// recheck_kernel: ~16 VALU per row and code tile pair instead of ~28 per code vector.
// =======================================================================================
constexpr int RC_CAP = 16;   // candidates listed per row; more: the row's lane scans all K in fp64

struct RcLds {
    uint32_t q, lut, cand, ncand, total;
};
__host__ __device__ inline RcLds rc_lds_layout(uint32_t K) {
    const uint32_t Kp = (K + 31) & ~31u;
    RcLds L;
    uint32_t o = Kp * 32;
    L.q = o;
    o += Kp * 24;
    o = (o + 15) & ~15u;
    L.lut = o;
    o += 256 * 8;
    L.cand = o;
    o += M32_WAVES * 64 * RC_CAP * 4;   // [wave][half][row][RC_CAP]: a list per lane
    L.ncand = o;
    o += M32_WAVES * 64 * 4;
    L.total = o;
    return L;
}
bool recheck_mf32_fits(uint32_t K) { return rc_lds_layout(K).total <= M32_LDS_MAX; }

__global__ __launch_bounds__(M32_THREADS) void recheck_mf32_kernel(
    const uint8_t *__restrict__ codes, const uint32_t *__restrict__ flags, const unsigned *__restrict__ flag_cnt,
    const _Float16 *__restrict__ g_rows, const double *__restrict__ C64, uint32_t K,
    const double *__restrict__ g_lut64, MfThresholds th, double tie_rel, double tie_abs, uint32_t *__restrict__ A,
    uint32_t *__restrict__ ties, unsigned *__restrict__ tie_cnt, uint64_t *__restrict__ xslab,
    uint32_t *__restrict__ xcnt, const uint64_t *__restrict__ plut) {
    extern __shared__ __attribute__((aligned(16))) unsigned char lds[];
    const unsigned nflag = *flag_cnt;
    const uint32_t ntile_rows = (nflag + 31) / 32;
    // tile-rows go round the blocks first (tr = blockIdx + grid * wave ...): a level's few
    // hundred tile-rows spread over every CU, not packed 16 to a CU on the first few
    if (blockIdx.x >= ntile_rows) return;   // (uniform) no rows for this block
    const uint32_t Kp = (K + 31) & ~31u;
    const RcLds L = rc_lds_layout(K);
    const int tid = threadIdx.x;
    m32_stage_pq(lds, L.q, g_rows, Kp, tid);
    double *lut = reinterpret_cast<double *>(lds + L.lut);
    for (uint32_t i = tid; i < 256; i += M32_THREADS) lut[i] = g_lut64[i];
    const int lane = tid & 63, wave = tid >> 6;
    const int r32 = lane & 31, h = lane >> 5;
    // each lane lists its own half's candidates of its row (no shared counter, no atomics)
    uint32_t *cand = reinterpret_cast<uint32_t *>(lds + L.cand) + wave * 64 * RC_CAP;
    uint32_t *ncand = reinterpret_cast<uint32_t *>(lds + L.ncand) + wave * 64;
    uint32_t *mine = cand + lane * RC_CAP;
    __syncthreads();
    const uint32_t ntiles = Kp / 32;
    const unsigned char *pa = lds + r32 * 32 + 16 * (h ^ ((r32 >> 3) & 1));
    const unsigned char *qa = lds + L.q + r32 * 24 + 8 * (1 - h);
    auto load_a = [&](uint32_t t, half8 &a1, half8 &a2) {
        const u32x4v v1 = *reinterpret_cast<const u32x4v *>(pa + (size_t)t * (32 * 32));
        const uint64_t *q = reinterpret_cast<const uint64_t *>(qa + (size_t)t * (32 * 24));
        const u64x2v v2 = {q[0], q[1]};
        a1 = __builtin_bit_cast(half8, v1);
        a2 = __builtin_bit_cast(half8, v2);
    };
    const uint32_t ones = h ? 0u : 0x3C003C00u;
    const f32x16 zero16 = {};
    const float scale_t = 1.0f / th.inv_scale;
    for (uint32_t tr = blockIdx.x + gridDim.x * wave; tr < ntile_rows; tr += gridDim.x * M32_WAVES) {
        const uint32_t f = tr * 32 + r32;
        const bool valid = f < nflag;
        const uint32_t row = flags[valid ? f : nflag - 1];
        const uint32_t *cw = reinterpret_cast<const uint32_t *>(codes + (uint64_t)row * MF_D);
        const uint32_t w0 = cw[0], w1 = cw[1], w2 = cw[2];
        half8 b1, b2;
        {
            uint32_t w01, w23, w45, w67, w89, wab;
            byte_quad_w(w0, w01, w23);
            byte_quad_w(w1, w45, w67);
            byte_quad_w(w2, w89, wab);
            const u32x4v v1 = {w01, w23, w45, w67};
            const u32x4v v2 = {w89, wab, ones, 0u};
            b1 = __builtin_bit_cast(half8, v1);
            b2 = __builtin_bit_cast(half8, v2);
        }
        uint32_t sad = __builtin_amdgcn_sad_u8(w0 ^ 0x80808080u, 0x7F7F7F7Fu, 0);
        sad = __builtin_amdgcn_sad_u8(w1 ^ 0x80808080u, 0x7F7F7F7Fu, sad);
        sad = __builtin_amdgcn_sad_u8(w2 ^ 0x80808080u, 0x7F7F7F7Fu, sad);
        // two scores' MFMA bounds, scaled, with a margin for the fp32 band arithmetic
        const float band_add = 2.002f * scale_t * __fmaf_rn((float)(2 * sad + MF_D), th.m1, th.m0);
        auto min16 = [](const f32x16 &c) {
            return min2f(min3f(min3f(min3f(c[0], c[1], c[2]), min3f(c[3], c[4], c[5]), min3f(c[6], c[7], c[8])),
                               min3f(c[9], c[10], c[11]), min3f(c[12], c[13], c[14])),
                         c[15]);
        };
        // scores of code tiles t and t + 1 (clamped: an odd count repeats the last tile), both
        // tiles' MFMAs issued before either result is read
        half8 a1, a2, a3, a4;
        auto pair = [&](uint32_t t, f32x16 &c, f32x16 &d) {
            load_a(t, a1, a2);
            load_a(t + 1 < ntiles ? t + 1 : t, a3, a4);
            c = __builtin_amdgcn_mfma_f32_32x32x16_f16(a1, b1, zero16, 0, 0, 0);
            d = __builtin_amdgcn_mfma_f32_32x32x16_f16(a3, b1, zero16, 0, 0, 0);
            c = __builtin_amdgcn_mfma_f32_32x32x16_f16(a2, b2, c, 0, 0, 0);
            d = __builtin_amdgcn_mfma_f32_32x32x16_f16(a4, b2, d, 0, 0, 0);
        };
        // pass 1: the row's minimum score
        float m = INFINITY;
        for (uint32_t t = 0; t < ntiles; t += 2) {
            f32x16 c, d;
            pair(t, c, d);
            m = min3f(m, min16(c), min16(d));
        }
        m = min2f(m, xor32_f32(m));
        const float band = valid ? m + band_add * (1.0f + 1e-6f) + fabsf(m) * 1e-6f : -INFINITY;
        // pass 2: list the code vectors inside the band, each lane into its own list (one
        // shared counter per row made every listing a returning LDS atomic, and the 16
        // listing branches of a tile ran whenever any of the wave's 32 rows had a candidate
        // there: pass 2 took 3-4x pass 1)
        uint32_t nmine = 0;
        auto list = [&](const f32x16 &c, uint32_t t) {
            if (__ballot(min16(c) <= band)) {   // some row of the wave has a candidate here
#pragma unroll
                for (int v = 0; v < 16; v++) {
                    if (c[v] <= band) {
                        if (nmine < RC_CAP) mine[nmine] = t * 32 + (v & 3) + 8 * (v >> 2) + 4 * h;
                        nmine++;
                    }
                }
            }
        };
        for (uint32_t t = 0; t < ntiles; t += 2) {
            f32x16 c, d;
            pair(t, c, d);
            list(c, t);
            if (t + 1 < ntiles) list(d, t + 1);
        }
        ncand[lane] = nmine;
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        if (valid && h == 0) {
            // the row's fp64 values, and its candidates (all K if the list overflowed)
            double x[MF_D];
#pragma unroll
            for (int d = 0; d < MF_D; d++) x[d] = lut[((d < 4 ? w0 : d < 8 ? w1 : w2) >> (8 * (d % 4))) & 0xFF];
            const uint32_t n0 = nmine, n1 = ncand[lane + 32];   // this half's, the other half's
            const uint32_t *other = mine + 32 * RC_CAP;
            const bool all = n0 > RC_CAP || n1 > RC_CAP;
            const uint32_t n = all ? K : n0 + n1;
            auto cand_at = [&](uint32_t i) { return i < n0 ? mine[i] : other[i - n0]; };
            double d1 = INFINITY, d2 = INFINITY;
            uint32_t k1 = 0xFFFFFFFFu;
            auto take = [&](uint32_t k, double d) {
                if (k >= K) return;   // padding positions
                if (d < d1 || (d == d1 && k < k1)) {
                    d2 = d1;
                    d1 = d;
                    k1 = k;
                } else if (d < d2) {
                    d2 = d;
                }
            };
            // two candidates per trip, both rows' loads in flight together (one round trip each
            // through L2 was the chain of a row with several candidates)
            for (uint32_t i = 0; i < n; i += 2) {
                const uint32_t ka = all ? i : cand_at(i);
                const bool two = i + 1 < n;
                const uint32_t kb = two ? (all ? i + 1 : cand_at(i + 1)) : ka;
                const RowN<MF_D> ra = load_row<MF_D>(C64 + (uint64_t)min(ka, K - 1) * MF_D);
                const RowN<MF_D> rb = load_row<MF_D>(C64 + (uint64_t)min(kb, K - 1) * MF_D);
                take(ka, ref_l2_n<MF_D>(x, ra));
                if (two) take(kb, ref_l2_n<MF_D>(x, rb));
            }
            if (in_tie_band(d1, d2, tie_rel, tie_abs)) {   // a tie for the reference: the kd-tree decides
                ties[atomicAdd(tie_cnt, 1u)] = row;   // A keeps the provisional index
            } else {
                const uint32_t from = A[row];   // the search's index (its terms are in the slabs when fused)
                if (k1 != from) {
                    if (xslab) {
                        for (int d = 0; d < MF_D; d++) {
                            const unsigned long long tm =
                                plut[((d < 4 ? w0 : d < 8 ? w1 : w2) >> (8 * (d % 4))) & 0xFF];
                            atomicAdd((unsigned long long *)&xslab[(uint64_t)d * K + k1], tm);
                            atomicAdd((unsigned long long *)&xslab[(uint64_t)K * MF_D + (uint64_t)d * K + from], tm);
                        }
                        atomicAdd(&xcnt[k1], 1u);
                        atomicAdd(&xcnt[K + from], 1u);
                    }
                    A[row] = k1;
                }
            }
        }
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    }
}

hipError_t launch_recheck_mf32(hipStream_t s, int num_cu, const uint8_t *codes, const uint32_t *flags,
                               const unsigned *flag_cnt, const _Float16 *cb_rows, const double *C64, uint32_t K,
                               const double *lut64, const MfThresholds &th, double tie_rel, double tie_abs, uint32_t *A,
                               uint32_t *ties, unsigned *tie_cnt, uint64_t *xslab, uint32_t *xcnt,
                               const uint64_t *plut) {
    if (!recheck_mf32_fits(K)) return hipErrorInvalidValue;
    hipLaunchKernelGGL(recheck_mf32_kernel, dim3(num_cu), dim3(M32_THREADS), rc_lds_layout(K).total, s, codes, flags,
                       flag_cnt, cb_rows, C64, K, lut64, th, tie_rel, tie_abs, A, ties, tie_cnt, xslab, xcnt, plut);
    return hipGetLastError();
}

template <bool F, bool S, int U, bool TAG, bool P = false>
static void launch_mf32_variant(hipStream_t s, int grid, size_t lds, const uint8_t *codes, uint64_t N,
                                const _Float16 *cb_rows, uint32_t K, const float *C32, const uint64_t *plut,
                                const MfThresholds &th, uint32_t idbits, float orrel, uint32_t *A, uint32_t *flags,
                                unsigned *flag_cnt, uint64_t *part, uint32_t *part_cnt, uint32_t copies,
                                const uint32_t *perm, const int32_t *tint, uint64_t *z1, uint32_t nz1) {
    hipLaunchKernelGGL((assign_mf32_kernel<F, S, U, TAG, P>), dim3(grid), dim3(M32_THREADS), lds, s, codes, N, cb_rows,
                       K, C32, plut, th, idbits, orrel, A, flags, flag_cnt, part, part_cnt, copies, perm, tint, z1, nz1);
}

bool mf32_fits(uint32_t K, bool fuse) { return m32_lds_layout(K, fuse, false).total <= M32_LDS_MAX; }

bool mf32_prune_fits(uint32_t K, bool fuse) {
    return K <= 65536 && m32_lds_layout(K, fuse, false, 1, true).total <= M32_LDS_MAX;
}

hipError_t launch_assign_mf32(hipStream_t s, int grid, bool fuse, const uint8_t *codes, uint64_t N,
                              const _Float16 *cb_rows, uint32_t K, const float *C32, const uint64_t *plut,
                              const MfThresholds &th, uint32_t *A, uint32_t *flags, unsigned *flag_cnt,
                              uint64_t *part, uint32_t *part_cnt, const uint32_t *perm, const int32_t *tint,
                              uint64_t *z1, uint32_t nz1) {
    if (!mf32_fits(K, fuse)) return hipErrorInvalidValue;
    if (!fuse) z1 = nullptr, nz1 = 0;   // (cleared in the fused set-up block only)
    const bool prune = perm && tint;
    if (prune && !mf32_prune_fits(K, fuse)) return hipErrorInvalidValue;
    const bool staged = m32_lds_layout(K, fuse, true, 1, prune).total <= M32_LDS_MAX;
    // sums copies (fused, 64 <= K <= 512): the most, up to 16, that fit.  With the padded copy
    // strides, C3: K = 64 / 128 / 256 / 512 -6 / -22 / -19 / -16 us against the wave run
    // reduction; K = 1024 has no room for a second copy (the run reduction at the pruned K = 256:
    // 123.3-123.9 vs 113.6-116.2 us, profiles/r05ap).
    uint32_t copies = 1;
    if (fuse && K >= 64 && K <= 512)
        while (copies < 16 && m32_lds_layout(K, fuse, staged, copies * 2, prune).total <= M32_LDS_MAX) copies *= 2;
    const size_t lds = m32_lds_layout(K, fuse, staged, copies, prune).total;
    // 4-code-vector units while the tile loop is short (the recompute dominates); K = 256 takes
    // 8-code-vector units, which the pruned search needs (the unpruned 4-unit search there:
    // 129.2 / 123.4 vs 112.7 / 114.1 us, profiles/r05al)
    const bool u4 = K <= 128;
    // unit tags: ids t * NU + q < (Kp / 32) * NU per lane fit the low mantissa bits up to 12 bits
    const uint32_t units = ((K + 31) / 32) * (u4 ? 4 : 2);
    uint32_t idbits = 0;
    while ((1u << idbits) < units) idbits++;
    const float orrel = std::ldexp(1.0f, (int)idbits - 22);
    using Fn = void (*)(hipStream_t, int, size_t, const uint8_t *, uint64_t, const _Float16 *, uint32_t, const float *,
                        const uint64_t *, const MfThresholds &, uint32_t, float, uint32_t *, uint32_t *, unsigned *,
                        uint64_t *, uint32_t *, uint32_t, const uint32_t *, const int32_t *, uint64_t *, uint32_t);
#define QVQ_MF32_PICK(TG)                                                                                          \
    if (fuse) {                                                                                                    \
        if (u4) fn = staged ? launch_mf32_variant<true, true, 4, TG> : launch_mf32_variant<true, false, 4, TG>;    \
        else fn = staged ? launch_mf32_variant<true, true, 8, TG> : launch_mf32_variant<true, false, 8, TG>;       \
    } else {                                                                                                       \
        if (u4) fn = staged ? launch_mf32_variant<false, true, 4, TG> : launch_mf32_variant<false, false, 4, TG>;  \
        else fn = staged ? launch_mf32_variant<false, true, 8, TG> : launch_mf32_variant<false, false, 8, TG>;     \
    }
    Fn fn;
    if (prune && !u4 && idbits <= 12) {   // pruned search: 8-code-vector units, tagged
        if (fuse) fn = staged ? launch_mf32_variant<true, true, 8, true, true> : launch_mf32_variant<true, false, 8, true, true>;
        else fn = staged ? launch_mf32_variant<false, true, 8, true, true> : launch_mf32_variant<false, false, 8, true, true>;
    } else if (idbits <= 12) {
        QVQ_MF32_PICK(true)
    } else {
        QVQ_MF32_PICK(false)
    }
#undef QVQ_MF32_PICK
    if (!(prune && !u4 && idbits <= 12)) perm = nullptr, tint = nullptr;   // (the unpruned order: identity)
    fn(s, grid, lds, codes, N, cb_rows, K, C32, plut, th, idbits, orrel, A, flags, flag_cnt, part, part_cnt, copies, perm,
       tint, z1, nz1);
    return hipGetLastError();
}

}  // namespace qvq
