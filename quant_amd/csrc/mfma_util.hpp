// mfma_util.hpp -- device helpers shared by the MFMA search kernels (k_assign.hip, k_wide.hip).
#pragma once
#include "common.hpp"

namespace qvq {

typedef _Float16 half8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

// min/min3 as compiler builtins: the hazard recognizer does not look inside inline asm, and
// an asm v_min3 reading an MFMA result right after the MFMA reads stale registers.  The
// search TUs build with -fno-honor-nans (no NaNs occur), so these become v_min3/v_min
// without canonicalising v_max instructions.
__device__ inline float min3f(float a, float b, float c) { return __builtin_fminf(__builtin_fminf(a, b), c); }
__device__ inline float min2f(float a, float b) { return __builtin_fminf(a, b); }
__device__ inline float med3f(float a, float b, float c) { return __builtin_amdgcn_fmed3f(a, b, c); }

// Cross-lane moves on the VALU (no LDS traffic; tools/micro/lane_ops_check.hip verifies them
// against __shfl_*).  v_permlane16_swap exchanges the odd 16-lane rows of its first operand
// with the even rows of its second; v_permlane32_swap the upper half of the first with the
// lower half of the second.  With both operands x, the x of lane ^ 16 (^ 32) lands in the
// first result on odd rows (upper half) and in the second on even rows (lower half).
__device__ inline uint32_t xor16_u32(uint32_t x) {
    const auto r = __builtin_amdgcn_permlane16_swap(x, x, false, false);
    return (__lane_id() & 16) ? r[0] : r[1];
}
__device__ inline uint32_t xor32_u32(uint32_t x) {
    const auto r = __builtin_amdgcn_permlane32_swap(x, x, false, false);
    return (__lane_id() & 32) ? r[0] : r[1];
}
// Both results of a swap.  swap32(x, y): lo = lanes < 32: x, lanes >= 32: y of lane - 32;
// hi = lanes < 32: x of lane + 32, lanes >= 32: y.  swap16 the same on 16-lane rows (even
// rows keep x in lo and take x of lane + 16 in hi; odd rows take y of lane - 16 in lo and
// keep y in hi).
struct LanePair {
    uint32_t lo, hi;
};
struct LanePairF {
    float lo, hi;
};
__device__ inline LanePair swap32_u32(uint32_t x, uint32_t y) {
    const auto r = __builtin_amdgcn_permlane32_swap(x, y, false, false);
    return {r[0], r[1]};
}
__device__ inline LanePair swap16_u32(uint32_t x, uint32_t y) {
    const auto r = __builtin_amdgcn_permlane16_swap(x, y, false, false);
    return {r[0], r[1]};
}
__device__ inline LanePairF swap32_f32(float x, float y) {
    const LanePair p = swap32_u32(__float_as_uint(x), __float_as_uint(y));
    return {__uint_as_float(p.lo), __uint_as_float(p.hi)};
}
__device__ inline LanePairF swap16_f32(float x, float y) {
    const LanePair p = swap16_u32(__float_as_uint(x), __float_as_uint(y));
    return {__uint_as_float(p.lo), __uint_as_float(p.hi)};
}
__device__ inline float xor16_f32(float x) { return __uint_as_float(xor16_u32(__float_as_uint(x))); }
__device__ inline float xor32_f32(float x) { return __uint_as_float(xor32_u32(__float_as_uint(x))); }
// x of lane - 1 (lane 0 keeps its own) and of lane + 1 (lane 63 keeps its own): DPP
// wave_shr:1 / wave_shl:1.
__device__ inline uint32_t wave_prev_u32(uint32_t x) {
    return (uint32_t)__builtin_amdgcn_update_dpp((int)x, (int)x, 0x138, 0xF, 0xF, false);
}
__device__ inline uint32_t wave_next_u32(uint32_t x) {
    return (uint32_t)__builtin_amdgcn_update_dpp((int)x, (int)x, 0x130, 0xF, 0xF, false);
}

// Wave64 inclusive scans with DPP (row_shr within rows of 16, then row_bcast:15/31 across
// rows): one VALU instruction per step, no LDS traffic.
template <int CTRL, int ROW_MASK>
__device__ inline uint32_t dpp_get(uint32_t v) {
    return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, CTRL, ROW_MASK, 0xF, true);
}
__device__ inline uint32_t wave_scan_add(uint32_t v) {
    v += dpp_get<0x111, 0xF>(v);   // row_shr:1
    v += dpp_get<0x112, 0xF>(v);   // row_shr:2
    v += dpp_get<0x114, 0xF>(v);   // row_shr:4
    v += dpp_get<0x118, 0xF>(v);   // row_shr:8
    v += dpp_get<0x142, 0xA>(v);   // row_bcast:15 into rows 1, 3
    v += dpp_get<0x143, 0xC>(v);   // row_bcast:31 into rows 2, 3
    return v;
}
__device__ inline uint32_t wave_scan_max(uint32_t v) {
    v = max(v, dpp_get<0x111, 0xF>(v));
    v = max(v, dpp_get<0x112, 0xF>(v));
    v = max(v, dpp_get<0x114, 0xF>(v));
    v = max(v, dpp_get<0x118, 0xF>(v));
    v = max(v, dpp_get<0x142, 0xA>(v));
    v = max(v, dpp_get<0x143, 0xC>(v));
    return v;
}

// fp64 minimum over the wave (or over lanes 0..15 with ROWS = 1) by DPP steps on the two
// dword halves: VALU-only, no LDS round trips on the walk's serial path.  Uniform result.
template <int CTRL, int ROW_MASK>
__device__ inline double dpp_min_step(double v) {
    const uint64_t b = (uint64_t)__double_as_longlong(v);
    constexpr uint64_t inf = 0x7FF0000000000000ull;   // what lanes without a source read
    const uint32_t lo = (uint32_t)__builtin_amdgcn_update_dpp((int)(uint32_t)inf, (int)(uint32_t)b, CTRL, ROW_MASK,
                                                              0xF, false);
    const uint32_t hi = (uint32_t)__builtin_amdgcn_update_dpp((int)(uint32_t)(inf >> 32), (int)(uint32_t)(b >> 32),
                                                              CTRL, ROW_MASK, 0xF, false);
    return fmin(v, __longlong_as_double((long long)(((uint64_t)hi << 32) | lo)));
}
template <int ROWS>
__device__ inline double wave_min_f64(double v) {
    v = dpp_min_step<0x111, 0xF>(v);   // row_shr:1
    v = dpp_min_step<0x112, 0xF>(v);   // row_shr:2
    v = dpp_min_step<0x114, 0xF>(v);   // row_shr:4
    v = dpp_min_step<0x118, 0xF>(v);   // row_shr:8: lane 15 of each row holds the row's
    int src = 15;
    if (ROWS > 1) {
        v = dpp_min_step<0x142, 0xA>(v);   // row_bcast:15 into rows 1, 3
        v = dpp_min_step<0x143, 0xC>(v);   // row_bcast:31 into rows 2, 3
        src = 63;
    }
    const uint64_t b = (uint64_t)__double_as_longlong(v);
    const uint32_t lo = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)b, src);
    const uint32_t hi = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(b >> 32), src);
    return __longlong_as_double((long long)(((uint64_t)hi << 32) | lo));
}

// u32 minimum over the wave by DPP steps (lanes without a source read ~0); uniform.
template <int CTRL, int ROW_MASK>
__device__ inline uint32_t dpp_min_u32_step(uint32_t v) {
    return min(v, (uint32_t)__builtin_amdgcn_update_dpp((int)0xFFFFFFFFu, (int)v, CTRL, ROW_MASK, 0xF, false));
}
__device__ inline uint32_t wave_min_u32(uint32_t v) {
    v = dpp_min_u32_step<0x111, 0xF>(v);   // row_shr:1
    v = dpp_min_u32_step<0x112, 0xF>(v);   // row_shr:2
    v = dpp_min_u32_step<0x114, 0xF>(v);   // row_shr:4
    v = dpp_min_u32_step<0x118, 0xF>(v);   // row_shr:8
    v = dpp_min_u32_step<0x142, 0xA>(v);   // row_bcast:15 into rows 1, 3
    v = dpp_min_u32_step<0x143, 0xC>(v);   // row_bcast:31 into rows 2, 3
    return (uint32_t)__builtin_amdgcn_readlane((int)v, 63);
}

// Centred integer of a byte: w = 2*((int8)b + 128) - 255 = 2*(b ^ 0x80) - 255 (both colour
// spaces), so v(b) = mu + w*sx.  Exact in f16.
__device__ inline float byte_w(uint32_t word, int j) {
    return __fmaf_rn(2.f, (float)(((word ^ 0x80808080u) >> (8 * j)) & 0xFF), -255.f);
}

// The four centred integers w = 2*(b ^ 0x80) - 255 of a word's bytes as two f16 pairs, exact:
// v_perm puts each u = b ^ 0x80 under an f16 exponent byte 0x64 (f16 0x64uu = 1024 + u), then
// (h - 1024) * 2 - 255 on packed f16 (every intermediate an integer below 2^11).
typedef _Float16 half2v __attribute__((ext_vector_type(2)));
__device__ inline uint32_t quad_pair_w(uint32_t h) {
    const half2v x = __builtin_bit_cast(half2v, h) + half2v{-1024, -1024};
    return __builtin_bit_cast(uint32_t, __builtin_elementwise_fma(x, half2v{2, 2}, half2v{-255, -255}));
}
__device__ inline void byte_quad_w(uint32_t word, uint32_t &w01, uint32_t &w23) {
    const uint32_t u = word ^ 0x80808080u;
    w01 = quad_pair_w(__builtin_amdgcn_perm(0x64646464u, u, 0x04010400u));   // [u0, 64, u1, 64]
    w23 = quad_pair_w(__builtin_amdgcn_perm(0x64646464u, u, 0x04030402u));   // [u2, 64, u3, 64]
}

// Epilogue of one tile pair for one data tile: minimum of the lane's 8 scores, then the
// running best pair, best score and second-best pair minimum.
__device__ inline void pair_update(const f32x4 &p0, const f32x4 &p1, uint32_t pair, float &b1, float &b2,
                                   uint32_t &bp) {
    const float m = min2f(min3f(min3f(p0[0], p0[1], p0[2]), p0[3], p1[0]), min3f(p1[1], p1[2], p1[3]));
    b2 = med3f(b1, b2, m);
    bp = m < b1 ? pair : bp;
    b1 = min2f(b1, m);
}

// One code tile for one data tile: minimum of the lane's 4 scores, then the running best tile,
// best score and second-best tile minimum.
__device__ inline void tile_update(const f32x4 &p, uint32_t tile, float &b1, float &b2, uint32_t &bt) {
    const float m = min2f(min3f(p[0], p[1], p[2]), p[3]);
    b2 = med3f(b1, b2, m);
    bt = m < b1 ? tile : bt;
    b1 = min2f(b1, m);
}
// The search's unit update: 8-code-vector units (a tile pair) or, with U4, 4-code-vector
// units (one tile; bp then counts tiles) -- half the recompute for 4 more VALU per pair.
template <bool U4>
__device__ inline void unit_update(const f32x4 &p0, const f32x4 &p1, uint32_t pair, float &b1, float &b2,
                                   uint32_t &bp) {
    if constexpr (U4) {
        tile_update(p0, 2 * pair, b1, b2, bp);
        tile_update(p1, 2 * pair + 1, b1, b2, bp);
    } else {
        pair_update(p0, p1, pair, b1, b2, bp);
    }
}

// Same, keeping the best two pairs (b1 at bp, b2 at bq) and the third-best minimum b3.
__device__ inline void pair_update2(const f32x4 &p0, const f32x4 &p1, uint32_t pair, float &b1, float &b2, float &b3,
                                    uint32_t &bp, uint32_t &bq) {
    const float m = min2f(min3f(min3f(p0[0], p0[1], p0[2]), p0[3], p1[0]), min3f(p1[1], p1[2], p1[3]));
    b3 = med3f(b2, b3, m);
    bq = m < b1 ? bp : (m < b2 ? pair : bq);
    b2 = med3f(b1, b2, m);
    bp = m < b1 ? pair : bp;
    b1 = min2f(b1, m);
}

}  // namespace qvq
