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

// Centred integer of a byte: w = 2*((int8)b + 128) - 255 = 2*(b ^ 0x80) - 255 (both colour
// spaces), so v(b) = mu + w*sx.  Exact in f16.
__device__ inline float byte_w(uint32_t word, int j) {
    return __fmaf_rn(2.f, (float)(((word ^ 0x80808080u) >> (8 * j)) & 0xFF), -255.f);
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
