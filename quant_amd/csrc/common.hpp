// common.hpp -- shared numerics and kernel launch interface of the qvq engine.
#pragma once
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdint>

#include "kdtree_dev.hpp"

namespace qvq {

// ---------------------------------------------------------------------------------------
// Exact-sum decomposition of a colour space's byte -> value map.
// Every value v[b] is an integer multiple of 2^-scale: q[b] = v[b] * 2^scale.  We write
// q[b] = R * hi[b] + (lo[b] - bias) with hi[b] <= 255 and 0 <= lo[b] <= 2*bias small, so one
// u64 LDS atomic of (hi << 32 | lo) per component accumulates both parts without carries
// for up to 2^24 rows per workgroup; the finaliser rebuilds the exact 128-bit sum.
//
// For the MFMA search every value is also an exact small integer in centred form:
// v[b] - mu = w[b] * sx with |w[b]| <= 255 (f16-exact), up to fl() rounding of v.
// ---------------------------------------------------------------------------------------
struct Terms {
    double v64[256];
    float v32[256];
    uint32_t hi[256];
    uint32_t lo[256];
    float w[256];       // centred integer value of each byte
    int64_t R;
    int64_t bias;
    int scale;
    uint8_t pad_code;   // byte whose value is exactly 0.0 (padding past the raster end)
    double vmax;        // max |v|
    double mu, sx;      // v ~= mu + w * sx
};

bool make_terms(int cs, Terms &t);

// Correctly rounded (nearest-even) conversion of a signed 128-bit integer to double.
__host__ __device__ inline double i128_to_double(__int128 v) {
    const bool neg = v < 0;
    unsigned __int128 m = neg ? (unsigned __int128)0 - (unsigned __int128)v : (unsigned __int128)v;
    const uint64_t hi = (uint64_t)(m >> 64), lo = (uint64_t)m;
    if (hi == 0 && (lo >> 53) == 0) {
        const double d = (double)lo;   // exact
        return neg ? -d : d;
    }
#ifdef __HIP_DEVICE_COMPILE__
    const int lz = hi ? __clzll((long long)hi) : 64 + __clzll((long long)lo);
#else
    const int lz = hi ? __builtin_clzll(hi) : 64 + __builtin_clzll(lo);
#endif
    const int sh = (128 - lz) - 53;
    uint64_t top = (uint64_t)(m >> sh);
    const unsigned __int128 rem = m & (((unsigned __int128)1 << sh) - 1);
    const unsigned __int128 half = (unsigned __int128)1 << (sh - 1);
    if (rem > half || (rem == half && (top & 1))) top++;
    const double d = ldexp((double)top, sh);
    return neg ? -d : d;
}

// Centroid component from reduced sums: round(R*hi + lo - bias*cnt) * 2^-scale * fl(1/cnt).
// Empty cell -> zero vector (src/Quantizer.cpp:81-85).  The reciprocal multiply is the
// reference's operator/= under -freciprocal-math (include/VectorOperations.hpp:96-98).
__host__ __device__ inline double centroid_value(uint64_t hi, uint64_t lo, uint64_t cnt, int64_t R, int64_t bias,
                                                 int scale) {
    if (cnt == 0) return 0.0;
    const __int128 S = (__int128)R * (__int128)hi + (__int128)lo - (__int128)bias * (__int128)cnt;
    return ldexp(i128_to_double(S), -scale) * (1.0 / (double)cnt);
}

// MFMA search layout (D = 12): per code vector one 56-byte row of 28 f16
// [hi0..3, lo0..3, hi4..7, lo4..7, hi8..11, lo8..11, nhi, nlo, 0, 0], where hi+lo ~=
// -2*sx*(c-mu)*2^t and nhi+nlo ~= 2^t*||c-mu||^2, so that score = 2^t*(||x-c||^2 - ||x-mu||^2).
// K-slot group g < 3 (slots 8g..8g+7) then meets components 4g..4g+3 twice: one word of the
// data row per B fragment.
constexpr int MF_D = 12;
constexpr int MF_ROW_F16 = 28;
constexpr int MF_ROW_BYTES = 2 * MF_ROW_F16;
constexpr float MF_PAD_SCORE = 65504.0f;   // nhi = nlo = f16 max for padding code vectors

// Wide MFMA layout (every D != 12, Dp <= 64): per code vector KS k-steps of 32 f16 slots,
// [hi(DH) | lo(DH) | nhi nlo | 0 ...] with DH = Dp rounded up to 8 (hi/lo of components
// D..DH-1 are 0), same hi/lo/n meaning as above.
__host__ __device__ constexpr uint32_t wide_dh(uint32_t Dp) { return (Dp + 7) & ~7u; }
__host__ __device__ constexpr uint32_t wide_ks(uint32_t Dp) { return (2 * wide_dh(Dp) + 2 + 31) / 32; }
__host__ __device__ constexpr uint32_t wide_row_f16(uint32_t Dp) { return 32 * wide_ks(Dp); }
// f16 slots per code-vector row and the offset of the lo half, for either layout
__host__ __device__ inline uint32_t cb_row_f16(uint32_t D, uint32_t Dp) { return D == MF_D ? MF_ROW_F16 : wide_row_f16(Dp); }
__host__ __device__ inline uint32_t cb_lo_off(uint32_t D, uint32_t Dp) { return D == MF_D ? MF_D : wide_dh(Dp); }
// f16 slot of component d's hi and lo part in a row of either layout (norm: slots 2*LO, +1)
__host__ __device__ inline uint32_t cb_hi_slot(uint32_t D, uint32_t Dp, uint32_t d) {
    return D == MF_D ? 8 * (d / 4) + d % 4 : d;
}
__host__ __device__ inline uint32_t cb_lo_slot(uint32_t D, uint32_t Dp, uint32_t d) {
    return D == MF_D ? 8 * (d / 4) + 4 + d % 4 : wide_dh(Dp) + d;
}

// ---------------------------------------------------------------------------------------
// Launch wrappers (each defined next to its kernel).  All take the stream last-but-args.
// ---------------------------------------------------------------------------------------
hipError_t launch_gen(hipStream_t s, uint8_t *rgb, uint32_t S, uint64_t seed0, uint64_t npix);
// Decode gather (CompressedImage::decompress): codebook bytes [K][D], A [wB*hB] -> raster [xs*ys*3].
// With orig (the original raster) the squared signed-byte differences are added to *sqerr.
hipError_t launch_decode(hipStream_t s, const uint8_t *cb, uint32_t K, uint32_t D, const uint32_t *A, uint32_t xs,
                         uint32_t ys, uint32_t w, uint32_t h, uint8_t *rgb, const uint8_t *orig, uint64_t *sqerr,
                         uint32_t *bad);
hipError_t launch_tile(hipStream_t s, const uint8_t *rgb, uint8_t *codes, uint32_t n_images, uint32_t xSize,
                       uint32_t ySize, uint32_t bw, uint32_t bh, uint32_t D, uint32_t Dp, uint8_t pad);
// VALU fp32 search for any Dp (multiple of 4, <= 64); codebook C32 [K][Dp].
hipError_t launch_assign_valu(hipStream_t s, int num_cu, uint32_t Dp, const uint8_t *codes, uint64_t N,
                              const float *C32, uint32_t K, const float *lut32, float alpha, float beta, float gamma,
                              uint32_t *A, uint32_t *flags, unsigned *flag_cnt);
// MFMA f16 search for D = 12, optionally with the centroid sums fused (K <= mf_fuse_max_k()).
// Flag rule (distances, unscaled): second - best <= mfma + 2*(alpha*sqrt(second) + beta*second)
// + gamma, where `mfma` bounds the error of one MFMA score and the rest the fp32 direct-form
// recompute ("near-tie flags").
// A re-assigned row of the fused path (the search added its terms at its provisional index
// `from`): its packed terms (hi << 32 | lo, plut) go to slab G (xslab [d][k], xcnt [k]) at
// `to` and to slab G + 1 (xslab + K*D, xcnt + K; subtracted by the reduce) at `from`.
// Called by the lanes of one wave (lane < D does component lane).
__device__ inline void move_row_terms(const uint8_t *codes, uint32_t Dp, uint32_t D, uint32_t row, uint32_t from,
                                      uint32_t to, uint32_t K, uint64_t *xslab, uint32_t *xcnt, const uint64_t *plut,
                                      uint32_t lane) {
    if (lane < D) {
        const unsigned long long t = plut[codes[(uint64_t)row * Dp + lane]];
        atomicAdd((unsigned long long *)&xslab[(uint64_t)lane * K + to], t);
        atomicAdd((unsigned long long *)&xslab[(uint64_t)K * D + (uint64_t)lane * K + from], t);
    }
    if (lane == 0) {
        atomicAdd(&xcnt[to], 1u);
        atomicAdd(&xcnt[K + from], 1u);
    }
}

// The same move into a second copy of the final sums (layout hi[D][K] | lo[D][K] | cnt[K], u64,
// added mod 2^64 to copy 0 by the finalize): kd_reduce_kernel's ties, concurrent with the
// reduce of the slabs into copy 0.
__device__ inline void move_row_sums(const uint8_t *codes, uint32_t Dp, uint32_t D, uint32_t row, uint32_t from,
                                     uint32_t to, uint32_t K, uint64_t *xs, const uint64_t *plut, uint32_t lane) {
    const uint64_t KD = (uint64_t)K * D;
    if (lane < D) {
        const uint64_t t = plut[codes[(uint64_t)row * Dp + lane]];
        const unsigned long long hi = t >> 32, lo = t & 0xFFFFFFFFull;
        atomicAdd((unsigned long long *)&xs[(uint64_t)lane * K + to], hi);
        atomicAdd((unsigned long long *)&xs[KD + (uint64_t)lane * K + to], lo);
        atomicAdd((unsigned long long *)&xs[(uint64_t)lane * K + from], 0ull - hi);
        atomicAdd((unsigned long long *)&xs[KD + (uint64_t)lane * K + from], 0ull - lo);
    }
    if (lane == 0) {
        atomicAdd((unsigned long long *)&xs[2 * KD + to], 1ull);
        atomicAdd((unsigned long long *)&xs[2 * KD + from], ~0ull);
    }
}

// Column reduce of G slabs into sums (copy 0 of the final layout) by one 1024-thread block: 64
// columns, 16 waves each adding every 16th slab, combined through red (2 x 16 x 64 u64).  The
// last nsub slabs are subtracted (hi and lo separately: the corrections of re-assigned rows,
// whose terms the search had added at their provisional index); every total stays >= 0.
__device__ inline void reduce_columns_block(const uint64_t *__restrict__ part, const uint32_t *__restrict__ part_cnt,
                                            uint32_t G, uint32_t nsub, uint32_t K, uint32_t D,
                                            uint64_t *__restrict__ sums, uint32_t bid, uint64_t *red) {
    uint64_t(*red_hi)[64] = reinterpret_cast<uint64_t(*)[64]>(red);
    uint64_t(*red_lo)[64] = reinterpret_cast<uint64_t(*)[64]>(red + 16 * 64);
    const uint64_t KD = (uint64_t)K * D;
    const uint64_t col = (uint64_t)bid * 64 + (threadIdx.x & 63);
    const int sg = threadIdx.x >> 6;
    uint64_t hi = 0, lo = 0;
    if (col < KD) {
#pragma unroll 4
        for (uint32_t g = sg; g < G; g += 16) {
            const uint64_t p = part[g * KD + col];
            const uint64_t sgn = g < G - nsub ? 0 : ~0ull;   // x ^ sgn - sgn: +x or -x (mod 2^64)
            hi += ((p >> 32) ^ sgn) - sgn;
            lo += ((p & 0xFFFFFFFFull) ^ sgn) - sgn;
        }
    } else if (col < KD + K) {
#pragma unroll 4
        for (uint32_t g = sg; g < G; g += 16) {
            const uint64_t c = part_cnt[(uint64_t)g * K + (col - KD)];
            hi += g < G - nsub ? c : 0ull - c;
        }
    }
    red_hi[sg][threadIdx.x & 63] = hi;
    red_lo[sg][threadIdx.x & 63] = lo;
    __syncthreads();
    if (sg == 0) {
        for (int i = 1; i < 16; i++) {
            hi += red_hi[i][threadIdx.x];
            lo += red_lo[i][threadIdx.x];
        }
        if (col < KD) {
            sums[col] = hi;
            sums[KD + col] = lo;
        } else if (col < KD + K) {
            sums[2 * KD + (col - KD)] = hi;
        }
    }
}

// Rows the kd-tree answers: their best two fp64 distances are within tie_rel relative (ties of
// the reference's own arithmetic), or close enough that the reference's centroid bits -- which
// may differ from the exact sums' by tie_abs / (2 sqrt(D)) per component -- can decide them
// (DESIGN.md 3.8): |d' - d| <= tie_abs sqrt(d) + tie_abs^2 / 2 for each distance.
__host__ __device__ inline bool in_tie_band(double d1, double d2, double tie_rel, double tie_abs) {
    const double gap = d2 - d1;   // d2 = inf: one candidate only, never a tie
    const double band = tie_abs * (sqrt(d1) + sqrt(fmin(d2, 1e300))) + tie_abs * tie_abs;
    return gap <= tie_rel * d1 || gap <= band;
}

struct MfThresholds {
    float mfma, alpha, beta, gamma;
    float inv_scale;   // 2^-t
    float mu, sx;      // x = mu + w * sx
    // small-K scan (expanded fp32 scores): flag when second - best <= e0 + e1 * sum_d |w_d|
    float e0, e1;
    // the mfma bound for one row (k_mf32.hip): m0 + m1 * sum_d |w_d| <= mfma
    float m0, m1;
};
uint32_t mf_fuse_max_k();
bool mf_can_search(uint32_t K);
// K <= 32: expanded fp32 scores from E32 [Kp][16] = [c''(0..11) | n | 0 0 0] (the MFMA row's
// terms in fp32; padding rows n = 1e30).
// perm / tint (finalize's prune_order, K <= PRUNE_MAXK): the pruned tile order of the MFMA
// search (assign_mf32_kernel PRUNE); null: every tile in index order.
hipError_t launch_assign_mfma(hipStream_t s, int grid, bool fuse, const uint8_t *codes, uint64_t N,
                              const _Float16 *cb_rows, const float *E32, uint32_t K, const float *C32,
                              const uint64_t *plut,
                              const MfThresholds &th, uint32_t *A, uint32_t *flags, unsigned *flag_cnt,
                              uint64_t *part, uint32_t *part_cnt, const uint32_t *perm = nullptr,
                              const int32_t *tint = nullptr, uint64_t *z1 = nullptr, uint32_t nz1 = 0);
// (z1, nz1: fused searches also clear these nz1 u64 -- copy 1 of the final sums -- spread over the grid)
// The same search on v_mfma_f32_32x32x16_f16 tiles (k_mf32.hip); launch_assign_mfma uses it
// for K above the small-K scan whenever mf32_fits.
bool mf32_fits(uint32_t K, bool fuse);
bool mf32_prune_fits(uint32_t K, bool fuse);
hipError_t launch_assign_mf32(hipStream_t s, int grid, bool fuse, const uint8_t *codes, uint64_t N,
                              const _Float16 *cb_rows, uint32_t K, const float *C32, const uint64_t *plut,
                              const MfThresholds &th, uint32_t *A, uint32_t *flags, unsigned *flag_cnt,
                              uint64_t *part, uint32_t *part_cnt, const uint32_t *perm = nullptr,
                              const int32_t *tint = nullptr,
                              uint64_t *z1 = nullptr, uint32_t nz1 = 0);
constexpr uint32_t PRUNE_MAXK_HOST = 4096;   // prune_order's capacity (k_misc.hip PRUNE_MAXK)
// d_tint: the envelopes (2 int32 per tile, PRUNE_MAXK_HOST / 32 tiles), then Kpad floats of
// projections (finalize -> prune_order)
inline size_t tint_bytes(uint32_t Kp) { return (size_t)2 * (PRUNE_MAXK_HOST / 32) * 4 + (size_t)Kp * 4; }
// MFMA f16 search for D != 12 (wide layout), no fused sums: K >= 32, codebook staged in LDS
// whole or in double-buffered slices.  Same flag rule as launch_assign_mfma.
// perm / tint (prune_order): the pruned variant for streamed codebooks (wide_prune_fits); cpr:
// 64-row chunks per image column of blocks (the workgroup's chunks stack across it; 1 = none).
bool wide_can_search(uint32_t Dp);
bool wide_prune_fits(uint32_t Dp, uint32_t K);
// the whole codebook sits in one workgroup's LDS (the search is not streamed)
bool wide_codebook_resident(uint32_t Dp, uint32_t K);
hipError_t launch_assign_wide(hipStream_t s, int num_cu, uint32_t Dp, uint32_t D, const uint8_t *codes, uint64_t N,
                              const _Float16 *cb_rows, uint32_t K, const float *C32, const MfThresholds &th,
                              uint32_t *A, uint32_t *flags, unsigned *flag_cnt, const uint32_t *perm = nullptr,
                              const int32_t *tint = nullptr, uint32_t cpr = 1, unsigned *sched = nullptr);
// (sched: two zeroed u32 the pruned variant's task counter uses and leaves zeroed)
// perm / tint / qscale = D / sx^2 (the level's pruned order; the chunked sweep only): only the
// positions the projection bound admits for the rows' fp32 bands are swept.
// Recheck of flagged rows: fp32 distances to all K code vectors (C32 [Kpad][Dp]), fp64 in
// the reference's order for those inside the fp32 error band (alpha, beta, gamma as the VALU
// search's); exact ties are listed in ties (tie_cnt) for launch_kd_resolve or the host.
// With xslab != nullptr adds every other row's packed terms (hi << 32 | lo) to xslab [d][k]
// and its count to xcnt [k] (the search's extra slab G).
hipError_t launch_recheck(hipStream_t s, int num_cu, const uint8_t *codes, uint32_t Dp, uint32_t D,
                          const uint32_t *flags, const unsigned *flag_cnt, const double *C64, const float *C32,
                          uint32_t K, const double *lut64, float alpha, float beta, float gamma, double tie_rel, double tie_abs,
                          uint32_t *A, uint32_t *ties, unsigned *tie_cnt, uint64_t *xslab, uint32_t *xcnt,
                          const uint64_t *plut,
                          const uint32_t *perm = nullptr, const int32_t *tint = nullptr, float qscale = 0.f);
// The recheck on the search's MFMA scores (D = 12, k_mf32.hip): same contract as launch_recheck
// (the band from th.m0 / th.m1), for K with recheck_mf32_fits.
bool recheck_mf32_fits(uint32_t K);
hipError_t launch_recheck_mf32(hipStream_t s, int num_cu, const uint8_t *codes, const uint32_t *flags,
                               const unsigned *flag_cnt, const _Float16 *cb_rows, const double *C64, uint32_t K,
                               const double *lut64, const MfThresholds &th, double tie_rel, double tie_abs, uint32_t *A,
                               uint32_t *ties, unsigned *tie_cnt, uint64_t *xslab, uint32_t *xcnt,
                               const uint64_t *plut);
// Device kd-tree answers for the listed ties (tree image in mapped host memory); adds their
// terms to sums when given.  kd_resolve_fits: the tree, stacks and one wave's point
// distances fit the LDS.
bool kd_resolve_fits(const KdView &kd, uint32_t K);
// kd_reduce_kernel: launch_kd_resolve (ties into copy 1 of sums) + launch_reduce (into copy 0).
// The reference kd-tree of P (K x D fp64, row-major) built on the device (k_kdbuild.hip), one
// workgroup: vind / nodes / nbox / cbox are scratch of K, 2K, 2K x 2D, 2K x 2D entries; flat gets
// kd_resolve's image (lo | hi | KdNodeDev[n] | vind, tree_bytes(K, D) at most), himg (mapped host
// memory, kdb_host_layout) the whole tree, its header's seq set to seq last.
bool kd_build_fits(uint32_t K, uint32_t D);
hipError_t launch_kd_build(hipStream_t s, const double *P, uint32_t K, uint32_t D, uint32_t *vind, KdbNode *nodes,
                           double *nbox, double *cbox, uint8_t *flat, uint8_t *himg, uint64_t seq);
bool kd_reduce_fits(const KdView &kd, uint32_t K);
hipError_t launch_kd_reduce(hipStream_t s, const uint8_t *codes, uint32_t Dp, uint32_t D, const uint32_t *ties,
                            const unsigned *tie_cnt, const double *C64, uint32_t K, const double *lut64,
                            const KdView &kd, uint32_t *A, const uint64_t *plut, const uint64_t *part,
                            const uint32_t *part_cnt, uint32_t G, uint32_t nsub, uint64_t *sums, uint64_t *sums1);
hipError_t launch_kd_resolve(hipStream_t s, const uint8_t *codes, uint32_t Dp, uint32_t D, const uint32_t *ties,
                             const unsigned *tie_cnt, const double *C64, uint32_t K, const double *lut64,
                             const KdView &kd, uint32_t *A, uint64_t *xslab, uint32_t *xcnt, const uint64_t *plut,
                             uint64_t *xsums = nullptr);   // xsums: moves into a final-sums copy (move_row_sums)
hipError_t launch_update(hipStream_t s, uint32_t Dp, uint32_t G, const uint8_t *codes, uint64_t N, const uint32_t *A,
                         uint32_t K, uint32_t D, const uint64_t *plut, uint64_t *part, uint32_t *part_cnt);
// Sums of a final assignment straight into sums [hi KD][lo KD][cnt K] (no slabs, no reduce)
// through a counting sort of the rows by index: hist [G][K], scratch 2K + 1, idx / ks [N].
bool sorted_sums_fits(uint32_t K);
hipError_t launch_sorted_sums(hipStream_t s, uint32_t Dp, uint32_t G, const uint8_t *codes, uint64_t N,
                              const uint32_t *A, uint32_t K, uint32_t D, const uint64_t *plut, uint32_t *hist,
                              uint32_t *scratch, uint32_t *idx, uint32_t *ks, uint64_t *sums);
// A counter published to mapped host memory by a kernel: *dst = *cnt, then *flag = seq
// (flag null: nothing).
struct PubArgs {
    const unsigned *cnt = nullptr;
    uint32_t *dst = nullptr;
    uint64_t *flag = nullptr;
    uint64_t seq = 0;
};
// Sums of G slabs, the last nsub of them subtracted (fused path: slab G + 1 holds the terms
// of re-assigned rows at their provisional index).  pub: a tie count to publish first.
hipError_t launch_reduce(hipStream_t s, const uint64_t *part, const uint32_t *part_cnt, uint32_t G, uint32_t nsub,
                         uint32_t K, uint32_t D, uint64_t *sums, PubArgs pub = PubArgs());
// Up to three device ranges (sizes multiples of 4 bytes, 0 = unused) copied in one launch,
// e.g. into mapped pinned host memory; with flag (mapped) the copy then publishes *flag = seq
// (done: a block counter at 0, left at 0).
hipError_t launch_copy_out(hipStream_t s, const void *src0, void *dst0, uint64_t bytes0, const void *src1, void *dst1,
                           uint64_t bytes1, const void *src2, void *dst2, uint64_t bytes2, uint64_t *flag = nullptr,
                           uint64_t seq = 0, unsigned *done = nullptr);
// Mean sums (K = 1): block b adds into copy b mod MEAN_COPIES of [hi D][lo D][n] (stride
// 2D + 1; n in copy 0 only), so the blocks' closing atomics spread over MEAN_COPIES addresses
// per component; the K = 1 finalize adds the copies.  Also clears zero[0..n_zero) and sets
// dist[0] = sum ||x||^2 and dist[1] = rows from the byte histogram hist (values v64).
constexpr uint32_t MEAN_COPIES = 8;
hipError_t launch_mean_sums(hipStream_t s, uint32_t Dp, const uint8_t *codes, uint64_t N, uint32_t D,
                            const uint64_t *plut, uint64_t *sums, unsigned *zero, uint32_t n_zero, double *dist,
                            const uint64_t *hist, const double *v64);
// Centroids of the reduced sums (C_cent [K][D]); with split also the next level's K' = 2K
// code vectors (C64n and, if host_cb, mapped host memory) and their search tables (see
// launch_prep) padded to Kpad_next; without split, given dist_out, dist_out[0] =
// sum_k (2 c_k.S_k - n_k ||c_k||^2) (closed-form distortion).  With done (a counter at 0,
// left at 0) the last block also publishes *ready = seq in mapped host memory; dist_part
// holds the per-block partials (<= 8000).
// The level's tie rows exported with the codebook (the speculative Kahan check, engine.cpp):
// out (mapped host memory) = [u32 count][u32 pad] then per row [u32 row][u32 A[row]][Dp code
// bytes], the first cap rows; released with the ready flag.
struct TieExport {
    const uint32_t *rows = nullptr;
    const unsigned *cnt = nullptr;
    const uint32_t *A = nullptr;
    const uint8_t *codes = nullptr;
    uint32_t cap = 0;
    uint64_t n_rows = 0;   // rows in codes / A (a row index past it is written as ~0, nothing read)
    uint8_t *out = nullptr;
};
hipError_t launch_finalize_prep(hipStream_t s, const uint64_t *sums, uint32_t K, uint32_t D, uint32_t Dp, int64_t R,
                                int64_t bias, int scale, double *C_cent, bool split, double *C64n, uint32_t Kpad_next,
                                double mu, double sx, int t, float *C32, _Float16 *cb_rows, float *E32,
                                double *host_cb, double *dist_part, unsigned *done, double *dist_out, uint64_t *ready, uint64_t seq,
                                bool zero_sums, uint32_t ncopy = 1, uint32_t *perm = nullptr, int32_t *tint = nullptr,
                                uint32_t zero_skip = 0, uint64_t copy_stride = 0, const unsigned *copy_gate = nullptr,
                                const TieExport &ties = TieExport());
// (zero_sums: clears copies zero_skip .. ncopy - 1; copy_stride 0: the copies follow each other,
// 2KD + K apart; copy_gate: copies past the first are read and cleared only if *copy_gate != 0)
hipError_t launch_finalize(hipStream_t s, const uint64_t *sums, uint32_t K, uint32_t D, int64_t R, int64_t bias,
                           int scale, double *C_cent);
// f16 MFMA tables (D = 12) and fp32 VALU table from an fp64 codebook of K code vectors.
// With E32 (D = 12) also the expanded fp32 table of launch_assign_mfma.
hipError_t launch_prep(hipStream_t s, const double *C64, uint32_t K, uint32_t Kpad, uint32_t D, uint32_t Dp,
                       double mu, double sx, int t, float *C32, _Float16 *cb_rows, float *E32);
hipError_t launch_gather_codes(hipStream_t s, const uint8_t *codes, uint32_t Dp, const uint32_t *rows, uint32_t n,
                               uint8_t *out);
// Host-resolved rows: A[rows[i]] = vals[i]; with xslab their terms move from the
// provisional index (A before) to the new one (move_row_terms).
hipError_t launch_fix_rows(hipStream_t s, const uint8_t *codes, uint32_t Dp, uint32_t D, uint32_t *A,
                           const uint32_t *rows, const uint32_t *vals, uint32_t n, uint32_t K, uint64_t *xslab,
                           uint32_t *xcnt, const uint64_t *plut, uint64_t *xsums = nullptr);
// 256-bin histogram of the first D bytes of every row (hist zeroed first).
hipError_t launch_byte_hist(hipStream_t s, const uint8_t *codes, uint64_t N, uint32_t D, uint32_t Dp,
                            uint64_t *hist);
// Exact mode (k_exact.hip): fp64 rows X [N][D].
hipError_t launch_exact_assign(hipStream_t s, const double *X, uint64_t N, uint32_t D, const double *C, uint32_t K,
                               double tie_rel, uint32_t *A, uint32_t *ties, unsigned *tie_cnt);
size_t exact_sort_temp_bytes(uint64_t N);
hipError_t launch_exact_iota(hipStream_t s, uint32_t *v, uint64_t N);
// Kahan centroids of assignment A (nullptr: the mean of all rows, K = 1) into C [K][D] and
// counts cnt [K] (may be null); keys_out / order [N], koff [K + 1] and temp are scratch.
hipError_t launch_exact_centroids(hipStream_t s, const double *X, uint64_t N, uint32_t D, const uint32_t *A, uint32_t K,
                                  uint32_t *keys_out, uint32_t *iota, uint32_t *order, uint32_t *koff, void *temp,
                                  size_t temp_bytes, double *C, uint64_t *cnt);
hipError_t launch_exact_distortion(hipStream_t s, const double *X, uint64_t N, uint32_t D, const double *C,
                                   const uint32_t *A, double *part, double *out);
hipError_t launch_exact_gather(hipStream_t s, const double *X, uint32_t D, const uint32_t *rows, uint32_t n,
                               double *out);
hipError_t launch_exact_fix(hipStream_t s, uint32_t *A, const uint32_t *rows, const uint32_t *vals, uint32_t n);
// The reference's Kahan centroids on the device (k_kahan.hip, kahan_par.hpp): scratch for one
// computation over N rows and up to k_cap cells (sizes from KahanWork::caps).
struct KahanWork {
    uint32_t *hist = nullptr;          // [G][K] sort histograms (G = sort_blocks(N))
    uint32_t *tot = nullptr;           // [K] rows per cell
    uint32_t *koff = nullptr, *segoff = nullptr, *blkoff = nullptr;   // [K + 1] each
    uint8_t *planes = nullptr;         // [D][plane_len(N)]: the chains' bytes, component-major
    void *meta = nullptr;              // [D][seg_cap] segment metadata
    void *bsum = nullptr;              // [D][blk_cap] 128-bit block totals, then prefixes
    void *bfn = nullptr;               // [D][blk_cap] block functions
    void *sfn = nullptr;               // [D][seg_cap] segment functions
    void *bfn8 = nullptr;              // [D][blk_cap][8] 8-segment sub-block functions
    void *tab = nullptr;               // the byte table (kahan::ByteTab)
    unsigned *stats = nullptr;         // [4] blocks not composable, block misses, segment replays
    uint32_t n_one = 0;                // K = 1: N (the mean's single cell)
    uint64_t seg_cap = 0, blk_cap = 0, n_cap = 0;
    uint32_t k_cap = 0, d_cap = 0;
    static size_t tab_bytes();
    static void make_tab(const uint64_t *X, void *out);
    static void caps(uint64_t N, uint32_t K, uint64_t &segs, uint64_t &blks);
    static uint64_t plane_len(uint64_t N);
    static size_t meta_bytes();
    static size_t fn_bytes();
    static size_t segfn_bytes();
    static uint32_t sort_blocks(uint64_t N);
};
// C [K][D] = the reference's centroids of assignment A (nullptr: K = 1, the mean of every row):
// Kahan sums in ascending row order times fl(1/n), empty cells 0, bit for bit (SCALED byte
// values; w.tab from KahanWork::make_tab).  With split_out also the split [2K][D] (x1.2 | x0.8).
// sel (n_sel entries, device; nullptr: every cell): the selected cells only, compacted: sel[a] =
// slot + 1 for a selected cell a, 0 otherwise; K is then the number of slots, and C / split_out
// rows are slots (split_out: slot | K + slot).  The sort skips the other rows' bytes.
// max_rows: a bound on the rows of any cell summed (0: unknown); at most kahan_direct_max()
// rows, each chain runs step by step on one lane (ks_direct_kernel) instead of through the
// segment functions, whose set-up costs more than short chains.
hipError_t launch_kahan_centroids(hipStream_t s, const KahanWork &w, const uint8_t *codes, uint32_t Dp, uint32_t D,
                                  uint64_t N, const uint32_t *A, uint32_t K, double *C, double *split_out,
                                  const uint32_t *sel = nullptr, uint32_t n_sel = 0, uint64_t max_rows = 0);
uint64_t kahan_direct_max();   // QVQ_KAHAN_DIRECT_MAX (default 4096; 0: never)
// The same centroids when a cell's rows are split over ranks (each rank holds a contiguous
// range of the global rows, ranks in row order; engine.cpp kahan_chained).  gather: u64
// [nranks][K * D][2] chain totals | [nranks][K] row counts, zeroed by the caller; each rank
// writes its slice (chain_local) and the caller sums gather over the ranks (an all-gather);
// chain_build then takes each chain's exact prefix from the lower ranks' totals.  state: u64
// [K * D][2], the reference's (sum, c) bits: chain_eval (once per rank, in rank order, each from
// the previous rank's output; rank 0 from zeros) advances it over this rank's rows; chain_finish
// divides by the global row count (C [K][D], split_out [2K][D] as launch_kahan_centroids).
hipError_t launch_kahan_chain_local(hipStream_t s, const KahanWork &w, const uint8_t *codes, uint32_t Dp, uint32_t D,
                                    uint64_t N, const uint32_t *A, uint32_t K, const uint32_t *sel, uint32_t n_sel,
                                    uint64_t *gather, uint32_t rank, uint32_t nranks);
hipError_t launch_kahan_chain_build(hipStream_t s, const KahanWork &w, uint32_t D, uint64_t N, uint32_t K,
                                    const uint64_t *gather, uint32_t rank);
hipError_t launch_kahan_chain_eval(hipStream_t s, const KahanWork &w, uint32_t D, uint64_t N, uint32_t K,
                                   uint64_t *state, const uint64_t *gather, uint32_t rank);
hipError_t launch_kahan_chain_finish(hipStream_t s, uint32_t D, uint32_t K, const uint64_t *state,
                                     const uint64_t *gather, uint32_t nranks, double *C, double *split_out);
}  // namespace qvq
