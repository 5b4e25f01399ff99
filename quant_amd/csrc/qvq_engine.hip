// qvq_engine.hip -- MI355X (gfx950) LBG vector-quantization engine behind the C ABI of
// include/qvq.h.
//
// Hot path (reference: src/Quantizer.cpp:122-143, one Lloyd step per split level):
//   tile      raw u8 raster -> per-block byte codes [N][Dp]            (Compressor.cpp:31-62)
//   assign    fp32 brute-force L2 argmin, codebook staged in LDS, best + second best per
//             row, rows whose fp32 gap is inside a rigorous error bound are flagged
//                                                                      (Quantizer.cpp:24-32)
//   recheck   flagged rows only: fp64 distances in the reference build's association;
//             rows whose fp64 gap is ~0 go to the host kd-tree resolver (kdtree.cpp)
//   update    exact per-code-vector sums: LDS u64 atomics of (hi<<32 | lo) byte terms,
//             per-workgroup slabs, column reduce                      (Quantizer.cpp:59-87)
//   finalize  centroid = round(exact sum) * fl(1/count), then split x1.2 / x0.8
//                                                                      (Quantizer.cpp:134-138)
//   [RCCL all-reduce of the sums between update and finalize when ranks > 1]
//
// Everything runs on one HIP stream; the host synchronises once per level to learn how
// many rows need the kd-tree (almost always zero).
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <string>
#include <vector>

#include "kdtree.hpp"
#include "qvq.h"

namespace qvq {

// ---------------------------------------------------------------------------------------
// Exact-sum decomposition of a colour space's byte -> value map.
// Every value v[b] is an integer multiple of 2^-scale: q[b] = v[b] * 2^scale.  We write
// q[b] = R * hi[b] + (lo[b] - bias) with hi[b] <= 255 and 0 <= lo[b] <= 2*bias small, so one
// u64 LDS atomic of (hi << 32 | lo) per component accumulates both parts without carries
// for up to 2^24 rows per workgroup; the finaliser rebuilds the exact 128-bit sum.
// ---------------------------------------------------------------------------------------
struct Terms {
    double v64[256];
    float v32[256];
    uint32_t hi[256];
    uint32_t lo[256];
    int64_t R;
    int64_t bias;
    int scale;
    uint8_t pad_code;   // byte whose value is exactly 0.0 (padding past the raster end)
    double vmax;        // max |v|
};

// src/ColorSpace.cpp:4-6 (NORMAL) and :16-21 (SCALED, reciprocal multiply under fast-math)
static double cs_value(int cs, int b) {
    const double s = (double)(signed char)(unsigned char)b;
    return cs == QVQ_CS_NORMAL ? s : (s + 128.0) * (1.0 / 255);
}

static bool make_terms(int cs, Terms &t) {
    if (cs != QVQ_CS_NORMAL && cs != QVQ_CS_SCALED) return false;
    t.scale = cs == QVQ_CS_SCALED ? 60 : 0;
    t.vmax = 0;
    for (int b = 0; b < 256; b++) {
        t.v64[b] = cs_value(cs, b);
        t.v32[b] = (float)t.v64[b];
        t.vmax = std::max(t.vmax, std::fabs(t.v64[b]));
    }
    // u = (int8)b + 128 orders the bytes by value; q = R*u + E with |E| small.
    t.R = cs == QVQ_CS_SCALED ? (int64_t)std::ldexp(1.0 / 255, 60) : 1;
    const int64_t off = cs == QVQ_CS_SCALED ? 0 : -128;
    int64_t E[256], emax = 0;
    for (int b = 0; b < 256; b++) {
        const double qd = std::ldexp(t.v64[b], t.scale);
        if (qd != std::floor(qd)) return false;
        const int64_t q = (int64_t)qd;
        const int64_t u = (int64_t)(signed char)(unsigned char)b + 128;
        E[b] = q - t.R * u;   // includes the constant offset for NORMAL
        (void)off;
        emax = std::max<int64_t>(emax, E[b] < 0 ? -E[b] : E[b]);
        t.hi[b] = (uint32_t)u;
    }
    t.bias = emax;
    for (int b = 0; b < 256; b++) t.lo[b] = (uint32_t)(E[b] + t.bias);
    t.pad_code = cs == QVQ_CS_SCALED ? 0x80 : 0x00;
    return t.v64[t.pad_code] == 0.0;
}

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
    const int nbits = 128 - lz;
    const int sh = nbits - 53;
    uint64_t top = (uint64_t)(m >> sh);
    const unsigned __int128 rem = m & (((unsigned __int128)1 << sh) - 1);
    const unsigned __int128 half = (unsigned __int128)1 << (sh - 1);
    if (rem > half || (rem == half && (top & 1))) top++;
    const double d = ldexp((double)top, sh);
    return neg ? -d : d;
}

// Centroid component from reduced sums: round(R*hi + lo - bias*cnt) * 2^-scale * fl(1/cnt).
__host__ __device__ inline double centroid_value(uint64_t hi, uint64_t lo, uint64_t cnt, int64_t R, int64_t bias,
                                                 int scale) {
    if (cnt == 0) return 0.0;   // empty cell -> zero vector (src/Quantizer.cpp:81-85)
    const __int128 S = (__int128)R * (__int128)hi + (__int128)lo - (__int128)bias * (__int128)cnt;
    return ldexp(i128_to_double(S), -scale) * (1.0 / (double)cnt);
}

// The reference build's nanoflann distance (see kdtree.hpp): must match ref_l2 bit for bit.
__device__ inline double ref_l2_dev(const double *a, const double *b, int dim) {
    double r = 0;
    int d = 0;
    for (; d + 3 < dim; d += 4) {
        const double e0 = a[d] - b[d], e1 = a[d + 1] - b[d + 1];
        const double e2 = a[d + 2] - b[d + 2], e3 = a[d + 3] - b[d + 3];
        r += (e1 * e1 + e2 * e2) + (e0 * e0 + e3 * e3);
    }
    for (; d < dim; d++) {
        const double e = a[d] - b[d];
        r += e * e;
    }
    return r;
}

// ---------------------------------------------------------------------------------------
// Kernels
// ---------------------------------------------------------------------------------------
__device__ inline uint64_t splitmix64(uint64_t z) {
    z += 0x9E3779B97F4A7C15ULL;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
    return z ^ (z >> 31);
}

// Synthetic S x S rasters; image i uses seed0 + i.  One thread per pixel.
__global__ void gen_kernel(uint8_t *__restrict__ rgb, uint32_t S, uint64_t seed0, uint64_t npix_total) {
    const uint64_t S2 = (uint64_t)S * S;
    for (uint64_t g = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; g < npix_total;
         g += (uint64_t)gridDim.x * blockDim.x) {
        const uint64_t img = g / S2, p = g - img * S2;
        const uint64_t r = p / S, c = p - r * S;
        const uint64_t seed = seed0 + img;
        const int64_t sm[3] = {(int64_t)(r * 255 / (S - 1)), (int64_t)(c * 255 / (S - 1)),
                               (int64_t)((r + c) * 255 / (2 * (uint64_t)(S - 1)))};
#pragma unroll
        for (int ch = 0; ch < 3; ch++) {
            const uint64_t h = splitmix64((seed << 40) ^ (p * 3 + ch));
            int64_t v = sm[ch] + (int64_t)(h % 33) - 16;
            v = v < 0 ? 0 : (v > 255 ? 255 : v);
            rgb[g * 3 + ch] = (uint8_t)v;
        }
    }
}

// getBlocksAsVectorsFromImage (src/Compressor.cpp:31-62) over n_images rasters, writing
// each block's raw bytes (component order (x*h + y)*3 + c) into codes[g][0..D), padding
// [D, Dp) with the zero-valued byte.  One thread per block.
__global__ void tile_kernel(const uint8_t *__restrict__ rgb, uint8_t *__restrict__ codes, uint32_t n_images,
                            uint32_t xSize, uint32_t ySize, uint32_t bw, uint32_t bh, uint32_t D, uint32_t Dp,
                            uint8_t pad) {
    const uint64_t wB = (xSize + bw - 1) / bw, hB = (ySize + bh - 1) / bh, nb = wB * hB;
    const uint64_t total = (uint64_t)xSize * ySize;
    const uint64_t nall = nb * n_images;
    for (uint64_t g = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; g < nall;
         g += (uint64_t)gridDim.x * blockDim.x) {
        const uint64_t img = g / nb, b = g - img * nb;
        const uint64_t i = b / hB, j = b - i * hB;
        const uint8_t *src = rgb + img * total * 3;
        uint8_t *dst = codes + g * Dp;
        for (uint64_t x = i * bw; x < i * bw + bw; x++)
            for (uint64_t y = j * bh; y < j * bh + bh; y++) {
                const uint64_t imgIndex = x * ySize + y;
                const uint64_t vec = ((x - i * bw) * bh + (y - j * bh)) * 3;
                for (int c = 0; c < 3; c++) dst[vec + c] = imgIndex < total ? src[imgIndex * 3 + c] : pad;
            }
        for (uint32_t d = D; d < Dp; d++) dst[d] = pad;
    }
}

constexpr int ASSIGN_THREADS = 256;
constexpr int ASSIGN_LDS_BYTES = 64 * 1024;

template <int DP>
struct AssignCfg {
    static constexpr int R = DP <= 16 ? 4 : (DP <= 48 ? 2 : 1);   // rows per thread
};

// Nearest code vector, fp32.  Each thread keeps R rows in registers, the codebook is
// staged in LDS (whole when it fits, else in tiles) and read by broadcast.  Per row we
// keep the best and second-best distance; if their gap is inside the fp32 error bound
// 2*(alpha*sqrt(d2) + beta*d2) + gamma the row is flagged for the fp64 recheck.
template <int DP>
__global__ __launch_bounds__(ASSIGN_THREADS) void assign_kernel(
    const uint8_t *__restrict__ codes, uint64_t N, const float *__restrict__ C32, uint32_t K, uint32_t KT,
    const float *__restrict__ lut32, float alpha, float beta, float gamma, uint32_t *__restrict__ A,
    uint32_t *__restrict__ flags, unsigned int *__restrict__ flag_cnt) {
    constexpr int R = AssignCfg<DP>::R;
    constexpr int D4 = DP / 4;
    extern __shared__ __attribute__((aligned(16))) float smem[];
    float *lut = smem;                 // 256
    float *cb = smem + 256;            // KT x DP
    const int tid = threadIdx.x;
    lut[tid] = lut32[tid];             // blockDim == 256
    const bool whole = K <= KT;
    if (whole) {
        const float4 *src = reinterpret_cast<const float4 *>(C32);
        float4 *dst = reinterpret_cast<float4 *>(cb);
        for (uint32_t i = tid; i < K * D4; i += ASSIGN_THREADS) dst[i] = src[i];
    }
    __syncthreads();
    const uint64_t rows_per_block = (uint64_t)ASSIGN_THREADS * R;
    const uint64_t nchunks = (N + rows_per_block - 1) / rows_per_block;
    for (uint64_t chunk = blockIdx.x; chunk < nchunks; chunk += gridDim.x) {
        float x[R][DP];
        uint64_t row[R];
#pragma unroll
        for (int r = 0; r < R; r++) {
            row[r] = chunk * rows_per_block + (uint64_t)r * ASSIGN_THREADS + tid;
            if (row[r] < N) {
                const uint32_t *w = reinterpret_cast<const uint32_t *>(codes + row[r] * DP);
#pragma unroll
                for (int q = 0; q < D4; q++) {
                    const uint32_t v = w[q];
                    x[r][4 * q + 0] = lut[v & 0xFF];
                    x[r][4 * q + 1] = lut[(v >> 8) & 0xFF];
                    x[r][4 * q + 2] = lut[(v >> 16) & 0xFF];
                    x[r][4 * q + 3] = lut[v >> 24];
                }
            } else {
#pragma unroll
                for (int d = 0; d < DP; d++) x[r][d] = 0.f;
            }
        }
        float b1[R], b2[R];
        uint32_t bi[R];
#pragma unroll
        for (int r = 0; r < R; r++) {
            b1[r] = INFINITY;
            b2[r] = INFINITY;
            bi[r] = 0;
        }
        for (uint32_t k0 = 0; k0 < K; k0 += KT) {
            const uint32_t kn = min(KT, K - k0);
            if (!whole) {
                __syncthreads();
                const float4 *src = reinterpret_cast<const float4 *>(C32 + (uint64_t)k0 * DP);
                float4 *dst = reinterpret_cast<float4 *>(cb);
                for (uint32_t i = tid; i < kn * D4; i += ASSIGN_THREADS) dst[i] = src[i];
                __syncthreads();
            }
            for (uint32_t kk = 0; kk < kn; kk++) {
                const float4 *c4 = reinterpret_cast<const float4 *>(cb + kk * DP);
                float acc[R];
#pragma unroll
                for (int r = 0; r < R; r++) acc[r] = 0.f;
#pragma unroll
                for (int q = 0; q < D4; q++) {
                    const float4 c = c4[q];
#pragma unroll
                    for (int r = 0; r < R; r++) {
                        float t;
                        t = x[r][4 * q + 0] - c.x; acc[r] = __fmaf_rn(t, t, acc[r]);
                        t = x[r][4 * q + 1] - c.y; acc[r] = __fmaf_rn(t, t, acc[r]);
                        t = x[r][4 * q + 2] - c.z; acc[r] = __fmaf_rn(t, t, acc[r]);
                        t = x[r][4 * q + 3] - c.w; acc[r] = __fmaf_rn(t, t, acc[r]);
                    }
                }
                const uint32_t k = k0 + kk;
#pragma unroll
                for (int r = 0; r < R; r++) {
                    b2[r] = __builtin_amdgcn_fmed3f(b1[r], b2[r], acc[r]);
                    bi[r] = acc[r] < b1[r] ? k : bi[r];
                    b1[r] = fminf(b1[r], acc[r]);
                }
            }
        }
#pragma unroll
        for (int r = 0; r < R; r++) {
            if (row[r] < N) {
                A[row[r]] = bi[r];
                const float thr = 2.f * (alpha * sqrtf(b2[r]) + beta * b2[r]) + gamma;
                if (!(b2[r] - b1[r] > thr)) flags[atomicAdd(flag_cnt, 1u)] = (uint32_t)row[r];
            }
        }
    }
}

// fp64 recheck of flagged rows: one wave per row, lanes stride over the codebook.  The
// row gets the fp64 argmin (lowest index among exact ties); if the two best fp64
// distances are within tie_rel (relative) the row is handed to the host kd-tree.
constexpr int RECHECK_THREADS = 256;
__global__ __launch_bounds__(RECHECK_THREADS) void recheck_kernel(
    const uint8_t *__restrict__ codes, uint32_t Dp, uint32_t D, const uint32_t *__restrict__ flags,
    const unsigned int *__restrict__ flag_cnt, const double *__restrict__ C64, uint32_t K,
    const double *__restrict__ lut64, double tie_rel, uint32_t *__restrict__ A, uint32_t *__restrict__ ties,
    unsigned int *__restrict__ tie_cnt) {
    __shared__ double xs[RECHECK_THREADS / 64][64];
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const unsigned nflag = *flag_cnt;
    for (unsigned base = blockIdx.x * (RECHECK_THREADS / 64); base < nflag;
         base += gridDim.x * (RECHECK_THREADS / 64)) {
        const unsigned f = base + wave;
        const bool active = f < nflag;
        const uint32_t row = active ? flags[f] : 0;
        __syncthreads();
        if (active && lane < (int)D) xs[wave][lane] = lut64[codes[(uint64_t)row * Dp + lane]];
        __syncthreads();
        if (!active) continue;
        double d1 = INFINITY, d2 = INFINITY;
        uint32_t k1 = 0xFFFFFFFFu;
        for (uint32_t k = lane; k < K; k += 64) {
            const double d = ref_l2_dev(xs[wave], C64 + (uint64_t)k * D, D);
            if (d < d1) {
                d2 = d1;
                d1 = d;
                k1 = k;
            } else if (d < d2) {
                d2 = d;
            }
        }
#pragma unroll
        for (int off = 32; off >= 1; off >>= 1) {
            const double od1 = __shfl_xor(d1, off);
            const double od2 = __shfl_xor(d2, off);
            const uint32_t ok1 = __shfl_xor(k1, off);
            if (od1 < d1 || (od1 == d1 && ok1 < k1)) {
                d2 = fmin(od2, d1);
                d1 = od1;
                k1 = ok1;
            } else {
                d2 = fmin(d2, od1);
            }
        }
        if (lane == 0) {
            A[row] = k1;
            if (d2 - d1 <= tie_rel * d1) ties[atomicAdd(tie_cnt, 1u)] = row;
        }
    }
}

// Exact per-code-vector sums of the rows (A == nullptr: every row belongs to code 0, the
// mean initialisation).  Grid (G, passes): workgroup g folds its contiguous row range into
// LDS for code vectors [k0, k0 + KR), then writes one slab of packed partials.
constexpr int UPDATE_THREADS = 1024;
template <int DP>
__global__ __launch_bounds__(UPDATE_THREADS) void update_kernel(
    const uint8_t *__restrict__ codes, uint64_t N, const uint32_t *__restrict__ A, uint32_t K, uint32_t KR,
    uint32_t D, uint64_t rows_per_group, const uint64_t *__restrict__ plut, uint64_t *__restrict__ part,
    uint32_t *__restrict__ part_cnt) {
    extern __shared__ __attribute__((aligned(16))) uint64_t lsum[];   // [KR*D] then cnt (u32) then lut
    const uint32_t k0 = blockIdx.y * KR;
    const uint32_t kr = min(KR, K - k0);
    uint32_t *lcnt = reinterpret_cast<uint32_t *>(lsum + (uint64_t)KR * D);
    uint64_t *llut = lsum + (uint64_t)KR * D + (KR + 1) / 2;
    const int tid = threadIdx.x;
    for (uint32_t i = tid; i < kr * D; i += UPDATE_THREADS) lsum[i] = 0;
    for (uint32_t i = tid; i < kr; i += UPDATE_THREADS) lcnt[i] = 0;
    for (int i = tid; i < 256; i += UPDATE_THREADS) llut[i] = plut[i];
    __syncthreads();
    const uint64_t start = blockIdx.x * rows_per_group;
    const uint64_t end = min(N, start + rows_per_group);
    for (uint64_t row = start + tid; row < end; row += UPDATE_THREADS) {
        const uint32_t k = A ? A[row] : 0u;
        const uint32_t kl = k - k0;
        if (kl < kr) {
            const uint32_t *w = reinterpret_cast<const uint32_t *>(codes + row * DP);
            uint64_t *dst = lsum + (uint64_t)kl * D;
#pragma unroll
            for (int q = 0; q < DP / 4; q++) {
                const uint32_t v = w[q];
#pragma unroll
                for (int j = 0; j < 4; j++)
                    if (4 * q + j < (int)D) atomicAdd((unsigned long long *)&dst[4 * q + j], (unsigned long long)llut[(v >> (8 * j)) & 0xFF]);
            }
            atomicAdd(&lcnt[kl], 1u);
        }
    }
    __syncthreads();
    uint64_t *pdst = part + ((uint64_t)blockIdx.x * K + k0) * D;
    for (uint32_t i = tid; i < kr * D; i += UPDATE_THREADS) pdst[i] = lsum[i];
    uint32_t *cdst = part_cnt + (uint64_t)blockIdx.x * K + k0;
    for (uint32_t i = tid; i < kr; i += UPDATE_THREADS) cdst[i] = lcnt[i];
}

// Column reduce of the G slabs into sums = [hi K*D][lo K*D][cnt K] (u64).
__global__ void reduce_kernel(const uint64_t *__restrict__ part, const uint32_t *__restrict__ part_cnt, uint32_t G,
                              uint32_t K, uint32_t D, uint64_t *__restrict__ sums) {
    const uint64_t KD = (uint64_t)K * D;
    for (uint64_t c = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; c < KD + K;
         c += (uint64_t)gridDim.x * blockDim.x) {
        if (c < KD) {
            uint64_t hi = 0, lo = 0;
            for (uint32_t g = 0; g < G; g++) {
                const uint64_t p = part[g * KD + c];
                hi += p >> 32;
                lo += p & 0xFFFFFFFFull;
            }
            sums[c] = hi;
            sums[KD + c] = lo;
        } else {
            const uint64_t k = c - KD;
            uint64_t n = 0;
            for (uint32_t g = 0; g < G; g++) n += part_cnt[g * (uint64_t)K + k];
            sums[2 * KD + k] = n;
        }
    }
}

// Centroids from the reduced sums; optionally the next level's split codebook
// (src/Quantizer.cpp:134-138: concat, then x(1+0.2) and x(1-0.2)) in fp64 and fp32.
__global__ void finalize_kernel(const uint64_t *__restrict__ sums, uint32_t K, uint32_t D, uint32_t Dp, int64_t R,
                                int64_t bias, int scale, double *__restrict__ C_cent, int split,
                                double *__restrict__ C64n, float *__restrict__ C32n) {
    const uint64_t KD = (uint64_t)K * D;
    for (uint64_t t = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; t < (uint64_t)K * Dp;
         t += (uint64_t)gridDim.x * blockDim.x) {
        const uint64_t k = t / Dp, d = t - k * Dp;
        if (d < D) {
            const uint64_t c = k * D + d;
            const double v = centroid_value(sums[c], sums[KD + c], sums[2 * KD + k], R, bias, scale);
            C_cent[c] = v;
            if (split) {
                const double a = v * (double)(1 + 0.2), b = v * (double)(1 - 0.2);
                C64n[c] = a;
                C64n[KD + c] = b;
                C32n[k * Dp + d] = (float)a;
                C32n[(k + K) * Dp + d] = (float)b;
            }
        } else if (split) {
            C32n[k * Dp + d] = 0.f;
            C32n[(k + K) * Dp + d] = 0.f;
        }
    }
}

// out[i] = codes of row rows[i] (the rows the host kd-tree resolves).
__global__ void gather_codes_kernel(const uint8_t *__restrict__ codes, uint32_t Dp, const uint32_t *__restrict__ rows,
                                    uint32_t n, uint8_t *__restrict__ out) {
    for (uint64_t t = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; t < (uint64_t)n * Dp;
         t += (uint64_t)gridDim.x * blockDim.x) {
        const uint64_t i = t / Dp, d = t - i * Dp;
        out[t] = codes[(uint64_t)rows[i] * Dp + d];
    }
}

// A[rows[i]] = vals[i] (host tie resolutions).
__global__ void scatter_kernel(uint32_t *__restrict__ A, const uint32_t *__restrict__ rows,
                               const uint32_t *__restrict__ vals, uint32_t n) {
    for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) A[rows[i]] = vals[i];
}

// Sum over rows of norm(x - c_A(x)) (src/Quantizer.cpp:9-22), one partial per workgroup.
constexpr int DIST_THREADS = 256;
__global__ __launch_bounds__(DIST_THREADS) void distortion_kernel(
    const uint8_t *__restrict__ codes, uint64_t N, uint32_t D, uint32_t Dp, const uint32_t *__restrict__ A,
    const double *__restrict__ C, const double *__restrict__ lut64, double *__restrict__ partial) {
    __shared__ double red[DIST_THREADS];
    double s = 0;
    for (uint64_t row = blockIdx.x * (uint64_t)DIST_THREADS + threadIdx.x; row < N;
         row += (uint64_t)gridDim.x * DIST_THREADS) {
        const double *c = C + (uint64_t)A[row] * D;
        const uint8_t *x = codes + row * Dp;
        double r = 0;
        for (uint32_t d = 0; d < D; d++) {
            const double e = lut64[x[d]] - c[d];
            r += e * e;
        }
        s += r;
    }
    red[threadIdx.x] = s;
    __syncthreads();
    for (int w = DIST_THREADS / 2; w > 0; w >>= 1) {
        if ((int)threadIdx.x < w) red[threadIdx.x] += red[threadIdx.x + w];
        __syncthreads();
    }
    if (threadIdx.x == 0) partial[blockIdx.x] = red[0];
}

// ---------------------------------------------------------------------------------------
// Kernel dispatch over Dp (multiples of 4 up to 64).
// ---------------------------------------------------------------------------------------
#define QVQ_FOR_EACH_DP(X) X(4) X(8) X(12) X(16) X(20) X(24) X(28) X(32) X(36) X(40) X(44) X(48) X(52) X(56) X(60) X(64)

static uint32_t assign_rows_per_thread(uint32_t Dp) {
    switch (Dp) {
#define X(DPV) case DPV: return AssignCfg<DPV>::R;
        QVQ_FOR_EACH_DP(X)
#undef X
    }
    return 1;
}

static hipError_t launch_assign(uint32_t Dp, int grid, size_t lds, hipStream_t s, const uint8_t *codes, uint64_t N,
                                const float *C32, uint32_t K, uint32_t KT, const float *lut32, float alpha, float beta,
                                float gamma, uint32_t *A, uint32_t *flags, unsigned *flag_cnt) {
    switch (Dp) {
#define X(DPV)                                                                                                   \
    case DPV:                                                                                                    \
        hipLaunchKernelGGL(assign_kernel<DPV>, dim3(grid), dim3(ASSIGN_THREADS), lds, s, codes, N, C32, K, KT,  \
                           lut32, alpha, beta, gamma, A, flags, flag_cnt);                                       \
        return hipGetLastError();
        QVQ_FOR_EACH_DP(X)
#undef X
    }
    return hipErrorInvalidValue;
}

static hipError_t launch_update(uint32_t Dp, dim3 grid, size_t lds, hipStream_t s, const uint8_t *codes, uint64_t N,
                                const uint32_t *A, uint32_t K, uint32_t KR, uint32_t D, uint64_t rows_per_group,
                                const uint64_t *plut, uint64_t *part, uint32_t *part_cnt) {
    switch (Dp) {
#define X(DPV)                                                                                                     \
    case DPV:                                                                                                      \
        hipLaunchKernelGGL(update_kernel<DPV>, grid, dim3(UPDATE_THREADS), lds, s, codes, N, A, K, KR, D,          \
                           rows_per_group, plut, part, part_cnt);                                                  \
        return hipGetLastError();
        QVQ_FOR_EACH_DP(X)
#undef X
    }
    return hipErrorInvalidValue;
}

}  // namespace qvq

// =======================================================================================
// Context and C ABI
// =======================================================================================
using namespace qvq;

struct qvq_ctx {
    int dev = 0;
    int num_cu = 256;
    hipStream_t stream = nullptr;
    std::string err;

    // training set
    uint64_t N = 0;
    uint32_t D = 0, Dp = 0;
    int cs = -1;
    Terms terms;
    uint8_t *d_codes = nullptr;
    float *d_lut32 = nullptr;
    double *d_lut64 = nullptr;
    uint64_t *d_plut = nullptr;
    uint32_t *d_A = nullptr, *d_flags = nullptr, *d_ties = nullptr;
    unsigned *d_counters = nullptr;   // [0] flags, [1] ties

    // level buffers
    uint32_t Kcap = 0;
    uint32_t G = 0;   // update row groups
    double *d_C64_cent = nullptr, *d_C64_split = nullptr;
    float *d_C32_split = nullptr;
    uint64_t *d_part = nullptr, *d_sums = nullptr;
    uint32_t *d_part_cnt = nullptr;
    double *d_dist_part = nullptr;
    uint32_t *d_scatter = nullptr;
    uint64_t scatter_bytes = 0;

    // multi-GPU
    ncclComm_t comm = nullptr;
    int nranks = 1, rank = 0;

    qvq_timings tm;
    hipEvent_t ev[32][4];
    bool ev_ready = false;
};

namespace {

thread_local std::string g_static_err;

qvq_status fail(qvq_ctx *c, qvq_status st, const std::string &msg) {
    if (c) c->err = msg;
    else g_static_err = msg;
    return st;
}

#define HIPCHK(expr)                                                                                  \
    do {                                                                                              \
        hipError_t e_ = (expr);                                                                       \
        if (e_ != hipSuccess)                                                                         \
            return fail(ctx, QVQ_EDEVICE, std::string(#expr) + ": " + hipGetErrorString(e_));         \
    } while (0)

#define NCCLCHK(expr)                                                                                 \
    do {                                                                                              \
        ncclResult_t r_ = (expr);                                                                     \
        if (r_ != ncclSuccess)                                                                        \
            return fail(ctx, QVQ_ECOMM, std::string(#expr) + ": " + ncclGetErrorString(r_));          \
    } while (0)

template <typename T>
void dfree(T *&p) {
    if (p) (void)hipFree(p);
    p = nullptr;
}

qvq_status free_training(qvq_ctx *ctx) {
    dfree(ctx->d_codes);
    dfree(ctx->d_A);
    dfree(ctx->d_flags);
    dfree(ctx->d_ties);
    ctx->N = 0;
    ctx->D = ctx->Dp = 0;
    return QVQ_OK;
}

void free_levels(qvq_ctx *ctx) {
    dfree(ctx->d_C64_cent);
    dfree(ctx->d_C64_split);
    dfree(ctx->d_C32_split);
    dfree(ctx->d_part);
    dfree(ctx->d_part_cnt);
    dfree(ctx->d_sums);
    ctx->Kcap = 0;
}

// Allocate the per-row buffers and upload the colour-space tables.
qvq_status alloc_training(qvq_ctx *ctx, uint64_t N, uint32_t D, int cs) {
    free_training(ctx);
    free_levels(ctx);
    if (!make_terms(cs, ctx->terms)) return fail(ctx, QVQ_EUNSUPPORTED, "colour space has no exact byte sums");
    if (N == 0 || D == 0) return fail(ctx, QVQ_EINVAL, "empty training set");
    if (N >= (1ull << 32)) return fail(ctx, QVQ_EINVAL, "more than 2^32-1 rows per rank");
    const uint32_t Dp = (D + 3) & ~3u;
    if (Dp > 64) return fail(ctx, QVQ_EINVAL, "block dimension above 64 (3*w*h) is not supported");
    ctx->N = N;
    ctx->D = D;
    ctx->Dp = Dp;
    ctx->cs = cs;
    HIPCHK(hipMalloc(&ctx->d_codes, N * Dp));
    HIPCHK(hipMalloc(&ctx->d_A, N * 4));
    HIPCHK(hipMalloc(&ctx->d_flags, N * 4));
    HIPCHK(hipMalloc(&ctx->d_ties, N * 4));
    uint64_t plut[256];
    for (int b = 0; b < 256; b++) plut[b] = ((uint64_t)ctx->terms.hi[b] << 32) | ctx->terms.lo[b];
    HIPCHK(hipMemcpyAsync(ctx->d_lut32, ctx->terms.v32, sizeof(ctx->terms.v32), hipMemcpyHostToDevice, ctx->stream));
    HIPCHK(hipMemcpyAsync(ctx->d_lut64, ctx->terms.v64, sizeof(ctx->terms.v64), hipMemcpyHostToDevice, ctx->stream));
    HIPCHK(hipMemcpyAsync(ctx->d_plut, plut, sizeof(plut), hipMemcpyHostToDevice, ctx->stream));
    return QVQ_OK;
}

qvq_status ensure_levels(qvq_ctx *ctx, uint32_t Kmax) {
    if (ctx->Kcap >= Kmax) return QVQ_OK;
    free_levels(ctx);
    const uint64_t KD = (uint64_t)Kmax * ctx->D;
    HIPCHK(hipMalloc(&ctx->d_C64_cent, KD * 8));
    HIPCHK(hipMalloc(&ctx->d_C64_split, KD * 8));
    HIPCHK(hipMalloc(&ctx->d_C32_split, (uint64_t)Kmax * ctx->Dp * 4));
    HIPCHK(hipMalloc(&ctx->d_part, (uint64_t)ctx->G * KD * 8));
    HIPCHK(hipMalloc(&ctx->d_part_cnt, (uint64_t)ctx->G * Kmax * 4));
    HIPCHK(hipMalloc(&ctx->d_sums, (2 * KD + Kmax) * 8));
    ctx->Kcap = Kmax;
    return QVQ_OK;
}

// fp32 error-bound coefficients for the assignment flag ("near-tie flag").
void flag_coeffs(const qvq_ctx *ctx, float &alpha, float &beta, float &gamma) {
    const double u = std::ldexp(1.0, -24);
    const double vmax = ctx->terms.vmax;
    const double L = std::sqrt((double)ctx->D) * (vmax + 1.2 * vmax) * 1.001;   // >= || |x| + |c| ||
    alpha = (float)(2.0 * 4.01 * u * L);                                         // x2 safety
    beta = (float)(2.0 * ((ctx->Dp + 4) * u * 1.01 + 4e-15));
    gamma = (float)(2.0 * 4.01 * u * u * L * L + 1e-30);
}

qvq_status run_update(qvq_ctx *ctx, const uint32_t *d_A, uint32_t K) {
    const uint32_t D = ctx->D;
    const size_t lds_cap = 150 * 1024;
    const size_t per_k = (size_t)D * 8 + 4;
    uint32_t KR = (uint32_t)std::min<size_t>(K, (lds_cap - 2048 - 16) / per_k);
    if (KR == 0) return fail(ctx, QVQ_EINVAL, "dimension too large for the update kernel");
    const uint32_t passes = (K + KR - 1) / KR;
    const size_t lds = (size_t)KR * D * 8 + ((KR + 1) / 2) * 8 + 256 * 8;
    const uint64_t rpg = (ctx->N + ctx->G - 1) / ctx->G;
    HIPCHK(launch_update(ctx->Dp, dim3(ctx->G, passes), lds, ctx->stream, ctx->d_codes, ctx->N, d_A, K, KR, D, rpg,
                         ctx->d_plut, ctx->d_part, ctx->d_part_cnt));
    const uint64_t cols = (uint64_t)K * D + K;
    const int rgrid = (int)std::min<uint64_t>((cols + 255) / 256, 4096);
    hipLaunchKernelGGL(reduce_kernel, dim3(rgrid), dim3(256), 0, ctx->stream, ctx->d_part, ctx->d_part_cnt, ctx->G, K,
                       D, ctx->d_sums);
    HIPCHK(hipGetLastError());
    if (ctx->comm) {
        NCCLCHK(ncclAllReduce(ctx->d_sums, ctx->d_sums, 2 * (uint64_t)K * D + K, ncclUint64, ncclSum, ctx->comm,
                              ctx->stream));
    }
    return QVQ_OK;
}

qvq_status run_finalize(qvq_ctx *ctx, uint32_t K, bool split) {
    const uint64_t n = (uint64_t)K * ctx->Dp;
    const int grid = (int)std::min<uint64_t>((n + 255) / 256, 4096);
    hipLaunchKernelGGL(finalize_kernel, dim3(grid), dim3(256), 0, ctx->stream, ctx->d_sums, K, ctx->D, ctx->Dp,
                       ctx->terms.R, ctx->terms.bias, ctx->terms.scale, ctx->d_C64_cent, split ? 1 : 0,
                       ctx->d_C64_split, ctx->d_C32_split);
    HIPCHK(hipGetLastError());
    return QVQ_OK;
}

// Assignment of every row against the split codebook in d_C64_split / d_C32_split (K
// code vectors): fp32 search, fp64 recheck, host kd-tree for the rows still tied.
qvq_status run_assign(qvq_ctx *ctx, uint32_t K, int level_slot, uint64_t *flagged_out, uint64_t *ties_out) {
    const uint32_t Dp = ctx->Dp;
    HIPCHK(hipMemsetAsync(ctx->d_counters, 0, 2 * sizeof(unsigned), ctx->stream));
    const uint32_t KT_max = (uint32_t)((ASSIGN_LDS_BYTES - 1024) / (Dp * 4));
    const uint32_t KT = std::min(K, KT_max);
    const size_t lds = 1024 + (size_t)KT * Dp * 4;
    float alpha, beta, gamma;
    flag_coeffs(ctx, alpha, beta, gamma);
    const uint32_t R = assign_rows_per_thread(Dp);
    const uint64_t chunks = (ctx->N + (uint64_t)ASSIGN_THREADS * R - 1) / ((uint64_t)ASSIGN_THREADS * R);
    const int grid = (int)std::min<uint64_t>(chunks, (uint64_t)ctx->num_cu * 8);
    if (level_slot >= 0) HIPCHK(hipEventRecord(ctx->ev[level_slot][0], ctx->stream));
    HIPCHK(launch_assign(Dp, grid, lds, ctx->stream, ctx->d_codes, ctx->N, ctx->d_C32_split, K, KT, ctx->d_lut32,
                         alpha, beta, gamma, ctx->d_A, ctx->d_flags, &ctx->d_counters[0]));
    if (level_slot >= 0) HIPCHK(hipEventRecord(ctx->ev[level_slot][1], ctx->stream));
    hipLaunchKernelGGL(recheck_kernel, dim3(ctx->num_cu * 4), dim3(RECHECK_THREADS), 0, ctx->stream, ctx->d_codes, Dp,
                       ctx->D, ctx->d_flags, &ctx->d_counters[0], ctx->d_C64_split, K, ctx->d_lut64, 1e-12, ctx->d_A,
                       ctx->d_ties, &ctx->d_counters[1]);
    HIPCHK(hipGetLastError());
    unsigned counters[2];
    HIPCHK(hipMemcpyAsync(counters, ctx->d_counters, sizeof(counters), hipMemcpyDeviceToHost, ctx->stream));
    HIPCHK(hipStreamSynchronize(ctx->stream));
    if (flagged_out) *flagged_out = counters[0];
    if (ties_out) *ties_out = counters[1];
    const uint32_t nt = counters[1];
    if (nt) {
        // Rows whose fp64 minimum is (nearly) shared: ask the reference kd-tree.
        const uint32_t D = ctx->D;
        std::vector<uint32_t> rows(nt);
        std::vector<double> C((uint64_t)K * D);
        HIPCHK(hipMemcpyAsync(rows.data(), ctx->d_ties, nt * 4, hipMemcpyDeviceToHost, ctx->stream));
        HIPCHK(hipMemcpyAsync(C.data(), ctx->d_C64_split, C.size() * 8, hipMemcpyDeviceToHost, ctx->stream));
        HIPCHK(hipStreamSynchronize(ctx->stream));
        std::sort(rows.begin(), rows.end());
        const uint64_t need = (uint64_t)nt * (8 + Dp);   // rows | resolved indices | gathered codes
        if (ctx->scatter_bytes < need) {
            dfree(ctx->d_scatter);
            HIPCHK(hipMalloc(&ctx->d_scatter, need));
            ctx->scatter_bytes = need;
        }
        uint32_t *d_rows = ctx->d_scatter, *d_vals = ctx->d_scatter + nt;
        uint8_t *d_gath = reinterpret_cast<uint8_t *>(ctx->d_scatter + 2 * (uint64_t)nt);
        std::vector<uint8_t> code((uint64_t)nt * Dp);
        HIPCHK(hipMemcpyAsync(d_rows, rows.data(), nt * 4, hipMemcpyHostToDevice, ctx->stream));
        hipLaunchKernelGGL(gather_codes_kernel, dim3((int)std::min<uint64_t>(((uint64_t)nt * Dp + 255) / 256, 4096)),
                           dim3(256), 0, ctx->stream, ctx->d_codes, Dp, d_rows, nt, d_gath);
        HIPCHK(hipGetLastError());
        HIPCHK(hipMemcpyAsync(code.data(), d_gath, code.size(), hipMemcpyDeviceToHost, ctx->stream));
        HIPCHK(hipStreamSynchronize(ctx->stream));
        std::vector<double> q(D);
        std::vector<uint32_t> vals(nt);
        RefKDTree tree(C.data(), K, (int)D);
        for (uint32_t i = 0; i < nt; i++) {
            for (uint32_t d = 0; d < D; d++) q[d] = ctx->terms.v64[code[(uint64_t)i * Dp + d]];
            vals[i] = tree.nearest(q.data());
        }
        HIPCHK(hipMemcpyAsync(d_vals, vals.data(), nt * 4, hipMemcpyHostToDevice, ctx->stream));
        hipLaunchKernelGGL(scatter_kernel, dim3((nt + 255) / 256), dim3(256), 0, ctx->stream, ctx->d_A, d_rows,
                           d_vals, nt);
        HIPCHK(hipGetLastError());
    }
    return QVQ_OK;
}

qvq_status tile_from_device(qvq_ctx *ctx, const uint8_t *d_rgb, uint32_t n_images, uint32_t xSize, uint32_t ySize,
                            uint32_t bw, uint32_t bh) {
    const uint64_t nb = (uint64_t)((xSize + bw - 1) / bw) * ((ySize + bh - 1) / bh) * n_images;
    const int grid = (int)std::min<uint64_t>((nb + 255) / 256, 65536);
    hipLaunchKernelGGL(tile_kernel, dim3(grid), dim3(256), 0, ctx->stream, d_rgb, ctx->d_codes, n_images, xSize, ySize,
                       bw, bh, ctx->D, ctx->Dp, ctx->terms.pad_code);
    HIPCHK(hipGetLastError());
    return QVQ_OK;
}

qvq_status check_image_args(qvq_ctx *ctx, uint32_t n_images, uint32_t xSize, uint32_t ySize, uint32_t bw,
                            uint32_t bh, uint64_t &N, uint32_t &D) {
    if (!ctx) return QVQ_EINVAL;
    if (n_images == 0 || xSize == 0 || ySize == 0 || bw == 0 || bh == 0)
        return fail(ctx, QVQ_EINVAL, "image and block sizes must be positive");
    N = (uint64_t)((xSize + bw - 1) / bw) * ((ySize + bh - 1) / bh) * n_images;
    D = 3 * bw * bh;
    return QVQ_OK;
}

}  // namespace

extern "C" {

QVQ_API const char *qvq_version(void) { return "qvq 0.1 (gfx950)"; }

QVQ_API const char *qvq_last_error(const qvq_ctx *ctx) { return ctx ? ctx->err.c_str() : g_static_err.c_str(); }

QVQ_API qvq_status qvq_create(int hip_device, qvq_ctx **out) {
    if (!out) return QVQ_EINVAL;
    *out = nullptr;
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess || n == 0) return fail(nullptr, QVQ_EDEVICE, "no HIP device");
    if (hip_device < 0 || hip_device >= n) return fail(nullptr, QVQ_EINVAL, "bad device index");
    qvq_ctx *ctx = new qvq_ctx();
    ctx->dev = hip_device;
    std::memset(&ctx->tm, 0, sizeof(ctx->tm));
    auto bail = [&](hipError_t e, const char *what) {
        g_static_err = std::string(what) + ": " + hipGetErrorString(e);
        delete ctx;
        return QVQ_EDEVICE;
    };
    hipError_t e;
    if ((e = hipSetDevice(hip_device)) != hipSuccess) return bail(e, "hipSetDevice");
    hipDeviceProp_t prop;
    if ((e = hipGetDeviceProperties(&prop, hip_device)) != hipSuccess) return bail(e, "hipGetDeviceProperties");
    if (std::strncmp(prop.gcnArchName, "gfx950", 6) != 0) {
        g_static_err = std::string("libqvq is built for gfx950, device is ") + prop.gcnArchName;
        delete ctx;
        return QVQ_EDEVICE;
    }
    ctx->num_cu = prop.multiProcessorCount;
    ctx->G = (uint32_t)ctx->num_cu;
    if ((e = hipStreamCreateWithFlags(&ctx->stream, hipStreamNonBlocking)) != hipSuccess) return bail(e, "stream");
    if ((e = hipMalloc(&ctx->d_lut32, 256 * 4)) != hipSuccess) return bail(e, "hipMalloc");
    if ((e = hipMalloc(&ctx->d_lut64, 256 * 8)) != hipSuccess) return bail(e, "hipMalloc");
    if ((e = hipMalloc(&ctx->d_plut, 256 * 8)) != hipSuccess) return bail(e, "hipMalloc");
    if ((e = hipMalloc(&ctx->d_counters, 4 * sizeof(unsigned))) != hipSuccess) return bail(e, "hipMalloc");
    if ((e = hipMalloc(&ctx->d_dist_part, 4096 * 8)) != hipSuccess) return bail(e, "hipMalloc");
    for (int l = 0; l < 32; l++)
        for (int j = 0; j < 4; j++)
            if ((e = hipEventCreate(&ctx->ev[l][j])) != hipSuccess) return bail(e, "hipEventCreate");
    ctx->ev_ready = true;
    *out = ctx;
    return QVQ_OK;
}

QVQ_API void qvq_destroy(qvq_ctx *ctx) {
    if (!ctx) return;
    (void)hipSetDevice(ctx->dev);
    if (ctx->stream) (void)hipStreamSynchronize(ctx->stream);
    if (ctx->comm) ncclCommDestroy(ctx->comm);
    free_training(ctx);
    free_levels(ctx);
    dfree(ctx->d_lut32);
    dfree(ctx->d_lut64);
    dfree(ctx->d_plut);
    dfree(ctx->d_counters);
    dfree(ctx->d_dist_part);
    dfree(ctx->d_scatter);
    if (ctx->ev_ready)
        for (int l = 0; l < 32; l++)
            for (int j = 0; j < 4; j++) (void)hipEventDestroy(ctx->ev[l][j]);
    if (ctx->stream) (void)hipStreamDestroy(ctx->stream);
    delete ctx;
}

QVQ_API uint64_t qvq_num_vectors(const qvq_ctx *ctx) { return ctx ? ctx->N : 0; }
QVQ_API uint32_t qvq_dim(const qvq_ctx *ctx) { return ctx ? ctx->D : 0; }
QVQ_API const uint32_t *qvq_assign_device(const qvq_ctx *ctx) { return ctx ? ctx->d_A : nullptr; }

QVQ_API qvq_status qvq_set_images_device(qvq_ctx *ctx, const void *d_rgb, uint32_t n_images, uint32_t xSize,
                                         uint32_t ySize, uint32_t bw, uint32_t bh, int colorspace) {
    uint64_t N;
    uint32_t D;
    qvq_status st = check_image_args(ctx, n_images, xSize, ySize, bw, bh, N, D);
    if (st != QVQ_OK) return st;
    if (!d_rgb) return fail(ctx, QVQ_EINVAL, "null raster");
    HIPCHK(hipSetDevice(ctx->dev));
    if ((st = alloc_training(ctx, N, D, colorspace)) != QVQ_OK) return st;
    if ((st = tile_from_device(ctx, (const uint8_t *)d_rgb, n_images, xSize, ySize, bw, bh)) != QVQ_OK) return st;
    HIPCHK(hipStreamSynchronize(ctx->stream));
    return QVQ_OK;
}

QVQ_API qvq_status qvq_set_images(qvq_ctx *ctx, const uint8_t *rgb, uint32_t n_images, uint32_t xSize, uint32_t ySize,
                                  uint32_t bw, uint32_t bh, int colorspace) {
    uint64_t N;
    uint32_t D;
    qvq_status st = check_image_args(ctx, n_images, xSize, ySize, bw, bh, N, D);
    if (st != QVQ_OK) return st;
    if (!rgb) return fail(ctx, QVQ_EINVAL, "null raster");
    HIPCHK(hipSetDevice(ctx->dev));
    const uint64_t bytes = (uint64_t)xSize * ySize * 3 * n_images;
    uint8_t *d_rgb = nullptr;
    HIPCHK(hipMalloc(&d_rgb, bytes));
    st = QVQ_OK;
    hipError_t e = hipMemcpyAsync(d_rgb, rgb, bytes, hipMemcpyHostToDevice, ctx->stream);
    if (e != hipSuccess) st = fail(ctx, QVQ_EDEVICE, std::string("raster upload: ") + hipGetErrorString(e));
    if (st == QVQ_OK) st = alloc_training(ctx, N, D, colorspace);
    if (st == QVQ_OK) st = tile_from_device(ctx, d_rgb, n_images, xSize, ySize, bw, bh);
    (void)hipStreamSynchronize(ctx->stream);
    (void)hipFree(d_rgb);
    return st;
}

QVQ_API qvq_status qvq_set_synthetic(qvq_ctx *ctx, uint32_t S, uint64_t seed0, uint32_t n_images, uint32_t bw,
                                     uint32_t bh, int colorspace) {
    uint64_t N;
    uint32_t D;
    if (S < 2) return fail(ctx, QVQ_EINVAL, "synthetic images need S >= 2");
    qvq_status st = check_image_args(ctx, n_images, S, S, bw, bh, N, D);
    if (st != QVQ_OK) return st;
    HIPCHK(hipSetDevice(ctx->dev));
    const uint64_t npix = (uint64_t)S * S * n_images;
    uint8_t *d_rgb = nullptr;
    HIPCHK(hipMalloc(&d_rgb, npix * 3));
    hipLaunchKernelGGL(gen_kernel, dim3((int)std::min<uint64_t>((npix + 255) / 256, 65536)), dim3(256), 0, ctx->stream,
                       d_rgb, S, seed0, npix);
    st = QVQ_OK;
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) st = fail(ctx, QVQ_EDEVICE, std::string("gen_kernel: ") + hipGetErrorString(e));
    if (st == QVQ_OK) st = alloc_training(ctx, N, D, colorspace);
    if (st == QVQ_OK) st = tile_from_device(ctx, d_rgb, n_images, S, S, bw, bh);
    (void)hipStreamSynchronize(ctx->stream);
    (void)hipFree(d_rgb);
    return st;
}

QVQ_API qvq_status qvq_set_vectors(qvq_ctx *ctx, const double *X, uint64_t n, uint32_t dim) {
    if (!ctx) return QVQ_EINVAL;
    if (!X || n == 0 || dim == 0) return fail(ctx, QVQ_EINVAL, "empty training set");
    // Recognise the colour space from the values: every value must be a byte's image
    // under NORMAL or SCALED (or 0.0, the tiling pad), so the exact sums apply.
    int cs_found = -1;
    std::vector<uint8_t> codes;
    for (int cs : {QVQ_CS_SCALED, QVQ_CS_NORMAL}) {
        Terms t;
        make_terms(cs, t);
        std::vector<std::pair<double, uint8_t>> inv;
        for (int b = 0; b < 256; b++) inv.push_back({t.v64[b], (uint8_t)b});
        std::sort(inv.begin(), inv.end());
        const uint32_t Dp = (dim + 3) & ~3u;
        codes.assign(n * Dp, t.pad_code);
        bool ok = true;
        for (uint64_t i = 0; i < n && ok; i++)
            for (uint32_t d = 0; d < dim; d++) {
                const double v = X[i * dim + d];
                auto it = std::lower_bound(inv.begin(), inv.end(), std::make_pair(v, (uint8_t)0));
                if (it == inv.end() || it->first != v || std::signbit(v)) {
                    if (v == 0.0 && !std::signbit(v)) {
                        codes[i * Dp + d] = t.pad_code;
                        continue;
                    }
                    ok = false;
                    break;
                }
                codes[i * Dp + d] = it->second;
            }
        if (ok) {
            cs_found = cs;
            break;
        }
    }
    if (cs_found < 0)
        return fail(ctx, QVQ_EUNSUPPORTED,
                    "training values are not NORMAL/SCALED colour-space values; exact device sums need them");
    HIPCHK(hipSetDevice(ctx->dev));
    qvq_status st = alloc_training(ctx, n, dim, cs_found);
    if (st != QVQ_OK) return st;
    HIPCHK(hipMemcpyAsync(ctx->d_codes, codes.data(), codes.size(), hipMemcpyHostToDevice, ctx->stream));
    HIPCHK(hipStreamSynchronize(ctx->stream));
    return QVQ_OK;
}

QVQ_API qvq_status qvq_lbg(qvq_ctx *ctx, uint32_t bits, double eps, double *codebook, uint32_t *assign,
                           double *distortion) {
    (void)eps;   // cannot change the outputs: one Lloyd step per level
    if (!ctx) return QVQ_EINVAL;
    if (ctx->N == 0) return fail(ctx, QVQ_ESTATE, "no training set");
    if (bits > 20) return fail(ctx, QVQ_EINVAL, "bits must be <= 20");
    HIPCHK(hipSetDevice(ctx->dev));
    const auto t0 = std::chrono::steady_clock::now();
    const uint32_t Kmax = 1u << bits;
    qvq_status st = ensure_levels(ctx, std::max<uint32_t>(Kmax, 2));
    if (st != QVQ_OK) return st;
    std::memset(&ctx->tm, 0, sizeof(ctx->tm));
    ctx->tm.levels = (int)bits;

    // codeVectors[0] = trainingSetSum() / N, then the first split (src/Quantizer.cpp:129-138)
    if ((st = run_update(ctx, nullptr, 1)) != QVQ_OK) return st;
    if ((st = run_finalize(ctx, 1, bits > 0)) != QVQ_OK) return st;
    HIPCHK(hipMemsetAsync(ctx->d_A, 0, ctx->N * 4, ctx->stream));

    for (uint32_t lvl = 1; lvl <= bits; lvl++) {
        const uint32_t K = 1u << lvl;
        const int slot = lvl < 32 ? (int)lvl - 1 : -1;
        const auto h0 = std::chrono::steady_clock::now();
        if ((st = run_assign(ctx, K, slot, &ctx->tm.flagged[slot], &ctx->tm.host_ties[slot])) != QVQ_OK) return st;
        HIPCHK(hipEventRecord(ctx->ev[slot][2], ctx->stream));
        if ((st = run_update(ctx, ctx->d_A, K)) != QVQ_OK) return st;
        HIPCHK(hipEventRecord(ctx->ev[slot][3], ctx->stream));
        if ((st = run_finalize(ctx, K, lvl < bits)) != QVQ_OK) return st;
        (void)h0;
    }
    // Returned distortion: updateDistortion after the last fix (src/Quantizer.cpp:9-22,103)
    const int dgrid = (int)std::min<uint64_t>((ctx->N + DIST_THREADS - 1) / DIST_THREADS, 4096);
    hipLaunchKernelGGL(distortion_kernel, dim3(dgrid), dim3(DIST_THREADS), 0, ctx->stream, ctx->d_codes, ctx->N, ctx->D,
                       ctx->Dp, ctx->d_A, ctx->d_C64_cent, ctx->d_lut64, ctx->d_dist_part);
    HIPCHK(hipGetLastError());
    std::vector<double> dpart(dgrid);
    HIPCHK(hipMemcpyAsync(dpart.data(), ctx->d_dist_part, dgrid * 8, hipMemcpyDeviceToHost, ctx->stream));
    if (codebook)
        HIPCHK(hipMemcpyAsync(codebook, ctx->d_C64_cent, (uint64_t)Kmax * ctx->D * 8, hipMemcpyDeviceToHost,
                              ctx->stream));
    if (assign) HIPCHK(hipMemcpyAsync(assign, ctx->d_A, ctx->N * 4, hipMemcpyDeviceToHost, ctx->stream));
    HIPCHK(hipStreamSynchronize(ctx->stream));
    double dsum = 0;
    for (double v : dpart) dsum += v;
    double ntot = (double)ctx->N;
    if (ctx->comm) {
        double *d_tmp = ctx->d_dist_part;
        double host2[2] = {dsum, ntot};
        HIPCHK(hipMemcpyAsync(d_tmp, host2, 16, hipMemcpyHostToDevice, ctx->stream));
        NCCLCHK(ncclAllReduce(d_tmp, d_tmp, 2, ncclDouble, ncclSum, ctx->comm, ctx->stream));
        HIPCHK(hipMemcpyAsync(host2, d_tmp, 16, hipMemcpyDeviceToHost, ctx->stream));
        HIPCHK(hipStreamSynchronize(ctx->stream));
        dsum = host2[0];
        ntot = host2[1];
    }
    if (distortion) *distortion = dsum / (ntot * (double)ctx->D);
    for (uint32_t lvl = 1; lvl <= bits && lvl <= 32; lvl++) {
        float a = 0, u = 0;
        (void)hipEventElapsedTime(&a, ctx->ev[lvl - 1][0], ctx->ev[lvl - 1][1]);
        (void)hipEventElapsedTime(&u, ctx->ev[lvl - 1][2], ctx->ev[lvl - 1][3]);
        ctx->tm.assign_ms[lvl - 1] = a;
        ctx->tm.update_ms[lvl - 1] = u;
    }
    ctx->tm.total_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    return QVQ_OK;
}

QVQ_API qvq_status qvq_assign(qvq_ctx *ctx, const double *C, uint32_t K, uint32_t *assign) {
    if (!ctx) return QVQ_EINVAL;
    if (ctx->N == 0) return fail(ctx, QVQ_ESTATE, "no training set");
    if (!C || K == 0) return fail(ctx, QVQ_EINVAL, "empty codebook");
    HIPCHK(hipSetDevice(ctx->dev));
    qvq_status st = ensure_levels(ctx, K);
    if (st != QVQ_OK) return st;
    const uint32_t D = ctx->D, Dp = ctx->Dp;
    std::vector<float> c32((uint64_t)K * Dp, 0.f);
    for (uint64_t k = 0; k < K; k++)
        for (uint32_t d = 0; d < D; d++) c32[k * Dp + d] = (float)C[k * D + d];
    HIPCHK(hipMemcpyAsync(ctx->d_C64_split, C, (uint64_t)K * D * 8, hipMemcpyHostToDevice, ctx->stream));
    HIPCHK(hipMemcpyAsync(ctx->d_C32_split, c32.data(), c32.size() * 4, hipMemcpyHostToDevice, ctx->stream));
    uint64_t fl = 0, ti = 0;
    if ((st = run_assign(ctx, K, 0, &fl, &ti)) != QVQ_OK) return st;
    ctx->tm.flagged[0] = fl;
    ctx->tm.host_ties[0] = ti;
    if (assign) HIPCHK(hipMemcpyAsync(assign, ctx->d_A, ctx->N * 4, hipMemcpyDeviceToHost, ctx->stream));
    HIPCHK(hipStreamSynchronize(ctx->stream));
    return QVQ_OK;
}

QVQ_API qvq_status qvq_update(qvq_ctx *ctx, const uint32_t *assign, uint32_t K, double *C_out, uint64_t *counts) {
    if (!ctx) return QVQ_EINVAL;
    if (ctx->N == 0) return fail(ctx, QVQ_ESTATE, "no training set");
    if (!assign || K == 0) return fail(ctx, QVQ_EINVAL, "empty assignment");
    for (uint64_t i = 0; i < ctx->N; i++)
        if (assign[i] >= K) return fail(ctx, QVQ_EINVAL, "assignment index out of range");
    HIPCHK(hipSetDevice(ctx->dev));
    qvq_status st = ensure_levels(ctx, K);
    if (st != QVQ_OK) return st;
    HIPCHK(hipMemcpyAsync(ctx->d_A, assign, ctx->N * 4, hipMemcpyHostToDevice, ctx->stream));
    if ((st = run_update(ctx, ctx->d_A, K)) != QVQ_OK) return st;
    if ((st = run_finalize(ctx, K, false)) != QVQ_OK) return st;
    if (C_out)
        HIPCHK(hipMemcpyAsync(C_out, ctx->d_C64_cent, (uint64_t)K * ctx->D * 8, hipMemcpyDeviceToHost, ctx->stream));
    if (counts)
        HIPCHK(hipMemcpyAsync(counts, ctx->d_sums + 2 * (uint64_t)K * ctx->D, (uint64_t)K * 8, hipMemcpyDeviceToHost,
                              ctx->stream));
    HIPCHK(hipStreamSynchronize(ctx->stream));
    return QVQ_OK;
}

QVQ_API qvq_status qvq_comm_unique_id(uint8_t id[128]) {
    static_assert(sizeof(ncclUniqueId) == 128, "RCCL unique id size");
    ncclUniqueId u;
    const ncclResult_t r = ncclGetUniqueId(&u);
    if (r != ncclSuccess) return fail(nullptr, QVQ_ECOMM, std::string("ncclGetUniqueId: ") + ncclGetErrorString(r));
    std::memcpy(id, &u, 128);
    return QVQ_OK;
}

QVQ_API qvq_status qvq_comm_init(qvq_ctx *ctx, int nranks, int rank, const uint8_t id[128]) {
    if (!ctx || !id || nranks < 1 || rank < 0 || rank >= nranks) return QVQ_EINVAL;
    HIPCHK(hipSetDevice(ctx->dev));
    if (ctx->comm) {
        ncclCommDestroy(ctx->comm);
        ctx->comm = nullptr;
    }
    if (nranks == 1) return QVQ_OK;
    ncclUniqueId u;
    std::memcpy(&u, id, 128);
    NCCLCHK(ncclCommInitRank(&ctx->comm, nranks, u, rank));
    ctx->nranks = nranks;
    ctx->rank = rank;
    return QVQ_OK;
}

QVQ_API qvq_status qvq_get_timings(const qvq_ctx *ctx, qvq_timings *out) {
    if (!ctx || !out) return QVQ_EINVAL;
    *out = ctx->tm;
    return QVQ_OK;
}

QVQ_API qvq_status qvq_host_kdtree_nn(const double *C, uint32_t K, uint32_t dim, const double *Q, uint64_t nq,
                                      uint32_t *out) {
    if (!C || !Q || !out || K == 0 || dim == 0) return QVQ_EINVAL;
    RefKDTree tree(C, K, (int)dim);
    for (uint64_t i = 0; i < nq; i++) out[i] = tree.nearest(Q + i * dim);
    return QVQ_OK;
}

QVQ_API qvq_status qvq_host_finalize(const uint64_t *hi, const uint64_t *lo, const uint64_t *cnt, uint32_t K,
                                     uint32_t dim, int colorspace, double *C_out) {
    Terms t;
    if (!hi || !lo || !cnt || !C_out) return QVQ_EINVAL;
    if (!make_terms(colorspace, t)) return QVQ_EUNSUPPORTED;
    for (uint64_t k = 0; k < K; k++)
        for (uint32_t d = 0; d < dim; d++)
            C_out[k * dim + d] = centroid_value(hi[k * dim + d], lo[k * dim + d], cnt[k], t.R, t.bias, t.scale);
    return QVQ_OK;
}

QVQ_API qvq_status qvq_host_row_terms(const uint8_t *codes, uint32_t dim, int colorspace, uint64_t *hi,
                                      uint64_t *lo) {
    Terms t;
    if (!codes || !hi || !lo) return QVQ_EINVAL;
    if (!make_terms(colorspace, t)) return QVQ_EUNSUPPORTED;
    for (uint32_t d = 0; d < dim; d++) {
        hi[d] = t.hi[codes[d]];
        lo[d] = t.lo[codes[d]];
    }
    return QVQ_OK;
}

}  // extern "C"
