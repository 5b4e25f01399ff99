// k_misc.hip -- tiling, synthetic rasters, exact centroid sums, finalisation, split and
// codebook preparation, tie scatter, distortion.
//
// Global sums layout (also the RCCL all-reduce buffer, u64):
//   hi[d][k] (K*D) | lo[d][k] (K*D) | cnt[k] (K)
// Workgroup slabs (update kernels): part[g][d][k] packed (hi << 32 | lo), part_cnt[g][k].
#include "common.hpp"
#include "mfma_util.hpp"

namespace qvq {

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

hipError_t launch_gen(hipStream_t s, uint8_t *rgb, uint32_t S, uint64_t seed0, uint64_t npix) {
    hipLaunchKernelGGL(gen_kernel, dim3((int)std::min<uint64_t>((npix + 255) / 256, 65536)), dim3(256), 0, s, rgb, S,
                       seed0, npix);
    return hipGetLastError();
}

// getBlocksAsVectorsFromImage (src/Compressor.cpp:31-62) over n_images rasters, writing
// each block's raw bytes (component order ((x-iw)*h + (y-jh))*3 + c) into codes[g][0..D),
// padding [D, Dp) with the zero-valued byte.  One thread per block.
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
                const uint64_t imgIndex = x * ySize + y;   // wraps past ySize into the next row
                const uint64_t vec = ((x - i * bw) * bh + (y - j * bh)) * 3;
                for (int c = 0; c < 3; c++) dst[vec + c] = imgIndex < total ? src[imgIndex * 3 + c] : pad;
            }
        for (uint32_t d = D; d < Dp; d++) dst[d] = pad;
    }
}

// The 2x2 case without wrap or padding (xSize even, ySize % 4 == 0: every block inside its image,
// raster rows 4-byte aligned): a thread takes two horizontally adjacent blocks -- 12 bytes of
// raster row 2i and 12 of row 2i + 1, three dword loads each -- and writes their 24 code bytes
// with six dword stores (block j: row 2i pixels 2j, 2j+1, then row 2i+1's; D = Dp = 12).  The
// generic kernel moved these 100 MB (C3) at ~2 TB/s with byte stores and 64-bit divisions.
__global__ __launch_bounds__(256) void tile22_kernel(const uint32_t *__restrict__ rgb, uint32_t *__restrict__ codes,
                                                     uint64_t pairs_total, uint32_t pairs_per_row, uint32_t words_per_row,
                                                     uint64_t pairs_per_image, uint64_t words_per_image) {
    for (uint64_t t = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; t < pairs_total;
         t += (uint64_t)gridDim.x * blockDim.x) {
        const uint64_t img = t / pairs_per_image, r = t - img * pairs_per_image;
        const uint32_t i = (uint32_t)(r / pairs_per_row), jp = (uint32_t)(r - (uint64_t)i * pairs_per_row);
        const uint32_t *a = rgb + img * words_per_image + (uint64_t)(2 * i) * words_per_row + 3 * jp;
        const uint32_t *b = a + words_per_row;
        const uint32_t a0 = a[0], a1 = a[1], a2 = a[2], b0 = b[0], b1 = b[1], b2 = b[2];
        // row bytes a0..a11: block j = a[0..5] b[0..5], block j+1 = a[6..11] b[6..11]
        uint32_t *o = codes + t * 6;
        o[0] = a0;
        o[1] = __builtin_amdgcn_perm(b0, a1, 0x05040100u);   // a4 a5 b0 b1
        o[2] = __builtin_amdgcn_alignbyte(b1, b0, 2);        // b2 b3 b4 b5
        o[3] = __builtin_amdgcn_alignbyte(a2, a1, 2);        // a6 a7 a8 a9
        o[4] = __builtin_amdgcn_perm(b1, a2, 0x07060302u);   // a10 a11 b6 b7
        o[5] = b2;                                           // b8 b9 b10 b11
    }
}

hipError_t launch_tile(hipStream_t s, const uint8_t *rgb, uint8_t *codes, uint32_t n_images, uint32_t xSize,
                       uint32_t ySize, uint32_t bw, uint32_t bh, uint32_t D, uint32_t Dp, uint8_t pad) {
    if (bw == 2 && bh == 2 && xSize % 2 == 0 && ySize % 4 == 0 && ((uintptr_t)rgb & 3) == 0) {
        const uint32_t ppr = ySize / 4, wpr = ySize * 3 / 4;
        const uint64_t ppi = (uint64_t)(xSize / 2) * ppr, wpi = (uint64_t)xSize * wpr;
        const uint64_t total = ppi * n_images;
        hipLaunchKernelGGL(tile22_kernel, dim3((int)std::min<uint64_t>((total + 255) / 256, 1u << 16)), dim3(256), 0, s,
                           reinterpret_cast<const uint32_t *>(rgb), reinterpret_cast<uint32_t *>(codes), total, ppr,
                           wpr, ppi, wpi);
        return hipGetLastError();
    }
    const uint64_t nb = (uint64_t)((xSize + bw - 1) / bw) * ((ySize + bh - 1) / bh) * n_images;
    hipLaunchKernelGGL(tile_kernel, dim3((int)std::min<uint64_t>((nb + 255) / 256, 65536)), dim3(256), 0, s, rgb,
                       codes, n_images, xSize, ySize, bw, bh, D, Dp, pad);
    return hipGetLastError();
}

// ---------------------------------------------------------------------------------------
// Exact centroid sums for an arbitrary assignment (the path not fused into the search).
// Grid (G, passes): workgroup g folds its contiguous row range into LDS for code vectors
// [k0, k0 + KR), layout [d][k], then writes its packed slab.
// ---------------------------------------------------------------------------------------
constexpr int UPDATE_THREADS = 1024;
constexpr size_t UPDATE_LDS = 150 * 1024;

template <int DP>
__global__ __launch_bounds__(UPDATE_THREADS) void update_kernel(
    const uint8_t *__restrict__ codes, uint64_t N, const uint32_t *__restrict__ A, uint32_t K, uint32_t KR,
    uint32_t D, uint64_t rows_per_group, const uint64_t *__restrict__ plut, uint64_t *__restrict__ part,
    uint32_t *__restrict__ part_cnt) {
    extern __shared__ __attribute__((aligned(16))) uint64_t lsum[];   // [D][KR] | cnt u32 [KR] | lut [256]
    const uint32_t k0 = blockIdx.y * KR;
    const uint32_t kr = min(KR, K - k0);
    uint32_t *lcnt = reinterpret_cast<uint32_t *>(lsum + (uint64_t)KR * D);
    uint64_t *llut = lsum + (uint64_t)KR * D + (KR + 1) / 2;
    const int tid = threadIdx.x;
    for (uint32_t i = tid; i < KR * D; i += UPDATE_THREADS) lsum[i] = 0;
    for (uint32_t i = tid; i < KR; i += UPDATE_THREADS) lcnt[i] = 0;
    for (int i = tid; i < 256; i += UPDATE_THREADS) llut[i] = plut[i];
    __syncthreads();
    const uint64_t start = blockIdx.x * rows_per_group;
    const uint64_t end = min(N, start + rows_per_group);
    for (uint64_t row = start + tid; row < end; row += UPDATE_THREADS) {
        const uint32_t kl = A[row] - k0;
        if (kl < kr) {
            const uint32_t *w = reinterpret_cast<const uint32_t *>(codes + row * DP);
#pragma unroll
            for (int q = 0; q < DP / 4; q++) {
                const uint32_t v = w[q];
#pragma unroll
                for (int j = 0; j < 4; j++)
                    if (4 * q + j < (int)D)
                        atomicAdd((unsigned long long *)&lsum[(uint32_t)(4 * q + j) * KR + kl],
                                  (unsigned long long)llut[(v >> (8 * j)) & 0xFF]);
            }
            atomicAdd(&lcnt[kl], 1u);
        }
    }
    __syncthreads();
    uint64_t *pdst = part + (uint64_t)blockIdx.x * K * D;
    for (uint32_t i = tid; i < kr * D; i += UPDATE_THREADS) {
        const uint32_t d = i / kr, k = i - d * kr;
        pdst[(uint64_t)d * K + k0 + k] = lsum[d * KR + k];
    }
    uint32_t *cdst = part_cnt + (uint64_t)blockIdx.x * K + k0;
    for (uint32_t i = tid; i < kr; i += UPDATE_THREADS) cdst[i] = lcnt[i];
}

#define QVQ_FOR_EACH_DP(X) X(4) X(8) X(12) X(16) X(20) X(24) X(28) X(32) X(36) X(40) X(44) X(48) X(52) X(56) X(60) X(64)

// Centroid sums of a final assignment, HBM-bound.  A wave takes 64*R consecutive rows per
// round, lane L rows R*L..R*L+R-1 (coalesced), R = 4, 2 or 1 rows by width so that the codes
// stay in registers.  A lane adds the exact terms of its rows in registers (u << 16 | lo per
// component) while the index repeats, across rounds, and flushes the run to the LDS sums
// [d][k] when the index changes or after 256 rows (the 16-bit fields never carry).  At small
// K many lanes flush to the same few addresses, which the LDS serialises: the sums are
// replicated C times (lane L adds into copy L mod C) and the copies are summed when the
// workgroup writes its slab [g][d][k] for reduce_kernel.
constexpr size_t URUN_LDS = 160 * 1024;
// wide rows keep 4 + DP/4 + DP registers per lane live: fewer waves, up to 256 VGPRs
__host__ __device__ constexpr int urun_threads(int DP) { return DP > 32 ? 512 : 1024; }

// copies' strides one word past K*D (u64) and an even K (u32): the copies of one term then sit
// on different LDS banks (as the MFMA search's, k_mf32.hip)
__host__ __device__ inline uint32_t urun_sstride(uint32_t K, uint32_t D) { return K * D + 1; }
__host__ __device__ inline uint32_t urun_cstride(uint32_t K) { return ((K + 1) & ~1u) + 2; }
static size_t urun_bytes(uint32_t K, uint32_t D, uint32_t C) {
    return (size_t)C * urun_sstride(K, D) * 8 + (size_t)C * urun_cstride(K) * 4 + 256;
}
static uint32_t urun_copies(uint32_t K, uint32_t D) {
    for (uint32_t C : {16u, 8u, 4u, 2u})
        if (urun_bytes(K, D, C) <= URUN_LDS / 2) return C;   // replicas only while they are cheap
    return 1;
}
bool update_runs_fits(uint32_t K, uint32_t D) { return urun_bytes(K, D, 1) <= URUN_LDS; }

template <int DP>
__global__ __launch_bounds__(urun_threads(DP)) void update_runs_kernel(const uint8_t *__restrict__ codes, uint64_t N,
                                                                   const uint32_t *__restrict__ A, uint32_t K,
                                                                   uint32_t D, uint32_t C, const uint64_t *__restrict__ plut,
                                                                   uint64_t *__restrict__ part,
                                                                   uint32_t *__restrict__ part_cnt) {
    constexpr int T = urun_threads(DP);
    constexpr int R = DP <= 16 ? 4 : (DP <= 32 ? 2 : 1);   // rows per lane and round
    constexpr int W4 = DP / 4;                               // code words per row
    extern __shared__ __attribute__((aligned(16))) uint64_t usm[];
    const uint32_t SS = urun_sstride(K, D), K2 = urun_cstride(K);
    uint64_t *sums_all = usm;                                                         // [C][SS] ([D][K] each)
    uint32_t *cnt_all = reinterpret_cast<uint32_t *>(usm + (size_t)C * SS);          // [C][K2]
    uint8_t *lo8 = reinterpret_cast<uint8_t *>(cnt_all + (size_t)C * K2);            // [256]
    const int tid = threadIdx.x, lane = tid & 63;
    for (uint32_t i = tid; i < C * SS; i += T) sums_all[i] = 0;
    for (uint32_t i = tid; i < C * K2; i += T) cnt_all[i] = 0;
    uint64_t *sums = sums_all + (size_t)(lane % C) * SS;   // this lane's copy
    uint32_t *cnt = cnt_all + (size_t)(lane % C) * K2;
    if (tid < 256) lo8[tid] = (uint8_t)(plut[tid] & 0xFF);
    __syncthreads();
    uint32_t acc[DP + 1];
    uint32_t cur = 0xFFFFFFFFu;
#pragma unroll
    for (int i = 0; i <= DP; i++) acc[i] = 0;
    auto flush = [&]() {
        if (acc[DP]) {
#pragma unroll
            for (int d = 0; d < DP; d++)
                if ((uint32_t)d < D)
                    atomicAdd((unsigned long long *)&sums[(uint32_t)d * K + cur],
                              (unsigned long long)((((uint64_t)(acc[d] >> 16)) << 32) | (acc[d] & 0xFFFF)));
            atomicAdd(&cnt[cur], acc[DP]);
        }
#pragma unroll
        for (int i = 0; i <= DP; i++) acc[i] = 0;
    };
    auto add_row = [&](const uint32_t *w, uint32_t k) {
        if (k != cur || acc[DP] == 256) {
            flush();
            cur = k;
        }
#pragma unroll
        for (int d = 0; d < DP; d++) {
            const uint32_t b = (w[d / 4] >> (8 * (d % 4))) & 0xFF;
            acc[d] += (b ^ 0x80u) << 16 | lo8[b];
        }
        acc[DP] += 1;
    };
    const uint64_t wave_g = ((uint64_t)blockIdx.x * T + tid) >> 6;
    const uint64_t n_waves = ((uint64_t)gridDim.x * T) >> 6;
    // (a prefetching loop holding the next round in registers measured slower: C4's update
    // 102 -> 132 us per quantize)
    for (uint64_t r0 = wave_g * 64 * R; r0 < N; r0 += n_waves * 64 * R) {
        const uint64_t row = r0 + (uint64_t)R * lane;
        if (r0 + 64 * R <= N) {
            uint32_t w[R * W4];
            const uint32_t *p = reinterpret_cast<const uint32_t *>(codes + row * DP);
#pragma unroll
            for (int i = 0; i < R * W4; i++) w[i] = p[i];
            uint32_t a[R];
#pragma unroll
            for (int r = 0; r < R; r++) a[r] = A[row + r];
#pragma unroll
            for (int r = 0; r < R; r++) add_row(w + r * W4, a[r]);
        } else {
            for (uint64_t r = row; r < row + R && r < N; r++) {
                uint32_t w[W4];
#pragma unroll
                for (int i = 0; i < W4; i++) w[i] = reinterpret_cast<const uint32_t *>(codes + r * DP)[i];
                add_row(w, A[r]);
            }
        }
    }
    flush();
    __syncthreads();
    uint64_t *pdst = part + (uint64_t)blockIdx.x * K * D;
    for (uint32_t i = tid; i < K * D; i += T) {
        uint64_t t = 0;
        for (uint32_t c = 0; c < C; c++) t += sums_all[(size_t)c * SS + i];
        pdst[i] = t;
    }
    uint32_t *cdst = part_cnt + (uint64_t)blockIdx.x * K;
    for (uint32_t i = tid; i < K; i += T) {
        uint32_t t = 0;
        for (uint32_t c = 0; c < C; c++) t += cnt_all[(size_t)c * K2 + i];
        cdst[i] = t;
    }
}

hipError_t launch_update(hipStream_t s, uint32_t Dp, uint32_t G, const uint8_t *codes, uint64_t N, const uint32_t *A,
                         uint32_t K, uint32_t D, const uint64_t *plut, uint64_t *part, uint32_t *part_cnt) {
    if (update_runs_fits(K, D)) {
        const uint32_t C = urun_copies(K, D);
        const size_t lds = urun_bytes(K, D, C);
        switch (Dp) {
#define X(DPV)                                                                                                     \
    case DPV:                                                                                                      \
        hipLaunchKernelGGL(update_runs_kernel<DPV>, dim3(G), dim3(urun_threads(DPV)), lds, s, codes, N, A, K, D, C,    \
                           plut, part, part_cnt);                                                                  \
        return hipGetLastError();
            QVQ_FOR_EACH_DP(X)
#undef X
        }
        return hipErrorInvalidValue;
    }
    const size_t per_k = (size_t)D * 8 + 4;
    const uint32_t KR = (uint32_t)std::min<size_t>(K, (UPDATE_LDS - 2048 - 16) / per_k);
    if (KR == 0) return hipErrorInvalidValue;
    const uint32_t passes = (K + KR - 1) / KR;
    const size_t lds = (size_t)KR * D * 8 + ((KR + 1) / 2) * 8 + 256 * 8;
    const uint64_t rpg = (N + G - 1) / G;
    switch (Dp) {
#define X(DPV)                                                                                                    \
    case DPV:                                                                                                     \
        hipLaunchKernelGGL(update_kernel<DPV>, dim3(G, passes), dim3(UPDATE_THREADS), lds, s, codes, N, A, K, KR, \
                           D, rpg, plut, part, part_cnt);                                                         \
        return hipGetLastError();
        QVQ_FOR_EACH_DP(X)
#undef X
    }
    return hipErrorInvalidValue;
}

// ---------------------------------------------------------------------------------------
// Centroid sums of a final assignment for big K * D (the non-fused levels of 4x4 blocks): a
// counting sort of the rows by index, then every lane folds 8 consecutive rows of the order
// (mostly one code vector) in registers, a wave sums its lanes' runs, and each run's last lane
// adds it to sums [hi KD][lo KD][cnt K] with global atomics.  The LDS update needs one pass per KR code vectors and leaves G slabs of
// K*D u64 for reduce_kernel (C4, K = 4096: 400 MB written and read again per level).
// ---------------------------------------------------------------------------------------
constexpr int SRT_THREADS = 1024;
constexpr int SRT_UB = 8;                    // row indices in flight per thread
constexpr uint32_t SRT_ROWS_PER_LANE = 8;    // consecutive sorted rows per lane, gathered at once
constexpr uint32_t SRT_SLOTS = 64;           // code vectors a block sums in LDS before the global atomics

// hist[g][k]: rows of block g's range with index k.  The blocks also clear the nzero u64 of the
// sums (no separate memset launch: ~3 us per level).
__global__ __launch_bounds__(SRT_THREADS) void sort_hist_kernel(const uint32_t *__restrict__ A, uint64_t N, uint32_t K,
                                                                uint64_t rpg, uint32_t *__restrict__ hist,
                                                                uint64_t *__restrict__ zero, uint64_t nzero) {
    extern __shared__ uint32_t h[];
    for (uint64_t i = (uint64_t)blockIdx.x * SRT_THREADS + threadIdx.x; i < nzero; i += (uint64_t)gridDim.x * SRT_THREADS)
        zero[i] = 0;
    for (uint32_t i = threadIdx.x; i < K; i += SRT_THREADS) h[i] = 0;
    __syncthreads();
    const uint64_t start = (uint64_t)blockIdx.x * rpg, end = min(N, start + rpg);
    for (uint64_t r0 = start + threadIdx.x; r0 < end; r0 += (uint64_t)SRT_UB * SRT_THREADS) {
        uint32_t a[SRT_UB];
#pragma unroll
        for (int u = 0; u < SRT_UB; u++) a[u] = A[min(r0 + (uint64_t)u * SRT_THREADS, end - 1)];
#pragma unroll
        for (int u = 0; u < SRT_UB; u++)
            if (r0 + (uint64_t)u * SRT_THREADS < end) atomicAdd(&h[a[u]], 1u);
    }
    __syncthreads();
    for (uint32_t i = threadIdx.x; i < K; i += SRT_THREADS) hist[(uint64_t)blockIdx.x * K + i] = h[i];
}

// hist[g][k] <- rows of blocks g' < g with index k; tot[k] = all rows with index k
__global__ __launch_bounds__(256) void sort_colscan_kernel(uint32_t *__restrict__ hist, uint32_t G, uint32_t K,
                                                           uint32_t *__restrict__ tot) {
    const uint32_t k = blockIdx.x * 256 + threadIdx.x;
    if (k >= K) return;
    uint32_t s = 0;
    constexpr uint32_t CU = 16;   // loads in flight (a dependent load per block was ~60 us)
    for (uint32_t g0 = 0; g0 < G; g0 += CU) {
        uint32_t v[CU];
#pragma unroll
        for (uint32_t u = 0; u < CU; u++) v[u] = hist[(uint64_t)min(g0 + u, G - 1) * K + k];
#pragma unroll
        for (uint32_t u = 0; u < CU; u++)
            if (g0 + u < G) {
                hist[(uint64_t)(g0 + u) * K + k] = s;
                s += v[u];
            }
    }
    tot[k] = s;
}

// The same for G <= 256 with four times the parallelism: a block owns 64 columns, its wave w
// the blocks w*QG .. of each (QG <= 64 values held in registers, all loads in flight), the
// waves' totals meet in LDS and each wave writes its part with the offset of the ones before.
// (The one-thread-per-column scan was 16 dependent load rounds: ~16 us per C4 level.)
constexpr uint32_t CS_QG = 64;
__global__ __launch_bounds__(256) void sort_colscan4_kernel(uint32_t *__restrict__ hist, uint32_t G, uint32_t K,
                                                            uint32_t *__restrict__ tot) {
    __shared__ uint32_t part[4][64];
    const uint32_t lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const uint32_t k = blockIdx.x * 64 + lane;
    const uint32_t QG = (G + 3) / 4, g0 = w * QG, g1 = min(G, g0 + QG);
    uint32_t v[CS_QG];
#pragma unroll
    for (uint32_t u = 0; u < CS_QG; u++) {
        const uint32_t g = g0 + u;
        v[u] = k < K && u < QG && g < g1 ? hist[(uint64_t)g * K + k] : 0u;
    }
    uint32_t s = 0;
#pragma unroll
    for (uint32_t u = 0; u < CS_QG; u++) {
        const uint32_t x = v[u];
        v[u] = s;
        s += x;
    }
    part[w][lane] = s;
    __syncthreads();
    uint32_t off = 0;
    for (uint32_t i = 0; i < w; i++) off += part[i][lane];
    if (k < K) {
#pragma unroll
        for (uint32_t u = 0; u < CS_QG; u++) {
            const uint32_t g = g0 + u;
            if (u < QG && g < g1) hist[(uint64_t)g * K + k] = v[u] + off;
        }
        if (w == 3) tot[k] = off + s;
    }
}

// koff[k] = rows with index < k (exclusive scan of tot in one block)
__global__ __launch_bounds__(SRT_THREADS) void sort_koff_kernel(const uint32_t *__restrict__ tot, uint32_t K,
                                                                uint32_t *__restrict__ koff) {
    __shared__ uint32_t part[SRT_THREADS];
    const uint32_t seg = (K + SRT_THREADS - 1) / SRT_THREADS;
    const uint32_t b = min(K, threadIdx.x * seg), e = min(K, b + seg);
    uint32_t s = 0;
    for (uint32_t i = b; i < e; i++) s += tot[i];
    part[threadIdx.x] = s;
    __syncthreads();
    for (int off = 1; off < SRT_THREADS; off <<= 1) {   // inclusive scan of the segment sums
        const uint32_t v = threadIdx.x >= (uint32_t)off ? part[threadIdx.x - off] : 0u;
        __syncthreads();
        part[threadIdx.x] += v;
        __syncthreads();
    }
    uint32_t base = part[threadIdx.x] - s;
    for (uint32_t i = b; i < e; i++) {
        koff[i] = base;
        base += tot[i];
    }
}

// idx[pos] = row, ks[pos] = its index, pos = koff[k] + hist[g][k] + rank within block g
// (any order within a code vector: the sums are exact integers)
__global__ __launch_bounds__(SRT_THREADS) void sort_scatter_kernel(const uint32_t *__restrict__ A, uint64_t N, uint32_t K,
                                                                   uint64_t rpg, const uint32_t *__restrict__ hist,
                                                                   const uint32_t *__restrict__ koff,
                                                                   uint32_t *__restrict__ idx, uint32_t *__restrict__ ks) {
    extern __shared__ uint32_t cur[];
    for (uint32_t i = threadIdx.x; i < K; i += SRT_THREADS) cur[i] = koff[i] + hist[(uint64_t)blockIdx.x * K + i];
    __syncthreads();
    const uint64_t start = (uint64_t)blockIdx.x * rpg, end = min(N, start + rpg);
    for (uint64_t r0 = start + threadIdx.x; r0 < end; r0 += (uint64_t)SRT_UB * SRT_THREADS) {
        uint32_t a[SRT_UB];
#pragma unroll
        for (int u = 0; u < SRT_UB; u++) a[u] = A[min(r0 + (uint64_t)u * SRT_THREADS, end - 1)];
#pragma unroll
        for (int u = 0; u < SRT_UB; u++) {
            const uint64_t row = r0 + (uint64_t)u * SRT_THREADS;
            if (row < end) {
                const uint32_t pos = atomicAdd(&cur[a[u]], 1u);
                idx[pos] = (uint32_t)row;
                ks[pos] = a[u];
            }
        }
    }
}

template <int DP>
__global__ __launch_bounds__(256) void sorted_sums_kernel(const uint8_t *__restrict__ codes, uint64_t N,
                                                          const uint32_t *__restrict__ idx, const uint32_t *__restrict__ ks,
                                                          uint32_t K, uint32_t D, const uint64_t *__restrict__ plut,
                                                          uint64_t *__restrict__ sums) {
    constexpr int W4 = DP / 4;
    constexpr int B = (int)SRT_ROWS_PER_LANE;   // rows gathered together
    constexpr uint32_t NS = 2 * DP + 1;         // hi | lo | count per code vector
    __shared__ uint8_t lo8[256];
    // the block's runs: its positions cover code vectors kbase .. (sorted), the first
    // SRT_SLOTS of them summed here and added to the global sums once per block
    __shared__ uint32_t tab[SRT_SLOTS * NS];
    if (threadIdx.x < 256) lo8[threadIdx.x] = (uint8_t)(plut[threadIdx.x] & 0xFF);
    for (uint32_t i = threadIdx.x; i < SRT_SLOTS * NS; i += 256) tab[i] = 0;
    const uint64_t bp = (uint64_t)blockIdx.x * 256 * SRT_ROWS_PER_LANE;
    const uint32_t kbase = ks[bp < N ? bp : N - 1];
    __syncthreads();
    const uint64_t p0 = ((uint64_t)blockIdx.x * 256 + threadIdx.x) * SRT_ROWS_PER_LANE;
    const uint64_t p1 = min(N, p0 + SRT_ROWS_PER_LANE);   // p0 >= N: no rows (the lane still joins the wave sums)
    const uint64_t KD = (uint64_t)K * D;
    uint32_t acc[DP + 1];
    uint32_t cur = 0xFFFFFFFFu;
#pragma unroll
    for (int i = 0; i <= DP; i++) acc[i] = 0;
    auto flush = [&]() {   // a run ending inside the lane's rows (a code vector boundary)
        if (acc[DP]) {
#pragma unroll
            for (int d = 0; d < DP; d++)
                if ((uint32_t)d < D) {
                    atomicAdd((unsigned long long *)&sums[(uint64_t)d * K + cur], (unsigned long long)(acc[d] >> 16));
                    atomicAdd((unsigned long long *)&sums[KD + (uint64_t)d * K + cur],
                              (unsigned long long)(acc[d] & 0xFFFF));
                }
            atomicAdd((unsigned long long *)&sums[2 * KD + cur], (unsigned long long)acc[DP]);
        }
#pragma unroll
        for (int i = 0; i <= DP; i++) acc[i] = 0;
    };
    for (uint64_t p = p0; p < p1; p += B) {   // <= 8 rows per lane: the 16-bit fields never carry
        uint32_t r[B], k[B], w[B][W4];
#pragma unroll
        for (int u = 0; u < B; u++) {
            const uint64_t q = min(p + u, p1 - 1);
            r[u] = idx[q];
            k[u] = ks[q];
        }
#pragma unroll
        for (int u = 0; u < B; u++) {
            if constexpr (DP % 16 == 0) {   // 16-byte rows: vector loads
                const uint4 *src = reinterpret_cast<const uint4 *>(codes + (uint64_t)r[u] * DP);
#pragma unroll
                for (int i = 0; i < W4 / 4; i++) {
                    const uint4 v = src[i];
                    w[u][4 * i] = v.x;
                    w[u][4 * i + 1] = v.y;
                    w[u][4 * i + 2] = v.z;
                    w[u][4 * i + 3] = v.w;
                }
            } else {
                const uint32_t *src = reinterpret_cast<const uint32_t *>(codes + (uint64_t)r[u] * DP);
#pragma unroll
                for (int i = 0; i < W4; i++) w[u][i] = src[i];
            }
        }
#pragma unroll
        for (int u = 0; u < B; u++) {
            if (p + u >= p1) continue;
            if (k[u] != cur) {
                flush();
                cur = k[u];
            }
#pragma unroll
            for (int d = 0; d < DP; d++) {
                const uint32_t b = (w[u][d / 4] >> (8 * (d % 4))) & 0xFF;
                acc[d] += (b ^ 0x80u) << 16 | lo8[b];
            }
            acc[DP] += 1;
        }
    }
    // The lanes' last runs: consecutive lanes mostly share a code vector (the order is sorted),
    // so they are summed over the wave first and only each run's last lane adds to the global
    // sums (device-scope atomics on one address serialise: a large cell's thousands of lanes
    // cost ~400 us per level that way).  hi and lo apart (up to 512 rows per run).
    {
        const int lane = threadIdx.x & 63;
        const uint32_t key = acc[DP] ? cur : 0xFFFFFFFFu;
        const uint32_t prev = wave_prev_u32(key), next = wave_next_u32(key);
        const bool head = lane == 0 || prev != key;
        const uint32_t h = wave_scan_max(head ? (uint32_t)lane : 0u);
        const int src = h == 0 ? 0 : (int)h - 1;
        const bool tail = lane == 63 || next != key;
        auto seg = [&](uint32_t v) {   // the run's sum on its last lane
            const uint32_t pre = wave_scan_add(v);
            const uint32_t before = __shfl(pre, src);
            return pre - (h == 0 ? 0u : before);
        };
        const bool mine = tail && key != 0xFFFFFFFFu;
        const uint32_t slot = key - kbase;   // < SRT_SLOTS: the block table (u32: <= 2048 rows)
#pragma unroll
        for (int d = 0; d < DP; d++) {
            if ((uint32_t)d >= D) continue;   // (uniform; continue keeps the loop unrolled)
            const uint32_t hs = seg(acc[d] >> 16), ls = seg(acc[d] & 0xFFFF);
            if (mine) {
                if (slot < SRT_SLOTS) {
                    atomicAdd(&tab[slot * NS + d], hs);
                    atomicAdd(&tab[slot * NS + DP + d], ls);
                } else {
                    atomicAdd((unsigned long long *)&sums[(uint64_t)d * K + key], (unsigned long long)hs);
                    atomicAdd((unsigned long long *)&sums[KD + (uint64_t)d * K + key], (unsigned long long)ls);
                }
            }
        }
        const uint32_t cs = seg(acc[DP]);
        if (mine) {
            if (slot < SRT_SLOTS) atomicAdd(&tab[slot * NS + 2 * DP], cs);
            else atomicAdd((unsigned long long *)&sums[2 * KD + key], (unsigned long long)cs);
        }
    }
    __syncthreads();
    // the block's table to the global sums: one atomic per (code vector, term) per block
    for (uint32_t i = threadIdx.x; i < SRT_SLOTS * NS; i += 256) {
        const uint32_t slot = i / NS, c = i - slot * NS;
        if (tab[slot * NS + 2 * DP] == 0 || kbase + slot >= K) continue;   // no rows of it here
        const uint32_t k = kbase + slot;
        uint64_t *dst;
        if (c < DP) {
            if (c >= D) continue;
            dst = &sums[(uint64_t)c * K + k];
        } else if (c < 2 * DP) {
            if (c - DP >= D) continue;
            dst = &sums[KD + (uint64_t)(c - DP) * K + k];
        } else {
            dst = &sums[2 * KD + k];
        }
        atomicAdd((unsigned long long *)dst, (unsigned long long)tab[i]);
    }
}

bool sorted_sums_fits(uint32_t K) { return (size_t)K * 4 <= 64 * 1024; }

hipError_t launch_sorted_sums(hipStream_t s, uint32_t Dp, uint32_t G, const uint8_t *codes, uint64_t N,
                              const uint32_t *A, uint32_t K, uint32_t D, const uint64_t *plut, uint32_t *hist,
                              uint32_t *scratch, uint32_t *idx, uint32_t *ks, uint64_t *sums) {
    if (!sorted_sums_fits(K) || N == 0 || N > 0xFFFFFFFFull) return hipErrorInvalidValue;
    uint32_t *tot = scratch, *koff = scratch + K;
    const uint64_t rpg = (N + G - 1) / G;
    hipLaunchKernelGGL(sort_hist_kernel, dim3(G), dim3(SRT_THREADS), K * 4, s, A, N, K, rpg, hist, sums,
                       2 * (uint64_t)K * D + K);
    if (G <= 4 * CS_QG)
        hipLaunchKernelGGL(sort_colscan4_kernel, dim3((K + 63) / 64), dim3(256), 0, s, hist, G, K, tot);
    else
        hipLaunchKernelGGL(sort_colscan_kernel, dim3((K + 255) / 256), dim3(256), 0, s, hist, G, K, tot);
    hipLaunchKernelGGL(sort_koff_kernel, dim3(1), dim3(SRT_THREADS), 0, s, tot, K, koff);
    hipLaunchKernelGGL(sort_scatter_kernel, dim3(G), dim3(SRT_THREADS), K * 4, s, A, N, K, rpg, hist, koff, idx, ks);
    const uint64_t lanes = (N + SRT_ROWS_PER_LANE - 1) / SRT_ROWS_PER_LANE;
    const uint32_t grid = (uint32_t)((lanes + 255) / 256);
    switch (Dp) {
#define X(DPV)                                                                                                     \
    case DPV:                                                                                                      \
        hipLaunchKernelGGL(sorted_sums_kernel<DPV>, dim3(grid), dim3(256), 0, s, codes, N, idx, ks, K, D, plut, sums); \
        return hipGetLastError();
        QVQ_FOR_EACH_DP(X)
#undef X
    }
    return hipErrorInvalidValue;
}

// Column reduce of G slabs into sums (layout in the file header; common.hpp reduce_columns_block).
constexpr int REDUCE_THREADS = 1024;
__global__ __launch_bounds__(REDUCE_THREADS) void reduce_kernel(const uint64_t *__restrict__ part,
                                                                const uint32_t *__restrict__ part_cnt, uint32_t G,
                                                                uint32_t nsub, uint32_t K, uint32_t D,
                                                                uint64_t *__restrict__ sums, PubArgs pub) {
    if (pub.flag && blockIdx.x == 0 && threadIdx.x == 0) {   // the count (final: the recheck ran before)
        *reinterpret_cast<volatile uint32_t *>(pub.dst) = *pub.cnt;
        __threadfence_system();
        *reinterpret_cast<volatile uint64_t *>(pub.flag) = pub.seq;
    }
    __shared__ uint64_t red[2 * 16 * 64];
    reduce_columns_block(part, part_cnt, G, nsub, K, D, sums, blockIdx.x, red);
}

hipError_t launch_reduce(hipStream_t s, const uint64_t *part, const uint32_t *part_cnt, uint32_t G, uint32_t nsub,
                         uint32_t K, uint32_t D, uint64_t *sums, PubArgs pub) {
    if (nsub > G) return hipErrorInvalidValue;
    const uint64_t cols = (uint64_t)K * D + K;
    hipLaunchKernelGGL(reduce_kernel, dim3((int)((cols + 63) / 64)), dim3(REDUCE_THREADS), 0, s, part, part_cnt, G,
                       nsub, K, D, sums, pub);
    return hipGetLastError();
}

// K = 1 (the mean initialisation, trainingSetSum, src/Quantizer.cpp:46-57): every row in
// one cluster, so a register + LDS reduction; sums must be zero on entry (the engine's mean
// buffer is cleared once at creation and again by the finalize that consumes it).  A thread takes
// groups of 4 consecutive rows (4*DP bytes: DP/4 16-byte loads), two groups per trip so the
// loads of both are in flight together, and adds each component's exact term as
// (b ^ 0x80) << 16 | lo8[b] in u32 registers: the grid gives every thread at most 256 rows,
// so neither 16-bit field carries.  Block 0 also writes the quantize's initial state (the
// distortion inputs, zeroed counters), which saves two host calls per quantize.
constexpr int MEAN_THREADS = 1024;
constexpr uint64_t MEAN_ROWS_PER_THREAD = 256;
constexpr int MEAN_U = 4;   // groups of 4 rows in flight per thread
struct MeanInit {
    unsigned *zero;     // n_zero counters to clear
    uint32_t n_zero;
    double *dist;       // dist[0..1] = sum ||x||^2, rows (from the byte histogram)
    const uint64_t *hist;   // byte histogram of the training set (over all ranks)
    const double *v64;      // byte -> value
};

// dist[0] = sum_b hist[b] v(b)^2 and dist[1] = sum_b hist[b] / D, by one wave in a fixed order
// (double-double terms and a fixed lane tree): a function of the histogram only, so every rank
// count gives the same bits (the histogram is all-reduced exactly, as integers).
__device__ inline void dd_add(double &h, double &l, double b, double bl) {
    const double s = h + b, bb = s - h;
    const double e = (h - (s - bb)) + (b - bb);
    const double t = e + l + bl;
    h = s + t;
    l = t - (h - s);
}
__device__ void hist_moments(const uint64_t *hist, const double *v64, uint32_t D, double *dist) {
    const int lane = threadIdx.x;   // wave 0
    double h = 0, l = 0;
    uint64_t n = 0;
    for (int b = lane; b < 256; b += 64) {
        const double c = (double)hist[b];   // exact: < 2^53
        const double v2 = v64[b] * v64[b], v2l = __fma_rn(v64[b], v64[b], -v2);
        const double p = c * v2, pl = __fma_rn(c, v2, -p) + c * v2l;
        dd_add(h, l, p, pl);
        n += hist[b];
    }
    for (int off = 32; off >= 1; off >>= 1) {
        const double oh = __shfl_xor(h, off), ol = __shfl_xor(l, off);
        const uint64_t on = __shfl_xor(n, off);
        // both partners add the same pair in the same order: lane-independent result
        if (lane & off) dd_add(h, l, oh, ol);
        else {
            double hh = oh, ll = ol;
            dd_add(hh, ll, h, l);
            h = hh, l = ll;
        }
        n += on;
    }
    if (lane == 0) {
        dist[0] = h + l;
        dist[1] = (double)(n / D);
    }
}
// Per thread: the high parts u = b ^ 0x80 of the four components of a word are added two at a
// time as 16-bit fields (u of components 4q, 4q+2 in ue[q], of 4q+1, 4q+3 in uo[q]: three VALU
// per word), the low parts (<= 128 each) from a 256-BYTE LDS table (ds_read_u8: at most two
// lanes' dwords per bank, where a dword table conflicts up to 8-way), also as 16-bit fields.
// <= MEAN_ROWS_PER_THREAD rows per thread keep every field from carrying.
template <int DP>
__global__ __launch_bounds__(MEAN_THREADS) void mean_sums_kernel(const uint8_t *__restrict__ codes, uint64_t N,
                                                                 uint32_t D, const uint64_t *__restrict__ plut,
                                                                 uint64_t *__restrict__ sums, MeanInit init) {
    constexpr int Q3 = DP / 4;   // component quads (words per row)
    __shared__ uint8_t lo8[256];
    __shared__ uint32_t red[MEAN_THREADS / 64][DP][2];
    // the last block only initialises (the count, the distortion's moments, the zeroed words):
    // in block 0 of the summing grid that serial work held one CU's loads back by ~2 us
    const uint32_t nblk = gridDim.x - 1;
    if (blockIdx.x == nblk) {
        if (threadIdx.x == 0) sums[2 * D] = N;   // cnt[0]
        if (threadIdx.x < 64) hist_moments(init.hist, init.v64, D, init.dist);
        if (threadIdx.x < init.n_zero) init.zero[threadIdx.x] = 0;
        return;
    }
    if (threadIdx.x < 256) lo8[threadIdx.x] = (uint8_t)(plut[threadIdx.x] & 0xFF);
    __syncthreads();
    // low parts two components per register too: lo2[2q] = (4q, 4q+1), lo2[2q+1] = (4q+2, 4q+3)
    uint32_t ue[Q3], uo[Q3], lo2[DP / 2];
#pragma unroll
    for (int q = 0; q < Q3; q++) ue[q] = uo[q] = 0;
#pragma unroll
    for (int d = 0; d < DP / 2; d++) lo2[d] = 0;
    auto add_word = [&](uint32_t w, int q) {
        const uint32_t u = w ^ 0x80808080u;
        ue[q] += u & 0x00FF00FFu;
        uo[q] += (u >> 8) & 0x00FF00FFu;
#pragma unroll
        for (int j = 0; j < 4; j++) lo2[2 * q + j / 2] += (uint32_t)lo8[(w >> (8 * j)) & 0xFF] << (16 * (j & 1));
    };
    constexpr int Q = DP / 4;   // 16-byte loads per group of 4 rows
    const uint64_t groups = N / 4;
    uint64_t g_begin = 0;   // groups before this are done by the wave-chunk loop
    if constexpr (Q <= 4) {
        // Wave chunks of 64 groups (64 Q 16-byte words), loaded lane-contiguously: load j of lane
        // l is 16-byte word 64 j + l of the chunk, whose 4-byte word k is word 4(64 j + l) + k,
        // i.e. component quad (256 j + 4 l + k) mod Q.  Words go to slot (256 j + k) mod Q; the
        // lane's slots are rotated by 4 l mod Q at the end.  MEAN_U chunks per trip in flight.
        const uint64_t chunks = groups / 64;
        const uint64_t wave_id = (uint64_t)blockIdx.x * (MEAN_THREADS / 64) + (threadIdx.x >> 6);
        const uint64_t nwaves = (uint64_t)nblk * (MEAN_THREADS / 64);
        const int lane = threadIdx.x & 63;
        for (uint64_t c = wave_id; c < chunks; c += MEAN_U * nwaves) {
            uint4 v[MEAN_U][Q];
#pragma unroll
            for (int u = 0; u < MEAN_U; u++) {
                const uint64_t cu = c + u * nwaves < chunks ? c + u * nwaves : c;   // repeats skipped
                const uint4 *p = reinterpret_cast<const uint4 *>(codes + cu * 64 * 4 * DP);
#pragma unroll
                for (int j = 0; j < Q; j++) v[u][j] = p[64 * j + lane];
            }
#pragma unroll
            for (int u = 0; u < MEAN_U; u++) {
                if (u > 0 && c + u * nwaves >= chunks) break;
#pragma unroll
                for (int j = 0; j < Q; j++) {
                    add_word(v[u][j].x, (256 * j + 0) % Q);
                    add_word(v[u][j].y, (256 * j + 1) % Q);
                    add_word(v[u][j].z, (256 * j + 2) % Q);
                    add_word(v[u][j].w, (256 * j + 3) % Q);
                }
            }
        }
        // slot s of this lane holds quad (s + 4 lane) mod Q
        const uint32_t r = (4u * (uint32_t)lane) % Q;
        uint32_t e2[Q], o2[Q], l2[DP / 2];
#pragma unroll
        for (int qd = 0; qd < Q; qd++) {
            e2[qd] = o2[qd] = l2[2 * qd] = l2[2 * qd + 1] = 0;
#pragma unroll
            for (int sl = 0; sl < Q; sl++) {
                const bool hit = (uint32_t)((sl + r) % Q) == (uint32_t)qd;
                e2[qd] += hit ? ue[sl] : 0u;
                o2[qd] += hit ? uo[sl] : 0u;
                l2[2 * qd] += hit ? lo2[2 * sl] : 0u;
                l2[2 * qd + 1] += hit ? lo2[2 * sl + 1] : 0u;
            }
        }
#pragma unroll
        for (int qd = 0; qd < Q; qd++) {
            ue[qd] = e2[qd];
            uo[qd] = o2[qd];
            lo2[2 * qd] = l2[2 * qd];
            lo2[2 * qd + 1] = l2[2 * qd + 1];
        }
        g_begin = chunks * 64;
    }
    // groups past the wave chunks (every group for wide rows): one group per thread, MEAN_U
    // groups per trip with all their loads issued first
    constexpr int U = DP <= 16 ? MEAN_U : (DP <= 32 ? 2 : 1);   // (wide rows: fewer, by registers)
    const uint64_t stride = (uint64_t)nblk * MEAN_THREADS;
    for (uint64_t g = g_begin + (uint64_t)blockIdx.x * MEAN_THREADS + threadIdx.x; g < groups; g += U * stride) {
        if constexpr (DP > 32) {   // wide rows: the group's 16-byte loads one by one (registers)
            const uint4 *p = reinterpret_cast<const uint4 *>(codes + g * 4 * DP);
#pragma unroll
            for (int q = 0; q < Q; q++) {
                const uint4 w = p[q];
                add_word(w.x, (4 * q + 0) % Q3);
                add_word(w.y, (4 * q + 1) % Q3);
                add_word(w.z, (4 * q + 2) % Q3);
                add_word(w.w, (4 * q + 3) % Q3);
            }
            continue;
        }
        uint4 v[U][Q];
#pragma unroll
        for (int u = 0; u < U; u++) {
            const uint64_t gu = g + u * stride < groups ? g + u * stride : g;   // repeats are skipped
            const uint4 *p = reinterpret_cast<const uint4 *>(codes + gu * 4 * DP);
#pragma unroll
            for (int q = 0; q < Q; q++) v[u][q] = p[q];
        }
        // word i of the group holds components (i mod DP/4)*4 .. +3 of row i / (DP/4)
#pragma unroll
        for (int u = 0; u < U; u++) {
            if (u > 0 && g + u * stride >= groups) break;
#pragma unroll
            for (int q = 0; q < Q; q++) {
                add_word(v[u][q].x, (4 * q + 0) % Q3);
                add_word(v[u][q].y, (4 * q + 1) % Q3);
                add_word(v[u][q].z, (4 * q + 2) % Q3);
                add_word(v[u][q].w, (4 * q + 3) % Q3);
            }
        }
    }
    // the last N mod 4 rows, one per thread of block 0
    if (blockIdx.x == 0 && threadIdx.x < N % 4) {
        const uint32_t *w = reinterpret_cast<const uint32_t *>(codes + (groups * 4 + threadIdx.x) * DP);
#pragma unroll
        for (int q = 0; q < Q3; q++) add_word(w[q], q);
    }
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
#pragma unroll
    for (int d = 0; d < DP; d++) {
        // wave totals (< 2^22) by DPP scans on the VALU: lane 63 holds them
        const uint32_t f = (d & 1 ? uo[d / 4] : ue[d / 4]) >> (d & 2 ? 16 : 0);
        const uint32_t g = lo2[d / 2] >> (d & 1 ? 16 : 0);
        const uint32_t h = wave_scan_add(f & 0xFFFF), l = wave_scan_add(g & 0xFFFF);
        if (lane == 63) {
            red[wave][d][0] = h;
            red[wave][d][1] = l;
        }
    }
    __syncthreads();
    if (threadIdx.x < (unsigned)D) {
        uint64_t h = 0, l = 0;
        for (int w = 0; w < MEAN_THREADS / 64; w++) {
            h += red[w][threadIdx.x][0];
            l += red[w][threadIdx.x][1];
        }
        uint64_t *dst = sums + (blockIdx.x % MEAN_COPIES) * (2 * (uint64_t)D + 1);
        atomicAdd((unsigned long long *)&dst[threadIdx.x], (unsigned long long)h);
        atomicAdd((unsigned long long *)&dst[D + threadIdx.x], (unsigned long long)l);
    }
}

hipError_t launch_mean_sums(hipStream_t s, uint32_t Dp, const uint8_t *codes, uint64_t N, uint32_t D,
                            const uint64_t *plut, uint64_t *sums, unsigned *zero, uint32_t n_zero, double *dist,
                            const uint64_t *hist, const double *v64) {
    if (n_zero > MEAN_THREADS) return hipErrorInvalidValue;
    // one block per CU (few same-address atomics at the end), more only where a thread would
    // otherwise take over MEAN_ROWS_PER_THREAD rows (u32 fields)
    constexpr uint64_t grid_cap = 256;
    const uint64_t per_block = MEAN_THREADS * MEAN_ROWS_PER_THREAD;
    const uint64_t grid_min = (N + per_block - 1) / per_block;
    const uint64_t grid = std::max<uint64_t>(std::max<uint64_t>(grid_min, 1),
                                             std::min<uint64_t>((N + 4 * MEAN_THREADS - 1) / (4 * MEAN_THREADS), grid_cap));
    if (grid > 0x7FFFFFFFull) return hipErrorInvalidValue;
    const MeanInit init{zero, n_zero, dist, hist, v64};
    switch (Dp) {
#define X(DPV)                                                                                              \
    case DPV:                                                                                               \
        hipLaunchKernelGGL(mean_sums_kernel<DPV>, dim3((unsigned)grid + 1), dim3(MEAN_THREADS), 0, s, codes, N, D, plut, \
                           sums, init);                                                                     \
        return hipGetLastError();
        QVQ_FOR_EACH_DP(X)
#undef X
    }
    return hipErrorInvalidValue;
}

// Result hand-off at the end of a quantize: up to three device ranges copied in one launch
// straight into mapped pinned host memory (replacing three staged device-to-host copies).
struct CopySeg {
    const uint32_t *src;
    uint32_t *dst;
    uint64_t words;
};
struct CopySegs {
    CopySeg seg[3];
    uint64_t *flag;   // with a flag: the last block to finish publishes seq (mapped memory)
    uint64_t seq;
    unsigned *done;   // block counter for that (0 on entry, left at 0)
};
__global__ __launch_bounds__(256) void copy_out_kernel(CopySegs a) {
#pragma unroll
    for (int k = 0; k < 3; k++) {
        const CopySeg &c = a.seg[k];
        for (uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x; i < c.words; i += (uint64_t)gridDim.x * 256)
            c.dst[i] = c.src[i];
    }
    if (a.flag) {   // every wave's stores complete, one system-scope release per block, and
                    // the last block to count itself in publishes the flag
        __asm__ volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        if (threadIdx.x == 0) {
            __threadfence_system();
            if (atomicAdd(a.done, 1u) == gridDim.x - 1) {
                *a.done = 0;
                __threadfence_system();
                *reinterpret_cast<volatile uint64_t *>(a.flag) = a.seq;
            }
        }
    }
}

hipError_t launch_copy_out(hipStream_t s, const void *src0, void *dst0, uint64_t bytes0, const void *src1, void *dst1,
                           uint64_t bytes1, const void *src2, void *dst2, uint64_t bytes2, uint64_t *flag,
                           uint64_t seq, unsigned *done) {
    if (flag && !done) return hipErrorInvalidValue;
    if ((bytes0 | bytes1 | bytes2) & 3) return hipErrorInvalidValue;
    CopySegs a;
    a.seg[0] = {static_cast<const uint32_t *>(src0), static_cast<uint32_t *>(dst0), bytes0 / 4};
    a.seg[1] = {static_cast<const uint32_t *>(src1), static_cast<uint32_t *>(dst1), bytes1 / 4};
    a.seg[2] = {static_cast<const uint32_t *>(src2), static_cast<uint32_t *>(dst2), bytes2 / 4};
    a.flag = flag;
    a.seq = seq;
    a.done = done;
    const uint64_t words = std::max(bytes0, std::max(bytes1, bytes2)) / 4;
    const int grid = (int)std::min<uint64_t>(std::max<uint64_t>((words + 255) / 256, 1), 256);
    hipLaunchKernelGGL(copy_out_kernel, dim3(grid), dim3(256), 0, s, a);
    return hipGetLastError();
}

// finalize (src/Quantizer.cpp:79-94 fixCodebook + :129-138 split) fused with the next
// level's search tables.  Block = 256/L rows x L component lanes.  With split, row j < 2K is
// split code vector j (cluster j mod K, factor 1.2 for j < K, 0.8 above) and rows
// 2K..Kpad_next-1 are padding; the split codebook also goes to host_cb (mapped pinned
// memory, for the host's kd-tree build; then the K cells' row counts, u32).  L = 16, 32 or 64 lanes per row (>= Dp).  Without split (last level) row k < K writes
// centroid k and its distortion term sum_d (2 c S - n c^2).  The last block to finish sums
// the per-block distortion terms in block order and then publishes *ready = seq (system
// scope), which tells the host that host_cb holds the codebook.

struct FinArgs {
    const uint64_t *sums;
    uint32_t K, D, Dp;
    int64_t R, bias;
    int scale;
    double *C_cent;
    int split;
    double *C64n;
    uint32_t Kpad_next;
    double mu, sx, scale_t;
    float *C32;
    _Float16 *rows;
    float *E32;   // D = 12: expanded fp32 terms [c''(12) | n | 0 0 0] (small-K scan)
    double *host_cb;
    bool dist;
    uint64_t *zero_after;   // cleared by the last block once every block has read sums (mean)
    uint32_t n_zero;
    uint32_t ncopy;         // copies of the sums to add: the mean's MEAN_COPIES, or 2 (kd_reduce_kernel)
    uint64_t cstride;       // u64 from one copy to the next (2KD + K, or the capacity's)
    const unsigned *gate;   // non-null: copies past the first only when *gate != 0 (the level's
                            // tie count: without ties copy 1 is all zero, read nor cleared)
    uint32_t *perm;         // split: the next search's tile order (prune_order), or null
    int32_t *tint;
    float *qproj;           // with perm: the split code vectors' projections (finalize_split_item)
    TieExport ties;         // out != null: the level's tie rows to mapped memory (TieExport)
};

// A split row j (< 2K: child of code vector j mod K, from that code vector's sums hs, ls, cnt of
// component d; Kpad_next > j >= 2K: padding) -- its C64n / C32 / host values and the MFMA tables.
__device__ inline void finalize_split_item(const FinArgs &a, uint32_t j, uint32_t d, uint32_t L, uint64_t hs,
                                           uint64_t ls, uint64_t cnt) {
    const uint32_t K = a.K, D = a.D, Dp = a.Dp;
    if (j < 2 * K) {
        const uint32_t k = j < K ? j : j - K;
        double v = 0;
        if (d < D) {
            const double cv = centroid_value(hs, ls, cnt, a.R, a.bias, a.scale);
            if (j < K) a.C_cent[(uint64_t)k * D + d] = cv;
            v = cv * (j < K ? (double)(1 + 0.2) : (double)(1 - 0.2));
            a.C64n[(uint64_t)j * D + d] = v;
            if (a.host_cb) a.host_cb[(uint64_t)j * D + d] = v;
        }
        // after the split rows: the K cells' row counts (the tie check: a cell of <= 2 rows has
        // the reference's bits, a Kahan sum of one or two values being the rounded exact sum)
        if (a.host_cb && j < K && d == 0)
            reinterpret_cast<uint32_t *>(a.host_cb + 2ull * K * D)[k] = cnt > 0xFFFFFFFFull ? 0xFFFFFFFFu : (uint32_t)cnt;
        if (d < Dp) a.C32[(uint64_t)j * Dp + d] = (float)v;
        if (a.rows) {   // MFMA row (common.hpp): hi / lo at their slots, norm at 2 LO
            const uint32_t RF = cb_row_f16(D, Dp), LO = cb_lo_off(D, Dp);
            _Float16 *row = a.rows + (uint64_t)j * RF;
            const double cp = d < D ? v - a.mu : 0.0;
            if (a.qproj) {   // the projection sum_d (c_d - mu) / sx for prune_order (any order: it
                             // is widened by 1 there)
                double qs = cp;
                for (uint32_t off = L / 2; off >= 1; off >>= 1) qs += __shfl_xor(qs, (int)off, (int)L);
                if (d == 0) a.qproj[j] = (float)(qs / a.sx);
            }
            double n = cp * cp;   // L >= LO lanes per row
            for (uint32_t off = L / 2; off >= 1; off >>= 1) n += __shfl_xor(n, (int)off, (int)L);
            if (d < D) {
                const double c2 = -2.0 * a.sx * cp * a.scale_t;
                const _Float16 h = (_Float16)(float)c2;
                row[cb_hi_slot(D, Dp, d)] = h;
                row[cb_lo_slot(D, Dp, d)] = (_Float16)(float)(c2 - (double)(float)h);
            } else if (d < LO) {
                row[cb_hi_slot(D, Dp, d)] = (_Float16)0.f;
                row[cb_lo_slot(D, Dp, d)] = (_Float16)0.f;
            }
            n *= a.scale_t;
            const _Float16 h = (_Float16)(float)n;
            const _Float16 l = (_Float16)(float)(n - (double)(float)h);
            for (uint32_t i = 2 * LO + d; i < RF; i += L)
                row[i] = i == 2 * LO ? h : (i == 2 * LO + 1 ? l : (_Float16)0.f);
            if (a.E32 && d < 16)   // L = 16 lanes for D = 12
                a.E32[(uint64_t)j * 16 + d] =
                    d < D ? (float)(-2.0 * a.sx * cp * a.scale_t) : (d == D ? (float)n : 0.f);
        }
    } else if (j < a.Kpad_next) {
        if (d < Dp) a.C32[(uint64_t)j * Dp + d] = 0.f;
        if (a.E32 && d < 16) a.E32[(uint64_t)j * 16 + d] = d == D ? 1e30f : 0.f;   // never wins
        if (a.rows) {
            const uint32_t RF = cb_row_f16(D, Dp), LO = cb_lo_off(D, Dp);
            _Float16 *row = a.rows + (uint64_t)j * RF;
            for (uint32_t i = d; i < RF; i += L)
                row[i] = (_Float16)(i == 2 * LO || i == 2 * LO + 1 ? MF_PAD_SCORE : 0.f);
        }
    }
}

// One (row j, component lane d) item of the finalize; L lanes per row (16 when D == 12: the
// norm of a row is a 16-lane butterfly).  Returns the item's distortion term (no split).
__device__ inline double finalize_item(const FinArgs &a, uint32_t j, uint32_t d, uint32_t L) {
    const uint32_t K = a.K, D = a.D;
    const uint64_t KD = (uint64_t)K * D;
    const uint32_t ncopy = a.gate && *a.gate == 0 ? 1 : a.ncopy;
    auto sums_at = [&](uint64_t i) {   // the sum of the ncopy copies
        uint64_t v = a.sums[i];
        for (uint32_t c = 1; c < ncopy; c++) v += a.sums[c * a.cstride + i];
        return v;
    };
    if (a.split) {
        const uint32_t k = j < K ? j : j - K;
        const uint64_t c = (uint64_t)d * K + k;
        const bool have = j < 2 * K && d < D;
        finalize_split_item(a, j, d, L, have ? sums_at(c) : 0, have ? sums_at(KD + c) : 0,
                            j < 2 * K ? sums_at(2 * KD + k) : 0);
        return 0.0;
    }
    if (j < K && d < D) {
        const uint64_t c = (uint64_t)d * K + j;
        const uint64_t cnt = sums_at(2 * KD + j), hs = sums_at(c), ls = sums_at(KD + c);
        const double cv = centroid_value(hs, ls, cnt, a.R, a.bias, a.scale);
        a.C_cent[(uint64_t)j * D + d] = cv;
        if (a.dist && cnt) {
            const __int128 Sq = (__int128)a.R * (__int128)hs + (__int128)ls - (__int128)a.bias * (__int128)cnt;
            const double S = ldexp(i128_to_double(Sq), -a.scale);
            return 2.0 * cv * S - (double)cnt * cv * cv;
        }
    }
    return 0.0;
}

// The next search's code-vector order for tile pruning (assign_mf32_kernel / assign_wide_kernel
// PRUNE): the K2 split code vectors bucket-sorted by their projection q = sum_d (c_d - mu) / sx on
// the all-ones direction (in the units of a row's sum_d w_d, w the centred byte integers), so that
// each 32-code-vector tile spans a short q interval.  perm[p] = the code vector at position p
// (padding positions K2 .. Kpad map to themselves); tint[2t], tint[2t + 1] = tile t's envelope:
// the floor / ceil of its q interval widened by 1 (empty tile: INT_MAX, INT_MIN), then the suffix
// minimum of the lows and the prefix maximum of the highs.  Any grouping keeps the search exact
// (the bound holds for every tile); the sort only makes it prune.  Run by the finalize's last
// block (any size >= 256: threads past 256 only meet the barriers), K2 <= PRUNE_MAXK.
constexpr uint32_t PRUNE_MAXK = 4096, PRUNE_NB = 256, PRUNE_MAXT = PRUNE_MAXK / 32;
__device__ void prune_order(const float *__restrict__ qproj, uint32_t K2, uint32_t Kpad, uint32_t *__restrict__ perm,
                            int32_t *__restrict__ tint) {
    __shared__ float q[PRUNE_MAXK];
    __shared__ float qs[PRUNE_MAXK];   // q by position
    __shared__ uint32_t hist[PRUNE_NB];
    __shared__ int32_t tlo[PRUNE_MAXT], thi[PRUNE_MAXT];
    __shared__ uint32_t wtot[4], wlo[4], whi[4];
    const uint32_t tid = threadIdx.x;
    const bool act = tid < 256;
    float mn = INFINITY, mx = -INFINITY;
    for (uint32_t j = tid; act && j < K2; j += 256) {   // (the finalize items wrote them)
        q[j] = __builtin_nontemporal_load(&qproj[j]);
        mn = fminf(mn, q[j]);
        mx = fmaxf(mx, q[j]);
    }
    // the range of q: DPP wave minima of the floats as order-preserving u32, then the four waves'
    auto ford = [](float f) {
        const uint32_t b = __float_as_uint(f);
        return b ^ ((b >> 31) ? 0xFFFFFFFFu : 0x80000000u);
    };
    auto fdec = [](uint32_t u) { return __uint_as_float(u ^ ((u >> 31) ? 0x80000000u : 0xFFFFFFFFu)); };
    const uint32_t umn = wave_min_u32(ford(mn)), umx = ~wave_min_u32(~ford(mx));
    if (act) {
        hist[tid] = 0;
        if ((tid & 63) == 0) {
            wlo[tid >> 6] = umn;
            whi[tid >> 6] = umx;
        }
    }
    __syncthreads();
    const float qmin = fdec(min(min(wlo[0], wlo[1]), min(wlo[2], wlo[3])));
    const float qmax = fdec(max(max(whi[0], whi[1]), max(whi[2], whi[3])));
    const float inv = (float)PRUNE_NB / (qmax - qmin + 1.0f);
    auto bucket = [&](float v) { return min((uint32_t)((v - qmin) * inv), PRUNE_NB - 1); };
    if (act)
        for (uint32_t j = tid; j < K2; j += 256) atomicAdd(&hist[bucket(q[j])], 1u);
    __syncthreads();
    {   // exclusive scan of the 256 bucket counts (one per thread): DPP scans within the four
        // waves, then each wave adds the totals of the waves before it (two barriers, not 16)
        static_assert(PRUNE_NB == 256, "one bucket per thread");
        const uint32_t own = act ? hist[tid] : 0u;
        const uint32_t inc = wave_scan_add(own);
        if (act && (tid & 63) == 63) wtot[tid >> 6] = inc;
        __syncthreads();
        uint32_t pre = 0;
        for (uint32_t w = 0; act && w < (tid >> 6); w++) pre += wtot[w];
        if (act) hist[tid] = pre + inc - own;
    }
    __syncthreads();
    if (act) {
        for (uint32_t j = tid; j < K2; j += 256) {   // (order inside a bucket: any)
            const uint32_t p = atomicAdd(&hist[bucket(q[j])], 1u);
            perm[p] = j;
            qs[p] = q[j];
        }
        for (uint32_t p = K2 + tid; p < Kpad; p += 256) perm[p] = p;
    }
    __syncthreads();
    // tile t = positions 32t .. 32t + 31: thread t < nt scans its tile
    const uint32_t nt = Kpad / 32;
    if (act && tid < nt) {
        float lo = INFINITY, hi = -INFINITY;
        for (uint32_t p = 32 * tid; p < min(32 * tid + 32, K2); p++) {
            lo = fminf(lo, qs[p]);
            hi = fmaxf(hi, qs[p]);
        }
        tlo[tid] = lo <= hi ? (int32_t)floorf(lo) - 1 : 0x7FFFFFFF;
        thi[tid] = lo <= hi ? (int32_t)ceilf(hi) + 1 : (int32_t)0x80000000;
    }
    // Tiles sharing a bucket can overlap out of order: monotone envelopes (lo: the suffix
    // minimum, hi: the prefix maximum; still bounds of every tile), so that the tiles a bound
    // admits form one contiguous range.  DPP max-scans over nt <= 128 entries in two waves (the
    // lows in reversed tile order, mapped so that a smaller int is a larger u32; 0 is the
    // neutral value of both maps, as INT_MAX / INT_MIN are of the envelopes).
    __syncthreads();
    const int r = (int)nt - 1 - (int)tid;   // this thread's tile for the suffix scan
    uint32_t hm = act && tid < nt ? (uint32_t)thi[tid] ^ 0x80000000u : 0u;
    uint32_t lm = act && r >= 0 ? ~((uint32_t)tlo[r] ^ 0x80000000u) : 0u;
    hm = wave_scan_max(hm);
    lm = wave_scan_max(lm);
    if (act && (tid & 63) == 63) {
        whi[tid >> 6] = hm;
        wlo[tid >> 6] = lm;
    }
    __syncthreads();
    for (uint32_t w = 0; act && w < (tid >> 6); w++) {
        hm = max(hm, whi[w]);
        lm = max(lm, wlo[w]);
    }
    if (act && tid < nt) tint[2 * tid + 1] = (int32_t)(hm ^ 0x80000000u);
    if (act && r >= 0) tint[2 * r] = (int32_t)(~lm ^ 0x80000000u);
}

__device__ inline uint32_t fin_rows(const FinArgs &a) { return a.split ? max(2 * a.K, a.Kpad_next) : a.K; }

// Grid-stride over groups of 256/L rows.  Each wave fences its mapped-host writes once, after
// its last row (a system fence writes back the L2: per row it cost ~25 ns x rows).
// The end of a finalize block: its distortion partial (red: blockDim doubles of LDS, tree order
// over the block's threads; none without red), the done count, and in the last block the
// distortion total (block order), the clearing, the next search's tile order and the host's
// ready number.
__device__ void finalize_block_done(const FinArgs &a, double term, double *red, double *__restrict__ dist_part,
                                    unsigned *__restrict__ done, double *__restrict__ dist_out,
                                    volatile uint64_t *ready, uint64_t seq) {
    __shared__ bool last;
    // one block (small codebooks): no count and no agent fence, only the system fence before the
    // ready number (two fences of ~2-3.5 us each were most of a small level's finalize)
    const bool one = gridDim.x == 1;
    if (red) red[threadIdx.x] = term;
    // host_cb: every wave's mapped stores complete before the barrier, and thread 0's
    // system-scope fence below releases them with the block's count (MI355X guide's
    // producer pattern: one fence per block, not one per thread)
    if (a.host_cb || a.ties.out) __asm__ volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (red)
        for (int w = (int)blockDim.x / 2; w > 0; w >>= 1) {
            if ((int)threadIdx.x < w) red[threadIdx.x] += red[threadIdx.x + w];
            __syncthreads();
        }
    if (threadIdx.x == 0) {
        if (one) {
            last = true;
        } else {
            if (red) dist_part[blockIdx.x] = red[0];
            if (a.host_cb || a.ties.out) __threadfence_system();
            else __threadfence();
            last = atomicAdd(done, 1u) == gridDim.x - 1;
        }
    }
    __syncthreads();
    if (!last) return;
    if (one) {
        if (dist_out && threadIdx.x == 0) dist_out[0] = red[0];
    } else {
        __threadfence();
    }
    if (dist_out && !one) {   // the block partials, loaded in parallel, then added in block order
        __shared__ double parts[512];
        for (uint32_t b = threadIdx.x; b < gridDim.x; b += blockDim.x) parts[b] = __builtin_nontemporal_load(&dist_part[b]);
        __syncthreads();
        if (threadIdx.x == 0) {
            double t = 0;
            for (uint32_t b = 0; b < gridDim.x; b++) t += parts[b];
            dist_out[0] = t;
        }
    }
    if (!a.gate || *a.gate)
        for (uint32_t i = threadIdx.x; i < a.n_zero; i += blockDim.x) a.zero_after[i] = 0;
    if (a.perm) prune_order(a.qproj, 2 * a.K, a.Kpad_next, a.perm, a.tint);
    if (threadIdx.x == 0) {
        *done = 0;
        if (ready) {
            __threadfence_system();
            *ready = seq;
        }
    }
}

// Grid-stride over groups of 256/L rows.  Each wave fences its mapped-host writes once, after
// its last row (a system fence writes back the L2: per row it cost ~25 ns x rows).
__global__ __launch_bounds__(256) void finalize_prep_kernel(FinArgs a, double *__restrict__ dist_part,
                                                            unsigned *__restrict__ done, double *__restrict__ dist_out,
                                                            volatile uint64_t *ready, uint64_t seq, uint32_t L) {
    const uint32_t d = threadIdx.x % L, r = threadIdx.x / L;
    const uint32_t per = 256 / L, n = fin_rows(a);
    double term = 0.0;
    for (uint32_t j0 = blockIdx.x * per; j0 < n; j0 += gridDim.x * per) term += finalize_item(a, j0 + r, d, L);
    if (a.ties.out) {   // the tie rows, a thread per 4 bytes of a row record
        const TieExport &t = a.ties;
        const uint32_t nt = *t.cnt, m = min(nt, t.cap), words = 2 + a.Dp / 4;
        uint32_t *o = reinterpret_cast<uint32_t *>(t.out);
        if (blockIdx.x == 0 && threadIdx.x == 0) o[0] = nt;
        for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < (uint64_t)m * words;
             i += (uint64_t)gridDim.x * blockDim.x) {
            const uint32_t k = (uint32_t)(i / words), w = (uint32_t)(i % words), row = t.rows[k];
            if (row >= t.n_rows) {   // (never: the recheck lists rows)
                o[2 + i] = ~0u;
                continue;
            }
            o[2 + i] = w == 0 ? row
                              : (w == 1 ? t.A[row] : reinterpret_cast<const uint32_t *>(t.codes + (uint64_t)row * a.Dp)[w - 2]);
        }
    }
    if (!done) return;
    __shared__ double red[256];
    // (the distortion's block tree only on the level that returns it: 8 barriers fewer elsewhere)
    finalize_block_done(a, term, a.dist ? red : nullptr, dist_part, done, dist_out, ready, seq);
}

static FinArgs fin_args(const uint64_t *sums, uint32_t K, uint32_t D, uint32_t Dp, int64_t R, int64_t bias,
                        int scale, double *C_cent, bool split, double *C64n, uint32_t Kpad_next, double mu, double sx,
                        int t, float *C32, _Float16 *cb_rows, float *E32, double *host_cb, bool dist) {
    FinArgs a;
    a.sums = sums;
    a.K = K;
    a.D = D;
    a.Dp = Dp;
    a.R = R;
    a.bias = bias;
    a.scale = scale;
    a.C_cent = C_cent;
    a.split = split ? 1 : 0;
    a.C64n = C64n;
    a.Kpad_next = Kpad_next;
    a.mu = mu;
    a.sx = sx;
    a.scale_t = std::ldexp(1.0, t);
    a.C32 = C32;
    a.rows = cb_rows;
    a.E32 = D == MF_D ? E32 : nullptr;
    a.host_cb = host_cb;
    a.dist = dist;
    a.zero_after = nullptr;
    a.n_zero = 0;
    a.ncopy = 1;
    a.cstride = 2 * (uint64_t)K * D + K;
    a.gate = nullptr;
    a.perm = nullptr;
    a.tint = nullptr;
    a.qproj = nullptr;
    a.ties = TieExport();
    return a;
}

constexpr uint32_t FIN_ONE_BLOCK_ROWS = 64;   // split rows: K <= 32
hipError_t launch_finalize_prep(hipStream_t s, const uint64_t *sums, uint32_t K, uint32_t D, uint32_t Dp, int64_t R,
                                int64_t bias, int scale, double *C_cent, bool split, double *C64n, uint32_t Kpad_next,
                                double mu, double sx, int t, float *C32, _Float16 *cb_rows, float *E32,
                                double *host_cb, double *dist_part, unsigned *done, double *dist_out, uint64_t *ready,
                                uint64_t seq, bool zero_sums, uint32_t ncopy, uint32_t *perm, int32_t *tint,
                                uint32_t zero_skip, uint64_t copy_stride, const unsigned *copy_gate,
                                const TieExport &ties) {
    if (D == 0 || D > 64) return hipErrorInvalidValue;
    if (ties.out && (!done || !ready || !ties.rows || !ties.cnt || !ties.A || !ties.codes || (Dp & 3) || !ties.n_rows))
        return hipErrorInvalidValue;   // released with the ready flag
    if (zero_sums && !done) return hipErrorInvalidValue;   // the clearing is the last block's
    const uint32_t L = D <= 16 ? 16 : (D <= 32 ? 32 : 64);
    const uint32_t n = split ? std::max(2 * K, Kpad_next) : K;
    // <= dist_part capacity; small codebooks in one block (the grid-stride loop takes several rows
    // per thread), which needs no cross-block count or fence (finalize_block_done)
    const uint32_t grid = n <= FIN_ONE_BLOCK_ROWS ? 1u : std::min<uint32_t>((n + 256 / L - 1) / (256 / L), 512);
    FinArgs a = fin_args(sums, K, D, Dp, R, bias, scale, C_cent, split, C64n, Kpad_next, mu, sx, t, C32, cb_rows,
                         E32, host_cb, dist_out != nullptr);
    a.ncopy = ncopy ? ncopy : 1;
    a.gate = copy_gate;
    a.ties = ties;
    if (copy_stride) {
        if (copy_stride < 2 * (uint64_t)K * D + K) return hipErrorInvalidValue;
        a.cstride = copy_stride;
    }
    if (perm) {   // the last block orders the next search's code vectors (needs the done counter)
        if (!done || !split || 2 * K > PRUNE_MAXK || Kpad_next % 32 || Kpad_next > PRUNE_MAXK) return hipErrorInvalidValue;
        a.perm = perm;
        a.tint = tint;
        a.qproj = reinterpret_cast<float *>(tint + 2 * PRUNE_MAXT);   // (the envelopes' region is fixed)
    }
    if (zero_sums) {   // copies zero_skip .. ncopy - 1
        if (zero_skip >= a.ncopy) return hipErrorInvalidValue;
        a.zero_after = const_cast<uint64_t *>(sums) + (uint64_t)zero_skip * a.cstride;
        a.n_zero = (uint32_t)((a.ncopy - zero_skip - 1) * a.cstride + 2 * (uint64_t)K * D + K);
    }
    hipLaunchKernelGGL(finalize_prep_kernel, dim3(grid), dim3(256), 0, s, a, dist_part, done, dist_out,
                       (volatile uint64_t *)ready, seq, L);
    return hipGetLastError();
}

// finalize without the tables (qvq_update): C_cent only.
hipError_t launch_finalize(hipStream_t s, const uint64_t *sums, uint32_t K, uint32_t D, int64_t R, int64_t bias,
                           int scale, double *C_cent) {
    return launch_finalize_prep(s, sums, K, D, (D + 3) & ~3u, R, bias, scale, C_cent, false, nullptr, 0, 0, 0, 0,
                                nullptr, nullptr, nullptr, nullptr, nullptr, nullptr, nullptr, nullptr, 0, false, 1,
                                nullptr, nullptr, 0, 0, nullptr);
}

// Search tables from an fp64 codebook: fp32 [Kpad][Dp] (VALU path and the MFMA recompute)
// and the f16 MFMA rows (D = 12 or wide layout, common.hpp).  Code vectors K..Kpad-1 are padding
// that never wins.
__device__ inline void prep_row(const double *v, uint32_t D, uint32_t Dp, double mu, double sx, double scale_t,
                                float *__restrict__ c32, _Float16 *__restrict__ r, float *__restrict__ e32) {
    const uint32_t RF = cb_row_f16(D, Dp), LO = cb_lo_off(D, Dp);
    double n = 0;
    for (uint32_t i = 0; i < RF; i++) r[i] = (_Float16)0.f;
    for (uint32_t d = 0; d < Dp; d++) {
        const double x = d < D ? v[d] : 0.0;
        c32[d] = (float)x;
        if (d < D) {
            const double cp = x - mu;
            n += cp * cp;
            const double c2 = -2.0 * sx * cp * scale_t;
            const _Float16 h = (_Float16)(float)c2;
            r[cb_hi_slot(D, Dp, d)] = h;
            r[cb_lo_slot(D, Dp, d)] = (_Float16)(float)(c2 - (double)(float)h);
            if (e32) e32[d] = (float)c2;
        }
    }
    n *= scale_t;
    if (e32)
        for (uint32_t d = D; d < 16; d++) e32[d] = d == D ? (float)n : 0.f;
    const _Float16 h = (_Float16)(float)n;
    r[2 * LO] = h;
    r[2 * LO + 1] = (_Float16)(float)(n - (double)(float)h);
}

__device__ inline void prep_pad_row(uint32_t D, uint32_t Dp, float *__restrict__ c32, _Float16 *__restrict__ r,
                                    float *__restrict__ e32) {
    const uint32_t RF = cb_row_f16(D, Dp), LO = cb_lo_off(D, Dp);
    for (uint32_t d = 0; d < Dp; d++) c32[d] = 0.f;
    if (e32)
        for (uint32_t d = 0; d < 16; d++) e32[d] = d == D ? 1e30f : 0.f;   // never wins
    for (uint32_t i = 0; i < RF; i++) r[i] = (_Float16)0.f;
    r[2 * LO] = (_Float16)MF_PAD_SCORE;
    r[2 * LO + 1] = (_Float16)MF_PAD_SCORE;
}

__global__ void prep_kernel(const double *__restrict__ C64, uint32_t K, uint32_t Kpad, uint32_t D, uint32_t Dp,
                            double mu, double sx, double scale_t, float *__restrict__ C32,
                            _Float16 *__restrict__ rows, float *__restrict__ E32) {
    const uint32_t RF = cb_row_f16(D, Dp);
    for (uint32_t k = blockIdx.x * blockDim.x + threadIdx.x; k < Kpad; k += gridDim.x * blockDim.x) {
        float *e32 = E32 ? E32 + (uint64_t)k * 16 : nullptr;
        if (k >= K) {
            prep_pad_row(D, Dp, C32 + (uint64_t)k * Dp, rows + (uint64_t)k * RF, e32);
            continue;
        }
        double v[64];
        for (uint32_t d = 0; d < D; d++) v[d] = C64[(uint64_t)k * D + d];
        prep_row(v, D, Dp, mu, sx, scale_t, C32 + (uint64_t)k * Dp, rows + (uint64_t)k * RF, e32);
    }
}

hipError_t launch_prep(hipStream_t s, const double *C64, uint32_t K, uint32_t Kpad, uint32_t D, uint32_t Dp,
                       double mu, double sx, int t, float *C32, _Float16 *cb_rows, float *E32) {
    hipLaunchKernelGGL(prep_kernel, dim3((Kpad + 255) / 256), dim3(256), 0, s, C64, K, Kpad, D, Dp, mu, sx,
                       std::ldexp(1.0, t), C32, cb_rows, D == MF_D ? E32 : nullptr);
    return hipGetLastError();
}

// out[i] = codes of row rows[i] (rows the host kd-tree resolves).
__global__ void gather_codes_kernel(const uint8_t *__restrict__ codes, uint32_t Dp, const uint32_t *__restrict__ rows,
                                    uint32_t n, uint8_t *__restrict__ out) {
    for (uint64_t t = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; t < (uint64_t)n * Dp;
         t += (uint64_t)gridDim.x * blockDim.x) {
        const uint64_t i = t / Dp, d = t - i * Dp;
        out[t] = codes[(uint64_t)rows[i] * Dp + d];
    }
}

hipError_t launch_gather_codes(hipStream_t s, const uint8_t *codes, uint32_t Dp, const uint32_t *rows, uint32_t n,
                               uint8_t *out) {
    hipLaunchKernelGGL(gather_codes_kernel, dim3((int)std::min<uint64_t>(((uint64_t)n * Dp + 255) / 256, 4096)),
                       dim3(256), 0, s, codes, Dp, rows, n, out);
    return hipGetLastError();
}

// A[rows[i]] = vals[i] (host tie resolutions).
// Host-resolved tie rows: A[rows[i]] = vals[i], and with xslab the row's terms move from its
// provisional index (the search's, still in A) to the new one: added to slab G (xslab,
// xcnt) at the new index and to slab G + 1 (subtracted by the reduce) at the old one.  One
// wave per row.
__global__ void fix_rows_kernel(const uint8_t *__restrict__ codes, uint32_t Dp, uint32_t D, uint32_t *__restrict__ A,
                                const uint32_t *__restrict__ rows, const uint32_t *__restrict__ vals, uint32_t n,
                                uint32_t K, uint64_t *__restrict__ xslab, uint32_t *__restrict__ xcnt,
                                const uint64_t *__restrict__ plut, uint64_t *__restrict__ xsums) {
    const uint32_t lane = threadIdx.x & 63;
    for (uint32_t i = (blockIdx.x * blockDim.x + threadIdx.x) / 64; i < n; i += gridDim.x * blockDim.x / 64) {
        const uint32_t row = rows[i], to = vals[i];
        const uint32_t from = A[row];
        if (from != to && xslab) move_row_terms(codes, Dp, D, row, from, to, K, xslab, xcnt, plut, lane);
        else if (from != to && xsums) move_row_sums(codes, Dp, D, row, from, to, K, xsums, plut, lane);
        if (lane == 0) A[row] = to;
    }
}

hipError_t launch_fix_rows(hipStream_t s, const uint8_t *codes, uint32_t Dp, uint32_t D, uint32_t *A,
                           const uint32_t *rows, const uint32_t *vals, uint32_t n, uint32_t K, uint64_t *xslab,
                           uint32_t *xcnt, const uint64_t *plut, uint64_t *xsums) {
    if (n == 0) return hipSuccess;
    const int blocks = (int)std::min<uint32_t>((n + 3) / 4, 1024);
    hipLaunchKernelGGL(fix_rows_kernel, dim3(blocks), dim3(256), 0, s, codes, Dp, D, A, rows, vals, n, K, xslab, xcnt,
                       plut, xsums);
    return hipGetLastError();
}

// Histogram of the bytes of the first D components of every row (for sum ||x||^2).
__global__ void byte_hist_kernel(const uint8_t *__restrict__ codes, uint64_t N, uint32_t D, uint32_t Dp,
                                 unsigned long long *__restrict__ hist) {
    __shared__ uint32_t h[256];
    h[threadIdx.x] = 0;
    __syncthreads();
    const uint64_t total = N * Dp;
    for (uint64_t i = (blockIdx.x * (uint64_t)blockDim.x + threadIdx.x) * 4; i < total;
         i += (uint64_t)gridDim.x * blockDim.x * 4) {
        const uint32_t w = *(const uint32_t *)(codes + i);   // Dp is a multiple of 4
        const uint32_t d0 = (uint32_t)(i % Dp);
#pragma unroll
        for (int j = 0; j < 4; j++)
            if (d0 + j < D) atomicAdd(&h[(w >> (8 * j)) & 0xFF], 1u);
    }
    __syncthreads();
    if (h[threadIdx.x]) atomicAdd(&hist[threadIdx.x], (unsigned long long)h[threadIdx.x]);
}

hipError_t launch_byte_hist(hipStream_t s, const uint8_t *codes, uint64_t N, uint32_t D, uint32_t Dp,
                            uint64_t *hist) {
    hipError_t e = hipMemsetAsync(hist, 0, 256 * 8, s);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(byte_hist_kernel, dim3(1024), dim3(256), 0, s, codes, N, D, Dp, (unsigned long long *)hist);
    return hipGetLastError();
}

}  // namespace qvq

namespace qvq {

// Decode (CompressedImage::decompress, src/Compressor.cpp:156-165 over getImageFromVectors,
// src/Compressor.cpp:64-85 there): gather code-vector bytes into the raster.  Each output
// pixel is computed by one thread, so there are no write races.  The reference writes block
// by block in loop order (i, j, dx, dy), "last writer wins", and a block column that
// overhangs ySize wraps into the next raster row(s).  Pixel (x, y) = P / ys, P % ys is
// written by (x - m, y + m*ys) for every m >= 0 with y + m*ys < hB*h; the last of them in
// that order has the largest block row i, then the largest j, then the largest dx.  Only m
// <= dx0 = x % w keep i = x / w; j grows with m, and among equal j the smallest m wins:
//   M = min(dx0, (yspan - 1 - y) / ys),  jM = (y + M*ys) / h,  m* = max(0, ceil((jM*h - y)/ys)).
// Without an overhang (ys % h == 0) m* = 0 for every pixel: a plain gather.
// Out-of-range indices (undefined behaviour in the reference, which indexes codeVectors with
// operator[]) write 0 and raise *bad.  With orig the kernel also sums the raport's squared
// signed-byte differences (src/Compressor.cpp:137-146) into *sqerr.
struct DecodeArgs {
    const uint8_t *cb;
    uint32_t K, D;
    const uint32_t *A;
    uint32_t xs, ys, w, h, hB, yspan, overhang;
    uint8_t *rgb;
    const uint8_t *orig;
    unsigned long long *sqerr;
    uint32_t *bad;
};

// (block index, byte offset in its code vector) of the last writer of pixel (x, y)
__device__ inline void decode_writer(const DecodeArgs &a, uint32_t x, uint32_t y, uint32_t i0, uint32_t dx0,
                                     uint32_t &blk, uint32_t &off) {
    uint32_t m = 0;
    if (y < a.overhang && dx0 > 0) {
        const uint32_t M = min(dx0, (a.yspan - 1 - y) / a.ys);
        const uint32_t jM = (y + M * a.ys) / a.h;
        const uint32_t need = jM * a.h;   // >= y is not guaranteed: clamp at 0
        m = need > y ? (need - y + a.ys - 1) / a.ys : 0;
    }
    const uint32_t yp = y + m * a.ys, j = yp / a.h;
    blk = i0 * a.hB + j;
    off = ((dx0 - m) * a.h + (yp - j * a.h)) * 3;
}

__device__ inline uint32_t decode_pixel(const DecodeArgs &a, const uint8_t *cb, uint32_t blk, uint32_t off,
                                        bool &bad) {
    const uint32_t code = a.A[blk];
    if (code >= a.K) {
        bad = true;
        return 0;
    }
    const uint8_t *p = cb + code * a.D + off;
    return (uint32_t)p[0] | (uint32_t)p[1] << 8 | (uint32_t)p[2] << 16;
}

__device__ inline uint32_t sq_diff_bytes(uint32_t u, uint32_t v) {   // signed bytes, all four
    uint32_t s = 0;
#pragma unroll
    for (int k = 0; k < 4; k++) {
        const int d = (int)(int8_t)(u >> (8 * k)) - (int)(int8_t)(v >> (8 * k));
        s += (uint32_t)(d * d);
    }
    return s;
}

__device__ inline void decode_finish(const DecodeArgs &a, uint64_t sq, bool bad) {
    if (bad) atomicOr(a.bad, 1u);
    if (a.orig) {   // one atomic per wave
#pragma unroll
        for (int off = 32; off >= 1; off >>= 1) sq += __shfl_xor(sq, off);
        if ((threadIdx.x & 63) == 0 && sq) atomicAdd(a.sqerr, (unsigned long long)sq);
    }
}

// The codebook's n bytes into LDS: whole words when the source is 4-byte aligned, the tail
// (n % 4 bytes) and any unaligned source byte by byte -- never past cb + n (a
// caller's device codebook may be a slice of odd length).
__device__ inline void stage_codebook(uint8_t *scb, const uint8_t *cb, uint32_t n) {
    uint32_t head = 0;
    if (((uintptr_t)cb & 3) == 0) {
        head = n & ~3u;
        for (uint32_t i = threadIdx.x; i < head / 4; i += blockDim.x)
            reinterpret_cast<uint32_t *>(scb)[i] = reinterpret_cast<const uint32_t *>(cb)[i];
    }
    for (uint32_t i = head + threadIdx.x; i < n; i += blockDim.x) scb[i] = cb[i];
}

// Rows of ys % 8 == 0 pixels: thread (x, q) produces pixels y = 8q .. 8q + 7 of raster row x,
// 24 contiguous 8-byte-aligned bytes stored as three dwordx2 (and the original read the same
// way for the MSE).  The codebook sits in LDS when it is small (C3: 12 KB).
template <bool LDSCB>
__global__ __launch_bounds__(256) void decode_rows_kernel(DecodeArgs a) {
    extern __shared__ __attribute__((aligned(16))) uint8_t scb[];
    if (LDSCB) {
        stage_codebook(scb, a.cb, a.K * a.D);
        __syncthreads();
    }
    const uint8_t *cb = LDSCB ? scb : a.cb;
    const uint32_t qpr = a.ys / 8;
    const uint64_t total = (uint64_t)a.xs * qpr;
    uint64_t sq = 0;
    bool bad = false;
    for (uint64_t t = blockIdx.x * 256ull + threadIdx.x; t < total; t += (uint64_t)gridDim.x * 256) {
        const uint32_t x = (uint32_t)(t / qpr), y0 = (uint32_t)(t - (uint64_t)x * qpr) * 8;
        const uint32_t i0 = x / a.w, dx0 = x - i0 * a.w;
        uint32_t px[8];
#pragma unroll
        for (int k = 0; k < 8; k++) {
            uint32_t blk, off;
            decode_writer(a, x, y0 + k, i0, dx0, blk, off);
            px[k] = decode_pixel(a, cb, blk, off, bad);
        }
        // 8 pixels x 3 bytes -> 6 words
        uint32_t wv[6];
        wv[0] = px[0] | px[1] << 24;
        wv[1] = px[1] >> 8 | px[2] << 16;
        wv[2] = px[2] >> 16 | px[3] << 8;
        wv[3] = px[4] | px[5] << 24;
        wv[4] = px[5] >> 8 | px[6] << 16;
        wv[5] = px[6] >> 16 | px[7] << 8;
        const uint64_t byte0 = ((uint64_t)x * a.ys + y0) * 3;
        uint2 *dst = reinterpret_cast<uint2 *>(a.rgb + byte0);
        dst[0] = make_uint2(wv[0], wv[1]);
        dst[1] = make_uint2(wv[2], wv[3]);
        dst[2] = make_uint2(wv[4], wv[5]);
        if (a.orig) {
            const uint2 *o = reinterpret_cast<const uint2 *>(a.orig + byte0);
            const uint2 o0 = o[0], o1 = o[1], o2 = o[2];
            sq += sq_diff_bytes(wv[0], o0.x) + sq_diff_bytes(wv[1], o0.y) + sq_diff_bytes(wv[2], o1.x) +
                  sq_diff_bytes(wv[3], o1.y) + sq_diff_bytes(wv[4], o2.x) + sq_diff_bytes(wv[5], o2.y);
        }
    }
    decode_finish(a, sq, bad);
}

// No overhang (ys % h == 0) and h dividing 8: the 8 pixels (x, 8q .. 8q+7) of a thread are the
// column dx0 = x mod w of 8 / H consecutive blocks of one block column -- 3H contiguous bytes of
// each block's code vector at byte 3 H dx0 -- so no per-pixel divisions: one vector load of the
// 8 / H consecutive indices (16-byte aligned: hB = ys / H and 8q / H are multiples of 8 / H),
// 16-bit codebook reads from LDS (3H is even for H >= 2), three dwordx2 stores.
// COAL (ys % 512 == 0: a wave's 64 threads are 1536 contiguous output bytes of one raster row):
// the wave stages its three 8-byte pieces per lane in LDS and stores the chunk lane-contiguously,
// 512 bytes per store instruction (the direct stores have a 24-byte lane stride); the raport's
// original bytes are read the same coalesced way.
template <int H, bool LDSCB, bool COAL>
__global__ __launch_bounds__(256) void decode_rows_h_kernel(DecodeArgs a, uint32_t stage_off) {
    constexpr int NB = 8 / H;   // blocks per thread
    extern __shared__ __attribute__((aligned(16))) uint8_t scb[];
    const int lane = threadIdx.x & 63;
    uint2 *stage = reinterpret_cast<uint2 *>(scb + stage_off) + (threadIdx.x >> 6) * 192;   // 1536 B per wave
    if (LDSCB) {
        stage_codebook(scb, a.cb, a.K * a.D);
        __syncthreads();
    }
    const uint8_t *cb = LDSCB ? scb : a.cb;
    const uint32_t qpr = a.ys / 8;
    const uint64_t total = (uint64_t)a.xs * qpr;
    uint64_t sq = 0;
    bool bad = false;
    const bool small = total < (1ull << 32);   // 32-bit index math (C3: 2M items)
    for (uint64_t t = blockIdx.x * 256ull + threadIdx.x; t < total; t += (uint64_t)gridDim.x * 256) {
        uint32_t x, q;
        if (small) {
            x = (uint32_t)t / qpr;
            q = (uint32_t)t - x * qpr;
        } else {
            x = (uint32_t)(t / qpr);
            q = (uint32_t)(t - (uint64_t)x * qpr);
        }
        const uint32_t i0 = x / a.w, dx0 = x - i0 * a.w;
        const uint32_t *ap = a.A + (uint64_t)i0 * a.hB + (uint64_t)q * NB;
        uint32_t code[NB];
        if constexpr (NB == 8) {
            const uint4 c0 = reinterpret_cast<const uint4 *>(ap)[0], c1 = reinterpret_cast<const uint4 *>(ap)[1];
            code[0] = c0.x, code[1] = c0.y, code[2] = c0.z, code[3] = c0.w;
            code[4] = c1.x, code[5] = c1.y, code[6] = c1.z, code[7] = c1.w;
        } else if constexpr (NB == 4) {
            const uint4 c0 = reinterpret_cast<const uint4 *>(ap)[0];
            code[0] = c0.x, code[1] = c0.y, code[2] = c0.z, code[3] = c0.w;
        } else if constexpr (NB == 2) {
            const uint2 c0 = reinterpret_cast<const uint2 *>(ap)[0];
            code[0] = c0.x, code[1] = c0.y;
        } else {
            code[0] = ap[0];
        }
        // branch-free: an out-of-range index reads code vector 0 and is masked to zero
        uint32_t wv[6];
        if constexpr (H == 1) {
            uint32_t px[8];
#pragma unroll
            for (int b = 0; b < NB; b++) {
                const bool ok = code[b] < a.K;
                bad |= !ok;
                const uint8_t *src = cb + (ok ? code[b] : 0u) * a.D + 3 * dx0;
                const uint32_t v = (uint32_t)src[0] | (uint32_t)src[1] << 8 | (uint32_t)src[2] << 16;
                px[b] = ok ? v : 0u;
            }
            wv[0] = px[0] | px[1] << 24;
            wv[1] = px[1] >> 8 | px[2] << 16;
            wv[2] = px[2] >> 16 | px[3] << 8;
            wv[3] = px[4] | px[5] << 24;
            wv[4] = px[5] >> 8 | px[6] << 16;
            wv[5] = px[6] >> 16 | px[7] << 8;
        } else {
            constexpr int HB = 3 * H / 2;   // 16-bit halves per block
            uint32_t hv[12];
#pragma unroll
            for (int b = 0; b < NB; b++) {
                const bool ok = code[b] < a.K;
                bad |= !ok;
                const uint16_t *src = reinterpret_cast<const uint16_t *>(cb + (ok ? code[b] : 0u) * a.D + 3 * H * dx0);
                const uint32_t m = ok ? 0xFFFFu : 0u;
#pragma unroll
                for (int k = 0; k < HB; k++) hv[HB * b + k] = (uint32_t)src[k] & m;
            }
#pragma unroll
            for (int k = 0; k < 6; k++) wv[k] = hv[2 * k] | hv[2 * k + 1] << 16;
        }
        const uint64_t byte0 = ((uint64_t)x * a.ys + 8ull * q) * 3;
        if constexpr (COAL) {
            // lane l's 24 bytes are chunk bytes [24 l, 24 l + 24); stored piece k of lane l is
            // chunk bytes [512 k + 8 l, + 8) (ds_write_b64 at a 24-byte stride is conflict-free)
            stage[3 * lane] = make_uint2(wv[0], wv[1]);
            stage[3 * lane + 1] = make_uint2(wv[2], wv[3]);
            stage[3 * lane + 2] = make_uint2(wv[4], wv[5]);
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
            uint2 pc[3];
#pragma unroll
            for (int k = 0; k < 3; k++) pc[k] = stage[64 * k + lane];
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");   // reads before the next writes
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
            const uint64_t c0 = byte0 - 24ull * lane;   // the wave's chunk start (lane 0's byte0)
            uint2 *dst = reinterpret_cast<uint2 *>(a.rgb + c0);
#pragma unroll
            for (int k = 0; k < 3; k++) dst[64 * k + lane] = pc[k];
            if (a.orig) {
                const uint2 *o = reinterpret_cast<const uint2 *>(a.orig + c0);
#pragma unroll
                for (int k = 0; k < 3; k++) {
                    const uint2 ov = o[64 * k + lane];
                    sq += sq_diff_bytes(pc[k].x, ov.x) + sq_diff_bytes(pc[k].y, ov.y);
                }
            }
        } else {
            uint2 *dst = reinterpret_cast<uint2 *>(a.rgb + byte0);
            dst[0] = make_uint2(wv[0], wv[1]);
            dst[1] = make_uint2(wv[2], wv[3]);
            dst[2] = make_uint2(wv[4], wv[5]);
            if (a.orig) {
                const uint2 *o = reinterpret_cast<const uint2 *>(a.orig + byte0);
                const uint2 o0 = o[0], o1 = o[1], o2 = o[2];
                sq += sq_diff_bytes(wv[0], o0.x) + sq_diff_bytes(wv[1], o0.y) + sq_diff_bytes(wv[2], o1.x) +
                      sq_diff_bytes(wv[3], o1.y) + sq_diff_bytes(wv[4], o2.x) + sq_diff_bytes(wv[5], o2.y);
            }
        }
    }
    decode_finish(a, sq, bad);
}

// Any raster: one thread per pixel, byte stores (ys % 8 != 0).
__global__ __launch_bounds__(256) void decode_pixels_kernel(DecodeArgs a) {
    const uint64_t npix = (uint64_t)a.xs * a.ys;
    uint64_t sq = 0;
    bool bad = false;
    for (uint64_t P = blockIdx.x * 256ull + threadIdx.x; P < npix; P += (uint64_t)gridDim.x * 256) {
        const uint32_t x = (uint32_t)(P / a.ys), y = (uint32_t)(P - (uint64_t)x * a.ys);
        const uint32_t i0 = x / a.w, dx0 = x - i0 * a.w;
        uint32_t blk, off;
        decode_writer(a, x, y, i0, dx0, blk, off);
        const uint32_t v = decode_pixel(a, a.cb, blk, off, bad);
        uint8_t *o = a.rgb + P * 3;
        o[0] = (uint8_t)v, o[1] = (uint8_t)(v >> 8), o[2] = (uint8_t)(v >> 16);
        if (a.orig) {
            const uint8_t *q = a.orig + P * 3;
            sq += sq_diff_bytes(v, (uint32_t)q[0] | (uint32_t)q[1] << 8 | (uint32_t)q[2] << 16);
        }
    }
    decode_finish(a, sq, bad);
}

hipError_t launch_decode(hipStream_t s, const uint8_t *cb, uint32_t K, uint32_t D, const uint32_t *A, uint32_t xs,
                         uint32_t ys, uint32_t w, uint32_t h, uint8_t *rgb, const uint8_t *orig,
                         uint64_t *sqerr, uint32_t *bad) {
    DecodeArgs a;
    a.cb = cb, a.K = K, a.D = D, a.A = A, a.xs = xs, a.ys = ys, a.w = w, a.h = h;
    a.hB = (uint32_t)(((uint64_t)ys + h - 1) / h);   // the caller checks ys + h - 1 < 2^32
    a.yspan = a.hB * h;
    a.overhang = a.yspan - ys;
    a.rgb = rgb, a.orig = orig, a.sqerr = (unsigned long long *)sqerr, a.bad = bad;
    // the row kernels store (and read the original) in 8-byte pieces and load 8 / H indices per
    // vector load: caller pointers (qvq_decode_device) without that alignment take the
    // per-pixel kernel
    const bool aligned = (uintptr_t)rgb % 8 == 0 && (!orig || (uintptr_t)orig % 8 == 0) && (uintptr_t)A % 16 == 0;
    if (aligned && ys % 8 == 0 && (uint64_t)xs * ys < (1ull << 40)) {
        const uint64_t items = (uint64_t)xs * (ys / 8);
        const size_t cbB = (size_t)K * D;
        const bool lds = cbB <= 48 * 1024;
        // with the codebook staged in LDS, a block loops over several 256-item rounds (C3: 8192
        // one-round blocks staged 100 MB of codebook copies for 67 MB of output)
        constexpr uint64_t cap = 2048;
        const int grid = (int)std::max<uint64_t>(1, std::min<uint64_t>((items + 255) / 256, lds ? cap : 1u << 16));
        const size_t ldsB = lds ? (cbB + 15) & ~(size_t)15 : 0;
        if (a.overhang == 0 && (h == 1 || h == 2 || h == 4 || h == 8)) {
            // wave-contiguous output chunks need whole waves inside one raster row: 64 | ys / 8
            const bool coal = (ys / 8) % 64 == 0;
            const uint32_t soff = (uint32_t)ldsB;
            const size_t lb = ldsB + (coal ? 4 * 1536 : 0);
#define QVQ_DEC_H(HV)                                                                                                  \
    if (h == HV) {                                                                                                     \
        if (coal) {                                                                                                    \
            if (lds) hipLaunchKernelGGL((decode_rows_h_kernel<HV, true, true>), dim3(grid), dim3(256), lb, s, a, soff); \
            else hipLaunchKernelGGL((decode_rows_h_kernel<HV, false, true>), dim3(grid), dim3(256), lb, s, a, soff);    \
        } else {                                                                                                       \
            if (lds) hipLaunchKernelGGL((decode_rows_h_kernel<HV, true, false>), dim3(grid), dim3(256), lb, s, a, soff);\
            else hipLaunchKernelGGL((decode_rows_h_kernel<HV, false, false>), dim3(grid), dim3(256), lb, s, a, soff);   \
        }                                                                                                              \
    }
            QVQ_DEC_H(1) QVQ_DEC_H(2) QVQ_DEC_H(4) QVQ_DEC_H(8)
#undef QVQ_DEC_H
        } else if (lds) {
            hipLaunchKernelGGL(decode_rows_kernel<true>, dim3(grid), dim3(256), ldsB, s, a);
        } else {
            hipLaunchKernelGGL(decode_rows_kernel<false>, dim3(grid), dim3(256), 0, s, a);
        }
    } else {
        const uint64_t npix = (uint64_t)xs * ys;
        const int grid = (int)std::max<uint64_t>(1, std::min<uint64_t>((npix + 255) / 256, 1u << 16));
        hipLaunchKernelGGL(decode_pixels_kernel, dim3(grid), dim3(256), 0, s, a);
    }
    return hipGetLastError();
}

}  // namespace qvq
