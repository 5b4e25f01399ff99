// k_exact.hip -- the general training-set mode: qvq_set_vectors with values that are not byte
// images of a colour space (arbitrary fp64 data, CIE1931-like values).  The exact integer sums
// of the byte path do not apply, so this mode reproduces the reference's own arithmetic:
//   assign   every row against every code vector in fp64 in nanoflann's order (ref_l2_hd,
//            nanoflann.hpp:320-345), the lexicographic (distance, index) minimum; rows whose best
//            two are within tie_rel are exact ties and get the kd-tree's answer (host RefKDTree),
//   update   the rows of each code vector in ascending order (a stable radix sort of the
//            assignment, hipCUB) and one Kahan sum per (code vector, component) in that order,
//            times fl(1/n) -- sumInArea + operator/= (src/Quantizer.cpp:59-87) under
//            -freciprocal-math; an empty cell is the zero vector,
//   mean     the same Kahan over all rows in order (trainingSetSum, src/Quantizer.cpp:46-57).
// Kahan is sequential by definition: one thread per (code vector, component) chain, the row
// loads prefetched ahead of the dependent adds.  Built with -ffp-contract=off (no FMA
// contraction inside the compensation).
#include <cstdlib>
#include <cstring>

#include <hipcub/hipcub.hpp>

#include "common.hpp"

namespace qvq {

constexpr int EX_THREADS = 256;

// A[row] = the lexicographic (fp64 distance, index) minimum over the K code vectors of C ([K][D]);
// rows whose best two distances are within tie_rel go to ties.  The codebook is staged in LDS
// in chunks of kc code vectors (kc * D * 8 <= EX_LDS_BYTES; one chunk when it fits), ascending,
// so every row still scans k in ascending order; each lane keeps its row's best two across chunks.
constexpr uint32_t EX_LDS_BYTES = 64 * 1024;

// ref_l2_hd (kdtree_dev.hpp) with the dimension known at compile time: the same operations in
// the same order, the row held in registers (with a run-time dimension every code vector re-read
// the row's D values from memory: 96 B per lane per code vector at D = 12).
template <int DT>
__device__ inline double ref_l2_fixed(const double (&x)[DT], const double *__restrict__ c) {
    double r = 0;
    int d = 0;
#pragma unroll
    for (; d + 3 < DT; d += 4) {
        const double e0 = x[d] - c[d], e1 = x[d + 1] - c[d + 1];
        const double e2 = x[d + 2] - c[d + 2], e3 = x[d + 3] - c[d + 3];
        r += (e1 * e1 + e2 * e2) + (e0 * e0 + e3 * e3);
    }
#pragma unroll
    for (; d < DT; d++) {
        const double e = x[d] - c[d];
        r += e * e;
    }
    return r;
}

// One row against code vectors [k0, k0 + n) of cb (LDS), updating its best two (ascending k).
template <int DT>
__device__ inline void scan_codes(const double *__restrict__ xg, uint32_t D, const double *cb, uint32_t k0, uint32_t n,
                                  double &d1, double &d2, uint32_t &k1) {
    if constexpr (DT > 0) {
        double x[DT];
#pragma unroll
        for (int d = 0; d < DT; d++) x[d] = xg[d];
        for (uint32_t k = 0; k < n; k++) {
            const double d = ref_l2_fixed<DT>(x, cb + (size_t)k * DT);
            if (d < d1) {   // ascending k: the first minimum is the lowest index
                d2 = d1;
                d1 = d;
                k1 = k0 + k;
            } else if (d < d2) {
                d2 = d;
            }
        }
    } else {
        for (uint32_t k = 0; k < n; k++) {
            const double d = ref_l2_hd(xg, cb + (size_t)k * D, (int)D);
            if (d < d1) {
                d2 = d1;
                d1 = d;
                k1 = k0 + k;
            } else if (d < d2) {
                d2 = d;
            }
        }
    }
}

template <int DT>
__global__ __launch_bounds__(EX_THREADS) void exact_assign_kernel(const double *__restrict__ X, uint64_t N, uint32_t D,
                                                                  const double *__restrict__ C, uint32_t K, uint32_t kc,
                                                                  double tie_rel, uint32_t *__restrict__ A,
                                                                  uint32_t *__restrict__ ties,
                                                                  unsigned *__restrict__ tie_cnt) {
    extern __shared__ double cs[];
    const uint64_t stride = (uint64_t)gridDim.x * EX_THREADS;
    const uint64_t first = (uint64_t)blockIdx.x * EX_THREADS + threadIdx.x;
    if (kc >= K) {   // the whole codebook in LDS: grid-stride over rows
        for (uint32_t i = threadIdx.x; i < K * D; i += EX_THREADS) cs[i] = C[i];
        __syncthreads();
        for (uint64_t row = first; row < N; row += stride) {
            double d1 = INFINITY, d2 = INFINITY;
            uint32_t k1 = 0;
            scan_codes<DT>(X + row * D, D, cs, 0, K, d1, d2, k1);
            A[row] = k1;
            if (d2 - d1 <= tie_rel * d1) ties[atomicAdd(tie_cnt, 1u)] = (uint32_t)row;
        }
        return;
    }
    // chunked: one row per lane per pass (the grid covers N), the chunks staged in turn
    for (uint64_t base = (uint64_t)blockIdx.x * EX_THREADS; base < N; base += stride) {
        const uint64_t row = base + threadIdx.x;
        const bool live = row < N;
        double d1 = INFINITY, d2 = INFINITY;
        uint32_t k1 = 0;
        for (uint32_t k0 = 0; k0 < K; k0 += kc) {
            const uint32_t n = min(kc, K - k0);
            __syncthreads();   // the previous chunk is read by every lane
            for (uint32_t i = threadIdx.x; i < n * D; i += EX_THREADS) cs[i] = C[(size_t)k0 * D + i];
            __syncthreads();
            if (live) scan_codes<DT>(X + row * D, D, cs, k0, n, d1, d2, k1);
        }
        if (live) {
            A[row] = k1;
            if (d2 - d1 <= tie_rel * d1) ties[atomicAdd(tie_cnt, 1u)] = (uint32_t)row;
        }
    }
}

// koff[k] = first position of code vector k in the sorted keys (lower bound), koff[K] = N.
__global__ void exact_koff_kernel(const uint32_t *__restrict__ keys, uint64_t N, uint32_t K, uint32_t *__restrict__ koff) {
    const uint32_t k = blockIdx.x * blockDim.x + threadIdx.x;
    if (k > K) return;
    uint64_t lo = 0, hi = N;
    while (lo < hi) {
        const uint64_t mid = (lo + hi) / 2;
        if (keys[mid] < k) lo = mid + 1;
        else hi = mid;
    }
    koff[k] = (uint32_t)lo;
}

// C[k][d] = Kahan sum of X[row][d] over the rows of code vector k in ascending order (order
// positions koff[k] .. koff[k+1]; order = nullptr: rows 0 .. N-1, K = 1), times fl(1/n); an
// empty cell is 0 (sumInArea of nothing, no division).  One thread per (k, d) chain.
__global__ __launch_bounds__(EX_THREADS) void kahan_centroids_kernel(const double *__restrict__ X, uint64_t N,
                                                                     uint32_t D, const uint32_t *__restrict__ order,
                                                                     const uint32_t *__restrict__ koff, uint32_t K,
                                                                     double *__restrict__ C, uint64_t *__restrict__ cnt) {
    const uint64_t t = (uint64_t)blockIdx.x * EX_THREADS + threadIdx.x;
    if (t >= (uint64_t)K * D) return;
    const uint32_t k = (uint32_t)(t / D), d = (uint32_t)(t - (uint64_t)k * D);
    const uint64_t b = order ? koff[k] : 0, e = order ? koff[k + 1] : N;
    double sum = 0.0, c = 0.0;
    constexpr int U = 16;   // loads in flight ahead of the dependent Kahan chain
    uint64_t i = b;
    for (; i + U <= e; i += U) {
        double v[U];
#pragma unroll
        for (int u = 0; u < U; u++) v[u] = X[(uint64_t)(order ? order[i + u] : i + u) * D + d];
#pragma unroll
        for (int u = 0; u < U; u++) {
            const double y = v[u] - c;
            const double s = sum + y;
            c = (s - sum) - y;
            sum = s;
        }
    }
    for (; i < e; i++) {
        const double y = X[(uint64_t)(order ? order[i] : i) * D + d] - c;
        const double s = sum + y;
        c = (s - sum) - y;
        sum = s;
    }
    const uint64_t n = e - b;
    if (n) sum *= 1.0 / (double)n;   // operator/= by a scalar under -freciprocal-math
    C[t] = sum;
    if (cnt && d == 0) cnt[k] = n;
}

// The same chains, staged (D <= 64; the mean's chain is N steps, and a level's time is its
// largest cell's chain, which on skewed data stays long at every K): one workgroup per code
// vector; waves 1-3 stage the cell's rows, tile by tile (KC_TILE_BYTES, double-buffered), from
// HBM into LDS while wave 0's lanes run the D chains over the previous tile from LDS.  The per-thread kernel above waits on two dependent
// global loads (order, then the row) per 16 steps; here the chain only waits on LDS reads issued
// 16 ahead of the dependent adds.
constexpr int KC_THREADS = 256;
constexpr uint32_t KC_TILE_BYTES = 32 * 1024;   // two buffers: the 64 KB dynamic LDS default
constexpr uint32_t KC_MAX_K = 1u << 20;   // every level (the largest cell sets a level's time)

__global__ __launch_bounds__(KC_THREADS) void kahan_chains_lds_kernel(const double *__restrict__ X, uint64_t N,
                                                                      uint32_t D, const uint32_t *__restrict__ order,
                                                                      const uint32_t *__restrict__ koff, double *__restrict__ C,
                                                                      uint64_t *__restrict__ cnt) {
    extern __shared__ double tiles[];   // [2][T * D]
    const uint32_t k = blockIdx.x;
    const uint32_t T = KC_TILE_BYTES / 8 / D;
    const uint64_t b = order ? koff[k] : 0, e = order ? koff[k + 1] : N;
    const uint64_t n = e - b, ntiles = (n + T - 1) / T;
    const uint32_t wave = threadIdx.x / 64, lane = threadIdx.x % 64;
    // waves 1..3: tile t of the cell into buffer t & 1.  Every load of a lane's share is issued
    // before the first is used (order entries, then the values, then the LDS stores): a loop
    // that waits on each element's two dependent loads in turn took ~100 ns per row.
    constexpr uint32_t LOADERS = KC_THREADS - 64;
    constexpr uint32_t EPL = (KC_TILE_BYTES / 8 + LOADERS - 1) / LOADERS;   // elements per loader lane
    auto stage = [&](uint64_t t) {
        double *buf = tiles + (t & 1) * (size_t)T * D;
        const uint64_t r0 = b + t * T;
        const uint32_t cnt_el = (uint32_t)min<uint64_t>(T, e - r0) * D;
        const uint32_t i0 = threadIdx.x - 64;
        // past the tile's end a lane loads the tile's last element again (no branch around the
        // loads, so they all issue back to back) and does not store it
        uint64_t src[EPL];
        uint32_t dd[EPL];
#pragma unroll
        for (uint32_t j = 0; j < EPL; j++) {
            const uint32_t i = min(i0 + j * LOADERS, cnt_el - 1);
            const uint32_t r = i / D;
            dd[j] = i - r * D;
            src[j] = r0 + r;
        }
        if (order) {   // one uniform branch around all the order loads (they issue together)
            uint32_t o[EPL];
#pragma unroll
            for (uint32_t j = 0; j < EPL; j++) o[j] = order[src[j]];
#pragma unroll
            for (uint32_t j = 0; j < EPL; j++) src[j] = o[j];
        }
#pragma unroll
        for (uint32_t j = 0; j < EPL; j++) src[j] = src[j] * D + dd[j];
        double v[EPL];
#pragma unroll
        for (uint32_t j = 0; j < EPL; j++) v[j] = X[src[j]];
#pragma unroll
        for (uint32_t j = 0; j < EPL; j++)
            if (i0 + j * LOADERS < cnt_el) buf[i0 + j * LOADERS] = v[j];
    };
    double sum = 0.0, c = 0.0;
    if (wave != 0 && ntiles) stage(0);
    __syncthreads();
    for (uint64_t t = 0; t < ntiles; t++) {
        if (wave != 0) {
            if (t + 1 < ntiles) stage(t + 1);
        } else if (lane < D) {
            const double *cur = tiles + (t & 1) * (size_t)T * D + lane;
            const uint32_t rows = (uint32_t)min<uint64_t>(T, e - (b + t * T));
            uint32_t r = 0;
            constexpr int U = 16;
            for (; r + U <= rows; r += U) {
                double v[U];
#pragma unroll
                for (int u = 0; u < U; u++) v[u] = cur[(size_t)(r + u) * D];
#pragma unroll
                for (int u = 0; u < U; u++) {
                    const double y = v[u] - c;
                    const double s = sum + y;
                    c = (s - sum) - y;
                    sum = s;
                }
            }
            for (; r < rows; r++) {
                const double y = cur[(size_t)r * D] - c;
                const double s = sum + y;
                c = (s - sum) - y;
                sum = s;
            }
        }
        __syncthreads();
    }
    if (wave == 0 && lane < D) {
        if (n) sum *= 1.0 / (double)n;   // operator/= by a scalar under -freciprocal-math
        C[(size_t)k * D + lane] = sum;
        if (cnt && lane == 0) cnt[k] = n;
    }
}

// Per-block partials of sum_rows ||x - C[A[row]]||^2 (norm of the difference: squares added in
// component order, include/VectorOperations.hpp:107-111); exact_sum_kernel adds them in order.
__global__ __launch_bounds__(EX_THREADS) void exact_dist_kernel(const double *__restrict__ X, uint64_t N, uint32_t D,
                                                                const double *__restrict__ C,
                                                                const uint32_t *__restrict__ A,
                                                                double *__restrict__ part) {
    __shared__ double red[EX_THREADS];
    double acc = 0.0;
    for (uint64_t row = (uint64_t)blockIdx.x * EX_THREADS + threadIdx.x; row < N;
         row += (uint64_t)gridDim.x * EX_THREADS) {
        const double *x = X + row * D, *c = C + (uint64_t)A[row] * D;
        double r = 0.0;
        for (uint32_t d = 0; d < D; d++) {
            const double e = x[d] - c[d];
            r += e * e;
        }
        acc += r;
    }
    red[threadIdx.x] = acc;
    __syncthreads();
    for (int s = EX_THREADS / 2; s > 0; s >>= 1) {
        if ((int)threadIdx.x < s) red[threadIdx.x] += red[threadIdx.x + s];
        __syncthreads();
    }
    if (threadIdx.x == 0) part[blockIdx.x] = red[0];
}
__global__ void exact_sum_kernel(const double *__restrict__ part, uint32_t n, double scale, double *__restrict__ out) {
    double s = 0.0;
    for (uint32_t i = 0; i < n; i++) s += part[i];
    *out = s * scale;
}

// out[i][d] = X[rows[i]][d] (the tie rows for the host kd-tree); A[rows[i]] = vals[i].
__global__ void exact_gather_kernel(const double *__restrict__ X, uint32_t D, const uint32_t *__restrict__ rows,
                                    uint32_t n, double *__restrict__ out) {
    const uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (t < (uint64_t)n * D) out[t] = X[(uint64_t)rows[t / D] * D + t % D];
}
__global__ void exact_fix_kernel(uint32_t *__restrict__ A, const uint32_t *__restrict__ rows,
                                 const uint32_t *__restrict__ vals, uint32_t n) {
    const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
    if (t < n) A[rows[t]] = vals[t];
}

static int grid_for(uint64_t items, int cap = 4096) {
    return (int)std::max<uint64_t>(1, std::min<uint64_t>((items + EX_THREADS - 1) / EX_THREADS, (uint64_t)cap));
}

hipError_t launch_exact_assign(hipStream_t s, const double *X, uint64_t N, uint32_t D, const double *C, uint32_t K,
                               double tie_rel, uint32_t *A, uint32_t *ties, unsigned *tie_cnt) {
    const uint32_t kc = (uint32_t)std::max<size_t>(1, EX_LDS_BYTES / (8 * (size_t)D));   // code vectors per chunk
    const size_t lds = (size_t)std::min(kc, K) * D * 8;
    const dim3 grid(grid_for(N, 8192)), block(EX_THREADS);
    switch (D) {   // the dimensions of the reference's block shapes held in registers
    case 3: hipLaunchKernelGGL(exact_assign_kernel<3>, grid, block, lds, s, X, N, D, C, K, kc, tie_rel, A, ties, tie_cnt); break;
    case 6: hipLaunchKernelGGL(exact_assign_kernel<6>, grid, block, lds, s, X, N, D, C, K, kc, tie_rel, A, ties, tie_cnt); break;
    case 12: hipLaunchKernelGGL(exact_assign_kernel<12>, grid, block, lds, s, X, N, D, C, K, kc, tie_rel, A, ties, tie_cnt); break;
    case 48: hipLaunchKernelGGL(exact_assign_kernel<48>, grid, block, lds, s, X, N, D, C, K, kc, tie_rel, A, ties, tie_cnt); break;
    default: hipLaunchKernelGGL(exact_assign_kernel<0>, grid, block, lds, s, X, N, D, C, K, kc, tie_rel, A, ties, tie_cnt);
    }
    return hipGetLastError();
}

size_t exact_sort_temp_bytes(uint64_t N) {
    size_t bytes = 0;
    (void)hipcub::DeviceRadixSort::SortPairs(nullptr, bytes, (const uint32_t *)nullptr, (uint32_t *)nullptr,
                                             (const uint32_t *)nullptr, (uint32_t *)nullptr, (int)N);
    return bytes;
}

hipError_t launch_exact_centroids(hipStream_t s, const double *X, uint64_t N, uint32_t D, const uint32_t *A, uint32_t K,
                                  uint32_t *keys_out, uint32_t *iota, uint32_t *order, uint32_t *koff, void *temp,
                                  size_t temp_bytes, double *C, uint64_t *cnt) {
    // LDS-staged chains (a thread per chain only beyond their limits: D > 64 or K > KC_MAX_K)
    const bool lds_chains = D <= 64 && (!A || K <= KC_MAX_K);
    const size_t lds_bytes = lds_chains ? 2 * (size_t)(KC_TILE_BYTES / 8 / D) * D * 8 : 0;
    if (!A) {   // the mean: every row, in order
        if (lds_chains)
            hipLaunchKernelGGL(kahan_chains_lds_kernel, dim3(1), dim3(KC_THREADS), lds_bytes, s, X, N, D,
                               (const uint32_t *)nullptr, (const uint32_t *)nullptr, C, cnt);
        else
            hipLaunchKernelGGL(kahan_centroids_kernel, dim3(grid_for((uint64_t)D)), dim3(EX_THREADS), 0, s, X, N, D,
                               (const uint32_t *)nullptr, (const uint32_t *)nullptr, 1u, C, cnt);
        return hipGetLastError();
    }
    int bits = 1;
    while (bits < 32 && (1ull << bits) < K) bits++;
    // stable: equal keys keep the input (ascending row) order
    hipError_t e = hipcub::DeviceRadixSort::SortPairs(temp, temp_bytes, A, keys_out, iota, order, (int)N, 0, bits, s);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(exact_koff_kernel, dim3((K + 1 + 255) / 256), dim3(256), 0, s, keys_out, N, K, koff);
    if (lds_chains)
        hipLaunchKernelGGL(kahan_chains_lds_kernel, dim3(K), dim3(KC_THREADS), lds_bytes, s, X, N, D, order, koff, C,
                           cnt);
    else
        hipLaunchKernelGGL(kahan_centroids_kernel, dim3(grid_for((uint64_t)K * D, 1u << 30)), dim3(EX_THREADS), 0, s, X,
                           N, D, order, koff, K, C, cnt);
    return hipGetLastError();
}

__global__ void exact_iota_kernel(uint32_t *__restrict__ v, uint64_t N) {
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < N; i += (uint64_t)gridDim.x * blockDim.x)
        v[i] = (uint32_t)i;
}
hipError_t launch_exact_iota(hipStream_t s, uint32_t *v, uint64_t N) {
    hipLaunchKernelGGL(exact_iota_kernel, dim3(grid_for(N)), dim3(EX_THREADS), 0, s, v, N);
    return hipGetLastError();
}

hipError_t launch_exact_distortion(hipStream_t s, const double *X, uint64_t N, uint32_t D, const double *C,
                                   const uint32_t *A, double *part, double *out) {
    const int g = grid_for(N, 1024);
    hipLaunchKernelGGL(exact_dist_kernel, dim3(g), dim3(EX_THREADS), 0, s, X, N, D, C, A, part);
    hipLaunchKernelGGL(exact_sum_kernel, dim3(1), dim3(1), 0, s, part, (uint32_t)g, 1.0 / ((double)N * (double)D), out);
    return hipGetLastError();
}

hipError_t launch_exact_gather(hipStream_t s, const double *X, uint32_t D, const uint32_t *rows, uint32_t n,
                               double *out) {
    hipLaunchKernelGGL(exact_gather_kernel, dim3((unsigned)(((uint64_t)n * D + 255) / 256)), dim3(256), 0, s, X, D,
                       rows, n, out);
    return hipGetLastError();
}
hipError_t launch_exact_fix(hipStream_t s, uint32_t *A, const uint32_t *rows, const uint32_t *vals, uint32_t n) {
    hipLaunchKernelGGL(exact_fix_kernel, dim3((n + 255) / 256), dim3(256), 0, s, A, rows, vals, n);
    return hipGetLastError();
}

}  // namespace qvq
