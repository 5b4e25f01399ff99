// k_kahan.hip -- the reference's Kahan centroids (sumInArea, src/Quantizer.cpp:59-87) on the
// device, exactly, for the byte engine's SCALED values: the rows sorted stably by their index,
// one chain per (code vector, component), each chain cut into segments whose tables compose
// (kahan_par.hpp).  Used on the levels whose tie band is not empty.
#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>

#include "common.hpp"
#include "kahan_par.hpp"

namespace qvq {

using kahan::Chain;
using kahan::Fn;
using kahan::i128;
using kahan::u128;

namespace {

constexpr int KT = 256;   // threads per block

__device__ inline uint32_t find_cell(const uint32_t *off, uint32_t K, uint32_t s) {   // off[k] <= s < off[k+1]
    uint32_t lo = 0, hi = K;
    while (hi - lo > 1) {
        const uint32_t mid = (lo + hi) / 2;
        if (off[mid] <= s) lo = mid;
        else hi = mid;
    }
    return lo;
}

// koff[k] = first sorted position with key >= k (keys sorted ascending)
__global__ void kc_koff_kernel(const uint32_t *__restrict__ keys, uint64_t N, uint32_t K, uint32_t *__restrict__ koff) {
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

// Per cell: segments (L), groups (L*S), supergroups (L*S*S); exclusive scans into off[3][K+1].
// One block, each thread a contiguous run of cells.
__global__ __launch_bounds__(1024) void kc_offsets_kernel(const uint32_t *__restrict__ koff, uint32_t K, uint32_t L,
                                                          uint32_t S, uint32_t *__restrict__ off) {
    __shared__ uint32_t part[3][1024];
    const uint32_t per = (K + 1023) / 1024, b = min(K, threadIdx.x * per), e = min(K, b + per);
    const uint64_t span[3] = {L, (uint64_t)L * S, (uint64_t)L * S * S};
    uint32_t s[3] = {0, 0, 0};
    for (uint32_t k = b; k < e; k++) {
        const uint64_t n = koff[k + 1] - koff[k];
        for (int l = 0; l < 3; l++) s[l] += (uint32_t)((n + span[l] - 1) / span[l]);
    }
    for (int l = 0; l < 3; l++) part[l][threadIdx.x] = s[l];
    __syncthreads();
    for (int o = 1; o < 1024; o <<= 1) {
        uint32_t v[3];
        for (int l = 0; l < 3; l++) v[l] = threadIdx.x >= (uint32_t)o ? part[l][threadIdx.x - o] : 0u;
        __syncthreads();
        for (int l = 0; l < 3; l++) part[l][threadIdx.x] += v[l];
        __syncthreads();
    }
    uint32_t base[3];
    for (int l = 0; l < 3; l++) base[l] = part[l][threadIdx.x] - s[l];
    for (uint32_t k = b; k < e; k++) {
        const uint64_t n = koff[k + 1] - koff[k];
        for (int l = 0; l < 3; l++) {
            off[(uint64_t)l * (K + 1) + k] = base[l];
            base[l] += (uint32_t)((n + span[l] - 1) / span[l]);
        }
    }
    if (threadIdx.x == 1023)
        for (int l = 0; l < 3; l++) off[(uint64_t)l * (K + 1) + K] = part[l][1023];
}

// planes[d][p] = codes[order[p]][d] (order null: row p)
__global__ void kc_gather_kernel(const uint8_t *__restrict__ codes, uint32_t Dp, uint32_t D, uint64_t N,
                                 const uint32_t *__restrict__ order, uint8_t *__restrict__ planes) {
    for (uint64_t p = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; p < N; p += (uint64_t)gridDim.x * blockDim.x) {
        const uint64_t row = order ? order[p] : p;
        const uint8_t *src = codes + row * Dp;
        for (uint32_t d = 0; d < D; d++) planes[(uint64_t)d * N + p] = src[d];
    }
}

struct Geo {   // where the chains live
    const uint8_t *planes;
    uint64_t N;
    const uint32_t *koff, *off;   // off: [3][K+1] segment / group / supergroup offsets
    uint32_t K, D, L, S;
    Fn *fn0, *fn1, *fn2;
    uint32_t NS, NG, NU;          // capacities per component
    __device__ Chain chain(uint32_t k, uint32_t d, const uint64_t *Xt) const {
        Chain c;
        c.b = planes + (uint64_t)d * N + koff[k];
        c.Xt = Xt;
        c.n = koff[k + 1] - koff[k];
        c.f0 = fn0 + (uint64_t)d * NS + off[k];
        c.f1 = fn1 + (uint64_t)d * NG + off[(K + 1) + k];
        c.f2 = fn2 + (uint64_t)d * NU + off[2 * (K + 1) + k];
        c.L = L;
        c.S = S;
        return c;
    }
};

__device__ inline void stage_xt(const uint64_t *__restrict__ g, uint64_t *s) {
    for (int i = threadIdx.x; i < 256; i += blockDim.x) s[i] = g[i];
    __syncthreads();
}

// Exact sum of X over each segment: P0[d][seg] (then scanned per chain into the prefixes).
__global__ __launch_bounds__(KT) void kc_segsum_kernel(Geo g, const uint64_t *__restrict__ gXt, i128 *__restrict__ P0) {
    __shared__ uint64_t Xt[256];
    stage_xt(gXt, Xt);
    const uint32_t tot = g.off[g.K];
    for (uint64_t t = (uint64_t)blockIdx.x * KT + threadIdx.x; t < (uint64_t)tot * g.D; t += (uint64_t)gridDim.x * KT) {
        const uint32_t d = (uint32_t)(t / tot), seg = (uint32_t)(t - (uint64_t)d * tot);
        const uint32_t k = find_cell(g.off, g.K, seg);
        const uint64_t a = g.koff[k] + (uint64_t)(seg - g.off[k]) * g.L;
        const uint64_t e = min((uint64_t)g.koff[k + 1], a + g.L);
        const uint8_t *b = g.planes + (uint64_t)d * g.N;
        u128 s = 0;
        for (uint64_t p = a; p < e; p++) s += Xt[b[p]];
        P0[(uint64_t)d * g.NS + seg] = (i128)s;
    }
}

// Exclusive scan of the segment sums along every chain: a wave per (cell, component).
__global__ __launch_bounds__(KT) void kc_prefix_kernel(Geo g, i128 *__restrict__ P0) {
    const uint32_t lane = threadIdx.x & 63;
    const uint64_t w = ((uint64_t)blockIdx.x * KT + threadIdx.x) >> 6;
    if (w >= (uint64_t)g.K * g.D) return;
    const uint32_t k = (uint32_t)(w / g.D), d = (uint32_t)(w - (uint64_t)k * g.D);
    const uint32_t s0 = g.off[k], s1 = g.off[k + 1];
    i128 *p = P0 + (uint64_t)d * g.NS;
    u128 carry = 0;
    for (uint32_t base = s0; base < s1; base += 64) {
        const uint32_t s = base + lane;
        u128 v = s < s1 ? (u128)p[s] : 0, inc = v;
        for (int o = 1; o < 64; o <<= 1) {
            const uint64_t lo = __shfl_up((unsigned long long)(uint64_t)inc, o, 64);
            const uint64_t hi = __shfl_up((unsigned long long)(uint64_t)(inc >> 64), o, 64);
            if (lane >= (uint32_t)o) inc += ((u128)hi << 64) | lo;
        }
        if (s < s1) p[s] = (i128)(carry + inc - v);
        const uint64_t tlo = __shfl((unsigned long long)(uint64_t)inc, 63, 64);
        const uint64_t thi = __shfl((unsigned long long)(uint64_t)(inc >> 64), 63, 64);
        carry += ((u128)thi << 64) | tlo;
    }
}

// Segment tables: P0 holds each segment's exact prefix; Etr (pass 2, may be null) the trusted
// walk's state at each segment start, the better estimate.
__global__ __launch_bounds__(KT) void kc_build_kernel(Geo g, const uint64_t *__restrict__ gXt,
                                                      const i128 *__restrict__ P0, const i128 *__restrict__ Etr) {
    __shared__ uint64_t Xt[256];
    stage_xt(gXt, Xt);
    const uint32_t tot = g.off[g.K];
    for (uint64_t t = (uint64_t)blockIdx.x * KT + threadIdx.x; t < (uint64_t)tot * g.D; t += (uint64_t)gridDim.x * KT) {
        const uint32_t d = (uint32_t)(t / tot), seg = (uint32_t)(t - (uint64_t)d * tot);
        const uint32_t k = find_cell(g.off, g.K, seg);
        const uint64_t a = g.koff[k] + (uint64_t)(seg - g.off[k]) * g.L;
        const uint32_t len = (uint32_t)min((uint64_t)g.L, (uint64_t)g.koff[k + 1] - a);
        const uint64_t idx = (uint64_t)d * g.NS + seg;
        const i128 P = P0[idx];
        const int64_t dest = Etr ? (int64_t)(Etr[idx] - P) : 0;
        g.fn0[idx] = kahan::build_segment(g.planes + (uint64_t)d * g.N + a, Xt, len, P, dest);
    }
}

// Groups (level 1) or supergroups (level 2): a thread per (function, component).
template <int LEVEL>
__global__ __launch_bounds__(KT) void kc_compose_kernel(Geo g, const uint64_t *__restrict__ gXt) {
    __shared__ uint64_t Xt[256];
    stage_xt(gXt, Xt);
    const uint32_t *off = g.off + (uint64_t)LEVEL * (g.K + 1);
    const uint32_t tot = off[g.K];
    for (uint64_t t = (uint64_t)blockIdx.x * KT + threadIdx.x; t < (uint64_t)tot * g.D; t += (uint64_t)gridDim.x * KT) {
        const uint32_t d = (uint32_t)(t / tot), f = (uint32_t)(t - (uint64_t)d * tot);
        const uint32_t k = find_cell(off, g.K, f);
        const Chain c = g.chain(k, d, Xt);
        if (LEVEL == 1) g.fn1[(uint64_t)d * g.NG + f] = kahan::compose1(c, f - off[k]);
        else g.fn2[(uint64_t)d * g.NU + f] = kahan::compose2(c, f - off[k]);
    }
}

// Trusted walk over a chain's pass-1 tables: the estimated state at every segment start.
__global__ __launch_bounds__(KT) void kc_trust_kernel(Geo g, const uint64_t *__restrict__ gXt, const i128 *__restrict__ P0,
                                                      i128 *__restrict__ Etr) {
    __shared__ uint64_t Xt[256];
    stage_xt(gXt, Xt);
    for (uint64_t t = (uint64_t)blockIdx.x * KT + threadIdx.x; t < (uint64_t)g.K * g.D; t += (uint64_t)gridDim.x * KT) {
        const uint32_t k = (uint32_t)(t / g.D), d = (uint32_t)(t - (uint64_t)k * g.D);
        const Chain c = g.chain(k, d, Xt);
        const uint64_t base = (uint64_t)d * g.NS + g.off[k];
        const uint64_t nseg = (c.n + c.L - 1) / c.L;
        // estimate_dest writes E - P; keep E itself (pass 2 adds back nothing)
        int64_t *dest = reinterpret_cast<int64_t *>(Etr + base);   // scratch: one int64 per segment first
        kahan::estimate_dest(c, P0 + base, dest);
        for (uint64_t s = nseg; s-- > 0;) Etr[base + s] = P0[base + s] + (i128)dest[s];
    }
}

// Every chain evaluated exactly: C[k][d] = Kahan sum * fl(1/n) (empty cell: 0).
__global__ __launch_bounds__(KT) void kc_eval_kernel(Geo g, const uint64_t *__restrict__ gXt, double *__restrict__ C,
                                                     unsigned *__restrict__ stats) {
    __shared__ uint64_t Xt[256];
    stage_xt(gXt, Xt);
    for (uint64_t t = (uint64_t)blockIdx.x * KT + threadIdx.x; t < (uint64_t)g.K * g.D; t += (uint64_t)gridDim.x * KT) {
        const uint32_t k = (uint32_t)(t / g.D), d = (uint32_t)(t - (uint64_t)k * g.D);
        const Chain c = g.chain(k, d, Xt);
        uint32_t miss[3] = {0, 0, 0};
        double s = c.n ? kahan::eval_chain(c, miss) : 0.0;
        if (c.n) s = __dmul_rn(s, 1.0 / (double)c.n);   // operator/= by a scalar under -freciprocal-math
        C[t] = s;
        if (stats && (miss[0] | miss[1] | miss[2])) {
            atomicAdd(&stats[0], miss[0]);
            atomicAdd(&stats[1], miss[1]);
            atomicAdd(&stats[2], miss[2]);
        }
    }
}

// The split (src/Quantizer.cpp:134-138): S[k] = C[k] * (1 + 0.2), S[K + k] = C[k] * (1 - 0.2).
__global__ void kc_split_kernel(const double *__restrict__ C, uint32_t K, uint32_t D, double *__restrict__ Sp) {
    const uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= (uint64_t)K * D) return;
    Sp[t] = __dmul_rn(C[t], (double)(1 + 0.2));
    Sp[(uint64_t)K * D + t] = __dmul_rn(C[t], (double)(1 - 0.2));
}

int grid_of(uint64_t items) { return (int)std::max<uint64_t>(1, std::min<uint64_t>((items + KT - 1) / KT, 16384)); }

}  // namespace

size_t KahanWork::fn_bytes() { return sizeof(Fn); }

// Capacity per component: every cell's last segment may be partial.
void KahanWork::caps(uint64_t N, uint32_t K, uint32_t L, uint32_t S, uint32_t &NS, uint32_t &NG, uint32_t &NU) {
    NS = (uint32_t)((N + L - 1) / L + K);
    NG = (uint32_t)((N + (uint64_t)L * S - 1) / ((uint64_t)L * S) + K);
    NU = (uint32_t)((N + (uint64_t)L * S * S - 1) / ((uint64_t)L * S * S) + K);
}

size_t kahan_sort_temp_bytes(uint64_t N) {
    size_t bytes = 0;
    (void)hipcub::DeviceRadixSort::SortPairs(nullptr, bytes, (const uint32_t *)nullptr, (uint32_t *)nullptr,
                                             (const uint32_t *)nullptr, (uint32_t *)nullptr, (int)N);
    return bytes;
}

hipError_t launch_kahan_centroids(hipStream_t s, const KahanWork &w, const uint8_t *codes, uint32_t Dp, uint32_t D,
                                  uint64_t N, const uint32_t *A, uint32_t K, const uint64_t *Xt, double *C,
                                  double *split_out, int passes) {
    if (N == 0 || N > 0xFFFFFFFFull || D == 0 || K == 0) return hipErrorInvalidValue;
    const uint32_t *order = nullptr;
    if (A) {
        int bits = 1;
        while (bits < 32 && (1ull << bits) < K) bits++;
        size_t tb = w.temp_bytes;
        hipError_t e = hipcub::DeviceRadixSort::SortPairs(w.temp, tb, A, w.keys, (const uint32_t *)w.iota, w.order,
                                                          (int)N, 0, bits, s);
        if (e != hipSuccess) return e;
        hipLaunchKernelGGL(kc_koff_kernel, dim3((K + 1 + 255) / 256), dim3(256), 0, s, w.keys, N, K, w.koff);
        order = w.order;
    } else {
        if (K != 1) return hipErrorInvalidValue;
        const uint32_t ko[2] = {0, (uint32_t)N};
        hipError_t e = hipMemcpyAsync(w.koff, ko, sizeof(ko), hipMemcpyHostToDevice, s);
        if (e != hipSuccess) return e;
    }
    hipLaunchKernelGGL(kc_offsets_kernel, dim3(1), dim3(1024), 0, s, w.koff, K, w.L, w.S, w.off);
    hipLaunchKernelGGL(kc_gather_kernel, dim3(grid_of(N)), dim3(KT), 0, s, codes, Dp, D, N, order, w.planes);
    uint32_t NS, NG, NU;
    KahanWork::caps(N, K, w.L, w.S, NS, NG, NU);
    Geo g{w.planes, N, w.koff, w.off, K, D, w.L, w.S, reinterpret_cast<Fn *>(w.fn0), reinterpret_cast<Fn *>(w.fn1),
          reinterpret_cast<Fn *>(w.fn2), NS, NG, NU};
    i128 *P0 = reinterpret_cast<i128 *>(w.P0), *Etr = reinterpret_cast<i128 *>(w.Etr);
    hipLaunchKernelGGL(kc_segsum_kernel, dim3(grid_of((uint64_t)NS * D)), dim3(KT), 0, s, g, Xt, P0);
    hipLaunchKernelGGL(kc_prefix_kernel, dim3((unsigned)(((uint64_t)K * D * 64 + KT - 1) / KT)), dim3(KT), 0, s, g, P0);
    hipLaunchKernelGGL(kc_build_kernel, dim3(grid_of((uint64_t)NS * D)), dim3(KT), 0, s, g, Xt, P0, (const i128 *)nullptr);
    if (passes > 1) {
        hipLaunchKernelGGL(kc_trust_kernel, dim3(grid_of((uint64_t)K * D)), dim3(KT), 0, s, g, Xt, P0, Etr);
        hipLaunchKernelGGL(kc_build_kernel, dim3(grid_of((uint64_t)NS * D)), dim3(KT), 0, s, g, Xt, P0,
                           (const i128 *)Etr);
    }
    hipLaunchKernelGGL(kc_compose_kernel<1>, dim3(grid_of((uint64_t)NG * D)), dim3(KT), 0, s, g, Xt);
    hipLaunchKernelGGL(kc_compose_kernel<2>, dim3(grid_of((uint64_t)NU * D)), dim3(KT), 0, s, g, Xt);
    hipLaunchKernelGGL(kc_eval_kernel, dim3(grid_of((uint64_t)K * D)), dim3(KT), 0, s, g, Xt, C, w.stats);
    if (split_out)
        hipLaunchKernelGGL(kc_split_kernel, dim3((unsigned)(((uint64_t)K * D + 255) / 256)), dim3(256), 0, s, C, K, D,
                           split_out);
    return hipGetLastError();
}

}  // namespace qvq
