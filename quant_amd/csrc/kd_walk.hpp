// kd_walk.hpp -- device code shared by the kd-tree tie kernels (k_assign.hip: kd_resolve_kernel
// and kd_reduce_kernel) and the rechecks: the reference-order fp64 distance
// (nanoflann.hpp:320-345 as the reference build computes it) and the wave-parallel walk of the
// reference kd-tree (nanoflann.hpp:1212-1270).
#pragma once
#include <algorithm>

#include "common.hpp"
#include "mfma_util.hpp"

namespace qvq {

// ref_l2_hd for D = N (12) against a code vector in global memory: the row's N/2 16-byte
// loads are issued together (the generic loop waits for each group of four), then the
// reference's order: per group of four (e1^2 + e2^2) + (e0^2 + e3^2), groups added in turn.
template <int N>
struct RowN {
    double2 v[N / 2];
};
template <int N>
__device__ inline RowN<N> load_row(const double *c) {
    RowN<N> r;
    const double2 *p = reinterpret_cast<const double2 *>(c);
#pragma unroll
    for (int i = 0; i < N / 2; i++) r.v[i] = p[i];
    return r;
}
template <int N>
__device__ inline double ref_l2_n(const double *a, const RowN<N> &c) {
    double r = 0;
#pragma unroll
    for (int g = 0; g < N / 4; g++) {
        const double e0 = a[4 * g] - c.v[2 * g].x, e1 = a[4 * g + 1] - c.v[2 * g].y;
        const double e2 = a[4 * g + 2] - c.v[2 * g + 1].x, e3 = a[4 * g + 3] - c.v[2 * g + 1].y;
        r += (e1 * e1 + e2 * e2) + (e0 * e0 + e3 * e3);
    }
    return r;
}
// fp64 reference distance of row a (LDS) to code vector k of C64 (global), any D
__device__ inline double ref_l2_cv(const double *a, const double *C64, uint32_t k, uint32_t D) {
    if (D == 12) return ref_l2_n<12>(a, load_row<12>(C64 + (uint64_t)k * 12));
    return ref_l2_hd(a, C64 + (uint64_t)k * D, (int)D);   // (a D = 48 row in registers costs the recheck occupancy)
}

// The same for D = 48 with the row's loads in flight two 8-component chunks ahead (the generic
// loop waits for every group of four: 12 dependent round trips per point); the kd kernels'
// point distances only (not inlined: its rows get their own register allocation).
static __device__ __attribute__((noinline)) double ref_l2_48(const double *a, const double *c) {
    const double2 *p = reinterpret_cast<const double2 *>(c);
    double2 b[2][4];
#pragma unroll
    for (int i = 0; i < 4; i++) b[0][i] = p[i];
#pragma unroll
    for (int i = 0; i < 4; i++) b[1][i] = p[4 + i];
    double r = 0;
#pragma unroll
    for (int ch = 0; ch < 6; ch++) {   // chunk ch: components 8 ch .. 8 ch + 7, two groups of four
        const double2 *v = b[ch & 1];
#pragma unroll
        for (int g = 0; g < 2; g++) {
            const int d = 8 * ch + 4 * g;
            const double e0 = a[d] - v[2 * g].x, e1 = a[d + 1] - v[2 * g].y;
            const double e2 = a[d + 2] - v[2 * g + 1].x, e3 = a[d + 3] - v[2 * g + 1].y;
            r += (e1 * e1 + e2 * e2) + (e0 * e0 + e3 * e3);
        }
        if (ch + 2 < 6) {
#pragma unroll
            for (int i = 0; i < 4; i++) b[ch & 1][i] = p[4 * (ch + 2) + i];
        }
    }
    return r;
}
// pv[j] for j = j0, j0 + step, ... < K: the fp64 reference distance of row a to point vind[j]
__device__ inline void kd_point_dists(const double *a, const double *C64, const uint32_t *vind, uint32_t K, uint32_t D,
                                      uint32_t j0, uint32_t step, double *pv) {
#pragma unroll 1
    for (uint32_t j = j0; j < K; j += step)
        pv[j] = D == 48 ? ref_l2_48(a, C64 + (uint64_t)vind[j] * 48) : ref_l2_cv(a, C64, vind[j], D);
}

// LDS written by some lanes of a wave and then read by others: order the accesses.
__device__ inline void wave_lds_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// kd_nearest_flat with the leaf scan spread over the wave: every lane runs the same
// descent (uniform values), lane i takes leaf point i, and the leaf's winner is the first
// point in leaf order with the smallest distance below the leaf-entry worst -- what the
// sequential strict-'<' scan picks.  Leaves hold at most 10 points (< 64 lanes).  pv holds
// every point's distance in vind order; subtrees none of whose points is below best are
// skipped (same result), and the walk stops once best is gmin, the smallest of all K
// distances (when known; -inf: never).
__device__ inline uint32_t kd_nearest_wave(const double *q, uint32_t D, const KdView &t, const double *pv, double *sd,
                                    int32_t *sn, double *dl, int lane, double gmin = -INFINITY) {
    double distsq = 0;   // dl: per-dimension cell distances (LDS, uniform across lanes)
    for (uint32_t d = 0; d < D; d++) {
        const double x = q[d];
        dl[d] = 0;
        if (x < t.lo[d]) {
            dl[d] = (x - t.lo[d]) * (x - t.lo[d]);
            distsq += dl[d];
        }
        if (x > t.hi[d]) {
            dl[d] = (x - t.hi[d]) * (x - t.hi[d]);
            distsq += dl[d];
        }
    }
    double best = 1.7976931348623157e308;
    uint32_t best_idx = 0;
    int sp = 0;
    sd[0] = distsq;
    sn[0] = 0;
    while (sp >= 0) {
        const int32_t node = sn[sp] >> 2, phase = sn[sp] & 3;
        const KdNodeDev n = t.nodes[node];
        // A subtree none of whose points is below best cannot change best (updates need
        // dist < worst <= best) and its walk has no other effect: skip it.  Its points are
        // vind[first, b), so the test is a range minimum of pv.
        if (phase == 0 && n.child1 >= 0 && best < 1.7976931348623157e308) {
            double m = INFINITY;
            for (int32_t j = kd_first(n) + lane; j < n.b; j += 64) m = fmin(m, pv[j]);
            m = wave_min_f64<4>(m);
            if (m >= best) {
                sp--;
                continue;
            }
        }
        if (n.child1 < 0) {
            const double worst = best;
            const int32_t cnt = n.b - n.a;
            double dist = INFINITY;
            if (lane < cnt) {
                const double dd = pv[n.a + lane];   // ref_l2_hd(q, point vind[n.a + lane])
                if (dd < worst) dist = dd;
            }
            // leaves hold <= 10 points: lanes 0..15 suffice; the winner is the lowest lane
            // with the minimum
            const double m = wave_min_f64<1>(dist);
            if (m < worst) {
                const uint64_t hit = __ballot(dist == m);
                best = m;
                best_idx = t.vind[n.a + __ffsll((unsigned long long)hit) - 1];
                if (m == gmin) break;   // the smallest of all K distances: nothing can follow
            }
            sp--;
            continue;
        }
        const int f = kd_feat(n);
        const double val = q[f];
        const double diff1 = val - n.lo, diff2 = val - n.hi;
        const bool left_first = (diff1 + diff2) < 0;
        if (phase == 0) {
            sn[sp] = node << 2 | 1;
            sd[sp + 1] = sd[sp];
            sn[sp + 1] = (left_first ? n.child1 : n.child2) << 2;
            sp++;
            continue;
        }
        if (phase == 1) {
            const double cut_dist = left_first ? (val - n.hi) * (val - n.hi) : (val - n.lo) * (val - n.lo);
            const double dst = dl[f];
            const double m2 = (sd[sp] - dst) + cut_dist;
            dl[f] = cut_dist;
            sd[sp] = dst;
            sn[sp] = node << 2 | 2;
            if (m2 <= best) {
                sd[sp + 1] = m2;
                sn[sp + 1] = (left_first ? n.child2 : n.child1) << 2;
                sp++;
                continue;
            }
        }
        dl[f] = sd[sp];
        sp--;
    }
    return best_idx;
}

// Wave-uniform doubles held one per lane (lane l = element l), read and written by lane index.
__device__ inline double lane_get_f64(double v, int l) {
    const uint64_t b = (uint64_t)__double_as_longlong(v);
    const uint32_t lo = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)b, l);
    const uint32_t hi = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(b >> 32), l);
    return __longlong_as_double((long long)((uint64_t)hi << 32 | lo));
}
__device__ inline double lane_set_f64(double v, double x, int l) { return (int)__lane_id() == l ? x : v; }

// Direct answer for a tie row, without the walk.  The walk (nanoflann's search) ends on the
// first point it reaches among T, the points at the smallest of all K distances gmin: later
// points need dist < best.  Before it reaches one, best is >= gnext, the smallest distance
// above gmin, so a point p of T is reached whenever every cell bound m2 on p's root-to-leaf
// path where p lies in the far child is <= gnext (near children are always entered; a far
// child's test reads dists[] as at its node's entry: the near subtree restores what it
// changes).  Ignoring pruning the walk meets the points of T in path order: at the node where
// two paths part, the near child's first, and in vind order within a leaf.  So: the first of T
// in path order, if its own path passes the test, is the walk's answer.  Otherwise (or more
// than 64 points in T, or D > 64) returns false and the walk decides.  Lane d holds query
// component d and the root cell distance of dimension d; candl: 64 ints of LDS.  gmin is
// returned either way (the walk stops at it).
__device__ inline bool kd_tie_direct(const double *q, uint32_t D, const KdView &t, const double *pv, uint32_t K,
                                     int32_t *candl, int lane, uint32_t &out, double &gmin_out) {
    double a1 = INFINITY, a2 = INFINITY;   // this lane's smallest distance and its smallest above a1
    for (uint32_t j0 = 0; j0 < K; j0 += 256) {
        double p[4];
#pragma unroll
        for (int u = 0; u < 4; u++) {
            const uint32_t j = j0 + 64 * u + lane;
            p[u] = j < K ? pv[j] : INFINITY;
        }
#pragma unroll
        for (int u = 0; u < 4; u++) {
            if (p[u] < a1) {
                a2 = a1;
                a1 = p[u];
            } else if (p[u] > a1 && p[u] < a2) {
                a2 = p[u];
            }
        }
    }
    const double gmin = wave_min_f64<4>(a1);
    const double gnext = wave_min_f64<4>(a1 > gmin ? a1 : a2);
    gmin_out = gmin;
    if (D > 64) return false;
    int nt = 0;
    for (uint32_t j0 = 0; j0 < K && nt <= 64; j0 += 64) {
        const uint32_t j = j0 + lane;
        const bool take = j < K && pv[j] == gmin;
        const uint64_t bal = __ballot(take);
        const int pre = (int)__builtin_amdgcn_mbcnt_hi((uint32_t)(bal >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)bal, 0u));
        if (take && nt + pre < 64) candl[nt + pre] = (int32_t)j;
        nt += __popcll(bal);
    }
    wave_lds_sync();
    if (nt < 1 || nt > 64) return false;
    const int32_t mine = lane < nt ? candl[lane] : -1;
    wave_lds_sync();
    const double ql = lane < (int)D ? q[lane] : 0.0;
    double dll = 0.0;
    if (lane < (int)D) {
        const double lo = t.lo[lane], hi = t.hi[lane];
        if (ql < lo) dll = (ql - lo) * (ql - lo);
        if (ql > hi) dll = (ql - hi) * (ql - hi);
    }
    double sdv = 0;   // the root's cell bound, in dimension order (zero terms add exactly)
    for (uint32_t d = 0; d < D; d++) sdv += lane_get_f64(dll, (int)d);
    const int max_steps = t.depth + 1;
    // the first of T in path order: each point against the current first, both positions
    // descending together to the node where they part
    int32_t w = __builtin_amdgcn_readlane(mine, 0);
    for (int c = 1; c < nt; c++) {
        const int32_t j = __builtin_amdgcn_readlane(mine, c);
        bool j_first = j < w;   // one leaf: vind order
        KdNodeDev n = t.nodes[0];
        for (int it = 0; it < max_steps && n.child1 >= 0; it++) {
            const KdNodeDev c1 = t.nodes[n.child1], c2 = t.nodes[n.child2];
            const bool wl = w < c1.b, jl = j < c1.b;   // child1 holds vind[first, c1.b)
            if (wl != jl) {
                const double val = lane_get_f64(ql, kd_feat(n));
                j_first = jl == (((val - n.lo) + (val - n.hi)) < 0);   // j in the near child
                break;
            }
            n = wl ? c1 : c2;
        }
        if (j_first) w = j;
    }
    // w's path: the cell-bound test at every far step
    bool ok = true;
    KdNodeDev n = t.nodes[0];
    for (int it = 0; it < max_steps && n.child1 >= 0; it++) {
        const KdNodeDev c1 = t.nodes[n.child1], c2 = t.nodes[n.child2];
        const bool go_left = w < c1.b;
        const int f = kd_feat(n);
        const double val = lane_get_f64(ql, f);
        const bool left_first = ((val - n.lo) + (val - n.hi)) < 0;
        if (go_left != left_first) {
            const double cut_dist = left_first ? (val - n.hi) * (val - n.hi) : (val - n.lo) * (val - n.lo);
            const double m2 = (sdv - lane_get_f64(dll, f)) + cut_dist;
            ok = ok && m2 <= gnext;
            dll = lane_set_f64(dll, cut_dist, f);
            sdv = m2;
        }
        n = go_left ? c1 : c2;
    }
    if (!ok || n.child1 >= 0) return false;
    out = t.vind[w];
    return true;
}

// The direct answer when it applies, else the walk, which stops at gmin (QVQ_KDWALK_LDS
// builds: the walk always, A/B).
__device__ inline uint32_t kd_walk(const double *q, uint32_t D, const KdView &t, const double *pv, uint32_t K, double *sd,
                                   int32_t *sn, double *dl, int lane) {
    double gmin = -INFINITY;
#ifndef QVQ_KDWALK_LDS
    uint32_t k;
    if (kd_tie_direct(q, D, t, pv, K, reinterpret_cast<int32_t *>(dl), lane, k, gmin)) return k;
#endif
    return kd_nearest_wave(q, D, t, pv, sd, sn, dl, lane, gmin);
}

// Exact ties listed by the recheck, answered by the reference kd-tree traversal
// (kd_nearest_flat).  The tree image (kd.lo .. ) lives in mapped pinned host memory (or a
// device copy) and is staged into LDS by each block that has tie rows; one wave walks it per
// tie, lanes spread over the leaf scans and the K point distances.
constexpr int KDR_MAX_WAVES = 16;
constexpr int KDR_BLOCKS = 64;   // blocks without ties exit before staging the tree (C3 level 6: 39 -> 27 us)

// LDS: per wave the row, cell distances, stack and the K point distances; plus the tree.
inline size_t kd_wave_bytes(const KdView &kd, uint32_t K) {
    return 128 * 8 + (((size_t)kd.depth * KD_FRAME_BYTES + 7) & ~(size_t)7) + (size_t)K * 8;
}
inline size_t kd_tree_bytes(const KdView &kd) { return ((size_t)kd.bytes + 7) & ~(size_t)7; }
// waves whose state fits next to the tree in `budget` bytes of LDS (0: the tree does not fit)
inline int kd_waves_within(const KdView &kd, uint32_t K, size_t budget) {
    const size_t wb = kd_wave_bytes(kd, K), tb = kd_tree_bytes(kd);
    if (kd.depth <= 0 || tb + wb > budget) return 0;
    return (int)std::min<size_t>(KDR_MAX_WAVES, (budget - tb) / wb);
}

struct KdArgs {
    const uint8_t *codes;
    uint32_t Dp, D;
    const uint32_t *ties;
    const double *C64;   // the split codebook being searched
    uint32_t K;
    const double *lut64;
    KdView kd;
    uint32_t *A;
    uint64_t *xslab;     // fused sums: the correction slabs (move_row_terms), else nullptr
    uint32_t *xcnt;
    const uint64_t *plut;
    uint64_t *xsums;     // or: copy 1 of the final sums (move_row_sums; kd_reduce_kernel), else nullptr
};

// Block b of nb answers ties f = b + nb wave, + nb W, ... (waves >= W only help staging): ties
// go round the blocks first, so a level's few hundred spread over all nb blocks' CUs.
// whole_block (W = 1): ties f = b, b + nb, ..., the block's waves compute the tie's K point
// distances together and wave 0 walks (big K * D: one wave spent most of a tie on them).
// Uniform per block (it contains __syncthreads); ksm: kd_tree_bytes + W kd_wave_bytes of LDS.
__device__ inline void kd_resolve_block(const KdArgs &a, unsigned nt, uint32_t b, uint32_t nb, int W, double *ksm,
                                        bool whole_block = false) {
    if (b >= nt) return;
    const KdView &kd = a.kd;
    const uint32_t D = a.D, K = a.K;
    const int Z = kd.depth;
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    double *tr = ksm;   // tree image
    double *wb = ksm + ((size_t)kd.bytes + 7) / 8 +
                 (size_t)(whole_block ? 0 : wave) * (128 + ((size_t)Z * KD_FRAME_BYTES + 7) / 8 + K);
    double *xs = wb, *dl = wb + 64;
    double *sd = wb + 128;
    int32_t *sn = reinterpret_cast<int32_t *>(sd + Z);
    double *pv = wb + 128 + ((size_t)Z * KD_FRAME_BYTES + 7) / 8;   // [K] distances in vind order
    {   // stage the tree image: 16-byte loads, eight in flight per lane (one round trip over
        // PCIe when the image is read in place from mapped host memory)
        const uint4 *src = reinterpret_cast<const uint4 *>(kd.lo);
        uint4 *dst = reinterpret_cast<uint4 *>(tr);
        const uint32_t n16 = kd.bytes / 16;
        constexpr int U = 8;
        for (uint32_t i0 = threadIdx.x; i0 < n16; i0 += U * blockDim.x) {
            uint4 v[U];   // clamped (always valid) loads: a predicated array went to scratch,
                          // and a kernel with scratch costs more to launch
#pragma unroll
            for (int u = 0; u < U; u++) v[u] = src[min(i0 + u * blockDim.x, n16 - 1)];
#pragma unroll
            for (int u = 0; u < U; u++)
                if (i0 + u * blockDim.x < n16) dst[i0 + u * blockDim.x] = v[u];
        }
        const uint32_t tail = (kd.bytes & 15) / 4;   // the image is a whole number of dwords
        if (threadIdx.x < tail)
            reinterpret_cast<uint32_t *>(tr)[n16 * 4 + threadIdx.x] =
                reinterpret_cast<const uint32_t *>(kd.lo)[n16 * 4 + threadIdx.x];
    }
    KdView kv = kd;
    kv.lo = tr;
    kv.hi = tr + D;
    kv.nodes = reinterpret_cast<const KdNodeDev *>(tr + 2 * D);
    kv.vind = reinterpret_cast<const uint32_t *>(kv.nodes + kd.n_nodes);
    __syncthreads();
    if (whole_block) {
        for (unsigned f = b; f < nt; f += nb) {
            const uint32_t row = a.ties[f];
            if (threadIdx.x < D) xs[threadIdx.x] = a.lut64[a.codes[(uint64_t)row * a.Dp + threadIdx.x]];
            __syncthreads();
            kd_point_dists(xs, a.C64, kv.vind, K, D, threadIdx.x, blockDim.x, pv);
            __syncthreads();
            if (wave == 0) {
                const uint32_t k = kd_walk(xs, D, kv, pv, K, sd, sn, dl, lane);
                const uint32_t from = __builtin_amdgcn_readfirstlane(a.A[row]);
                if (k != from) {
                    if (a.xslab) move_row_terms(a.codes, a.Dp, D, row, from, k, K, a.xslab, a.xcnt, a.plut, lane);
                    else if (a.xsums) move_row_sums(a.codes, a.Dp, D, row, from, k, K, a.xsums, a.plut, lane);
                    if (lane == 0) a.A[row] = k;
                }
            }
            __syncthreads();
        }
        return;
    }
    if (wave >= W) return;
    for (unsigned f = b + nb * wave; f < nt; f += nb * W) {
        const uint32_t row = a.ties[f];
        if (lane < (int)D) xs[lane] = a.lut64[a.codes[(uint64_t)row * a.Dp + lane]];
        wave_lds_sync();
        if (D == 12) {   // four points per lane in flight (their 24 loads together)
            for (uint32_t j0 = lane; j0 < K; j0 += 4 * 64) {
                RowN<12> c[4];
#pragma unroll
                for (int u = 0; u < 4; u++) {
                    const uint32_t j = j0 + 64 * u;
                    c[u] = load_row<12>(a.C64 + (uint64_t)kv.vind[j < K ? j : j0] * 12);
                }
#pragma unroll
                for (int u = 0; u < 4; u++)
                    if (j0 + 64 * u < K) pv[j0 + 64 * u] = ref_l2_n<12>(xs, c[u]);
            }
        } else {
            kd_point_dists(xs, a.C64, kv.vind, K, D, lane, 64, pv);
        }
        wave_lds_sync();
        const uint32_t k = kd_walk(xs, D, kv, pv, K, sd, sn, dl, lane);
        const uint32_t from = __builtin_amdgcn_readfirstlane(a.A[row]);   // the search's index
        if (k != from) {
            if (a.xslab) move_row_terms(a.codes, a.Dp, D, row, from, k, K, a.xslab, a.xcnt, a.plut, lane);
            else if (a.xsums) move_row_sums(a.codes, a.Dp, D, row, from, k, K, a.xsums, a.plut, lane);
            if (lane == 0) a.A[row] = k;
        }
        wave_lds_sync();
    }
}

}  // namespace qvq
