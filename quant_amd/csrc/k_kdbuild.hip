// k_kdbuild.hip -- the reference kd-tree of a level's split codebook, built on the device.
//
// The tree is nanoflann 1.2.3's (buildIndex / divideTree / middleSplit_ / planeSplit,
// nanoflann.hpp:863-871, :1046-1094, :1108-1147, :1159-1186, leaf_max_size 10 from
// KDTreeVectorOfVectorsAdaptor.hpp:59) exactly as RefKDTree builds it on the host (kdtree.cpp):
// the same cut dimensions, cut values, point order (vind), divlow / divhigh and point boxes.
//
// Parallel form of the two sequential pieces:
//  * planeSplit's two Hoare passes.  Pass 1 over [0, n) leaves lim1 = #(v < cutval) and swaps
//    the k-th element with v >= cutval in [0, lim1) (from the left) with the k-th element with
//    v < cutval in [lim1, n) (from the right); pass 2 does the same over [lim1, n) with <=.  So
//    each element's rank among its kind (a prefix count) gives its partner: two block (or wave)
//    scans per pass instead of a serial walk.  (tools/kd_shapes.py checks the pairing against the
//    serial passes on real codebooks and tie-heavy random sets.)
//  * the point boxes.  A node's box is its points' exact per-dimension min / max; the parent
//    computes its children's: the smaller child's by a scan, the larger child's by keeping the
//    node's extreme wherever the smaller child does not reach it (a point holding it is in the
//    larger child) and scanning only the other dimensions.  Degenerate trees (the duplicate zero
//    code vectors of empty cells: C4's level-12 tree is 174 levels deep, its chain nodes ~1900
//    points each) then cost a scan of the few peeled points per level.
//
// One workgroup builds the tree: nodes of more than KB_SMALL points one at a time with every
// thread (phase 1, depth first, the larger child kept in LDS), then the subtrees of at most
// KB_SMALL points one per wave (phase 2).  Node ids are creation order (root 0); the host renumbers
// them depth first (RefKDTree's own order) when it imports the image.  The kd_resolve image
// (kdtree_dev.hpp KdView: root box | KdNodeDev[n] | vind) goes to device memory, the full image
// (nodes, boxes, vind) to mapped host memory for the host's tie certificate.
#include <cstdint>

#include "common.hpp"
#include "kdtree_dev.hpp"
#include "mfma_util.hpp"

namespace qvq {

constexpr int KB_THREADS = 1024;
constexpr int KB_WAVES = KB_THREADS / 64;
constexpr uint32_t KB_SMALL = 128;   // points per wave-built subtree (two per lane)
constexpr uint32_t KB_STACK = 256;   // pending big nodes
constexpr uint32_t KB_LIST = 1024;   // subtrees left to the waves
constexpr uint32_t KB_WSTACK = 96;   // a wave's pending nodes (a subtree of KB_SMALL points)

// Ordered 64-bit keys of doubles (integer min / max in LDS): monotone, -0.0 below +0.0 (the
// engine's codebooks hold no -0.0).
__device__ inline unsigned long long kb_key(double x) {
    const uint64_t b = (uint64_t)__double_as_longlong(x);
    return (b >> 63) ? ~b : (b | 0x8000000000000000ull);
}
__device__ inline double kb_unkey(unsigned long long k) {
    const uint64_t b = (k >> 63) ? (k & 0x7FFFFFFFFFFFFFFFull) : ~k;
    return __longlong_as_double((long long)b);
}

// fp64 maximum over the wave by DPP steps (no LDS round trips: the cut choice is on every
// node's serial path); lanes without a source read -inf.  Uniform result.
template <int CTRL, int ROW_MASK>
__device__ inline double kb_dpp_max_step(double v) {
    const uint64_t b = (uint64_t)__double_as_longlong(v);
    constexpr uint64_t ninf = 0xFFF0000000000000ull;
    const uint32_t lo = (uint32_t)__builtin_amdgcn_update_dpp((int)(uint32_t)ninf, (int)(uint32_t)b, CTRL, ROW_MASK,
                                                              0xF, false);
    const uint32_t hi = (uint32_t)__builtin_amdgcn_update_dpp((int)(uint32_t)(ninf >> 32), (int)(uint32_t)(b >> 32),
                                                              CTRL, ROW_MASK, 0xF, false);
    return fmax(v, __longlong_as_double((long long)(((uint64_t)hi << 32) | lo)));
}
__device__ inline double kb_wave_max(double v) {
    v = kb_dpp_max_step<0x111, 0xF>(v);   // row_shr:1
    v = kb_dpp_max_step<0x112, 0xF>(v);   // row_shr:2
    v = kb_dpp_max_step<0x114, 0xF>(v);   // row_shr:4
    v = kb_dpp_max_step<0x118, 0xF>(v);   // row_shr:8
    v = kb_dpp_max_step<0x142, 0xA>(v);   // row_bcast:15 into rows 1, 3
    v = kb_dpp_max_step<0x143, 0xC>(v);   // row_bcast:31 into rows 2, 3
    const uint64_t b = (uint64_t)__double_as_longlong(v);
    const uint32_t lo = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)b, 63);
    const uint32_t hi = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(b >> 32), 63);
    return __longlong_as_double((long long)(((uint64_t)hi << 32) | lo));
}
__device__ inline double kb_readlane(double v, int l) {
    const uint64_t b = (uint64_t)__double_as_longlong(v);
    const uint32_t lo = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)b, l);
    const uint32_t hi = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(b >> 32), l);
    return __longlong_as_double((long long)(((uint64_t)hi << 32) | lo));
}

// middleSplit_'s choice for one node (kdtree.cpp middle_split): lane d < D holds the node's cell
// box and point box in dimension d.  Every lane returns the same values.
struct KbCut {
    int cf;
    double cutval, split_val, spread_gap;
    uint64_t cand;
};
__device__ inline KbCut kb_choose_cut(uint32_t lane, uint32_t D, double plo, double phi, double clo, double chi) {
    const double NEG = -__builtin_huge_val();
    const bool in = lane < D;
    const double span = in ? chi - clo : NEG;
    const double max_span = kb_wave_max(span);
    const double EPS = 0.00001;
    const bool cand = in && span > (1 - EPS) * max_span;
    const uint64_t cmask = __ballot(cand);
    const double spread = phi - plo;
    // the first candidate with the greatest spread (spread > max_spread, ascending dimensions)
    const double best = kb_wave_max(cand ? spread : NEG);
    const uint64_t at = __ballot(cand && spread == best);
    KbCut c;
    const bool have = cmask != 0;
    c.cf = have ? (int)__builtin_ctzll(at) : 0;
    const double second = kb_wave_max(cand && (int)lane != c.cf ? spread : NEG);
    c.spread_gap = have ? best - second : -1.0;
    const double mn = kb_readlane(plo, c.cf), mx = kb_readlane(phi, c.cf);
    const double blo = kb_readlane(clo, c.cf), bhi = kb_readlane(chi, c.cf);
    c.split_val = (blo + bhi) / 2;
    c.cutval = c.split_val < mn ? mn : (c.split_val > mx ? mx : c.split_val);
    c.cand = cmask;
    return c;
}

// Min / max keys over the points pts[0..n) (row indices of P) in nd dimensions (dl[j] & 0xFF, or
// j itself without dl; with dl, bit 8 / 9 of dl[j] select the minimum / maximum), the (point,
// dimension) pairs q = first, first + step, ... spread over the calling threads; LDS key arrays
// lo / hi indexed by dimension.  Eight pairs per trip: their loads are all issued before the
// first atomic (one round trip to L2 per eight pairs, not per pair).
__device__ inline void kb_pairs_minmax(const double *__restrict__ P, uint32_t D, const uint32_t *pts, uint32_t n,
                                       uint32_t first, uint32_t step, uint32_t nd, const uint32_t *dl,
                                       unsigned long long *lo, unsigned long long *hi) {
    const uint32_t total = n * nd;
    constexpr int U = 8;
    for (uint32_t q0 = first; q0 < total; q0 += U * step) {
        double v[U];
        uint32_t e[U];
#pragma unroll
        for (int u = 0; u < U; u++) {
            const uint32_t q = q0 + u * step;
            const uint32_t qq = q < total ? q : total - 1;
            const uint32_t p = qq / nd, j = qq - p * nd;
            e[u] = dl ? dl[j] : (j | 0x300u);
            v[u] = P[(size_t)pts[p] * D + (e[u] & 0xFF)];
        }
#pragma unroll
        for (int u = 0; u < U; u++) {
            if (q0 + u * step >= total) break;
            const unsigned long long k = kb_key(v[u]);
            const uint32_t d = e[u] & 0xFF;
            if (e[u] & 0x100) atomicMin(&lo[d], k);
            if (e[u] & 0x200) atomicMax(&hi[d], k);
        }
    }
}

struct KbArgs {
    const double *P;   // K x D split codebook (row-major)
    uint32_t K, D;
    uint32_t *vind;     // [K] device
    KdbNode *nodes;     // [2K] device
    double *nbox;       // [2K][2][D] device: point boxes (lo row, hi row)
    double *cbox;       // [2K][2][D] device: cell boxes
    uint8_t *flat;      // kd_resolve image: lo[D] | hi[D] | KdNodeDev[n] | vind[K]
    uint8_t *himg;      // mapped host image (kdb_host_layout)
    uint64_t seq;
};

__device__ inline void kb_write_leaf(const KbArgs &a, uint32_t id, uint32_t left, uint32_t right, uint32_t depth) {
    KdbNode n{};
    n.child1 = n.child2 = -1;
    n.left = left;
    n.right = right;
    n.depth = depth;
    a.nodes[id] = n;
}

__global__ __launch_bounds__(KB_THREADS) void kd_build_kernel(KbArgs a) {
    const uint32_t K = a.K, D = a.D;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const uint64_t t_start = wall_clock64();
    __shared__ uint32_t s_ind[KDB_MAXK];
    __shared__ double s_val[KDB_MAXK];
    __shared__ uint16_t s_mpos[KDB_MAXK / 2 + 1], s_ppos[KDB_MAXK / 2 + 1];
    __shared__ double s_pb[2][64], s_cb[2][64];
    __shared__ unsigned long long s_ks[2][64], s_kg[2][64];   // children's box keys: smaller, larger
    __shared__ uint32_t s_wsum[KB_WAVES];
    __shared__ uint32_t s_stack[KB_STACK], s_list[KB_LIST];
    __shared__ uint32_t s_nstack, s_nlist, s_nnodes, s_depth, s_fail, s_lnext;
    __shared__ uint32_t s_me, s_l, s_n, s_dep, s_keep;
    __shared__ KbCut s_cut;
    __shared__ uint32_t s_dl[64], s_ndl;
    __shared__ uint32_t w_ind[KB_WAVES][KB_SMALL];
    __shared__ double w_val[KB_WAVES][KB_SMALL];
    __shared__ uint8_t w_mpos[KB_WAVES][KB_SMALL / 2 + 1], w_ppos[KB_WAVES][KB_SMALL / 2 + 1];
    __shared__ uint32_t w_stack[KB_WAVES][KB_WSTACK];
    __shared__ unsigned long long w_key[KB_WAVES][256];
    __shared__ uint32_t w_dl[KB_WAVES][64];

    // ---- root: identity order, its point box (= its cell box) --------------------------------
    for (uint32_t i = tid; i < K; i += KB_THREADS) a.vind[i] = i;
    if (tid < 64) {
        s_ks[0][tid] = ~0ull;
        s_ks[1][tid] = 0ull;
    }
    if (tid == 0) {
        s_nstack = s_nlist = s_fail = s_lnext = 0;
        s_nnodes = 1;
        s_depth = 1;
    }
    __syncthreads();
    for (uint32_t q = tid; q < K * D; q += KB_THREADS) {
        const unsigned long long k = kb_key(a.P[q]);
        atomicMin(&s_ks[0][q % D], k);
        atomicMax(&s_ks[1][q % D], k);
    }
    __syncthreads();
    if (tid < (int)D) {
        const double lo = kb_unkey(s_ks[0][tid]), hi = kb_unkey(s_ks[1][tid]);
        a.nbox[tid] = lo;
        a.nbox[D + tid] = hi;
        a.cbox[tid] = lo;
        a.cbox[D + tid] = hi;
    }
    if (tid == 0) {
        if (K <= 10) {
            kb_write_leaf(a, 0, 0, K, 1);
        } else if (K > KB_SMALL) {
            s_stack[0] = 0;
            s_nstack = 1;
        } else {
            s_list[0] = 0;
            s_nlist = 1;
        }
        KdbNode r{};
        r.left = 0;
        r.right = K;
        r.depth = 1;
        if (K > 10) a.nodes[0] = r;
    }
    __syncthreads();

    // ---- phase 1: nodes of more than KB_SMALL points, every thread ---------------------------
    // s_keep: the node to split next is already in LDS (the larger child of the last one)
    if (tid == 0) s_keep = 0;
    __syncthreads();
    for (;;) {
        if (tid == 0) {
            if (!s_keep) {
                if (s_nstack == 0 || s_fail) {
                    s_me = ~0u;
                } else {
                    s_me = s_stack[--s_nstack];
                    const KdbNode nd = a.nodes[s_me];
                    s_l = nd.left;
                    s_n = nd.right - nd.left;
                    s_dep = nd.depth;
                }
            }
        }
        __syncthreads();
        const uint32_t me = s_me;
        if (me == ~0u) break;
        const uint32_t l = s_l, n = s_n, dep = s_dep;
        if (!s_keep) {   // the node's boxes and points from global memory
            if (tid < (int)D) {
                s_pb[0][tid] = a.nbox[(size_t)me * 2 * D + tid];
                s_pb[1][tid] = a.nbox[(size_t)me * 2 * D + D + tid];
                s_cb[0][tid] = a.cbox[(size_t)me * 2 * D + tid];
                s_cb[1][tid] = a.cbox[(size_t)me * 2 * D + D + tid];
            }
            for (uint32_t i = tid; i < n; i += KB_THREADS) s_ind[i] = a.vind[l + i];
        }
        __syncthreads();
        if (wave == 0) {
            const KbCut c = kb_choose_cut(lane, D, lane < (int)D ? s_pb[0][lane] : 0.0, lane < (int)D ? s_pb[1][lane] : 0.0,
                                          lane < (int)D ? s_cb[0][lane] : 0.0, lane < (int)D ? s_cb[1][lane] : 0.0);
            if (lane == 0) s_cut = c;
        }
        __syncthreads();
        const KbCut c = s_cut;
        // this thread's chunk of positions [b0, b1)
        const uint32_t E = (n + KB_THREADS - 1) / KB_THREADS;
        const uint32_t b0 = min((uint32_t)tid * E, n), b1 = min(b0 + E, n);
        uint32_t r_ind[KDB_MAXK / KB_THREADS];
        double r_val[KDB_MAXK / KB_THREADS];
#pragma unroll
        for (uint32_t j = 0; j < KDB_MAXK / KB_THREADS; j++)   // every load issued before the first use
            if (j < b1 - b0) {
                r_ind[j] = s_ind[b0 + j];
                r_val[j] = a.P[(size_t)r_ind[j] * D + c.cf];
            }
        for (uint32_t j = 0; j < b1 - b0; j++) s_val[b0 + j] = r_val[j];
        // two passes: pass 0 over [0, n) with <, pass 1 over [lim1, n) with <=
        uint32_t lim1 = 0, lim2 = 0;
        for (int pass = 0; pass < 2; pass++) {
            const uint32_t from = pass ? lim1 : 0;
            uint32_t cnt = 0;
            for (uint32_t j = 0; j < b1 - b0; j++) {
                const uint32_t i = b0 + j;
                const bool f = pass ? r_val[j] <= c.cutval : r_val[j] < c.cutval;
                cnt += (i >= from && f) ? 1u : 0u;
            }
            const uint32_t inc = wave_scan_add(cnt);
            if (lane == 63) s_wsum[wave] = inc;
            __syncthreads();
            uint32_t wpre = 0, tot = 0;
            for (int w = 0; w < KB_WAVES; w++) {
                const uint32_t ws = s_wsum[w];
                wpre += w < wave ? ws : 0u;
                tot += ws;
            }
            const uint32_t lim = from + tot;   // lim1 or lim2
            uint32_t pf = wpre + inc - cnt;     // kind before this chunk (within [from, n))
            uint32_t src[KDB_MAXK / KB_THREADS];
            for (uint32_t j = 0; j < b1 - b0; j++) {
                const uint32_t i = b0 + j;
                src[j] = i;
                if (i < from) continue;
                const bool f = pass ? r_val[j] <= c.cutval : r_val[j] < c.cutval;
                if (i < lim && !f) s_mpos[(i - from) - pf] = (uint16_t)i;        // k-th misfit from the left
                if (i >= lim && f) s_ppos[(lim - from) - pf - 1] = (uint16_t)i;  // k-th partner from the right
                pf += f ? 1u : 0u;
            }
            __syncthreads();
            pf = wpre + inc - cnt;
            for (uint32_t j = 0; j < b1 - b0; j++) {
                const uint32_t i = b0 + j;
                if (i < from) continue;
                const bool f = pass ? r_val[j] <= c.cutval : r_val[j] < c.cutval;
                if (i < lim && !f) src[j] = s_ppos[(i - from) - pf];
                if (i >= lim && f) src[j] = s_mpos[(lim - from) - pf - 1];
                pf += f ? 1u : 0u;
            }
            for (uint32_t j = 0; j < b1 - b0; j++) {
                r_ind[j] = s_ind[src[j]];
                r_val[j] = s_val[src[j]];
            }
            __syncthreads();
            for (uint32_t j = 0; j < b1 - b0; j++) {
                s_ind[b0 + j] = r_ind[j];
                s_val[b0 + j] = r_val[j];
            }
            if (pass) lim2 = lim;
            else lim1 = lim;
            __syncthreads();
        }
        const uint32_t index = lim1 > n / 2 ? lim1 : (lim2 < n / 2 ? lim2 : n / 2);
        for (uint32_t j = 0; j < b1 - b0; j++) a.vind[l + b0 + j] = r_ind[j];
        // the children's point boxes: the smaller one scanned, the larger one from the node's
        const bool first_small = index <= n - index;
        const uint32_t sb = first_small ? 0 : index, sn = first_small ? index : n - index;
        const uint32_t gb = first_small ? index : 0, gn = n - sn;
        if (tid < 64) {
            s_ks[0][tid] = ~0ull;
            s_ks[1][tid] = 0ull;
        }
        __syncthreads();
        kb_pairs_minmax(a.P, D, s_ind + sb, sn, tid, KB_THREADS, D, nullptr, s_ks[0], s_ks[1]);
        __syncthreads();
        if (wave == 0) {   // the dimensions where the smaller child reaches the node's extreme
            bool nlo = false, nhi = false;
            if (lane < (int)D) {
                nlo = !(kb_unkey(s_ks[0][lane]) > s_pb[0][lane]);
                nhi = !(kb_unkey(s_ks[1][lane]) < s_pb[1][lane]);
                s_kg[0][lane] = nlo ? ~0ull : kb_key(s_pb[0][lane]);
                s_kg[1][lane] = nhi ? 0ull : kb_key(s_pb[1][lane]);
            }
            const uint64_t m = __ballot(nlo || nhi);
            const uint32_t pos = (uint32_t)__popcll(m & ((1ull << lane) - 1));
            if (nlo || nhi) s_dl[pos] = (uint32_t)lane | (nlo ? 0x100u : 0u) | (nhi ? 0x200u : 0u);
            if (lane == 0) s_ndl = (uint32_t)__popcll(m);
        }
        __syncthreads();
        const uint32_t ndl = s_ndl;
        if (ndl) kb_pairs_minmax(a.P, D, s_ind + gb, gn, tid, KB_THREADS, ndl, s_dl, s_kg[0], s_kg[1]);
        __syncthreads();
        // ids, records, the children's boxes
        uint32_t c1 = 0;
        if (tid == 0) {
            c1 = s_nnodes;
            s_nnodes = c1 + 2;
            if (c1 + 2 > 2 * K) s_fail = 1;
            s_me = c1;   // (broadcast)
            s_depth = max(s_depth, dep + 1);
        }
        __syncthreads();
        c1 = s_me;
        const bool fail = s_fail != 0;
        __syncthreads();
        if (fail) break;
        const uint32_t n1 = index, n2 = n - index;
        if (tid < (int)D) {
            const double slo = kb_unkey(s_ks[0][tid]), shi = kb_unkey(s_ks[1][tid]);
            const double glo = kb_unkey(s_kg[0][tid]), ghi = kb_unkey(s_kg[1][tid]);
            const double lo1 = first_small ? slo : glo, hi1 = first_small ? shi : ghi;
            const double lo2 = first_small ? glo : slo, hi2 = first_small ? ghi : shi;
            double *nb1 = a.nbox + (size_t)c1 * 2 * D, *nb2 = nb1 + 2 * D;
            double *cb1 = a.cbox + (size_t)c1 * 2 * D, *cb2 = cb1 + 2 * D;
            nb1[tid] = lo1;
            nb1[D + tid] = hi1;
            nb2[tid] = lo2;
            nb2[D + tid] = hi2;
            const double clo = s_cb[0][tid], chi = s_cb[1][tid];
            cb1[tid] = clo;
            cb1[D + tid] = tid == c.cf ? c.cutval : chi;
            cb2[tid] = tid == c.cf ? c.cutval : clo;
            cb2[D + tid] = chi;
            if (tid == c.cf) {   // the node's record (divlow / divhigh: the children's boxes)
                KdbNode nd{};
                nd.child1 = (int32_t)c1;
                nd.child2 = (int32_t)c1 + 1;
                nd.left = l;
                nd.right = l + n;
                nd.divfeat = c.cf;
                nd.depth = dep;
                nd.divlow = hi1;
                nd.divhigh = lo2;
                nd.cutval = c.cutval;
                nd.split_val = c.split_val;
                nd.spread_gap = c.spread_gap;
                nd.cand = c.cand;
                a.nodes[me] = nd;
            }
        }
        if (tid == 0) {
            // children: leaves now; subtrees of <= KB_SMALL points to the waves (phase 2); larger
            // ones split next by every thread (the larger of the two kept in LDS)
            const uint32_t cl[2] = {l, l + n1}, cn[2] = {n1, n2};
            int keep = -1;
            for (int h = 0; h < 2; h++) {
                const uint32_t id = c1 + h;
                if (cn[h] <= 10) {
                    kb_write_leaf(a, id, cl[h], cl[h] + cn[h], dep + 1);
                    continue;
                }
                KdbNode cdn{};
                cdn.left = cl[h];
                cdn.right = cl[h] + cn[h];
                cdn.depth = dep + 1;
                a.nodes[id] = cdn;
                if (cn[h] <= KB_SMALL) {
                    if (s_nlist < KB_LIST) s_list[s_nlist++] = id;
                    else s_fail = 1;
                } else if (keep < 0 && cn[h] == max(n1, n2)) {
                    keep = h;
                } else {
                    if (s_nstack < KB_STACK) s_stack[s_nstack++] = id;
                    else s_fail = 1;
                }
            }
            s_keep = keep >= 0 ? 1u : 0u;
            if (keep >= 0) {
                s_me = c1 + keep;
                s_l = cl[keep];
                s_n = cn[keep];
                s_dep = dep + 1;
            }
        }
        __syncthreads();
        if (s_keep) {   // the kept child's points and boxes stay in LDS
            const uint32_t off = s_l - l;
            uint32_t tmp[KDB_MAXK / KB_THREADS];
            const uint32_t kn = s_n;
            const uint32_t E2 = (kn + KB_THREADS - 1) / KB_THREADS;
            const uint32_t k0 = min((uint32_t)tid * E2, kn), k1 = min(k0 + E2, kn);
            for (uint32_t j = 0; j < k1 - k0; j++) tmp[j] = s_ind[off + k0 + j];
            __syncthreads();
            for (uint32_t j = 0; j < k1 - k0; j++) s_ind[k0 + j] = tmp[j];
            if (tid < (int)D) {
                const bool one = s_me == c1;
                const double *nb = a.nbox + (size_t)(one ? c1 : c1 + 1) * 2 * D;   // (just written by this thread)
                s_pb[0][tid] = nb[tid];
                s_pb[1][tid] = nb[D + tid];
                const double clo = s_cb[0][tid], chi = s_cb[1][tid];
                s_cb[0][tid] = (!one && tid == c.cf) ? c.cutval : clo;
                s_cb[1][tid] = (one && tid == c.cf) ? c.cutval : chi;
            }
        }
        __syncthreads();
    }
    __syncthreads();

    const uint64_t t_p1 = wall_clock64();
    // ---- phase 2: subtrees of at most KB_SMALL points, one wave each --------------------------
    uint32_t *wi = w_ind[wave];
    double *wv = w_val[wave];
    uint8_t *wm = w_mpos[wave], *wp = w_ppos[wave];
    uint32_t *ws = w_stack[wave];
    for (;;) {
        uint32_t root = 0;
        if (lane == 0) {
            const uint32_t t = atomicAdd(&s_lnext, 1u);
            root = t < s_nlist && !s_fail ? s_list[t] : ~0u;
        }
        root = (uint32_t)__builtin_amdgcn_readlane((int)root, 0);
        if (root == ~0u) break;
        uint32_t nst = 1;
        if (lane == 0) ws[0] = root;
        for (;;) {
            __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
            __builtin_amdgcn_wave_barrier();
            if (nst == 0) break;
            const uint32_t me = ws[--nst];
            const KdbNode nd = a.nodes[me];
            const uint32_t l = nd.left, n = nd.right - nd.left, dep = nd.depth;
            const double *nb = a.nbox + (size_t)me * 2 * D, *cb = a.cbox + (size_t)me * 2 * D;
            const bool in = lane < (int)D;
            const double plo = in ? nb[lane] : 0.0, phi = in ? nb[D + lane] : 0.0;
            const double clo = in ? cb[lane] : 0.0, chi = in ? cb[D + lane] : 0.0;
            const KbCut c = kb_choose_cut(lane, D, plo, phi, clo, chi);
            // two positions per lane: 2 lane, 2 lane + 1
            uint32_t r_ind[2];
            double r_val[2];
            const uint32_t b0 = min(2u * lane, n), b1 = min(b0 + 2, n);
            for (uint32_t j = 0; j < b1 - b0; j++) {
                r_ind[j] = a.vind[l + b0 + j];
                r_val[j] = a.P[(size_t)r_ind[j] * D + c.cf];
                wi[b0 + j] = r_ind[j];
                wv[b0 + j] = r_val[j];
            }
            uint32_t lim1 = 0, lim2 = 0;
            for (int pass = 0; pass < 2; pass++) {
                const uint32_t from = pass ? lim1 : 0;
                uint32_t cnt = 0;
                for (uint32_t j = 0; j < b1 - b0; j++) {
                    const bool f = pass ? r_val[j] <= c.cutval : r_val[j] < c.cutval;
                    cnt += (b0 + j >= from && f) ? 1u : 0u;
                }
                const uint32_t inc = wave_scan_add(cnt);
                const uint32_t tot = (uint32_t)__builtin_amdgcn_readlane((int)inc, 63);
                const uint32_t lim = from + tot;
                uint32_t pf = inc - cnt;
                uint32_t src[2] = {b0, b0 + 1};
                for (uint32_t j = 0; j < b1 - b0; j++) {
                    const uint32_t i = b0 + j;
                    if (i < from) continue;
                    const bool f = pass ? r_val[j] <= c.cutval : r_val[j] < c.cutval;
                    if (i < lim && !f) wm[(i - from) - pf] = (uint8_t)i;
                    if (i >= lim && f) wp[(lim - from) - pf - 1] = (uint8_t)i;
                    pf += f ? 1u : 0u;
                }
                __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
                __builtin_amdgcn_wave_barrier();
                pf = inc - cnt;
                for (uint32_t j = 0; j < b1 - b0; j++) {
                    const uint32_t i = b0 + j;
                    if (i < from) continue;
                    const bool f = pass ? r_val[j] <= c.cutval : r_val[j] < c.cutval;
                    if (i < lim && !f) src[j] = wp[(i - from) - pf];
                    if (i >= lim && f) src[j] = wm[(lim - from) - pf - 1];
                    pf += f ? 1u : 0u;
                }
                for (uint32_t j = 0; j < b1 - b0; j++) {
                    r_ind[j] = wi[src[j]];
                    r_val[j] = wv[src[j]];
                }
                __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
                __builtin_amdgcn_wave_barrier();
                for (uint32_t j = 0; j < b1 - b0; j++) {
                    wi[b0 + j] = r_ind[j];
                    wv[b0 + j] = r_val[j];
                }
                __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
                __builtin_amdgcn_wave_barrier();
                if (pass) lim2 = lim;
                else lim1 = lim;
            }
            const uint32_t index = lim1 > n / 2 ? lim1 : (lim2 < n / 2 ? lim2 : n / 2);
            for (uint32_t j = 0; j < b1 - b0; j++) a.vind[l + b0 + j] = r_ind[j];
            // children's boxes, a dimension per lane
            const bool first_small = index <= n - index;
            const uint32_t sb = first_small ? 0 : index, sn = first_small ? index : n - index;
            const uint32_t gb = first_small ? index : 0, gn = n - sn;
            // (point, dimension) pairs over the lanes, LDS key min / max per dimension: every
            // lane's loads are independent, so they are all in flight at once
            unsigned long long *wk = w_key[wave];   // [0]: smaller child lo, [1] hi, [2] larger lo, [3] hi
            wk[lane] = ~0ull;
            wk[64 + lane] = 0ull;
            wk[128 + lane] = ~0ull;
            wk[192 + lane] = 0ull;
            __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
            __builtin_amdgcn_wave_barrier();
            kb_pairs_minmax(a.P, D, wi + sb, sn, lane, 64, D, nullptr, wk, wk + 64);
            __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
            __builtin_amdgcn_wave_barrier();
            double slo = in ? kb_unkey(wk[lane]) : 0.0, shi = in ? kb_unkey(wk[64 + lane]) : 0.0;
            const bool nlo = in && !(slo > plo), nhi = in && !(shi < phi);
            const uint64_t need = __ballot(nlo || nhi);
            const uint32_t ndl = (uint32_t)__popcll(need);
            uint32_t *wdl = w_dl[wave];
            if (nlo || nhi)
                wdl[__popcll(need & ((1ull << lane) - 1))] = (uint32_t)lane | (nlo ? 0x100u : 0u) | (nhi ? 0x200u : 0u);
            __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
            __builtin_amdgcn_wave_barrier();
            if (ndl) kb_pairs_minmax(a.P, D, wi + gb, gn, lane, 64, ndl, wdl, wk + 128, wk + 192);
            __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
            __builtin_amdgcn_wave_barrier();
            double glo = plo, ghi = phi;
            if (nlo) glo = kb_unkey(wk[128 + lane]);
            if (nhi) ghi = kb_unkey(wk[192 + lane]);
            uint32_t c1 = 0;
            if (lane == 0) {
                c1 = atomicAdd(&s_nnodes, 2u);
                atomicMax(&s_depth, dep + 1);
            }
            c1 = (uint32_t)__builtin_amdgcn_readlane((int)c1, 0);
            if (c1 + 2 > 2 * K) {
                if (lane == 0) s_fail = 1;
                break;
            }
            const uint32_t n1 = index, n2 = n - index;
            if (in) {
                const double lo1 = first_small ? slo : glo, hi1 = first_small ? shi : ghi;
                const double lo2 = first_small ? glo : slo, hi2 = first_small ? ghi : shi;
                double *nb1 = a.nbox + (size_t)c1 * 2 * D, *nb2 = nb1 + 2 * D;
                double *cb1 = a.cbox + (size_t)c1 * 2 * D, *cb2 = cb1 + 2 * D;
                nb1[lane] = lo1;
                nb1[D + lane] = hi1;
                nb2[lane] = lo2;
                nb2[D + lane] = hi2;
                cb1[lane] = clo;
                cb1[D + lane] = lane == c.cf ? c.cutval : chi;
                cb2[lane] = lane == c.cf ? c.cutval : clo;
                cb2[D + lane] = chi;
                if (lane == c.cf) {
                    KdbNode o{};
                    o.child1 = (int32_t)c1;
                    o.child2 = (int32_t)c1 + 1;
                    o.left = l;
                    o.right = l + n;
                    o.divfeat = c.cf;
                    o.depth = dep;
                    o.divlow = hi1;
                    o.divhigh = lo2;
                    o.cutval = c.cutval;
                    o.split_val = c.split_val;
                    o.spread_gap = c.spread_gap;
                    o.cand = c.cand;
                    a.nodes[me] = o;
                }
            }
            // (the records above are read back by this wave only: vector stores, then loads of
            // the same addresses by the same wave, in order)
            if (lane == 0) {
                const uint32_t cl[2] = {l, l + n1}, cn[2] = {n1, n2};
                for (int h = 1; h >= 0; h--) {   // child 1 on top: depth first, child 1 first
                    const uint32_t id = c1 + h;
                    if (cn[h] <= 10) {
                        kb_write_leaf(a, id, cl[h], cl[h] + cn[h], dep + 1);
                    } else {
                        KdbNode cdn{};
                        cdn.left = cl[h];
                        cdn.right = cl[h] + cn[h];
                        cdn.depth = dep + 1;
                        a.nodes[id] = cdn;
                        if (nst < KB_WSTACK) ws[nst] = id;
                        else s_fail = 1;
                        nst++;
                    }
                }
            }
            nst = (uint32_t)__builtin_amdgcn_readlane((int)nst, 0);
            if (nst > KB_WSTACK) break;
            // global writes of this wave (vind, records, boxes) before its next node reads them
            __threadfence_block();
        }
    }
    __syncthreads();

    const uint64_t t_p2 = wall_clock64();
    // ---- the images: kd_resolve's (device) and the host's (mapped) -----------------------------
    const uint32_t nn = s_nnodes;
    const bool ok = s_fail == 0;
    __threadfence_block();
    __syncthreads();
    if (ok) {
        double *flo = reinterpret_cast<double *>(a.flat);
        KdNodeDev *fn = reinterpret_cast<KdNodeDev *>(flo + 2 * D);
        uint32_t *fv = reinterpret_cast<uint32_t *>(fn + nn);
        if (tid < (int)D) {
            flo[tid] = a.nbox[tid];
            flo[D + tid] = a.nbox[D + tid];
        }
        for (uint32_t i = tid; i < nn; i += KB_THREADS) {
            const KdbNode nd = a.nodes[i];
            KdNodeDev o;
            o.child1 = nd.child1;
            o.child2 = nd.child2;
            if (nd.child1 < 0) {
                o.a = (int32_t)nd.left;
                o.lo = o.hi = 0;
            } else {
                o.a = (int32_t)((uint32_t)nd.divfeat | nd.left << 8);
                o.lo = nd.divlow;
                o.hi = nd.divhigh;
            }
            o.b = (int32_t)nd.right;
            fn[i] = o;
        }
        for (uint32_t i = tid; i < K; i += KB_THREADS) fv[i] = a.vind[i];
        // host image (kdb_host_layout): header | nodes | boxes | vind, at fixed offsets
        const KdbHostLayout L = kdb_host_layout(K, D);
        KdbNode *hn = reinterpret_cast<KdbNode *>(a.himg + L.nodes);
        double *hb = reinterpret_cast<double *>(a.himg + L.boxes);
        uint32_t *hv = reinterpret_cast<uint32_t *>(a.himg + L.vind);
        for (uint32_t i = tid; i < nn; i += KB_THREADS) hn[i] = a.nodes[i];
        for (uint32_t i = tid; i < nn * 2 * D; i += KB_THREADS) hb[i] = a.nbox[i];
        for (uint32_t i = tid; i < K; i += KB_THREADS) hv[i] = a.vind[i];
    }
    __threadfence_system();
    __syncthreads();
    if (tid == 0) {
        KdbHeader *h = reinterpret_cast<KdbHeader *>(a.himg);
        h->n_nodes = nn;
        h->depth = s_depth;
        h->status = ok ? 1u : 2u;
        h->pad2[0] = t_p1 - t_start;   // wall-clock ticks (100 MHz): phase 1, phase 2, the images
        h->pad2[1] = t_p2 - t_p1;
        h->pad2[2] = wall_clock64() - t_p2;
        __threadfence_system();
        __hip_atomic_store(&h->seq, a.seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
    }
}

bool kd_build_fits(uint32_t K, uint32_t D) { return K >= 1 && K <= KDB_MAXK && D >= 1 && D <= 64; }

hipError_t launch_kd_build(hipStream_t s, const double *P, uint32_t K, uint32_t D, uint32_t *vind, KdbNode *nodes,
                           double *nbox, double *cbox, uint8_t *flat, uint8_t *himg, uint64_t seq) {
    if (!kd_build_fits(K, D)) return hipErrorInvalidValue;
    const KbArgs a{P, K, D, vind, nodes, nbox, cbox, flat, himg, seq};
    hipLaunchKernelGGL(kd_build_kernel, dim3(1), dim3(KB_THREADS), 0, s, a);
    return hipGetLastError();
}

}  // namespace qvq
