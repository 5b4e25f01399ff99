// kdtree_dev.hpp -- flattened reference kd-tree and its device traversal.
//
// The host builds the tree over a level's codebook (kdtree.cpp, nanoflann 1.2.3 build) while
// the GPU searches; the recheck kernel then resolves exact fp64 ties on the device with the
// same traversal as RefKDTree::nearest (nanoflann.hpp:906-920, :1188-1270): first point
// visited wins on equal distances, the leaf's worst distance is captured at leaf entry and
// the pruning bound is updated as (mindistsq - dst) + cut_dist.
#pragma once
#include <cstdint>

#if defined(__HIPCC__)
#define QVQ_HD __host__ __device__
#else
#define QVQ_HD
#endif

namespace qvq {

// Squared L2 as the reference's Release build evaluates nanoflann's L2_Adaptor
// (nanoflann.hpp:320-339 under g++ -O3 -ffast-math): each group of four squares is added
// as (s1 + s2) + (s0 + s3), then the 0-3 leftover components one by one.
QVQ_HD inline double ref_l2_hd(const double *a, const double *b, int dim) {
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

struct KdNodeDev {
    int32_t child1, child2;   // -1: leaf
    int32_t a, b;             // leaf: vind[a, b); inner: a = divfeat | first << 8, vind[first, b)
    double lo, hi;            // inner: divlow, divhigh
};
QVQ_HD inline int kd_feat(const KdNodeDev &n) { return n.a & 0xFF; }
QVQ_HD inline int32_t kd_first(const KdNodeDev &n) { return n.child1 < 0 ? n.a : (int32_t)((uint32_t)n.a >> 8); }

struct KdView {
    const KdNodeDev *nodes = nullptr;
    const uint32_t *vind = nullptr;
    const double *lo = nullptr, *hi = nullptr;   // root bounding box
    int depth = 0;                               // 0: no device tree (host resolves ties)
    uint32_t n_nodes = 0;
    uint32_t bytes = 0;   // contiguous image lo[D] | hi[D] | nodes | vind from lo
};

// ---- the device build (k_kdbuild.hip) -------------------------------------------------------
// One node as the device builds it (ids in creation order, root 0; child1 < 0: leaf).  The host
// import (RefKDTree's image constructor) renumbers depth first.
constexpr uint32_t KDB_MAXK = 4096;   // code vectors the device build takes (its LDS arrays)
struct KdbNode {
    int32_t child1, child2;
    uint32_t left, right;   // vind[left, right)
    int32_t divfeat;
    uint32_t depth;         // the root is 1
    double divlow, divhigh, cutval, split_val, spread_gap;
    uint64_t cand;          // candidate dimensions (bit d)
};
struct KdbHeader {
    uint32_t n_nodes, depth, status, pad;   // status 1: built, 2: failed (the host builds instead)
    uint64_t seq;                           // written last: the launch's sequence number
    uint64_t pad2[5];
};
// The mapped host image: header | nodes[2K] | point boxes [2K][lo row D | hi row D] | vind[K].
struct KdbHostLayout {
    uint64_t nodes, boxes, vind, total;
};
QVQ_HD inline KdbHostLayout kdb_host_layout(uint32_t K, uint32_t D) {
    KdbHostLayout L;
    L.nodes = sizeof(KdbHeader);
    L.boxes = L.nodes + (uint64_t)2 * K * sizeof(KdbNode);
    L.vind = L.boxes + (uint64_t)2 * K * 2 * D * sizeof(double);
    L.total = L.vind + (uint64_t)K * 4;
    return L;
}

// Device stack frames are 12 bytes: one double (the cell bound mindistsq, replaced by the
// saved dists[f] once the first child is done) and node << 2 | phase.
constexpr int KD_FRAME_BYTES = 12;

// The reference search for query q over points pts (row stride S doubles): the recursive
// searchLevel unrolled onto an explicit stack of t.depth frames (sd, sn); dists holds D
// doubles.
QVQ_HD inline uint32_t kd_nearest_flat(const double *q, uint32_t D, const KdView &t, const double *pts, uint32_t S,
                                       double *sd, int32_t *sn, double *dists) {
    double distsq = 0;
    for (uint32_t d = 0; d < D; d++) {
        const double x = q[d];
        dists[d] = 0;
        if (x < t.lo[d]) {
            dists[d] = (x - t.lo[d]) * (x - t.lo[d]);
            distsq += dists[d];
        }
        if (x > t.hi[d]) {
            dists[d] = (x - t.hi[d]) * (x - t.hi[d]);
            distsq += dists[d];
        }
    }
    double best = 1.7976931348623157e308;   // numeric_limits<double>::max()
    uint32_t best_idx = 0;
    bool have = false;
    int sp = 0;
    sd[0] = distsq;
    sn[0] = 0;
    while (sp >= 0) {
        const int32_t node = sn[sp] >> 2, phase = sn[sp] & 3;
        const KdNodeDev n = t.nodes[node];
        if (n.child1 < 0) {
            const double worst = best;   // captured once per leaf
            for (int32_t i = n.a; i < n.b; i++) {
                const uint32_t idx = t.vind[i];
                const double dist = ref_l2_hd(q, pts + (uint64_t)idx * S, (int)D);
                if (dist < worst && (!have || best > dist)) {
                    best = dist;
                    best_idx = idx;
                    have = true;
                }
            }
            sp--;
            continue;
        }
        const int f = kd_feat(n);
        const double val = q[f];
        const double diff1 = val - n.lo, diff2 = val - n.hi;
        const bool left_first = (diff1 + diff2) < 0;
        if (phase == 0) {   // descend into the closer child
            sn[sp] = node << 2 | 1;
            sd[sp + 1] = sd[sp];
            sn[sp + 1] = (left_first ? n.child1 : n.child2) << 2;
            sp++;
            continue;
        }
        if (phase == 1) {   // then the other child if its cell can still hold a closer point
            const double cut_dist = left_first ? (val - n.hi) * (val - n.hi) : (val - n.lo) * (val - n.lo);
            const double dst = dists[f];
            const double m2 = (sd[sp] - dst) + cut_dist;   // the reference build's association
            dists[f] = cut_dist;
            sd[sp] = dst;
            sn[sp] = node << 2 | 2;
            if (m2 <= best) {   // mindistsq * epsError(1.0f) <= worstDist
                sd[sp + 1] = m2;
                sn[sp + 1] = (left_first ? n.child2 : n.child1) << 2;
                sp++;
                continue;
            }
        }
        dists[f] = sd[sp];
        sp--;
    }
    return best_idx;
}

}  // namespace qvq
