// See kdtree.hpp.  Build: nanoflann.hpp:863-871 (buildIndex), :1014-1036 (bounding box),
// :1046-1094 (divideTree), :1108-1147 (middleSplit_), :1159-1186 (planeSplit).
// Search (kdtree_dev.hpp, kd_nearest_flat): :906-920 (findNeighbors), :1188-1205 (initial
// distances), :1212-1270 (searchLevel) with KNNResultSet capacity 1 (:77-138): strict '<'
// everywhere, so among equal distances the first point visited wins.
#include "kdtree.hpp"

#include <algorithm>
#include <cmath>
#include <limits>
#include <memory>

namespace qvq {


double ref_l2(const double *a, const double *b, int dim) { return ref_l2_hd(a, b, dim); }

namespace {
constexpr int KD_MAX_DIM = 64;

// children's boxes per tree level, [2][KD_MAX_DIM] each: allocated on first use and kept
// (duplicated points make degenerate trees hundreds of levels deep)
Box *level_boxes(int level) {
    static thread_local std::vector<std::unique_ptr<Box[]>> levels;
    while ((int)levels.size() <= level) levels.emplace_back(new Box[2 * KD_MAX_DIM]);
    return levels[level].get();
}

// Per-dimension minima and maxima over the rows ind[0..count) of a row-major point set (the
// inner loop over a row's contiguous coordinates vectorises; built for AVX2 and baseline
// x86-64, picked at load time).  Exact min / max, so any instruction set gives the same values.
template <int DIM>
inline void rows_min_max_t(const double *pts, const size_t *ind, size_t count, int dim, double *mn, double *mx) {
    const int D = DIM ? DIM : dim;
    const double *p0 = pts + ind[0] * (size_t)D;
    for (int d = 0; d < D; d++) mn[d] = mx[d] = p0[d];
    for (size_t i = 1; i < count; i++) {
        const double *p = pts + ind[i] * (size_t)D;
        for (int d = 0; d < D; d++) {
            mn[d] = p[d] < mn[d] ? p[d] : mn[d];
            mx[d] = p[d] > mx[d] ? p[d] : mx[d];
        }
    }
}
__attribute__((target_clones("avx2", "default"))) void rows_min_max(const double *pts, const size_t *ind,
                                                                     size_t count, int dim, double *mn, double *mx) {
    if (dim == 48) rows_min_max_t<48>(pts, ind, count, dim, mn, mx);
    else if (dim == 12) rows_min_max_t<12>(pts, ind, count, dim, mn, mx);
    else rows_min_max_t<0>(pts, ind, count, dim, mn, mx);
}
}  // namespace

RefKDTree::RefKDTree(const double *pts, size_t K, int dim) : pts_(pts), dim_(dim), K_(K) {
    static thread_local std::vector<double> cols;   // reused: a fresh 1.5 MB buffer per level page-faults
    if (cols.size() < K * (size_t)dim) cols.resize(K * (size_t)dim);
    double *const cbuf = cols.data();
    cols_ = cbuf;
    vind_.resize(K);
    for (size_t i = 0; i < K; i++) vind_[i] = i;
    root_bbox_.resize(dim);
    // column-major copy and root box, 64 points at a time (their rows stay in L1 while
    // every column takes its 64 values)
    for (int d = 0; d < dim; d++) root_bbox_[d].low = root_bbox_[d].high = pts[d];
    for (size_t k0 = 0; k0 < K; k0 += 64) {
        const size_t k1 = std::min(K, k0 + 64);
        for (int d = 0; d < dim; d++) {
            double *col = cbuf + (size_t)d * K;
            double lo = root_bbox_[d].low, hi = root_bbox_[d].high;
            for (size_t k = k0; k < k1; k++) {
                const double v = pts[k * (size_t)dim + d];
                col[k] = v;
                lo = v < lo ? v : lo;
                hi = v > hi ? v : hi;
            }
            root_bbox_[d].low = lo;
            root_bbox_[d].high = hi;
        }
    }
    nodes_.reserve(2 * (K / 5 + 1));
    node_box_.clear();
    node_box_.reserve(2 * (K / 5 + 1) * (size_t)dim);
    std::vector<Box> box(root_bbox_);
    divide(0, K, box.data(), 1, nodes_, depth_);
    flat_nodes_.resize(nodes_.size());
    flat_vind_.resize(K);
    flat_box_.resize(2 * (size_t)dim);
    flatten(flat_nodes_.data(), flat_vind_.data(), flat_box_.data(), flat_box_.data() + dim);
    cols_ = nullptr;
}

// Branch-free minima and maxima: the comparisons are data-dependent, and mispredicted
// branches dominated the build (min / max are exact, so any form gives the same values).
void RefKDTree::min_max(const size_t *ind, size_t count, int e, double &mn, double &mx) const {
    double a = pt(ind[0], e), b = a;
    for (size_t i = 1; i < count; i++) {
        const double v = pt(ind[i], e);
        a = v < a ? v : a;
        b = v > b ? v : b;
    }
    mn = a;
    mx = b;
}

void RefKDTree::plane_split(size_t *ind, size_t count, int cutfeat, double cutval, size_t &lim1,
                            size_t &lim2) {
    // Two Hoare-style passes: [< cutval | == cutval | > cutval].  'right' is unsigned, so
    // the reference stops when it reaches 0 as well.
    size_t left = 0, right = count - 1;
    for (;;) {
        while (left <= right && pt(ind[left], cutfeat) < cutval) ++left;
        while (right && left <= right && pt(ind[right], cutfeat) >= cutval) --right;
        if (left > right || !right) break;
        std::swap(ind[left], ind[right]);
        ++left;
        --right;
    }
    lim1 = left;
    right = count - 1;
    for (;;) {
        while (left <= right && pt(ind[left], cutfeat) <= cutval) ++left;
        while (right && left <= right && pt(ind[right], cutfeat) > cutval) --right;
        if (left > right || !right) break;
        std::swap(ind[left], ind[right]);
        ++left;
        --right;
    }
    lim2 = left;
}

void RefKDTree::middle_split(size_t *ind, size_t count, size_t &index, int &cutfeat, double &cutval,
                             const Box *bbox, Node *info) {
    const double EPS = 0.00001;
    double max_span = bbox[0].high - bbox[0].low;
    for (int i = 1; i < dim_; i++) max_span = std::max(max_span, bbox[i].high - bbox[i].low);
    // Candidate dimensions: span within EPS of the widest.  In real codebooks (empty cells at
    // 0, saturated colours) every dimension not yet cut along the path has the root's span,
    // so upper nodes need the point min/max of most dimensions, from the column copy.
    int q[64], nq = 0;
    for (int i = 0; i < dim_; i++)
        if (bbox[i].high - bbox[i].low > (1 - EPS) * max_span) q[nq++] = i;
    double qmn[64], qmx[64];
    if (nq * 4 >= dim_ && dim_ >= 8) {
        // most dimensions are candidates (real codebooks: every dimension not yet cut on the
        // path keeps the root's span): one row-major pass over the node's points gives all
        // of them -- each point's contiguous row once, instead of nq column gathers
        double mn[64], mx[64];
        rows_min_max(pts_, ind, count, dim_, mn, mx);
        for (int j = 0; j < nq; j++) {
            qmn[j] = mn[q[j]];
            qmx[j] = mx[q[j]];
        }
    } else {
        for (int j = 0; j < nq; j++) min_max(ind, count, q[j], qmn[j], qmx[j]);
    }
    double max_spread = -1, mn = 0, mx = 0;
    cutfeat = 0;
    bool have = false;
    for (int j = 0; j < nq; j++)
        if (qmx[j] - qmn[j] > max_spread) {
            cutfeat = q[j];
            max_spread = qmx[j] - qmn[j];
            mn = qmn[j];
            mx = qmx[j];
            have = true;
        }
    if (!have) min_max(ind, count, cutfeat, mn, mx);
    const double split_val = (bbox[cutfeat].low + bbox[cutfeat].high) / 2;
    cutval = split_val < mn ? mn : (split_val > mx ? mx : split_val);
    {   // what a later change of one coordinate can move (unchanged_under)
        double second = -std::numeric_limits<double>::infinity();
        uint64_t cand = 0;
        for (int j = 0; j < nq; j++) {
            cand |= 1ull << q[j];
            if (q[j] != cutfeat) second = std::max(second, qmx[j] - qmn[j]);
        }
        info->cand = cand;
        info->spread_gap = have ? max_spread - second : -1.0;
        info->split_val = split_val;
    }
    size_t lim1, lim2;
    plane_split(ind, count, cutfeat, cutval, lim1, lim2);
    if (lim1 > count / 2) index = lim1;
    else if (lim2 < count / 2) index = lim2;
    else index = count / 2;
}

// bbox is in/out: the caller's cell box on entry, the node's actual point box on exit.
int RefKDTree::divide(size_t left, size_t right, Box *bbox, int level, std::vector<Node> &nodes, int &depth) {
    const int me = (int)nodes.size();
    depth = std::max(depth, level);
    nodes.push_back(Node());
    node_box_.resize(node_box_.size() + dim_);
    if (right - left <= 10) {   // leaf_max_size (KDTreeVectorOfVectorsAdaptor.hpp:59)
        Node &n = nodes[me];
        n.leaf = true;
        n.left = left;
        n.right = right;
        n.child1 = n.child2 = -1;
        n.cutval = 0;
        double mn[64], mx[64];
        rows_min_max(pts_, vind_.data() + left, right - left, dim_, mn, mx);   // row-major: a point's coordinates are contiguous
        for (int d = 0; d < dim_; d++) {
            bbox[d].low = mn[d];
            bbox[d].high = mx[d];
        }
        std::copy(bbox, bbox + dim_, node_box_.begin() + (size_t)me * dim_);
        return me;
    }
    size_t idx;
    int cutfeat;
    double cutval;
    Node info;
    middle_split(vind_.data() + left, right - left, idx, cutfeat, cutval, bbox, &info);
    // children's boxes (a vector per node cost two heap allocations each)
    Box *lb = level_boxes(level), *rb = lb + dim_;
    std::copy(bbox, bbox + dim_, lb);
    std::copy(bbox, bbox + dim_, rb);
    lb[cutfeat].high = cutval;
    rb[cutfeat].low = cutval;
    const int c1 = divide(left, left + idx, lb, level + 1, nodes, depth);
    const int c2 = divide(left + idx, right, rb, level + 1, nodes, depth);
    Node &n = nodes[me];
    n.leaf = false;
    n.left = left;
    n.right = right;
    n.divfeat = cutfeat;
    n.child1 = c1;
    n.child2 = c2;
    n.divlow = lb[cutfeat].high;
    n.divhigh = rb[cutfeat].low;
    n.cutval = cutval;
    n.split_val = info.split_val;
    n.spread_gap = info.spread_gap;
    n.cand = info.cand;
    for (int d = 0; d < dim_; d++) {
        bbox[d].low = std::min(lb[d].low, rb[d].low);
        bbox[d].high = std::max(lb[d].high, rb[d].high);
    }
    std::copy(bbox, bbox + dim_, node_box_.begin() + (size_t)me * dim_);
    return me;
}

bool RefKDTree::unchanged_under(const double *pts2) const {
    std::vector<uint32_t> pos;   // point -> its place in vind (built on the first changed coordinate)
    for (size_t p = 0; p < K_; p++)
        for (int d = 0; d < dim_; d++) {
            const double x = pts_[p * (size_t)dim_ + d], y = pts2[p * (size_t)dim_ + d];
            if (x == y && std::signbit(x) == std::signbit(y)) continue;
            if (pos.empty()) {
                pos.resize(K_);
                for (size_t i = 0; i < K_; i++) pos[vind_[i]] = (uint32_t)i;
            }
            const double dev = std::fabs(x - y);
            // the root box is every cell box's origin
            if (!(x > root_bbox_[d].low && x < root_bbox_[d].high && y > root_bbox_[d].low && y < root_bbox_[d].high))
                return false;
            const size_t at = pos[p];
            int node = 0;
            while (!nodes_[node].leaf) {
                const Node &n = nodes_[node];
                const Box &b = node_box_[(size_t)node * dim_ + d];
                const bool extreme = !(x > b.low && x < b.high && y > b.low && y < b.high);
                if (extreme && ((n.cand >> d) & 1)) {
                    // the spread of a candidate moves by at most dev: the choice must keep its margin
                    if (!(n.spread_gap > 2 * dev)) return false;
                    // and the cut dimension's clamp must stay inactive on both sides
                    if (d == n.divfeat && (n.cutval != n.split_val || !((x < n.cutval) == (y < n.cutval))))
                        return false;
                }
                if (n.divfeat == d) {   // the partition compares against the cut: same side, never equal
                    const double c = n.cutval;
                    if ((x < c) != (y < c) || x == c || y == c) return false;
                }
                const Node &c1 = nodes_[n.child1];
                const bool left = at < c1.right;
                if (n.divfeat == d) {   // the children's boxes give divlow / divhigh
                    const Box &cb = node_box_[(size_t)(left ? n.child1 : n.child2) * dim_ + d];
                    if (left ? !(x < cb.high && y < cb.high) : !(x > cb.low && y > cb.low)) return false;
                }
                node = left ? n.child1 : n.child2;
            }
        }
    return true;
}

void RefKDTree::flatten(KdNodeDev *nodes, uint32_t *vind, double *lo, double *hi) const {
    for (size_t i = 0; i < nodes_.size(); i++) {
        const Node &n = nodes_[i];
        KdNodeDev &o = nodes[i];
        if (n.leaf) {
            o.child1 = o.child2 = -1;
            o.a = (int32_t)n.left;
            o.b = (int32_t)n.right;
            o.lo = o.hi = 0;
        } else {
            o.child1 = n.child1;
            o.child2 = n.child2;
            o.a = (int32_t)((uint32_t)n.divfeat | (uint32_t)n.left << 8);
            o.b = (int32_t)n.right;
            o.lo = n.divlow;
            o.hi = n.divhigh;
        }
    }
    for (size_t i = 0; i < vind_.size(); i++) vind[i] = (uint32_t)vind_[i];
    for (int d = 0; d < dim_; d++) {
        lo[d] = root_bbox_[d].low;
        hi[d] = root_bbox_[d].high;
    }
}

// The traversal the device runs (kdtree_dev.hpp), so host tests check the device's code.
uint32_t RefKDTree::nearest(const double *q) const {
    KdView v;
    v.nodes = flat_nodes_.data();
    v.vind = flat_vind_.data();
    v.lo = flat_box_.data();
    v.hi = flat_box_.data() + dim_;
    v.depth = depth_;
    std::vector<double> sd((size_t)depth_ + 1), dists((size_t)dim_);
    std::vector<int32_t> sn((size_t)depth_ + 1);
    return kd_nearest_flat(q, (uint32_t)dim_, v, pts_, (uint32_t)dim_, sd.data(), sn.data(), dists.data());
}

}  // namespace qvq
