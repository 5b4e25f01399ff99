// See kdtree.hpp.  Build: nanoflann.hpp:863-871 (buildIndex), :1014-1036 (bounding box),
// :1046-1094 (divideTree), :1108-1147 (middleSplit_), :1159-1186 (planeSplit).
// Search (kdtree_dev.hpp, kd_nearest_flat): :906-920 (findNeighbors), :1188-1205 (initial
// distances), :1212-1270 (searchLevel) with KNNResultSet capacity 1 (:77-138): strict '<'
// everywhere, so among equal distances the first point visited wins.
#include "kdtree.hpp"

#include <algorithm>
#include <cmath>
#include <cstdlib>
#include <cstring>
#include <immintrin.h>
#include <limits>
#include <memory>
#include <thread>

namespace qvq {

namespace {
// The pool behind Recycled<T>: at most 8 buffers per type (the largest kept), the smallest that
// fits and is at most 1.5x the request is taken.
template <class T>
struct BufPool {
    std::mutex m;
    std::vector<std::pair<size_t, std::unique_ptr<T[]>>> free;
    static BufPool &get() {
        static BufPool *p = new BufPool;   // never destroyed: trees may die at exit
        return *p;
    }
};
}  // namespace

template <class T>
void Recycled<T>::align() {   // (threads that share a buffer write whole cache lines)
    const uintptr_t a = reinterpret_cast<uintptr_t>(p_.get());
    base_ = reinterpret_cast<T *>((a + 63) & ~(uintptr_t)63);
}

template <class T>
void Recycled<T>::resize(size_t n) {
    n_ = n;
    if (n <= cap_) return;
    release();
    n_ = n;
    BufPool<T> &P = BufPool<T>::get();
    {
        std::lock_guard<std::mutex> g(P.m);
        size_t best = P.free.size();
        // (not one of more than 1.5x the request: the levels' sizes double, and a level that
        // took the next one's buffer left the largest level to write fresh pages -- C4 level
        // 12 ~0.5 ms a call)
        for (size_t i = 0; i < P.free.size(); i++)
            if (P.free[i].first >= n && P.free[i].first <= n + n / 2 + 1024 &&
                (best == P.free.size() || P.free[i].first < P.free[best].first))
                best = i;
        if (best < P.free.size()) {
            cap_ = P.free[best].first;
            p_ = std::move(P.free[best].second);
            P.free.erase(P.free.begin() + (std::ptrdiff_t)best);
            align();
            return;
        }
    }
    // cap_ usable elements after the 64-byte alignment of the base
    p_.reset(new T[n + 64 / sizeof(T) + 1]);
    cap_ = n;
    align();
}

template <class T>
void Recycled<T>::release() {
    if (!p_) return;
    BufPool<T> &P = BufPool<T>::get();
    std::lock_guard<std::mutex> g(P.m);
    if (P.free.size() >= 8) {   // drop the smallest
        size_t s = 0;
        for (size_t i = 1; i < P.free.size(); i++)
            if (P.free[i].first < P.free[s].first) s = i;
        if (P.free[s].first >= cap_) {
            p_.reset();
            base_ = nullptr;
            cap_ = n_ = 0;
            return;
        }
        P.free.erase(P.free.begin() + (std::ptrdiff_t)s);
    }
    P.free.emplace_back(cap_, std::move(p_));
    base_ = nullptr;
    cap_ = n_ = 0;
}
template class Recycled<double>;
template class Recycled<RefKDTree::Iv>;
template class Recycled<RefKDTree::Node>;
template class Recycled<Box>;


double ref_l2(const double *a, const double *b, int dim) { return ref_l2_hd(a, b, dim); }

namespace {
// ref_l2_hd's sum with an early exit: once a prefix exceeds cap it is returned (the terms are
// nonnegative and rounding is monotone, so the whole sum, in the same order, exceeds cap too).
inline double ref_l2_cap(const double *a, const double *b, int dim, double cap) {
    double r = 0;
    int d = 0;
    for (; d + 3 < dim; d += 4) {
        const double e0 = a[d] - b[d], e1 = a[d + 1] - b[d + 1];
        const double e2 = a[d + 2] - b[d + 2], e3 = a[d + 3] - b[d + 3];
        r += (e1 * e1 + e2 * e2) + (e0 * e0 + e3 * e3);
        if (r > cap) return r;
    }
    for (; d < dim; d++) {
        const double e = a[d] - b[d];
        r += e * e;
    }
    return r;
}
}  // namespace

namespace {
constexpr int KD_MAX_DIM = 64;
inline uint64_t all_dims(int dim) { return dim >= 64 ? ~0ull : (1ull << dim) - 1; }

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

namespace {
bool has_avx2() {
    static const bool v = __builtin_cpu_supports("avx2");
    return v;
}
// cols[d][k] = pts[k][d]: 4 x 4 blocks through registers (4 rows' loads, 4 columns' stores),
// the points 64 at a time (their rows stay in L1 while every column takes its 64 values)
__attribute__((target("avx2"))) void transpose_rows_avx2(const double *pts, size_t K, int dim, double *cols) {
    const size_t K4 = K & ~(size_t)3;
    const int d4 = dim & ~3;
    for (size_t k0 = 0; k0 < K4; k0 += 64) {
        const size_t k1 = std::min(K4, k0 + 64);
        for (int d = 0; d < d4; d += 4)
            for (size_t k = k0; k < k1; k += 4) {
                const double *p = pts + k * (size_t)dim + d;
                const __m256d r0 = _mm256_loadu_pd(p), r1 = _mm256_loadu_pd(p + dim), r2 = _mm256_loadu_pd(p + 2 * dim),
                              r3 = _mm256_loadu_pd(p + 3 * dim);
                const __m256d t0 = _mm256_unpacklo_pd(r0, r1), t1 = _mm256_unpackhi_pd(r0, r1),
                              t2 = _mm256_unpacklo_pd(r2, r3), t3 = _mm256_unpackhi_pd(r2, r3);
                double *c = cols + (size_t)d * K + k;
                _mm256_storeu_pd(c, _mm256_permute2f128_pd(t0, t2, 0x20));
                _mm256_storeu_pd(c + K, _mm256_permute2f128_pd(t1, t3, 0x20));
                _mm256_storeu_pd(c + 2 * K, _mm256_permute2f128_pd(t0, t2, 0x31));
                _mm256_storeu_pd(c + 3 * K, _mm256_permute2f128_pd(t1, t3, 0x31));
            }
    }
    for (int d = 0; d < dim; d++)   // the ragged edges
        for (size_t k = d < d4 ? K4 : 0; k < K; k++) cols[(size_t)d * K + k] = pts[k * (size_t)dim + d];
}
void transpose_rows(const double *pts, size_t K, int dim, double *cols) {
    if (has_avx2()) {
        transpose_rows_avx2(pts, K, dim, cols);
        return;
    }
    for (size_t k0 = 0; k0 < K; k0 += 64) {
        const size_t k1 = std::min(K, k0 + 64);
        for (int d = 0; d < dim; d++) {
            double *col = cols + (size_t)d * K;
            for (size_t k = k0; k < k1; k++) col[k] = pts[k * (size_t)dim + d];
        }
    }
}
}  // namespace

RefKDTree::RefKDTree(const double *pts, size_t K, int dim, const std::atomic<bool> *cancel)
    : pts_(pts), dim_(dim), K_(K), cancel_(cancel) {
    static std::atomic<uint64_t> next_id{1};
    id_ = next_id.fetch_add(1);
    static thread_local std::vector<double> cols;   // reused: a fresh 1.5 MB buffer per level page-faults
    if (cols.size() < K * (size_t)dim) cols.resize(K * (size_t)dim);
    double *const cbuf = cols.data();
    cols_ = cbuf;
    vind_.resize(K);
    for (size_t i = 0; i < K; i++) vind_[i] = i;
    root_bbox_.resize(dim);
    // the root box from one vectorised row-major pass; the column-major copy 64 points at a
    // time (their rows stay in L1 while every column takes its 64 values), plain copies (a
    // min / max chain per column here cost a dependent compare per value)
    if (K) {
        double mn[64], mx[64];
        rows_min_max(pts, vind_.data(), K, dim, mn, mx);
        for (int d = 0; d < dim; d++) root_bbox_[d] = Box{mn[d], mx[d]};
    }
    transpose_rows(pts, K, dim, cbuf);
    // every node's record and box in one pooled buffer each (a tree of K points has fewer than
    // 2K + 1 nodes unless empty leaves pile up; push_back grows then)
    nodes_.reserve(2 * K + 1);
    node_box_.reserve((2 * K + 1) * (size_t)dim);
    std::vector<Box> box(root_bbox_);
    Known &rk = level_known(0)[0];   // the root's extremes: its box
    std::copy(root_bbox_.begin(), root_bbox_.end(), rk.b);
    rk.mask = K ? all_dims(dim) : 0;
    divide(0, K, box.data(), rk, 1, nodes_, depth_);
    flat_nodes_.resize(nodes_.size());
    flat_vind_.resize(K);
    flat_box_.resize(2 * (size_t)dim);
    flatten(flat_nodes_.data(), flat_vind_.data(), flat_box_.data(), flat_box_.data() + dim);
    cols_ = nullptr;
}

RefKDTree::RefKDTree(const double *pts, size_t K, int dim, const uint8_t *img) : pts_(pts), dim_(dim), K_(K) {
    static std::atomic<uint64_t> next_id{1};
    id_ = next_id.fetch_add(1);
    const KdbHeader &h = *reinterpret_cast<const KdbHeader *>(img);
    const KdbHostLayout L = kdb_host_layout((uint32_t)K, (uint32_t)dim);
    const KdbNode *dn = reinterpret_cast<const KdbNode *>(img + L.nodes);
    const double *db = reinterpret_cast<const double *>(img + L.boxes);
    const uint32_t *dv = reinterpret_cast<const uint32_t *>(img + L.vind);
    const uint32_t nn = h.n_nodes;
    // depth-first order, child 1 first: the host build's node numbering
    std::vector<uint32_t> order, pre(nn, 0);
    order.reserve(nn);
    std::vector<uint32_t> st(1, 0);
    while (!st.empty()) {
        const uint32_t d = st.back();
        st.pop_back();
        pre[d] = (uint32_t)order.size();
        order.push_back(d);
        if (dn[d].child1 >= 0) {
            st.push_back((uint32_t)dn[d].child2);
            st.push_back((uint32_t)dn[d].child1);
        }
    }
    nodes_.resize(order.size());
    node_box_.resize(order.size() * (size_t)dim);
    for (size_t i = 0; i < order.size(); i++) {
        const KdbNode &d = dn[order[i]];
        Node &n = nodes_[i];
        n = Node();
        n.leaf = d.child1 < 0;
        n.left = d.left;
        n.right = d.right;
        if (n.leaf) {
            n.child1 = n.child2 = -1;
        } else {
            n.divfeat = d.divfeat;
            n.divlow = d.divlow;
            n.divhigh = d.divhigh;
            n.cutval = d.cutval;
            n.split_val = d.split_val;
            n.spread_gap = d.spread_gap;
            n.cand = d.cand;
            n.child1 = (int)pre[(uint32_t)d.child1];
            n.child2 = (int)pre[(uint32_t)d.child2];
        }
        const double *b = db + (size_t)order[i] * 2 * dim;
        for (int e = 0; e < dim; e++) node_box_[i * (size_t)dim + e] = Box{b[e], b[dim + e]};
    }
    vind_.assign(dv, dv + K);
    root_bbox_.assign(node_box_.begin(), node_box_.begin() + dim);
    depth_ = (int)h.depth;
    flat_nodes_.resize(nodes_.size());
    flat_vind_.resize(K);
    flat_box_.resize(2 * (size_t)dim);
    flatten(flat_nodes_.data(), flat_vind_.data(), flat_box_.data(), flat_box_.data() + dim);
}

bool RefKDTree::same_as(const RefKDTree &o, std::string *why) const {
    auto fail = [&](const std::string &w) {
        if (why) *why = w;
        return false;
    };
    if (K_ != o.K_ || dim_ != o.dim_) return fail("shape");
    if (nodes_.size() != o.nodes_.size()) return fail("node count " + std::to_string(nodes_.size()) + " vs " +
                                                      std::to_string(o.nodes_.size()));
    if (depth_ != o.depth_) return fail("depth " + std::to_string(depth_) + " vs " + std::to_string(o.depth_));
    for (size_t i = 0; i < K_; i++)
        if (vind_[i] != o.vind_[i]) return fail("vind at " + std::to_string(i));
    for (size_t i = 0; i < nodes_.size(); i++) {
        const Node &a = nodes_[i], &b = o.nodes_[i];
        const std::string at = " at node " + std::to_string(i);
        if (a.leaf != b.leaf || a.left != b.left || a.right != b.right) return fail("structure" + at);
        if (!a.leaf && (a.divfeat != b.divfeat || a.child1 != b.child1 || a.child2 != b.child2 ||
                        a.divlow != b.divlow || a.divhigh != b.divhigh || a.cutval != b.cutval ||
                        a.split_val != b.split_val || a.spread_gap != b.spread_gap || a.cand != b.cand))
            return fail("split" + at);
        for (int d = 0; d < dim_; d++) {
            const Box &x = node_box_[i * (size_t)dim_ + d], &y = o.node_box_[i * (size_t)dim_ + d];
            if (x.low != y.low || x.high != y.high) return fail("point box" + at + " dim " + std::to_string(d));
        }
    }
    for (int d = 0; d < dim_; d++)
        if (root_bbox_[d].low != o.root_bbox_[d].low || root_bbox_[d].high != o.root_bbox_[d].high) return fail("root box");
    return true;
}

void RefKDTree::to_device_image(uint8_t *img) const {
    const KdbHostLayout L = kdb_host_layout((uint32_t)K_, (uint32_t)dim_);
    KdbHeader &h = *reinterpret_cast<KdbHeader *>(img);
    KdbNode *dn = reinterpret_cast<KdbNode *>(img + L.nodes);
    double *db = reinterpret_cast<double *>(img + L.boxes);
    uint32_t *dv = reinterpret_cast<uint32_t *>(img + L.vind);
    // breadth first from the root: node q of the queue gets id q, its children the next two ids
    std::vector<int> queue(1, 0);
    std::vector<uint32_t> depth(1, 1);
    for (size_t q = 0; q < queue.size(); q++) {
        const Node &n = nodes_[(size_t)queue[q]];
        KdbNode o{};
        o.left = (uint32_t)n.left;
        o.right = (uint32_t)n.right;
        o.depth = depth[q];
        if (n.leaf) {
            o.child1 = o.child2 = -1;
        } else {
            o.child1 = (int32_t)queue.size();
            o.child2 = o.child1 + 1;
            queue.push_back(n.child1);
            queue.push_back(n.child2);
            depth.push_back(depth[q] + 1);
            depth.push_back(depth[q] + 1);
            o.divfeat = n.divfeat;
            o.divlow = n.divlow;
            o.divhigh = n.divhigh;
            o.cutval = n.cutval;
            o.split_val = n.split_val;
            o.spread_gap = n.spread_gap;
            o.cand = n.cand;
        }
        dn[q] = o;
        for (int e = 0; e < dim_; e++) {
            const Box &bx = node_box_[(size_t)queue[q] * dim_ + e];
            db[q * 2 * (size_t)dim_ + e] = bx.low;
            db[q * 2 * (size_t)dim_ + dim_ + e] = bx.high;
        }
    }
    for (size_t i = 0; i < K_; i++) dv[i] = (uint32_t)vind_[i];
    h = KdbHeader{};
    h.n_nodes = (uint32_t)queue.size();
    h.depth = (uint32_t)depth_;
    h.status = 1;
}

// Branch-free minima and maxima: the comparisons are data-dependent, and mispredicted
// branches dominated the build; four independent chains, since one chain waits on a dependent
// compare per value (min / max are exact, so any order gives the same values).
void RefKDTree::min_max(const size_t *ind, size_t count, int e, double &mn, double &mx) const {
    const double *col = cols_ + (size_t)e * K_;
    double a0 = col[ind[0]], b0 = a0, a1 = a0, b1 = a0, a2 = a0, b2 = a0, a3 = a0, b3 = a0;
    size_t i = 1;
    for (; i + 4 <= count; i += 4) {
        const double v0 = col[ind[i]], v1 = col[ind[i + 1]], v2 = col[ind[i + 2]], v3 = col[ind[i + 3]];
        a0 = v0 < a0 ? v0 : a0;
        b0 = v0 > b0 ? v0 : b0;
        a1 = v1 < a1 ? v1 : a1;
        b1 = v1 > b1 ? v1 : b1;
        a2 = v2 < a2 ? v2 : a2;
        b2 = v2 > b2 ? v2 : b2;
        a3 = v3 < a3 ? v3 : a3;
        b3 = v3 > b3 ? v3 : b3;
    }
    for (; i < count; i++) {
        const double v = col[ind[i]];
        a0 = v < a0 ? v : a0;
        b0 = v > b0 ? v : b0;
    }
    a0 = a1 < a0 ? a1 : a0;
    a2 = a3 < a2 ? a3 : a2;
    b0 = b1 > b0 ? b1 : b0;
    b2 = b3 > b2 ? b3 : b2;
    mn = a2 < a0 ? a2 : a0;
    mx = b2 > b0 ? b2 : b0;
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
                             const Box *bbox, Known &kn, Node *info) {
    const double EPS = 0.00001;
    double max_span = bbox[0].high - bbox[0].low;
    for (int i = 1; i < dim_; i++) max_span = std::max(max_span, bbox[i].high - bbox[i].low);
    // Candidate dimensions: span within EPS of the widest.  In real codebooks (empty cells at
    // 0, saturated colours) every dimension not yet cut along the path has the root's span,
    // so upper nodes need the point min/max of most dimensions.  Those the parent's extremes
    // do not settle (child_known) are computed here.
    int q[64], nq = 0, nu = 0;
    for (int i = 0; i < dim_; i++)
        if (bbox[i].high - bbox[i].low > (1 - EPS) * max_span) {
            nu += !(kn.mask >> i & 1);
            q[nq++] = i;
        }
    if (nu * 4 >= dim_ && dim_ >= 8) {
        // most dimensions wanted (real codebooks: every dimension not yet cut on the path
        // keeps the root's span): one row-major pass over the node's points gives all of
        // them -- each point's contiguous row once, instead of nu column gathers
        double mn[64], mx[64];
        rows_min_max(pts_, ind, count, dim_, mn, mx);
        for (int d = 0; d < dim_; d++) kn.b[d] = Box{mn[d], mx[d]};
        kn.mask = all_dims(dim_);
    } else if (nu) {
        for (int j = 0; j < nq; j++)
            if (!(kn.mask >> q[j] & 1)) {
                min_max(ind, count, q[j], kn.b[q[j]].low, kn.b[q[j]].high);
                kn.mask |= 1ull << q[j];
            }
    }
    double qmn[64], qmx[64];
    for (int j = 0; j < nq; j++) {
        qmn[j] = kn.b[q[j]].low;
        qmx[j] = kn.b[q[j]].high;
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
    if (!have) {
        if (!(kn.mask >> cutfeat & 1)) {
            min_max(ind, count, cutfeat, kn.b[cutfeat].low, kn.b[cutfeat].high);
            kn.mask |= 1ull << cutfeat;
        }
        mn = kn.b[cutfeat].low;
        mx = kn.b[cutfeat].high;
    }
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

// The children's known extremes (ind[0, n1) and ind[n1, count)): the smaller child's from its
// rows; the larger child keeps each known parent extreme the smaller child stays strictly
// inside of (the point attaining it is the larger child's).  A degenerate chain (a node peeling
// a few points off the duplicated code vectors per level) then skips most of its row passes and
// column scans: C4 level 12 49.6 K rows and 0.89 M column values -> 21.2 K and 0.36 M.  Below
// 32 dimensions (D = 12: short rows, few column scans) only from a node whose extremes are all
// known -- the smaller child's row pass at every node cost more than it saved there.
void RefKDTree::child_known(const size_t *ind, size_t n1, size_t count, const Known &kn, Known &k1,
                            Known &k2) const {
    k1.mask = k2.mask = 0;
    if (dim_ < 32 && kn.mask != all_dims(dim_)) return;
    const bool first_small = n1 <= count - n1;
    const size_t s = first_small ? n1 : count - n1;
    Known &ks = first_small ? k1 : k2, &kb = first_small ? k2 : k1;
    if (s == 0) {   // (an empty child is a leaf; it reads nothing)
        kb = kn;
        return;
    }
    double mn[64], mx[64];
    rows_min_max(pts_, first_small ? ind : ind + n1, s, dim_, mn, mx);
    uint64_t m = 0;
    for (int d = 0; d < dim_; d++) {
        ks.b[d] = Box{mn[d], mx[d]};
        kb.b[d] = kn.b[d];
        m |= (uint64_t)(mn[d] > kn.b[d].low && mx[d] < kn.b[d].high) << d;
    }
    ks.mask = all_dims(dim_);
    kb.mask = m & kn.mask;
}

RefKDTree::Known *RefKDTree::level_known(int level) {
    static thread_local std::vector<std::unique_ptr<Known[]>> levels;
    while ((int)levels.size() <= level) levels.emplace_back(new Known[2]);
    return levels[level].get();
}

// bbox is in/out: the caller's cell box on entry, the node's actual point box on exit.
int RefKDTree::divide(size_t left, size_t right, Box *bbox, Known &kn, int level, RecycledVec<Node> &nodes,
                      int &depth) {
    const int me = (int)nodes.size();
    depth = std::max(depth, level);
    nodes.push_back(Node());
    node_box_.resize(node_box_.size() + dim_);
    if (cancel_ && !cancelled_ && cancel_->load(std::memory_order_relaxed)) cancelled_ = true;
    if (right - left <= 10 || cancelled_) {   // leaf_max_size (KDTreeVectorOfVectorsAdaptor.hpp:59)
        Node &n = nodes[me];
        n.leaf = true;
        n.left = left;
        n.right = right;
        n.child1 = n.child2 = -1;
        n.cutval = 0;
        if (right > left && kn.mask == all_dims(dim_)) {
            std::copy(kn.b, kn.b + dim_, bbox);
        } else {   // (an empty leaf reads the point at 'left', as the reference's loop)
            double mn[64], mx[64];
            rows_min_max(pts_, vind_.data() + left, right - left, dim_, mn, mx);   // row-major: a point's coordinates are contiguous
            for (int d = 0; d < dim_; d++) {
                bbox[d].low = mn[d];
                bbox[d].high = mx[d];
            }
        }
        std::copy(bbox, bbox + dim_, node_box_.begin() + (size_t)me * dim_);
        return me;
    }
    size_t idx;
    int cutfeat;
    double cutval;
    Node info;
    middle_split(vind_.data() + left, right - left, idx, cutfeat, cutval, bbox, kn, &info);
    // children's boxes (a vector per node cost two heap allocations each)
    Box *lb = level_boxes(level), *rb = lb + dim_;
    std::copy(bbox, bbox + dim_, lb);
    std::copy(bbox, bbox + dim_, rb);
    lb[cutfeat].high = cutval;
    rb[cutfeat].low = cutval;
    Known *kc = level_known(level);   // (level 0 holds the root's, and level >= 1 here)
    child_known(vind_.data() + left, idx, right - left, kn, kc[0], kc[1]);
    const int c1 = divide(left, left + idx, lb, kc[0], level + 1, nodes, depth);
    const int c2 = divide(left + idx, right, rb, kc[1], level + 1, nodes, depth);
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

void RefKDTree::near_set(const double *q, double slack_rel, double slack_abs, std::vector<uint32_t> &out,
                         double &dmin) const {
    static thread_local std::vector<std::pair<double, uint32_t>> seen;
    static thread_local std::vector<int> stack;
    seen.clear();
    stack.assign(1, 0);
    double best = std::numeric_limits<double>::infinity();
    // a box's squared distance is rounded a few ulps at most: the bound keeps a relative margin
    auto limit = [&] { return (best * (1 + slack_rel) + slack_abs) * (1 + 1e-12); };
    auto box_dist = [&](int node) {
        const Box *b = &node_box_[(size_t)node * dim_];
        double s = 0;
        for (int d = 0; d < dim_; d++) {
            const double x = q[d], e = x < b[d].low ? b[d].low - x : (x > b[d].high ? x - b[d].high : 0.0);
            s += e * e;
        }
        return s;
    };
    while (!stack.empty()) {
        const int node = stack.back();
        stack.pop_back();
        if (box_dist(node) > limit()) continue;
        const Node &n = nodes_[node];
        if (n.leaf) {
            for (size_t i = n.left; i < n.right; i++) {
                const uint32_t p = (uint32_t)vind_[i];
                const double cap = best * (1 + slack_rel) + slack_abs;   // beyond it: no candidate
                const double d = ref_l2_cap(q, pts_ + (size_t)p * dim_, dim_, cap);
                if (d > cap) continue;
                seen.emplace_back(d, p);
                best = std::min(best, d);
            }
            continue;
        }
        const double d1 = box_dist(n.child1), d2 = box_dist(n.child2);
        stack.push_back(d1 <= d2 ? n.child2 : n.child1);   // the closer child pops first
        stack.push_back(d1 <= d2 ? n.child1 : n.child2);
    }
    dmin = best;
    out.clear();
    const double lim = best * (1 + slack_rel) + slack_abs;
    for (const auto &s : seen)
        if (s.first <= lim) out.push_back(s.second);
}

// Blame (the collecting run): the points holding the least and greatest value in dimension d
// among node's points whose bits are not known, every one at that value (duplicated code
// vectors).  A large node finds them by descending to a leaf through the children whose
// aggregate holds the value (O(depth), not a scan).
void RefKDTree::blame_extremes(int node, int d) const {
    CertScratch &S = cert_scratch();
    for (int s = 0; s < 2; s++) {
        const size_t off = (size_t)s * dim_ + d;
        const double v = agg_[(size_t)node * dim_ * 4 + off];
        if (std::isinf(v)) continue;   // no unknown point
        int m = node;
        while (nodes_[m].right - nodes_[m].left > 256 && !nodes_[m].leaf) {
            const Node &n = nodes_[m];
            m = agg_[(size_t)n.child1 * dim_ * 4 + off] == v ? n.child1 : n.child2;
        }
        const Node &n = nodes_[m];
        for (size_t i = n.left; i < n.right; i++) {
            const size_t p = vind_[i];
            if (ptr(p, d) == v && !S.known[p * (size_t)dim_ + d]) S.blame->push_back((uint32_t)p);
        }
    }
}

// ... and with_cell those of the node's cell box's origin in d too (the root's box and every
// ancestor that cut along d).
void RefKDTree::blame_dim(int node, int d, bool with_cell) const {
    blame_extremes(node, d);
    if (!with_cell) return;
    for (int a = parent_[node]; a >= 0; a = parent_[a])
        if (nodes_[a].divfeat == d) blame_extremes(a, d);
    if (node != 0) blame_extremes(0, d);
}

// One node of the build replayed over every codebook within delta of this one (interval
// endpoints: each build quantity is a monotone function of the coordinates it reads, so the
// endpoints' values bound it).  True when the candidate dimensions, the cut dimension, the cut's
// clamp and every point's side of the cut are the same for all of them; then the children's
// cell boxes and divlow / divhigh get their intervals.  Collecting, an open decision blames the
// points it reads and the replay goes on with the exact split's decision.
bool RefKDTree::cert_split(int node) const {
    CertScratch &S = cert_scratch();
    const Node &n = nodes_[node];
    CertNode &cn = cnode_[node];
    const bool collect = S.blame != nullptr;
    const int D = dim_;
    const Iv *cb = &cbox_[(size_t)node * D * 2];
    const size_t *ind = vind_.data() + n.left;
    const size_t count = n.right - n.left;
    const double EPS = 0.00001;
    double sp_lo[64], sp_hi[64], ms_lo = 0, ms_hi = 0;
    for (int d = 0; d < D; d++) {
        sp_lo[d] = cb[2 * d + 1].lo - cb[2 * d].hi;
        sp_hi[d] = cb[2 * d + 1].hi - cb[2 * d].lo;
        ms_lo = d ? std::max(ms_lo, sp_lo[d]) : sp_lo[d];
        ms_hi = d ? std::max(ms_hi, sp_hi[d]) : sp_hi[d];
    }
    const double th_lo = (1 - EPS) * ms_lo, th_hi = (1 - EPS) * ms_hi;
    uint64_t cand = 0;
    for (int d = 0; d < D; d++) {
        if (sp_lo[d] > th_hi) {
            cand |= 1ull << d;
        } else if (!(sp_hi[d] <= th_lo)) {   // open: the dimension's span and the widest's
            if (!collect) return false;
            blame_dim(node, d, true);
            for (int e = 0; e < D; e++)
                if (sp_hi[e] >= ms_lo) blame_dim(node, e, true);
        }
    }
    if (!collect && cand != n.cand) return false;
    cand = n.cand;
    const int c = n.divfeat;
    const Iv mn = iv_min(node, c), mx = iv_max(node, c);
    if (cand) {   // the first candidate of greatest spread, strictly ahead of the others
        const double sc_lo = mx.lo - mn.hi;
        for (int j = 0; j < D; j++) {
            if (j == c || !((cand >> j) & 1)) continue;
            const double sj_hi = iv_max(node, j).hi - iv_min(node, j).lo;
            if (j < c ? !(sj_hi < sc_lo) : !(sj_hi <= sc_lo)) {
                if (!collect) return false;
                blame_dim(node, j, false);
                blame_dim(node, c, false);
            }
        }
    } else if (c != 0) {
        return false;
    }
    // the exact split's children: their exact boxes along c tell whether a point sits on the cut
    const Node &c1 = nodes_[n.child1], &c2 = nodes_[n.child2];
    const double e1 = node_box_[(size_t)n.child1 * D + c].high, e2 = node_box_[(size_t)n.child2 * D + c].low;
    const Iv sv{(cb[2 * c].lo + cb[2 * c + 1].lo) / 2, (cb[2 * c].hi + cb[2 * c + 1].hi) / 2};
    Iv cut;
    if (n.cutval == n.split_val) {   // not clamped, for all; no point meets the cut unless both are exact
        if (!(sv.lo >= mn.hi && sv.hi <= mx.lo)) {
            if (!collect) return false;
            blame_dim(node, c, true);
        }
        cut = sv;
        bool blamed = false;
        // no point on the cut: each child strictly on its side (O(1)); else point by point
        const bool plain = e1 < n.cutval && e2 > n.cutval;
        if (plain && iv_max(n.child1, c).hi < cut.lo && iv_min(n.child2, c).lo > cut.hi) {
        } else for (size_t i = 0; i < count; i++) {   // and on the exact split's side of it
            const double e = ptr(ind[i], c);
            const int side_e = e < n.cutval ? 0 : (e == n.cutval ? 1 : 2);
            const Iv v = piv(ind[i], c);
            int side;
            if (v.hi < cut.lo) side = 0;
            else if (v.lo > cut.hi) side = 2;
            else if (v.lo == v.hi && cut.lo == cut.hi && v.lo == cut.lo) side = 1;
            else side = -1;
            if (side != side_e) {
                if (!collect) return false;
                if (!S.known[ind[i] * (size_t)D + c]) S.blame->push_back((uint32_t)ind[i]);
                if (!blamed) blame_dim(node, c, true);
                blamed = true;
            }
        }
    } else {   // clamped to the points' minimum (maximum): the points at it stay the extreme ones
        const bool low = n.cutval > n.split_val;
        if (low ? !(sv.hi < mn.lo) : !(sv.lo > mx.hi)) {
            if (!collect) return false;
            blame_dim(node, c, true);
        }
        cut = low ? mn : mx;
        // the usual shape: one child is exactly the points at the clamp value (O(1) then)
        const int at_child = low ? n.child1 : n.child2, rest = low ? n.child2 : n.child1;
        const bool shaped = low ? (e1 == n.cutval && e2 > n.cutval) : (e2 == n.cutval && e1 < n.cutval);
        bool quick = false;
        if (shaped) {
            const Iv am = iv_min(at_child, c), ax = iv_max(at_child, c);
            const bool one = nodes_[at_child].right - nodes_[at_child].left == 1;
            const bool ex = am.lo == ax.hi;   // all known, one value
            if (ex || one) {
                const double lim = ex ? am.lo : (low ? ax.hi : am.lo);
                quick = low ? iv_min(rest, c).lo > lim : iv_max(rest, c).hi < lim;
            }
        }
        size_t nat = 0;
        bool exact = true;   // every one of them known, all at one value
        Iv at{0, 0};
        for (size_t i = 0; i < count; i++)
            if (ptr(ind[i], c) == n.cutval) {
                const Iv v = piv(ind[i], c);
                exact = exact && v.lo == v.hi && (nat == 0 || v.lo == at.lo);
                at = v;
                nat++;
            }
        bool open = !quick && !exact && nat != 1;
        const double lim = exact ? at.lo : (low ? at.hi : at.lo);
        for (size_t i = 0; i < count && !open && !quick; i++) {
            if (ptr(ind[i], c) == n.cutval) continue;
            const Iv v = piv(ind[i], c);
            open = low ? !(v.lo > lim) : !(v.hi < lim);
        }
        if (open) {
            if (!collect) return false;
            blame_dim(node, c, false);
            for (size_t i = 0; i < count; i++) {   // and every point that may reach the extreme
                const Iv v = piv(ind[i], c);
                if ((low ? v.lo <= cut.hi : v.hi >= cut.lo) && !S.known[ind[i] * (size_t)D + c])
                    S.blame->push_back((uint32_t)ind[i]);
            }
        }
    }
    Iv *lb = &cbox_[(size_t)n.child1 * D * 2], *rb = &cbox_[(size_t)n.child2 * D * 2];
    std::copy(cb, cb + 2 * D, lb);
    std::copy(cb, cb + 2 * D, rb);
    lb[2 * c + 1] = cut;
    rb[2 * c] = cut;
    cn.dl = iv_max(n.child1, c);
    cn.dh = iv_min(n.child2, c);
    (void)c1;
    (void)c2;
    return true;
}

RefKDTree::CertScratch &RefKDTree::cert_scratch() {
    static thread_local CertScratch s;
    return s;
}

void RefKDTree::cert_ensure_agg(uint64_t gen, const double *kpts, const uint8_t *known) const {
    if (agg_gen_.load(std::memory_order_acquire) == gen && agg_k_ == kpts && agg_known_ == known) return;
    std::lock_guard<std::mutex> g(agg_mu_);
    if (agg_gen_.load(std::memory_order_acquire) == gen && agg_k_ == kpts && agg_known_ == known) return;
    agg_prepare(kpts, known);
    // per node and dimension: min / max over its points whose bits are not known (exact-sum
    // values) and over those known (the reference's values), children before parents
    for (size_t i = nodes_.size(); i-- > 0;) cert_agg_node(i);
    agg_gen_.store(gen, std::memory_order_release);
}

// (under agg_mu_) the parent / leaf maps and the aggregates' storage for (kpts, known)
void RefKDTree::agg_prepare(const double *kpts, const uint8_t *known) const {
    const size_t nn = nodes_.size();
    if (parent_.size() != nn) {
        parent_.assign(nn, -1);
        leaf_of_.resize(K_);
        for (size_t i = 0; i < nn; i++) {
            const Node &n = nodes_[i];
            if (!n.leaf) parent_[n.child1] = parent_[n.child2] = (int)i;
            else
                for (size_t j = n.left; j < n.right; j++) leaf_of_[vind_[j]] = (int)i;
        }
    }
    agg_k_ = kpts;
    agg_known_ = known;
    agg_.resize(nn * dim_ * 4);
}

void RefKDTree::cert_reset(double delta, const double *kpts, const uint8_t *known) const {
    CertScratch &S = cert_scratch();
    const bool collect = S.blame != nullptr;
    const uint64_t gen = cert_gen_.load(std::memory_order_acquire);
    cert_ensure_agg(gen, kpts, known);
    S.owner = id_;
    S.gen = gen;
    S.k = kpts;
    S.known = known;
    S.collect = collect;
    S.delta = delta;
    // the shared node states for this key: reset by the first thread that brings a new key
    // (the replays of one key start after it; a phase's threads share its key)
    if (ckey_gen_.load(std::memory_order_acquire) == gen && ckey_delta_ == delta && ckey_k_ == kpts &&
        ckey_known_ == known && ckey_collect_ == collect)
        return;
    std::lock_guard<std::mutex> g(agg_mu_);
    if (ckey_gen_.load(std::memory_order_acquire) == gen && ckey_delta_ == delta && ckey_k_ == kpts &&
        ckey_known_ == known && ckey_collect_ == collect)
        return;
    const int D = dim_;
    const size_t nn = nodes_.size();
    if (!cstate_ || cnode_.size() != nn) {
        cstate_.reset(new std::atomic<int8_t>[nn]);
        cnode_.assign(nn, CertNode());
        cbox_.resize(nn * D * 2);
    }
    for (size_t i = 0; i < nn; i++) cstate_[i].store(0, std::memory_order_relaxed);
    for (int d = 0; d < D; d++) {   // the root's cell box: the points' box
        cbox_[2 * d] = iv_min(0, d);
        cbox_[2 * d + 1] = iv_max(0, d);
    }
    ckey_delta_ = delta;
    ckey_k_ = kpts;
    ckey_known_ = known;
    ckey_collect_ = collect;
    ckey_gen_.store(gen, std::memory_order_release);
}

// One node's aggregates (children's first): min / max over the unknown points and over the known
// points, stored [min unknown | max unknown | min known | max known][dim] so that the loops
// below are plain element-wise min / max (vectorised; a branch per value mispredicted on the
// irregular known pattern).
namespace {
// One leaf point's row into a node's aggregates, four dimensions at a time (blends on the
// known mask, then min / max; the values are finite, so min_pd / max_pd are exact): returns the
// first dimension left to the scalar loop.
__attribute__((target("avx2"))) int agg_row_avx2(const double *x, const double *kv, const uint8_t *k, int D,
                                                 double *mnu, double *mxu, double *mnk, double *mxk) {
    const __m256d inf = _mm256_set1_pd(std::numeric_limits<double>::infinity()), ninf = _mm256_sub_pd(_mm256_setzero_pd(), inf);
    int d = 0;
    for (; d + 4 <= D; d += 4) {
        int32_t kb;
        std::memcpy(&kb, k + d, 4);
        const __m256i k64 = _mm256_cvtepu8_epi64(_mm_cvtsi32_si128(kb));
        const __m256d m = _mm256_castsi256_pd(_mm256_cmpgt_epi64(k64, _mm256_setzero_si256()));   // known
        const __m256d xv = _mm256_loadu_pd(x + d), kk = _mm256_loadu_pd(kv + d);
        _mm256_storeu_pd(mnu + d, _mm256_min_pd(_mm256_loadu_pd(mnu + d), _mm256_blendv_pd(xv, inf, m)));
        _mm256_storeu_pd(mxu + d, _mm256_max_pd(_mm256_loadu_pd(mxu + d), _mm256_blendv_pd(xv, ninf, m)));
        _mm256_storeu_pd(mnk + d, _mm256_min_pd(_mm256_loadu_pd(mnk + d), _mm256_blendv_pd(inf, kk, m)));
        _mm256_storeu_pd(mxk + d, _mm256_max_pd(_mm256_loadu_pd(mxk + d), _mm256_blendv_pd(ninf, kk, m)));
    }
    return d;
}
// A whole leaf into its aggregates, four dimensions at a time with the four running values in
// registers over the leaf's points (one store per dimension block, no read-modify-write chain
// through memory per point): returns the first dimension left to the scalar loop.
__attribute__((target("avx2"))) int agg_leaf_avx2(const double *pts, const double *kpts, const uint8_t *known,
                                                  const size_t *ind, size_t n, int D, int d0, int d1, double *mnu,
                                                  double *mxu, double *mnk, double *mxk) {
    const __m256d inf = _mm256_set1_pd(std::numeric_limits<double>::infinity()), ninf = _mm256_sub_pd(_mm256_setzero_pd(), inf);
    for (size_t j = 0; j < n; j++) {   // every row of the leaf requested first (rows are scattered)
        const size_t r = ind[j] * (size_t)D;
        for (int o = d0; o < d1; o += 8) {
            _mm_prefetch((const char *)(pts + r + o), _MM_HINT_T0);
            _mm_prefetch((const char *)(kpts + r + o), _MM_HINT_T0);
        }
        _mm_prefetch((const char *)(known + r + d0), _MM_HINT_T0);
    }
    int d = d0;
    for (; d + 4 <= d1; d += 4) {
        __m256d a = inf, b = ninf, c = inf, e = ninf;
        for (size_t j = 0; j < n; j++) {
            const size_t r = ind[j] * (size_t)D + d;
            int32_t kb;
            std::memcpy(&kb, known + r, 4);
            const __m256d m = _mm256_castsi256_pd(
                _mm256_cmpgt_epi64(_mm256_cvtepu8_epi64(_mm_cvtsi32_si128(kb)), _mm256_setzero_si256()));
            const __m256d xv = _mm256_loadu_pd(pts + r), kk = _mm256_loadu_pd(kpts + r);
            a = _mm256_min_pd(a, _mm256_blendv_pd(xv, inf, m));
            b = _mm256_max_pd(b, _mm256_blendv_pd(xv, ninf, m));
            c = _mm256_min_pd(c, _mm256_blendv_pd(inf, kk, m));
            e = _mm256_max_pd(e, _mm256_blendv_pd(ninf, kk, m));
        }
        _mm256_storeu_pd(mnu + d, a);
        _mm256_storeu_pd(mxu + d, b);
        _mm256_storeu_pd(mnk + d, c);
        _mm256_storeu_pd(mxk + d, e);
    }
    return d;
}
// An inner node's aggregates from its children's (element-wise min / max of the two rows).
__attribute__((target("avx2"))) void agg_inner_avx2(const double *b, const double *c, double *o, int D, int d0,
                                                    int d1) {
    for (int q = 0; q < 4; q++) {
        const double *bq = b + q * D, *cq = c + q * D;
        double *oq = o + q * D;
        int d = d0;
        for (; d + 4 <= d1; d += 4) {
            const __m256d u = _mm256_loadu_pd(bq + d), v = _mm256_loadu_pd(cq + d);
            _mm256_storeu_pd(oq + d, (q & 1) ? _mm256_max_pd(v, u) : _mm256_min_pd(v, u));
        }
        for (; d < d1; d++) oq[d] = (q & 1) ? (cq[d] > bq[d] ? cq[d] : bq[d]) : (cq[d] < bq[d] ? cq[d] : bq[d]);
    }
}
}  // namespace

void RefKDTree::cert_agg_node(size_t i) const { cert_agg_dims(i, 0, dim_); }

// cert_agg_node over dimensions [d0, d1) only (the parallel warm-up splits the dimensions).
void RefKDTree::cert_agg_dims(size_t i, int d0, int d1) const {
    constexpr double INF = std::numeric_limits<double>::infinity();
    const int D = dim_;
    double *__restrict mnu = &agg_[i * D * 4], *__restrict mxu = mnu + D, *__restrict mnk = mxu + D,
                       *__restrict mxk = mnk + D;
    const Node &n = nodes_[i];
    const bool avx2 = has_avx2();
    if (n.leaf && avx2) {
        const int e = agg_leaf_avx2(pts_, agg_k_, agg_known_, vind_.data() + n.left, n.right - n.left, D, d0, d1, mnu,
                                    mxu, mnk, mxk);
        for (int d = e; d < d1; d++) {
            mnu[d] = mnk[d] = INF, mxu[d] = mxk[d] = -INF;
            for (size_t j = n.left; j < n.right; j++) {
                const size_t r = vind_[j] * (size_t)D + d;
                const bool kk = agg_known_[r] != 0;
                const double x = pts_[r], kv = agg_k_[r];
                const double xu_lo = kk ? INF : x, xu_hi = kk ? -INF : x, xk_lo = kk ? kv : INF, xk_hi = kk ? kv : -INF;
                mnu[d] = mnu[d] < xu_lo ? mnu[d] : xu_lo;
                mxu[d] = mxu[d] > xu_hi ? mxu[d] : xu_hi;
                mnk[d] = mnk[d] < xk_lo ? mnk[d] : xk_lo;
                mxk[d] = mxk[d] > xk_hi ? mxk[d] : xk_hi;
            }
        }
        return;
    }
    if (n.leaf) {
        for (int d = d0; d < d1; d++) mnu[d] = mnk[d] = INF, mxu[d] = mxk[d] = -INF;
        for (size_t j = n.left; j < n.right; j++) {
            const size_t r = vind_[j] * (size_t)D + d0;
            const double *__restrict x = pts_ + r, *__restrict kv = agg_k_ + r;
            const uint8_t *__restrict k = agg_known_ + r;
            const int w = d1 - d0;
            int e = 0;
            if (has_avx2()) e = agg_row_avx2(x, kv, k, w, mnu + d0, mxu + d0, mnk + d0, mxk + d0);
            // (the compiler keeps this loop scalar: its selects on a loaded byte are control flow)
            for (; e < w; e++) {
                const int d = d0 + e;
                const bool kk = k[e] != 0;
                const double xu_lo = kk ? INF : x[e], xu_hi = kk ? -INF : x[e];
                const double xk_lo = kk ? kv[e] : INF, xk_hi = kk ? kv[e] : -INF;
                mnu[d] = xu_lo < mnu[d] ? xu_lo : mnu[d];
                mxu[d] = xu_hi > mxu[d] ? xu_hi : mxu[d];
                mnk[d] = xk_lo < mnk[d] ? xk_lo : mnk[d];
                mxk[d] = xk_hi > mxk[d] ? xk_hi : mxk[d];
            }
        }
        return;
    }
    const double *__restrict b = &agg_[(size_t)n.child1 * D * 4], *__restrict c = &agg_[(size_t)n.child2 * D * 4];
    if (avx2) {
        agg_inner_avx2(b, c, mnu, D, d0, d1);
        return;
    }
    for (int q = 0; q < 4; q++)   // [min unknown | max unknown | min known | max known]
        for (int d = d0; d < d1; d++) {
            const double u = b[q * D + d], v = c[q * D + d];
            mnu[q * D + d] = (q & 1) ? (v > u ? v : u) : (v < u ? v : u);
        }
}

// The least (greatest) value of dimension d over node's points, over every allowed codebook.
RefKDTree::Iv RefKDTree::iv_min(int node, int d) const {
    CertScratch &S = cert_scratch();
    const double *a = &agg_[(size_t)node * dim_ * 4 + d];
    return {std::min(a[0] - S.delta, a[2 * dim_]), std::min(a[0] + S.delta, a[2 * dim_])};
}
RefKDTree::Iv RefKDTree::iv_max(int node, int d) const {
    CertScratch &S = cert_scratch();
    const double *a = &agg_[(size_t)node * dim_ * 4 + d];
    return {std::max(a[dim_] - S.delta, a[3 * dim_]), std::max(a[dim_] + S.delta, a[3 * dim_])};
}

namespace {
// x * x over x in [e.lo, e.hi] (a product of a value with itself rounds monotonically in |x|)
inline void sq_iv(double elo, double ehi, double &lo, double &hi) {
    if (elo >= 0) lo = elo * elo, hi = ehi * ehi;
    else if (ehi <= 0) lo = ehi * ehi, hi = elo * elo;
    else lo = 0, hi = std::max(elo * elo, ehi * ehi);
}
}  // namespace

void RefKDTree::certify_blame(const double *q, double delta, const double *kpts, const uint8_t *known,
                              std::vector<uint32_t> &blame) const {
    CertScratch &S = cert_scratch();
    // the collecting replay keeps a cache of its own (a node it replayed has blamed already)
    S.blame = &blame;
    certified_search(q, delta, kpts, known);
    S.blame = nullptr;
}

void RefKDTree::cert_clear() const { cert_gen_.fetch_add(1, std::memory_order_acq_rel); }

void RefKDTree::cert_warm(double delta, const double *kpts, const uint8_t *known, unsigned nthr,
                          const std::function<void(unsigned, const std::function<void(unsigned)> &)> &run) const {
    if (dim_ > 64 || nodes_.empty()) return;
    {   // the aggregates, the dimensions split over nthr threads (memory-bound: ~4.6 MB at
        // K = 4096, D = 48; whole 64-byte lines per thread and node)
        const uint64_t gen = cert_gen_.load(std::memory_order_acquire);
        std::lock_guard<std::mutex> g(agg_mu_);
        if (!(agg_gen_.load(std::memory_order_acquire) == gen && agg_k_ == kpts && agg_known_ == known)) {
            agg_prepare(kpts, known);
            const size_t nn = nodes_.size();
            const int D = dim_;
            const unsigned nt = run && nthr > 1 ? std::min<unsigned>(nthr, (unsigned)(D + 7) / 8) : 1;
            auto part = [&](unsigned t) {
                const int d0 = (int)((D * (uint64_t)t / nt) & ~7ull), d1 = t + 1 == nt ? D : (int)((D * (uint64_t)(t + 1) / nt) & ~7ull);
                for (size_t i = nn; i-- > 0;) cert_agg_dims(i, d0, d1);
            };
            if (nt > 1) run(nt, part);
            else part(0);
            agg_gen_.store(gen, std::memory_order_release);
        }
    }
    CertScratch &S = cert_scratch();
    std::vector<uint32_t> *keep = S.blame;
    S.blame = nullptr;   // the strict replay's key (the node states reset, the root's box)
    cert_reset(delta, kpts, known);
    S.blame = keep;
}

void RefKDTree::cert_prepare(double delta, const double *kpts, const uint8_t *known) const {
    if (dim_ > 64 || nodes_.empty()) return;
    CertScratch &S = cert_scratch();
    std::vector<uint32_t> *keep = S.blame;
    S.blame = nullptr;   // the strict replay's key
    cert_reset(delta, kpts, known);
    // parents before children (a node's cell box is its parent's split), with the node states'
    // protocol of certified_search (0 -> 3 -> 1 / 2)
    std::vector<int> stack = {0};
    while (!stack.empty()) {
        const int node = stack.back();
        stack.pop_back();
        const Node &n = nodes_[node];
        if (n.leaf) continue;
        int8_t st = cstate_[node].load(std::memory_order_acquire);
        if (st == 0) {
            int8_t z = 0;
            if (cstate_[node].compare_exchange_strong(z, 3, std::memory_order_acq_rel)) {
                st = cert_split(node) ? 1 : 2;
                cstate_[node].store(st, std::memory_order_release);
            } else {
                st = z;
            }
        }
        while (st == 3) {
            std::this_thread::yield();
            st = cstate_[node].load(std::memory_order_acquire);
        }
        if (st == 1) {
            stack.push_back(n.child1);
            stack.push_back(n.child2);
        }
    }
    S.blame = keep;
}

void RefKDTree::cert_update(const uint32_t *pts, size_t n) const {
    std::lock_guard<std::mutex> g(agg_mu_);
    const uint64_t gen = cert_gen_.fetch_add(1, std::memory_order_acq_rel) + 1;   // the node states: all anew
    if (agg_gen_.load(std::memory_order_acquire) + 1 != gen || parent_.size() != nodes_.size())
        return;   // the next replay recomputes every aggregate
    const size_t nn = nodes_.size();
    std::vector<uint8_t> dirty(nn, 0);
    for (size_t i = 0; i < n; i++)
        for (int a = leaf_of_[pts[i]]; a >= 0 && !dirty[a]; a = parent_[a]) dirty[a] = 1;
    for (size_t i = nn; i-- > 0;)   // children before parents
        if (dirty[i]) cert_agg_node(i);
    agg_gen_.store(gen, std::memory_order_release);
}

// kd_nearest_flat (the reference's search) replayed over every codebook the certificate allows:
// each quantity an interval, each decision taken only when all of them take it (collecting:
// an open decision blames the points it reads and the exact split's decision is taken).
int64_t RefKDTree::certified_search(const double *q, double delta, const double *kpts, const uint8_t *known) const {
    CertScratch &S = cert_scratch();
    if (dim_ > 64) return -1;
    const bool collect = S.blame != nullptr;
    cert_reset(delta, kpts, known);
    const int D = dim_;
    constexpr double U = 1.1102230246251565e-16;   // unit roundoff
    double dlo[64], dhi[64];
    double mlo = 0, mhi = 0;
    for (int d = 0; d < D; d++) {   // the initial distances against the root box
        const double x = q[d];
        const Iv lo = cbox_[2 * d], hi = cbox_[2 * d + 1];
        dlo[d] = dhi[d] = 0;
        if ((!(x < lo.lo) && x < lo.hi) || (!(x > hi.hi) && x > hi.lo)) {
            if (!collect) return -1;
            blame_extremes(0, d);
        }
        if (x < lo.lo) {
            sq_iv(x - lo.hi, x - lo.lo, dlo[d], dhi[d]);
            mlo += dlo[d];
            mhi += dhi[d];
        }
        if (x > hi.hi) {
            sq_iv(x - hi.hi, x - hi.lo, dlo[d], dhi[d]);
            mlo += dlo[d];
            mhi += dhi[d];
        }
    }
    const double MAXD = 1.7976931348623157e308;
    double blo = MAXD, bhi = MAXD;   // the best distance so far
    int64_t idx = 0;
    bool amb = false, ok = true;
    std::vector<int> path;
    // sum_d 2 |q_d - c_d| delta + delta^2 over the coordinates, at most (Cauchy-Schwarz, with
    // sum_d (q_d - c_d)^2 <= de (1 + D u)), and both evaluations' rounding; de - pert(de) grows
    // with de
    auto pert = [&](double de) {
        const double lin = 2 * delta * std::sqrt(D * de * (1 + (D + 4) * U)) + D * delta * delta;
        return (lin + (D + 4) * U * (2 * de + lin)) * (1 + 1e-9) + 1e-300;
    };
    // a point's distance: exact when all its coordinates are known, else around the exact-sum
    // split's; a prefix past the best so far (bhi) settles a rejection early
    auto pdist = [&](uint32_t p, double bound, double &lo, double &hi) {
        const size_t r = (size_t)p * D;
        bool all = true;
        for (int d = 0; d < D; d++) all = all && known[r + d];
        if (all) {
            lo = hi = ref_l2_cap(q, kpts + r, D, bound);
            return;
        }
        double de = ref_l2_cap(q, pts_ + r, D, bound);
        if (de > bound && !(de - pert(de) >= bound)) de = ref_l2(q, pts_ + r, D);
        lo = de - pert(de);
        hi = de + pert(de);
    };
    auto blame_pt = [&](uint32_t p) {
        for (int d = 0; d < D; d++)
            if (!known[(size_t)p * D + d]) {
                S.blame->push_back(p);
                return;
            }
    };
    auto search = [&](auto &&self, int node, double slo, double shi) -> void {
        if (!ok) return;
        const Node &n = nodes_[node];
        if (n.leaf) {
            const double wlo = blo, whi = bhi;   // the leaf's worst, captured at entry
            for (size_t i = n.left; i < n.right; i++) {
                const uint32_t p = (uint32_t)vind_[i];
                double lo, hi;
                pdist(p, bhi, lo, hi);
                // kept iff dist < worst and best > dist: with best <= worst, iff dist < best
                const bool yes = hi < wlo && hi < blo, no = lo >= whi || lo >= bhi;
                if (yes) {
                    blo = lo, bhi = hi, idx = p, amb = false;
                } else if (!no) {
                    if (collect) {
                        blame_pt(p);
                        blame_pt((uint32_t)idx);
                    }
                    blo = std::min(blo, lo), bhi = std::min(bhi, hi), amb = true;
                }
            }
            return;
        }
        int8_t st = cstate_[node].load(std::memory_order_acquire);
        if (st == 0) {   // replayed once, by whichever thread gets here first
            int8_t z = 0;
            if (cstate_[node].compare_exchange_strong(z, 3, std::memory_order_acq_rel)) {
                st = cert_split(node) ? 1 : 2;
                cstate_[node].store(st, std::memory_order_release);
            } else {
                st = z;
            }
        }
        while (st == 3) {
            std::this_thread::yield();
            st = cstate_[node].load(std::memory_order_acquire);
        }
        if (st != 1) {
            ok = false;
            return;
        }
        const int f = n.divfeat;
        const double val = q[f];
        const CertNode &cn = cnode_[node];
        const double s_hi = (val - cn.dl.lo) + (val - cn.dh.lo), s_lo = (val - cn.dl.hi) + (val - cn.dh.hi);
        bool left_first = s_hi < 0;
        if (!(s_hi < 0) && !(s_lo >= 0)) {
            if (!collect) {
                ok = false;
                return;
            }
            blame_extremes(n.child1, f);
            blame_extremes(n.child2, f);
            left_first = (val - n.divlow) + (val - n.divhigh) < 0;
        }
        path.push_back(node);
        self(self, left_first ? n.child1 : n.child2, slo, shi);
        path.pop_back();
        if (!ok) return;
        double clo, chi;
        if (left_first) sq_iv(val - cn.dh.hi, val - cn.dh.lo, clo, chi);
        else sq_iv(val - cn.dl.hi, val - cn.dl.lo, clo, chi);
        const double tlo = dlo[f], thi = dhi[f];
        const double m2lo = (slo - thi) + clo, m2hi = (shi - tlo) + chi;
        dlo[f] = clo;
        dhi[f] = chi;
        bool visit = m2hi <= blo;
        if (!visit && !(m2lo > bhi)) {
            if (!collect) {
                ok = false;
                return;
            }
            blame_pt((uint32_t)idx);
            for (int a : path) {
                blame_extremes(nodes_[a].child1, nodes_[a].divfeat);
                blame_extremes(nodes_[a].child2, nodes_[a].divfeat);
            }
            blame_extremes(n.child1, f);
            blame_extremes(n.child2, f);
            visit = true;
        }
        if (visit) {
            path.push_back(node);
            self(self, left_first ? n.child2 : n.child1, m2lo, m2hi);
            path.pop_back();
        }
        dlo[f] = tlo;
        dhi[f] = thi;
    };
    search(search, 0, mlo, mhi);
    return ok && !amb && blo < MAXD ? idx : -1;
}

int64_t certify_tie(const RefKDTree &t, const double *q, const std::vector<uint32_t> &cand, const double *kpts,
                    const uint8_t *known, int dim, double delta) {
    if (cand.empty()) return -1;
    for (uint32_t j : cand)
        for (int d = 0; d < dim; d++)
            if (!known[(size_t)j * dim + d]) return -1;
    return t.certified_search(q, delta, kpts, known);
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
