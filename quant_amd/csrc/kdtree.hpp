// Host-side exact nearest-neighbour resolver with nanoflann 1.2.3 semantics.
//
// The device assigns every block by brute force.  A handful of rows per level have two
// code vectors at (nearly) the same fp64 distance; for those the reference's answer is
// whatever its kd-tree search visits first (src/KDTree.cpp:20-29 over
// include/external/nanoflann.hpp).  This class rebuilds that tree over the level's
// codebook and answers exactly those rows.  It is part of the product (not the oracle):
// the C-ABI engine builds it per level while the GPU searches, and either uploads it for
// the device traversal (k_assign.hip, kd_nearest_dev) or answers handed-back rows here.
#pragma once
#include <atomic>
#include <cstddef>
#include <memory>
#include <mutex>
#include <cstdint>
#include <cstring>
#include <functional>
#include <string>
#include <vector>

#include "kdtree_dev.hpp"

namespace qvq {

// Squared L2 in the reference build's order (kdtree_dev.hpp, ref_l2_hd).
double ref_l2(const double *a, const double *b, int dim);

struct Box { double low, high; };

// A per-tree buffer of a trivial type, uninitialised, whose storage returns to a small process
// pool when the tree dies: a level's tree lives one level, and a fresh multi-MB buffer page-
// faults on its first touch and is unmapped again on free (at K = 4096, D = 48 the certificate's
// aggregates and cell boxes cost more in faults, zero-fill and unmap than in the work on them).
template <class T>
class Recycled {
public:
    Recycled() = default;
    Recycled(const Recycled &) = delete;
    Recycled &operator=(const Recycled &) = delete;
    ~Recycled() { release(); }
    void resize(size_t n);   // contents undefined; data() 64-byte aligned
    void swap(Recycled &o) {
        std::swap(p_, o.p_);
        std::swap(base_, o.base_);
        std::swap(cap_, o.cap_);
        std::swap(n_, o.n_);
    }
    size_t size() const { return n_; }
    T *data() { return base_; }
    const T *data() const { return base_; }
    T &operator[](size_t i) { return base_[i]; }
    const T &operator[](size_t i) const { return base_[i]; }

private:
    void release();
    void align();
    std::unique_ptr<T[]> p_;
    T *base_ = nullptr;
    size_t cap_ = 0, n_ = 0;
};

// A growable array of a trivially copyable type on Recycled storage: a level's tree allocates
// its node records and boxes (MBs at K = 4096, D = 48) from the pool instead of fresh pages
// (first-touch faults cost ~0.45 ms of the 1.5 ms K = 4096 build on the GPU box's host).
template <class T>
class RecycledVec {
public:
    void reserve(size_t n) {
        if (n > buf_.size()) grow(n);
    }
    void resize(size_t n) {
        reserve(n);
        n_ = n;
    }
    void push_back(const T &v) {
        if (n_ == buf_.size()) grow(n_ < 16 ? 16 : 2 * n_);
        buf_[n_++] = v;
    }
    size_t size() const { return n_; }
    bool empty() const { return n_ == 0; }
    T *begin() { return buf_.data(); }
    const T *begin() const { return buf_.data(); }
    T *data() { return buf_.data(); }
    const T *data() const { return buf_.data(); }
    T &operator[](size_t i) { return buf_[i]; }
    const T &operator[](size_t i) const { return buf_[i]; }

private:
    void grow(size_t cap) {
        Recycled<T> nb;
        nb.resize(cap);
        if (n_) std::memcpy(static_cast<void *>(nb.data()), buf_.data(), n_ * sizeof(T));
        buf_.swap(nb);
    }
    Recycled<T> buf_;
    size_t n_ = 0;
};

class RefKDTree {
public:
    // pts: K x dim, row-major, borrowed for the lifetime of the tree.  cancel (optional): the
    // build stops early once it reads true, leaving a tree to be discarded (cancelled()).
    RefKDTree(const double *pts, size_t K, int dim, const std::atomic<bool> *cancel = nullptr);
    // The tree the device built over pts (k_kdbuild.hip; image in kdb_host_layout): its nodes
    // renumbered depth first, child 1 first, as this class builds them; the same tree.
    RefKDTree(const double *pts, size_t K, int dim, const uint8_t *device_image);
    bool cancelled() const { return cancelled_; }
    // Node for node the same tree as o (structure, vind, cut dimensions and values, divlow /
    // divhigh, the build's split records, point boxes, root box, depth); why: the first difference.
    bool same_as(const RefKDTree &o, std::string *why = nullptr) const;
    // This tree as the device build writes it (kdb_host_layout: nodes numbered breadth first, the
    // two children of a node consecutive), for the import's CPU tests.  img: kdb_host_layout(K,
    // dim).total bytes.
    void to_device_image(uint8_t *img) const;
    // Index the reference's kd-tree search returns for query q (dim values).
    uint32_t nearest(const double *q) const;
    // Flattened copy for the device search (kdtree_dev.hpp); depth = longest root-to-leaf
    // path in nodes (the search's stack depth).
    size_t num_nodes() const { return nodes_.size(); }
    int depth() const { return depth_; }
    void flatten(KdNodeDev *nodes, uint32_t *vind, double *lo, double *hi) const;
    // True when the tree the reference would build over pts2 (K x dim, the same shape; e.g. the
    // Kahan-bit codebook next to the exact-sum one) is this tree bit for bit: structure, cut
    // values, boxes (a sufficient test, per differing coordinate along its point's path: the
    // root box, the cut choices, cut values, partitions and children's boxes it can reach stay).
    bool unchanged_under(const double *pts2) const;

    // ---- the reference's answer without the reference's whole split ----------
    // This tree is built over the exact-sum split; the reference's (Kahan-bit) split differs
    // from it by at most delta per coordinate.
    // Every point whose ref_l2 distance to q is at most dmin (1 + slack_rel) + slack_abs, dmin
    // the least distance; the points' own box per node prunes the walk.
    void near_set(const double *q, double slack_rel, double slack_abs, std::vector<uint32_t> &out,
                  double &dmin) const;
    // The index the reference's search over its own (Kahan-bit) split returns for q, from this
    // tree: the search replayed over every split within delta of this one that equals kpts on
    // the coordinates known marks (K x dim bytes), each build and search quantity an interval
    // (each is a monotone function of what it reads), each decision taken only when all of them
    // take it; the build's decisions per node are cached for one (delta, kpts, known).  -1 when
    // a decision is not the same for all: the caller then computes the reference's split and
    // its tree.
    int64_t certified_search(const double *q, double delta, const double *kpts, const uint8_t *known) const;
    // The same replay collecting instead of deciding: every point whose reference bits would
    // settle a decision the intervals leave open is appended to blame (then the exact split's
    // decision is taken), so that one round of Kahan sums can make the strict replay succeed.
    void certify_blame(const double *q, double delta, const double *kpts, const uint8_t *known,
                       std::vector<uint32_t> &blame) const;
    // Forget the replays' caches, on every thread (kpts or known changed in place).
    void cert_clear() const;
    // The replays' shared state for (delta, kpts, known) built ahead of any query: the per-node
    // aggregates and every node's replayed split, top down (a later certified_search with the
    // same key then only walks).  The caller keeps kpts / known unchanged until its replays.
    void cert_prepare(double delta, const double *kpts, const uint8_t *known) const;
    // Only the shared state's cheap part for (delta, kpts, known): the per-node aggregates and
    // the reset node states (every node's split is then replayed by the first search reaching it).
    // run(n, fn): fn(t) for t < n on n threads (nullptr / nthr 1: this thread only).
    void cert_warm(double delta, const double *kpts, const uint8_t *known, unsigned nthr = 1,
                   const std::function<void(unsigned, const std::function<void(unsigned)> &)> &run = nullptr) const;
    // The same after kpts / known changed on the rows pts[0..n) only: the calling thread's
    // cache keeps its per-node values but those of these points' leaves and their ancestors.
    void cert_update(const uint32_t *pts, size_t n) const;

private:
    struct Node {
        bool leaf;
        size_t left, right;      // the node's points: vind[left, right)
        int divfeat;
        double divlow, divhigh;
        double cutval, split_val;   // the cut and the cell-box midpoint it was clamped from
        double spread_gap;          // the cut dimension's spread minus the next candidate's
        uint64_t cand;              // dimensions that were split candidates
        int child1, child2;
    };
    // the build reads one coordinate of many points at a time: a column-major copy keeps
    // those reads in cache (row-major, every read of a 48-D codebook was a cache miss)
    double pt(size_t i, int d) const { return cols_[(size_t)d * K_ + i]; }
    double ptr(size_t i, int d) const { return pts_[i * (size_t)dim_ + d]; }   // row-major
    // The exact point min / max of a node's points in the dimensions of mask (the rest unknown).
    struct Known {
        Box b[64];
        uint64_t mask;
    };
    // bbox: the node's cell box (dim entries); children's boxes live in boxes_ at their level.
    // kn: what is known of the node's point extremes (middle_split adds what it computes).
    int divide(size_t left, size_t right, Box *bbox, Known &kn, int level, RecycledVec<Node> &nodes, int &depth);
    void middle_split(size_t *ind, size_t count, size_t &index, int &cutfeat, double &cutval, const Box *bbox,
                      Known &kn, Node *info);
    void child_known(const size_t *ind, size_t n1, size_t count, const Known &kn, Known &k1, Known &k2) const;
    static Known *level_known(int level);   // two per tree level
    void plane_split(size_t *ind, size_t count, int cutfeat, double cutval, size_t &lim1, size_t &lim2);
    void min_max(const size_t *ind, size_t count, int e, double &mn, double &mx) const;
    const double *pts_;
    int dim_;
    size_t K_;
    const std::atomic<bool> *cancel_ = nullptr;
    bool cancelled_ = false;
    const double *cols_ = nullptr;   // [dim][K], thread-local scratch valid during the build
    std::vector<size_t> vind_;
    RecycledVec<Node> nodes_;
    std::vector<Box> root_bbox_;
    RecycledVec<Box> node_box_;   // [node][dim]: the node's actual point box (the build's in/out bbox)
    int depth_ = 0;
    std::vector<KdNodeDev> flat_nodes_;
    std::vector<uint32_t> flat_vind_;
    std::vector<double> flat_box_;

    // certified_search's replay: the values each build quantity takes over all splits allowed
    struct Iv { double lo, hi; };
    struct CertNode {
        Iv dl{0, 0}, dh{0, 0};   // divlow, divhigh
    };
    // the replay's state, per thread (replays of one tree may run on several threads) and
    // reused from tree to tree (no fresh pages per level); owned by the tree that reset it last
    struct CertScratch {
        uint64_t owner = 0;   // the owning tree's id_
        uint64_t gen = 0;     // and its cert_gen_ then
        double delta = -1;
        const double *k = nullptr;       // the reference's split where known
        const uint8_t *known = nullptr;
        bool collect = false;            // the cache's mode
        std::vector<uint32_t> *blame = nullptr;   // collecting (certify_blame)
    };
    // the replayed nodes, shared by the threads that replay with one key (cert_gen_, delta,
    // kpts, known, mode): a node's state goes 0 -> 3 (being replayed by one thread) -> 1 (the
    // same split for every allowed codebook; its children's cell boxes and its divlow /
    // divhigh set) or 2 (not shown)
    mutable std::unique_ptr<std::atomic<int8_t>[]> cstate_;
    mutable std::vector<CertNode> cnode_;   // dl, dh
    mutable Recycled<Iv> cbox_;             // [node][dim][lo, hi]: the node's cell box
    mutable std::atomic<uint64_t> ckey_gen_{~0ull};
    mutable double ckey_delta_ = -1;
    mutable const double *ckey_k_ = nullptr;
    mutable const uint8_t *ckey_known_ = nullptr;
    mutable bool ckey_collect_ = false;
    // the per-node aggregates, shared by the threads that replay (computed by the first of them
    // for one (cert_gen_, kpts, known), then read only)
    mutable std::mutex agg_mu_;
    mutable std::atomic<uint64_t> agg_gen_{~0ull};
    mutable const double *agg_k_ = nullptr;
    mutable const uint8_t *agg_known_ = nullptr;
    mutable Recycled<double> agg_;         // [node][min unknown | max unknown | min known | max known][dim]
    mutable std::vector<int> parent_;
    mutable std::vector<int> leaf_of_;     // point -> its leaf
    void cert_ensure_agg(uint64_t gen, const double *kpts, const uint8_t *known) const;
    static CertScratch &cert_scratch();
    Iv piv(size_t p, int d) const {
        const CertScratch &S = cert_scratch();
        const size_t i = p * (size_t)dim_ + d;
        if (S.known[i]) return {S.k[i], S.k[i]};
        return {pts_[i] - S.delta, pts_[i] + S.delta};
    }
    bool cert_split(int node) const;
    void cert_reset(double delta, const double *kpts, const uint8_t *known) const;
    void blame_extremes(int node, int d) const;
    void cert_agg_node(size_t i) const;
    void cert_agg_dims(size_t i, int d0, int d1) const;
    void agg_prepare(const double *kpts, const uint8_t *known) const;
    Iv iv_min(int node, int d) const;
    Iv iv_max(int node, int d) const;

    void blame_dim(int node, int d, bool with_cell) const;

    uint64_t id_;   // unique per tree (a later tree may reuse this one's address)
    mutable std::atomic<uint64_t> cert_gen_{0};   // cert_clear: every thread's cache is stale
};

// The reference's index for tie row q: certified_search, once the candidates cand (near_set
// over the exact-sum split, slack covering the reference's bits) are all known; else -1.
int64_t certify_tie(const RefKDTree &t, const double *q, const std::vector<uint32_t> &cand, const double *kpts,
                    const uint8_t *known, int dim, double delta);

}  // namespace qvq
