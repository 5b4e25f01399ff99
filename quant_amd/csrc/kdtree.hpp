// Host-side exact nearest-neighbour resolver with nanoflann 1.2.3 semantics.
//
// The device assigns every block by brute force.  A handful of rows per level have two
// code vectors at (nearly) the same fp64 distance; for those the reference's answer is
// whatever its kd-tree search visits first (src/KDTree.cpp:20-29 over
// include/external/nanoflann.hpp).  This class rebuilds that tree over the level's
// codebook and answers exactly those rows.  It is part of the product (not the oracle):
// the C-ABI engine calls it for rows the fp64 recheck kernel hands back.
#pragma once
#include <cstddef>
#include <cstdint>
#include <vector>

namespace qvq {

// Squared L2 as the reference's Release build evaluates nanoflann's L2_Adaptor
// (nanoflann.hpp:320-339 under g++ -O3 -ffast-math): each group of four squares is
// added as (s1 + s2) + (s0 + s3), then the 0-3 leftover components one by one.  Must
// stay bit-identical to the device recheck (qvq_engine.hip, ref_l2_dev).
double ref_l2(const double *a, const double *b, int dim);

class RefKDTree {
public:
    // pts: K x dim, row-major, borrowed for the lifetime of the tree.
    RefKDTree(const double *pts, size_t K, int dim);
    // Index the reference's kd-tree search returns for query q (dim values).
    uint32_t nearest(const double *q) const;

private:
    struct Box { double low, high; };
    struct Node {
        bool leaf;
        size_t left, right;      // leaf: vind[left, right)
        int divfeat;
        double divlow, divhigh;
        int child1, child2;
    };
    double pt(size_t i, int d) const { return pts_[i * (size_t)dim_ + d]; }
    int divide(size_t left, size_t right, std::vector<Box> &bbox);
    void middle_split(size_t *ind, size_t count, size_t &index, int &cutfeat, double &cutval,
                      const std::vector<Box> &bbox);
    void plane_split(size_t *ind, size_t count, int cutfeat, double cutval, size_t &lim1, size_t &lim2);
    void min_max(const size_t *ind, size_t count, int e, double &mn, double &mx) const;
    void search(const double *q, int node, double mindistsq, std::vector<double> &dists, double &best,
                size_t &best_idx, bool &have) const;

    const double *pts_;
    int dim_;
    std::vector<size_t> vind_;
    std::vector<Node> nodes_;
    std::vector<Box> root_bbox_;
};

}  // namespace qvq
