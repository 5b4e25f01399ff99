// ref_nn.cpp -- TEST INFRASTRUCTURE ONLY.  A thin driver over the reference's vendored
// nanoflann headers, compiled from where they lie (/root/reference/include/external) with
// the reference's Release flags (-O3 -ffast-math, CMakeLists.txt:9-10), mirroring
// KDTree::nearestNeighbour (src/KDTree.cpp:8-29).  It never ships: the built .so lives in
// oracle/_ref/ (git-ignored) and is only used by tests to check the restated kd-tree in
// lbg_oracle.c and quant_amd/csrc/kdtree.cpp.  Training-set storage is std::vector
// instead of boost::container::small_vector (Boost is absent; the storage type does not
// enter the arithmetic).
#include <cstdint>
#include <vector>
#include "nanoflann.hpp"
#include "KDTreeVectorOfVectorsAdaptor.hpp"

typedef std::vector<std::vector<double>> Points;
typedef KDTreeVectorOfVectorsAdaptor<Points, double> Tree;

extern "C" __attribute__((visibility("default"))) void ref_kdtree_nn(const double *C, size_t K, int D,
                                                                     const double *Q, size_t nq, uint32_t *out) {
    Points pts(K);
    for (size_t k = 0; k < K; k++) pts[k].assign(C + k * D, C + (k + 1) * D);
    Tree tree(D, pts);
    tree.index->buildIndex();
    std::vector<double> q(D);
    #pragma omp parallel for firstprivate(q)
    for (size_t i = 0; i < nq; i++) {
        size_t idx = 0;
        double dist = 0;
        nanoflann::KNNResultSet<double> rs(1);
        rs.init(&idx, &dist);
        q.assign(Q + i * D, Q + (i + 1) * D);
        tree.index->findNeighbors(rs, &q[0], nanoflann::SearchParams(10));
        out[i] = (uint32_t)idx;
    }
}
