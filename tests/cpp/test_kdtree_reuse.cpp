// CPU check of RefKDTree::unchanged_under (quant_amd/csrc/kdtree.cpp): the level's tree over the
// exact-sum split codebook may stand for the tree over the Kahan-bit one only when the two
// trees are bit for bit the same image (nanoflann.hpp:1046-1186 as RefKDTree restates it).
// Input: [u32 K][u32 D] then pairs of K x D doubles (exact split, Kahan split), repeated.  For
// each pair and for random one-ulp perturbations of each exact codebook, a claim "unchanged"
// must be true.  Prints one summary line; exit status 1 on a wrong claim.
#include <cmath>
#include <cstdio>
#include <cstring>
#include <random>
#include <vector>

#include "kdtree.hpp"

using namespace qvq;

static bool same_image(const std::vector<double> &a, const std::vector<double> &b, uint32_t K, int D) {
    RefKDTree ta(a.data(), K, D), tb(b.data(), K, D);
    if (ta.num_nodes() != tb.num_nodes() || ta.depth() != tb.depth()) return false;
    const size_t nn = ta.num_nodes();
    std::vector<KdNodeDev> na(nn), nb(nn);
    std::vector<uint32_t> va(K), vb(K);
    std::vector<double> la(2 * D), lb(2 * D);
    ta.flatten(na.data(), va.data(), la.data(), la.data() + D);
    tb.flatten(nb.data(), vb.data(), lb.data(), lb.data() + D);
    return !memcmp(na.data(), nb.data(), nn * sizeof(KdNodeDev)) && va == vb && la == lb;
}

int main(int argc, char **argv) {
    if (argc < 2) return 2;
    FILE *f = fopen(argv[1], "rb");
    if (!f) return 2;
    std::mt19937_64 rng(7);
    int wrong = 0, pairs = 0, claims = 0, truths = 0;
    uint32_t hdr[2];
    while (fread(hdr, 4, 2, f) == 2) {
        const uint32_t K = hdr[0];
        const int D = (int)hdr[1];
        std::vector<double> x((size_t)K * D), k((size_t)K * D);
        if (fread(x.data(), 8, x.size(), f) != x.size() || fread(k.data(), 8, k.size(), f) != k.size()) return 2;
        RefKDTree t(x.data(), K, D);
        auto check = [&](const std::vector<double> &y) {
            const bool claim = t.unchanged_under(y.data());
            const bool truth = same_image(x, y, K, D);
            claims += claim;
            truths += truth;
            if (claim && !truth) wrong++;
        };
        check(k);
        pairs++;
        for (int rep = 0; rep < 100; rep++) {
            std::vector<double> y = x;
            const int nch = 1 + (int)(rng() % 30);
            for (int c = 0; c < nch; c++) {
                const size_t i = rng() % y.size();
                y[i] = std::nextafter(y[i], (rng() & 1) ? 10.0 : -10.0);
            }
            check(y);
        }
    }
    printf("kdtree reuse: codebooks %d, claimed unchanged %d of %d truly unchanged, wrong claims %d\n", pairs, claims,
           truths, wrong);
    return wrong ? 1 : 0;
}
