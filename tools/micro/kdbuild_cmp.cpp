#include "kdtree_old.hpp"
#include "kdtree.hpp"
#include <chrono>
#include <cstdio>
#include <cstring>
#include <random>
#include <vector>
int main(int argc, char **argv) {
    const char *f = argv[1]; int K = atoi(argv[2]), D = atoi(argv[3]);
    std::vector<double> p((size_t)K * D);
    if (f[0] == '@') {   // random with duplicates
        std::mt19937_64 r(atoi(f + 1));
        for (int k = 0; k < K; k++) {
            bool z = r() % 4 == 0;
            for (int d = 0; d < D; d++) p[(size_t)k * D + d] = z ? 0.0 : (r() % 1000) / 997.0;
        }
    } else { FILE *fp = fopen(f, "rb"); if (fread(p.data(), 8, p.size(), fp) != p.size()) return 2; fclose(fp); }
    double tn = 1e9, to = 1e9;
    for (int rep = 0; rep < 20; rep++) {
        auto t0 = std::chrono::steady_clock::now();
        qvq_old::RefKDTree a(p.data(), K, D);
        auto t1 = std::chrono::steady_clock::now();
        qvq::RefKDTree b(p.data(), K, D);
        auto t2 = std::chrono::steady_clock::now();
        to = std::min(to, std::chrono::duration<double, std::milli>(t1 - t0).count());
        tn = std::min(tn, std::chrono::duration<double, std::milli>(t2 - t1).count());
        if (rep) continue;
        if (a.num_nodes() != b.num_nodes() || a.depth() != b.depth()) { printf("MISMATCH shape\n"); return 1; }
        size_t nn = a.num_nodes();
        std::vector<qvq_old::KdNodeDev> na(nn); std::vector<qvq::KdNodeDev> nb(nn);
        std::vector<uint32_t> va(K), vb(K); std::vector<double> la(D), ha(D), lb(D), hb(D);
        a.flatten(na.data(), va.data(), la.data(), ha.data());
        b.flatten(nb.data(), vb.data(), lb.data(), hb.data());
        if (memcmp(na.data(), nb.data(), nn * sizeof(nb[0])) || va != vb || la != lb || ha != hb) { printf("MISMATCH image\n"); return 1; }
        std::mt19937_64 r(5);
        for (int q = 0; q < 300; q++) {
            std::vector<double> x(D);
            for (auto &v : x) v = (r() % 1200) / 1000.0;
            std::vector<uint32_t> ca, cb; double da, db;
            a.near_set(x.data(), 1e-3, 1e-3, ca, da); b.near_set(x.data(), 1e-3, 1e-3, cb, db);
            if (ca != cb || da != db || a.nearest(x.data()) != b.nearest(x.data())) { printf("MISMATCH query %d\n", q); return 1; }
        }
    }
    printf("%s K=%d D=%d identical; build old %.3f ms new %.3f ms\n", f, K, D, to, tn);
}
