// Writes the host build's device image for a set of point sets (tie-heavy random, clustered,
// the C4 level codebooks) to argv[1]: two builds of kdtree.cpp must write the same bytes.
#include "kdtree.hpp"
#include "kdtree_dev.hpp"
#include <cstdio>
#include <random>
#include <vector>
int main(int argc, char **argv) {
    FILE *o = std::fopen(argv[1], "wb");
    std::vector<std::vector<double>> sets;
    std::vector<std::pair<int, int>> shp;
    std::mt19937_64 r(7);
    for (int D : {3, 12, 48})
        for (int K : {2, 7, 16, 64, 256, 1024, 4096})
            for (int levels : {2, 5, 50, 1000000}) {
                std::vector<double> p((size_t)K * D);
                for (auto &v : p) v = (r() % 10 < 3) ? 0.0 : (double)(r() % levels) / levels;
                sets.push_back(p);
                shp.push_back({K, D});
            }
    for (const char *f : {"tools/micro/data/b2_L10.f64", "tools/micro/data/b4_L11.f64", "tools/micro/data/b4_L12.f64"}) {
        FILE *i = std::fopen(f, "rb");
        std::vector<double> p;
        double v;
        while (std::fread(&v, 8, 1, i) == 1) p.push_back(v);
        std::fclose(i);
        const int D = std::string(f).find("b2_") != std::string::npos ? 12 : 48;
        sets.push_back(p);
        shp.push_back({(int)(p.size() / D), D});
    }
    for (size_t s = 0; s < sets.size(); s++) {
        const int K = shp[s].first, D = shp[s].second;
        qvq::RefKDTree t(sets[s].data(), K, D);
        std::vector<uint8_t> img(qvq::kdb_host_layout(K, D).total);
        t.to_device_image(img.data());
        std::fwrite(img.data(), 1, img.size(), o);
        for (int q = 0; q < 64; q++) {   // and some nearest answers
            std::vector<double> x(D);
            for (auto &v : x) v = (double)(r() % 7) / 7;
            const uint32_t a = t.nearest(x.data());
            std::fwrite(&a, 4, 1, o);
        }
    }
    std::fclose(o);
    std::printf("%zu sets\n", sets.size());
}
