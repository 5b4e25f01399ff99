// One kdtree.cpp build on level codebooks (data/b4_L12.f64, b4_L11.f64: C4, D = 48;
// b2_L10.f64: D = 12): median build time warm (back to back, 31 builds), cold (a 256 MB
// sweep before each, 15 builds) and novel (each of 15 builds on its own row permutation of the
// set: the branch predictors have not seen the build before, as in the engine, where a level's
// tree is built once -- the same build repeated in the engine runs at the warm time).
#include "kdtree.hpp"
#include <algorithm>
#include <chrono>
#include <cstdio>
#include <random>
#include <string>
#include <vector>
int main() {
    std::vector<char> sweep(256u << 20, 1);
    for (const char *f : {"tools/micro/data/b4_L12.f64", "tools/micro/data/b4_L11.f64", "tools/micro/data/b2_L10.f64"}) {
        std::vector<double> p;
        FILE *i = std::fopen(f, "rb");
        if (!i) return 1;
        double v;
        while (std::fread(&v, 8, 1, i) == 1) p.push_back(v);
        std::fclose(i);
        const int D = std::string(f).find("b2_") != std::string::npos ? 12 : 48, K = (int)(p.size() / D);
        std::vector<std::vector<double>> perm(15);
        std::mt19937_64 rng(5);
        for (auto &q : perm) {
            std::vector<int> o(K);
            for (int k = 0; k < K; k++) o[k] = k;
            std::shuffle(o.begin(), o.end(), rng);
            q.resize(p.size());
            for (int k = 0; k < K; k++) std::copy(p.begin() + (size_t)o[k] * D, p.begin() + (size_t)(o[k] + 1) * D, q.begin() + (size_t)k * D);
        }
        for (int cold = 0; cold < 3; cold++) {
            std::vector<double> t;
            for (int r = 0; r < (cold ? 15 : 31); r++) {
                if (cold == 1) {
                    volatile char s = 0;
                    for (size_t j = 0; j < sweep.size(); j += 64) { sweep[j]++; s = s + sweep[j]; }
                }
                const auto t0 = std::chrono::steady_clock::now();
                qvq::RefKDTree tr(cold == 2 ? perm[r].data() : p.data(), K, D);
                t.push_back(std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count());
            }
            std::sort(t.begin(), t.end());
            std::printf("D %d K %d %s: median %.3f ms min %.3f\n", D, K, cold == 2 ? "novel" : cold ? "cold" : "warm", t[t.size() / 2], t[0]);
        }
    }
}
