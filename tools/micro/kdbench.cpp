#include "kdtree.hpp"
#include <chrono>
#include <cstdio>
#include <random>
#include <vector>
int main() {
    for (int D : {12, 48}) for (int K : {1024, 2048, 4096}) {
        std::vector<double> p((size_t)K * D);
        std::mt19937_64 r(1);
        for (auto &v : p) v = (r() % 100000) / 100000.0;
        auto t0 = std::chrono::steady_clock::now();
        int reps = 20;
        size_t nn = 0;
        for (int i = 0; i < reps; i++) { qvq::RefKDTree t(p.data(), K, D); nn += t.num_nodes(); }
        auto t1 = std::chrono::steady_clock::now();
        printf("D=%d K=%d build %.3f ms (nodes %zu)\n", D, K, std::chrono::duration<double, std::milli>(t1 - t0).count() / reps, nn / reps);
    }
}
