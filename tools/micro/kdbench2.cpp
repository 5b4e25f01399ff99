#include "kdtree.hpp"
#include <algorithm>
#include <chrono>
#include <cstdio>
#include <random>
#include <vector>
// median-of-reps build time; codebook like a split level: centroids of clustered data x 1.2 / 0.8
int main() {
    for (int D : {12, 48}) for (int K : {1024, 4096}) {
        std::vector<double> p((size_t)K * D);
        std::mt19937_64 r(1);
        for (int k = 0; k < K / 2; k++)
            for (int d = 0; d < D; d++) {
                const double v = (r() % 100000) / 100000.0 * (d % 3 == 0 ? 1.0 : 0.6);
                p[(size_t)k * D + d] = v * 1.2;
                p[(size_t)(k + K / 2) * D + d] = v * 0.8;
            }
        std::vector<double> t;
        for (int i = 0; i < 31; i++) {
            auto t0 = std::chrono::steady_clock::now();
            qvq::RefKDTree tr(p.data(), K, D);
            t.push_back(std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count());
        }
        std::sort(t.begin(), t.end());
        printf("D=%d K=%d build median %.3f ms  min %.3f\n", D, K, t[15], t[0]);
    }
}
