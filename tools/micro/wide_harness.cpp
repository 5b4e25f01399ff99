// Standalone check of launch_assign_wide against a CPU evaluation of the same scores.
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <random>
#include <vector>

#include "common.hpp"

using namespace qvq;

int main(int argc, char **argv) {
    const uint32_t D = argc > 1 ? atoi(argv[1]) : 3, K = argc > 2 ? atoi(argv[2]) : 32;
    const uint64_t N = argc > 3 ? atoll(argv[3]) : 4096;
    const uint32_t Dp = (D + 3) & ~3u, Kp = (K + 31) & ~31u, RF = wide_row_f16(Dp), LO = wide_dh(Dp);
    const double mu = 0.5, sx = 1.0 / 510.0;
    const int t = 10;
    std::mt19937_64 rng(1);
    std::vector<uint8_t> codes(N * Dp);
    for (auto &b : codes) b = rng() & 0xFF;
    std::vector<double> C(K * D);
    for (auto &v : C) v = (rng() % 1000) / 1000.0;
    std::vector<float> C32(Kp * Dp, 0.f);
    std::vector<_Float16> rows(Kp * RF, (_Float16)0.f);
    for (uint32_t k = 0; k < Kp; k++) {
        _Float16 *r = &rows[k * RF];
        if (k >= K) {
            r[2 * LO] = r[2 * LO + 1] = (_Float16)MF_PAD_SCORE;
            continue;
        }
        double n = 0;
        for (uint32_t d = 0; d < D; d++) {
            const double x = C[k * D + d];
            C32[k * Dp + d] = (float)x;
            const double cp = x - mu;
            n += cp * cp;
            const double c2 = -2.0 * sx * cp * std::ldexp(1.0, t);
            const _Float16 h = (_Float16)(float)c2;
            r[d] = h;
            r[LO + d] = (_Float16)(float)(c2 - (double)(float)h);
        }
        n *= std::ldexp(1.0, t);
        const _Float16 h = (_Float16)(float)n;
        r[2 * LO] = h;
        r[2 * LO + 1] = (_Float16)(float)(n - (double)(float)h);
    }
    MfThresholds th{};
    th.mfma = 1e-5f;
    th.alpha = 1e-6f;
    th.beta = 1e-6f;
    th.gamma = 1e-12f;
    th.inv_scale = (float)std::ldexp(1.0, -t);
    th.mu = (float)mu;
    th.sx = (float)sx;
    uint8_t *d_codes;
    _Float16 *d_rows;
    float *d_C32;
    uint32_t *d_A, *d_flags;
    unsigned *d_cnt;
    hipMalloc(&d_codes, codes.size());
    hipMalloc(&d_rows, rows.size() * 2);
    hipMalloc(&d_C32, C32.size() * 4);
    hipMalloc(&d_A, N * 4);
    hipMalloc(&d_flags, N * 4);
    hipMalloc(&d_cnt, 4);
    hipMemcpy(d_codes, codes.data(), codes.size(), hipMemcpyHostToDevice);
    hipMemcpy(d_rows, rows.data(), rows.size() * 2, hipMemcpyHostToDevice);
    hipMemcpy(d_C32, C32.data(), C32.size() * 4, hipMemcpyHostToDevice);
    hipMemset(d_cnt, 0, 4);
    hipError_t e = launch_assign_wide(0, 256, Dp, D, d_codes, N, d_rows, K, d_C32, th, d_A, d_flags, d_cnt);
    hipError_t e2 = hipDeviceSynchronize();
    std::vector<uint32_t> A(N), flags(N);
    unsigned cnt = 0;
    hipMemcpy(A.data(), d_A, N * 4, hipMemcpyDeviceToHost);
    hipMemcpy(&cnt, d_cnt, 4, hipMemcpyDeviceToHost);
    hipMemcpy(flags.data(), d_flags, N * 4, hipMemcpyDeviceToHost);
    std::vector<char> isf(N, 0);
    for (unsigned i = 0; i < cnt && i < N; i++) isf[flags[i]] = 1;
    uint64_t bad = 0;
    for (uint64_t i = 0; i < N; i++) {
        double best = 1e300;
        uint32_t bk = 0;
        double sc_best = 1e300;
        for (uint32_t k = 0; k < K; k++) {
            double dist = 0, sc = 0;
            for (uint32_t d = 0; d < D; d++) {
                const int w = 2 * (codes[i * Dp + d] ^ 0x80) - 255;
                const double x = mu + w * sx;
                dist += (x - C[k * D + d]) * (x - C[k * D + d]);
                sc += ((double)rows[k * RF + d] + (double)rows[k * RF + LO + d]) * w;
            }
            sc += (double)rows[k * RF + 2 * LO] + (double)rows[k * RF + 2 * LO + 1];
            if (dist < best) {
                best = dist;
                bk = k;
                sc_best = sc;
            }
        }
        if (A[i] != bk && !isf[i]) {
            if (bad < 8) printf("row %lu: gpu %u cpu %u (score %g)\n", (unsigned long)i, A[i], bk, sc_best);
            bad++;
        }
    }
    printf("D=%u K=%u N=%lu: launch %s sync %s, flagged %u, unflagged mismatches %lu\n", D, K, (unsigned long)N,
           hipGetErrorString(e), hipGetErrorString(e2), cnt, (unsigned long)bad);
    return bad != 0;
}
