// CPU check of the segment-parallel Kahan evaluator (quant_amd/csrc/kahan_par.hpp): for
// random SCALED chains of many kinds, eval_chain must return the bits of the reference's
// sequential sumInArea (src/Quantizer.cpp:59-70), and the builder/composer are exercised at
// several segment and group sizes.  Prints one line per case; exit status 1 on any mismatch.
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
#include <vector>

#include "kahan_par.hpp"

using namespace qvq::kahan;

static double scaled(int b) { return ((double)(signed char)(unsigned char)b + 128.0) * (1.0 / 255); }

static double kahan_ref(const std::vector<double> &x) {
    double sum = 0, c = 0;
    for (double v : x) {
        double y = v - c;
        double t = sum + y;
        c = (t - sum) - y;
        sum = t;
    }
    return sum;
}

struct Result {
    double v;
    uint32_t stats[3];
};

// The engine's two passes over one chain: tables from dest 0, a trusted walk for the
// estimates, tables again, composition, exact evaluation.
static Result run_chain(const std::vector<uint8_t> &b, const uint64_t *Xt, uint32_t L, uint32_t S, int passes) {
    const uint64_t n = b.size();
    const uint64_t nseg = (n + L - 1) / L, GL = (uint64_t)L * S, ngrp = (n + GL - 1) / GL;
    const uint64_t SL = GL * S, nsup = (n + SL - 1) / SL;
    std::vector<Fn> f0(nseg), f1(ngrp), f2(nsup);
    std::vector<i128> P0(nseg + 1);
    std::vector<int64_t> dest(nseg, 0);
    Chain c{b.data(), Xt, n, f0.data(), f1.data(), f2.data(), L, S};
    for (int pass = 0; pass < passes; pass++) {
        i128 P = 0;
        for (uint64_t s = 0; s < nseg; s++) {
            const uint64_t a = s * L;
            const uint32_t len = (uint32_t)c.len0(s);
            P0[s] = P;
            f0[s] = build_segment(b.data() + a, Xt, len, P, dest[s]);
            for (uint32_t j = 0; j < len; j++) P += (i128)Xt[b[a + j]];
        }
        if (pass + 1 < passes) estimate_dest(c, P0.data(), dest.data());
    }
    for (uint64_t g = 0; g < ngrp; g++) f1[g] = compose1(c, g);
    for (uint64_t g = 0; g < nsup; g++) f2[g] = compose2(c, g);
    Result r{};
    r.v = eval_chain(c, r.stats);
    return r;
}

int main(int argc, char **argv) {
    const int reps = argc > 1 ? atoi(argv[1]) : 200;
    uint64_t Xt[256];
    for (int b = 0; b < 256; b++) Xt[b] = (uint64_t)ldexp(scaled(b), 60);
    std::mt19937_64 rng(12345);
    int bad = 0, cases = 0;
    uint64_t tot_seg = 0, fail_seg = 0, tot_grp = 0, fail_grp = 0, tot_sup = 0, fail_sup = 0;
    // byte codes: code b has value (int8(b) + 128)/255, so u = b ^ 0x80 is the value index
    auto code = [](int u) { return (uint8_t)(u ^ 0x80); };
    for (int rep = 0; rep < reps; rep++) {
        const int kind = rep % 8;
        uint64_t n;
        if (rep % 5 == 0) n = 1 + rng() % 50;
        else if (rep % 5 == 1) n = 1 + rng() % 5000;
        else if (rep % 5 == 2) n = 1 + rng() % 200000;
        else n = 1 + rng() % 1000000;
        std::vector<uint8_t> b(n);
        std::vector<double> x(n);
        const int lo = (int)(rng() % 256), span = 1 + (int)(rng() % 40);
        for (uint64_t i = 0; i < n; i++) {
            int u;
            switch (kind) {
            case 0: u = (int)(rng() % 256); break;                                  // noise
            case 1: u = (rng() % 4 == 0) ? 255 : (int)(rng() % 256); break;          // saturated
            case 2: u = (int)(rng() % 8); break;                                     // dark
            case 3: u = std::min(255, lo + (int)(rng() % span)); break;             // narrow band
            case 4: u = (rng() % 3 == 0) ? 0 : (int)(rng() % 256); break;            // zeros
            case 5: u = 255; break;                                                  // flat 1.0
            case 6: u = (rng() % 2) ? 255 : 128 + (int)(rng() % 8); break;           // 1.0 and mid
            default: u = (int)(64 + rng() % 64); break;                              // [0.25, 0.5)
            }
            b[i] = code(u);
            x[i] = scaled(b[i]);
        }
        const double ref = kahan_ref(x);
        static const uint32_t Ls[] = {16, 64, 128, 256};
        static const uint32_t Ss[] = {4, 16, 32};
        const uint32_t L = Ls[rep % 4], S = Ss[rep % 3];
        const int mode = argc > 2 ? atoi(argv[2]) : 2;
        Result r = run_chain(b, Xt, L, S, mode);
        cases++;
        const uint64_t nseg = (n + L - 1) / L, ngrp = (nseg + S - 1) / S, nsup = (ngrp + S - 1) / S;
        tot_seg += nseg;
        tot_grp += ngrp;
        tot_sup += nsup;
        fail_seg += r.stats[0];
        fail_grp += r.stats[1];
        fail_sup += r.stats[2];
        if (getenv("KVERBOSE")) printf("kind %d n %llu L %u S %u misses %u/%llu %u/%llu %u/%llu\n", kind, (unsigned long long)n, L, S,
                                       r.stats[0], (unsigned long long)nseg, r.stats[1], (unsigned long long)ngrp,
                                       r.stats[2], (unsigned long long)nsup);
        if (memcmp(&ref, &r.v, 8) != 0) {
            bad++;
            printf("MISMATCH rep %d kind %d n %llu L %u S %u: ref %.17g got %.17g\n", rep, kind,
                   (unsigned long long)n, L, S, ref, r.v);
        }
    }
    printf("cases %d mismatches %d | table misses: segments %llu/%llu groups %llu/%llu super %llu/%llu\n", cases, bad,
           (unsigned long long)fail_seg, (unsigned long long)tot_seg, (unsigned long long)fail_grp,
           (unsigned long long)tot_grp, (unsigned long long)fail_sup, (unsigned long long)tot_sup);
    return bad ? 1 : 0;
}
