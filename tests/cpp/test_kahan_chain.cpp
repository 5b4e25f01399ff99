// CPU check of the segment-parallel Kahan evaluator (quant_amd/csrc/kahan_par.hpp): for chains of
// many kinds, the pipeline the device runs (segment metadata, prefix sums, segment functions,
// 64-segment block composites, the checked evaluation with replays) must return the bits of the
// reference's sequential sumInArea (src/Quantizer.cpp:59-70).  Prints one summary line; exit
// status 1 on any mismatch.
//   test_kahan_chain [reps]            random chains
//   test_kahan_chain /path/chains.bin  chains from a file ([u32 count] then per chain [u32 n][n bytes])
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
#include <algorithm>
#include <vector>

#include "kahan_par.hpp"

using namespace qvq::kahan;

static double scaled(int b) { return ((double)(signed char)(unsigned char)b + 128.0) * (1.0 / 255); }

static double kahan_ref(const std::vector<uint8_t> &b, const ByteTab &tb) {
    double sum = 0, c = 0;
    for (uint8_t v : b) {
        double y = ldexp((double)tb.X[v], -60) - c;
        double t = sum + y;
        c = (t - sum) - y;
        sum = t;
    }
    return sum;
}

struct Stats {
    uint64_t segs = 0, raw = 0, blocks = 0, blk_bad = 0, blk_miss = 0, seg_miss = 0, replays = 0;
};

// The device pipeline on one chain, serially.
static double run_chain(const std::vector<uint8_t> &b, const ByteTab &tb, Stats &st) {
    const uint32_t n = (uint32_t)b.size();
    if (n == 0) return 0.0;
    const uint32_t nseg = (n + L - 1) / L;
    std::vector<SegMeta> meta(nseg);
    std::vector<u128> P(nseg + 1);
    P[0] = 0;
    for (uint32_t j = 0; j < nseg; j++) {
        const uint32_t len = std::min(L, n - j * L);
        meta[j] = seg_meta(tb, b.data() + j * L, len);
        P[j + 1] = P[j] + meta_sum(meta[j]);
    }
    auto build = [&](uint32_t j, int64_t D_est, Fn &f) {
        int c_in;
        uint32_t off_in;
        input_structure([&](int i) { return meta[j - i]; }, (int)std::min<uint32_t>(8, j), c_in, off_in);
        build_fn(tb, b.data() + j * L, std::min(L, n - j * L), P[j], meta[j], c_in, off_in, j + 1 == nseg, D_est, f);
    };
    // block composites (estimates 0), a tree as on the device
    const uint32_t nblk = (nseg + SPB - 1) / SPB;
    std::vector<Fn> blk(nblk);
    std::vector<bool> blk_ok(nblk);
    std::vector<SegFn> segfn(nseg);   // stored for the evaluation's re-walks (estimates 0)
    for (uint32_t bi = 0; bi < nblk; bi++) {
        const uint32_t s0 = bi * SPB, s1 = std::min(nseg, s0 + SPB);
        std::vector<Fn> f(SPB);
        std::vector<bool> ok(SPB, false);
        for (uint32_t s = s0; s < s1; s++) {
            build(s, 0, f[s - s0]);
            pack_seg(f[s - s0], segfn[s]);
            ok[s - s0] = fkind(f[s - s0]) != FK_RAW;
            st.segs++;
            st.raw += !ok[s - s0];
        }
        for (uint32_t w = 1; w < SPB; w <<= 1)
            for (uint32_t i = 0; i + w < SPB; i += 2 * w) {
                if (s0 + i + w >= s1) continue;
                Fn h;
                const bool c = ok[i] && ok[i + w] && compose(f[i], f[i + w], h);
                ok[i] = c;
                if (c) f[i] = h;
            }
        blk[bi] = f[0];
        blk_ok[bi] = ok[0];
        st.blocks++;
        st.blk_bad += !ok[0];
    }
    // evaluation
    double sum;
    u128 Pt, E;
    const uint32_t tau = transient(tb, b.data(), n, sum, Pt, E);
    if (!(sum >= 2.0)) return sum;
    int64_t D = (int64_t)(E - Pt);
    uint32_t F = (uint32_t)E & 511;
    uint32_t j = (tau + L - 1) / L;
    if (tau % L) {   // to the next boundary, exactly
        const uint32_t end = std::min(n, j * L);
        D += replay(tb, b.data() + tau, end - tau, Pt, F, D);
        st.replays++;
    }
    while (j < nseg) {
        if ((uint32_t)((P[j] + (u128)(i128)D) & 511) != F) abort();   // state consistency
        const uint32_t bi = j / SPB;
        if (j % SPB == 0 && blk_ok[bi]) {
            uint32_t F2 = F;
            int64_t D2 = D;
            if (apply(blk[bi], F2, D2)) {
                F = F2;
                D = D2;
                j = std::min(nseg, j + SPB);
                continue;
            }
            st.blk_miss++;
        }
        const uint32_t end = std::min(nseg, (bi + 1) * SPB);
        for (; j < end; j++) {
            Fn f;
            unpack_seg(segfn[j], f);
            uint32_t F2 = F;
            int64_t D2 = D;
            if (apply(f, F2, D2)) {
                F = F2;
                D = D2;
                continue;
            }
            st.seg_miss += fkind(f) != FK_RAW;
            st.replays++;
            D += replay(tb, b.data() + j * L, std::min(L, n - j * L), P[j], F, D);
        }
    }
    return to_double(P[nseg] + (u128)(i128)D);
}

// The chained evaluation (k_kahan.hip, several ranks): the chain split at cuts into pieces, each
// piece's segment functions built with the global exact prefix, each piece evaluated from the
// state (sum, c) the previous piece left -- rank by rank, as engine.cpp's relay runs it.
static double run_chain_split(const std::vector<uint8_t> &b, const std::vector<uint32_t> &cuts, const ByteTab &tb,
                              Stats &st) {
    double sum = 0, c = 0;
    u128 P0 = 0;
    for (size_t r = 0; r + 1 < cuts.size(); r++) {
        const uint8_t *pb = b.data() + cuts[r];
        const uint32_t n = cuts[r + 1] - cuts[r];
        if (n == 0) continue;
        const uint32_t nseg = (n + L - 1) / L;
        std::vector<SegMeta> meta(nseg);
        std::vector<u128> P(nseg + 1);
        P[0] = P0;
        for (uint32_t j = 0; j < nseg; j++) {
            meta[j] = seg_meta(tb, pb + j * L, std::min(L, n - j * L));
            P[j + 1] = P[j] + meta_sum(meta[j]);
        }
        const u128 Pn = P[nseg];
        const u128 Pin = P0;
        P0 = Pn;   // the next piece's prefix
        if (Pn == Pin && !(c != 0.0 && !(sum >= 2.0))) continue;   // nothing changes the state
        std::vector<SegFn> segfn(nseg);
        for (uint32_t j = 0; j < nseg; j++) {   // (the piece's own segments only: a new rank knows nothing before)
            int c_in;
            uint32_t off_in;
            input_structure([&](int i) { return meta[j - i]; }, (int)std::min<uint32_t>(8, j), c_in, off_in);
            Fn f;
            build_fn(tb, pb + j * L, std::min(L, n - j * L), P[j], meta[j], c_in, off_in, j + 1 == nseg, 0, f);
            pack_seg(f, segfn[j]);
            st.segs++;
            st.raw += fkind(f) == FK_RAW;
        }
        // the transient from the incoming state
        uint32_t i = 0;
        u128 Pt = Pin;
        while (i < n && !(sum >= 2.0)) {
            fstep(sum, c, ldexp((double)tb.X[pb[i]], -60));
            Pt += tb.X[pb[i]];
            i++;
        }
        if (!(sum >= 2.0)) continue;
        const u128 E = (u128)(to_units(sum) - to_units(c));
        int64_t D = (int64_t)(E - Pt);
        uint32_t F = (uint32_t)E & 511;
        uint32_t j = (i + L - 1) / L;
        if (i % L) {
            D += replay(tb, pb + i, std::min(n, j * L) - i, Pt, F, D);
            st.replays++;
        }
        for (; j < nseg; j++) {
            if ((uint32_t)((P[j] + (u128)(i128)D) & 511) != F) abort();
            Fn f;
            unpack_seg(segfn[j], f);
            if (apply(f, F, D)) continue;
            st.replays++;
            D += replay(tb, pb + j * L, std::min(L, n - j * L), P[j], F, D);
        }
        const u128 Ef = Pn + (u128)(i128)D;
        sum = to_double(Ef);
        c = ldexp((double)(int64_t)(to_units(sum) - (i128)Ef), -60);
    }
    return sum;
}

static int check(const std::vector<uint8_t> &b, const ByteTab &tb, Stats &st, const char *what) {
    const double ref = kahan_ref(b, tb);
    const Stats before = st;
    const double got = run_chain(b, tb, st);
    if (getenv("KCHAIN"))   // per chain: blocks, re-walked blocks, replays
        printf("chain n %zu blocks %llu bad %llu miss %llu replays %llu\n", b.size(),
               (unsigned long long)(st.blocks - before.blocks), (unsigned long long)(st.blk_bad - before.blk_bad),
               (unsigned long long)(st.blk_miss - before.blk_miss), (unsigned long long)(st.replays - before.replays));
    if (memcmp(&ref, &got, 8) != 0) {
        printf("MISMATCH %s n %zu: ref %.17g got %.17g\n", what, b.size(), ref, got);
        return 1;
    }
    // the same chain split over 2..9 "ranks" at random cuts (some early: inside the transient,
    // some empty pieces), each piece evaluated from the state the previous one left
    static std::mt19937_64 rng(777);
    const uint32_t n = (uint32_t)b.size();
    for (int rep = 0; rep < 3; rep++) {
        const int pieces = 2 + (int)(rng() % 8);
        std::vector<uint32_t> cuts = {0, n};
        for (int p = 1; p < pieces; p++) {
            const uint64_t r = rng();
            cuts.push_back(r % 4 == 0 ? (uint32_t)(r % std::min<uint32_t>(n + 1, 300)) : (uint32_t)(r % (n + 1)));
        }
        std::sort(cuts.begin(), cuts.end());
        const double got2 = run_chain_split(b, cuts, tb, st);
        if (memcmp(&ref, &got2, 8) != 0) {
            printf("MISMATCH (split %d) %s n %zu: ref %.17g got %.17g\n", pieces, what, b.size(), ref, got2);
            return 1;
        }
    }
    return 0;
}

static void report(const char *what, int cases, int bad, const Stats &st) {
    printf("%s: cases %d mismatches %d | segments %llu raw %llu | blocks %llu not composable %llu missed %llu | "
           "segment misses %llu replays %llu\n",
           what, cases, bad, (unsigned long long)st.segs, (unsigned long long)st.raw, (unsigned long long)st.blocks,
           (unsigned long long)st.blk_bad, (unsigned long long)st.blk_miss, (unsigned long long)st.seg_miss,
           (unsigned long long)st.replays);
}

int main(int argc, char **argv) {
    uint64_t Xt[256];
    for (int b = 0; b < 256; b++) Xt[b] = (uint64_t)ldexp(scaled(b), 60);
    static ByteTab tb;
    make_tab(Xt, tb);
    Stats st;
    int bad = 0, cases = 0;
    if (argc > 1 && argv[1][0] == '/') {
        FILE *fp = fopen(argv[1], "rb");
        if (!fp) return 2;
        uint32_t nc = 0;
        if (fread(&nc, 4, 1, fp) != 1) return 2;
        for (uint32_t i = 0; i < nc; i++) {
            uint32_t n = 0;
            if (fread(&n, 4, 1, fp) != 1) return 2;
            std::vector<uint8_t> b(n);
            if (n && fread(b.data(), 1, n, fp) != n) return 2;
            bad += check(b, tb, st, "file");
            cases++;
        }
        report(argv[1], cases, bad, st);
        return bad ? 1 : 0;
    }
    const int reps = argc > 1 ? atoi(argv[1]) : 200;
    std::mt19937_64 rng(12345);
    // byte codes: code b has value (int8(b) + 128)/255, so u = b ^ 0x80 is the value index
    auto code = [](int u) { return (uint8_t)(u ^ 0x80); };
    for (int rep = 0; rep < reps; rep++) {
        const int kind = rep % 10;
        uint64_t n;
        if (rep % 5 == 0) n = 1 + rng() % 50;
        else if (rep % 5 == 1) n = 1 + rng() % 5000;
        else if (rep % 5 == 2) n = 1 + rng() % 200000;
        else n = 1 + rng() % 600000;
        std::vector<uint8_t> b(n);
        const int lo = (int)(rng() % 256), span = 1 + (int)(rng() % 40);
        const uint64_t period = 50 + rng() % 20000;
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
            case 7: u = (int)(64 + rng() % 64); break;                               // [0.25, 0.5)
            case 8: u = ((i / period) % 2) ? (int)(rng() % 4) : (int)(128 + rng() % 128); break;   // dark/bright regions
            default: u = ((i / period) % 3 == 0) ? 0 : ((i / period) % 3 == 1) ? (int)(rng() % 6) : 255; break;
            }
            b[i] = code(u);
        }
        char what[64];
        snprintf(what, sizeof(what), "rep %d kind %d", rep, kind);
        bad += check(b, tb, st, what);
        cases++;
    }
    report("random", cases, bad, st);
    return bad ? 1 : 0;
}
