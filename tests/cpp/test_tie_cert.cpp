// CPU check of the tie certificate (quant_amd/csrc/kdtree.cpp: near_set, certified_search,
// certify_tie): for each level of a reference run, the tree over the exact-sum split answers the
// tie band's rows with the reference's (Kahan-bit) split known only on the candidates' rows;
// every answer it gives must be the reference's index.  Prints one summary line per level and a
// total; exit status 1 on a wrong answer or a coordinate off by more than delta.
//   test_tie_cert levels.bin
// file: per level [u32 K][u32 D][u32 n] exact split (K x D f64) | Kahan split (K x D f64) |
//       rows (n x D f64) | the reference's indices (n u32)
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "kdtree.hpp"

using namespace qvq;

int main(int argc, char **argv) {
    if (argc < 2) return 2;
    FILE *fp = fopen(argv[1], "rb");
    if (!fp) return 2;
    const double delta = std::ldexp(1.0, -49);   // engine.cpp: the per-component bound
    long tot_rows = 0, tot_cert = 0, tot_wrong = 0, tot_multi = 0, bad_delta = 0;
    for (int level = 0;; level++) {
        uint32_t hdr[3];
        if (fread(hdr, 4, 3, fp) != 3) break;
        const uint32_t K = hdr[0], D = hdr[1], n = hdr[2];
        std::vector<double> ex((size_t)K * D), ka((size_t)K * D), q((size_t)n * D);
        std::vector<uint32_t> want(n);
        if (fread(ex.data(), 8, ex.size(), fp) != ex.size() || fread(ka.data(), 8, ka.size(), fp) != ka.size() ||
            fread(q.data(), 8, q.size(), fp) != q.size() || fread(want.data(), 4, n, fp) != n)
            return 2;
        // coordinates the reference's bits equal without computing them: a cell's exact mean is
        // 0 or 1 only when all its values are (SCALED values lie in [0, 1]; Kahan sums of 0s and
        // 1s are exact), and the split scales it by 1.2 or 0.8 (engine: tie_cert_known)
        std::vector<double> kp(ex);   // the reference's split where known
        std::vector<uint8_t> known((size_t)K * D, 0);
        for (size_t i = 0; i < ex.size(); i++) {
            const double u = i / D < K / 2 ? 1 + 0.2 : 1 - 0.2;
            known[i] = ex[i] == 0 || std::fabs(ex[i] - u) <= 1e-14;
            if (!(std::fabs(ex[i] - ka[i]) <= (known[i] ? 0.0 : delta))) bad_delta++;
        }
        RefKDTree tree(ex.data(), K, (int)D);
        std::vector<uint32_t> cand;
        long cert = 0, wrong = 0, multi = 0, cells = 0;
        // the engine's order (engine.cpp certify_rows): short searches replay every row at once,
        // long ones (48-D) first list each row's candidates and replay at once only rows whose
        // candidates are all known; for the others (and those left open), one
        // round: the parent cells (both split rows of each) of the candidates and of the points
        // a collecting replay blames, from the reference's sums, then the replay again
        const auto t0 = std::chrono::steady_clock::now();
        std::vector<uint32_t> blame, ready, pend, left;
        std::vector<int64_t> got(n, -1);
        std::vector<std::vector<uint32_t>> cands(n);
        auto all_known = [&](uint32_t j) {
            for (uint32_t d = 0; d < D; d++)
                if (!known[(size_t)j * D + d]) return false;
            return true;
        };
        const bool long_search = (uint64_t)K * D >= 65536;   // (near_set first)
        for (uint32_t r = 0; r < n; r++) {
            bool k = true;
            if (long_search) {
                double dmin;
                tree.near_set(q.data() + (size_t)r * D, 1e-9, 1e-9, cands[r], dmin);
                for (uint32_t j : cands[r]) k = k && all_known(j);
            }
            (k ? ready : pend).push_back(r);
        }
        for (uint32_t r : ready)
            if ((got[r] = tree.certified_search(q.data() + (size_t)r * D, delta, kp.data(), known.data())) < 0) {
                pend.push_back(r);
                if (!long_search) {
                    double dmin;
                    tree.near_set(q.data() + (size_t)r * D, 1e-9, 1e-9, cands[r], dmin);
                }
            }
        std::vector<uint32_t> changed;
        auto need = [&](uint32_t j) {
            if (all_known(j)) return;
            const uint32_t par = j % (K / 2);
            for (uint32_t s : {par, par + K / 2}) {
                std::memcpy(&kp[(size_t)s * D], &ka[(size_t)s * D], D * 8);
                std::memset(&known[(size_t)s * D], 1, D);
                changed.push_back(s);
            }
            cells++;
        };
        if (!getenv("TIE_CERT_NO_BLAME"))
            for (uint32_t r : pend) tree.certify_blame(q.data() + (size_t)r * D, delta, kp.data(), known.data(), blame);
        for (uint32_t r : pend)
            for (uint32_t j : cands[r]) need(j);
        for (uint32_t j : blame) need(j);
        tree.cert_update(changed.data(), changed.size());   // kp / known changed on these rows
        for (uint32_t r : pend) got[r] = tree.certified_search(q.data() + (size_t)r * D, delta, kp.data(), known.data());
        const auto t1 = std::chrono::steady_clock::now();
        for (uint32_t r = 0; r < n; r++) {
            if (got[r] < 0) {
                if (getenv("TIE_CERT_VERBOSE")) printf("undecided level %d row %u want %u\n", level, r, want[r]);
                continue;
            }
            cert++;
            if ((uint32_t)got[r] != want[r]) {
                wrong++;
                if (wrong <= 5) printf("WRONG level %d row %u: got %lld want %u\n", level, r, (long long)got[r], want[r]);
            }
        }
        const auto t2 = std::chrono::steady_clock::now();
        // rows whose candidates tie exactly under the reference's bits
        for (uint32_t r = 0; r < n; r++) {
            const double *x = q.data() + (size_t)r * D;
            double dmin;
            tree.near_set(x, 1e-9, 1e-9, cand, dmin);
            double best = INFINITY;
            int at = 0;
            for (uint32_t j : cand) {
                const double d = ref_l2(x, ka.data() + (size_t)j * D, (int)D);
                if (d < best) best = d, at = 1;
                else if (d == best) at++;
            }
            multi += at > 1;
        }
        printf("level K %u: rows %u certified %ld wrong %ld exact ties %ld cells computed %ld (host %.3f + %.3f ms)\n",
               K, n, cert, wrong, multi, cells, std::chrono::duration<double, std::milli>(t1 - t0).count(),
               std::chrono::duration<double, std::milli>(t2 - t1).count());
        tot_rows += n;
        tot_cert += cert;
        tot_wrong += wrong;
        tot_multi += multi;
    }
    printf("total: rows %ld certified %ld wrong %ld exact ties %ld off by more than delta %ld\n", tot_rows, tot_cert,
           tot_wrong, tot_multi, bad_delta);
    return (tot_wrong || bad_delta) ? 1 : 0;
}
