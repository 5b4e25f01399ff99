// kahan_par.hpp -- the reference's Kahan centroid chains (sumInArea, src/Quantizer.cpp:59-70),
// evaluated exactly and in parallel over segments of each chain.  Host and device code.
//
// The fast path sums centroids exactly (order-free 2^-60 integers).  The reference sums each
// (code vector, component) chain with Kahan's compensation in ascending row order, and that
// result can sit one ulp away from the exact sum.  On levels where a row's answer can depend on
// that ulp (the kd-tree tie band), the engine recomputes the previous level's centroids with the
// reference's bits; this file is the arithmetic.
//
// The model (SCALED values: every value is a multiple of 2^-60 in [0, 1]; "units" below):
//  * Once sum >= 2, the state (sum, c) is exactly E = sum - c, an integer number of units, with
//    sum = RN(E).  One reference step (y = x - c; t = sum + y; c = (t - sum) - y; sum = t) is
//        E' = E + X + delta,   delta = RN_g(X + r) - (X + r),   r = E - RN(E),
//    where g is the rounding grid of X's binade (2^lg units, lg = 0..7 for x < 1): delta depends
//    only on F = E mod 512 (ties to even read one bit above the grid; ulp(sum) >= 512 units).
//    x = 1.0 is the exception: X + r rounds to 256 units when r >= 0 and to 128 below, so that
//    step also depends on the sign of r, i.e. on E mod ulp(sum) -- a "decision".
//  * Before sum reaches 2 the chain runs in doubles (the transient, evaluated serially).
//  * A step of grid 2^g leaves E == 0 mod 2^g ("collapse"), and a later step of a finer grid
//    does not look at bits >= g: after an anchor of grade c, E = A + 2^c q with A determined by
//    the steps since the anchor and q unknown ("class").  A segment's function therefore needs
//    one entry per value of the input class bits its steps read: 2^lne entries, lne =
//    max(0, G + 1 - c_in) (G: the segment's highest grade read, 8 for x = 1.0), and bits above
//    pass through.  Each entry records the segment's sum of deltas; decisions add an interval of
//    the input D = E - P (P: the exact prefix sum) inside which every decision holds.
//  * Segments are L steps; the class structure at a segment's start is the anchor of the
//    previous segment (its last step of the highest collapse grade) plus that segment's tail.
//  * Functions compose (the classes of the composite are the first function's), so a block of
//    64 segments becomes one function; a chain is evaluated from its start: the transient in
//    doubles, then block functions, each checked (input class structure, D inside the
//    interval), and where a check fails (or a segment has more than NE entries) the block's
//    segments or steps are replayed with the exact state.  The checks make the result exact.
#pragma once
#include <cmath>
#include <cstdint>

#include "kdtree_dev.hpp"   // QVQ_HD

namespace qvq {
namespace kahan {

typedef unsigned __int128 u128;
typedef __int128 i128;

constexpr uint32_t L = 64;               // steps per segment
constexpr uint32_t SPB = 64;             // segments per block
constexpr int NE = 16;                   // entries per function (lne <= 4)
constexpr int64_t DLIM = 1ll << 30;      // |D| inside every table interval
constexpr u128 MIN_STATE = (u128)1 << 61;   // sum >= 2
constexpr uint64_t ONE = 1ull << 60;      // x = 1.0

// Per byte value: X in units; the step's parameters packed in one word:
//   bits 0..40  X mod 2^41 (the running prefix for decisions: ulp(sum) <= 2^40 units)
//   bits 41..49 X mod 512
//   bits 50..54 parity shift (lg; 31 for exact steps, 8 for x = 1.0 -- unused there)
//   bits 55..61 hm1 = 2^(lg-1) - 1 (0 for exact steps)
//   bit  62     x = 1.0
// plus the anchor grade cg (-1: none) and the dependence grade dg (-1: none; 8 for x = 1.0).
struct ByteTab {
    uint64_t X[256];
    uint64_t pk[256];
    int8_t cg[256], dg[256];
};
QVQ_HD inline int bitlen(u128 v) {
    const uint64_t hi = (uint64_t)(v >> 64), lo = (uint64_t)v;
#if defined(__HIP_DEVICE_COMPILE__)
    return hi ? 128 - __clzll((long long)hi) : (lo ? 64 - __clzll((long long)lo) : 0);
#else
    return hi ? 128 - __builtin_clzll(hi) : (lo ? 64 - __builtin_clzll(lo) : 0);
#endif
}
QVQ_HD inline void make_tab(const uint64_t *X, ByteTab &t) {
    for (int b = 0; b < 256; b++) {
        const uint64_t x = X[b];
        int lg;   // grid exponent; -1: the step is exact (x = 0, or x < 2^-7: grid 1 unit)
        if (x == ONE) lg = 8;
        else if (x == 0) lg = -1;
        else lg = bitlen((u128)x) - 53 > 0 ? bitlen((u128)x) - 53 : -1;
        const uint64_t sh = lg < 0 ? 31 : (uint64_t)lg;
        const uint64_t hm1 = lg > 0 && lg < 8 ? (1ull << (lg - 1)) - 1 : 0;
        t.X[b] = x;
        t.pk[b] = (x & ((1ull << 41) - 1)) | ((x & 511) << 41) | (sh << 50) | (hm1 << 55) | ((uint64_t)(lg == 8) << 62);
        t.cg[b] = (int8_t)(lg == 8 ? 7 : lg);
        t.dg[b] = (int8_t)lg;
    }
}

// t rounded to a multiple of 2^lg, ties to even (lg >= 1)
QVQ_HD inline uint32_t rnd(uint32_t t, uint32_t lg) {
    return (t + ((1u << (lg - 1)) - 1) + ((t >> lg) & 1)) & ~((1u << lg) - 1);
}

// ---- one trajectory ------------------------------------------------------------------------
// Steps b[0..n) from E = P + D0 with E mod 512 = F (the caller's class representative).  bl0:
// the binade of every E on the way (0: compute it at each decision from the exact E).  Out: the
// final F, the sum of deltas, and [lo, hi] narrowed to the input D for which every decision
// would be the same.
template <bool EXACT_BL>
QVQ_HD inline void sim(const ByteTab &tb, const uint8_t *b, uint32_t n, u128 P, int bl0, uint32_t &F, int64_t D0,
                       int32_t &dsum, int64_t &lo, int64_t &hi) {
    uint64_t q = (uint64_t)P;
    u128 Pj = P;
    int32_t d = 0;
    for (uint32_t i = 0; i < n; i++) {
        const uint8_t c = b[i];
        const uint64_t pk = tb.pk[c];
        if (pk >> 62) {   // x = 1.0: a decision
            const uint64_t E64 = q + (uint64_t)(D0 + d);
            int bl = bl0;
            if (EXACT_BL) bl = bitlen(Pj + (u128)(i128)(D0 + d));
            const int su = bl - 53;
            const uint64_t U = 1ull << su, h = U >> 1, e = E64 & (U - 1);
            const bool pos = e < h || (e == h && !((E64 >> su) & 1));
            const uint32_t r8 = rnd(F, 8), r7 = rnd(F, 7), r = pos ? r8 : r7;
            if (r8 != r7) {
                int64_t l, u;
                if (e == h) l = u = 0;
                else if (pos) l = -(int64_t)e, u = (int64_t)(h - 1 - e);
                else l = (int64_t)(h + 1 - e), u = (int64_t)(U - 1 - e);
                if (EXACT_BL) {   // the shift must also keep E in its binade
                    const i128 E = (i128)(Pj + (u128)(i128)(D0 + d));
                    const i128 bl_lo = ((i128)1 << (bl - 1)) - E, bl_hi = ((i128)1 << bl) - 1 - E;
                    if (bl_lo > (i128)l) l = bl_lo > (i128)DLIM ? DLIM : (int64_t)bl_lo;
                    if (bl_hi < (i128)u) u = bl_hi < -(i128)DLIM ? -DLIM : (int64_t)bl_hi;
                }
                if (D0 + l > lo) lo = D0 + l;
                if (D0 + u < hi) hi = D0 + u;
            }
            d += (int32_t)r - (int32_t)F;
            F = r & 511;
        } else {
            const uint32_t t = F + (uint32_t)((pk >> 41) & 511), sh = (uint32_t)((pk >> 50) & 31);
            const uint32_t hm1 = (uint32_t)((pk >> 55) & 127);
            const uint32_t m = ~(2 * hm1 + 1);   // exact steps: hm1 = 0 -> ~1, but the parity bit is 0 and t & ~1 ...
            uint32_t r;
            if (sh == 31) r = t;   // exact step
            else r = (t + hm1 + ((t >> sh) & 1)) & ~((1u << sh) - 1);
            (void)m;
            d += (int32_t)r - (int32_t)t;
            F = r & 511;
        }
        q += tb.X[c];
        if (EXACT_BL) Pj += tb.X[c];
    }
    dsum = d;
}

// The binade of every state E in [P - DLIM, P + S + DLIM] (S: the steps' sum), or 0 when they
// straddle a power of two.
QVQ_HD inline int fixed_binade(u128 P, u128 S) {
    const int a = bitlen(P - (u128)DLIM), b = bitlen(P + S + (u128)DLIM);
    return a == b ? a : 0;
}

// ---- functions -------------------------------------------------------------------------------
enum : uint8_t { FK_TRANS = 0, FK_TABLE = 1, FK_RAW = 2 };
constexpr uint8_t FK_FINAL = 0x80;   // flag: the function runs to the chain's end

// A function from a segment start to a later boundary.  TABLE: input F == off_in (mod 2^c_in);
// entry e = ((F - off_in) mod 512 >> c_in) & (2^lne - 1); D_in must lie in [lo, hi]; out:
// D += dlt[e], F += sx9 + dlt[e] (mod 512), and F == off_out (mod 2^c_out).  TRANS: F += sx9
// (no class reads, no decisions).  RAW: not tabulated (the evaluation replays it).
struct Fn {
    uint8_t kind, c_in, lne, c_out;
    uint16_t off_in, off_out, sx9, pad;
    int32_t lo, hi;
    int32_t dlt[NE];
};

QVQ_HD inline uint8_t fkind(const Fn &f) { return f.kind & 0x7F; }
QVQ_HD inline void set_raw(Fn &f) {
    f.kind = FK_RAW;
    f.c_in = f.lne = f.c_out = 0;
    f.off_in = f.off_out = f.sx9 = f.pad = 0;
    f.lo = 1;
    f.hi = 0;
}

// Apply f to (F, D).  false: f cannot answer this input (RAW, class structure, interval).
QVQ_HD inline bool apply(const Fn &f, uint32_t &F, int64_t &D) {
    const uint8_t k = fkind(f);
    if (k == FK_TRANS) {
        F = (F + f.sx9) & 511;
        return true;
    }
    if (k != FK_TABLE) return false;
    const uint32_t rel = (F - f.off_in) & 511;
    if (rel & ((1u << f.c_in) - 1)) return false;
    if (D < (int64_t)f.lo || D > (int64_t)f.hi) return false;
    const int e = (int)((rel >> f.c_in) & ((1u << f.lne) - 1));
    D += f.dlt[e];
    F = (F + f.sx9 + (uint32_t)f.dlt[e]) & 511;
    return true;
}

// h = g after f (f's steps first).  false: not representable (RAW, class structures that do
// not meet, more than NE entries).
QVQ_HD inline bool compose(const Fn &f, const Fn &g, Fn &h) {
    const uint8_t kf = fkind(f), kg = fkind(g);
    const uint8_t fin = (uint8_t)((f.kind | g.kind) & FK_FINAL);
    if (kf == FK_RAW || kg == FK_RAW) return false;
    if (kf == FK_TRANS && kg == FK_TRANS) {
        h = f;
        h.sx9 = (uint16_t)((f.sx9 + g.sx9) & 511);
        h.kind = (uint8_t)(FK_TRANS | fin);
        return true;
    }
    if (kf == FK_TRANS) {   // translate g's input
        h = g;
        h.off_in = (uint16_t)((g.off_in - f.sx9) & 511);
        h.sx9 = (uint16_t)((f.sx9 + g.sx9) & 511);
        h.kind = (uint8_t)(FK_TABLE | fin);
        return true;
    }
    if (kg == FK_TRANS) {   // translate f's output
        h = f;
        h.off_out = (uint16_t)((f.off_out + g.sx9) & 511);
        h.sx9 = (uint16_t)((f.sx9 + g.sx9) & 511);
        h.kind = (uint8_t)(FK_TABLE | fin);
        return true;
    }
    // f's output structure must refine g's input structure
    if (f.c_out < g.c_in || ((f.off_out - g.off_in) & ((1u << g.c_in) - 1))) return false;
    int lne = f.lne;
    if ((int)g.c_in + g.lne - (int)f.c_in > lne) lne = (int)g.c_in + g.lne - (int)f.c_in;
    if (lne > 4) return false;
    h.kind = (uint8_t)(FK_TABLE | fin);
    h.c_in = f.c_in;
    h.lne = (uint8_t)lne;
    h.c_out = g.c_out;
    h.off_in = f.off_in;
    h.off_out = g.off_out;
    h.sx9 = (uint16_t)((f.sx9 + g.sx9) & 511);
    h.pad = 0;
    int64_t lo = f.lo, hi = f.hi;
    const uint32_t mf = (1u << f.lne) - 1, mg = (1u << g.lne) - 1;
    for (int e = 0; e < (1 << lne); e++) {
        const uint32_t F0 = (f.off_in + ((uint32_t)e << f.c_in)) & 511;
        const int32_t d1 = f.dlt[e & mf];
        const uint32_t F1 = (F0 + f.sx9 + (uint32_t)d1) & 511;
        const int32_t d2 = g.dlt[(((F1 - g.off_in) & 511) >> g.c_in) & mg];
        h.dlt[e] = d1 + d2;
        if ((int64_t)g.lo - d1 > lo) lo = (int64_t)g.lo - d1;
        if ((int64_t)g.hi - d1 < hi) hi = (int64_t)g.hi - d1;
    }
    for (int e = 1 << lne; e < NE; e++) h.dlt[e] = 0;
    h.lo = (int32_t)(lo < -DLIM ? -DLIM : lo);
    h.hi = (int32_t)(hi > DLIM ? DLIM : hi);
    if (h.lo > h.hi) h.lo = 1, h.hi = 0;   // never answers (every input re-walked)
    return true;
}

// ---- per-segment metadata (one pass over the steps) ------------------------------------------
// cmax: the highest anchor grade (-1: every step is exact); off: E mod 2^cmax at the segment's
// end relative to its last anchor (the tail's steps are finer, so deterministic); G: the
// highest grade any step reads; S: the exact sum of X.
struct SegMeta {
    uint64_t s_lo;
    uint8_t s_hi;
    int8_t cmax, G;
    uint8_t pad;
    uint16_t off, sx9;
};
QVQ_HD inline SegMeta seg_meta(const ByteTab &tb, const uint8_t *b, uint32_t n) {
    SegMeta m;
    int cmax = -1, G = -1;
    uint32_t apos = 0;
    u128 s = 0;
    for (uint32_t i = 0; i < n; i++) {
        const uint8_t c = b[i];
        if (tb.cg[c] >= cmax && tb.cg[c] >= 0) cmax = tb.cg[c], apos = i;
        if (tb.dg[c] > G) G = tb.dg[c];
        s += tb.X[c];
    }
    uint32_t F = 0;
    if (cmax >= 0)
        for (uint32_t i = apos + 1; i < n; i++) {   // grades below cmax: no decisions, no class reads
            const uint64_t pk = tb.pk[b[i]];
            const uint32_t t = F + (uint32_t)((pk >> 41) & 511), sh = (uint32_t)((pk >> 50) & 31);
            const uint32_t hm1 = (uint32_t)((pk >> 55) & 127);
            F = sh == 31 ? t : (t + hm1 + ((t >> sh) & 1)) & ~((1u << sh) - 1);
            F &= (1u << cmax) - 1;
        }
    m.s_lo = (uint64_t)s;
    m.s_hi = (uint8_t)(s >> 64);
    m.cmax = (int8_t)cmax;
    m.G = (int8_t)G;
    m.pad = 0;
    m.off = (uint16_t)F;
    m.sx9 = (uint16_t)(s & 511);
    return m;
}
QVQ_HD inline u128 meta_sum(const SegMeta &m) { return ((u128)m.s_hi << 64) | m.s_lo; }

// ---- building a segment's function -------------------------------------------------------------
// Segment j of a chain (n_j steps at b, exact prefix P at its start).  prev[-i] (i = 1..nprev) are
// the metadata of the preceding segments (nearest first); final: the chain's last segment.
// D_est: the estimate of the input D that decides the x = 1.0 steps (any value is safe).
QVQ_HD inline void build_fn(const ByteTab &tb, const uint8_t *b, uint32_t n, u128 P, const SegMeta &self,
                            const SegMeta *prev, int nprev, bool final, int64_t D_est, Fn &f) {
    f.pad = 0;
    for (int e = 0; e < NE; e++) f.dlt[e] = 0;
    if (self.G < 0) {   // every step exact: a translation
        f.kind = (uint8_t)(FK_TRANS | (final ? FK_FINAL : 0));
        f.c_in = f.lne = f.c_out = 0;
        f.off_in = f.off_out = 0;
        f.sx9 = self.sx9;
        f.lo = -(int32_t)DLIM;
        f.hi = (int32_t)DLIM;
        return;
    }
    // the input class structure: the nearest preceding segment with an anchor, translated by the
    // exact segments in between
    int c_in = -1;
    uint32_t off_in = 0, trans = 0;
    for (int i = 0; i < nprev; i++) {
        const SegMeta &m = prev[i];
        if (m.cmax >= 0) {
            c_in = m.cmax;
            off_in = (m.off + trans) & 511;
            break;
        }
        trans += m.sx9;
    }
    const int bl0 = fixed_binade(P, meta_sum(self));
    if (c_in < 0 || P < MIN_STATE + (u128)DLIM) {
        set_raw(f);
        return;
    }
    const int lne = self.G + 1 - c_in > 0 ? self.G + 1 - c_in : 0;
    if (lne > 4) {
        set_raw(f);
        return;
    }
    f.kind = (uint8_t)(FK_TABLE | (final ? FK_FINAL : 0));
    f.c_in = (uint8_t)c_in;
    f.lne = (uint8_t)lne;
    f.c_out = (uint8_t)(self.cmax >= 0 ? self.cmax : c_in);
    f.off_in = (uint16_t)(off_in & ((1u << c_in) - 1));
    f.sx9 = self.sx9;
    int64_t lo = -DLIM, hi = DLIM;
    for (int e = 0; e < (1 << lne); e++) {
        uint32_t F = (f.off_in + ((uint32_t)e << c_in)) & 511;
        // the representative input D: D == F - P (mod 512), next to D_est
        const int64_t D0 = D_est + (int64_t)(((F - (uint32_t)(uint64_t)P - (uint32_t)D_est + 256) & 511)) - 256;
        int32_t ds;
        if (bl0) sim<false>(tb, b, n, P, bl0, F, D0, ds, lo, hi);
        else sim<true>(tb, b, n, P, 0, F, D0, ds, lo, hi);
        f.dlt[e] = ds;
        if (e == 0) f.off_out = (uint16_t)(F & (f.c_out < 9 ? (1u << f.c_out) - 1 : 511));
    }
    // the output structure: the segment's own anchor, or (no anchor) the input's, carried
    if (self.cmax >= 0) f.off_out = self.off;
    else f.off_out = (uint16_t)((f.off_in + self.sx9 + (uint32_t)f.dlt[0]) & ((1u << c_in) - 1));
    f.lo = (int32_t)lo;
    f.hi = (int32_t)hi;
    if (f.lo > f.hi) f.lo = 1, f.hi = 0;
}

// ---- the transient and the final rounding -------------------------------------------------------
QVQ_HD inline void fstep(double &sum, double &c, double x) {
#if defined(__HIP_DEVICE_COMPILE__)
    const double y = __dsub_rn(x, c);
    const double t = __dadd_rn(sum, y);
    c = __dsub_rn(__dsub_rn(t, sum), y);
#else
    const double y = x - c;
    const double t = sum + y;
    c = (t - sum) - y;
#endif
    sum = t;
}
// A double on the 2^-60 grid (|v| < 2^67) in units.
QVQ_HD inline i128 to_units(double v) {
    if (v == 0) return 0;
    const bool neg = v < 0;
    const double a = neg ? -v : v;
    const uint64_t bits = __builtin_bit_cast(uint64_t, a);
    const int ex = (int)((bits >> 52) & 0x7FF);
    const uint64_t man = (bits & ((1ull << 52) - 1)) | (ex ? (1ull << 52) : 0);
    const int sh = (ex ? ex : 1) - 1075 + 60;
    const u128 m = sh >= 0 ? (u128)man << sh : (u128)(man >> -sh);
    return neg ? -(i128)m : (i128)m;
}
// RN(E) as a double (E >= 0)
QVQ_HD inline double to_double(u128 E) {
    const int bl = bitlen(E);
    if (bl <= 53) return ldexp((double)(uint64_t)E, -60);
    const int sh = bl - 53;
    const u128 U = (u128)1 << sh, rem = E & (U - 1), half = U >> 1;
    u128 base = E - rem;
    if (rem > half || (rem == half && ((base >> sh) & 1))) base += U;
    const int bl2 = bitlen(base);
    const int sh2 = bl2 > 53 ? bl2 - 53 : 0;
    return ldexp((double)(uint64_t)(base >> sh2), sh2 - 60);
}

// The reference's steps in doubles from the chain's start until sum >= 2 (or the end).  Returns
// the steps taken; P = their exact sum; E = sum - c in units (valid when sum >= 2).
QVQ_HD inline uint32_t transient(const ByteTab &tb, const uint8_t *b, uint32_t n, double &sum, u128 &P, u128 &E) {
    double c = 0;
    sum = 0;
    P = 0;
    uint32_t i = 0;
    while (i < n && !(sum >= 2.0)) {
        fstep(sum, c, ldexp((double)tb.X[b[i]], -60));
        P += tb.X[b[i]];
        i++;
    }
    E = sum >= 2.0 ? (u128)(to_units(sum) - to_units(c)) : 0;
    return i;
}

}  // namespace kahan
}  // namespace qvq
