// kahan_par.hpp -- the reference's Kahan centroid chains (sumInArea, src/Quantizer.cpp:59-70),
// evaluated exactly and in parallel over segments of a chain.
//
// The fast path sums centroids exactly (order-free 2^-60 integers).  The reference sums each
// (code vector, component) chain with Kahan's compensation, in ascending row order, and that
// result can sit one ulp away from the exact sum.  On levels where a row's decision depends on
// that ulp (the kd-tree tie band), the engine recomputes the previous level's centroids with
// the reference's bits; this file is the arithmetic.
//
// The model (SCALED values only: every value is v = k/255 rounded, a multiple of 2^-60 in
// [0, 1]; NORMAL values are integers and their Kahan sums are exact):
//  * A Kahan state (sum, c) with sum >= 2 is exactly E = sum - c, an integer in units of
//    2^-60: every later y = x - c has |y| < 2 <= sum, so (t - sum) - y is the exact rounding
//    error of sum + y (Fast2Sum) and sum = RN(E), c = RN(E) - E.  One step is then
//        s = RN(E), r = E - s, y = RN(X + r), E' = s + y          (step(), integers)
//    which is the reference's four double operations, exactly.  Before sum reaches 2 the
//    chain runs in doubles (the transient).
//  * step() commutes with shifts of E by multiples of 512 (= 2 ulp(2)), as long as the sign
//    of r at each x = 1.0 step is unchanged (y = RN(1 + r) rounds to 2^-52 when r > 0 and to
//    2^-53 below).  Every other step's rounding depends only on E mod 512.
//  * After a step with x >= 0.5 (a "collapse" step) E is a multiple of 128: E mod 512 is one
//    of 4 classes q.  A segment of a chain is therefore summarised by: its head (the steps
//    through its first collapse step, replayed at evaluation), and per class q the state
//    increment T[q] to the segment's end, valid while err = E_true - (B + 128 q) stays in
//    [lo[q], hi[q]] -- B is the estimate of the state at the collapse point the table was
//    built from, the interval the set of shifts that keep every x = 1.0 decision the same.
//  * Segment functions compose (groups of segments, groups of groups) in the same form, and a
//    chain is evaluated exactly from its start: the transient in doubles, then the functions,
//    each one checked (head replayed exactly, err inside the interval) and, where the check
//    fails, its children or its steps replayed exactly.  The check is what makes the result
//    exact; the estimates only decide how often it passes.
#pragma once
#include <cmath>
#include <cstdint>

#include "kdtree_dev.hpp"   // QVQ_HD

namespace qvq {
namespace kahan {

typedef unsigned __int128 u128;
typedef __int128 i128;

constexpr uint64_t ONE = 1ull << 60;    // x = 1.0 in units of 2^-60
constexpr uint64_t HALF = 1ull << 59;   // x = 0.5: steps with x >= 0.5 collapse E mod 128
constexpr int64_t I64_MIN = (int64_t)(1ull << 63);
constexpr int64_t I64_MAX = (int64_t)((1ull << 63) - 1);
constexpr u128 MIN_STATE = (u128)1 << 61;   // sum >= 2

QVQ_HD inline int bitlen(u128 v) {
    const uint64_t hi = (uint64_t)(v >> 64), lo = (uint64_t)v;
#if defined(__HIP_DEVICE_COMPILE__)
    return hi ? 128 - __clzll((long long)hi) : (lo ? 64 - __clzll((long long)lo) : 0);
#else
    return hi ? 128 - __builtin_clzll(hi) : (lo ? 64 - __builtin_clzll(lo) : 0);
#endif
}

// v rounded to 53 significant bits, ties to even (a positive integer's double value)
QVQ_HD inline u128 rn53(u128 v) {
    const int bl = bitlen(v);
    if (bl <= 53) return v;
    const int sh = bl - 53;
    const u128 U = (u128)1 << sh, rem = v & (U - 1), half = U >> 1;
    u128 base = v - rem;
    if (rem > half || (rem == half && ((base >> sh) & 1))) base += U;
    return base;
}

// One Kahan step of the model (E >= MIN_STATE): y = x - c, t = sum + y, c = (t - sum) - y, sum = t.
QVQ_HD inline u128 step(u128 E, uint64_t X) {
    const u128 s = rn53(E);
    const i128 r = (i128)(E - s);   // |r| <= ulp(sum) / 2
    const i128 v = (i128)X + r;
    const u128 y = v >= 0 ? rn53((u128)v) : (u128)v;   // v < 0 only when X == 0: |r| < 2^53, exact
    return s + y;                                       // modulo 2^128: a negative y subtracts
}

// The reference's step in doubles (the transient, sum < 2).  Device code uses the _rn
// intrinsics so that no contraction or reassociation can touch it.
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

// A double on the 2^-60 grid (|v| < 2^67) in units of 2^-60.
QVQ_HD inline i128 to_units(double v) {
    if (v == 0) return 0;
    const bool neg = v < 0;
    const double a = neg ? -v : v;
    const uint64_t bits = __builtin_bit_cast(uint64_t, a);
    const int ex = (int)((bits >> 52) & 0x7FF);
    const uint64_t man = (bits & ((1ull << 52) - 1)) | (ex ? (1ull << 52) : 0);
    const int sh = (ex ? ex : 1) - 1075 + 60;   // a = man * 2^(ex - 1075)
    const u128 m = sh >= 0 ? (u128)man << sh : (u128)(man >> -sh);
    return neg ? -(i128)m : (i128)m;
}

// RN(E) as a double (E > 0)
QVQ_HD inline double to_double(u128 E) {
    const u128 s = rn53(E);
    const int bl = bitlen(s);
    const int sh = bl > 53 ? bl - 53 : 0;
    return ldexp((double)(uint64_t)(s >> sh), sh - 60);   // exact: the mantissa has <= 53 bits
}

// The interval of shifts err (multiples of 512) of a state E >= MIN_STATE that keep the sign
// of r = E - RN(E) -- the decision at an x = 1.0 step -- and the binade of E, intersected into
// [lo, hi].  Conservative: the decision boundaries themselves are excluded.
QVQ_HD inline void margin(u128 E, int64_t &lo, int64_t &hi) {
    const int bl = bitlen(E);
    const int sh = bl - 53;   // >= 9
    const i128 U = (i128)1 << sh, H = U >> 1;
    const i128 m = (i128)(E & (u128)(U - 1));
    i128 l, u;
    if (m == 0) {
        l = -(H - 1);
        u = 0;
    } else if (m < H) {
        l = -(m - 1);
        u = H - 1 - m;
    } else if (m == H) {
        l = 0;
        u = 0;
    } else {
        l = H + 1 - m;
        u = U - m;
    }
    const i128 lb = (i128)((u128)1 << (bl - 1)) - (i128)E, ub = (i128)((u128)1 << bl) - 1 - (i128)E;
    if (l < lb) l = lb;
    if (u > ub) u = ub;
    if (l > (i128)lo) lo = l > (i128)I64_MAX ? I64_MAX : (int64_t)l;
    if (u < (i128)hi) hi = u < (i128)I64_MIN ? I64_MIN : (int64_t)u;
}

// Grid (ulp in units of 2^-60, as a shift) of a step's value: x in [2^-k, 2^-k+1) -> 2^(8-k);
// x = 1.0 -> 8 (its rounding also depends on the sign of r); x = 0 -> 0.
QVQ_HD inline uint32_t grid_shift(uint64_t X) {
    const int bl = bitlen((u128)X);
    return bl > 53 ? (uint32_t)(bl - 53) : 0u;
}

// A chain function over a range of steps: a segment, a group of segments, a group of groups.
//  FN_BRIGHT: the range has a step with x >= 0.5.  Its collapse point is after the first one;
//             class q = (E >> 7) & 3 there, T[q] valid while err in [lo[q], hi[q]].
//  FN_DARK (segments only): every x < 0.5.  The collapse point is after the first step with the
//             range's coarsest grid 2^gs; from there E mod 2^(gs+1) decides everything (no x = 1.0
//             decisions): class q = (E >> gs) & 1, T[q] valid for any err = 0 mod 2^(gs+1).
//  FN_SEQ (groups only): no bright child; the children are evaluated in turn.
// head: segments, the steps through the collapse step; groups, the child holding the collapse point.
enum : uint32_t { FN_SEQ = 0, FN_DARK = 1, FN_BRIGHT = 2 };
struct Fn {
    uint32_t kind, head, gs, pad;
    i128 B;             // state estimate at the collapse point (its class bits clear)
    i128 T[4];          // state increment from the collapse point to the range's end, per class
    int64_t lo[4], hi[4];
};

QVQ_HD inline void clamp_in(i128 l, i128 u, int64_t &lo, int64_t &hi) {
    if (l > (i128)lo) lo = l > (i128)I64_MAX ? I64_MAX : (int64_t)l;
    if (u < (i128)hi) hi = u < (i128)I64_MIN ? I64_MIN : (int64_t)u;
}

// The table of steps b[0, n) (X = Xt[b]): P_in is the exact sum of X before the range (over
// the whole chain), dest the estimate of E - P at the range's collapse point.
QVQ_HD inline Fn build_segment(const uint8_t *b, const uint64_t *Xt, uint32_t n, i128 P_in, int64_t dest) {
    Fn f;
    f.pad = 0;
    f.gs = 0;
    uint32_t h = 0;
    while (h < n && Xt[b[h]] < HALF) h++;
    uint32_t cls_shift = 7, ncls = 4;
    if (h == n) {   // dark: the first step with the coarsest grid
        uint32_t gs = 0;
        h = 0;
        for (uint32_t j = 0; j < n; j++) {
            const uint64_t X = Xt[b[j]];
            if (X && (grid_shift(X) > gs || (gs == 0 && Xt[b[h]] == 0))) {
                gs = grid_shift(X);
                h = j;
            }
        }
        f.kind = FN_DARK;
        f.gs = gs;
        cls_shift = gs;
        ncls = 2;
    } else {
        f.kind = FN_BRIGHT;
    }
    i128 P = P_in;
    for (uint32_t j = 0; j <= h && j < n; j++) P += (i128)Xt[b[j]];
    f.head = n ? h + 1 : 0;
    const i128 cmask = ((i128)ncls << cls_shift) - 1;   // class bits and below
    i128 B = (P + (i128)dest) & ~cmask;
    if (B < (i128)MIN_STATE) B = (i128)MIN_STATE;
    f.B = B;
    u128 E[4];
    for (uint32_t q = 0; q < 4; q++) {
        E[q] = (u128)(B + ((i128)(q % ncls) << cls_shift));
        f.lo[q] = q < ncls ? I64_MIN : 1;
        f.hi[q] = q < ncls ? I64_MAX : 0;
    }
    for (uint32_t j = f.head; j < n; j++) {
        const uint64_t X = Xt[b[j]];
        if (X == ONE)
            for (uint32_t q = 0; q < ncls; q++) margin(E[q], f.lo[q], f.hi[q]);
        for (uint32_t q = 0; q < ncls; q++) E[q] = step(E[q], X);
    }
    for (uint32_t q = 0; q < 4; q++) f.T[q] = q < ncls ? (i128)E[q] - (B + ((i128)q << cls_shift)) : 0;
    return f;
}

// A chain: its step bytes, the byte -> X table, and its functions at three levels -- segments
// of L steps, groups of S segments, supergroups of S groups (the last of each shorter).
struct Chain {
    const uint8_t *b;
    const uint64_t *Xt;
    uint64_t n;
    const Fn *f0, *f1, *f2;
    uint32_t L, S;
    QVQ_HD uint64_t X(uint64_t i) const { return Xt[b[i]]; }
    QVQ_HD uint64_t len0(uint64_t s) const { const uint64_t a = s * L; return n - a < L ? n - a : L; }
    QVQ_HD uint64_t len1(uint64_t g) const { const uint64_t a = g * L * S, GL = (uint64_t)L * S; return n - a < GL ? n - a : GL; }
    QVQ_HD uint64_t len2(uint64_t g) const { const uint64_t SL = (uint64_t)L * S * S, a = g * SL; return n - a < SL ? n - a : SL; }
    QVQ_HD uint32_t kids1(uint64_t g) const { return (uint32_t)((len1(g) + L - 1) / L); }
    QVQ_HD uint32_t kids2(uint64_t g) const { const uint64_t GL = (uint64_t)L * S; return (uint32_t)((len2(g) + GL - 1) / GL); }
};

// The class and error of a state at a function's collapse point.
QVQ_HD inline void classify(const Fn &f, u128 e, int &q, i128 &err) {
    const uint32_t sh = f.kind == FN_BRIGHT ? 7 : f.gs;
    q = (int)((e >> sh) & (f.kind == FN_BRIGHT ? 3 : 1));
    err = (i128)e - (f.B + ((i128)q << sh));
}

// ---- exact evaluation (the state E is the true one, >= MIN_STATE) ------------------------
// Segment s: replay its head, then the table if err is inside the class interval, else its steps.
QVQ_HD inline void eval0(const Chain &c, uint64_t s, u128 &E, uint32_t *miss) {
    const Fn &f = c.f0[s];
    const uint64_t a = s * c.L, n = c.len0(s);
    u128 e = E;
    for (uint32_t j = 0; j < f.head; j++) e = step(e, c.X(a + j));
    int q;
    i128 err;
    classify(f, e, q, err);
    if (f.kind == FN_DARK || (err >= (i128)f.lo[q] && err <= (i128)f.hi[q])) {
        E = e + (u128)f.T[q];
        return;
    }
    if (miss) miss[0]++;
    for (uint64_t j = f.head; j < n; j++) e = step(e, c.X(a + j));
    E = e;
}
// Group g: its leading children, the collapse child's head, the check; children on a miss.
QVQ_HD inline void eval1(const Chain &c, uint64_t g, u128 &E, uint32_t *miss) {
    const Fn &f = c.f1[g];
    const uint64_t s0 = g * c.S;
    const uint32_t nk = c.kids1(g);
    uint32_t i = 0;
    if (f.kind == FN_BRIGHT) {
        for (; i < f.head; i++) eval0(c, s0 + i, E, miss);
        const Fn &k = c.f0[s0 + i];
        const uint64_t a = (s0 + i) * c.L;
        u128 e = E;
        for (uint32_t j = 0; j < k.head; j++) e = step(e, c.X(a + j));
        int q;
        i128 err;
        classify(f, e, q, err);
        if (err >= (i128)f.lo[q] && err <= (i128)f.hi[q]) {
            E = e + (u128)f.T[q];
            return;
        }
        if (miss) miss[1]++;
    }
    for (; i < nk; i++) eval0(c, s0 + i, E, miss);
}
QVQ_HD inline void head1(const Chain &c, uint64_t g, u128 &e, uint32_t *miss) {   // to the group's collapse point
    const Fn &f = c.f1[g];
    const uint64_t s0 = g * c.S;
    for (uint32_t i = 0; i < f.head; i++) eval0(c, s0 + i, e, miss);
    const uint64_t a = (s0 + f.head) * c.L;
    for (uint32_t j = 0; j < c.f0[s0 + f.head].head; j++) e = step(e, c.X(a + j));
}
QVQ_HD inline void eval2(const Chain &c, uint64_t G, u128 &E, uint32_t *miss) {
    const Fn &f = c.f2[G];
    const uint64_t g0 = G * c.S;
    const uint32_t nk = c.kids2(G);
    uint32_t i = 0;
    if (f.kind == FN_BRIGHT) {
        for (; i < f.head; i++) eval1(c, g0 + i, E, miss);
        u128 e = E;
        head1(c, g0 + i, e, miss);
        int q;
        i128 err;
        classify(f, e, q, err);
        if (err >= (i128)f.lo[q] && err <= (i128)f.hi[q]) {
            E = e + (u128)f.T[q];
            return;
        }
        if (miss) miss[2]++;
    }
    for (; i < nk; i++) eval1(c, g0 + i, E, miss);
}

// ---- estimated evaluation (E carries an unknown shift err, a multiple of 512; [lo, hi]
// collects the err values for which every decision taken holds) ----------------------------
QVQ_HD inline void est_steps(const Chain &c, uint64_t a, uint64_t n, u128 &E, int64_t &lo, int64_t &hi) {
    for (uint64_t j = 0; j < n; j++) {
        const uint64_t X = c.X(a + j);
        if (X == ONE) margin(E, lo, hi);
        E = step(E, X);
    }
}
QVQ_HD inline void est0(const Chain &c, uint64_t s, u128 &E, int64_t &lo, int64_t &hi) {
    const Fn &f = c.f0[s];
    est_steps(c, s * c.L, f.head, E, lo, hi);
    int q;
    i128 err;
    classify(f, E, q, err);
    if (f.kind == FN_BRIGHT) clamp_in((i128)f.lo[q] - err, (i128)f.hi[q] - err, lo, hi);
    E += (u128)f.T[q];
}
QVQ_HD inline void est1(const Chain &c, uint64_t g, u128 &E, int64_t &lo, int64_t &hi) {
    const Fn &f = c.f1[g];
    const uint64_t s0 = g * c.S;
    const uint32_t nk = c.kids1(g);
    if (f.kind != FN_BRIGHT) {
        for (uint32_t i = 0; i < nk; i++) est0(c, s0 + i, E, lo, hi);
        return;
    }
    for (uint32_t i = 0; i < f.head; i++) est0(c, s0 + i, E, lo, hi);
    est_steps(c, (s0 + f.head) * c.L, c.f0[s0 + f.head].head, E, lo, hi);
    int q;
    i128 err;
    classify(f, E, q, err);
    clamp_in((i128)f.lo[q] - err, (i128)f.hi[q] - err, lo, hi);
    E += (u128)f.T[q];
}

// ---- composition ---------------------------------------------------------------------------
// Group g from its segments (level 1) / supergroup G from its groups (level 2).
QVQ_HD inline Fn compose1(const Chain &c, uint64_t g) {
    Fn f{};
    const uint64_t s0 = g * c.S;
    const uint32_t nk = c.kids1(g);
    uint32_t js = 0;
    while (js < nk && c.f0[s0 + js].kind != FN_BRIGHT) js++;
    if (js == nk) {
        f.kind = FN_SEQ;
        return f;
    }
    const Fn &k = c.f0[s0 + js];
    f.kind = FN_BRIGHT;
    f.head = js;
    f.B = k.B;
    for (int q = 0; q < 4; q++) {
        int64_t lo = k.lo[q], hi = k.hi[q];
        u128 E = (u128)(k.B + 128 * q + k.T[q]);
        for (uint32_t i = js + 1; i < nk && lo <= hi; i++) est0(c, s0 + i, E, lo, hi);
        f.lo[q] = lo;
        f.hi[q] = hi;
        f.T[q] = (i128)E - (f.B + 128 * q);
    }
    return f;
}
QVQ_HD inline Fn compose2(const Chain &c, uint64_t G) {
    Fn f{};
    const uint64_t g0 = G * c.S;
    const uint32_t nk = c.kids2(G);
    uint32_t js = 0;
    while (js < nk && c.f1[g0 + js].kind != FN_BRIGHT) js++;
    if (js == nk) {
        f.kind = FN_SEQ;
        return f;
    }
    const Fn &k = c.f1[g0 + js];
    f.kind = FN_BRIGHT;
    f.head = js;
    f.B = k.B;
    for (int q = 0; q < 4; q++) {
        int64_t lo = k.lo[q], hi = k.hi[q];
        u128 E = (u128)(k.B + 128 * q + k.T[q]);
        for (uint32_t i = js + 1; i < nk && lo <= hi; i++) est1(c, g0 + i, E, lo, hi);
        f.lo[q] = lo;
        f.hi[q] = hi;
        f.T[q] = (i128)E - (f.B + 128 * q);
    }
    return f;
}

// The transient: the reference's double steps from (0, 0) until sum >= 2 (or the chain's
// end).  Returns the position reached; E = sum - c in units once sum >= 2.
QVQ_HD inline uint64_t transient(const Chain &c, double &sum, u128 &E) {
    double cc = 0;
    sum = 0;
    uint64_t pos = 0;
    while (pos < c.n && !(sum >= 2.0)) fstep(sum, cc, ldexp((double)c.X(pos++), -60));
    E = sum >= 2.0 ? (u128)(to_units(sum) - to_units(cc)) : 0;
    return pos;
}

// Exact Kahan sum of the whole chain (sumInArea's result before the division).  miss[0..2]
// count the segments / groups / supergroups whose table was not used (may be null).
QVQ_HD inline double eval_chain(const Chain &c, uint32_t *miss) {
    double sum;
    u128 E;
    uint64_t pos = transient(c, sum, E);
    if (!(sum >= 2.0)) return sum;
    const uint64_t L = c.L, GL = L * c.S, SL = GL * c.S;
    for (; pos < c.n && pos % L; pos++) E = step(E, c.X(pos));
    for (; pos < c.n && pos % GL; pos += L) eval0(c, pos / L, E, miss);
    for (; pos < c.n && pos % SL; pos += GL) eval1(c, pos / GL, E, miss);
    for (; pos < c.n; pos += SL) eval2(c, pos / SL, E, miss);
    return to_double(E);
}

// Trusted walk (no checks) from the chain's start: dest[s] = E - P at the start of every
// segment s, the estimates for a second build of the segment tables.  P0[s]: exact sums of X
// before segment s.
QVQ_HD inline void estimate_dest(const Chain &c, const i128 *P0, int64_t *dest) {
    const uint64_t nseg = (c.n + c.L - 1) / c.L;
    double sum;
    u128 E;
    uint64_t pos = transient(c, sum, E);
    for (uint64_t s = 0; s < nseg && s * c.L < pos; s++) dest[s] = 0;
    if (!(sum >= 2.0)) return;
    for (; pos < c.n && pos % c.L; pos++) E = step(E, c.X(pos));
    for (; pos < c.n; pos += c.L) {
        const uint64_t s = pos / c.L;
        dest[s] = (int64_t)((i128)E - P0[s]);
        const Fn &f = c.f0[s];
        for (uint32_t j = 0; j < f.head; j++) E = step(E, c.X(pos + j));
        int q;
        i128 err;
        classify(f, E, q, err);
        E += (u128)f.T[q];
    }
}

}  // namespace kahan
}  // namespace qvq
