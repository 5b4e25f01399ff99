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
    uint64_t op[256];   // lo: X mod 512 | hm1 << 9 | parity shift << 16 (31: exact); hi: rounding mask
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
        const uint32_t mask = lg <= 0 || lg == 8 ? 0xFFFFFFFFu : ~((1u << lg) - 1);
        t.op[b] = (x & 511) | (hm1 << 9) | (sh << 16) | ((uint64_t)mask << 32);
        t.cg[b] = (int8_t)(lg == 8 ? 7 : lg);
        t.dg[b] = (int8_t)lg;
    }
}

// t rounded to a multiple of 2^lg, ties to even (lg >= 1)
QVQ_HD inline uint32_t rnd(uint32_t t, uint32_t lg) {
    return (t + ((1u << (lg - 1)) - 1) + ((t >> lg) & 1)) & ~((1u << lg) - 1);
}

// ---- trajectories ------------------------------------------------------------------------------
// NEN trajectories over steps b[0..n), all from the prefix P: entry e starts at E = P + D0[e]
// with E mod 512 = F[e] (the caller's class representatives).  bl0: the binade of every E on
// the way (0: computed at each decision from the exact E).  Out: the final F[e], the sums of
// deltas ds[e], and [lo, hi] narrowed to the input D for which every decision of every entry
// would be the same (absolute D of each entry's own input).
// One step of NEN trajectories (byte c).  R[e] is the trajectory's fine state without the mod
// 512 (only bits below 9 are ever read), so a step is four VALU per entry; Sxm accumulates X mod
// 512 for the deltas: sum(delta) = R_end - R_start - Sxm (mod 2^32).
template <int NEN, bool EXACT_BL>
QVQ_HD inline void step_n(const ByteTab &tb, uint32_t c, uint64_t &q, u128 &Pj, uint32_t &Sxm, int bl0, uint32_t *R,
                          const int64_t *D0, const uint32_t *R0, int64_t &lo, int64_t &hi) {
    const uint64_t pk = tb.pk[c];
    if (pk >> 62) {   // x = 1.0: a decision per entry
#pragma unroll
        for (int e = 0; e < NEN; e++) {
            const int64_t d = (int64_t)(int32_t)(R[e] - R0[e] - Sxm);   // deltas so far
            const uint64_t E64 = q + (uint64_t)(D0[e] + d);
            int bl = bl0;
            if (EXACT_BL) bl = bitlen(Pj + (u128)(i128)(D0[e] + d));
            const int su = bl - 53;
            const uint64_t U = 1ull << su, h = U >> 1, ee = E64 & (U - 1);
            const bool pos = ee < h || (ee == h && !((E64 >> su) & 1));
            const uint32_t F = R[e] & 511;
            const uint32_t r8 = rnd(F, 8), r7 = rnd(F, 7), r = pos ? r8 : r7;
            if (r8 != r7) {
                int64_t l, u2;
                if (ee == h) l = u2 = 0;
                else if (pos) l = -(int64_t)ee, u2 = (int64_t)(h - 1 - ee);
                else l = (int64_t)(h + 1 - ee), u2 = (int64_t)(U - 1 - ee);
                if (EXACT_BL) {   // the shift must also keep E in its binade
                    const i128 E = (i128)(Pj + (u128)(i128)(D0[e] + d));
                    const i128 bl_lo = ((i128)1 << (bl - 1)) - E, bl_hi = ((i128)1 << bl) - 1 - E;
                    if (bl_lo > (i128)l) l = bl_lo > (i128)DLIM ? DLIM : (int64_t)bl_lo;
                    if (bl_hi < (i128)u2) u2 = bl_hi < -(i128)DLIM ? -DLIM : (int64_t)bl_hi;
                }
                if (D0[e] + l > lo) lo = D0[e] + l;
                if (D0[e] + u2 < hi) hi = D0[e] + u2;
            }
            R[e] += r - F;   // (X mod 512 = 0 for x = 1.0)
        }
    } else {
        const uint64_t op = tb.op[c];
        const uint32_t xm = (uint32_t)op & 511, hm1 = ((uint32_t)op >> 9) & 127, sh = ((uint32_t)op >> 16) & 31;
        const uint32_t mask = (uint32_t)(op >> 32);
#pragma unroll
        for (int e = 0; e < NEN; e++) {
            const uint32_t t = R[e] + xm;
            R[e] = (t + hm1 + ((t >> sh) & 1)) & mask;   // sh = 31 (exact): t < 2^31 reads 0
        }
        Sxm += xm;
    }
    q += pk & ((1ull << 41) - 1);
    if (EXACT_BL) Pj += tb.X[c];
}

// NEN trajectories over steps b[0..n), all from the prefix P: entry e starts at E = P + D0[e]
// with E mod 512 = F[e] (the caller's class representatives).  bl0: the binade of every E on
// the way (0: computed at each decision from the exact E).  Out: the final F[e], the sums of
// deltas ds[e], and [lo, hi] narrowed to the input D for which every decision of every entry
// would be the same (absolute D of each entry's own input).
template <int NEN, bool EXACT_BL>
QVQ_HD inline void sim_n(const ByteTab &tb, const uint8_t *b, uint32_t n, u128 P, int bl0, uint32_t *F,
                         const int64_t *D0, int32_t *ds, int64_t &lo, int64_t &hi) {
    uint64_t q = (uint64_t)P;   // the prefix mod 2^64 (only bits < 41 are read)
    u128 Pj = P;
    uint32_t Sxm = 0, R[NEN], R0[NEN];
#pragma unroll
    for (int e = 0; e < NEN; e++) R[e] = R0[e] = F[e];
    if (((uintptr_t)b & 3) == 0) {   // whole words
        const uint32_t nw = n / 4;
        for (uint32_t w = 0; w < nw; w++) {
            const uint32_t word = reinterpret_cast<const uint32_t *>(b)[w];
#pragma unroll
            for (int u = 0; u < 4; u++) step_n<NEN, EXACT_BL>(tb, (word >> (8 * u)) & 0xFF, q, Pj, Sxm, bl0, R, D0, R0, lo, hi);
        }
        for (uint32_t i = nw * 4; i < n; i++) step_n<NEN, EXACT_BL>(tb, b[i], q, Pj, Sxm, bl0, R, D0, R0, lo, hi);
    } else {
        for (uint32_t i = 0; i < n; i++) step_n<NEN, EXACT_BL>(tb, b[i], q, Pj, Sxm, bl0, R, D0, R0, lo, hi);
    }
#pragma unroll
    for (int e = 0; e < NEN; e++) {
        ds[e] = (int32_t)(R[e] - R0[e] - Sxm);
        F[e] = R[e] & 511;
    }
}

// One trajectory (the exact replay: D0 is the true input D, so every decision is the true one).
QVQ_HD inline int32_t replay(const ByteTab &tb, const uint8_t *b, uint32_t n, u128 P, uint32_t &F, int64_t D0) {
    int32_t ds;
    int64_t lo = -DLIM, hi = DLIM;
    sim_n<1, true>(tb, b, n, P, 0, &F, &D0, &ds, lo, hi);
    return ds;
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

// A segment's function as stored for the evaluation's re-walks (a segment's sums of deltas fit
// 16 bits: 64 steps of at most 128 units).
struct SegFn {
    uint8_t kind, c_in, lne, c_out;
    uint16_t off_in, off_out, sx9, pad;
    int32_t lo, hi;
    int16_t dlt[NE];
};
QVQ_HD inline void pack_seg(const Fn &f, SegFn &s) {
    s.kind = f.kind;
    s.c_in = f.c_in;
    s.lne = f.lne;
    s.c_out = f.c_out;
    s.off_in = f.off_in;
    s.off_out = f.off_out;
    s.sx9 = f.sx9;
    s.pad = 0;
    s.lo = f.lo;
    s.hi = f.hi;
#pragma unroll
    for (int e = 0; e < NE; e++) s.dlt[e] = (int16_t)f.dlt[e];
}
QVQ_HD inline void unpack_seg(const SegFn &s, Fn &f) {
    f.kind = s.kind;
    f.c_in = s.c_in;
    f.lne = s.lne;
    f.c_out = s.c_out;
    f.off_in = s.off_in;
    f.off_out = s.off_out;
    f.sx9 = s.sx9;
    f.pad = 0;
    f.lo = s.lo;
    f.hi = s.hi;
#pragma unroll
    for (int e = 0; e < NE; e++) f.dlt[e] = s.dlt[e];
}
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
    int32_t dl = 0;
#pragma unroll
    for (int i = 0; i < NE; i++) dl = i == e ? f.dlt[i] : dl;   // (a select chain: f may be in registers)
    D += dl;
    F = (F + f.sx9 + (uint32_t)dl) & 511;
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
#pragma unroll
    for (int e = 0; e < NE; e++) {   // (a fixed trip count: h stays in registers)
        const uint32_t F0 = (f.off_in + ((uint32_t)e << f.c_in)) & 511;
        const int32_t d1 = f.dlt[e & mf];
        const uint32_t F1 = (F0 + f.sx9 + (uint32_t)d1) & 511;
        const int32_t d2 = g.dlt[(((F1 - g.off_in) & 511) >> g.c_in) & mg];
        const bool live = e < (1 << lne);
        h.dlt[e] = live ? d1 + d2 : 0;
        if (live && (int64_t)g.lo - d1 > lo) lo = (int64_t)g.lo - d1;
        if (live && (int64_t)g.hi - d1 < hi) hi = (int64_t)g.hi - d1;
    }
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
    int key = -1, G = -1;   // key = cg << 8 | position: its maximum is the last step of the top grade
    uint64_t slo = 0, shi = 0;
    const bool aligned = ((uintptr_t)b & 3) == 0;
    for (uint32_t i0 = 0; i0 < n; i0 += 4) {
        uint32_t word;
        if (aligned && i0 + 4 <= n) word = *reinterpret_cast<const uint32_t *>(b + i0);
        else {
            word = 0;
            for (uint32_t u = 0; u < 4 && i0 + u < n; u++) word |= (uint32_t)b[i0 + u] << (8 * u);
        }
        const uint32_t m4 = n - i0 < 4 ? n - i0 : 4;
#pragma unroll
        for (uint32_t u = 0; u < 4; u++) {
            const uint32_t c = (word >> (8 * u)) & 0xFF;
            const int cg = u < m4 ? tb.cg[c] : -1, dg = u < m4 ? tb.dg[c] : -1;
            const int kk = cg << 8 | (int)(i0 + u);
            key = cg >= 0 && kk > key ? kk : key;
            G = G > dg ? G : dg;
            const uint64_t x = u < m4 ? tb.X[c] : 0, t = slo + x;
            shi += t < slo;
            slo = t;
        }
    }
    const int cmax = key < 0 ? -1 : key >> 8;
    uint32_t F = 0;
    if (cmax >= 0) {   // the tail after the anchor: grades below cmax, no decisions, no class reads
        const uint32_t mk = (1u << cmax) - 1;
        for (uint32_t i = (uint32_t)(key & 0xFF) + 1; i < n; i++) {
            const uint64_t op = tb.op[b[i]];
            const uint32_t xm = (uint32_t)op & 511, hm1 = ((uint32_t)op >> 9) & 127, sh = ((uint32_t)op >> 16) & 31;
            const uint32_t t = F + xm;
            F = ((t + hm1 + ((t >> sh) & 1)) & (uint32_t)(op >> 32)) & mk;
        }
    }
    m.s_lo = slo;
    m.s_hi = (uint8_t)shi;
    m.cmax = (int8_t)cmax;
    m.G = (int8_t)G;
    m.pad = 0;
    m.off = (uint16_t)F;
    m.sx9 = (uint16_t)(slo & 511);
    return m;
}
QVQ_HD inline u128 meta_sum(const SegMeta &m) { return ((u128)m.s_hi << 64) | m.s_lo; }

// ---- building a segment's function -------------------------------------------------------------
// The input class structure of a segment: the nearest preceding segment with an anchor (its
// cmax and tail offset), translated by the exact segments in between.  prev(i) (i = 1..np) gives
// the metadata of the i-th preceding segment.  c_in = -1: none within np segments.
template <class PrevFn>
QVQ_HD inline void input_structure(PrevFn prev, int np, int &c_in, uint32_t &off_in) {
    c_in = -1;
    off_in = 0;
    uint32_t trans = 0;
    for (int i = 1; i <= np; i++) {
        const SegMeta m = prev(i);
        if (m.cmax >= 0) {
            c_in = m.cmax;
            off_in = (m.off + trans) & ((1u << c_in) - 1);
            return;
        }
        trans += m.sx9;
    }
}

// Entries [e0, e0 + NEN) of f through sim_n (f's header already set); [lo, hi] narrowed.
template <int NEN, bool EXACT_BL>
QVQ_HD inline void build_group(const ByteTab &tb, const uint8_t *b, uint32_t n, u128 P, int bl0, int64_t D_est,
                               int e0, Fn &f, int64_t &lo, int64_t &hi, bool active = true) {
    uint32_t F[NEN];
    int64_t D0[NEN];
    int32_t ds[NEN];
#pragma unroll
    for (int e = 0; e < NEN; e++) {
        F[e] = (f.off_in + ((uint32_t)(e0 + e) << f.c_in)) & 511;
        // the representative input D: D == F - P (mod 512), next to D_est
        D0[e] = D_est + (int64_t)((F[e] - (uint32_t)(uint64_t)P - (uint32_t)D_est + 256) & 511) - 256;
    }
    int64_t l2 = lo, h2 = hi;
    sim_n<NEN, EXACT_BL>(tb, b, n, P, bl0, F, D0, ds, l2, h2);
    if (!active) return;   // (a lane that ran along with its wave)
    lo = l2;
    hi = h2;
#pragma unroll
    for (int e = 0; e < NE; e++)   // (a fixed trip count: f stays in registers)
        if (e >= e0 && e < e0 + NEN) f.dlt[e] = ds[(e - e0) & (NEN - 1)];
}

// Segment j of a chain (n steps at b, exact prefix P at its start, metadata self, input class
// structure (c_in, off_in) from input_structure); final: the chain's last segment.  The header
// of its function (kind, classes, output structure); returns the entries to simulate (0: none,
// the function is complete) and in bl0 the binade of the segment's states (0: a power of two
// inside its range, each decision then takes the exact binade).
QVQ_HD inline int build_header(const uint8_t *b, uint32_t n, u128 P, const SegMeta &self, int c_in, uint32_t off_in,
                               bool final, Fn &f, int &bl0) {
    (void)b;
    (void)n;
    f.pad = 0;
    bl0 = 0;
    for (int e = 0; e < NE; e++) f.dlt[e] = 0;
    if (self.G < 0) {   // every step exact: a translation
        f.kind = (uint8_t)(FK_TRANS | (final ? FK_FINAL : 0));
        f.c_in = f.lne = f.c_out = 0;
        f.off_in = f.off_out = 0;
        f.sx9 = self.sx9;
        f.lo = -(int32_t)DLIM;
        f.hi = (int32_t)DLIM;
        return 0;
    }
    const int lne = self.G + 1 - c_in > 0 ? self.G + 1 - c_in : 0;
    if (c_in < 0 || P < MIN_STATE + (u128)DLIM || lne > 4) {
        set_raw(f);
        return 0;
    }
    f.kind = (uint8_t)(FK_TABLE | (final ? FK_FINAL : 0));
    f.c_in = (uint8_t)c_in;
    f.lne = (uint8_t)lne;
    f.c_out = (uint8_t)self.cmax;   // G >= 0 means some step rounds: an anchor exists
    f.off_in = (uint16_t)off_in;
    f.off_out = self.off;
    f.sx9 = self.sx9;
    f.lo = -(int32_t)DLIM;
    f.hi = (int32_t)DLIM;
    bl0 = fixed_binade(P, meta_sum(self));
    return 1 << lne;
}

// Entries [e0, e0 + NEN) of f (header set by build_header), f's interval narrowed.
template <int NEN, bool EXACT_BL>
QVQ_HD inline void build_entries(const ByteTab &tb, const uint8_t *b, uint32_t n, u128 P, int bl0, int64_t D_est,
                                 int e0, Fn &f, bool active = true) {
    int64_t lo = f.lo, hi = f.hi;
    build_group<NEN, EXACT_BL>(tb, b, n, P, bl0, D_est, e0, f, lo, hi, active);
    if (!active) return;
    f.lo = (int32_t)lo;
    f.hi = (int32_t)hi;
    if (f.lo > f.hi) f.lo = 1, f.hi = 0;
}

// The whole function (host; the device runs the entries wave-uniformly, k_kahan.hip).
QVQ_HD inline void build_fn(const ByteTab &tb, const uint8_t *b, uint32_t n, u128 P, const SegMeta &self, int c_in,
                            uint32_t off_in, bool final, int64_t D_est, Fn &f) {
    int bl0;
    const int ne = build_header(b, n, P, self, c_in, off_in, final, f, bl0);
    if (!ne) return;
    if (bl0) {
        if (ne <= 2) build_entries<2, false>(tb, b, n, P, bl0, D_est, 0, f);
        else
            for (int e0 = 0; e0 < ne; e0 += 4) build_entries<4, false>(tb, b, n, P, bl0, D_est, e0, f);
    } else {
        for (int e0 = 0; e0 < ne; e0++) build_entries<1, true>(tb, b, n, P, 0, D_est, e0, f);
    }
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
