"""The reference kd-tree build (nanoflann 1.2.3 as quant_amd/csrc/kdtree.cpp restates it) in numpy,
for studying the trees of real level codebooks (tools/dump_splits.py) and as the model of the
device build (k_kdbuild.hip).  usage: python tools/kd_shapes.py SPLITS.npz [KEY ...]"""
import sys
import numpy as np

LEAF = 10
EPS = 0.00001


def build(P):
    """Returns (nodes, vind, root_box): nodes in DFS pre-order, each a dict."""
    K, D = P.shape
    vind = np.arange(K)
    lo, hi = P.min(0), P.max(0)
    nodes = []

    def divide(left, right, box_lo, box_hi, depth):
        me = len(nodes)
        nodes.append(None)
        idx = vind[left:right]
        if right - left <= LEAF:
            nodes[me] = dict(leaf=True, left=left, right=right, depth=depth)
            return me, P[idx].min(0), P[idx].max(0)
        span = box_hi - box_lo
        max_span = span.max()
        cand = np.nonzero(span > (1 - EPS) * max_span)[0]
        mn, mx = P[idx][:, cand].min(0), P[idx][:, cand].max(0)
        spread = mx - mn
        j = 0
        best = -1.0
        for t in range(len(cand)):
            if spread[t] > best:
                best, j = spread[t], t
        cutfeat = int(cand[j]) if len(cand) else 0
        cmn, cmx = (mn[j], mx[j]) if len(cand) else (P[idx, 0].min(), P[idx, 0].max())
        split_val = (box_lo[cutfeat] + box_hi[cutfeat]) / 2
        cutval = cmn if split_val < cmn else (cmx if split_val > cmx else split_val)
        lim1, lim2 = plane_split(left, right - left, cutfeat, cutval)
        count = right - left
        index = lim1 if lim1 > count // 2 else (lim2 if lim2 < count // 2 else count // 2)
        lb_lo, lb_hi = box_lo.copy(), box_hi.copy()
        lb_hi[cutfeat] = cutval
        rb_lo, rb_hi = box_lo.copy(), box_hi.copy()
        rb_lo[cutfeat] = cutval
        c1, l1, h1 = divide(left, left + index, lb_lo, lb_hi, depth + 1)
        c2, l2, h2 = divide(left + index, right, rb_lo, rb_hi, depth + 1)
        nodes[me] = dict(leaf=False, left=left, right=right, depth=depth, cutfeat=cutfeat, cutval=cutval,
                         divlow=h1[cutfeat], divhigh=l2[cutfeat], child1=c1, child2=c2, ncand=len(cand),
                         lim1=lim1, lim2=lim2, index=index)
        return me, np.minimum(l1, l2), np.maximum(h1, h2)

    def plane_split(left, count, f, cv):
        ind = vind[left:left + count]   # view: swaps act on vind
        v = lambda i: P[ind[i], f]
        l, r = 0, count - 1
        while True:
            while l <= r and v(l) < cv:
                l += 1
            while r and l <= r and v(r) >= cv:
                r -= 1
            if l > r or not r:
                break
            ind[l], ind[r] = ind[r], ind[l]
            l += 1
            r -= 1
        lim1 = l
        r = count - 1
        while True:
            while l <= r and v(l) <= cv:
                l += 1
            while r and l <= r and v(r) > cv:
                r -= 1
            if l > r or not r:
                break
            ind[l], ind[r] = ind[r], ind[l]
            l += 1
            r -= 1
        return lim1, l

    sys.setrecursionlimit(100000)
    divide(0, K, lo.copy(), hi.copy(), 1)
    return nodes, vind, (lo, hi)


def main():
    z = np.load(sys.argv[1])
    keys = sys.argv[2:] or list(z.keys())
    for k in keys:
        P = z[k]
        nodes, vind, _ = build(P)
        inner = [n for n in nodes if not n["leaf"]]
        depth = max(n["depth"] for n in nodes)
        zero = int((np.abs(P).sum(1) == 0).sum())
        dup = P.shape[0] - len(np.unique(P, axis=0))
        work = sum((n["right"] - n["left"]) for n in inner)
        big = [n for n in inner if n["right"] - n["left"] > 64]
        unbal = [n for n in inner if min(n["index"], n["right"] - n["left"] - n["index"]) * 8 < (n["right"] - n["left"])]
        print("%s K=%d D=%d: nodes %d (inner %d), depth %d, zero rows %d, duplicate rows %d, sum of inner sizes %d "
              "(%.1f per point), inner > 64 pts %d, 1:8-unbalanced %d, depth of those %s" %
              (k, P.shape[0], P.shape[1], len(nodes), len(inner), depth, zero, dup, work, work / P.shape[0], len(big),
               len(unbal), sorted(set(n["depth"] for n in unbal))[:5]))
        ds = {}
        for n in inner:
            ds.setdefault(n["depth"], []).append(n["right"] - n["left"])
        print("   per depth: " + " ".join("%d:%d/%d" % (d, len(v), max(v)) for d, v in sorted(ds.items())[:40]))


if __name__ == "__main__":
    main()
