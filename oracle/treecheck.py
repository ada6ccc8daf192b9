"""Host re-derivation of one lane's optimal tree from its stored train scores.

TEST INFRASTRUCTURE ONLY (tests/, never the product package).  At full size (7.7e9
cells) the oracle cannot rerun the whole DP, but every number that reaches the CVfile --
the root's train score and the root's test -2LL -- is decided by the cells on the optimal
tree and by the scores of their split children.  Given a lane's stored float32 train
scores (read back cell by cell from the device, ``gather``), this walks the tree top-down
and re-derives every decision with the reference's own recurrence, computed here on the
host:

  * split candidates in the reference's scan order: positions ascending, only ambiguous
    codes, pairs in complements_tab order (CV :37-51, pattern_utils.py:48-84);
    ``new = f32(S[c1] + S[c2])``, taken on a strict ``<`` (first minimum wins);
  * the single-pattern term in float64 from the node's train counts (sums over its
    k-mers), with the C library's log (CV :56-71; Fit :56-64): it replaces the best split
    only if ``s < f64(best)``, and is stored as f32(s);
  * k-mer cells (level 0): ``f32(-2 (xlogy(M, p) + xlog1py(U, -p)) + c)`` (CV :15-20);
  * the node's stored score must equal the re-derived value bit for bit;
  * test -2LL: leaves take the single-pattern test term (CV :73-78; :19 at k-mers), split
    nodes ``f32(test[c1] + test[c2])`` (CV :47), summed bottom-up -- the root's value is
    ``test_score_mem[root]`` (CV :158-163);
  * the leaf list in backtrack order, left = first child of the winning pair (Fit :17-24).

It shares no code with the product: its own IUPAC tables (``oracle.oracle``), its own
k-mer index arithmetic and ``log`` / ``log1p`` from the host C library through ctypes
(what numba's ``np.log`` lowers to; scipy's ``xlogy`` / ``xlog1py`` are ``x * log(y)`` /
``x * log1p(y)``, tests/test_libm.py).
"""
import ctypes
import ctypes.util
import math

import numpy as np

from .oracle import _PERM, _SPLIT

_libm = ctypes.CDLL(ctypes.util.find_library("m") or "libm.so.6")
_libm.log.argtypes = [ctypes.c_double]
_libm.log.restype = ctypes.c_double
_libm.log1p.argtypes = [ctypes.c_double]
_libm.log1p.restype = ctypes.c_double
c_log, c_log1p = _libm.log, _libm.log1p

IUPAC = {"A": "A", "C": "C", "G": "G", "T": "T", "R": "AG", "Y": "CT", "S": "CG", "W": "AT", "K": "GT",
         "M": "AC", "B": "CGT", "D": "AGT", "H": "ACT", "V": "ACG", "N": "ACGT"}
F32 = np.float32


def _xlogy(x, y):
    return 0.0 if (x == 0 and not math.isnan(y)) else float(x) * c_log(y)


def _xlog1py(x, y):
    return 0.0 if (x == 0 and not math.isnan(y)) else float(x) * c_log1p(y)


class Lattice:
    """IUPAC index arithmetic of one general pattern: cell index = mixed radix over
    positions, position 0 least significant, digit = index in perm_code[g]
    (pattern_utils.py:86-100, :253-257); k-mer index = position 0 fastest, digit = rank of
    the nucleotide among the general code's nucleotides (alphabetical)."""

    def __init__(self, gen_pat):
        self.gp = gen_pat
        self.k = len(gen_pat)
        self.radix = [len(_PERM[g]) for g in gen_pat]
        self.cw = [1] * self.k
        self.kw = [1] * self.k
        self.nn = [len(IUPAC[g]) for g in gen_pat]
        for i in range(1, self.k):
            self.cw[i] = self.cw[i - 1] * self.radix[i - 1]
            self.kw[i] = self.kw[i - 1] * self.nn[i - 1]
        self.root = sum((r - 1) * w for r, w in zip(self.radix, self.cw))
        self.n_kmers = self.kw[-1] * self.nn[-1]
        # per position: letter digit -> (nucleotide-rank mask, split pairs as digit pairs)
        self.mask = []
        self.pairs = []
        for g in gen_pat:
            nucs = IUPAC[g]
            self.mask.append([sum(1 << nucs.index(n) for n in IUPAC[x]) for x in _PERM[g]])
            self.pairs.append([[(_PERM[g].index(p[0]), _PERM[g].index(p[1])) for p in _SPLIT.get(x, "").split()]
                               for x in _PERM[g]])
        x = np.arange(self.n_kmers, dtype=np.int64)
        self.kdig = np.empty((self.k, self.n_kmers), np.uint8)
        for i in range(self.k):
            self.kdig[i] = (x // self.kw[i]) % self.nn[i]

    def digits(self, cell):
        out = []
        for r in self.radix:
            cell, d = divmod(int(cell), r)
            out.append(d)
        return out

    def pattern(self, cell):
        return "".join(_PERM[g][d] for g, d in zip(self.gp, self.digits(cell)))


class TreeMismatch(AssertionError):
    pass


def rederive(lat, gather, Mtr, Utr, Mte, Ute, alpha, beta, penalty):
    """Walk the optimal tree of one lane and re-derive every node.

    ``gather(cells)`` -> float32 train scores of the lane at those cell indices (uint64).
    ``Mtr``/``Utr`` = train counts per k-mer (k-mer index order), ``Mte``/``Ute`` = test
    counts (zeros in fit mode), int64.  Returns ``dict(root_train, root_test, leaves,
    nodes)`` (float32, float32, uint64 array in backtrack order, nodes visited); raises
    :class:`TreeMismatch` naming the first node whose stored score differs from the
    re-derived one."""
    Mtr, Utr = np.asarray(Mtr, np.int64), np.asarray(Utr, np.int64)
    Mte, Ute = np.asarray(Mte, np.int64), np.asarray(Ute, np.int64)
    a, b, c = float(alpha), float(beta), float(penalty)
    # a node: (cell, k-mer index array); processed depth by depth so that each depth's
    # candidate children are read back in one gather
    nodes = {}  # id -> [cell, kidx, kind, children(id1, id2) | None, test f32]
    frontier = [0]
    nodes[0] = [lat.root, np.arange(lat.n_kmers, dtype=np.int64), None, None, None]
    next_id = 1
    visited = 0
    while frontier:
        # every candidate child (and the node itself) of the frontier, in scan order
        cand = []
        for nid in frontier:
            cell = nodes[nid][0]
            dig = lat.digits(cell)
            lst = []
            for i, d in enumerate(dig):
                base = cell - d * lat.cw[i]
                for pa, pb in lat.pairs[i][d]:
                    lst.append((i, pa, pb, base + pa * lat.cw[i], base + pb * lat.cw[i]))
            cand.append((dig, lst))
        flat = []
        for nid, (dig, lst) in zip(frontier, cand):
            flat.append(nodes[nid][0])
            for (_, _, _, c1, c2) in lst:
                flat.extend((c1, c2))
        vals = np.asarray(gather(np.asarray(flat, np.uint64)), np.float32)
        q = 0
        nxt = []
        for nid, (dig, lst) in zip(frontier, cand):
            node = nodes[nid]
            cell, kidx = node[0], node[1]
            stored = vals[q]
            q += 1
            mtr, utr = int(Mtr[kidx].sum()), int(Utr[kidx].sum())
            mte, ute = int(Mte[kidx].sum()), int(Ute[kidx].sum())
            p = (mtr + a) / (((mtr + utr) + a) + b)
            if not lst:  # a k-mer: level-0 terms (CV :15-20)
                got = F32(-2.0 * (_xlogy(mtr, p) + _xlog1py(utr, -p)) + c)
                node[2] = "kmer"
                node[4] = F32(-2.0 * (_xlogy(mte, p) + _xlog1py(ute, -p)))
            else:
                best, win = F32(np.inf), None
                for (i, pa, pb, c1, c2) in lst:
                    s1, s2 = vals[q], vals[q + 1]
                    q += 2
                    nt = F32(s1 + s2)
                    if nt < best:  # strict: the first minimum wins (CV :49)
                        best, win = nt, (i, pa, pb, c1, c2)
                logp, log1mp = c_log(p), c_log(1.0 - p)
                s = c
                if mtr > 0:
                    s += (-2.0 * mtr) * logp
                if utr > 0:
                    s += (-2.0 * utr) * log1mp
                if s < float(best):  # CV :71, float64 against the stored float32
                    got, win = F32(s), None
                    t = 0.0
                    if mte > 0:
                        t += (-2.0 * mte) * logp
                    if ute > 0:
                        t += (-2.0 * ute) * log1mp
                    node[4] = F32(t)
                    node[2] = "single"
                else:
                    got = best
                    i, pa, pb, c1, c2 = win
                    ch = []
                    for dd, cc in ((pa, c1), (pb, c2)):
                        m = lat.mask[i][dd]
                        keep = ((m >> lat.kdig[i][kidx].astype(np.int64)) & 1).astype(bool)
                        nodes[next_id] = [cc, kidx[keep], None, None, None]
                        ch.append(next_id)
                        nxt.append(next_id)
                        next_id += 1
                    node[2] = "split"
                    node[3] = tuple(ch)
            visited += 1
            if got.view(np.uint32) != stored.view(np.uint32) and not (np.isnan(got) and np.isnan(stored)):
                raise TreeMismatch(f"cell {cell} ({lat.pattern(cell)}): stored {stored!r} "
                                   f"(0x{int(stored.view(np.uint32)):08x}), re-derived {got!r} "
                                   f"(0x{int(got.view(np.uint32)):08x}) [{node[2]}]")
            node[1] = None  # (the children hold their own k-mer sets)
        frontier = nxt
    # test values bottom-up (ids grow with depth, so children come after parents)
    for nid in sorted(nodes, reverse=True):
        node = nodes[nid]
        if node[2] == "split":
            t1, t2 = nodes[node[3][0]][4], nodes[node[3][1]][4]
            node[4] = F32(t1 + t2)
    # leaves in backtrack order: left subtree first (Fit :17-24)
    leaves, stack = [], [0]
    while stack:
        nid = stack.pop()
        node = nodes[nid]
        if node[2] == "split":
            stack.append(node[3][1])
            stack.append(node[3][0])
        else:
            leaves.append(node[0])
    root_train = F32(gather(np.asarray([lat.root], np.uint64))[0])
    return {"root_train": root_train, "root_test": nodes[0][4], "leaves": np.asarray(leaves, np.uint64),
            "nodes": visited}
