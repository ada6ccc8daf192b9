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
  * the leaf list in backtrack order, left = first child of the winning pair (Fit :17-24);
  * with ``offtree=True`` (default) every split CANDIDATE child of every tree node -- the
    cells whose stored scores the node's first minimum was taken against, on the tree or
    not -- is re-derived one level down as well: its own split candidates' stored scores
    (one more gather per depth) and its single-pattern term from its train counts (the
    node's k-mers restricted at the split position) must give its stored score bit for bit
    (``local_values``).  A candidate stored too HIGH (a wrong gather, count table or store in
    some block) could otherwise flip a node's argmin to a worse split that the walk would
    then reproduce faithfully; a too-high candidate fails its own re-derivation unless every
    one of its split sums and its single term were too high as well, and the single term is
    computed here from the true counts.

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
        # the same tables as arrays, padded: split pair j of digit d at position i, -1 past the
        # last pair (positions ascending, pairs in table order = the reference's scan order)
        self.PA = np.full((self.k, 15, 7), -1, np.int64)
        self.PB = np.full((self.k, 15, 7), -1, np.int64)
        self.MB = np.zeros((self.k, 15, 4), np.int64)  # nucleotide-rank membership of digit d
        for i in range(self.k):
            for d, prs in enumerate(self.pairs[i]):
                for j, (pa, pb) in enumerate(prs):
                    self.PA[i, d, j], self.PB[i, d, j] = pa, pb
            for d, m in enumerate(self.mask[i]):
                for n in range(4):
                    self.MB[i, d, n] = (m >> n) & 1
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

    def digit_array(self, cells):
        """``[n, k]`` digits of an array of cells."""
        x = np.asarray(cells, np.int64).copy()
        out = np.empty((x.size, self.k), np.int64)
        for i, r in enumerate(self.radix):
            out[:, i] = x % r
            x //= r
        return out


def _libm_array(x, fn):
    try:
        from .oracle import libm
        return libm(x, fn)
    except OSError:  # the oracle library is not built: the same calls one by one
        f = c_log1p if fn == "log1p" else c_log
        return np.array([f(float(v)) for v in np.asarray(x, np.float64).ravel()], np.float64)


def local_values(lat, cells, mtr, utr, gather, alpha, beta, penalty):
    """Re-derived float32 train score of each cell in ``cells`` from the STORED scores of its
    own split children (``gather``) and its train counts ``mtr``/``utr`` (int arrays): the
    reference's recurrence for one cell, vectorised -- k-mer cells (no split pairs)
    ``f32(-2 (xlogy(M, p) + xlog1py(U, -p)) + c)`` (CV :15-20); other cells the smallest
    ``f32(S[c1] + S[c2])`` over their split pairs (a NaN sum never wins a strict ``<``, CV :49;
    the smallest value is the first minimum's value), replaced by ``f32(s)`` if the float64
    single-pattern term ``s`` (CV :56-70, the C library's log) is strictly smaller (CV :71)."""
    cells = np.asarray(cells, np.int64)
    n = cells.size
    a, b, c = float(alpha), float(beta), float(penalty)
    mtr = np.asarray(mtr, np.int64)
    utr = np.asarray(utr, np.int64)
    D = lat.digit_array(cells)
    P = lat.k * 7
    c1 = np.zeros((n, P), np.int64)
    c2 = np.zeros((n, P), np.int64)
    ok = np.zeros((n, P), bool)
    for i in range(lat.k):
        d = D[:, i]
        for j in range(7):
            pa, pb = lat.PA[i, d, j], lat.PB[i, d, j]
            v = pa >= 0
            col = i * 7 + j
            ok[:, col] = v
            c1[:, col] = np.where(v, cells + (pa - d) * lat.cw[i], 0)
            c2[:, col] = np.where(v, cells + (pb - d) * lat.cw[i], 0)
    need = np.concatenate([c1[ok], c2[ok]])
    vals = np.asarray(gather(need.astype(np.uint64)), np.float32) if need.size else np.zeros(0, np.float32)
    m = int(ok.sum())
    sums = np.full((n, P), np.inf, np.float32)
    with np.errstate(invalid="ignore", over="ignore"):
        s12 = vals[:m] + vals[m:]  # float32 + float32 -> float32 (CV :46)
    s12 = np.where(np.isnan(s12), np.float32(np.inf), s12)
    sums[ok] = s12
    best = sums.min(axis=1) if P else np.full(n, np.inf, np.float32)
    kmer = ~ok.any(axis=1)
    with np.errstate(invalid="ignore", divide="ignore", over="ignore"):
        p = (mtr.astype(np.float64) + a) / (((mtr + utr).astype(np.float64) + a) + b)
        logp = _libm_array(p, "log")
        log1mp = _libm_array(1.0 - p, "log")
        s = np.full(n, c)
        s = np.where(mtr > 0, s + (-2.0 * mtr.astype(np.float64)) * logp, s)
        s = np.where(utr > 0, s + (-2.0 * utr.astype(np.float64)) * log1mp, s)
        out = np.where(s < best.astype(np.float64), s.astype(np.float32), best)
        if kmer.any():
            pk, mk, uk = p[kmer], mtr[kmer].astype(np.float64), utr[kmer].astype(np.float64)
            xa = np.where((mk == 0) & ~np.isnan(pk), 0.0, mk * logp[kmer])
            xb = np.where((uk == 0) & ~np.isnan(-pk), 0.0, uk * _libm_array(-pk, "log1p"))
            out[kmer] = (-2.0 * (xa + xb) + c).astype(np.float32)
    return out


class TreeMismatch(AssertionError):
    pass


def rederive(lat, gather, Mtr, Utr, Mte, Ute, alpha, beta, penalty, offtree=True):
    """Walk the optimal tree of one lane and re-derive every node.

    ``gather(cells)`` -> float32 train scores of the lane at those cell indices (uint64).
    ``Mtr``/``Utr`` = train counts per k-mer (k-mer index order), ``Mte``/``Ute`` = test
    counts (zeros in fit mode), int64.  Returns ``dict(root_train, root_test, leaves,
    nodes, candidates)`` (float32, float32, uint64 array in backtrack order, nodes visited,
    split candidates re-derived one level down); raises :class:`TreeMismatch` naming the
    first node (or candidate) whose stored score differs from the re-derived one."""
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
    checked = 0
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
        if offtree:
            checked += _check_candidates(lat, frontier, nodes, cand, vals, gather, Mtr, Utr, a, b, c)
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
            "nodes": visited, "candidates": checked}


def _check_candidates(lat, frontier, nodes, cand, vals, gather, Mtr, Utr, a, b, c):
    """Every split candidate child of the frontier's nodes (``cand``, ``vals`` as gathered by
    rederive: per node its own score, then c1, c2 of each pair) re-derived by local_values
    from ITS split children's stored scores and its train counts.  A candidate's k-mers are
    its parent's restricted at the split position, so its counts are sums of per-node,
    per-position nucleotide histograms."""
    nfr = len(frontier)
    kid = [nodes[nid][1] for nid in frontier]
    K = np.concatenate(kid)
    lab = np.repeat(np.arange(nfr), [k.size for k in kid])
    wm, wu = Mtr[K].astype(np.float64), Utr[K].astype(np.float64)  # exact: sums < 2^53
    HM, HU = [], []
    for i in range(lat.k):
        key = lab * 4 + lat.kdig[i][K].astype(np.int64)
        HM.append(np.rint(np.bincount(key, weights=wm, minlength=nfr * 4)).astype(np.int64).reshape(nfr, 4))
        HU.append(np.rint(np.bincount(key, weights=wu, minlength=nfr * 4)).astype(np.int64).reshape(nfr, 4))
    cnode, cpos, cdig, ccell, cval = [], [], [], [], []
    q = 0
    for fi, (dig, lst) in enumerate(cand):
        q += 1
        for (i, pa, pb, c1, c2) in lst:
            cnode += [fi, fi]
            cpos += [i, i]
            cdig += [pa, pb]
            ccell += [c1, c2]
            cval += [vals[q], vals[q + 1]]
            q += 2
    if not ccell:
        return 0
    cnode, cpos, cdig = np.asarray(cnode), np.asarray(cpos), np.asarray(cdig)
    ccell = np.asarray(ccell, np.int64)
    cval = np.asarray(cval, np.float32)
    mtr = np.zeros(ccell.size, np.int64)
    utr = np.zeros(ccell.size, np.int64)
    for i in range(lat.k):
        sel = cpos == i
        if sel.any():
            mb = lat.MB[i, cdig[sel]]
            mtr[sel] = (HM[i][cnode[sel]] * mb).sum(axis=1)
            utr[sel] = (HU[i][cnode[sel]] * mb).sum(axis=1)
    got = local_values(lat, ccell, mtr, utr, gather, a, b, c)
    bad = (got.view(np.uint32) != cval.view(np.uint32)) & ~(np.isnan(got) & np.isnan(cval))
    if bad.any():
        j = int(np.argmax(bad))
        parent = nodes[frontier[cnode[j]]][0]
        raise TreeMismatch(f"split candidate cell {int(ccell[j])} ({lat.pattern(int(ccell[j]))}) of tree node "
                           f"{parent} ({lat.pattern(parent)}): stored {cval[j]!r} (0x{int(cval[j].view(np.uint32)):08x}), "
                           f"re-derived {got[j]!r} (0x{int(got[j].view(np.uint32)):08x}) [{int(bad.sum())} candidates differ]")
    return int(ccell.size)
