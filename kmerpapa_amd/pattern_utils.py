"""IUPAC pattern algebra for the k-mer pattern lattice (host side).

Public names, argument meanings and enumeration ORDERS follow the reference module
``kmerpapa.pattern_utils`` (src/kmerpapa/pattern_utils.py, v0.2.4) so that callers and
tests written against it keep working.  The lattice tables below are the data the
device planner (`kmerpapa_amd/csrc/kp_hip.hip`, ``kp_plan_create``) rebuilds in C++.

Facts the whole build relies on (checked by tests/test_pattern_utils.py):
  * cell index = mixed radix over positions, position 0 least significant; the digit at
    position i is the index of the sub-code in ``perm_code[g_i]``   (ref :247-266)
  * ``perm_code[g]`` lists the nucleotides of ``g`` first, in ``code[g]`` order, so a
    k-mer's digit equals its nucleotide's index in ``code[g]``     (ref :86-100, :5-19)
  * every split child has a strictly smaller digit than its parent at the split
    position, so ascending cell index is a topological order of the DP.
"""
from itertools import chain, product

import numpy as np

NUCLEOTIDES = "ACGT"

# IUPAC code -> nucleotides in the reference's order (pattern_utils.py:5-19).
_CODE = {"A": "A", "C": "C", "G": "G", "T": "T",
         "R": "AG", "Y": "CT", "S": "GC", "W": "AT", "K": "GT", "M": "AC",
         "B": "CGT", "D": "AGT", "H": "ACT", "V": "ACG", "N": "ACGT"}
# IUPAC code -> all sub-codes, the digit order of the lattice index (pattern_utils.py:86-100).
_PERM = {"A": "A", "C": "C", "G": "G", "T": "T",
         "R": "AGR", "Y": "CTY", "S": "GCS", "W": "ATW", "K": "GTK", "M": "ACM",
         "B": "CGTSYKB", "D": "AGTRWKD", "H": "ACTMWYH", "V": "ACGMRSV",
         "N": "ACGTRYSWKMBDHVN"}
# IUPAC code -> ordered two-way splits (pattern_utils.py:48-57).  The order is the
# scan order of the DP's strict "<" and therefore decides ties.
_SPLITS = {"R": "AG", "Y": "CT", "S": "GC", "W": "AT", "K": "GT", "M": "AC",
           "V": "AS CR GM", "H": "AY CW TM", "D": "AK GW TR", "B": "CK GY TS",
           "N": "SW KM RY AB CD GH TV"}

code = {x: list(v) for x, v in _CODE.items()}
perm_code = {x: list(v) for x, v in _PERM.items()}
complements = {x: [tuple(p) for p in v.split()] for x, v in _SPLITS.items()}

set_code = {x: frozenset(v) for x, v in _CODE.items()}
set_perm_code = {x: frozenset(v) for x, v in _PERM.items()}
inv_code = {frozenset(v): x for x, v in _CODE.items()}

# code_level[x] = |x| - 1 : how many splits separate x from single nucleotides
code_level = {x: len(v) - 1 for x, v in _CODE.items()}
code_lev = code_level

# perm_code_no[g][x] = digit of sub-code x under general code g (pattern_utils.py:112-116)
perm_code_no = {g: {x: i for i, x in enumerate(v)} for g, v in _PERM.items()}
# code_no[g][n] = index of nucleotide n inside code g (pattern_utils.py:122-126)
code_no = {g: {n: i for i, n in enumerate(v)} for g, v in _CODE.items()}

# minus_set[c][x] = the other half of the split of c that contains x (pattern_utils.py:184-189)
minus_set = {c: dict(chain.from_iterable(((a, b), (b, a)) for a, b in pairs))
             for c, pairs in complements.items()}

n_complements_of = {x: len(complements.get(x, ())) for x in _CODE}


def _ord_table(fill, shape, items):
    t = np.full(shape, fill, dtype=int)
    for key, val in items:
        t[key] = val
    return t


# ord-indexed numpy views used by the reference's numeric callers and tests
perm_code_no_np = _ord_table(-100, (90, 90), (((ord(g), ord(x)), i)
                                              for g, v in _PERM.items() for i, x in enumerate(v)))
code_no_np = _ord_table(-100, (90, 90), (((ord(g), ord(n)), i)
                                         for g, v in _CODE.items() for i, n in enumerate(v)))
code_len_ord_np = _ord_table(-100, (90,), ((ord(x), len(v)) for x, v in _CODE.items()))
code_lev_ord_np = _ord_table(-100, (90,), ((ord(x), len(v) - 1) for x, v in _CODE.items()))
n_complements = _ord_table(0, (90,), ((ord(x), len(v)) for x, v in complements.items()))


def pattern_level(pattern):
    """Level of a pattern: number of splits needed to reach single k-mers (ref :219-230)."""
    return sum(code_level[x] for x in pattern)


def get_genpat_pos_level(genpat):
    """Radix of every position: number of sub-codes of each general code (ref :233-234)."""
    return [len(_PERM[x]) for x in genpat]


def get_cum_genpat_pos_level(genpat):
    """Place values of the mixed-radix cell index, position 0 first (ref :237-244)."""
    out, acc = [], 1
    for r in get_genpat_pos_level(genpat):
        out.append(acc)
        acc *= r
    return out


def pattern_max(general_pattern):
    """Number of sub-patterns (lattice cells) of a general pattern (ref :587-599)."""
    n = 1
    for x in general_pattern:
        n *= len(_PERM[x])
    return n


def generality(pat):
    """Number of k-mers matching a pattern (ref :554-568)."""
    n = 1
    for x in pat:
        n *= len(_CODE[x])
    return n


def generality_ord(pat):
    """:func:`generality` for a pattern given as ord() codes (ref :571-585)."""
    n = 1
    for c in pat:
        n *= len(_CODE[chr(c)])
    return n


class PatternEnumeration:
    """Mixed-radix bijection pattern <-> lattice cell index (ref :247-266)."""

    def __init__(self, general_pattern):
        self.genpat = general_pattern
        self.gppl = get_genpat_pos_level(general_pattern)
        self.cgppl = get_cum_genpat_pos_level(general_pattern)
        self._digit = [perm_code_no[g] for g in general_pattern]

    def pattern2num(self, pattern):
        return sum(d[x] * w for d, x, w in zip(self._digit, pattern, self.cgppl))

    def num2pattern(self, num):
        num = int(num)
        chars = []
        for g, r in zip(self.genpat, self.gppl):
            num, d = divmod(num, r)
            chars.append(_PERM[g][d])
        return "".join(chars)


class KmerEnumeration:
    """Mixed-radix bijection k-mer <-> index over the nucleotides of each position (ref :268-373)."""

    def __init__(self, general_pattern):
        self.genpat = general_pattern
        self.gppl = [len(_CODE[x]) for x in general_pattern]
        self.cgppl = []
        acc = 1
        for r in self.gppl:
            self.cgppl.append(acc)
            acc *= r

    def kmer2num(self, kmer):
        return sum(code_no[g][n] * w for g, n, w in zip(self.genpat, kmer, self.cgppl))

    def num2kmer(self, num):
        num = int(num)
        chars = []
        for g, r in zip(self.genpat, self.gppl):
            num, d = divmod(num, r)
            chars.append(_CODE[g][d])
        return "".join(chars)


def pattern2num_new_ord(cgppl, genpat, pat):
    """Cell index of a pattern given as ord() codes under an ord()-coded general pattern (ref :376-380)."""
    return sum(int(perm_code_no_np[g][p]) * w for g, p, w in zip(genpat, pat, cgppl))


def LCA_pattern_of_kmers(contexts):
    """Most specific IUPAC pattern covering all k-mers (ref :382-388)."""
    width = len(contexts[0])
    return "".join(inv_code[frozenset(c[i] for c in contexts)] for i in range(width))


def LCA_pattern_of_patterns(patterns):
    """Most specific IUPAC pattern covering all patterns (ref :390-396)."""
    width = len(patterns[0])
    return "".join(inv_code[frozenset(chain.from_iterable(_CODE[p[i]] for p in patterns))]
                   for i in range(width))


def match(pattern, context):
    """True if the k-mer ``context`` is covered by ``pattern`` (ref :399-412)."""
    return all(c in set_code[p] for p, c in zip(pattern, context))


def matches(pattern):
    """Yield every k-mer matching ``pattern``; position 0 varies fastest (ref :415-429)."""
    for tail in product(*(_CODE[x] for x in reversed(pattern))):
        yield "".join(reversed(tail))


def matches_list(pattern):
    """List form of :func:`matches`, same order (ref :602-610)."""
    return list(matches(pattern))


def subpatterns(pattern):
    """Yield every sub-pattern; position 0 varies fastest = cell-index order (ref :538-552)."""
    for tail in product(*(_PERM[x] for x in reversed(pattern))):
        yield "".join(reversed(tail))


def _level_tuples(genpat, level):
    """Sub-patterns of ``genpat`` at ``level`` as tuples of codes.

    Order = the reference's per-level generator (ref :469-478, :513-535): position 0 is
    the OUTERMOST loop, each position walks ``perm_code`` order, and a code is admitted
    only if the remaining positions can still reach the required level.
    """
    k = len(genpat)
    cap = [0] * (k + 1)
    for i in range(k - 1, -1, -1):
        cap[i] = cap[i + 1] + code_level[genpat[i]]

    def walk(i, need):
        if i == k:
            if need == 0:
                yield ()
            return
        lo = need - cap[i + 1]
        for x in _PERM[genpat[i]]:
            lv = code_level[x]
            if lo <= lv <= need:
                for rest in walk(i + 1, need - lv):
                    yield (x,) + rest

    if 0 <= level <= cap[0]:
        yield from walk(0, level)


def subpatterns_level(pattern, level):
    """Yield all sub-patterns of ``pattern`` at ``level`` as strings (ref :469-478)."""
    for t in _level_tuples(pattern, level):
        yield "".join(t)


def subpatterns_level_ord(pattern, level):
    """As :func:`subpatterns_level` but yields lists of ord() codes (ref :480-489)."""
    for t in _level_tuples(pattern, level):
        yield [ord(x) for x in t]


def subpatterns_level_ord_np(pattern, cur_level, level):
    """Ord-coded per-level generator (ref :513-535).

    ``pattern`` is the general pattern as a tuple of ord() codes and ``cur_level`` its
    level (kept for signature compatibility; it is recomputed).
    """
    gp = "".join(chr(c) for c in pattern)
    for t in _level_tuples(gp, level):
        yield tuple(ord(x) for x in t)


def get_M_U(pattern, contextD, index_mut=0):
    """Sum the (positive, negative) counts of every k-mer matching ``pattern`` (ref :192-215)."""
    M = U = None
    for kmer in matches(pattern):
        counts = contextD[kmer]
        nm, nu = counts[index_mut], counts[-1]
        if M is None:
            M, U = nm, nu
        else:
            M += nm
            U += nu
    return M, U


# ----------------------------------------------------------------------------
# compact numeric description of a general pattern, consumed by the device planner
# ----------------------------------------------------------------------------

def lattice_tables(gen_pat):
    """Per-position digit tables of the lattice of ``gen_pat``.

    Returns a dict with, for every position i, the radix r_i, the number of nucleotides
    n_i, and for every digit d < r_i: the code, its level and its ordered split pairs as
    digit pairs ``(a, b)``.  This is the same information the C++ planner derives.
    """
    pos = []
    for g in gen_pat:
        subs = _PERM[g]
        digit = perm_code_no[g]
        rows = []
        for x in subs:
            rows.append({"code": x, "level": code_level[x],
                         "pairs": [(digit[a], digit[b]) for a, b in complements.get(x, ())]})
        pos.append({"gen": g, "radix": len(subs), "nucs": len(_CODE[g]), "digits": rows})
    return pos
