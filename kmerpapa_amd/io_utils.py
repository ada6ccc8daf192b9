"""Reading k-mer count files into the ``contextD`` table the DP consumes (host side).

Behaviour (filters, down-sizing to a centred k, assertions) follows the reference's
``kmerpapa.io_utils`` (src/kmerpapa/io_utils.py:3-217); SURVEY.md §8(f) row 1.

Two forms:

* ``read_dict`` / ``read_joint_kmer_counts`` / ``read_postive_and_other`` /
  ``read_input``: the reference's API, returning plain dicts (pure Python, as the
  reference; kept for API users and as the cross-check of the native reader);
* ``read_input_table``: what the CLI uses -- the C++ reader of libkmerpapa_hip.so
  (``kp_kmer_parse``, kmerpapa_amd/csrc/kp_io.h) into a :class:`KmerCounts` table of
  sorted 2-bit k-mer codes and count arrays, which the CV, fit and output steps consume
  as arrays (no per-k-mer Python objects).  ~50x faster at 11-mers (2 M lines per file).
"""
from collections.abc import Mapping

import numpy as np

from .pattern_utils import code as _code, inv_code as _inv_code

_NUC = frozenset("ACGT")
_LETTERS = np.frombuffer(b"ACGT", dtype=np.uint8)


def _as_count(tok):
    try:
        return int(tok)
    except ValueError:
        return int(float(tok))


def _centre_window(width, length):
    """Slice bounds that keep the central ``length`` letters of a ``width``-mer (ref :50-79)."""
    lo = width // 2 - length // 2
    return lo, lo + length


def read_joint_kmer_counts(f, super_pattern, n_scale=1):
    """Read ``kmer n_positive n_background`` lines (ref io_utils.py:3-46).

    Returns ``(contextD, n_negative_total, n_positive_total)``.
    """
    table = {}
    n_sites = n_pos = 0
    for line in f:
        kmer, pos_tok, bg_tok = line.split()
        if not set(kmer) <= _NUC:
            continue
        bg = _as_count(bg_tok)
        pos = _as_count(pos_tok)
        assert n_scale * bg - pos >= 0, (
            "background counts should be larger than the positive counts so that a negative "
            f"set can be created by subtraction the positive count from the background count. "
            f"Problematic kmer: {kmer}")
        if super_pattern is not None and kmer not in super_pattern:
            continue
        n_sites += n_scale * bg
        n_pos += pos
        table[kmer] = (pos, n_scale * bg - pos)
    f.close()
    return table, n_sites - n_pos, n_pos


def downsize_contextD(D, general_pattern, length):
    """Collapse k-mer counts onto their central ``length``-mers (ref io_utils.py:50-79)."""
    out = {}
    lo = hi = None
    for context, counts in D.items():
        if lo is None:
            assert length is not None
            assert len(context) > length, f"k-mer:{context} cannot be reduced to length {length}"
            lo, hi = _centre_window(len(context), length)
        key = context[lo:hi]
        acc = out.setdefault(key, [0] * len(counts))
        for i, v in enumerate(counts):
            acc[i] += v
    return out, general_pattern[lo:hi]


def read_dict(f, super_pattern, length=None):
    """Read ``kmer count`` lines, optionally down-sizing and filtering (ref io_utils.py:82-136).

    Returns ``(counts_by_kmer, total_count)``.
    """
    if length is None and super_pattern is not None:
        length = len(super_pattern)
    table = {}
    total = 0
    lo = hi = None
    for line in f:
        context, tok = line.split()
        if not set(context) <= _NUC:
            continue
        count = _as_count(tok)
        assert count >= 0, f"negative counts are not allowed, bad line:\n{line.strip()}"
        if lo is None:
            if length is not None and length != len(context):
                assert len(context) > length
                lo, hi = _centre_window(len(context), length)
            else:
                lo, hi = 0, len(context)
        context = context[lo:hi]
        if super_pattern is not None:
            assert len(super_pattern) == len(context)
            if context not in super_pattern:
                continue
        total += count
        table[context] = table.get(context, 0) + count
    return table, total


def read_postive_and_other(fpos, fother, super_pattern, n_scale=1, background=True):
    """Combine a positive and a background/negative count file (ref io_utils.py:139-184).

    Returns ``(contextD, n_negative_total, n_positive_total)``.
    """
    posD, allpos = read_dict(fpos, super_pattern)
    otherD, allother = read_dict(fother, super_pattern, length=len(next(iter(posD.keys()))))
    table = {}
    for context in sorted(set(posD) | set(otherD)):
        n_pos = posD.get(context, 0)
        n_other = n_scale * otherD.get(context, 0)
        if background:
            assert n_other >= n_pos, (
                "background counts should be larger than the positive counts so that a negative "
                "set can be created by subtraction the positive count from the background count. "
                f"Problematic k-mer: {context}")
            n_other -= n_pos
        table[context] = (n_pos, n_other)
    if background:
        allother -= allpos
    return table, allother, allpos


def read_input(args, super_pattern):
    """Dispatch on the CLI's input options (ref io_utils.py:187-217)."""
    assert (args.positive is None) != (args.joint_context_counts is None), (
        "Either the --positive option or the --join_context_counts option (but not both) "
        "must be used to provide input data.")
    if args.positive is not None:
        assert (args.negative is None) != (args.background is None), (
            "If the --joint_context_counts option is not used then either the --negative or the "
            "--background option (but not both) must be used.")
        if args.negative is not None:
            return read_postive_and_other(args.positive, args.negative, super_pattern,
                                          n_scale=1, background=False)
        return read_postive_and_other(args.positive, args.background, super_pattern,
                                      n_scale=1, background=True)
    return read_joint_kmer_counts(args.joint_context_counts, super_pattern, n_scale=1)


# ----------------------------------------------------------------------------
# native reader and the array-backed count table (the CLI's path)
# ----------------------------------------------------------------------------

def _codes_of_pattern(pattern):
    """Sorted 2-bit codes of every k-mer matching an IUPAC pattern."""
    codes = np.zeros(1, np.uint64)
    for g in pattern:
        bases = np.array(sorted("ACGT".index(c) for c in _code[g]), np.uint64)
        codes = (codes[:, None] * np.uint64(4) + bases[None, :]).reshape(-1)
    return codes


class KmerCounts(Mapping):
    """k-mer -> (positive, negative) counts as arrays: ``codes`` (uint64, sorted and
    unique; 2 bits per letter, A=0 C=1 G=2 T=3, first letter most significant, so code
    order is sorted k-mer order) and ``M``/``U`` (int64).  A read-only ``contextD`` for
    every reader of the reference's dict (lookup, ``in``, sorted iteration, ``len``);
    the engine takes the arrays directly (``letters()``)."""

    def __init__(self, k, codes, M, U):
        self.k = int(k)
        self.codes = np.ascontiguousarray(codes, np.uint64)
        self.M = np.ascontiguousarray(M, np.int64)
        self.U = np.ascontiguousarray(U, np.int64)
        self._keys = None

    def letters(self):
        """ASCII letters ``[n, k]`` (uint8) of every k-mer, in table order."""
        shifts = np.arange(2 * (self.k - 1), -1, -2, dtype=np.uint64)
        return _LETTERS[((self.codes[:, None] >> shifts[None, :]) & np.uint64(3)).astype(np.intp)]

    def kmer_at(self, i):
        return self.letters()[i].tobytes().decode("ascii") if self._keys is None else self._keys[i]

    def _key_list(self):
        if self._keys is None:
            raw = self.letters()
            self._keys = [] if raw.shape[0] == 0 else \
                np.ascontiguousarray(raw).view(f"S{self.k}").reshape(-1).astype(str).tolist()
        return self._keys

    def _find(self, kmer):
        if not isinstance(kmer, str) or len(kmer) != self.k:
            return None
        c = 0
        for ch in kmer:
            d = "ACGT".find(ch)
            if d < 0:
                return None
            c = 4 * c + d
        i = int(np.searchsorted(self.codes, np.uint64(c)))
        return i if i < self.codes.shape[0] and int(self.codes[i]) == c else None

    def __getitem__(self, kmer):
        i = self._find(kmer)
        if i is None:
            raise KeyError(kmer)
        return int(self.M[i]), int(self.U[i])

    def __contains__(self, kmer):
        return self._find(kmer) is not None

    def __iter__(self):
        return iter(self._key_list())

    def __len__(self):
        return int(self.codes.shape[0])

    def lca_pattern(self):
        """LCA_pattern_of_kmers over the table's k-mers (pattern_utils.py:382-388)."""
        out = []
        for i in range(self.k):
            d = (self.codes >> np.uint64(2 * (self.k - 1 - i))) & np.uint64(3)
            present = np.bincount(d.astype(np.intp), minlength=4) > 0
            out.append(_inv_code[frozenset(b for b, f in zip("ACGT", present) if f)])
        return "".join(out)

    def zero_filled(self, gen_pat):
        """Every k-mer of ``gen_pat``, missing ones with (0, 0): the CLI's zero fill
        (cli.py:185-187) as a new table."""
        allc = _codes_of_pattern(gen_pat)
        idx = np.searchsorted(allc, self.codes)
        if self.codes.shape[0] and (idx.max() >= allc.shape[0] or (allc[np.minimum(idx, allc.shape[0] - 1)]
                                                                     != self.codes).any()):
            raise ValueError(f"k-mers outside the general pattern {gen_pat}")
        M = np.zeros(allc.shape[0], np.int64)
        U = np.zeros(allc.shape[0], np.int64)
        M[idx] = self.M
        U[idx] = self.U
        return KmerCounts(len(gen_pat), allc, M, U)

    def downsized(self, general_pattern, length):
        """downsize_contextD (io_utils.py:50-79): counts summed onto the central ``length``
        letters; returns ``(table, general_pattern[lo:hi])``."""
        assert len(self) > 0 and self.k > length, f"k-mers cannot be reduced to length {length}"
        lo = self.k // 2 - length // 2
        drop = np.uint64(2 * (self.k - lo - length))
        mask = np.uint64((1 << (2 * length)) - 1)
        sub = (self.codes >> drop) & mask
        order = np.argsort(sub, kind="stable")
        sub = sub[order]
        first = np.flatnonzero(np.r_[True, sub[1:] != sub[:-1]])
        M = np.add.reduceat(self.M[order], first)
        U = np.add.reduceat(self.U[order], first)
        return KmerCounts(length, sub[first], M, U), general_pattern[lo:lo + length]

    def match_rows(self, pattern):
        """(k-mers, positive counts, negative counts) of every k-mer matching ``pattern``, in
        :func:`matches` order (position 0 fastest), as Python lists."""
        codes = np.zeros(1, np.uint64)
        for i in range(len(pattern) - 1, -1, -1):  # position 0 innermost = fastest
            bases = np.array(["ACGT".index(c) for c in _code[pattern[i]]], np.uint64)
            codes = (codes[:, None] + bases[None, :] * np.uint64(4 ** (len(pattern) - 1 - i))).reshape(-1)
        idx = np.searchsorted(self.codes, codes)
        sub = KmerCounts(self.k, codes, self.M[idx], self.U[idx])
        return sub._key_list(), sub.M.tolist(), sub.U.tolist()

    def partition_rows(self, patterns):
        """Every k-mer of every pattern, as :meth:`match_rows` lists them (patterns in order,
        each one's k-mers in :func:`matches` order), vectorised over all patterns at once.
        Returns ``(codes, pid)``: the k-mers' 2-bit codes and each row's pattern index."""
        P = len(patterns)
        if P == 0:
            return np.zeros(0, np.uint64), np.zeros(0, np.int64)
        k = len(patterns[0])
        raw = np.frombuffer("".join(patterns).encode("ascii"), np.uint8).reshape(P, k)
        size = np.zeros(256, np.int64)
        base = np.zeros((256, 4), np.uint64)
        for c, nucs in _code.items():
            size[ord(c)] = len(nucs)
            base[ord(c), :len(nucs)] = ["ACGT".index(n) for n in nucs]
        pid = np.arange(P, dtype=np.int64)
        codes = np.zeros(P, np.uint64)
        for i in range(k - 1, -1, -1):  # position 0 last = innermost = fastest
            ch = raw[pid, i]
            rep = size[ch]
            start = np.cumsum(rep) - rep
            pid = np.repeat(pid, rep)
            codes = np.repeat(codes, rep)
            j = np.arange(pid.size) - np.repeat(start, rep)
            codes = codes + base[np.repeat(ch, rep), j] * np.uint64(4 ** (k - 1 - i))
        return codes, pid

    def pattern_counts(self, patterns):
        """get_M_U (pattern_utils.py:192-215) for many patterns: summed (M, U) of the
        k-mers each pattern matches (every one must be in the table)."""
        out = []
        for pat in patterns:
            idx = np.searchsorted(self.codes, _codes_of_pattern(pat))
            out.append((int(self.M[idx].sum()), int(self.U[idx].sum())))
        return out


def _read_bytes(f):
    data = f.buffer.read() if hasattr(f, "buffer") else f.read()
    return data.encode() if isinstance(data, str) else bytes(data)


def _native(text, columns, super_pattern, length=0):
    from . import engine  # the C++ reader lives in libkmerpapa_hip.so
    return engine.parse_kmer_counts(text, columns, str(super_pattern) if super_pattern is not None else None,
                                    length)


def read_input_table(args, super_pattern):
    """read_input (ref io_utils.py:187-217) through the native reader.

    Returns ``(KmerCounts, n_negative_total, n_positive_total)``; the same tables, totals
    and input errors as :func:`read_input` (tests/test_io_native.py)."""
    assert (args.positive is None) != (args.joint_context_counts is None), (
        "Either the --positive option or the --join_context_counts option (but not both) "
        "must be used to provide input data.")
    if args.positive is None:
        f = args.joint_context_counts
        k, codes, pos, neg, n_neg, n_pos = _native(_read_bytes(f), 3, super_pattern)
        f.close()
        return KmerCounts(k, codes, pos, neg), n_neg, n_pos
    assert (args.negative is None) != (args.background is None), (
        "If the --joint_context_counts option is not used then either the --negative or the "
        "--background option (but not both) must be used.")
    background = args.negative is None
    fother = args.background if background else args.negative
    kp, cp, mp, _, allpos, _ = _native(_read_bytes(args.positive), 2, super_pattern)
    if cp.shape[0] == 0:
        raise StopIteration  # next(iter(posD.keys())) on an empty table (ref :148)
    ko, co, mo, _, allother, _ = _native(_read_bytes(fother), 2, super_pattern, kp)
    codes = np.union1d(cp, co)
    n_pos = np.zeros(codes.shape[0], np.int64)
    n_other = np.zeros(codes.shape[0], np.int64)
    n_pos[np.searchsorted(codes, cp)] = mp
    n_other[np.searchsorted(codes, co)] = mo
    table = KmerCounts(kp, codes, n_pos, n_other)
    if background:
        bad = np.flatnonzero(n_other < n_pos)
        assert bad.shape[0] == 0, (
            "background counts should be larger than the positive counts so that a negative "
            "set can be created by subtraction the positive count from the background count. "
            f"Problematic k-mer: {table.kmer_at(int(bad[0])) if bad.shape[0] else ''}")
        table.U = n_other - n_pos
        allother -= allpos
    return table, allother, allpos
