"""Reading k-mer count files into the ``contextD`` table the DP consumes (host side).

Behaviour (filters, down-sizing to a centred k, assertions) follows the reference's
``kmerpapa.io_utils`` (src/kmerpapa/io_utils.py:3-217).  This is SURVEY.md §8(f) row 1
("next"): a text parser that feeds the hot path, kept in Python for round 1.
"""

_NUC = frozenset("ACGT")


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
