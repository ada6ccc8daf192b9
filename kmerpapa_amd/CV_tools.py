"""Cross-validation fold splitting (host side, numpy legacy RNG).

Same API and, crucially, the same random stream as the reference module
``kmerpapa.CV_tools`` (src/kmerpapa/CV_tools.py): every fold is a multivariate
hypergeometric draw made colour by colour with ``RandomState.hypergeometric``, in the
order the reference walks the colours, so a given seed yields bit-identical folds.

The device path never sees the ``[npat, nf]`` arrays of the reference (a 9-mer lattice
has 7.7e9 rows): :func:`fold_tables` returns only the per-k-mer fold counts, which the
C-ABI uploads (``kp_set_counts``).
"""
import threading

import numpy as np

from .pattern_utils import PatternEnumeration, generality, matches


def sample(m, colors, itype, prng):
    """Draw ``m`` balls from an urn with ``colors[i]`` balls of colour i (ref CV_tools.py:5-27).

    Colours are visited in order; colour i gets ``hypergeometric(colors[i], rest, m_left)``
    where ``rest`` counts the balls of all later colours; the walk stops once nothing is
    left to draw and the last colour takes the remainder.
    """
    colors = np.asarray(colors)
    n = len(colors)
    tail = np.cumsum(colors[::-1])[::-1]  # tail[i] = balls in colours i..n-1
    out = np.zeros(n, dtype=itype)
    left = int(m)
    draw = prng.hypergeometric
    for i in range(n - 1):
        if left < 1:
            break
        got = int(draw(int(colors[i]), int(tail[i + 1]), left))
        out[i] = got
        left -= got
    out[-1] = left
    return out


def _split_colors(colors, n_folds, itype, prng):
    """Folds 0..nf-2 by :func:`sample`, the last fold takes what is left (ref :53-57).

    Runs in C++ (``kp_fold_split`` of the engine library: the same MT19937 stream and
    legacy hypergeometric samplers, ~10x faster than one numpy call per colour); the numpy
    walk below is used only when the library is not built."""
    try:
        from . import engine
        engine.load()
    except ImportError:
        return _split_colors_numpy(colors, n_folds, itype, prng)
    return engine.fold_split(np.asarray(colors), n_folds, prng).astype(itype)


def _split_colors_numpy(colors, n_folds, itype, prng):
    """The reference's fold loop with numpy draws (kept as the executable specification)."""
    colors = np.array(colors, dtype=itype, copy=True)
    per_fold = int(colors.sum()) // n_folds
    folds = np.empty((len(colors), n_folds), dtype=itype)
    for f in range(n_folds - 1):
        s = sample(per_fold, colors, itype, prng)
        folds[:, f] = s
        colors -= s
    folds[:, n_folds - 1] = colors
    return folds


def _colors(contextD, itype):
    """Contexts in sorted order and the urn of :func:`make_all_folds_contextD_patterns`
    (ref :44-50): M counts of every context, then U counts."""
    if hasattr(contextD, "letters"):  # io_utils.KmerCounts: already in sorted order, as arrays
        contexts = contextD
        colors = np.concatenate([contextD.M, contextD.U]).astype(itype)
    else:
        contexts = sorted(contextD)
        nk = len(contexts)
        colors = np.empty(2 * nk, dtype=itype)
        for i, c in enumerate(contexts):
            nm, nu = contextD[c]
            colors[i] = nm
            colors[nk + i] = nu
    return contexts, colors


def fold_tables(contextD, n_folds, prng, itype=np.uint64):
    """Fold counts per k-mer, in sorted-context order.

    Returns ``(contexts, M, U)`` with ``M, U`` of shape ``[n_kmers, n_folds]``: exactly the
    level-0 rows :func:`make_all_folds_contextD_patterns` scatters into ``M_mem``/``U_mem``.
    """
    contexts, colors = _colors(contextD, itype)
    nk = len(contexts)
    folds = _split_colors(colors, n_folds, itype, prng)
    return contexts, folds[:nk], folds[nk:]


def all_counts(contextD, itype=np.uint64):
    """``(contexts, M, U)``: every context's counts of all data, in :func:`fold_tables`'
    order (the sum of its folds)."""
    contexts, colors = _colors(contextD, itype)
    nk = len(contexts)
    return contexts, colors[:nk], colors[nk:]


def fold_stream(contextD, n_folds, prng, itype=np.uint64):
    """:func:`fold_tables` one fold at a time: yields ``(f, M_f, U_f)`` (``[n_kmers]``,
    sorted-context order) for f = 0 .. n_folds-1 as each fold is drawn, the same draws
    from the same stream (each fold is one :func:`sample` in C++, ``kp_fold_sample``; the
    last fold takes what is left).  The CV driver starts the GPU passes of fold 0 while
    the later folds are still being drawn."""
    from . import engine
    contexts, colors = _colors(contextD, itype)
    nk = len(contexts)
    col = colors.astype(np.uint64)
    per_fold = int(col.sum()) // n_folds  # n_samples = n // n_folds (ref :51)
    for f in range(n_folds - 1):
        s = engine.fold_sample(col, per_fold, prng)
        col -= s
        yield f, s[:nk].astype(itype), s[nk:].astype(itype)
    yield n_folds - 1, col[:nk].astype(itype), col[nk:].astype(itype)


def fold_feed(contextD, gen_pat, n_folds, prng, itype=np.uint64, on_done=None):
    """Start the pipelined fold split of the CV driver: returns ``(feed, thread)``, an
    engine.FoldFeed that receives fold f's counts in k-mer order as soon as
    :func:`fold_stream` has drawn it, and the producer thread (the caller joins it).  The
    draws start first: the all-data counts and the k-mer order, which only the scatter into
    k-mer order needs, are computed beside fold 0's draw (the native sampler drops the
    GIL), so fold 0 arrives one k-mer ordering earlier.  ``on_done()`` runs after the last
    fold.  Same draws from the same stream as :func:`fold_tables`."""
    from . import engine
    nk = generality(gen_pat)
    box = {}
    ready = threading.Event()

    def produce():
        try:
            for f, Mf, Uf in fold_stream(contextD, n_folds, prng, itype):
                ready.wait()
                if "feed" not in box:  # the caller's side failed and raises its own error
                    return
                mk = np.zeros(nk, itype)
                uk = np.zeros(nk, itype)
                mk[box["idx"]] = Mf
                uk[box["idx"]] = Uf
                box["feed"].put(f, mk, uk)
            if on_done is not None:
                on_done()
        except BaseException as e:  # the GPU side raises it from feed.get
            ready.wait()
            if "feed" in box:
                box["feed"].fail(e)

    th = threading.Thread(target=produce)
    th.start()
    try:
        contexts, Ma, Ua = all_counts(contextD, itype)
        idx = engine.kmer_order(gen_pat, contexts if hasattr(contexts, "letters") else list(contexts))
        M_all = np.zeros(nk, itype)
        U_all = np.zeros(nk, itype)
        M_all[idx] = Ma
        U_all[idx] = Ua
        box["idx"] = idx
        box["feed"] = engine.FoldFeed(M_all, U_all, n_folds)
    finally:
        ready.set()
    return box["feed"], th


def make_all_folds_contextD_patterns(contextD, U_mem, M_mem, general_pattern, prng, itype=np.uint64):
    """Fill the k-mer rows of ``M_mem``/``U_mem`` ``[npat, nf]`` with fold counts (ref :30-62)."""
    PE = PatternEnumeration(general_pattern)
    contexts, M, U = fold_tables(contextD, U_mem.shape[1], prng, itype)
    for i, c in enumerate(contexts):
        row = PE.pattern2num(c)
        M_mem[row] = M[i]
        U_mem[row] = U[i]


def make_all_folds_contextD_kmers(contextD, U_mem, M_mem, general_pattern, prng):
    """Fold counts for every k-mer of ``general_pattern`` in :func:`matches` order (ref :65-96)."""
    if hasattr(contextD, "letters"):  # io_utils.KmerCounts: matches() order = KmerEnumeration order
        from .engine import kmer_order
        nk = generality(general_pattern)
        idx = kmer_order(general_pattern, contextD)
        if len(contextD) != nk:
            raise KeyError("the count table must hold every k-mer of the general pattern (zero-filled)")
        colors = np.zeros(2 * nk, dtype=np.uint64)
        colors[idx] = contextD.M
        colors[nk + idx] = contextD.U
    else:
        contexts = list(matches(general_pattern))
        nk = len(contexts)
        colors = np.zeros(2 * nk, dtype=np.uint64)
        for i, c in enumerate(contexts):
            nm, nu = contextD[c]
            colors[i] = nm
            colors[nk + i] = nu
    folds = _split_colors(colors, U_mem.shape[1], np.uint64, prng)
    M_mem[:nk] = folds[:nk]
    U_mem[:nk] = folds[nk:]


def make_all_folds(kmer_table, n_folds, n_repeats, prng):
    """Split a count table into ``n_folds`` folds, ``n_repeats`` times (ref :124-147).

    Returns an array of shape ``(n_repeats, n_folds) + kmer_table.shape``.
    """
    kmer_table = np.asarray(kmer_table)
    itype = kmer_table.dtype
    out = np.zeros((n_repeats, n_folds) + kmer_table.shape, dtype=itype)
    for r in range(n_repeats):
        folds = _split_colors(kmer_table.reshape(-1), n_folds, itype, prng)
        for f in range(n_folds):
            out[r, f] = folds[:, f].reshape(kmer_table.shape)
    return out
