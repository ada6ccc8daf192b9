"""The native k-mer count reader (kp_kmer_parse, kmerpapa_amd/csrc/kp_io.h) and the
array-backed KmerCounts table against the pure-Python readers that mirror the
reference's io_utils (src/kmerpapa/io_utils.py:3-217).  CPU only: the parser is host
code in libkmerpapa_hip.so."""
import io
import itertools
import types

import numpy as np
import pytest

from kmerpapa_amd import engine, io_utils
from kmerpapa_amd.papa import Pattern
from kmerpapa_amd.pattern_utils import LCA_pattern_of_kmers, get_M_U, matches


class _F(io.TextIOWrapper):
    """A text file over bytes, like argparse.FileType('r') gives (has .buffer)."""

    def __init__(self, data):
        super().__init__(io.BytesIO(data), encoding="utf-8")


def _args(**kw):
    base = dict(positive=None, negative=None, background=None, joint_context_counts=None)
    base.update(kw)
    return types.SimpleNamespace(**base)


def _rand_lines(rng, k, n, alphabet="ACGT", dup=True):
    out = []
    for _ in range(n):
        kmer = "".join(rng.choice(list(alphabet), size=k))
        out.append(kmer)
    if dup:
        out += out[: n // 5]
    return out


def _write2(kmers, counts, sep=" ", eol="\n"):
    return "".join(f"{a}{sep}{b}{eol}" for a, b in zip(kmers, counts)).encode()


def _same_table(native, pydict):
    assert len(native) == len(pydict)
    assert dict(native.items()) == {k: tuple(v) for k, v in pydict.items()}
    assert list(native) == sorted(pydict)


@pytest.mark.parametrize("sep,eol", [(" ", "\n"), ("\t", "\r\n"), ("  ", "\r")])
def test_positive_background_matches_python(sep, eol):
    rng = np.random.RandomState(3)
    km = _rand_lines(rng, 5, 300) + ["ACGNT", "acgta"]  # non-ACGT lines are skipped
    bg = [int(x) for x in rng.randint(5, 50, len(km))]
    pos = [int(x) for x in rng.randint(0, 5, len(km))]
    pos_txt = _write2(km, pos, sep, eol)
    bg_txt = _write2(km, bg, sep, eol)
    ref = io_utils.read_input(_args(positive=_F(pos_txt), background=_F(bg_txt)), None)
    got = io_utils.read_input_table(_args(positive=_F(pos_txt), background=_F(bg_txt)), None)
    _same_table(got[0], ref[0])
    assert got[1:] == ref[1:]
    # negative file instead of background
    ref = io_utils.read_input(_args(positive=_F(pos_txt), negative=_F(bg_txt)), None)
    got = io_utils.read_input_table(_args(positive=_F(pos_txt), negative=_F(bg_txt)), None)
    _same_table(got[0], ref[0])
    assert got[1:] == ref[1:]


def test_downsizing_and_super_pattern():
    rng = np.random.RandomState(5)
    km = _rand_lines(rng, 7, 400)
    counts = [str(int(x)) for x in rng.randint(0, 30, len(km))]
    counts[0], counts[1], counts[2] = "1_000", "2.9", "1e2"  # int() and int(float()) forms
    txt = _write2(km, counts)
    for sp in ("NNNNN", "NRNYN", "ANNNA"):
        ref = io_utils.read_dict(_F(txt), Pattern(sp))
        k, codes, c0, c1, tot, _ = engine.parse_kmer_counts(txt, 2, sp)
        table = io_utils.KmerCounts(k, codes, c0, c1)
        assert k == 5 and tot == ref[1]
        assert {kk: v[0] for kk, v in table.items()} == ref[0]
    ref = io_utils.read_dict(_F(txt), None, length=3)
    k, codes, c0, c1, tot, _ = engine.parse_kmer_counts(txt, 2, None, 3)
    assert k == 3 and tot == ref[1]
    assert {kk: v[0] for kk, v in io_utils.KmerCounts(k, codes, c0, c1).items()} == ref[0]


def test_joint_counts_last_line_wins():
    rng = np.random.RandomState(7)
    km = _rand_lines(rng, 4, 200)
    lines = []
    for x in km:
        bg = int(rng.randint(3, 40))
        lines.append(f"{x} {int(rng.randint(0, 3))} {bg}\n")
    lines.append("NNNN 5 1\n")  # skipped before the counts are checked
    txt = "".join(lines).encode()
    for sp in (None, "NRNN"):
        patt = Pattern(sp) if sp else None
        ref = io_utils.read_input(_args(joint_context_counts=_F(txt)), patt)
        got = io_utils.read_input_table(_args(joint_context_counts=_F(txt)), patt)
        assert dict(got[0].items()) == ref[0]
        assert got[1:] == ref[1:]


@pytest.mark.parametrize("text,columns", [
    (b"ACGT 1\n\nACGA 2\n", 2),          # blank line: tuple unpacking fails
    (b"ACGT 1 2\n", 2),                  # too many tokens
    (b"ACGT\n", 2),                      # too few
    (b"ACGT -1\n", 2),                   # negative count
    (b"ACGT x1\n", 2),                   # not a number
    (b"ACGT inf\n", 2),
    (b"ACGT nan\n", 2),
    (b"ACGT 1__0\n", 2),
    (b"ACGT 5 2\n", 3),                  # background < positive
])
def test_input_errors_match_python(text, columns):
    if columns == 2:
        with pytest.raises(Exception):
            io_utils.read_dict(_F(text), None)
    else:
        with pytest.raises(Exception):
            io_utils.read_joint_kmer_counts(_F(text), None)
    with pytest.raises(ValueError):
        engine.parse_kmer_counts(text, columns)


def test_error_messages():
    with pytest.raises(ValueError, match="not enough values to unpack"):
        engine.parse_kmer_counts(b"ACGT 1\n\n", 2)
    with pytest.raises(ValueError, match="could not convert string to float: 'x1'"):
        engine.parse_kmer_counts(b"ACGT x1\n", 2)
    with pytest.raises(ValueError, match="Problematic kmer: ACGT"):
        engine.parse_kmer_counts(b"ACGT 5 2\n", 3)
    with pytest.raises(ValueError, match="different lengths"):
        engine.parse_kmer_counts(b"ACGT 5\nACG 2\n", 2)
    with pytest.raises(StopIteration):
        io_utils.read_input_table(_args(positive=_F(b"NNNN 1\n"), background=_F(b"ACGT 1\n")), None)
    with pytest.raises(AssertionError, match="Problematic k-mer: ACGT"):
        io_utils.read_input_table(_args(positive=_F(b"ACGT 5\n"), background=_F(b"ACGT 1\n")), None)


def test_table_helpers_match_dict_forms():
    rng = np.random.RandomState(11)
    gen_pat = "NMRN"
    kmers = [k for k in matches(gen_pat) if rng.rand() < 0.7]
    D = {k: (int(rng.randint(0, 9)), int(rng.randint(0, 99))) for k in kmers}
    codes = np.array([int("".join(str("ACGT".index(c)) for c in k), 4) for k in sorted(D)], np.uint64)
    T = io_utils.KmerCounts(4, codes, [D[k][0] for k in sorted(D)], [D[k][1] for k in sorted(D)])
    assert T.lca_pattern() == LCA_pattern_of_kmers(list(D))
    full = T.zero_filled(gen_pat)
    Dz = dict(D)
    for c in matches(gen_pat):
        Dz.setdefault(c, (0, 0))
    assert dict(full.items()) == Dz
    pats = ["NMRN", "AMRN", "NAGT", "GMAN"]
    assert full.pattern_counts(pats) == [get_M_U(p, Dz) for p in pats]
    small, gp = full.downsized(gen_pat, 2)
    ref, rgp = io_utils.downsize_contextD(Dz, gen_pat, 2)
    assert gp == rgp and dict(small.items()) == {k: tuple(v) for k, v in ref.items()}
    # the engine's k-mer order from letters == from strings
    assert (engine.kmer_order(gen_pat, full) == engine.kmer_order(gen_pat, list(full))).all()
    assert "AGAA" not in full and "ACGT" in full and full.get("AAAA") == Dz.get("AAAA")


def test_all_4mers_roundtrip():
    kmers = ["".join(p) for p in itertools.product("ACGT", repeat=4)]
    txt = _write2(kmers, range(len(kmers)))
    k, codes, c0, c1, tot, _ = engine.parse_kmer_counts(txt, 2)
    assert k == 4 and (codes == np.arange(256, dtype=np.uint64)).all() and (c0 == np.arange(256)).all()
    assert tot == sum(range(256))


def test_reference_test_data_tables(tmp_path):
    """The reference's 5-mer files (tests/golden/test_data.npz), as -p/-b, -p/-n and -j
    inputs: the native table equals the Python reader's dict, and the CLI's LCA/zero-fill
    steps agree."""
    from tests.fixtures import write_count_files, write_joint_file
    pos, bg = write_count_files(5, str(tmp_path))
    joint = write_joint_file(5, str(tmp_path))
    for kw in (dict(positive=pos, background=bg), dict(positive=pos, negative=bg), dict(joint_context_counts=joint)):
        ref = io_utils.read_input(_args(**{k: open(v) for k, v in kw.items()}), None)
        got = io_utils.read_input_table(_args(**{k: open(v) for k, v in kw.items()}), None)
        assert dict(got[0].items()) == {k: tuple(v) for k, v in ref[0].items()}
        assert got[1:] == ref[1:]
        gp = LCA_pattern_of_kmers(list(ref[0]))
        assert got[0].lca_pattern() == gp == "NNMNN"
        full = got[0].zero_filled(gp)
        assert len(full) == 512 and full.pattern_counts([gp]) == [get_M_U(gp, dict(full.items()))]


def test_match_rows_order():
    """KmerCounts.match_rows: the k-mers of a pattern in matches() order (position 0
    fastest) with their counts, as the long output walks them (cli.py:305-311)."""
    rng = np.random.RandomState(1)
    gp = "NMRS"
    D = {k: (int(rng.randint(0, 9)), int(rng.randint(1, 99))) for k in matches(gp)}
    codes = np.array([int("".join(str("ACGT".index(c)) for c in k), 4) for k in sorted(D)], np.uint64)
    T = io_utils.KmerCounts(4, codes, [D[k][0] for k in sorted(D)], [D[k][1] for k in sorted(D)])
    for pat in ["NMRS", "ACRS", "NAGS", "TMGC"]:
        ks, m, u = T.match_rows(pat)
        assert ks == list(matches(pat))
        assert m == [D[x][0] for x in ks] and u == [D[x][1] for x in ks]
