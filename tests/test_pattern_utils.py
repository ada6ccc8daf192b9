"""Pattern algebra API (kmerpapa_amd.pattern_utils) against the reference's own test
(tests/test_pattern_utils.py:4-28 of the reference: per-level enumeration, index round
trips) and against the enumeration orders the reference produced (tests/golden/enum.json)."""
import hashlib

import pytest

from kmerpapa_amd import pattern_utils as pu
from tests.fixtures import golden_json

ENUM = golden_json("enum.json")


@pytest.mark.parametrize("gp", ["NNMNN", "SWSW"])
def test_enumeration_api(gp):
    npat = pu.pattern_max(gp)
    cgppl = pu.get_cum_genpat_pos_level(gp)
    level = pu.pattern_level(gp)
    PE = pu.PatternEnumeration(gp)
    seen = 0
    for lv in range(level + 1):
        for pat in pu.subpatterns_level(gp, lv):
            assert pu.pattern_level(pat) == lv
            assert PE.num2pattern(PE.pattern2num(pat)) == pat
            seen += 1
    assert seen == npat
    gpo = tuple(ord(x) for x in gp)
    seen = 0
    for lv in range(level + 1):
        for op in pu.subpatterns_level_ord_np(gpo, level, lv):
            pat = "".join(chr(x) for x in op)
            assert pu.pattern_level(pat) == lv
            assert PE.num2pattern(pu.pattern2num_new_ord(cgppl, gpo, op)) == pat
            seen += 1
    assert seen == npat


@pytest.mark.parametrize("gp", sorted(ENUM["enum"]))
def test_enumeration_order_matches_reference(gp):
    ref = ENUM["enum"][gp]
    level = pu.pattern_level(gp)
    assert level == ref["level"]
    assert pu.pattern_max(gp) == ref["pattern_max"]
    per = [list(pu.subpatterns_level(gp, lv)) for lv in range(level + 1)]
    gpo = tuple(ord(x) for x in gp)
    per_ord = [["".join(chr(c) for c in t) for t in pu.subpatterns_level_ord_np(gpo, level, lv)]
               for lv in range(level + 1)]
    PE = pu.PatternEnumeration(gp)
    assert [len(x) for x in per] == ref["level_sizes"]
    assert hashlib.sha256("|".join(",".join(x) for x in per).encode()).hexdigest() == ref["sha_levels"]
    assert hashlib.sha256("|".join(",".join(x) for x in per_ord).encode()).hexdigest() == ref["sha_levels_ord"]
    nums = ",".join(str(PE.pattern2num(p)) for x in per for p in x)
    assert hashlib.sha256(nums.encode()).hexdigest() == ref["sha_nums"]
    if ref.get("matches") is not None:
        assert list(pu.matches(gp)) == ref["matches"]


def test_lca():
    for key, want in ENUM["lca"].items():
        assert pu.LCA_pattern_of_kmers(key.split("|")) == want


def test_split_children_have_smaller_digits():
    """Every split child has a strictly smaller digit at the split position (the fact
    that makes ascending cell index a topological order of the DP)."""
    for g, subs in pu.perm_code.items():
        for x in subs:
            for a, b in pu.complements.get(x, ()):
                assert pu.perm_code_no[g][a] < pu.perm_code_no[g][x]
                assert pu.perm_code_no[g][b] < pu.perm_code_no[g][x]
                assert pu.set_code[a] | pu.set_code[b] == pu.set_code[x]
                assert not (pu.set_code[a] & pu.set_code[b])


def test_nucleotides_come_first_in_perm_code():
    for g, subs in pu.perm_code.items():
        assert subs[:len(pu.code[g])] == pu.code[g]
        assert subs[-1] == g


def test_kmer_enumeration_roundtrip_and_get_M_U():
    gp = "NMN"
    KE = pu.KmerEnumeration(gp)
    kmers = list(pu.matches(gp))
    assert [KE.kmer2num(k) for k in kmers] == list(range(len(kmers)))
    assert all(KE.num2kmer(i) == k for i, k in enumerate(kmers))
    ctx = {k: (i, 2 * i) for i, k in enumerate(kmers)}
    M, U = pu.get_M_U("NMN", ctx)
    assert (M, U) == (sum(range(len(kmers))), 2 * sum(range(len(kmers))))
    assert pu.get_M_U("ACA", ctx) == ctx["ACA"]
