"""The block list's closed form (kp_block_slot, the rule kp_blocks_kernel builds the
device block list by) against the host's block walk (kp_plan.h build_plan), every block
of each lattice: slot, packed digits and split-pair counts (host code, no GPU)."""
import os

import pytest

from kmerpapa_amd import engine


@pytest.mark.parametrize("gen_pat,max_block", [
    ("NNNNMNNNN", 0),       # the headline 9-mer (2,278,125 blocks)
    ("ANNNNMNNNNA", 0),     # the 11-mer config
    ("NNNNNNN", 16),        # one low position, six high
    ("RYSWKMBDHVN", 16),    # every IUPAC class at a high position
    ("BDHVNSWR", 64),
    ("NNNRNNN", 16),
    ("NNNN", 0),            # a single block (no high position)
    ("ACGT", 0),
])
def test_closed_form_block_order_matches_host_walk(gen_pat, max_block):
    assert engine.block_order_check(gen_pat, max_block) == 0


def test_closed_form_under_explicit_block_permutation():
    """KP_BLOCK_PERM (an experiment order, fastest high position first) goes through the
    same closed form."""
    old = os.environ.get("KP_BLOCK_PERM")
    try:
        for perm in ("0-1-2-3-4-5", "3-0-5", "5-4-3-2-1-0"):
            os.environ["KP_BLOCK_PERM"] = perm
            assert engine.block_order_check("NNNNNNN", 16) == 0
            assert engine.block_order_check("RYSWKMBDHVN", 16) == 0
    finally:
        if old is None:
            os.environ.pop("KP_BLOCK_PERM", None)
        else:
            os.environ["KP_BLOCK_PERM"] = old
