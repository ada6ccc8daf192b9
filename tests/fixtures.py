"""Test inputs rebuilt from committed fixtures (tests/golden/), no /root/reference needed."""
import json
import os

import numpy as np

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def golden_json(name):
    path = os.path.join(GOLDEN, name)
    if not os.path.exists(path):
        return None
    with open(path) as fh:
        return json.load(fh)


def golden_npz(name):
    return np.load(os.path.join(GOLDEN, name), allow_pickle=False)


def write_count_files(k, directory):
    """Write the reference's k-mer count files (from test_data.npz); returns (positive, background)."""
    d = golden_npz("test_data.npz")
    paths = []
    for kind in ("mutated", "background"):
        p = os.path.join(directory, f"{kind}_{k}mers.txt")
        with open(p, "w") as fh:
            for kmer, c in zip(d[f"{kind}{k}_kmers"], d[f"{kind}{k}_counts"]):
                fh.write(f"{kmer} {int(c)}\n")
        paths.append(p)
    return tuple(paths)


def write_joint_file(k, directory):
    """The "kmer positive background" file make_golden.py's cli5b job writes (background
    file order, positive = 0 where the k-mer has no positive line)."""
    d = golden_npz("test_data.npz")
    pos = {str(a): int(b) for a, b in zip(d[f"mutated{k}_kmers"], d[f"mutated{k}_counts"])}
    p = os.path.join(directory, f"joint_{k}mers.txt")
    with open(p, "w") as fh:
        for kmer, c in zip(d[f"background{k}_kmers"], d[f"background{k}_counts"]):
            fh.write(f"{kmer} {pos.get(str(kmer), 0)} {int(c)}\n")
    return p


def context_table(k):
    """contextD as cli.main builds it (read_input + zero fill), plus gen_pat and totals."""
    from kmerpapa_amd.io_utils import read_postive_and_other
    from kmerpapa_amd.pattern_utils import LCA_pattern_of_kmers, matches
    d = golden_npz("test_data.npz")
    pos = (f"{a} {int(b)}\n" for a, b in zip(d[f"mutated{k}_kmers"], d[f"mutated{k}_counts"]))
    bg = (f"{a} {int(b)}\n" for a, b in zip(d[f"background{k}_kmers"], d[f"background{k}_counts"]))
    ctx, n_unmut, n_mut = read_postive_and_other(pos, bg, None)
    gp = LCA_pattern_of_kmers(list(ctx))
    for c in matches(gp):
        ctx.setdefault(c, (0, 0))
    return ctx, gp, n_mut, n_unmut


def bits_equal(a, b):
    """float32 arrays equal bit for bit, any NaN equal to any NaN (NaN sign is meaningless)."""
    a = np.asarray(a, np.float32)
    b = np.asarray(b, np.float32)
    same = a.view(np.uint32) == b.view(np.uint32)
    return bool(np.all(same | (np.isnan(a) & np.isnan(b))))
