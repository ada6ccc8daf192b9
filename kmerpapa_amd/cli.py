"""Command line front-end -- same flags, flow and output as the reference's
``kmerpapa.cli`` (src/kmerpapa/cli.py:16-318, v0.2.4).

The flow: read counts -> penalty presets -> general pattern (LCA) + zero fill ->
(optional) grid cross-validation on the GPU -> final fit on the GPU -> partition table.
Out of scope in this build: ``--greedy``, ``--greedyCV`` and ``--BayesOpt``;
they are accepted by the parser and rejected with a message.  ``--score all_kmers`` (one
rate per k-mer, no lattice DP) evaluates its loss terms on the GPU (algorithms/all_kmers_CV.py, kp_allkmers_cv).
"""
import argparse
import json
import os
import sys
import time
from math import log

import numpy as np

from . import __version__
from .algorithms import all_kmers_CV, bottum_up_array_penalty_plus_pseudo_CV, bottum_up_array_w_numba
from .io_utils import read_input_table
from .papa import Pattern
from .score_utils import get_loss


def get_parser():
    """The argument parser (flags as cli.py:16-115)."""
    p = argparse.ArgumentParser(prog="kmerpapa",
                                description="Finds optimal k-mer pattern partition in fx. mutation data")
    p.add_argument("-p", "--positive", type=argparse.FileType("r"),
                   help="File with k-mer counts in positive set")
    p.add_argument("-n", "--negative", type=argparse.FileType("r"),
                   help="File with k-mer counts in negative set. If the negative set is created with a larger k "
                        "than the positive set then the k-mers will be collapsed so that they have the same length.")
    p.add_argument("-b", "--background", type=argparse.FileType("r"),
                   help="File with k-mer counts in backgound set (includes both positive and negative regions). "
                        "If the background set is created with a larger k than the positive set then the k-mers "
                        "will be collapsed so that they have the same length.")
    p.add_argument("-j", "--joint_context_counts", type=argparse.FileType("r"),
                   help="File with k-mer counts in positive set and background set. This option can be used "
                        "instead of having positive and negative counts in seperate files.")
    p.add_argument("-o", "--output", type=argparse.FileType("w"), default="-", metavar="PATH",
                   help="Output file (default: standard output)")
    p.add_argument("-f", "--CVfile", type=argparse.FileType("w"),
                   help="File with training and test likelihood values from cross validation.")
    p.add_argument("--verbosity", type=int, default=1,
                   help="Amount of info printed to stderr during execution. 0:silent, 1:default, 2:verbose")
    p.add_argument("--CV_only", action="store_true",
                   help="Only run crossvalidation. Do not run on whole data set using best values afterwards.")
    p.add_argument("--greedy", action="store_true",
                   help="Use a fast greedy heuristic (not available in this build).")
    p.add_argument("--BayesOpt", action="store_true",
                   help="Bayesian Optimization of pseudo_count and penalty (not available in this build).")
    p.add_argument("--greedyCV", action="store_true",
                   help="Greedy heuristic during CV (not available in this build).")
    p.add_argument("-l", "--long_output", action="store_true", help="Print all k-mers in output format.")
    p.add_argument("-s", "--super_pattern", type=str,
                   help="If a super-pattern is provided the program will only consider k-mers that match that "
                        "pattern. If for instance the \"--positive\" file contain all 5-mers at A->T mutated sites "
                        "but the \"--background\" file contains 5-mers from all sites in the genome. Then "
                        "\"--super_pattern NNANN\" should be specified to ignore 5-mers where A->T mutations cannot "
                        "happen.")
    p.add_argument("--score", type=str, default="penalty_and_pseudo",
                   choices=["penalty_and_pseudo", "all_kmers", "BIC", "AIC", "HQ", "LL"],
                   help='Type of score function. Default is "penalty_and_pseudo". '
                        '"all_kmers" will calculate a rate for each k-mer.')
    p.add_argument("-N", "--nfolds", type=int, metavar="N",
                   help="Perform cross validation with N folds. If more than one value of pseudo_count and "
                        "penalty is given then default is 2. Otherwise default is not to run cross validation "
                        "if --nfolds option is not set.")
    p.add_argument("-i", "--iterations", type=int, default=1, metavar="i", help="Repeat cross validation i times")
    p.add_argument("-a", "--pseudo_counts", type=float, metavar="a", nargs="+", default=[0.8],
                   help="Different pseudo count (alpha) values to test using cross validation")
    p.add_argument("-c", "--penalty_values", type=float, metavar="c", nargs="+",
                   help="Different penalty values to test using cross validation. If no value is set for the "
                        "default scoring function then log(#k-mers) will be used.")
    p.add_argument("--test_smaller_k", action="store_true",
                   help="By standard k is the width of the k-mers in the input data. If this option is supplied "
                        "it will test all odd numbern up to the width using CV and use the best.")
    p.add_argument("--seed", type=int, help="seed for numpy.random")
    p.add_argument("-V", "--version", action="store_true", help="Print version number and return")
    return p


def _out_of_scope(args):
    if args.greedy or args.greedyCV or args.BayesOpt:
        return "--greedy / --greedyCV / --BayesOpt"
    return None


class _Phases:
    """Wall-clock per phase of one run.  With $KMERPAPA_METRICS set to a file path, one JSON
    line is appended there at the end (no reference counterpart; SURVEY.md 5 metrics)."""

    def __init__(self):
        self.t0 = self.last = time.perf_counter()
        self.phases = {}

    def mark(self, name):
        now = time.perf_counter()
        self.phases[name] = self.phases.get(name, 0.0) + (now - self.last)
        self.last = now

    def write(self, **extra):
        path = os.environ.get("KMERPAPA_METRICS")
        if not path:
            return
        rec = dict(extra, phases_s={k: round(v, 4) for k, v in self.phases.items()},
                   total_s=round(time.perf_counter() - self.t0, 4))
        with open(path, "a") as fh:
            fh.write(json.dumps(rec) + "\n")


def write_partition(out, names, counts, contextD, alpha, beta, long_output):
    """The output table (cli.py:301-316): one row per pattern ``pattern p_neg p_pos p_rate``,
    or with ``-l`` one row per k-mer of each pattern (``matches`` order) ``context c_neg c_pos
    c_rate pattern p_neg p_pos p_rate``; rates are Python float reprs.  The -l rows are built
    from the table's arrays for all patterns at once (KmerCounts.partition_rows) and
    formatted natively (engine.format_long_rows, the same text as the reference's f-string)."""
    if long_output:
        print("context", "c_neg", "c_pos", "c_rate", "pattern", "p_neg", "p_pos", "p_rate", file=out)
        tails = [f" {pat} {Up} {Mp} {(Mp + alpha) / (Mp + Up + alpha + beta)}\n" for pat, (Mp, Up) in zip(names, counts)]
        codes, pid = contextD.partition_rows(names)
        idx = np.searchsorted(contextD.codes, codes)
        from .engine import format_long_rows
        from .io_utils import KmerCounts
        rows = KmerCounts(contextD.k, codes, contextD.M[idx], contextD.U[idx])
        try:
            text = format_long_rows(rows.letters(), rows.U, rows.M, pid, tails)
        except ZeroDivisionError:
            # a k-mer without counts: the reference prints every row before it and then
            # raises (c_rate = c_pos / 0); write those rows the same way, then raise
            letters = rows.letters()
            for i in range(len(pid)):
                cn, cp = int(rows.U[i]), int(rows.M[i])
                ctx = letters[i].tobytes().decode("ascii")
                out.write(f"{ctx} {cn} {cp} {float(cp) / (cp + cn)}{tails[int(pid[i])]}")
            raise
        out.flush()
        if hasattr(out, "buffer"):
            out.buffer.write(text)
            out.buffer.flush()
        else:
            out.write(text.decode("ascii"))
    else:
        print("pattern", "p_neg", "p_pos", "p_rate", file=out)
        for pat, (Mp, Up) in zip(names, counts):
            p = (Mp + alpha) / (Mp + Up + alpha + beta)
            print(pat, Up, Mp, p, file=out)


def main(args=None):
    """Run the program (cli.py:118-318).  Returns an exit code: 0 as the reference's, 1
    with a message on stderr when the lattice does not fit the GPU's memory (the
    reference's numpy allocation would fail there, CV :93-102)."""
    from .engine import KPError
    try:
        return _main(args)
    except KPError as e:
        if e.code != -2:  # KP_E_NOMEM
            raise
        print(f"kmerpapa: {e}", file=sys.stderr)
        return 1


def _main(args=None):
    clock = _Phases()
    parser = get_parser()
    args = parser.parse_args(args=args)
    if args.version:
        print("version:", __version__)
        print()
        return 0
    missing = _out_of_scope(args)
    if missing:
        print(f"{missing} is not part of this MI355X build (only the optimal lattice DP is).", file=sys.stderr)
        return 2
    super_pattern = Pattern(args.super_pattern) if args.super_pattern is not None else None
    try:
        contextD, n_unmut, n_mut = read_input_table(args, super_pattern)  # native reader (io_utils)
    except Exception as e:  # the reference prints help and returns 0 on bad input (cli.py:144-153)
        parser.print_help()
        print("=" * 80, file=sys.stderr)
        print("input error:", file=sys.stderr)
        print(e, file=sys.stderr)
        print("=" * 80, file=sys.stderr)
        return 0
    clock.mark("read_input")
    verbose = args.verbosity > 0
    if verbose:
        print(f"Input data read. {n_mut} positive k-mers and {n_unmut} negative k-mers", file=sys.stderr)

    if args.penalty_values is not None:
        assert args.score == "penalty_and_pseudo", \
            f"you cannot specify penalty values when using the {args.score} score function"
    else:
        presets = {"BIC": lambda: [log(n_mut)], "AIC": lambda: [2.0], "HQ": lambda: [log(log(n_mut))],
                   "LL": lambda: [0.0]}
        if args.score in presets:
            args.penalty_values = presets[args.score]()
        elif args.score == "all_kmers":
            pass
        elif args.score == "penalty_and_pseudo":
            args.penalty_values = [log(len(contextD))]  # before zero fill (cli.py:171-175)
            if verbose:
                print(f"penalty values not set. Using {args.penalty_values[0]}", file=sys.stderr)
        else:
            raise AssertionError(f"illegal score option {args.score}")

    gen_pat = contextD.lca_pattern()  # LCA_pattern_of_kmers over the table (cli.py:180)
    if args.super_pattern is not None:
        assert gen_pat == args.super_pattern
    contextD = contextD.zero_filled(gen_pat)  # every k-mer of gen_pat, missing ones (0, 0) (cli.py:185-187)
    if verbose:
        print(f"General pattern: {gen_pat}", file=sys.stderr)
    if args.CVfile is not None:
        print("k alpha P LL_test", file=args.CVfile)
    clock.mark("pattern_and_zero_fill")

    best_alpha = best_penalty = best_k = None
    ks = range(len(gen_pat), 1, -2) if args.test_smaller_k else [len(gen_pat)]
    this_contextD, this_gen_pat = contextD, gen_pat
    best_score = 1e100
    if args.nfolds is None and (len(ks) > 1 or len(args.pseudo_counts) > 1 or len(args.penalty_values) > 1
                                or args.CV_only):
        args.nfolds = 2
    if args.nfolds is not None and args.nfolds > 1:
        for k in ks:
            if verbose:
                print(f"Running {args.nfolds}-fold cross validation on {k}-mers", file=sys.stderr)
            if k != len(this_gen_pat):
                this_contextD, this_gen_pat = this_contextD.downsized(this_gen_pat, k)  # downsize_contextD
            if args.score == "all_kmers":
                this_alpha, test_score = all_kmers_CV.all_kmers(this_gen_pat, this_contextD, args.pseudo_counts,
                                                                args, n_mut, n_unmut)
                this_penalty = None
            else:
                this_alpha, this_penalty, test_score = \
                    bottum_up_array_penalty_plus_pseudo_CV.pattern_partition_bottom_up(
                        this_gen_pat, this_contextD, args.pseudo_counts, args, n_mut, n_unmut, args.penalty_values)
            if test_score < best_score:
                best_score, best_k, best_alpha, best_penalty = test_score, k, this_alpha, this_penalty
        if verbose:
            print(f"CV DONE. best_k={best_k}, best_alpha={best_alpha}, best_penalty={best_penalty}, "
                  f"best_test_LL={best_score}", file=sys.stderr)
    if args.CVfile is not None:
        args.CVfile.close()
    clock.mark("cross_validation")
    if args.CV_only:
        clock.write(gen_pat=gen_pat, cv_only=True)
        return 0

    if best_alpha is None:
        assert len(args.pseudo_counts) == 1
        best_alpha = args.pseudo_counts[0]
    if args.score != "all_kmers" and best_penalty is None:
        assert len(args.penalty_values) == 1
        best_penalty = args.penalty_values[0]
    if best_k is None:
        best_k = len(gen_pat)
    if best_k != len(gen_pat):
        contextD, gen_pat = contextD.downsized(gen_pat, best_k)

    my = n_mut / (n_mut + n_unmut)
    best_beta = (best_alpha * (1.0 - my)) / my
    if verbose:
        print(f"Training on whole data set with k={best_k} alpha={best_alpha} penalty={best_penalty}",
              file=sys.stderr)
    if args.score == "all_kmers":  # every k-mer is its own pattern, matches() order (cli.py:266-271)
        names, Ms, Us = contextD.match_rows(gen_pat)
        best_score, M, U, counts = 0, n_mut, n_unmut, list(zip(Ms, Us))
    else:
        best_score, M, U, names = bottum_up_array_w_numba.pattern_partition_bottom_up(
            gen_pat, contextD, best_alpha, best_beta, best_penalty, args, n_mut, n_unmut)
        counts = contextD.pattern_counts(names)  # get_M_U per pattern (cli.py:287)
    clock.mark("final_fit")
    # partition sanity checks of the reference (cli.py:289-292)
    assert M == n_mut
    assert U == n_unmut
    assert n_mut == sum(x[0] for x in counts)
    assert n_unmut == sum(x[1] for x in counts)
    if verbose:
        print(f"Optimal k-mer pattern partition contains {len(names)} patterns.", file=sys.stderr)
        print(f"loss={best_score}", file=sys.stderr)
        print(f"LL={get_loss(counts, best_alpha, best_beta)}", file=sys.stderr)

    write_partition(args.output, names, counts, contextD, best_alpha, best_beta, args.long_output)
    clock.mark("output")
    clock.write(gen_pat=gen_pat, patterns=len(names), best_alpha=best_alpha, best_penalty=best_penalty)
    return 0
