"""--score all_kmers (one rate per k-mer) against golden CLI runs of
the reference on its own 5-mer test data (tests/golden/make_golden.py job allk5):
output table byte-identical, per-alpha test losses and the selection identical.
Host code only (no lattice DP), so this runs on the CPU."""
import pytest

from tests.fixtures import golden_json, write_count_files

G = golden_json("allk5.json")


@pytest.mark.parametrize("run", ["grid", "iter"])
def test_all_kmers_cli_matches_reference(run, tmp_path, capsys):
    if G is None:
        pytest.skip("all_kmers golden not generated")
    from kmerpapa_amd import cli
    g = G[run]
    pos, bg = write_count_files(5, str(tmp_path))
    argv = list(g["argv"])
    argv[argv.index("-p") + 1] = str(pos)
    argv[argv.index("-b") + 1] = str(bg)
    out = tmp_path / "out.txt"
    rc = cli.main(argv + ["-o", str(out)])
    err = capsys.readouterr().err
    assert rc == g["rc"]
    assert out.read_text() == g["output"]
    want = [ln for ln in g["stderr"].splitlines() if ln.startswith(("alpha=", "CV DONE", "LL=", "loss="))]
    got = [ln for ln in err.splitlines() if ln.startswith(("alpha=", "CV DONE", "LL=", "loss="))]
    assert got == want
