"""A lattice whose single lane does not fit the GPU: a clean KP_E_NOMEM error naming the
lattice, never a pass of zero lanes (engine.pass_cap / plan_passes with cap 0), and the
CLI prints it and exits 1.  The reference allocates its [npat, nf] arrays regardless
(CV :93-102, Fit :79-87) and fails inside numpy.  CPU test: the plan object is the real
engine.Plan's check over a stand-in device that reports 288 GB of HBM."""
import io
import os

import pytest

from kmerpapa_amd import engine


class _Dev:
    device = 0

    def mem(self):
        return 250 * 10 ** 9, 288 * 10 ** 9


def _plan(gen_pat):
    p = engine.Plan.__new__(engine.Plan)
    p._h = None
    p.device = _Dev()
    p.gen_pat = gen_pat
    p.info = engine.plan_info(gen_pat)
    p.lanes_held = 0
    p.nf = p.itype = None
    return p


def test_require_lanes_message():
    ok = _plan("NNNNMNNNN")
    assert ok.require_lanes() == ok.lanes_that_fit() >= 7
    big = _plan("NNNNNNNNNR")  # 1.15e11 cells: 461 GB per lane
    assert big.lanes_that_fit() == 0
    with pytest.raises(engine.KPError) as e:
        big.require_lanes()
    assert e.value.code == -2
    msg = str(e.value)
    assert "NNNNNNNNNR" in msg and "115,330,078,125 cells" in msg and "463.7 GB" in msg and "--super_pattern" in msg
    with pytest.raises(engine.KPError):
        engine.plan_passes([(0, 1.0, 1.0, [3.0])], 0, 5)


class _BigPlan:
    """engine.Plan stand-in for run_groups / the fit: counts accepted, no lane fits."""

    def __init__(self, gen_pat):
        self._p = _plan(gen_pat)
        self._p.device.mem = lambda: (1 * 10 ** 9, 288 * 10 ** 9)
        self.info = self._p.info
        self.ran = False

    def set_counts(self, M, U):
        pass

    def counts_begin(self, M, U, nf):
        pass

    def counts_fold(self, f, M, U):
        pass

    def lanes_that_fit(self):
        return self._p.lanes_that_fit()

    def require_lanes(self, n=1):
        return self._p.require_lanes(n)

    def reserve(self, lanes):
        raise AssertionError("no lane may be reserved")

    def run(self, groups):
        self.ran = True
        raise AssertionError("no pass may run")


@pytest.mark.parametrize("cv", [False, True])
def test_cli_lattice_too_big_message(monkeypatch, tmp_path, capsys, cv):
    from kmerpapa_amd import cli
    from tests.fixtures import write_count_files
    pos, bg = write_count_files(5, str(tmp_path))
    monkeypatch.setenv("KMERPAPA_DEVICES", "0")
    monkeypatch.setattr(engine, "get_plan", lambda dev, gp, mb=0, replica=0: _BigPlan(gp))
    args = ["-p", pos, "-b", bg, "-c", "3", "-a", "0.5", "-o", os.path.join(str(tmp_path), "out.txt")]
    if cv:
        args += ["-c", "3", "5", "--nfolds", "2", "--seed", "1"]
    assert cli.main(args) == 1
    err = capsys.readouterr().err
    assert "kmerpapa: " in err and "NNMNN" in err and "does not fit" not in err.split("kmerpapa:")[0]
    assert "per lane" in err and "--super_pattern" in err
