"""CLI behaviour that needs no GPU (reference tests/test_cli.py:8-23 and cli.py:130-153)."""
import pytest

from kmerpapa_amd import cli


def test_main_without_input_prints_help_and_returns_0(capsys):
    assert cli.main([]) == 0
    assert "usage: kmerpapa" in capsys.readouterr().out


def test_show_help(capsys):
    with pytest.raises(SystemExit):
        cli.main(["-h"])
    assert "kmerpapa" in capsys.readouterr().out


def test_version(capsys):
    assert cli.main(["-V"]) == 0
    assert "version: 0.2.4" in capsys.readouterr().out


def test_out_of_scope_options_are_rejected(capsys):
    assert cli.main(["--greedy"]) == 2
    assert "not part of this MI355X build" in capsys.readouterr().err
