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


def test_empty_count_files_print_help_and_return_0(tmp_path, capsys):
    """Empty positive/background files are an input error: help on stdout, the framed
    'input error:' block on stderr, exit code 0 -- as the reference's cli.py:144-153 does
    (checked against the reference's own run of the same command in this container)."""
    pos, bg = tmp_path / "pos.txt", tmp_path / "bg.txt"
    pos.write_text("")
    bg.write_text("")
    assert cli.main(["-p", str(pos), "-b", str(bg), "-c", "3", "-a", "0.5"]) == 0
    out, err = capsys.readouterr()
    assert out.startswith("usage: kmerpapa")
    assert err.splitlines()[:2] == ["=" * 80, "input error:"] and err.splitlines()[-1] == "=" * 80
