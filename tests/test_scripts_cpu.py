"""Host-side logic of the two drop-in scripts (khmer_amd/khmer_args.py,
khmer_amd/scripts.py): option parsing, table sizing and the -U / --fp-rate
messages, pinned to the strings and numbers the reference's own script tests
assert (tests/test_scripts.py:108-150, 293-360 of the reference).  Nothing
here creates a device table; tests that do are in test_gpu_scripts.py."""
import os
import subprocess
import sys

import pytest

from tests.conftest import ROOT, data

KA = pytest.importorskip("khmer_amd.khmer_args")
from khmer_amd import scripts as S  # noqa: E402


def lic_args(argv):
    return S.load_into_counting_parser().parse_args(argv)


@pytest.mark.parametrize("label,value", [
    ("1", 1.0), ("1000", 1e3), ("1e9", 1e9), ("2K", 2e3), ("2k", 2e3),
    ("1.5M", 1.5e6), ("4G", 4e9), ("3t", 3e12),
])
def test_memory_setting(label, value):
    assert KA.memory_setting(label) == value


@pytest.mark.parametrize("label", ["1X", "GG", "", "1.2.3G"])
def test_memory_setting_rejects(label):
    with pytest.raises(ValueError, match="cannot parse memory setting"):
        KA.memory_setting(label)


def test_estimates():
    r = KA.estimate_optimal_with_K_and_f(1e7, 0.08)
    assert (r.num_htables, "%5g" % r.htable_size) == (3, "1.77407e+07")
    r = KA.estimate_optimal_with_K_and_M(1e7, 1e6)
    assert (r.num_htables, r.htable_size) == (1, 1000000)
    assert str(r.fp_rate).startswith("0.9999546")
    r = KA.optimal_size(1e7, fp_rate=0.1)
    assert "%3g" % r.mem_use == "4.80833e+07"
    with pytest.raises(TypeError):
        KA.optimal_size(1e7)


def test_autoargs_fp_override_and_small_table(capsys):
    """reference test_load_into_counting_autoargs_0"""
    KA.configure_logging(False)
    a = KA._check_fp_rate(lic_args(["-U", "1e7", "--fp-rate", "0.08", "out", "in"]), 0.1)
    err = capsys.readouterr().err
    assert "INFO: Overriding default fp 0.1 with new fp: 0.08" in err
    assert " tablesize is too small!" in err
    assert "Estimated FP rate with current config is: 0.9999546" in err
    assert "Recommended tablesize is: 1.77407e+07 bytes" in err
    assert a.max_memory_usage is None


def test_autoargs_sets_ceiling(capsys):
    """reference test_load_into_counting_autoargs_1"""
    KA.configure_logging(False)
    a = KA._check_fp_rate(lic_args(["-U", "1e7", "--max-tablesize", "3e7", "out", "in"]), 0.1)
    err = capsys.readouterr().err
    assert "Ceiling is: 4.80833e+07 bytes" in err
    assert "set memory ceiling automatically." in err
    assert KA.calculate_graphsize(a, "countgraph") == pytest.approx(4.80833e7 / 4, rel=1e-5)


def test_autoargs_memory_too_small_aborts(capsys):
    a = lic_args(["-U", "1e9", "-M", "1e6", "out", "in"])
    with pytest.raises(SystemExit) as e:
        KA._check_fp_rate(a, 0.1)
    assert e.value.code == 1
    assert "above the recommended false positive ceiling" in capsys.readouterr().err
    a = lic_args(["-U", "1e9", "-M", "1e6", "--force", "out", "in"])
    KA._check_fp_rate(a, 0.1)


@pytest.mark.parametrize("graphtype,bpb", [("countgraph", 1), ("smallcountgraph", 2), ("nodegraph", 8)])
def test_graphsize_from_memory(graphtype, bpb):
    a = lic_args(["-M", "2e3", "-N", "4", "out", "in"])
    assert KA.calculate_graphsize(a, graphtype) == bpb * 2e3 / 4
    a = lic_args(["-x", "1e3", "out", "in"])
    assert KA.calculate_graphsize(a, graphtype) == 1e3
    with pytest.raises(ValueError):
        KA.calculate_graphsize(a, "bogus")


def test_x_and_M_exclusive(capsys):
    with pytest.raises(SystemExit):
        lic_args(["-x", "1e3", "-M", "1e3", "out", "in"])


def test_default_tablesize_warning(capsys):
    KA.report_on_config(lic_args(["-k", "20", "out", "in"]))
    assert "WARNING: tablesize is default!" in capsys.readouterr().err
    KA.report_on_config(lic_args(["-M", "2e3", "-k", "20", "out", "in"]))
    assert "WARNING: tablesize is default!" not in capsys.readouterr().err


def test_report_on_config_text(capsys):
    KA.configure_logging(False)
    KA.report_on_config(lic_args(["-x", "1e3", "-N", "2", "-k", "20", "out", "in"]))
    err = capsys.readouterr().err
    assert " - kmer size =     20 \t\t(-k)" in err
    assert " - n tables =      2 \t\t(-N)" in err
    assert "Estimated memory usage is 0.0 Gb (2e+03 bytes = 2 bytes x 1e+03 entries / 1 entries per byte)" in err


def test_quiet_silences_info(capsys):
    a = lic_args(["-q", "-x", "1e3", "out", "in"])
    KA.report_on_config(a)
    assert capsys.readouterr().err == ""
    KA.configure_logging(False)


def test_table_shape_errors(capsys):
    with pytest.raises(SystemExit):
        KA._check_table_shape(lic_args(["-N", "21", "out", "in"]), 20)
    assert "number of tables <= 20" in capsys.readouterr().err
    with pytest.raises(SystemExit):
        KA._check_table_shape(lic_args(["out", "in"]), 33)
    assert "k-mer sizes <= 32" in capsys.readouterr().err
    KA._check_table_shape(lic_args(["-N", "21", "-f", "out", "in"]), 20)


def test_bad_summary_format(capsys):
    """reference test_load_into_counting_bad_summary_fmt"""
    with pytest.raises(SystemExit) as e:
        lic_args(["-s", "badfmt", "out", "in"])
    assert e.value.code != 0
    assert "invalid choice: 'badfmt'" in capsys.readouterr().err


def test_missing_and_empty_input(tmp_path, capsys):
    with pytest.raises(SystemExit) as e:
        KA.check_input_files(str(tmp_path / "nope.fa"), False)
    assert e.value.code == 1
    assert "does not exist" in capsys.readouterr().err
    KA.check_input_files(str(tmp_path / "nope.fa"), True)
    with pytest.raises(SystemExit):
        KA.check_input_files(data("empty-file"), False)
    assert "is empty" in capsys.readouterr().err
    KA.check_input_files(data("random-20-a.fa"), False)
    KA.check_input_files("-", False)


def test_space_check(tmp_path, capsys):
    out = str(tmp_path / "o.ct")
    with pytest.raises(SystemExit) as e:
        KA.check_space_for_graph(out, 1e12, False, _testhook_free_space=0)
    assert "ERROR: Not enough free space on disk" in str(e.value.code)
    KA.check_space_for_graph(out, 1e12, True, _testhook_free_space=0)
    assert "WARNING: Not enough free space" in capsys.readouterr().err
    KA.check_space_for_graph(out, 10, False)


@pytest.mark.skipif(os.geteuid() == 0, reason="root can write anything")
def test_nonwritable(tmp_path, capsys):
    p = tmp_path / "ro"
    p.write_text("x")
    os.chmod(str(p), 0o444)
    with pytest.raises(SystemExit):
        KA.check_file_writable(str(p))
    assert "does not have write permission; exiting" in capsys.readouterr().err


def test_load_graph_parser():
    a = S.load_graph_parser().parse_args(["-x", "1e7", "-N", "2", "-k", "20", "-n", "-T", "8",
                                          "out", "a.fa", "b.fa"])
    assert (a.max_tablesize, a.n_tables, a.ksize, a.no_build_tagset, a.threads) == (1e7, 2, 20, True, 8)
    assert a.input_filenames == ["a.fa", "b.fa"] and a.output_filename == "out"


def test_script_without_device_fails_loudly(tmp_path):
    """No HIP device here: the script must stop with an error, not count on
    the CPU."""
    import torch
    if torch.cuda.is_available():
        pytest.skip("device present")
    out = str(tmp_path / "o.ct")
    r = subprocess.run([sys.executable, os.path.join(ROOT, "scripts", "load-into-counting.py"),
                        "-x", "1e3", "-N", "2", "-k", "20", out, data("test-abund-read-2.fa")],
                       capture_output=True, text=True, timeout=300)
    assert r.returncode != 0
    assert "Total number of unique k-mers" not in r.stderr
    assert not os.path.exists(out) or os.path.getsize(out) == 0
