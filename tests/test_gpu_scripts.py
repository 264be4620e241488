"""The two drop-in scripts on the device, in-process, pinned to the reference's
own script tests (reference tests/test_scripts.py:65-360 and 521-800): the
unique-k-mer counts, the `.info` / `.info.tsv` / `.info.json` contents and the
"too small" failure.  Beyond the reference's assertions, the saved table and
tagset files must equal, byte for byte, what the oracle writes after
consuming the same inputs."""
import json
import os
import subprocess
import sys

import pytest

from oracle import oracle as O
from tests.conftest import ROOT, data

khmer = pytest.importorskip("khmer_amd")
from khmer_amd import scripts as S  # noqa: E402
from khmer_amd import khmer_args as KA  # noqa: E402

pytestmark = pytest.mark.gpu

ABUND = data("test-abund-read-2.fa")
RAND = data("random-20-a.fa")


def run(fn, argv, capsys):
    KA.configure_logging(False)
    try:
        status = fn(argv)
    except SystemExit as e:
        status = e.code if isinstance(e.code, int) else 1
    out, err = capsys.readouterr()
    return status, out, err


def oracle_file(kind, k, x, n, inputs, path, bigcount=True, tag=False):
    o = O.Table(kind, k, O.get_n_primes_near_x(n, int(x)))
    if kind == O.BYTE:
        o.set_use_bigcount(bigcount)
    for f in inputs:
        o.consume_fastx(f, tag=tag)
    o.save(path)
    return o


def same_file(a, b):
    with open(a, "rb") as fa, open(b, "rb") as fb:
        return fa.read() == fb.read()


def test_load_into_counting(tmp_path, capsys):
    out = str(tmp_path / "out.ct")
    st, _, err = run(S.load_into_counting, ["-x", "1e3", "-N", "2", "-k", "20", out, ABUND], capsys)
    assert st == 0 and "Total number of unique k-mers: 94" in err, err
    oracle_file(O.BYTE, 20, 1e3, 2, [ABUND], str(tmp_path / "o.ct"))
    assert same_file(out, str(tmp_path / "o.ct"))
    info = open(out + ".info").read().splitlines()
    assert info[0].startswith("khmer version:")
    assert info[1] == "through " + ABUND
    assert info[2] == "Total number of unique k-mers: 94"
    assert info[3].startswith("fp rate estimated to be ")


def test_load_into_counting_smallcount(tmp_path, capsys):
    out = str(tmp_path / "out.ct")
    st, _, err = run(S.load_into_counting, ["-x", "1e3", "--small-count", out, ABUND], capsys)
    assert st == 0 and "Total number of unique k-mers: 83" in err, err
    oracle_file(O.NIBBLE, 32, 1e3, 4, [ABUND], str(tmp_path / "o.ct"))
    assert same_file(out, str(tmp_path / "o.ct"))


def test_load_into_counting_quiet(tmp_path, capsys):
    out = str(tmp_path / "out.ct")
    st, o, err = run(S.load_into_counting, ["-q", "-x", "1e3", "-N", "2", "-k", "20", out, ABUND], capsys)
    assert st == 0 and o == "" and err == ""
    assert os.path.exists(out)


def test_load_into_counting_nobigcount(tmp_path, capsys):
    out = str(tmp_path / "out.ct")
    st, _, err = run(S.load_into_counting, ["-x", "1e3", "-N", "2", "-k", "20", "-b", out, ABUND], capsys)
    assert st == 0 and "Total number of unique k-mers: 94" in err
    oracle_file(O.BYTE, 20, 1e3, 2, [ABUND], str(tmp_path / "o.ct"), bigcount=False)
    assert same_file(out, str(tmp_path / "o.ct"))


def test_load_into_counting_max_memory(tmp_path, capsys):
    out = str(tmp_path / "out.ct")
    st, _, err = run(S.load_into_counting, ["-M", "2e3", "-k", "20", out, ABUND], capsys)
    assert st == 0 and "WARNING: tablesize is default!" not in err
    cg = khmer.Countgraph.load(out)
    assert sum(cg.hashsizes()) < 3e8
    assert cg.hashsizes() == O.get_n_primes_near_x(4, 500)


def test_load_into_counting_fail(tmp_path, capsys):
    out = str(tmp_path / "out.ct")
    st, _, err = run(S.load_into_counting, ["-x", "1e2", "-N", "2", "-k", "20", out, ABUND], capsys)
    assert st == 1
    assert "** ERROR: the graph structure is too small" in err


def test_load_into_counting_multifile(tmp_path, capsys):
    out = str(tmp_path / "out.kh")
    st, _, err = run(S.load_into_counting, ["-x", "1e7", "-N", "2", "-k", "20", out] + [ABUND] * 11,
                     capsys)
    assert st == 0 and "Total number of unique k-mers: 95" in err, err
    assert "mid-save" in err
    oracle_file(O.BYTE, 20, 1e7, 2, [ABUND] * 11, str(tmp_path / "o.ct"))
    assert same_file(out, str(tmp_path / "o.ct"))


def test_load_into_counting_tsv(tmp_path, capsys):
    out = str(tmp_path / "out.ct")
    st, _, err = run(S.load_into_counting, ["-x", "1e7", "-N", "2", "-k", "20", "-s", "tsv", out, ABUND],
                     capsys)
    assert st == 0 and "Total number of unique k-mers: 95" in err
    lines = open(out + ".info.tsv").readlines()
    assert lines == ["ht_name\tfpr\tnum_kmers\tnum_reads\tfiles\n",
                     "\t".join(["out.ct", "0.000", "95", "1001", ABUND]) + "\n"]


def test_load_into_counting_json(tmp_path, capsys):
    out = str(tmp_path / "out.ct")
    st, _, _ = run(S.load_into_counting, ["-x", "1e7", "-N", "2", "-k", "20", "-s", "json", out, ABUND],
                   capsys)
    assert st == 0
    got = json.load(open(out + ".info.json"))
    assert got == {"files": [ABUND], "ht_name": "out.ct", "num_kmers": 95, "num_reads": 1001,
                   "fpr": 9.025048735197377e-11, "mrinfo_version": "0.2.0"}


def test_load_graph(tmp_path, capsys):
    out = str(tmp_path / "out")
    st, _, err = run(S.load_graph, ["-x", "1e7", "-N", "2", "-k", "20", out, RAND], capsys)
    assert st == 0 and "Total number of unique k-mers: 3960" in err, err
    o = oracle_file(O.BIT, 20, 1e7, 2, [RAND], str(tmp_path / "o.pt"), tag=True)
    assert same_file(out, str(tmp_path / "o.pt"))
    o.save_tagset(str(tmp_path / "o.tagset"))
    assert same_file(out + ".tagset", str(tmp_path / "o.tagset"))
    ng = khmer.Nodegraph.load(out)
    ng.load_tagset(out + ".tagset")
    assert ng.n_tags == len(o.tags()) > 0


def test_load_graph_no_tags(tmp_path, capsys):
    out = str(tmp_path / "out")
    st, _, err = run(S.load_graph, ["-x", "1e7", "-N", "2", "-k", "20", "-n", out, RAND], capsys)
    assert st == 0 and "We WILL NOT build the tagset." in err
    assert os.path.exists(out) and not os.path.exists(out + ".tagset")
    assert khmer.Nodegraph.load(out)


def test_load_graph_fail(tmp_path, capsys):
    out = str(tmp_path / "out")
    st, _, err = run(S.load_graph, ["-x", "1e3", "-N", "2", "-k", "20", out, RAND], capsys)
    assert st == 1
    assert "** ERROR: the graph structure is too small" in err


def test_load_graph_write_fp(tmp_path, capsys):
    out = str(tmp_path / "out")
    st, _, _ = run(S.load_graph, ["-x", "1e5", "-N", "2", "-k", "20", out, RAND], capsys)
    assert st == 0
    lines = set(x.strip() for x in open(out + ".info"))
    assert "3959 unique k-mers" in lines, lines
    assert "false positive rate estimated to be 0.002" in lines


def test_load_graph_max_memory_and_threads(tmp_path, capsys):
    out = str(tmp_path / "out")
    st, _, err = run(S.load_graph, ["-M", "2e7", "-k", "20", "-n", "-T", "8", out, RAND], capsys)
    assert st == 0 and "Total number of unique k-mers: 3960" in err, err
    oracle_file(O.BIT, 20, 8 * 2e7 / 4, 4, [RAND], str(tmp_path / "o.pt"))
    assert same_file(out, str(tmp_path / "o.pt"))


def test_script_entry_points(tmp_path):
    """The files under scripts/ run as programs (one child process each)."""
    out = str(tmp_path / "out.ct")
    r = subprocess.run([sys.executable, os.path.join(ROOT, "scripts", "load-into-counting.py"),
                        "-x", "1e3", "-N", "2", "-k", "20", out, ABUND],
                       capture_output=True, text=True, timeout=300)
    assert r.returncode == 0 and "Total number of unique k-mers: 94" in r.stderr, r.stderr
    out = str(tmp_path / "g")
    r = subprocess.run([sys.executable, os.path.join(ROOT, "scripts", "load-graph.py"),
                        "-x", "1e7", "-N", "2", "-k", "20", out, RAND],
                       capture_output=True, text=True, timeout=300)
    assert r.returncode == 0 and "Total number of unique k-mers: 3960" in r.stderr, r.stderr
    assert os.path.exists(out + ".tagset")


@pytest.mark.parametrize("suffix", [".gz", ".bz2"])
def test_load_into_counting_compressed(tmp_path, capsys, suffix):
    """Compressed inputs give the same table as the plain file."""
    src = data("test-abund-read-2.fa" + suffix) if suffix == ".bz2" else None
    if src is None:
        import gzip
        src = str(tmp_path / "in.fa.gz")
        with open(ABUND, "rb") as fi, gzip.open(src, "wb") as fo:
            fo.write(fi.read())
    out = str(tmp_path / "out.ct")
    st, _, err = run(S.load_into_counting, ["-x", "1e3", "-N", "2", "-k", "20", out, src], capsys)
    assert st == 0 and "Total number of unique k-mers: 94" in err, err
    oracle_file(O.BYTE, 20, 1e3, 2, [ABUND], str(tmp_path / "o.ct"))
    assert same_file(out, str(tmp_path / "o.ct"))


def test_c1_exact_command(tmp_path, capsys):
    """BASELINE configs[0] / SURVEY §8(d) C1 as written: load-into-counting.py
    -k 21 -N 4 -x 1e7 out.ct data/25k.fq.gz (bigcount on by default):
    25,000 reads, 1,223,896 k-mers; the saved .ct equals the oracle's byte for
    byte and the logged unique k-mer count equals the oracle's n_unique_kmers
    (VERDICT r3 "Next round" #8)."""
    fq = data("25k.fq.gz")
    out = str(tmp_path / "out.ct")
    st, _, err = run(S.load_into_counting, ["-k", "21", "-N", "4", "-x", "1e7", out, fq], capsys)
    assert st == 0, err
    o = oracle_file(O.BYTE, 21, 1e7, 4, [fq], str(tmp_path / "o.ct"))
    assert "Total number of unique k-mers: %d" % o.n_unique_kmers() in err, err
    assert same_file(out, str(tmp_path / "o.ct"))
    import khmer_amd
    g = khmer_amd.Countgraph.load(out)
    assert g.hashsizes() == [9999991, 9999973, 9999971, 9999943]
    assert g.n_occupied() == o.n_occupied()
    reads, kmers = khmer_amd.Countgraph(21, 1e7, 4).consume_seqfile(fq)
    assert (reads, kmers) == (25000, 1223896)
