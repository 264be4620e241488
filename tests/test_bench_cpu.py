"""bench.py's host-side logic on CPU: the golden-fixture match that makes a
bench line carry its own parity check (VERDICT r2 "Next round" #1c), and the
algorithmic-bytes figures of SURVEY.md §8(d)."""
import importlib.util
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope="module")
def bench():
    spec = importlib.util.spec_from_file_location("bench_under_test", os.path.join(ROOT, "bench.py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


def _args(bench, argv):
    old = sys.argv
    sys.argv = ["bench.py"] + argv
    try:
        return bench.parse()
    finally:
        sys.argv = old


def test_default_workload_is_c2_full(bench):
    a = _args(bench, [])
    fx, exact = bench.matching_fixture(a, a.reads)
    assert fx is not None and fx["config"] == "c2_full" and exact
    # strong scaling over 8 ranks is the same stream (broadcast mode: rank order)
    a8 = _args(bench, ["--gpus", "8", "--strong", "--group-mode", "broadcast"])
    assert bench.matching_fixture(a8, 8 * ((a8.reads + 7) // 8)) == (bench.matching_fixture(a, a.reads)[0], True)


def _have(name):
    from tests import full_digest as FD
    return os.path.exists(FD.fixture_path(name))


@pytest.mark.parametrize("world", [2, 4, 8])
def test_weak_scaling_lines_have_fixtures(bench, world):
    """every `bench.py --gpus G` line the driver runs (C2, weak
    scaling, 50M reads per rank, the default delta mode and batch) matches a
    fixture made in its own stream order, so the line carries counters_match
    and tables_match; other group modes fall back to the same reads in
    another order (tables and n_occupied)."""
    name = "c2_w%d_d" % world
    if not _have(name):
        pytest.skip("fixture %s not generated yet" % name)
    a = _args(bench, ["--gpus", str(world)])
    assert a.group_mode == "delta"
    fx, exact = bench.matching_fixture(a, world * a.reads, (a.group_mode, [world, a.batch_kmers]))
    assert fx["config"] == name and exact
    assert fx["params"]["reads"] == world * 50_000_000
    ax = _args(bench, ["--gpus", str(world), "--group-mode", "exchange"])
    fx, exact = bench.matching_fixture(ax, world * ax.reads, ("exchange", [world, ax.batch_kmers]))
    assert fx is not None and fx["params"]["reads"] == world * 50_000_000
    assert exact == (fx["config"] == "c2_w%d_x" % world)


def test_exchange_fixture_order(bench):
    """Exchange mode's pass-interleaved stream: the fixture made in that
    order (c2_full_x2b: 2 ranks at the default batch) is an exact match; with
    none for the order (8 ranks at the default batch) the rank-order fixture
    checks the order-free outputs only."""
    a = _args(bench, ["--gpus", "2", "--strong", "--group-mode", "exchange"])
    fx, exact = bench.matching_fixture(a, 50_000_000, ("exchange", [2, a.batch_kmers]))
    assert fx["config"] == "c2_full_x2b" and exact
    fx, exact = bench.matching_fixture(a, 50_000_000, ("exchange", [8, a.batch_kmers]))
    assert fx["config"] == "c2_full" and not exact
    part = bench.compare_fixture(fx, 1, fx["n_occupied"], fx["table_sha256"], stream_order=False)
    assert part["n_occupied_match"] and part["tables_match"] and "counters_match" not in part


@pytest.mark.parametrize("argv,name", [(["--config", "C3", "--reads", "4000000"], "c3_shape"),
                                       (["--config", "C4", "--reads", "4000000"], "c4_shape"),
                                       (["--config", "C5", "--reads", "4000000"], "c5_shape"),
                                       (["--config", "C5", "--reads", "4000000", "--genome", "5e7"], "c5_genomic"),
                                       (["--config", "C5M", "--reads", "1000000", "--genome", "1e7"], "c5m_genomic"),
                                       (["--genome", "2e6", "--reads", "10000000"], "genomic_c2"),
                                       (["--reads", "49999999"], None),
                                       (["--no-bigcount"], None)])
def test_fixture_match(bench, argv, name):
    a = _args(bench, argv)
    fx, _ = bench.matching_fixture(a, a.reads)
    assert (fx["config"] if fx else None) == name


def test_compare_fixture(bench):
    a = _args(bench, [])
    fx, _ = bench.matching_fixture(a, a.reads)
    ok = bench.compare_fixture(fx, fx["n_unique_kmers"], fx["n_occupied"], fx["table_sha256"])
    assert ok == {"fixture": "c2_full", "counters_match": True, "tables_match": True}
    bad = bench.compare_fixture(fx, fx["n_unique_kmers"] + 1, fx["n_occupied"], None)
    assert bad == {"fixture": "c2_full", "counters_match": False}


def test_algorithmic_bytes(bench):
    assert abs(bench.algorithmic_bytes_per_kmer(150, 21, 4) - 8.288461538) < 1e-6
    assert abs(bench.query_bytes_per_kmer(150, 51, 4) - 4.475) < 1e-9


@pytest.mark.parametrize("argv,mode", [
    ([], "delta"),
    (["--gpus", "8"], "delta"),                                  # C2 weak: 4 GB vs 3.25e9 k-mers a rank-pass
    (["--gpus", "8", "--strong"], "delta"),                      # C2 strong: 4 GB vs 0.8e9 k-mers
    (["--gpus", "8", "--config", "C4"], "delta"),                # C4 weak: 32 GB vs 3.25e9 k-mers
    (["--gpus", "8", "--config", "C4", "--strong"], "exchange"), # C4 strong: 32 GB vs 0.8e9 k-mers
    (["--gpus", "8", "--config", "C4", "--strong", "--group-mode", "delta"], "delta"),
])
def test_auto_group_mode(bench, argv, mode):
    """bench.py picks the group mode per configuration from the
    crossover DESIGN.md §6 derives (table bytes against 4 x tables x the
    k-mers of a rank-pass); an explicit --group-mode wins."""
    assert _args(bench, argv).group_mode == mode
