"""extract_countgraph_info / extract_nodegraph_info / calc_expected_collisions
(khmer/__init__.py:95-215) on CPU: table files written by the oracle's saver
(the reference's file layout), read through the library's raw header reader.
Mirrors tests/test_functions.py:191-250 of the reference."""
import pytest

from oracle import oracle as O
from tests.conftest import data

khmer = pytest.importorskip("khmer_amd")


@pytest.mark.parametrize("size", [1e6, 2e6, 5e6, 1e7])
def test_extract_countgraph_info(tmp_path, size):
    fn = str(tmp_path / "c.ct")
    t = O.Table(O.BYTE, 25, O.get_n_primes_near_x(4, size))
    t.save(fn)
    ksize, n_tables, table_size, use_bigcount, version, ht_type, occupied = khmer.extract_countgraph_info(fn)
    assert (ksize, n_tables, table_size) == (25, 4, size)
    assert (use_bigcount, version, ht_type, occupied) == (0, 4, 1, 0)


@pytest.mark.parametrize("size", [1e6, 2e6, 5e6, 1e7])
def test_extract_nodegraph_info(tmp_path, size):
    fn = str(tmp_path / "n.pt")
    t = O.Table(O.BIT, 25, O.get_n_primes_near_x(4, size))
    t.consume("ACGT" * 20)
    t.save(fn)
    ksize, table_size, n_tables, version, ht_type, occupied = khmer.extract_nodegraph_info(fn)
    assert (ksize, table_size, n_tables, version, ht_type) == (25, size, 4, 4, 2)
    assert occupied == t.n_occupied()


def test_extract_smallcount_info_has_no_bigcount(tmp_path):
    fn = str(tmp_path / "s.ct")
    O.Table(O.NIBBLE, 21, O.get_n_primes_near_x(2, 1e5)).save(fn)
    info = khmer.extract_countgraph_info(fn)
    assert info.use_bigcount is None and info.ht_type == 7 and info.ksize == 21


@pytest.mark.parametrize("fn", ["test-abund-read-2.fa", "empty-file", "normC20k20.ct.gz"])
def test_extract_info_badfile(fn):
    with pytest.raises(ValueError):
        khmer.extract_countgraph_info(data(fn))
    with pytest.raises(ValueError):
        khmer.extract_nodegraph_info(data(fn))


class _G(object):
    def __init__(self, sizes, occ):
        self.sizes, self.occ = sizes, occ

    def hashsizes(self):
        return self.sizes

    def n_occupied(self):
        return self.occ


def test_calc_expected_collisions(capsys):
    assert khmer.calc_expected_collisions(_G([100, 200], 10)) == pytest.approx(0.01)
    with pytest.raises(SystemExit):
        khmer.calc_expected_collisions(_G([100], 90))
    err = capsys.readouterr().err
    assert "** ERROR: the graph structure is too small for" in err
    assert "(estimated false positive rate of 0.900; max recommended 0.200)" in err
    assert khmer.calc_expected_collisions(_G([100], 90), force=True) == pytest.approx(0.9)
