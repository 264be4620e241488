"""consume_seqfile_banding / _with_mask / _banding_with_mask on the device
(kh_consume_parser_filtered), against the reference's own tests
(tests/test_banding.py, tests/test_counttable.py:83-187) and the oracle's
filtered consume (oracle/khmer_oracle.c or_consume_fastx_filtered)."""
import pytest

from oracle import oracle as O
from tests.conftest import data
from tests.test_gpu_parity import HASH, KIND, assert_same

khmer = pytest.importorskip("khmer_amd")
from khmer_amd import synth  # noqa: E402
from khmer_amd._lib import lib  # noqa: E402

pytestmark = pytest.mark.gpu

SEQB_KMERS = ["GATTTGAGAAAAA", "ATTTGAGAAAAAA", "TTTGAGAAAAAAG", "TTGAGAAAAAAGT"]


@pytest.mark.parametrize("cls", ["Nodetable", "Counttable"])
def test_banding(cls):
    """tests/test_banding.py:140-157."""
    t = getattr(khmer, cls)(31, 1e5, 4)
    assert t.consume_seqfile_banding(data("bogus.fa"), 8, 3) == (1, 3)
    assert t.get("CGGCTATTATCTGAGCTCAAGACTAATACGC") == 1
    assert t.get("TATTATCTGAGCTCAAGACTAATACGCGCTG") == 1
    assert t.get("TGAGCTCAAGACTAATACGCGCTGGCCACTG") == 1
    assert t.get("GTACGGCTATTATCTGAGCTCAAGACTAATA") == 0
    assert t.get("TTATCTGAGCTCAAGACTAATACGCGCTGGC") == 0
    assert t.get("GCTCAAGACTAATACGCGCTGGCCACTGGTA") == 0


@pytest.mark.parametrize("cls", ["Nodetable", "Counttable"])
def test_banding_bad_params(cls):
    """tests/test_banding.py:120-136."""
    t = getattr(khmer, cls)(31, 1e5, 4)
    with pytest.raises(ValueError, match="'band' must be in the interval \\[0, 'num_bands'\\)"):
        t.consume_seqfile_banding(data("bogus.fa"), 8, 13)
    with pytest.raises(OSError, match="does not exist"):
        t.consume_seqfile_banding("file-no-exist.fa", 16, 3)


@pytest.mark.parametrize("numbands", [3, 11, 23, 29])
def test_banding_to_disk(tmp_path, numbands):
    """tests/test_banding.py:85-117: byte-identical saved table."""
    reads = data("banding-reads.fq.gz")
    a = khmer.Counttable(21, 5e6 / 4, 4)
    a.consume_seqfile(reads)
    a.save(str(tmp_path / "a.ct"))
    b = khmer.Counttable(21, 5e6 / 4, 4)
    for band in range(numbands):
        b.consume_seqfile_banding(reads, numbands, band)
    b.save(str(tmp_path / "b.ct"))
    assert open(str(tmp_path / "a.ct"), "rb").read() == open(str(tmp_path / "b.ct"), "rb").read()


@pytest.mark.parametrize("numbands", [2, 4, 8, 16])
def test_banding_in_memory(numbands):
    """tests/test_banding.py:42-82: banded counts sum to the plain count
    (within the reference's epsilon of 1 for false positives)."""
    reads = data("banding-reads.fq.gz")
    normal = khmer.Counttable(21, 5e6 / 4, 4)
    normal.consume_seqfile(reads)
    banded = []
    for band in range(numbands):
        t = khmer.Counttable(21, 5e6 / 4 / numbands, 4)
        t.consume_seqfile_banding(reads, numbands, band)
        banded.append(t)
    for n, rec in enumerate(khmer.ReadParser(reads)):
        if not (n > 0 and n % 100 == 0):
            continue
        for kmer in normal.get_kmers(rec.sequence):
            abunds = [t.get(kmer) for t in banded]
            assert abs(sum(abunds) - normal.get(kmer)) <= 1
            nz = [a for a in abunds if a > 0]
            assert len(nz) <= 2
            if len(nz) > 1:
                assert min(nz) == 1


def _seq_a_mask():
    mask = khmer.Counttable(13, 1e3, 4)
    mask.consume_seqfile(data("seq-a.fa"))
    return mask


def test_consume_with_mask():
    """tests/test_counttable.py:83-110."""
    ct = khmer.Counttable(13, 1e3, 4)
    assert ct.consume_seqfile_with_mask(data("seq-b.fa"), _seq_a_mask()) == (1, 3)
    assert [ct.get(k) for k in SEQB_KMERS] == [0, 1, 1, 1]


def test_consume_banding_with_mask():
    """tests/test_counttable.py:113-136."""
    ct = khmer.Counttable(13, 1e3, 4)
    assert ct.consume_seqfile_banding_with_mask(data("seq-b.fa"), 4, 1, _seq_a_mask()) == (1, 1)
    assert [ct.get(k) for k in SEQB_KMERS] == [0, 0, 0, 1]


def test_consume_with_mask_threshold():
    """tests/test_counttable.py:139-173."""
    mask = khmer.Counttable(13, 1e3, 4)
    for _ in range(3):
        mask.consume("TAGATCTGCTTGAAACAAGTGGATTTGAGAAAAA")
    for _ in range(2):
        mask.consume("TAGATCTGCTTGAAACAAGTGGATTTGAGAAAAAAGT")
    ct = khmer.Counttable(13, 1e3, 4)
    assert ct.consume_seqfile_with_mask(data("seq-b.fa"), mask, 3) == (1, 3)
    assert [ct.get(k) for k in SEQB_KMERS] == [0, 1, 1, 1]


def test_consume_with_mask_complement():
    """tests/test_counttable.py:176-187."""
    mask = khmer.Nodetable(13, 1e3, 4)
    mask.consume("TGCTTGAAACAAGTG")
    ct = khmer.Counttable(13, 1e3, 4)
    ct.consume_seqfile_with_mask(data("seq-b.fa"), mask, threshold=1, consume_masked=True)
    assert ct.get_kmer_counts("TGCTTGAAACAAGTG") == [1, 1, 1]
    assert ct.get_kmer_counts("GAAACAAGTGGATTT") == [0, 0, 0]


def test_mask_errors():
    ct = khmer.Counttable(13, 1e3, 4)
    with pytest.raises(TypeError):
        ct.consume_seqfile_with_mask(data("seq-b.fa"), "not a table")
    with pytest.raises(ValueError):
        ct.consume_seqfile_with_mask(data("seq-b.fa"), ct)


@pytest.mark.parametrize("cls,mcls", [("Countgraph", "Countgraph"), ("Nodegraph", "SmallCountgraph"),
                                      ("SmallCountgraph", "Nodegraph"), ("Counttable", "Counttable")])
@pytest.mark.parametrize("numbands,band", [(0, 0), (5, 2), (3, 3)])
@pytest.mark.parametrize("threshold,masked", [(None, False), (0, False), (2, True), (257, False), (257, True)])
def test_filtered_matches_oracle(tmp_path, cls, mcls, numbands, band, threshold, masked):
    """Device filtered consume == oracle, over several device batches, with a
    saturated bigcount mask (thresholds above 255 read the bigcount map)."""
    path = str(tmp_path / "syn.fq")
    synth.write_fastq(path, 600, 120)
    k = 15 if HASH[cls] == O.MURMUR else 21
    msizes = O.get_n_primes_near_x(3, 503)
    mask_g = mask_o = None
    if threshold is not None:
        mask_g = getattr(khmer, mcls)(k, 1, 1, primes=msizes)
        mask_o = O.Table(KIND[mcls], k, msizes, hash=HASH[mcls])
        if KIND[mcls] == O.BYTE:
            mask_g.set_use_bigcount(True)
            mask_o.set_use_bigcount(True)
        for _ in range(3):
            mask_g.consume_seqfile(path)
            mask_o.consume_fastx(path)
    sizes = O.get_n_primes_near_x(4, 100003)
    g = getattr(khmer, cls)(k, 1, 1, primes=sizes)
    o = O.Table(KIND[cls], k, sizes, hash=HASH[cls])
    lib.kh_graph_set_batch_kmers(g._g, 8192)
    thr = 0 if threshold is None else threshold
    if numbands == 0 and mask_g is None:
        got = g.consume_seqfile(path)
    elif numbands == 0:
        got = g.consume_seqfile_with_mask(path, mask_g, thr, masked)
    elif mask_g is None:
        got = g.consume_seqfile_banding(path, numbands, band)
    else:
        got = g.consume_seqfile_banding_with_mask(path, numbands, band, mask_g, thr, masked)
    want = o.consume_fastx_filtered(path, numbands, band, mask_o, thr, masked)
    assert got == want
    assert_same(g, o, "%s/%s bands=%d/%d thr=%s" % (cls, mcls, band, numbands, threshold))
