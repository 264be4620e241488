"""Pin the CPU restatement (oracle/) against the reference's own known answers.

Every expected value below is transcribed from the reference test-suite
(file:line cited per test).  The reference itself could not be executed in
this environment, so these KATs are what pins the oracle;
the oracle in turn pins the HIP path (tests/test_gpu_parity.py).
CPU only.
"""
import gzip
import os
import shutil

import pytest

from oracle import oracle as O
from tests.conftest import data

PRIMES_1M_CG = [1000003, 1009837]     # tests/test_countgraph.py:54
PRIMES_1M_TF = [100003, 1000007]      # tests/table_fixtures.py:47
PARAMS_1M = (1000003, 2)              # tests/table_fixtures.py:46


def primes(n, x):
    return O.get_n_primes_near_x(n, x)


# --- hashing: tests/test_functions.py:51-169 ---------------------------------
def test_forward_hash():
    assert O.forward_hash("AAAA", 4) == 0
    assert O.forward_hash("TTTT", 4) == 0
    assert O.forward_hash("CCCC", 4) == 170
    assert O.forward_hash("GGGG", 4) == 170
    assert O.forward_hash("GGTTGACGGGGCTCAGGGGGCGGCTGACTCCG", 32) == 13607885392109549066


def test_forward_hash_no_rc():
    assert O.forward_hash_no_rc("AAAA", 4) == 0
    assert O.forward_hash_no_rc("TTTT", 4) == 85
    assert O.forward_hash_no_rc("CCCC", 4) == 170
    assert O.forward_hash_no_rc("GGGG", 4) == 255


def test_reverse_hash():
    assert O.reverse_hash(0, 4) == "AAAA"
    assert O.reverse_hash(85, 4) == "TTTT"
    assert O.reverse_hash(170, 4) == "CCCC"
    assert O.reverse_hash(255, 4) == "GGGG"


def test_reverse_complement():
    # tests/test_functions.py:101-120
    assert O.reverse_complement("AATTCCGG") == "CCGGAATT"
    for a, b in zip("ATCG", "TAGC"):
        assert O.reverse_complement(a) == b
    assert O.reverse_complement("FGF") == "FCF"


def test_hash_murmur3():
    assert O.hash_murmur3("AAAA") == 526240128537019279
    assert O.hash_murmur3("TTTT") == 526240128537019279
    assert O.hash_murmur3("CCCC") == 14391997331386449225
    assert O.hash_murmur3("GGGG") == 14391997331386449225
    for s in ("TATATATATATATATATATA", "TTTTGCAAAA", "GAAAATTTTC"):
        assert O.hash_murmur3(s) != 0


def test_hash_no_rc_murmur3():
    assert O.hash_no_rc_murmur3("AAAA") == 5231866503566620412
    assert O.hash_no_rc_murmur3("TTTT") == 5753003579327329651
    assert O.hash_no_rc_murmur3("CCCC") == 3789793362494378039
    assert O.hash_no_rc_murmur3("GGGG") == 17519752047064575358


def test_smallcounttable_murmur_hashes():
    # tests/test_nibblestorage.py:49-66
    t = O.Table(O.NIBBLE, 4, [4], hash=O.MURMUR)
    assert t.kmer_hashes("AAAC") == [11898086063751343884]
    assert t.kmer_hashes("AAAG") == [10548630838975263317]
    t.add(t.kmer_hashes("AAAC")[0])
    assert t.get(t.kmer_hashes("AAAC")[0]) == 1
    assert t.get(t.kmer_hashes("AAAG")[0]) == 0


# --- primes: tests/test_functions.py:172-189 ---------------------------------
def test_get_primes():
    assert primes(7, 20) == [19, 17, 13, 11, 7, 5, 3]
    with pytest.raises(RuntimeError, match="unable to find 5 prime numbers < 5"):
        primes(5, 5)


def test_config_primes():
    # SURVEY.md §8 table (computed with the same algorithm)
    assert primes(4, 1e7) == [9999991, 9999973, 9999971, 9999943]
    assert primes(4, 1e9) == [999999937, 999999929, 999999893, 999999883]


# --- collisions: tests/test_countgraph.py:117-197, 251-282 -------------------
def test_collision_hashes():
    assert O.forward_hash("G" * 12, 12) == 11184810
    assert O.forward_hash("AAACGTATGACT", 12) == 184777
    assert O.forward_hash("AAATACCGAGCG", 12) == 76603
    assert O.forward_hash("AAACGTATCGAG", 12) == 184755


@pytest.mark.parametrize("others,expect", [
    (["AAACGTATGACT"], 1),
    (["AAATACCGAGCG"], 1),
    (["AAACGTATGACT", "AAATACCGAGCG"], 2),
])
def test_collisions_2tables(others, expect):
    t = O.Table(O.BYTE, 12, PRIMES_1M_CG)
    t.consume("G" * 12)
    for s in others:
        t.consume(s)
    assert t.get(t.hash("G" * 12)) == expect


def test_3_tables():
    t = O.Table(O.BYTE, 12, PRIMES_1M_CG + [1000005])
    gg = t.hash("G" * 12)
    t.consume("G" * 12)
    assert t.get(gg) == 1
    for s in ("AAACGTATGACT", "AAATACCGAGCG"):
        t.consume(s)
        assert t.get(gg) == 1
    t.consume("AAACGTATCGAG")
    assert t.get(gg) == 2


# --- tests/test_counting_single.py ------------------------------------------
def test_collision_aaaa_tttt():
    # :56-63
    t = O.Table(O.BYTE, 4, primes(1, 100))
    t.add(t.hash("AAAA"))
    assert t.get(t.hash("AAAA")) == 1
    t.add(t.hash("TTTT"))
    assert t.get(t.hash("TTTT")) == 2


def test_complete_no_collision():
    # :80-105
    t = O.Table(O.BYTE, 4, [4 ** 4])
    for i in range(256):
        t.add(t.hash(O.reverse_hash(i, 4)))
    rc_filled = pal = fwd = 0
    for i in range(256):
        c = t.get(t.hash(O.reverse_hash(i, 4)))
        rc_filled += bool(c)
        pal += (c == 1)
        fwd += bool(t.get(i))
    assert rc_filled == 256
    assert pal == 16
    assert fwd == 256 // 2 + 16 // 2


def test_maxcount_consume():
    # :199-219
    t = O.Table(O.BYTE, 4, primes(1, 100))
    t.consume("A" * 10000)
    assert t.get(t.hash("AAAA")) == 255
    t = O.Table(O.BYTE, 4, primes(1, 100))
    t.set_use_bigcount(True)
    t.consume("A" * 10000)
    assert t.get(t.hash("AAAA")) == 10000 - 3


def test_very_short_read():
    # :317-327
    t = O.Table(O.BYTE, 9, primes(1, 4))
    assert t.consume_fastx(data("test-short.fa")) == (1, 0)
    t = O.Table(O.BYTE, 8, primes(1, 4))
    assert t.consume_fastx(data("test-short.fa")) == (1, 1)


# --- saturation / bigcount: tests/test_countgraph.py:890-992 -----------------
def test_maxcount_and_bigcount():
    for bc, expect in ((False, 255), (True, 1000)):
        t = O.Table(O.BYTE, 4, primes(4, 4 ** 4))
        t.set_use_bigcount(bc)
        h = t.hash("AAAA")
        for _ in range(1000):
            t.add(h)
        assert t.get(h) == expect


def test_bigcount_300():
    # tests/test_tabletype.py:426-439
    t = O.Table(O.BYTE, 12, primes(2, 1000003))
    t.set_use_bigcount(True)
    h = t.hash("G" * 12)
    for _ in range(300):
        t.add(h)
    assert t.get(h) == 300


# --- raw tables: tests/test_countgraph.py:200-240 ----------------------------
def test_raw_tables_views():
    t = O.Table(O.BYTE, 20, primes(4, 1e5))
    t.consume("AAAATTTTCCCCGGGGAAAA")
    for i in range(4):
        assert sum(t.table_bytes(i)) == 1
    s = O.Table(O.NIBBLE, 4, primes(4, 1e5))
    for i, p in enumerate(s.sizes):
        assert len(s.table_bytes(i)) == p // 2 + 1
    s.consume("AAAA")
    for i in range(4):
        assert sum(s.table_bytes(i)) == 16  # count 1 in the high nibble


# --- nibble saturation: tests/test_nibblestorage.py:69-92 --------------------
def test_nibble_overflow():
    for a, b in (("AAAA", "AAAT"), ("AAAT", "AAAA")):
        t = O.Table(O.NIBBLE, 4, primes(4, 1e6), hash=O.MURMUR)
        ha, hb = t.hash(a), t.hash(b)
        for _ in range(17):
            t.add(ha)
        assert t.get(ha) == 15
        assert t.get(hb) == 0


# --- file-level counters ------------------------------------------------------
def test_random20_countgraph_occupied():
    # tests/test_countgraph.py:634-666
    for kind in (O.BYTE, O.NIBBLE):
        t = O.Table(kind, 12, primes(4, 1e5))
        t.consume_fastx(data("random-20-a.fa"))
        assert t.n_occupied() == 3886


def test_random20_abundance_distribution():
    # tests/test_countgraph.py:669-692
    sizes = PRIMES_1M_CG + [1000005]
    t = O.Table(O.BYTE, 12, sizes)
    t.consume_fastx(data("random-20-a.fa"))
    tracking = O.Table(O.BIT, 12, sizes)
    assert sum(t.abundance_distribution(data("random-20-a.fa"), tracking)) == 3966


def test_nodegraph_random20():
    # tests/test_nodegraph.py:219-278
    t = O.Table(O.BIT, 20, primes(1, 100000))
    for _, seq, _ in O.read_fastx(data("random-20-a.fa")):
        t.consume(seq)
    assert t.n_occupied() == 3884
    t = O.Table(O.BIT, 20, primes(3, 100000))
    for _, seq, _ in O.read_fastx(data("random-20-a.fa")):
        t.consume(seq)
    assert t.n_occupied() == 3884
    assert t.n_unique_kmers() == 3960


def test_nodegraph_tiny_primes():
    # tests/test_nodegraph.py:281-341
    t = O.Table(O.BIT, 4, [11])
    occ = []
    uniq = []
    for s in ("AAAA", "ACTG", "AACG", "AGAC"):
        t.add(t.hash(s))
        occ.append(t.n_occupied())
        uniq.append(t.n_unique_kmers())
    assert occ == [1, 2, 2, 2]
    assert uniq == [1, 2, 2, 2]
    t = O.Table(O.BIT, 4, [11, 13])
    uniq = []
    for s in ("AAAA", "ACTG", "AACG", "AGAC"):
        t.add(t.hash(s))
        uniq.append(t.n_unique_kmers())
    assert uniq[1:] == [2, 3, 3]


# --- read cleaning: tests/test_sequence_validation.py:57-125 -----------------
@pytest.mark.parametrize("kind,hashfn", [(O.BYTE, O.TWOBIT), (O.NIBBLE, O.TWOBIT),
                                         (O.BYTE, O.MURMUR), (O.NIBBLE, O.MURMUR)])
def test_read_cleaning(kind, hashfn):
    sizes = primes(PARAMS_1M[1], PARAMS_1M[0])
    x = O.Table(kind, 15, sizes, hash=hashfn)
    x.consume_fastx(data("valid-read-testing.fq"))
    for kmer in ("caggcgcccaccacc".upper(), "CCTCATCGGCACCAG", "ACTGAGCTTCATGTC"):
        assert x.get(x.hash(kmer)) == 2
    y = O.Table(kind, 15, sizes, hash=hashfn)
    for _, seq, _ in O.read_fastx(data("valid-read-testing.fq")):
        y.consume(seq)   # raw, not cleaned
    assert y.get(y.hash("caggcgcccaccacc".upper())) == 1
    if hashfn == O.TWOBIT:
        # 2-bit hashing maps invalid bases to G: still counted twice
        assert y.get(y.hash("CCTCATCGGCACCAG")) == 2
        assert y.get(y.hash("ACTGAGCTTCATGTC")) == 2
    tracking = O.Table(O.BIT, 15, PRIMES_1M_TF, hash=hashfn)
    dist = x.abundance_distribution(data("valid-read-testing.fq"), tracking)
    assert dist[1] == 35
    assert dist[2] == 69


# --- read parser: tests/test_read_parsers.py:84-175 --------------------------
def test_read_properties():
    recs = list(O.read_fastx(data("single-read.fq")))
    assert recs == [("895:1:1:1246:14654 1:N:0:NNNNN",
                     "CAGGCGCCCACCACCGTGCCCTCCAACCTGATGGT",
                     "][aaX__aa[`ZUZ[NONNFNNNNNO_____^RQ_")]
    recs = list(O.read_fastx(data("single-read.fa")))
    assert recs[0][:2] == ("895:1:1:1246:14654 1:N:0:NNNNN",
                           "CAGGCGCCCACCACCGTGCCCTCCAACCTGATGGT")


def test_num_reads_gz():
    assert len(list(O.read_fastx(data("100-reads.fq.gz")))) == 100
    names = sorted(int(n) for n, _, _ in O.read_fastx(data("random-20-a.fa")))
    assert names == list(range(len(names)))


def test_truncated():
    n = 0
    with pytest.raises(ValueError, match="Sequence is empty"):
        for _ in O.read_fastx(data("truncated.fq")):
            n += 1
    assert n == 1


def test_empty_and_missing():
    with pytest.raises(OSError, match="does not contain any sequences"):
        list(O.read_fastx(data("empty-file")))
    with pytest.raises(OSError):
        list(O.read_fastx(data("no-such-file.fa")))


# --- script-level numbers: tests/test_scripts.py -----------------------------
def test_load_into_counting_unique():
    # :65-90 (-x 1e3 -N 2 -k 20 -> 94), :278-345 (-x 1e7 -> 95, 1001 reads)
    t = O.Table(O.BYTE, 20, primes(2, 1e3))
    t.set_use_bigcount(True)
    assert t.consume_fastx(data("test-abund-read-2.fa"))[0] == 1001
    assert t.n_unique_kmers() == 94
    t = O.Table(O.BYTE, 20, primes(2, 1e7))
    t.consume_fastx(data("test-abund-read-2.fa"))
    assert t.n_unique_kmers() == 95
    # --small-count with defaults k=32, N=4, -x 1e3 -> 83
    s = O.Table(O.NIBBLE, 32, primes(4, 1e3))
    s.consume_fastx(data("test-abund-read-2.fa"))
    assert s.n_unique_kmers() == 83


def test_load_graph_unique():
    # :521-552 (-x 1e7 -N 2 -k 20, tagging path) -> 3960
    t = O.Table(O.BIT, 20, primes(2, 1e7))
    t.consume_fastx(data("random-20-a.fa"), tag=True)
    assert t.n_unique_kmers() == 3960
    # :717-736 (-x 1e5) -> 3959 unique, fp rate 0.002
    t = O.Table(O.BIT, 20, primes(2, 1e5))
    t.consume_fastx(data("random-20-a.fa"), tag=True)
    assert t.n_unique_kmers() == 3959
    fp = (t.n_occupied() / min(t.sizes)) ** 2
    assert "%1.3f" % fp == "0.002"


def test_fpr_json():
    # tests/test_scripts.py:323-345: fpr 9.025048735197377e-11 for -x 1e7 -N 2 -k 20
    t = O.Table(O.BYTE, 20, primes(2, 1e7))
    t.consume_fastx(data("test-abund-read-2.fa"))
    fp = (float(t.n_occupied()) / min(t.sizes)) ** 2.0
    assert fp == 9.025048735197377e-11


# --- file format: a reference-written Countgraph (tests/test-data/normC20k20.ct)
def test_normc20k20_header(tmp_path):
    src = data("normC20k20.ct.gz")
    raw = gzip.open(src).read()
    assert raw[:4] == b"OXLI" and raw[4] == 4 and raw[5] == 1
    k = int.from_bytes(raw[7:11], "little")
    n = raw[11]
    first = int.from_bytes(raw[20:28], "little")
    assert (k, n, first) == (20, 4, 999983)


def test_normc20k20_layout():
    # the reference-written file follows the layout our writers use:
    # header, N x (u64 size + size bytes), u64 n_bigcounts, n x (u64 key, u16 val)
    raw = gzip.open(data("normC20k20.ct.gz")).read()
    sizes, tables = [], []
    off = 20
    for _ in range(raw[11]):
        p = int.from_bytes(raw[off:off + 8], "little")
        sizes.append(p)
        tables.append(raw[off + 8:off + 8 + p])
        off += 8 + p
    nbig = int.from_bytes(raw[off:off + 8], "little")
    assert off + 8 + 10 * nbig == len(raw)
    # (this fixture's occupied field is 0: it was written before occupancy
    # tracking, so only the layout is checked here)
    for i in range(nbig):
        rec = raw[off + 8 + 10 * i: off + 18 + 10 * i]
        key = int.from_bytes(rec[:8], "little")
        val = int.from_bytes(rec[8:], "little")
        assert val > 255
        # a bigcount only exists where every table's bin is saturated
        assert all(t[key % p] == 255 for t, p in zip(tables, sizes))


# --- banding / mask consume: tests/test_banding.py, tests/test_counttable.py:83-187 ---
def _get(o, kmer):
    return o.get(o.hash(kmer))


@pytest.mark.parametrize("kind", [O.BIT, O.BYTE])
def test_oracle_banding_kat(kind):
    """tests/test_banding.py:140-157 (Nodetable / Counttable, k=31, 1e5 x 4)."""
    o = O.Table(kind, 31, primes(4, 100000), hash=O.MURMUR)
    assert o.consume_fastx_filtered(data("bogus.fa"), 8, 3) == (1, 3)
    for kmer, want in [("CGGCTATTATCTGAGCTCAAGACTAATACGC", 1), ("TATTATCTGAGCTCAAGACTAATACGCGCTG", 1),
                       ("TGAGCTCAAGACTAATACGCGCTGGCCACTG", 1), ("GTACGGCTATTATCTGAGCTCAAGACTAATA", 0),
                       ("TTATCTGAGCTCAAGACTAATACGCGCTGGC", 0), ("GCTCAAGACTAATACGCGCTGGCCACTGGTA", 0)]:
        assert _get(o, kmer) == want, kmer


def test_oracle_banding_bad_band():
    """tests/test_banding.py:120-136."""
    o = O.Table(O.BYTE, 31, primes(4, 100000), hash=O.MURMUR)
    with pytest.raises(ValueError, match="'band' must be in the interval"):
        o.consume_fastx_filtered(data("bogus.fa"), 8, 13)
    with pytest.raises(OSError):
        o.consume_fastx_filtered("file-no-exist.fa", 16, 3)


@pytest.mark.parametrize("numbands", [3, 11, 23, 29])
def test_oracle_banding_to_disk(tmp_path, numbands):
    """tests/test_banding.py:85-117: all bands consumed in turn give the same
    saved table bytes as one plain consume (Counttable k=21, 5e6/4 x 4)."""
    a = O.Table(O.BYTE, 21, primes(4, 5e6 / 4), hash=O.MURMUR)
    a.consume_fastx(data("banding-reads.fq.gz"))
    b = O.Table(O.BYTE, 21, primes(4, 5e6 / 4), hash=O.MURMUR)
    total = 0
    for band in range(numbands):
        total += b.consume_fastx_filtered(data("banding-reads.fq.gz"), numbands, band)[1]
    a.save(str(tmp_path / "a.ct"))
    b.save(str(tmp_path / "b.ct"))
    assert open(str(tmp_path / "a.ct"), "rb").read() == open(str(tmp_path / "b.ct"), "rb").read()


def _mask_from(path):
    m = O.Table(O.BYTE, 13, primes(4, 1e3), hash=O.MURMUR)
    m.consume_fastx(path)
    return m


def test_oracle_consume_with_mask():
    """tests/test_counttable.py:83-110."""
    mask = _mask_from(data("seq-a.fa"))
    o = O.Table(O.BYTE, 13, primes(4, 1e3), hash=O.MURMUR)
    assert o.consume_fastx_filtered(data("seq-b.fa"), mask=mask) == (1, 3)
    assert [_get(o, k) for k in ["GATTTGAGAAAAA", "ATTTGAGAAAAAA", "TTTGAGAAAAAAG", "TTGAGAAAAAAGT"]] == [0, 1, 1, 1]


def test_oracle_consume_banding_with_mask():
    """tests/test_counttable.py:113-136."""
    mask = _mask_from(data("seq-a.fa"))
    o = O.Table(O.BYTE, 13, primes(4, 1e3), hash=O.MURMUR)
    assert o.consume_fastx_filtered(data("seq-b.fa"), 4, 1, mask=mask) == (1, 1)
    assert [_get(o, k) for k in ["GATTTGAGAAAAA", "ATTTGAGAAAAAA", "TTTGAGAAAAAAG", "TTGAGAAAAAAGT"]] == [0, 0, 0, 1]


def test_oracle_consume_with_mask_threshold():
    """tests/test_counttable.py:139-173."""
    mask = O.Table(O.BYTE, 13, primes(4, 1e3), hash=O.MURMUR)
    for _ in range(3):
        mask.consume("TAGATCTGCTTGAAACAAGTGGATTTGAGAAAAA")
    for _ in range(2):
        mask.consume("TAGATCTGCTTGAAACAAGTGGATTTGAGAAAAAAGT")
    o = O.Table(O.BYTE, 13, primes(4, 1e3), hash=O.MURMUR)
    assert o.consume_fastx_filtered(data("seq-b.fa"), mask=mask, threshold=3) == (1, 3)
    assert [_get(o, k) for k in ["GATTTGAGAAAAA", "ATTTGAGAAAAAA", "TTTGAGAAAAAAG", "TTGAGAAAAAAGT"]] == [0, 1, 1, 1]


def test_oracle_consume_with_mask_complement():
    """tests/test_counttable.py:176-187."""
    mask = O.Table(O.BIT, 13, primes(4, 1e3), hash=O.MURMUR)
    mask.consume("TGCTTGAAACAAGTG")
    o = O.Table(O.BYTE, 13, primes(4, 1e3), hash=O.MURMUR)
    o.consume_fastx_filtered(data("seq-b.fa"), mask=mask, threshold=1, consume_masked=True)
    assert [_get(o, k) for k in ["TGCTTGAAACAAG", "GCTTGAAACAAGT", "CTTGAAACAAGTG"]] == [1, 1, 1]
    assert [_get(o, k) for k in ["GAAACAAGTGGAT", "AAACAAGTGGATT", "AACAAGTGGATTT"]] == [0, 0, 0]
