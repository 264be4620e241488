"""CPU-only checks of libkhmer_hip.so: it loads, exports every symbol the
C-ABI header declares, and its host-side logic (scalar hashing, primes, the
FASTA/FASTQ reader) matches the oracle.  No device calls."""
import os
import re

import pytest

from oracle import oracle as O
from tests.conftest import ROOT, data

khmer = pytest.importorskip("khmer_amd")
from khmer_amd import _lib  # noqa: E402


def declared_symbols():
    text = open(os.path.join(ROOT, "include", "khmer_hip.h")).read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"\b(kh_[a-z0-9_]+)\s*\(", text)))


def test_header_symbols_exported():
    syms = declared_symbols()
    assert len(syms) > 40
    missing = [s for s in syms if not hasattr(_lib.lib, s)]
    assert not missing, missing


def test_bindings_cover_header():
    # every declared entry point has a ctypes signature in khmer_amd._lib
    assert set(declared_symbols()) == set(_lib.SIGNATURES)


def test_abi_version():
    assert _lib.lib.kh_abi_version() == 1


@pytest.mark.parametrize("kmer", ["AAAA", "TTTT", "CCCC", "GGGG", "ACGTNacgt", "G" * 12,
                                  "GGTTGACGGGGCTCAGGGGGCGGCTGACTCCG", "AAACGTATGACT"])
def test_hash_helpers_match_oracle(kmer):
    k = len(kmer)
    if k <= 32:
        assert khmer.forward_hash(kmer, k) == O.forward_hash(kmer, k)
        assert khmer.forward_hash_no_rc(kmer, k) == O.forward_hash_no_rc(kmer, k)
        h = O.forward_hash(kmer, k)
        assert khmer.reverse_hash(h, k) == O.reverse_hash(h, k)
    assert khmer.hash_murmur3(kmer) == O.hash_murmur3(kmer)
    assert khmer.hash_no_rc_murmur3(kmer) == O.hash_no_rc_murmur3(kmer)
    assert khmer.reverse_complement(kmer) == O.reverse_complement(kmer)


def test_murmur_lengths():
    # every Murmur tail length and multi-block keys
    s = "ACGTTGCAAGGCTTAACCGGTATATCGCGATAGCTAGCTAGGATCCATGCAT"
    for n in range(1, len(s) + 1):
        assert khmer.hash_murmur3(s[:n]) == O.hash_murmur3(s[:n]), n
        assert khmer.hash_no_rc_murmur3(s[:n]) == O.hash_no_rc_murmur3(s[:n]), n


def test_hash_errors():
    with pytest.raises(ValueError):
        khmer.forward_hash("AAAA", 5)
    with pytest.raises(ValueError):
        khmer.forward_hash("A" * 33, 33)
    with pytest.raises(TypeError):
        khmer.reverse_hash("2345", 4)


def test_primes():
    assert khmer.get_n_primes_near_x(7, 20) == [19, 17, 13, 11, 7, 5, 3]
    assert khmer.get_n_primes_near_x(7, 20.) == [19, 17, 13, 11, 7, 5, 3]
    with pytest.raises(RuntimeError, match="unable to find 5 prime numbers < 5"):
        khmer.get_n_primes_near_x(5, 5)
    for x in (1e3, 1e5, 1e7, 123457, 4 ** 4):
        assert khmer.get_n_primes_near_x(4, x) == O.get_n_primes_near_x(4, x)
    assert khmer.get_n_primes_near_x(1, 1) == [1]
    assert khmer.is_prime(999999937) and not khmer.is_prime(999999939)


def test_kmer_hashes_helper():
    seq = "ACGTACGTTTGACCAGTNNACGTAGGCTAacgtTTTTAAAAC"
    for k in (4, 9, 21):
        o = O.Table(O.BYTE, k, [101])
        assert _hashes(khmer._lib.HASH_TWOBIT, k, seq) == o.kmer_hashes(seq)
        m = O.Table(O.BYTE, k, [101], hash=O.MURMUR)
        assert _hashes(khmer._lib.HASH_MURMUR, k, seq) == m.kmer_hashes(seq)


def _hashes(kind, k, seq):
    import ctypes
    b = seq.encode()
    out = (ctypes.c_uint64 * len(b))()
    n = ctypes.c_uint64()
    _lib.check(_lib.lib.kh_kmer_hashes(kind, k, b, len(b), out, ctypes.byref(n)))
    return list(out[:n.value])


PARSE_FILES = ["random-20-a.fa", "random-20-a.fa.gz", "random-20-a.fq", "test-abund-read-2.fa",
               "valid-read-testing.fq", "single-read.fq", "single-read.fa", "100-reads.fq.gz",
               "test-short.fa", "all-A.fa", "bogus.fa", "random-31-c.fa", "25k.fq.gz"]


@pytest.mark.parametrize("fname", PARSE_FILES)
def test_parser_matches_oracle(fname):
    ours = [(r.name, r.sequence, getattr(r, "quality", "")) for r in khmer.ReadParser(data(fname))]
    theirs = list(O.read_fastx(data(fname)))
    assert ours == theirs


BZ2_FILES = ["100-reads.fq.bz2", "random-20-a.fa.bz2", "random-20-a.fq.bz2", "test-abund-read-2.fa.bz2"]


def _decompressed(tmp_path, fname):
    import bz2
    out = tmp_path / fname.replace(".bz2", "")
    out.write_bytes(bz2.decompress(open(data(fname), "rb").read()))
    return str(out)


@pytest.mark.parametrize("fname", BZ2_FILES)
def test_parser_bzip2(tmp_path, fname):
    """bzip2 input (seqan autodetection, reference tests/test_read_parsers.py:208-215):
    the records equal the oracle's on Python's bz2-decompressed copy."""
    ours = [(r.name, r.sequence, getattr(r, "quality", "")) for r in khmer.ReadParser(data(fname))]
    assert ours == list(O.read_fastx(_decompressed(tmp_path, fname)))
    if fname == "100-reads.fq.bz2":
        assert len(ours) == 100


def test_parser_bzip2_multistream(tmp_path):
    import bz2
    raw = open(data("random-20-a.fq"), "rb").read()
    cut = raw.index(b"@", len(raw) // 2)
    f = tmp_path / "multi.fq.bz2"
    f.write_bytes(bz2.compress(raw[:cut]) + bz2.compress(raw[cut:]))
    ours = [(r.name, r.sequence, r.quality) for r in khmer.ReadParser(str(f))]
    assert ours == list(O.read_fastx(data("random-20-a.fq")))


@pytest.mark.parametrize("fname", ["100-reads.fq.truncated.bz2", "100-reads.fq.truncated.gz"])
def test_parser_truncated_compressed(fname):
    """Opening succeeds; iterating raises OSError (reference
    tests/test_read_parsers.py:183-228)."""
    p = khmer.ReadParser(data(fname))
    with pytest.raises(OSError):
        for _ in p:
            pass


@pytest.mark.parametrize("fname", ["test-empty.fa.bz2", "empty-file.bz2"])
def test_parser_empty_bzip2(fname):
    with pytest.raises(OSError, match="does not contain any sequences"):
        khmer.ReadParser(data(fname))


def test_parser_corrupt_bzip2(tmp_path):
    import bz2
    blob = bytearray(bz2.compress(open(data("random-20-a.fa"), "rb").read()))
    blob[len(blob) // 2] ^= 0xFF
    f = tmp_path / "corrupt.fa.bz2"
    f.write_bytes(bytes(blob))
    with pytest.raises(OSError):
        list(khmer.ReadParser(str(f)))


def test_parser_errors(tmp_path):
    p = khmer.ReadParser(data("truncated.fq"))
    n = 0
    with pytest.raises(ValueError, match="Sequence is empty"):
        for _ in p:
            n += 1
    assert n == 1 and p.num_reads == 1
    with pytest.raises(OSError, match="does not contain any sequences"):
        khmer.ReadParser(data("empty-file"))
    with pytest.raises(OSError):
        khmer.ReadParser(data("does-not-exist.fa"))
    bad = tmp_path / "bad.fq"
    bad.write_text("@r1\nACGT\n+x\nIIII\n")
    with pytest.raises(OSError):
        list(khmer.ReadParser(str(bad)))
    ragged = tmp_path / "ragged.fq"
    ragged.write_text("@r1\nACGT\n+\nIIII\n@r2\nAC GT\nT\n+r2\nII\nIII\n@r3\nAAAA\n+\nIII")
    ours, theirs = [], []
    with pytest.raises(ValueError, match="lengths differ"):
        for r in khmer.ReadParser(str(ragged)):
            ours.append((r.name, r.sequence, r.quality))
    with pytest.raises(ValueError, match="lengths differ"):
        for rec in O.read_fastx(str(ragged)):
            theirs.append(rec)
    assert ours == theirs and len(ours) == 2


def test_parser_threads():
    import threading
    p = khmer.ReadParser(data("100-reads.fq.gz"))
    seen = []

    def run():
        for r in p:
            seen.append(r.name)

    ts = [threading.Thread(target=run) for _ in range(4)]
    for t in ts:
        t.start()
    for t in ts:
        t.join()
    assert p.num_reads == 100 and len(set(seen)) == 100


def test_read_object():
    r = khmer.Read(sequence="ACGTN", quality="good", name="1234", description="desc")
    assert r.name == "1234" and r.description == "desc"
    assert r.cleaned_seq == "ACGTA"
    r2 = khmer.Read(sequence="acgt")
    assert not hasattr(r2, "quality") and r2.cleaned_seq == "ACGT"


def test_no_device_graph_raises():
    if _lib.device_count() > 0:
        pytest.skip("device present")
    with pytest.raises(RuntimeError):
        khmer.Countgraph(21, 1e5, 4)


# ---- compressed input off the parsing thread (kh_parser.cpp BgzfSource /
# ReadAheadSource): same records and errors as the serial zlib path ----

def _plain_25k(tmp_path):
    import gzip
    raw = gzip.decompress(open(data("25k.fq.gz"), "rb").read())
    f = tmp_path / "25k.fq"
    f.write_bytes(raw)
    return raw, str(f)


def _records(path):
    return [(r.name, r.sequence, r.quality) for r in khmer.ReadParser(path)]


def test_parser_bgzf(tmp_path):
    """A BGZF file (worker-thread inflate of member groups) parses to the
    oracle's records of the plain file; Python's gzip reads the same bytes."""
    import gzip
    from tests import bgzf
    raw, plain = _plain_25k(tmp_path)
    blob = bgzf.compress(raw)
    assert gzip.decompress(blob) == raw and len(bgzf.member_offsets(blob)) > 32
    f = tmp_path / "25k.fq.bgz"
    f.write_bytes(blob)
    ours = _records(str(f))
    assert len(ours) == 25000
    assert ours == list(O.read_fastx(plain))


def test_parser_bgzf_small_members(tmp_path):
    """Members of a few hundred bytes: records cross many member and group
    boundaries."""
    from tests import bgzf
    raw, plain = _plain_25k(tmp_path)
    f = tmp_path / "small.fq.gz"
    f.write_bytes(bgzf.compress(raw, block=777))
    assert _records(str(f)) == list(O.read_fastx(plain))


def test_parser_bgzf_eof_member_alone(tmp_path):
    """64q + 1 members: the 28-byte empty EOF member is alone in the last
    member group, whose ring slot has never held data (zlib refused
    the null output buffer and the parser raised OSError after the last
    record).  Default BGZF threshold, so the worker-thread inflate runs."""
    from tests import bgzf
    raw, plain = _plain_25k(tmp_path)
    blob = bgzf.compress(raw, block=len(raw) // 128 + 1)
    assert len(bgzf.member_offsets(blob)) % 64 == 1 and len(blob) > (1 << 20)
    f = tmp_path / "eof_alone.fq.gz"
    f.write_bytes(blob)
    assert _records(str(f)) == list(O.read_fastx(plain))


@pytest.mark.parametrize("where", ["member", "crc"])
def test_parser_bgzf_corrupt(tmp_path, where):
    """Damage in a middle member: OSError, after exactly the records that lie
    wholly before that member's group (never a record past the damage)."""
    from tests import bgzf
    raw, plain = _plain_25k(tmp_path)
    blob = bytearray(bgzf.compress(raw))
    offs = bgzf.member_offsets(bytes(blob))
    i = len(offs) // 2
    if where == "member":
        blob[offs[i] + 40] ^= 0xFF              # inside the deflate data
    else:
        blob[offs[i + 1] - 8] ^= 0x01           # the member's CRC32
    f = tmp_path / "bad.fq.gz"
    f.write_bytes(bytes(blob))
    ours = []
    with pytest.raises(OSError):
        for r in khmer.ReadParser(str(f)):
            ours.append((r.name, r.sequence, r.quality))
    theirs = list(O.read_fastx(plain))
    assert 0 < len(ours) < len(theirs) and ours == theirs[:len(ours)]
    # the records returned end inside the damaged member (its bytes decoded
    # before the damage is found), and every earlier member's records came
    end = 0
    for _ in range(4 * len(ours)):
        end = raw.index(b"\n", end) + 1
    assert i * 65280 - 1000 <= end <= (i + 1) * 65280


def test_parser_bgzf_truncated(tmp_path):
    """A BGZF file cut inside a member is not a clean chain: zlib's path
    (read-ahead thread), OSError after a prefix of the records."""
    from tests import bgzf
    raw, plain = _plain_25k(tmp_path)
    blob = bgzf.compress(raw)
    f = tmp_path / "cut.fq.gz"
    f.write_bytes(blob[:len(blob) // 2 + 123])
    ours = []
    with pytest.raises(OSError):
        for r in khmer.ReadParser(str(f)):
            ours.append((r.name, r.sequence, r.quality))
    theirs = list(O.read_fastx(plain))
    assert 0 < len(ours) < len(theirs) and ours == theirs[:len(ours)]


def test_parser_multimember_gzip(tmp_path):
    """Concatenated plain gzip members (no BC field): the zlib path reads
    them all, as gzread does."""
    import gzip
    raw, plain = _plain_25k(tmp_path)
    cut = raw.index(b"\n@", len(raw) // 3) + 1
    f = tmp_path / "cat.fq.gz"
    f.write_bytes(gzip.compress(raw[:cut]) + gzip.compress(raw[cut:]))
    assert _records(str(f)) == list(O.read_fastx(plain))


def test_parser_gzip_closed_early(tmp_path):
    """A parser closed after one read (decompression still running ahead)
    shuts its threads down."""
    from tests import bgzf
    raw, _ = _plain_25k(tmp_path)
    f = tmp_path / "early.fq.gz"
    f.write_bytes(bgzf.compress(raw))
    for path in (str(f), data("25k.fq.gz")):
        for _ in range(20):
            p = khmer.ReadParser(path)
            next(iter(p))
            del p
