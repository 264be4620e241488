"""The host feed of consume_seqfile (kh_capi.cpp consume_pipelined): the
chunk-parallel path for plain files must give exactly what the serial parser
gives -- (reads, k-mers), every table byte, n_unique, n_occupied, the error
and the reads consumed before it -- for any chunk size, record layout
(FASTA, four-line FASTQ, wrapped FASTQ, CRLF) and malformed input.
Reference semantics: Hashtable::consume_seqfile over FastxReader
(src/oxli/hashtable.cc:125-150, src/oxli/read_parsers.cc:329-372)."""
import os

import pytest

from khmer_amd import synth

pytestmark = pytest.mark.gpu

DATA = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "data")


def _consume(monkeypatch, path, chunk, threads, k=21):
    import khmer_amd
    monkeypatch.setenv("KH_FEED_CHUNK", str(chunk))
    monkeypatch.setenv("KH_FEED_THREADS", str(threads))
    g = khmer_amd.Countgraph(k, 1e5, 3)
    g.set_use_bigcount(True)
    err = None
    try:
        rk = g.consume_seqfile(path)
    except (ValueError, OSError) as e:
        rk, err = None, (type(e), str(e))
    tabs = [bytes(t) for t in g.get_raw_tables()]
    return rk, err, tabs, g.n_unique_kmers(), g.n_occupied()


def _write_fastq(path, n, L=120, wrap=0, crlf=False, bad_at=None, at_quals=False):
    rows = synth.read_ascii(0, n, L)
    nl = "\r\n" if crlf else "\n"
    with open(path, "w") as fh:
        for i in range(n):
            s = rows[i].tobytes().decode()
            q = ("@" if at_quals else "I") + "I" * (L - 1)
            if bad_at is not None and i == bad_at:
                q = q[:-3]
            if wrap:
                s = nl.join(s[j:j + wrap] for j in range(0, len(s), wrap))
                q = nl.join(q[j:j + wrap] for j in range(0, len(q), wrap))
            fh.write("@r%d%s%s%s+%s%s%s" % (i, nl, s, nl, nl, q, nl))


def _write_fasta(path, n, L=100, wrap=60):
    rows = synth.read_ascii(0, n, L)
    with open(path, "w") as fh:
        for i in range(n):
            s = rows[i].tobytes().decode()
            fh.write(">r%d\n%s\n" % (i, "\n".join(s[j:j + wrap] for j in range(0, len(s), wrap))))


CASES = {
    "fastq4": dict(kind="fq"),
    "fastq_wrapped": dict(kind="fq", wrap=50),
    "fastq_crlf": dict(kind="fq", crlf=True),
    "fastq_at_quals": dict(kind="fq", at_quals=True),
    "fastq_bad_record": dict(kind="fq", bad_at=2345),
    "fasta_wrapped": dict(kind="fa"),
}


@pytest.mark.parametrize("case", sorted(CASES))
@pytest.mark.parametrize("chunk", [777, 65536])
def test_chunked_feed_matches_serial(tmp_path, monkeypatch, case, chunk):
    c = dict(CASES[case])
    path = str(tmp_path / ("in." + c.pop("kind")))
    if path.endswith(".fq"):
        _write_fastq(path, 4000, **c)
    else:
        _write_fasta(path, 4000)
    serial = _consume(monkeypatch, path, 1 << 30, 1)
    chunked = _consume(monkeypatch, path, chunk, 8)
    assert chunked == serial
    if case == "fastq_bad_record":   # a short quality line: the record reader fails mid-file
        assert serial[1] is not None and serial[0] is None


@pytest.mark.parametrize("name", ["random-20-a.fa", "random-20-a.fq", "valid-read-testing.fq",
                                  "test-abund-read-2.fa", "single-read.fq", "truncated.fq", "bogus.fa"])
def test_chunked_feed_fixtures(monkeypatch, name):
    path = os.path.join(DATA, name)
    assert _consume(monkeypatch, path, 101, 8) == _consume(monkeypatch, path, 1 << 30, 1)


def test_chunked_feed_parser_object(monkeypatch):
    """A shared ReadParser drained by the chunk path reports every read."""
    import khmer_amd
    monkeypatch.setenv("KH_FEED_CHUNK", "555")
    monkeypatch.setenv("KH_FEED_THREADS", "8")
    path = os.path.join(DATA, "random-20-a.fa")
    rp = khmer_amd.ReadParser(path)
    g = khmer_amd.Countgraph(20, 1e5, 2)
    reads, kmers = g.consume_seqfile(rp)
    assert rp.num_reads == reads == 99
    assert g.consume_seqfile(rp) == (0, 0)


@pytest.mark.parametrize("how", ["bgzf", "gzip", "bz2"])
def test_compressed_feed_matches_plain(tmp_path, monkeypatch, how):
    """Compressed input (BGZF member groups inflated on worker threads, other
    gzip / bzip2 streams on a read-ahead thread) consumes to exactly the
    plain file's tables and counters."""
    import bz2
    import gzip
    from tests import bgzf
    plain = str(tmp_path / "in.fq")
    _write_fastq(plain, 40000)
    raw = open(plain, "rb").read()
    blob = {"bgzf": lambda: bgzf.compress(raw, block=8192), "gzip": lambda: gzip.compress(raw),
            "bz2": lambda: bz2.compress(raw)}[how]()
    if how == "bgzf":
        assert len(blob) > (1 << 20)   # large enough for the worker-thread path
    comp = str(tmp_path / ("in.fq." + how))
    open(comp, "wb").write(blob)
    want = _consume(monkeypatch, plain, 1 << 30, 1)
    assert _consume(monkeypatch, comp, 1 << 30, 8) == want
    assert want[0] == (40000, 40000 * 100)


def test_bgzf_feed_corrupt_member(tmp_path, monkeypatch):
    """A damaged BGZF member: consume_seqfile raises OSError."""
    from tests import bgzf
    plain = str(tmp_path / "in.fq")
    _write_fastq(plain, 40000)
    blob = bytearray(bgzf.compress(open(plain, "rb").read(), block=8192))
    offs = bgzf.member_offsets(bytes(blob))
    blob[offs[len(offs) // 2] + 30] ^= 0xFF
    comp = str(tmp_path / "bad.fq.gz")
    open(comp, "wb").write(bytes(blob))
    rk, err, _, _, _ = _consume(monkeypatch, comp, 1 << 30, 8)
    assert rk is None and err[0] is OSError


@pytest.mark.parametrize("case", sorted(CASES))
@pytest.mark.parametrize("chunk", [777, 65536])
def test_bgzf_chunked_feed(tmp_path, monkeypatch, case, chunk):
    """BGZF input through the chunk-parallel feed (each chunk inflates only the
    members under its window): the plain file's serial result, for every
    layout (CRLF and wrapped FASTQ fall back to the streaming feed, a
    malformed record raises after the same reads), and the same as streaming
    the BGZF file through one parser (KH_BGZF_CHUNKED=0)."""
    from tests import bgzf
    c = dict(CASES[case])
    plain = str(tmp_path / ("in." + c.pop("kind")))
    if plain.endswith(".fq"):
        _write_fastq(plain, 4000, **c)
    else:
        _write_fasta(plain, 4000)
    raw = open(plain, "rb").read()
    comp = plain + ".bgz"
    open(comp, "wb").write(bgzf.compress(raw, block=1000))
    monkeypatch.setenv("KH_BGZF_MIN_BYTES", "1")   # the BGZF paths for a small file
    serial = _consume(monkeypatch, plain, 1 << 30, 1)
    assert _consume(monkeypatch, comp, chunk, 8) == serial
    monkeypatch.setenv("KH_BGZF_CHUNKED", "0")
    assert _consume(monkeypatch, comp, chunk, 8) == serial


@pytest.mark.parametrize("where", ["early", "middle", "late"])
def test_bgzf_chunked_feed_damage(tmp_path, monkeypatch, where):
    """A damaged member under some chunk's window: the chunked feed consumes
    exactly the reads the streaming parser returns before the damage, then
    raises OSError (same tables, same counters)."""
    from tests import bgzf
    plain = str(tmp_path / "in.fq")
    _write_fastq(plain, 4000)
    blob = bytearray(bgzf.compress(open(plain, "rb").read(), block=1000))
    offs = bgzf.member_offsets(bytes(blob))
    i = {"early": 2, "middle": len(offs) // 2, "late": len(offs) - 3}[where]
    blob[offs[i] + 30] ^= 0xFF
    comp = str(tmp_path / "bad.fq.bgz")
    open(comp, "wb").write(bytes(blob))
    monkeypatch.setenv("KH_BGZF_MIN_BYTES", "1")
    chunked = _consume(monkeypatch, comp, 4096, 8)
    monkeypatch.setenv("KH_BGZF_CHUNKED", "0")
    streamed = _consume(monkeypatch, comp, 4096, 8)
    assert chunked[1] is not None and chunked[1][0] is OSError
    assert chunked == streamed
