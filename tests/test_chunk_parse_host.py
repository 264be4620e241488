"""Host-only check of the chunk-parallel parse (kh_parser.cpp
plain_parse_chunk / plain_parse_rest, driven in consume_chunked's order by
tools/chunk_check.cpp) against the streaming parser over the same file:
reads parsed, a digest of the reads of >= k bases, and the error -- for plain
and BGZF files, every record layout of tests/test_gpu_feed.py, damaged BGZF
members and chunk sizes from 101 bytes.  No device."""
import os
import shutil
import subprocess

import pytest

from tests.conftest import ROOT

pytest.importorskip("khmer_amd")

LIB = os.path.join(ROOT, "khmer_amd", "libkhmer_hip.so")


@pytest.fixture(scope="module")
def checker(tmp_path_factory):
    if not shutil.which("g++") or not os.path.exists(LIB):
        pytest.skip("needs g++ and the built library")
    out = str(tmp_path_factory.mktemp("cc") / "chunk_check")
    subprocess.run(["bash", os.path.join(ROOT, "tools", "chunk_check.sh"), out], check=True,
                   capture_output=True)
    return out


def _run(checker, path, chunk):
    import json
    env = dict(os.environ, KH_BGZF_MIN_BYTES="1")
    r = subprocess.run([checker, path, str(chunk), "21"], capture_output=True, text=True, env=env, timeout=120)
    return json.loads(r.stdout.strip().splitlines()[-1])


LAYOUTS = {
    "fastq4": dict(kind="fq"),
    "fastq_wrapped": dict(kind="fq", wrap=50),
    "fastq_crlf": dict(kind="fq", crlf=True),
    "fastq_at_quals": dict(kind="fq", at_quals=True),
    "fastq_bad_record": dict(kind="fq", bad_at=2345),
    "fasta_wrapped": dict(kind="fa"),
}


@pytest.mark.parametrize("layout", sorted(LAYOUTS))
@pytest.mark.parametrize("bgzf", [False, True])
def test_chunk_parse_matches_streaming(tmp_path, checker, layout, bgzf):
    from tests import bgzf as B
    from tests.test_gpu_feed import _write_fasta, _write_fastq
    c = dict(LAYOUTS[layout])
    path = str(tmp_path / ("in." + c.pop("kind")))
    if path.endswith(".fq"):
        _write_fastq(path, 4000, **c)
    else:
        _write_fasta(path, 4000)
    if bgzf:
        blob = B.compress(open(path, "rb").read(), block=1000)
        path += ".bgz"
        open(path, "wb").write(blob)
    for chunk in ((4096, 65536) if bgzf else (101, 4096, 65536)):   # a BGZF chunk inflates >= 4 MiB
        r = _run(checker, path, chunk)
        assert r["same"], (chunk, r)
        assert r["reads"][0] == (2346 if layout == "fastq_bad_record" else 4000)


@pytest.mark.parametrize("where", ["early", "middle", "late"])
def test_chunk_parse_bgzf_damage(tmp_path, checker, where):
    from tests import bgzf as B
    from tests.test_gpu_feed import _write_fastq
    path = str(tmp_path / "in.fq")
    _write_fastq(path, 4000)
    blob = bytearray(B.compress(open(path, "rb").read(), block=1000))
    offs = B.member_offsets(bytes(blob))
    i = {"early": 2, "middle": len(offs) // 2, "late": len(offs) - 3}[where]
    blob[offs[i] + 30] ^= 0xFF
    bad = str(tmp_path / "bad.fq.bgz")
    open(bad, "wb").write(bytes(blob))
    for chunk in (4096, 65536):
        r = _run(checker, bad, chunk)
        assert r["same"] and r["err"][0].startswith("File "), (chunk, r)
        assert 0 < r["reads"][0] < 4000 or where == "early"


@pytest.mark.parametrize("scalar", ["0", "1"])
def test_pack_matches_restatement(checker, scalar):
    """HostBatch::append's cleaned 2-bit packing (BMI2 fast path, or the
    table loop with KH_PACK_SCALAR=1) against a scalar restatement of
    _to_valid_dna + twobit_repr over random reads of every byte value."""
    import json
    env = dict(os.environ, KH_PACK_SCALAR=scalar)
    r = subprocess.run([checker, "--pack", "20000"], capture_output=True, text=True, env=env, timeout=120)
    d = json.loads(r.stdout.strip().splitlines()[-1])
    assert d["mismatches"] == 0 and d["pack_bases"] > 3_000_000
    assert d["merge_mismatch"] == 0   # HostBatch::merge of random batch splits == one batch
