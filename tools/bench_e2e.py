#!/usr/bin/env python3
"""End-to-end (host-fed) rate of the drop-in path: Countgraph.consume_seqfile
on a synthetic FASTQ in the page cache -- parse, clean, 2-bit pack, upload and
count (src/oxli/hashtable.cc:125-150 via scripts/load-into-counting.py:143-158).
Not the headline metric (bench.py's value is device-resident input); this is
the PCIe/host-inclusive rate DESIGN.md reports beside it.

--compress gzip|bgzf: the same FASTQ gzip-compressed (one member, zlib level
6) or BGZF-compressed (htslib's bgzip layout, tests/bgzf.py; members
compressed on a thread pool here), to time the compressed-input feed
(KH_ASYNC_INFLATE=0 selects the serial inflate for an A/B).

--tag: the default load-graph.py path instead (Nodegraph.consume_seqfile_and_tag,
src/oxli/hashgraph.cc:290-320: the device sets the bits and returns the per-k-mer
is_new flags, the host runs the reference's per-read tag state machine),
C3's Nodegraph k=31 4 x 4e9 unless -k / -x say otherwise.

Prints one JSON line.  The FASTQ is the benchmark's synthetic stream
(khmer_amd/synth.py), written once with fixed-width names, then read once
untimed so it sits in the page cache.
"""
import argparse
import json
import os
import sys
import tempfile
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def write_fastq(path, nreads, L, chunk=1_000_000):
    from khmer_amd import synth
    width = len(str(nreads))
    rec = 1 + 1 + width + 1 + L + 3 + L + 1     # "@r<idx>\n" seq "\n+\n" qual "\n"
    with open(path, "wb") as fh:
        for r0 in range(0, nreads, chunk):
            n = min(chunk, nreads - r0)
            out = np.empty((n, rec), dtype=np.uint8)
            names = np.char.zfill(np.arange(r0, r0 + n).astype("U%d" % width), width).astype("S%d" % width)
            out[:, 0] = ord("@")
            out[:, 1] = ord("r")
            out[:, 2:2 + width] = np.frombuffer(names.tobytes(), dtype=np.uint8).reshape(n, width)
            out[:, 2 + width] = ord("\n")
            o = 3 + width
            out[:, o:o + L] = synth.read_ascii(r0, n, L)
            out[:, o + L:o + L + 3] = np.frombuffer(b"\n+\n", dtype=np.uint8)
            out[:, o + L + 3:o + 2 * L + 3] = ord("I")
            out[:, o + 2 * L + 3] = ord("\n")
            fh.write(out.tobytes())


def _bgzf_part(args):
    from tests import bgzf
    raw, block = args
    return b"".join(bgzf.member(raw[i:i + block]) for i in range(0, len(raw), block))


def compress(fq, how):
    """The FASTQ at fq compressed as `how` (the plain file is removed)."""
    if how == "none":
        return fq
    import zlib
    out = fq + (".gz" if how == "gzip" else ".bgz")
    with open(fq, "rb") as src, open(out, "wb") as dst:
        if how == "gzip":
            z = zlib.compressobj(6, zlib.DEFLATED, 31)
            while True:
                b = src.read(1 << 24)
                if not b:
                    break
                dst.write(z.compress(b))
            dst.write(z.flush())
        else:
            from multiprocessing.pool import ThreadPool   # zlib releases the GIL
            from tests import bgzf
            block, span = 65280, 65280 * 64
            with ThreadPool(min(16, os.cpu_count() or 1)) as pool:
                def spans():
                    while True:
                        b = src.read(span)
                        if not b:
                            return
                        yield b, block
                for part in pool.imap(_bgzf_part, spans(), chunksize=4):
                    dst.write(part)
            dst.write(bgzf.member(b""))
    os.remove(fq)
    with open(out, "rb") as fh:
        while fh.read(1 << 26):
            pass
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reads", type=int, default=10_000_000)
    ap.add_argument("--read-len", type=int, default=150)
    ap.add_argument("-k", type=int, default=None)
    ap.add_argument("-x", type=float, default=None)
    ap.add_argument("--tag", action="store_true", help="Nodegraph consume_seqfile_and_tag (load-graph.py default)")
    ap.add_argument("--tables", type=int, default=4)
    ap.add_argument("--cpu-reads", type=int, default=300_000)
    ap.add_argument("--compress", choices=["none", "gzip", "bgzf"], default="none")
    ap.add_argument("--make", default=None, help="only write the (compressed) FASTQ to this path and exit")
    ap.add_argument("--input", default=None, help="time this file (written by --make with the same --reads)")
    ap.add_argument("--dir", default=None, help="where to write the FASTQ (default: a temporary directory)")
    a = ap.parse_args()
    if a.make:
        write_fastq(a.make, a.reads, a.read_len)
        fq_bytes = os.path.getsize(a.make)
        t0 = time.perf_counter()
        out = compress(a.make, a.compress)
        print(json.dumps({"made": out, "fastq_bytes": fq_bytes, "file_bytes": os.path.getsize(out),
                          "compress_s": time.perf_counter() - t0}), flush=True)
        return
    a.k = a.k or (31 if a.tag else 21)
    a.x = a.x or (4e9 if a.tag else 1e9)
    import khmer_amd
    from khmer_amd import _lib
    _lib.set_default_device(int(os.environ.get("LOCAL_RANK", "0")))
    with tempfile.TemporaryDirectory(dir=a.dir) as tmp:
        if a.input:
            fq, t_write, t_compress = a.input, 0.0, 0.0
            w = len(str(a.reads))
            fq_bytes = a.reads * (2 * a.read_len + 7 + w)
            a.compress = {".gz": "gzip", ".bgz": "bgzf"}.get(os.path.splitext(fq)[1], "none")
        else:
            fq = os.path.join(tmp, "reads.fq")
            t0 = time.perf_counter()
            write_fastq(fq, a.reads, a.read_len)
            t_write = time.perf_counter() - t0
            fq_bytes = os.path.getsize(fq)
            t0 = time.perf_counter()
            fq = compress(fq, a.compress)
            t_compress = time.perf_counter() - t0
        size = os.path.getsize(fq)
        with open(fq, "rb") as fh:
            while fh.read(1 << 26):
                pass
        def graph():
            if a.tag:
                return khmer_amd.Nodegraph(a.k, a.x, a.tables)
            g = khmer_amd.Countgraph(a.k, a.x, a.tables)
            g.set_use_bigcount(True)
            return g
        cg = graph()
        # warm-up: the device pipeline's first use (workspace, code objects)
        cg.consume("A" * (a.k + 10))
        cg = graph()
        t0 = time.perf_counter()
        nr, nk = cg.consume_seqfile_and_tag(fq) if a.tag else cg.consume_seqfile(fq)
        dt = time.perf_counter() - t0
        n_new = None
        if a.tag:   # consume_sequence_and_tag counts the new k-mers (src/oxli/hashgraph.cc:219-221)
            n_new, nk = nk, a.reads * (a.read_len - a.k + 1)
        assert nr == a.reads and nk == a.reads * (a.read_len - a.k + 1), (nr, nk)
        cpu = None
        if a.cpu_reads:
            from oracle import oracle as O
            sub = os.path.join(tmp, "sample.fq")
            write_fastq(sub, a.cpu_reads, a.read_len)
            with open(sub, "rb") as fh:
                while fh.read(1 << 26):
                    pass
            t = O.Table(O.BIT if a.tag else O.BYTE, a.k, cg.hashsizes())
            t.set_use_bigcount(not a.tag)
            t0 = time.perf_counter()
            _, ck = t.consume_fastx(sub, tag=a.tag)
            cpu = {"value": ck / (time.perf_counter() - t0), "unit": "k-mers/s", "cores": 1, "kind": "port",
                   "sample": "%d reads of the same FASTQ layout, oracle/khmer_oracle.c consume_fastx "
                             "(parse + clean + count), 1 thread" % a.cpu_reads}
    feed = int(os.environ.get("KH_FEED_THREADS", "0")) or None
    print(json.dumps({
        "metric": ("k-mers/sec consume_seqfile_and_tag end to end (page-cached FASTQ -> parse -> pack -> H2D -> "
                   "set bits + is_new -> host tag state machine) into Nodegraph (k=%d, %dx%.0e)" if a.tag else
                   "k-mers/sec consume_seqfile end to end (page-cached FASTQ -> parse -> pack -> H2D -> count) "
                   "into Countgraph (k=%d, %dx%.0e)") % (a.k, a.tables, a.x),
        "n_tags": cg.n_tags if a.tag else None,
        "new_kmers_returned": n_new,
        "value": nk / dt, "unit": "k-mers/s", "reads": nr, "kmers": nk, "seconds": dt,
        "compress": a.compress, "async_inflate": os.environ.get("KH_ASYNC_INFLATE", "1") != "0",
        "file_bytes": size, "file_GBps": size / dt / 1e9, "fastq_bytes": fq_bytes, "fastq_GBps": fq_bytes / dt / 1e9,
        "write_s": t_write, "compress_s": t_compress,
        "host_threads": os.environ.get("OMP_NUM_THREADS"), "feed_threads_override": feed,
        "n_unique_kmers": cg.n_unique_kmers(), "n_occupied": cg.n_occupied(),
        "cpu_baseline": cpu,
    }), flush=True)


if __name__ == "__main__":
    main()
