"""Development probe: the synthetic collision workload of
tests/test_gpu_parity.py::test_synthetic_1m_reads, printing how the device
tables differ from the oracle (for debugging partition variants)."""
import ctypes
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import khmer_amd  # noqa: E402
from khmer_amd import synth  # noqa: E402
from khmer_amd._lib import lib, check  # noqa: E402
from oracle import oracle as O  # noqa: E402

seqs, offs = synth.batch(0, 200000, 150)
sizes = O.get_n_primes_near_x(4, 4000037)
o = O.Table(O.BYTE, 21, sizes)
o.set_use_bigcount(True)
o.consume_batch(seqs, [int(v) for v in offs])
ref = [np.frombuffer(o.table_bytes(i), dtype=np.uint8).astype(np.int32) for i in range(4)]
arr = (ctypes.c_uint64 * len(offs))(*[int(v) for v in offs])
for rep in range(int(sys.argv[1]) if len(sys.argv) > 1 else 2):
    g = khmer_amd.Countgraph(21, 1, 1, primes=sizes)
    g.set_use_bigcount(True)
    out = ctypes.c_uint64()
    check(lib.kh_consume_seqs(g._g, seqs, arr, len(offs) - 1, 1, ctypes.byref(out)))
    tabs = g.get_raw_tables()
    msg = []
    for i in range(4):
        a = np.frombuffer(bytes(tabs[i]), dtype=np.uint8).astype(np.int32)
        d = a - ref[i]
        nz = np.nonzero(d)[0]
        msg.append("t%d: %d bins differ, sum(ours-ref)=%d, min %d max %d, first %s" % (
            i, len(nz), int(d.sum()), int(d.min()), int(d.max()), nz[:5].tolist()))
    print("rep", rep, "n_unique", g.n_unique_kmers(), "| " + " | ".join(msg), flush=True)
dbg = (ctypes.c_uint64 * 64)()
if hasattr(lib, "kh_debug_read"):
    lib.kh_debug_read(dbg)
    print("dbg", {i: dbg[i] for i in range(64) if dbg[i]})
