"""Seeded synthetic reads.

Counter-based SplitMix64: word t of read r is
    mix(seed + (r * 2**20 + t) * 0x9E3779B97F4A7C15)   (mod 2**64)
with mix = SplitMix64's output function; base i of read r is the 2-bit code
(A=0, T=1, C=2, G=3) at bits 63-2*(i%32) .. 62-2*(i%32) of word i // 32.
The same definition is implemented on the device (kh_synth_packed_device) so a
benchmark batch can be generated straight into HBM and checked on a host
sample.
"""
import numpy as np

SEED = 0x6b686d6572  # "khmer"
GOLDEN = np.uint64(0x9E3779B97F4A7C15)
_ASCII = np.frombuffer(b"ATCG", dtype=np.uint8)


def _mix(z):
    z = z.copy()
    z ^= z >> np.uint64(30)
    z *= np.uint64(0xBF58476D1CE4E5B9)
    z ^= z >> np.uint64(27)
    z *= np.uint64(0x94D049BB133111EB)
    z ^= z >> np.uint64(31)
    return z


def read_codes(r0, nreads, length, seed=SEED):
    """uint8 array [nreads, length] of 2-bit base codes for reads r0..r0+n-1."""
    nw = (length + 31) // 32
    r = np.arange(r0, r0 + nreads, dtype=np.uint64)[:, None]
    t = np.arange(nw, dtype=np.uint64)[None, :]
    with np.errstate(over="ignore"):
        key = np.uint64(seed) + (r * np.uint64(1 << 20) + t) * GOLDEN
    words = _mix(key)                                   # [n, nw]
    shifts = (np.uint64(62) - np.uint64(2) * (np.arange(32, dtype=np.uint64)))
    codes = (words[:, :, None] >> shifts[None, None, :]) & np.uint64(3)
    return codes.reshape(nreads, nw * 32)[:, :length].astype(np.uint8)


def read_ascii(r0, nreads, length, seed=SEED):
    """bytes rows [nreads, length] of ASCII bases."""
    return _ASCII[read_codes(r0, nreads, length, seed)]


def write_fastq(path, nreads, length, seed=SEED, chunk=100000, r0=0):
    """FASTQ with quality 'I' (the script-path input of SURVEY §8(d))."""
    qual = b"I" * length
    with open(path, "wb") as fh:
        for a in range(r0, r0 + nreads, chunk):
            n = min(chunk, r0 + nreads - a)
            rows = read_ascii(a, n, length, seed)
            out = []
            for i in range(n):
                out.append(b"@r%d\n%s\n+\n%s\n" % (a + i, rows[i].tobytes(), qual))
            fh.write(b"".join(out))


def batch(r0, nreads, length, seed=SEED):
    """(concatenated ASCII bytes, offsets) for kh_consume_seqs / oracle batches."""
    rows = read_ascii(r0, nreads, length, seed)
    offs = np.arange(nreads + 1, dtype=np.uint64) * np.uint64(length)
    return rows.tobytes(), offs
