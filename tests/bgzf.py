"""BGZF writer for tests (SAM/BAM format specification 4.1, htslib's bgzip
layout): gzip members of <= 65280 input bytes, each with FLG.FEXTRA and a
'BC' subfield holding the member size - 1, and the 28-byte empty end-of-file
member.  Python's gzip module reads the result as multi-member gzip."""
import struct
import zlib


def member(chunk, level=6):
    c = zlib.compressobj(level, zlib.DEFLATED, -15)
    d = c.compress(chunk) + c.flush()
    bsize = 10 + 2 + 6 + len(d) + 8 - 1
    hdr = (b"\x1f\x8b\x08\x04" + b"\x00\x00\x00\x00" + b"\x00\xff" + struct.pack("<H", 6) + b"BC" +
           struct.pack("<HH", 2, bsize))
    return hdr + d + struct.pack("<II", zlib.crc32(chunk) & 0xFFFFFFFF, len(chunk))


def compress(raw, block=65280, eof=True):
    out = [member(raw[i:i + block]) for i in range(0, len(raw), block)]
    if eof:
        out.append(member(b""))
    return b"".join(out)


def member_offsets(blob):
    """Start offset of every member of a BGZF blob."""
    offs, off = [], 0
    while off < len(blob):
        offs.append(off)
        xlen = struct.unpack_from("<H", blob, off + 10)[0]
        assert blob[off + 12:off + 14] == b"BC" and xlen == 6
        off += struct.unpack_from("<H", blob, off + 16)[0] + 1
    return offs
