"""Reads and the shared FASTA/FASTQ parser.

Mirrors khmer.Read / khmer.ReadParser (src/khmer/_cpy_readparsers.cc:392-550
over oxli::read_parsers, src/oxli/read_parsers.cc:257-382).  Parsing runs in
libkhmer_hip.so (C++, gzip aware); one parser may be drained by several
threads, each read is returned exactly once.
"""
import ctypes

from . import _lib
from ._lib import lib, check


def _to_valid_dna(seq):
    """read_parsers.cc:53-69: ACGT kept, acgt upper-cased, anything else 'A'."""
    out = []
    for c in seq:
        if c in "ACGT":
            out.append(c)
        elif c in "acgt":
            out.append(c.upper())
        else:
            out.append("A")
    return "".join(out)


class Read(object):
    """A sequence record; absent fields are absent attributes (as in khmer)."""

    def __init__(self, name=None, sequence=None, quality=None, description=None):
        if name is not None:
            self.name = name
        if sequence is not None:
            self.sequence = sequence
        if quality is not None:
            self.quality = quality
        if description is not None:
            self.description = description

    @property
    def cleaned_seq(self):
        return _to_valid_dna(self.sequence)

    def __len__(self):
        return len(self.sequence)

    def __repr__(self):
        return "Read(name=%r, sequence=%r)" % (getattr(self, "name", None),
                                               getattr(self, "sequence", None))


class ReadParser(object):
    """khmer.ReadParser(filename): iterable of Read, thread-safe."""

    def __init__(self, filename):
        self._h = None
        self.filename = filename
        h = ctypes.c_void_p()
        check(lib.kh_parser_open(str(filename).encode(), ctypes.byref(h)))
        self._h = h

    @property
    def handle(self):
        if self._h is None:
            raise ValueError("I/O operation on closed parser")
        return self._h

    def __iter__(self):
        return self

    def __next__(self):
        n, s, q = ctypes.c_char_p(), ctypes.c_char_p(), ctypes.c_char_p()
        nl, sl, ql = ctypes.c_size_t(), ctypes.c_size_t(), ctypes.c_size_t()
        rc = lib.kh_parser_next_read(self.handle, ctypes.byref(n), ctypes.byref(nl),
                                     ctypes.byref(s), ctypes.byref(sl),
                                     ctypes.byref(q), ctypes.byref(ql))
        if rc == _lib.KH_END:
            raise StopIteration
        check(rc)
        name = ctypes.string_at(n, nl.value).decode("latin-1")
        seq = ctypes.string_at(s, sl.value).decode("latin-1")
        qual = ctypes.string_at(q, ql.value).decode("latin-1") if ql.value else None
        return Read(name=name, sequence=seq, quality=qual)

    next = __next__

    @property
    def num_reads(self):
        out = ctypes.c_uint64()
        check(lib.kh_parser_num_reads(self.handle, ctypes.byref(out)))
        return out.value

    def is_complete(self):
        out = ctypes.c_int()
        check(lib.kh_parser_is_complete(self.handle, ctypes.byref(out)))
        return bool(out.value)

    def close(self):
        if self._h is not None:
            lib.kh_parser_close(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass
