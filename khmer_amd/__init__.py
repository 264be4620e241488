"""khmer_amd: khmer's k-mer counting path (Countgraph / Nodegraph /
SmallCountgraph and the Murmur *table family) on AMD Instinct MI355X.

Drop-in for the `khmer` names that scripts/load-into-counting.py and
scripts/load-graph.py use (khmer/__init__.py:36-215); `import khmer_amd as
khmer` in a script is the whole integration.  Tables live in HBM and are
updated by hand-written HIP kernels in libkhmer_hip.so.
"""
import ctypes
from collections import namedtuple
import sys

from . import _lib
from ._lib import lib, check
from .parsing import Read, ReadParser
from .graphs import (Hashtable, Hashgraph, Countgraph, SmallCountgraph, Nodegraph,
                     Counttable, SmallCounttable, Nodetable)
from .utils import get_n_primes_near_x, is_prime

__version__ = "3.0.0a3+mi355x"

FILETYPES = {  # src/khmer/_cpy_khmer.cc:281-291
    "COUNTING_HT": 1, "HASHBITS": 2, "TAGS": 3, "STOPTAGS": 4,
    "SUBSET": 5, "LABELSET": 6, "SMALLCOUNT": 7,
}

_buckets_per_byte = {  # khmer/__init__.py:86-92
    'qfcounttable': 1 / 1.26,
    'countgraph': 1,
    'smallcountgraph': 2,
    'nodegraph': 8,
}


def _check_ksize(ksize):
    if not -128 <= ksize <= 127:
        raise OverflowError("signed char is greater than maximum")
    if ksize > 32:
        raise ValueError("k-mer size must be <= 32")


def forward_hash(kmer, ksize):
    """Canonical 2-bit hash (src/khmer/_cpy_khmer.cc:63-91)."""
    _check_ksize(ksize)
    if len(kmer) != ksize:
        raise ValueError("k-mer size different from ksize")
    out = ctypes.c_uint64()
    check(lib.kh_hash_twobit(kmer.encode("latin-1"), ksize, None, None, ctypes.byref(out)))
    return out.value


def forward_hash_no_rc(kmer, ksize):
    """Forward-strand 2-bit hash (src/khmer/_cpy_khmer.cc:93-117)."""
    _check_ksize(ksize)
    if len(kmer) != ksize:
        raise ValueError("k-mer length must equal the k-size")
    out = ctypes.c_uint64()
    check(lib.kh_hash_twobit(kmer.encode("latin-1"), ksize, ctypes.byref(out), None, None))
    return out.value


def reverse_hash(hash_value, ksize):
    """2-bit hash -> k-mer (src/khmer/_cpy_khmer.cc:119-145)."""
    if not isinstance(hash_value, int) or isinstance(hash_value, bool):
        raise TypeError("Hash value must be an integer.")
    _check_ksize(ksize)
    buf = ctypes.create_string_buffer(ksize + 1)
    check(lib.kh_reverse_hash(hash_value, ksize, buf))
    return buf.value.decode()


def hash_murmur3(kmer):
    """Canonical MurmurHash3 k-mer hash (src/khmer/_cpy_khmer.cc:147-159)."""
    b = kmer.encode("latin-1")
    out = ctypes.c_uint64()
    check(lib.kh_hash_murmur(b, len(b), ctypes.byref(out), None))
    return out.value


def hash_no_rc_murmur3(kmer):
    """Forward MurmurHash3 (src/khmer/_cpy_khmer.cc:161-173)."""
    b = kmer.encode("latin-1")
    out = ctypes.c_uint64()
    check(lib.kh_hash_murmur(b, len(b), None, ctypes.byref(out)))
    return out.value


def reverse_complement(sequence):
    """IUPAC-aware reverse complement (src/khmer/_cpy_khmer.cc:175-190)."""
    b = sequence.encode("latin-1")
    buf = ctypes.create_string_buffer(len(b) + 1)
    check(lib.kh_reverse_complement(b, len(b), buf))
    return buf.raw[:len(b)].decode("latin-1")


def _file_header(filename, layout, what):
    """Header fields through the library's raw reader (kh_file_header); any
    failure is the reference's "corrupt" ValueError (khmer/__init__.py:95-178)."""
    out = (ctypes.c_int64 * 7)()
    try:
        check(lib.kh_file_header(str(filename).encode(), layout, out))
    except (OSError, ValueError, TypeError):
        raise ValueError("{} '{}' is corrupt ".format(what, filename))
    version, ht_type, bigcount, ksize, n_tables, occupied, size0 = list(out)
    return version, ht_type, (None if bigcount < 0 else bigcount), ksize, n_tables, occupied, size0


def extract_nodegraph_info(filename):
    """(ksize, table size rounded to 100, n tables, version, type, occupied)
    of a saved nodegraph."""
    version, ht_type, _, ksize, n_tables, occupied, size0 = _file_header(filename, 0, "Node graph")
    return ksize, round(size0, -2), n_tables, version, ht_type, occupied


CgInfo = namedtuple("CgInfo", ["ksize", "n_tables", "table_size", "use_bigcount", "version", "ht_type",
                               "n_occupied"])


def extract_countgraph_info(filename):
    """CgInfo of a saved countgraph (use_bigcount is None for SMALLCOUNT files)."""
    version, ht_type, bigcount, ksize, n_tables, occupied, size0 = _file_header(filename, 1, "Count graph file")
    return CgInfo(ksize, n_tables, round(size0, -2), bigcount, version, ht_type, occupied)


_TOO_SMALL = """**
** ERROR: the graph structure is too small for 
** this data set.  Increase data structure size
** with --max_memory_usage/-M.
**
** Do not use these results!!
**
** (estimated false positive rate of {fp:.3f}; max recommended {mx:.3f})
**"""


def calc_expected_collisions(graph, force=False, max_false_pos=.2):
    """False-positive rate expected from table-0 occupancy: (occupied / the
    smallest table) ** n_tables.  Above max_false_pos it prints the
    reference's warning block and exits 1 unless force."""
    sizes = graph.hashsizes()
    fp_all = (float(graph.n_occupied()) / min(sizes)) ** float(len(sizes))
    if fp_all > max_false_pos:
        print(_TOO_SMALL.format(fp=fp_all, mx=max_false_pos), file=sys.stderr)
        if not force:
            sys.exit(1)
    return fp_all


def device_count():
    """Number of visible HIP devices."""
    return _lib.device_count()
