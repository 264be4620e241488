"""khmer_amd: khmer's k-mer counting path (Countgraph / Nodegraph /
SmallCountgraph and the Murmur *table family) on AMD Instinct MI355X.

Drop-in for the `khmer` names that scripts/load-into-counting.py and
scripts/load-graph.py use (khmer/__init__.py:36-215); `import khmer_amd as
khmer` in a script is the whole integration.  Tables live in HBM and are
updated by hand-written HIP kernels in libkhmer_hip.so.
"""
import ctypes
from collections import namedtuple
from struct import pack, unpack
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


def extract_nodegraph_info(filename):
    """(ksize, table size, n tables, version, type, occupied) of a nodegraph
    file (khmer/__init__.py:95-136)."""
    uint_size = len(pack('I', 0))
    uchar_size = len(pack('B', 0))
    ulonglong_size = len(pack('Q', 0))
    try:
        with open(filename, 'rb') as nodegraph:
            signature, = unpack('4s', nodegraph.read(4))
            version, = unpack('B', nodegraph.read(1))
            ht_type, = unpack('B', nodegraph.read(1))
            ksize, = unpack('I', nodegraph.read(uint_size))
            n_tables, = unpack('B', nodegraph.read(uchar_size))
            occupied, = unpack('Q', nodegraph.read(ulonglong_size))
            table_size, = unpack('Q', nodegraph.read(ulonglong_size))
        if signature != b"OXLI":
            raise ValueError("Node graph '{}' is missing file type "
                             "signature".format(filename) + str(signature))
    except:  # noqa: E722  (reference behaviour: any failure -> corrupt)
        raise ValueError("Node graph '{}' is corrupt ".format(filename))
    return ksize, round(table_size, -2), n_tables, version, ht_type, occupied


def extract_countgraph_info(filename):
    """CgInfo of a countgraph file (khmer/__init__.py:139-178)."""
    CgInfo = namedtuple("CgInfo", ['ksize', 'n_tables', 'table_size', 'use_bigcount',
                                   'version', 'ht_type', 'n_occupied'])
    uint_size = len(pack('I', 0))
    ulonglong_size = len(pack('Q', 0))
    try:
        with open(filename, 'rb') as countgraph:
            signature, = unpack('4s', countgraph.read(4))
            version, = unpack('B', countgraph.read(1))
            ht_type, = unpack('B', countgraph.read(1))
            if ht_type != FILETYPES['SMALLCOUNT']:
                use_bigcount, = unpack('B', countgraph.read(1))
            else:
                use_bigcount = None
            ksize, = unpack('I', countgraph.read(uint_size))
            n_tables, = unpack('B', countgraph.read(1))
            occupied, = unpack('Q', countgraph.read(ulonglong_size))
            table_size, = unpack('Q', countgraph.read(ulonglong_size))
        if signature != b'OXLI':
            raise ValueError("Count graph file '{}' is missing file type "
                             "signature. ".format(filename) + str(signature))
    except:  # noqa: E722
        raise ValueError("Count graph file '{}' is corrupt ".format(filename))
    return CgInfo(ksize, n_tables, round(table_size, -2), use_bigcount, version, ht_type, occupied)


def calc_expected_collisions(graph, force=False, max_false_pos=.2):
    """Expected false-positive rate from table-0 occupancy
    (khmer/__init__.py:181-215)."""
    sizes = graph.hashsizes()
    n_ht = float(len(sizes))
    occupancy = float(graph.n_occupied())
    min_size = min(sizes)
    fp_one = occupancy / min_size
    fp_all = fp_one ** n_ht
    if fp_all > max_false_pos:
        print("**", file=sys.stderr)
        print("** ERROR: the graph structure is too small for ", file=sys.stderr)
        print("** this data set.  Increase data structure size", file=sys.stderr)
        print("** with --max_memory_usage/-M.", file=sys.stderr)
        print("**", file=sys.stderr)
        print("** Do not use these results!!", file=sys.stderr)
        print("**", file=sys.stderr)
        print("** (estimated false positive rate of %.3f;" % fp_all, file=sys.stderr, end=' ')
        print("max recommended %.3f)" % max_false_pos, file=sys.stderr)
        print("**", file=sys.stderr)
        if not force:
            sys.exit(1)
    return fp_all


def device_count():
    """Number of visible HIP devices."""
    return _lib.device_count()
