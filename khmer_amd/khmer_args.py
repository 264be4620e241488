"""Command-line plumbing for the two drop-in scripts (scripts/load-into-counting.py,
scripts/load-graph.py).

Behaviour follows khmer/khmer_args.py and khmer/khmer_logger.py of the
reference: the same option names and defaults, the same table-sizing rules
and the same messages on stderr, so a pipeline that greps the reference
script's log or its `.info` files reads ours the same way.  Graph creation
goes to khmer_amd's device-backed classes; nothing here computes k-mers.
"""
import argparse
import math
import os
import sys
import textwrap
from collections import namedtuple

DEFAULT_K = 32                  # khmer_args.py:64-67
DEFAULT_N_TABLES = 4
DEFAULT_MAX_TABLESIZE = 1e6
DEFAULT_N_THREADS = 1

# ---------------------------------------------------------------------------
# stderr logging (khmer_logger.py:41-74): info is silenced by -q, warnings and
# errors are not.
_QUIET = False


def configure_logging(quiet):
    global _QUIET
    _QUIET = bool(quiet)


def _emit(message, kwargs):
    print(message.format(**kwargs) if kwargs else message, file=sys.stderr)


def log_info(message, **kwargs):
    if not _QUIET:
        _emit(message, kwargs)


def log_warn(message, **kwargs):
    _emit(message, kwargs)


def log_error(message, **kwargs):
    _emit(message, kwargs)


# ---------------------------------------------------------------------------
# sizing


def memory_setting(label):
    """Bytes from '1e9', '2000', '4G', '500m' ... (khmer_args.py:175-205)."""
    try:
        return float(label)
    except ValueError:
        pass
    scale = {"K": 1e3, "M": 1e6, "G": 1e9, "T": 1e12}.get(label[-1:].upper())
    try:
        if scale is None:
            raise ValueError
        return float(label[:-1]) * scale
    except ValueError:
        raise ValueError('cannot parse memory setting "{}"'.format(label))


SizeEstimate = namedtuple("result", ["num_htables", "htable_size", "mem_use", "fp_rate"])


def _bloom_fp(n_kmers, table_size, n_tables):
    return (1.0 - math.exp(-n_kmers / float(table_size))) ** n_tables


def estimate_optimal_with_K_and_M(num_kmers, mem_cap):
    """Tables/size for a memory cap: Z = ln2 * M / N (khmer_args.py:282-298)."""
    z = max(1, int(math.log(2) * (mem_cap / float(num_kmers))))
    h = int(mem_cap / z)
    return SizeEstimate(z, h, h * z, _bloom_fp(num_kmers, h, z))


def estimate_optimal_with_K_and_f(num_kmers, des_fp_rate):
    """Tables/size for a target false-positive rate: Z = log_0.5 f,
    H = -N / ln(1 - f^(1/Z)) (khmer_args.py:301-320)."""
    z = max(1, int(math.log(des_fp_rate, 0.5)))
    h = int(-num_kmers / math.log(1.0 - des_fp_rate ** (1.0 / z)))
    return SizeEstimate(z, h, h * z, _bloom_fp(num_kmers, h, z))


def optimal_size(num_kmers, mem_cap=None, fp_rate=None):
    if num_kmers is not None and mem_cap is not None and fp_rate is None:
        return estimate_optimal_with_K_and_M(num_kmers, mem_cap)
    if num_kmers is not None and mem_cap is None and fp_rate is not None:
        return estimate_optimal_with_K_and_f(num_kmers, fp_rate)
    raise TypeError("num_kmers and either mem_cap or fp_rate must be defined.")


def _buckets_per_byte():
    from . import _buckets_per_byte as bpb
    return bpb


def calculate_graphsize(args, graphtype, multiplier=1.0):
    """Per-table target size in buckets: -M spread over N tables at the graph
    type's buckets-per-byte, else -x (khmer_args.py:497-513)."""
    bpb = _buckets_per_byte()
    if graphtype not in bpb:
        raise ValueError("unknown graph type: " + graphtype)
    if args.max_memory_usage:
        return float(multiplier) * (bpb[graphtype] * args.max_memory_usage / args.n_tables)
    return args.max_tablesize


def _check_fp_rate(args, desired_max_fp):
    """Use -U (expected unique k-mers) to pick or vet the table size
    (khmer_args.py:375-430)."""
    if not args.unique_kmers:
        return args
    if args.fp_rate:
        log_info("*** INFO: Overriding default fp {def_fp} with new fp: {new_fp}",
                 def_fp=desired_max_fp, new_fp=args.fp_rate)
        desired_max_fp = args.fp_rate

    if args.max_memory_usage:
        res = estimate_optimal_with_K_and_M(args.unique_kmers, args.max_memory_usage)
        if res.fp_rate > desired_max_fp:
            print("\n*** ERROR: The given restrictions yield an estimate false positive rate of {0},"
                  "\n*** which is above the recommended false positive ceiling of {1}!"
                  .format(res.fp_rate, desired_max_fp), file=sys.stderr)
            if not args.force:
                print("NOTE: This can be overridden using the --force argument", file=sys.stderr)
                print("*** Aborting...!", file=sys.stderr)
                sys.exit(1)
        return args

    res = estimate_optimal_with_K_and_f(args.unique_kmers, desired_max_fp)
    if args.max_tablesize and args.max_tablesize < res.htable_size:
        log_warn("\n*** Warning: The given tablesize is too small!")
        log_warn("*** Recommended tablesize is: {tsize:5g} bytes", tsize=res.htable_size)
        log_warn("*** Current is: {tsize:5g} bytes", tsize=args.max_tablesize)
        res = estimate_optimal_with_K_and_M(args.unique_kmers, args.max_tablesize)
        log_warn("*** Estimated FP rate with current config is: {fp}\n", fp=res.fp_rate)
    else:
        args.max_memory_usage = max(1e6, res.mem_use)
        log_info("*** INFO: set memory ceiling automatically.")
        log_info("*** Ceiling is: {ceil:3g} bytes\n", ceil=float(args.max_memory_usage))
        args.max_mem = res.mem_use
    return args


def _check_table_shape(args, ksize):
    if hasattr(args, "force") and args.n_tables > 20:
        if not args.force:
            log_error("\n** ERROR: khmer only supports number of tables <= 20.\n")
            sys.exit(1)
        log_warn("\n*** Warning: Maximum recommended number of tables is 20, "
                 "discarded by force nonetheless!\n")
    if ksize > 32:
        log_error("\n** ERROR: khmer only supports k-mer sizes <= 32.\n")
        sys.exit(1)


def create_countgraph(args, ksize=None, multiplier=1.0, fp_rate=0.1):
    """Countgraph (or SmallCountgraph with --small-count) sized from the
    arguments (khmer_args.py:541-576)."""
    import khmer_amd
    args = _check_fp_rate(args, fp_rate)
    ksize = args.ksize if ksize is None else ksize
    _check_table_shape(args, ksize)
    if args.small_count:
        size = calculate_graphsize(args, "smallcountgraph", multiplier=multiplier)
        return khmer_amd.SmallCountgraph(ksize, size, args.n_tables)
    size = calculate_graphsize(args, "countgraph", multiplier=multiplier)
    graph = khmer_amd.Countgraph(ksize, size, args.n_tables)
    if hasattr(args, "bigcount"):
        graph.set_use_bigcount(args.bigcount)
    return graph


def create_nodegraph(args, ksize=None, multiplier=1.0, fp_rate=0.01):
    """Nodegraph sized from the arguments (khmer_args.py:516-538)."""
    import khmer_amd
    args = _check_fp_rate(args, fp_rate)
    ksize = args.ksize if ksize is None else ksize
    _check_table_shape(args, ksize)
    size = calculate_graphsize(args, "nodegraph", multiplier)
    return khmer_amd.Nodegraph(ksize, size, args.n_tables)


def report_on_config(args, graphtype="countgraph"):
    """Print the table parameters and memory estimate (khmer_args.py:587-617)."""
    if getattr(args, "quiet", None):
        configure_logging(args.quiet)
    bpb = _buckets_per_byte()
    if graphtype not in bpb:
        raise ValueError("unknown graph type: " + graphtype)
    size = calculate_graphsize(args, graphtype)
    maxmem = args.n_tables * size / bpb[graphtype]
    log_info("\nPARAMETERS:")
    log_info(" - kmer size =     {ksize} \t\t(-k)", ksize=args.ksize)
    log_info(" - n tables =      {ntables} \t\t(-N)", ntables=args.n_tables)
    log_info(" - max tablesize = {tsize:5.2g} \t(-x)", tsize=size)
    log_info("Estimated memory usage is {mem:.1f} Gb ({bytes:.2g} bytes = {ntables} bytes x "
             "{tsize:5.2g} entries / {div:d} entries per byte)", bytes=maxmem, mem=maxmem / 1e9,
             div=bpb[graphtype], ntables=args.n_tables, tsize=size)
    log_info("-" * 8)
    if size == DEFAULT_MAX_TABLESIZE and not getattr(args, "loadgraph", None):
        log_warn("\n** WARNING: tablesize is default!\n"
                 "** You probably want to increase this with -M/--max-memory-usage!\n"
                 "** Please read the docs!\n")


# ---------------------------------------------------------------------------
# argument parsers


class _VersionAction(argparse.Action):
    def __init__(self, option_strings, version=None, dest=argparse.SUPPRESS,
                 default=argparse.SUPPRESS, help="show program's version number and exit"):
        super(_VersionAction, self).__init__(option_strings=option_strings, dest=dest,
                                             default=default, nargs=0, help=help)
        self.version = version

    def __call__(self, parser, namespace, values, option_string=None):
        print(self.version, file=sys.stderr)   # the reference prints the version to stderr
        parser.exit()


class KhmerArgumentParser(argparse.ArgumentParser):
    """ArgumentParser with the reference's --version/-h and the startup banner
    (khmer_args.py:125-155)."""

    def __init__(self, citations=None, **kwargs):
        kwargs.setdefault("formatter_class", argparse.RawDescriptionHelpFormatter)
        super(KhmerArgumentParser, self).__init__(add_help=False, **kwargs)
        from . import __version__
        self.add_argument("--version", action=_VersionAction, version="khmer {}".format(__version__))
        self.add_argument("-h", "--help", action="help", default=argparse.SUPPRESS,
                          help="show this help message and exit")

    def parse_args(self, args=None, namespace=None):
        ns = super(KhmerArgumentParser, self).parse_args(args=args, namespace=namespace)
        if not getattr(ns, "quiet", False):
            from . import __version__
            log_info("\n|| This is the script {name} in khmer.\n"
                     "|| You are running khmer version {version}\n||", name=self.prog,
                     version=__version__)
        return ns


def build_graph_args(descr=None, epilog=None, parser=None, citations=None):
    """-k, -N, -U, --fp-rate and the exclusive -x / -M (khmer_args.py:433-469)."""
    if parser is None:
        parser = KhmerArgumentParser(description=descr, epilog=epilog, citations=citations)
    parser.add_argument("-k", "--ksize", type=int, default=DEFAULT_K, help="k-mer size to use")
    parser.add_argument("--n_tables", "-N", type=int, default=DEFAULT_N_TABLES,
                        help="number of tables to use in k-mer countgraph")
    parser.add_argument("-U", "--unique-kmers", type=float, default=0,
                        help="approximate number of unique kmers in the input set")
    parser.add_argument("--fp-rate", type=float, default=None,
                        help="Override the automatic FP rate setting for the current script")
    group = parser.add_mutually_exclusive_group()
    group.add_argument("--max-tablesize", "-x", type=float, default=DEFAULT_MAX_TABLESIZE,
                       help="upper bound on tablesize to use; overrides --max-memory-usage/-M")
    group.add_argument("-M", "--max-memory-usage", type=memory_setting,
                       help="maximum amount of memory to use for data structure")
    return parser


def build_counting_args(descr=None, epilog=None, citations=None):
    parser = build_graph_args(descr=descr, epilog=epilog, citations=citations)
    parser.add_argument("--small-count", default=False, action="store_true",
                        help="Reduce memory usage by using a smaller counter for individual kmers.")
    return parser


def build_nodegraph_args(descr=None, epilog=None, parser=None, citations=None):
    return build_graph_args(descr=descr, epilog=epilog, parser=parser, citations=citations)


def add_threading_args(parser):
    parser.add_argument("-T", "--threads", default=DEFAULT_N_THREADS, type=int,
                        help="Accepted for compatibility; the device consumes each file "
                             "with all of its CUs whatever the value.")


def dedent(text):
    return textwrap.dedent(text)


# ---------------------------------------------------------------------------
# file checks (khmer/kfile.py:46-185)


def check_input_files(file_path, force):
    """Exit when an input is missing or empty, unless --force."""
    if file_path == "-":
        return
    try:
        st = os.stat(file_path)
    except OSError:
        print("ERROR: Input file %s does not exist" % file_path, file=sys.stderr)
        if not force:
            print("NOTE: This can be overridden using the --force argument", file=sys.stderr)
            print("Exiting", file=sys.stderr)
            sys.exit(1)
        return
    import stat as _stat
    if _stat.S_ISFIFO(st.st_mode) or _stat.S_ISBLK(st.st_mode) or _stat.S_ISCHR(st.st_mode):
        return
    if st.st_size == 0:
        print("ERROR: Input file %s is empty; exiting." % file_path, file=sys.stderr)
        if not force:
            print("NOTE: This can be overridden using the --force argument", file=sys.stderr)
            sys.exit(1)


def check_file_writable(file_path):
    """Exit 1 when file_path cannot be opened for append."""
    import errno
    try:
        fh = open(file_path, "a")
    except IOError as error:
        if error.errno == errno.EACCES:
            print("ERROR: File %s does not have write permission; exiting" % file_path,
                  file=sys.stderr)
            sys.exit(1)
        print("ERROR: " + error.strerror, file=sys.stderr)
    else:
        fh.close()


def check_space_for_graph(outfile_name, hash_size, force, _testhook_free_space=None):
    """Exit when the saved tables (hash_size bytes) will not fit on disk."""
    st = os.statvfs(os.path.dirname(os.path.realpath(outfile_name)))
    free = st.f_frsize * st.f_bavail if _testhook_free_space is None else _testhook_free_space
    short = hash_size - free
    if short > 0:
        msg = ("Not enough free space on disk for saved graph files;"
               "\n       Need at least {:.1f} GB more."
               "\n       Table size: {:.1f} GB"
               "\n       Free space: {:.1f} GB").format(short / 1e9, hash_size / 1e9, free / 1e9)
        if force:
            print("WARNING:", msg, file=sys.stderr)
        else:
            raise SystemExit("ERROR: " + msg +
                             "\nNOTE: This can be overridden using the --force argument")
