"""The two drop-in scripts on the hot path, as importable functions.

`load_into_counting(argv)` is scripts/load-into-counting.py
(reference scripts/load-into-counting.py:60-218) and `load_graph(argv)` is
scripts/load-graph.py (reference scripts/load-graph.py + oxli/build_graph.py:
40-123).  Options, stderr messages, the saved table, the `.info` file, the
`.info.json` / `.info.tsv` summaries and the `.tagset` file match the
reference's.  Each input file is consumed as the reference does it: `-T`
Python threads all call consume_seqfile[_and_tag] on one shared ReadParser
(scripts/load-into-counting.py:143-158, oxli/functions.py:56-66).  The first
call drains the parser into the device pipeline; the others find it drained
and return their (empty) share, so the tables and counters do not depend on
-T.  One deliberate difference: an exception in a consuming thread is
re-raised in the main thread after the join (the reference's thread prints
it and the script carries on).  The tests call these functions in-process;
the files under scripts/ are two-line wrappers.
"""
import json
import os
import sys
import threading

from . import khmer_args as KA


def consume_threads(eat, parser, num_threads):
    """`num_threads` threads calling eat(parser) on one shared parser; their
    (reads, k-mers) shares, and the first exception re-raised after the join."""
    shares, errors = [], []

    def run():
        try:
            shares.append(eat(parser))
        except BaseException as e:   # re-raised in the caller below
            errors.append(e)

    threads = [threading.Thread(target=run) for _ in range(max(1, int(num_threads)))]
    for t in threads:
        t.start()
    for t in threads:
        t.join()
    if errors:
        raise errors[0]
    return shares


# ---------------------------------------------------------------------------
# load-into-counting.py

_LIC_EPILOG = """\
    Note: with -b/--no-bigcount the output will be the exact size of the
    k-mer countgraph and this script will use a constant amount of memory.
    In exchange k-mer counts will stop at 255.

    Example:

        load-into-counting.py -k 20 -x 5e7 out data/100k-filtered.fa
    """


def load_into_counting_parser():
    parser = KA.build_counting_args("Build a k-mer countgraph from the given sequences.",
                                    epilog=KA.dedent(_LIC_EPILOG))
    parser.prog = "load-into-counting.py"
    KA.add_threading_args(parser)
    parser.add_argument("output_countgraph_filename",
                        help="The name of the file to write the k-mer countgraph to.")
    parser.add_argument("input_sequence_filename", nargs="+",
                        help="The names of one or more FAST[AQ] input sequence files.")
    parser.add_argument("-b", "--no-bigcount", dest="bigcount", default=True,
                        action="store_false",
                        help="Turn bigcount off, limiting counts to 255.")
    parser.add_argument("-s", "--summary-info", type=str, default=None, metavar="FORMAT",
                        choices=["json", "tsv"],
                        help="What format should the machine readable run summary be in? "
                             "(`json` or `tsv`, disabled by default)")
    parser.add_argument("-f", "--force", default=False, action="store_true",
                        help="Overwrite output file if it exists")
    parser.add_argument("-q", "--quiet", dest="quiet", default=False, action="store_true")
    return parser


def _write_summary(fmt, path, base, fp_rate, n_kmers, n_reads, filenames):
    with open(path, "w") as fh:
        if fmt == "json":
            json.dump({"ht_name": os.path.basename(base), "fpr": fp_rate, "num_kmers": n_kmers,
                       "files": filenames, "mrinfo_version": "0.2.0", "num_reads": n_reads}, fh)
            fh.write("\n")
        else:
            fh.write("ht_name\tfpr\tnum_kmers\tnum_reads\tfiles\n")
            fh.write("\t".join([os.path.basename(base), "{:1.3f}".format(fp_rate), str(n_kmers),
                                str(n_reads), ";".join(filenames)]) + "\n")


def load_into_counting(argv=None):
    import khmer_amd
    args = load_into_counting_parser().parse_args(argv)
    KA.configure_logging(args.quiet)
    KA.report_on_config(args)

    base = args.output_countgraph_filename
    filenames = args.input_sequence_filename
    for name in filenames:
        KA.check_input_files(name, args.force)
    KA.check_space_for_graph(base, KA.calculate_graphsize(args, "countgraph"), args.force)
    info_filename = base + ".info"
    KA.check_file_writable(base)
    KA.check_file_writable(info_filename)

    KA.log_info("Saving k-mer countgraph to {base}", base=base)
    KA.log_info("Loading kmers from sequences in {filenames}", filenames=repr(filenames))
    with open(info_filename, "w") as fh:
        print("khmer version:", khmer_amd.__version__, file=fh)

    KA.log_info("making countgraph")
    countgraph = KA.create_countgraph(args)

    total_reads = 0
    for index, filename in enumerate(filenames):
        parser = khmer_amd.ReadParser(filename)
        KA.log_info("consuming input {input}", input=filename)
        consume_threads(countgraph.consume_seqfile, parser, args.threads)
        if index > 0 and index % 10 == 0:     # periodic checkpoint, as the reference
            KA.check_space_for_graph(base, KA.calculate_graphsize(args, "countgraph"), args.force)
            KA.log_info("mid-save {base}", base=base)
            countgraph.save(base)
        with open(info_filename, "a") as fh:
            print("through", filename, file=fh)
        total_reads += parser.num_reads
        parser.close()

    n_kmers = countgraph.n_unique_kmers()
    KA.log_info("Total number of unique k-mers: {nk}", nk=n_kmers)
    with open(info_filename, "a") as fh:
        print("Total number of unique k-mers:", n_kmers, file=fh)

    KA.log_info("saving {base}", base=base)
    countgraph.save(base)

    fp_rate = khmer_amd.calc_expected_collisions(countgraph, args.force, max_false_pos=.2)
    with open(info_filename, "a") as fh:
        print("fp rate estimated to be %1.3f\n" % fp_rate, file=fh)

    if args.summary_info:
        fmt = args.summary_info.lower()
        mr_file = base + ".info." + fmt
        KA.log_info("Writing summmary info to {mr_file}", mr_file=mr_file)
        _write_summary(fmt, mr_file, base, fp_rate, n_kmers, total_reads, filenames)

    KA.log_info("fp rate estimated to be {fpr:1.3f}", fpr=fp_rate)
    KA.log_info("DONE.")
    KA.log_info("wrote to: {filename}", filename=info_filename)
    return 0


# ---------------------------------------------------------------------------
# load-graph.py


def load_graph_parser():
    parser = KA.build_nodegraph_args(
        descr="Load sequences into the compressible graph format plus optional tagset.")
    parser.prog = "load-graph.py"
    KA.add_threading_args(parser)
    parser.add_argument("--no-build-tagset", "-n", default=False, action="store_true",
                        dest="no_build_tagset",
                        help="Do NOT construct tagset while loading sequences")
    parser.add_argument("output_filename", metavar="output_nodegraph_filename",
                        help="output k-mer nodegraph filename.")
    parser.add_argument("input_filenames", metavar="input_sequence_filename", nargs="+",
                        help="input FAST[AQ] sequence filename")
    parser.add_argument("-f", "--force", default=False, action="store_true",
                        help="Overwrite output file if it exists")
    return parser


def build_graph(filenames, graph, num_threads=1, tags=False):
    """Consume every file into graph, tagging when asked
    (oxli/functions.py:42-66)."""
    import khmer_amd
    eat = graph.consume_seqfile_and_tag if tags else graph.consume_seqfile
    for name in filenames:
        parser = khmer_amd.ReadParser(name)
        consume_threads(eat, parser, num_threads)
        parser.close()


def load_graph(argv=None):
    import khmer_amd
    args = load_graph_parser().parse_args(argv)
    KA.report_on_config(args, graphtype="nodegraph")
    base = args.output_filename
    filenames = args.input_filenames
    for name in filenames:
        KA.check_input_files(name, args.force)
    size = KA.calculate_graphsize(args, "nodegraph")
    KA.check_space_for_graph(base, args.n_tables * size / khmer_amd._buckets_per_byte["nodegraph"],
                             args.force)

    err = sys.stderr
    print("Saving k-mer nodegraph to %s" % base, file=err)
    print("Loading kmers from sequences in %s" % repr(filenames), file=err)
    if args.no_build_tagset:
        print("We WILL NOT build the tagset.", file=err)
    else:
        print("We WILL build the tagset (for partitioning/traversal).", file=err)

    print("making nodegraph", file=err)
    nodegraph = KA.create_nodegraph(args)
    build_graph(filenames, nodegraph, args.threads, not args.no_build_tagset)

    n_unique = nodegraph.n_unique_kmers()
    print("Total number of unique k-mers: {0}".format(n_unique), file=err)
    print("saving k-mer nodegraph in", base, file=err)
    nodegraph.save(base)
    if not args.no_build_tagset:
        print("saving tagset in", base + ".tagset", file=err)
        nodegraph.save_tagset(base + ".tagset")

    with open(base + ".info", "w") as info:
        info.write("%d unique k-mers" % n_unique)
        fp_rate = khmer_amd.calc_expected_collisions(nodegraph, args.force, max_false_pos=.15)
        print("false positive rate estimated to be %1.3f" % fp_rate, file=err)
        print("\nfalse positive rate estimated to be %1.3f" % fp_rate, file=info)

    print("wrote to " + base + ".info and " + base, file=err)
    if not args.no_build_tagset:
        print("and " + base + ".tagset", file=err)
    return 0


def run(fn):
    """Entry used by scripts/*.py: exit with fn's status."""
    sys.exit(fn())
