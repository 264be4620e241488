#!/bin/bash
# C5 query: the table gathers as plain vs non-temporal loads -- the round-6
# A/B (profiles/r6/ab_runs/query_nt/): var/libqnt.so was built with
# -DKH_QUERY_NT when plain loads were the default; non-temporal is now the
# default and -DKH_QUERY_TEMPORAL builds the plain variant.  Timing twice
# each, then one FETCH_SIZE pass each.
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
out=gpurun_out/qnt; mkdir -p $out
tools/ab_libs.sh 2 "plain=" "nt=var/libqnt.so" -- --config C5 --query --steps 3 --no-unprofiled || exit 1
for v in plain nt; do
    lib=""; [ $v = nt ] && lib=var/libqnt.so
    KHMER_AMD_LIB=$lib timeout -s KILL 300 rocprofv3 --kernel-trace --pmc FETCH_SIZE -d $out/pmc_$v -o run --output-format csv -- \
        python3 bench.py --config C5 --query --steps 1 --warmup 0 --cpu-reads 0 --no-unprofiled > $out/pmc_$v.json 2> $out/pmc_$v.err || exit 1
done
python3 - <<'PY'
import csv, glob
for v in ("plain", "nt"):
    f = glob.glob("gpurun_out/qnt/pmc_%s/**/run_counter_collection.csv" % v, recursive=True)[0]
    tot, n = 0.0, 0
    for r in csv.DictReader(open(f)):
        if "median" in r["Kernel_Name"]:
            tot += float(r["Counter_Value"]); n += 1
    print(v, "k_median_fixed FETCH_SIZE raw KiB per launch (sum of dims/agents):", tot / max(1, len({1})), "rows", n)
PY
