#!/bin/bash
# Secondary bench lines on one GPU (each its own process, one JSON line each):
# C2 genomic stream, C3, C4 (one-GPU anchor), C5 (2-bit nibble), C5M
# (SmallCounttable k=51, Murmur), C5 and C5M get_median_count query, C5M
# at BASELINE configs[4]'s 500M reads, and the query on the genomic nibble
# fixtures' streams (c5_genomic / c5m_genomic: medians 1..15, digest-checked).
# Usage: tools/bench_modes.sh <tag>   -> gpurun_out/modes_<tag>/*.json
set -u
tag=${1:?tag}
cd "$(dirname "$0")/.."
out=gpurun_out/modes_$tag
mkdir -p "$out"
run() {
    name=$1; shift
    timeout -k 10 400 python3 bench.py "$@" > "$out/$name.json" 2> "$out/$name.err" || { echo "FAIL $name rc=$?"; tail -3 "$out/$name.err"; return 1; }
    python3 - "$name" "$out/$name.json" <<'PY'
import json, sys
d = json.loads(open(sys.argv[2]).read().strip().splitlines()[-1])
r = d["roofline"] or {}
print("%-10s %.3e %s  %.1f ms/step (unprofiled %s)  frac %.4f  %s  %s" % (sys.argv[1], d["value"], d["unit"], d["ms_per_step"], d.get("ms_per_step_unprofiled") and "%.1f" % d["ms_per_step_unprofiled"], r.get("frac", 0), d["cpu_baseline"] and "%.3e" % d["cpu_baseline"]["value"], d.get("check")), flush=True)
PY
}
run c2_genomic --config C2 --genome 1e8 --steps 3 --cpu-reads 300000 &&
run c3 --config C3 --steps 3 --cpu-reads 300000 &&
run c4 --config C4 --steps 2 --cpu-reads 200000 &&
run c5 --config C5 --steps 2 --cpu-reads 200000 &&
run c5m --config C5M --steps 2 --cpu-reads 100000 &&
run c5_query --config C5 --query --steps 3 --cpu-reads 100000 &&
run c5m_query --config C5M --query --steps 3 --cpu-reads 50000 &&
run c5m_500m --config C5M --reads 500000000 --steps 1 --warmup 1 --cpu-reads 0 --batch-kmers 2147483648 &&
run c5g_query --config C5 --query --genome 5e7 --reads 4000000 --steps 3 --cpu-reads 50000 &&
run c5mg_query --config C5M --query --genome 1e7 --reads 1000000 --steps 3 --cpu-reads 20000
