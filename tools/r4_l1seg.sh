#!/bin/bash
# Exact level 1 (k_scatter_l1) tail mode A/B at 1908 buckets (C4, C5):
# 2-record tails (one workgroup per CU) against none (the default above 1024
# buckets).  Usage: tools/r4_l1seg.sh <tag>
set -u
tag=${1:?tag}
cd "$(dirname "$0")/.."
out=gpurun_out/r4_$tag
mkdir -p "$out"
one() {
  name=$1; shift; envs=$1; shift
  env $envs timeout -k 10 300 python3 bench.py --steps 3 --cpu-reads 0 --no-unprofiled "$@" > "$out/$name.json" 2> "$out/$name.err" || { echo "bench $name failed"; tail -5 "$out/$name.err"; return 1; }
  python3 -c "
import json; d=json.loads(open('$out/$name.json').read().strip().splitlines()[-1]); r=d['roofline']
print('$name', round(d['ms_per_step'],1), 'ms/step', '%.3e'%d['value'], (d['check'].get('counters_match'), d['check'].get('tables_match')), {k:v for k,v in r['kernels_ms_per_step'].items() if v>1})"
}
one c4_seg0 KH_L1_SEG=0 --config C4 && one c4_seg2 KH_L1_SEG=2 --config C4 && one c3_seg0 KH_L1_SEG=0 --config C3
