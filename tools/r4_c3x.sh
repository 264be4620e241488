#!/bin/bash
# C3 (Nodegraph 4 x 4e9, 956 level-1 buckets): the one-launch k_scatter_l1f
# (one workgroup per CU at this LDS size) against the exact two-pass level 1
# (KH_L1_EXACT=1).  Usage: tools/r4_c3x.sh <tag>
set -u
tag=${1:?tag}
cd "$(dirname "$0")/.."
out=gpurun_out/r4_$tag
mkdir -p "$out"
one() {
  name=$1; cfg=$2; shift 2
  env "$@" timeout -k 10 300 python3 bench.py --config $cfg --steps 3 --cpu-reads 0 --no-unprofiled > "$out/$name.json" 2> "$out/$name.err" || { echo "bench $name failed"; tail -5 "$out/$name.err"; return 1; }
  python3 -c "
import json; d=json.loads(open('$out/$name.json').read().strip().splitlines()[-1]); r=d['roofline']
print('$name', round(d['ms_per_step'],1), 'ms/step', '%.3e'%d['value'], (d['check'].get('counters_match'), d['check'].get('tables_match')), {k:v for k,v in r['kernels_ms_per_step'].items() if v>1})"
}
one c3_l1f C3 KH_L1_EXACT=0 && one c3_exact C3 KH_L1_EXACT=1
