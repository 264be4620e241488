#!/bin/bash
# C4 (one GPU) A/B: 2^13-bin regions (KH_S0=13: 512-thread apply, two
# workgroups per CU) and the per-region winner lists (KH_WINNERS=1) against
# the default.  Usage: tools/r4_c4ab.sh <tag>
set -u
tag=${1:?tag}
cd "$(dirname "$0")/.."
out=gpurun_out/r4_$tag
mkdir -p "$out"
one() {
  name=$1; shift
  env "$@" timeout -k 10 300 python3 bench.py --config C4 --steps 2 --cpu-reads 0 --no-unprofiled > "$out/$name.json" 2> "$out/$name.err" || { echo "bench $name failed"; tail -5 "$out/$name.err"; return 1; }
  python3 -c "
import json; d=json.loads(open('$out/$name.json').read().strip().splitlines()[-1]); r=d['roofline']
print('$name', round(d['ms_per_step'],1), 'ms/step', '%.3e'%d['value'], {k:v for k,v in r['kernels_ms_per_step'].items() if v>1})"
}
one c4_base KH_S0=14 && one c4_s013 KH_S0=13 && one c4_lists KH_WINNERS=1
