#!/bin/bash
# Timing of bench.py under several env settings (one run each, in order).
# Usage: tools/ab_multi.sh "<env1>" "<env2>" ... -- [bench args]
set -u
envs=()
while [ $# -gt 0 ] && [ "$1" != "--" ]; do envs+=("$1"); shift; done
[ $# -gt 0 ] && shift
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
i=0
for e in "${envs[@]}"; do
    i=$((i+1))
    env $e timeout -k 10 240 python3 bench.py --cpu-reads 0 "$@" > gpurun_out/abm_$i.json 2> gpurun_out/abm_$i.err || exit $?
    python3 - "$e" gpurun_out/abm_$i.json <<'PY'
import json, sys
d = json.load(open(sys.argv[2]))
k = d["roofline"]["kernels_ms_per_step"]
big = sorted(k.items(), key=lambda kv: -kv[1])[:6]
print("%-40s" % sys.argv[1], "%.1f ms/step" % d["ms_per_step"], " ".join("%s=%.1f" % kv for kv in big), flush=True)
PY
done
