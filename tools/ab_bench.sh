#!/bin/bash
# A/B timing on the GPU box: alternating runs of bench.py under two env
# settings; prints one summary line per run (ms/step and the big kernels).
# Usage: tools/ab_bench.sh <runs> "<envA>" "<envB>" [bench args...]
set -u
runs=$1; ea=$2; eb=$3; shift 3
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
for r in $(seq 1 "$runs"); do
    for tag in A B; do
        if [ $tag = A ]; then e=$ea; else e=$eb; fi
        env $e timeout -k 10 240 python3 bench.py --cpu-reads 0 "$@" > gpurun_out/ab_$tag$r.json 2> gpurun_out/ab_$tag$r.err || exit $?
        python3 - "$tag" "$e" gpurun_out/ab_$tag$r.json <<'PY'
import json, sys
d = json.load(open(sys.argv[3]))
k = d["roofline"]["kernels_ms_per_step"]
big = sorted(k.items(), key=lambda kv: -kv[1])[:6]
print(sys.argv[1], "%-22s" % sys.argv[2], "%.1f ms/step" % d["ms_per_step"], " ".join("%s=%.1f" % kv for kv in big), flush=True)
PY
    done
done
