#!/bin/bash
# A/B/C timing of library builds on the GPU box: for each of <runs> rounds,
# one bench.py run per "tag=KHMER_AMD_LIB path" (empty path: the product
# library); prints ms/step, the big kernels and the parity check per run.
# Usage: tools/ab_libs.sh <runs> "<tag>=<lib>" ... -- [bench args...]
set -u
runs=$1; shift
cfgs=()
while [ $# -gt 0 ] && [ "$1" != "--" ]; do cfgs+=("$1"); shift; done
[ "${1:-}" = "--" ] && shift
cd "$(dirname "$0")/.."
out=gpurun_out/ab; mkdir -p $out
for r in $(seq 1 "$runs"); do
    for c in "${cfgs[@]}"; do
        tag=${c%%=*}; lib=${c#*=}
        if [ -n "$lib" ]; then export KHMER_AMD_LIB=$lib; else unset KHMER_AMD_LIB; fi
        timeout -k 10 300 python3 bench.py --cpu-reads 0 "$@" > $out/$tag$r.json 2> $out/$tag$r.err || exit $?
        python3 - "$tag" $out/$tag$r.json <<'PY'
import json, sys
d = json.load(open(sys.argv[2]))
k = d["roofline"]["kernels_ms_per_step"]
big = sorted(k.items(), key=lambda kv: -kv[1])[:5]
c = d.get("check", {})
print("%-6s %.1f ms/step" % (sys.argv[1], d["ms_per_step"]), " ".join("%s=%.1f" % kv for kv in big),
      "tables_match=%s counters_match=%s" % (c.get("tables_match"), c.get("counters_match")), flush=True)
PY
    done
done
