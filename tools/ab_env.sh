#!/bin/bash
# A/B timing of development knobs on the GPU box: for each of <runs> rounds,
# one bench.py run per "tag=VAR=v,VAR=v" (empty after '=': no knob) with the
# library <lib> (a `make DEV=1` build: the knobs are read only there).
# Prints ms/step, the big kernels and the parity check per run.
# Usage: tools/ab_env.sh <runs> <lib> "<tag>=<VAR=v,...>" ... -- [bench args...]
set -u
runs=$1; lib=$2; shift 2
cfgs=()
while [ $# -gt 0 ] && [ "$1" != "--" ]; do cfgs+=("$1"); shift; done
[ "${1:-}" = "--" ] && shift
cd "$(dirname "$0")/.."
out=gpurun_out/abenv; mkdir -p $out
for r in $(seq 1 "$runs"); do
    for c in "${cfgs[@]}"; do
        tag=${c%%=*}; kv=${c#*=}
        envs=()
        IFS=',' read -ra parts <<< "$kv"
        for p in "${parts[@]}"; do [ -n "$p" ] && envs+=("$p"); done
        env "${envs[@]}" KHMER_AMD_LIB="$lib" timeout -k 10 400 python3 bench.py --cpu-reads 0 "$@" \
            > $out/$tag$r.json 2> $out/$tag$r.err || exit $?
        python3 - "$tag" $out/$tag$r.json <<'PY'
import json, sys
d = json.load(open(sys.argv[2]))
k = d["roofline"]["kernels_ms_per_step"]
big = sorted(k.items(), key=lambda kv: -kv[1])[:6]
c = d.get("check", {})
print("%-8s %.1f ms/step" % (sys.argv[1], d["ms_per_step"]), " ".join("%s=%.1f" % kv for kv in big),
      "tables_match=%s counters_match=%s" % (c.get("tables_match"), c.get("counters_match")), flush=True)
PY
    done
done
