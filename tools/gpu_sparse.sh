#!/bin/bash
# Record-driven apply: its parity tests (and the near-prime / schedule ones,
# whose sparse regions take it), then the C4 / C5 / C5M / C2 bench lines with
# their fixture checks.  Usage: tools/gpu_sparse.sh <tag>
set -o pipefail
tag=${1:?tag}
cd "$(dirname "$0")/.."
mkdir -p gpurun_out/$tag
timeout -k 10 700 python -u -m pytest tests/test_gpu_sparse_apply.py tests/test_gpu_nearprime.py tests/test_gpu_schedule.py tests/test_gpu_shard.py -k "delta or sparse or schedule or nearprime or apply" -x -v --timeout 170 --timeout-method thread > gpurun_out/$tag/t.log 2>&1 || { echo "tests failed"; tail -40 gpurun_out/$tag/t.log; exit 1; }
tail -3 gpurun_out/$tag/t.log
for cfg in C4 C5 C5M C2; do
    timeout -k 10 400 python -u bench.py --config $cfg --steps 3 --warmup 1 --cpu-reads 0 > gpurun_out/$tag/bench_$cfg.json 2> gpurun_out/$tag/bench_$cfg.err || { echo "bench $cfg failed"; tail -20 gpurun_out/$tag/bench_$cfg.err; exit 1; }
    python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], round(d['ms_per_step'],1), sorted(d['roofline']['kernels_ms_per_step'].items(), key=lambda x:-x[1])[:6], d['check'])" gpurun_out/$tag/bench_$cfg.json $cfg
done
