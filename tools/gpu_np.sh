#!/bin/bash
# Near-prime parity tests, then the C4 (three-level) and C2 bench lines, each
# checked against its oracle fixture.  Usage: tools/gpu_np.sh <tag>
set -o pipefail
tag=${1:?tag}
cd "$(dirname "$0")/.."
mkdir -p gpurun_out/$tag
timeout -k 10 700 python -u -m pytest tests/test_gpu_nearprime.py -x -v --timeout 170 --timeout-method thread > gpurun_out/$tag/t_np.log 2>&1 || { echo "np tests failed"; tail -40 gpurun_out/$tag/t_np.log; exit 1; }
tail -3 gpurun_out/$tag/t_np.log
for cfg in C4 C2; do
    timeout -k 10 400 python -u bench.py --config $cfg --steps 3 --warmup 1 --cpu-reads 0 > gpurun_out/$tag/bench_$cfg.json 2> gpurun_out/$tag/bench_$cfg.err || { echo "bench $cfg failed"; tail -20 gpurun_out/$tag/bench_$cfg.err; exit 1; }
    python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], round(d['ms_per_step'],1), d['roofline']['kernels_ms_per_step'], d['check'])" gpurun_out/$tag/bench_$cfg.json $cfg
done
