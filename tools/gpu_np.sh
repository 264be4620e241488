set -o pipefail
mkdir -p gpurun_out/r6
timeout -k 10 700 python -u -m pytest tests/test_gpu_nearprime.py -x -v --timeout 170 --timeout-method thread > gpurun_out/r6/t_np.log 2>&1 || { echo "np tests failed"; tail -40 gpurun_out/r6/t_np.log; exit 1; }
tail -5 gpurun_out/r6/t_np.log
timeout -k 10 300 python -u bench.py --steps 5 --warmup 1 --cpu-reads 0 > gpurun_out/r6/bench_np.json 2> gpurun_out/r6/bench_np.err || { echo bench failed; tail -20 gpurun_out/r6/bench_np.err; exit 1; }
cat gpurun_out/r6/bench_np.json
