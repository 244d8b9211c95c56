set -u
mkdir -p gpurun_out/r06/final
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > gpurun_out/r06/final/pytest_gpu.log 2>&1; rc=$?
tail -2 gpurun_out/r06/final/pytest_gpu.log
[ $rc -le 1 ] || { echo "pytest crashed rc=$rc"; exit 1; }
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r06/final/smoke.log 2>&1 || { echo "smoke failed"; tail gpurun_out/r06/final/smoke.log; exit 1; }
tail -1 gpurun_out/r06/final/smoke.log
bash tools/profile.sh > gpurun_out/r06/final/profile.log 2>&1 || { echo "profile failed"; tail -20 gpurun_out/r06/final/profile.log; exit 1; }
tail -3 gpurun_out/r06/final/profile.log
cp gpurun_out/op_stats.csv gpurun_out/traffic.json gpurun_out/mfma.json profiles/ && cp gpurun_out/op_stats.csv gpurun_out/traffic.json gpurun_out/mfma.json gpurun_out/piped_steps.json gpurun_out/bench_ops.json gpurun_out/r06/final/ && cp gpurun_out/prof/run_kernel_stats.csv gpurun_out/r06/final/kernel_stats.csv
timeout -k 10 700 python -u bench.py > gpurun_out/r06/final/bench_default.json 2> gpurun_out/r06/final/bench_default.err || { echo "bench failed"; tail gpurun_out/r06/final/bench_default.err; exit 1; }
echo bench done
