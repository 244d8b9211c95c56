set -u
mkdir -p gpurun_out/r06/final3
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > gpurun_out/r06/final3/pytest_gpu.log 2>&1; rc=$?
tail -2 gpurun_out/r06/final3/pytest_gpu.log
[ $rc -le 1 ] || { echo "pytest crashed rc=$rc"; exit 1; }
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r06/final3/smoke.log 2>&1 || { echo "smoke failed"; tail gpurun_out/r06/final3/smoke.log; exit 1; }
tail -1 gpurun_out/r06/final3/smoke.log
bash tools/profile.sh > gpurun_out/r06/final3/profile.log 2>&1 || { echo "profile failed"; tail -20 gpurun_out/r06/final3/profile.log; exit 1; }
tail -3 gpurun_out/r06/final3/profile.log
cp gpurun_out/op_stats.csv gpurun_out/traffic.json gpurun_out/mfma.json profiles/ && cp gpurun_out/op_stats.csv gpurun_out/traffic.json gpurun_out/mfma.json gpurun_out/piped_steps.json gpurun_out/bench_ops.json gpurun_out/r06/final3/ && cp gpurun_out/prof/run_kernel_stats.csv gpurun_out/r06/final3/kernel_stats.csv
timeout -k 10 700 python -u bench.py > gpurun_out/r06/final3/bench_default.json 2> gpurun_out/r06/final3/bench_default.err || { echo "bench failed"; tail gpurun_out/r06/final3/bench_default.err; exit 1; }
echo bench done
timeout -k 10 400 python tools/serve_load.py --rounds 3 --seconds 6 --trace --back-frames 2 --out gpurun_out/r06/final3/serve_bf2.json > gpurun_out/r06/final3/serve_bf2.log 2>&1 || { echo "serve_load failed"; tail gpurun_out/r06/final3/serve_bf2.log; exit 1; }
tail -1 gpurun_out/r06/final3/serve_bf2.log
