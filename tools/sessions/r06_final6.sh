set -u
D=gpurun_out/r06/final6
mkdir -p $D
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > $D/pytest_gpu.log 2>&1; rc=$?
tail -2 $D/pytest_gpu.log
[ $rc -le 1 ] || { echo "pytest crashed rc=$rc"; exit 1; }
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > $D/smoke.log 2>&1 || { echo "smoke failed"; tail $D/smoke.log; exit 1; }
tail -1 $D/smoke.log
bash tools/profile.sh > $D/profile.log 2>&1 || { echo "profile failed"; tail -20 $D/profile.log; exit 1; }
tail -3 $D/profile.log
cp gpurun_out/op_stats.csv gpurun_out/traffic.json gpurun_out/mfma.json profiles/ && cp gpurun_out/op_stats.csv gpurun_out/traffic.json gpurun_out/mfma.json gpurun_out/piped_steps.json gpurun_out/bench_ops.json $D/ && cp gpurun_out/prof/run_kernel_stats.csv $D/kernel_stats.csv
timeout -k 10 700 python -u bench.py > $D/bench_default.json 2> $D/bench_default.err || { echo "bench failed"; tail $D/bench_default.err; exit 1; }
echo bench done
timeout -k 10 400 python tools/serve_load.py --rounds 3 --seconds 6 --trace --back-frames 2 --out $D/serve_bf2.json > $D/serve_bf2.log 2>&1 || { echo "serve_load failed"; tail $D/serve_bf2.log; exit 1; }
tail -1 $D/serve_bf2.log
