set -o pipefail
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; rc=$?
tail -5 gpurun_out/pytest_gpu.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python tools/head_stamps.py > gpurun_out/head_stamps.log 2>&1 || exit $?
grep -v amdgpu.ids gpurun_out/head_stamps.log
timeout -k 10 300 python bench.py --no-cpu-baseline --no-latency --no-quant-variant --ops-out gpurun_out/ops_chain.json > gpurun_out/bench_chain.log 2>&1 || exit $?
tail -1 gpurun_out/bench_chain.log | cut -c1-300
