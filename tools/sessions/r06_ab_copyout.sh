set -o pipefail
mkdir -p gpurun_out/tr2
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_gpu_preview.py tests/test_gpu_serve.py tests/test_gpu_bench_shape.py tests/test_gpu_configs.py > gpurun_out/pre.log 2>&1 || { echo PRE FAILED; tail -30 gpurun_out/pre.log; exit 1; }
tail -2 gpurun_out/pre.log
ROOT=$(pwd)
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace -d $ROOT/gpurun_out/tr2 -o run --output-format csv -- python $ROOT/bench.py --warmup 5 --profile-frames 30 --no-cpu-baseline --no-quant-variant --no-latency --no-distinct-voices --no-voice-bench --no-text-bench --no-op-times > $ROOT/gpurun_out/tr2/log.txt 2>&1) || { echo trace failed; exit 1; }
ARMS="base:PTTS_LIB=gpubin/libbase.so new:-" REPS=4 bash tools/ab.sh gpurun_out/ab_copyout.txt
tail -3 gpurun_out/ab_copyout.txt
