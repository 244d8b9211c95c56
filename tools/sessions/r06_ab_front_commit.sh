set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_gpu_preview.py tests/test_gpu_edges.py > gpurun_out/pre.log 2>&1 || { echo PRE FAILED; tail -30 gpurun_out/pre.log; exit 1; }
tail -2 gpurun_out/pre.log
ARMS="base:PTTS_LIB=gpubin/libbase.so new:-" REPS=3 bash tools/ab.sh gpurun_out/ab_fc.txt
tail -4 gpurun_out/ab_fc.txt
