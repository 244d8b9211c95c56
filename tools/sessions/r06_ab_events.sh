set -o pipefail
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_gpu_preview.py tests/test_gpu_serve.py tests/test_gpu_bench_shape.py > gpurun_out/pre.log 2>&1 || { echo PRE FAILED; tail -30 gpurun_out/pre.log; exit 1; }
tail -2 gpurun_out/pre.log
timeout -k 10 120 python -u tools/first_chunk_probe.py --admissions 40 > gpurun_out/fcp_new.json 2>&1 || { echo probe failed; tail gpurun_out/fcp_new.json; exit 1; }
tail -1 gpurun_out/fcp_new.json
ARMS="base:PTTS_LIB=gpubin/libbase.so new:-" REPS=4 bash tools/ab.sh gpurun_out/ab_ev.txt
tail -3 gpurun_out/ab_ev.txt
