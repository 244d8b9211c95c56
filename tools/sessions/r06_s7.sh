set -u
mkdir -p gpurun_out/r06
T="timeout -k 10 900 python -u -m pytest -v --timeout 300 --timeout-method thread"
$T tests/test_gpu_parity.py -k "flush or varying or frame_pairs or batch_scheduler or pipelined" > gpurun_out/r06/s7_tests.log 2>&1; rc=$?
tail -2 gpurun_out/r06/s7_tests.log
[ $rc -eq 0 ] || { grep -E "^(FAILED|ERROR)" gpurun_out/r06/s7_tests.log | head; exit 1; }
$T tests/test_gpu_bench_shape.py tests/test_gpu_streaming.py > gpurun_out/r06/s7_shape.log 2>&1; rc=$?
tail -2 gpurun_out/r06/s7_shape.log
[ $rc -eq 0 ] || { grep -E "^(FAILED|ERROR)" gpurun_out/r06/s7_shape.log | head; exit 1; }
ARMS="base2:PTTS_LIB=gpubin/libbase.so base4:PTTS_LIB=gpubin/libbase.so,BENCH=--back-frames+4 bf2:- bf4:BENCH=--back-frames+4" REPS=3 bash tools/ab.sh gpurun_out/r06/ab_partial.txt > gpurun_out/r06/ab_partial.log 2>&1 || { echo "ab failed"; tail gpurun_out/r06/ab_partial.log; exit 1; }
tail -5 gpurun_out/r06/ab_partial.log
