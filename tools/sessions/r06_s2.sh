set -u
mkdir -p gpurun_out/r06
T="timeout -k 10 900 python -u -m pytest -v --timeout 300 --timeout-method thread"
$T tests/test_gpu_parity.py -k "frame_pairs or varying_rows or flush or batch_scheduler" tests/test_gpu_streaming.py tests/test_fp8.py > gpurun_out/r06/quad_tests.log 2>&1; rc=$?
tail -3 gpurun_out/r06/quad_tests.log
[ $rc -le 1 ] || { echo "tests crashed rc=$rc"; tail -30 gpurun_out/r06/quad_tests.log; exit 1; }
[ $rc -eq 0 ] || { grep -E "^(FAILED|ERROR)" gpurun_out/r06/quad_tests.log | head -20; exit 1; }
$T tests/test_gpu_bench_shape.py > gpurun_out/r06/quad_bench_shape.log 2>&1; rc=$?
tail -3 gpurun_out/r06/quad_bench_shape.log
[ $rc -eq 0 ] || { grep -E "^(FAILED|ERROR)|Error" gpurun_out/r06/quad_bench_shape.log | head -20; exit 1; }
ARMS="bf2:- bf4:BENCH=--back-frames+4" REPS=3 bash tools/ab.sh gpurun_out/r06/ab_quad.txt > gpurun_out/r06/ab_quad.log 2>&1 || { echo "ab failed"; tail gpurun_out/r06/ab_quad.log; exit 1; }
tail -3 gpurun_out/r06/ab_quad.log
