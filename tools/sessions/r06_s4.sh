set -u
mkdir -p gpurun_out/r06
timeout -k 10 600 python -u -m pytest -v --timeout 300 --timeout-method thread tests/test_gpu_bench_shape.py > gpurun_out/r06/s4_bench_shape.log 2>&1; rc=$?
tail -2 gpurun_out/r06/s4_bench_shape.log
[ $rc -eq 0 ] || { grep -E "^(FAILED|ERROR)|Error" gpurun_out/r06/s4_bench_shape.log | head; exit 1; }
B4=BENCH=--back-frames+4
ARMS="bf2:- bf4:$B4 bp0:PTTS_LIB=gpubin/libback_prio0.so,$B4 cap2:PTTS_LIB=gpubin/libback_cap2.so,$B4 fp2:PTTS_LIB=gpubin/libfront_prio2.so,$B4" REPS=3 bash tools/ab.sh gpurun_out/r06/ab_quad_prio.txt > gpurun_out/r06/ab_quad_prio.log 2>&1 || { echo "ab failed"; tail gpurun_out/r06/ab_quad_prio.log; exit 1; }
tail -6 gpurun_out/r06/ab_quad_prio.log
