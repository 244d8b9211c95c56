set -u
mkdir -p gpurun_out/r06
T="timeout -k 10 900 python -u -m pytest -v --timeout 300 --timeout-method thread"
$T tests/test_gpu_bench_shape.py tests/test_gpu_bf16.py > gpurun_out/r06/s8_tests.log 2>&1; rc=$?
tail -2 gpurun_out/r06/s8_tests.log
[ $rc -eq 0 ] || { grep -E "^(FAILED|ERROR)" gpurun_out/r06/s8_tests.log | head; exit 1; }
for v in resblock_s12 resblock_s012; do
  timeout -k 10 200 python tools/lib_diff.py gpubin/libbase.so gpubin/lib$v.so 40 4 > gpurun_out/r06/diff_$v.txt 2>&1 || { echo "diff $v failed"; tail gpurun_out/r06/diff_$v.txt; exit 1; }
  tail -1 gpurun_out/r06/diff_$v.txt
done
ARMS="base:PTTS_LIB=gpubin/libbase.so rbload:- s12:PTTS_LIB=gpubin/libresblock_s12.so s012:PTTS_LIB=gpubin/libresblock_s012.so" REPS=3 bash tools/ab.sh gpurun_out/r06/ab_resblock.txt > gpurun_out/r06/ab_resblock.log 2>&1 || { echo "ab failed"; tail gpurun_out/r06/ab_resblock.log; exit 1; }
tail -5 gpurun_out/r06/ab_resblock.log
