set -u
mkdir -p gpurun_out/r06
timeout -k 10 400 python -u -m pytest tests/test_fp8.py tests/test_quantize.py -m gpu -v --timeout 120 --timeout-method thread > gpurun_out/r06/fp8_tests.log 2>&1; rc=$?; [ $rc -le 1 ] || { echo "fp8 tests crashed rc=$rc"; tail -30 gpurun_out/r06/fp8_tests.log; exit 1; }
tail -2 gpurun_out/r06/fp8_tests.log
for v in up0s1 c0s1; do
  timeout -k 10 200 python tools/lib_diff.py pocket-tts_amd/lib/libpocket_tts_hip.so gpubin/lib$v.so 40 > gpurun_out/r06/diff_$v.txt 2>&1 || { echo "diff $v failed"; tail gpurun_out/r06/diff_$v.txt; exit 1; }
  tail -2 gpurun_out/r06/diff_$v.txt
done
ARMS="prod:- up0s1:PTTS_LIB=gpubin/libup0s1.so c0s1:PTTS_LIB=gpubin/libc0s1.so bf1:BENCH=--back-frames+1" REPS=3 bash tools/ab.sh gpurun_out/r06/ab1.txt > gpurun_out/r06/ab1.log 2>&1 || { echo "ab failed"; tail gpurun_out/r06/ab1.log; exit 1; }
tail -5 gpurun_out/r06/ab1.log
timeout -k 10 600 python -u bench.py > gpurun_out/r06/bench_start.json 2> gpurun_out/r06/bench_start.err || { echo "bench failed"; tail gpurun_out/r06/bench_start.err; exit 1; }
