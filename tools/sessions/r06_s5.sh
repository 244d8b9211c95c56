set -u
mkdir -p gpurun_out/r06
timeout -k 10 300 python -u -m pytest -v --timeout 200 --timeout-method thread tests/test_gpu_parity.py -k "flush or varying" > gpurun_out/r06/s5_tests.log 2>&1; rc=$?
tail -2 gpurun_out/r06/s5_tests.log
[ $rc -le 1 ] || { echo "crash"; exit 1; }
timeout -k 10 200 python tools/lib_diff.py pocket-tts_amd/lib/libpocket_tts_hip.so pocket-tts_amd/lib/libpocket_tts_hip.so 40 8 > gpurun_out/r06/diff_bf8.txt 2>&1 || { echo "bf8 run failed"; tail gpurun_out/r06/diff_bf8.txt; exit 1; }
tail -1 gpurun_out/r06/diff_bf8.txt
ARMS="bf2:- bf4:BENCH=--back-frames+4 bf8:BENCH=--back-frames+8 bp0_4:PTTS_LIB=gpubin/libback_prio0.so,BENCH=--back-frames+4 bp0_8:PTTS_LIB=gpubin/libback_prio0.so,BENCH=--back-frames+8" REPS=3 bash tools/ab.sh gpurun_out/r06/ab_bf8.txt > gpurun_out/r06/ab_bf8.log 2>&1 || { echo "ab failed"; tail gpurun_out/r06/ab_bf8.log; exit 1; }
tail -6 gpurun_out/r06/ab_bf8.log
