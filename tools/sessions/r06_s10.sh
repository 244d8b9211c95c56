set -u
mkdir -p gpurun_out/r06
timeout -k 10 600 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > gpurun_out/r06/s10_pytest.log 2>&1; rc=$?
tail -2 gpurun_out/r06/s10_pytest.log
[ $rc -eq 0 ] || { grep -E "^(FAILED|ERROR)" gpurun_out/r06/s10_pytest.log | head; exit 1; }
ARMS="base:PTTS_LIB=gpubin/libbase.so compact:-" REPS=4 bash tools/ab.sh gpurun_out/r06/ab_compact_admission.txt > gpurun_out/r06/ab_compact.log 2>&1 || { echo "ab failed"; tail gpurun_out/r06/ab_compact.log; exit 1; }
tail -3 gpurun_out/r06/ab_compact.log
METRIC=admit_ms ARMS="base:PTTS_LIB=gpubin/libbase.so compact:-" REPS=2 bash tools/ab.sh gpurun_out/r06/ab_compact_admission.txt > gpurun_out/r06/ab_compact2.log 2>&1 || { echo "ab2 failed"; tail gpurun_out/r06/ab_compact2.log; exit 1; }
tail -3 gpurun_out/r06/ab_compact2.log
