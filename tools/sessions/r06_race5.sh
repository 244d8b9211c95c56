set -u
mkdir -p gpurun_out
for L in gpubin/libqprio_fix.so product gpubin/libqprio_fix.so product gpubin/libqprio_fix.so; do
  if [ "$L" = product ]; then timeout -k 10 120 python -u tools/race_probe.py --jobs 80 >> gpurun_out/race5.txt 2>&1 || { echo "probe failed $L"; tail -5 gpurun_out/race5.txt; exit 1; }
  else PTTS_LIB=$L timeout -k 10 120 python -u tools/race_probe.py --jobs 80 >> gpurun_out/race5.txt 2>&1 || { echo "probe failed $L"; tail -5 gpurun_out/race5.txt; exit 1; }; fi
done
cut -c1-200 gpurun_out/race5.txt
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_gpu_preview.py tests/test_gpu_serve.py tests/test_gpu_bench_shape.py > gpurun_out/pre5.log 2>&1 || { echo TESTS FAILED; tail -30 gpurun_out/pre5.log; exit 1; }
tail -1 gpurun_out/pre5.log
