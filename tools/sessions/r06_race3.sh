set -u
mkdir -p gpurun_out
for L in gpubin/libqp_waits.so gpubin/libqp_callev.so gpubin/libqp_waits.so gpubin/libqp_callev.so; do
  PTTS_LIB=$L timeout -k 10 120 python -u tools/race_probe.py --jobs 60 >> gpurun_out/race3.txt 2>&1 || { echo "probe failed $L"; tail -5 gpurun_out/race3.txt; exit 1; }
done
cut -c1-200 gpurun_out/race3.txt
