set -u
mkdir -p gpurun_out
for L in gpubin/libqp_f3aff65.so product gpubin/libqp_f3aff65.so product gpubin/libqp_f3aff65.so product; do
  if [ "$L" = product ]; then timeout -k 10 120 python -u tools/race_probe.py --jobs 80 >> gpurun_out/race4.txt 2>&1 || { echo "probe failed $L"; tail -5 gpurun_out/race4.txt; exit 1; }
  else PTTS_LIB=$L timeout -k 10 120 python -u tools/race_probe.py --jobs 80 >> gpurun_out/race4.txt 2>&1 || { echo "probe failed $L"; tail -5 gpurun_out/race4.txt; exit 1; }; fi
done
cut -c1-200 gpurun_out/race4.txt
