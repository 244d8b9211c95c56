set -u
mkdir -p gpurun_out
for L in product gpubin/libqueue_prio.so gpubin/libqprio_old.so product gpubin/libqueue_prio.so gpubin/libqprio_old.so; do
  if [ "$L" = product ]; then timeout -k 10 120 python -u tools/race_probe.py --jobs 60 >> gpurun_out/race.txt 2>&1 || { echo "probe failed $L"; tail -5 gpurun_out/race.txt; exit 1; }
  else PTTS_LIB=$L timeout -k 10 120 python -u tools/race_probe.py --jobs 60 >> gpurun_out/race.txt 2>&1 || { echo "probe failed $L"; tail -5 gpurun_out/race.txt; exit 1; }; fi
done
cat gpurun_out/race.txt | cut -c1-400
