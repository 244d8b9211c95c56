set -u
mkdir -p gpurun_out
for L in gpubin/libqp_f3aff65.so gpubin/libqp_760904d.so gpubin/libqp_bc691db.so gpubin/libqueue_prio.so; do
  PTTS_LIB=$L timeout -k 10 120 python -u tools/race_probe.py --jobs 60 >> gpurun_out/race2.txt 2>&1 || { echo "probe failed $L"; tail -5 gpurun_out/race2.txt; exit 1; }
done
cut -c1-300 gpurun_out/race2.txt
