set -o pipefail
mkdir -p gpurun_out
timeout -k 10 200 python -u tools/overlap_probe.py > gpurun_out/overlap.txt 2>&1; tail -4 gpurun_out/overlap.txt
ARMS="prod:- ffnkeep:PTTS_LIB=gpubin/libffn_keep.so gemvkeep:PTTS_LIB=gpubin/libgemv_keep.so" REPS=3 bash tools/ab.sh gpurun_out/ab_keep.txt
tail -4 gpurun_out/ab_keep.txt
