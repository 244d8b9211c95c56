set -o pipefail
mkdir -p gpurun_out
ARMS="prod:- qprio:PTTS_LIB=gpubin/libqueue_prio.so" REPS=4 bash tools/ab.sh gpurun_out/ab_qprio.txt
tail -3 gpurun_out/ab_qprio.txt
