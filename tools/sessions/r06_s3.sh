set -u
mkdir -p gpurun_out/r06
timeout -k 10 200 python tools/lib_diff.py pocket-tts_amd/lib/libpocket_tts_hip.so gpubin/libqd.so 40 4 > gpurun_out/r06/diff_qd.txt 2>&1 || { echo "diff failed"; tail gpurun_out/r06/diff_qd.txt; exit 1; }
tail -1 gpurun_out/r06/diff_qd.txt
ARMS="bf2:- bf4:BENCH=--back-frames+4 qa:PTTS_LIB=gpubin/libqa.so,BENCH=--back-frames+4 qb:PTTS_LIB=gpubin/libqb.so,BENCH=--back-frames+4 qd:PTTS_LIB=gpubin/libqd.so,BENCH=--back-frames+4 qe:PTTS_LIB=gpubin/libqe.so,BENCH=--back-frames+4" REPS=3 bash tools/ab.sh gpurun_out/r06/ab_quad_splits.txt > gpurun_out/r06/ab_quad_splits.log 2>&1 || { echo "ab failed"; tail gpurun_out/r06/ab_quad_splits.log; exit 1; }
tail -7 gpurun_out/r06/ab_quad_splits.log
