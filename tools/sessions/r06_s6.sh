set -u
mkdir -p gpurun_out/r06
timeout -k 10 600 python -u -m pytest -v --timeout 300 --timeout-method thread tests/test_gpu_parity.py -k "flush or varying or frame_pairs or batch_scheduler" tests/test_gpu_bench_shape.py > gpurun_out/r06/s6_tests.log 2>&1; rc=$?
tail -2 gpurun_out/r06/s6_tests.log
[ $rc -eq 0 ] || { grep -E "^(FAILED|ERROR)" gpurun_out/r06/s6_tests.log | head; exit 1; }
B4=BENCH=--back-frames+4
ARMS="bf2:- bf4:$B4 m35:PTTS_LIB=gpubin/libmimi_tiles35.so,$B4 t35:PTTS_LIB=gpubin/libconvtr_tiles35.so,$B4" REPS=3 bash tools/ab.sh gpurun_out/r06/ab_quad_tiles.txt > gpurun_out/r06/ab_quad_tiles.log 2>&1 || { echo "ab failed"; tail gpurun_out/r06/ab_quad_tiles.log; exit 1; }
tail -5 gpurun_out/r06/ab_quad_tiles.log
timeout -k 10 400 python tools/serve_load.py --rounds 3 --seconds 6 --trace --back-frames 2 --out gpurun_out/r06/serve_bf2.json > gpurun_out/r06/serve_bf2.log 2>&1 || { echo "serve_load failed"; tail gpurun_out/r06/serve_bf2.log; exit 1; }
tail -2 gpurun_out/r06/serve_bf2.log
