# k_gemv with one shared LDS block (X slice / reduction): GPU tests, then the product bench
# against the previous library (pocket-tts_amd/lib-base), both back-pass modes
set -e
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { tail -n 30 gpurun_out/pytest_gpu.log; exit 1; }
tail -n 1 gpurun_out/pytest_gpu.log
bash tools/bf_ab.sh
