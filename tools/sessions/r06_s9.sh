set -u
mkdir -p gpurun_out/r06
P=gpubin/libprobes.so
NOV="--no-cpu-baseline --no-quant-variant --no-op-times --no-latency --no-distinct-voices --no-voice-bench --no-text-bench"
for bf in 4 2; do
  PTTS_LIB=$P PTTS_STAMPS=gpurun_out/r06/stamps_bf$bf.txt timeout -k 10 240 python bench.py $NOV --back-frames $bf > gpurun_out/r06/stamps_bf$bf.json 2>&1 || { echo "stamps $bf failed"; tail gpurun_out/r06/stamps_bf$bf.json; exit 1; }
  python tools/stamps.py gpurun_out/r06/stamps_bf$bf.txt gpurun_out/r06/stamps_bf$bf.sum.json | tail -12
done
PTTS_LIB=$P PTTS_STAMPS=gpurun_out/r06/opstamps_bf4.txt PTTS_STAMP_OPS=1 timeout -k 10 240 python bench.py $NOV --back-frames 4 > gpurun_out/r06/opstamps_bf4.json 2>&1 || { echo "opstamps failed"; tail gpurun_out/r06/opstamps_bf4.json; exit 1; }
python tools/op_stamps.py gpurun_out/r06/opstamps_bf4.txt gpurun_out/r06/opstamps_bf4.sum.json > gpurun_out/r06/opstamps_bf4.log 2>&1; tail -5 gpurun_out/r06/opstamps_bf4.log
