# FlowLM linear1 tile / split-K choices (probe build, PTTS_OVR): per-op HIP-event time and the
# pipelined step, to price a fused (no split-K, GELU in the epilogue) linear1.
set -e
export PTTS_LIB=pocket-tts_amd/lib-probes/libpocket_tts_hip.so
ovr() { s=""; for l in 0 1 2 3 4 5; do s="$s${s:+,}flow.l$l.ff1_gemm=$1"; done; echo $s; }
timeout -k 10 400 python -u tools/variant_probe.py "[{}, {\"PTTS_OVR\": \"$(ovr 0:1)\"}, {\"PTTS_OVR\": \"$(ovr 0:2)\"}, {\"PTTS_OVR\": \"$(ovr 18:1)\"}, {\"PTTS_OVR\": \"$(ovr 7:2)\"}, {\"PTTS_OVR\": \"$(ovr 6:1)\"}]" flow.l0.ff1_gemm,flow.l0.ff1_reduce_gelu,flow.l0.out_gemm,flow.l0.qkv_gemm > gpurun_out/ff1_var.log 2>&1
cat gpurun_out/ff1_var.log
