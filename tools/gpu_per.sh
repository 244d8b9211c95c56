# Persistent back-part tiles (layouts 40/41/42: 3/4/5 LDS buffers) against the 64x64 ILV tile
# (layout 32), probe build: numerics (first frames vs the default variant) and the steady
# pipelined step, same box.
set -e
export PTTS_LIB=pocket-tts_amd/lib-probes/libpocket_tts_hip.so
ovr() { echo "mimi.qkv=$1,mimi.out=$1:4,mimi.ff1=$1,mimi.ff2=$1:4,seanet.conv0=$1:4,seanet.up0.convtr=$1:4,seanet.up1.convtr=$1,seanet.up2.convtr=$1"; }
timeout -k 10 300 python -u tools/variant_probe.py "[{}, {\"PTTS_OVR\": \"$(ovr 41)\"}, {\"PTTS_OVR\": \"$(ovr 42)\"}]" seanet.conv0,seanet.up2.convtr > gpurun_out/per_var.log 2>&1
cat gpurun_out/per_var.log
VAR=PTTS_OVR VALUES="- $(ovr 40) $(ovr 41) $(ovr 42)" REPS=3 timeout -k 10 500 python -u tools/env_ab.py > gpurun_out/per_ab.log 2>&1
grep MEDIAN gpurun_out/per_ab.log
