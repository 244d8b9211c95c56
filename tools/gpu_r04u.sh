#!/bin/bash
# Round 4: the back part's short launches without the one-workgroup-per-CU cap (probe build,
# PTTS_OP_CAP name=0): the row reduces, the Mimi RoPE / append, quantizer + upsample, the final
# conv and the commit (A), and A + the Mimi attention (B); bench steady ms/step, interleaved.
set -u
cd "$(dirname "$0")/.."
export PTTS_LIB=pocket-tts_amd/lib-probes/libpocket_tts_hip.so
A="mimi.quant_upsample=0,mimi.l0.qkv_rope=0,mimi.l1.qkv_rope=0,mimi.l0.out_reduce_ln2=0,mimi.l1.out_reduce_ln2=0,mimi.l0.ff2_reduce=0,mimi.l1.ff2_reduce=0,seanet.conv0_reduce=0,seanet.up0.convtr_reduce=0,seanet.conv_final=0,commit=0"
B="$A,mimi.l0.attention=0,mimi.l1.attention=0"
rm -f gpurun_out/sweep_all.txt
VAR=PTTS_OP_CAP REPS=3 VALUES="- $A $B" bash tools/sweep_env.sh
