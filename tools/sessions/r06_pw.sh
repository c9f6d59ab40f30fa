#!/bin/bash
# Round 6, session pw: the stage-wise pointwise split of VERDICT r05 item 1 (tools/pointwise_stages.py)
# for the product library and the A/B builds initf64 (init transcendentals in double), phase (library
# sincosf), rcp (1.0f / |k|), acc (all three), plus OCEAN_Q=0 (four-plane frame) at cfg3.
set -o pipefail
OUT=gpurun_out/r06_pw; mkdir -p $OUT
export TMPDIR=/tmp
L=$PWD/ocean-simulation_amd/ocean_hip
run() {  # label lib cfgs rows [env]
  env $5 OCEAN_HIP_LIB=$L/$2 timeout -k 10 400 python -u tools/pointwise_stages.py $1 $OUT/$1.json $3 $4 2>> $OUT/$1.err || { tail $OUT/$1.err; exit 3; }
}
run base liboceanhip.so cfg2,cfg3 init,frame,evolve,operator
run initf64 liboceanhip_initf64.so cfg2,cfg3 init,frame
run phase liboceanhip_phase.so cfg2,cfg3 frame
run rcp liboceanhip_rcp.so cfg3 frame
run acc liboceanhip_acc.so cfg2,cfg3 init,frame
run q0 liboceanhip.so cfg3 frame OCEAN_Q=0
echo session done
