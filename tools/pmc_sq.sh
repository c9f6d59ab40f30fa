#!/bin/bash
# SQ counters (one --pmc pass per group) for the bench workload under several env settings.
# Usage: tools/pmc_sq.sh "<env,env> <env>..."; output gpurun_out/sq_<i>/
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
ARGS=${ARGS:-"--steps 50 --warmup 5 --no-cpu-baseline --no-ifft-stage --no-beyond-cache"}
i=0
for cfg in $1; do
  i=$((i+1)); OUT=gpurun_out/sq_$i; mkdir -p $OUT; echo "$cfg" > $OUT/cfg
  g=0
  for grp in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY" \
             "SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD SQ_ACTIVE_INST_VALU" \
             "SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_BRANCH SQ_ACTIVE_INST_MISC SQ_ACTIVE_INST_SCA"; do
    g=$((g+1))
    env $(echo $cfg | tr ',' ' ') timeout -k 10 200 rocprofv3 --pmc $grp --output-format csv -d $OUT/g$g -o run -- python3 bench.py $ARGS > $OUT/g$g.log 2>&1 || { echo "fail $cfg $grp"; tail -5 $OUT/g$g.log; exit 1; }
  done
done
echo done
