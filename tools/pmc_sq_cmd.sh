#!/bin/bash
# SQ counters of any command, one --pmc pass per group (never combined with tracing domains), plus a
# kernel-trace pass for the per-kernel VGPR / LDS / duration record.
#   bash tools/pmc_sq_cmd.sh <outdir> <command...>     e.g.  gpurun_out/sq_cfg3 python3 bench.py --steps 50 ...
set -o pipefail
OUT=$1; shift
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- "$@" > $OUT/trace.log 2>&1 || { echo "trace failed"; tail -5 $OUT/trace.log; exit 1; }
g=0
for grp in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY" \
           "SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD SQ_ACTIVE_INST_VALU" \
           "SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_BRANCH SQ_ACTIVE_INST_MISC SQ_ACTIVE_INST_SCA"; do
  g=$((g+1))
  timeout -s KILL 200 rocprofv3 --pmc $grp --output-format csv -d $OUT/g$g -o run -- "$@" > $OUT/g$g.log 2>&1 || { echo "fail $grp"; tail -5 $OUT/g$g.log; exit 1; }
done
echo done
