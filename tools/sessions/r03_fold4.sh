#!/bin/bash
# Folded operator, fold formed in the last row's emit: parity, A/B timing, rocprofv3 stats of the 4096 operator
set -o pipefail
O=gpurun_out/r03fold4; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -v --timeout 300 --timeout-method thread -k "operator" > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -3 $O/pytest.log
for r in 1 2; do
  OCEAN_OP_FOLD=1 timeout -k 10 120 python3 tools/ifft_op.py 4096 4 1 20 > $O/op4k_fold.r$r.json 2>> $O/err.log || exit 3
  OCEAN_OP_FOLD=0 timeout -k 10 120 python3 tools/ifft_op.py 4096 4 1 20 > $O/op4k_grouped.r$r.json 2>> $O/err.log || exit 5
  OCEAN_OP_FOLD=1 timeout -k 10 120 python3 tools/ifft_op.py 2048 4 1 30 > $O/op2k_fold.r$r.json 2>> $O/err.log || exit 4
done
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o op4k -- python3 tools/ifft_op.py 4096 4 1 20 > $O/prof.log 2>&1 || exit 6
for f in $O/op*.json; do echo "$f $(cat $f)"; done
find $O/prof -name "*kernel_stats.csv" | head -3
