#!/bin/bash
# Folded operator columns at N = 2048 / 4096 (fft2.hip k_rowsf / k_colsf): parity, then A/B timing
# against the XCD-grouped whole-column tiles -> gpurun_out/r03fold
set -o pipefail
O=gpurun_out/r03fold; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -v --timeout 300 --timeout-method thread -k "operator_large or operator_2048" > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -3 $O/pytest.log
for r in 1 2; do
for m in 1 0; do
  OCEAN_OP_FOLD=$m timeout -k 10 120 python3 tools/ifft_op.py 4096 4 1 20 > $O/op4k_fold$m.r$r.json 2>> $O/err.log || exit 3
  OCEAN_OP_FOLD=$m timeout -k 10 120 python3 tools/ifft_op.py 2048 4 1 30 > $O/op2k_fold$m.r$r.json 2>> $O/err.log || exit 4
done
OCEAN_OP_FOLD=1 OCEAN_FOLD_COLS=16 timeout -k 10 120 python3 tools/ifft_op.py 4096 4 1 20 > $O/op4k_fold16.r$r.json 2>> $O/err.log || exit 5
done
for f in $O/op*.json; do echo "$f $(cat $f)"; done
