#!/bin/bash
# Read-side fold (OCEAN_OP_FOLD=2) against the row-side fold (1) and the grouped tiles (0) -> gpurun_out/r03fold5
set -o pipefail
O=gpurun_out/r03fold5; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -v --timeout 300 --timeout-method thread -k "operator" > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -3 $O/pytest.log
for r in 1 2; do
  for m in 2 1 0; do
    OCEAN_OP_FOLD=$m timeout -k 10 120 python3 tools/ifft_op.py 4096 4 1 20 > $O/op4k_fold$m.r$r.json 2>> $O/err.log || exit 3
  done
  OCEAN_OP_FOLD=2 timeout -k 10 120 python3 tools/ifft_op.py 2048 4 1 30 > $O/op2k_fold2.r$r.json 2>> $O/err.log || exit 4
  OCEAN_OP_FOLD=2 OCEAN_OP_CHUNK_MIB=256 timeout -k 10 120 python3 tools/ifft_op.py 4096 4 1 20 > $O/op4k_fold2_c256.r$r.json 2>> $O/err.log || exit 4
done
for f in $O/op*.json; do echo "$f $(cat $f)"; done
