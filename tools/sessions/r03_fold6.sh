#!/bin/bash
# Fold factor at 4096: two rows (2048-point columns) against four (1024-point) and the grouped tiles
set -o pipefail
O=gpurun_out/r03fold6; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -v --timeout 300 --timeout-method thread -k "operator" > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -3 $O/pytest.log
for r in 1 2; do
  OCEAN_FOLD_F=2 timeout -k 10 120 python3 tools/ifft_op.py 4096 4 1 20 > $O/op4k_f2.r$r.json 2>> $O/err.log || exit 3
  OCEAN_FOLD_F=2 OCEAN_OP_CHUNK_MIB=256 timeout -k 10 120 python3 tools/ifft_op.py 4096 4 1 20 > $O/op4k_f2_c256.r$r.json 2>> $O/err.log || exit 3
  OCEAN_FOLD_F=4 timeout -k 10 120 python3 tools/ifft_op.py 4096 4 1 20 > $O/op4k_f4.r$r.json 2>> $O/err.log || exit 3
  OCEAN_OP_FOLD=0 timeout -k 10 120 python3 tools/ifft_op.py 4096 4 1 20 > $O/op4k_grouped.r$r.json 2>> $O/err.log || exit 3
done
OCEAN_FOLD_F=2 timeout -k 10 120 python3 tools/ifft_op.py 4096 1 1 20 > $O/op4k1_f2.json 2>> $O/err.log || exit 4
for f in $O/op*.json; do echo "$f $(cat $f)"; done
