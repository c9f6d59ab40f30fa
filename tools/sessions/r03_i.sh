#!/bin/bash
# Four-step operator at 4096: rows per workgroup 1 vs 2.
set -o pipefail
O=gpurun_out/r03i; mkdir -p $O
for r in 1 2; do for b in 1 2; do
  OCEAN_OP_ROWS_B=$b timeout -k 10 120 python tools/ifft_op.py 4096 4 1 10 > $O/b$b.json 2>/dev/null || exit 2
  echo "$r rows_b=$b $(cat $O/b$b.json)"
done; done
