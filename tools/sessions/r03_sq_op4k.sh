#!/bin/bash
# SQ counters of the 4 x 4096^2 operator with the 2-way folded columns (k_rowsf<4096, 2> / k_colsf) and,
# for comparison, the in-place grouped tiles (k_rows2<4096, 1> / k_cols2<4096, 4, 4>) -> gpurun_out/sq_op4k_*
set -o pipefail
bash tools/pmc_sq_cmd.sh gpurun_out/sq_op4k_fold python3 tools/ifft_op.py 4096 4 1 10 || exit 1
OCEAN_OP_FOLD=0 bash tools/pmc_sq_cmd.sh gpurun_out/sq_op4k_grouped python3 tools/ifft_op.py 4096 4 1 10 || exit 2
echo done
