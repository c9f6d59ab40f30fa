#!/bin/bash
# Round 5, session k: the whole GPU suite on the product (DISP cached + nontemporal loads tied together), then
# cfg3 / cfg4 A/B against nodc.
set -o pipefail
OUT=gpurun_out/r05_k; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -2 $OUT/pytest.log
bash tools/ab_lib.sh cfg3 "base nodc" 300 3 > $OUT/ab_cfg3.txt 2>&1 || { tail $OUT/ab_cfg3.txt; exit 3; }
cat $OUT/ab_cfg3.txt
bash tools/ab_lib.sh cfg4 "base nodc" 100 2 > $OUT/ab_cfg4.txt 2>&1 || { tail $OUT/ab_cfg4.txt; exit 4; }
cat $OUT/ab_cfg4.txt
echo session done
