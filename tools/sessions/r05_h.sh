#!/bin/bash
# Round 5, session h: pass BQ's texture store policy.  Part of the textures with default-policy stores (they
# land in the Infinity Cache and are written back while the next pass A runs, when HBM has headroom) instead of
# nontemporal: DISP (dpl), TURB (tpl), both (dtpl), against the product (all nontemporal).  cfg3 and cfg4 A/B.
set -o pipefail
OUT=gpurun_out/r05_h; mkdir -p $OUT
export TMPDIR=/tmp
bash tools/ab_lib.sh cfg3 "base dpl tpl dtpl lnt dlnt" 300 3 > $OUT/ab_cfg3.txt 2>&1 || { tail $OUT/ab_cfg3.txt; exit 3; }
cat $OUT/ab_cfg3.txt
bash tools/ab_lib.sh cfg4 "base dpl lnt dlnt" 100 2 > $OUT/ab_cfg4.txt 2>&1 || { tail $OUT/ab_cfg4.txt; exit 4; }
cat $OUT/ab_cfg4.txt
echo session done
