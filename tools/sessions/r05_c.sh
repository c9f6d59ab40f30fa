#!/bin/bash
# Round 5, session c: the full GPU suite on the product with the split pass 1 (k_pass_aq), cfg3 and cfg4 A/B
# against the pre-split build (liboceanhip_prev.so, three alternating rounds), the chip ceilings with their
# stamp (tools/ceilings.sh, bqbench now with the flat-with-foam and foam-from-TURB shapes), and the pointwise
# clause with per-(frame, cascade, channel) ratios (tools/pointwise.py).
set -o pipefail
OUT=gpurun_out/r05_c; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -2 $OUT/pytest.log
bash tools/ab_lib.sh cfg3 "base prev" 300 3 > $OUT/ab_cfg3.txt 2>&1 || { tail $OUT/ab_cfg3.txt; exit 3; }
cat $OUT/ab_cfg3.txt
bash tools/ab_lib.sh cfg4 "base prev" 100 3 > $OUT/ab_cfg4.txt 2>&1 || { tail $OUT/ab_cfg4.txt; exit 4; }
cat $OUT/ab_cfg4.txt
bash tools/ceilings.sh $OUT/ceilings || exit 5
cat $OUT/ceilings/bqbench.txt
timeout -k 10 420 python -u tools/pointwise.py $OUT/pointwise.json > $OUT/pointwise.log 2>&1 || { tail $OUT/pointwise.log; exit 6; }
echo session done
