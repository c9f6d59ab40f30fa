#!/bin/bash
# Round 5, session i: DISP written with default-policy stores when the frame fits the Infinity Cache
# (disp_fits_cache; product) -- parity subset, then cfg3 / cfg4 / cfg2 A/B against the same library without it
# (nodc) and with nontemporal intermediate loads in pass BQ (lnt).
set -o pipefail
OUT=gpurun_out/r05_i; mkdir -p $OUT
export TMPDIR=/tmp
K="frames_vs_oracle or large_time or cfg4_shape or five_cascades or three_plane or golden or pointwise or normals or mips"
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py -m gpu -k "$K" -q -x --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
bash tools/ab_lib.sh cfg3 "base nodc lnt" 300 4 > $OUT/ab_cfg3.txt 2>&1 || { tail $OUT/ab_cfg3.txt; exit 3; }
cat $OUT/ab_cfg3.txt
bash tools/ab_lib.sh cfg4 "base nodc lnt" 100 3 > $OUT/ab_cfg4.txt 2>&1 || { tail $OUT/ab_cfg4.txt; exit 4; }
cat $OUT/ab_cfg4.txt
echo session done
