#!/bin/bash
# Round 4 session 6: R[Q3] stored for rows <= N/2 only (liboceanhip_half.so, -DOCEAN_Q3HALF=1; pass BQ forms
# the rows above N/2 from their mirror rows): parity subset, then cfg3 / cfg4 A/B against the base library
set -o pipefail
OUT=gpurun_out/r04_ab6; mkdir -p $OUT
export TMPDIR=/tmp
K="frames_vs_oracle or large_time or five_cascades or three_plane or split_ocean or column_band_narrow or narrow_column or past_4gib or shallow or cfg4_shape or golden or chunked_frame or tiles_are_independent or normals"
OCEAN_HIP_LIB=$PWD/ocean-simulation_amd/ocean_hip/liboceanhip_half.so timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py \
  -m gpu -k "$K" -q --maxfail=5 --timeout 300 --timeout-method thread -p no:cacheprovider > $OUT/pytest_half.log 2>&1
rc=$?; echo "half pytest rc=$rc $(tail -1 $OUT/pytest_half.log)"
grep -E "FAILED|assert|Error" $OUT/pytest_half.log | head -20
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
bash tools/ab_lib.sh cfg3 "base half" 300 3 > $OUT/ab_cfg3.txt 2>&1 || { tail $OUT/ab_cfg3.txt; exit 3; }
cat $OUT/ab_cfg3.txt
bash tools/ab_lib.sh cfg4 "base half" 100 2 > $OUT/ab_cfg4.txt 2>&1 || { tail $OUT/ab_cfg4.txt; exit 4; }
cat $OUT/ab_cfg4.txt
echo session done
