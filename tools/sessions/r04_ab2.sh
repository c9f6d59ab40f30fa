#!/bin/bash
# Round 4 session 2: parity of the pass-AQ variants aqx4 (Q3 of row y2 synthesized in pass 1) and aqx5 / aqx5w
# (one LDS pass of five sequences), then cfg3 / cfg4 A/B against the base library
set -o pipefail
OUT=gpurun_out/r04_ab2; mkdir -p $OUT
export TMPDIR=/tmp
K="frames_vs_oracle or large_time or cfg4_shape or five_cascades or three_plane or split_ocean or column_band_narrow or narrow_column or golden or past_4gib or chunked_frame or tiles_are_independent"
for v in aqx4 aqx5; do
  OCEAN_HIP_LIB=$PWD/ocean-simulation_amd/ocean_hip/liboceanhip_$v.so timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py \
    -m gpu -k "$K" -q --maxfail=3 --timeout 300 --timeout-method thread -p no:cacheprovider > $OUT/pytest_$v.log 2>&1
  rc=$?; echo "$v pytest rc=$rc $(tail -1 $OUT/pytest_$v.log)"
  [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
done
bash tools/ab_lib.sh cfg3 "base aqx4 aqx5" 300 3 > $OUT/ab_cfg3.txt 2>&1 || { tail $OUT/ab_cfg3.txt; exit 3; }
cat $OUT/ab_cfg3.txt
bash tools/ab_lib.sh cfg4 "base aqx5" 100 2 > $OUT/ab_cfg4.txt 2>&1 || { tail $OUT/ab_cfg4.txt; exit 4; }
cat $OUT/ab_cfg4.txt
echo session done
