#!/bin/bash
# Round 4 session 3: pass AQW (one wave per mirror-row pair, N = 1024): parity, then cfg3 A/B against base
set -o pipefail
OUT=gpurun_out/r04_ab3; mkdir -p $OUT
export TMPDIR=/tmp
K="frames_vs_oracle or large_time or five_cascades or three_plane or split_ocean or column_band_narrow or narrow_column or past_4gib or normals or shallow or cfg4_shape or golden or chunked_frame or tiles_are_independent"
OCEAN_HIP_LIB=$PWD/ocean-simulation_amd/ocean_hip/liboceanhip_aqx6.so timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py \
  -m gpu -k "$K" -q --maxfail=5 --timeout 300 --timeout-method thread -p no:cacheprovider > $OUT/pytest_aqx6.log 2>&1
rc=$?; echo "aqx6 pytest rc=$rc $(tail -1 $OUT/pytest_aqx6.log)"
grep -E "FAILED|rel err|Error" $OUT/pytest_aqx6.log | head -20
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
bash tools/ab_lib.sh cfg3 "base aqx6" 300 3 > $OUT/ab_cfg3.txt 2>&1 || { tail $OUT/ab_cfg3.txt; exit 3; }
cat $OUT/ab_cfg3.txt
bash tools/ab_lib.sh cfg4 "base aqx6" 100 2 > $OUT/ab_cfg4.txt 2>&1 || { tail $OUT/ab_cfg4.txt; exit 4; }
cat $OUT/ab_cfg4.txt
echo session done
