#!/bin/bash
# Round 4 session 8: pass AQ (mirror-pair rows, h0k: 32 instead of 40 B per texel) at
# N = 4096 in place of pass A3Q (liboceanhip_aq4k.so, -DOCEAN_AQ4K=1): 4096 parity, then cfg5 A/B
set -o pipefail
OUT=gpurun_out/r04_ab8; mkdir -p $OUT
export TMPDIR=/tmp
K="4096 and (frames_vs_oracle or shallow or three_plane or split_ocean or large_n or four_step or column_parity)"
OCEAN_HIP_LIB=$PWD/ocean-simulation_amd/ocean_hip/liboceanhip_aq4k.so timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py \
  -m gpu -k "$K" -q --maxfail=3 --timeout 400 --timeout-method thread -p no:cacheprovider > $OUT/pytest_aq4k.log 2>&1
rc=$?; echo "aq4k pytest rc=$rc $(tail -1 $OUT/pytest_aq4k.log)"
grep -E "FAILED|assert|Error" $OUT/pytest_aq4k.log | head -20
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
bash tools/ab_lib.sh cfg5 "base aq4k" 100 3 > $OUT/ab_cfg5.txt 2>&1 || { tail $OUT/ab_cfg5.txt; exit 3; }
cat $OUT/ab_cfg5.txt
echo session done
