#!/bin/bash
# Round 4 session 9: passes A8 / B8 with their twiddles in registers, loaded
# beside the first item's data (liboceanhip_twreg.so, -DOCEAN_TWREG=1): parity, then cfg2 A/B
set -o pipefail
OUT=gpurun_out/r04_ab9; mkdir -p $OUT
export TMPDIR=/tmp
K="frames_vs_oracle and 512 or launch_variants or narrow or column_band_narrow or split_ocean"
OCEAN_HIP_LIB=$PWD/ocean-simulation_amd/ocean_hip/liboceanhip_twreg.so timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py \
  -m gpu -k "$K" -q --maxfail=3 --timeout 300 --timeout-method thread -p no:cacheprovider > $OUT/pytest_twreg.log 2>&1
rc=$?; echo "twreg pytest rc=$rc $(tail -1 $OUT/pytest_twreg.log)"
[ $rc -eq 0 ] || exit $rc
bash tools/ab_lib.sh cfg2 "base twreg" 2000 4 > $OUT/ab_cfg2.txt 2>&1 || { tail $OUT/ab_cfg2.txt; exit 3; }
cat $OUT/ab_cfg2.txt
echo session done
