#!/bin/bash
# Round 5, session j: the product (DISP cached when it fits + nontemporal intermediate loads in pass BQ) against
# the build without either (nodc) on cfg3 / cfg4; cfg5 with pass C2's loads nontemporal (c2nt) against the product.
set -o pipefail
OUT=gpurun_out/r05_j; mkdir -p $OUT
export TMPDIR=/tmp
OCEAN_HIP_LIB=$PWD/ocean-simulation_amd/ocean_hip/liboceanhip_c2nt.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu \
  -k "frames_vs_oracle and 4096 or column_parity_shards" -q -x --timeout 300 --timeout-method thread > $OUT/pytest_c2nt.log 2>&1 || { tail -30 $OUT/pytest_c2nt.log; exit 1; }
tail -1 $OUT/pytest_c2nt.log
bash tools/ab_lib.sh cfg3 "base nodc" 300 4 > $OUT/ab_cfg3.txt 2>&1 || { tail $OUT/ab_cfg3.txt; exit 3; }
cat $OUT/ab_cfg3.txt
bash tools/ab_lib.sh cfg4 "base nodc" 100 3 > $OUT/ab_cfg4.txt 2>&1 || { tail $OUT/ab_cfg4.txt; exit 4; }
cat $OUT/ab_cfg4.txt
bash tools/ab_lib.sh cfg5 "base c2nt" 40 3 > $OUT/ab_cfg5.txt 2>&1 || { tail $OUT/ab_cfg5.txt; exit 5; }
cat $OUT/ab_cfg5.txt
echo session done
