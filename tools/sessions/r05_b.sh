#!/bin/bash
# Round 5, session b: the full GPU suite on the product (ABI v3: device scope, readback copy timing, the
# parity call orders), then the split-barrier pass AQ (candidate 1: AQ_SPLIT build)
# on the parity subset and cfg3 A/B against the product, three alternating rounds.
set -o pipefail
OUT=gpurun_out/r05_b; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -2 $OUT/pytest.log
K="frames_vs_oracle or large_time or cfg4_shape or five_cascades or three_plane or golden"
OCEAN_HIP_LIB=$PWD/ocean-simulation_amd/ocean_hip/liboceanhip_split.so timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py \
    -m gpu -k "$K" -q --maxfail=3 --timeout 300 --timeout-method thread -p no:cacheprovider > $OUT/pytest_split.log 2>&1
rc=$?; echo "split pytest rc=$rc $(tail -1 $OUT/pytest_split.log)"
[ $rc -eq 0 ] || exit 2
bash tools/ab_lib.sh cfg3 "base split" 300 3 > $OUT/ab_cfg3.txt 2>&1 || { tail $OUT/ab_cfg3.txt; exit 3; }
cat $OUT/ab_cfg3.txt
echo session done
