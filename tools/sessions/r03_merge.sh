#!/bin/bash
# Pass AQ with rows 0 and N/2 as one item (8 items per CU at cfg3; mg3 build: compiled for 3 waves per
# SIMD) against the N/2 + 1 deal (mg0 build): frame parity with the merged build, then A/B on cfg3 / cfg4
set -o pipefail
O=gpurun_out/r03merge; mkdir -p $O
OCEAN_HIP_LIB=$PWD/ocean-simulation_amd/ocean_hip/liboceanhip_mg3.so timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread -k "frames or cfg4 or large_time or three_plane or normal or foam or band" > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
bash tools/ab_lib.sh cfg3 "mg3 mg0" 500 3 > $O/ab_cfg3.txt 2>&1 || exit 3
bash tools/ab_lib.sh cfg4 "mg3 mg0" 50 2 > $O/ab_cfg4.txt 2>&1 || exit 4
cat $O/ab_cfg3.txt $O/ab_cfg4.txt
