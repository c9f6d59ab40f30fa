#!/bin/bash
# Round 4 session 5 (exploratory): pass A of chunk k + 1 on a second stream beside pass B
# of chunk k (liboceanhip_ovl.so, -DOCEAN_OVERLAP, two intermediate regions): parity of the chunked frame,
# then cfg4 A/B against the base library at 96 / 128 / 192 MiB chunks.  Kill criterion: >= 5 % over 51.0 k.
set -o pipefail
OUT=gpurun_out/r04_ab5; mkdir -p $OUT
export TMPDIR=/tmp
K="cfg4_shape or chunked_frame or tiles_are_independent"
OCEAN_HIP_LIB=$PWD/ocean-simulation_amd/ocean_hip/liboceanhip_ovl.so timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py \
  -m gpu -k "$K" -q --maxfail=3 --timeout 300 --timeout-method thread -p no:cacheprovider > $OUT/pytest_ovl.log 2>&1
rc=$?; echo "ovl pytest rc=$rc $(tail -1 $OUT/pytest_ovl.log)"
[ $rc -eq 0 ] || exit $rc
bash tools/ab_env_lib.sh cfg4 "base:- ovl:- ovl:OCEAN_CHUNK_MIB=96 ovl:OCEAN_CHUNK_MIB=128 base:OCEAN_CHUNK_MIB=96" 100 3 > $OUT/ab_cfg4.txt 2>&1 || { tail $OUT/ab_cfg4.txt; exit 3; }
cat $OUT/ab_cfg4.txt
echo session done
