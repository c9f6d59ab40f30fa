#!/bin/bash
# Round 4: the facades' readback ring after the in-place slice change (Python + C++ host), then the probe
set -o pipefail
OUT=gpurun_out/r04_ring; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_host.py -m gpu -k "water_body or host" -v --timeout 300 \
  --timeout-method thread -p no:cacheprovider > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
for v in base rbss; do
  lib=ocean-simulation_amd/ocean_hip/liboceanhip.so; [ $v != base ] && lib=ocean-simulation_amd/ocean_hip/liboceanhip_$v.so
  o=$(OCEAN_HIP_LIB=$PWD/$lib timeout -k 10 250 python tools/readback_probe.py 200 2> $OUT/probe_$v.err) || { tail $OUT/probe_$v.err; exit 2; }
  echo "$v $o" | tee -a $OUT/probe.txt
done
echo session done
