#!/bin/bash
# Round 4: where the Update loop's readback time goes (tools/readback_probe.py), with the product library
# and with the readback snapshot as a copy kernel (liboceanhip_snapk.so, -DOCEAN_SNAPKERN=1)
set -o pipefail
OUT=gpurun_out/r04_rb; mkdir -p $OUT
export TMPDIR=/tmp
for v in base snapk base snapk; do
  lib=ocean-simulation_amd/ocean_hip/liboceanhip.so; [ $v != base ] && lib=ocean-simulation_amd/ocean_hip/liboceanhip_$v.so
  o=$(OCEAN_HIP_LIB=$PWD/$lib timeout -k 10 200 python tools/readback_probe.py 200 2> $OUT/probe_$v.err) || { tail $OUT/probe_$v.err; exit 1; }
  echo "$v $o" | tee -a $OUT/probe.txt
done
echo session done
