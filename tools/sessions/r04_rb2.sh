#!/bin/bash
# Round 4: readback ring depth and stream placement (tools/readback_probe.py): the product library and the
# device-to-host copy on the context stream (liboceanhip_rbss.so, -DOCEAN_RB_SAMESTREAM=1)
set -o pipefail
OUT=gpurun_out/r04_rb2; mkdir -p $OUT
export TMPDIR=/tmp
for v in base rbss; do
  lib=ocean-simulation_amd/ocean_hip/liboceanhip.so; [ $v != base ] && lib=ocean-simulation_amd/ocean_hip/liboceanhip_$v.so
  o=$(OCEAN_HIP_LIB=$PWD/$lib timeout -k 10 250 python tools/readback_probe.py 200 2> $OUT/probe_$v.err) || { tail $OUT/probe_$v.err; exit 1; }
  echo "$v $o" | tee -a $OUT/probe.txt
done
echo session done
