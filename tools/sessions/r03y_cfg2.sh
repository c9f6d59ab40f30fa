#!/bin/bash
# A/B cfg2 (512^2 x 1, displacement only): pre-change library vs current, alternating.
set -e
out=gpurun_out/r03y
mkdir -p $out
: > $out/cfg2_ab.txt
pre=$PWD/ocean-simulation_amd/ocean_hip/liboceanhip_pre.so
for r in 1 2 3; do
  echo "pre" >> $out/cfg2_ab.txt
  OCEAN_HIP_LIB=$pre timeout -k 10 200 python3 bench.py --config cfg2 --no-cpu-baseline >> $out/cfg2_ab.txt 2>/dev/null
  echo "new" >> $out/cfg2_ab.txt
  timeout -k 10 200 python3 bench.py --config cfg2 --no-cpu-baseline >> $out/cfg2_ab.txt 2>/dev/null
done
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $out/prof -o cfg2 -- python3 bench.py --config cfg2 --no-cpu-baseline > /dev/null 2>&1
python3 -c "
import json
for l in open('$out/cfg2_ab.txt'):
    l=l.strip()
    if l.startswith('{'):
        d=json.loads(l); print(d['value'], d.get('kernels_us'))
    else: print(l)
"
