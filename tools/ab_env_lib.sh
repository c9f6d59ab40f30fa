# A/B of (library variant, env) pairs on one bench config, interleaved over rounds:
#   bash tools/ab_env_lib.sh <config> "<variant>:<env,env> ..." [steps] [rounds]
# variant "base" = ocean_hip/liboceanhip.so, else ocean_hip/liboceanhip_<variant>.so; env "-" = none
set -e
mkdir -p gpurun_out
for r in $(seq 1 ${4:-2}); do
  i=0
  for vc in $2; do
    i=$((i+1)); v=${vc%%:*}; e=${vc#*:}; [ "$e" = "-" ] && e=
    lib=ocean-simulation_amd/ocean_hip/liboceanhip.so
    [ "$v" != base ] && lib=ocean-simulation_amd/ocean_hip/liboceanhip_$v.so
    env OCEAN_HIP_LIB=$PWD/$lib $(echo $e | tr ',' ' ') timeout -k 10 300 python bench.py --config $1 --steps ${3:-50} \
      --warmup 5 --no-cpu-baseline --no-ifft-stage --no-beyond-cache --no-update-loop > gpurun_out/abe_$i.json 2> gpurun_out/abe_$i.err
    echo "$r $vc $(python -c "import json;d=json.load(open('gpurun_out/abe_$i.json'));print(d['value'],d['kernels_us'])")"
  done
done
