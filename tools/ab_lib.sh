# A/B of library builds on one bench config, interleaved A B A B ... to spread drift:
#   bash tools/ab_lib.sh <config> "<variant> <variant> ..." [steps] [rounds]
# variant "base" = ocean_hip/liboceanhip.so, else ocean_hip/liboceanhip_<variant>.so
# (make -C ocean-simulation_amd VARIANT=<variant> EXTRA=-D...).  Prints value + kernel us.
set -e
mkdir -p gpurun_out
for r in $(seq 1 ${4:-2}); do
  for v in $2; do
    lib=ocean-simulation_amd/ocean_hip/liboceanhip.so
    [ "$v" != base ] && lib=ocean-simulation_amd/ocean_hip/liboceanhip_$v.so
    OCEAN_HIP_LIB=$PWD/$lib timeout -k 10 300 python bench.py --config $1 --steps ${3:-300} --warmup 20 \
      --no-cpu-baseline --no-ifft-stage --no-beyond-cache --no-update-loop > gpurun_out/ab_$v.json 2> gpurun_out/ab_$v.err
    echo "$r $v $(python -c "import json;d=json.load(open('gpurun_out/ab_$v.json'));print(d['value'],d['kernels_us'])")"
  done
done
