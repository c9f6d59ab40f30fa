# A/B of env settings on one bench config: bash tools/ab_cfg.sh cfg5 "<env,env> <env> ..." [steps]
set -e
mkdir -p gpurun_out
i=0
for cfg in $2; do
  i=$((i+1))
  env $(echo $cfg | tr ',' ' ') timeout -k 10 300 python bench.py --config $1 --steps ${3:-20} --warmup 3 --no-cpu-baseline --no-ifft-stage --no-beyond-cache > gpurun_out/abc_$i.json 2> gpurun_out/abc_$i.err
  echo "$cfg $(python -c "import json;d=json.load(open('gpurun_out/abc_$i.json'));print(d['value'],d['kernels_us'])")"
done
