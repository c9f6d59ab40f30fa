# A/B timing of pass-A variants on cfg3; usage: bash tools/ab_a3.sh "<env-assignments> ..." [pytest-env]
#   e.g. bash tools/ab_a3.sh "OCEAN_A3_VARIANT=0 OCEAN_A3_VARIANT=3,OCEAN_XCD_REMAP=0" OCEAN_A3_VARIANT=3
set -e
mkdir -p gpurun_out
i=0
for cfg in $1; do
  i=$((i+1))
  env $(echo $cfg | tr ',' ' ') timeout -k 10 120 python bench.py --steps 200 --warmup 20 > gpurun_out/ab_$i.json 2> gpurun_out/ab_$i.err
  echo "$cfg $(python -c "import json;d=json.load(open('gpurun_out/ab_$i.json'));print(d['value'],d['kernels_us'])")"
done
if [ -n "$2" ]; then env $(echo $2 | tr ',' ' ') timeout -k 10 300 python -m pytest tests -m gpu -x -q 2>&1 | tail -3; fi
