# A/B timing of the operator IFFT kernels: bash tools/ab_ifft.sh "<env,env> <env> ..."
set -e
for cfg in $1; do
  echo "$cfg $(env $(echo $cfg | tr ',' ' ') timeout -k 10 120 python tools/ifft_bench.py 100)"
done
