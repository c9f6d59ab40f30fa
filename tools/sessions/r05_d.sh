#!/bin/bash
# Round 5, session d: the in-place 4096 operator (k_rowsf onto the planes + k_colsf_ip):
# its parity tests, then A/B against the scratch operator (liboceanhip_prev.so) on 4 x 4096^2 x 4 planes,
# three alternating rounds, and the chunk sweep.
set -o pipefail
OUT=gpurun_out/r05_d; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -q -x --timeout 200 --timeout-method thread \
  -k "operator_large or ifft2d_operator or delta_and_linearity or frames_vs_oracle and 4096" > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -2 $OUT/pytest.log
for r in 1 2 3; do
  for v in base prev; do
    lib=ocean-simulation_amd/ocean_hip/liboceanhip.so
    [ "$v" != base ] && lib=ocean-simulation_amd/ocean_hip/liboceanhip_$v.so
    OCEAN_HIP_LIB=$PWD/$lib timeout -k 10 120 python tools/ifft_op.py 4096 4 1 12 > $OUT/op_$v.json 2>> $OUT/op.err || exit 3
    echo "$r $v $(cat $OUT/op_$v.json)"
  done
done
for c in 128 512 1024; do
  OCEAN_OP_CHUNK_MIB=$c timeout -k 10 120 python tools/ifft_op.py 4096 4 1 12 > $OUT/op_c$c.json 2>> $OUT/op.err || exit 4
  echo "chunk $c $(cat $OUT/op_c$c.json)"
done
echo session done
