#!/bin/bash
# Round-3 closing measurements on the GPU box -> gpurun_out/r03z (copied into profiles/r03z by hand):
# part 1: -m gpu suite, smoke, default bench line, rocprofv3 of the cfg3 frame (trace + FETCH + WRITE),
# the chip ceilings the bench line quotes (wrbench, aqbench, bqbench).
set -o pipefail
O=gpurun_out/r03z; mkdir -p $O
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit 2
timeout -k 10 60 ./tools/wrbench > $O/wrbench.txt 2>&1 || exit 3
timeout -k 10 60 ./tools/aqbench > $O/aqbench.txt 2>&1 || exit 4
timeout -k 10 60 ./tools/bqbench > $O/bqbench.txt 2>&1 || exit 5
bash tools/profile.sh r03z || exit 6
echo done
