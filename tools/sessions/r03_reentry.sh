#!/bin/bash
# Round-3 re-entry check on HEAD -> gpurun_out/r03re: -m gpu suite, smoke, default bench line.
set -o pipefail
O=gpurun_out/r03re; mkdir -p $O
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit 2
timeout -k 10 300 python3 bench.py > $O/bench_cfg3.json 2> $O/bench_cfg3.err || exit 7
cat $O/bench_cfg3.json
echo done
