#!/bin/bash
# usage: tools/gpu_bench_par.sh <tag> [pytest files...] — short bench line (no CPU leg) + GPU parity files
set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${1:-bp}; shift
mkdir -p $OUT
timeout -k 10 300 python3 bench.py --no-cpu --no-conv > $OUT/bench.json 2> $OUT/bench.err || { tail -20 $OUT/bench.err; exit 1; }
python3 -c "import json,sys; d=json.load(open('$OUT/bench.json')); print('value', d['value'], 'ms', d['ms_per_step'], 'gpu', d['round_gpu_ms'], 'rowpass', d['roofline']['avg_launch_ms'], 'sock', d['modes']['socket_faithful']['ms_per_step'])"
F=${@:-tests/test_gpu_parity.py}
timeout -k 10 700 python -u -m pytest -x -q --timeout 120 --timeout-method thread $F > $OUT/pytest.log 2>&1
rc=$?; tail -3 $OUT/pytest.log; exit $rc
