#!/bin/bash
# usage: tools/gpu_ab.sh <tag> [ENV=VAL ...] — GPU parity tests, then for the baseline and each
# ENV=VAL variant: quick timing and a rocprofv3 kernel-trace summary of a short bench (dev A/B loop)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
TAG=${1:-ab}; shift
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1
rc=$?; tail -5 $OUT/pytest_gpu.log; [ $rc -ne 0 ] && exit $rc
n=0
for v in BASE "$@"; do
  n=$((n+1))
  if [ "$v" = BASE ]; then E=""; else E="$v"; fi
  env $E timeout -k 10 200 python tools/quick_perf.py 65536 20 > $OUT/perf_$n.log 2>&1 || exit 1
  echo "[$v] $(grep N= $OUT/perf_$n.log)"
  # rocprofv3 must exec python directly: the variant goes in through the environment of this shell
  ([ -n "$E" ] && export $E; timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/$OUT/prof_$n" -o run --output-format csv -- \
    python3 bench.py --steps 20 --warmup 5 --no-cpu --no-conv > $OUT/bench_$n.json 2> $OUT/bench_$n.err) || exit 1
  python3 tools/prof_summary.py stats $OUT/prof_$n > $OUT/stats_$n.txt; head -12 $OUT/stats_$n.txt
done
