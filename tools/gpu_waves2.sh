#!/bin/bash
# usage: tools/gpu_waves2.sh <tag> — per-wave kernel trace of the aged 64K workload + the bench rank path
set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${1:-waves}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace -d "$GRAFT_REPO_ROOT/$OUT/prof" -o run --output-format csv -- \
  python3 tools/quick_perf.py 65536 12 > $OUT/quick.log 2>&1 || { tail -20 $OUT/quick.log; exit 1; }
f=$(find $OUT/prof -name "*kernel_trace.csv" | head -1)
python3 tools/wave_prof.py "$f" > $OUT/waves.txt; tail -60 $OUT/waves.txt
KB_DEBUG_WAVES=1 timeout -k 10 200 python3 tools/quick_perf.py 65536 6 > $OUT/debug_waves.log 2>&1 || exit 1
grep "round 7" $OUT/debug_waves.log | head -20
timeout -k 10 300 python3 -u bench.py --rank-mesh --steps 10 --warmup 3 --no-cpu > $OUT/bench_rank.json 2> $OUT/bench_rank.err
rc=$?; cat $OUT/bench_rank.json; tail -3 $OUT/bench_rank.err; exit $rc
