#!/bin/bash
# usage: tools/gpu_benchwaves.sh <tag> [mode] — per-wave kernel trace of the bench workload in its benched state
# (30 warmup rounds, then 8 traced rounds), plus the idle gaps between kernels
set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${1:-bw}; MODE=${2:-sim_sender}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace -d "$GRAFT_REPO_ROOT/$OUT/prof" -o run --output-format csv -- \
  python3 bench.py --no-cpu --no-conv --no-modes --failed-mode $MODE --warmup 30 --steps 8 > $OUT/bench.json 2> $OUT/bench.err || { tail -5 $OUT/bench.err; exit 1; }
f=$(find $OUT/prof -name "*kernel_trace.csv" | head -1)
python3 tools/wave_prof.py "$f" > $OUT/waves.txt; tail -24 $OUT/waves.txt
python3 tools/round_gaps.py "$f" | tail -4
