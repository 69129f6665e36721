#!/bin/bash
# usage: tools/gpu_final.sh <tag>: PMC HBM traffic of the row pass and fold (2 counter passes), the
# bench line with that traffic, and the rocprofv3 kernel statistics of the bench command.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
TAG=${1:-r02final}
OUT=gpurun_out/$TAG; mkdir -p $OUT
export TMPDIR=/tmp
bash tools/gpu_pmc.sh $TAG/pmc > $OUT/pmc.log 2>&1 || { tail -20 $OUT/pmc.log; exit 1; }
for f in $OUT/pmc/pmc_*.json; do cp "$f" "profiles/${TAG}_$(basename $f)"; done
ls profiles/${TAG}_pmc_*.json
timeout -k 10 600 python3 bench.py > $OUT/bench.json 2> $OUT/bench.err || { tail -20 $OUT/bench.err; exit 1; }
cat $OUT/bench.json
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/$OUT/prof" -o run --output-format csv -- \
  python3 bench.py --no-cpu --no-conv --no-modes > $OUT/prof_bench.json 2> $OUT/prof_bench.err || { tail -20 $OUT/prof_bench.err; exit 1; }
python3 tools/prof_summary.py stats $OUT/prof 50 > $OUT/kernel_stats.txt
head -30 $OUT/kernel_stats.txt
