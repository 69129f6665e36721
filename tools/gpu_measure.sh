#!/bin/bash
# usage: tools/gpu_measure.sh <tag> [pmc]
# On the GPU box: the driver's bench command, then rocprofv3 kernel-trace statistics of the same command
# (per-round kernel time over the timed rounds), and with `pmc` the two HBM counter passes
# (FETCH_SIZE, WRITE_SIZE cannot share a pass on gfx950) summarised per kernel over the timed rounds.
# Everything lands in gpurun_out/<tag>/.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
TAG=${1:-measure}; PMC=${2:-}
OUT=gpurun_out/$TAG; mkdir -p $OUT
export TMPDIR=/tmp
STEPS=20; WARM=5
CMD="bench.py --gpus 1 --steps $STEPS --warmup $WARM"
timeout -k 10 400 python3 $CMD > $OUT/bench.json 2> $OUT/bench.err || { tail -20 $OUT/bench.err; exit 1; }
tail -c 600 $OUT/bench.json; echo
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/$OUT/prof" -o run --output-format csv -- \
  python3 $CMD --no-cpu --no-conv --no-modes > $OUT/prof_bench.json 2> $OUT/prof_bench.err || { tail -20 $OUT/prof_bench.err; exit 1; }
python3 tools/prof_summary.py stats $OUT/prof > $OUT/kernel_stats.txt
python3 tools/prof_summary.py rounds $OUT/prof $WARM $STEPS > $OUT/kernel_rounds.json || exit 1
head -12 $OUT/kernel_stats.txt
if [ "$PMC" = pmc ]; then
  for c in FETCH_SIZE WRITE_SIZE; do
    timeout -s KILL 300 rocprofv3 --pmc $c --kernel-trace -d "$GRAFT_REPO_ROOT/$OUT/$c" -o run --output-format csv -- \
      python3 $CMD --no-cpu --no-conv --no-modes > $OUT/$c.log 2>&1 || { tail -20 $OUT/$c.log; exit 1; }
  done
  CAP=$(python3 -c "import json;print(json.load(open('$OUT/bench.json'))['config']['capacity'])")
  WL=$(python3 -c "import json;print(json.load(open('$OUT/bench.json'))['config']['workload'])")
  A3=$(python3 -c "import json;print(json.load(open('$OUT/bench.json'))['config']['a3_order'])")
  python3 tools/prof_summary.py pmc $OUT "{\"workload\": \"$WL\", \"capacity\": $CAP, \"steps\": $STEPS, \"warmup\": $WARM, \"failed_mode\": \"sim_sender\", \"a3_order\": \"$A3\", \"command\": \"python3 $CMD\"}" > $OUT/pmc.json || exit 1
  head -30 $OUT/pmc.json
fi
