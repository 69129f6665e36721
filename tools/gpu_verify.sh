#!/bin/bash
# usage: tools/gpu_verify.sh <tag> — the RCCL rank path on one GPU (1-rank communicator, full bench
# workload), then the sweep's HIP-event duration against rocprofv3's for the same command
set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${1:-verify}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python -u bench.py --rank-mesh --steps 10 --warmup 3 --no-cpu --no-conv > $OUT/rank_mesh.json 2> $OUT/rank_mesh.err
rc=$?; cat $OUT/rank_mesh.json; tail -3 $OUT/rank_mesh.err; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/$OUT/prof" -o run --output-format csv -- \
  python3 bench.py --steps 20 --warmup 5 --no-cpu --no-conv > $OUT/prof_bench.json 2> $OUT/prof_bench.err || exit $?
python3 tools/prof_summary.py stats $OUT/prof > $OUT/stats.txt; head -4 $OUT/stats.txt
python3 -c "import json; print('event avg_launch_ms', json.load(open('$OUT/prof_bench.json'))['roofline']['avg_launch_ms'])"
