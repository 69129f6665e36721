#!/bin/bash
# usage: tools/gpu_rp_ablate.sh <tag> — row pass time with parts skipped (KB_DEV bits; results are wrong by design)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${1:-rpab}
mkdir -p $OUT
for dv in ${DVS:-0 2 4 8 14 15}; do
  KB_DEV=$dv timeout -k 10 200 python3 tools/quick_perf.py 65536 20 sim lat > $OUT/q_$dv.log 2>&1 || { tail -3 $OUT/q_$dv.log; }
  echo "dev=$dv: $(grep N= $OUT/q_$dv.log)"
done
