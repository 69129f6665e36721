#!/bin/bash
# A/B of KnownPeers group splits (KP_COLS 4 / 2 / 1): kernel time of k_kp_group per mode
set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${1:-abkp}; mkdir -p $OUT
export TMPDIR=/tmp
for v in "" _kp2 _kp1; do
  for mode in sim sock; do
    KB_LIB_PATH=$PWD/kaboodle_amd/libkaboodle_sim$v.so timeout -k 10 200 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/$OUT/p$v$mode" -o run --output-format csv -- \
      python3 tools/quick_perf.py 65536 12 $mode lat > $OUT/q$v$mode.log 2>&1 || { tail -5 $OUT/q$v$mode.log; exit 1; }
    echo "variant [$v] $mode: $(grep N= $OUT/q$v$mode.log)"
    f=$(find $OUT/p$v$mode -name "*kernel_stats.csv" | head -1)
    grep -E "k_kp_group|k_proc\b|\"k_proc\"" "$f" | cut -d, -f1-5
  done
done
