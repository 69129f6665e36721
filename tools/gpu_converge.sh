#!/bin/bash
# rounds to fingerprint convergence of configs[2] in both failed modes (tools/converge.py)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${1:-conv}; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 ${2:-300} python3 -u tools/converge.py --mode sock --budget-s $((${2:-300} - 40)) --out $OUT/converge_sock.json \
  2>&1 | tee $OUT/converge_sock.log
timeout -k 10 ${3:-800} python3 -u tools/converge.py --mode sim --budget-s $((${3:-800} - 40)) --out $OUT/converge_sim.json \
  2>&1 | tee $OUT/converge_sim.log
