#!/bin/bash
# usage: tools/gpu_pmc.sh <tag> [bench args...]   (summaries for k_rowpass<true> and k_fold)
# Two counter passes over the bench workload (FETCH_SIZE and WRITE_SIZE cannot share a pass on gfx950),
# kernel-trace only (no runtime/sys trace with --pmc on this pool).  Summary -> gpurun_out/<tag>/pmc.json
set -o pipefail
cd "$GRAFT_REPO_ROOT"
TAG=${1:-pmc}; shift
mkdir -p gpurun_out/$TAG
export TMPDIR=/tmp
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 500 rocprofv3 --pmc $c --kernel-trace -d "$GRAFT_REPO_ROOT/gpurun_out/$TAG/$c" -o run \
    --output-format csv -- python3 bench.py --no-cpu --no-conv --no-modes "$@" > gpurun_out/$TAG/$c.log 2>&1 || exit $?
done
for k in "k_rowpass<true>" k_fold; do
  f=gpurun_out/$TAG/pmc_$(echo $k | tr -d '<>').json
  python3 tools/prof_summary.py pmc gpurun_out/$TAG "$k" "$@" > $f && cat $f
done
