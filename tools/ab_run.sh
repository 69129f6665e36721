#!/bin/bash
# On the GPU box: quick_perf (64K, the bench's workload with the latency EWMA, 25 rounds after 2) for each
# variant library, twice, alternating.  tools/ab_run.sh OUTDIR variant...   (KB_AB_ARGS: extra quick_perf args,
# default "lat exact": the bench's A3 order)
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/$1; shift
mkdir -p $OUT
for rep in 1 2; do
  for v in "$@"; do
    KB_LIB_PATH=kaboodle_amd/variants/$v.so timeout -k 10 120 python3 tools/quick_perf.py 65536 25 sim ${KB_AB_ARGS:-lat exact} > $OUT/$v.$rep.log 2>&1 || { tail -5 $OUT/$v.$rep.log; exit 1; }
    echo "$v.$rep: $(grep 'wall' $OUT/$v.$rep.log)"
  done
done
