#!/bin/bash
# On the GPU box: quick_perf (64K, the bench's workload with the latency EWMA) under kb_config.debug_flags values
# (kernel variants with identical results), alternating, twice.  tools/dbg_ab.sh OUTDIR flags...
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/$1; shift
mkdir -p $OUT
for rep in 1 2; do
  for f in "$@"; do
    KB_QP_DBG=$f timeout -k 10 120 python3 tools/quick_perf.py 65536 25 sim lat > $OUT/dbg$f.$rep.log 2>&1 || { tail -5 $OUT/dbg$f.$rep.log; exit 1; }
    echo "dbg$f.$rep: $(grep 'wall' $OUT/dbg$f.$rep.log)"
  done
done
