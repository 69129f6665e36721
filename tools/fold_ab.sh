#!/bin/bash
# On the GPU box: the fold by decimal blocks vs by htab (KB_DEV=8192), quick_perf at 64K sim_sender with the
# latency EWMA, alternating, twice.  tools/fold_ab.sh OUTDIR
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/$1
mkdir -p $OUT
for rep in 1 2; do
  for v in dec htab; do
    dev=0; [ $v = htab ] && dev=8192
    KB_DEV=$dev timeout -k 10 120 python3 tools/quick_perf.py 65536 25 sim lat > $OUT/$v.$rep.log 2>&1 || { tail -5 $OUT/$v.$rep.log; exit 1; }
    echo "$v.$rep: $(grep 'wall' $OUT/$v.$rep.log)"
  done
done
