#!/bin/bash
# On the GPU box: the driver's bench (timed part only) for each variant library, twice, alternating.
# tools/ab_bench.sh OUTDIR variant...
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/$1; shift
mkdir -p $OUT
for rep in 1 2; do
  for v in "$@"; do
    KB_LIB_PATH=kaboodle_amd/variants/$v.so timeout -k 10 200 python3 bench.py --no-cpu --no-conv --no-modes --seeds "" --no-replay > $OUT/$v.$rep.json 2> $OUT/$v.$rep.err || { tail -5 $OUT/$v.$rep.err; exit 1; }
    python3 -c "import json;d=json.load(open('$OUT/$v.$rep.json'));print('$v.$rep', round(d['value']/1e6,3), round(d['ms_per_step'],3), {k:v['ms_per_round'] for k,v in list(d['kernels'].items())[:5]})"
  done
done
