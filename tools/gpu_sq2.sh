#!/bin/bash
# usage: tools/gpu_sq2.sh <tag> — counter passes (SQ issue/LDS/VMEM, TA/TD busy) over the main kernels of a short 64K run
set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${1:-sq2}
mkdir -p $OUT
export TMPDIR=/tmp
rocprofv3 -L > $OUT/avail.txt 2>&1 || true
RX='k_fold|k_rowpass|k_resp_wave|k_proc|k_kp_group|k_scatter|k_route'
P1="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE"
P2="SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INST_CYCLES_VMEM SQ_INSTS_SALU TA_BUSY_avr TD_BUSY_avr"
n=0
for P in "$P1" "$P2"; do
  n=$((n+1))
  timeout -s KILL 200 rocprofv3 --pmc $P --kernel-include-regex "$RX" --kernel-trace -d "$GRAFT_REPO_ROOT/$OUT/p$n" -o run --output-format csv -- python3 tools/quick_perf.py 65536 6 sim lat > $OUT/p$n.log 2>&1 || { tail -5 $OUT/p$n.log; exit 1; }
  python3 tools/prof_summary.py sq $OUT/p$n > $OUT/p$n.txt; cat $OUT/p$n.txt
done
