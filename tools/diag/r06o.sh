set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r06o; mkdir -p $O
bash tools/ab_run.sh r06o base new &&
KB_LIB_PATH=kaboodle_amd/variants/new.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_bigmesh.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_new.log 2>&1 &&
tail -2 $O/pytest_new.log &&
for v in base new; do
  KB_LIB_PATH=kaboodle_amd/variants/$v.so timeout -s KILL 120 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_BUSY_CYCLES SQ_INSTS_SALU SQ_WAVES --kernel-trace -d "$GRAFT_REPO_ROOT/$O/lds_$v" -o run --output-format csv -- python3 tools/quick_perf.py 65536 6 sim lat exact > $O/lds_$v.log 2>&1 || exit 1
  python3 tools/prof_summary.py sq $O/lds_$v > $O/lds_$v.txt || exit 1
  grep -E "k_resp_wave|kernel" $O/lds_$v.txt
done
