set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r06r; mkdir -p $O
export KB_LIB_PATH=kaboodle_amd/variants/cur.so
KB_DEBUG_WAVES=1 KB_DEV=512 timeout -k 10 120 python3 tools/quick_perf.py 65536 8 sim lat exact > $O/phases.log 2>&1 && grep "k_resp_wave" $O/phases.log | tail -3 &&
for rep in 1 2; do
  for fl in 0 64; do
    KB_QP_DBG=$fl timeout -k 10 120 python3 tools/quick_perf.py 65536 25 sim lat exact > $O/f$fl.$rep.log 2>&1 || exit 1
    echo "f$fl.$rep $(grep wall $O/f$fl.$rep.log | cut -c1-40) $(grep -o 'k_resp_wave [0-9.]*' $O/f$fl.$rep.log)"
  done
done
