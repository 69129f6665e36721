set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r06q; mkdir -p $O
KB_LIB_PATH=kaboodle_amd/variants/r4u3.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_bigmesh.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_r4u3.log 2>&1 &&
tail -2 $O/pytest_r4u3.log &&
bash tools/ab_run.sh r06q new r4u4 r4u3 r4u2 r3u4 && for f in gpurun_out/r06q/*.log; do echo "$f $(grep -o 'k_resp_wave [0-9.]*' $f)"; done
