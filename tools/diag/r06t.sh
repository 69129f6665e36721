set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r06t; mkdir -p $O
KB_LIB_PATH=kaboodle_amd/variants/a3s.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py -m gpu -x -q --timeout 120 --timeout-method thread -k "exact or horizon or wide" > $O/pytest_a3s.log 2>&1 &&
tail -2 $O/pytest_a3s.log &&
bash tools/ab_run.sh r06t fin a3s a3s8 && for f in gpurun_out/r06t/*.[12].log; do echo "$(basename $f) $(grep -o 'wall [0-9.]* ms/round' $f) $(grep -o 'round(ev) [0-9.]* ms' $f)"; done
