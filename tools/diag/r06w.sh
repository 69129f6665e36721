set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r06w; mkdir -p $O
KB_LIB_PATH=kaboodle_amd/variants/f5.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py -m gpu -x -q --timeout 120 --timeout-method thread -k "every_round or horizon or wide" > $O/pytest_f5.log 2>&1 &&
tail -1 $O/pytest_f5.log &&
bash tools/ab_run.sh r06w fin f5 && for f in gpurun_out/r06w/*.[12].log; do echo "$(basename $f) $(grep -o 'wall [0-9.]* ms/round' $f) $(grep -o 'fold [0-9.]* ms' $f) $(grep -o 'round(ev) [0-9.]* ms' $f)"; done
