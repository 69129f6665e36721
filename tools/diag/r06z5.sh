set -o pipefail
cd $GRAFT_REPO_ROOT
bash tools/ab_run.sh r06z5 fin w7 && for f in gpurun_out/r06z5/*.[12].log; do echo "$(basename $f .log) $(grep -o 'wall [0-9.]* ms/round' $f) $(grep -o 'fold [0-9.]* ms' $f) $(grep -o 'round(ev) [0-9.]* ms' $f)"; done
