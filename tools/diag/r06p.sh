set -o pipefail
cd $GRAFT_REPO_ROOT
bash tools/ab_run.sh r06p new u3 u5 u9 && grep -h "^kernels" gpurun_out/r06p/*.log
