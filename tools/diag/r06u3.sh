set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r06u
bash tools/final_extra.sh r06u/extra > gpurun_out/r06u/extra.log 2>&1
