set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r06z
bash tools/final_conv.sh r06z/conv > gpurun_out/r06z/conv.log 2>&1 &&
bash tools/final_extra.sh r06z/extra > gpurun_out/r06z/extra.log 2>&1
