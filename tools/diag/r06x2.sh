set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r06x
bash tools/final_conv.sh r06x/conv > gpurun_out/r06x/conv.log 2>&1 &&
bash tools/final_extra.sh r06x/extra > gpurun_out/r06x/extra.log 2>&1
