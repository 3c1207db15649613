#!/bin/bash
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/q9


bash tools_dev/gpu_quad.sh quad9
