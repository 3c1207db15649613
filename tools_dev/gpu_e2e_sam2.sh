set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/e2esam2
timeout -k 10 400 python -u -m pytest tests/test_sam_parity.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/e2esam2/tests.log 2>&1 || { tail -30 gpurun_out/e2esam2/tests.log; exit 1; }
tail -1 gpurun_out/e2esam2/tests.log
bash tools_dev/gpu_e2e_sam.sh e2esam2 100000 16
