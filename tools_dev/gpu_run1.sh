set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -m pytest tests/test_gpu_parity.py -x -q > gpurun_out/gpu_tests.log 2>&1 || { echo "pytest failed rc=$?" >> gpurun_out/gpu_tests.log; exit 1; }
timeout -k 10 400 python bench.py --pairs 200000 --steps 12 --warmup 2 --cpu-budget 10 > gpurun_out/bench_small.json 2> gpurun_out/bench_small.err || exit 2
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof1 -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --pairs 200000 --steps 12 --warmup 2 --no-cpu > $GRAFT_REPO_ROOT/gpurun_out/prof1.log 2>&1 || exit 3
