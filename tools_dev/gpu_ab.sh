# GPU A/B: parity tests (group kernels on), then bench with group kernels on and off
# usage: bash tools_dev/gpu_ab.sh <tag> [pytest -k expr]
set -o pipefail
TAG=${1:-ab}; K=${2:-}
cd $GRAFT_REPO_ROOT
OUT=$GRAFT_REPO_ROOT/gpurun_out/$TAG
mkdir -p $OUT
if [ -n "$K" ]; then KA="-k $K"; else KA=""; fi
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread $KA > $OUT/gpu_tests.log 2>&1 || { echo "pytest failed"; tail -40 $OUT/gpu_tests.log; exit 1; }
tail -3 $OUT/gpu_tests.log
timeout -k 10 200 python bench.py --pairs 300000 --steps 10 --warmup 2 --no-cpu --no-host-path > $OUT/bench_grp.json 2> $OUT/bench_grp.err || { tail -20 $OUT/bench_grp.err; exit 2; }
BWAGPU_C2A_GRP=0 timeout -k 10 200 python bench.py --pairs 300000 --steps 10 --warmup 2 --no-cpu --no-host-path > $OUT/bench_wave.json 2> $OUT/bench_wave.err || { tail -20 $OUT/bench_wave.err; exit 3; }
python - <<PY
import json
for k in ("grp","wave"):
    d=json.load(open("$OUT/bench_%s.json"%k))
    print(k, d["value"], "Mreads/s", d["ms_per_step"], "ms/batch", d.get("gcups"), "GCUPS", "parity", d.get("parity_batch0_vs_cpu"))
PY
