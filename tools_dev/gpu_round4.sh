#!/bin/bash
# Round-4 measurement on the GPU box, one tree: every -m gpu test, smoke(),
# the default bench line, kernel traces of the stage bench (2 and 1 caller
# streams), and the PMC passes (SQ issue/wait/LDS counters; FETCH_SIZE and
# WRITE_SIZE each alone).  Summaries are made from gpurun_out/ afterwards
# (tools_dev/trace_busy.py, pmc_round.py, pmc_traffic.py).
# usage (GPU box): bash tools_dev/gpu_round4.sh <tag> [nop]   (nop: without the trace and PMC passes,
# which tools_dev/gpu_round4_prof.sh <tag> runs as a call of its own)
set -o pipefail
T=${1:-r04}
cd $GRAFT_REPO_ROOT
OUT=$GRAFT_REPO_ROOT/gpurun_out/$T
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/ -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/gpu_tests.log 2>&1 || { echo "pytest failed"; tail -30 $OUT/gpu_tests.log; exit 1; }
tail -1 $OUT/gpu_tests.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { tail $OUT/smoke.log; exit 2; }
tail -1 $OUT/smoke.log
timeout -k 10 900 python -u bench.py > $OUT/bench.json 2> $OUT/bench.err || { tail $OUT/bench.err; exit 3; }
python3 -c "import json;d=json.load(open('$OUT/bench.json'));print(d['value'],d['ms_per_step'],d['parity_all_steps'])"
[ "$2" = "nop" ] || { bash tools_dev/gpu_trace.sh $T/trace || exit 4; bash tools_dev/gpu_pmc4.sh $T/pmc all || exit 5; }
echo done > $OUT/rc.txt
