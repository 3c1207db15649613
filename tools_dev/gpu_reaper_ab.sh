# A/B of the drop-in stage's chain frees (BWAGPU_CHAIN_REAPER): one background
# reaper thread vs inline on each stage worker; end_to_end leg of bench.py,
# after the host-stage tests.  usage (on the GPU box): bash tools_dev/gpu_reaper_ab.sh <tag>
set -o pipefail
TAG=${1:-reaper}
cd $GRAFT_REPO_ROOT
OUT=$GRAFT_REPO_ROOT/gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_host_stage.py -x -v --timeout 120 --timeout-method thread > $OUT/host_stage.log 2>&1 || { tail -30 $OUT/host_stage.log; exit 1; }
tail -1 $OUT/host_stage.log
for rep in 1 2; do
  BWAGPU_CHAIN_REAPER=0 timeout -k 10 200 python -u bench.py --no-cpu --no-cigar --no-seeding --steps 5 > $OUT/off$rep.json 2> $OUT/off$rep.err || { tail $OUT/off$rep.err; exit 2; }
  timeout -k 10 200 python -u bench.py --no-cpu --no-cigar --no-seeding --steps 5 > $OUT/on$rep.json 2> $OUT/on$rep.err || { tail $OUT/on$rep.err; exit 3; }
done
for f in off1 on1 off2 on2; do python3 -c "import json; d=json.load(open('$OUT/$f.json'))['end_to_end']; print('$f', d['value'], d['wall_s'], d['phases'], d['parity_last_rep'])"; done
