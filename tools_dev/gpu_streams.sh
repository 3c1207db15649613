# bench.py at 1..4 streams (batches ping-ponged over that many slots)
set -o pipefail
TAG=${1:-streams}
cd $GRAFT_REPO_ROOT
OUT=$GRAFT_REPO_ROOT/gpurun_out/$TAG
mkdir -p $OUT
for s in 1 2 3 4; do
timeout -k 10 200 python bench.py --no-cpu --no-cigar --no-host-path --streams $s --steps 40 > $OUT/bench_s$s.json 2> $OUT/bench_s$s.err || { tail $OUT/bench_s$s.err; exit 1; }
python3 -c "import json; d=json.load(open('$OUT/bench_s$s.json')); print($s, d['value'], d['ms_per_step'], d['parity_all_steps'], d['roofline']['avg_launch_ms'])"
done
