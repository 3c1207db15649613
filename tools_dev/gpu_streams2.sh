set -o pipefail
TAG=${1:-streams2}
cd $GRAFT_REPO_ROOT
OUT=$GRAFT_REPO_ROOT/gpurun_out/$TAG
mkdir -p $OUT
for a in "--streams 1" "--streams 1 --no-prof" "--streams 2 --no-prof" "--streams 4 --no-prof"; do
timeout -k 10 200 python bench.py --no-cpu --no-cigar --no-host-path $a --steps 40 > $OUT/b.json 2> $OUT/b.err || { tail $OUT/b.err; exit 1; }
python3 -c "import json; d=json.load(open('$OUT/b.json')); print('$a', d['value'], d['ms_per_step'], d['parity_all_steps'], d['roofline']['avg_launch_ms'], d['roofline_hbm']['launch_sequence_ms'])"
done
