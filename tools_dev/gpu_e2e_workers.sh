# end_to_end leg with 1/2/3 stage workers on the device
set -o pipefail
TAG=${1:-e2ew}
cd $GRAFT_REPO_ROOT
OUT=$GRAFT_REPO_ROOT/gpurun_out/$TAG
mkdir -p $OUT
for W in 1 2 3 4; do
  BWAGPU_E2E_WORKERS=$W timeout -k 10 300 python bench.py --no-cpu --no-cigar --steps 10 > $OUT/b$W.json 2> $OUT/b$W.err || { tail $OUT/b$W.err; exit 1; }
  python3 -c "import json; d=json.load(open('$OUT/b$W.json')); e=d['end_to_end']; print('workers $W', e.get('value'), e.get('stage_workers'), e.get('phases'), e.get('parity_last_rep'), 'main', d['value'])"
done
