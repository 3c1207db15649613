# stream path C2 timing, claim 1 (lib/) vs claim 2 (alt_c2/), 2 reps each
set -o pipefail
TAG=${1:-streamab}
cd $GRAFT_REPO_ROOT
OUT=$GRAFT_REPO_ROOT/gpurun_out/$TAG
mkdir -p $OUT
for rep in 1 2; do
  for L in lib alt_c2; do
    BWAGPU_LIB=$GRAFT_REPO_ROOT/bwa-flow_amd/$L/libbwagpu.so timeout -k 10 200 python3 -u tools_dev/stream_bench.py > $OUT/$L.$rep.json 2> $OUT/$L.$rep.err || { tail $OUT/$L.$rep.err; exit 1; }
    python3 -c "import json; d=json.load(open('$OUT/$L.$rep.json')); print('$L', $rep, d['ms_per_call'], d['parity'])"
  done
done
