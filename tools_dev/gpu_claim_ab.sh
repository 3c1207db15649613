# A/B of spec_ext_kernel's claim size (BWAGPU_EXT_CLAIM 2 = lib/, 1 and 4 = alt builds)
# usage (on the GPU box): bash tools_dev/gpu_claim_ab.sh <tag>
set -o pipefail
TAG=${1:-claim}
cd $GRAFT_REPO_ROOT
OUT=$GRAFT_REPO_ROOT/gpurun_out/$TAG
mkdir -p $OUT
for rep in 1 2; do
  for L in lib alt_c1 alt_c4; do
    BWAGPU_LIB=$GRAFT_REPO_ROOT/bwa-flow_amd/$L/libbwagpu.so timeout -k 10 200 python -u bench.py --no-cpu --no-cigar --no-host-path --no-seeding > $OUT/$L.$rep.json 2> $OUT/$L.$rep.err || { tail $OUT/$L.$rep.err; exit 1; }
    python3 -c "import json; d=json.load(open('$OUT/$L.$rep.json')); print('$L', $rep, d['value'], d['ms_per_step'], d['parity_all_steps'], d['roofline']['avg_launch_ms'])"
  done
done
