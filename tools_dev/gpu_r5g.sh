#!/bin/bash
# round-5 change check: issue microbenchmark, the touched tests, the bench
set -o pipefail
T=${1:-r5f}
OUT=$GRAFT_REPO_ROOT/gpurun_out/$T
mkdir -p $OUT
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
ISSUE_MODE0=14 timeout -k 10 200 ./tools_dev/micro/issue > $OUT/issue.json || { echo issue failed; exit 1; }
timeout -k 10 400 python -u bench.py --no-cpu --no-cigar --no-e2e --no-seeding --no-regime > $OUT/b.json 2> $OUT/b.err || { tail $OUT/b.err; exit 3; }
python3 -c "
import json;d=json.load(open('$OUT/b.json'));r=d['roofline']
print('bench', d['value'], d['ms_per_step'], d['parity_all_steps'], r['kernel'], r.get('kernel_ms_per_step'), r['frac'], r['frac_pk16'], r['alg_bytes_per_launch'], r['traffic_over_alg'])
print('host_buffer_path', d.get('host_buffer_path'))
print('end_to_end', json.dumps(d.get('end_to_end')))"
# side-stream A/B: 0 = a plain side stream (default), 3 = none (heavy selection after the light on one stream)
for p in 3 0; do
  BWAGPU_SIDE_PRIO=$p timeout -k 10 300 python -u tools_dev/regime_state_ab.py > $OUT/st$p.json 2> $OUT/st$p.err || { tail $OUT/st$p.err; exit 4; }
  echo "side $p" $(cat $OUT/st$p.json)
  BWAGPU_SIDE_PRIO=$p timeout -k 10 300 python -u tools_dev/regime_ab.py --modes c2alt,c2b0,c3r > $OUT/ab$p.json 2> $OUT/ab$p.err || { tail $OUT/ab$p.err; exit 5; }
  echo "side $p" $(cat $OUT/ab$p.json)
done
for bl in 2 1; do
  BWAGPU_EXT2_BLOCKS_PER_CU=$bl timeout -k 10 300 python -u bench.py --no-cpu --no-cigar --no-host-path --no-e2e --no-seeding --no-regime > $OUT/bb$bl.json 2> $OUT/bb$bl.err || { tail $OUT/bb$bl.err; exit 6; }
  python3 -c "
import json;d=json.load(open('$OUT/bb$bl.json'));r=d['roofline']
print('blocks/CU $bl', d['value'], d['ms_per_step'], d['parity_all_steps'], r['kernel_ms_per_step'], r['isolated_launch_ms'])"
done
# caller streams x side stream
for ns in 3 4; do
for p in 3 0; do
  BWAGPU_SIDE_PRIO=$p timeout -k 10 300 python -u bench.py --no-cpu --no-cigar --no-host-path --no-e2e --no-seeding --no-regime --streams $ns > $OUT/bs$ns$p.json 2> $OUT/bs$ns$p.err || { tail $OUT/bs$ns$p.err; exit 7; }
  python3 -c "
import json;d=json.load(open('$OUT/bs$ns$p.json'));r=d['roofline']
print('streams $ns side $p', d['value'], d['ms_per_step'], d['parity_all_steps'], r['kernel_ms_per_step'])"
done
done
bash tools_dev/gpu_strace.sh r5f_strace || exit 8
