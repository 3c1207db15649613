"""diagnostic: per-read timeline of one chain2aln launch"""
import sys, os, json
sys.path.insert(0, 'bwa-flow_amd/python'); sys.path.insert(0, '.')
import numpy as np, torch
from bwagpu import abi
from bwagpu.engine import Engine
from bwagpu.synth import SynthRef, synth_batch
import bench
dev = torch.device('cuda', 0)
ref = SynthRef(42, 46_709_983, 1)
pac_t = torch.from_numpy(ref.pac).to(dev)
eng = Engine(0, abi.default_opt(), ref.l_pac, ref.ann_offset, ref.ann_len, pac_device_ptr=pac_t.data_ptr())
b = synth_batch(ref, 1000, 35000, int(os.environ.get('RL', '150')))
bs = bench.split_batches(b, 10_000_000)
d = bench.DevBatch(bs[0], dev)
st = torch.cuda.Stream(device=dev); torch.cuda.set_stream(st)
for _ in range(3): d.run(eng, st.cuda_stream)
torch.cuda.synchronize()
tr = torch.zeros(d.b.n_reads * 8, dtype=torch.int32, device=dev)
eng.lib.bwagpu_debug_set_trace(eng.ctx, tr.data_ptr())
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
e0.record(st); d.run(eng, st.cuda_stream); e1.record(st); torch.cuda.synchronize()
eng.lib.bwagpu_debug_set_trace(eng.ctx, None)
t = tr.cpu().numpy().view(np.uint32).reshape(-1, 8).astype(np.int64)
t0 = t[:, 0] | (t[:, 1] << 32); t1 = t[:, 2] | (t[:, 3] << 32)
ok = t0 > 0
base = t0[ok].min()
s = (t0 - base) / 100.0; e = (t1 - base) / 100.0; dur = e - s  # microseconds
out = dict(kernel_ms=e0.elapsed_time(e1), n_reads=int(ok.sum()), span_us=float(e[ok].max()),
           dur_us_pct=[float(np.percentile(dur[ok], q)) for q in (50, 90, 99, 99.9, 100)],
           rows_pct=[float(np.percentile(t[ok, 4], q)) for q in (50, 90, 99, 100)],
           us_per_row_median=float(np.median(dur[ok & (t[:, 4] > 0)] / t[ok & (t[:, 4] > 0), 4])),
           start_us_pct=[float(np.percentile(s[ok], q)) for q in (0, 50, 90, 99, 100)],
           end_us_pct=[float(np.percentile(e[ok], q)) for q in (50, 90, 99, 100)])
# concurrency over time
grid = np.linspace(0, out['span_us'], 41)
out['active_reads_over_time'] = [int(((s[ok] <= g) & (e[ok] > g)).sum()) for g in grid]
print(json.dumps(out))
np.save('gpurun_out/trace.npy', t)
