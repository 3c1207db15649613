"""diagnostic: per-wave phase breakdown of chain2aln_fast_kernel (trace-gated stamps)"""
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
b = synth_batch(ref, 1000, 35000, 150)
bs = bench.split_batches(b, 10_000_000)
d = bench.DevBatch(bs[0], dev)
st = torch.cuda.Stream(device=dev); torch.cuda.set_stream(st)
for _ in range(3): d.run(eng, st.cuda_stream)
torch.cuda.synchronize()
tr = torch.zeros(3 * 65536 * 8, dtype=torch.int32, device=dev)
eng.lib.bwagpu_debug_set_trace(eng.ctx, tr.data_ptr())
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
e0.record(st); d.run(eng, st.cuda_stream); e1.record(st); torch.cuda.synchronize()
eng.lib.bwagpu_debug_set_trace(eng.ctx, None)
t = tr.cpu().numpy().view(np.uint32).reshape(3, 65536, 8).astype(np.float64)
t[:, :, :7] /= 100.0  # us
out = {"launch_ms_traced": e0.elapsed_time(e1)}
names = ["desc+ticket", "contain", "fill", "dp", "tail", "contents", "first_grab", "reads"]
for v in range(2):
    x = t[v]
    live = x.sum(1) > 0
    x = x[live]
    if len(x) == 0:
        continue
    out[f"variant{v}"] = dict(waves=int(len(x)), mean_us={n: round(float(x[:, k].mean()), 2) for k, n in enumerate(names)},
                              total_mean_us=round(float(x.sum(1).mean()), 1), total_max_us=round(float(x.sum(1).max()), 1))
print(json.dumps(out, indent=1))
