"""diagnostic: per-task cells/rows/lane time of the lane-path extension kernels"""
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
nc = d.b.n_chains
tr = torch.zeros(max(2 * nc * 4, d.b.n_reads * 8), dtype=torch.int32, device=dev)
eng.lib.bwagpu_debug_set_trace(eng.ctx, tr.data_ptr())
d.run(eng, st.cuda_stream); torch.cuda.synchronize()
eng.lib.bwagpu_debug_set_trace(eng.ctx, None)
t = tr.cpu().numpy()[:2 * nc * 4].view(np.uint32).reshape(2, nc, 4).astype(np.int64)
out = {}
for side in range(2):
    x = t[side]
    n = int((x[:, 1] > 0).sum())  # tasks with rows
    x = x[:n] if n else x[:0]
    cells, rows, tus, blk = x[:, 0], x[:, 1], x[:, 2] / 100.0, x[:, 3]
    waves = {}
    for bb in np.unique(blk):
        m = blk == bb
        waves[int(bb)] = (cells[m].sum(), cells[m].max(), rows[m].max(), tus[m].max(), m.sum())
    W = np.array(list(waves.values()), dtype=np.float64)
    out[f"side{side}"] = dict(
        tasks=n, cells=int(cells.sum()), cells_pct=[float(np.percentile(cells, q)) for q in (50, 90, 99, 100)],
        rows_pct=[float(np.percentile(rows, q)) for q in (50, 90, 99, 100)],
        lane_us_pct=[float(np.percentile(tus, q)) for q in (50, 90, 99, 100)],
        waves=len(W), wave_us_pct=[float(np.percentile(W[:, 3], q)) for q in (50, 90, 99, 100)],
        util_cells_mean_over_max=float((W[:, 0] / (W[:, 4] * W[:, 1])).mean()),
        ns_per_cell_step=float(np.median(W[:, 3] * 1e3 / W[:, 1])))
print(json.dumps(out, indent=1))
