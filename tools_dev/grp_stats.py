"""diagnostic (library built with -DBWAGPU_GRP_STATS, BWAGPU_LIB pointing at it):
chain2aln_grp_kernel wave time split into control vs DP rows and the mean
number of groups per DP row iteration, for one C2 batch"""
import sys, json
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
d = bench.DevBatch(bench.split_batches(b, 10_000_000)[0], dev)
st = torch.cuda.Stream(device=dev); torch.cuda.set_stream(st)
d.run(eng, st.cuda_stream); torch.cuda.synchronize()
tr = torch.zeros(1 << 20, dtype=torch.int32, device=dev)
eng.lib.bwagpu_debug_set_trace(eng.ctx, tr.data_ptr())
d.run(eng, st.cuda_stream); torch.cuda.synchronize()
eng.lib.bwagpu_debug_set_trace(eng.ctx, None)
T = tr.cpu().numpy()[:8 * 17].view(np.uint32).astype(np.int64).reshape(17, 8)
for cpl in range(17):
    t = T[cpl]
    if not t[4]:
        continue
    ctrl, dp, it, gr, waves = t[0] * 256, t[1] * 256, t[2], t[3], t[4]
    print(json.dumps(dict(cpl=cpl, waves=int(waves), ctrl_cycles_per_wave=float(ctrl / waves),
                          dp_cycles_per_wave=float(dp / waves), row_iters_per_wave=float(it / waves),
                          groups_per_row_iter=float(gr / max(it, 1)), dp_cycles_per_row_iter=float(dp / max(it, 1)))))
