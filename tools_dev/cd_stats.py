"""diagnostic (build with -DBWAGPU_CD_STATS): DP rows/cells/calls per segment count CD"""
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
tr = torch.zeros(1 << 20, dtype=torch.int32, device=dev)
eng.lib.bwagpu_debug_set_trace(eng.ctx, tr.data_ptr())
d.run(eng, st.cuda_stream); torch.cuda.synchronize()
eng.lib.bwagpu_debug_set_trace(eng.ctx, None)
t = tr.cpu().numpy()[:4 * 17].view(np.uint32).reshape(17, 4)
print(json.dumps({f"CD{k}": dict(rows=int(t[k, 0]), cells=int(t[k, 1]), calls=int(t[k, 2])) for k in range(1, 17) if t[k, 2]}))
