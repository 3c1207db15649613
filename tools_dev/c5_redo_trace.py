#!/usr/bin/env python3
"""Per-read timeline of the c5_refseed batch's selection passes, the redo
pass (pass 2) included: which reads the redo pass takes, how long each takes
and how many extensions it computes inline (shape >> 4)."""
import json
import os
import sys

REPO = os.path.normpath(os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
sys.path.insert(0, REPO)
import bench  # noqa: E402
import numpy as np  # noqa: E402
import torch  # noqa: E402
from bwagpu import workload  # noqa: E402
from bwagpu.engine import Engine  # noqa: E402

dev = torch.device("cuda:0")
opt, gref, _ = workload.load_fixture(with_ref=True)
pac_t = torch.from_numpy(gref.pac).to(dev)
opt5, _, rbs = workload.load_fixture(workload.C5_FIXTURE, with_ref=False)
rb = rbs[0]
b = rb.batch
eng = Engine(0, opt5, gref.l_pac, gref.ann_offset, gref.ann_len, pac_device_ptr=pac_t.data_ptr())
lens = np.diff(b.seq_off)
eng.set_device_read_len(int(lens.max()))
st = torch.cuda.Stream()
d = bench.DevBatch(b, dev)
for _ in range(2):
    d.run(eng, st.cuda_stream, 0, stats=False)
torch.cuda.synchronize()
tr = torch.zeros(b.n_reads * 24, dtype=torch.int32, device=dev)
eng.lib.bwagpu_debug_set_trace(eng.ctx, C_ptr := __import__("ctypes").c_void_p(tr.data_ptr()))
d.run(eng, st.cuda_stream, 0, stats=False)
torch.cuda.synchronize()
eng.lib.bwagpu_debug_set_trace(eng.ctx, None)
T = tr.cpu().numpy().view(np.uint32).reshape(3, b.n_reads, 8).astype(np.int64)
out = {}
base = None
for ps, name in ((0, "emulate"), (1, "final"), (2, "redo")):
    t0 = T[ps, :, 0] | (T[ps, :, 1] << 32)
    t1 = T[ps, :, 2] | (T[ps, :, 3] << 32)
    m = t1 > 0
    if not m.any():
        out[name] = None
        continue
    if base is None:
        base = t0[m].min()
    dur = (t1 - t0)[m] / 100.0
    idx = np.nonzero(m)[0]
    top = np.argsort(-dur)[:12]
    out[name] = {"reads": int(m.sum()), "span_us": round(float((t1[m].max() - t0[m].min()) / 100.0), 1),
                 "start_us": round(float((t0[m].min() - base) / 100.0), 1),
                 "p50_us": round(float(np.percentile(dur, 50)), 2), "max_us": round(float(dur.max()), 1),
                 "slowest": [{"read": int(idx[k]), "len": int(lens[idx[k]]), "us": round(float(dur[k]), 1),
                              "seeds": int(T[ps, idx[k], 4]), "regions": int(T[ps, idx[k], 5]),
                              "inline": int(T[ps, idx[k], 7] >> 4)} for k in top]}
print(json.dumps(out, indent=1))
