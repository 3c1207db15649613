#!/usr/bin/env python3
"""The c5_refseed batch's speculative-path counters (bwagpu_debug_spec_counters):
tasks of rounds A / B / C, inline extensions (final-pass and redo misses),
heavy reads, redo reads; and the batch alone on one stream, timed."""
import ctypes as C
import json
import os
import sys
import time

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
eng = Engine(0, opt5, gref.l_pac, gref.ann_offset, gref.ann_len, pac_device_ptr=pac_t.data_ptr())
eng.set_device_read_len(int(np.diff(rb.batch.seq_off).max()))
st = torch.cuda.Stream()
d = bench.DevBatch(rb.batch, dev)
for rep in range(3):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    d.run(eng, st.cuda_stream, 0, stats=False)
    torch.cuda.synchronize()
    ms = (time.perf_counter() - t0) * 1e3
sc = np.zeros(8, np.int64)
assert eng.lib.bwagpu_debug_spec_counters(eng.ctx, C.c_void_p(st.cuda_stream), sc.ctypes.data_as(C.c_void_p)) == 0
print(json.dumps({"tasks_a_b_c": [int(x) for x in sc[:3]], "inline_extensions": int(sc[4]), "heavy_reads": int(sc[5]),
                  "redo_reads": int(sc[6]), "one_stream_ms": round(ms, 3), "parity": bool(rb.check(*d.results(0)))}))
