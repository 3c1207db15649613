#!/usr/bin/env python3
"""Host-buffer path, phase by phase: per batch the time in bwagpu_chain2aln_submit
(check, staging copy, launches) and in wait + results_dense, at 2 and 3 slots,
plus the submit alone on an idle device."""
import os
import sys
import time

REPO = os.path.normpath(os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
sys.path.insert(0, os.path.join(REPO, "bwa-flow_amd", "python"))
os.environ.setdefault("GPU_MAX_HW_QUEUES", "16")
import numpy as np  # noqa: E402
import torch  # noqa: E402

from bwagpu import workload  # noqa: E402
from bwagpu.engine import Engine  # noqa: E402

dev = torch.device("cuda:0")
opt, ref, rbs = workload.load_fixture()
bs = [rb.batch for rb in rbs]
pac_t = torch.from_numpy(np.ascontiguousarray(ref.pac)).to(dev)
eng = Engine(0, opt, ref.l_pac, ref.ann_offset, ref.ann_len, pac_device_ptr=pac_t.data_ptr())
for k in range(4):
    eng.submit(k, bs[k % 2])
    eng.wait_dense(k, bs[k % 2])
# submit alone, device idle
ts = []
for i in range(6):
    t0 = time.perf_counter()
    eng.submit(0, bs[i % 2])
    ts.append(time.perf_counter() - t0)
    torch.cuda.synchronize()
    t1 = time.perf_counter()
    eng.wait_dense(0, bs[i % 2])
    ts[-1] = (ts[-1], time.perf_counter() - t1)
print("idle device: submit ms", [round(a * 1e3, 3) for a, _ in ts], "wait_dense after sync ms", [round(b * 1e3, 3) for _, b in ts])
for depth in (2, 3, 4):
    n = 12
    sub, wt = [], []
    t0 = time.perf_counter()
    for i in range(depth - 1):
        eng.submit(i, bs[i % 2])
    for i in range(n):
        if i + depth - 1 < n:
            a = time.perf_counter()
            eng.submit((i + depth - 1) % depth, bs[(i + depth - 1) % 2])
            sub.append(time.perf_counter() - a)
            if sub[-1] > 3e-3:
                print(f"  depth {depth}: submit of batch {i + depth - 1} (slot {(i + depth - 1) % depth}) took {sub[-1] * 1e3:.2f} ms")
        a = time.perf_counter()
        eng.wait_dense(i % depth, bs[i % 2])
        wt.append(time.perf_counter() - a)
        if wt[-1] > 3e-3:
            print(f"  depth {depth}: wait of batch {i} (slot {i % depth}) took {wt[-1] * 1e3:.2f} ms")
    dt = time.perf_counter() - t0
    print(f"depth {depth}: ms/batch {dt * 1e3 / n:.3f} submit ms {np.mean(sub) * 1e3:.3f} (max {np.max(sub) * 1e3:.3f}) "
          f"wait ms {np.mean(wt) * 1e3:.3f} (max {np.max(wt) * 1e3:.3f})")
