#!/usr/bin/env python3
"""c5_refseed leg alone (bench.c5_refseed_stage) in a fresh process."""
import json, os, sys
REPO = os.path.normpath(os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
sys.path.insert(0, REPO)
import bench  # noqa: E402  (sets GPU_MAX_HW_QUEUES before torch)
import torch  # noqa: E402
from bwagpu import workload  # noqa: E402
dev = torch.device("cuda:0")
opt, gref, rbs = workload.load_fixture(with_ref=True)
pac_t = torch.from_numpy(gref.pac).to(dev)
for _ in range(2):
    r = bench.c5_refseed_stage(pac_t, gref, dev)
    print(json.dumps({k: r.get(k) for k in ("ms_per_batch", "value", "gcups", "parity_all_steps")}), flush=True)
