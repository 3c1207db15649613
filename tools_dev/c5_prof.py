#!/usr/bin/env python3
"""The c5_refseed leg alone (BASELINE.json configs[4]: one mixed 2x100 / 2x150
/ 2x250 reference-seeded ChainsRecord), for kernel traces and PMC passes of
its extension kernels (bench.c5_refseed_stage, 10 steps, 2 streams)."""
import json
import os
import sys

REPO = os.path.normpath(os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
sys.path.insert(0, REPO)
import bench  # noqa: E402
import torch  # noqa: E402
from bwagpu import workload  # noqa: E402

dev = torch.device("cuda:0")
opt, ref, _ = workload.load_fixture()
pac_t = torch.from_numpy(ref.pac).to(dev)
print(json.dumps(bench.c5_refseed_stage(pac_t, ref, dev)))
