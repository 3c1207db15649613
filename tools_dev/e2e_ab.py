#!/usr/bin/env python3
"""The drop-in stage end to end (bench.end_to_end_stage) under a few host
settings: stage workers (contexts), reaper threads, chain ownership.
    python tools_dev/e2e_ab.py"""
import json
import os
import sys

REPO = os.path.normpath(os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "bwa-flow_amd", "python"))
import bench  # noqa: E402
from bwagpu import workload  # noqa: E402

opt, gref, rbs = workload.load_fixture(with_ref=True)
batches = [rb.batch for rb in rbs]
for workers in (2, 3, 4):
    for mode in (1, 0):
        r = bench.end_to_end_stage(opt, gref, batches, rbs, workers=workers, chain_mode=mode)
        print(json.dumps({"workers": workers, "chain_mode": mode, "reaper": os.environ.get("BWAGPU_REAPER_THREADS"),
                          "value": r.get("value"), "parity": r.get("parity_last_rep"), "per": r.get("ms_per_record"),
                          "err": r.get("error")}), flush=True)
