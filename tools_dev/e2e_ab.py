#!/usr/bin/env python3
"""The drop-in stage end to end (bench.end_to_end_stage) under host settings
given on the command line: stage workers (contexts) x slots in flight
(BWAGPU_STAGE_SLOTS, read once per process), chain ownership.
    BWAGPU_STAGE_SLOTS=2 python tools_dev/e2e_ab.py 1 2 3"""
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
for workers in [int(x) for x in sys.argv[1:]] or [2]:
    r = bench.end_to_end_stage(opt, gref, batches, rbs, workers=workers, chain_mode=1)
    print(json.dumps({"workers": workers, "slots": os.environ.get("BWAGPU_STAGE_SLOTS"),
                      "value": r.get("value"), "parity": r.get("parity_last_rep"), "per": r.get("ms_per_record"),
                      "err": r.get("error")}), flush=True)
