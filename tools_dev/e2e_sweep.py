#!/usr/bin/env python3
"""The drop-in stage end to end (bench.py's end_to_end leg) under host-side
settings, each in a process of its own (the settings are read once):
BWAGPU_HOST_THREADS, BWAGPU_UNPACK_THREADS, BWAGPU_REAPER_THREADS,
BWAGPU_E2E_WORKERS, sink workers.  One JSON line per setting.
    python tools_dev/e2e_sweep.py [reps] [modes, e.g. 1,0] [rounds]     (GPU box)"""
import json
import os
import subprocess
import sys

REPO = os.path.normpath(os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
CHILD = r'''
import json, os, sys
sys.path.insert(0, %r)
import bench
from bwagpu import workload
opt, ref, rbs = workload.load_fixture()
r = bench.end_to_end_stage(opt, ref, [rb.batch for rb in rbs], rbs, reps=%d, chain_mode=%d, sink_workers=%d)
print(json.dumps(r))
'''
SETTINGS = [
    dict(BWAGPU_POST_THREADS="0"),
    dict(),
    dict(BWAGPU_REAPER_THREADS="4"),
    dict(BWAGPU_REAPER_THREADS="6"),
    dict(BWAGPU_POST_THREADS="6", BWAGPU_REAPER_THREADS="4"),
    dict(BWAGPU_REAPER_THREADS="4", BWAGPU_HOST_THREADS="16"),
    dict(BWAGPU_REAPER_THREADS="4", BWAGPU_E2E_WORKERS="4"),
    dict(BWAGPU_REAPER_THREADS="4", BWAGPU_UNPACK_THREADS="2"),
]


def main():
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 20
    modes = (1, 0) if len(sys.argv) < 3 else tuple(int(x) for x in sys.argv[2].split(","))
    for rnd in range(int(sys.argv[3]) if len(sys.argv) > 3 else 1):
      for st in SETTINGS:
        for mode in modes:
          env = dict(os.environ, **st)
          r = subprocess.run([sys.executable, "-c", CHILD % (REPO, reps, mode, 4)], env=env, cwd=REPO,
                             capture_output=True, text=True, timeout=300)
          try:
              d = json.loads(r.stdout.strip().splitlines()[-1])
          except Exception:
              d = {"error": r.stderr[-400:]}
          print(json.dumps({"round": rnd, "settings": st, "chain_mode": mode, "value": d.get("value"),
                            "ms_per_record": d.get("ms_per_record"), "parity": d.get("parity_last_rep"),
                            "workers": d.get("stage_workers"), "error": d.get("error")}), flush=True)


if __name__ == "__main__":
    main()
