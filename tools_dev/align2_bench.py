#!/usr/bin/env python3
"""Batched ksw_align2 (mate rescue) throughput on one GPU, with the
reference's own ksw_align2 (oracle/_ref) timed on a subsample of the same
tasks on the host as the CPU figure.  One JSON line on stdout.

    python tools_dev/align2_bench.py [--tasks N] [--reps K] [--qlens 100,150,250]
"""
import argparse
import json
import os
import sys
import time

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.normpath(os.path.join(HERE, ".."))
sys.path.insert(0, os.path.join(REPO, "bwa-flow_amd", "python"))
sys.path.insert(0, os.path.join(REPO, "oracle"))
sys.path.insert(0, os.path.join(REPO, "tests"))

from bwagpu import abi, synth  # noqa: E402
from bwagpu.engine import Engine  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--tasks", type=int, default=32768)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--qlens", default="100,150,250")
    ap.add_argument("--win", default="300,700")
    ap.add_argument("--check", type=int, default=2000, help="tasks checked against the oracle")
    ap.add_argument("--cpu-sample", type=int, default=2000)
    a = ap.parse_args()
    opt = abi.default_opt()
    rng = np.random.default_rng(1234)
    qlens = tuple(int(x) for x in a.qlens.split(","))
    w0, w1 = (int(x) for x in a.win.split(","))
    t0 = time.time()
    tasks, qp, tp = synth.mate_rescue_tasks(rng, a.tasks, qlens=qlens, win=(w0, w1), xtra_mode="matesw")
    gen_s = time.time() - t0
    import golden_io as G
    r = G.load_ref()
    eng = Engine(0, opt, r["l_pac"], r["ann_offset"], r["ann_len"], pac=r["pac"])
    got = eng.align2_batch(tasks, qp, tp)  # warm-up (and allocations)
    kms, walls = [], []
    for _ in range(a.reps):
        t0 = time.time()
        got = eng.align2_batch(tasks, qp, tp)
        walls.append(time.time() - t0)
        kms.append(eng.last_stats()["kernel_ms"])
    st = eng.last_stats()
    out = dict(metric="ksw_align2 mate-rescue tasks/s", tasks=a.tasks, qlens=qlens, win=[w0, w1],
               kernel_ms=float(np.median(kms)), wall_ms=1e3 * float(np.median(walls)),
               tasks_per_s=a.tasks / (1e-3 * float(np.median(kms))),
               gcups=st["cells"] / (1e-3 * float(np.median(kms))) / 1e9, cells=st["cells"], rows=st["rows"],
               passes=st["ext_calls"], gen_s=gen_s)
    import oracle
    n = min(a.check, a.tasks)
    sub = tasks[:n]
    want, _ = oracle.align2("oracle", opt, sub, qp, tp)
    out["parity_checked"] = n
    out["parity_mismatch"] = int((got[:n].view(np.int32).reshape(-1, 7) != want.view(np.int32).reshape(-1, 7))
                                 .any(axis=1).sum())
    if oracle.ref_lib() is not None and hasattr(oracle.ref_lib(), "ref_align2_batch"):
        m = min(a.cpu_sample, a.tasks)
        t0 = time.time()
        oracle.align2("ref", opt, tasks[:m], qp, tp)
        dt = time.time() - t0
        out["cpu_reference_1thread_tasks_per_s"] = m / dt
        out["cpu_sample"] = m
    print(json.dumps(out))
    eng.close()


if __name__ == "__main__":
    main()
