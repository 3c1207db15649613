"""Bare ksw_extend2 task-list throughput: wave kernels vs 16-lane-group kernels.

Replicates each golden task set R times (tasks only; pools shared), runs
bwagpu_extend_batch with BWAGPU_EXT_WAVE=1 (wave kernels) and =0 (groups for
qlen+1 <= 128), checks both against the golden results, prints kernel ms/GCUPS.
"""
import os
import sys

sys.path.insert(0, "bwa-flow_amd/python"); sys.path.insert(0, "oracle"); sys.path.insert(0, "tests")
import numpy as np  # noqa: E402
import golden_io as G  # noqa: E402
from bwagpu.engine import Engine  # noqa: E402

R = int(sys.argv[1]) if len(sys.argv) > 1 else 20
refd = G.load_ref()
for name in G.CHAIN_SETS + G.KSW_SETS:
    opt, tasks, want, qp, tp = G.load_tasks(name)
    big = np.tile(tasks, R)
    wbig = np.tile(want, R)
    eng = Engine(0, opt, refd["l_pac"], refd["ann_offset"], refd["ann_len"], pac=refd["pac"])
    line = [f"{name:18s} n={len(big):7d}"]
    for mode in ("1", "0"):
        os.environ["BWAGPU_EXT_WAVE"] = mode
        best = None
        for _ in range(3):
            got = eng.extend_batch(big, qp, tp)
            st = eng.last_stats()
            best = st if best is None or st["kernel_ms"] < best["kernel_ms"] else best
        g, w = got.view(np.int32).reshape(-1, 6), wbig.view(np.int32).reshape(-1, 6)
        bad = int((g != w).any(axis=1).sum())
        line.append(f"{'wave' if mode == '1' else 'grp '}: {best['kernel_ms']:8.3f} ms "
                    f"{best['cells'] / best['kernel_ms'] / 1e6:7.1f} GCUPS bad={bad}")
    eng.close()
    print(" | ".join(line), flush=True)
