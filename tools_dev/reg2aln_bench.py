#!/usr/bin/env python3
"""Batched mem_reg2aln CIGAR throughput on one GPU (bwagpu_reg2aln_batch) on the
regions of one C2-shaped batch (66.7k synthetic 2x150 reads vs a chr21-sized
synthetic reference; regions from the GPU mem_chain2aln of the same batch), with
the reference's own mem_reg2aln (oracle/_ref) timed on a subsample on one host
thread as the CPU figure and the oracle as the checker.  One JSON line.

    python tools_dev/reg2aln_bench.py [--pairs N] [--reps K]
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

from bwagpu import abi  # noqa: E402
from bwagpu.engine import Engine, unflatten  # noqa: E402
from bwagpu.synth import SynthRef, synth_batch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--pairs", type=int, default=33334)
    ap.add_argument("--len", type=int, default=150)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--check", type=int, default=4000)
    ap.add_argument("--cpu-sample", type=int, default=4000)
    a = ap.parse_args()
    opt = abi.default_opt()
    ref = SynthRef(42, 46_709_983, 1)
    b = synth_batch(ref, 1000, a.pairs, a.len)
    eng = Engine(0, opt, ref.l_pac, ref.ann_offset, ref.ann_len, pac=ref.pac)
    regs, n = eng.chain2aln(b)
    parts = unflatten(b, regs, n)
    jobs = []
    for r, p in enumerate(parts):
        for g in p:
            jobs.append((g["rb"], g["re"], b.seq_off[r], b.seq_off[r + 1] - b.seq_off[r], g["qb"], g["qe"],
                         g["truesc"], g["w"], 0))
    tasks = np.array(jobs, dtype=abi.REG2ALN_TASK_DTYPE)
    qpool = b.seq
    out, cig, md = eng.reg2aln_batch(tasks, qpool, 64, 512)  # warm-up
    kms, walls = [], []
    for _ in range(a.reps):
        t0 = time.time()
        out, cig, md = eng.reg2aln_batch(tasks, qpool, 64, 512)
        walls.append(time.time() - t0)
        kms.append(eng.last_stats()["kernel_ms"])
    st = eng.last_stats()
    km = float(np.median(kms))
    res = dict(metric="mem_reg2aln CIGAR jobs/s", jobs=len(tasks), reads=int(b.n_reads), kernel_ms=km,
               wall_ms=1e3 * float(np.median(walls)), jobs_per_s=len(tasks) / (1e-3 * km),
               cells=st["cells"], rows=st["rows"], gen_cigar2_calls=st["ext_calls"],
               gcups=st["cells"] / (1e-3 * km) / 1e9, status=np.bincount(out["status"], minlength=4).tolist())
    import golden_io as G
    import oracle
    R = oracle.Ref(ref.l_pac, ref.ann_offset, ref.ann_len, ref.pac)
    m = min(a.check, len(tasks))
    want, wc, wm = oracle.reg2aln("oracle", opt, R, tasks[:m], qpool, 64, 512)
    res["parity_checked"] = m
    res["parity_ok"] = G.aln_mismatch(tasks[:m], out[:m], cig[:m], md[:m], *G.aln_expected_from(want, wc, wm)) is None
    if oracle.ref_lib() is not None and hasattr(oracle.ref_lib(), "ref_reg2aln_batch"):
        m = min(a.cpu_sample, len(tasks))
        t0 = time.time()
        oracle.reg2aln("ref", opt, R, tasks[:m], qpool, 64, 512)
        dt = time.time() - t0
        res["cpu_reference_1thread_jobs_per_s"] = m / dt
        res["cpu_sample"] = m
    print(json.dumps(res))
    eng.close()


if __name__ == "__main__":
    main()
