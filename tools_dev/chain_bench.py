"""Chaining benchmark: bwagpu_seqs2chains / bwagpu_seqs2regions over the C2
batch's reads against the chr21-sized genome's bwa index (bench_data/e2e);
parity against the reference's ChainsRecord / regions.  One JSON line."""
import argparse
import json
import os
import sys
import time

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
sys.path.insert(0, os.path.join(ROOT, "bwa-flow_amd", "python"))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import torch  # noqa: E402,F401
from bwagpu import workload  # noqa: E402
from bwagpu.engine import Batch, Engine  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--fused", action="store_true")
    ap.add_argument("--budget", type=int, default=-1, help="seeding tier-1 budget (-1: library default)")
    ap.add_argument("--concurrent", type=int, default=0,
                    help="also: N contexts on N host threads, each running seqs2chains (pipeline throughput)")
    a = ap.parse_args()
    opt, gref, rbs = workload.load_fixture()
    rb = rbs[0]
    b = rb.batch
    eng = Engine(0, opt, gref.l_pac, gref.ann_offset, gref.ann_len, pac=gref.pac)
    hdr, words, sa, sa_intv = workload.load_bwa_index(os.path.join(ROOT, "bench_data", "e2e", "ref.fa"))
    eng.set_bwt(hdr, words, sa, sa_intv)
    if a.budget >= 0:
        eng.seed_budget(a.budget)
    so = np.ascontiguousarray(b.seq_off, np.int64)
    sq = np.ascontiguousarray(b.seq, np.uint8)
    eng.seqs2chains(so, sq, copy=False)
    t0 = time.perf_counter()
    for _ in range(a.reps):
        eng.seqs2chains(so, sq, copy=False)
    ms = (time.perf_counter() - t0) * 1e3 / a.reps
    out = eng.seqs2chains(so, sq)
    rco, ch, cso, sd = out
    got = Batch(b.seq_off, b.seq, rco, cso, ch["rid"].copy(), ch["frac_rep"].copy(), sd)
    res = {"budget": a.budget, "seqs2chains_ms": round(ms, 3), "chains_ok": workload.batch_digest(got) == workload.batch_digest(b)}
    if a.fused:
        eng.seqs2regions(so, sq, copy=False)
        t0 = time.perf_counter()
        for _ in range(a.reps):
            eng.seqs2regions(so, sq, copy=False)
        res["seqs2regions_ms"] = round((time.perf_counter() - t0) * 1e3 / a.reps, 3)
        n, regs = eng.seqs2regions(so, sq)
        res["regions_ok"] = bool(rb.check_compact(regs, n))
    if a.concurrent:
        import threading
        engs = [eng] + [Engine(0, opt, gref.l_pac, gref.ann_offset, gref.ann_len, pac=gref.pac)
                        for _ in range(a.concurrent - 1)]
        for e in engs[1:]:
            e.set_bwt(hdr, words, sa, sa_intv)
            e.seqs2chains(so, sq, copy=False)
        for fn, key in (("seqs2chains", "conc_seqs2chains_ms_per_batch"), ("seqs2regions", "conc_seqs2regions_ms_per_batch")):
            bar = threading.Barrier(len(engs) + 1)

            def work(e):
                bar.wait()
                for _ in range(a.reps):
                    getattr(e, fn)(so, sq, copy=False)

            th = [threading.Thread(target=work, args=(e,)) for e in engs]
            for t in th:
                t.start()
            bar.wait()
            t0 = time.perf_counter()
            for t in th:
                t.join()
            res[key] = round((time.perf_counter() - t0) * 1e3 / (a.reps * len(engs)), 3)
        res["concurrent"] = a.concurrent
    print(json.dumps(res))


if __name__ == "__main__":
    main()
