#!/usr/bin/env python3
"""Kernel iteration bench on reference-seeded ChainsRecords (dev tool).

Makes C2-sized batches with the reference's own seeding (tests/refseed.py ->
oracle/_ref/gen_golden), runs the GPU stage through bwagpu_chain2aln_device
with inputs resident in HBM, checks every batch byte-for-byte against the
reference's regions, and prints one JSON line: ms per batch, reads/s, GCUPS,
evaluated cells / rows / extension calls per batch.

    python tools_dev/realbench.py [--batches 2] [--reps 10] [--length 150|mix]
"""
import argparse
import ctypes as C
import json
import os
import sys
import time

REPO = os.path.normpath(os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
for p in ("bwa-flow_amd/python", "tests", "oracle"):
    sys.path.insert(0, os.path.join(REPO, p))

import numpy as np  # noqa: E402
import torch  # noqa: E402

import golden_io as G  # noqa: E402
import refseed  # noqa: E402
from bwagpu import abi  # noqa: E402
from bwagpu.engine import Engine, compact  # noqa: E402

FIELDS = ("seq_off", "seq", "read_chain_off", "chain_seed_off", "chain_rid", "chain_frac_rep", "seeds")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batches", type=int, default=2)
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--pairs", type=int, default=33334)
    ap.add_argument("--length", default="150")
    ap.add_argument("--opt-mode", type=int, default=0)
    ap.add_argument("--path", default="spec", help="spec (default) | fast (per-read kernels)")
    a = ap.parse_args()
    if a.path == "spec":
        os.environ.pop("BWAGPU_C2A_PATH", None)
    else:
        os.environ["BWAGPU_C2A_PATH"] = a.path
    dev = torch.device("cuda:0")
    sets = []
    t0 = time.time()
    for k in range(a.batches):
        sets.append(refseed.make(pairs=a.pairs, seed=100 + k, length=a.length, opt_mode=a.opt_mode))
    t_gen = time.time() - t0
    opt, ref = sets[0][0], sets[0][1]
    eng = Engine(0, opt, ref["l_pac"], ref["ann_offset"], ref["ann_len"], pac=ref["pac"])
    dbs = []
    for (_, _, b, want, want_n) in sets:
        t = {k: torch.from_numpy(np.ascontiguousarray(getattr(b, k)).view(np.uint8).copy()).to(dev) for k in FIELDS}
        c = abi.BatchC()
        c.n_reads, c.n_chains, c.n_seeds = b.n_reads, b.n_chains, b.n_seeds
        c.seq_bytes = int(b.seq_off[-1])
        for k in FIELDS:
            setattr(c, k, t[k].data_ptr())
        out = torch.zeros(max(b.n_seeds, 1) * 88, dtype=torch.uint8, device=dev)
        nn = torch.zeros(max(b.n_reads, 1), dtype=torch.int32, device=dev)
        st = torch.zeros(4, dtype=torch.int64, device=dev)
        dbs.append((b, t, c, out, nn, st, want, want_n))
    stream = torch.cuda.Stream()  # a real stream: the engine maps NULL to its own
    # warm-up + parity on every batch
    parity = True
    stats = []
    spec = []
    for (b, t, c, out, nn, st, want, want_n) in dbs:
        st.zero_()
        eng.chain2aln_device(c, out.data_ptr(), nn.data_ptr(), st.data_ptr(), stream.cuda_stream)
        torch.cuda.synchronize()
        regs = out.cpu().numpy().view(abi.ALNREG_DTYPE)[:b.n_seeds]
        n = nn.cpu().numpy()[:b.n_reads]
        ok = np.array_equal(n, want_n) and G.region_mismatch(compact(b, regs, n), want) is None
        parity &= ok
        stats.append(st.cpu().numpy().tolist())
        sc = np.zeros(8, np.int64)
        if a.path == "spec":
            eng.lib.bwagpu_debug_spec_counters(eng.ctx, C.c_void_p(stream.cuda_stream), sc.ctypes.data_as(C.c_void_p))
        spec.append(sc.tolist())
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    torch.cuda.set_stream(stream)
    e0.record(stream)
    for r in range(a.reps):
        for (b, t, c, out, nn, st, want, want_n) in dbs:
            eng.chain2aln_device(c, out.data_ptr(), nn.data_ptr(), None, stream.cuda_stream)
    e1.record(stream)
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / (a.reps * len(dbs))
    reads = sum(d[0].n_reads for d in dbs) / len(dbs)
    cells = sum(s[0] for s in stats) / len(stats)
    rows = sum(s[1] for s in stats) / len(stats)
    calls = sum(s[2] for s in stats) / len(stats)
    print(json.dumps(dict(ms_per_batch=round(ms, 4), mreads_s=round(reads / ms / 1e3, 3), gcups=round(cells / ms / 1e6, 2),
                          reads=reads, chains=sum(d[0].n_chains for d in dbs) / len(dbs),
                          seeds=sum(d[0].n_seeds for d in dbs) / len(dbs), cells=cells, rows=rows, ext_calls=calls,
                          parity_all_batches=bool(parity), length=a.length, path=a.path, gen_s=round(t_gen, 1),
                          spec_tasks_abc=[s[:3] for s in spec], spec_cells=[s[3] for s in spec],
                          redo_inline=[s[4] for s in spec], heavy_reads=[s[5] for s in spec],
                          redo_reads=[s[6] for s in spec])), flush=True)
    eng.close()


if __name__ == "__main__":
    main()
