#!/usr/bin/env python3
"""Diagnostic: per-read timeline of the speculative path's selection passes
(emulate = pass 0, final = pass 1) on one reference-seeded C2 batch.
Prints per pass and shape (light / heavy): span, per-read duration
percentiles, the slowest reads, and how many reads are in flight over time."""
import json
import os
import sys

REPO = os.path.normpath(os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
for p in ("bwa-flow_amd/python", "tests", "oracle"):
    sys.path.insert(0, os.path.join(REPO, p))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import refseed  # noqa: E402
from bwagpu import abi  # noqa: E402
from bwagpu.engine import Engine  # noqa: E402

FIELDS = ("seq_off", "seq", "read_chain_off", "chain_seed_off", "chain_rid", "chain_frac_rep", "seeds")
dev = torch.device("cuda:0")
opt, ref, b, want, want_n = refseed.make(pairs=33334, seed=100)
eng = Engine(0, opt, ref["l_pac"], ref["ann_offset"], ref["ann_len"], pac=ref["pac"])
t = {k: torch.from_numpy(np.ascontiguousarray(getattr(b, k)).view(np.uint8).copy()).to(dev) for k in FIELDS}
c = abi.BatchC()
c.n_reads, c.n_chains, c.n_seeds = b.n_reads, b.n_chains, b.n_seeds
c.seq_bytes = int(b.seq_off[-1])
for k in FIELDS:
    setattr(c, k, t[k].data_ptr())
out = torch.zeros(b.n_seeds * 88, dtype=torch.uint8, device=dev)
nn = torch.zeros(b.n_reads, dtype=torch.int32, device=dev)
st = torch.cuda.Stream()
for _ in range(2):
    eng.chain2aln_device(c, out.data_ptr(), nn.data_ptr(), None, st.cuda_stream)
torch.cuda.synchronize()
tr = torch.zeros(b.n_reads * 24, dtype=torch.int32, device=dev)  # passes emulate / final / redo
eng.lib.bwagpu_debug_set_trace(eng.ctx, tr.data_ptr())
eng.chain2aln_device(c, out.data_ptr(), nn.data_ptr(), None, st.cuda_stream)
torch.cuda.synchronize()
eng.lib.bwagpu_debug_set_trace(eng.ctx, None)
T = tr.cpu().numpy().view(np.uint32).reshape(3, b.n_reads, 8).astype(np.int64)
res = {}
for ps, name in ((0, "emulate"), (1, "final")):
    t0 = T[ps, :, 0] | (T[ps, :, 1] << 32)
    t1 = T[ps, :, 2] | (T[ps, :, 3] << 32)
    ok = t0 > 0
    base = t0[ok].min()
    s, e = (t0 - base) / 100.0, (t1 - base) / 100.0
    dur = e - s
    r = {"span_us": float(e[ok].max())}
    for shape, sn in ((1, "light"), (2, "heavy"), (3, "heavy_mat")):
        m = ok & (T[ps, :, 7] == shape)
        if not m.any():
            continue
        idx = np.nonzero(m)[0]
        top = idx[np.argsort(-dur[idx])[:6]]
        r[sn] = dict(n=int(m.sum()), start_max_us=float(s[m].max()), end_max_us=float(e[m].max()),
                     dur_pct=[round(float(np.percentile(dur[m], q)), 1) for q in (50, 90, 99, 100)],
                     busy_us_total=round(float(dur[m].sum()), 1),
                     slowest=[(int(i), int(T[ps, i, 4]), int(T[ps, i, 5]), round(float(dur[i]), 1)) for i in top])
    grid = np.linspace(0, r["span_us"], 21)
    r["in_flight"] = [int(((s[ok] <= g) & (e[ok] > g)).sum()) for g in grid]
    res[name] = r
print(json.dumps(res))
