#!/usr/bin/env python3
"""Diagnostic: per-task DP work of the speculative path's extension tasks on
one reference-seeded C2 batch (SeedExt records: rows, cells, ksw calls per
seed), against the task's side lengths — how heavy the tail tasks are."""
import ctypes as C
import json
import os
import sys

REPO = os.path.normpath(os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
for p in ("bwa-flow_amd/python", "tests", "oracle"):
    sys.path.insert(0, os.path.join(REPO, p))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from bwagpu import abi, workload  # noqa: E402
from bwagpu.engine import Engine  # noqa: E402

EXT = np.dtype([("rb", "<i8"), ("re", "<i8"), ("qb", "<i4"), ("qe", "<i4"), ("score", "<i4"), ("truesc", "<i4"),
                ("w", "<i4"), ("cells", "<i4"), ("rows", "<i4"), ("calls", "<i4")])
FIELDS = ("seq_off", "seq", "read_chain_off", "chain_seed_off", "chain_rid", "chain_frac_rep", "seeds")
dev = torch.device("cuda:0")
opt, ref, bs = workload.load_fixture()
eng = Engine(0, opt, ref.l_pac, ref.ann_offset, ref.ann_len, pac=ref.pac)
res = {}
for k, rb in enumerate(bs):
    b = rb.batch
    t = {f: torch.from_numpy(np.ascontiguousarray(getattr(b, f)).view(np.uint8).copy()).to(dev) for f in FIELDS}
    c = abi.BatchC()
    c.n_reads, c.n_chains, c.n_seeds = b.n_reads, b.n_chains, b.n_seeds
    c.seq_bytes = int(b.seq_off[-1])
    for f in FIELDS:
        setattr(c, f, t[f].data_ptr())
    out = torch.zeros(b.n_seeds * 88, dtype=torch.uint8, device=dev)
    nn = torch.zeros(b.n_reads, dtype=torch.int32, device=dev)
    st = torch.cuda.Stream()
    eng.chain2aln_device(c, out.data_ptr(), nn.data_ptr(), None, st.cuda_stream)
    e = np.zeros(b.n_seeds, EXT)
    assert eng.lib.bwagpu_debug_spec_ext(eng.ctx, C.c_void_p(st.cuda_stream), e.ctypes.data_as(C.c_void_p), b.n_seeds) == 0
    # seeds in processing order (descending score<<32|i per chain, bwamem.c:671-676) -> widest side
    cols = np.zeros(b.n_seeds, np.int64)
    lq_read = np.diff(b.seq_off)
    for ch in range(b.n_chains):
        s0, s1 = int(b.chain_seed_off[ch]), int(b.chain_seed_off[ch + 1])
        if s1 == s0:
            continue
        sd = b.seeds[s0:s1]
        key = (sd["score"].astype(np.int64) << 32) | np.arange(s1 - s0)
        o_ = np.argsort(-key, kind="stable")
        rd = int(np.searchsorted(b.read_chain_off, ch, side="right") - 1)
        lq = int(lq_read[rd])
        q = sd["qbeg"][o_].astype(np.int64)
        ln = sd["len"][o_].astype(np.int64)
        cols[s0:s1] = np.maximum(q, lq - q - ln) + 1
    m = e["calls"] > 0
    bins = np.digitize(cols, [65, 129, 193])
    res[f"batch{k}_bins"] = {int(x): dict(tasks=int((m & (bins == x)).sum()), rows=int(e["rows"][m & (bins == x)].sum()),
                                          cells=int(e["cells"][m & (bins == x)].sum())) for x in range(4)}
    comp = e[e["calls"] > 0]
    rows = np.sort(comp["rows"])[::-1]
    res[f"batch{k}"] = dict(tasks=int(len(comp)), rows_total=int(rows.sum()), cells_total=int(comp["cells"].sum()),
                            rows_top=[int(x) for x in rows[:12]], rows_pct=[int(np.percentile(rows, q)) for q in (50, 90, 99, 99.9)],
                            calls_hist=np.bincount(comp["calls"] - 1).tolist(),
                            top_share_rows=round(float(rows[:200].sum() / rows.sum()), 4))
print(json.dumps(res))
