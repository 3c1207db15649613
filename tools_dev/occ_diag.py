#!/usr/bin/env python3
"""Occupancy of the packed extension kernels on the C2 batches, from a build
with tools_dev/ab/quad_occupancy_diag.patch (+ the two beyond-qlen counters of
round 5): group-rows run, slot columns run, call-rows, and per live call
sum(rows x (qlen + 1)) against sum(rows x columns run) -- the share of a live
call's columns that lie beyond its own query.  BWAGPU_LIB=<that build>."""
import ctypes as C
import json
import os
import sys

REPO = os.path.normpath(os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
sys.path.insert(0, os.path.join(REPO, "bwa-flow_amd", "python"))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from bwagpu import abi, workload  # noqa: E402
from bwagpu.engine import Engine  # noqa: E402

FIELDS = ("seq_off", "seq", "read_chain_off", "chain_seed_off", "chain_rid", "chain_frac_rep", "seeds")
dev = torch.device("cuda:0")
opt, ref, bs = workload.load_fixture()
eng = Engine(0, opt, ref.l_pac, ref.ann_offset, ref.ann_len, pac=ref.pac)
out = {}
for k, rb in enumerate(bs):
    b = rb.batch
    t = {f: torch.from_numpy(np.ascontiguousarray(getattr(b, f)).view(np.uint8).copy()).to(dev) for f in FIELDS}
    c = abi.BatchC()
    c.n_reads, c.n_chains, c.n_seeds = b.n_reads, b.n_chains, b.n_seeds
    c.seq_bytes = int(b.seq_off[-1])
    for f in FIELDS:
        setattr(c, f, t[f].data_ptr())
    regs = torch.zeros(b.n_seeds * 88, dtype=torch.uint8, device=dev)
    nn = torch.zeros(b.n_reads, dtype=torch.int32, device=dev)
    stats = torch.zeros(4, dtype=torch.int64, device=dev)
    st = torch.cuda.Stream()
    eng.chain2aln_device(c, regs.data_ptr(), nn.data_ptr(), stats.data_ptr(), st.cuda_stream)
    sc = np.zeros(16, np.int64)
    assert eng.lib.bwagpu_debug_spec_counters(eng.ctx, C.c_void_p(st.cuda_stream), sc.ctypes.data_as(C.c_void_p)) == 0
    s = stats.cpu().numpy()
    loops, cols, rows, qcols, live = (int(x) for x in sc[8:13])
    out[f"batch{k}"] = {"cells_reference": int(s[0]), "cells_computed": int(sc[3]), "group_rows": loops,
                        "slot_cells": cols, "call_rows": rows, "row_occupancy": round(rows / max(2 * loops, 1), 4),
                        "cell_occupancy": round(int(sc[3]) / max(cols, 1), 4),
                        "live_call_slot_cells": live, "live_call_query_cells": qcols,
                        "beyond_qlen_share_of_live": round(1 - qcols / max(live, 1), 4),
                        "band_share_of_query_cells": round(int(sc[3]) / max(qcols, 1), 4)}
print(json.dumps(out, indent=1))
