"""Diagnostic: the speculative path's extension work on a reference-seeded C2
batch — tasks per round (A: each chain's first seed; B: the emulation's
predictions; C: mispredictions), DP cells of every computed task against the
cells of the extensions the reference performs, and where the unused cells
sit (per round, by the SeedExt records: computed but not counted)."""
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

FIELDS = ("seq_off", "seq", "read_chain_off", "chain_seed_off", "chain_rid", "chain_frac_rep", "seeds")
dev = torch.device("cuda:0")
opt, ref, bs = workload.load_fixture()
eng = Engine(0, opt, ref.l_pac, ref.ann_offset, ref.ann_len, pac=ref.pac)
if os.environ.get("EXT_FORM"):  # bwagpu_debug_ext_form for the A/B
    abi.load().bwagpu_debug_ext_form(int(os.environ["EXT_FORM"]))
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
    torch.cuda.synchronize()
    s = stats.cpu().numpy()
    out[f"batch{k}"] = {"tasks_A": int(sc[0]), "tasks_B": int(sc[1]), "tasks_C": int(sc[2]),
                        "cells_computed": int(sc[3]), "cells_reference": int(s[0]), "ext_calls_reference": int(s[2]),
                        "waste_frac": round(1 - s[0] / sc[3], 4), "redo_inline": int(sc[4]),
                        "heavy_reads": int(sc[5]), "redo_reads": int(sc[6])}
    if sc[8]:  # a lib with tools_dev/ab/quad_occupancy_diag.patch: four-per-wave loop occupancy
        loops, cols, rows = int(sc[8]), int(sc[9]), int(sc[10])
        # loops: group-rows (x 2 call slots), cols: call-slot columns over the rows
        out[f"batch{k}"]["quad"] = {"group_rows": loops, "call_rows": rows, "row_occupancy": round(rows / (2 * loops), 4),
                                    "slot_cells": cols, "cell_occupancy": round(sc[3] / cols, 4)}
print(json.dumps(out))
