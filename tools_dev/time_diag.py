#!/usr/bin/env python3
"""Where a packed extension wave's time goes (C2 batches), from a build with
clock64() brackets around the phases of spec_ext4_kernel's generation loop
(claim + qtask_start, qtask_call, extend_quad, qtask_advance + store; each
bracket ends with s_waitcnt 0) summed per wave into ctr words 32-45 and
copied out by bwagpu_debug_spec_counters.  BWAGPU_LIB=<that build>."""
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
    for rep in range(3):
        eng.chain2aln_device(c, regs.data_ptr(), nn.data_ptr(), stats.data_ptr(), st.cuda_stream)
        sc = np.zeros(16, np.int64)
        assert eng.lib.bwagpu_debug_spec_counters(eng.ctx, C.c_void_p(st.cuda_stream), sc.ctypes.data_as(C.c_void_p)) == 0
    tot, tcl, tca, tro, tad, gens, waves = (int(x) for x in sc[8:15])
    out[f"batch{k}"] = {"wave_clocks": tot, "waves": waves, "generations": gens,
                        "share_claim_start": round(tcl / tot, 4), "share_call_fill": round(tca / tot, 4),
                        "share_rows": round(tro / tot, 4), "share_advance_store": round(tad / tot, 4),
                        "clocks_per_generation": round(tot / max(gens, 1), 1),
                        "row_clocks_per_generation": round(tro / max(gens, 1), 1)}
print(json.dumps(out, indent=1))
