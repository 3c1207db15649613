#!/usr/bin/env python3
"""Where the packed extension kernels' issued cells go, on the C2 fixture
batches: a library built with -DBWAGPU_OCC_DIAG (make LIB=lib/diag
EXTRA=-DBWAGPU_OCC_DIAG lib/diag/libbwagpu.so) counts per extend_quad
generation the rows run, the live calls' rows, the call-slot cells, the
cells beyond a live call's query, outside ksw's band, and computed
(bwagpu_debug_occupancy).  Split of the call-slot cells:
  ended      calls that already ended (the wave runs until its longest ends)
  beyond_q   columns past a live call's own query (columns set by the longest)
  out_band   inside the query but outside ksw's band
  computed   cells computed (the row bound's live rows only)
With spec_sidep_kernel (the producer wave) start_claim is a DP wave's wait for
its next buffer, and claim / taskrec are the producer wave's busy / idle cycles.
    BWAGPU_LIB=bwa-flow_amd/lib/diag/libbwagpu.so python tools_dev/occ_diag.py [row_bound 0|1]"""
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
KEYS = ("generations", "rows_run", "call_slot_rows", "live_call_rows", "slot_cells", "live_slot_cells",
        "query_cells", "computed_cells", "cyc_start_claim", "cyc_setup", "cyc_dp", "cyc_advance", "cyc_claim",
        "cyc_taskrec")


def main():
    bound = int(sys.argv[1]) if len(sys.argv) > 1 else 1
    dev = torch.device("cuda:0")
    opt, ref, bs = workload.load_fixture()
    eng = Engine(0, opt, ref.l_pac, ref.ann_offset, ref.ann_len, pac=ref.pac)
    eng.row_bound(bound)
    out = {"row_bound": bound, "lib": abi.lib_path(), "kernel": eng.ext_kernel(160),
           "env": {k: v for k, v in os.environ.items() if k.startswith("BWAGPU_")}}
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
        st = torch.cuda.Stream()
        eng.chain2aln_device(c, regs.data_ptr(), nn.data_ptr(), None, st.cuda_stream)
        oc = np.zeros(14, np.int64)
        rc = eng.lib.bwagpu_debug_occupancy(eng.ctx, C.c_void_p(st.cuda_stream), oc.ctypes.data_as(C.c_void_p))
        if rc != 0:
            raise SystemExit(f"bwagpu_debug_occupancy rc={rc}: {eng.lib.bwagpu_last_error(eng.ctx)}")
        d = dict(zip(KEYS, (int(x) for x in oc)))
        S = max(d["slot_cells"], 1)
        d["split"] = {"ended": round(1 - d["live_slot_cells"] / S, 4),
                      "beyond_q": round((d["live_slot_cells"] - d["query_cells"]) / S, 4),
                      "out_band": round((d["query_cells"] - d["computed_cells"]) / S, 4),
                      "computed": round(d["computed_cells"] / S, 4)}
        cyc = sum(d[k] for k in KEYS[8:12])
        d["cycle_split"] = {k[4:]: round(d[k] / max(cyc, 1), 4) for k in KEYS[8:]}
        d["cycles_per_generation"] = {k[4:]: round(d[k] / max(d["generations"], 1), 1) for k in KEYS[8:]}
        d["row_occupancy"] = round(d["live_call_rows"] / max(d["call_slot_rows"], 1), 4)
        d["rows_per_generation"] = round(d["rows_run"] / max(d["generations"], 1), 2)
        d["parity"] = bool(rb.check(regs.cpu().numpy().view(abi.ALNREG_DTYPE), nn.cpu().numpy()))
        out[f"batch{k}"] = d
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
