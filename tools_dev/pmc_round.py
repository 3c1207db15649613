"""Summarise tools_dev/gpu_pmc4.sh's SQ passes of the stage bench.

    python tools_dev/pmc_round.py <dir with pmc_a/ pmc_b/> <bench json of pass a>

Per kernel (short name): dispatches and each counter summed over the run and
divided by the launch sequences (spec_reads_kernel dispatches: one per
batch).  For the extension kernels (spec_ext*): issued VALU lane-ops per
ALGORITHMIC cell (the phased pair spec_side4_kernel<G, P, K8>: both sides summed) = SQ_INSTS_VALU * 64 / the reference's cells of one batch
(bench roofline.cells_per_step), and the SIMD-cycle shares: VALU issue =
INSTS_VALU * 2 cycles (a wave64 VALU op on a SIMD-32) over the kernel's
wave-resident SIMD-cycles, and the SQ_WAVE_CYCLES split (quad-cycles) into
active / issue-stall (WAIT_INST_ANY) / parked (WAIT_ANY)."""
import collections
import csv
import glob
import json
import sys

d, bj = sys.argv[1], sys.argv[2]
bench = json.loads(open(bj).read().strip().splitlines()[-1])
cells = bench["roofline"]["cells_per_step"]
tot = collections.defaultdict(lambda: collections.defaultdict(float))
disp = collections.defaultdict(set)
for sub in ("pmc_a", "pmc_b"):
    for f in glob.glob(f"{d}/{sub}/*counter_collection.csv"):
        for r in csv.DictReader(open(f)):
            if "bwagpu::" not in r["Kernel_Name"]:
                continue
            k = r["Kernel_Name"].split("(")[0].replace("void ", "").replace("bwagpu::", "")
            tot[k][r["Counter_Name"]] += float(r["Counter_Value"])
            if sub == "pmc_a":
                disp[k].add(r["Dispatch_Id"])
n_seq = len(disp.get("spec_reads_kernel", ())) or 1
for k in [k for k in tot if k.startswith(("spec_side4_kernel<", "spec_sidep_kernel<")) and k.endswith(", false>")]:  # the phased pair
    r, pk = k[:-len(", false>")] + ", true>", k[:-len(", false>")] + ">"
    if r in tot:
        for n in set(tot[k]) | set(tot[r]):
            tot[pk][n] = tot[k][n] + tot[r][n]
        disp[pk] = disp[k]
out = {"sequences": n_seq, "cells_per_step": cells, "kernels": {}}
for k, c in sorted(tot.items(), key=lambda x: -x[1].get("SQ_WAVE_CYCLES", 0)):
    e = {"dispatches_per_seq": round(len(disp[k]) / n_seq, 3)}
    e.update({n: v / n_seq for n, v in sorted(c.items())})
    wc = c.get("SQ_WAVE_CYCLES", 0)
    if wc:
        e["share_active"] = round(c.get("SQ_ACTIVE_INST_ANY", 0) / wc, 4)
        e["share_wait_inst"] = round(c.get("SQ_WAIT_INST_ANY", 0) / wc, 4)
        e["share_wait_any"] = round(c.get("SQ_WAIT_ANY", 0) / wc, 4)
    if k.startswith("spec_ext") or (k.startswith(("spec_side4", "spec_sidep")) and k.count(",") == 2):
        e["valu_lane_ops_per_cell"] = round(c["SQ_INSTS_VALU"] / n_seq * 64 / cells, 2)
        e["lds_insts_per_kcell"] = round(c.get("SQ_INSTS_LDS", 0) / n_seq / cells * 1e3, 3)
        if c.get("SQ_INSTS_LDS"):
            e["lds_bank_conflict_per_lds_inst"] = round(c.get("SQ_LDS_BANK_CONFLICT", 0) / c["SQ_INSTS_LDS"], 4)
    out["kernels"][k] = e
print(json.dumps(out, indent=1))
