"""Summarise rocprofv3 FETCH_SIZE / WRITE_SIZE passes of bench.py
(tools_dev/gpu_round.sh) into profiles/<tag>_<workload>_traffic.json:
HBM-side bytes per launch of every engine kernel, and per step (one batch's
launch sequence).  bench.py reads the dominant kernel's entry as
roofline.traffic.

FETCH_SIZE/WRITE_SIZE are in KiB per dispatch (TCC_EA0_RDREQ/WRREQ based).
Per MI355X_MICROARCH.md §HBM, gfx950 FETCH_SIZE reads 1/2 of the bytes of a
wide (16 B/lane) streaming read; our loads are narrow (1-8 B/lane, gathers),
a width the guide lists as uncalibrated, so both the raw and the x2 figure are
recorded and the raw one is reported (a lower bound).

    python tools_dev/pmc_traffic.py <dir with pmc_fetch/ pmc_write/> <tag> <workload> <steps per run>"""
import collections
import csv
import glob
import json
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "bwa-flow_amd", "python"))
from bwagpu.provenance import source_digest  # noqa: E402

d, tag, wl, steps = sys.argv[1], sys.argv[2], sys.argv[3], int(sys.argv[4])
ours = ("bwagpu::",)
out = {"tag": tag, "workload": wl, "source_digest": source_digest(), "per_launch": {}}
tot = collections.defaultdict(float)
for sub, c in (("pmc_fetch", "FETCH_SIZE"), ("pmc_write", "WRITE_SIZE")):
    per = collections.defaultdict(list)
    for f in glob.glob(f"{d}/{sub}/*counter_collection.csv"):
        for r in csv.DictReader(open(f)):
            if r["Counter_Name"] == c and any(k in r["Kernel_Name"] for k in ours):
                per[r["Kernel_Name"].split("(")[0].replace("void ", "").replace("bwagpu::", "")].append(
                    float(r["Counter_Value"]) * 1024)
    for k, v in per.items():
        e = out["per_launch"].setdefault(k, {"dispatches": len(v)})
        e["fetch_bytes" if c == "FETCH_SIZE" else "write_bytes"] = sum(v) / len(v)
        tot[c] += sum(v)
# the phased extension's side pair (spec_side4_kernel<G, P, K8, false|true>:
# every left call, then every right call) is one "launch" of the dominant
# kernel: its entry sums the two sides' per-dispatch bytes
for k in [k for k in out["per_launch"] if k.startswith(("spec_side4_kernel<", "spec_sidep_kernel<")) and k.endswith(", false>")]:
    r = k[:-len(", false>")] + ", true>"
    if r in out["per_launch"]:
        L, R = out["per_launch"][k], out["per_launch"][r]
        out["per_launch"][k[:-len(", false>")] + ">"] = {
            "dispatches": min(L["dispatches"], R["dispatches"]), "pair": "left + right side launch",
            **{f: L.get(f, 0.0) + R.get(f, 0.0) for f in ("fetch_bytes", "write_bytes")}}
for k, e in out["per_launch"].items():
    e["traffic_bytes"] = e.get("fetch_bytes", 0.0) + e.get("write_bytes", 0.0)
    e["traffic_bytes_fetch_x2"] = 2 * e.get("fetch_bytes", 0.0) + e.get("write_bytes", 0.0)
# the bench runs warmup + timed steps + the launch-sequence timing pass; the
# per-step figure divides the chain2aln kernels' totals by the launches of the
# first kernel of a sequence (spec_chain_kernel: one per batch)
n_seq = out["per_launch"].get("spec_chain_kernel", {}).get("dispatches", steps)
out["per_step"] = {"fetch_bytes": tot["FETCH_SIZE"] / n_seq, "write_bytes": tot["WRITE_SIZE"] / n_seq,
                   "traffic_bytes": (tot["FETCH_SIZE"] + tot["WRITE_SIZE"]) / n_seq, "sequences": n_seq,
                   "note": "all engine kernels of the run / chain2aln launch sequences (includes the CIGAR and "
                           "host-path legs' kernels if they ran)"}
json.dump(out, open(f"profiles/{tag}_{wl}_traffic.json", "w"), indent=1)
print(json.dumps({k: round(v["traffic_bytes"]) for k, v in out["per_launch"].items()}))
