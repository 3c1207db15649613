"""Summarise rocprofv3 FETCH_SIZE / WRITE_SIZE passes (tools_dev/gpu_official.sh) into
profiles/<tag>_traffic.json: HBM-side bytes per SW-stage launch sequence.

FETCH_SIZE/WRITE_SIZE are in KiB per dispatch (TCC_EA0_RDREQ/WRREQ based).
Per MI355X_MICROARCH.md §HBM, gfx950 FETCH_SIZE reads 1/2 of the bytes of a
wide (16 B/lane) streaming read; our loads are narrow (1-8 B/lane, gathers),
a width the guide lists as uncalibrated, so both the raw and the x2 figure are
recorded and the raw one is reported (a lower bound)."""
import csv
import collections
import json
import sys

d, tag = sys.argv[1], sys.argv[2]
ours = ("bwagpu::", "rocprim::")
out = {"tag": tag, "kernels": {}}
for f, c in ((f"{d}/pmc_fetch/f_counter_collection.csv", "FETCH_SIZE"),
             (f"{d}/pmc_write/w_counter_collection.csv", "WRITE_SIZE")):
    per = collections.defaultdict(list)
    for r in csv.DictReader(open(f)):
        if r["Counter_Name"] == c and any(k in r["Kernel_Name"] for k in ours):
            per[r["Kernel_Name"].split("(")[0]].append(float(r["Counter_Value"]) * 1024)
    for k, v in per.items():
        out["kernels"].setdefault(k, {})[c] = {"dispatches": len(v), "bytes_mean": sum(v) / len(v)}
seq_f = seq_w = 0.0
launches = max(v["FETCH_SIZE"]["dispatches"] for k, v in out["kernels"].items() if "chain2aln_kernel" in k)
for k, v in out["kernels"].items():
    for c in ("FETCH_SIZE", "WRITE_SIZE"):
        if c in v:
            tot = v[c]["bytes_mean"] * v[c]["dispatches"] / launches
            if c == "FETCH_SIZE":
                seq_f += tot
            else:
                seq_w += tot
out["per_launch_sequence"] = {"fetch_bytes": seq_f, "write_bytes": seq_w, "traffic_bytes": seq_f + seq_w,
                              "traffic_bytes_fetch_x2": 2 * seq_f + seq_w, "launches": launches}
json.dump(out, open(f"profiles/{tag}_traffic.json", "w"), indent=1)
print(json.dumps(out["per_launch_sequence"]))
