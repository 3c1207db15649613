"""Print the per-launch timeline of the last chain2aln batch in a rocprofv3
kernel trace (dev tool): python tools_dev/timeline.py <run_kernel_trace.csv> [first-kernel-name]"""
import csv
import sys

rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
first = sys.argv[2] if len(sys.argv) > 2 else "spec_chain_kernel"
starts = [i for i, r in enumerate(rows) if first in r["Kernel_Name"]]
seq = rows[starts[-2]:starts[-1]] if len(starts) > 1 else rows[starts[-1]:]
t0 = int(seq[0]["Start_Timestamp"])
busy = {}
for r in seq:
    n = r["Kernel_Name"].replace("bwagpu::", "").replace("void ", "").split("(")[0]
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    busy[n] = busy.get(n, 0) + (e - s)
    print(f"{n:36s} start {(s - t0) / 1e3:9.1f} dur {(e - s) / 1e3:8.1f} us  vgpr {r['VGPR_Count']} lds {r['LDS_Block_Size']} scr {r['Scratch_Size']}")
print("span", (int(seq[-1]["End_Timestamp"]) - t0) / 1e3, "us")
for k, v in sorted(busy.items(), key=lambda x: -x[1]):
    print(f"  {k:36s} {v / 1e3:9.1f} us")
