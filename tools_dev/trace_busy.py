"""Busy time and critical path of the stage bench from a rocprofv3 kernel trace
(tools_dev/gpu_trace.sh).

    python tools_dev/trace_busy.py <run_kernel_trace.csv> [warmup] [steps] [kernel] [--timeline K]

Launch sequences are split at spec_reads_kernel (the first launch of every
mem_chain2aln batch) in launch (correlation) order; sequences warmup ..
warmup+steps-1 are the timed steps.  For the named kernel (default the
dominant spec_ext2_kernel<5>; a name without its last template argument
takes both sides of the phased pair) it prints the SUM of its launch durations and the
UNION of its launch intervals inside the timed window (the busy time: overlapping
launches of the two caller streams count once), per step, beside the window's
wall time per step; then each kernel family's union per step.  --timeline K
prints sequence K's launches relative to its first start (queue, start, end).
"""
import csv
import json
import sys
from collections import defaultdict


def union(iv):
    tot, cur_s, cur_e = 0, None, None
    for s, e in sorted(iv):
        if cur_e is None or s > cur_e:
            if cur_e is not None:
                tot += cur_e - cur_s
            cur_s, cur_e = s, e
        else:
            cur_e = max(cur_e, e)
    if cur_e is not None:
        tot += cur_e - cur_s
    return tot


def short(name):
    n = name.split("(")[0].replace("void ", "").replace("bwagpu::", "").replace("(anonymous namespace)::", "")
    return n


def load(path):
    rows = []
    for r in csv.DictReader(open(path)):
        rows.append(dict(name=short(r["Kernel_Name"]), q=int(r["Queue_Id"]), cid=int(r["Correlation_Id"]),
                         s=int(r["Start_Timestamp"]), e=int(r["End_Timestamp"])))
    rows.sort(key=lambda r: r["cid"])
    return rows


def sequences(rows):
    seqs, cur = [], None
    for r in rows:
        if r["name"] == "spec_reads_kernel":
            cur = []
            seqs.append(cur)
        if cur is not None and not r["name"].startswith("__amd"):
            cur.append(r)
    return seqs


def analyse(path, warmup=3, steps=20, kernel="spec_ext2_kernel<5>"):
    rows = load(path)
    seqs = sequences(rows)
    timed = [r for q in seqs[warmup:warmup + steps] for r in q]
    t0 = min(r["s"] for r in timed)
    t1 = max(r["e"] for r in timed)
    wall = (t1 - t0) / 1e6
    # a name without its last template argument (spec_side4_kernel<16, 10, true>)
    # takes every instance (the phased pair's left and right sides)
    pre = kernel[:-1] + ", "
    k = [(r["s"], r["e"]) for r in timed if r["name"] == kernel or r["name"].startswith(pre)]
    per = 2 if any(r["name"].startswith(pre) for r in timed) else 1  # launches per pair
    fam = defaultdict(list)
    for r in timed:
        fam[r["name"]].append((r["s"], r["e"]))
    out = {
        "trace": path, "sequences": len(seqs), "timed_steps": steps,
        "window_ms_per_step": round(wall / steps, 4),
        "gpu_busy_ms_per_step": round(union([(r["s"], r["e"]) for r in timed]) / 1e6 / steps, 4),
        "kernel": kernel, "launches": len(k),
        "kernel_sum_ms_per_step": round(sum(e - s for s, e in k) / 1e6 / steps, 4),
        "kernel_busy_ms_per_step": round(union(k) / 1e6 / steps, 4),
        "kernel_avg_launch_ms": round(sum(e - s for s, e in k) / 1e6 / max(len(k), 1), 4),
        "kernel_avg_pair_ms": round(per * sum(e - s for s, e in k) / 1e6 / max(len(k), 1), 4),
        "families_busy_ms_per_step": {n: round(union(v) / 1e6 / steps, 4)
                                      for n, v in sorted(fam.items(), key=lambda x: -union(x[1]))},
    }
    return out, seqs


def timeline(seqs, k):
    q = seqs[k]
    t0 = min(r["s"] for r in q)
    for r in sorted(q, key=lambda r: r["s"]):
        print(f"q{r['q']:<3} {(r['s'] - t0) / 1e3:9.1f} {(r['e'] - t0) / 1e3:9.1f} {(r['e'] - r['s']) / 1e3:8.1f}  {r['name']}")


if __name__ == "__main__":
    a = [x for x in sys.argv[1:] if not x.startswith("--")]
    tl = None
    if "--timeline" in sys.argv:
        tl = int(sys.argv[sys.argv.index("--timeline") + 1])
        a = [x for x in a if x != str(tl)]
    path = a[0]
    warmup = int(a[1]) if len(a) > 1 else 3
    steps = int(a[2]) if len(a) > 2 else 20
    kern = a[3] if len(a) > 3 else "spec_ext2_kernel<5>"
    out, seqs = analyse(path, warmup, steps, kern)
    print(json.dumps(out, indent=1))
    if tl is not None:
        timeline(seqs, tl)
