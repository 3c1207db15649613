"""Selection-kernel time per mem_chain2aln batch from a rocprofv3 kernel trace
(tools_dev/gpu_trace.sh): the union of the intervals of every spec_* launch
that is not an extension round (spec_ext*), per batch sequence, averaged over
the timed sequences; beside it each selection kernel's mean duration.

    python tools_dev/sel_union.py <run_kernel_trace.csv> [warmup]
"""
import sys
from collections import defaultdict

from trace_busy import load, sequences, union

path = sys.argv[1]
warmup = int(sys.argv[2]) if len(sys.argv) > 2 else 3
seqs = sequences(load(path))[warmup:]
tot, per = [], defaultdict(list)
for sq in seqs:
    sel = [r for r in sq if r["name"].startswith("spec_") and not r["name"].startswith("spec_ext")]
    tot.append(union([(r["s"], r["e"]) for r in sel]))
    for r in sel:
        per[r["name"]].append(r["e"] - r["s"])
print(f"batches {len(seqs)}  selection union {sum(tot) / len(tot) / 1e6:.3f} ms/batch")
for n, v in sorted(per.items(), key=lambda kv: -sum(kv[1])):
    print(f"  {n:40s} {len(v) / len(seqs):5.1f}/batch  mean {sum(v) / len(v) / 1e3:8.1f} us")
