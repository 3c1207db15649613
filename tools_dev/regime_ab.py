#!/usr/bin/env python3
"""Where the GRCh38 regime's extra time per batch goes.

The bench's `regime_grch38.c3_refseed` leg is C2's batch 0 translated into the
GRCh38-shaped genome (0.8 GB pac, past the MALL) and runs that ONE batch on
both caller streams; the headline C2 leg alternates two different batches.
This tool times the same stage on one genome at a time in these patterns:

    c2alt   C2 batches 0/1 alternating over 2 streams (the headline)
    c2b0    C2 batch 0 on both streams (the regime leg's pattern, chr21-sized pac)
    c2b1    C2 batch 1 on both streams
    c2b0s1  C2 batch 0, 1 stream
    c3r     c3_refseed (batch 0 in the GRCh38-shaped genome) on both streams
    c3rs1   c3_refseed, 1 stream

c2b0 vs c2alt separates batch 0's own shape (its serial heavy-read tail lands
on both streams at once) from the genome; c3r vs c2b0 is the genome alone.

    python tools_dev/regime_ab.py --modes c2alt,c2b0,c3r [--steps 20]
"""
import argparse
import json
import os
import sys
import time

REPO = os.path.normpath(os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "bwa-flow_amd", "python"))

import numpy as np  # noqa: E402
import torch  # noqa: E402

import bench  # noqa: E402
from bwagpu import workload  # noqa: E402
from bwagpu.engine import Engine  # noqa: E402


STREAMS = []


def timed(eng, dbs, pattern, n_streams, steps, warm=2, stats=False, prof=False):
    """pattern: list of batch indices, step i runs dbs[pattern[i % len]] on stream i % n_streams;
    stats / prof: the bench's per-batch counters and HIP events around the extension launches"""
    streams = STREAMS[:n_streams]
    slots = []
    for i in range(steps):
        d, _ = dbs[pattern[i % len(pattern)]]
        slots.append(d.add_out())
    for i in range(warm):
        d, _ = dbs[pattern[i % len(pattern)]]
        d.run(eng, streams[i % n_streams].cuda_stream, 0, stats=False)
    torch.cuda.synchronize()
    if prof:
        eng.prof_start(3 * steps)
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    t0 = time.perf_counter()
    ev0.record(streams[0])
    for x in streams[1:]:
        x.wait_event(ev0)
    for i in range(steps):
        d, _ = dbs[pattern[i % len(pattern)]]
        d.run(eng, streams[i % n_streams].cuda_stream, slots[i], stats=stats)
    for x in streams[1:]:
        e = torch.cuda.Event()
        e.record(x)
        streams[0].wait_event(e)
    ev1.record(streams[0])
    torch.cuda.synchronize()
    el = max(time.perf_counter() - t0, ev0.elapsed_time(ev1) / 1e3)
    if prof:
        eng.prof_start(0)
    ok = True
    for i in range(steps):
        d, chk = dbs[pattern[i % len(pattern)]]
        ok &= bool(chk(*d.results(slots[i])))
    return round(el * 1e3 / steps, 4), ok


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--modes", default="c2alt,c2b0,c2b1,c2b0s1,c3r,c3rs1")
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--stats", action="store_true")
    ap.add_argument("--prof", action="store_true")
    a = ap.parse_args()
    modes = a.modes.split(",")
    dev = torch.device("cuda:0")
    STREAMS.extend(torch.cuda.Stream(device=dev) for _ in range(2))  # one context takes <= 4 caller streams
    out = {}
    if any(m.startswith("c2") for m in modes):
        opt, gref, rbs = workload.load_fixture(with_ref=True)
        pac_t = torch.from_numpy(gref.pac).to(dev)
        eng = Engine(0, opt, gref.l_pac, gref.ann_offset, gref.ann_len, pac_device_ptr=pac_t.data_ptr())
        eng.set_device_read_len(max(int(np.diff(rb.batch.seq_off).max()) for rb in rbs))
        dbs = [(bench.DevBatch(rb.batch, dev), rb.check) for rb in rbs]
        pats = {"c2alt": ([0, 1], 2), "c2b0": ([0], 2), "c2b1": ([1], 2), "c2b0s1": ([0], 1)}
        for m in modes:
            if m in pats:
                p, ns = pats[m]
                out[m] = timed(eng, dbs, p, ns, a.steps, stats=a.stats, prof=a.prof)
                print(m, out[m], file=sys.stderr, flush=True)
        eng.close()
        del pac_t, dbs
        torch.cuda.empty_cache()
    if any(m.startswith("c3r") for m in modes):
        opt, g2, s = workload.load_c3_refseed()
        pac_t = torch.from_numpy(g2.pac).to(dev)
        eng = Engine(0, opt, g2.l_pac, g2.ann_offset, g2.ann_len, pac_device_ptr=pac_t.data_ptr())
        eng.set_device_read_len(int(np.diff(s.batch.seq_off).max()))

        def chk(regs, n):
            return s.check(regs, n) is None
        dbs = [(bench.DevBatch(s.batch, dev), chk)]
        pats = {"c3r": ([0], 2), "c3rs1": ([0], 1)}
        for m in modes:
            if m in pats:
                p, ns = pats[m]
                out[m] = timed(eng, dbs, p, ns, a.steps, stats=a.stats, prof=a.prof)
                print(m, out[m], file=sys.stderr, flush=True)
        eng.close()
    print(json.dumps({k: {"ms_per_batch": v[0], "parity": v[1]} for k, v in out.items()}), flush=True)


if __name__ == "__main__":
    main()
