"""Timing of bwagpu_sw_stream (the FPGA wire format entry) on a C2 batch.

The stream is what the reference's host packs (packReadData,
src/fpga/FPGAPipeline.cpp:194-343); here the oracle's restatement packs it from
the C2 fixture's reference-seeded chains, outside any timed region, the way a
bwa-flow host would hand it over.  Timed: the whole call (host buffers in,
records out: H2D + decode + extension + D2H), and the oracle computing the
same records on one core.  Prints one JSON line.
"""
import argparse
import json
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "bwa-flow_amd", "python"))
sys.path.insert(0, os.path.join(REPO, "oracle"))
sys.path.insert(0, os.path.join(REPO, "tests"))

import oracle  # noqa: E402
from bwagpu import workload  # noqa: E402
from bwagpu.engine import Engine  # noqa: E402
from test_fpga_stream_oracle import sub_batch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--cpu-reads", type=int, default=4000)
    args = ap.parse_args()
    opt, ref, bs = workload.load_fixture()
    b = bs[0].batch
    r = oracle.Ref(ref.l_pac, ref.ann_offset, ref.ann_len, ref.pac)
    words, nt, packed, _ = oracle.fpga_pack(opt, r, b)
    eng = Engine(0, opt, ref.l_pac, ref.ann_offset, ref.ann_len, pac=ref.pac)
    got = eng.sw_stream(words, nt)  # warm-up (allocations)
    ts = []
    for _ in range(args.reps):
        t0 = time.perf_counter()
        got = eng.sw_stream(words, nt)
        ts.append(time.perf_counter() - t0)
    t = float(np.median(ts))
    # parity of the whole stream, and the oracle's time on a slice
    want = oracle.fpga_sw(opt, r, words, nt)
    same = bool(np.array_equal(got, want))
    sb = sub_batch(b, 0, args.cpu_reads)
    w2, n2, _, _ = oracle.fpga_pack(opt, r, sb)
    t0 = time.perf_counter()
    oracle.fpga_sw(opt, r, w2, n2)
    tc = time.perf_counter() - t0
    print(json.dumps({
        "entry": "bwagpu_sw_stream", "reads_packed": int(packed.sum()), "tasks": int(nt),
        "stream_MB": round(words.nbytes / 1e6, 2), "ms_per_call": round(t * 1e3, 3),
        "mreads_s": round(packed.sum() / t / 1e6, 3), "mtasks_s": round(nt / t / 1e6, 3),
        "parity": same, "cpu_oracle_tasks_s_1core": round(n2 / tc, 1), "cpu_sample_reads": args.cpu_reads,
    }))


if __name__ == "__main__":
    main()
