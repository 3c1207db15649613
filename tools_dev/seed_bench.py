"""Seeding benchmark: bwagpu_collect_intv (mem_collect_intv on the device) over
the reference-seeded C2 batch's reads (tests/golden/c2_refseed.npz, 66,668 x
150 bp) against the chr21-sized golden genome's FM-index
(bench_data/c2_bwt.npz, built by the reference's bwa_idx_build:
`oracle/_ref/gen_seed /tmp/x 1 0 150 46709983 0`, then saved with np.savez_compressed).
Parity: a sample of reads checked against the oracle (oracle/seed.c).
CPU: the oracle restatement, one thread, on a bounded sample.
Prints one JSON line."""
import argparse
import json
import os
import sys
import time

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
sys.path.insert(0, os.path.join(ROOT, "bwa-flow_amd", "python"))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
sys.path.insert(0, os.path.join(ROOT, "tests"))

import golden_io as G  # noqa: E402
import oracle  # noqa: E402
from bwagpu.engine import Engine  # noqa: E402
from bwagpu.workload import load_fixture  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--check", type=int, default=2000)
    ap.add_argument("--cpu-reads", type=int, default=4000)
    ap.add_argument("--budget", type=int, default=-1, help="bwt_extend calls per read on one lane (-1: library default)")
    ap.add_argument("--mult", type=str, default="", help="comma list: also time k copies of the batch in one call")
    ap.add_argument("--reads", type=str, default="", help="first:count: only these reads of the batch")
    a = ap.parse_args()
    z = np.load(os.path.join(ROOT, "bench_data", "c2_bwt.npz"))
    hdr, words = z["hdr"], z["words"]
    _, _, batches = load_fixture(with_ref=False)
    b = batches[0].batch
    if a.reads:
        f, c = (int(v) for v in a.reads.split(":"))
        so = b.seq_off[f:f + c + 1]
        b = type("B", (), dict(seq_off=(so - so[0]).astype(np.int64), seq=b.seq[so[0]:so[-1]], n_reads=c))
        a.check = min(a.check, c)
        a.cpu_reads = min(a.cpu_reads, c)
    refd = G.load_ref()
    opt, *_ = G.load_chain_set("c1_default")
    eng = Engine(0, opt, refd["l_pac"], refd["ann_offset"], refd["ann_len"], pac=refd["pac"])
    eng.set_bwt(hdr, words)
    if a.budget >= 0:
        eng.seed_budget(a.budget)
    n, iv = eng.collect_intv(b.seq_off, b.seq)  # warm-up
    t0 = time.perf_counter()
    for _ in range(a.reps):
        n, iv = eng.collect_intv(b.seq_off, b.seq)
    ms = (time.perf_counter() - t0) * 1e3 / a.reps
    k = a.check
    sub_off = b.seq_off[:k + 1]
    want_n, want = oracle.collect_intv(hdr, words, np.array([19, 10, 20], np.int32), 1.5, sub_off,
                                       b.seq[:sub_off[-1]])
    got = np.column_stack([iv["x"], iv["info"]]).astype(np.uint64)[:int(want_n.sum())]
    parity = bool(np.array_equal(n[:k], want_n) and np.array_equal(got, want))
    c = a.cpu_reads
    t0 = time.perf_counter()
    oracle.collect_intv(hdr, words, np.array([19, 10, 20], np.int32), 1.5, b.seq_off[:c + 1], b.seq[:b.seq_off[c]])
    cpu_s = time.perf_counter() - t0
    scaling = {}
    for k in [int(x) for x in a.mult.split(",") if x]:
        so = np.concatenate([[0], np.cumsum(np.tile(np.diff(b.seq_off), k))]).astype(np.int64)
        sq = np.tile(b.seq, k)
        eng.collect_intv(so, sq, out_cap=int(n.sum()) * k)
        t0 = time.perf_counter()
        for _ in range(3):
            eng.collect_intv(so, sq, out_cap=int(n.sum()) * k)
        scaling[k] = round((time.perf_counter() - t0) * 1e3 / 3, 2)
    slen = (iv["info"] & 0xffffffff).astype(np.int64) - (iv["info"] >> 32).astype(np.int64)
    print(json.dumps({
        "metric": "seeding_reads_per_s", "reads": int(b.n_reads), "ms_per_batch": round(ms, 3),
        "gpu_reads_per_s": round(b.n_reads / ms * 1e3), "intervals": int(n.sum()),
        "intervals_per_read": round(float(n.mean()), 2), "mean_interval_len": round(float(slen.mean()), 1),
        "parity_sample_reads": k, "parity": parity,
        "cpu_baseline": {"kind": "port", "threads": 1, "reads": c, "reads_per_s": round(c / cpu_s)},
        "ms_for_k_batches_in_one_call": scaling,
        "scope": "host API wall incl. H2D of reads, D2H of packed intervals; BWT resident"}))


if __name__ == "__main__":
    main()
