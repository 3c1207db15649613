#!/usr/bin/env python3
"""TEST INFRASTRUCTURE: make tests/golden/c3_grch38.npz, the C3 / C5 regime
fixture (BASELINE.json configs[2] and configs[4]).

The reference is GRCh38-shaped (bwa-flow_amd/tools/synth.cpp grch38_layout /
grch38_genome): 195 contigs, l_pac = 3,099,734,149, so forward coordinates
pass 2^31, 2-strand coordinates pass 2^32 and the 0.78 GB pac does not fit the
256 MB MALL.  A bwa index of it cannot be built here (hours, tens of GB), so
the chains are the synthetic generator's (exact-match seeds along each read's
true origin, bwa-flow_amd/tools/synth.cpp reads_core placement 1: contigs
weighted by length, one pair in ten across a contig junction).  The expected
answers are the REFERENCE's own:

  * mem_chain2aln (bwa/bwamem.c:641-795) per chain, through
    oracle/_ref/libbwaref.so (compiled from /root/reference/bwa) — it needs only
    the bns contig table and the pac;
  * mem_reg2aln (bwa/bwamem.c:1104-1174) on every output region
    (ref_reg2aln_batch), whose bns_pos2rid search runs over all 195 contigs.

Stored: the generator parameters, SHA-256 of the pac and of each regenerated
batch (so a generator change is caught before any comparison), per-read region
counts, the SHA-256 of the reference's 88-byte records, and per-256-read chunk
digests of regions and CIGAR/MD output (to localise a mismatch).  Two batches:
"c3" (2x150 bp, 33,334 pairs = 10.0 Mbases) and "c5" (thirds of 2x100 /
2x150 / 2x250, 30,000 pairs = 10.0 Mbases).

    python oracle/gen_c3_fixture.py [--out tests/golden/c3_grch38.npz]
"""
import argparse
import hashlib
import os
import sys
import time

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
sys.path.insert(0, HERE)
sys.path.insert(0, os.path.join(REPO, "bwa-flow_amd", "python"))

import oracle  # noqa: E402
from bwagpu import abi, workload  # noqa: E402
from bwagpu.engine import compact  # noqa: E402
from bwagpu.synth import Grch38Ref, synth_batch  # noqa: E402

GENOME_SEED = 38
SETS = {"c3": dict(read_seed=3003, pairs=33_334, len_mode=150),
        "c5": dict(read_seed=5005, pairs=30_000, len_mode=0)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default=workload.C3_FIXTURE)
    ap.add_argument("--threads", type=int, default=min(8, os.cpu_count() or 1))
    a = ap.parse_args()
    if oracle.ref_lib() is None:
        sys.exit("oracle/_ref/libbwaref.so is required (make -C oracle ref)")
    t0 = time.time()
    g = Grch38Ref(GENOME_SEED)
    print(f"genome: l_pac {g.l_pac}, {len(g.ann_len)} contigs, {time.time() - t0:.1f} s", file=sys.stderr)
    opt = abi.default_opt()
    R = oracle.Ref(g.l_pac, g.ann_offset, g.ann_len, g.pac)
    out = dict(genome_seed=np.int64(GENOME_SEED), l_pac=np.int64(g.l_pac), ann_offset=g.ann_offset,
               ann_len=g.ann_len, pac_sha256=np.frombuffer(hashlib.sha256(g.pac).digest(), np.uint8),
               opt_int=np.array([opt[k] for k in workload.OPT_KEYS], np.int32), opt_mat=opt["mat"].astype(np.int8))
    for name, p in SETS.items():
        b = synth_batch(g, p["read_seed"], p["pairs"], p["len_mode"], genome_wide=True)
        t1 = time.time()
        regs, n, _ = oracle.chain2aln("ref", opt, R, b, n_threads=a.threads)
        t_ref = time.time() - t1
        c = np.ascontiguousarray(compact(b, regs, n))
        jobs = workload.reg2aln_jobs(b, regs, n)
        t1 = time.time()
        aln, cig, md = oracle.reg2aln("ref", opt, R, jobs, b.seq, workload.C3_MAX_OPS, workload.C3_MAX_MD)
        t_cig = time.time() - t1
        st = workload.c3_coverage(g, b, c)
        out.update({
            f"{name}_read_seed": np.int64(p["read_seed"]), f"{name}_pairs": np.int32(p["pairs"]),
            f"{name}_len_mode": np.int32(p["len_mode"]),
            f"{name}_batch_sha256": np.frombuffer(workload.batch_digest(b), np.uint8),
            f"{name}_reg_n": n.astype(np.uint16),
            f"{name}_regs_sha256": np.frombuffer(hashlib.sha256(c.tobytes()).digest(), np.uint8),
            f"{name}_regs_chunks": workload.chunk_digests(b, c, n),
            f"{name}_cigar_chunks": workload.cigar_chunk_digests(jobs, aln, cig, md),
            f"{name}_coverage": np.array([st[k] for k in workload.C3_COVERAGE_KEYS], np.int64),
        })
        print(f"{name}: {b.n_reads} reads, {b.n_chains} chains, {b.n_seeds} seeds, {len(c)} regions "
              f"(reference mem_chain2aln {t_ref:.1f} s on {a.threads} threads), {len(jobs)} CIGAR jobs "
              f"({t_cig:.1f} s, 1 thread); {st}", file=sys.stderr)
    np.savez_compressed(a.out, **out)
    print(f"wrote {a.out}: {os.path.getsize(a.out) / 1e6:.2f} MB", file=sys.stderr)


if __name__ == "__main__":
    main()
