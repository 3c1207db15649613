#!/usr/bin/env python3
"""TEST INFRASTRUCTURE: make tests/golden/c3_refseed.npz — reference-seeded
chains in the GRCh38 regime.

The C2 fixture's batch 0 (tests/golden/c2_refseed.npz: 66,668 reads whose
chains bwa's own seeding + chaining produced on a chr21-sized genome) is
translated into a GRCh38-shaped reference: the golden genome twice, before
and after the 195 GRCh38-shaped contigs (bwagpu.workload.GoldenInGrch38); the
even reads' chains go to the first copy (its reverse strand lies past 2-strand
2^32), the odd reads' to the second (past forward 2^31); the pac is 0.80 GB.
The expected answers are the REFERENCE's, through oracle/_ref/libbwaref.so on
the combined genome: mem_chain2aln (bwa/bwamem.c:641-795) and mem_reg2aln
(bwa/bwamem.c:1104-1174) on every output region.  Stored: the pac digest, the
translated batch's digest, per-read region counts, the SHA-256 of the 88-byte
records, per-256-read chunk digests of the regions and of the CIGAR/MD output.

    python oracle/gen_c3r_fixture.py [--out tests/golden/c3_refseed.npz]
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
from bwagpu import workload  # noqa: E402
from bwagpu.engine import compact  # noqa: E402

C2_BATCH = 0


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default=workload.C3R_FIXTURE)
    ap.add_argument("--threads", type=int, default=min(8, os.cpu_count() or 1))
    a = ap.parse_args()
    if oracle.ref_lib() is None:
        sys.exit("oracle/_ref/libbwaref.so is required (make -C oracle ref)")
    t0 = time.time()
    opt, _, bs = workload.load_fixture(with_ref=False)
    g = workload.GoldenInGrch38()
    b = g.translate(bs[C2_BATCH].batch)
    print(f"genome: l_pac {g.l_pac} ({len(g.ann_len)} contigs, golden copies at 0 and {g.off_b}), {time.time() - t0:.1f} s",
          file=sys.stderr)
    R = oracle.Ref(g.l_pac, g.ann_offset, g.ann_len, g.pac)
    t1 = time.time()
    regs, n, _ = oracle.chain2aln("ref", opt, R, b, n_threads=a.threads)
    t_ref = time.time() - t1
    c = np.ascontiguousarray(compact(b, regs, n))
    jobs = workload.reg2aln_jobs(b, regs, n)
    t1 = time.time()
    aln, cig, md = oracle.reg2aln("ref", opt, R, jobs, b.seq, workload.C3_MAX_OPS, workload.C3_MAX_MD)
    t_cig = time.time() - t1
    st = workload.c3_coverage(g, b, c)
    # the translation must not change the answer's shape: same counts as on the golden genome
    assert np.array_equal(n.astype(np.int32), bs[C2_BATCH].reg_n), "region counts differ from the C2 fixture's"
    out = dict(opt_int=np.array([opt[k] for k in workload.OPT_KEYS], np.int32), opt_mat=opt["mat"].astype(np.int8),
               c2_batch=np.int32(C2_BATCH), l_pac=np.int64(g.l_pac), off_b=np.int64(g.off_b),
               pac_sha256=np.frombuffer(hashlib.sha256(g.pac).digest(), np.uint8),
               batch_sha256=np.frombuffer(workload.batch_digest(b), np.uint8),
               reg_n=n.astype(np.uint16),
               regs_sha256=np.frombuffer(hashlib.sha256(c.tobytes()).digest(), np.uint8),
               regs_chunks=workload.chunk_digests(b, c, n),
               cigar_chunks=workload.cigar_chunk_digests(jobs, aln, cig, md),
               coverage=np.array([st[k] for k in workload.C3_COVERAGE_KEYS], np.int64))
    print(f"{b.n_reads} reads, {b.n_chains} chains, {b.n_seeds} seeds, {len(c)} regions (reference "
          f"mem_chain2aln {t_ref:.1f} s on {a.threads} threads), {len(jobs)} CIGAR jobs ({t_cig:.1f} s); {st}", file=sys.stderr)
    np.savez_compressed(a.out, **out)
    print(f"wrote {a.out}: {os.path.getsize(a.out) / 1e6:.2f} MB", file=sys.stderr)


if __name__ == "__main__":
    main()
