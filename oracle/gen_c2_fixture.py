#!/usr/bin/env python3
"""TEST INFRASTRUCTURE: make tests/golden/c2_refseed.npz, the bench's C2 workload
(and, with --length mix, tests/golden/c5_refseed.npz: one mixed 2x100/150/250
ChainsRecord of the same genome, the bench's c5_refseed leg).

Runs oracle/_ref/gen_golden (the REFERENCE's own bwa index + seeding +
chaining + mem_chain2aln, see gen_golden.c) on a chr21-sized synthetic genome
(46,709,983 bases, three contigs, the golden genome's per-Mb repeat / tandem /
N-run structure) with 2x150 bp pairs, and packs two ChainsRecord-sized batches
(66,668 reads = 10.0 Mbases nominal each, src/Pipeline.cpp:123,146) as the
SeqsToChains stage hands them to ChainsToRegions (src/Pipeline.cpp:503-544):

  * reads: 2-bit packed bases + the positions of N (nt4 code 4) + lengths;
  * chains: seeds per chain, chains per read, rid, frac_rep;
  * seeds: mem_seed_t fields (rbeg delta-coded along the batch);
  * expected output: regions per read and the SHA-256 of the reference's
    mem_alnreg_t records (88 B each, read order) — the bench checks every
    timed step's output against it;
  * the genome's parameters and the SHA-256 of the reference's .pac, which
    bench.py regenerates with bwa-flow_amd/tools/synth.cpp (golden_genome)
    and checks before use.

The genome itself is not stored (11.7 MB of 2-bit bases): it is a pure
function of (length, seed 1234) and bwa's N filling (bntseq.c:261, srand48(11)).

    python oracle/gen_c2_fixture.py [--out tests/golden/c2_refseed.npz]
    python oracle/gen_c2_fixture.py --length mix --pairs 30000 --batches 1 --read-seed 2027 \
        --out tests/golden/c5_refseed.npz
"""
import argparse
import hashlib
import os
import subprocess
import sys
import tempfile

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
GENOME_LEN = 46_709_983  # GRCh38 chr21
READ_SEED = 2026
PAIRS = 66_668           # two batches of 33,334 pairs
BATCH_READS = 66_668

SEED_DT = np.dtype([("rbeg", "<i8"), ("qbeg", "<i4"), ("len", "<i4"), ("score", "<i4"), ("pad_", "<i4")])


def rd(d, name, dt):
    return np.fromfile(os.path.join(d, name + ".bin"), dtype=dt)


def pack_reads(seq, seq_off):
    lens = np.diff(seq_off).astype(np.int64)
    assert lens.max() <= 255
    npos = np.nonzero(seq == 4)[0].astype(np.int32)
    s = (seq & 3).astype(np.uint8)
    s = np.concatenate([s, np.zeros((-len(s)) % 4, np.uint8)]).reshape(-1, 4)
    packed = (s[:, 0] << 6 | s[:, 1] << 4 | s[:, 2] << 2 | s[:, 3]).astype(np.uint8)
    return packed, npos, lens.astype(np.uint8)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default=os.path.join(REPO, "tests", "golden", "c2_refseed.npz"))
    ap.add_argument("--length", default="150", help="150 | mix (2x100 / 2x150 / 2x250 pairs in thirds)")
    ap.add_argument("--pairs", type=int, default=PAIRS)
    ap.add_argument("--batches", type=int, default=2)
    ap.add_argument("--read-seed", type=int, default=READ_SEED)
    a = ap.parse_args()
    gen = os.path.join(HERE, "_ref", "gen_golden")
    with tempfile.TemporaryDirectory(prefix="c2fix_") as d:
        subprocess.run([gen, d, str(a.read_seed), str(a.pairs), a.length, "0", str(GENOME_LEN), "0"], check=True)
        pac = rd(d, "pac", np.uint8)
        l_pac = int(rd(d, "l_pac", np.int64)[0])
        ann_offset, ann_len = rd(d, "ann_offset", np.int64), rd(d, "ann_len", np.int32)
        seq_off, seq = rd(d, "seq_off", np.int64), rd(d, "seq", np.uint8)
        rco, cso = rd(d, "read_chain_off", np.int32), rd(d, "chain_seed_off", np.int32)
        rid, frac = rd(d, "chain_rid", np.int32), rd(d, "chain_frac_rep", np.float32)
        seeds = rd(d, "seeds", SEED_DT)
        regs, reg_n = rd(d, "regs", np.uint8).reshape(-1, 88), rd(d, "reg_n", np.int32)
        opt_int, opt_mat = rd(d, "opt_int", np.int32), rd(d, "opt_mat", np.int8)
    assert l_pac == GENOME_LEN
    n_reads = len(seq_off) - 1
    assert n_reads == 2 * a.pairs, n_reads
    per = n_reads // a.batches
    per -= per & 1  # whole pairs per batch
    out = dict(genome_len=np.int64(l_pac), genome_seed=np.int64(1234), ann_offset=ann_offset, ann_len=ann_len,
               pac_sha256=np.frombuffer(hashlib.sha256(pac.tobytes()).digest(), np.uint8),
               opt_int=opt_int, opt_mat=opt_mat, n_batches=np.int32(a.batches), read_seed=np.int64(a.read_seed))
    reg_off = np.concatenate([[0], np.cumsum(reg_n)])
    for k in range(a.batches):
        r0, r1 = k * per, (k + 1) * per
        c0, c1 = int(rco[r0]), int(rco[r1])
        s0, s1 = int(cso[c0]), int(cso[c1])
        q0, q1 = int(seq_off[r0]), int(seq_off[r1])
        packed, npos, lens = pack_reads(seq[q0:q1], seq_off[r0:r1 + 1] - q0)
        sd = seeds[s0:s1]
        rb = sd["rbeg"].astype(np.int64)
        assert rb.max() < 2 ** 31 and sd["len"].max() < 65536 and reg_n.max() < 65536
        want = regs[reg_off[r0]:reg_off[r1]]
        p = f"b{k}_"
        out.update({
            p + "seq2": packed, p + "npos": npos, p + "lens": lens,
            p + "read_nchain": np.diff(rco[r0:r1 + 1]).astype(np.uint16),
            p + "chain_nseed": np.diff(cso[c0:c1 + 1]).astype(np.uint16),
            p + "chain_rid": rid[c0:c1].astype(np.int8), p + "chain_frac_rep": frac[c0:c1],
            p + "rbeg_delta": np.diff(np.concatenate([[0], rb])).astype(np.int32),
            p + "qbeg": sd["qbeg"].astype(np.uint16), p + "slen": sd["len"].astype(np.uint16),
            p + "score": sd["score"].astype(np.uint16),
            p + "reg_n": reg_n[r0:r1].astype(np.uint16),
            p + "regs_sha256": np.frombuffer(hashlib.sha256(np.ascontiguousarray(want).tobytes()).digest(), np.uint8),
        })
        print(f"batch {k}: {r1 - r0} reads, {c1 - c0} chains, {s1 - s0} seeds, {len(want)} regions", file=sys.stderr)
    np.savez_compressed(a.out, **out)
    print(f"wrote {a.out}: {os.path.getsize(a.out) / 1e6:.2f} MB", file=sys.stderr)


if __name__ == "__main__":
    main()
