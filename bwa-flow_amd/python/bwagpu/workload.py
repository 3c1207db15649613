"""The bench's C2 workload: reference-seeded ChainsRecords from
tests/golden/c2_refseed.npz (made by oracle/gen_c2_fixture.py with the
reference's own bwa index + seeding + chaining on a chr21-sized synthetic
genome).  The genome is regenerated here (tools/synth.cpp golden_genome) and
checked against the SHA-256 of the reference's pac; every batch carries the
reference's region count per read and the SHA-256 of its mem_alnreg_t
records, so any run can be checked bit for bit without the reference.
Input loading only — never part of the measured path."""
from __future__ import annotations

import hashlib
import os

import numpy as np

from . import abi
from .engine import Batch, compact
from .synth import GoldenRef

REPO = os.path.normpath(os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "..", ".."))
C2_FIXTURE = os.path.join(REPO, "tests", "golden", "c2_refseed.npz")
# one mixed 2x100 / 2x150 / 2x250 ChainsRecord on the same genome, seeded and
# chained by the reference (oracle/gen_c2_fixture.py --length mix): BASELINE.json configs[4]
C5_FIXTURE = os.path.join(REPO, "tests", "golden", "c5_refseed.npz")
OPT_KEYS = ("a", "b", "o_del", "e_del", "o_ins", "e_ins", "pen_clip5", "pen_clip3", "w", "zdrop")


class RefBatch:
    """one reference-seeded ChainsRecord and the reference's answer for it"""

    def __init__(self, batch: Batch, reg_n: np.ndarray, regs_sha256: bytes):
        self.batch, self.reg_n, self.regs_sha256 = batch, reg_n, regs_sha256

    def check(self, regs: np.ndarray, n: np.ndarray) -> bool:
        """bit-exact: per-read counts and every byte of every region; regs in
        the ABI's slot layout (read r's regions from chain_seed_off[read_chain_off[r]])"""
        if not np.array_equal(np.asarray(n, np.int64), self.reg_n.astype(np.int64)):
            return False
        return self.check_compact(compact(self.batch, regs, n), n)

    def check_compact(self, regs: np.ndarray, n: np.ndarray) -> bool:
        """the same for regions already concatenated in read order"""
        if not np.array_equal(np.asarray(n, np.int64), self.reg_n.astype(np.int64)):
            return False
        c = np.ascontiguousarray(regs[:int(np.asarray(n, np.int64).sum())])
        return hashlib.sha256(c.view(np.uint8).tobytes()).digest() == self.regs_sha256


def load_bwa_index(prefix: str):
    """a bwa index's FM-index and sampled suffix array from its files
    (bwt_dump_bwt / bwt_dump_sa, bwa/bwt.c:385-407; restored as
    bwt_restore_bwt / bwt_restore_sa do, 421-462) -> (hdr int64[8]: primary,
    L2[0..4], seq_len, bwt_size; occurrence words uint32; sa uint64 with
    sa[0] = -1 as bwa sets it; sa_intv)"""
    raw = np.fromfile(prefix + ".bwt", np.uint8)
    head = raw[:40].view(np.uint64)
    words = raw[40:].view(np.uint32)
    primary, l2 = int(head[0]), [0] + [int(x) for x in head[1:5]]
    sraw = np.fromfile(prefix + ".sa", np.uint8)
    sh = sraw[:56].view(np.uint64)
    if int(sh[0]) != primary or int(sh[6]) != l2[4]:
        raise RuntimeError("SA-BWT inconsistency")
    sa_intv, seq_len = int(sh[5]), int(sh[6])
    n_sa = (seq_len + sa_intv) // sa_intv
    sa = np.empty(n_sa, np.uint64)
    sa[0] = np.uint64(0xFFFFFFFFFFFFFFFF)
    sa[1:] = sraw[56:56 + 8 * (n_sa - 1)].view(np.uint64)
    hdr = np.array([primary, *l2, seq_len, len(words)], np.int64)
    return hdr, words, sa, sa_intv


# ---------------------------------------------------------------- C3 / C5 regime
# tests/golden/c3_grch38.npz (oracle/gen_c3_fixture.py): synthetic chains on a
# GRCh38-shaped genome (195 contigs, l_pac 3.1e9) with the reference's own
# mem_chain2aln / mem_reg2aln answers as digests.
C3_FIXTURE = os.path.join(REPO, "tests", "golden", "c3_grch38.npz")
C3_MAX_OPS, C3_MAX_MD = 128, 1024
C3_CHUNK = 256  # reads (regions) / jobs per chunk digest
C3_COVERAGE_KEYS = ("seeds_fwd_ge_2^31", "seeds_ge_2^32", "regs_fwd_ge_2^31", "regs_ge_2^32", "contigs_hit",
                    "regs_small_contigs", "regs_at_contig_edge")
ALN_FIELDS = ("pos", "rid", "is_rev", "n_cigar", "NM", "md_len", "status")


def batch_digest(b: Batch) -> bytes:
    """SHA-256 over every array of a flattened ChainsRecord"""
    h = hashlib.sha256()
    for a in (b.seq_off, b.seq, b.read_chain_off, b.chain_seed_off, b.chain_rid, b.chain_frac_rep, b.seeds):
        h.update(np.ascontiguousarray(a).view(np.uint8).tobytes())
    return h.digest()


def chunk_digests(b: Batch, regs_compact: np.ndarray, n: np.ndarray) -> np.ndarray:
    """uint8[n_chunks, 32]: SHA-256 of the regions of reads [256k, 256k+256)"""
    off = np.concatenate([[0], np.cumsum(np.asarray(n, np.int64))])
    raw = np.ascontiguousarray(regs_compact).view(np.uint8).reshape(-1, 88) if len(regs_compact) else \
        np.zeros((0, 88), np.uint8)
    out = []
    for r0 in range(0, b.n_reads, C3_CHUNK):
        r1 = min(r0 + C3_CHUNK, b.n_reads)
        out.append(np.frombuffer(hashlib.sha256(raw[off[r0]:off[r1]].tobytes()).digest(), np.uint8))
    return np.array(out, np.uint8).reshape(-1, 32)


def cigar_chunk_digests(jobs, aln, cig, md) -> np.ndarray:
    """uint8[n_chunks, 32]: SHA-256 of 256 jobs' mem_reg2aln outputs (the record
    fields the reference fills, the CIGAR ops and the MD string)"""
    out = []
    rec = np.stack([aln[f].astype(np.int64) for f in ALN_FIELDS], axis=1) if len(aln) else np.zeros((0, 7), np.int64)
    for k0 in range(0, len(jobs), C3_CHUNK):
        h = hashlib.sha256()
        for k in range(k0, min(k0 + C3_CHUNK, len(jobs))):
            h.update(rec[k].tobytes())
            if aln["status"][k] == abi.ALN_OK:
                h.update(np.ascontiguousarray(cig[k, :int(aln["n_cigar"][k])]).tobytes())
                h.update(bytes(md[k, :int(aln["md_len"][k])]))
        out.append(np.frombuffer(h.digest(), np.uint8))
    return np.array(out, np.uint8).reshape(-1, 32)


def reg2aln_jobs(b: Batch, regs, n):
    """the SAM stage's mem_reg2aln jobs for one batch: every region of every read
    (bwa_wrapper.cpp:611 runs it on the regions a read outputs; all of them here)"""
    c = compact(b, regs, n)
    rd = np.repeat(np.arange(b.n_reads), n)
    jobs = np.zeros(len(c), abi.REG2ALN_TASK_DTYPE)
    for f in ("rb", "re", "qb", "qe", "truesc", "w"):
        jobs[f] = c[f]
    jobs["qoff"] = b.seq_off[rd]
    jobs["l_seq"] = b.seq_off[rd + 1] - b.seq_off[rd]
    return jobs


def c3_coverage(ref, b: Batch, regs_compact: np.ndarray) -> dict:
    """how much of the GRCh38 regime a batch exercises: coordinates past 2^31
    (forward) and 2^32 (2-strand), contigs, regions clipped at a contig edge"""
    L = int(ref.l_pac)
    s, c = b.seeds["rbeg"].astype(np.int64), regs_compact
    rb, re = c["rb"].astype(np.int64), c["re"].astype(np.int64)
    fwd = rb < L
    cb = np.asarray(ref.ann_offset, np.int64)[c["rid"]]
    ce = cb + np.asarray(ref.ann_len, np.int64)[c["rid"]]
    lo = np.where(fwd, cb, 2 * L - ce)  # the contig's span on the region's strand
    hi = np.where(fwd, ce, 2 * L - cb)
    return {"seeds_fwd_ge_2^31": int(((s >= 2 ** 31) & (s < L)).sum()), "seeds_ge_2^32": int((s >= 2 ** 32).sum()),
            "regs_fwd_ge_2^31": int(((rb >= 2 ** 31) & fwd).sum()), "regs_ge_2^32": int((rb >= 2 ** 32).sum()),
            "contigs_hit": int(len(np.unique(c["rid"]))), "regs_small_contigs": int((c["rid"] >= 25).sum()),
            "regs_at_contig_edge": int(((rb == lo) | (re == hi)).sum())}


class C3Set:
    """one C3/C5 batch regenerated from the fixture's seeds, with the
    reference's answers (region digests, CIGAR digests)"""

    def __init__(self, z, name: str, ref):
        from .synth import synth_batch
        self.name = name
        self.batch = synth_batch(ref, int(z[f"{name}_read_seed"]), int(z[f"{name}_pairs"]),
                                 int(z[f"{name}_len_mode"]), genome_wide=True)
        if batch_digest(self.batch) != z[f"{name}_batch_sha256"].tobytes():
            raise RuntimeError(f"regenerated {name} batch differs from the fixture's (tools/synth.cpp reads_core)")
        self.reg_n = z[f"{name}_reg_n"].astype(np.int32)
        self.regs_sha256 = z[f"{name}_regs_sha256"].tobytes()
        self.regs_chunks = z[f"{name}_regs_chunks"]
        self.cigar_chunks = z[f"{name}_cigar_chunks"]
        self.coverage = dict(zip(C3_COVERAGE_KEYS, z[f"{name}_coverage"].tolist()))

    def check(self, regs, n) -> str | None:
        """None when bit-exact with the reference, else where it first differs"""
        n = np.asarray(n, np.int32)
        if not np.array_equal(n, self.reg_n):
            k = int(np.argmax(n != self.reg_n))
            return f"region count of read {k}: {n[k]} vs {self.reg_n[k]}"
        c = np.ascontiguousarray(compact(self.batch, regs, n))
        if hashlib.sha256(c.tobytes()).digest() == self.regs_sha256:
            return None
        got = chunk_digests(self.batch, c, n)
        k = int(np.argmax(np.any(got != self.regs_chunks, axis=1)))
        return f"regions of reads [{k * C3_CHUNK}, {(k + 1) * C3_CHUNK}) differ"

    def check_cigar(self, jobs, aln, cig, md) -> str | None:
        got = cigar_chunk_digests(jobs, aln, cig, md)
        if got.shape == self.cigar_chunks.shape and np.array_equal(got, self.cigar_chunks):
            return None
        if got.shape != self.cigar_chunks.shape:
            return f"{len(jobs)} jobs: chunk count {len(got)} vs {len(self.cigar_chunks)}"
        k = int(np.argmax(np.any(got != self.cigar_chunks, axis=1)))
        return f"CIGAR jobs [{k * C3_CHUNK}, {(k + 1) * C3_CHUNK}) differ"


def load_c3(path: str = C3_FIXTURE, names=("c3", "c5"), ref=None):
    """-> (opt dict, Grch38Ref, {name: C3Set}); raises if the regenerated genome
    or a batch differs from the one the reference was run on"""
    from .synth import Grch38Ref
    z = np.load(path, allow_pickle=False)
    opt = dict(zip(OPT_KEYS, z["opt_int"].tolist()))
    opt["mat"] = z["opt_mat"].astype(np.int8)
    if ref is None:
        ref = Grch38Ref(int(z["genome_seed"]))
    if ref.l_pac != int(z["l_pac"]) or not np.array_equal(ref.ann_offset, z["ann_offset"]):
        raise RuntimeError("regenerated GRCh38 contig table differs from the fixture's")
    if hashlib.sha256(ref.pac).digest() != z["pac_sha256"].tobytes():
        raise RuntimeError("regenerated GRCh38-shaped genome differs from the fixture's (tools/synth.cpp)")
    return opt, ref, {nm: C3Set(z, nm, ref) for nm in names}


def _unpack_seq(seq2: np.ndarray, npos: np.ndarray, n: int) -> np.ndarray:
    s = np.empty(4 * len(seq2), np.uint8)
    for k in range(4):
        s[k::4] = (seq2 >> (6 - 2 * k)) & 3
    s = s[:n]
    s[npos] = 4
    return s


C3R_FIXTURE = os.path.join(REPO, "tests", "golden", "c3_refseed.npz")


class GoldenInGrch38:
    """the reference-seeded C2 genome (GoldenRef, the c2_refseed fixture's, 3
    contigs) twice around the GRCh38-shaped one: copy A at forward offset 0
    (contigs 0-2), the 195 GRCh38 contigs, copy B at the end (contigs 198-200);
    every offset is a multiple of 4 (the contig before a gap takes the pad
    bases, A).  Even reads of a translated batch go to copy A, whose reverse
    strand lies past 2-strand 2^32; odd reads to copy B, past forward 2^31.
    A golden coordinate x (either strand) becomes, in copy B, x + offB (forward
    p -> p + offB, reverse 2l-1-p -> 2L-1-(p + offB) = x + offB as L = offB + l);
    in copy A, x on the forward strand and x + 2(L - l) on the reverse."""

    def __init__(self, grch=None, golden=None):
        from .synth import GoldenRef, Grch38Ref
        z = np.load(C2_FIXTURE, allow_pickle=False)
        grch = grch if grch is not None else Grch38Ref(38)
        golden = golden if golden is not None else GoldenRef(int(z["genome_len"]), int(z["genome_seed"]))

        def body(pac, n):  # the bytes of n bases, pad bases of the last byte zeroed (A)
            h = np.asarray(pac[:(n + 3) // 4], np.uint8).copy()
            if n & 3:
                h[-1] &= np.uint8((0xff << (2 * (4 - (n & 3)))) & 0xff)
            return h

        self.lg = lg = int(golden.l_pac)
        lr = int(grch.l_pac)
        self.off_grch = (lg + 3) & ~3
        self.off_b = (self.off_grch + lr + 3) & ~3
        self.l_pac = self.off_b + lg
        ga, gl = np.asarray(golden.ann_offset, np.int64), np.asarray(golden.ann_len, np.int64)
        self.ann_offset = np.concatenate([ga, np.asarray(grch.ann_offset, np.int64) + self.off_grch, ga + self.off_b])
        ann_len = np.concatenate([gl, np.asarray(grch.ann_len, np.int64), gl])
        ann_len[len(gl) - 1] += self.off_grch - lg
        ann_len[len(gl) + len(grch.ann_len) - 1] += self.off_b - self.off_grch - lr
        self.ann_len = ann_len.astype(np.int32)
        self.rid_b = len(gl) + len(grch.ann_len)
        self.pac = np.concatenate([body(golden.pac, lg), body(grch.pac, lr), body(golden.pac, lg)])

    def translate(self, b: Batch) -> Batch:
        """a batch on the golden genome -> the same batch here (even reads on
        copy A, odd reads on copy B)"""
        nch = np.diff(b.read_chain_off)
        chain_b = np.repeat((np.arange(b.n_reads) & 1).astype(bool), nch)
        seed_b = np.repeat(chain_b, np.diff(b.chain_seed_off))
        seeds = b.seeds.copy()
        x = seeds["rbeg"].astype(np.int64)
        seeds["rbeg"] = np.where(seed_b, x + self.off_b, np.where(x < self.lg, x, x + 2 * (self.l_pac - self.lg)))
        rid = np.where(chain_b, b.chain_rid + self.rid_b, b.chain_rid).astype(np.int32)
        return Batch(b.seq_off, b.seq, b.read_chain_off, b.chain_seed_off, rid, b.chain_frac_rep, seeds)


class C3RefSet:
    """C2 batch 0's reference-seeded chains, translated into the GRCh38-shaped
    genome past 2^31 (GoldenInGrch38), with the reference's answers there"""

    def __init__(self, z, batch: Batch):
        self.name = "c3_refseed"
        self.batch = batch
        if batch_digest(batch) != z["batch_sha256"].tobytes():
            raise RuntimeError("translated c3_refseed batch differs from the fixture's")
        self.reg_n = z["reg_n"].astype(np.int32)
        self.regs_sha256 = z["regs_sha256"].tobytes()
        self.regs_chunks = z["regs_chunks"]
        self.cigar_chunks = z["cigar_chunks"]
        self.coverage = dict(zip(C3_COVERAGE_KEYS, z["coverage"].tolist()))

    check = C3Set.check
    check_cigar = C3Set.check_cigar


def load_c3_refseed(path: str = C3R_FIXTURE, grch=None, golden=None):
    """-> (opt dict, GoldenInGrch38, C3RefSet); raises if the regenerated
    genome or the translated batch differs from the one the reference ran on"""
    z = np.load(path, allow_pickle=False)
    opt = dict(zip(OPT_KEYS, z["opt_int"].tolist()))
    opt["mat"] = z["opt_mat"].astype(np.int8)
    g = GoldenInGrch38(grch, golden)
    if hashlib.sha256(g.pac).digest() != z["pac_sha256"].tobytes():
        raise RuntimeError("regenerated golden-in-GRCh38 genome differs from the fixture's")
    _, _, bs = load_fixture(with_ref=False)
    return opt, g, C3RefSet(z, g.translate(bs[int(z["c2_batch"])].batch))


def load_fixture(path: str = C2_FIXTURE, with_ref: bool = True):
    """-> (opt dict, GoldenRef or None, [RefBatch]); raises if the regenerated
    genome differs from the one the reference indexed"""
    z = np.load(path, allow_pickle=False)
    opt = dict(zip(OPT_KEYS, z["opt_int"].tolist()))
    opt["mat"] = z["opt_mat"].astype(np.int8)
    ref = None
    if with_ref:
        ref = GoldenRef(int(z["genome_len"]), int(z["genome_seed"]))
        if hashlib.sha256(ref.pac.tobytes()).digest() != z["pac_sha256"].tobytes():
            raise RuntimeError("regenerated genome differs from the reference's pac (tools/synth.cpp golden_genome)")
        if not (np.array_equal(ref.ann_offset, z["ann_offset"]) and np.array_equal(ref.ann_len, z["ann_len"])):
            raise RuntimeError("regenerated contig table differs from the reference's")
    out = []
    for k in range(int(z["n_batches"])):
        p = f"b{k}_"
        lens = z[p + "lens"].astype(np.int64)
        seq_off = np.concatenate([[0], np.cumsum(lens)])
        seq = _unpack_seq(z[p + "seq2"], z[p + "npos"], int(seq_off[-1]))
        rco = np.concatenate([[0], np.cumsum(z[p + "read_nchain"].astype(np.int64))])
        cso = np.concatenate([[0], np.cumsum(z[p + "chain_nseed"].astype(np.int64))])
        seeds = np.zeros(int(cso[-1]), abi.SEED_DTYPE)
        seeds["rbeg"] = np.cumsum(z[p + "rbeg_delta"].astype(np.int64))
        seeds["qbeg"] = z[p + "qbeg"]
        seeds["len"] = z[p + "slen"]
        seeds["score"] = z[p + "score"]
        b = Batch(seq_off, seq, rco, cso, z[p + "chain_rid"].astype(np.int32), z[p + "chain_frac_rep"], seeds)
        out.append(RefBatch(b, z[p + "reg_n"].astype(np.int32), z[p + "regs_sha256"].tobytes()))
    return opt, ref, out
