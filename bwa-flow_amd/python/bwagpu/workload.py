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


def _unpack_seq(seq2: np.ndarray, npos: np.ndarray, n: int) -> np.ndarray:
    s = np.empty(4 * len(seq2), np.uint8)
    for k in range(4):
        s[k::4] = (seq2 >> (6 - 2 * k)) & 3
    s = s[:n]
    s[npos] = 4
    return s


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
