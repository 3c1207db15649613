"""The FPGA wire format on the CPU: the oracle's
restatement of packReadData (src/fpga/FPGAPipeline.cpp:194-343) and of what
sw_top must return for it.

Pinning: processOutput (FPGAPipeline.cpp:90-105) rebuilds a region from each
record; every region of the reference's own mem_chain2aln in the golden chain
sets (oracle/gen_golden.py, bwa's C) must be one of the regions rebuilt for
its read — each such region is one seed's extension in its chain's window,
and getChainRef's window is mem_chain2aln's.
"""
import numpy as np
import pytest

import golden_io as G
import oracle
from bwagpu import abi
from bwagpu.engine import Batch


@pytest.fixture(scope="module")
def ref():
    r = G.load_ref()
    return oracle.Ref(r["l_pac"], r["ann_offset"], r["ann_len"], r["pac"])


def sub_batch(b: Batch, r0: int, r1: int) -> Batch:
    c0, c1 = int(b.read_chain_off[r0]), int(b.read_chain_off[r1])
    s0, s1 = int(b.chain_seed_off[c0]), int(b.chain_seed_off[c1])
    q0, q1 = int(b.seq_off[r0]), int(b.seq_off[r1])
    return Batch(b.seq_off[r0:r1 + 1] - q0, b.seq[q0:q1], b.read_chain_off[r0:r1 + 1] - c0,
                 b.chain_seed_off[c0:c1 + 1] - s0, b.chain_rid[c0:c1], b.chain_frac_rep[c0:c1], b.seeds[s0:s1])


def apply_records(batch: Batch, rec: np.ndarray, task_seed: np.ndarray) -> np.ndarray:
    """processOutput's arithmetic (FPGAPipeline.cpp:91-105) from the packer's
    initial region (FPGAPipeline.cpp:231-242) -> per task (rb, re, qb, qe,
    score, truesc, w)"""
    s = batch.seeds[task_seed]
    t = rec.astype(np.int64)
    idx = (t[:, 1] << 16) | (t[:, 0] & 0xffff)
    assert np.array_equal(idx, np.arange(len(rec)))
    rb = s["rbeg"] + t[:, 4]
    re = s["rbeg"] + s["len"] + t[:, 5]
    qb = t[:, 2]
    qe = s["qbeg"] + s["len"] + t[:, 3]
    return np.stack([rb, re, qb, qe, t[:, 6], t[:, 7], t[:, 8]], axis=1)


def seed_read(batch: Batch) -> np.ndarray:
    chain_of_seed = np.repeat(np.arange(batch.n_chains), np.diff(batch.chain_seed_off))
    read_of_chain = np.repeat(np.arange(batch.n_reads), np.diff(batch.read_chain_off))
    return read_of_chain[chain_of_seed]


def test_pack_layout_by_hand(ref):
    """one read, one chain of three seeds (one of them the whole read): the
    word layout of packReadData"""
    lq = 10
    seq = np.array([0, 1, 2, 3, 4, 3, 2, 1, 0, 1], np.uint8)
    seeds = np.zeros(3, abi.SEED_DTYPE)
    seeds[0] = (1000, 0, 10, 10, 0)   # qbeg 0, len = lq: no task
    seeds[1] = (1002, 2, 5, 5, 0)
    seeds[2] = (1001, 1, 3, 3, 0)
    b = Batch([0, lq], seq, [0, 1], [0, 3], [0], [0.0], seeds)
    opt, _, _, _ = G.load_chain_set("c1_default")
    words, nt, packed, task_seed = oracle.fpga_pack(opt, ref, b)
    assert nt == 2 and packed.tolist() == [1] and task_seed.tolist() == [2, 1]  # seeds n-1 .. 0
    w = words.view(np.uint32)
    assert words[0] == len(words) and words[1] == lq
    assert w[2] == 0x01234321 and w[3] == 0x01000000  # first base in the high nibble, zero padded
    assert words[4] == 1  # chains
    lo = int(w[5]) | int(w[6]) << 32
    hi = int(w[7]) | int(w[8]) << 32
    assert lo < 1000 and hi > 1010
    assert words[9] == 2  # tasks of the chain
    assert words[10] == 0 and (int(w[11]) | int(w[12]) << 32) == 1001 and words[13] == 1 and words[14] == 3
    assert words[15] == 1 and (int(w[16]) | int(w[17]) << 32) == 1002 and words[18] == 2 and words[19] == 5
    assert len(words) == 20


@pytest.mark.parametrize("name", G.CHAIN_SETS)
def test_records_rebuild_the_reference_regions(ref, name):
    opt, batch, want, want_n = G.load_chain_set(name)
    words, nt, packed, task_seed = oracle.fpga_pack(opt, ref, batch)
    rec = oracle.fpga_sw(opt, ref, words, nt)
    assert rec is not None and len(rec) == nt
    got = apply_records(batch, rec, task_seed)
    rd_of_task = seed_read(batch)[task_seed]
    by_read = {}
    for r, row in zip(rd_of_task.tolist(), map(tuple, got.tolist())):
        by_read.setdefault(r, set()).add(row)
    roff = np.concatenate([[0], np.cumsum(want_n)])
    lq = np.diff(batch.seq_off)
    checked = missing = 0
    for r in range(batch.n_reads):
        for k in range(roff[r], roff[r + 1]):
            g = want[k]
            if g["qb"] == 0 and g["qe"] == lq[r] and g["re"] - g["rb"] == lq[r] and g["seedlen0"] == lq[r]:
                continue  # a whole-read seed: no task (FPGAPipeline.cpp:298-329)
            assert packed[r]
            key = (int(g["rb"]), int(g["re"]), int(g["qb"]), int(g["qe"]), int(g["score"]), int(g["truesc"]),
                   int(g["w"]))
            checked += 1
            missing += key not in by_read.get(r, ())
    assert checked > 100 and missing == 0, f"{missing}/{checked} reference regions not rebuilt"


def test_malformed_streams(ref):
    opt, batch, _, _ = G.load_chain_set("c1_default")
    b = sub_batch(batch, 0, 50)
    words, nt, packed, _ = oracle.fpga_pack(opt, ref, b)
    assert nt > 10 and oracle.fpga_sw(opt, ref, words, nt) is not None
    assert oracle.fpga_sw(opt, ref, words[:0], 0).shape == (0, 10)
    bad = words.copy()
    bad[0] = len(words) + 5  # end word past the stream
    assert oracle.fpga_sw(opt, ref, bad, nt) is None
    assert oracle.fpga_sw(opt, ref, words, nt - 1) is None  # the last index is out of range
    # a repeated task index: the first task's index rewritten to the second's
    p = task_word(words, 0)
    q = task_word(words, 1)
    bad = words.copy()
    bad[p] = bad[q]
    assert oracle.fpga_sw(opt, ref, bad, nt) is None
    bad = words.copy()
    bad[p + 4] = 10_000  # seed longer than its read
    assert oracle.fpga_sw(opt, ref, bad, nt) is None


def task_word(words: np.ndarray, t: int) -> int:
    """the word holding task t's index (walks the stream)"""
    p = 0
    while p < len(words):
        end, lq = int(words[p]), int(words[p + 1])
        c = p + 2 + (lq + 7) // 8
        nch = int(words[c])
        c += 1
        for _ in range(nch):
            ns = int(words[c + 4])
            c += 5
            for _ in range(ns):
                if int(words[c]) == t:
                    return c
                c += 5
        p = end
    raise KeyError(t)
