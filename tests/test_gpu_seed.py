"""GPU parity of seeding's interval collection:
bwagpu_collect_intv returns, per read, the intervals mem_collect_intv
(bwa/bwamem.c:120-167) leaves — same SA intervals, same info, same order
(klib introsort's order for equal info) — on the golden sets produced by the
reference's own bwt_smem1 / bwt_seed_strategy1 / ks_introsort_mem_intv
(oracle/gen_seed.c), and on fresh reads against the oracle (oracle/seed.c).

Edge cases: empty reads, all-N reads, reads shorter than min_seed_len,
non-default seeding options (the re-seeding and LAST-like passes switched by
split_factor / split_width / max_mem_intv), a read with more intervals than
max_per_read (E_UNSUPPORTED, flagged count), missing index."""
import numpy as np
import pytest

import golden_io as G
import oracle
from bwagpu import abi
from bwagpu.engine import BwaGpuError, Engine

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def eng():
    refd = G.load_ref()
    opt, *_ = G.load_chain_set("c1_default")
    e = Engine(0, opt, refd["l_pac"], refd["ann_offset"], refd["ann_len"], pac=refd["pac"])
    hdr, words = G.load_seed_bwt()
    intv, sa, _, _ = G.load_seed_sa()
    e.set_bwt(hdr, words, sa, intv)
    return e


def as_u64(iv):
    return np.column_stack([iv["x"], iv["info"]]).astype(np.uint64) if len(iv) else np.zeros((0, 4), np.uint64)


@pytest.mark.parametrize("budget", [1024, 0, 200])
@pytest.mark.parametrize("name", G.SEED_SETS)
def test_collect_intv_golden(eng, name, budget):
    """budget 0: every read on the wave kernel; 200: a mix of both tiers"""
    opt, sf, seq_off, seq, want_n, want = G.load_seed_set(name)
    eng.seed_budget(budget)
    try:
        n, iv = eng.collect_intv(seq_off, seq, int(opt[0]), int(opt[1]), int(opt[2]), sf)
    finally:
        eng.seed_budget(1024)
    assert np.array_equal(n, want_n)
    assert np.array_equal(as_u64(iv), want)


def _fresh_reads(rng, n, genome_len=1_000_000):
    """reads cut from random BWT-independent sequence and from the golden genome's pac"""
    refd = G.load_ref()
    pac = refd["pac"]
    lens = rng.choice([12, 19, 20, 33, 76, 101, 150, 151, 250, 300], n)
    out, off = [], [0]
    for L in lens:
        p = int(rng.integers(0, genome_len - L))
        idx = np.arange(p, p + L)
        q = (pac[idx >> 2] >> ((~idx & 3) << 1)) & 3
        if rng.random() < 0.5:
            q = 3 - q[::-1]
        q = q.astype(np.uint8)
        mut = rng.random(L) < 0.02
        q[mut] = rng.integers(0, 4, int(mut.sum()))
        q[rng.random(L) < 0.01] = 4
        out.append(q)
        off.append(off[-1] + L)
    return np.array(off, np.int64), np.concatenate(out)


@pytest.mark.parametrize("opts", [(19, 10, 20, 1.5), (15, 20, 0, 1.0), (25, 5, 50, 2.0)])
def test_collect_intv_fresh_vs_oracle(eng, opts):
    rng = np.random.default_rng(sum(opts[:3]))
    seq_off, seq = _fresh_reads(rng, 800)
    msl, sw, mmi, sf = opts
    hdr, words = G.load_seed_bwt()
    want_n, want = oracle.collect_intv(hdr, words, np.array([msl, sw, mmi], np.int32), sf, seq_off, seq)
    n, iv = eng.collect_intv(seq_off, seq, msl, sw, mmi, sf)
    assert np.array_equal(n, want_n)
    assert np.array_equal(as_u64(iv), want)


def test_collect_intv_edge_reads(eng):
    reads = [np.zeros(0, np.uint8), np.full(40, 4, np.uint8), np.array([0, 1, 2], np.uint8),
             np.array([2] * 200, np.uint8), np.array([0, 1, 2, 3] * 60, np.uint8)]
    seq_off = np.concatenate([[0], np.cumsum([len(r) for r in reads])]).astype(np.int64)
    seq = np.concatenate(reads)
    hdr, words = G.load_seed_bwt()
    want_n, want = oracle.collect_intv(hdr, words, np.array([19, 10, 20], np.int32), 1.5, seq_off, seq)
    for budget in (1024, 0):
        eng.seed_budget(budget)
        n, iv = eng.collect_intv(seq_off, seq, max_per_read=8192)  # the homopolymer has thousands
        assert n[0] == 0 and n[1] == 0 and n[2] == 0 and n[3] > 1000
        assert np.array_equal(n, want_n) and np.array_equal(as_u64(iv), want)
    eng.seed_budget(1024)


def test_collect_intv_overflow_and_missing_index(eng):
    opt, sf, seq_off, seq, want_n, want = G.load_seed_set("c1")
    r = int(np.argmax(want_n))
    sub_off = np.array([0, seq_off[r + 1] - seq_off[r]], np.int64)
    sub = seq[seq_off[r]:seq_off[r + 1]]
    with pytest.raises(BwaGpuError) as ei:
        eng.collect_intv(sub_off, sub, max_per_read=int(want_n[r]) - 1)
    assert ei.value.code == 6  # BWAGPU_E_UNSUPPORTED
    bad = sub.copy()
    bad[len(bad) // 2] = 5  # not an nt4 base
    with pytest.raises(BwaGpuError) as ei:
        eng.collect_intv(sub_off, bad)
    assert ei.value.code == 1  # BWAGPU_E_INVAL
    refd = G.load_ref()
    e2 = Engine(0, {k: v for k, v in G.load_chain_set("c1_default")[0].items()}, refd["l_pac"],
                refd["ann_offset"], refd["ann_len"], pac=refd["pac"])
    with pytest.raises(BwaGpuError):
        e2.collect_intv(sub_off, sub)


def test_bwt_sa_golden(eng):
    """bwt_sa on the device equals the reference's at 20 010 BWT positions
    (random, sample boundaries, primary and neighbours, seq_len)"""
    intv, sa, q, want = G.load_seed_sa()
    assert np.array_equal(eng.bwt_sa(q), want)
    hdr, words = G.load_seed_bwt()
    with pytest.raises(BwaGpuError):
        eng.bwt_sa(np.array([hdr[6] + 1], np.uint64))  # past seq_len


def test_bwt_sa_of_collected_intervals(eng):
    """the seeds mem_chain would take from the golden intervals
    (bwamem.c:282-288: up to max_occ positions per interval, stepped): the
    device's rbeg values equal the oracle's"""
    opt, sf, seq_off, seq, want_n, want = G.load_seed_set("c1")
    ks = []
    for x0, _, x2, _ in want[:4000]:
        step = x2 // 500 if x2 > 500 else 1
        ks.extend(int(x0) + k for k in range(0, int(min(x2, 500 * step)), int(step)))
    ks = np.array(ks[:20000], np.uint64)
    hdr, words = G.load_seed_bwt()
    intv, sa, _, _ = G.load_seed_sa()
    assert np.array_equal(eng.bwt_sa(ks), oracle.bwt_sa(hdr, words, sa, intv, ks))


def test_expanded_suffix_array_equals_the_walk(monkeypatch):
    """bwagpu_set_bwt expands the sampled suffix array into every row's entry
    (one load per bwt_sa); BWAGPU_SA_FULL=0 keeps bwt.c's walk to a sampled
    row.  Both give the reference's values at the golden positions, and the
    two agree at EVERY row 0..seq_len of the golden index"""
    refd = G.load_ref()
    opt, *_ = G.load_chain_set("c1_default")
    hdr, words = G.load_seed_bwt()
    intv, sa, q, want = G.load_seed_sa()
    engs = {}
    for mode in ("1", "64", "0"):  # 32-bit entries, 64-bit entries, the walk
        monkeypatch.setenv("BWAGPU_SA_FULL", mode)
        e = Engine(0, opt, refd["l_pac"], refd["ann_offset"], refd["ann_len"], pac=refd["pac"])
        e.set_bwt(hdr, words, sa, intv)
        assert np.array_equal(e.bwt_sa(q), want)
        engs[mode] = e
    rows = np.arange(int(hdr[6]) + 1, dtype=np.uint64)
    full, walk = engs["1"].bwt_sa(rows), engs["0"].bwt_sa(rows)
    assert np.array_equal(full, walk)
    assert np.array_equal(engs["64"].bwt_sa(rows), walk)
    # a permutation of 0..seq_len-1 plus row 0's stored -1 (bwt_cal_sa, bwt.c:181)
    want_set = np.append(np.arange(len(rows) - 1, dtype=np.uint64), np.uint64(2**64 - 1))
    assert np.array_equal(np.sort(full), want_set)
    for e in engs.values():
        e.close()
