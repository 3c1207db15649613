"""GPU parity of seeding's chaining: bwagpu_seqs2chains
runs bwa-flow's SeqsToChains on the device — mem_collect_intv, mem_chain's
body (bwt_sa, bns_intv2rid, the kbtree of chains, test_and_merge),
mem_chain_flt and mem_flt_chained_seeds — and bwagpu_seqs2regions fuses it with
mem_chain2aln.

Pins:
  * tests/golden/chain_*.npz (oracle/gen_chain.c, the reference's own
    mem_chain / mem_chain_flt / mem_flt_chained_seeds): raw chains in kbtree
    order and the filtered chains, every field (pos, rid, n, w, kept, first,
    is_alt, frac_rep bits, seeds with scores) — default and non-default
    options, an ALT contig, 750-1000 bp reads (mem_seed_sw through ksw_align2),
    repeat-rich reads with equal chain positions;
  * the chain sets gen_golden.c recorded with the reference's mem_chain2aln
    (c1_default, c5_mixed, opt1_scoring, opt2_band): reads in, the same chains,
    and through bwagpu_seqs2regions the reference's regions;
  * fresh reads against the oracle (oracle/chain.c); edge reads."""
import numpy as np
import pytest

import golden_io as G
import oracle
from bwagpu import abi
from bwagpu.engine import Engine

pytestmark = pytest.mark.gpu


def make_engine(opt, sup_shift=None):
    refd = G.load_ref()
    e = Engine(0, opt, refd["l_pac"], refd["ann_offset"], refd["ann_len"], pac=refd["pac"])
    if sup_shift is not None:
        e.sup_shift(sup_shift)
    hdr, words = G.load_seed_bwt()
    sa_intv, sa, _, _ = G.load_seed_sa()
    e.set_bwt(hdr, words, sa, sa_intv)
    return e


@pytest.fixture(scope="module")
def engines():
    cache = {}

    def get(opt):
        key = (opt["a"], opt["b"], opt["w"], opt["o_del"], opt["e_del"], opt["o_ins"], opt["e_ins"])
        if key not in cache:
            cache[key] = make_engine(opt)
        return cache[key]
    yield get
    for e in cache.values():
        e.close()


def dev_chains(eng, g, raw):
    eng.set_alt(g["is_alt"] if g["is_alt"].any() else None)
    return eng.seqs2chains(g["seq_off"], g["seq"], g["seedopt"], g["split_factor"], g["copt"], raw=raw)


@pytest.mark.parametrize("name", G.CHAIN_GOLD_SETS)
def test_raw_chains_golden(engines, name):
    from test_chain_oracle import raw_mismatch
    g = G.load_chain_gold(name)
    got = dev_chains(engines(g["opt"]), g, True)
    assert raw_mismatch(got, g["raw"]) is None


@pytest.mark.parametrize("name", G.CHAIN_GOLD_SETS)
def test_filtered_chains_golden(engines, name):
    from test_chain_oracle import final_mismatch
    g = G.load_chain_gold(name)
    got = dev_chains(engines(g["opt"]), g, False)
    assert final_mismatch(got, g["final"]) is None


@pytest.mark.parametrize("shift", [9, 16])
def test_chains_golden_across_superblocks(shift):
    """the occurrence layout's superblock table and its 32-bit relative counts
    (seed.hip block_counts64 / sup_c) only come into play past 2^32 positions,
    i.e. on a human-sized index; with superblocks of 2^shift positions the
    golden index (~2 M positions) crosses hundreds of them, and every interval
    and chain must stay the reference's"""
    from test_chain_oracle import final_mismatch, raw_mismatch
    eng, key = None, None
    try:
        for name in G.CHAIN_GOLD_SETS:
            g = G.load_chain_gold(name)
            o = g["opt"]
            k = (o["a"], o["b"], o["w"], o["o_del"], o["e_del"], o["o_ins"], o["e_ins"])
            if k != key:
                if eng is not None:
                    eng.close()
                eng, key = make_engine(o, shift), k
            assert raw_mismatch(dev_chains(eng, g, True), g["raw"]) is None, name
            assert final_mismatch(dev_chains(eng, g, False), g["final"]) is None, name
    finally:
        if eng is not None:
            eng.close()


@pytest.mark.parametrize("name", G.CHAIN_SETS)
def test_reads_to_chains_and_regions_vs_gen_golden(engines, name):
    """gen_golden's reads: the device chains equal the chains the reference
    handed to mem_chain2aln, and the fused path's regions equal the reference's"""
    opt, batch, want_regs, want_n = G.load_chain_set(name)
    eng = engines(opt)
    eng.set_alt(None)
    copt = abi.default_chainopt()
    rco, ch, cso, sd = eng.seqs2chains(batch.seq_off, batch.seq, (19, 10, 20), 1.5, copt)
    assert np.array_equal(rco, batch.read_chain_off)
    assert np.array_equal(ch["rid"], batch.chain_rid)
    assert np.array_equal(ch["frac_rep"].view(np.uint32), np.asarray(batch.chain_frac_rep, np.float32).view(np.uint32))
    assert np.array_equal(cso, batch.chain_seed_off)
    for f in ("rbeg", "qbeg", "len", "score"):
        assert np.array_equal(sd[f], batch.seeds[f]), f
    n, regs = eng.seqs2regions(batch.seq_off, batch.seq, (19, 10, 20), 1.5, copt)
    assert np.array_equal(n, want_n)
    assert G.region_mismatch(regs, want_regs) is None


def fresh_reads(rng, n):
    """reads cut from the golden genome (both strands, 2% substitutions, some
    N) plus tandem-repeat-like and random junk reads"""
    refd = G.load_ref()
    pac, l_pac = refd["pac"], refd["l_pac"]
    lens = rng.choice([19, 33, 76, 101, 150, 151, 250, 300, 760, 900], n)
    out = []
    for L in lens:
        kind = rng.random()
        if kind < 0.05:
            q = rng.integers(0, 4, L).astype(np.uint8)
        elif kind < 0.15:  # a short unit repeated: many seeds with equal positions
            unit = rng.integers(0, 4, int(rng.integers(2, 12))).astype(np.uint8)
            q = np.resize(unit, L)
        else:
            p = int(rng.integers(0, l_pac - L))
            idx = np.arange(p, p + L)
            q = ((pac[idx >> 2] >> ((~idx & 3) << 1)) & 3).astype(np.uint8)
            if rng.random() < 0.5:
                q = (3 - q[::-1]).astype(np.uint8)
            mut = rng.random(L) < 0.02
            q[mut] = rng.integers(0, 4, int(mut.sum()))
            q[rng.random(L) < 0.005] = 4
        out.append(q)
    off = np.concatenate([[0], np.cumsum([len(q) for q in out])]).astype(np.int64)
    return off, np.concatenate(out)


@pytest.mark.parametrize("case", ["default", "stepped", "alt"])
def test_fresh_reads_vs_oracle(engines, case):
    from test_chain_oracle import final_mismatch, raw_mismatch
    rng = np.random.default_rng({"default": 7, "stepped": 8, "alt": 9}[case])
    seq_off, seq = fresh_reads(rng, 600)
    opt = abi.default_opt()
    copt = abi.default_chainopt()
    alt = None
    if case == "stepped":
        copt.update(max_occ=7, max_chain_gap=150, min_chain_weight=30, max_chain_extend=2, drop_ratio=0.7)
    if case == "alt":
        alt = np.array([0, 1, 1], np.uint8)
    eng = engines(opt)
    eng.set_alt(alt)
    refd = G.load_ref()
    hdr, words = G.load_seed_bwt()
    sa_intv, sa, _, _ = G.load_seed_sa()
    R = oracle.Ref(refd["l_pac"], refd["ann_offset"], refd["ann_len"], refd["pac"])
    so = np.array([19, 10, 20], np.int32)
    for raw in (True, False):
        want = oracle.seqs2chains(opt, copt, so, 1.5, R, alt, hdr, words, sa, sa_intv, seq_off, seq, raw=raw)
        got = eng.seqs2chains(seq_off, seq, so, 1.5, copt, raw=raw)
        if raw:
            w = (want[0], np.column_stack([want[1]["pos"], want[1]["rid"], want[1]["n"], want[1]["is_alt"]]),
                 np.column_stack([want[3]["rbeg"], want[3]["qbeg"], want[3]["len"]]))
            assert raw_mismatch(got, w) is None
        else:
            w = (want[0], np.column_stack([want[1][f] for f in ("pos", "rid", "n", "w", "kept", "first", "is_alt")]),
                 want[1]["frac_rep"], np.column_stack([want[3][f] for f in ("rbeg", "qbeg", "len", "score")]))
            assert final_mismatch(got, w) is None
    eng.set_alt(None)


def test_edge_batches(engines):
    eng = engines(abi.default_opt())
    eng.set_alt(None)
    rco, ch, cso, sd = eng.seqs2chains(np.zeros(1, np.int64), np.zeros(0, np.uint8))
    assert len(rco) == 1 and len(ch) == 0 and len(sd) == 0
    reads = [np.zeros(0, np.uint8), np.full(40, 4, np.uint8), np.array([0, 1, 2], np.uint8),
             np.array([2] * 200, np.uint8), np.array([0, 1, 2, 3] * 60, np.uint8)]
    seq_off = np.concatenate([[0], np.cumsum([len(r) for r in reads])]).astype(np.int64)
    seq = np.concatenate(reads)
    rco, ch, cso, sd = eng.seqs2chains(seq_off, seq)
    assert rco[1] == 0 and rco[2] == 0 and rco[3] == 0  # empty, all-N, shorter than min_seed_len
    refd = G.load_ref()
    hdr, words = G.load_seed_bwt()
    sa_intv, sa, _, _ = G.load_seed_sa()
    R = oracle.Ref(refd["l_pac"], refd["ann_offset"], refd["ann_len"], refd["pac"])
    want = oracle.seqs2chains(abi.default_opt(), abi.default_chainopt(), np.array([19, 10, 20], np.int32), 1.5, R,
                              None, hdr, words, sa, sa_intv, seq_off, seq)
    assert np.array_equal(rco, want[0]) and np.array_equal(ch, want[1]) and np.array_equal(sd, want[3])
    n, regs = eng.seqs2regions(seq_off, seq)
    assert n[0] == 0 and n[1] == 0 and n[2] == 0


def test_two_stage_workers_on_two_contexts():
    """bwa-flow runs SeqsToChains on several worker threads; two contexts on
    one device (Engine.clone, each with its own copy of the index and its
    expanded suffix array) called from two host threads at once give the
    reference's chains and regions on every call"""
    import threading
    name = G.CHAIN_SETS[0]
    opt, batch, want_regs, want_n = G.load_chain_set(name)
    e1 = make_engine(opt)
    e2 = e1.clone()
    hdr, words = G.load_seed_bwt()
    sa_intv, sa, _, _ = G.load_seed_sa()
    e2.set_bwt(hdr, words, sa, sa_intv)
    copt = abi.default_chainopt()
    bad = []

    def work(e, tag):
        for k in range(4):
            rco, ch, cso, sd = e.seqs2chains(batch.seq_off, batch.seq, (19, 10, 20), 1.5, copt)
            if not (np.array_equal(rco, batch.read_chain_off) and np.array_equal(cso, batch.chain_seed_off) and
                    all(np.array_equal(sd[f], batch.seeds[f]) for f in ("rbeg", "qbeg", "len", "score"))):
                bad.append((tag, k, "chains"))
            n, regs = e.seqs2regions(batch.seq_off, batch.seq, (19, 10, 20), 1.5, copt)
            if not np.array_equal(n, want_n) or G.region_mismatch(regs, want_regs) is not None:
                bad.append((tag, k, "regions"))

    th = [threading.Thread(target=work, args=(e, i)) for i, e in enumerate((e1, e2))]
    for t in th:
        t.start()
    for t in th:
        t.join()
    e1.close()
    e2.close()
    assert not bad, bad
