"""The CPU restatement of seeding's chaining (oracle/chain.c: mem_chain's body
with its kbtree, test_and_merge, mem_chain_flt, mem_flt_chained_seeds /
mem_seed_sw) against the reference's own output (tests/golden/chain_*.npz,
oracle/gen_chain.c), field by field and in order — the checker the device
chaining (tests/test_gpu_chain.py) relies on.

The sets cover: default options at 150 bp; 12-250 bp reads with an ALT
contig; 750-1000 bp reads, where mem_flt_chained_seeds runs ksw_align2 on
every seed; non-default w / max_occ / max_chain_gap / min_chain_weight /
max_chain_extend / mask_level / drop_ratio / scoring; repeat-rich reads (>= 6
raw chains each: kbtree splits, chains with EQUAL positions, whose order and
kb_intervalp choice follow the tree's shape)."""
import numpy as np
import pytest

import golden_io as G
import oracle


@pytest.fixture(scope="module")
def env():
    refd = G.load_ref()
    hdr, words = G.load_seed_bwt()
    sa_intv, sa, _, _ = G.load_seed_sa()
    ref = oracle.Ref(refd["l_pac"], refd["ann_offset"], refd["ann_len"], refd["pac"])
    return ref, hdr, words, sa, sa_intv


def run(env, g, raw):
    ref, hdr, words, sa, sa_intv = env
    return oracle.seqs2chains(g["opt"], g["copt"], g["seedopt"], g["split_factor"], ref, g["is_alt"], hdr, words,
                              sa, sa_intv, g["seq_off"], g["seq"], raw=raw)


def raw_mismatch(got, want):
    rco, ch, cso, sd = got
    wrco, wch, wsd = want
    if not np.array_equal(rco, wrco):
        r = int(np.argmax(rco != wrco))
        return f"chain counts differ from read {r - 1}"
    g = np.column_stack([ch["pos"], ch["rid"], ch["n"], ch["is_alt"]]).astype(np.int64)
    if not np.array_equal(g, wch):
        return f"chain {int(np.argmax(np.any(g != wch, axis=1)))} differs"
    s = np.column_stack([sd["rbeg"], sd["qbeg"], sd["len"]]).astype(np.int64)
    if not np.array_equal(s, wsd):
        return f"seed {int(np.argmax(np.any(s != wsd, axis=1)))} differs"
    return None


def final_mismatch(got, want):
    rco, ch, cso, sd = got
    wrco, wch, wfr, wsd = want
    if not np.array_equal(rco, wrco):
        r = int(np.argmax(rco != wrco))
        return f"chain counts differ from read {r - 1}"
    g = np.column_stack([ch["pos"], ch["rid"], ch["n"], ch["w"], ch["kept"], ch["first"],
                         ch["is_alt"]]).astype(np.int64)
    if not np.array_equal(g, wch):
        k = int(np.argmax(np.any(g != wch, axis=1)))
        return f"chain {k} differs: {g[k].tolist()} vs {wch[k].tolist()}"
    if not np.array_equal(ch["frac_rep"].view(np.uint32), wfr.view(np.uint32)):
        return "frac_rep differs"
    s = np.column_stack([sd["rbeg"], sd["qbeg"], sd["len"], sd["score"]]).astype(np.int64)
    if not np.array_equal(s, wsd):
        k = int(np.argmax(np.any(s != wsd, axis=1)))
        return f"seed {k} differs: {s[k].tolist()} vs {wsd[k].tolist()}"
    return None


@pytest.mark.parametrize("name", G.CHAIN_GOLD_SETS)
def test_raw_chains_match_reference(env, name):
    g = G.load_chain_gold(name)
    assert raw_mismatch(run(env, g, True), g["raw"]) is None


@pytest.mark.parametrize("name", G.CHAIN_GOLD_SETS)
def test_filtered_chains_match_reference(env, name):
    g = G.load_chain_gold(name)
    assert final_mismatch(run(env, g, False), g["final"]) is None


def test_sets_reach_the_hard_cases():
    z = {n: np.load(f"{G.GOLD}/chain_{n}.npz") for n in G.CHAIN_GOLD_SETS}
    assert z["rep"]["stats"][0] >= 100      # reads with equal raw chain positions
    assert z["rep"]["raw_n"].max() > 9      # kbtree root splits (9 keys per node)
    assert z["long"]["stats"][1] >= 500     # mem_flt_chained_seeds ran
    assert z["longopt"]["stats"][1] == 300
    assert (z["opt"]["chn"][:, 4] == 1).any() and (z["opt"]["chn"][:, 4] == 2).any()
    assert (z["mix"]["chn"][:, 6] == 1).any()  # ALT chains
