"""CPU: pin the oracle (our C restatement) to the reference's golden vectors.

The fixtures were produced by the reference's own C compiled from
/root/reference/bwa (oracle/gen_golden.py): chains from its seeding, regions
from its mem_chain2aln (bwa/bwamem.c:641-795), ksw_extend2 (bwa/ksw.c:380-479)
outputs for recorded and randomised edge-case calls."""
import numpy as np
import pytest

import golden_io as G
import oracle
from bwagpu import abi
from bwagpu.engine import compact


@pytest.fixture(scope="module")
def ref():
    r = G.load_ref()
    return oracle.Ref(r["l_pac"], r["ann_offset"], r["ann_len"], r["pac"])


@pytest.mark.parametrize("name", G.CHAIN_SETS)
@pytest.mark.parametrize("threads", [1, 3])
def test_oracle_regions_match_reference(ref, name, threads):
    opt, batch, want, want_n = G.load_chain_set(name)
    regs, n, st = oracle.chain2aln("oracle", opt, ref, batch, n_threads=threads)
    assert np.array_equal(n, want_n)
    assert G.region_mismatch(compact(batch, regs, n), want) is None
    assert st[0] > 0 and st[1] > 0 and st[2] > 0


@pytest.mark.parametrize("name", G.CHAIN_SETS + G.KSW_SETS)
def test_oracle_ksw_extend2_matches_reference(name):
    opt, tasks, want, qp, tp = G.load_tasks(name)
    got, cells = oracle.extend("oracle", opt, tasks, qp, tp)
    bad = np.nonzero(got.view(np.int32).reshape(-1, 6) != want.view(np.int32).reshape(-1, 6))[0]
    assert len(bad) == 0, f"{len(set(bad))} tasks differ, first {tasks[bad[0]]}: {got[bad[0]]} vs {want[bad[0]]}"


def test_fixture_coverage():
    """the golden sets exercise the corners the reference code has"""
    seen = dict(multi_region=0, retry=0, to_end=0, tlen0=0, n_query=0, zero_chain_reads=0, long_reads=0)
    for name in G.CHAIN_SETS:
        opt, batch, regs, n = G.load_chain_set(name)
        seen["multi_region"] += int((n > 1).sum())
        seen["retry"] += int((regs["w"] > opt["w"]).sum())
        seen["zero_chain_reads"] += int((np.diff(batch.read_chain_off) == 0).sum())
        seen["n_query"] += int((batch.seq == 4).sum())
        seen["long_reads"] += int((np.diff(batch.seq_off) > 160).sum())
        seen["to_end"] += int(((regs["qb"] == 0) & (regs["truesc"] != regs["score"])).sum())
    for name in G.KSW_SETS:
        _, tasks, res, _, _ = G.load_tasks(name)
        seen["tlen0"] += int((tasks["tlen"] == 0).sum())
    for k, v in seen.items():
        assert v > 0, f"golden vectors never exercise {k}"


def test_reference_layout():
    lib = oracle.ref_lib()
    if lib is None:
        pytest.skip("oracle/_ref not built")
    assert lib.ref_abi_check() == 88 * 1000 + 24  # sizeof(mem_alnreg_t), sizeof(mem_seed_t)


def test_oracle_vs_reference_fresh_random_tasks():
    """beyond the committed vectors: fresh random calls, oracle vs the compiled reference"""
    if oracle.ref_lib() is None:
        pytest.skip("oracle/_ref not built")
    import gen_golden
    rng = np.random.default_rng(99)
    for opt in (abi.default_opt(),
                dict(a=2, b=3, o_del=3, e_del=3, o_ins=2, e_ins=1, pen_clip5=7, pen_clip3=1, w=15, zdrop=10,
                     mat=abi.fill_scmat(2, 3))):
        tasks, qp, tp = gen_golden.edge_tasks(rng, 600, allow_t5=True)
        a, _ = oracle.extend("oracle", opt, tasks, qp, tp)
        b, _ = oracle.extend("ref", opt, tasks, qp, tp)
        assert np.array_equal(a.view(np.int32), b.view(np.int32))
