"""CPU: pin the oracle (our C restatement) to the reference's golden vectors.

The fixtures were produced by the reference's own C compiled from
/root/reference/bwa (oracle/gen_golden.py): chains from its seeding, regions
from its mem_chain2aln (bwa/bwamem.c:641-795), ksw_extend2 (bwa/ksw.c:380-479)
outputs for recorded and randomised edge-case calls, ksw_align2
(bwa/ksw.c:337-357) outputs for mate-rescue-shaped and edge-case calls."""
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


@pytest.mark.parametrize("name", G.CHAIN_SETS + G.KSW_SETS)
def test_row_bound_changes_no_output(name):
    """the GPU kernels' row bound restated on the CPU:
    ending a call once no later cell can reach gscore leaves all six outputs
    of every recorded ksw_extend2 call as the reference's, with fewer rows"""
    opt, tasks, want, qp, tp = G.load_tasks(name)
    full, cells = oracle.extend("oracle", opt, tasks, qp, tp)
    got, bcells = oracle.extend("oracle_bounded", opt, tasks, qp, tp)
    bad = np.nonzero((got.view(np.int32).reshape(-1, 6) != want.view(np.int32).reshape(-1, 6)).any(axis=1))[0]
    assert len(bad) == 0, f"{len(bad)} tasks differ, first {tasks[bad[0]]}: {got[bad[0]]} vs {want[bad[0]]}"
    assert bcells[0] <= cells[0] and bcells[1] <= cells[1]


@pytest.mark.parametrize("name", G.ALIGN2_SETS)
def test_oracle_ksw_align2_matches_reference(name):
    opt, tasks, want, qp, tp = G.load_align2(name)
    got, cells = oracle.align2("oracle", opt, tasks, qp, tp)
    assert G.kswr_mismatch(tasks, got, want) is None
    assert cells[0] > 0


def test_align2_fixture_coverage():
    """the ksw_align2 sets reach u8 and i16, the 255 saturation, XSTOP, the
    2nd-best score, the start pass, scores below minsc and o_ins == 0"""
    seen = dict(u8=0, i16=0, sat255=0, xstop=0, score2=0, start=0, below_minsc=0, o_ins0=0, qlen_gt_256=0,
                tlen_le_qlen=0)
    for name in G.ALIGN2_SETS:
        opt, t, r, _, _ = G.load_align2(name)
        u8 = (t["xtra"] & abi.KSW_XBYTE) != 0
        seen["u8"] += int(u8.sum())
        seen["i16"] += int((~u8).sum())
        seen["sat255"] += int((u8 & (r["score"] == 255)).sum())
        seen["xstop"] += int(((t["xtra"] & abi.KSW_XSTOP) != 0).sum())
        seen["score2"] += int((r["score2"] >= 0).sum())
        seen["start"] += int((r["tb"] >= 0).sum())
        sub = (t["xtra"] & abi.KSW_XSUBO) != 0
        seen["below_minsc"] += int((sub & (r["score"] < (t["xtra"] & 0xffff))).sum())
        seen["o_ins0"] += len(t) if opt["o_ins"] == 0 else 0
        seen["qlen_gt_256"] += int((t["qlen"] > 256).sum())
        seen["tlen_le_qlen"] += int((t["tlen"] <= t["qlen"]).sum())
    for k, v in seen.items():
        assert v > 0, f"ksw_align2 golden vectors never exercise {k}"


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


def test_oracle_align2_vs_reference_fresh_random_tasks():
    """fresh random ksw_align2 calls, oracle vs the compiled reference"""
    if oracle.ref_lib() is None:
        pytest.skip("oracle/_ref not built")
    import gen_golden
    from bwagpu import synth
    rng = np.random.default_rng(123)
    for o in gen_golden.ALIGN2_OPTS.values():
        opt = abi.default_opt() if o is None else dict(o, mat=abi.fill_scmat(o["a"], o["b"]))
        tasks, qp, tp = synth.mate_rescue_tasks(rng, 150, a=opt["a"], qlens=gen_golden.A2_SHORT, win=(0, 300),
                                                xtra_mode="mix")
        a, _ = oracle.align2("oracle", opt, tasks, qp, tp)
        b, _ = oracle.align2("ref", opt, tasks, qp, tp)
        assert G.kswr_mismatch(tasks, a, b) is None
