"""GPU parity of the CIGAR step: bwagpu_reg2aln_batch (mem_reg2aln's CIGAR,
NM, MD, strand, contig and position; bwa/bwamem.c:1104-1174) against
* the reference's own mem_reg2aln outputs on every region of the golden
  chain sets (tests/golden/cigar_*.npz), and
* the oracle (oracle/ksw_global.c) on fresh synthetic jobs: both strands,
  indels, N bases, clipped query ranges, band doubling, 100-1000 bp reads,
  matrices past the LDS bins (HBM path), unmapped / rejected jobs and
  output capacity overflow.
Bit-exact: every record field, every CIGAR op and every MD byte."""
import numpy as np
import pytest

import golden_io as G
import oracle
from bwagpu import abi
from bwagpu.engine import BwaGpuError, Engine

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def refd():
    return G.load_ref()


@pytest.fixture(scope="module")
def R(refd):
    return oracle.Ref(refd["l_pac"], refd["ann_offset"], refd["ann_len"], refd["pac"])


def engine(refd, opt):
    return Engine(0, opt, refd["l_pac"], refd["ann_offset"], refd["ann_len"], pac=refd["pac"])


@pytest.mark.parametrize("name", G.CIGAR_SETS)
def test_reg2aln_golden_sets_bit_exact(refd, name):
    opt, tasks, qpool, exp, ops, mds = G.load_cigar_set(name)
    eng = engine(refd, opt)
    out, cig, md = eng.reg2aln_batch(tasks, qpool, 64, 512)
    assert G.aln_mismatch(tasks, out, cig, md, exp, ops, mds) is None
    st = eng.last_stats()
    assert st["cells"] > 0 and st["ext_calls"] == len(tasks)
    eng.close()


@pytest.mark.parametrize("lens,n", [((100, 150, 250), 700), ((400, 700, 1000), 120)])
@pytest.mark.parametrize("optname", ["default", "scoring"])
def test_reg2aln_synthetic_vs_oracle(refd, R, lens, n, optname):
    opt = abi.default_opt() if optname == "default" else dict(
        a=2, b=5, o_del=7, e_del=2, o_ins=5, e_ins=3, pen_clip5=3, pen_clip3=9, w=30, zdrop=40,
        mat=abi.fill_scmat(2, 5))
    rng = np.random.default_rng(41 + len(lens) + n)
    tasks, qpool = G.synth_reg2aln_jobs(rng, refd["pac"], int(refd["l_pac"]), refd["ann_offset"], refd["ann_len"], n,
                                        lens=lens, mat=opt["mat"])
    eng = engine(refd, opt)
    out, cig, md = eng.reg2aln_batch(tasks, qpool, 256, 2048)
    want, wc, wm = oracle.reg2aln("oracle", opt, R, tasks, qpool, 256, 2048)
    assert G.aln_mismatch(tasks, out, cig, md, *G.aln_expected_from(want, wc, wm)) is None
    eng.close()


def test_reg2aln_edge_jobs(refd, R):
    """unmapped (rb < 0), rejected windows (strand-spanning, past the reference
    end, empty query range), the ungapped shortcut (w = 0) and capacity overflow"""
    opt = abi.default_opt()
    rng = np.random.default_rng(9)
    tasks, qpool = G.synth_reg2aln_jobs(rng, refd["pac"], int(refd["l_pac"]), refd["ann_offset"], refd["ann_len"], 40)
    l_pac = int(refd["l_pac"])
    t = tasks.copy()
    t[0]["rb"], t[0]["re"] = -1, -1                      # unmapped record
    t[1]["rb"], t[1]["re"] = l_pac - 50, l_pac + 50      # spans both strands
    t[2]["rb"], t[2]["re"] = 2 * l_pac - 10, 2 * l_pac + 40  # past the end
    t[3]["qe"] = t[3]["qb"]                              # empty query range
    for k in range(4, 10):                               # ungapped: equal lengths, high local score
        t[k]["re"] = t[k]["rb"] + (t[k]["qe"] - t[k]["qb"])
        t[k]["truesc"] = 0
    eng = engine(refd, opt)
    for max_ops, max_md in [(64, 512), (3, 8)]:          # the second overflows most jobs
        out, cig, md = eng.reg2aln_batch(t, qpool, max_ops, max_md)
        want, wc, wm = oracle.reg2aln("oracle", opt, R, t, qpool, max_ops, max_md)
        assert G.aln_mismatch(t, out, cig, md, *G.aln_expected_from(want, wc, wm)) is None
    assert out["status"][0] == abi.ALN_UNMAPPED and (out["status"][1:4] == abi.ALN_NO_CIGAR).all()
    assert (out["status"][4:] == abi.ALN_OVERFLOW).any()
    eng.close()


def test_reg2aln_errors(refd):
    opt = abi.default_opt()
    eng = engine(refd, opt)
    t = np.zeros(1, abi.REG2ALN_TASK_DTYPE)
    t[0] = (100, 250, 0, 150, 0, 150, 140, 100, 0)
    with pytest.raises(BwaGpuError):
        eng.reg2aln_batch(t, np.zeros(10, np.uint8))  # read outside the pool
    out, _, _ = eng.reg2aln_batch(t[:0], np.zeros(1, np.uint8))
    assert len(out) == 0
    eng.close()
