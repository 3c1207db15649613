"""CPU: pin the CIGAR oracle (oracle/ksw_global.c) to the reference.

mem_reg2aln (bwa/bwamem.c:1104-1174: infer_bw, the band-doubling loop,
bwa_gen_cigar2 bwa/bwa.c:121-207, ksw_global2 bwa/ksw.c:504-606, the
deletion squeeze and soft clips) on
* every region of the golden chain sets, with the outputs the reference's
  own mem_reg2aln produced (oracle/gen_golden.c, tests/golden/cigar_*.npz),
* fresh synthetic jobs on both strands (indels, Ns, clipped query ranges,
  local scores above the global score so the band doubles) against the
  reference compiled from /root/reference (oracle/_ref/libbwaref.so)."""
import numpy as np
import pytest

import golden_io as G
import oracle
from bwagpu import abi


@pytest.fixture(scope="module")
def refd():
    return G.load_ref()


@pytest.fixture(scope="module")
def ref(refd):
    return oracle.Ref(refd["l_pac"], refd["ann_offset"], refd["ann_len"], refd["pac"])


@pytest.mark.parametrize("name", G.CIGAR_SETS)
def test_oracle_reg2aln_matches_reference_fixtures(ref, name):
    opt, tasks, qpool, exp, ops, mds = G.load_cigar_set(name)
    out, cig, md = oracle.reg2aln("oracle", opt, ref, tasks, qpool, 64, 512)
    assert G.aln_mismatch(tasks, out, cig, md, exp, ops, mds) is None
    # the sets reach both strands, indels, clipping and mismatches
    assert exp["is_rev"].any() and (~exp["is_rev"].astype(bool)).any()
    allops = np.concatenate(ops)
    assert {0, 1, 2, 3} <= set((allops & 0xf).tolist())


@pytest.mark.parametrize("optname", ["default", "scoring"])
def test_oracle_reg2aln_matches_compiled_reference(refd, ref, optname):
    if oracle.ref_lib() is None or not hasattr(oracle.ref_lib(), "ref_reg2aln_batch"):
        pytest.skip("reference library not built here")
    opt = abi.default_opt() if optname == "default" else dict(
        a=2, b=5, o_del=7, e_del=2, o_ins=5, e_ins=3, pen_clip5=3, pen_clip3=9, w=30, zdrop=40,
        mat=abi.fill_scmat(2, 5))
    rng = np.random.default_rng(31 if optname == "default" else 32)
    tasks, qpool = G.synth_reg2aln_jobs(rng, refd["pac"], int(refd["l_pac"]), refd["ann_offset"], refd["ann_len"],
                                        600, mat=opt["mat"])
    want, wc, wm = oracle.reg2aln("ref", opt, ref, tasks, qpool, 128, 1024)
    got, gc, gm = oracle.reg2aln("oracle", opt, ref, tasks, qpool, 128, 1024)
    exp, ops, mds = G.aln_expected_from(want, wc, wm)
    assert G.aln_mismatch(tasks, got, gc, gm, exp, ops, mds,
                          fields=("pos", "rid", "is_rev", "n_cigar", "NM", "md_len", "status")) is None
    assert (got["status"] == abi.ALN_OK).all()
