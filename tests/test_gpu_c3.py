"""GPU parity in the GRCh38 regime (BASELINE.json configs[2] / [4]).

The GRCh38-shaped genome of tests/golden/c3_grch38.npz (195 contigs, l_pac
3,099,734,149, a 0.78 GB resident pac) with one C3 batch (2x150 bp) and one C5
batch (thirds of 2x100 / 2x150 / 2x250), each a 10 Mbase ChainsRecord whose
seeds sit past 2^31 (forward) and 2^32 (2-strand), in all 195 contigs and
across contig junctions.  The GPU's mem_chain2aln output must match the
reference's (oracle/_ref mem_chain2aln, recorded as digests) byte for byte, on
both kernel paths; the CIGAR kernel (bns_pos2rid over 195 contigs) must match
the reference's mem_reg2aln on every region.  And the C2 fixture's
reference-seeded chains (bwa's own seeding) translated into that regime
(tests/golden/c3_refseed.npz: two copies of the golden genome around the
GRCh38-shaped contigs, seeds past forward 2^31 and 2-strand 2^32).
"""
import numpy as np
import pytest

from bwagpu import workload
from conftest import set_c2a_path
from bwagpu.engine import Engine

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def c3():
    return workload.load_c3()


@pytest.fixture(scope="module")
def eng(c3):
    opt, ref, _ = c3
    e = Engine(0, opt, ref.l_pac, ref.ann_offset, ref.ann_len, pac=ref.pac)
    yield e
    e.close()


@pytest.mark.parametrize("path", ["spec", "quad", "pair", "fast"])
@pytest.mark.parametrize("name", ["c3", "c5"])
def test_chain2aln_grch38(c3, eng, name, path, monkeypatch):
    restore = set_c2a_path(path, monkeypatch)
    s = c3[2][name]
    regs, n = eng.chain2aln(s.batch)
    restore()
    why = s.check(regs, n)
    assert why is None, why
    assert eng.last_stats()["ext_calls"] > 0


@pytest.mark.parametrize("name", ["c3", "c5"])
def test_reg2aln_grch38(c3, eng, name):
    s = c3[2][name]
    regs, n = eng.chain2aln(s.batch)
    jobs = workload.reg2aln_jobs(s.batch, regs, n)
    assert len(jobs) == int(np.sum(s.reg_n))
    aln, cig, md = eng.reg2aln_batch(jobs, s.batch.seq, workload.C3_MAX_OPS, workload.C3_MAX_MD)
    why = s.check_cigar(jobs, aln, cig, md)
    assert why is None, why
    assert len(np.unique(aln["rid"])) == 195


@pytest.mark.parametrize("path", ["spec", "quad", "pair", "fast"])
def test_chain2aln_refseed_in_grch38(c3, path, monkeypatch):
    opt, g, s = workload.load_c3_refseed(grch=c3[1])
    e = Engine(0, opt, g.l_pac, g.ann_offset, g.ann_len, pac=g.pac)
    restore = set_c2a_path(path, monkeypatch)
    regs, n = e.chain2aln(s.batch)
    restore()
    why = s.check(regs, n)
    e.close()
    assert why is None, why


def test_reg2aln_refseed_in_grch38(c3):
    opt, g, s = workload.load_c3_refseed(grch=c3[1])
    e = Engine(0, opt, g.l_pac, g.ann_offset, g.ann_len, pac=g.pac)
    regs, n = e.chain2aln(s.batch)
    jobs = workload.reg2aln_jobs(s.batch, regs, n)
    aln, cig, md = e.reg2aln_batch(jobs, s.batch.seq, workload.C3_MAX_OPS, workload.C3_MAX_MD)
    e.close()
    assert len(jobs) == int(np.sum(s.reg_n))
    why = s.check_cigar(jobs, aln, cig, md)
    assert why is None, why
    assert set(np.unique(aln["rid"]).tolist()) <= {0, 1, 2, 198, 199, 200}
