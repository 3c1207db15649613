"""The C3 / C5 regime fixture (tests/golden/c3_grch38.npz, made by
oracle/gen_c3_fixture.py): a GRCh38-shaped genome (195 contigs, l_pac
3,099,734,149; coordinates past 2^31 forward and 2^32 on the reverse strand;
a 0.78 GB pac) regenerates bit for bit, the synthetic batches regenerate, they
exercise that regime, and the CPU restatement (and the compiled reference,
when present) reproduce the reference's recorded digests — the checker the GPU
test (tests/test_gpu_c3.py) relies on."""
import os

import numpy as np
import pytest

import oracle
from bwagpu import workload


@pytest.fixture(scope="module")
def c3():
    return workload.load_c3()


def test_genome_shape(c3):
    opt, ref, sets = c3
    assert ref.l_pac == 3_099_734_149 and len(ref.ann_len) == 195
    assert int(ref.ann_offset[-1]) + int(ref.ann_len[-1]) == ref.l_pac
    assert len(ref.pac) == ref.l_pac // 4 + 1 and ref.pac.nbytes > 256 << 20  # larger than the MALL
    assert int(ref.ann_len[0]) == 248_956_422 and int(ref.ann_len.min()) >= 1000


@pytest.mark.parametrize("name", ["c3", "c5"])
def test_batch_covers_the_regime(c3, name):
    _, _, sets = c3
    s = sets[name]
    cov = s.coverage
    assert cov["seeds_fwd_ge_2^31"] > 10_000 and cov["seeds_ge_2^32"] > 10_000
    assert cov["regs_fwd_ge_2^31"] > 5_000 and cov["regs_ge_2^32"] > 5_000
    assert cov["contigs_hit"] == 195 and cov["regs_small_contigs"] > 1_000 and cov["regs_at_contig_edge"] > 500
    b = s.batch
    assert int(b.seq_off[-1]) >= 9_900_000  # one 10 Mbase ChainsRecord
    if name == "c5":
        assert set(np.unique(np.diff(b.seq_off)).tolist()) >= {100, 150, 250} or np.diff(b.seq_off).max() > 200


@pytest.mark.parametrize("which", ["oracle", "ref"])
def test_cpu_paths_match_fixture(c3, which):
    opt, ref, sets = c3
    if which == "ref" and oracle.ref_lib() is None:
        pytest.skip("oracle/_ref not built")
    R = oracle.Ref(ref.l_pac, ref.ann_offset, ref.ann_len, ref.pac)
    for s in sets.values():
        regs, n, _ = oracle.chain2aln(which, opt, R, s.batch, n_threads=min(8, os.cpu_count() or 1))
        assert s.check(regs, n) is None
    # a corrupted region is caught
    s = sets["c3"]
    regs, n, _ = oracle.chain2aln(which, opt, R, s.batch, n_threads=min(8, os.cpu_count() or 1))
    k = int(np.argmax(n > 0))
    regs[s.batch.read_seed_off()[k]]["rb"] += 1
    assert s.check(regs, n) is not None


def test_cigar_oracle_matches_fixture(c3):
    opt, ref, sets = c3
    R = oracle.Ref(ref.l_pac, ref.ann_offset, ref.ann_len, ref.pac)
    s = sets["c3"]
    regs, n, _ = oracle.chain2aln("oracle", opt, R, s.batch, n_threads=min(8, os.cpu_count() or 1))
    jobs = workload.reg2aln_jobs(s.batch, regs, n)
    out = oracle.reg2aln("oracle", opt, R, jobs, s.batch.seq, workload.C3_MAX_OPS, workload.C3_MAX_MD)
    assert s.check_cigar(jobs, *out) is None


@pytest.fixture(scope="module")
def c3r(c3):
    return workload.load_c3_refseed(grch=c3[1])


def test_refseed_in_grch38_covers_the_regime(c3r):
    """C2's reference-seeded chains (bwa's own seeding) translated past forward
    2^31 (copy B) and 2-strand 2^32 (copy A's reverse strand) in a 0.8 GB pac"""
    opt, g, s = c3r
    assert len(g.ann_len) == 201 and g.l_pac > 3_190_000_000 and g.pac.nbytes > 256 << 20
    assert int(g.ann_offset[-1]) + int(g.ann_len[-1]) == g.l_pac
    cov = s.coverage
    assert cov["seeds_fwd_ge_2^31"] > 50_000 and cov["seeds_ge_2^32"] > 50_000
    assert cov["regs_fwd_ge_2^31"] > 20_000 and cov["regs_ge_2^32"] > 20_000


@pytest.mark.parametrize("which", ["oracle", "ref"])
def test_refseed_in_grch38_cpu_paths_match_fixture(c3r, which):
    opt, g, s = c3r
    if which == "ref" and oracle.ref_lib() is None:
        pytest.skip("oracle/_ref not built")
    R = oracle.Ref(g.l_pac, g.ann_offset, g.ann_len, g.pac)
    regs, n, _ = oracle.chain2aln(which, opt, R, s.batch, n_threads=min(8, os.cpu_count() or 1))
    assert s.check(regs, n) is None


def test_refseed_in_grch38_cigars_match_fixture(c3r):
    opt, g, s = c3r
    R = oracle.Ref(g.l_pac, g.ann_offset, g.ann_len, g.pac)
    regs, n, _ = oracle.chain2aln("oracle", opt, R, s.batch, n_threads=min(8, os.cpu_count() or 1))
    jobs = workload.reg2aln_jobs(s.batch, regs, n)
    aln, cig, md = oracle.reg2aln("oracle", opt, R, jobs, s.batch.seq, workload.C3_MAX_OPS, workload.C3_MAX_MD)
    assert s.check_cigar(jobs, aln, cig, md) is None
