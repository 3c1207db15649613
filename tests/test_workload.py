"""The bench's C2 workload fixture (tests/golden/c2_refseed.npz, made by
oracle/gen_c2_fixture.py from the reference's own seeding on a chr21-sized
genome): the genome regenerates bit for bit, and the oracle/_ref reference and
the C restatement both reproduce the recorded region digests."""
import os
import sys

import numpy as np
import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "bwa-flow_amd", "python"))
sys.path.insert(0, os.path.join(REPO, "oracle"))

import oracle  # noqa: E402
from bwagpu import workload  # noqa: E402
from bwagpu.synth import GoldenRef  # noqa: E402


@pytest.fixture(scope="module")
def c2():
    return workload.load_fixture()


def test_golden_genome_1mb_is_the_golden_ref():
    r = np.load(os.path.join(REPO, "tests", "golden", "ref.npz"))
    g = GoldenRef(1_000_000)
    assert np.array_equal(g.pac, r["pac"])
    assert np.array_equal(g.ann_offset, r["ann_offset"]) and np.array_equal(g.ann_len, r["ann_len"])


def test_fixture_shape(c2):
    opt, ref, bs = c2
    assert ref.l_pac == 46_709_983 and len(bs) == 2
    for rb in bs:
        b = rb.batch
        assert b.n_reads == 66_668 and int(b.seq_off[-1]) > 9_990_000  # 2x150 nominal: 10.0 Mbases
        assert b.n_chains > 1.4 * b.n_reads and b.n_seeds > 4 * b.n_reads  # reference-seeded, not synthetic
        assert len(rb.reg_n) == b.n_reads


@pytest.mark.parametrize("which", ["oracle", "ref"])
def test_cpu_paths_match_fixture_digest(c2, which):
    opt, ref, bs = c2
    if which == "ref" and oracle.ref_lib() is None:
        pytest.skip("oracle/_ref not built")
    R = oracle.Ref(ref.l_pac, ref.ann_offset, ref.ann_len, ref.pac)
    rb = bs[0]
    regs, n, _ = oracle.chain2aln(which, opt, R, rb.batch, n_threads=min(8, os.cpu_count() or 1))
    assert rb.check(regs, n)
    n2 = n.copy()
    if len(n2):
        regs2 = regs.copy()
        k = int(np.argmax(n2 > 0))
        regs2[rb.batch.read_seed_off()[k]]["score"] += 1
        assert not rb.check(regs2, n2)
