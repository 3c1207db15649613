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


def test_c5_refseed_fixture_matches_the_oracle(c2):
    """tests/golden/c5_refseed.npz (the bench's c5_refseed leg): one mixed
    2x100 / 2x150 / 2x250 ChainsRecord seeded by the reference on the C2 genome;
    the oracle reproduces the reference's regions on it (per-read counts and
    the SHA-256 of every record)"""
    _, ref, _ = c2
    opt, _, bs = workload.load_fixture(workload.C5_FIXTURE, with_ref=False)
    z = np.load(workload.C5_FIXTURE)
    import hashlib
    assert hashlib.sha256(ref.pac.tobytes()).digest() == z["pac_sha256"].tobytes()
    rb = bs[0]
    lens = set(np.diff(rb.batch.seq_off).tolist())
    assert {100, 150, 250} <= lens and int(rb.batch.seq_off[-1]) > 9_000_000
    R = oracle.Ref(ref.l_pac, ref.ann_offset, ref.ann_len, ref.pac)
    regs, n, _ = oracle.chain2aln("oracle", opt, R, rb.batch, n_threads=min(8, os.cpu_count() or 1))
    assert rb.check(regs, n)
