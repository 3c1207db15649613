"""CPU: the seeding restatement (oracle/seed.c: mem_collect_intv with bwt_occ4,
bwt_extend, bwt_smem1a, bwt_seed_strategy1 and klib's introsort restated)
reproduces the reference's intervals exactly.

The golden sets (tests/golden/seed_*.npz, oracle/gen_seed.py) come from
oracle/_ref/gen_seed: mem_collect_intv's control flow (bwamem.c:120-167)
around the REFERENCE's own bwt_smem1, bwt_seed_strategy1 and
ks_introsort_mem_intv, on a bwa index of the golden genome built by the
reference's bwa_idx_build.  Reads: 150 bp (c1) and 100/150/250/40/19/12 bp
(mix) with substitutions, indels, junk reads and N bases."""
import numpy as np
import pytest

import golden_io as G
import oracle


def test_bwt_fixture_is_consistent():
    hdr, words = G.load_seed_bwt()
    primary, L2, seq_len, size = hdr[0], hdr[1:6], hdr[6], hdr[7]
    assert L2[0] == 0 and L2[4] == seq_len and np.all(np.diff(L2) >= 0)
    assert size == len(words) and size >= (seq_len + 127) // 128 * 16 and 0 <= primary <= seq_len
    # the first block's counts are zero; the last block's counts plus its bases are L2's totals
    assert np.all(words[:8] == 0)


@pytest.mark.parametrize("name", G.SEED_SETS)
def test_oracle_collect_intv_matches_reference(name):
    hdr, words = G.load_seed_bwt()
    opt, sf, seq_off, seq, want_n, want = G.load_seed_set(name)
    n, got = oracle.collect_intv(hdr, words, opt, sf, seq_off, seq)
    assert np.array_equal(n, want_n)
    assert np.array_equal(got, want)
    # the sets exercise ties in info (their order is introsort's), N bases and short reads
    off = np.concatenate([[0], np.cumsum(want_n)])
    ties = sum(len(want[off[r]:off[r + 1], 3]) - len(np.unique(want[off[r]:off[r + 1], 3])) for r in range(len(want_n)))
    assert ties > 0
    assert (seq == 4).any()


def test_oracle_bwt_sa_matches_reference():
    """bwt_sa (bwt.c:86-96) restated: 20 000 random BWT positions plus 0, the
    sample boundaries, primary and its neighbours, seq_len"""
    hdr, words = G.load_seed_bwt()
    intv, sa, q, want = G.load_seed_sa()
    assert intv == 32 and hdr[0] in q
    assert np.array_equal(oracle.bwt_sa(hdr, words, sa, intv, q), want)
