"""GPU parity of the opt-in one-seed-per-lane extension kernel (spec_extl_kernel,
DESIGN.md §3) on chains the REFERENCE seeded.

The kernel is off by default (it loses to the two-seeds-per-wave kernel in the
bench), so the default-path tests never run it.  Here it is switched on
(bwagpu_debug_ext_lane, process-wide) for a C2-sized batch and a mixed-length
(C5) batch, beside the pair kernel (mode 2) and before it (mode 1); every
mem_alnreg_t byte, the region order and the per-read counts must equal the
reference's mem_chain2aln output, as on the default path.
"""
import numpy as np
import pytest

import golden_io as G
import refseed
from bwagpu.engine import Engine, compact

pytestmark = [pytest.mark.gpu, pytest.mark.skipif(not refseed.available(), reason="oracle/_ref/gen_golden not built")]


@pytest.fixture
def lane_mode():
    from bwagpu import abi
    lib = abi.load()
    prev = lib.bwagpu_debug_ext_lane(-1)

    def set_mode(m):
        lib.bwagpu_debug_ext_lane(m)

    yield set_mode
    lib.bwagpu_debug_ext_lane(prev)


@pytest.mark.parametrize("mode", [2, 1])
@pytest.mark.parametrize("length,pairs", [("150", 33334), ("mix", 24000)])
def test_lane_kernel_reference_seeded(length, pairs, mode, lane_mode):
    opt, ref, batch, want, want_n = refseed.make(pairs=pairs, seed=7, length=length)
    eng = Engine(0, opt, ref["l_pac"], ref["ann_offset"], ref["ann_len"], pac=ref["pac"])
    lane_mode(mode)
    for _ in range(2):  # the second batch reuses the context's scratch and queue heads
        regs, n = eng.chain2aln(batch)
        assert np.array_equal(n, want_n), f"{int((n != want_n).sum())} reads with a different region count"
        assert G.region_mismatch(compact(batch, regs, n), want) is None
    eng.close()
