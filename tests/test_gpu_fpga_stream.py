"""GPU parity of bwagpu_sw_stream, the FPGA wire format entry (SURVEY.md §8f
rank 4): streams packed by the oracle's restatement of packReadData
(FPGAPipeline.cpp:194-343) from the golden chain sets and from the C2
workload's reference-seeded chains, records bit-exact against the oracle
(tests/test_fpga_stream_oracle.py pins that oracle to the reference's
regions), and the error behaviour of processOutput's checks
(FPGAPipeline.cpp:38-74 -> BWAGPU_E_RESULTS)."""
import numpy as np
import pytest

import golden_io as G
import oracle
from bwagpu import abi, workload
from bwagpu.engine import BwaGpuError, Engine
from test_fpga_stream_oracle import sub_batch, task_word

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def refd():
    return G.load_ref()


def engine_for(refd, opt):
    return Engine(0, opt, refd["l_pac"], refd["ann_offset"], refd["ann_len"], pac=refd["pac"])


def oref(refd):
    return oracle.Ref(refd["l_pac"], refd["ann_offset"], refd["ann_len"], refd["pac"])


def first_diff(got, want):
    bad = np.nonzero((got != want).any(axis=1))[0]
    return None if len(bad) == 0 else f"{len(bad)} records differ; first task {bad[0]}: {got[bad[0]]} vs {want[bad[0]]}"


@pytest.mark.parametrize("name", G.CHAIN_SETS)
def test_chain_sets_bit_exact(refd, name):
    opt, batch, _, _ = G.load_chain_set(name)
    words, nt, _, _ = oracle.fpga_pack(opt, oref(refd), batch)
    want = oracle.fpga_sw(opt, oref(refd), words, nt)
    got = engine_for(refd, opt).sw_stream(words, nt)
    assert got.shape == want.shape
    assert first_diff(got, want) is None


def test_c2_reference_seeded_slice():
    """the bench workload's first 8000 reads (reference seeding on the
    chr21-sized genome): every non-whole-read seed is a task"""
    opt, ref, bs = workload.load_fixture()
    b = sub_batch(bs[0].batch, 0, 8000)
    r = oracle.Ref(ref.l_pac, ref.ann_offset, ref.ann_len, ref.pac)
    words, nt, packed, _ = oracle.fpga_pack(opt, r, b)
    assert nt > 20000
    want = oracle.fpga_sw(opt, r, words, nt)
    eng = Engine(0, opt, ref.l_pac, ref.ann_offset, ref.ann_len, pac=ref.pac)
    got = eng.sw_stream(words, nt)
    assert first_diff(got, want) is None


def test_empty_and_errors(refd):
    opt, batch, _, _ = G.load_chain_set("c1_default")
    eng = engine_for(refd, opt)
    r = oref(refd)
    assert eng.sw_stream(np.zeros(0, np.int32), 0).shape == (0, 10)
    b = sub_batch(batch, 0, 60)
    words, nt, _, _ = oracle.fpga_pack(opt, r, b)
    assert first_diff(eng.sw_stream(words, nt + 100), oracle.fpga_sw(opt, r, words, nt)) is None
    bad = words.copy()
    bad[0] = len(words) + 3
    with pytest.raises(BwaGpuError) as e:
        eng.sw_stream(bad, nt)
    assert e.value.code == abi.E_INVAL
    with pytest.raises(BwaGpuError) as e:
        eng.sw_stream(words, nt - 1)  # task nt-1 out of range
    assert e.value.code == abi.E_RESULTS
    bad = words.copy()
    bad[task_word(words, 0)] = bad[task_word(words, 1)]  # repeated index
    with pytest.raises(BwaGpuError) as e:
        eng.sw_stream(bad, nt)
    assert e.value.code == abi.E_RESULTS
    bad = words.copy()
    bad[task_word(words, 2) + 4] = 10_000  # seed past its read
    with pytest.raises(BwaGpuError) as e:
        eng.sw_stream(bad, nt)
    assert e.value.code == abi.E_RESULTS
    bad = words.copy()
    bad[2] |= 0x70000000  # first base 7
    with pytest.raises(BwaGpuError) as e:
        eng.sw_stream(bad, nt)
    assert e.value.code == abi.E_RESULTS
    bad = words.copy()
    bad[1] = abi.MAX_READ_LEN + 1
    with pytest.raises(BwaGpuError) as e:
        eng.sw_stream(bad, nt)
    assert e.value.code in (abi.E_UNSUPPORTED,)
    # the engine still serves after every refusal
    assert first_diff(eng.sw_stream(words, nt), oracle.fpga_sw(opt, r, words, nt)) is None
