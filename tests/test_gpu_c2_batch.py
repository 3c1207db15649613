"""GPU parity at full ChainsRecord size on chains the REFERENCE seeded.

One C2-sized batch (33,334 2x150 pairs = 66,668 reads, >= 10 Mbases: one
ChainsRecord, src/Pipeline.cpp:123,146) is seeded and chained by the
reference's own bwa (mem_chain -> mem_chain_flt -> mem_flt_chained_seeds, run
by oracle/_ref/gen_golden on the golden genome with repeats, N runs and contig
junctions), and the reference's own mem_chain2aln gives the expected regions.
The GPU stage must reproduce every mem_alnreg_t byte, the region order and the
per-read counts — through the host-buffer entry and through the device entry.
The mixed-length set (C5: 2x100 / 2x150 / 2x250) runs the same way.
"""
import numpy as np
import pytest

import golden_io as G
import refseed
from conftest import set_c2a_path
from bwagpu import abi
from bwagpu.engine import Engine, compact

pytestmark = [pytest.mark.gpu, pytest.mark.skipif(not refseed.available(), reason="oracle/_ref/gen_golden not built")]


@pytest.fixture(params=["spec", "quad", "pair", "fast"])
def c2a_path(request, monkeypatch):
    restore = set_c2a_path(request.param, monkeypatch)
    yield request.param
    restore()


@pytest.mark.parametrize("length,pairs", [("150", 33334), ("mix", 24000)])
def test_reference_seeded_full_batch(length, pairs, c2a_path):
    opt, ref, batch, want, want_n = refseed.make(pairs=pairs, seed=7, length=length)
    assert int(batch.seq_off[-1]) >= 3_000_000 * (2 if length == "150" else 1)
    eng = Engine(0, opt, ref["l_pac"], ref["ann_offset"], ref["ann_len"], pac=ref["pac"])
    regs, n = eng.chain2aln(batch)
    assert np.array_equal(n, want_n), f"{int((n != want_n).sum())} reads with a different region count"
    assert G.region_mismatch(compact(batch, regs, n), want) is None
    st = eng.last_stats()
    assert st["ext_calls"] > batch.n_reads  # reference-seeded chains: > 1 extension per read
    eng.close()


def test_reference_seeded_device_entry():
    torch = pytest.importorskip("torch")
    opt, ref, batch, want, want_n = refseed.make(pairs=33334, seed=11, length="150")
    eng = Engine(0, opt, ref["l_pac"], ref["ann_offset"], ref["ann_len"], pac=ref["pac"])
    dev = torch.device("cuda:0")
    fields = ("seq_off", "seq", "read_chain_off", "chain_seed_off", "chain_rid", "chain_frac_rep", "seeds")
    t = {k: torch.from_numpy(np.ascontiguousarray(getattr(batch, k)).view(np.uint8).copy()).to(dev) for k in fields}
    out = torch.zeros(max(batch.n_seeds, 1) * 88, dtype=torch.uint8, device=dev)
    nn = torch.zeros(max(batch.n_reads, 1), dtype=torch.int32, device=dev)
    c = abi.BatchC()
    c.n_reads, c.n_chains, c.n_seeds = batch.n_reads, batch.n_chains, batch.n_seeds
    c.seq_bytes = int(batch.seq_off[-1])
    for k in fields:
        setattr(c, k, t[k].data_ptr())
    stream = torch.cuda.current_stream()
    for _ in range(2):  # the second launch reuses the context's scratch
        eng.chain2aln_device(c, out.data_ptr(), nn.data_ptr(), None, stream.cuda_stream)
    torch.cuda.synchronize()
    regs = out.cpu().numpy().view(abi.ALNREG_DTYPE)[:batch.n_seeds]
    n = nn.cpu().numpy()[:batch.n_reads]
    assert np.array_equal(n, want_n)
    assert G.region_mismatch(compact(batch, regs, n), want) is None
    eng.close()


def test_full_batch_malformed_refused():
    """a C2-sized batch goes through the multi-threaded stage-and-check pass of
    bwagpu_chain2aln_submit (blocks of 1024 reads on 8 threads): a bad seed deep
    inside it, or offsets that turn back at a block boundary, are refused with
    E_INVAL before anything is enqueued, and the same context then serves the
    intact batch with the reference's regions"""
    from bwagpu import workload
    from bwagpu.engine import Batch, BwaGpuError
    opt, ref, rbs = workload.load_fixture()
    rb = rbs[0]
    b = rb.batch
    assert b.n_seeds >= 1 << 16 and b.n_reads > 8 * 1024
    eng = Engine(0, opt, ref.l_pac, ref.ann_offset, ref.ann_len, pac=ref.pac)
    sd = b.seeds.copy()
    k = int(b.chain_seed_off[b.read_chain_off[40_000]])  # a seed of read 40 000 (block 39, thread 4)
    sd[k]["qbeg"] = 10_000  # outside its read
    bad_seed = Batch(b.seq_off, b.seq, b.read_chain_off, b.chain_seed_off, b.chain_rid, b.chain_frac_rep, sd)
    rco = b.read_chain_off.copy()
    rco[5 * 1024] = rco[5 * 1024 + 1] + 1  # turns back at the boundary of blocks 4 and 5
    bad_off = Batch(b.seq_off, b.seq, rco, b.chain_seed_off, b.chain_rid, b.chain_frac_rep, b.seeds)
    for bad in (bad_seed, bad_off):
        with pytest.raises(BwaGpuError) as e:
            eng.chain2aln(bad)
        assert e.value.code == abi.E_INVAL
    regs, n = eng.chain2aln(b)
    assert rb.check(regs, n)
    eng.close()


def test_slot_results_survive_the_next_stage():
    """bwagpu_chain2aln_results stays valid until the slot's next _submit
    (include/bwagpu.h): wait(NULL) -> _stage of the NEXT batch over the slot's
    pinned input -> _results must still give the finished batch's slot layout
    (its offsets are moved out of the staging buffer before it is overwritten);
    a submit that is refused leaves the slot with no results at all"""
    import ctypes as C
    from bwagpu import workload
    from bwagpu.engine import BwaGpuError
    opt, ref, rbs = workload.load_fixture()
    b0, b1 = rbs[0].batch, rbs[1].batch
    eng = Engine(0, opt, ref.l_pac, ref.ann_offset, ref.ann_len, pac=ref.pac)
    lib = eng.lib
    eng.submit(1, b0)
    assert lib.bwagpu_chain2aln_wait(eng.ctx, 1, None, None) == 0
    view = abi.BatchC()
    assert lib.bwagpu_chain2aln_stage(eng.ctx, 1, b1.n_reads, b1.n_chains, b1.n_seeds, int(b1.seq_off[-1]),
                                      C.byref(view)) == 0
    # the caller packs b1 into the pinned input (its offsets overwrite b0's)
    for k, dt in (("read_chain_off", np.int32), ("chain_seed_off", np.int32), ("seq_off", np.int64)):
        a = np.ascontiguousarray(getattr(b1, k), dt)
        C.memmove(getattr(view, k), a.ctypes.data, a.nbytes)
    rp, np_ = C.c_void_p(), C.c_void_p()
    assert lib.bwagpu_chain2aln_results(eng.ctx, 1, C.byref(rp), C.byref(np_)) == 0
    n = np.ctypeslib.as_array(C.cast(np_, C.POINTER(C.c_int32)), (b0.n_reads,)).copy()
    regs = np.ctypeslib.as_array(C.cast(rp, C.POINTER(C.c_uint8)), (b0.n_seeds * 88,)).copy().view(abi.ALNREG_DTYPE)
    assert rbs[0].check(regs, n)
    # a refused submit on the slot: no results until a batch finishes there again
    bad = workload.Batch(b0.seq_off, b0.seq, b0.read_chain_off, b0.chain_seed_off, b0.chain_rid,
                         b0.chain_frac_rep, b0.seeds.copy())
    bad.seeds[5]["qbeg"] = 10_000
    with pytest.raises(BwaGpuError):
        eng.submit(1, bad)
    op = C.c_void_p()
    assert lib.bwagpu_chain2aln_results(eng.ctx, 1, C.byref(rp), C.byref(np_)) == abi.E_INVAL
    assert lib.bwagpu_chain2aln_results_dense(eng.ctx, 1, C.byref(rp), C.byref(np_), C.byref(op)) == abi.E_INVAL
    eng.submit(1, b1)
    got = eng.wait_dense(1, b1)
    assert rbs[1].check_compact(*got)
    eng.close()
