"""GPU parity of the batched ksw_align2 (mate rescue):
the HIP kernels, called through bwagpu_align2_batch / bwagpu_align2_device,
return the reference's kswr_t bit for bit.

* golden sets from the reference's own ksw_align2 (oracle/gen_golden.py):
  mate-rescue-shaped calls (XSUBO|XSTART|XBYTE as mem_matesw passes them,
  bwamem_pair.c:150) and edge cases (u8 saturation at 255, XSTOP, plain
  calls, qlen 1..1023 over every segment-count bucket)
* o_ins == 0 is refused with E_UNSUPPORTED (the reference's lazy-F early
  exit then depends on its SIMD lane order; the caller keeps the CPU path)
* fresh seeded batches against the oracle, the device-pointer entry, cell
  counts, empty / zero-length tasks
"""
import numpy as np
import pytest

import golden_io as G
import oracle
from bwagpu import abi, synth
from bwagpu.engine import BwaGpuError, Engine

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def refd():
    return G.load_ref()


def make_engine(refd, opt):
    return Engine(0, opt, refd["l_pac"], refd["ann_offset"], refd["ann_len"], pac=refd["pac"])


@pytest.mark.parametrize("name", G.ALIGN2_SETS)
def test_align2_golden_bit_exact(refd, name):
    opt, tasks, want, qp, tp = G.load_align2(name)
    eng = make_engine(refd, opt)
    if opt["o_ins"] == 0:
        with pytest.raises(BwaGpuError) as ei:
            eng.align2_batch(tasks, qp, tp)
        assert ei.value.code == abi.E_UNSUPPORTED
        eng.close()
        return
    got = eng.align2_batch(tasks, qp, tp)
    assert G.kswr_mismatch(tasks, got, want) is None
    _, cells = oracle.align2("oracle", opt, tasks, qp, tp)
    st = eng.last_stats()
    assert st["cells"] == cells[0] and st["kernel_ms"] > 0
    eng.close()


def _concat(parts):
    ts, qs, tps, qo, to = [], [], [], 0, 0
    for t, q, tp in parts:
        t = t.copy()
        t["qoff"] += qo
        t["toff"] += to
        ts.append(t)
        qs.append(q)
        tps.append(tp)
        qo += len(q)
        to += len(tp)
    return np.concatenate(ts), np.concatenate(qs), np.concatenate(tps)


@pytest.mark.parametrize("optname", ["default", "scoring", "cheapdel"])
def test_align2_fresh_batches_vs_oracle(refd, optname):
    import gen_golden
    o = gen_golden.ALIGN2_OPTS[optname]
    opt = abi.default_opt() if o is None else dict(o, mat=abi.fill_scmat(o["a"], o["b"]))
    rng = np.random.default_rng(77)
    tasks, qp, tp = _concat([
        synth.mate_rescue_tasks(rng, 600, a=opt["a"], qlens=(100, 150, 250), xtra_mode="matesw"),
        synth.mate_rescue_tasks(rng, 400, a=opt["a"], qlens=gen_golden.A2_SHORT, win=(0, 300), xtra_mode="mix"),
        # every bucket of both widths: 16*ceil(q/16) and 8*ceil(q/8) columns over 64 lanes
        synth.mate_rescue_tasks(rng, 120, a=opt["a"], qlens=(320, 384, 385, 448, 512, 513, 640, 767, 768, 1023),
                                win=(0, 600), xtra_mode="mix"),
    ])
    eng = make_engine(refd, opt)
    got = eng.align2_batch(tasks, qp, tp)
    want, cells = oracle.align2("oracle", opt, tasks, qp, tp)
    assert G.kswr_mismatch(tasks, got, want) is None
    assert eng.last_stats()["cells"] == cells[0]
    eng.close()


def test_align2_empty_and_zero_length(refd):
    opt = abi.default_opt()
    eng = make_engine(refd, opt)
    assert len(eng.align2_batch(np.zeros(0, abi.ALIGN2_TASK_DTYPE), np.zeros(0, np.uint8),
                                np.zeros(0, np.uint8))) == 0
    rng = np.random.default_rng(5)
    q = rng.integers(0, 4, 50).astype(np.uint8)
    t = rng.integers(0, 4, 80).astype(np.uint8)
    tasks = np.zeros(8, abi.ALIGN2_TASK_DTYPE)
    flags = [0, abi.KSW_XSTART, abi.KSW_XBYTE | abi.KSW_XSTART, abi.KSW_XSUBO | abi.KSW_XSTART]
    for k in range(8):  # qlen 0 or tlen 0 under every flag combination
        tasks[k] = (0, 0, 0 if k < 4 else 50, 80 if k < 4 else 0, flags[k % 4], 0)
    got = eng.align2_batch(tasks, q, t)
    want, _ = oracle.align2("oracle", opt, tasks, q, t)
    assert G.kswr_mismatch(tasks, got, want) is None
    eng.close()


def test_align2_errors(refd):
    opt = abi.default_opt()
    eng = make_engine(refd, opt)
    q = np.zeros(10, np.uint8)
    t = np.zeros(10, np.uint8)
    bad = np.zeros(1, abi.ALIGN2_TASK_DTYPE)
    bad[0] = (5, 0, 10, 10, 0, 0)  # query runs past its pool
    with pytest.raises(BwaGpuError) as ei:
        eng.align2_batch(bad, q, t)
    assert ei.value.code == abi.E_INVAL
    longq = np.zeros(1100, np.uint8)
    bad[0] = (0, 0, 1024, 10, abi.KSW_XBYTE, 0)
    with pytest.raises(BwaGpuError) as ei:
        eng.align2_batch(bad, longq, t)
    assert ei.value.code == abi.E_UNSUPPORTED
    q5 = np.full(10, 5, np.uint8)
    bad[0] = (0, 0, 10, 10, 0, 0)
    with pytest.raises(BwaGpuError) as ei:
        eng.align2_batch(bad, q5, t)
    assert ei.value.code == abi.E_INVAL
    # the context stays usable
    ok = np.zeros(1, abi.ALIGN2_TASK_DTYPE)
    ok[0] = (0, 0, 10, 10, abi.KSW_XSTART, 0)
    got = eng.align2_batch(ok, q, t)
    want, _ = oracle.align2("oracle", opt, ok, q, t)
    assert G.kswr_mismatch(ok, got, want) is None
    eng.close()


def test_align2_device_entry_with_torch_buffers(refd):
    import torch
    opt = abi.default_opt()
    rng = np.random.default_rng(11)
    tasks, qp, tp = _concat([
        synth.mate_rescue_tasks(rng, 700, qlens=(100, 150, 250), xtra_mode="matesw"),
        synth.mate_rescue_tasks(rng, 200, qlens=(33, 300, 700, 1023), win=(0, 500), xtra_mode="mix"),
    ])
    eng = make_engine(refd, opt)
    dev = torch.device("cuda:0")
    d_tasks = torch.from_numpy(tasks.view(np.uint8).copy()).to(dev)
    d_q = torch.from_numpy(qp.copy()).to(dev)
    d_t = torch.from_numpy(tp.copy()).to(dev)
    d_out = torch.zeros(len(tasks) * abi.KSWR_DTYPE.itemsize, dtype=torch.uint8, device=dev)
    d_scr = torch.zeros(8 * (int(tasks["tlen"].sum()) + len(tasks)), dtype=torch.uint8, device=dev)
    stream = torch.cuda.current_stream(dev)
    eng.align2_device(len(tasks), d_tasks.data_ptr(), d_q.data_ptr(), d_t.data_ptr(), d_out.data_ptr(),
                      d_scr.data_ptr(), stream.cuda_stream)
    torch.cuda.synchronize(dev)
    got = d_out.cpu().numpy().view(abi.KSWR_DTYPE)
    want, _ = oracle.align2("oracle", opt, tasks, qp, tp)
    assert G.kswr_mismatch(tasks, got, want) is None
    # same answers as the host-staged entry
    assert np.array_equal(eng.align2_batch(tasks, qp, tp).view(np.int32), got.view(np.int32))
    eng.close()
