"""GPU parity: the HIP engine, called through its C ABI, reproduces the
reference bit for bit.

* golden chain sets (reference seeding + mem_chain2aln): every mem_alnreg_t
  byte, region order and per-read count
* recorded + randomised ksw_extend2 calls: all six outputs
* the double-buffered submit/wait slots, the device-pointer entry, empty and
  ragged batches, and the reference's error conditions
* larger synthetic batches against the oracle (same seeded inputs)
"""
import ctypes as C

import numpy as np
import pytest

import golden_io as G
from conftest import set_c2a_path
import oracle
from bwagpu import abi
from bwagpu.engine import Batch, BwaGpuError, Engine, compact

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def refd():
    return G.load_ref()


@pytest.fixture(params=["spec", "quad", "pair", "fast"])
def c2a_path(request, monkeypatch):
    """mem_chain2aln paths (conftest.set_c2a_path)"""
    restore = set_c2a_path(request.param, monkeypatch)
    yield request.param
    restore()


@pytest.fixture(params=["quad", "wave"])
def ext_path(request):
    """bare ksw_extend2 lists: four per wave with packed 16-bit DP where a task
    fits (default), or the wave kernels only (bwagpu_debug_ext_form(1))"""
    lib = abi.load()
    prev = lib.bwagpu_debug_ext_form(0 if request.param == "quad" else 1)
    yield request.param
    lib.bwagpu_debug_ext_form(prev)


def make_engine(refd, opt):
    return Engine(0, opt, refd["l_pac"], refd["ann_offset"], refd["ann_len"], pac=refd["pac"])


def assert_counts(st, ost, bound):
    """(cells, rows, calls) against the oracle's: equal with the row bound off;
    with it on the same calls, none of them longer"""
    got, want = (st["cells"], st["rows"], st["ext_calls"]), tuple(int(x) for x in ost[:3])
    if bound:
        assert got[2] == want[2] and got[0] <= want[0] and got[1] <= want[1], (got, want)
    else:
        assert got == want


@pytest.mark.parametrize("name", G.CHAIN_SETS)
def test_chain_sets_bit_exact(refd, name, c2a_path):
    opt, batch, want, want_n = G.load_chain_set(name)
    eng = make_engine(refd, opt)
    regs, n = eng.chain2aln(batch)
    assert np.array_equal(n, want_n), f"{int((n != want_n).sum())} reads with a different region count"
    assert G.region_mismatch(compact(batch, regs, n), want) is None
    st = eng.last_stats()
    assert st["cells"] > 0 and st["kernel_ms"] > 0
    eng.close()


@pytest.mark.parametrize("name", G.CHAIN_SETS + G.KSW_SETS)
def test_ksw_extend2_tasks_bit_exact(refd, name, ext_path):
    opt, tasks, want, qp, tp = G.load_tasks(name)
    eng = make_engine(refd, opt)
    _, cells = oracle.extend("oracle", opt, tasks, qp, tp)
    for bound in (1, 0):  # the packed kernels' row bound on (default) and off
        eng.row_bound(bound)
        got = eng.extend_batch(tasks, qp, tp)
        g, w = got.view(np.int32).reshape(-1, 6), want.view(np.int32).reshape(-1, 6)
        bad = np.nonzero((g != w).any(axis=1))[0]
        assert len(bad) == 0, f"{len(bad)} tasks differ; first {tasks[bad[0]]}: got {got[bad[0]]} want {want[bad[0]]}"
        st = eng.last_stats()
        if bound:  # calls end early, never late
            assert st["cells"] <= cells[0] and st["rows"] <= cells[1]
        else:  # the evaluated-cell count agrees with the oracle's count of ksw.c:424 iterations
            assert st["cells"] == cells[0] and st["rows"] == cells[1]
    eng.close()


def test_cell_and_call_counts_match_oracle(refd, c2a_path):
    opt, batch, want, want_n = G.load_chain_set("c1_default")
    eng = make_engine(refd, opt)
    ref = oracle.Ref(refd["l_pac"], refd["ann_offset"], refd["ann_len"], refd["pac"])
    _, _, ost = oracle.chain2aln("oracle", opt, ref, batch)
    for bound in (0, 1):
        eng.row_bound(bound)
        regs, n = eng.chain2aln(batch)
        assert np.array_equal(n, want_n) and G.region_mismatch(compact(batch, regs, n), want) is None
        st = eng.last_stats()
        assert_counts(st, ost, bound)


def test_slots_double_buffered(refd):
    opt, batch, want, want_n = G.load_chain_set("c1_default")
    eng = make_engine(refd, opt)
    half = batch.n_reads // 2
    b0 = batch.subset(range(half))
    b1 = batch.subset(range(half, batch.n_reads))
    eng.submit(0, b0)
    eng.submit(1, b1)
    with pytest.raises(BwaGpuError):  # a slot holds one batch at a time
        eng.submit(0, b0)
    r1, n1 = eng.wait(1, b1)
    r0, n0 = eng.wait(0, b0)
    got = np.concatenate([compact(b0, r0, n0), compact(b1, r1, n1)])
    assert G.region_mismatch(got, want) is None
    eng.close()


def test_reordered_and_ragged_batches(refd, c2a_path):
    opt, batch, want, want_n = G.load_chain_set("c5_mixed")
    eng = make_engine(refd, opt)
    rng = np.random.default_rng(5)
    perm = rng.permutation(batch.n_reads)
    sub = batch.subset(perm)
    regs, n = eng.chain2aln(sub)
    off = np.concatenate([[0], np.cumsum(want_n)])
    exp = np.concatenate([want[off[r]:off[r + 1]] for r in perm])
    assert G.region_mismatch(compact(sub, regs, n), exp) is None
    # empty batch, one read, reads with no chains only
    empty = batch.subset([])
    r, n = eng.chain2aln(empty)
    assert len(r) == 0 and len(n) == 0
    nochain = [i for i in range(batch.n_reads) if batch.read_chain_off[i + 1] == batch.read_chain_off[i]][:5]
    r, n = eng.chain2aln(batch.subset(nochain))
    assert (n == 0).all()
    one = batch.subset([int(np.argmax(want_n))])
    r, n = eng.chain2aln(one)
    assert n[0] == want_n.max()
    eng.close()


def test_error_conditions(refd):
    opt, batch, _, _ = G.load_chain_set("c1_default")
    eng = make_engine(refd, opt)
    # a chain whose rid does not hold its first seed: the reference asserts (bwamem.c:669)
    sub = batch.subset(range(20))
    bad = Batch(sub.seq_off, sub.seq, sub.read_chain_off, sub.chain_seed_off,
                (sub.chain_rid + 1) % len(refd["ann_len"]), sub.chain_frac_rep, sub.seeds)
    with pytest.raises(BwaGpuError) as e:
        eng.chain2aln(bad)
    assert e.value.code == abi.E_RESULTS
    # the engine keeps working after a failed batch
    regs, n = eng.chain2aln(sub)
    assert n.sum() > 0
    # reads longer than BWAGPU_MAX_READ_LEN are refused up front
    long = Batch(np.array([0, 1100]), np.zeros(1100, np.uint8), np.array([0, 0]), np.array([0]),
                 np.zeros(0, np.int32), np.zeros(0, np.float32), np.zeros(0, abi.SEED_DTYPE))
    with pytest.raises(BwaGpuError) as e:
        eng.chain2aln(long)
    assert e.value.code == abi.E_UNSUPPORTED
    # malformed offsets
    mal = Batch(np.array([0, 5]), np.zeros(5, np.uint8), np.array([0, 1]), np.array([0]),
                np.zeros(0, np.int32), np.zeros(0, np.float32), np.zeros(0, abi.SEED_DTYPE))
    with pytest.raises(BwaGpuError) as e:
        eng.chain2aln(mal)
    assert e.value.code == abi.E_INVAL
    # offsets that span their arrays but are not monotone: refused before any
    # offset indexes past the caller's arrays (read 0 claims chains 0..4 of 2,
    # chain 0 claims seeds 0..2 of 1)
    sd = np.zeros(2, abi.SEED_DTYPE)
    sd["len"] = 1
    for rco, cso, ns in (([0, 5, 2], [0, 1, 2], 2), ([0, 2, 2], [0, 3, 1], 1)):
        mal = Batch(np.array([0, 5, 10]), np.zeros(10, np.uint8), np.array(rco, np.int32), np.array(cso, np.int32),
                    np.zeros(2, np.int32), np.zeros(2, np.float32), sd[:ns])
        with pytest.raises(BwaGpuError) as e:
            eng.chain2aln(mal)
        assert e.value.code == abi.E_INVAL
    regs, n = eng.chain2aln(sub)  # and the engine still serves
    assert n.sum() > 0
    eng.close()


def test_lds_refusal_before_enqueue(refd):
    """options whose LDS row buffer cannot fit a launch (huge band and clipping
    bonus) are refused before the H2D is queued: the slot is not left busy, a
    second submit on the same slot gets the same answer, and the device entry
    refuses them too"""
    opt, batch, _, _ = G.load_chain_set("c1_default")
    big = dict(opt, w=40000, pen_clip5=40000, pen_clip3=40000)
    eng = make_engine(refd, big)
    sub = batch.subset(range(50))
    for _ in range(2):
        with pytest.raises(BwaGpuError) as e:
            eng.submit(0, sub)
        assert e.value.code == abi.E_UNSUPPORTED
    eng.close()
    eng = make_engine(refd, opt)  # the ordinary options on a fresh context still run
    regs, n = eng.chain2aln(sub)
    assert n.sum() > 0
    eng.close()


def test_device_and_submit_entries_concurrently(refd):
    """the device entry and the submit/wait slots keep separate scratch: both in
    flight on one context give the reference's regions"""
    torch = pytest.importorskip("torch")
    opt, batch, want, want_n = G.load_chain_set("c1_default")
    eng = make_engine(refd, opt)
    dev = torch.device("cuda", 0)
    t = {k: torch.from_numpy(np.ascontiguousarray(getattr(batch, k)).view(np.uint8).copy()).to(dev)
         for k in ("seq_off", "seq", "read_chain_off", "chain_seed_off", "chain_rid", "chain_frac_rep", "seeds")}
    out = torch.zeros(batch.n_seeds * 88, dtype=torch.uint8, device=dev)
    n = torch.zeros(batch.n_reads, dtype=torch.int32, device=dev)
    bc = abi.BatchC()
    bc.n_reads, bc.n_chains, bc.n_seeds = batch.n_reads, batch.n_chains, batch.n_seeds
    bc.seq_bytes = int(batch.seq_off[-1])
    for k in t:
        setattr(bc, k, t[k].data_ptr())
    s = torch.cuda.Stream()
    for _ in range(3):
        eng.chain2aln_device(bc, out.data_ptr(), n.data_ptr(), None, s.cuda_stream)
        eng.submit(0, batch)
        r0, n0 = eng.wait(0, batch)
        assert G.region_mismatch(compact(batch, r0, n0), want) is None
    torch.cuda.synchronize()
    regs = out.cpu().numpy().view(abi.ALNREG_DTYPE)
    nn = n.cpu().numpy()
    assert np.array_equal(nn, want_n)
    assert G.region_mismatch(compact(batch, regs, nn), want) is None
    eng.close()


def test_device_entry_point_with_torch_buffers(refd):
    torch = pytest.importorskip("torch")
    opt, batch, want, want_n = G.load_chain_set("opt2_band")
    eng = make_engine(refd, opt)
    dev = torch.device("cuda", 0)
    t = {k: torch.from_numpy(np.ascontiguousarray(getattr(batch, k)).view(np.uint8)).to(dev)
         for k in ("seq_off", "seq", "read_chain_off", "chain_seed_off", "chain_rid", "chain_frac_rep", "seeds")}
    out = torch.zeros(batch.n_seeds * 88, dtype=torch.uint8, device=dev)
    n = torch.zeros(batch.n_reads, dtype=torch.int32, device=dev)
    stats = torch.zeros(4, dtype=torch.int64, device=dev)
    bc = abi.BatchC()
    bc.n_reads, bc.n_chains, bc.n_seeds = batch.n_reads, batch.n_chains, batch.n_seeds
    bc.seq_bytes = int(batch.seq_off[-1])
    for k in t:
        setattr(bc, k, t[k].data_ptr())
    stream = torch.cuda.current_stream().cuda_stream
    eng.chain2aln_device(bc, out.data_ptr(), n.data_ptr(), stats.data_ptr(), stream)
    torch.cuda.synchronize()
    regs = out.cpu().numpy().view(abi.ALNREG_DTYPE)
    nn = n.cpu().numpy()
    assert np.array_equal(nn, want_n)
    assert G.region_mismatch(compact(batch, regs, nn), want) is None
    assert int(stats[0]) > 0 and int(stats[3]) == 0
    eng.close()


def test_device_entry_read_len_bound(refd):
    """bwagpu_set_device_read_len: the exact bound gives the same regions (the
    longer length bins are not launched); a bound below the longest read sets
    the length error flag; out-of-range bounds are refused"""
    torch = pytest.importorskip("torch")
    from bwagpu.synth import SynthRef, synth_batch
    sref = SynthRef(78, 2_000_000, 3)
    batch = synth_batch(sref, 9, 300, 0, 19)  # mixed read lengths
    opt = abi.default_opt()
    eng = Engine(0, opt, sref.l_pac, sref.ann_offset, sref.ann_len, pac=sref.pac)
    want, want_n = eng.chain2aln(batch)
    lq = np.diff(batch.seq_off)
    dev = torch.device("cuda", 0)
    t = {k: torch.from_numpy(np.ascontiguousarray(getattr(batch, k)).view(np.uint8)).to(dev)
         for k in ("seq_off", "seq", "read_chain_off", "chain_seed_off", "chain_rid", "chain_frac_rep", "seeds")}
    bc = abi.BatchC()
    bc.n_reads, bc.n_chains, bc.n_seeds = batch.n_reads, batch.n_chains, batch.n_seeds
    bc.seq_bytes = int(batch.seq_off[-1])
    for k in t:
        setattr(bc, k, t[k].data_ptr())
    stream = torch.cuda.current_stream().cuda_stream
    for bound, err in ((int(lq.max()), 0), (160, 2 if lq.max() > 160 else 0), (int(lq.max()) - 1, 2)):
        eng.set_device_read_len(bound)
        out = torch.zeros(batch.n_seeds * 88, dtype=torch.uint8, device=dev)
        n = torch.zeros(batch.n_reads, dtype=torch.int32, device=dev)
        stats = torch.zeros(4, dtype=torch.int64, device=dev)
        eng.chain2aln_device(bc, out.data_ptr(), n.data_ptr(), stats.data_ptr(), stream)
        torch.cuda.synchronize()
        assert int(stats[3]) & 2 == err, bound
        if err == 0:
            nn = n.cpu().numpy()
            assert np.array_equal(nn, want_n)
            regs = out.cpu().numpy().view(abi.ALNREG_DTYPE)
            assert G.region_mismatch(compact(batch, regs, nn), compact(batch, want, want_n)) is None
    for bad in (0, abi.MAX_READ_LEN + 1):
        with pytest.raises(BwaGpuError):
            eng.set_device_read_len(bad)
    eng.close()


@pytest.mark.parametrize("len_mode,min_seed,pairs", [(150, 19, 800), (0, 19, 600), (250, 12, 400), (400, 12, 300),
                                                     (700, 8, 150), (1000, 8, 60)])
def test_synthetic_batches_vs_oracle(len_mode, min_seed, pairs, c2a_path):
    """seeded synthetic reads of every kernel variant's shape — 100-256 bp on
    the fast kernel, > 32 seeds (short min seed length) and 257-1023 bp on the
    generic kernel — against the oracle on the same inputs, bit for bit"""
    from bwagpu.synth import SynthRef, synth_batch
    ref = SynthRef(77, 2_000_000, 3)
    b = synth_batch(ref, 5 + len_mode, pairs, len_mode, min_seed)
    opt = abi.default_opt()
    eng = Engine(0, opt, ref.l_pac, ref.ann_offset, ref.ann_len, pac=ref.pac)
    R = oracle.Ref(ref.l_pac, ref.ann_offset, ref.ann_len, ref.pac)
    oregs, on, ostats = oracle.chain2aln("oracle", opt, R, b, n_threads=4)
    for bound in (1, 0):
        eng.row_bound(bound)
        regs, n = eng.chain2aln(b)
        st = eng.last_stats()
        assert np.array_equal(n, on), f"{int((n != on).sum())} reads with a different region count"
        assert G.region_mismatch(compact(b, regs, n), compact(b, oregs, on)) is None
        assert_counts(st, ostats, bound)
    eng.close()


def split_seeds(b: Batch, piece: int) -> Batch:
    """every seed cut into exact sub-matches of `piece` bases (score = length):
    valid mem_chain2aln input with many seeds per chain"""
    seeds, cso = [], [0]
    for c in range(b.n_chains):
        for s in b.seeds[b.chain_seed_off[c]:b.chain_seed_off[c + 1]]:
            for k in range(0, int(s["len"]), piece):
                ln = min(piece, int(s["len"]) - k)
                seeds.append((int(s["rbeg"]) + k, int(s["qbeg"]) + k, ln, ln, 0))
        cso.append(len(seeds))
    arr = np.array(seeds, dtype=abi.SEED_DTYPE) if seeds else np.zeros(0, abi.SEED_DTYPE)
    return Batch(b.seq_off, b.seq, b.read_chain_off, np.array(cso, np.int32), b.chain_rid, b.chain_frac_rep, arr)


@pytest.mark.parametrize("len_mode,piece", [(150, 6), (250, 9), (400, 14)])
def test_many_seed_reads_vs_oracle(len_mode, piece, c2a_path):
    """reads with more seeds or chains than the fast kernel keeps per wave
    (> 32) go to the generic kernel; both against the oracle"""
    from bwagpu.synth import SynthRef, synth_batch
    ref = SynthRef(78, 1_000_000, 2)
    b = split_seeds(synth_batch(ref, 9 + len_mode, 120, len_mode), piece)
    spr = b.chain_seed_off[b.read_chain_off[1:]] - b.chain_seed_off[b.read_chain_off[:-1]]
    assert (spr > 32).any() and (spr <= 32).any()
    opt = abi.default_opt()
    eng = Engine(0, opt, ref.l_pac, ref.ann_offset, ref.ann_len, pac=ref.pac)
    regs, n = eng.chain2aln(b)
    R = oracle.Ref(ref.l_pac, ref.ann_offset, ref.ann_len, ref.pac)
    oregs, on, _ = oracle.chain2aln("oracle", opt, R, b, n_threads=4)
    assert np.array_equal(n, on)
    assert G.region_mismatch(compact(b, regs, n), compact(b, oregs, on)) is None
    eng.close()


def far_seed_batch(b: Batch, ann_offset, ann_len, dist: int, n_reads: int) -> Batch:
    """a copy of the batch where the first chain of each of the first n_reads
    reads with a forward-strand chain gets one more seed `dist` bases
    downstream of its first seed (same query interval): a chain window of
    more than `dist` bases, as a chain collected along a tandem repeat has"""
    seeds, cso = [], [0]
    done = 0
    for c in range(b.n_chains):
        s0, s1 = int(b.chain_seed_off[c]), int(b.chain_seed_off[c + 1])
        chain = [tuple(int(x) for x in sd) for sd in b.seeds[s0:s1]]
        first_of_read = c in set(int(x) for x in b.read_chain_off[:-1])
        if chain and first_of_read and done < n_reads:
            rid = int(b.chain_rid[c])
            rb, qb, ln, sc, _ = chain[0]
            end = int(ann_offset[rid]) + int(ann_len[rid])
            if rb >= int(ann_offset[rid]) and rb + dist + ln < end:
                chain.append((rb + dist, qb, ln, sc, 0))
                done += 1
        seeds.extend(chain)
        cso.append(len(seeds))
    assert done == n_reads
    arr = np.array(seeds, dtype=abi.SEED_DTYPE)
    return Batch(b.seq_off, b.seq, b.read_chain_off, np.array(cso, np.int32), b.chain_rid, b.chain_frac_rep, arr)


@pytest.mark.parametrize("dist", [40_000, 70_000])
def test_chain_window_past_16_bits(refd, dist, c2a_path):
    """chain windows of 40 and 70 kb: a seed's target length (the window
    distance, ksw_extend2's tlen) no longer fits the packed kernels' 16-bit
    row counters; rows past qlen + w + 1 have an empty band (ksw.c:415-419),
    so the call is capped there with every output unchanged, on every path,
    against the oracle"""
    opt, batch, _, _ = G.load_chain_set("c1_default")
    sub = batch.subset(range(400))
    b = far_seed_batch(sub, refd["ann_offset"], refd["ann_len"], dist, 120)
    eng = make_engine(refd, opt)
    ref = oracle.Ref(refd["l_pac"], refd["ann_offset"], refd["ann_len"], refd["pac"])
    oregs, on, ost = oracle.chain2aln("oracle", opt, ref, b)
    for bound in (1, 0):
        eng.row_bound(bound)
        regs, n = eng.chain2aln(b)
        st = eng.last_stats()
        assert np.array_equal(n, on), f"{int((n != on).sum())} reads with a different region count"
        assert G.region_mismatch(compact(b, regs, n), compact(b, oregs, on)) is None
        assert_counts(st, ost, bound)
    eng.close()
