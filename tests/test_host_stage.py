"""The C++ host side: bwa-flow_amd/host/ (kflow mirror + ChainsToRegionsGPU,
the replacement of ChainsToRegionsFPGA, src/fpga/FPGAPipeline.cpp:367-579)
driven like bwa-flow's stage 4 by tests/cpp/test_pipeline.cpp on the golden
chain sets; regions must equal the reference's, record ownership must follow
ChainsToRegions::compute (src/Pipeline.cpp:503-544).

CPU tier: the pipeline with the CPU stage only (oracle as the stage body),
and with a GPU back end that has no device — its workers retire at once and
switch accx dispatch off (FPGAPipeline.cpp:402-405), so every record must
drain back to the CPU stage.  GPU tier: the GPU back end attached with
priority 10 (main.cpp:365) and as the sole stage (--disable_sw_cpu)."""
import json
import os
import subprocess

import numpy as np
import pytest

import golden_io as G
from bwagpu import abi

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CPP = os.path.join(REPO, "tests", "cpp")
EXE = os.path.join(CPP, "build", "test_pipeline")


@pytest.fixture(scope="module")
def exe():
    subprocess.run(["make", "-s", "-C", CPP], check=True)
    return EXE


def write_inputs(d, name):
    opt, b, regs, n = G.load_chain_set(name)
    ref = G.load_ref()
    o = abi.opt_from_dict(opt)
    open(os.path.join(d, "opt.bin"), "wb").write(bytes(o))
    np.array([ref["l_pac"]], np.int64).tofile(os.path.join(d, "l_pac.bin"))
    np.asarray(ref["ann_offset"], np.int64).tofile(os.path.join(d, "ann_offset.bin"))
    np.asarray(ref["ann_len"], np.int32).tofile(os.path.join(d, "ann_len.bin"))
    np.asarray(ref["pac"], np.uint8).tofile(os.path.join(d, "pac.bin"))
    for k in ("seq_off", "seq", "read_chain_off", "chain_seed_off", "chain_rid", "chain_frac_rep", "seeds"):
        getattr(b, k).tofile(os.path.join(d, k + ".bin"))
    return b, regs, n


def run(exe, d, mode, per_rec, workers, rc=0, chain_mode="forward"):
    env = dict(os.environ, TEST_CHAIN_MODE=chain_mode)
    p = subprocess.run([exe, d, mode, str(per_rec), str(workers)], capture_output=True, text=True, timeout=600,
                       env=env)
    assert p.returncode == rc, p.stderr
    info = json.loads(p.stdout.strip().splitlines()[-1])
    n = np.fromfile(os.path.join(d, "out_n.bin"), np.int32)
    regs = np.fromfile(os.path.join(d, "out_regs.bin"), np.uint8).view(abi.ALNREG_DTYPE)
    return info, regs, n


def check(regs, n, want_regs, want_n):
    assert np.array_equal(n, want_n)
    assert G.region_mismatch(regs, want_regs) is None


@pytest.mark.parametrize("mode,per_rec,workers", [("cpu", 97, 3), ("accx_none", 64, 2)])
def test_pipeline_cpu_paths(exe, tmp_path, mode, per_rec, workers):
    d = str(tmp_path)
    b, want_regs, want_n = write_inputs(d, "c1_default")
    info, regs, n = run(exe, d, mode, per_rec, workers)
    assert info["outputs"] == info["records"] == -(-b.n_reads // per_rec)
    assert info["bad_ownership"] == 0 and info["on_gpu"] == 0
    check(regs, n, want_regs, want_n)


@pytest.mark.parametrize("inline", [False, True])
def test_chain_reaper_frees_every_record(exe, tmp_path, inline):
    """ChainReaper (host/GPUPipeline.cpp): the GPU stage's background frees of
    the records' chains, released from 4 threads at once; after drain() the
    heap is back to its size before the records were built.  BWAGPU_CHAIN_REAPER=0
    frees inline in release()."""
    d = str(tmp_path)
    b, _, _ = write_inputs(d, "c1_default")
    env = dict(os.environ, BWAGPU_CHAIN_REAPER="0" if inline else "1")
    p = subprocess.run([exe, d, "reaper", "37", "4"], capture_output=True, text=True, timeout=120, env=env)
    assert p.returncode == 0, p.stderr
    info = json.loads(p.stdout.strip().splitlines()[-1])
    assert info["records"] == -(-b.n_reads // 37)
    # what may stay "in use" after the frees: the reaper's queue nodes and the
    # chunks glibc parks in the freeing thread's tcache (at most 7 per size
    # class); a leak would leave about all of built_bytes
    assert info["built_bytes"] > 400_000
    assert info["left_bytes"] < min(256 * 1024, info["built_bytes"] // 2), info
    # with the reaper off every free is inline and none is counted as a fallback
    assert not inline or info["inline_frees"] == 0


def test_chain_reaper_bounded_queue(exe, tmp_path):
    """a reaper that has fallen behind (held: it frees nothing) queues at most
    ChainReaper::kMaxQueued records; every later release frees inline on the
    releasing thread, and after drain() the heap is back where it started"""
    d = str(tmp_path)
    b, _, _ = write_inputs(d, "c1_default")
    env = dict(os.environ, BWAGPU_CHAIN_REAPER="1", TEST_REAPER_HOLD="1")
    p = subprocess.run([exe, d, "reaper", "37", "4"], capture_output=True, text=True, timeout=120, env=env)
    assert p.returncode == 0, p.stderr
    info = json.loads(p.stdout.strip().splitlines()[-1])
    k_max_queued = 4 * 4  # 4 * BWAGPU_NUM_SLOTS
    assert info["records"] == -(-b.n_reads // 37) > k_max_queued
    assert info["inline_frees"] == info["records"] - k_max_queued, info
    assert info["left_bytes"] < min(256 * 1024, info["built_bytes"] // 2), info


@pytest.mark.gpu
@pytest.mark.parametrize("name", ["c1_default", "c5_mixed"])
@pytest.mark.parametrize("mode", ["gpu", "gpu_only"])
@pytest.mark.parametrize("chain_mode", ["forward", "free"])
def test_pipeline_gpu_stage(exe, tmp_path, name, mode, chain_mode):
    """chain ownership: forwarded in the GPU records for RegionsToSam to free
    (the FPGA stage's, FPGAPipeline.cpp:434) or freed by the stage with NULL
    forwarded (the CPU stage's, Pipeline.cpp:526-537); records the CPU stage
    made always carry NULL"""
    d = str(tmp_path)
    b, want_regs, want_n = write_inputs(d, name)
    info, regs, n = run(exe, d, mode, 50, 2, chain_mode=chain_mode)
    assert info["devices"] >= 1 and info["on_gpu"] > 0 and info["gpu_fallback_cpu"] == 0
    if mode == "gpu_only":
        assert info["on_gpu"] == info["records"]
    assert info["bad_ownership"] == 0
    assert info["forwarded"] == (info["on_gpu"] if chain_mode == "forward" else 0), info
    check(regs, n, want_regs, want_n)


@pytest.mark.gpu
def test_two_workers_per_device(exe, tmp_path):
    """two contexts on each device share one resident reference (GPUEnv
    per_device = 2): both workers pull records, outputs equal the golden regions"""
    d = str(tmp_path)
    b, want_regs, want_n = write_inputs(d, "c1_default")
    info, regs, n = run(exe, d, "gpu_2ctx", 40, 2)
    assert info["devices"] >= 2 and info["on_gpu"] == info["records"]
    assert info["w0"] > 0 and info["w1"] > 0, info
    check(regs, n, want_regs, want_n)


@pytest.mark.gpu
def test_reference_through_rccl_broadcast(exe, tmp_path):
    """GPUEnv's RCCL branch (ncclCommInitAll + grouped ncclBroadcast, the
    start-up broadcast of the packed reference over xGMI, BWAOCLEnv.h:67-114's
    per-device upload): forced on a one-rank communicator, the context's
    reference is the broadcast's output, and every region equals the golden one"""
    d = str(tmp_path)
    b, want_regs, want_n = write_inputs(d, "c1_default")
    info, regs, n = run(exe, d, "gpu_rccl", 50, 2)
    assert info["rccl"] == 1, info["env"]
    assert info["on_gpu"] == info["records"] and info["gpu_fallback_cpu"] == 0
    check(regs, n, want_regs, want_n)


@pytest.mark.gpu
def test_midstream_device_failure_recovers_on_cpu(exe, tmp_path):
    """the third wait fails as a watchdog expiry does (fpgaHangError path,
    FPGAPipeline.cpp:526-551): the records in flight are recomputed by the CPU
    stage, the worker retires and switches accx dispatch off, every output
    still equals the golden regions"""
    d = str(tmp_path)
    b, want_regs, want_n = write_inputs(d, "c1_default")
    info, regs, n = run(exe, d, "gpu_hang", 50, 2)
    assert info["on_gpu"] >= 1 and info["gpu_fallback_cpu"] >= 1
    assert info["accx_on_at_end"] == 0
    assert info["outputs"] == info["records"] and info["bad_ownership"] == 0
    check(regs, n, want_regs, want_n)


@pytest.mark.gpu
def test_malformed_record_takes_the_error_path(exe, tmp_path):
    """a chain outside its contig (bwa asserts, bwamem.c:669) in record 1: the
    stage reports it, emits the record with that chain skipped, never hands
    it to the CPU stage, and keeps the device in service"""
    d = str(tmp_path)
    b, want_regs, want_n = write_inputs(d, "c1_default")
    per = 50
    info, regs, n = run(exe, d, "gpu_badrid", per, 2, rc=7)  # the driver exits non-zero
    assert info["failed"] == 1 and info["gpu_fallback_cpu"] == 0
    assert info["on_gpu"] == info["records"]
    bad = info["bad_rid_read"]
    assert bad >= per
    off = np.concatenate([[0], np.cumsum(want_n)])
    got_off = np.concatenate([[0], np.cumsum(n)])
    keep = [r for r in range(b.n_reads) if r != bad]
    assert np.array_equal(n[keep], want_n[keep])
    for r in keep[::7] + keep[-3:]:
        assert G.region_mismatch(regs[got_off[r]:got_off[r + 1]], want_regs[off[r]:off[r + 1]]) is None


@pytest.mark.gpu
def test_record_with_overlong_read_falls_back_to_cpu(exe, tmp_path):
    """a read longer than BWAGPU_MAX_READ_LEN makes its record unsupported on
    the device (E_UNSUPPORTED before anything is enqueued): that record goes to
    the CPU stage (FPGAPipeline.cpp's per-record fallback), the others stay on
    the GPU, and every output equals the CPU stage's on the same input"""
    d_cpu, d_gpu = str(tmp_path / "cpu"), str(tmp_path / "gpu")
    os.makedirs(d_cpu)
    os.makedirs(d_gpu)
    per = 50
    for d in (d_cpu, d_gpu):
        b, _, _ = write_inputs(d, "c1_default")
        r = per + 3  # a read of record 1
        seq_off = b.seq_off.copy()
        ext = np.full(abi.MAX_READ_LEN + 10 - int(seq_off[r + 1] - seq_off[r]), 2, np.uint8)
        seq = np.concatenate([b.seq[:seq_off[r + 1]], ext, b.seq[seq_off[r + 1]:]])
        seq_off[r + 1:] += len(ext)
        seq_off.astype(np.int64).tofile(os.path.join(d, "seq_off.bin"))
        seq.astype(np.uint8).tofile(os.path.join(d, "seq.bin"))
    want_info, want_regs, want_n = run(exe, d_cpu, "cpu", per, 2)
    info, regs, n = run(exe, d_gpu, "gpu_only", per, 2)
    assert info["gpu_fallback_cpu"] == 1 and info["on_gpu"] >= info["records"] - 1, info
    assert info["outputs"] == info["records"] and info["bad_ownership"] == 0
    check(regs, n, want_regs, want_n)
