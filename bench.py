#!/usr/bin/env python3
"""Benchmark of the MI355X seed-extension stage (bwa-flow's ChainsToRegions,
src/Pipeline.cpp:503-544, as replaced by the GPU back end).

Workload (BASELINE.json configs[1], "C2"; --workload c2_stream, the default):
a STREAM of distinct ChainsRecords of 2x150 bp pairs on a chr21-sized
synthetic genome (46.7 Mb, three contigs, interspersed/tandem repeats, N runs;
chr21 itself is not available offline).  Global batch g holds 33,334 pairs
(66,668 reads, 10.0 Mbases: Pipeline.cpp:123,146) drawn by
bwa-flow_amd/tools/synth.cpp with seed STREAM_SEED + g; its chains are made by
the device's own SeqsToChains (bwagpu_seqs2chains, bit-exact with the
reference's mem_chain -> mem_chain_flt -> mem_flt_chained_seeds) against the
genome's bwa index (bench_data/e2e, built once per box by the reference's
bwa_idx_build).  The reference then checks the workload before any timing:
its own SeqsToChains must give the same chains, and its own mem_chain2aln
gives every batch's expected regions (oracle/_ref/libbwaref.so on the host
cores: also the CPU baseline).  One step = one batch through the stage (chain
windows, seed order, containment tests, left/right ksw_extend2 with band
retries, seedcov, regions); step i runs stream batch i mod D (D = min(steps,
--stream-batches), default 30 = 1M pairs) with every batch resident in HBM
before timing (far more than the 256 MB MALL holds), and after the timed
region EVERY step's output is checked bit for bit against the reference's.

Side figures: "two_batch_fixture" (round 5's headline: the two
reference-seeded batches of tests/golden/c2_refseed.npz cycled over the same
steps), "hw_queues_4" (that figure again in a child process with HIP's default
GPU_MAX_HW_QUEUES = 4), the PCIe-inclusive host-buffer path, the drop-in
C++ stage end to end, CIGARs, seeding, chaining, the GRCh38-shaped regime legs
and the whole bwa-mem pipeline against `bwa mem`.  --workload c2_refseed keeps
the two fixture batches as the headline; --workload synth round 1's generator
(exact-match chains along the true origin: lighter than the reference's).

Multi-GPU: one process per GPU (torchrun); the packed reference is broadcast
from rank 0 over RCCL/xGMI once; rank r takes global batches r, r + N, r + 2N,
... of the stream (bwa-flow's pull-scatter of read batches to workers,
src/mpi/MPIChannel.cpp:140-200): disjoint shards, no data-path collective,
weak scaling (D batches per rank).

The CPU baseline (rank 0, N=1) is the reference's own mem_chain2aln compiled
from /root/reference (oracle/_ref/libbwaref.so, "kind": "reference") — or our
C restatement ("port") when that library is absent — over the same batches,
using the host cores this job may use.
"""
from __future__ import annotations

import argparse
import ctypes
import glob
import hashlib
import json
import math
import os
import sys
import time

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(REPO, "bwa-flow_amd", "python"))
# Hardware queues per process (read once, at HIP's start): every stream HIP
# makes lands on one of GPU_MAX_HW_QUEUES queues (default 4), and streams that
# share a queue run in submission order.  The stage runs each batch on its
# caller's stream plus a selection side stream, and this job
# makes new caller streams leg after leg: with 4 queues the later legs' streams
# shared queues (the mixed C5 leg 6.8 against 4.1 ms per batch); with 16 none
# did.  INTEGRATION.md §2 gives the same setting for bwa-flow with --use_gpu.
# Every leg also takes its caller streams through caller_streams(), which
# keeps only streams that run concurrently with the others.
# The hw_queues_4 side figure runs this file again as a child process with
# BWAGPU_BENCH_KEEP_HWQ=1 and HIP's default of 4 queues.
if int(os.environ.get("GPU_MAX_HW_QUEUES", "4") or 4) < 16 and os.environ.get("BWAGPU_BENCH_KEEP_HWQ") != "1":
    os.environ["GPU_MAX_HW_QUEUES"] = "16"

import numpy as np  # noqa: E402
import torch  # noqa: E402  (imported before the engine: one HIP runtime)
import torch.distributed as dist  # noqa: E402

from bwagpu import abi  # noqa: E402
from bwagpu.engine import Batch, Engine, compact  # noqa: E402
from bwagpu import workload  # noqa: E402
from bwagpu.synth import SynthRef, synth_batch  # noqa: E402

METRIC = "million reads/sec (2×150 bp PE) end-to-end align; SW-extend GCUPS at 1/2/4/8 MI355X"
HBM_PEAK_GBS = 8000.0            # MI355X_MICROARCH.md chip table (spec)
# int32 VALU peak: 256 CU x 4 SIMD32 x 32 lanes x 2.4 GHz (a wave64 instruction
# issues over 2 cycles, MI355X_MICROARCH.md "CU") = 78.6 T lane-ops/s
VALU_PEAK_TOPS = 256 * 4 * 32 * 2.4e9 / 1e12
# measured issue: 2.64 SIMD cycles per independent VALU wave-instruction at 8
# waves/SIMD (profiles/r01e_issue_costs.json) -> 2/2.64 of the nominal peak
VALU_ISSUE_PEAK_TOPS = VALU_PEAK_TOPS * 2.0 / 2.642
# packed 16-bit peak: a v_pk_* lane-op does two 16-bit ops (157.3 T); the
# extension kernel computes in packed halves, so this is its roofline peak
PK16_PEAK_TOPS = 2 * VALU_PEAK_TOPS
# algorithmic integer ops per evaluated cell: the reference's inner loop
# (ksw.c:430-447) compiles (gcc -O2, x86-64; oracle/_ref/obj/ksw.o,
# ksw_extend2+0x340..0x3ad) to 34 instructions per cell: 20 integer ALU ops
# (test/add/sub/cmp/cmov), 5 memory, 5 moves, 4 loop/branch.  In max/select
# form (one v_max_i32 per cmp+cmov max) those 20 ALU ops are 17: M select 3,
# H max 2, row max + argmax 3, E 4, F 4, profile lookup 1.
OPS_PER_CELL = 17
# the first-bin extension launch of every round (set in run_stage from the options)
# the phased pair (left + right side launches; "spec_sidep_kernel<16, 10, true>"
# with BWAGPU_EXT_PRODUCER=1), "spec_ext4_kernel<16, 10, true>"
# with BWAGPU_EXT_PHASED=0, "spec_ext2_kernel<5>" with --ext-form 1 (engine.ext_kernel)
DOMINANT_KERNEL = "spec_side4_kernel<16, 10, true>"


def caller_streams(dev, n: int, tries: int = 16) -> list:
    """n torch streams that run concurrently with each other
    (bwagpu_streams_concurrent: none shares a hardware queue with another);
    a stream that shares one is left unused and another taken"""
    lib = abi.load()
    out = []
    for _ in range(tries):
        if len(out) == n:
            break
        s = torch.cuda.Stream(device=dev)
        if all(lib.bwagpu_streams_concurrent(ctypes.c_void_p(s.cuda_stream), ctypes.c_void_p(t.cuda_stream)) == 1 and
               lib.bwagpu_streams_concurrent(ctypes.c_void_p(t.cuda_stream), ctypes.c_void_p(s.cuda_stream)) == 1
               for t in out):
            out.append(s)
    while len(out) < n:  # no free queue left: share one
        out.append(torch.cuda.Stream(device=dev))
    return out


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def split_batches(b: Batch, min_bases: int) -> list[Batch]:
    """cut reads into ChainsRecords of >= min_bases bases and an even read count (getKseqBatch)"""
    so = b.seq_off
    out, r0 = [], 0
    while r0 < b.n_reads:
        r1 = int(np.searchsorted(so, so[r0] + min_bases, side="left"))
        r1 = max(r1, r0 + 2)
        r1 += (r1 - r0) & 1
        r1 = min(r1, b.n_reads)
        out.append(sub_range(b, r0, r1))
        r0 = r1
    return out


def sub_range(b: Batch, r0: int, r1: int) -> Batch:
    c0, c1 = int(b.read_chain_off[r0]), int(b.read_chain_off[r1])
    s0, s1 = int(b.chain_seed_off[c0]), int(b.chain_seed_off[c1])
    q0, q1 = int(b.seq_off[r0]), int(b.seq_off[r1])
    return Batch(b.seq_off[r0:r1 + 1] - q0, b.seq[q0:q1], b.read_chain_off[r0:r1 + 1] - c0,
                 b.chain_seed_off[c0:c1 + 1] - s0, b.chain_rid[c0:c1], b.chain_frac_rep[c0:c1], b.seeds[s0:s1])


FIELDS = ("seq_off", "seq", "read_chain_off", "chain_seed_off", "chain_rid", "chain_frac_rep", "seeds")


class DevBatch:
    """one batch resident in HBM + its output buffers (one set per step that
    runs it, so every timed step's output can be checked afterwards)"""

    def __init__(self, b: Batch, dev, check=None):
        self.b, self.dev, self.check = b, dev, check
        self.t = {k: torch.from_numpy(np.ascontiguousarray(getattr(b, k)).view(np.uint8).copy()).to(dev)
                  for k in FIELDS}
        self.outs = []
        self.stats = torch.zeros(4, dtype=torch.int64, device=dev)
        self.c = abi.BatchC()
        self.c.n_reads, self.c.n_chains, self.c.n_seeds = b.n_reads, b.n_chains, b.n_seeds
        self.c.seq_bytes = int(b.seq_off[-1])
        for k in FIELDS:
            setattr(self.c, k, self.t[k].data_ptr())
        self.in_bytes = sum(int(getattr(b, k).nbytes) for k in FIELDS)
        self.add_out()

    def add_out(self) -> int:
        self.outs.append((torch.zeros(max(self.b.n_seeds, 1) * 88, dtype=torch.uint8, device=self.dev),
                          torch.zeros(max(self.b.n_reads, 1), dtype=torch.int32, device=self.dev)))
        return len(self.outs) - 1

    def run(self, eng: Engine, stream, k: int = 0, stats: bool = True):
        out, n = self.outs[k]
        eng.chain2aln_device(self.c, out.data_ptr(), n.data_ptr(), self.stats.data_ptr() if stats else None, stream)

    def results(self, k: int = 0):
        out, n = self.outs[k]
        regs = out.cpu().numpy().view(abi.ALNREG_DTYPE)[:self.b.n_seeds]
        return regs, n.cpu().numpy()[:self.b.n_reads]


def cpu_model() -> str:
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def cpu_baseline(opt, ref, batches, budget_s, gpu_out, checks=None):
    """reference mem_chain2aln on the host over a bounded sample of the same
    batches; bit-exact parity of the GPU's output of each sampled batch
    against it (and of the CPU output against the fixture's digest)"""
    sys.path.insert(0, os.path.join(REPO, "oracle"))
    import oracle
    kind = "reference" if oracle.ref_lib() is not None else "port"
    which = "ref" if kind == "reference" else "oracle"
    cores = host_threads()
    R = oracle.Ref(ref.l_pac, ref.ann_offset, ref.ann_len, ref.pac)
    # batches in turn (again from the first when the distinct ones run out)
    # until ~budget_s CPU-seconds; every distinct batch's output is compared
    reads, t_used, k, parity, fix_ok = 0, 0.0, 0, True, True
    while True:
        j = k % len(batches)
        b = batches[j]
        t0 = time.perf_counter()
        regs, n, _ = oracle.chain2aln(which, opt, R, b, n_threads=cores)
        t_used += time.perf_counter() - t0
        if k < len(batches):
            g_regs, g_n = gpu_out[j]
            parity &= bool(np.array_equal(g_n, n) and
                           np.array_equal(compact(b, g_regs, g_n).view(np.uint8), compact(b, regs, n).view(np.uint8)))
            if checks is not None:
                fix_ok &= checks[j].check(regs, n)
        reads += b.n_reads
        k += 1
        if t_used * cores >= budget_s or k >= 200:
            break
    # the same on ONE host thread (SURVEY.md §8d asks for both), first batch only
    t0 = time.perf_counter()
    oracle.chain2aln(which, opt, R, batches[0], n_threads=1)
    t1c = time.perf_counter() - t0
    r = dict(value=reads / t_used / 1e6, unit="Mreads/s", cores=cores, cpu=cpu_model(), kind=kind,
             host_cpus=os.cpu_count(), value_1core=round(batches[0].n_reads / t1c / 1e6, 5),
             sample_1core=f"batch 0 ({batches[0].n_reads} reads) on one thread, {t1c:.2f} s",
             sample=f"{k} batch runs ({min(k, len(batches))} distinct), {reads} reads of the same workload, {t_used:.2f} s wall on {cores} threads "
                    f"({'oracle/_ref/libbwaref.so: the reference mem_chain2aln' if kind == 'reference' else 'oracle/liboracle.so'})",
             parity_gpu_vs_cpu=parity)
    if checks is not None:
        r["cpu_matches_fixture"] = fix_ok
    return r


reg2aln_jobs = workload.reg2aln_jobs


def cigar_stage(eng: Engine, b: Batch, regs, n, reps: int = 3):
    """§8f rank 2: batched mem_reg2aln on the regions of one batch
    (host buffers in and out; kernel time from HIP events)"""
    jobs = reg2aln_jobs(b, regs, n)
    out = eng.reg2aln_batch(jobs, b.seq, 64, 512)  # warm-up
    kms, walls = [], []
    for _ in range(reps):
        t0 = time.perf_counter()
        out = eng.reg2aln_batch(jobs, b.seq, 64, 512)
        walls.append(time.perf_counter() - t0)
        kms.append(eng.last_stats()["kernel_ms"])
    st = eng.last_stats()
    km = float(np.median(kms))
    return dict(jobs=len(jobs), kernel_ms=round(km, 4), jobs_per_s=round(len(jobs) / (km * 1e-3)),
                host_buffer_ms=round(1e3 * float(np.median(walls)), 3), dp_cells=int(st["cells"]),
                gen_cigar2_calls=int(st["ext_calls"])), jobs, out


def cigar_cpu_baseline(opt, ref, b: Batch, jobs, gpu_out) -> dict:
    """the reference mem_reg2aln (oracle/_ref) on one host thread over the same
    jobs, and bit-exact parity of the GPU records, CIGARs and MD strings"""
    sys.path.insert(0, os.path.join(REPO, "oracle"))
    sys.path.insert(0, os.path.join(REPO, "tests"))
    import oracle
    import golden_io as G
    lib = oracle.ref_lib()
    kind = "reference" if lib is not None and hasattr(lib, "ref_reg2aln_batch") else "port"
    R = oracle.Ref(ref.l_pac, ref.ann_offset, ref.ann_len, ref.pac)
    m = min(len(jobs), 200_000)
    t0 = time.perf_counter()
    want = oracle.reg2aln("ref" if kind == "reference" else "oracle", opt, R, jobs[:m], b.seq, 64, 512)
    dt = time.perf_counter() - t0
    o, c, md = gpu_out
    # the reference's mem_reg2aln fills the record, CIGAR and MD; score and w are
    # the last bwa_gen_cigar2 call's, checked against the golden
    # vectors in tests/test_gpu_cigar.py
    fields = ("pos", "rid", "is_rev", "n_cigar", "NM", "md_len", "status") if kind == "reference" else \
        ("pos", "rid", "is_rev", "n_cigar", "NM", "md_len", "score", "w", "status")
    why = G.aln_mismatch(jobs[:m], o[:m], c[:m], md[:m], *G.aln_expected_from(*want), fields=fields)
    r = dict(value=round(m / dt), unit="jobs/s", cores=1, kind=kind, sample=f"{m} jobs (batch 0)",
             parity_vs_cpu=why is None)
    if why is not None:
        r["mismatch"] = why[:600]
    return r


class HostRef:
    """the host view of the shared reference a rank needs to generate its reads"""

    def __init__(self, l_pac, pac, ann_offset, ann_len):
        self.l_pac, self.pac, self.ann_offset, self.ann_len = l_pac, pac, ann_offset, ann_len


def shared_reference(ref_len: int, contigs: int, rank: int, world: int, dev):
    """rank 0 generates the packed reference; one start-up broadcast (RCCL over
    xGMI on GPUs, gloo in the CPU tests) gives every rank the same pac and
    contig table.  Returns (HostRef, pac tensor on dev)."""
    return broadcast_reference(SynthRef(42, ref_len, contigs) if rank == 0 else None, rank, world, dev)


def broadcast_reference(src, rank: int, world: int, dev):
    """the one start-up collective: rank 0's packed reference and contig table
    (any contig count: the sizes go first in a meta tensor) to every rank, over
    RCCL/xGMI on GPUs (gloo in the CPU tests).  src: an object with l_pac, pac,
    ann_offset, ann_len on rank 0 (ignored elsewhere).  -> (HostRef, pac tensor on dev)"""
    meta = torch.tensor([src.l_pac, len(src.ann_len)] if rank == 0 else [0, 0], dtype=torch.int64, device=dev)
    if world > 1:
        dist.broadcast(meta, src=0)
    L, n_ctg = int(meta[0].item()), int(meta[1].item())
    if rank == 0:
        pac_t = torch.from_numpy(np.ascontiguousarray(src.pac)).to(dev)
        ann = torch.from_numpy(np.concatenate([np.asarray(src.ann_offset, np.int64),
                                               np.asarray(src.ann_len, np.int64)])).to(dev)
    else:
        pac_t = torch.empty(L // 4 + 1, dtype=torch.uint8, device=dev)
        ann = torch.empty(2 * n_ctg, dtype=torch.int64, device=dev)
    if world > 1:
        dist.broadcast(pac_t, src=0)
        dist.broadcast(ann, src=0)
        if pac_t.is_cuda:
            torch.cuda.synchronize()
    if rank == 0:
        return HostRef(L, src.pac, np.asarray(src.ann_offset, np.int64), np.asarray(src.ann_len, np.int32)), pac_t
    a = ann.cpu().numpy()
    return HostRef(L, pac_t.cpu().numpy(), a[:n_ctg].copy(), a[n_ctg:].astype(np.int32)), pac_t


def rank_reads(ref, rank: int, pairs: int, read_len: int):
    """this rank's shard: independent reads (seed 1000 + rank), weak scaling"""
    return synth_batch(ref, 1000 + rank, pairs, read_len)


def job_totals(elapsed: float, reads: int, world: int, dev):
    """whole-job numbers: the slowest rank's time, every rank's reads"""
    t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
    tot = torch.tensor([float(reads)], dtype=torch.float64, device=dev)
    if world > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dist.all_reduce(tot, op=dist.ReduceOp.SUM)
    return float(t.item()), float(tot.item())


def host_path_rate(eng: Engine, batches, n: int, checks=None, depth: int = 4) -> dict:
    """PCIe-inclusive rate: n batches (cycling over the distinct ones, as the
    timed steps do) from HOST buffers through the bwagpu_chain2aln_submit/wait
    pair on `depth` slots (batch i + depth - 1 is packed and submitted before
    batch i is waited for: with 2 slots only one batch runs on the device while
    the host packs the next, and the rate is one batch's latency), the regions
    written densely to pinned memory and read in place.  Reported beside the
    resident-input `value`, never as it."""
    def run(bs):
        for i in range(min(depth - 1, len(bs))):
            eng.submit(i, bs[i])
        got = [None] * depth
        for i in range(len(bs)):
            if i + depth - 1 < len(bs):
                eng.submit((i + depth - 1) % depth, bs[i + depth - 1])
            # the results as views onto the slot's pinned buffers (valid until its next submit)
            got[i % depth] = eng.wait_dense(i % depth, bs[i])
        return got

    for k in range(depth):  # warm every slot's buffers with every distinct batch (they only grow)
        for b in batches:
            eng.submit(k, b)
            eng.wait_dense(k, b)
    run([batches[i % len(batches)] for i in range(4 * depth)])  # and the pipelined loop itself, untimed
    bs = [batches[i % len(batches)] for i in range(n)]
    t0 = time.perf_counter()
    got = run(bs)
    dt = time.perf_counter() - t0
    reads = sum(b.n_reads for b in bs)
    parity = None
    if checks:  # the last batch of each slot against the reference (outside the timing)
        parity = True
        for i in range(max(len(bs) - depth, 0), len(bs)):
            k = i % len(batches)
            regs, cnt = got[i % depth]
            parity &= bool(checks[k].check_compact(regs, cnt))
    return {"value": round(reads / dt / 1e6, 4), "unit": "Mreads/s", "batches": len(bs),
            "distinct_batches": len(batches), "ms_per_batch": round(dt * 1e3 / len(bs), 3),
            "parity_last_batches": parity, "slots": depth,
            "path": f"host buffers -> bwagpu_chain2aln_submit/wait + results_dense (H2D + kernels + the "
                    f"regions written densely to pinned memory and read in place, {depth} slots)"}


SEED_BWT = os.path.join(REPO, "bench_data", "c2_bwt.npz")


def seeding_stage(eng: Engine, b: Batch, reps: int = 5) -> dict | None:
    """Seeding's interval collection on the device:
    bwagpu_collect_intv over the batch's reads against the chr21-sized golden
    genome's FM-index (bench_data/c2_bwt.npz: hdr + occurrence words, built by
    the reference's bwa_idx_build: `oracle/_ref/gen_seed <dir> 1 0 150
    46709983 0`; the leg is skipped when the file is absent).  Host API wall, H2D of the reads and
    D2H of the packed intervals included."""
    if os.path.exists(SEED_BWT):
        z = np.load(SEED_BWT)
        hdr, words = z["hdr"], z["words"]
    elif os.path.exists(os.path.join(E2E_DIR, "ref.fa.bwt")) and os.path.exists(os.path.join(E2E_DIR, "ref.fa.sa")):
        hdr, words, _, _ = workload.load_bwa_index(os.path.join(E2E_DIR, "ref.fa"))  # the same genome's index
    else:
        return None
    eng.set_bwt(hdr, words)
    n, iv = eng.collect_intv(b.seq_off, b.seq)
    # the caller's interval buffer, reused per batch as a pipeline stage would
    buf = np.zeros(int(n.sum()) * 5 // 4 + 1024, iv.dtype)
    seq_off = np.ascontiguousarray(b.seq_off, np.int64)
    seq = np.ascontiguousarray(b.seq, np.uint8)
    eng.collect_intv(seq_off, seq, out=buf)
    t0 = time.perf_counter()
    for _ in range(reps):
        n, iv = eng.collect_intv(seq_off, seq, out=buf)
    ms = (time.perf_counter() - t0) * 1e3 / reps
    iv = iv.copy()
    return {"reads": int(b.n_reads), "ms_per_batch": round(ms, 3), "value": round(b.n_reads / ms / 1e3, 4),
            "unit": "Mreads/s", "intervals": int(n.sum()),
            "index": "chr21-sized golden genome, 93.4 M BWT positions (47 MB occurrence array)",
            "path": "bwagpu_collect_intv: mem_collect_intv (bwamem.c:120-167) per read, two tiers",
            "_check": (hdr, words, n, iv)}


def chaining_stage(eng: Engine, rb, reps: int = 5) -> dict | None:
    """bwa-flow's SeqsToChains entirely on the device (bwagpu_seqs2chains:
    interval search, SA lookups, the kbtree chaining, mem_chain_flt,
    mem_flt_chained_seeds) and fused with ChainsToRegions
    (bwagpu_seqs2regions), over the C2 batch's reads against the bwa index of
    the chr21-sized genome (bench_data/e2e, which the end_to_end_align leg's
    harness builds with the reference's bwa_idx_build).  Parity: the chains must
    be the reference's ChainsRecord byte for byte (the fixture was seeded and
    chained by the reference's mem_chain -> mem_chain_flt ->
    mem_flt_chained_seeds) and the regions the reference's mem_chain2aln
    output.  Host API wall (reads H2D, results D2H)."""
    pre = os.path.join(E2E_DIR, "ref.fa")
    if not (os.path.exists(pre + ".bwt") and os.path.exists(pre + ".sa")):
        return None
    hdr, words, sa, sa_intv = workload.load_bwa_index(pre)
    eng.set_bwt(hdr, words, sa, sa_intv)
    b = rb.batch
    # timed: the C ABI call (its outputs stay in the context's pinned buffers); the
    # checked copy is made after the timing
    seq_off = np.ascontiguousarray(b.seq_off, np.int64)
    seq = np.ascontiguousarray(b.seq, np.uint8)
    eng.seqs2chains(seq_off, seq, copy=False)
    t0 = time.perf_counter()
    for _ in range(reps):
        eng.seqs2chains(seq_off, seq, copy=False)
    ms_c = (time.perf_counter() - t0) * 1e3 / reps
    rco, ch, cso, sd = eng.seqs2chains(seq_off, seq)
    got = Batch(b.seq_off, b.seq, rco, cso, ch["rid"].copy(), ch["frac_rep"].copy(), sd)
    chains_ok = workload.batch_digest(got) == workload.batch_digest(b)
    eng.seqs2regions(seq_off, seq, copy=False)
    t0 = time.perf_counter()
    for _ in range(reps):
        eng.seqs2regions(seq_off, seq, copy=False)
    ms_r = (time.perf_counter() - t0) * 1e3 / reps
    n, regs = eng.seqs2regions(seq_off, seq)
    pipe = None
    try:  # a side figure: the stage's throughput with two workers, as SeqsToChains runs (several threads)
        pipe = two_context_rate(eng, hdr, words, sa, sa_intv, seq_off, seq, reps)
    except Exception as e:
        pipe = {"error": repr(e)}
    return {"reads": int(b.n_reads), "seqs2chains_ms_per_batch": round(ms_c, 3),
            "seqs2chains_Mreads_per_s": round(b.n_reads / ms_c / 1e3, 4), "chains": int(len(ch)), "seeds": int(len(sd)),
            "chains_identical_to_reference": bool(chains_ok),
            "seqs2regions_ms_per_batch": round(ms_r, 3), "value": round(b.n_reads / ms_r / 1e3, 4),
            "unit": "Mreads/s", "regions_identical_to_reference": bool(rb.check_compact(regs, n)),
            "path": "bwagpu_seqs2regions: reads -> mem_collect_intv -> mem_chain -> mem_chain_flt -> "
                    "mem_flt_chained_seeds -> mem_chain2aln, all on the device (host API wall)",
            "two_workers": pipe}


def two_context_rate(eng: Engine, hdr, words, sa, sa_intv, seq_off, seq, reps: int) -> dict:
    """seqs2chains / seqs2regions throughput with two stage workers: two contexts
    (each with its own copy of the FM-index) called from two host threads, as
    bwa-flow runs SeqsToChains on several worker threads (src/Pipeline.cpp:
    the stage's MapStage workers); one batch's latency is the figure above.
    ms per batch = wall / batches over both workers."""
    import threading
    e2 = eng.clone()
    e2.set_bwt(hdr, words, sa, sa_intv)
    engs = [eng, e2]
    out = {}
    for fn in ("seqs2chains", "seqs2regions"):
        for e in engs:
            getattr(e, fn)(seq_off, seq, copy=False)
        bar = threading.Barrier(len(engs) + 1)

        def work(e):
            bar.wait()
            for _ in range(reps):
                getattr(e, fn)(seq_off, seq, copy=False)

        th = [threading.Thread(target=work, args=(e,)) for e in engs]
        for t in th:
            t.start()
        bar.wait()
        t0 = time.perf_counter()
        for t in th:
            t.join()
        out[f"{fn}_ms_per_batch"] = round((time.perf_counter() - t0) * 1e3 / (reps * len(engs)), 3)
    e2.close()
    out["workers"] = len(engs)
    return out


def host_threads() -> int:
    """the host threads a CPU leg may use: this job's CPU affinity, capped by
    OMP_NUM_THREADS (the box's CPU share for one GPU: 16) and 64"""
    try:
        cores = len(os.sched_getaffinity(0))
    except Exception:
        cores = os.cpu_count() or 1
    return max(1, min(cores, int(os.environ.get("OMP_NUM_THREADS", cores)), 64))


def ref_seeding_baseline(b: Batch, mode: int, reads_1core: int = 3000) -> dict | None:
    """the REFERENCE's own seeding on the host (oracle/_ref/libbwaref.so
    ref_seeding_bench): mode 0 = the interval search (mem_collect_intv's
    control flow around bwa's bwt_smem1 / bwt_seed_strategy1 /
    ks_introsort_mem_intv), mode 1 = SeqsToChains (mem_chain -> mem_chain_flt
    -> mem_flt_chained_seeds); the whole batch on every allowed core, and a
    sample on one; against the bwa index of bench_data/e2e"""
    import ctypes as C
    so_path = os.path.join(REPO, "oracle", "_ref", "libbwaref.so")
    pre = os.path.join(E2E_DIR, "ref.fa")
    if not os.path.exists(so_path) or not os.path.exists(pre + ".bwt"):
        return None
    lib = C.CDLL(so_path)
    lib.ref_seeding_bench.restype = C.c_double
    lib.ref_seeding_bench.argtypes = [C.c_char_p, C.c_int, C.c_int32, C.c_void_p, C.c_void_p, C.c_int, C.c_int,
                                      C.POINTER(C.c_int64)]
    cores = host_threads()
    so = np.ascontiguousarray(b.seq_off, np.int64)
    sq = np.ascontiguousarray(b.seq, np.uint8)
    cnt = C.c_int64()
    if lib.ref_seeding_bench(pre.encode(), mode, 0, so.ctypes.data, sq.ctypes.data, 1, 1, C.byref(cnt)) < 0:
        return None  # (index load, outside the timing)
    k = min(reads_1core, b.n_reads)
    t1 = lib.ref_seeding_bench(pre.encode(), mode, k, so.ctypes.data, sq.ctypes.data, 1, 1, C.byref(cnt))
    tn = lib.ref_seeding_bench(pre.encode(), mode, b.n_reads, so.ctypes.data, sq.ctypes.data, cores, 1, C.byref(cnt))
    return {"value": round(b.n_reads / tn / 1e6, 5), "unit": "Mreads/s", "cores": cores, "kind": "reference",
            "value_1core": round(k / t1 / 1e6, 5), "sample_1core": f"first {k} reads on one thread, {t1:.2f} s",
            "sample": f"the whole batch ({b.n_reads} reads) on {cores} threads, {tn:.2f} s wall",
            "count": int(cnt.value), "count_is": "intervals" if mode == 0 else "chains",
            "code": ("the reference's bwt_smem1 / bwt_seed_strategy1 / ks_introsort_mem_intv in mem_collect_intv's "
                     "control flow") if mode == 0 else
                    "the reference's mem_chain -> mem_chain_flt -> mem_flt_chained_seeds (bwa-flow SeqsToChains)"}


def seeding_cpu_baseline(b: Batch, hdr, words, n, iv, reads: int = 1500) -> dict:
    """the oracle restatement (oracle/seed.c), one thread, on the first reads;
    also the parity check of the device's intervals for them"""
    sys.path.insert(0, os.path.join(REPO, "oracle"))
    import oracle
    so = b.seq_off[:reads + 1]
    t0 = time.perf_counter()
    wn, want = oracle.collect_intv(hdr, words, np.array([19, 10, 20], np.int32), 1.5, so, b.seq[:so[-1]])
    dt = time.perf_counter() - t0
    got = np.column_stack([iv["x"], iv["info"]]).astype(np.uint64)[:int(wn.sum())]
    return {"value": round(reads / dt / 1e6, 5), "unit": "Mreads/s", "cores": 1, "kind": "port",
            "sample": f"first {reads} reads of the batch (oracle/seed.c)",
            "parity_gpu_vs_cpu": bool(np.array_equal(n[:reads], wn) and np.array_equal(got, want))}


def end_to_end_stage(opt, ref, batches, checks, reps: int = 20,
                     workers: int = int(os.environ.get("BWAGPU_E2E_WORKERS", "3")), chain_mode: int = 1,
                     sink_workers: int = 4) -> dict:
    """The drop-in stage end to end (bwa-flow_amd/lib/libgpustage.so,
    host/stage_bench.cpp): host ChainsRecords (malloc'd chains/seeds per read,
    as SeqsToChains hands them over) through a kflow pipeline whose stage 4 is
    ChainsToRegionsGPU alone — pack, pinned staging + H2D, kernels, the regions
    written densely to pinned memory, malloc'd mem_alnreg_v — with its slot
    ping-pong; a second kflow stage of sink_workers threads plays RegionsToSam
    (frees the regions, and the chains the stage forwards: chain_mode 0, the
    FPGA stage's ownership; 1: the stage frees them).  Reported beside the resident-input `value`, with the
    stage's per-phase totals (FPGAPipeline.cpp:557-578 prints the same split),
    per-record device times and bit-exact parity of the last rep against the
    reference's regions."""
    import ctypes as C
    lib = C.CDLL(os.path.join(abi.LIB_DIR, "libgpustage.so"))
    lib.gpustage_run.restype = C.c_int
    lib.gpustage_run.argtypes = [C.POINTER(abi.Opt), C.POINTER(abi.Bns), C.c_void_p, C.c_int,
                                 C.POINTER(abi.BatchC), C.c_int, C.c_int, C.c_int, C.c_int, C.c_int, C.c_void_p,
                                 C.c_void_p, C.c_void_p]
    o = abi.opt_from_dict(opt)
    bns = abi.Bns()
    bns.l_pac, bns.n_seqs = ref.l_pac, len(ref.ann_len)
    ann_off = np.ascontiguousarray(ref.ann_offset, np.int64)
    ann_len = np.ascontiguousarray(ref.ann_len, np.int32)
    bns.ann_offset = ann_off.ctypes.data_as(C.c_void_p)
    bns.ann_len = ann_len.ctypes.data_as(C.c_void_p)
    pac = np.ascontiguousarray(ref.pac, np.uint8)
    arr = (abi.BatchC * len(batches))(*[b.to_c() for b in batches])
    outs_n = [np.zeros(max(b.n_reads, 1), np.int32) for b in batches]
    outs_r = [np.zeros(max(b.n_seeds, 1), abi.ALNREG_DTYPE) for b in batches]
    pn = (C.c_void_p * len(batches))(*[x.ctypes.data for x in outs_n])
    pr = (C.c_void_p * len(batches))(*[x.ctypes.data for x in outs_r])
    times = np.zeros(12, np.float64)
    rc = lib.gpustage_run(C.byref(o), C.byref(bns), pac.ctypes.data_as(C.c_void_p), len(batches), arr, reps, 1,
                          workers, chain_mode, sink_workers, times.ctypes.data_as(C.c_void_p), C.cast(pn, C.c_void_p),
                          C.cast(pr, C.c_void_p))
    if rc != 0:
        return {"error": f"gpustage_run rc={rc}"}
    reads = reps * sum(b.n_reads for b in batches)
    par = None
    if checks:
        par = True
        for b, rb, n, r in zip(batches, checks, outs_n, outs_r):
            par &= rb.check_compact(r, n[:b.n_reads])  # regions concatenated in read order
    nrec = max(int(times[5]), 1)
    ph = {k: round(float(v), 4) for k, v in zip(("pack_s", "submit_s", "wait_s", "post_s"), times[1:5])}
    per = {k: round(float(v) * 1e3 / nrec, 3) for k, v in zip(("pack", "submit", "wait", "post"), times[1:5])}
    per.update(kernels=round(float(times[8]) * 1e3 / nrec, 3), h2d_and_results=round(float(times[9]) * 1e3 / nrec, 3),
               host_cpu_user=round(float(times[10]) * 1e3 / nrec, 3), host_cpu_sys=round(float(times[11]) * 1e3 / nrec, 3))
    own = (f"forwarded to RegionsToSam (the FPGA stage's ownership, FPGAPipeline.cpp:434); the sink stage "
           f"({sink_workers} threads) frees them"
           if chain_mode == 0 else f"freed by the stage's {os.environ.get('BWAGPU_REAPER_THREADS', '4')} reaper threads, "
           "NULL forwarded (the CPU stage's ownership, Pipeline.cpp:526-537)")
    return {"value": round(reads / times[0] / 1e6, 4), "unit": "Mreads/s", "records": int(times[5]),
            "cpu_fallback_records": int(times[6]), "wall_s": round(float(times[0]), 4), "phases": ph,
            "ms_per_record": per, "stage_workers": int(times[7]), "parity_last_rep": par, "chains": own,
            "path": f"host ChainsRecords -> ChainsToRegionsGPU (kflow, {workers} stage workers on the device, "
                    "4 slots each): pack, H2D, kernels, dense results to pinned memory, "
                    "malloc'd mem_alnreg_v (bwa-flow_amd/host/stage_bench.cpp)"}


# roofline.traffic: the PMC summary (tools_dev/pmc_traffic.py over separate
# rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes of bench.py) whose
# source_digest is this tree's (bwagpu.provenance): a summary of other kernel
# sources is never reported


E2E_DIR = os.path.join(REPO, "bench_data", "e2e")  # bwa index of the chr21-sized golden genome (sam_harness builds it once)


def end_to_end_align(pairs: int = 300_000, threads: int | None = None) -> dict | None:
    """The metric's "end-to-end align" (BASELINE.json): 2x150 pairs through the
    whole bwa-mem pipeline on the chr21-sized golden genome, batch by batch
    (10 Mbase ChainsRecords).  Two runs of oracle/_ref/sam_harness, the
    reference's own host code (bwa compiled from /root/reference) around the
    stages:
      * "ref": bwa mem's mem_process_seqs (bwamem.c:1220-1249), all on the CPU —
        the CPU baseline;
      * "gpuchain": the same pipeline with this repository's GPU stages dropped
        in — SeqsToChains + ChainsToRegions fused on the device
        (bwagpu_seqs2regions: interval search, SA lookups, the kbtree chaining,
        mem_chain_flt, mem_flt_chained_seeds, mem_chain2aln), then mate rescue
        and CIGARs (libbwagpu.so / libgpusam.so); sort/dedup, pairing and SAM
        text stay on the reference's host code.
    Both on the same host threads; the SAM outputs must be byte-identical.
    reads/s = reads / the pipeline's wall time (index load and read simulation
    excluded, the same for both)."""
    import hashlib
    import subprocess
    h = os.path.join(REPO, "oracle", "_ref", "sam_harness")
    if not os.access(h, os.X_OK):
        return None
    if threads is None:
        try:
            threads = len(os.sched_getaffinity(0))
        except Exception:
            threads = os.cpu_count() or 1
        threads = max(1, min(threads, 16))
    os.makedirs(E2E_DIR, exist_ok=True)
    out, shas = {}, {}
    tmp = os.environ.get("TMPDIR", "/tmp")
    for mode in ("ref", "gpuchain"):
        sam = os.path.join(tmp, f"bwagpu_e2e_{os.getpid()}_{mode}.sam")
        r = subprocess.run([h, mode, E2E_DIR, sam, "7", str(pairs), "150", "10000000", str(threads), "46709983"],
                           cwd=REPO, capture_output=True, text=True, timeout=900)
        if r.returncode != 0:
            return {"error": f"{mode}: rc={r.returncode} {r.stderr[-400:]}"}
        info = json.loads(r.stderr.strip().splitlines()[-1])
        shas[mode] = hashlib.sha256(open(sam, "rb").read()).hexdigest()
        os.remove(sam)
        out[mode] = info
    ref, gpu = out["ref"], out["gpuchain"]
    v_ref, v_gpu = ref["reads"] / ref["total_s"] / 1e6, gpu["reads"] / gpu["total_s"] / 1e6
    return {"value": round(v_gpu, 4), "unit": "Mreads/s", "reads": gpu["reads"], "threads": threads,
            "bwa_mem_cpu": round(v_ref, 4), "speedup_vs_bwa_mem": round(v_gpu / v_ref, 3),
            "sam_identical": shas["ref"] == shas["gpuchain"],
            "phases_s": {k: gpu[k] for k in ("seed_s", "seed_device_s", "ext_s", "post_s", "sam_s", "flush_s", "pass0_s",
                                             "pass1_s", "pass2_s", "clear_s", "out_s", "feeder_s", "total_s")},
            "bwa_mem_out_s": ref["out_s"],
            "sam_passes": gpu["sam_passes"], "bwa_mem_total_s": ref["total_s"],
            "path": "bwa mem host pipeline (reference code, oracle/_ref/sam_harness) with the GPU stages dropped in: "
                    "reads -> regions on the device (bwagpu_seqs2regions: seeding, chaining, chain2aln), mate rescue "
                    "(ksw_align2) and CIGAR (mem_reg2aln) on the device"}


def load_traffic(workload_tag: str):
    """HBM bytes per launch of the dominant kernel from the newest
    profiles/*_traffic.json of THIS source tree (same source_digest), with
    FETCH_SIZE doubled (MI355X_MICROARCH.md §HBM: gfx950 FETCH_SIZE reads half
    the bytes of a wide coalesced read) -> (bytes, source text, pmc counters) or
    (None, why, None)"""
    from bwagpu.provenance import source_digest
    dig = source_digest()
    best = None
    for f in sorted(glob.glob(os.path.join(REPO, "profiles", "*_traffic.json"))):
        try:
            d = json.load(open(f))
        except Exception:
            continue
        if d.get("source_digest") == dig and d.get("workload") == workload_tag and DOMINANT_KERNEL in d.get("per_launch", {}):
            best = (f, d)
    if best is None:
        return None, f"no PMC summary of this source tree (digest {dig}) under profiles/", None
    f, d = best
    k = d["per_launch"][DOMINANT_KERNEL]
    rel = os.path.relpath(f, REPO)
    return round(2 * k.get("fetch_bytes", 0.0) + k.get("write_bytes", 0.0)), \
        (f"{rel} (source digest {dig}): 2 x FETCH_SIZE + WRITE_SIZE per {DOMINANT_KERNEL} launch "
         f"(raw FETCH {round(k.get('fetch_bytes', 0.0))} B)"), d.get("counters")


def busy_ms(iv) -> float:
    """union of [start, end] intervals (ms): launches that overlap count once"""
    tot, cs, ce = 0.0, None, None
    for a, b in sorted(map(tuple, iv)):
        if ce is None or a > ce:
            if ce is not None:
                tot += ce - cs
            cs, ce = a, b
        else:
            ce = max(ce, b)
    if ce is not None:
        tot += ce - cs
    return tot


def regime_stage(dev, steps: int = 10, n_streams: int = 2, ext_form: int = 0) -> dict:
    """C3 / C5 regime legs (BASELINE.json configs[2] / [4]): the
    GRCh38-shaped genome of tests/golden/c3_grch38.npz (195 contigs, l_pac
    3.1e9, the 0.78 GB pac resident in HBM, far past the 256 MB MALL) with one
    10 Mbase ChainsRecord of 2x150 bp ("c3") and one of mixed 2x100/150/250 bp
    ("c5", which fills the C = 4 extension bin); synthetic chains (no bwa
    index of a 3.1 Gb genome can be built here), the reference's answers as
    digests.  Then "c3_refseed": the C2 fixture's reference-seeded chains (bwa's
    own seeding) translated into that regime (tests/golden/c3_refseed.npz: the
    golden genome twice around the GRCh38-shaped contigs, l_pac 3.19e9).  Each
    batch runs `steps` times over 2 streams, resident inputs; every step's
    output is checked."""
    t0 = time.perf_counter()
    opt, g, sets = workload.load_c3()
    out = {"l_pac": g.l_pac, "contigs": len(g.ann_len), "pac_bytes": int(g.pac.nbytes)}
    streams = caller_streams(dev, n_streams)

    def run_set(eng, name, s):
        d = DevBatch(s.batch, dev)
        for _ in range(steps - 1):
            d.add_out()
        for i in range(2):
            d.run(eng, streams[i % n_streams].cuda_stream, i, stats=False)
        torch.cuda.synchronize()
        d.stats.zero_()
        eng.prof_start(3 * steps)
        ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        t1 = time.perf_counter()
        ev0.record(streams[0])
        for x in streams[1:]:
            x.wait_event(ev0)
        for i in range(steps):
            d.run(eng, streams[i % n_streams].cuda_stream, i)
        t_enq = time.perf_counter() - t1
        for x in streams[1:]:
            e = torch.cuda.Event()
            e.record(x)
            streams[0].wait_event(e)
        ev1.record(streams[0])
        torch.cuda.synchronize()
        el = max(time.perf_counter() - t1, ev0.elapsed_time(ev1) / 1e3)
        ext_ms, ext_n = eng.prof_read()
        ext_busy = busy_ms(eng.prof_intervals(3 * steps))
        eng.prof_start(0)
        st = d.stats.cpu().numpy()
        why = None
        for i in range(steps):
            why = why or s.check(*d.results(i))
        r = {"reads_per_batch": s.batch.n_reads, "bases_per_batch": int(s.batch.seq_off[-1]),
             "ms_per_batch": round(el * 1e3 / steps, 4), "value": round(s.batch.n_reads * steps / el / 1e6, 4),
             "unit": "Mreads/s", "gcups": round(float(st[0]) / el / 1e9, 3),
             "parity_all_steps": why is None, "coverage": s.coverage,
             "ext_busy_ms_per_batch": round(ext_busy / steps, 4),
             # the host's enqueue of the batches' launches (~30 each): near ms_per_batch = launch-bound
             "host_enqueue_ms_per_batch": round(t_enq * 1e3 / steps, 4),
             "batch": ("tests/golden/c3_refseed.npz (the C2 fixture's batch 0 in the GRCh38-shaped regime)"
                       if name == "c3_refseed" else f"tests/golden/c3_grch38.npz set {name!r}") +
                      f", the same batch every step"}
        if why:
            r["mismatch"] = why
        if name in ("c3", "c3_refseed") and ext_busy > 0:  # 150 bp: every task is in the first length bin
            ach = float(st[0]) * OPS_PER_CELL / (ext_busy * 1e-3) / 1e12
            r["roofline"] = {"bound": "valu", "kernel": DOMINANT_KERNEL, "achieved": round(ach, 3),
                             "peak": round(PK16_PEAK_TOPS, 1), "unit": "Tops/s", "frac": round(ach / PK16_PEAK_TOPS, 5),
                             "frac_int32": round(ach / VALU_PEAK_TOPS, 5),
                             "avg_launch_ms": round(ext_ms / max(ext_n, 1), 4)}
        out[name] = r

    pac_t = torch.from_numpy(g.pac).to(dev)
    eng = Engine(dev.index or 0, opt, g.l_pac, g.ann_offset, g.ann_len, pac_device_ptr=pac_t.data_ptr())
    eng.ext_form(ext_form)
    eng.set_device_read_len(max(int(np.diff(s.batch.seq_off).max()) for s in sets.values() if s.batch.n_reads))
    out["setup_s"] = round(time.perf_counter() - t0, 2)
    for name, s in sets.items():
        run_set(eng, name, s)
    eng.close()
    del pac_t
    torch.cuda.empty_cache()
    # reference-seeded chains in the same regime (a second genome: two golden copies around GRCh38's contigs)
    opt, g2, s = workload.load_c3_refseed(grch=g)
    del g
    pac_t = torch.from_numpy(g2.pac).to(dev)
    eng = Engine(dev.index or 0, opt, g2.l_pac, g2.ann_offset, g2.ann_len, pac_device_ptr=pac_t.data_ptr())
    eng.ext_form(ext_form)
    eng.set_device_read_len(int(np.diff(s.batch.seq_off).max()))
    run_set(eng, "c3_refseed", s)
    out["c3_refseed"].update({"l_pac": g2.l_pac, "contigs": len(g2.ann_len)})
    eng.close()
    del pac_t
    torch.cuda.empty_cache()
    return out


def c5_refseed_stage(pac_t, ref, dev, steps: int = 10, n_streams: int = 2, ext_form: int = 0) -> dict:
    """C5 (BASELINE.json configs[4]) on chains the REFERENCE seeded: one mixed
    2x100 / 2x150 / 2x250 ChainsRecord of the chr21-sized genome
    (tests/golden/c5_refseed.npz, oracle/gen_c2_fixture.py --length mix) run
    `steps` times over 2 streams with inputs resident, every step's output
    checked against the reference's regions (per-read counts + SHA-256)."""
    opt, _, rbs = workload.load_fixture(workload.C5_FIXTURE, with_ref=False)
    z = np.load(workload.C5_FIXTURE)
    if hashlib.sha256(ref.pac.tobytes()).digest() != z["pac_sha256"].tobytes():
        return {"error": "c5_refseed fixture is for another genome"}
    rb = rbs[0]
    eng = Engine(dev.index or 0, opt, ref.l_pac, ref.ann_offset, ref.ann_len, pac_device_ptr=pac_t.data_ptr())
    eng.ext_form(ext_form)
    lens = np.diff(rb.batch.seq_off)
    eng.set_device_read_len(int(lens.max()))
    streams = caller_streams(dev, n_streams)
    d = DevBatch(rb.batch, dev)
    for _ in range(steps - 1):
        d.add_out()
    for i in range(2):
        d.run(eng, streams[i % n_streams].cuda_stream, i, stats=False)
    torch.cuda.synchronize()
    d.stats.zero_()
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    t1 = time.perf_counter()
    ev0.record(streams[0])
    for x in streams[1:]:
        x.wait_event(ev0)
    for i in range(steps):
        d.run(eng, streams[i % n_streams].cuda_stream, i)
    for x in streams[1:]:
        e = torch.cuda.Event()
        e.record(x)
        streams[0].wait_event(e)
    ev1.record(streams[0])
    torch.cuda.synchronize()
    el = max(time.perf_counter() - t1, ev0.elapsed_time(ev1) / 1e3)
    st = d.stats.cpu().numpy()
    ok = all(rb.check(*d.results(i)) for i in range(steps))
    eng.close()
    return {"reads_per_batch": rb.batch.n_reads, "bases_per_batch": int(rb.batch.seq_off[-1]),
            "read_lengths": {str(k): int(v) for k, v in zip(*np.unique(lens, return_counts=True))},
            "ms_per_batch": round(el * 1e3 / steps, 4), "value": round(rb.batch.n_reads * steps / el / 1e6, 4),
            "unit": "Mreads/s", "gcups": round(float(st[0]) / el / 1e9, 3), "parity_all_steps": bool(ok),
            "chain_source": "reference seeding (bwa mem_chain), chr21-sized genome"}


STREAM_SEED = 4000      # stream batch g: tools/synth.cpp reads with seed STREAM_SEED + g
STREAM_PAIRS = 33_334   # pairs per ChainsRecord: 66,668 reads = 10.0 Mbases (Pipeline.cpp:123,146)


def shard_ids(rank: int, world: int, per_rank: int) -> list[int]:
    """the global stream batches rank `rank` of `world` takes: r, r + N, r + 2N, ...
    (bwa-flow's pull-scatter hands read batches to workers in turn,
    src/mpi/MPIChannel.cpp:140-200); the shards are disjoint and their union is
    batches 0 .. N * per_rank - 1"""
    return [rank + world * k for k in range(per_rank)]


def ensure_bwa_index(local_rank: int, world: int) -> str | None:
    """the golden genome's bwa index under bench_data/e2e (ref.fa.bwt/.sa/.pac/
    .ann/.amb): kept when its stamp matches, else built by the reference's own
    bwa_idx_build (oracle/_ref/sam_harness index: ~30-60 s, once per box) — the
    index bwa-flow's SeqsToChains reads.  Local rank 0 builds, the others wait.
    -> the index prefix, or None when it cannot be had"""
    pre = os.path.join(E2E_DIR, "ref.fa")
    h = os.path.join(REPO, "oracle", "_ref", "sam_harness")
    have = os.path.exists(pre + ".bwt") and os.path.exists(pre + ".sa")
    if not have and local_rank == 0 and os.access(h, os.X_OK):
        import subprocess
        os.makedirs(E2E_DIR, exist_ok=True)
        t0 = time.perf_counter()
        r = subprocess.run([h, "index", E2E_DIR, os.devnull, "7", "0", "150", "10000000", "1", "46709983"],
                           cwd=REPO, capture_output=True, text=True, timeout=900)
        log(f"[bench] bwa index of the golden genome: rc={r.returncode}, {time.perf_counter() - t0:.1f} s")
    if world > 1:
        dist.barrier()
    return pre if os.path.exists(pre + ".bwt") and os.path.exists(pre + ".sa") else None


def stream_reads(ref, g: int, pairs: int = STREAM_PAIRS) -> Batch:
    """global stream batch g's reads (tools/synth.cpp, seed STREAM_SEED + g,
    uniform over the genome's contigs, 0.8 % substitutions, 0.1 % indels); only
    seq_off / seq are used"""
    return synth_batch(ref, STREAM_SEED + g, pairs, 150)


def stream_batches(dev, opt, ref, pac_t, index, gids: list[int], pairs: int = STREAM_PAIRS) -> tuple[list[Batch], float]:
    """the stream's ChainsRecords `gids`: stream_reads(g), chains from the
    DEVICE's SeqsToChains (bwagpu_seqs2chains) against `index` = a bwa index
    prefix or (hdr, words, sa, sa_intv), on a context of its own, closed before
    timing.  -> (batches, seconds)"""
    t0 = time.perf_counter()
    hdr, words, sa, sa_intv = workload.load_bwa_index(index) if isinstance(index, str) else index
    ech = Engine(dev.index or 0, opt, ref.l_pac, ref.ann_offset, ref.ann_len, pac_device_ptr=pac_t.data_ptr())
    ech.set_bwt(hdr, words, sa, sa_intv)
    out = []
    for g in gids:
        rd = stream_reads(ref, g, pairs)
        rco, ch, cso, sd = ech.seqs2chains(rd.seq_off, rd.seq)
        out.append(Batch(rd.seq_off, rd.seq, rco, cso, ch["rid"].copy(), ch["frac_rep"].copy(), sd))
    ech.close()
    torch.cuda.empty_cache()
    return out, time.perf_counter() - t0


def reference_answers(opt, ref, batches: list[Batch], prefix: str) -> dict:
    """THE CHECKER (and the CPU baseline) of the stream: for every batch, the
    reference's own SeqsToChains on the host must give the chains the device
    made (oracle.ref_seqs2chains: ref_seqs2chains_batch), and the reference's own
    mem_chain2aln (oracle/_ref/libbwaref.so, the host cores this job may use)
    gives the expected regions, kept as a RefBatch (per-read counts + SHA-256 of
    the 88-byte records) that every timed step's output is compared with.
    -> {"checks": [RefBatch], "chains_identical": bool, "chain2aln_s": wall of
    the reference mem_chain2aln calls, "cores": threads, "kind"}"""
    sys.path.insert(0, os.path.join(REPO, "oracle"))
    import oracle
    kind = "reference" if oracle.ref_lib() is not None else "port"
    which = "ref" if kind == "reference" else "oracle"
    cores = host_threads()
    R = oracle.Ref(ref.l_pac, ref.ann_offset, ref.ann_len, ref.pac)
    checks, same, t_c2a, t_chain = [], True, 0.0, 0.0
    for b in batches:
        if kind == "reference":
            t0 = time.perf_counter()
            rco, rid, fr, cso, sd = oracle.ref_seqs2chains(prefix, b.seq_off, b.seq, n_threads=cores)
            t_chain += time.perf_counter() - t0
            same &= bool(np.array_equal(rco, b.read_chain_off) and np.array_equal(cso, b.chain_seed_off) and
                         np.array_equal(rid, b.chain_rid) and np.array_equal(fr.view(np.uint32),
                                                                         b.chain_frac_rep.view(np.uint32)) and
                         all(np.array_equal(sd[f], b.seeds[f]) for f in ("rbeg", "qbeg", "len", "score")))
        t0 = time.perf_counter()
        regs, n, _ = oracle.chain2aln(which, opt, R, b, n_threads=cores)
        t_c2a += time.perf_counter() - t0
        c = np.ascontiguousarray(compact(b, regs, n))
        checks.append(workload.RefBatch(b, n.astype(np.int32), hashlib.sha256(c.view(np.uint8).tobytes()).digest()))
    return {"checks": checks, "chains_identical": same if kind == "reference" else None, "chain2aln_s": t_c2a,
            "seqs2chains_s": t_chain, "cores": cores, "kind": kind}


class Workload:
    """what a rank runs: opt, host reference + its device copy, the timed
    batches and their reference answers, the fixture's two batches (side
    figure, warm-up, the chaining leg), the data text and config extras"""

    def __init__(self, **kw):
        self.fixture = None      # [RefBatch] of tests/golden/c2_refseed.npz (c2_* workloads)
        self.ref_answers = None  # reference_answers() of the stream (c2_stream)
        self.__dict__.update(kw)


FIXTURE_DATA = ("synthetic (seeded) reads on a 46.7 Mb chr21-sized synthetic genome (3 contigs, interspersed + "
                "tandem repeats, N runs), 2x150 bp pairs, 0.8% subs / 0.1% indels")


def batch_stats(batches, checks) -> dict:
    nr = sum(b.n_reads for b in batches)
    st = dict(chains_per_read=round(sum(b.n_chains for b in batches) / nr, 3),
              seeds_per_read=round(sum(b.n_seeds for b in batches) / nr, 3))
    if checks:
        st["regions_per_read"] = round(sum(int(rb.reg_n.sum()) for rb in checks) / nr, 3)
    return st


def load_workload(args, rank, world, dev, local: int = 0) -> Workload:
    if args.workload in ("c2_refseed", "c2_stream"):
        opt, gref, refbatches = workload.load_fixture(with_ref=(rank == 0))
        L = int(np.load(workload.C2_FIXTURE)["genome_len"])
        ref, pac_t = broadcast_reference(gref, rank, world, dev)
        assert ref.l_pac == L
        prefix = ensure_bwa_index(local, world) if args.workload == "c2_stream" else None
        if args.workload == "c2_stream" and prefix is not None:
            n_use = max(1, min(args.stream_batches, args.steps))
            gids = shard_ids(rank, world, n_use)
            batches, t_gen = stream_batches(dev, opt, ref, pac_t, prefix, gids)
            t0 = time.perf_counter()
            ans = reference_answers(opt, ref, batches, prefix)
            t_ref = time.perf_counter() - t0
            data = (FIXTURE_DATA + f"; a stream of {world * n_use} distinct ChainsRecords ({n_use} per GPU: global "
                    f"batches rank + {world} k), reads from tools/synth.cpp (seed {STREAM_SEED} + batch), chains from "
                    "the device's own SeqsToChains (bwagpu_seqs2chains) against the reference's bwa index, checked "
                    "equal to the REFERENCE's own mem_chain/mem_chain_flt/mem_flt_chained_seeds before timing")
            extras = dict(chain_source="device SeqsToChains, checked against the reference's", **batch_stats(
                batches, ans["checks"]), stream_batches_per_gpu=n_use, stream_batches_total=world * n_use,
                          stream_reads_per_gpu=sum(b.n_reads for b in batches),
                          chains_identical_to_reference=ans["chains_identical"],
                          setup_s={"reads_and_device_chains": round(t_gen, 2), "reference_check": round(t_ref, 2)})
            return Workload(opt=opt, ref=ref, pac_t=pac_t, batches=batches, checks=ans["checks"], data=data,
                            extras=extras, fixture=refbatches, ref_answers=ans, gids=gids)
        if args.workload == "c2_stream":
            log("[bench] no bwa index of the golden genome: the fixture's two batches are the workload")
        batches = [rb.batch for rb in refbatches]
        checks = list(refbatches)
        if rank % len(batches):  # each rank starts at a different batch
            k = rank % len(batches)
            batches, checks = batches[k:] + batches[:k], checks[k:] + checks[:k]
        data = (FIXTURE_DATA + "; chains from the REFERENCE's own bwa index + mem_chain/mem_chain_flt/"
                "mem_flt_chained_seeds (tests/golden/c2_refseed.npz, oracle/gen_c2_fixture.py)")
        return Workload(opt=opt, ref=ref, pac_t=pac_t, batches=batches, checks=checks, data=data,
                        extras=dict(chain_source="reference seeding (bwa mem_chain)", **batch_stats(batches, checks)),
                        fixture=refbatches)
    opt = abi.default_opt()
    ref, pac_t = shared_reference(args.ref_len, args.contigs, rank, world, dev)
    allb = rank_reads(ref, rank, args.pairs, args.read_len)
    batches = split_batches(allb, args.batch_bases)
    data = ("synthetic (seeded): 46.7 Mb chr21-sized reference, 2x150 bp pairs with 0.8% subs/0.1% indels, "
            "chains = exact-match seeds along the true origin (bwa-flow_amd/tools/synth.cpp)")
    return Workload(opt=opt, ref=ref, pac_t=pac_t, batches=batches, checks=None, data=data,
                    extras=dict(chain_source="synth.cpp exact matches", **batch_stats(batches, None)))


def timed_steps(eng: Engine, dbs, slots, streams, steps: int, world: int, dev, prof: bool) -> dict:
    """exactly `steps` steps (step i: batch dbs[i % len(dbs)] into its output
    slots[i], on streams[i % len(streams)]) between a barrier + device sync on
    each side; the job's time is the max over ranks, reads summed over ranks"""
    stream = streams[0]
    nb = len(dbs)
    if prof:
        eng.prof_start(3 * steps)  # HIP events around the dominant kernel's launches
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    t0 = time.perf_counter()
    ev0.record(stream)
    for x in streams[1:]:
        x.wait_event(ev0)
    for i in range(steps):
        dbs[i % nb].run(eng, streams[i % len(streams)].cuda_stream, slots[i])
    t_enq = time.perf_counter() - t0  # the host's enqueue of every step's ~30 launches
    for x in streams[1:]:
        e = torch.cuda.Event()
        e.record(x)
        stream.wait_event(e)
    ev1.record(stream)
    torch.cuda.synchronize()
    wall = time.perf_counter() - t0
    if world > 1:
        dist.barrier()
    gpu_s = ev0.elapsed_time(ev1) / 1e3
    elapsed = max(wall, gpu_s)
    reads_done = sum(dbs[i % nb].b.n_reads for i in range(steps))
    elapsed, total_reads = job_totals(elapsed, reads_done, world, dev)
    r = dict(elapsed=elapsed, total_reads=total_reads, wall=wall, gpu_s=gpu_s, enqueue_s=t_enq)
    if prof:
        r["ext_ms"], r["ext_launches"] = eng.prof_read()
        r["ext_iv"] = eng.prof_intervals(3 * steps)
        eng.prof_start(0)
    return r


def steps_parity(dbs, slots, steps: int, world: int, dev) -> bool | None:
    """every timed step's output against its batch's reference answer, all ranks"""
    if any(d.check is None for d in dbs):
        return None
    ok = True
    for i in range(steps):
        d = dbs[i % len(dbs)]
        ok &= d.check.check(*d.results(slots[i]))
    pt = torch.tensor([0.0 if ok else 1.0], dtype=torch.float64, device=dev)
    if world > 1:
        dist.all_reduce(pt, op=dist.ReduceOp.SUM)
    return float(pt.item()) == 0.0


def make_slots(dbs, steps: int) -> list[int]:
    """step i's output slot in its batch (one per run, so every step can be checked)"""
    nb, slots = len(dbs), []
    for i in range(steps):
        slots.append(dbs[i % nb].add_out() if i >= nb else 0)
    return slots


def fixture_figure(eng: Engine, fixture, dev, streams, steps: int) -> dict:
    """round 5's headline as a side figure: the two reference-seeded fixture
    batches cycled over `steps` steps, same streams, parity on every step"""
    dbs = [DevBatch(rb.batch, dev, rb) for rb in fixture]
    slots = make_slots(dbs, steps)
    for i in range(2 * len(dbs)):
        dbs[i % len(dbs)].run(eng, streams[i % len(streams)].cuda_stream, 0, stats=False)
    torch.cuda.synchronize()
    t = timed_steps(eng, dbs, slots, streams, steps, 1, dev, prof=False)
    par = steps_parity(dbs, slots, steps, 1, dev)
    del dbs
    torch.cuda.empty_cache()
    return {"value": round(t["total_reads"] / t["elapsed"] / 1e6, 4), "unit": "Mreads/s",
            "ms_per_step": round(t["elapsed"] / steps * 1e3, 4), "steps": steps, "distinct_batches": len(fixture),
            "parity_all_steps": par, "streams": len(streams),
            "workload": "tests/golden/c2_refseed.npz: 2 reference-seeded batches of 66,668 reads cycled (round 5's "
                        "headline workload)"}


def hw_queues_4_figure(steps: int, warmup: int, ext_form: int) -> dict:
    """the fixture figure in a child process with HIP's default of 4 hardware
    queues per process (GPU_MAX_HW_QUEUES unset: what a bwa-flow process gets
    without INTEGRATION.md §2's setting); the parent's figure runs at 16"""
    import subprocess
    env = dict(os.environ, BWAGPU_BENCH_KEEP_HWQ="1")
    env.pop("GPU_MAX_HW_QUEUES", None)
    for k in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(k, None)
    r = subprocess.run([sys.executable, os.path.abspath(__file__), "--workload", "c2_refseed", "--steps", str(steps),
                        "--warmup", str(warmup), "--ext-form", str(ext_form), "--headline-only"],
                       cwd=REPO, env=env, capture_output=True, text=True, timeout=600)
    if r.returncode != 0:
        return {"error": f"rc={r.returncode} {r.stderr[-300:]}"}
    d = json.loads(r.stdout.strip().splitlines()[-1])
    return {"value": d["value"], "unit": "Mreads/s", "ms_per_step": d["ms_per_step"],
            "parity_all_steps": d["parity_all_steps"], "gpu_max_hw_queues": 4, "streams": d["config"]["streams"],
            "workload": "the two_batch_fixture workload, in a child process"}


def headline_line(args, world, W, eng, dbs, slots, streams, stream, sptr, elapsed, total_reads, cells, cells_all,
                  ext_ms, ext_launches, ext_busy_ms, parity) -> dict:
    """rank 0's JSON line: the headline, its roofline (the dominant kernel, VALU
    bound: packed 16-bit peak, the int32 figure beside it) and the HBM view"""
    dev = dbs[0].dev
    nb = len(dbs)
    batches = [d.b for d in dbs]
    # ---- launch-sequence duration (HIP events on the launch stream), outside the timed region
    per = []
    for i in range(min(nb, 8)):
        a, b_ = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record(stream)
        dbs[i].run(eng, sptr, 0, stats=False)
        b_.record(stream)
        torch.cuda.synchronize()
        per.append(a.elapsed_time(b_) / 1e3)
    launch_s = float(np.mean(per))
    # the same kernel with the GPU to itself: each distinct batch (up to 8) alone
    # on one stream, its first-bin launches (rounds A, B, C) timed by HIP events
    n_iso = min(nb, 8)
    iso, ext_tasks, tasks_ab, misses = [], [], [], []
    for i in range(n_iso):
        eng.prof_start(3)
        dbs[i].run(eng, sptr, 0, stats=False)
        torch.cuda.synchronize()
        iso.append([round(float(e - a), 4) for a, e in eng.prof_intervals(3)])
        sc = np.zeros(8, np.int64)  # tasks of rounds A / B / C (bwagpu_debug_spec_counters)
        eng.lib.bwagpu_debug_spec_counters(eng.ctx, ctypes.c_void_p(sptr), sc.ctypes.data_as(ctypes.c_void_p))
        ext_tasks.append(int(sc[0] + sc[1]))
        tasks_ab.append([int(sc[0]), int(sc[1])])
        misses.append(int(sc[4]))
    eng.prof_start(0)
    runs = {j: sum(1 for i in range(args.steps) if i % nb == j) for j in range(nb)}
    # the cells ksw_extend2 itself evaluates (ksw.c:424 iterations): each distinct
    # batch that ran once more, untimed, with the row bound off (bwagpu_ctx_row_bound)
    ref_cells = {}
    prev_bound = eng.row_bound(0)
    for i in range(nb):
        if not runs[i]:
            continue
        st0 = torch.zeros(4, dtype=torch.int64, device=dev)
        out, nn = dbs[i].outs[0]
        eng.chain2aln_device(dbs[i].c, out.data_ptr(), nn.data_ptr(), st0.data_ptr(), sptr)
        torch.cuda.synchronize()
        ref_cells[i] = int(st0.cpu().numpy()[0])
    eng.row_bound(prev_bound)
    # algorithmic HBM bytes of one launch sequence (batch average): inputs read
    # once, regions + counts written once, 2-bit reference rows read (rows/4
    # bytes), per-chain window + per-seed scratch written and read once
    alg, ext_alg, cells_batch = [], [], []
    for j, d in enumerate(dbs):
        if not runs[j]:
            continue
        s = d.stats.cpu().numpy()
        nreg = int(d.results(0)[1].sum())
        alg.append(d.in_bytes + nreg * 88 + d.b.n_reads * 4 + (int(s[1]) // runs[j]) / 4 +
                   2 * (d.b.n_chains * 16 + d.b.n_seeds * 8))
        cells_batch.append(float(s[0]) / runs[j])
    alg_bytes = float(np.mean(alg))
    # the extension kernel's own algorithmic bytes per launch (rounds A and B: two
    # launches per batch): per task its list entry 8 B, seed 24 B, chain window
    # 16 B, owner read 4 B, read offsets 16 B, the read's bases (lq B) and the
    # 48-byte SeedExt it writes; the 2-bit target rows the reference's DP reads
    # (stats rows / 4 B)
    for j in range(n_iso):
        s = dbs[j].stats.cpu().numpy()
        lq = float(dbs[j].b.seq_off[-1]) / max(dbs[j].b.n_reads, 1)
        ext_alg.append((ext_tasks[j] * (8 + 24 + 16 + 4 + 16 + lq + 48) + (int(s[1]) // max(runs[j], 1)) / 4) / 2)
    ext_alg_bytes = float(np.mean(ext_alg))
    cells_step = cells / args.steps
    cells_ref_step = sum(ref_cells[i % nb] for i in range(args.steps)) / args.steps
    ext_avg_ms = ext_ms / max(ext_launches, 1)
    # the dominant kernel's VALU roofline: algorithmic ops of the timed steps
    # over the busy union of its launches in those steps
    ach = cells * OPS_PER_CELL / (ext_busy_ms * 1e-3) / 1e12 if ext_busy_ms > 0 else None

    global DOMINANT_KERNEL
    DOMINANT_KERNEL = eng.ext_kernel(max(int(np.diff(b.seq_off).max()) for b in batches if b.n_reads))
    traffic, traffic_src, pmc = load_traffic(args.workload)
    iso_ms = [sum(x) for x in iso]
    frac_iso = (float(np.sum(cells_batch[:n_iso])) * OPS_PER_CELL / (float(np.sum(iso_ms)) * 1e-3) / 1e12 /
                PK16_PEAK_TOPS if iso and sum(iso_ms) > 0 else None)
    value = total_reads / elapsed / 1e6
    stream_wl = W.ref_answers is not None
    wl_text = ("STAGE-ONLY (the SW-extend stage, ChainsToRegions: mem_chain2aln + ksw_extend2, on the GPU; seeding, "
               "pairing and SAM are not in this number: end_to_end_align is the whole pipeline) C2: 2x150 bp pairs vs "
               "a chr21-sized reference, ChainsRecords of 66,668 reads, inputs resident in HBM; " +
               (f"a stream of {nb} distinct batches per GPU ({sum(b.n_reads for b in batches)} reads), each timed "
                f"step a different batch until the stream is used up" if stream_wl else
                f"{nb} distinct reference-seeded batches cycled"))
    return {
        "metric": METRIC, "value": round(value, 4), "unit": "Mreads/s", "n_gpus": world, "steps": args.steps,
        "warmup": args.warmup, "ms_per_step": round(elapsed / args.steps * 1e3, 4), "higher_is_better": True,
        "scaling": "weak", "vs_baseline": None, "dtype": "int32", "data": W.data,
        "config": {"workload": wl_text if args.workload != "synth" else
                   "STAGE-ONLY C2 (synth chains): SW-extend stage on GPU, inputs resident in HBM",
                   "reads_per_batch": int(np.mean([b.n_reads for b in batches])), "distinct_batches": nb,
                   "distinct_batches_timed": min(nb, args.steps),
                   "batch_bases": args.batch_bases, "read_len": 150 if args.workload != "synth" else args.read_len,
                   "parallelism": f"dp{world}", "streams": len(streams),
                   "sharding": (f"rank r runs global stream batches r, r+{world}, ... (disjoint shards)"
                                if stream_wl else "every rank runs the same batches"), **W.extras},
        "gcups": round(cells_all / elapsed / 1e9, 3),
        # the same over the cells the reference's ksw_extend2 evaluates (the row
        # bound ends calls early: those rows' cells are never computed)
        "gcups_reference_cells": round(cells_ref_step * args.steps * world / elapsed / 1e9, 3),
        "row_bound": bool(eng.row_bound(-1)),
        "stage_only": True,
        "parity_all_steps": parity,
        "roofline": {"bound": "valu", "kernel": DOMINANT_KERNEL,
                     # the kernel computes in packed 16-bit halves (v_pk_*: two DP cells per
                     # lane-op, issued at ~4 cycles per wave-instruction like every 3-input /
                     # DPP op it uses): the peak is the packed-16 one
                     "achieved": round(ach, 3) if ach else None, "peak": round(PK16_PEAK_TOPS, 1), "unit": "Tops/s",
                     "frac": round(ach / PK16_PEAK_TOPS, 5) if ach else None,
                     "arith": "int16x2 packed (v_pk_*), int32 guards and row-end state",
                     "peak_int32": round(VALU_PEAK_TOPS, 1),
                     "frac_int32": round(ach / VALU_PEAK_TOPS, 5) if ach else None,
                     "peak_measured_issue_int32": round(VALU_ISSUE_PEAK_TOPS, 1),
                     "frac_denominator": "busy union of the kernel's launch intervals (HIP events)",
                     "cells": "computed cells (the row bound's skipped rows are not counted)",
                     "ops_per_cell": OPS_PER_CELL, "cells_per_step": round(cells_step),
                     "cells_per_step_reference": round(cells_ref_step),
                     # busy time: the union of the kernel's launch intervals in the timed steps
                     # (HIP events on the launching streams), <= ms_per_step
                     "kernel_ms_per_step": round(ext_busy_ms / args.steps, 4),
                     "kernel_sum_ms_per_step": round(ext_ms / args.steps, 4), "launches_timed": ext_launches,
                     "avg_launch_ms": round(ext_avg_ms, 4),
                     "launch_unit": ("one round's left + right side launches (the phased pair, HIP events "
                                     "bracket both)" if "spec_side" in DOMINANT_KERNEL else "one launch per round"),
                     # the kernel alone on the GPU (one stream, one batch at a time)
                     "isolated_launch_ms": iso, "frac_isolated": round(frac_iso, 5) if frac_iso else None,
                     "tasks_round_a_b": tasks_ab,
                     # extensions the selection passes computed inline (a round-B prediction missed them)
                     "inline_extensions": misses,
                     "traffic": traffic, "traffic_source": traffic_src, "pmc": pmc,
                     "alg_bytes_per_launch": round(ext_alg_bytes),
                     "traffic_over_alg": round(traffic / ext_alg_bytes, 3) if traffic and ext_alg_bytes else None,
                     "formula": "cells_per_step * ops_per_cell / kernel_ms_per_step (busy union) / peak "
                                "(DESIGN.md §5)",
                     "frac_step": round(cells_step * OPS_PER_CELL / (elapsed / args.steps) / 1e12 / PK16_PEAK_TOPS, 5)},
        "roofline_hbm": {"bound": "hbm", "achieved": round(alg_bytes / launch_s / 1e9, 3), "peak": HBM_PEAK_GBS,
                         "unit": "GB/s", "frac": round(alg_bytes / launch_s / 1e9 / HBM_PEAK_GBS, 6),
                         "alg_bytes_per_launch_sequence": round(alg_bytes), "launch_sequence_ms": round(launch_s * 1e3, 4),
                         "kernel": "whole SW-stage launch sequence (all kernels of one batch)"},
    }


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=30)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--workload", default="c2_stream", choices=("c2_stream", "c2_refseed", "synth"))
    ap.add_argument("--stream-batches", type=int, default=30,
                    help="c2_stream: distinct ChainsRecords per GPU (30 = 1M pairs); step i runs batch i mod "
                         "min(this, steps)")
    ap.add_argument("--pairs", type=int, default=1_000_000, help="synth: read pairs per GPU (C2: 1M)")
    ap.add_argument("--ref-len", type=int, default=46_709_983, help="synth: reference length (chr21: 46.7 Mb)")
    ap.add_argument("--contigs", type=int, default=1)
    ap.add_argument("--read-len", type=int, default=150, help="synth: 100/150/250, or 0 = mixed thirds (C5)")
    ap.add_argument("--batch-bases", type=int, default=10_000_000, help="ChainsRecord size (Pipeline.cpp:146)")
    ap.add_argument("--cpu-budget", type=float, default=20.0, help="CPU-seconds for the cpu_baseline sample")
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--no-host-path", action="store_true", help="skip the PCIe-inclusive host-buffer rate")
    ap.add_argument("--host-slots", type=int, default=4, choices=(2, 3, 4),
                    help="host-buffer path: slots in flight (batch i + slots - 1 submitted before i is waited for)")
    ap.add_argument("--no-cigar", action="store_true", help="skip the CIGAR (mem_reg2aln) stage line")
    ap.add_argument("--no-seeding", action="store_true", help="skip the seeding (mem_collect_intv) line")
    ap.add_argument("--no-regime", action="store_true", help="skip the C3/C5 GRCh38-regime legs")
    ap.add_argument("--no-e2e", action="store_true", help="skip the whole-pipeline end-to-end align leg")
    ap.add_argument("--no-hwq4", action="store_true", help="skip the GPU_MAX_HW_QUEUES=4 side figure")
    ap.add_argument("--headline-only", action="store_true", help="the headline line only (no side legs)")
    ap.add_argument("--e2e-pairs", type=int, default=300_000)
    ap.add_argument("--no-prof", action="store_true", help="no HIP events around the dominant kernel (A/B of their cost)")
    ap.add_argument("--ext-form", type=int, default=0, choices=(0, 1, 2),
                    help="first two read-length bins: 0 packed 16-bit DP, eight seeds per wave in the first bin and "
                         "four in the second; 1 two per wave (32-bit DP); 2 four per wave in both")
    ap.add_argument("--streams", type=int, default=3, choices=(1, 2, 3, 4),
                    help="batches alternate over this many streams (the FPGA stage's ping-pong, SWTask.cpp:82-85, "
                         "one stream per stage worker): batch i+1's launches overlap batch i's tail; 3 since the row "
                         "bound (2 / 3 / 4: 45.7-46.3 / 48.0-51.2 / 42.8-43.8 Mreads/s, gpurun_out/r6z)")
    args = ap.parse_args()
    if args.headline_only:
        args.no_cpu = args.no_host_path = args.no_cigar = args.no_seeding = args.no_regime = True
        args.no_e2e = args.no_hwq4 = True

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)

    def new_engine(opt_, l_pac, ann_offset, ann_len, pac_ptr) -> Engine:
        """a context with this run's extension form (bwagpu_ctx_ext_form)"""
        e = Engine(local, opt_, l_pac, ann_offset, ann_len, pac_device_ptr=pac_ptr)
        e.ext_form(args.ext_form)
        return e

    # reference: on rank 0, broadcast over RCCL (xGMI) at start-up only
    t0 = time.perf_counter()
    W = load_workload(args, rank, world, dev, local)
    opt, ref, pac_t, batches, checks = W.opt, W.ref, W.pac_t, W.batches, W.checks
    setup_s = time.perf_counter() - t0
    eng = new_engine(opt, ref.l_pac, ref.ann_offset, ref.ann_len, pac_t.data_ptr())
    # the producer of the resident batches knows their longest read (bwagpu_set_device_read_len)
    eng.set_device_read_len(max(int(np.diff(b.seq_off).max()) for b in batches if b.n_reads))
    dbs = [DevBatch(b, dev, checks[i] if checks else None) for i, b in enumerate(batches)]
    nb = len(dbs)
    slots = make_slots(dbs, args.steps)
    torch.cuda.synchronize()
    log(f"[bench] rank {rank}: {nb} batches, {sum(b.n_reads for b in batches)} reads, "
        f"{sum(b.n_chains for b in batches)} chains, {sum(b.n_seeds for b in batches)} seeds "
        f"(setup {setup_s:.1f} s)")

    # a dedicated stream: the engine launches on it and every HIP event below is
    # recorded on it (the null stream would leave the engine on its own stream)
    streams = caller_streams(dev, args.streams)
    stream = streams[0]
    torch.cuda.set_stream(stream)
    sptr = stream.cuda_stream
    # warm-up: on the fixture's batches when there are any, so that the timed
    # stream batches start cold (not in the MALL)
    wdbs = [DevBatch(rb.batch, dev) for rb in W.fixture] if W.fixture and W.ref_answers else dbs
    for i in range(args.warmup):
        wdbs[i % len(wdbs)].run(eng, streams[i % len(streams)].cuda_stream, 0, stats=False)
    torch.cuda.synchronize()
    if wdbs is not dbs:
        del wdbs
    for d in dbs:
        d.stats.zero_()

    # ---- timed region: exactly K steps
    T = timed_steps(eng, dbs, slots, streams, args.steps, world, dev, prof=not args.no_prof)
    elapsed, total_reads = T["elapsed"], T["total_reads"]
    ext_ms, ext_launches = T.get("ext_ms", 0.0), T.get("ext_launches", 0)
    # the dominant kernel's busy time: the union of its launch intervals (the
    # caller streams' launches overlap; their summed durations can exceed the wall)
    ext_busy_ms = busy_ms(T.get("ext_iv", []))

    # per-step counters (cells/rows/calls) of the timed steps
    cells = rows = calls = 0
    for d in dbs:
        s = d.stats.cpu().numpy()  # accumulated over every run of the batch in the timed region
        cells += int(s[0])
        rows += int(s[1])
        calls += int(s[2])
        assert int(s[3]) == 0, "device flagged an error"
    ctot = torch.tensor([cells, rows, calls], dtype=torch.float64, device=dev)
    if world > 1:
        dist.all_reduce(ctot, op=dist.ReduceOp.SUM)
    cells_all = float(ctot[0].item())

    # bit-exact check of EVERY timed step's output against the reference's regions
    parity = steps_parity(dbs, slots, args.steps, world, dev) if checks else None

    result = None
    if rank == 0:
        result = headline_line(args, world, W, eng, dbs, slots, streams, stream, sptr, elapsed, total_reads,
                               cells, cells_all, ext_ms, ext_launches, ext_busy_ms, parity)
        # the host's enqueue of the timed steps' launches (~30 per batch), per step: near
        # ms_per_step would mean the stage is launch-bound on this host
        result["host_enqueue_ms_per_step"] = round(T["enqueue_s"] * 1e3 / args.steps, 4)
    regs0, n0 = dbs[0].results(0)
    fix_checks = W.fixture if W.fixture else checks
    if rank == 0 and world == 1 and W.fixture and W.ref_answers and not args.headline_only:
        try:  # a side line: a failure here must not cost the headline line
            result["two_batch_fixture"] = fixture_figure(eng, W.fixture, dev, streams, args.steps)
        except Exception as e:
            result["two_batch_fixture"] = {"error": repr(e)}
    if rank == 0 and world == 1 and not args.no_host_path:
        # host buffers through submit/wait: every distinct batch once at least
        result["host_buffer_path"] = host_path_rate(eng, batches, max(24, nb), checks, depth=args.host_slots)
        try:  # a side line: a failure here must not cost the headline line
            e2_batches = batches[:min(nb, 20)]
            e2_checks = checks[:len(e2_batches)] if checks else None
            reps = max(2, 40 // len(e2_batches))
            result["end_to_end"] = end_to_end_stage(opt, ref, e2_batches, e2_checks, reps=reps, chain_mode=1)
            e2f = end_to_end_stage(opt, ref, e2_batches, e2_checks, reps=reps, chain_mode=0)
            result["end_to_end"]["chains_forwarded"] = {k: e2f.get(k) for k in ("value", "ms_per_record",
                                                                                "parity_last_rep", "chains", "error")
                                                        if k in e2f}
        except Exception as e:
            result["end_to_end"] = {"error": repr(e)}
    cigar = None
    if rank == 0 and world == 1 and not args.no_cigar:
        try:  # a side line: a failure here must not cost the headline line
            cs, jobs0, gout0 = cigar_stage(eng, dbs[0].b, regs0, n0)
            result["cigar_stage"] = cs
            cigar = (jobs0, gout0)
        except Exception as e:
            result["cigar_stage"] = {"error": repr(e)}
    # the whole-pipeline leg first: its harness builds the chr21-sized genome's
    # bwa index (bench_data/e2e) on a fresh box when the stream has not, which
    # the seeding and chaining legs then read
    if rank == 0 and world == 1 and not args.no_e2e:
        try:  # a side line: a failure here must not cost the headline line
            e2e = end_to_end_align(args.e2e_pairs)
            if e2e is not None:
                result["end_to_end_align"] = e2e
        except Exception as e:
            result["end_to_end_align"] = {"error": repr(e)}
    seeding = None
    fix_b0 = fix_checks[0].batch if fix_checks else dbs[0].b
    if rank == 0 and world == 1 and not args.no_seeding:
        try:  # a side line: a failure here must not cost the headline line
            seeding = seeding_stage(eng, fix_b0)
            if seeding is not None:
                result["seeding_stage"] = {k: v for k, v in seeding.items() if k != "_check"}
        except Exception as e:
            result["seeding_stage"] = {"error": repr(e)}
        if fix_checks:
            try:  # a side line: a failure here must not cost the headline line
                chaining = chaining_stage(eng, fix_checks[0])  # reference chains: the fixture's
                if chaining is not None:
                    result["chaining_stage"] = chaining
            except Exception as e:
                result["chaining_stage"] = {"error": repr(e)}
    if rank == 0 and world == 1 and not args.no_regime:
        try:  # a side line: a failure here must not cost the headline line
            result["regime_grch38"] = regime_stage(dev, ext_form=args.ext_form)
        except Exception as e:
            result["regime_grch38"] = {"error": repr(e)}
    if rank == 0 and world == 1 and not args.no_regime and args.workload != "synth":
        try:  # a side line: a failure here must not cost the headline line
            result["c5_refseed"] = c5_refseed_stage(pac_t, ref, dev, ext_form=args.ext_form)
        except Exception as e:
            result["c5_refseed"] = {"error": repr(e)}
    if rank == 0 and world == 1 and not args.no_hwq4 and W.fixture:
        try:  # a side line: a failure here must not cost the headline line
            h4 = hw_queues_4_figure(args.steps, args.warmup, args.ext_form)
            h16 = result.get("two_batch_fixture") or {}
            h4["gpu_max_hw_queues_16_same_workload"] = h16.get("value")
            result["hw_queues_4"] = h4
        except Exception as e:
            result["hw_queues_4"] = {"error": repr(e)}
    if rank == 0 and world == 1 and not args.no_cpu:
        if seeding is not None:
            try:
                port = seeding_cpu_baseline(fix_b0, *seeding["_check"])
                refb = ref_seeding_baseline(fix_b0, 0)
                result["seeding_stage"]["cpu_baseline"] = refb if refb is not None else port
                result["seeding_stage"]["parity_gpu_vs_cpu"] = port["parity_gpu_vs_cpu"]
                if refb is not None:
                    result["seeding_stage"]["cpu_baseline"]["matches_gpu"] = refb["count"] == seeding["intervals"]
                    result["seeding_stage"]["speedup_vs_cpu"] = round(seeding["value"] / refb["value"], 2)
            except Exception as e:
                result["seeding_stage"]["cpu_baseline"] = {"error": repr(e)}
        if "chaining_stage" in result and "error" not in result["chaining_stage"]:
            try:
                refc = ref_seeding_baseline(fix_b0, 1)
                if refc is not None:
                    ch = result["chaining_stage"]
                    refc["matches_gpu"] = refc["count"] == ch["chains"]
                    ch["cpu_baseline"] = refc
                    ch["speedup_vs_cpu_seqs2chains"] = round(ch["seqs2chains_Mreads_per_s"] / refc["value"], 2)
            except Exception as e:
                result["chaining_stage"]["cpu_baseline"] = {"error": repr(e)}
        if W.ref_answers is not None:
            cb = stream_cpu_baseline(opt, ref, batches, W.ref_answers)
        else:
            cb = cpu_baseline(opt, ref, batches, args.cpu_budget, [d.results(0) for d in dbs], checks)
        result["cpu_baseline"] = cb
        result["speedup_vs_cpu"] = round(result["value"] / cb["value"], 2)
        # the CPU side scaled linearly to every CPU of the host (optimistic for the CPU)
        node_cpu = cb["value"] * cb["host_cpus"] / max(cb["cores"], 1)
        result["speedup_vs_cpu_note"] = (f"vs the reference on {cb['cores']} threads (this job's CPU affinity) of a "
                                         f"{cb['host_cpus']}-CPU host, the CPU share this pool gives one GPU; "
                                         f"vs one thread: {round(result['value'] / cb['value_1core'], 1)}x; an EXTRAPOLATION, not measured: "
                                         f"the stage-only value x 8 GPUs (perfect weak scaling assumed) vs the "
                                         f"reference on all {cb['host_cpus']} CPUs at {cb['cores']}-thread "
                                         f"efficiency: {round(8 * result['value'] / node_cpu, 2)}x")

        if cigar is not None:
            try:
                result["cigar_stage"]["cpu_baseline"] = cigar_cpu_baseline(opt, ref, dbs[0].b, *cigar)
            except Exception as e:
                result["cigar_stage"]["cpu_baseline"] = {"error": repr(e)}
    if rank == 0:
        print(json.dumps(result), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()
    eng.close()


def stream_cpu_baseline(opt, ref, batches, ans) -> dict:
    """the CPU baseline of the stream: the reference's mem_chain2aln already ran
    over every batch on the host cores (reference_answers, before timing: it made
    the expected regions), plus batch 0 again on one thread"""
    sys.path.insert(0, os.path.join(REPO, "oracle"))
    import oracle
    which = "ref" if ans["kind"] == "reference" else "oracle"
    R = oracle.Ref(ref.l_pac, ref.ann_offset, ref.ann_len, ref.pac)
    t0 = time.perf_counter()
    oracle.chain2aln(which, opt, R, batches[0], n_threads=1)
    t1c = time.perf_counter() - t0
    reads = sum(b.n_reads for b in batches)
    return dict(value=reads / ans["chain2aln_s"] / 1e6, unit="Mreads/s", cores=ans["cores"], cpu=cpu_model(),
                kind=ans["kind"], host_cpus=os.cpu_count(), value_1core=round(batches[0].n_reads / t1c / 1e6, 5),
                sample_1core=f"batch 0 ({batches[0].n_reads} reads) on one thread, {t1c:.2f} s",
                sample=f"every stream batch once ({len(batches)} distinct, {reads} reads), "
                       f"{ans['chain2aln_s']:.2f} s wall on {ans['cores']} threads "
                       f"({'oracle/_ref/libbwaref.so: the reference mem_chain2aln' if ans['kind'] == 'reference' else 'oracle/liboracle.so'}); "
                       "its regions are the expected output every timed step is checked against",
                reference_seqs2chains_s=round(ans["seqs2chains_s"], 3),
                chains_identical_to_reference=ans["chains_identical"])


if __name__ == "__main__":
    main()
