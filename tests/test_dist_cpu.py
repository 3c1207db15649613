"""The multi-GPU path of bench.py on the CPU: world_size-2 `gloo` process
group standing in for RCCL.  bench.py's data path has exactly one
collective — the start-up broadcast of the packed reference + contig table
from rank 0 — and the whole-job totals (max time, summed
reads) at the end; shards are independent (weak scaling): rank r takes the
stream's global batches r, r + N, ... (the reference's pull-scatter,
src/mpi/MPIChannel.cpp:140-200)."""
import os
import socket
import sys

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, out_dir):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import bench
    ref, pac_t = bench.shared_reference(300_000, 3, rank, world, torch.device("cpu"))
    b = bench.rank_reads(ref, rank, 400, 150)
    el, tot = bench.job_totals(1.0 + rank, b.n_reads, world, torch.device("cpu"))
    np.savez(os.path.join(out_dir, f"r{rank}.npz"), pac=ref.pac, ann_offset=ref.ann_offset, ann_len=ref.ann_len,
             seq=b.seq, seeds=b.seeds.view(np.uint8), n_reads=b.n_reads, el=el, tot=tot)
    dist.barrier()
    dist.destroy_process_group()


def test_bench_distributed_plumbing_gloo(tmp_path):
    world = 2
    mp.spawn(_worker, args=(world, _free_port(), str(tmp_path)), nprocs=world, join=True)
    r = [np.load(os.path.join(tmp_path, f"r{k}.npz")) for k in range(world)]
    # every rank holds rank 0's reference after the broadcast ...
    for k in range(1, world):
        assert np.array_equal(r[k]["pac"], r[0]["pac"])
        assert np.array_equal(r[k]["ann_offset"], r[0]["ann_offset"])
        assert np.array_equal(r[k]["ann_len"], r[0]["ann_len"])
    from bwagpu.synth import SynthRef
    want = SynthRef(42, 300_000, 3)
    assert np.array_equal(r[0]["pac"], want.pac)
    # ... its own, different shard ...
    assert not np.array_equal(r[0]["seq"], r[1]["seq"])
    # ... and the job totals are max-over-ranks time and summed reads
    for k in range(world):
        assert float(r[k]["el"]) == 2.0
        assert float(r[k]["tot"]) == float(sum(int(x["n_reads"]) for x in r))


def _worker_fixture(rank, world, port, out_dir):
    """bench.load_workload on the c2_refseed fixture path with 2 ranks: rank 0
    regenerates the genome, rank 1 only receives it (any contig count)"""
    import argparse
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import bench
    args = argparse.Namespace(workload="c2_refseed")
    W = bench.load_workload(args, rank, world, torch.device("cpu"))
    ref, batches, checks = W.ref, W.batches, W.checks
    # a 195-contig table (the GRCh38 layout) through the same broadcast
    from bwagpu.synth import _load
    import ctypes as C
    off, ln, lp = np.zeros(195, np.int64), np.zeros(195, np.int32), C.c_int64()
    _load().grch38_layout(off.ctypes.data, ln.ctypes.data, C.byref(lp))

    class Small:
        l_pac, pac, ann_offset, ann_len = 4000, (np.arange(1001) % 251).astype(np.uint8), off, ln
    g, _ = bench.broadcast_reference(Small if rank == 0 else None, rank, world, torch.device("cpu"))
    np.savez(os.path.join(out_dir, f"f{rank}.npz"), pac=ref.pac, ann_offset=ref.ann_offset, ann_len=ref.ann_len,
             l_pac=ref.l_pac, first_reads=batches[0].n_reads, first_seq=batches[0].seq[:1000],
             checks=checks is not None and all(c.batch is b for c, b in zip(checks, batches)),
             g_off=g.ann_offset, g_len=g.ann_len, g_lpac=g.l_pac, g_pac=g.pac[:1000])
    dist.barrier()
    dist.destroy_process_group()


def test_load_workload_fixture_gloo(tmp_path):
    world = 2
    mp.spawn(_worker_fixture, args=(world, _free_port(), str(tmp_path)), nprocs=world, join=True)
    r = [np.load(os.path.join(tmp_path, f"f{k}.npz")) for k in range(world)]
    from bwagpu import workload
    z = np.load(workload.C2_FIXTURE)
    for k in range(world):
        assert int(r[k]["l_pac"]) == int(z["genome_len"])
        assert np.array_equal(r[k]["ann_offset"], z["ann_offset"]) and np.array_equal(r[k]["ann_len"], z["ann_len"])
        assert np.array_equal(r[k]["pac"], r[0]["pac"])
        assert bool(r[k]["checks"])
        assert len(r[k]["g_off"]) == 195 and int(r[k]["g_lpac"]) == 4000
        assert np.array_equal(r[k]["g_off"], r[0]["g_off"]) and np.array_equal(r[k]["g_len"], r[0]["g_len"])
        assert np.array_equal(r[k]["g_pac"], (np.arange(1000) % 251).astype(np.uint8))
        assert int(r[k]["g_off"][-1]) + int(r[k]["g_len"][-1]) == 3_099_734_149
    # rank 1 starts at the other batch
    assert not np.array_equal(r[0]["first_seq"], r[1]["first_seq"])


def test_shards_are_deterministic():
    import bench
    from bwagpu.synth import SynthRef
    ref = SynthRef(42, 300_000, 3)
    a = bench.rank_reads(ref, 1, 200, 150)
    b = bench.rank_reads(ref, 1, 200, 150)
    assert np.array_equal(a.seq, b.seq) and np.array_equal(a.seeds, b.seeds)


def test_stream_shards_partition_the_stream():
    """bench.shard_ids: for every world size the ranks' shards are disjoint and
    their union is exactly the stream's first world * per_rank batches"""
    import bench
    for world in (1, 2, 3, 4, 8):
        for per in (1, 2, 15, 30):
            shards = [bench.shard_ids(r, world, per) for r in range(world)]
            flat = [g for sh in shards for g in sh]
            assert len(flat) == len(set(flat)) == world * per
            assert sorted(flat) == list(range(world * per))
            assert all(len(sh) == per for sh in shards)


def _worker_stream(rank, world, port, out_dir):
    """each rank draws the reads of its own stream shard (bench.stream_reads)
    on the broadcast genome; rank 0 gathers which global batches were made"""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import bench
    ref, _ = bench.shared_reference(400_000, 3, rank, world, torch.device("cpu"))
    gids = bench.shard_ids(rank, world, 3)
    digests = {g: __import__("hashlib").sha256(bench.stream_reads(ref, g, 300).seq.tobytes()).hexdigest()
               for g in gids}
    got = [None] * world
    dist.all_gather_object(got, digests)
    if rank == 0:
        import json
        json.dump(got, open(os.path.join(out_dir, "stream.json"), "w"))
    dist.barrier()
    dist.destroy_process_group()


def test_stream_shards_gloo(tmp_path):
    """world_size 2: the shards the two ranks generate are disjoint, their union
    is the whole stream, and each batch is the one a single process makes for
    the same global index (the stream does not depend on the world size)"""
    import json
    import hashlib
    import bench
    from bwagpu.synth import SynthRef
    world = 2
    mp.spawn(_worker_stream, args=(world, _free_port(), str(tmp_path)), nprocs=world, join=True)
    got = json.load(open(os.path.join(tmp_path, "stream.json")))
    ids = [int(g) for d in got for g in d]
    assert sorted(ids) == list(range(6)) and len(set(ids)) == 6
    assert set(int(g) for g in got[0]) == {0, 2, 4} and set(int(g) for g in got[1]) == {1, 3, 5}
    ref = SynthRef(42, 400_000, 3)
    merged = {int(g): h for d in got for g, h in d.items()}
    for g in range(6):
        assert merged[g] == hashlib.sha256(bench.stream_reads(ref, g, 300).seq.tobytes()).hexdigest()
    assert len(set(merged.values())) == 6
