"""The multi-GPU path of bench.py on the CPU: world_size-2 `gloo` process
group standing in for RCCL.  bench.py's data path has exactly one
collective — the start-up broadcast of the packed reference + contig table
from rank 0 — and the whole-job totals (max time, summed
reads) at the end; shards are independent (weak scaling)."""
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


def test_shards_are_deterministic():
    import bench
    from bwagpu.synth import SynthRef
    ref = SynthRef(42, 300_000, 3)
    a = bench.rank_reads(ref, 1, 200, 150)
    b = bench.rank_reads(ref, 1, 200, 150)
    assert np.array_equal(a.seq, b.seq) and np.array_equal(a.seeds, b.seeds)
