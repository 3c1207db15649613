"""The multi-rank path on one GPU box: two ranks (gloo process group; both on
cuda:0) share the work the way bench.py does — rank 0 holds the reference and
broadcasts the packed pac + contig table, each rank runs its own shard of
ChainsRecords through the engine — and the union of the shards' regions must
equal a single-rank run (the reference's golden regions)."""
import os
import socket
import sys

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, out_dir):
    for p in (os.path.join(REPO, "bwa-flow_amd", "python"), os.path.join(REPO, "tests")):
        sys.path.insert(0, p)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import golden_io as G
    from bwagpu.engine import Engine, compact
    opt, batch, _, _ = G.load_chain_set("c1_default")
    if rank == 0:
        refd = G.load_ref()
        pac = torch.from_numpy(np.asarray(refd["pac"], np.uint8).copy())
        ann = torch.from_numpy(np.concatenate([refd["ann_offset"], np.asarray(refd["ann_len"], np.int64)]))
        meta = torch.tensor([refd["l_pac"], len(refd["pac"]), len(refd["ann_len"])], dtype=torch.int64)
    else:
        meta = torch.zeros(3, dtype=torch.int64)
    dist.broadcast(meta, src=0)
    l_pac, npac, nseq = (int(x) for x in meta.tolist())
    if rank != 0:
        pac = torch.zeros(npac, dtype=torch.uint8)
        ann = torch.zeros(2 * nseq, dtype=torch.int64)
    dist.broadcast(pac, src=0)  # the one start-up collective
    dist.broadcast(ann, src=0)
    a = ann.numpy()
    eng = Engine(0, opt, l_pac, a[:nseq].copy(), a[nseq:].astype(np.int32), pac=pac.numpy())
    # records of 100 reads; rank r takes records r, r + world, ...
    per = 100
    recs = [range(r0, min(r0 + per, batch.n_reads)) for r0 in range(0, batch.n_reads, per)]
    mine = {}
    for k in range(rank, len(recs), world):
        sub = batch.subset(recs[k])
        regs, n = eng.chain2aln(sub)
        mine[k] = (compact(sub, regs, n).view(np.uint8).tobytes(), n.tolist())
    eng.close()
    gathered = [None] * world
    dist.all_gather_object(gathered, mine)
    if rank == 0:
        merged = {}
        for g in gathered:
            merged.update(g)
        regs = b"".join(merged[k][0] for k in range(len(recs)))
        n = sum((merged[k][1] for k in range(len(recs))), [])
        np.save(os.path.join(out_dir, "n.npy"), np.array(n, np.int32))
        open(os.path.join(out_dir, "regs.bin"), "wb").write(regs)
        np.save(os.path.join(out_dir, "owners.npy"), np.array([len(g) for g in gathered]))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.gpu
def test_two_rank_shards_merge_to_single_rank(tmp_path):
    import golden_io as G
    from bwagpu import abi
    world = 2
    mp.spawn(_worker, args=(world, _free_port(), str(tmp_path)), nprocs=world, join=True)
    _, batch, want_regs, want_n = G.load_chain_set("c1_default")
    n = np.load(os.path.join(tmp_path, "n.npy"))
    regs = np.frombuffer(open(os.path.join(tmp_path, "regs.bin"), "rb").read(), np.uint8).view(abi.ALNREG_DTYPE)
    owners = np.load(os.path.join(tmp_path, "owners.npy"))
    assert all(o > 0 for o in owners)  # both ranks processed records
    assert np.array_equal(n, want_n)
    assert G.region_mismatch(regs, want_regs) is None


def _worker_stream(rank, world, port, out_dir):
    """bench.py's stream path on one GPU with two ranks: rank r takes global
    batches r, r + 2 (bench.shard_ids), makes their chains with the device's
    SeqsToChains (bench.stream_batches) and their regions with the device's
    ChainsToRegions, and checks both against the oracle restatement (chains:
    oracle/chain.c, pinned by the reference's chain dumps; regions: the
    oracle's mem_chain2aln); rank 0 gathers every batch's regions"""
    for p in (os.path.join(REPO, "bwa-flow_amd", "python"), os.path.join(REPO, "tests"), REPO,
              os.path.join(REPO, "oracle")):
        sys.path.insert(0, p)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import hashlib
    import bench
    import golden_io as G
    import oracle
    from bwagpu import abi
    from bwagpu.engine import Engine, compact
    dev = torch.device("cuda:0")
    refd = G.load_ref() if rank == 0 else None

    class Src:
        pass
    if rank == 0:
        Src.l_pac, Src.pac, Src.ann_offset, Src.ann_len = refd["l_pac"], refd["pac"], refd["ann_offset"], refd["ann_len"]
    ref, pac_t = bench.broadcast_reference(Src if rank == 0 else None, rank, world, torch.device("cpu"))
    pac_d = torch.from_numpy(np.ascontiguousarray(ref.pac)).to(dev)
    hdr, words = G.load_seed_bwt()
    sa_intv, sa, _, _ = G.load_seed_sa()
    opt = abi.default_opt()
    gids = bench.shard_ids(rank, world, 2)
    batches, _ = bench.stream_batches(dev, opt, ref, pac_d, (hdr, words, sa, sa_intv), gids, pairs=400)
    R = oracle.Ref(ref.l_pac, ref.ann_offset, ref.ann_len, ref.pac)
    eng = Engine(0, opt, ref.l_pac, ref.ann_offset, ref.ann_len, pac=ref.pac)
    mine, ok = {}, True
    for g, b in zip(gids, batches):
        rco, ch, cso, sd = oracle.seqs2chains(opt, abi.default_chainopt(), np.array([19, 10, 20], np.int32), 1.5, R,
                                              None, hdr, words, sa, sa_intv, b.seq_off, b.seq)
        ok &= bool(np.array_equal(rco, b.read_chain_off) and np.array_equal(cso, b.chain_seed_off) and
                   np.array_equal(ch["rid"], b.chain_rid) and
                   all(np.array_equal(sd[f], b.seeds[f]) for f in ("rbeg", "qbeg", "len", "score")))
        regs, n = eng.chain2aln(b)
        oregs, on, _ = oracle.chain2aln("oracle", opt, R, b)
        got = compact(b, regs, n)
        ok &= bool(np.array_equal(n, on) and np.array_equal(got.view(np.uint8), compact(b, oregs, on).view(np.uint8)))
        mine[g] = hashlib.sha256(got.view(np.uint8).tobytes()).hexdigest()
    eng.close()
    gathered = [None] * world
    dist.all_gather_object(gathered, (mine, ok))
    if rank == 0:
        import json
        json.dump(gathered, open(os.path.join(out_dir, "stream.json"), "w"))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.gpu
def test_two_rank_stream_shards(tmp_path):
    """the shards are disjoint, cover the stream, and every batch's chains and
    regions equal the oracle's on whichever rank ran it"""
    import json
    world = 2
    mp.spawn(_worker_stream, args=(world, _free_port(), str(tmp_path)), nprocs=world, join=True)
    got = json.load(open(os.path.join(tmp_path, "stream.json")))
    ids = [int(g) for mine, _ in got for g in mine]
    assert sorted(ids) == [0, 1, 2, 3]
    assert all(ok for _, ok in got)
    assert len({h for mine, _ in got for h in mine.values()}) == 4
