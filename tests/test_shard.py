"""Multi-GPU path on the CPU: world_size-2 gloo ranks shard blocks round-robin,
encode their share and gather them back in order (fastqueeze_amd/shard.py).
Without a GPU the ranks encode with the CPU restatement (test infrastructure);
the sharding and the gather are the code bench.py / a multi-GPU host runs."""
import os
import socket

import pytest
import torch.distributed as dist
import torch.multiprocessing as mp

import oracle_py
import synth

from fastqueeze_amd import blocks_from_fastq
from fastqueeze_amd.shard import encode_shard, gather_blocks, shard_indices

BLOCK = 300_000


def _free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _oracle_encode(bl):
    return [oracle_py.encode_block(b, 3, 2, 1, 0) for b in bl]


def _rank(rank, world, port, text, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        blocks = blocks_from_fastq(text, None, BLOCK)
        local = encode_shard(blocks, rank, world, _oracle_encode)
        assert [i for i, _ in local] == shard_indices(len(blocks), rank, world)
        out = gather_blocks(local, len(blocks))
        q.put((rank, [len(b) for b in out], b"".join(out)))
    finally:
        dist.destroy_process_group()


def test_shard_indices_cover_every_block_once():
    for n in (0, 1, 5, 69):
        for world in (1, 2, 3, 8):
            got = sorted(i for r in range(world) for i in shard_indices(n, r, world))
            assert got == list(range(n))
    with pytest.raises(ValueError):
        shard_indices(4, 2, 2)


def test_two_gloo_ranks_gather_blocks_in_order():
    text, _ = synth.generate(4000, seed=21)
    blocks = blocks_from_fastq(text, None, BLOCK)
    assert len(blocks) >= 3
    want = _oracle_encode(blocks)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_rank, args=(r, 2, port, text, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = [q.get(timeout=300) for _ in procs]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for rank, lens, blob in res:
        assert lens == [len(w) for w in want], rank
        assert blob == b"".join(want), rank
