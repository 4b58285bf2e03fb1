"""Block sharding over GPUs.

Every model of the encoder is re-initialised per block (compressSeq@0x424934,
compressQual@0x426f10, compressLen_short@0x423f80, kModelInit), so blocks are
independent units: block i goes to rank i mod world, each rank encodes its
blocks on its own GPU (one process per GPU, `Encoder(local_rank)`), and the
encoded blocks are gathered back in input order.  There is no data-path
collective; the gather is a plain exchange of finished blocks (the reference's
writer thread likewise emits blocks as its encode threads finish them).
"""
from __future__ import annotations

from typing import Callable, Sequence


def shard_indices(nblocks: int, rank: int, world: int) -> list[int]:
    """Indices of the blocks rank `rank` encodes (round robin)."""
    if world < 1 or not 0 <= rank < world:
        raise ValueError(f"rank {rank} outside world of {world}")
    return list(range(rank, nblocks, world))


def encode_shard(blocks: Sequence, rank: int, world: int, encode: Callable[[list], list[bytes]]):
    """Encodes this rank's blocks with `encode` (e.g. `Encoder(local).encode(bl, cfg)`);
    returns [(block index, encoded bytes)]."""
    idx = shard_indices(len(blocks), rank, world)
    outs = encode([blocks[i] for i in idx]) if idx else []
    if len(outs) != len(idx):
        raise RuntimeError("encoder returned a different number of blocks")
    return list(zip(idx, outs))


def gather_blocks(local: list[tuple[int, bytes]], nblocks: int, group=None) -> list[bytes]:
    """All ranks' (index, bytes) pairs back in input order (torch.distributed
    all_gather_object over any backend; every rank gets the full list)."""
    import torch.distributed as dist

    world = dist.get_world_size(group)
    parts: list = [None] * world
    dist.all_gather_object(parts, local, group=group)
    out: list[bytes | None] = [None] * nblocks
    for part in parts:
        for i, b in part:
            if out[i] is not None:
                raise RuntimeError(f"block {i} encoded twice")
            out[i] = b
    missing = [i for i, b in enumerate(out) if b is None]
    if missing:
        raise RuntimeError(f"blocks {missing[:8]} not encoded by any rank")
    return out  # type: ignore[return-value]
