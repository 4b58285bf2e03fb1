"""Multi-GPU path on the CPU: `bench.py --gpus 2 --dry-run` launches two ranks
itself (its --gpus launcher), the ranks join a gloo group, deal the global
batches with fastqueeze_amd.shard.shard_indices, encode their share and gather
the per-block digests back in global order with shard.gather_blocks -- the code
the GPU bench runs, with the CPU restatement standing in for the GPU encoder
(dry run only; the product path has no CPU encoder)."""
import json
import os
import subprocess
import sys

import pytest

from fastqueeze_amd.shard import shard_indices

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_shard_indices_cover_every_block_once():
    for n in (0, 1, 5, 69):
        for world in (1, 2, 3, 8):
            got = sorted(i for r in range(world) for i in shard_indices(n, r, world))
            assert got == list(range(n))
    with pytest.raises(ValueError):
        shard_indices(4, 2, 2)


def _bench(*args):
    env = {k: v for k, v in os.environ.items() if k not in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "MASTER_PORT")}
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--dry-run", "--pairs", "2000", *args],
                       capture_output=True, text=True, timeout=600, env=env)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout
    return json.loads(lines[0])


def test_bench_gpus2_launches_two_gloo_ranks_and_gathers_in_order():
    one = _bench("--gpus", "1", "--batches", "4")
    two = _bench("--gpus", "2", "--batches", "2")
    assert one["n_gpus"] == 1 and two["n_gpus"] == 2
    assert one["batches"] == two["batches"] == 4
    # the same global batches, encoded on two ranks and gathered in order
    assert one["blocks_digest"] == two["blocks_digest"]
    # the whole-node end-to-end leg: rank 0's first batch, 2 x 2 times over, through one
    # seqarc_amd --devices 2 (here --ingest-only: the reader and the cut dealing batches)
    e2e = two["end_to_end"]
    assert e2e["devices"] == 2 and "--devices 2" in e2e["command"] and e2e["fastq_bytes"] > 0
    assert e2e["value"] > 0 and "block(s)" not in e2e["cli_stages"]
