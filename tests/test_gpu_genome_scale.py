"""configs[3] at genome scale: the HASH path on
a synthetic genome longer than 2^31 bases.  GRCh38 (3.1 Gb) puts reference
positions above 2^31, `shift = bits(genome) - 2 = 30` (HashAlignment::
loadRefIndex@0x40fe9b; compressOrder@0x424b70's order byte (pos >> shift) + 1)
and 30-bit position fields (int2bit@0x40dcd0 in compressAlignInfo_Pos@0x425d70):
a signed 32-bit position or a width bug on the device would show only there.

One test, its own timeout: the index of a 2^31 + 100 Mb genome built on the
GPU (sa_hash_build) and by the CPU restatement (oracle/hash_oracle.c), the
`.hash` files compared byte for byte; a sample of reads aligned by both; one
full 50 MiB PE block of reads drawn from beyond 2^31 encoded on the GPU
(sa_run_input_aligned) byte-equal to the oracle's encode_block_hash.  Parity
with SeqArc itself is unpinned."""
import numpy as np
import pytest

import fastqueeze_amd as fq
import oracle_py as orc
import synth

pytestmark = pytest.mark.gpu

GLEN = (1 << 31) + 100_000_000   # 2.247 Gb: bits(GLEN) = 32, shift 30, as GRCh38's 3.1 Gb


def first_difference(a: np.ndarray, b: np.ndarray, chunk: int = 1 << 28) -> int:
    """Index of the first differing byte of two uint8 arrays (-1: equal)."""
    if a.size != b.size:
        return min(a.size, b.size)
    for s in range(0, a.size, chunk):
        x, y = a[s:s + chunk], b[s:s + chunk]
        if not np.array_equal(x, y):
            return s + int(np.flatnonzero(x != y)[0])
    return -1


@pytest.mark.timeout(240)
def test_hash_path_beyond_2_31():
    fa, g = synth.big_reference(GLEN, 2031, chroms=3)
    enc = fq.Encoder(0)
    ix = None
    try:
        ix = fq.HashIndex(enc, fa)
        assert ix.genome_length == GLEN
        got = ix.file_array()
        want = orc.hash_index_array(fa)   # (the oracle keeps this index for the encodes below)
        del fa
        k = first_difference(got, want)
        assert k < 0, f".hash files differ at byte {k} of {want.size}"
        hdr = want[:16].view(np.uint32)
        npos, nwords = int(hdr[3]), int(hdr[2])
        positions = want[16 + 4 * (nwords + 2 * (1 << 28)):].view(np.uint32)
        assert positions.size == npos and int(positions.max()) > (1 << 31)   # seeds beyond 2^31 indexed
        del got, want, positions

        # reads drawn from beyond 2^31 (mates too), both strands, mismatches, N runs
        r1, r2 = synth.aligned_reads(g, 80_000, 2032, paired=True, random_frac=0.02, far_frac=0.02, lo=1 << 31)
        del g
        blocks = fq.blocks_from_fastq(r1, r2)
        assert blocks[0].nreads > 100_000   # a full 50 MiB block

        # the aligner on a sample: GPU against the oracle, positions beyond 2^31
        sample = [r for r in r1.split(b"\n")[1::4][:3000]]
        ga = ix.align(sample)
        oa = orc.hash_align(sample)
        for name, x, y in zip(("ret", "rev", "pos", "mispos", "mistype"), ga, oa):
            assert np.array_equal(x, y), f"aligner {name} differs"
        ok = ga[0] >= 0   # (synth.aligned_reads: 0-10 substitutions, a fifth beyond maxmis 7, 2 % random)
        assert ok.mean() > 0.7 and (ga[2][ok] > (1 << 31)).all()

        cfg = fq.Config()
        got_blk = enc.encode_aligned(blocks[:1], cfg, ix, True)
        carry = [0, 0]
        want_blk = [orc.encode_block_hash(blocks[0], True, carry)]
        assert len(got_blk[0]) == len(want_blk[0]), f"{len(got_blk[0])} vs {len(want_blk[0])} bytes"
        k = first_difference(np.frombuffer(got_blk[0], np.uint8), np.frombuffer(want_blk[0], np.uint8))
        assert k < 0, f"aligned block differs at byte {k}"
    finally:
        if ix is not None:
            ix.close()
        enc.close()
