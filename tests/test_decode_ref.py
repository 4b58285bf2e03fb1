"""Round trip of the reference (HASH index) path on the CPU: blocks encoded by
the oracle's doAlign + doAlignEncode restatement decode with the library's
host decoder (sa_decode_block_ref: decompressSeq@0x42e390, getRealPos@0x42de30,
AlignInfoToSeq@0x42e020) back to the input reads, MD5s included.  (The reads
are upper case: aligned bases come back from the genome in upper case, as in
the reference.)"""
import numpy as np
import pytest

import fastqueeze_amd as fq
import oracle_py as orc
import synth


@pytest.fixture(scope="module")
def ref():
    fa, g = synth.reference(1_500_000, 41, chroms=2)
    fa = fa.upper()
    return fa, g, orc.hash_index(fa)


@pytest.mark.parametrize("paired,kw", [(False, {}), (True, {}), (True, {"insert_size": 300}),
                                       (False, {"maxmis": 8}), (False, {"maxmis": 0})])
def test_round_trip(ref, paired, kw):
    fa, g, hfile = ref
    words, bases = fq.hash_file_genome(hfile)
    r1, r2 = synth.aligned_reads(g, 3000, 42, paired=paired, random_frac=0.2, far_frac=0.3, short_frac=0.3)
    blocks = fq.blocks_from_fastq(r1, r2, block_size=200_000)
    carry = [0, 0]
    for b in blocks:
        enc = orc.encode_block_hash(b, paired, carry, **kw)
        got, ok = fq.decode_block(enc, b.text_bytes or b.text1 + b.text2,
                                  ref=(words, bases, paired, kw.get("maxmis", 7), kw.get("insert_size", 0)))
        assert ok
        assert np.array_equal(got.seq_lens, b.seq_lens)
        assert got.seq.tobytes() == b.seq.tobytes()
        assert got.qual.tobytes() == b.qual.tobytes() and got.names.tobytes() == b.names.tobytes()
