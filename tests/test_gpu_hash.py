"""GPU parity of the HASH reference-index path (SURVEY.md section 8(f) 3,
configs[3]) against the CPU restatement oracle/hash_oracle.c: the `.hash`
file byte for byte (small K and the default K = 14), and every read's
alignment (mismatch count, strand, position, mismatch offsets and types).
Parity with SeqArc itself is unpinned."""
import numpy as np
import pytest

import fastqueeze_amd as fq
import oracle_py as orc

pytestmark = pytest.mark.gpu

COMP = bytes.maketrans(b"ACGTN", b"TGCAN")


def genome(n, seed):
    rng = np.random.default_rng(seed)
    return np.frombuffer(b"ACGT", dtype=np.uint8)[rng.integers(0, 4, n)].tobytes()


def fasta(chroms, width=60):
    out = []
    for i, c in enumerate(chroms):
        out.append(b">chr%d\n" % (i + 1))
        out += [c[j:j + width] + b"\n" for j in range(0, len(c), width)]
    return b"".join(out)


@pytest.fixture(scope="module")
def enc():
    e = fq.Encoder(0)
    yield e
    e.close()


def reads_from(g, n, seed, lens=(36, 50, 75, 100, 150)):
    rng = np.random.default_rng(seed)
    out = []
    for i in range(n):
        L = int(rng.choice(lens))
        p = int(rng.integers(0, len(g) - L))
        r = bytearray(g[p:p + L])
        for a in rng.integers(0, L, int(rng.integers(0, 10))):   # 0..9 substitutions: some exceed maxmis
            r[a] = b"ACGT"[(b"ACGT".index(r[a]) + 1 + int(rng.integers(0, 3))) % 4]
        if i % 5 == 0:
            r[int(rng.integers(0, L))] = ord("N")
        if i % 11 == 0:
            r[int(rng.integers(0, L))] = ord("R")
        r = bytes(r)
        out.append(r.translate(COMP)[::-1] if i % 2 else r)
    out += [genome(150, 99), b"N" * 20 + genome(80, 98), g[1000:1100].lower(), b"ACGT" * 40]
    return out


@pytest.mark.parametrize("k,step,cap", [(8, 2, 1 << 16), (10, 1, 64), (14, 2, 1 << 16)])
def test_index_file_identical(enc, k, step, cap):
    chroms = [genome(300_000, 1), b"ACGTNNNNN" + genome(40_000, 2) + b"nnnn", (b"ACGTAC" * 400) + genome(5_000, 3)]
    fa = fasta(chroms)
    want = orc.hash_index(fa, k=k, step=step, maxcount=cap)
    ix = fq.HashIndex(enc, fa, k=k, step=step, maxcount=cap)
    got = ix.file_bytes()
    ix.close()
    assert len(got) == len(want)
    assert got == want


@pytest.mark.parametrize("ai0", [0, -1])
def test_alignments_identical(enc, ai0):
    g = genome(1_000_000, 7)
    fa = fasta([g[:600_000], g[600_000:]])
    orc.hash_index(fa)
    ix = fq.HashIndex(enc, fa)
    reads = reads_from(g, 4000, 11)
    want = orc.hash_align(reads, ai_nmis=ai0)
    got = ix.align(reads, ai_nmis=ai0)
    ix.close()
    names = ["ret", "rev", "pos", "mispos", "mistype"]
    for nm, a, b in zip(names, got, want):
        bad = np.nonzero(a != b)[0] if a.ndim == 1 else np.nonzero((a != b).any(axis=1))[0]
        assert bad.size == 0, (nm, bad[:5], a[bad[:5]], b[bad[:5]])
    aligned = (want[0] >= 0).sum()
    assert aligned > 2000          # most reads with <= 7 substitutions align back


def test_empty_and_short_inputs(enc):
    fa = fasta([genome(20_000, 5)])
    orc.hash_index(fa)
    ix = fq.HashIndex(enc, fa)
    reads = [b"A", b"ACGTACGTACGTAC", b"", b"ACGTN"]
    want = orc.hash_align([r for r in reads if r])
    got = ix.align([r for r in reads if r])
    for a, b in zip(got, want):
        assert np.array_equal(a, b)
    ix.close()


def test_long_reads_identical(enc):
    """Reads beyond the row kernel's 512 bp (one lane of their row walks them,
    sa_hash.hip align_read_serial) mixed with short ones in one launch."""
    g = genome(1_000_000, 17)
    fa = fasta([g])
    orc.hash_index(fa)
    ix = fq.HashIndex(enc, fa)
    reads = reads_from(g, 600, 19, lens=(150, 300, 511, 512, 513, 700, 1000, 5000))
    want = orc.hash_align(reads)
    got = ix.align(reads)
    ix.close()
    for nm, a, b in zip(["ret", "rev", "pos", "mispos", "mistype"], got, want):
        assert np.array_equal(a, b), nm
    lens = np.array([len(r) for r in reads])
    assert ((want[0] >= 0) & (lens > 512)).sum() > 50   # long reads aligned, not only refused
