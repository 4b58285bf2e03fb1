"""CPU checks of the HASH-index oracle (oracle/hash_oracle.c; SURVEY.md
section 8(f) 3): the index layout against a direct Python count of the same
sampled seeds, and reads cut from the reference (forward and reverse
complement, with substitutions and an N) aligning back to where they came from
with the listed mismatches.  Parity with SeqArc itself is unpinned (DESIGN.md
section 9): the reference ships no index or alignment to compare with."""
import numpy as np
import pytest

import oracle_py as orc

COMP = bytes.maketrans(b"ACGT", b"TGCA")


def genome(n, seed):
    rng = np.random.default_rng(seed)
    return np.frombuffer(b"ACGT", dtype=np.uint8)[rng.integers(0, 4, n)].tobytes()


def fasta(chroms, width=60):
    out = []
    for i, c in enumerate(chroms):
        out.append(b">chr%d test\n" % (i + 1))
        out += [c[j:j + width] + b"\n" for j in range(0, len(c), width)]
    return b"".join(out)


def parse_index(blob, k):
    K, total, nwords, npos = np.frombuffer(blob[:16], dtype=np.uint32)
    nk = 4 ** k
    a = np.frombuffer(blob[16:], dtype=np.uint32)
    seq, num, ind, pos = a[:nwords], a[nwords:nwords + nk], a[nwords + nk:nwords + 2 * nk], a[nwords + 2 * nk:]
    assert K == k and len(pos) == npos
    return int(total), seq, num, ind, pos


def test_index_layout_small_k():
    k = 8
    chroms = [genome(5000, 1), b"ACGTNNNN" + genome(3000, 2), genome(17, 3)]
    blob = orc.hash_index(fasta(chroms), k=k, step=2, maxcount=1 << 16)
    total, seq, num, ind, pos = parse_index(blob, k)
    cat = b"".join(chroms)
    assert total == len(cat)
    # packed sequence: 16 bases a word, N -> A, last word left-aligned
    codes = np.frombuffer(cat.translate(bytes.maketrans(b"ACGTN", b"\0\1\2\3\0")), dtype=np.uint8)
    pad = (-len(codes)) % 16
    c2 = np.concatenate([codes, np.zeros(pad, dtype=np.uint8)]).reshape(-1, 16).astype(np.uint64)
    words = np.zeros(len(c2), dtype=np.uint64)
    for j in range(16):
        words = (words << np.uint64(2)) | c2[:, j]
    assert np.array_equal(seq, words.astype(np.uint32))
    # seeds: K-mers ending at 1-based p with p % step == 0 and no N among them
    # (the K-mer runs across chromosome boundaries, as the reference's does)
    want = {}
    for p in range(k, len(cat) + 1):
        w = cat[p - k:p]
        if p % 2 == 0 and b"N" not in w:
            v = 0
            for ch in w:
                v = v * 4 + b"ACGT".index(ch)
            want.setdefault(v, []).append(p - k + 1)
    for v, ps in want.items():
        assert num[v] == len(ps)
        assert list(pos[ind[v]:ind[v] + num[v]]) == ps
    assert int(num.sum()) == sum(map(len, want.values()))


def test_index_cap_drops_repeats():
    k = 6
    rep = b"ACGTAC" * 50
    blob = orc.hash_index(fasta([rep + genome(4000, 5)]), k=k, step=1, maxcount=16)
    _, _, num, ind, pos = parse_index(blob, k)
    v = 0
    for ch in b"ACGTAC":
        v = v * 4 + b"ACGT".index(ch)
    assert num[v] == 0 and (num < 16).all()


def test_reads_align_back():
    g = genome(200_000, 7)
    orc.hash_index(fasta([g]))
    rng = np.random.default_rng(11)
    reads, truth = [], []
    for i in range(300):
        L = int(rng.choice([50, 100, 150]))
        p = int(rng.integers(0, len(g) - L))
        r = bytearray(g[p:p + L])
        nmut = int(rng.integers(0, 4))
        at = sorted(set(int(x) for x in rng.integers(0, L, nmut)))
        for a in at:
            r[a] = b"ACGT"[(b"ACGT".index(r[a]) + 1 + int(rng.integers(0, 3))) % 4]
        if i % 7 == 0:
            r[L // 2] = ord("N")
            at = sorted(set(at) | {L // 2})
        rc = i % 2 == 1
        reads.append(bytes(r).translate(COMP)[::-1] if rc else bytes(r))
        truth.append((p + 1, rc, at))
    ret, rev, pos, mp, mt = orc.hash_align(reads)
    ok = 0
    for i, (p, rc, at) in enumerate(truth):
        if ret[i] < 0:
            continue
        assert rev[i] == rc and pos[i] == p, (i, ret[i], rev[i], pos[i], truth[i])
        got = [x for x in mp[i] if x >= 0]
        # (reverse strand: the aligned sequence is the read's reverse
        # complement, i.e. the reference segment: offsets along it)
        assert got == at
        assert ret[i] == len(at)
        ok += 1
    assert ok >= 290


def test_unalignable_reads():
    orc.hash_index(fasta([genome(50_000, 9)]))
    far = genome(150, 12345)
    many_n = b"N" * 10 + genome(140, 4)
    ret, *_ = orc.hash_align([far, many_n, b"ACGT" * 30])
    assert ret[1] == -1          # more N than maxmis
    assert ret[0] == -1 and ret[2] == -1


def test_unwrapped_chromosome_line():
    """A chromosome on one FASTA line (the seed buffer was flushed
    only between lines): 36 M bases give 18 M sampled seeds in that line, more
    than the oracle's 2^24-entry buffer.  Line wrapping does not change the
    index (positions count bases, the reference's getdelim loop keeps the
    K-mer across lines), so the unwrapped FASTA's index equals the wrapped
    one's."""
    k = 10
    chroms = [genome(36_000_000, 11), genome(300_000, 12)]
    wrapped = orc.hash_index(fasta(chroms), k=k, step=2, maxcount=1 << 16)
    one_line = orc.hash_index(fasta(chroms, width=1 << 40), k=k, step=2, maxcount=1 << 16)
    assert one_line == wrapped
    total, _, num, _, pos = parse_index(one_line, k)
    assert total == 36_300_000 and len(pos) > (1 << 24)
