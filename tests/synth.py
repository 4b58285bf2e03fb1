"""Deterministic synthetic FASTQ generator (SURVEY.md section 8(d) spec).

Test / bench infrastructure.  Genome of 5,000,000 uniform random bases; fragments
with uniform start and insert 250-449; r1 = forward read, r2 = reverse complement
of the fragment end; 0.2 % substitutions; qualities from {F, :, ,} with
p = {0.90, 0.07, 0.03}; 0.05 % N on r1 with quality '#'; Illumina-style headers
whose mate IDs differ (`1:N:0:` / `2:N:0:`), which keeps the reference out of its
identical-mate-ID PE livelock (defect i).
"""
from __future__ import annotations

import numpy as np

_COMP = np.frombuffer(b"TGCA", dtype=np.uint8)  # complement of ACGT by code
_BASES = np.frombuffer(b"ACGT", dtype=np.uint8)
_QUALS = np.frombuffer(b"F:,", dtype=np.uint8)


def _headers(rng: np.random.Generator, start: int, n: int, mate: int) -> list[bytes]:
    # tiles of 4000 reads; y increases within a tile, x random (variable width)
    idx = np.arange(start, start + n)
    tile = 1101 + (idx // 4000) % 78
    y = 1000 + (idx % 4000) * 8
    x = rng.integers(1000, 32000, size=n)
    return [
        b"@A00123:8:H5KJ2DSXX:1:%d:%d:%d %d:N:0:ACGTACGT" % (t, xx, yy, mate)
        for t, xx, yy in zip(tile.tolist(), x.tolist(), y.tolist())
    ]


def _records(names: list[bytes], seq: np.ndarray, qual: np.ndarray) -> bytes:
    L = seq.shape[1]
    n = seq.shape[0]
    body = np.empty((n, 2 * L + 4), dtype=np.uint8)
    body[:, 0] = ord("\n")
    body[:, 1 : L + 1] = seq
    body[:, L + 1] = ord("\n")
    body[:, L + 2] = ord("+")
    body[:, L + 3] = ord("\n")
    body[:, L + 4 :] = qual
    tail = b"\n"
    bodies = body.tobytes()
    w = 2 * L + 4
    return b"".join(nm + bodies[i * w : (i + 1) * w] + tail for i, nm in enumerate(names))


def generate(n_reads: int, read_len: int = 150, paired: bool = False, seed: int = 12345,
             genome_len: int = 5_000_000, chunk: int = 250_000, progress=None):
    """Return (r1_bytes, r2_bytes or None) of n_reads records (pairs if paired)."""
    rng = np.random.default_rng(seed)
    genome = rng.integers(0, 4, size=genome_len, dtype=np.uint8)
    out1: list[bytes] = []
    out2: list[bytes] = []
    ar = np.arange(read_len)
    for s in range(0, n_reads, chunk):
        n = min(chunk, n_reads - s)
        start = rng.integers(0, genome_len - max(450, read_len), size=n)
        ins = rng.integers(250, 450, size=n)
        r1 = genome[start[:, None] + ar[None, :]]
        sub = rng.random((n, read_len)) < 0.002
        r1 = np.where(sub, (r1 + rng.integers(1, 4, size=(n, read_len), dtype=np.uint8)) % 4, r1)
        s1 = _BASES[r1]
        q1 = _QUALS[rng.choice(3, size=(n, read_len), p=[0.90, 0.07, 0.03])]
        nmask = rng.random((n, read_len)) < 0.0005
        s1 = np.where(nmask, np.uint8(ord("N")), s1)
        q1 = np.where(nmask, np.uint8(ord("#")), q1)
        out1.append(_records(_headers(rng, s, n, 1), s1, q1))
        if paired:
            end = start + ins
            r2 = genome[(end - read_len)[:, None] + ar[None, :]][:, ::-1]
            sub2 = rng.random((n, read_len)) < 0.002
            r2 = np.where(sub2, (r2 + rng.integers(1, 4, size=(n, read_len), dtype=np.uint8)) % 4, r2)
            s2 = _COMP[r2]
            q2 = _QUALS[rng.choice(3, size=(n, read_len), p=[0.90, 0.07, 0.03])]
            out2.append(_records(_headers(rng, s, n, 2), s2, q2))
        if progress is not None and (s // chunk) % 40 == 39:
            progress(s + n)
    return b"".join(out1), (b"".join(out2) if paired else None)


def edge_cases() -> bytes:
    """Small SE FASTQ exercising the reference's edge paths: lowercase and IUPAC
    bases, all-N reads, trailing and all-'#' qualities, empty reads, variable
    read and name lengths, ':' and ' ' in names (tokenizer realignment)."""
    recs = [
        (b"r1", b"ACGTNNACGTacgtRYKM", b"IIII##IIIIIIII####"),
        (b"r1 extra:field", b"NNNNNNNN", b"########"),
        (b"r2:1:22", b"", b""),
        (b"r22:1:2 x", b"ACGTACGTACGTSWHBVD", b"ABCDEFGHIJKLMNOPQR"),
        (b"read:with:colons", b"GATTACA", b"#######"),
        (b"read:with:colons:and:more", b"GATTACAGATTACA", b"!!!!!!!!!!!!!!"),
        (b"x", b"N", b"5"),
        (b"", b"ACGT", b"~~~~"),
        (b"a:b c:d", b"ACNGTNNA", b"I#I#I##I"),
    ]
    for i in range(40):
        nm = b"tok:%d:%d %d" % (i, i * 37 % 1000, i % 3)
        s = (b"ACGTN"[i % 5:] + b"ACGTTGCA" * (i % 7 + 1))[: 3 + i]
        q = bytes((33 + (j * 7 + i) % 41) for j in range(len(s)))
        if i % 4 == 0 and len(q) > 2:
            q = q[:-2] + b"##"
        recs.append((nm, s, q))
    return b"".join(b"@" + n + b"\n" + s + b"\n+\n" + q + b"\n" for n, s, q in recs)
