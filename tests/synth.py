"""Deterministic synthetic FASTQ generator (SURVEY.md section 8(d) spec).

Test / bench infrastructure.  Genome of 5,000,000 uniform random bases; fragments
with uniform start and insert 250-449; r1 = forward read, r2 = reverse complement
of the fragment end; 0.2 % substitutions; qualities from {F, :, ,} with
p = {0.90, 0.07, 0.03}; 0.05 % N on r1 with quality '#'; Illumina-style headers
`@A00123:8:H5KJ2DSXX:1:<tile>:<x>:<y> {1|2}:N:0:ACGTACGT`: both mates of a pair
carry the same tile:x:y (as a sequencer writes them) and differ only in the
`1:`/`2:` comment, which keeps the reference out of its identical-mate-ID PE
livelock (defect i).

Chunks of `chunk` records are drawn from their own generator (seed, chunk index),
so the output does not depend on how many worker processes produce it.
Qualities are drawn as 16-bit integers (p = k / 65536, within 1e-5 of the spec);
substitutions and N are placed at a binomial number of uniform positions.
"""
from __future__ import annotations

import numpy as np

_COMP = np.frombuffer(b"TGCA", dtype=np.uint8)  # complement of ACGT by code
_BASES = np.frombuffer(b"ACGT", dtype=np.uint8)
_QUALS = np.frombuffer(b"F:,", dtype=np.uint8)
_Q1, _Q2 = 58982, 63570        # 0.90, 0.97 of 65536 -> 'F' / ':' / ','
_SUB = 131                     # 0.002 of 65536
_NRATE = 33                    # 0.0005 of 65536

_genome_cache: dict = {}


def _genome(seed: int, genome_len: int) -> np.ndarray:
    key = (seed, genome_len)
    g = _genome_cache.get(key)
    if g is None:
        g = np.random.default_rng(seed).integers(0, 4, size=genome_len, dtype=np.uint8)
        _genome_cache.clear()
        _genome_cache[key] = g
    return g


def _headers(start: int, x: np.ndarray, mate: int) -> list[bytes]:
    # tiles of 4000 reads; y increases within a tile, x random (variable width)
    n = x.shape[0]
    idx = np.arange(start, start + n)
    tile = 1101 + (idx // 4000) % 78
    y = 1000 + (idx % 4000) * 8
    return [
        b"@A00123:8:H5KJ2DSXX:1:%d:%d:%d %d:N:0:ACGTACGT" % (t, xx, yy, mate)
        for t, xx, yy in zip(tile.tolist(), x.tolist(), y.tolist())
    ]


def _records(names: list[bytes], seq: np.ndarray, qual: np.ndarray) -> bytes:
    L = seq.shape[1]
    n = seq.shape[0]
    body = np.empty((n, 2 * L + 5), dtype=np.uint8)
    body[:, 0] = ord("\n")
    body[:, 1 : L + 1] = seq
    body[:, L + 1] = ord("\n")
    body[:, L + 2] = ord("+")
    body[:, L + 3] = ord("\n")
    body[:, L + 4 : 2 * L + 4] = qual
    body[:, 2 * L + 4] = ord("\n")
    bodies = body.tobytes()
    w = 2 * L + 5
    return b"".join(nm + bodies[i * w : (i + 1) * w] for i, nm in enumerate(names))


def _sparse(rng: np.random.Generator, total: int, rate: float) -> np.ndarray:
    """Flat positions of a Bernoulli(rate) event over `total` cells (a binomial
    count of uniform positions; a repeated position counts once)."""
    return rng.integers(0, total, size=int(rng.binomial(total, rate)))


def _chunk(args):
    seed, ci, s, n, read_len, paired, genome_len, x_span = args
    genome = _genome(seed, genome_len)
    win = np.lib.stride_tricks.sliding_window_view(genome, read_len)
    rng = np.random.default_rng([seed, ci])
    start = rng.integers(0, genome_len - max(450, read_len), size=n)
    ins = rng.integers(250, 450, size=n)
    x = rng.integers(1000, 32000, size=n)
    if x_span:   # (the draw stays: every other byte is the same for any x_span)
        x = 1000 + (x - 1000) % x_span
    cells = n * read_len

    def quals():
        u = rng.bit_generator.random_raw((cells + 3) // 4).view(np.uint16)[:cells].reshape(n, read_len)
        return _QUALS[(u >= _Q1).astype(np.uint8) + (u >= _Q2)]

    def mutate(r):
        r = np.ascontiguousarray(r).reshape(-1)
        at = _sparse(rng, cells, _SUB / 65536)
        r[at] = (r[at] + rng.integers(1, 4, size=at.size, dtype=np.uint8)) & 3
        return r.reshape(n, read_len)

    s1 = _BASES[mutate(win[start])]
    q1 = quals()
    at = _sparse(rng, cells, _NRATE / 65536)
    s1.reshape(-1)[at] = ord("N")
    q1.reshape(-1)[at] = ord("#")
    out1 = _records(_headers(s, x, 1), s1, q1)
    out2 = None
    if paired:
        s2 = _COMP[mutate(win[start + ins - read_len][:, ::-1])]
        out2 = _records(_headers(s, x, 2), s2, quals())
    return out1, out2


def generate(n_reads: int, read_len: int = 150, paired: bool = False, seed: int = 12345,
             genome_len: int = 5_000_000, chunk: int = 250_000, progress=None, workers: int = 1,
             x_span: int = 0):
    """Return (r1_bytes, r2_bytes or None) of n_reads records (pairs if paired).
    workers > 1 draws the chunks in that many spawned processes (same bytes).
    x_span > 0 draws the header x coordinate from that many values (x_span = 8:
    a 50 MiB PE block's name stream is ~60 kB, near SURVEY 8's 58.7 kB; the
    default, uniform over 31000 values, gives ~195 kB)."""
    jobs = [(seed, ci, s, min(chunk, n_reads - s), read_len, paired, genome_len, x_span)
            for ci, s in enumerate(range(0, n_reads, chunk))]
    out1: list[bytes] = []
    out2: list[bytes] = []
    if workers > 1 and len(jobs) > 1:
        import multiprocessing as mp
        with mp.get_context("spawn").Pool(min(workers, len(jobs))) as pool:
            for k, (a, b) in enumerate(pool.imap(_chunk, jobs)):
                out1.append(a)
                if paired:
                    out2.append(b)
                if progress is not None and k % 40 == 39:
                    progress(jobs[k][2] + jobs[k][3])
    else:
        for k, job in enumerate(jobs):
            a, b = _chunk(job)
            out1.append(a)
            if paired:
                out2.append(b)
            if progress is not None and k % 40 == 39:
                progress(job[2] + job[3])
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


def reference(genome_len: int, seed: int, chroms: int = 3, width: int = 60) -> tuple[bytes, np.ndarray]:
    """FASTA of a random genome (`chroms` records, some lowercase and N runs)
    for the reference (HASH index) path, and its bases as uint8 ACGTN."""
    rng = np.random.default_rng([seed, 7])
    g = _BASES[rng.integers(0, 4, size=genome_len, dtype=np.uint8)].copy()
    for at in rng.integers(0, max(genome_len - 64, 1), size=max(genome_len // 200000, 1)):
        g[at:at + int(rng.integers(1, 40))] = ord("N")
    cuts = sorted(set(int(x) for x in rng.integers(1, genome_len, size=chroms - 1))) if chroms > 1 else []
    bounds = [0] + cuts + [genome_len]
    out = []
    for i in range(len(bounds) - 1):
        c = g[bounds[i]:bounds[i + 1]].tobytes()
        if i == 1:
            c = c.lower()
        out.append(b">chr%d synthetic\n" % (i + 1))
        out += [c[j:j + width] + b"\n" for j in range(0, len(c), width)]
    return b"".join(out), g


def big_reference(genome_len: int, seed: int, chroms: int = 3, width: int = 60) -> tuple[np.ndarray, np.ndarray]:
    """reference() at genome scale (numpy throughout, no per-line Python):
    FASTA as a uint8 array and the bases (ACGTN).  Random bases, N runs of
    1-39 every ~200 kb, the second record in lower case, `chroms` records of
    `width`-base lines."""
    rng = np.random.default_rng([seed, 8])
    g = _BASES[rng.integers(0, 4, size=genome_len, dtype=np.uint8)]
    at = rng.integers(0, max(genome_len - 64, 1), size=max(genome_len // 200000, 1))
    ln = rng.integers(1, 40, size=at.size)
    for a, l in zip(at.tolist(), ln.tolist()):
        g[a:a + l] = ord("N")
    cuts = sorted(set(int(x) for x in rng.integers(1, genome_len, size=chroms - 1))) if chroms > 1 else []
    bounds = [0] + cuts + [genome_len]
    parts = []
    for i in range(len(bounds) - 1):
        c = g[bounds[i]:bounds[i + 1]]
        n = c.size
        rows = (n + width - 1) // width
        body = np.full((rows, width + 1), ord("\n"), dtype=np.uint8)
        pad = np.zeros(rows * width, dtype=np.uint8)
        pad[:n] = c
        if i == 1:
            pad[:n] |= 0x20   # lower case (N -> n)
        body[:, :width] = pad.reshape(rows, width)
        del pad
        body = body.reshape(-1)
        if n % width:   # the last line holds n % width bases, then its newline
            body = body[: (rows - 1) * (width + 1) + n % width + 1]
            body[-1] = ord("\n")
        parts += [np.frombuffer(b">chr%d synthetic\n" % (i + 1), dtype=np.uint8), body]
    return np.concatenate(parts), g


def aligned_reads(genome: np.ndarray, n: int, seed: int, paired: bool = False, read_len: int = 150,
                  random_frac: float = 0.05, far_frac: float = 0.05, short_frac: float = 0.0,
                  lo: int = 0) -> tuple[bytes, bytes | None]:
    """Reads for the reference path: drawn from `genome` (either strand) with
    0-10 substitutions, some N runs (more than maxmis in some reads), a fraction
    of random (unalignable) reads; PE mates mostly 250-449 apart, a fraction
    far apart or on another chromosome region (the relation's other cases).
    Fragments start at or after genome position `lo` (0-based)."""
    rng = np.random.default_rng([seed, 11])
    G = genome.size
    comp = bytes.maketrans(b"ACGTN", b"TGCAN")

    def one(start, rev):
        s = genome[start:start + read_len].copy()
        k = int(rng.choice([0, 0, 0, 1, 1, 2, 3, 5, 8, 10]))
        if k:
            at = rng.integers(0, read_len, size=k)
            s[at] = _BASES[(np.searchsorted(_BASES, s[at]) + rng.integers(1, 4, size=k)) % 4]
        if rng.random() < 0.03:
            a = int(rng.integers(0, read_len))
            s[a:a + int(rng.integers(1, 12))] = ord("N")
        if rng.random() < random_frac:
            s = _BASES[rng.integers(0, 4, size=read_len)]
        if rng.random() < short_frac:   # short reads: few even-offset seeds survive a few substitutions
            s = s[:int(rng.integers(20, 60))].copy()
            k2 = int(rng.integers(1, 5))
            at = rng.integers(0, s.size, size=k2)
            s[at] = _BASES[(np.searchsorted(_BASES, s[at]) + 1) % 4]
        b = s.tobytes()
        return b.translate(comp)[::-1] if rev else b

    r1, r2 = [], []
    for i in range(n):
        st = int(rng.integers(lo, G - 1000 - read_len))
        rv = bool(rng.random() < 0.5)
        r1.append(one(st, rv))
        if paired:
            if rng.random() < far_frac:
                st2 = int(rng.integers(lo, G - read_len))
            else:
                st2 = min(st + int(rng.integers(250, 450)) - read_len, G - read_len)
            r2.append(one(max(st2, 0), not rv))

    x = rng.integers(1000, 32000, size=n)

    def fq(reads, mate):
        q = _QUALS[rng.integers(0, 3, size=(len(reads), read_len))]
        names = _headers(0, x, mate)
        return b"".join(b"%s\n%s\n+\n%s\n" % (names[i], s, q[i, :len(s)].tobytes()) for i, s in enumerate(reads))
    return fq(r1, 1), (fq(r2, 2) if paired else None)


_COMP256 = np.zeros(256, np.uint8)
_COMP256[list(b"ACGTN")] = list(b"TGCAN")


def fixed_fastq(seq: np.ndarray, mate: int, first: int, qual_seed: int) -> bytes:
    """Fixed-width FASTQ records (Illumina-style headers `@SYN:7:HXX3:1:<10-digit
    index> <mate>:N:0:1`, qualities from F : ,) for an n x L base array: numpy
    throughout, for genome-scale read sets."""
    n, L = seq.shape
    pre, suf, digits = b"@SYN:7:HXX3:1:", b" %d:N:0:1" % mate, 10
    rec = len(pre) + digits + len(suf) + 1 + L + 1 + 2 + L + 1
    a = np.empty((n, rec), np.uint8)
    o = 0
    a[:, o:o + len(pre)] = np.frombuffer(pre, np.uint8)
    o += len(pre)
    idx = np.arange(first, first + n, dtype=np.int64)
    for k in range(digits):
        a[:, o + digits - 1 - k] = 48 + (idx // 10 ** k) % 10
    o += digits
    a[:, o:o + len(suf)] = np.frombuffer(suf, np.uint8)
    o += len(suf)
    a[:, o] = 10
    a[:, o + 1:o + 1 + L] = seq
    o += 1 + L
    a[:, o:o + 3] = np.frombuffer(b"\n+\n", np.uint8)
    o += 3
    rng = np.random.default_rng([qual_seed, mate])
    a[:, o:o + L] = np.frombuffer(b"F:,F", np.uint8)[rng.integers(0, 4, (n, L), dtype=np.uint8)]
    a[:, o + L] = 10
    return a.tobytes()


def draw_reads(rng: np.random.Generator, g: np.ndarray, starts: np.ndarray, rev: np.ndarray, L: int,
               sub: float = 0.004, random_frac: float = 0.02) -> np.ndarray:
    """n x L reads from genome g (ACGTN) at `starts`, substitutions at rate
    `sub`, a fraction of random reads, reverse complement where `rev`."""
    seq = g[starts[:, None] + np.arange(L)]
    m = rng.random(seq.shape) < sub
    seq[m] = _BASES[rng.integers(0, 4, int(m.sum()), dtype=np.uint8)]
    rnd = rng.random(len(starts)) < random_frac
    seq[rnd] = _BASES[rng.integers(0, 4, (int(rnd.sum()), L), dtype=np.uint8)]
    seq[rev] = _COMP256[seq[rev][:, ::-1]]
    return seq


def pe_reads_fast(g: np.ndarray, pairs: int, seed: int, L: int = 150, first: int = 0) -> tuple[bytes, bytes]:
    """Genome-scale PE reads (configs[3] shape): fragments of 250-449 bp at
    uniform starts, either strand, 2 % of mates far away, 0.4 % substitutions,
    2 % random reads."""
    rng = np.random.default_rng([seed, 12])
    glen = g.size
    s1 = rng.integers(0, glen - 1000 - L, pairs)
    rv = rng.random(pairs) < 0.5
    s2 = np.minimum(s1 + rng.integers(250, 450, pairs) - L, glen - L)
    far = rng.random(pairs) < 0.02
    s2[far] = rng.integers(0, glen - L, int(far.sum()))
    return (fixed_fastq(draw_reads(rng, g, s1, rv, L), 1, first, seed),
            fixed_fastq(draw_reads(rng, g, s2, ~rv, L), 2, first, seed))
