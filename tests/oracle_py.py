"""ctypes binding of the CPU restatement (oracle/liboracle.so) -- test
infrastructure only: used by tests/, __graft_entry__.smoke() and bench.py's
cpu_baseline leg as the checker / CPU baseline, never by the product."""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ORACLE_DIR = os.path.join(ROOT, "oracle")
LIB = os.path.join(ORACLE_DIR, "_build", "liboracle.so")
CLI = os.path.join(ORACLE_DIR, "_build", "orc_cli")

_lib = None


class _Blk(C.Structure):
    _fields_ = [("names", C.c_void_p), ("name_lens", C.c_void_p), ("seq", C.c_void_p),
                ("seq_lens", C.c_void_p), ("qual", C.c_void_p), ("nreads", C.c_uint32)]


class _Cfg(C.Structure):
    _fields_ = [("slevel", C.c_int), ("qlevel", C.c_int), ("md5", C.c_int), ("bin_mode", C.c_int),
                ("lossy", C.c_double)]


def build():
    subprocess.run(["make", "-s", "-C", ORACLE_DIR], check=True)


def lib():
    global _lib
    if _lib is None:
        srcs = [os.path.join(ORACLE_DIR, f)
                for f in ("fqz_oracle.c", "fqz_decode.c", "hash_oracle.c", "align_oracle.c", "fqz_oracle.h",
                          "hash_oracle.h", "orc_cli.c")]
        if not os.path.exists(LIB) or any(os.path.getmtime(s) > os.path.getmtime(LIB) for s in srcs):
            build()
        l = C.CDLL(LIB)
        P = C.c_void_p
        l.orc_encode_block.argtypes = [P, P, P, C.c_size_t]
        l.orc_encode_block.restype = C.c_int64
        l.orc_analyze_idbin.argtypes = [P, C.c_int, P]
        l.orc_analyze_idbin.restype = C.c_int
        l.orc_rc_encode.argtypes = [P, P, P, C.c_size_t, P, C.c_size_t]
        l.orc_rc_encode.restype = C.c_int64
        l.orc_md5.argtypes = [P, C.c_size_t, P]
        l.orc_md5.restype = None
        l.orc_decode_block.argtypes = [P, C.c_size_t, P, P]
        l.orc_decode_block.restype = C.c_int64
        l.orc_rblock.argtypes = [P, C.c_size_t, C.c_double]
        l.orc_rblock.restype = None
        l.ho_build.argtypes = [P, C.c_uint64, C.c_uint32, C.c_uint32, C.c_uint32]
        l.ho_build.restype = C.c_int64
        l.ho_serialize.argtypes = [P, C.c_uint64]
        l.ho_serialize.restype = C.c_int
        l.ho_genome_length.argtypes = []
        l.ho_genome_length.restype = C.c_uint32
        l.ho_align_reads.argtypes = [P, P, P, C.c_int64, C.c_int32, C.c_int32, P, P, P, P, P, P]
        l.ho_align_reads.restype = C.c_int
        l.orc_encode_block_hash.argtypes = [P, P, C.c_int, C.c_int, C.c_int, C.c_uint32, P, P, C.c_size_t]
        l.orc_encode_block_hash.restype = C.c_int64
        _lib = l
    return _lib


def _p(a):
    return a.ctypes.data if a.size else 0


def _blk(b) -> _Blk:
    return _Blk(_p(b.names), _p(b.name_lens), _p(b.seq), _p(b.seq_lens), _p(b.qual), b.nreads)


def encode_block(b, slevel=3, qlevel=2, md5=True, bin_mode=0, lossy=0.0) -> bytes:
    cap = 2 * (b.seq.size + b.names.size) + 16 * b.nreads + 4096
    out = np.empty(cap, dtype=np.uint8)
    cb, cc = _blk(b), _Cfg(slevel, qlevel, 1 if md5 else 0, 1 if bin_mode else 0, float(lossy))
    n = lib().orc_encode_block(C.byref(cb), C.byref(cc), _p(out), cap)
    if n < 0:
        raise RuntimeError("oracle encode failed")
    return out[:n].tobytes()


class _Dec(C.Structure):
    _fields_ = [("names", C.c_void_p), ("name_lens", C.c_void_p), ("seq", C.c_void_p),
                ("seq_lens", C.c_void_p), ("qual", C.c_void_p), ("name_cap", C.c_size_t),
                ("seq_cap", C.c_size_t), ("max_reads", C.c_uint32), ("nreads", C.c_uint32),
                ("md5_ok", C.c_int)]


def decode_block(data: bytes, max_reads: int, name_cap: int, seq_cap: int, slevel=3, qlevel=2, md5=True,
                 lossy=0.0):
    """CPU decode of one encoded block (oracle/fqz_decode.c) -> (names, name_lens,
    seq, seq_lens, qual, md5_ok)."""
    names = np.empty(max(name_cap, 1), np.uint8)
    nl = np.empty(max(max_reads, 1), np.uint16)
    seq = np.empty(max(seq_cap, 1), np.uint8)
    sl = np.empty(max(max_reads, 1), np.int32)
    qual = np.empty(max(seq_cap, 1), np.uint8)
    d = _Dec(_p(names), _p(nl), _p(seq), _p(sl), _p(qual), name_cap, seq_cap, max_reads, 0, 0)
    src = np.frombuffer(data, np.uint8)
    cc = _Cfg(slevel, qlevel, 1 if md5 else 0, 0, float(lossy))
    n = lib().orc_decode_block(_p(src), src.size, C.byref(cc), C.byref(d))
    if n < 0:
        raise RuntimeError(f"oracle decode failed ({n})")
    n = int(n)
    ln, ls = int(nl[:n].astype(np.int64).sum()), int(sl[:n].astype(np.int64).sum())
    return names[:ln], nl[:n], seq[:ls], sl[:n], qual[:ls], bool(d.md5_ok)


def rblock(qual: np.ndarray, ratio: float) -> np.ndarray:
    """R-Block lossy pre-pass (rblock@0x426c10) over one block's qualities."""
    q = np.array(qual, dtype=np.uint8, copy=True)
    lib().orc_rblock(_p(q), q.size, float(ratio))
    return q


def analyze_ids(b, single_end: bool) -> np.ndarray:
    t = np.zeros(512, dtype=np.uint8)
    cb = _blk(b)
    if lib().orc_analyze_idbin(C.byref(cb), 1 if single_end else 0, _p(t)) != 0:
        raise RuntimeError("oracle id analysis failed")
    return t


def md5(data: bytes) -> bytes:
    a = np.frombuffer(data, dtype=np.uint8)
    d = np.zeros(16, dtype=np.uint8)
    lib().orc_md5(_p(a), a.size, _p(d))
    return d.tobytes()


def rc_encode(cum: np.ndarray, freq: np.ndarray, tot: np.ndarray) -> bytes:
    """The bare range coder over (cum, freq, tot) triples (uint16 arrays)."""
    cum, freq, tot = (np.ascontiguousarray(a, dtype=np.uint16) for a in (cum, freq, tot))
    cap = 2 * cum.size + 64
    out = np.empty(cap, dtype=np.uint8)
    n = lib().orc_rc_encode(_p(cum), _p(freq), _p(tot), cum.size, _p(out), cap)
    if n < 0:
        raise RuntimeError("oracle range coder rejected the records")
    return out[:n].tobytes()


def squeeze_streams(seed: int = 7, count: int = 12):
    """(cum, freq, tot) streams for the coder tests: random models plus streams
    that drive low towards all-ones (the same symbol at probability 1/2), which
    fire the carry-less squeeze of the reference coder."""
    rng = np.random.default_rng(seed)
    out = []
    for i in range(count):
        n = int(rng.integers(1, 30000)) if i > 1 else i * 5
        kind = i % 3
        if kind == 0:
            t = np.full(n, 2, np.uint16); f = np.ones(n, np.uint16); c = np.ones(n, np.uint16)
        elif kind == 1:
            t = rng.integers(2, 0xffe0, n, dtype=np.uint32)
            f = np.maximum(1, (rng.random(n) * t).astype(np.uint32))
            c = (rng.random(n) * (t - f + 1)).astype(np.uint32)
        else:
            t = rng.integers(12, 253, n, dtype=np.uint32)
            f = np.maximum(1, (rng.random(n) * (t - 1)).astype(np.uint32))
            c = (rng.random(n) * (t - f + 1)).astype(np.uint32)
        out.append((c.astype(np.uint16), f.astype(np.uint16), t.astype(np.uint16)))
    return out


# ---- HASH reference index + gapless seed alignment (oracle/hash_oracle.c) ----
HASH_K, HASH_STEP, HASH_MAXCOUNT, HASH_MAXMIS, HASH_GOOD = 14, 2, 1 << 16, 7, 1   # SeqArcParam ctor @0x407490


def hash_index(fasta: bytes, k: int = HASH_K, step: int = HASH_STEP, maxcount: int = HASH_MAXCOUNT) -> bytes:
    """The `.hash` file buildRefIndex@0x410190 writes for this FASTA (the
    oracle keeps the index for hash_align)."""
    out = hash_index_array(fasta, k, step, maxcount)
    return out.tobytes()


def hash_index_array(fasta, k: int = HASH_K, step: int = HASH_STEP, maxcount: int = HASH_MAXCOUNT) -> np.ndarray:
    """hash_index() as a uint8 array; fasta may be bytes or a uint8 array
    (genome-scale FASTA without a bytes copy)."""
    l = lib()
    if isinstance(fasta, np.ndarray):
        n = l.ho_build(_p(fasta), fasta.size, k, step, maxcount)
    else:
        n = l.ho_build(fasta, len(fasta), k, step, maxcount)
    if n < 0:
        raise ValueError("hash index build failed")
    out = np.empty(n, dtype=np.uint8)
    if l.ho_serialize(_p(out), n):
        raise ValueError("hash index serialize failed")
    return out


def hash_align(reads: list[bytes], maxmis: int = HASH_MAXMIS, good: int = HASH_GOOD, ai_nmis: int = 0):
    """getHashAlignInfo@0x4113c0 for the reads in order against the last
    hash_index, one align_info carried across them (ai_nmis: its state before
    the first read; 0 = a zero-filled AlignParam).  Arrays ret (mismatches or
    -1), rev, pos (1-based), mispos / mistype ([n, maxmis+1], -1 past the
    read's mismatches)."""
    l = lib()
    n = len(reads)
    seq = np.frombuffer(b"".join(reads) or b"\0", dtype=np.uint8)
    lens = np.array([len(r) for r in reads] or [0], dtype=np.int32)
    off = np.zeros(max(n, 1), dtype=np.uint64)
    if n > 1:
        off[1:n] = np.cumsum(lens[:n - 1])
    ret = np.zeros(max(n, 1), dtype=np.int32)
    rev = np.zeros(max(n, 1), dtype=np.uint8)
    pos = np.zeros(max(n, 1), dtype=np.uint64)
    mp = np.zeros((max(n, 1), maxmis + 1), dtype=np.int32)
    mt = np.zeros((max(n, 1), maxmis + 1), dtype=np.int32)
    st = np.array([ai_nmis], dtype=np.int32)
    if l.ho_align_reads(_p(seq), _p(off), _p(lens), n, maxmis, good, _p(st), _p(ret), _p(rev), _p(pos), _p(mp),
                        _p(mt)):
        raise ValueError("hash align failed")
    return ret[:n], rev[:n], pos[:n], mp[:n], mt[:n]


def encode_block_hash(b, paired: bool, carry=None, slevel=3, qlevel=2, md5=True, bin_mode=0, lossy=0.0,
                      maxmis: int = HASH_MAXMIS, good: int = HASH_GOOD, insert_size: int = 0):
    """The reference path's block encode (doAlign + doAlignEncode@0x42d4c0)
    against the last hash_index.  carry: [mate1/SE, mate2] align_info state in,
    updated in place (default: a fresh zero-filled AlignParam)."""
    cap = 3 * (b.seq.size + b.names.size) + 64 * b.nreads + 8192
    out = np.empty(cap, dtype=np.uint8)
    cb, cc = _blk(b), _Cfg(slevel, qlevel, 1 if md5 else 0, 1 if bin_mode else 0, float(lossy))
    cr = np.array(carry if carry is not None else [0, 0], dtype=np.int32)
    n = lib().orc_encode_block_hash(C.byref(cb), C.byref(cc), 1 if paired else 0, maxmis, good, insert_size,
                                    _p(cr), _p(out), cap)
    if n < 0:
        raise RuntimeError("oracle reference-path encode failed")
    if carry is not None:
        carry[0], carry[1] = int(cr[0]), int(cr[1])
    return out[:n].tobytes()
