"""fastqueeze_amd -- MI355X (gfx950) SeqArc no-reference block encoder.

Thin ctypes binding of libseqarc_amd.so (include/seqarc_amd.h) used by the
tests and bench.py.  The product path is the HIP library; there is no CPU
fallback: if the library or a gfx950 device is missing, the calls raise.

Reference interface mirrored (SeqArc-1.6, cited by address in the binary):
  Encoder.encode()   EncapFqzComp::doFqzEncode@0x42d2d0 for a batch of blocks
  cut_se / cut_pe    SeqArcRead::doReadJob@0x432a80 / doReadPEJob@0x432d10
  parse_se / parse_pe AlignEncodeSEJob::getBlockRead@0x411b60 / getBlockReadPE@0x412920
  analyze_ids        IDProcess::analysisIDBinType@0x4310a0
  Encoder.code_records  the inlined RangeCoder (encode_seq@0x422010-0x422085)
"""
from __future__ import annotations

import ctypes as C
import os
from dataclasses import dataclass

import numpy as np

from . import build as _build

__all__ = ["SeqArcError", "blocks_from_fastq", "Block", "Config", "Encoder", "cut_se", "cut_pe", "parse_se", "parse_pe", "analyze_ids",
           "load_library", "BLOCK_SIZE", "Input"]

BLOCK_SIZE = 50 << 20   # SeqArcParam BlockSize(M) = 50 (ctor @0x40776f)

_lib = None


class SeqArcError(RuntimeError):
    pass


class _SaBlock(C.Structure):
    _fields_ = [("names", C.c_void_p), ("name_lens", C.c_void_p), ("seq", C.c_void_p),
                ("seq_lens", C.c_void_p), ("qual", C.c_void_p), ("nreads", C.c_uint32)]


class _SaCfg(C.Structure):
    _fields_ = [("slevel", C.c_int32), ("qlevel", C.c_int32), ("md5", C.c_int32), ("bin_mode", C.c_int32),
                ("lossy", C.c_double)]


class _SaArcBlock(C.Structure):
    _fields_ = [("size", C.c_uint32), ("long_reads", C.c_uint32), ("text1", C.c_uint64), ("text2", C.c_uint64)]


class _SaArcInfo(C.Structure):
    _fields_ = [("file1", C.c_char_p), ("file2", C.c_char_p), ("paired", C.c_int32), ("gz1", C.c_int32),
                ("bare_plus", C.c_int32), ("md5", C.c_int32), ("lossy", C.c_int32), ("id_template", C.c_void_p),
                ("ref_md5", C.c_void_p), ("insert_size", C.c_uint32)]


class _SaDecoded(C.Structure):
    _fields_ = [("names", C.c_void_p), ("name_lens", C.c_void_p), ("seq", C.c_void_p), ("seq_lens", C.c_void_p),
                ("qual", C.c_void_p), ("name_cap", C.c_uint64), ("seq_cap", C.c_uint64), ("max_reads", C.c_uint32),
                ("nreads", C.c_uint32), ("md5_ok", C.c_int32)]


class _SaTextBlock(C.Structure):
    _fields_ = [("text1", C.c_void_p), ("len1", C.c_uint64), ("text2", C.c_void_p), ("len2", C.c_uint64)]


class _SaTextInfo(C.Structure):
    _fields_ = [("nreads", C.c_uint32), ("len_long", C.c_uint32), ("name_bytes", C.c_uint64),
                ("seq_bytes", C.c_uint64), ("out_bound", C.c_uint64)]


class _SaAlignCfg(C.Structure):
    _fields_ = [("index", C.c_void_p), ("paired", C.c_int32), ("maxmis", C.c_int32), ("good", C.c_int32),
                ("insert_size", C.c_uint32)]


class _SaRef(C.Structure):
    _fields_ = [("genome", C.c_void_p), ("bases", C.c_uint64), ("paired", C.c_int32), ("maxmis", C.c_int32),
                ("insert_size", C.c_uint32)]


class _SaOut(C.Structure):
    _fields_ = [("data", C.c_void_p), ("cap", C.c_uint64), ("size", C.c_uint64)]


def load_library(path: str | None = None):
    """Load libseqarc_amd.so (building it first if the sources are newer)."""
    global _lib
    if _lib is not None:
        return _lib
    if path is None and os.environ.get("SA_LIB"):   # (A/B runs: another build of the library)
        path = os.environ["SA_LIB"]
    if path is None:
        path = _build.LIB
        if _build.needs_build():
            if os.environ.get("SA_NO_BUILD"):   # (GPU runs: the library travels prebuilt)
                raise SeqArcError("libseqarc_amd.so is older than its sources and SA_NO_BUILD is set")
            _build.build()
    if not os.path.exists(path):
        raise SeqArcError(f"libseqarc_amd.so not found at {path}")
    lib = C.CDLL(path)
    P, U64, I64, I32 = C.c_void_p, C.c_uint64, C.c_int64, C.c_int
    sigs = {
        "sa_create": ([I32], P), "sa_destroy": ([P], None), "sa_last_error": ([P], C.c_char_p),
        "sa_version": ([], C.c_char_p), "sa_output_bound": ([P], U64),
        "sa_encode_blocks": ([P, P, I32, P, P], I32), "sa_stage": ([P, P, I32], I32),
        "sa_run": ([P, P], I32), "sa_fetch": ([P, P, I32], I32), "sa_fetch_sizes": ([P, P, I32], I32),
        "sa_phase_times": ([P, P, P, I32], I32), "sa_set_timing": ([P, I32], None),
        "sa_cut_se": ([P, U64, U64, P, U64], I64), "sa_cut_pe": ([P, U64, P, U64, U64, P, P, U64], I64),
        "sa_parse_se": ([P, U64, P, P, P, P, P], I64), "sa_parse_pe": ([P, U64, P, U64, P, P, P, P, P], I64),
        "sa_analyze_ids": ([P, I32, P], I32),
        "sa_code_records": ([P, I32, P, P, P, P, P, U64, P], I32), "sa_coder_restarts": ([P], C.c_uint32),
        "sa_stream_stats": ([P, P, P], None), "sa_device_bytes": ([P], U64), "sa_front_bytes": ([P], U64),
        "sa_create_shared": ([I32, P], P),
        "sa_input_create": ([I32, P, I32], P), "sa_input_destroy": ([P], None), "sa_run_input": ([P, P, P], I32),
        "sa_arc_header": ([U64, P], I32), "sa_arc_trailer": ([P, P, C.c_uint32, P, U64], I64),
        "sa_arc_trailer2": ([P, C.c_int32, P, C.c_uint32, P, U64], I64),
        "sa_decode_block": ([P, U64, P, P, I32, P], I64),
        "sa_host_register": ([P, U64], I32), "sa_host_unregister": ([P], I32),
        "sa_stage_text": ([P, P, I32, P], I32), "sa_host_alloc": ([U64], P), "sa_host_free": ([P], None),
        "sa_text_upload": ([P, P, I32, I32, I32, P, U64], I32), "sa_text_parse": ([P, P, I32, P, I32, U64, P], I32),
        "sa_hash_build": ([P, P, U64, C.c_uint32, C.c_uint32, C.c_uint32], P),
        "sa_hash_file_bytes": ([P], U64), "sa_hash_serialize": ([P, P, P, U64], I32),
        "sa_hash_genome_length": ([P], C.c_uint32), "sa_hash_destroy": ([P], None),
        "sa_hash_align": ([P, P, P, P, P, I64, C.c_int32, C.c_int32, P, P, P, P, P, P], I32),
        "sa_align_chain_create": ([C.c_int32, C.c_int32], P), "sa_align_chain_destroy": ([P], None),
        "sa_run_input_aligned": ([P, P, P, P, P, U64], I32), "sa_run_aligned": ([P, P, P, P, U64], I32),
        "sa_encode_blocks_aligned": ([P, P, I32, P, P, P, P], I32),
        "sa_hash_load": ([P, P, U64], P), "sa_hash_packed": ([P, P, P, U64], I32),
        "sa_hash_align_kernel_ms": ([P], C.c_float),
        "sa_decode_block_ref": ([P, U64, P, P, I32, P, P], I64),
    }
    for name, (args, res) in sigs.items():
        fn = getattr(lib, name)
        fn.argtypes = args
        fn.restype = res
    _lib = lib
    return lib


def _ptr(a: np.ndarray) -> int:
    return a.ctypes.data if a.size else 0


@dataclass
class Block:
    """One parsed block: the SeqArcMemBuf SoA (PE reads interleaved r1, r2)."""
    names: np.ndarray       # uint8, IDs without '@'
    name_lens: np.ndarray   # uint16
    seq: np.ndarray         # uint8
    seq_lens: np.ndarray    # int32
    qual: np.ndarray        # uint8
    text_bytes: int = 0     # FASTQ bytes this block was parsed from
    text1: int = 0          # ... of them in input 1 (ReadBuf+0xc)
    text2: int = 0          # ... in input 2 (ReadBuf+0x10)

    @property
    def nreads(self) -> int:
        return int(self.name_lens.shape[0])

    def _c(self) -> _SaBlock:
        return _SaBlock(_ptr(self.names), _ptr(self.name_lens), _ptr(self.seq), _ptr(self.seq_lens),
                        _ptr(self.qual), self.nreads)


@dataclass
class Config:
    """SeqArcParam fields of the no-ref path (defaults of SeqArcParam::SeqArcParam@0x407490)."""
    slevel: int = 3
    qlevel: int = 2
    md5: bool = True
    bin_mode: int = 0
    lossy: float = 0.0     # -l R (R-Block lossy qualities, rblock@0x426c10); 0 = lossless

    def _c(self) -> _SaCfg:
        return _SaCfg(self.slevel, self.qlevel, 1 if self.md5 else 0, 1 if self.bin_mode else 0, float(self.lossy))


def _as_u8(text) -> np.ndarray:
    if isinstance(text, np.ndarray):
        return text.view(np.uint8).reshape(-1)
    return np.frombuffer(text, dtype=np.uint8)


def cut_se(text, block_size: int = BLOCK_SIZE) -> list[tuple[int, int]]:
    lib = load_library()
    t = _as_u8(text)
    maxb = t.size // 1024 + 16
    ends = np.zeros(maxb, dtype=np.uint64)
    n = lib.sa_cut_se(_ptr(t), t.size, block_size, _ptr(ends), maxb)
    if n < 0:
        raise SeqArcError("block cut failed")
    e = [0] + ends[:n].astype(np.int64).tolist()
    return [(e[i], e[i + 1]) for i in range(n)]


def cut_pe(t1, t2, block_size: int = BLOCK_SIZE):
    lib = load_library()
    a, b = _as_u8(t1), _as_u8(t2)
    maxb = (a.size + b.size) // 1024 + 16
    e1 = np.zeros(maxb, dtype=np.uint64)
    e2 = np.zeros(maxb, dtype=np.uint64)
    n = lib.sa_cut_pe(_ptr(a), a.size, _ptr(b), b.size, block_size, _ptr(e1), _ptr(e2), maxb)
    if n < 0:
        raise SeqArcError("PE block cut failed")
    x = [0] + e1[:n].astype(np.int64).tolist()
    y = [0] + e2[:n].astype(np.int64).tolist()
    return [((x[i], x[i + 1]), (y[i], y[i + 1])) for i in range(n)]


def _alloc(nbytes: int):
    return (np.empty(nbytes + 16, np.uint8), np.empty(nbytes // 4 + 8, np.uint16), np.empty(nbytes + 16, np.uint8),
            np.empty(nbytes // 4 + 8, np.int32), np.empty(nbytes + 16, np.uint8))


def _trim(names, nl, seq, sl, qual, n, text_bytes) -> Block:
    nl = nl[:n].copy()
    sl = sl[:n].copy()
    tn = int(nl.sum(dtype=np.int64))
    ts = int(sl.sum(dtype=np.int64))
    return Block(names[:tn].copy(), nl, seq[:ts].copy(), sl, qual[:ts].copy(), text_bytes)


def parse_se(text) -> Block:
    lib = load_library()
    t = _as_u8(text)
    names, nl, seq, sl, qual = _alloc(t.size)
    n = lib.sa_parse_se(_ptr(t), t.size, _ptr(names), _ptr(nl), _ptr(seq), _ptr(sl), _ptr(qual))
    if n < 0:
        raise SeqArcError("FASTQ parse failed")
    return _trim(names, nl, seq, sl, qual, n, t.size)


def parse_pe(t1, t2) -> Block:
    lib = load_library()
    a, b = _as_u8(t1), _as_u8(t2)
    names, nl, seq, sl, qual = _alloc(a.size + b.size)
    n = lib.sa_parse_pe(_ptr(a), a.size, _ptr(b), b.size, _ptr(names), _ptr(nl), _ptr(seq), _ptr(sl), _ptr(qual))
    if n < 0:
        raise SeqArcError("PE FASTQ parse failed")
    return _trim(names, nl, seq, sl, qual, n, a.size + b.size)


def analyze_ids(first: Block, single_end: bool) -> np.ndarray:
    lib = load_library()
    tmpl = np.zeros(512, dtype=np.uint8)
    cb = first._c()
    if lib.sa_analyze_ids(C.byref(cb), 1 if single_end else 0, _ptr(tmpl)) != 0:
        raise SeqArcError("ID template analysis failed (the reference would throw)")
    return tmpl


def blocks_from_fastq(t1, t2=None, block_size: int = BLOCK_SIZE) -> list[Block]:
    """Cut and parse FASTQ text exactly as the reference's reader does."""
    if t2 is None:
        a = _as_u8(t1)
        return [parse_se(a[s:e]) for s, e in cut_se(a, block_size)]
    a, b = _as_u8(t1), _as_u8(t2)
    out = []
    for (s1, e1), (s2, e2) in cut_pe(a, b, block_size):
        blk = parse_pe(a[s1:e1], b[s2:e2])
        blk.text1, blk.text2 = e1 - s1, e2 - s2
        out.append(blk)
    return out


class Encoder:
    """A gfx950 device context of libseqarc_amd (one per device / host thread)."""

    PHASES = 11

    def __init__(self, device: int = 0, share_with: "Encoder | None" = None):
        """share_with: another Encoder of the same device whose front scratch this
        one shares (sa_create_shared): their fronts then run one at a time."""
        self._lib = load_library()
        self._ctx = (self._lib.sa_create_shared(device, share_with._ctx) if share_with is not None
                     else self._lib.sa_create(device))
        if not self._ctx:
            raise SeqArcError(f"no usable gfx950 device {device} (the HIP path is the only path)")
        self._staged: list[int] | None = []   # output bound of each staged block

    def close(self):
        if self._ctx:
            self._lib.sa_destroy(self._ctx)
            self._ctx = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def _err(self, what: str):
        msg = self._lib.sa_last_error(self._ctx)
        raise SeqArcError(f"{what}: {msg.decode() if msg else 'unknown error'}")

    def set_timing(self, on: bool = True):
        self._lib.sa_set_timing(self._ctx, 1 if on else 0)

    def stage(self, blocks: list[Block]):
        self._staged = [int(self._lib.sa_output_bound(C.byref(b._c()))) for b in blocks]
        arr = (_SaBlock * max(1, len(blocks)))(*[b._c() for b in blocks])
        if self._lib.sa_stage(self._ctx, arr, len(blocks)) != 0:
            self._err("sa_stage")

    def stage_text(self, texts) -> list[dict]:
        """sa_stage_text: blocks given as FASTQ text, [(text1, text2 or None)]
        as the reader cut them, parsed on the device.  Returns per-block counts."""
        keep = [(_as_u8(a), None if b is None else _as_u8(b)) for a, b in texts]
        dummy = np.zeros(1, np.uint8)   # (an empty PE mate text still needs a non-NULL pointer)
        arr = (_SaTextBlock * max(1, len(keep)))(*[
            _SaTextBlock(_ptr(a) or dummy.ctypes.data, a.size,
                         None if b is None else (_ptr(b) or dummy.ctypes.data), 0 if b is None else b.size)
            for a, b in keep])
        info = (_SaTextInfo * max(1, len(keep)))()
        if self._lib.sa_stage_text(self._ctx, arr, len(keep), info) != 0:
            self._staged = None
            self._err("sa_stage_text")
        self._staged = [int(info[i].out_bound) for i in range(len(keep))]
        return [{"nreads": int(info[i].nreads), "len_long": int(info[i].len_long),
                 "name_bytes": int(info[i].name_bytes), "seq_bytes": int(info[i].seq_bytes)} for i in range(len(keep))]

    def stage_text_streamed(self, texts, slot: int = 0, stride: int | None = None) -> list[dict]:
        """sa_text_upload block by block into text arena `slot`, then
        sa_text_parse: what the command line does as its reader cuts blocks.
        Returns per-block counts as stage_text does."""
        keep = [(_as_u8(a), None if b is None else _as_u8(b)) for a, b in texts]
        if stride is None:
            stride = max([a.size for a, _ in keep] + [0 if b is None else b.size for _, b in keep] + [1])
        dummy = np.zeros(1, np.uint8)
        blks = [_SaTextBlock(_ptr(a) or dummy.ctypes.data, a.size,
                             None if b is None else (_ptr(b) or dummy.ctypes.data), 0 if b is None else b.size)
                for a, b in keep]
        for i, tb in enumerate(blks):
            if self._lib.sa_text_upload(self._ctx, None, slot, i, len(blks), C.byref(tb), stride) != 0:
                self._staged = None
                self._err("sa_text_upload")
        arr = (_SaTextBlock * max(1, len(blks)))(*blks)
        info = (_SaTextInfo * max(1, len(keep)))()
        if self._lib.sa_text_parse(self._ctx, None, slot, arr, len(keep), stride, info) != 0:
            self._staged = None
            self._err("sa_text_parse")
        self._staged = [int(info[i].out_bound) for i in range(len(keep))]
        return [{"nreads": int(info[i].nreads), "len_long": int(info[i].len_long),
                 "name_bytes": int(info[i].name_bytes), "seq_bytes": int(info[i].seq_bytes)} for i in range(len(keep))]

    def run(self, cfg: Config):
        c = cfg._c()
        if self._lib.sa_run(self._ctx, C.byref(c)) != 0:
            self._err("sa_run")

    def fetch_sizes(self) -> list[int]:
        """The encoded size of each block of the last run (sa_fetch_sizes: what
        fetch() will return, known before the copies)."""
        if self._staged is None:
            raise SeqArcError("fetch_sizes(): nothing staged")
        n = len(self._staged)
        sizes = np.zeros(max(1, n), dtype=np.uint64)
        if self._lib.sa_fetch_sizes(self._ctx, _ptr(sizes), n) != 0:
            self._err("sa_fetch_sizes")
        return [int(x) for x in sizes[:n]]

    def fetch(self) -> list[bytes]:
        if self._staged is None:
            raise SeqArcError("fetch(): nothing staged (encode_blocks() fetched its own output; stage() or "
                              "run_input() first)")
        # (the host buffers are kept for the next fetch: freeing memory the
        # device-to-host copies page-locked stalls the GPU's queues while other
        # contexts run -- DESIGN.md, round 5)
        bufs = self.__dict__.setdefault("_fetch_bufs", [])
        outs, keep = [], []
        for i, cap in enumerate(self._staged):
            if i == len(bufs):
                bufs.append(np.empty(0, dtype=np.uint8))
            if bufs[i].size < cap:
                bufs[i] = np.empty(cap + cap // 8, dtype=np.uint8)
            keep.append(bufs[i])
            outs.append(_SaOut(_ptr(bufs[i]), cap, 0))
        arr = (_SaOut * max(1, len(outs)))(*outs)
        if self._lib.sa_fetch(self._ctx, arr, len(outs)) != 0:
            self._err("sa_fetch")
        return [keep[i][: arr[i].size].tobytes() for i in range(len(outs))]

    def encode_blocks(self, blocks: list[Block], cfg: Config) -> list[bytes]:
        """One sa_encode_blocks call (the drop-in for doFqzEncode over a batch;
        the library splits batches larger than its HBM cap into sub-batches)."""
        ins = (_SaBlock * max(1, len(blocks)))(*[b._c() for b in blocks])
        keep, outs = [], []
        for b in blocks:
            cb = b._c()
            cap = int(self._lib.sa_output_bound(C.byref(cb)))
            buf = np.empty(cap, dtype=np.uint8)
            keep.append(buf)
            outs.append(_SaOut(_ptr(buf), cap, 0))
        arr = (_SaOut * max(1, len(outs)))(*outs)
        c = cfg._c()
        if self._lib.sa_encode_blocks(self._ctx, ins, len(blocks), C.byref(c), arr) != 0:
            self._err("sa_encode_blocks")
        self._staged = None   # the context's last output is a sub-batch: nothing to fetch()
        return [keep[i][: arr[i].size].tobytes() for i in range(len(outs))]

    def run_input(self, inp: "Input", cfg: Config):
        """Encode a resident batch (sa_run_input); fetch() then returns its blocks."""
        c = cfg._c()
        if self._lib.sa_run_input(self._ctx, inp._h, C.byref(c)) != 0:
            self._err("sa_run_input")
        self._staged = [int(self._lib.sa_output_bound(C.byref(b._c()))) for b in inp.blocks]

    def run_aligned(self, cfg: Config, index: "HashIndex", paired: bool, chain: "AlignChain",
                    batch: int | None = None, inp: "Input | None" = None, maxmis: int = 7, good: int = 1,
                    insert_size: int = 0):
        """The staged batch (or `inp`) through the reference path
        (sa_run_input_aligned; doAlignEncode@0x42d4c0 per block); fetch() then."""
        c = cfg._c()
        a = _SaAlignCfg(index._h, 1 if paired else 0, maxmis, good, insert_size)
        b = 0xFFFFFFFFFFFFFFFF if batch is None else int(batch)
        if inp is None:
            rc = self._lib.sa_run_aligned(self._ctx, C.byref(c), C.byref(a), chain._h, b)
        else:
            rc = self._lib.sa_run_input_aligned(self._ctx, inp._h, C.byref(c), C.byref(a), chain._h, b)
            self._staged = [int(self._lib.sa_output_bound(C.byref(x._c()))) for x in inp.blocks]
        if rc != 0:
            self._err("sa_run_input_aligned")

    def encode_aligned(self, blocks: list[Block], cfg: Config, index: "HashIndex", paired: bool,
                       chain: "AlignChain | None" = None, **kw) -> list[bytes]:
        """stage + run_aligned + fetch (a fresh chain unless one is given)."""
        own = chain is None
        chain = chain or AlignChain()
        try:
            self.stage(blocks)
            self.run_aligned(cfg, index, paired, chain, **kw)
            return self.fetch()
        finally:
            if own:
                chain.close()

    def device_bytes(self) -> int:
        return int(self._lib.sa_device_bytes(self._ctx))

    def front_bytes(self) -> int:
        return int(self._lib.sa_front_bytes(self._ctx))

    def encode(self, blocks: list[Block], cfg: Config) -> list[bytes]:
        self.stage(blocks)
        self.run(cfg)
        return self.fetch()

    def code_records(self, streams) -> list[bytes]:
        """Range-code pre-modelled streams [(cum, freq, tot) uint16 arrays] on the GPU."""
        lens = np.array([len(c) for c, _, _ in streams], dtype=np.uint32)
        cat = [np.ascontiguousarray(np.concatenate([s[k] for s in streams]) if streams else np.zeros(0), dtype=np.uint16)
               for k in range(3)]
        cap = int(2 * lens.sum() + 64 * len(streams) + 16)
        out = np.empty(cap, dtype=np.uint8)
        ol = np.zeros(max(1, len(streams)), dtype=np.uint64)
        if self._lib.sa_code_records(self._ctx, len(streams), _ptr(lens), _ptr(cat[0]), _ptr(cat[1]), _ptr(cat[2]),
                                     _ptr(out), cap, _ptr(ol)) != 0:
            self._err("sa_code_records")
        res, o = [], 0
        for i in range(len(streams)):
            res.append(out[o:o + int(ol[i])].tobytes())
            o += int(ol[i])
        return res

    def coder_restarts(self) -> int:
        return int(self._lib.sa_coder_restarts(self._ctx))

    def stream_stats(self) -> tuple[int, int]:
        """(symbols of the longest coder stream, symbols of all streams) of the last run."""
        mx, tot = C.c_uint64(0), C.c_uint64(0)
        self._lib.sa_stream_stats(self._ctx, C.byref(mx), C.byref(tot))
        return int(mx.value), int(tot.value)

    def phase_times(self) -> dict[str, float]:
        names = (C.c_char_p * self.PHASES)()
        ms = (C.c_float * self.PHASES)()
        n = self._lib.sa_phase_times(self._ctx, names, ms, self.PHASES)
        return {names[i].decode(): float(ms[i]) for i in range(n)}


class HostBuffer:
    """Page-locked host memory (sa_host_alloc: portable across devices, so a copy
    from it is a DMA) seen as a numpy uint8 array: where sa_stage_text wants the
    reader's text windows."""

    def __init__(self, nbytes: int):
        self._lib = load_library()
        self._p = self._lib.sa_host_alloc(max(1, nbytes))
        if not self._p:
            raise SeqArcError(f"sa_host_alloc({nbytes}) failed")
        self.array = np.ctypeslib.as_array((C.c_uint8 * max(1, nbytes)).from_address(self._p))[:nbytes]

    def close(self):
        if self._p:
            self.array = None
            self._lib.sa_host_free(self._p)
            self._p = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class Input:
    """A batch of blocks resident in HBM (sa_input_create): uploaded once, encoded
    by any Encoder of the same device, concurrently from several host threads."""

    def __init__(self, blocks: list[Block], device: int = 0):
        self._lib = load_library()
        self.blocks = list(blocks)
        arr = (_SaBlock * max(1, len(blocks)))(*[b._c() for b in blocks])
        self._h = self._lib.sa_input_create(device, arr, len(blocks))
        if not self._h:
            raise SeqArcError(f"sa_input_create failed on device {device}")
        self.text_bytes = sum(b.text_bytes for b in blocks)

    def close(self):
        if self._h:
            self._lib.sa_input_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def bare_plus(text) -> int:
    """1 if the first record's '+' line carries no ID (getFirstLine@0x431eb0)."""
    t = _as_u8(text)
    nl = np.flatnonzero(t[: 1 << 16] == 10)[:3]
    if nl.size < 3:
        return 1
    return 0 if int(nl[2]) - int(nl[1]) > 2 else 1


def arc_archive(encaps: list[bytes], blocks: list[Block], file1: str, file2: str | None = None,
                template: np.ndarray | None = None, cfg: Config | None = None, gz1: bool = False,
                plus_bare: int = 1, ref_md5: bytes | None = None, insert_size: int = 0, maxmis: int = 7) -> bytes:
    """The .arc file around encoded blocks (header, blocks in input order, trailer):
    SeqArcFile::writeFileInfo@0x4171b0 / writeParam@0x416450 / writeBlockLenArry (arc_file.cpp)."""
    lib = load_library()
    cfg = cfg or Config()
    recs = (_SaArcBlock * max(1, len(encaps)))()
    for i, (e, b) in enumerate(zip(encaps, blocks)):
        lng = 1 if b.nreads and int(b.seq_lens.max()) > 0xffff else 0
        recs[i] = _SaArcBlock(len(e), lng, b.text1 or b.text_bytes, b.text2)
    tmpl = np.zeros(512, np.uint8) if template is None else np.ascontiguousarray(template, dtype=np.uint8)
    rm = None if ref_md5 is None else np.frombuffer(ref_md5, np.uint8)
    info = _SaArcInfo(file1.encode(), (file2 or "").encode(), 1 if file2 else 0, 1 if gz1 else 0, int(plus_bare),
                      1 if cfg.md5 else 0, 1 if cfg.lossy > 0 else 0, _ptr(tmpl), None if rm is None else _ptr(rm),
                      int(insert_size))
    cap = 4096 + 40 * len(encaps)
    tr = np.empty(cap, np.uint8)
    n = lib.sa_arc_trailer2(C.byref(info), int(maxmis), recs, len(encaps), _ptr(tr), cap)
    if n < 0:
        raise SeqArcError("sa_arc_trailer failed")
    hdr = np.zeros(16, np.uint8)
    lib.sa_arc_header(sum(map(len, encaps)), _ptr(hdr))
    return hdr.tobytes() + b"".join(encaps) + tr[:n].tobytes()


def hash_file_genome(hash_file: bytes) -> tuple[np.ndarray, int]:
    """(packed genome words, bases) of a `.hash` file (HashRefIndex32 layout:
    K, bases, words, positions, then the words)."""
    K, bases, nwords, npos = np.frombuffer(hash_file[:16], np.uint32)
    return np.frombuffer(hash_file, np.uint32, count=int(nwords), offset=16).copy(), int(bases)


def decode_block(data: bytes, text_bytes: int, cfg: Config | None = None, template: np.ndarray | None = None,
                 long_reads: bool = False, ref: tuple | None = None) -> tuple[Block, bool]:
    """Host decode of one encoded block (sa_decode_block; doFqzDecode@0x42c680):
    (the block's reads, stored MD5s match).  text_bytes bounds the arrays
    (the block's FASTQ size, from the archive's block table).  ref = (genome
    words, bases, paired, maxmis[, insert_size]): a block of the reference path."""
    lib = load_library()
    cfg = cfg or Config()
    cap = int(text_bytes) + 64
    names, seq, qual = (np.empty(cap, np.uint8) for _ in range(3))
    mr = cap // 4 + 8
    nl, sl = np.empty(mr, np.uint16), np.empty(mr, np.int32)
    d = _SaDecoded(_ptr(names), _ptr(nl), _ptr(seq), _ptr(sl), _ptr(qual), cap, cap, mr, 0, 0)
    src = np.frombuffer(data, np.uint8)
    tmpl = np.zeros(512, np.uint8) if template is None else np.ascontiguousarray(template, dtype=np.uint8)
    c = cfg._c()
    if ref is None:
        n = lib.sa_decode_block(_ptr(src), src.size, C.byref(c), _ptr(tmpl), 1 if long_reads else 0, C.byref(d))
    else:
        words = np.ascontiguousarray(ref[0], dtype=np.uint32)
        r = _SaRef(_ptr(words), int(ref[1]), 1 if ref[2] else 0, int(ref[3]), int(ref[4]) if len(ref) > 4 else 0)
        n = lib.sa_decode_block_ref(_ptr(src), src.size, C.byref(c), _ptr(tmpl), 1 if long_reads else 0, C.byref(r),
                                    C.byref(d))
    if n < 0:
        raise SeqArcError("sa_decode_block: malformed block")
    n = int(n)
    ln, ls = int(nl[:n].astype(np.int64).sum()), int(sl[:n].astype(np.int64).sum())
    return Block(names[:ln].copy(), nl[:n].copy(), seq[:ls].copy(), sl[:n].copy(), qual[:ls].copy(), text_bytes), \
        bool(d.md5_ok)


class AlignChain:
    """The align_info state an encode thread carries from read to read and block
    to block on the reference path (sa_align_chain): one per input, batches
    pass through it in order.  nmis: the states before the first read (0 for
    a fresh encode thread's AlignParam)."""

    def __init__(self, nmis_mate1: int = 0, nmis_mate2: int = 0):
        self._lib = load_library()
        self._h = self._lib.sa_align_chain_create(nmis_mate1, nmis_mate2)

    def close(self):
        if self._h:
            self._lib.sa_align_chain_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class HashIndex:
    """The HASH reference index of a FASTA (`SeqArc -i ref.fa`,
    buildRefIndex@0x410190), built and kept on an Encoder's device
    (sa_hash_build), and the gapless seed alignment of reads against it
    (sa_hash_align, getHashAlignInfo@0x4113c0)."""

    K, STEP, MAXCOUNT, MAXMIS, GOOD = 14, 2, 1 << 16, 7, 1   # SeqArcParam ctor @0x407490

    def __init__(self, enc: "Encoder", fasta: bytes | None, k: int = K, step: int = STEP, maxcount: int = MAXCOUNT,
                 hash_file: bytes | None = None):
        """From the FASTA (built on the device) or from its `.hash` file (hash_file)."""
        self._enc, self._lib = enc, enc._lib
        if hash_file is not None:
            f = np.frombuffer(hash_file, np.uint8)
            self._h = self._lib.sa_hash_load(enc._ctx, _ptr(f), f.size)
            if not self._h:
                enc._err("sa_hash_load")
            return
        if isinstance(fasta, np.ndarray):   # (a genome-scale FASTA as a uint8 array: no bytes copy)
            self._h = self._lib.sa_hash_build(enc._ctx, _ptr(fasta), fasta.size, k, step, maxcount)
        else:
            self._h = self._lib.sa_hash_build(enc._ctx, fasta, len(fasta), k, step, maxcount)
        if not self._h:
            enc._err("sa_hash_build")

    def close(self):
        if self._h:
            self._lib.sa_hash_destroy(self._h)
            self._h = None

    def __del__(self):
        self.close()

    @property
    def genome_length(self) -> int:
        return int(self._lib.sa_hash_genome_length(self._h))

    def file_bytes(self) -> bytes:
        """The `<ref.fa>.hash` file (HashRefIndex32::writeIndexFile@0x41ed00)."""
        return self.file_array().tobytes()

    def file_array(self) -> np.ndarray:
        """file_bytes() as a uint8 array."""
        n = int(self._lib.sa_hash_file_bytes(self._h))
        out = np.empty(n, dtype=np.uint8)
        if self._lib.sa_hash_serialize(self._enc._ctx, self._h, _ptr(out), n) != 0:
            self._enc._err("sa_hash_serialize")
        return out

    def packed(self) -> tuple[np.ndarray, int]:
        """(the genome's packed words, bases): what the aligned-read decoder
        reads (sa_hash_packed; HashAlignment::doGetSeq@0x40ff90)."""
        n = self.genome_length
        words = np.empty(max(1, (n + 15) // 16), np.uint32)
        if self._lib.sa_hash_packed(self._enc._ctx, self._h, _ptr(words), words.size) != 0:
            self._enc._err("sa_hash_packed")
        return words, n

    def align(self, reads: list[bytes], maxmis: int = MAXMIS, good: int = GOOD, ai_nmis: int = 0):
        """The reads in order, one align_info state carried across them
        (ai_nmis: before the first read; 0 = a zero-filled AlignParam).  Per
        read: ret (mismatches or -1), rev, pos (1-based), mispos and mistype
        ([n, maxmis + 1], -1 past the read's mismatches)."""
        n = len(reads)
        seq = np.frombuffer(b"".join(reads) or b"\0", dtype=np.uint8)
        lens = np.array([len(r) for r in reads] or [0], dtype=np.int32)
        off = np.zeros(max(n, 1), dtype=np.uint64)
        if n > 1:
            off[1:n] = np.cumsum(lens[:n - 1])
        return self.align_arrays(seq, off, lens, n, maxmis, good, ai_nmis)

    def align_arrays(self, seq: np.ndarray, off: np.ndarray, lens: np.ndarray, n: int, maxmis: int = MAXMIS,
                     good: int = GOOD, ai_nmis: int = 0):
        """align() over reads given as one uint8 array with uint64 offsets and
        int32 lengths (no per-read Python objects)."""
        seq = np.ascontiguousarray(seq, dtype=np.uint8)
        off = np.ascontiguousarray(off, dtype=np.uint64)
        lens = np.ascontiguousarray(lens, dtype=np.int32)
        ret = np.zeros(max(n, 1), dtype=np.int32)
        rev = np.zeros(max(n, 1), dtype=np.uint8)
        pos = np.zeros(max(n, 1), dtype=np.uint64)
        mp = np.zeros((max(n, 1), maxmis + 1), dtype=np.int32)
        mt = np.zeros((max(n, 1), maxmis + 1), dtype=np.int32)
        st = np.array([ai_nmis], dtype=np.int32)
        if self._lib.sa_hash_align(self._enc._ctx, self._h, _ptr(seq), _ptr(off), _ptr(lens), n, maxmis, good,
                                   _ptr(st), _ptr(ret), _ptr(rev), _ptr(pos), _ptr(mp), _ptr(mt)) != 0:
            self._enc._err("sa_hash_align")
        self.last_kernel_ms = float(self._lib.sa_hash_align_kernel_ms(self._enc._ctx))
        return ret[:n], rev[:n], pos[:n], mp[:n], mt[:n]
