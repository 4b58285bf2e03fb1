"""The .arc container (SeqArcFile::writeFileInfo@0x4171b0, writeParam@0x416450,
writeBlockLenArry{SE,PE}@0x416d60/0x416e90) around the encoded blocks.

Pinned by the reference's own run on its own test files:
the PE pair compresses to 821,500 bytes and file 1 alone to 379,069 bytes, and
the header's block-region VINT ends in ...0c8652.  Field values follow the
disassembly (arc_file.cpp); the per-field bytes beyond these sizes are
"parity unpinned" (the reference binary may not be run here)."""
import os
import struct

import numpy as np
import pytest

import oracle_py
from conftest import GOLDEN

import fastqueeze_amd as fq

T1 = os.path.join(GOLDEN, "ERR2755197_test_1.fq")
T2 = os.path.join(GOLDEN, "ERR2755197_test_2.fq")


def _archive(paths, cfg_kw=None):
    texts = [open(p, "rb").read() for p in paths]
    blocks = fq.blocks_from_fastq(*texts)
    tmpl = fq.analyze_ids(blocks[0], len(paths) == 1)
    cfg = fq.Config(bin_mode=int(tmpl[0]), **(cfg_kw or {}))
    enc = [oracle_py.encode_block(b, cfg.slevel, cfg.qlevel, cfg.md5, cfg.bin_mode, cfg.lossy) for b in blocks]
    names = [os.path.basename(p) for p in paths]
    return fq.arc_archive(enc, blocks, names[0], names[1] if len(names) > 1 else None, tmpl, cfg,
                          plus_bare=fq.bare_plus(texts[-1])), enc, blocks, tmpl


def _vint(b, i):
    """EBML VINT at b[i] -> (value, width)."""
    first = b[i]
    n = 1
    while not first & (0x80 >> (n - 1)):
        n += 1
    v = first & ((0x80 >> (n - 1)) - 1)
    for k in range(1, n):
        v = (v << 8) | b[i + k]
    return v, n


def _fields(tr):
    """Parse the trailer: {encap id: payload} of the params encap and the block table."""
    tid, n = _vint(tr, 0)
    assert tid == 3
    size = int.from_bytes(tr[n:n + 4], "big") & 0x0FFFFFFF
    body = tr[n + 4:]
    assert len(body) == size
    pid, n = _vint(body, 0)
    assert pid == 1
    psize = int.from_bytes(body[n:n + 2], "big") & 0x3FFF
    params, rest = body[n + 2:n + 2 + psize], body[n + 2 + psize:]
    out, i = {}, 0
    while i < len(params):
        fid, k = _vint(params, i)
        i += k
        w = 2 if fid == 15 else 1
        ln = int.from_bytes(params[i:i + w], "big") & ((1 << (7 * w)) - 1)
        i += w
        out[fid] = params[i:i + ln]
        i += ln
    bid, n = _vint(rest, 0)
    assert bid == 7
    bsize = int.from_bytes(rest[n:n + 4], "big") & 0x0FFFFFFF
    return out, rest[n + 4:n + 4 + bsize]


def test_reference_archive_sizes():
    pe, enc, _, _ = _archive([T1, T2])
    assert len(pe) == 821500                      # SeqArc-1.6 -c -t 1 on the test pair
    assert pe[:7] == b".arc\x01\x06\x00" and pe[7] == 0x82
    assert pe[8:16].hex().endswith("0c8652")      # block region bytes
    assert pe[16:16 + len(enc[0])] == enc[0]
    se, _, _, _ = _archive([T1])
    assert len(se) == 379069                      # SeqArc-1.6 -c -t 1 on file 1


def test_trailer_fields_pe_and_se():
    pe, enc, blocks, tmpl = _archive([T1, T2])
    f, table = _fields(pe[16 + sum(map(len, enc)):])
    assert sorted(f) == list(range(1, 19)) and f[14] == b"ERR2755197_test_2.fq"
    assert f[13] == b"ERR2755197_test_1.fq" and f[15] == tmpl.tobytes()
    assert f[1] == b"\x01" and f[17] == b"\x01" and f[16] == b"\x00"
    assert f[3] == b"\x00"                        # param+0x5: set by -1, cleared by -2 (parseOptFromCmd@0x40b460)
    assert struct.unpack("<H", f[9])[0] == 6 and struct.unpack("<I", f[11])[0] == 1
    size2, l1, l2, pad, off, o1, o2 = struct.unpack("<IIIIQQQ", table)
    assert size2 >> 1 == len(enc[0]) and size2 & 1 == 0 and off == 16
    assert (l1, l2) == (os.path.getsize(T1), os.path.getsize(T2)) and (pad, o1, o2) == (0, 0, 0)
    se, enc, _, _ = _archive([T1])
    f, table = _fields(se[16 + sum(map(len, enc)):])
    assert 14 not in f and len(table) == 32 and f[3] == b"\x01"   # single-end
    size2, fi, l1, pad, off, o1 = struct.unpack("<IIIIQQ", table)
    assert size2 >> 1 == len(enc[0]) and fi == 1 and l1 == os.path.getsize(T1) and off == 16


def test_multi_block_table_and_flags(tmp_path):
    import synth
    t1, _ = synth.generate(3000, seed=21)
    t_long, _ = synth.generate(3, seed=22, read_len=70000)
    text = t1 + t_long
    blocks = fq.blocks_from_fastq(text, block_size=300_000)
    enc = [oracle_py.encode_block(b, lossy=1.15) for b in blocks]
    a = fq.arc_archive(enc, blocks, "/data/run/x.fq.gz", None, None, fq.Config(lossy=1.15), gz1=True)
    f, table = _fields(a[16 + sum(map(len, enc)):])
    assert f[13] == b"x.fq" and f[4] == b"\x01" and f[16] == b"\x01"
    assert struct.unpack("<I", f[11])[0] == len(blocks) > 3
    recs = [struct.unpack("<IIIIQQ", table[32 * i:32 * i + 32]) for i in range(len(blocks))]
    off = in_off = 0
    for r, e, b in zip(recs, enc, blocks):
        assert r[0] >> 1 == len(e) and r[4] == 16 + off and r[5] == in_off
        assert r[0] & 1 == (1 if int(b.seq_lens.max()) > 0xFFFF else 0)
        off += len(e)
        in_off += r[2]
    assert in_off == len(text) and recs[-1][0] & 1 == 1
    assert int.from_bytes(a[8:16], "big") & ((1 << 56) - 1) == off
