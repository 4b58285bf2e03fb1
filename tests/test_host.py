"""Host-side checks (no GPU): the C-ABI library builds/loads and exports every
symbol include/seqarc_amd.h declares; the host block plumbing (cut, parse, ID
template analysis) agrees with the oracle."""
import ctypes
import os
import re

import numpy as np

import oracle_py
import synth
from conftest import ROOT

import fastqueeze_amd as fq


def test_library_exports_header_symbols():
    lib = fq.load_library()
    hdr = open(os.path.join(ROOT, "include", "seqarc_amd.h")).read()
    names = set(re.findall(r"\b(sa_[a-z_]+)\s*\(", hdr))
    assert {"sa_encode_blocks", "sa_create", "sa_run", "sa_analyze_ids"} <= names
    for n in sorted(names):
        assert hasattr(lib, n), n
    assert fq.load_library().sa_version().decode().startswith("seqarc_amd")


def _orc_blocks(t1, t2, bs):
    """Oracle cut + parse via its CLI-equivalent C entry points."""
    lib = oracle_py.lib()
    P = ctypes.c_void_p
    a = np.frombuffer(t1, np.uint8)
    maxb = len(t1) // 1024 + 16
    e1 = np.zeros(maxb, np.uint64)
    if t2 is None:
        lib.orc_cut_se.argtypes = [P, ctypes.c_size_t, ctypes.c_size_t, P, ctypes.c_size_t]
        lib.orc_cut_se.restype = ctypes.c_int64
        n = lib.orc_cut_se(a.ctypes.data, a.size, bs, e1.ctypes.data, maxb)
        return [int(x) for x in e1[:n]], None
    b = np.frombuffer(t2, np.uint8)
    e2 = np.zeros(maxb, np.uint64)
    lib.orc_cut_pe.argtypes = [P, ctypes.c_size_t, P, ctypes.c_size_t, ctypes.c_size_t, P, P, ctypes.c_size_t]
    lib.orc_cut_pe.restype = ctypes.c_int64
    n = lib.orc_cut_pe(a.ctypes.data, a.size, b.ctypes.data, b.size, bs, e1.ctypes.data, e2.ctypes.data, maxb)
    return [int(x) for x in e1[:n]], [int(x) for x in e2[:n]]


def test_cut_matches_oracle(test_pair):
    t1, t2 = test_pair
    for bs in (300000, 600000, 1 << 20, fq.BLOCK_SIZE):
        ours = fq.cut_se(t1, bs)
        o1, _ = _orc_blocks(t1, None, bs)
        assert [e for _, e in ours] == o1
        ours_pe = fq.cut_pe(t1, t2, bs)
        p1, p2 = _orc_blocks(t1, t2, bs)
        assert [x[0][1] for x in ours_pe] == p1 and [x[1][1] for x in ours_pe] == p2


def test_parse_and_ids(test_pair):
    t1, t2 = test_pair
    se = fq.parse_se(t1)
    assert se.nreads == 10000 and int(se.seq_lens.sum()) == 1_000_000
    assert bytes(se.names[:25]) == b"ERR2755197.1 1 length=100"
    pe = fq.parse_pe(t1, t2)
    assert pe.nreads == 20000
    np.testing.assert_array_equal(pe.seq_lens[0::2], se.seq_lens)
    for blk, single in ((se, True), (pe, False)):
        np.testing.assert_array_equal(fq.analyze_ids(blk, single), oracle_py.analyze_ids(blk, single))
    a, b = synth.generate(500, paired=True, seed=1)
    syn = fq.parse_pe(a, b)
    t = fq.analyze_ids(syn, False)
    assert t[0] == 0 and (t == oracle_py.analyze_ids(syn, False)).all()


def test_parse_rejects_truncated():
    import pytest
    with pytest.raises(fq.SeqArcError):
        fq.parse_se(b"@r\nACGT\n+\nII")
