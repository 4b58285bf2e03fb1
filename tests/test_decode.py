"""SeqArc -d path: the host block decoder (sa_decode_block, arc_decode.cpp)
and `seqarc_amd -d` over an archive.  Blocks are produced by the CPU
restatement (the GPU encoder is byte-identical to it, tests/test_gpu_parity.py),
so these run without a GPU.  The reference's own round trip on its test files
("-d reproduces the input MD5") is the bar: the decoded
FASTQ equals the input byte for byte."""
import os
import subprocess

import numpy as np
import pytest

import oracle_py
import synth
from conftest import GOLDEN
from test_oracle import _norm_seq

import fastqueeze_amd as fq

T1 = os.path.join(GOLDEN, "ERR2755197_test_1.fq")
T2 = os.path.join(GOLDEN, "ERR2755197_test_2.fq")
CLI = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "fastqueeze_amd", "bin", "seqarc_amd")


def _roundtrip(t1, t2=None, block_size=fq.BLOCK_SIZE, **kw):
    blocks = fq.blocks_from_fastq(t1, t2, block_size) if t2 else fq.blocks_from_fastq(t1, block_size=block_size)
    tmpl = fq.analyze_ids(blocks[0], t2 is None)
    cfg = fq.Config(bin_mode=int(tmpl[0]), **kw)
    out = []
    for b in blocks:
        enc = oracle_py.encode_block(b, cfg.slevel, cfg.qlevel, cfg.md5, cfg.bin_mode, cfg.lossy)
        lng = bool(b.nreads and int(b.seq_lens.max()) > 0xFFFF)
        d, ok = fq.decode_block(enc, b.text_bytes or b.text1 + b.text2, cfg, tmpl, lng)
        assert np.array_equal(d.name_lens, b.name_lens) and np.array_equal(d.seq_lens, b.seq_lens)
        assert d.names.tobytes() == b.names.tobytes()
        assert np.array_equal(d.seq, _norm_seq(b.seq))
        want_q = oracle_py.rblock(b.qual, cfg.lossy) if cfg.lossy else b.qual
        if not cfg.lossy or not (b.seq != _norm_seq(b.seq)).any():
            assert d.qual.tobytes() == want_q.tobytes()
        out.append(ok)
    return out


def test_reference_pair_bin_mode():
    t1, t2 = open(T1, "rb").read(), open(T2, "rb").read()
    assert all(_roundtrip(t1, t2))          # IDProcess::decodeIDS, PE type 1
    assert all(_roundtrip(t1))              # SE bin mode


@pytest.mark.parametrize("kw", [{}, {"slevel": 4, "qlevel": 3}, {"slevel": 9}, {"md5": False}, {"qlevel": 1}])
def test_tokenizer_configs(kw):
    a, b = synth.generate(2500, paired=True, seed=3)
    assert all(_roundtrip(a, b, block_size=300_000, **kw))


def test_edge_long_and_lossy():
    e = synth.edge_cases()
    oks = _roundtrip(e)
    assert oks == [False]                   # lowercase / non-IUPAC bases come back normalised: MD5 differs
    assert all(_roundtrip(synth.generate(12, read_len=70000, seed=5)[0]))   # compressLen_long
    a, _ = synth.generate(2000, seed=8)
    a = b"\n".join(l if i % 4 != 1 else l.replace(b"N", b"A") for i, l in enumerate(a.split(b"\n")))
    assert all(_roundtrip(a, lossy=1.15))   # qualities come back as rblock output (no quality MD5)
    a, _ = synth.generate(2000, seed=8)     # with N bases: placement uses lossy qualities (reference: fails)
    blk = fq.blocks_from_fastq(a)[0]
    d, ok = fq.decode_block(oracle_py.encode_block(blk, lossy=1.15), blk.text_bytes, fq.Config(lossy=1.15))
    assert d.names.tobytes() == blk.names.tobytes() and d.nreads == blk.nreads


def test_decoder_matches_oracle_decoder():
    a, b = synth.generate(1500, paired=True, seed=9)
    blk = fq.blocks_from_fastq(a, b)[0]
    enc = oracle_py.encode_block(blk)
    d, ok = fq.decode_block(enc, blk.text1 + blk.text2)
    names, nl, seq, sl, qual, ok2 = oracle_py.decode_block(enc, blk.nreads, blk.names.size, blk.seq.size)
    assert ok and ok2 and d.names.tobytes() == names.tobytes() and d.seq.tobytes() == seq.tobytes()
    assert d.qual.tobytes() == qual.tobytes()


def test_rejects_corrupt_block():
    a, _ = synth.generate(500, seed=10)
    blk = fq.blocks_from_fastq(a)[0]
    enc = bytearray(oracle_py.encode_block(blk))
    with pytest.raises(fq.SeqArcError):
        fq.decode_block(bytes(enc[: len(enc) // 2]), blk.text_bytes)
    enc[len(enc) // 2] ^= 0xFF
    try:
        _, ok = fq.decode_block(bytes(enc), blk.text_bytes)
        assert not ok
    except fq.SeqArcError:
        pass


def _write_archive(tmp_path, texts, names, block_size=fq.BLOCK_SIZE):
    paths = []
    for n, t in zip(names, texts):
        p = tmp_path / n
        p.write_bytes(t)
        paths.append(p)
    blocks = fq.blocks_from_fastq(*texts, block_size) if len(texts) == 2 else fq.blocks_from_fastq(texts[0], block_size=block_size)
    tmpl = fq.analyze_ids(blocks[0], len(texts) == 1)
    cfg = fq.Config(bin_mode=int(tmpl[0]))
    enc = [oracle_py.encode_block(b, bin_mode=cfg.bin_mode) for b in blocks]
    arc = fq.arc_archive(enc, blocks, names[0], names[1] if len(names) > 1 else None, tmpl, cfg,
                         plus_bare=fq.bare_plus(texts[-1]))
    ap = tmp_path / "in.arc"
    ap.write_bytes(arc)
    return ap


def test_cli_decode_reference_pair(tmp_path):
    texts = [open(T1, "rb").read(), open(T2, "rb").read()]
    ap = _write_archive(tmp_path, texts, ["ERR2755197_test_1.fq", "ERR2755197_test_2.fq"])
    r = subprocess.run([CLI, "-d", "-t", "2", str(ap), str(tmp_path / "out")], capture_output=True, text=True,
                       timeout=120)
    assert r.returncode == 0, r.stderr
    assert (tmp_path / "out_1.fastq").read_bytes() == texts[0]
    assert (tmp_path / "out_2.fastq").read_bytes() == texts[1]


def test_cli_decode_multi_block_se(tmp_path):
    t, _ = synth.generate(6000, seed=12)
    ap = _write_archive(tmp_path, [t], ["s.fq"], block_size=400_000)
    r = subprocess.run([CLI, "-d", "-t", "3", str(ap), str(tmp_path / "se")], capture_output=True, text=True,
                       timeout=120)
    assert r.returncode == 0, r.stderr
    assert (tmp_path / "se.fastq").read_bytes() == t


@pytest.mark.parametrize("kind", [1, 2, 3])
def test_bin_mode_pe_types(kind):
    """ID-bin names of the three PE types (analysisPEType@0x430f50 / decodeIDS@0x430610):
    1 identical mate IDs, 2 '/1' -> '/2', 3 '... length=' + the mate's own length."""
    rng = np.random.default_rng(kind)

    def rec(name, n):
        s = rng.choice(np.frombuffer(b"ACGT", np.uint8), n).tobytes()
        q = rng.choice(np.frombuffer(b"F:,", np.uint8), n).tobytes()
        return b"@" + name + b"\n" + s + b"\n+\n" + q + b"\n"

    r1, r2 = [], []
    for i in range(500):
        l1, l2 = 100 + i % 7, 90 + i % 5
        if kind == 1:
            n1 = n2 = b"SRR9.%d %d length=%d" % (i + 1, i + 1, l1)
            l2 = l1
        elif kind == 2:
            n1, n2 = b"SRR9.%d %d/1" % (i + 1, i + 1), b"SRR9.%d %d/2" % (i + 1, i + 1)
        else:
            n1, n2 = b"SRR9.%d %d length=%d" % (i + 1, i + 1, l1), b"SRR9.%d %d length=%d" % (i + 1, i + 1, l2)
        r1.append(rec(n1, l1))
        r2.append(rec(n2, l2))
    t1, t2 = b"".join(r1), b"".join(r2)
    blk = fq.blocks_from_fastq(t1, t2)[0]
    tmpl = fq.analyze_ids(blk, False)
    assert (tmpl[0], tmpl[1]) == (1, kind)
    cfg = fq.Config(bin_mode=1)
    d, ok = fq.decode_block(oracle_py.encode_block(blk, bin_mode=1), blk.text1 + blk.text2, cfg, tmpl)
    assert ok and d.names.tobytes() == blk.names.tobytes() and np.array_equal(d.name_lens, blk.name_lens)


def test_cli_decode_reference_shm(tmp_path):
    """-s (README.md:32, IHashRefIndex::createShm@0x41f280 /
    HashRefIndex32::loadRefIndexShm@0x41ef80): the first -d with -s copies
    ref.fa.hash into /dev/shm/<ref file name>, later runs map it instead of
    reading the file; an object of another size is refused ("is wrong file")."""
    import hashlib
    name = f"sa_shm_test_{os.getpid()}.fa"
    shm = os.path.join("/dev/shm", name)
    fa, g = synth.reference(150_000, 71, chroms=2)
    fa = fa.upper()
    (tmp_path / name).write_bytes(fa)
    hfile = oracle_py.hash_index(fa, k=10)   # (the decoder reads the genome words; K = 10 keeps the image at 8 MB)
    (tmp_path / (name + ".hash")).write_bytes(hfile)
    (tmp_path / (name + ".md5")).write_bytes(hashlib.md5(fa).digest())
    r1, r2 = synth.aligned_reads(g, 500, 72, paired=True, random_frac=0.1)
    blocks = fq.blocks_from_fastq(r1, r2, 1 << 16)
    tmpl = fq.analyze_ids(blocks[0], False)
    cfg = fq.Config(bin_mode=int(tmpl[0]))
    carry = [0, 0]
    enc = [oracle_py.encode_block_hash(b, True, carry, bin_mode=cfg.bin_mode) for b in blocks]
    arc = fq.arc_archive(enc, blocks, "a_1.fq", "a_2.fq", tmpl, cfg, plus_bare=fq.bare_plus(r1),
                         ref_md5=hashlib.md5(fa).digest())
    (tmp_path / "a.arc").write_bytes(arc)
    run = lambda args: subprocess.run([CLI] + args, capture_output=True, text=True, cwd=tmp_path, timeout=120)
    try:
        if os.path.exists(shm):
            os.remove(shm)
        r = run(["-d", "-s", "-v", name, "a.arc", "b1"])
        assert r.returncode == 0, r.stderr
        assert open(shm, "rb").read() == hfile
        assert (tmp_path / "b1_1.fastq").read_bytes() == r1 and (tmp_path / "b1_2.fastq").read_bytes() == r2
        os.remove(tmp_path / (name + ".hash"))   # from now on only the shared-memory image has the index
        r = run(["-d", "-s", "-v", name, "a.arc", "b2"])
        assert r.returncode == 0, r.stderr
        assert "from /dev/shm/" in r.stderr
        assert (tmp_path / "b2_1.fastq").read_bytes() == r1 and (tmp_path / "b2_2.fastq").read_bytes() == r2
        with open(shm, "r+b") as f:
            f.truncate(len(hfile) - 4)
        r = run(["-d", "-s", name, "a.arc", "b3"])
        assert r.returncode != 0 and "is wrong file" in r.stderr
    finally:
        for f in (shm, shm + ".sa_ref"):
            if os.path.exists(f):
                os.remove(f)


def test_cli_shm_two_references_same_name(tmp_path):
    """the shared-memory image is keyed by the reference's file name
    (loadRefIndexShm@0x41ef80), so two references of one name -- a/ref.fa and
    b/ref.fa -- would share it.  The object is bound to its FASTA's MD5 (the
    /dev/shm/<name>.sa_ref tag): -d -s with b/ref.fa does not decode against
    a's genome; it reads b's .hash and republishes; with b's image in /dev/shm
    and a's .hash gone, -d -s with a/ref.fa is refused."""
    import hashlib
    name = f"sa_shm_two_{os.getpid()}.fa"
    shm = os.path.join("/dev/shm", name)
    run = lambda args: subprocess.run([CLI] + args, capture_output=True, text=True, cwd=tmp_path, timeout=120)
    arcs = {}
    for d, seed in (("a", 81), ("b", 82)):
        (tmp_path / d).mkdir()
        fa, g = synth.reference(150_000, seed, chroms=2)
        fa = fa.upper()
        (tmp_path / d / name).write_bytes(fa)
        (tmp_path / d / (name + ".hash")).write_bytes(oracle_py.hash_index(fa, k=10))
        (tmp_path / d / (name + ".md5")).write_bytes(hashlib.md5(fa).digest())
        r1, r2 = synth.aligned_reads(g, 400, seed + 10, paired=True, random_frac=0.1)
        blocks = fq.blocks_from_fastq(r1, r2, 1 << 16)
        tmpl = fq.analyze_ids(blocks[0], False)
        cfg = fq.Config(bin_mode=int(tmpl[0]))
        carry = [0, 0]
        enc = [oracle_py.encode_block_hash(b, True, carry, bin_mode=cfg.bin_mode) for b in blocks]
        (tmp_path / f"{d}.arc").write_bytes(fq.arc_archive(enc, blocks, "x_1.fq", "x_2.fq", tmpl, cfg,
                                                           plus_bare=fq.bare_plus(r1),
                                                           ref_md5=hashlib.md5(fa).digest()))
        arcs[d] = (r1, r2)
    try:
        for f in (shm, shm + ".sa_ref"):
            if os.path.exists(f):
                os.remove(f)
        r = run(["-d", "-s", f"a/{name}", "a.arc", "ra"])
        assert r.returncode == 0, r.stderr
        assert (tmp_path / "ra_1.fastq").read_bytes() == arcs["a"][0]
        # b's reference under the same name: not decoded against a's image
        r = run(["-d", "-s", "-v", f"b/{name}", "b.arc", "rb"])
        assert r.returncode == 0, r.stderr
        assert "from /dev/shm/" not in r.stderr
        assert (tmp_path / "rb_1.fastq").read_bytes() == arcs["b"][0]
        assert (tmp_path / "rb_2.fastq").read_bytes() == arcs["b"][1]
        assert open(shm, "rb").read() == (tmp_path / "b" / (name + ".hash")).read_bytes()   # republished
        # a's .hash gone, b's image in /dev/shm: refused, not decoded wrongly
        os.remove(tmp_path / "a" / (name + ".hash"))
        r = run(["-d", "-s", f"a/{name}", "a.arc", "ra2"])
        assert r.returncode != 0 and "is not the index of" in r.stderr, r.stderr
        # b maps its own image with its .hash gone
        os.remove(tmp_path / "b" / (name + ".hash"))
        r = run(["-d", "-s", "-v", f"b/{name}", "b.arc", "rb2"])
        assert r.returncode == 0 and "from /dev/shm/" in r.stderr, r.stderr
        assert (tmp_path / "rb2_1.fastq").read_bytes() == arcs["b"][0]
    finally:
        for f in (shm, shm + ".sa_ref"):
            if os.path.exists(f):
                os.remove(f)
