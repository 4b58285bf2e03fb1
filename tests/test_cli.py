"""The seqarc_amd command line without a GPU: the decode side (-d, -P, -f, -p,
output naming of SeqArcParam::getDecodeFile@0x405f70) on archives built from
the CPU restatement's blocks, and the streaming block cut the -c reader uses
(sa_cut_next_se / sa_cut_next_pe) against the whole-buffer cut."""
import ctypes as C
import hashlib
import os
import subprocess

import numpy as np
import pytest

import oracle_py
import synth
from conftest import GOLDEN

import fastqueeze_amd as fq
from fastqueeze_amd import build

EXE = build.CLI


def _write_archive(tmp_path, texts, names, arc="t.arc", block_size=fq.BLOCK_SIZE, gz1=False):
    blocks = fq.blocks_from_fastq(texts[0], texts[1] if len(texts) > 1 else None, block_size)
    tmpl = fq.analyze_ids(blocks[0], len(texts) == 1)
    cfg = fq.Config(bin_mode=int(tmpl[0]))
    enc = [oracle_py.encode_block(b, cfg.slevel, cfg.qlevel, cfg.md5, cfg.bin_mode) for b in blocks]
    data = fq.arc_archive(enc, blocks, names[0], names[1] if len(names) > 1 else None, tmpl, cfg, gz1=gz1,
                          plus_bare=fq.bare_plus(texts[-1]))
    path = tmp_path / arc
    path.write_bytes(data)
    return str(path), len(blocks)


def _run(args, cwd, env=None):
    return subprocess.run([EXE] + args, capture_output=True, cwd=cwd, timeout=300,
                          env=None if env is None else dict(os.environ, **env))


def _records(text):
    lines = text.split(b"\n")
    return [b"\n".join(lines[i:i + 4]) + b"\n" for i in range(0, len(lines) - 1, 4)]


@pytest.fixture(scope="module")
def pair():
    a, b = synth.generate(3000, paired=True, seed=61)
    return a, b


def test_pipe_out_se_pe1_pe2_interleaved(tmp_path, pair):
    """-P 1 / 2 / 3 (DecodePipeOutJob::recoverData*@0x42f930): SE reads, PE1,
    PE2 and each pair in order, on stdout, over a multi-block archive."""
    a, b = pair
    arc, nb = _write_archive(tmp_path, (a, b), ["p_1.fq", "p_2.fq"], block_size=200_000)
    assert nb > 3
    assert _run(["-d", "-P", "1", arc], tmp_path).stdout == a
    assert _run(["-d", "-P", "2", arc], tmp_path).stdout == b
    inter = b"".join(x + y for x, y in zip(_records(a), _records(b)))
    assert _run(["-d", "-t", "4", "-P", "3", arc], tmp_path).stdout == inter
    se, _ = _write_archive(tmp_path, (a,), ["s.fq"], arc="s.arc", block_size=150_000)
    assert _run(["-d", "-P", "1", se], tmp_path).stdout == a
    with open(os.path.join(GOLDEN, "ERR2755197_test_1.fq"), "rb") as f:
        t1 = f.read()
    ref, _ = _write_archive(tmp_path, (t1,), ["ERR2755197_test_1.fq"], arc="r.arc")
    assert _run(["-d", "-P", "1", ref], tmp_path).stdout == t1   # ID-bin names, bare '+'


def test_decode_names_force_and_dir(tmp_path, pair):
    """Outputs: PREFIX_1/_2.fastq (PE) or PREFIX.fastq (SE) (appendname@0x405f10);
    without a prefix the stored input names (3 more bytes cut after a gzip
    input 1, as the binary does); an existing output stops the run ("has
    exist!") unless -f; -p writes next to the archive."""
    a, b = pair
    sub = tmp_path / "arcdir"
    sub.mkdir()
    arc, _ = _write_archive(sub, (a, b), ["m_1.fq", "m_2.fq"])
    r = _run(["-d", arc, "back"], tmp_path)
    assert r.returncode == 0, r.stderr
    assert (tmp_path / "back_1.fastq").read_bytes() == a and (tmp_path / "back_2.fastq").read_bytes() == b
    r = _run(["-d", arc, "-o", "back"], tmp_path)
    assert r.returncode == 1 and b"has exist!" in r.stderr
    r = _run(["-d", "-f", arc, "-o", "back"], tmp_path)
    assert r.returncode == 0
    r = _run(["-d", arc], tmp_path)   # the stored names
    assert r.returncode == 0 and (tmp_path / "m_1.fq").read_bytes() == a and (tmp_path / "m_2.fq").read_bytes() == b
    r = _run(["-d", "-p", arc, "x"], tmp_path)
    assert r.returncode == 0 and (sub / "x_1.fastq").read_bytes() == a
    se, _ = _write_archive(tmp_path, (a,), ["reads.fq.gz"], arc="se.arc", gz1=True)
    r = _run(["-d", se, "s"], tmp_path)
    assert r.returncode == 0 and (tmp_path / "s.fastq").read_bytes() == a
    r = _run(["-d", se], tmp_path)   # "reads.fq" stored, 3 more bytes cut for the gzip input
    assert r.returncode == 0 and (tmp_path / "reads").read_bytes() == a


def test_compress_usage_errors(tmp_path):
    """-c argument checks that need no GPU: missing / empty input, -q (the
    minimizer index, not part of this build), a missing reference."""
    r = _run(["-c", "-1", str(tmp_path / "missing.fq"), "-o", "x"], tmp_path)
    assert r.returncode == 1 and b"may be not exist or empty" in r.stderr
    (tmp_path / "e.fq").write_bytes(b"")
    r = _run(["-c", "-1", str(tmp_path / "e.fq"), "x"], tmp_path)
    assert r.returncode == 1
    r = _run(["-q", "-i", "ref.fa"], tmp_path)
    assert r.returncode == 2
    r = _run(["-i", str(tmp_path / "missing.fa")], tmp_path)
    assert r.returncode == 1 and b"may be not exist" in r.stderr
    r = _run(["-c", "--maxmis", "9", "-1", str(tmp_path / "e.fq"), "x"], tmp_path)   # (no Mis model beyond 8)
    assert r.returncode == 2 and b"0..8" in r.stderr


@pytest.mark.parametrize("maxmis,field19", [(0, True), (3, True), (8, True), (8, False), (0, False)])
def test_decode_reference_maxmis_from_archive(tmp_path, maxmis, field19):
    """An archive of the reference path made with a non-default maxmis carries it
    (params field 19, ours; SeqArc keeps maxmis in ./seqarc.config and stores
    none): -d rebuilds the Mis model without being told.  An archive without
    field 19 (SeqArc's own, or an earlier build's) takes -d --maxmis M (ADVICE
    r4: the option was accepted and ignored)."""
    fa, g = synth.reference(600_000, 73, chroms=2)
    fa = fa.upper()
    (tmp_path / "ref.fa").write_bytes(fa)
    (tmp_path / "ref.fa.hash").write_bytes(oracle_py.hash_index(fa))
    r1, _ = synth.aligned_reads(g, 2000, 74, short_frac=0.2)
    blocks = fq.blocks_from_fastq(r1, None, block_size=120_000)
    tmpl = fq.analyze_ids(blocks[0], True)
    cfg = fq.Config(bin_mode=int(tmpl[0]))
    carry = [0, 0]
    enc = [oracle_py.encode_block_hash(b, False, carry, bin_mode=cfg.bin_mode, maxmis=maxmis) for b in blocks]
    data = fq.arc_archive(enc, blocks, "s.fq", None, tmpl, cfg, plus_bare=fq.bare_plus(r1),
                          ref_md5=hashlib.md5(fa).digest(), maxmis=maxmis if field19 else 7)
    (tmp_path / "a.arc").write_bytes(data)
    r = _run(["-d", "-t", "2"] + ([] if field19 else ["--maxmis", str(maxmis)]) + ["ref.fa", "a.arc", "back"],
             tmp_path)
    assert r.returncode == 0, r.stderr
    assert (tmp_path / "back.fastq").read_bytes() == r1
    if not field19 and maxmis == 8:   # (without the option: the Mis model of 8 symbols, not 9)
        r = _run(["-d", "-f", "-t", "2", "ref.fa", "a.arc", "back"], tmp_path)
        assert r.returncode != 0 or (tmp_path / "back.fastq").read_bytes() != r1


@pytest.mark.parametrize("paired,with_hash", [(False, True), (True, False), (True, True)])
def test_decode_with_reference(tmp_path, paired, with_hash):
    """SeqArc -d ref.fa ARCHIVE PREFIX on an archive of the reference path
    (blocks from the oracle's doAlignEncode restatement, trailer field 1 = 0,
    the FASTA's MD5 after the params, writeMd5@0x416b10): the genome from
    ref.fa.hash or, without it, packed from ref.fa; the MD5 checked
    (checkMd5@0x416c40); no reference or another one: refused."""
    fa, g = synth.reference(800_000, 71, chroms=2)
    fa = fa.upper()
    hfile = oracle_py.hash_index(fa)
    (tmp_path / "ref.fa").write_bytes(fa)
    if with_hash:
        (tmp_path / "ref.fa.hash").write_bytes(hfile)
    r1, r2 = synth.aligned_reads(g, 2500, 72, paired=paired, random_frac=0.2, far_frac=0.3, short_frac=0.2)
    blocks = fq.blocks_from_fastq(r1, r2, block_size=150_000)
    assert len(blocks) >= 3
    tmpl = fq.analyze_ids(blocks[0], not paired)
    cfg = fq.Config(bin_mode=int(tmpl[0]))
    carry = [0, 0]
    ins = 400 if paired and with_hash else 0
    enc = [oracle_py.encode_block_hash(b, paired, carry, bin_mode=cfg.bin_mode, insert_size=ins) for b in blocks]
    data = fq.arc_archive(enc, blocks, "a_1.fq", "a_2.fq" if paired else None, tmpl, cfg,
                          plus_bare=fq.bare_plus(r1), ref_md5=hashlib.md5(fa).digest(), insert_size=ins)
    (tmp_path / "a.arc").write_bytes(data)
    r = _run(["-d", "-t", "3", "ref.fa", "a.arc", "back"], tmp_path)
    assert r.returncode == 0, r.stderr
    if paired:
        assert (tmp_path / "back_1.fastq").read_bytes() == r1 and (tmp_path / "back_2.fastq").read_bytes() == r2
    else:
        assert (tmp_path / "back.fastq").read_bytes() == r1
    r = _run(["-d", "-f", "a.arc", "x"], tmp_path)
    assert r.returncode == 1 and b"made with a reference" in r.stderr
    (tmp_path / "other.fa").write_bytes(fa.replace(b"ACGT", b"ACGA", 1))
    r = _run(["-d", "-f", "other.fa", "a.arc", "x"], tmp_path)
    assert r.returncode == 1 and b"MD5" in r.stderr


def _stream_cut(t1, t2, bs, step):
    """The -c reader's loop over windows that grow `step` bytes at a time."""
    lib = fq.load_library()
    lib.sa_cut_next_se.argtypes = [C.c_void_p, C.c_uint64, C.c_int, C.c_uint64, C.c_void_p, C.c_uint64]
    lib.sa_cut_next_se.restype = C.c_int64
    lib.sa_cut_next_pe.argtypes = [C.c_void_p, C.c_uint64, C.c_int, C.c_void_p, C.c_uint64, C.c_int, C.c_uint64,
                                   C.c_void_p, C.c_uint64, C.c_void_p, C.c_void_p]
    lib.sa_cut_next_pe.restype = C.c_int
    a = np.frombuffer(t1, np.uint8)
    b = np.frombuffer(t2, np.uint8) if t2 is not None else None
    first = a[: int(np.flatnonzero(a == 10)[0]) + 1].copy()
    o1 = o2 = 0
    h1 = h2 = 0   # bytes "read" so far
    out = []
    while o1 < a.size or (b is not None and o2 < b.size):
        h1 = min(a.size, max(h1, o1 + step))
        w1 = a[o1:h1]
        eof1 = int(h1 == a.size)
        if b is None:
            e = lib.sa_cut_next_se(w1.ctypes.data, w1.size, eof1, bs, first.ctypes.data, first.size)
            if e < 0:
                assert not eof1
                h1 += step
                continue
            out.append((o1, o1 + e))
            o1 += e
        else:
            h2 = min(b.size, max(h2, o2 + step))
            w2 = b[o2:h2]
            eof2 = int(h2 == b.size)
            e1, e2 = C.c_uint64(0), C.c_uint64(0)
            if lib.sa_cut_next_pe(w1.ctypes.data, w1.size, eof1, w2.ctypes.data, w2.size, eof2, bs,
                                  first.ctypes.data, first.size, C.byref(e1), C.byref(e2)) != 0:
                assert not (eof1 and eof2)
                h1 += step
                h2 += step
                continue
            out.append(((o1, o1 + e1.value), (o2, o2 + e2.value)))
            o1 += e1.value
            o2 += e2.value
    return out


@pytest.mark.parametrize("step", [70_000, 1 << 20])
def test_streaming_cut_equals_whole_buffer_cut(pair, step):
    a, b = pair
    bs = 300_000
    assert _stream_cut(a, None, bs, step) == [tuple(x) for x in fq.cut_se(a, bs)]
    _, short = synth.generate(3000, paired=True, seed=62, read_len=90)   # mates of unequal length
    assert _stream_cut(a, short, bs, step) == [tuple(map(tuple, x)) for x in fq.cut_pe(a, short, bs)]
    assert _stream_cut(a, b, bs, step) == [tuple(map(tuple, x)) for x in fq.cut_pe(a, b, bs)]


def test_host_only_reader_matches_the_cut(tmp_path):
    """-c --host-only: the streaming reader (parallel pread slices once a window
    is >= 16 MiB, counted PE cut, recycled windows) and the host parser, with no
    device: the block count and bytes read equal the whole-buffer cut's, for
    several block sizes, PE and SE."""
    a, b = synth.generate(70_000, paired=True, seed=63)   # ~2 x 25 MB: full 25 MiB PE windows
    pa, pb = tmp_path / "h_1.fq", tmp_path / "h_2.fq"
    pa.write_bytes(a)
    pb.write_bytes(b)
    for mib in (1, 8, 50):
        r = _run(["-c", "-f", "--host-only", "--block-size", str(mib), "-1", str(pa), "-2", str(pb), "-o",
                  str(tmp_path / "h")], tmp_path)
        assert r.returncode == 0, r.stderr
        want = len(fq.cut_pe(a, b, mib << 20))
        line = [ln for ln in r.stderr.decode().splitlines() if "block(s)" in ln][0]
        assert line.split()[1] == str(want) and f" {len(a) + len(b)} -> " in line, (mib, line)
        r = _run(["-c", "-f", "--host-only", "--block-size", str(mib), "-1", str(pa), "-o", str(tmp_path / "s")],
                 tmp_path)
        assert r.returncode == 0, r.stderr
        line = [ln for ln in r.stderr.decode().splitlines() if "block(s)" in ln][0]
        assert line.split()[1] == str(len(fq.cut_se(a, mib << 20))) and f" {len(a)} -> " in line, (mib, line)


def test_ingest_only_eight_way(tmp_path, capsys):
    """The -c reader and block cut alone (--ingest-only) feeding 8 devices x 1
    context of consumers, as a whole-node run deals batches: the block count and
    bytes equal the whole-buffer cut, and the ingest MB/s is reported."""
    a, b = synth.generate(60_000, paired=True, seed=64)
    pa, pb = tmp_path / "i_1.fq", tmp_path / "i_2.fq"
    pa.write_bytes(a)
    pb.write_bytes(b)
    want = len(fq.cut_pe(a, b, 1 << 20))
    rates = {}
    for dev in (1, 8):
        r = _run(["-c", "-f", "--ingest-only", "--devices", str(dev), "--contexts", "1", "--batch", "2",
                  "--block-size", "1", "-1", str(pa), "-2", str(pb), "-o", str(tmp_path / "g")], tmp_path)
        assert r.returncode == 0, r.stderr
        line = [ln for ln in r.stderr.decode().splitlines() if "block(s)" in ln][0]
        assert line.split()[1] == str(want) and f" {len(a) + len(b)} -> " in line, line
        rates[dev] = float(line.split()[-2])
    with capsys.disabled():
        print(f"\n[ingest] reader + PE cut, 1 MiB blocks: 1 consumer {rates[1]:.0f} MB/s, "
              f"8 consumers {rates[8]:.0f} MB/s")


def _bgzf(data: bytes, level: int = 1) -> bytes:
    """bgzip's format: gzip members of <= 64 KiB input with the 'BC' extra field
    (the member size), then the 28-byte empty end-of-file member."""
    import struct
    import zlib
    out = bytearray()
    for i in range(0, len(data), 65280):
        chunk = data[i:i + 65280]
        c = zlib.compressobj(level, zlib.DEFLATED, -15)
        cd = c.compress(chunk) + c.flush()
        out += b"\x1f\x8b\x08\x04\x00\x00\x00\x00\x00\xff\x06\x00BC\x02\x00"
        out += struct.pack("<H", 18 + len(cd) + 8 - 1) + cd + struct.pack("<II", zlib.crc32(chunk), len(chunk))
    return bytes(out) + bytes.fromhex("1f8b08040000000000ff0600424302001b0003000000000000000000")


def test_gzip_ingest_plain_multimember_bgzf(tmp_path, capsys):
    """gzip inputs through the inflate-ahead reader: one member, concatenated
    members and BGZF (members inflated in parallel) give the same blocks and
    the same text (CRC-32 over every block's text in order) as the plain file;
    a truncated gzip file is an error.  The ingest MB/s of each is reported."""
    import gzip
    a, b = synth.generate(40_000, paired=True, seed=65)
    files = {"plain": (a, b), "plain_windows": (a, b), "plain_segments": (a, b),
             "gz": (gzip.compress(a, 1), gzip.compress(b, 1)),
             "multi": (gzip.compress(a[:len(a) // 3], 1) + gzip.compress(a[len(a) // 3:], 1),
                       gzip.compress(b[:7], 1) + gzip.compress(b[7:], 1)),
             "bgzf": (_bgzf(a), _bgzf(b))}
    got = {}
    for k, (x, y) in files.items():
        p1, p2 = tmp_path / f"{k}_1.fq", tmp_path / f"{k}_2.fq"
        p1.write_bytes(x)
        p2.write_bytes(y)
        # plain: the segment reader (SegReader); plain_windows: the per-block window reader;
        # plain_segments: 4 MiB segments in a ring of 4 (every slot refilled)
        extra = ["--read-threads", "0"] if k == "plain_windows" else []
        env = {"SA_CLI_SEG_SLICES": "1"} if k == "plain_segments" else None
        r = _run(["-c", "-f", "--ingest-only", "--ingest-crc", "--devices", "2", "--contexts", "2", "--batch", "2",
                  "--block-size", "1", "-t", "8"] + extra + ["-1", str(p1), "-2", str(p2), "-o", str(tmp_path / k)],
                 tmp_path, env=env)
        assert r.returncode == 0, (k, r.stderr)
        err = r.stderr.decode()
        crc = [ln for ln in err.splitlines() if "crc32" in ln][0].split()[-1]
        line = [ln for ln in err.splitlines() if "block(s)" in ln][0]
        got[k] = (crc, line.split()[1], line.split(" -> ")[0].split()[-1], float(line.split()[-2]))
    assert len({v[:3] for v in got.values()}) == 1, got
    assert got["plain"][1] == str(len(fq.cut_pe(a, b, 1 << 20)))
    bad = tmp_path / "bad_1.fq"
    bad.write_bytes(files["gz"][0][: len(files["gz"][0]) // 2])
    r = _run(["-c", "-f", "--ingest-only", "-1", str(bad), "-o", str(tmp_path / "bad")], tmp_path)
    assert r.returncode != 0
    # BGZF cut inside a member, and with bytes that are no member after the last
    for k, data in (("bgzf_cut", files["bgzf"][0][: len(files["bgzf"][0]) * 2 // 3]),
                    ("bgzf_tail", files["bgzf"][0] + b"\x1f\x8bjunk")):
        bad = tmp_path / f"{k}_1.fq"
        bad.write_bytes(data)
        r = _run(["-c", "-f", "--ingest-only", "-t", "4", "-1", str(bad), "-o", str(tmp_path / k)], tmp_path)
        assert r.returncode != 0, k
    with capsys.disabled():
        print("\n[ingest] " + ", ".join(f"{k} {v[3]:.0f} MB/s" for k, v in got.items()))


def test_ingest_ring_at_its_floor(tmp_path):
    """The segment ring at its floor: a batch's blocks keep
    their segments until the batch is taken, so a ring smaller than one batch of
    windows plus two segments deadlocks (r5i, fixed in be7581d by the floor in
    SegReader::start).  4 MiB segments, 1 MiB blocks (576 KiB windows per file),
    32-block batches spanning four segments of each file, six consumers,
    SA_CLI_RING_SEGS=3 (clamped up to the floor, 7): the run ends in bounded
    time and delivers the same text (CRC-32 over the blocks in order) as an
    unconstrained ring.  (Checked when written: the same command with the
    floor removed from the build hangs.)"""
    a, b = synth.generate(60_000, paired=True, seed=66)
    p1, p2 = tmp_path / "r_1.fq", tmp_path / "r_2.fq"
    p1.write_bytes(a)
    p2.write_bytes(b)
    crcs = {}
    for name, env in (("floor", {"SA_CLI_SEG_SLICES": "1", "SA_CLI_RING_SEGS": "3"}), ("default", {})):
        r = subprocess.run([EXE, "-c", "-f", "--ingest-only", "--ingest-crc", "--devices", "2", "--contexts", "3",
                            "--batch", "32", "--block-size", "1", "-1", str(p1), "-2", str(p2), "-o",
                            str(tmp_path / name)], capture_output=True, cwd=tmp_path, timeout=120,
                           env=dict(os.environ, **env))
        assert r.returncode == 0, (name, r.stderr)
        err = r.stderr.decode()
        crcs[name] = ([ln for ln in err.splitlines() if "crc32" in ln][0].split()[-1],
                      [ln for ln in err.splitlines() if "block(s)" in ln][0].split()[1])
    assert crcs["floor"] == crcs["default"]
    assert crcs["floor"][1] == str(len(fq.cut_pe(a, b, 1 << 20)))


def test_archive_writer_reports_a_full_file_system(tmp_path):
    """The archive writer (ArcWriter) copies blocks into maps of the file's
    pages only where fallocate allocated them; elsewhere it uses pwrite.  A
    store into a page the file system cannot back raises SIGBUS (the
    process died silently with a partial archive); here the file cannot grow
    past RLIMIT_FSIZE (ftruncate / pwrite fail with EFBIG, SIGXFSZ ignored):
    the run must end with "write error" and a non-zero status, not a signal.
    The blocks are SA_CLI_TEST_OUT bytes of filler (--host-only: no device)."""
    import resource
    import signal
    a, b = synth.generate(20_000, paired=True, seed=67)
    p1, p2 = tmp_path / "w_1.fq", tmp_path / "w_2.fq"
    p1.write_bytes(a)
    p2.write_bytes(b)
    nblk = len(fq.cut_pe(a, b, 1 << 20))
    args = [EXE, "-c", "-f", "--host-only", "--block-size", "1", "-1", str(p1), "-2", str(p2)]
    env = dict(os.environ, SA_CLI_TEST_OUT="200000")
    ok = subprocess.run(args + ["-o", str(tmp_path / "ok")], capture_output=True, cwd=tmp_path, timeout=120, env=env)
    assert ok.returncode == 0, ok.stderr
    arc = (tmp_path / "ok.arc").read_bytes()
    assert arc[16:16 + nblk * 200000] == b"\x5a" * (nblk * 200000)

    def limit():
        signal.signal(signal.SIGXFSZ, signal.SIG_IGN)
        resource.setrlimit(resource.RLIMIT_FSIZE, (600_000, 600_000))

    r = subprocess.run(args + ["-o", str(tmp_path / "full")], capture_output=True, cwd=tmp_path, timeout=120,
                       env=env, preexec_fn=limit)
    assert r.returncode == 1, (r.returncode, r.stderr)
    assert b"write error" in r.stderr, r.stderr
