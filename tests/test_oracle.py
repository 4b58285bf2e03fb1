"""Oracle pinning (CPU): the restatement against the reference-run sizes recorded
in SURVEY.md section 6, RFC 1321 vectors, and the committed golden digests."""
import hashlib
import json
import os
import re
import subprocess

import numpy as np
import pytest

import oracle_py
import synth
from conftest import GOLDEN, ROOT, TEST1, TEST2

import fastqueeze_amd as fq


def _encaps(block: bytes):
    """Split a block (81 size4 ...) into {encap id: total encap length}."""
    assert block[0] == 0x81
    size = int.from_bytes(block[1:5], "big") & 0x0FFFFFFF
    assert size == len(block) - 5
    p, out = 5, {}
    while p < len(block):
        eid = block[p] & 0x7F
        if eid == 1:  # count: 81 84 u32
            out[1] = 6
            p += 6
            continue
        ln = int.from_bytes(block[p + 1:p + 5], "big") & 0x0FFFFFFF
        out[eid] = 1 + 4 + ln
        p += 5 + ln
    assert p == len(block)
    return out


def test_rfc1321_vectors():
    vec = {b"": "d41d8cd98f00b204e9800998ecf8427e", b"a": "0cc175b9c0f1b6a831c399e269772661",
           b"abc": "900150983cd24fb0d6963f7d28e17f72",
           b"message digest": "f96b697d7cb7938d525a2f31aaf161d0",
           b"12345678901234567890123456789012345678901234567890123456789012345678901234567890":
               "57edf4a22be3c955ac49da2e2107b67a"}
    for m, h in vec.items():
        assert oracle_py.md5(m).hex() == h
    data = bytes(range(256)) * 300
    assert oracle_py.md5(data) == hashlib.md5(data).digest()


def test_reference_size_pins(test_pair):
    """reference `SeqArc -c -t 1` on the test PE pair printed
    name 48, seq 74,610 (seq + len + dege encaps), qual 746,149 compressed bytes."""
    blocks = fq.blocks_from_fastq(*test_pair)
    assert len(blocks) == 1 and blocks[0].nreads == 20000
    tmpl = oracle_py.analyze_ids(blocks[0], False)
    assert (tmpl[0], tmpl[1]) == (1, 1)          # "bOrderBin 1 petype 1"
    enc = _encaps(oracle_py.encode_block(blocks[0], bin_mode=1))
    assert enc[5] == 48
    assert enc[7] == 746149
    assert enc[6] + enc[4] + sum(enc.get(i, 0) for i in (23, 14, 24, 25, 26)) == 74610
    # orgsize columns of the same table: name 655,576 = IDs + 2/read; seq 2,020,000
    assert int(blocks[0].name_lens.sum()) + 2 * 20000 == 655576
    assert int(blocks[0].seq_lens.sum()) + 20000 == 2020000



@pytest.fixture(scope="module")
def golden():
    import sys
    sys.path.insert(0, GOLDEN)
    import make_golden
    with open(os.path.join(GOLDEN, "golden.json")) as f:
        return make_golden, json.load(f)


@pytest.mark.parametrize("name", ["test_pe", "test_se", "test_pe_600k", "synth_pe_4k", "synth_pe_4k_s4",
                                  "synth_se_4k_q3", "edge_se", "edge_se_s9", "test_pe_lossy_115",
                                  "synth_se_lossy_16", "synth_long_70k"])
def test_oracle_golden(golden, name):
    mg, g = golden
    case = g[name]["case"]
    blocks, tmpl, outs = mg.run_case(case)
    assert [len(o) for o in outs] == g[name]["blocks"]
    assert hashlib.sha256(b"".join(outs)).hexdigest() == g[name]["sha256"]


def test_cpu_decomposition(tmp_path):
    """The GPU decomposition (sa_logic.h driven on the host) equals the oracle."""
    exe = tmp_path / "emu"
    src = os.path.join(ROOT, "tests", "cpu_emu", "emu.cpp")
    subprocess.run(["g++", "-O2", "-std=c++17", "-o", str(exe), src,
                    os.path.join(ROOT, "fastqueeze_amd", "csrc", "fastq_host.cpp"),
                    os.path.join(ROOT, "oracle", "fqz_oracle.c"), os.path.join(ROOT, "oracle", "hash_oracle.c"),
                    os.path.join(ROOT, "oracle", "align_oracle.c"), "-lm"], check=True)
    import synth
    pe1, pe2 = synth.generate(3000, paired=True, seed=3)
    (tmp_path / "a.fq").write_bytes(pe1)
    (tmp_path / "b.fq").write_bytes(pe2)
    (tmp_path / "e.fq").write_bytes(synth.edge_cases())
    (tmp_path / "long.fq").write_bytes(synth.generate(12, read_len=70000, seed=5)[0])
    # R-Block runs that span whole 8 KiB chunks (constant or two-level qualities):
    # the run values reach the chunks' bytes through rb_chase
    rng = np.random.default_rng(1)
    recs = []
    for i in range(6):
        n = 30000 + 1000 * i
        s = bytes(np.frombuffer(b"ACGT", np.uint8)[rng.integers(0, 4, n)])
        q = b"I" * n if i % 2 == 0 else bytes(b"5?"[(j // 9000) % 2] for j in range(n))
        recs.append(b"@c%d\n%s\n+\n%s\n" % (i, s, q))
    (tmp_path / "const.fq").write_bytes(b"".join(recs))
    runs = [[TEST1, TEST2], [TEST1], ["-b", "600000", TEST1, TEST2], [str(tmp_path / "a.fq"), str(tmp_path / "b.fq")],
            ["-s", "4", "-b", "300000", str(tmp_path / "a.fq"), str(tmp_path / "b.fq")],
            ["-q", "3", str(tmp_path / "a.fq")], [str(tmp_path / "e.fq")], ["-s", "9", str(tmp_path / "e.fq")],
            ["-l", "1.15", TEST1, TEST2], ["-l", "1.3", "-b", "300000", str(tmp_path / "a.fq")],
            ["-l", "1.05", str(tmp_path / "e.fq")], [str(tmp_path / "long.fq")],
            ["-l", "1.6", str(tmp_path / "long.fq")], ["-l", "1.15", str(tmp_path / "const.fq")],
            ["-l", "1.6", str(tmp_path / "const.fq")]]
    for args in runs:
        r = subprocess.run([str(exe)] + args, capture_output=True, text=True)
        assert r.returncode == 0 and r.stdout.startswith("OK"), (args, r.stdout, r.stderr)
    # the engine's other R-Block chunk lengths (SA_RB_CHUNK, also the arrays' stride;
    # the default is 7904)
    for chunk in ("8192", "4096", "1024"):
        for args in (["-l", "1.15", TEST1, TEST2], ["-l", "1.6", str(tmp_path / "long.fq")],
                     ["-l", "1.15", str(tmp_path / "const.fq")]):
            r = subprocess.run([str(exe)] + args, capture_output=True, text=True,
                               env=dict(os.environ, SA_RB_CHUNK=chunk))
            assert r.returncode == 0 and r.stdout.startswith("OK"), (chunk, args, r.stdout, r.stderr)


def test_cpu_decomposition_reference_path(tmp_path):
    """The reference (HASH index) path's decomposition on the host: the engine's
    chain / bail-out / insert-window bookkeeping (sa_align_host.h) and the
    alignment-stream emission (sa_logic.h) over the oracle's alignments, block
    for block equal to the oracle's doAlign + doAlignEncode restatement."""
    exe = tmp_path / "emu"
    src = os.path.join(ROOT, "tests", "cpu_emu", "emu.cpp")
    subprocess.run(["g++", "-O2", "-std=c++17", "-o", str(exe), src,
                    os.path.join(ROOT, "fastqueeze_amd", "csrc", "fastq_host.cpp"),
                    os.path.join(ROOT, "oracle", "fqz_oracle.c"), os.path.join(ROOT, "oracle", "hash_oracle.c"),
                    os.path.join(ROOT, "oracle", "align_oracle.c"), "-lm"], check=True)
    import synth
    fa, g = synth.reference(2_000_000, 5)
    (tmp_path / "ref.fa").write_bytes(fa)
    a, b = synth.aligned_reads(g, 8000, 9, paired=True, random_frac=0.1, far_frac=0.2, short_frac=0.5)
    (tmp_path / "p1.fq").write_bytes(a)
    (tmp_path / "p2.fq").write_bytes(b)
    a, _ = synth.aligned_reads(g, 6000, 7, random_frac=0.6, short_frac=0.3)
    (tmp_path / "s.fq").write_bytes(a)
    runs = [["-b", "500000", str(tmp_path / "p1.fq"), str(tmp_path / "p2.fq")],
            ["-I", "400", "-b", "700000", str(tmp_path / "p1.fq"), str(tmp_path / "p2.fq")],
            ["-b", "300000", str(tmp_path / "s.fq")]]
    for args in runs:
        r = subprocess.run([str(exe), "-r", str(tmp_path / "ref.fa")] + args, capture_output=True, text=True,
                           env=dict(os.environ, EMU_ALN="1"))
        assert r.returncode == 0 and r.stdout.splitlines()[-1].startswith("OK"), (args, r.stdout[-2000:], r.stderr)
        # the cases reached the paths: a bail-out / the carried-state variant / an estimated window
        lines = [l for l in r.stdout.splitlines() if l.startswith("block ")]
        assert lines


def test_coder_decomposition_selftest(tmp_path):
    """Decomposed coder (pass R / L1 / L2 / L3 + squeeze restarts) == serial coder on the host."""
    exe = tmp_path / "emu"
    src = os.path.join(ROOT, "tests", "cpu_emu", "emu.cpp")
    subprocess.run(["g++", "-O2", "-std=c++17", "-o", str(exe), src,
                    os.path.join(ROOT, "fastqueeze_amd", "csrc", "fastq_host.cpp"),
                    os.path.join(ROOT, "oracle", "fqz_oracle.c"), os.path.join(ROOT, "oracle", "hash_oracle.c"),
                    os.path.join(ROOT, "oracle", "align_oracle.c"), "-lm"], check=True)
    r = subprocess.run([str(exe), "--coder"], capture_output=True, text=True)
    assert r.returncode == 0 and r.stdout.startswith("OK"), r.stdout


def test_oracle_rc_squeeze_streams():
    """The oracle's bare coder accepts the squeeze streams the GPU coder test uses."""
    for c, f, t in oracle_py.squeeze_streams():
        out = oracle_py.rc_encode(c, f, t)
        assert len(out) >= 8


_IUPAC = b"MRYKSWHBVD"


def _norm_seq(seq: np.ndarray) -> np.ndarray:
    """What a decoder can return for stored bases: ACGT / IUPAC upper-cased,
    anything else 'N' (the encoder keeps base codes, seq_val_table@0x44b800)."""
    up = seq.copy()
    low = (up >= ord("a")) & (up <= ord("z"))
    up[low] -= 32
    keep = np.isin(up, np.frombuffer(b"ACGT" + _IUPAC, np.uint8))
    up[~keep] = ord("N")
    return up


def _roundtrip(b, slevel, qlevel, md5=True):
    import oracle_py as ob
    enc = ob.encode_block(b, slevel, qlevel, md5, 0)
    names, nl, seq, sl, qual, ok = ob.decode_block(enc, b.nreads, b.names.size, b.seq.size, slevel, qlevel, md5)
    assert np.array_equal(nl, b.name_lens) and np.array_equal(names, b.names)
    assert np.array_equal(sl, b.seq_lens)
    assert np.array_equal(qual, b.qual)
    assert np.array_equal(seq, _norm_seq(b.seq))
    return ok


@pytest.mark.parametrize("slevel,qlevel", [(3, 2), (1, 1), (4, 3), (9, 2)])
def test_decoder_round_trip_synthetic(slevel, qlevel):
    """encode -> decode (oracle/fqz_decode.c) gives the block back, MD5s match."""
    import fastqueeze_amd as fq
    text1, text2 = synth.generate(3000, paired=True, seed=40 + slevel)
    for b in fq.blocks_from_fastq(text1, text2, 400_000):
        assert _roundtrip(b, slevel, qlevel)


def test_decoder_round_trip_edge_cases():
    """N / IUPAC / lowercase bases, '#' runs, empty reads: the decoded block is the
    input with bases normalised; the MD5 check flags the lowercase input."""
    import fastqueeze_amd as fq
    b = fq.blocks_from_fastq(synth.edge_cases())[0]
    ok = _roundtrip(b, 3, 2)
    assert ok == bool(np.array_equal(_norm_seq(b.seq), b.seq))


def test_decoder_round_trip_reference_pair(test_pair):
    import fastqueeze_amd as fq
    t1, t2 = test_pair
    for b in fq.blocks_from_fastq(t1, t2):
        assert _roundtrip(b, 3, 2)
