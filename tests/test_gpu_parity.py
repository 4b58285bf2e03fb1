"""GPU parity: libseqarc_amd on MI355X against the CPU restatement, byte for byte,
through the C-ABI (sa_stage / sa_run / sa_fetch)."""
import json
import os

import numpy as np
import pytest

import oracle_py
import synth
from conftest import GOLDEN

import fastqueeze_amd as fq

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def enc():
    e = fq.Encoder(0)
    yield e
    e.close()


def _oracle_outs(blocks, cfg):
    return [oracle_py.encode_block(b, cfg.slevel, cfg.qlevel, cfg.md5, cfg.bin_mode, cfg.lossy) for b in blocks]


def _check(enc, blocks, cfg):
    got = enc.encode(blocks, cfg)
    want = _oracle_outs(blocks, cfg)
    assert len(got) == len(want)
    for i, (g, w) in enumerate(zip(got, want)):
        if g != w:
            at = next((k for k in range(min(len(g), len(w))) if g[k] != w[k]), min(len(g), len(w)))
            pytest.fail(f"block {i}: gpu {len(g)} B vs oracle {len(w)} B, first difference at byte {at}")
    return got


def test_reference_test_pair(enc, test_pair):
    blocks = fq.blocks_from_fastq(*test_pair)
    tmpl = fq.analyze_ids(blocks[0], False)
    out = _check(enc, blocks, fq.Config(bin_mode=int(tmpl[0])))
    assert len(out[0]) == 820818
    se = fq.blocks_from_fastq(test_pair[0])
    _check(enc, se, fq.Config(bin_mode=1))
    # tokenizer path on the same reads
    _check(enc, se, fq.Config(bin_mode=0))


@pytest.mark.parametrize("name", ["test_pe_600k", "synth_pe_4k", "synth_pe_4k_s4", "synth_se_4k_q3", "edge_se",
                                  "edge_se_s9", "test_pe_lossy_115", "synth_se_lossy_16", "synth_long_70k"])
def test_golden_cases(enc, name):
    import sys
    sys.path.insert(0, GOLDEN)
    import make_golden
    g = json.load(open(os.path.join(GOLDEN, "golden.json")))[name]
    case = g["case"]
    t1, t2 = make_golden.inputs(case)
    blocks = fq.blocks_from_fastq(t1, t2, case.get("bs", fq.BLOCK_SIZE))
    tmpl = fq.analyze_ids(blocks[0], t2 is None)
    cfg = fq.Config(slevel=case.get("slevel", 3), qlevel=case.get("qlevel", 2), bin_mode=int(tmpl[0]),
                    lossy=case.get("lossy", 0.0))
    out = _check(enc, blocks, cfg)
    assert [len(o) for o in out] == g["blocks"]


def test_name_prefix_suffix_lengths(enc):
    """k_prep_sq16's row-parallel name columns (name_prefix_suffix): consecutive
    names sharing prefixes and suffixes of 0..250 bytes, names that are prefixes
    or suffixes of their neighbour, equal names, 1-byte names; tokenizer mode."""
    rng = np.random.default_rng(7)
    alpha = np.frombuffer(b"ABCDEFGHIJKLMNOPQRSTUVWXYZ0123456789:_-./", dtype=np.uint8)

    def word(n):
        return bytes(alpha[rng.integers(0, len(alpha), n)])

    names, prev = [], word(40)
    for i in range(3000):
        kind = i % 6
        if kind == 0:
            p, s, m = int(rng.integers(0, 120)), int(rng.integers(0, 120)), int(rng.integers(0, 16))
            nm = prev[:p] + word(m) + prev[len(prev) - min(s, len(prev)):]
        elif kind == 1:
            nm = prev
        elif kind == 2:
            nm = prev[:int(rng.integers(1, len(prev) + 1))]
        elif kind == 3:
            nm = prev[int(rng.integers(0, len(prev))):]
        elif kind == 4:
            nm = word(int(rng.integers(1, 250)))
        else:
            nm = word(1) if rng.integers(0, 2) else prev + word(int(rng.integers(0, 60)))
        nm = (nm or b"X")[:245]
        names.append(nm)
        prev = nm
    # every header starts with the first one's first bytes (the block cut looks for
    # "\n@" + more than five bytes of the file's first line, end_pos)
    names = [b"SIMRD" + nm for nm in names]
    recs = []
    for nm in names:
        L = int(rng.integers(20, 120))
        seq = bytes(np.frombuffer(b"ACGT", dtype=np.uint8)[rng.integers(0, 4, L)])
        qual = bytes(rng.integers(35, 64, L).astype(np.uint8))   # (no '@' in the qualities)
        recs.append(b"@" + nm + b"\n" + seq + b"\n+\n" + qual + b"\n")
    blocks = fq.blocks_from_fastq(b"".join(recs), None, 100_000)
    assert len(blocks) > 2
    _check(enc, blocks, fq.Config(bin_mode=0))


def test_md5_off_and_empty_reads(enc):
    blocks = fq.blocks_from_fastq(synth.edge_cases())
    _check(enc, blocks, fq.Config(md5=False))
    empty = fq.parse_se(b"@a\n\n+\n\n@b\n\n+\n\n")
    _check(enc, [empty], fq.Config())


def test_many_blocks_one_batch(enc):
    a, b = synth.generate(30000, paired=True, seed=21)
    blocks = fq.blocks_from_fastq(a, b, 400_000)
    assert len(blocks) > 20
    _check(enc, blocks, fq.Config())


def test_encode_blocks_sub_batches(enc, monkeypatch):
    """sa_encode_blocks (the one-call drop-in) splits a batch over its HBM cap into
    consecutive sub-batches; a cap of ~2 blocks' bases forces several splits and
    the outputs stay equal to the oracle, in input order."""
    a, b = synth.generate(8000, paired=True, seed=23)
    blocks = fq.blocks_from_fastq(a, b, 300_000)
    assert len(blocks) >= 8
    want = _oracle_outs(blocks, fq.Config())
    assert enc.encode_blocks(blocks, fq.Config()) == want          # one batch
    monkeypatch.setenv("SA_BATCH_BASES", str(2 * int(blocks[0].seq.size)))
    assert enc.encode_blocks(blocks, fq.Config()) == want          # ~len/2 sub-batches
    monkeypatch.setenv("SA_BATCH_BASES", "1")
    assert enc.encode_blocks(blocks, fq.Config()) == want          # one block per sub-batch
    assert enc.encode_blocks([], fq.Config()) == []


def test_full_size_block(enc):
    """One full 50 MiB block (146,716 x 150 bp reads) -- the bench's unit of work --
    equal to the oracle, and decoding back to the input (CPU decoder, MD5s match)."""
    a, _ = synth.generate(150_000, seed=5)
    blocks = fq.blocks_from_fastq(a)
    assert blocks[0].text_bytes > 50_000_000
    got = _check(enc, blocks[:1], fq.Config())
    b = blocks[0]
    names, nl, seq, sl, qual, ok = oracle_py.decode_block(got[0], b.nreads, b.names.size, b.seq.size)
    assert ok
    assert np.array_equal(names, b.names) and np.array_equal(nl, b.name_lens)
    assert np.array_equal(seq, b.seq) and np.array_equal(sl, b.seq_lens) and np.array_equal(qual, b.qual)


def test_exact_payload_fallback(enc, monkeypatch):
    """The payload arena is sized from the streams' real byte counts after L2
    with slack for squeeze restarts; with no slack the tiny streams outgrow it
    (their 8 flush bytes) and the batch is re-encoded with the 2-byte-per-symbol
    caps -- same bytes."""
    blocks = fq.blocks_from_fastq(synth.edge_cases())
    monkeypatch.setenv("SA_PAYLOAD_SLACK", "0")
    _check(enc, blocks, fq.Config())


def test_fetch_sizes(enc):
    """sa_fetch_sizes after sa_run gives each block's encoded size (the command
    line sizes its output buffers by it), equal to what sa_fetch copies; a
    count that is not the batch's is refused."""
    a, b = synth.generate(6000, paired=True, seed=44)
    blocks = fq.blocks_from_fastq(a, b, 300_000)
    assert len(blocks) >= 4
    first = enc.encode(blocks, fq.Config())
    enc.run(fq.Config())
    sizes = enc.fetch_sizes()
    assert sizes == [len(o) for o in first]
    assert enc.fetch() == first
    bad = np.zeros(len(blocks) + 1, dtype=np.uint64)
    assert enc._lib.sa_fetch_sizes(enc._ctx, fq._ptr(bad), len(blocks) + 1) == -1


def test_deterministic_rerun(enc):
    a, b = synth.generate(2000, paired=True, seed=4)
    blocks = fq.blocks_from_fastq(a, b)
    first = enc.encode(blocks, fq.Config())
    enc.run(fq.Config())
    assert enc.fetch() == first


def test_pass_r_starved_long_runs(enc, monkeypatch):
    """Pass R codes while the long SIMPLE_MODEL runs are still replayed and
    waits for records they have not written (seg_retry).  With the long-run
    kernel never launched (SA_TEST_SKIP_LONG, a test hook) every such wait
    times out: the batch fails with E_CODER in about SA_RV_WAIT_MS, the L3 pass
    does not run on the missing records, and a context made afterwards encodes
    the same blocks exactly."""
    import time
    a, b = synth.generate(40_000, paired=True, seed=81)
    blocks = fq.blocks_from_fastq(a, b, 4 << 20)
    monkeypatch.setenv("SA_TEST_SKIP_LONG", "1")
    monkeypatch.setenv("SA_RV_WAIT_MS", "300")
    starved = fq.Encoder(0)
    try:
        t0 = time.perf_counter()
        with pytest.raises(fq.SeqArcError, match="E_CODER|0x"):
            starved.encode(blocks, fq.Config())
        assert time.perf_counter() - t0 < 20
    finally:
        starved.close()
    monkeypatch.delenv("SA_TEST_SKIP_LONG")
    monkeypatch.delenv("SA_RV_WAIT_MS")
    fresh = fq.Encoder(0)
    try:
        _check(fresh, blocks, fq.Config())
    finally:
        fresh.close()


def test_rejects_out_of_model_quality(enc):
    bad = fq.parse_se(b"@r\nACGT\n+\nII\x7fI\n")
    with pytest.raises(fq.SeqArcError):
        enc.encode([bad], fq.Config())


def test_coder_records_with_squeezes(enc):
    """Bare coder on streams that fire the carry-less squeeze: the GPU decomposition
    restarts those streams and still matches the serial reference coder."""
    streams = oracle_py.squeeze_streams()
    got = enc.code_records(streams)
    assert enc.coder_restarts() > 0
    for i, (s, g) in enumerate(zip(streams, got)):
        assert g == oracle_py.rc_encode(*s), f"stream {i}"


def test_low_complexity_context_runs(enc):
    """Poly-A / dinucleotide / triplet repeats: BASE_MODEL context runs far longer
    than the first halving (in-run index 242) and runs that cross sort tiles."""
    rng = np.random.default_rng(17)
    recs = []
    motifs = [b"A", b"AC", b"CAG", b"GATTACA"]
    for i in range(3000):
        m = motifs[i % len(motifs)]
        s = (m * 200)[: 100 + (i % 51)]
        if i % 7 == 0:   # sprinkle random bases and an N
            arr = bytearray(s)
            for p in rng.integers(0, len(arr), 3):
                arr[int(p)] = b"ACGTN"[int(rng.integers(0, 5))]
            s = bytes(arr)
        q = bytes(rng.choice(np.frombuffer(b"F:,#", np.uint8), size=len(s), p=[0.7, 0.2, 0.08, 0.02]))
        recs.append(b"@lc%d\n%s\n+\n%s\n" % (i, s, q))
    blocks = fq.blocks_from_fastq(b"".join(recs))
    for slevel in (3, 1):
        _check(enc, blocks, fq.Config(slevel=slevel))


def _low_complexity_fastq(seed, n):
    rng = np.random.default_rng(seed)
    recs = []
    motifs = [b"A", b"AC", b"CAG", b"GATTACA", b"TTTTTTTTTG"]
    for i in range(n):
        m = motifs[i % len(motifs)]
        s = (m * 200)[: 100 + (i % 51)]
        if i % 7 == 0:
            arr = bytearray(s)
            for p in rng.integers(0, len(arr), 3):
                arr[int(p)] = b"ACGTN"[int(rng.integers(0, 5))]
            s = bytes(arr)
        q = bytes(rng.choice(np.frombuffer(b"F:,#", np.uint8), size=len(s), p=[0.7, 0.2, 0.08, 0.02]))
        # (a common name prefix of more than five bytes: the block cut's record test)
        recs.append(b"@LOWCPLX%d\n%s\n+\n%s\n" % (i, s, q))
    return b"".join(recs)


@pytest.mark.parametrize("lanes,bucket,variant,inv,db,lpt", [(0, 0, 6, 1, 0, 1), (1, 1, 6, 1, 0, 1),
                                                             (1, 0, 6, 1, 0, 1), (0, 1, 6, 1, 0, 1),
                                                             (0, 1, 5, 1, 0, 1), (0, 1, 0, 1, 0, 1),
                                                             (0, 1, 5, 0, 0, 1), (0, 1, 5, 1, 9, 1),
                                                             (0, 1, 5, 1, 10, 1), (0, 1, 5, 1, 0, 0)])
def test_pass_r_and_seq_replay_paths(monkeypatch, lanes, bucket, variant, inv, db, lpt):
    """Both pass-R kernels (k_coder_rv: a chain per wave on the scalar unit --
    its operands through SMEM from the lanes' ring (6) or through
    v_readlane (5: batched, the default; 0: per step), SA_RV_VARIANT; k_coder_rl: a chain
    per lane in the VALU fed through an LDS ring, SA_RV_LANES) and both SEQ
    replays (the full sort + k_replay_seq; one bucket sort pass +
    k_replay_seq_bkt, SA_SEQ_BUCKET; its records stored in sorted order and
    gathered back through the bucket pass's inverse permutation, or stored
    scattered, SA_SEQ_INV; the bucket pass's digit bits, SA_BKT_DB = 0 (the
    default: 8 up to 20-bit contexts, 9 above), 9 or 10;
    the buckets largest first or in digit order, SA_BKT_LPT)
    give the oracle's bytes: multi-block PE
    batches (chains of ~2.9 M symbols and of a few), low-complexity reads
    (context runs far past the first halving, contexts shared inside a
    64-symbol step), Slevel 1 / 3 / 4 (8 / 12 / 13 low context bits per
    bucket)."""
    monkeypatch.setenv("SA_RV_LANES", str(lanes))
    monkeypatch.setenv("SA_SEQ_BUCKET", str(bucket))
    monkeypatch.setenv("SA_RV_VARIANT", str(variant))
    monkeypatch.setenv("SA_SEQ_INV", str(inv))
    monkeypatch.setenv("SA_BKT_DB", str(db))
    monkeypatch.setenv("SA_BKT_LPT", str(lpt))
    e = fq.Encoder(0)
    try:
        a, b = synth.generate(40_000, paired=True, seed=91)
        pe = fq.blocks_from_fastq(a, b, 4 << 20)
        assert len(pe) >= 4
        _check(e, pe, fq.Config())
        _check(e, pe[:2], fq.Config(slevel=4, qlevel=3))
        lc = fq.blocks_from_fastq(_low_complexity_fastq(33, 4000), None, 200_000)
        for slevel in (3, 1):
            _check(e, lc, fq.Config(slevel=slevel))
    finally:
        e.close()


def _long_read_fastq(seed, n):
    """Reads whose lengths straddle the 64-position steps of k_emit_sq, with N /
    IUPAC bases anywhere (so a step compacts its ACGT bases) and '#' runs that
    end the read across step boundaries (qual_nonhash) or fill it."""
    rng = np.random.default_rng(seed)
    lens = [0, 1, 2, 16, 17, 63, 64, 65, 127, 128, 129, 150, 191, 192, 200, 300, 1000]
    recs = []
    for i in range(n):
        L = lens[i % len(lens)]
        s = bytearray(rng.choice(np.frombuffer(b"ACGT", np.uint8), size=L))
        rate = (0.0, 0.01, 0.2)[i % 3]
        for p in np.nonzero(rng.random(L) < rate)[0]:
            s[int(p)] = b"NNRYKMSWacgtn"[int(rng.integers(0, 13))]
        q = bytearray(rng.integers(35, 75, size=L, dtype=np.uint8))
        if L and i % 4 == 0:
            tail = int(rng.integers(0, L + 1))
            q[L - tail:] = b"#" * tail
        if L and i % 5 == 1:
            for p in np.nonzero(rng.random(L) < 0.1)[0]:
                q[int(p)] = ord("#")
        recs.append(b"@lr%d\n%s\n+\n%s\n" % (i, bytes(s), bytes(q)))
    return b"".join(recs)


@pytest.mark.parametrize("slevel,qlevel", [(3, 2), (1, 3), (4, 1), (9, 2)])
def test_long_reads_emit_steps(enc, slevel, qlevel):
    """SEQ contexts and QUAL contexts carried across k_emit_sq's 64-position steps."""
    blocks = fq.blocks_from_fastq(_long_read_fastq(5 + slevel, 700))
    _check(enc, blocks, fq.Config(slevel=slevel, qlevel=qlevel))


def test_prep_wave_per_read(monkeypatch):
    """k_prep_sq16 with a whole wave per read (SA_PREP_ROW=64, opt-in) gives the
    oracle's bytes: long reads with N / IUPAC bases and '#' runs, lossy
    qualities, and short PE reads."""
    monkeypatch.setenv("SA_PREP_ROW", "64")
    e = fq.Encoder(0)
    try:
        _check(e, fq.blocks_from_fastq(_long_read_fastq(77, 500)), fq.Config(slevel=3, qlevel=3))
        t1, _ = synth.generate(40, paired=False, seed=12, read_len=20000)
        _check(e, fq.blocks_from_fastq(t1), fq.Config(lossy=1.15))
        a, b = synth.generate(20_000, paired=True, seed=13)
        _check(e, fq.blocks_from_fastq(a, b, 4 << 20)[:2], fq.Config())
    finally:
        e.close()


@pytest.mark.parametrize("ratio", [1.05, 1.15, 1.6])
def test_lossy_rblock(enc, test_pair, ratio):
    """-l R (rblock@0x426c10 + no quality MD5): GPU chunked R-Block == the oracle's serial pass,
    incl. a block of long reads whose runs cross many 8 KiB chunks."""
    blocks = fq.blocks_from_fastq(*test_pair)
    tmpl = fq.analyze_ids(blocks[0], False)
    _check(enc, blocks, fq.Config(bin_mode=int(tmpl[0]), lossy=ratio))
    t1, _ = synth.generate(60, paired=False, seed=11, read_len=20000)
    _check(enc, fq.blocks_from_fastq(t1), fq.Config(lossy=ratio))
    _check(enc, fq.blocks_from_fastq(synth.edge_cases()), fq.Config(lossy=ratio, md5=False))


def _rblock_runs_fastq(seed, n, read_len):
    """Long reads whose qualities alternate long near-constant stretches (runs
    of rblock that cross many R-Block chunks: their speculative exits differ
    from the true ones, so the entry pass takes rb_carry) with noisy ones
    (chunks that converge), at random lengths, so the failing chunks fall at
    every position of the 64-chunk windows of k_rb_fix_w."""
    rng = np.random.default_rng(seed)
    recs = []
    for i in range(n):
        q = bytearray()
        while len(q) < read_len:
            # (qualities below '@': a quality line never looks like a header to the cut)
            if rng.random() < 0.5:
                v = int(rng.integers(40, 62))
                m = int(rng.integers(500, 40000))
                q += bytes(np.where(rng.random(m) < 0.5, v, v + 1).astype(np.uint8))
            else:
                q += bytes(rng.integers(35, 64, size=int(rng.integers(50, 6000)), dtype=np.uint8))
        q = bytes(q[:read_len])
        s = bytes(rng.choice(np.frombuffer(b"ACGT", np.uint8), size=read_len))
        recs.append(b"@SIMRDrb%d\n%s\n+\n%s\n" % (i, s, q))   # (the cut matches > 5 bytes of the first header)
    return b"".join(recs)


@pytest.mark.parametrize("serial,spec_wg", [("0", "2"), ("1", "2"), ("0", "0")])
def test_rblock_entry_pass(monkeypatch, serial, spec_wg):
    """The R-Block entry pass -- k_rb_fix_w (a wave per block, 64 chunks a step,
    the default) and k_rb_fix (SA_RB_FIX_SERIAL=1) -- where many chunks do not
    converge (rb_carry at arbitrary window positions), blocks of several
    windows, and a constant-quality block where no chunk converges: == the
    oracle's serial rblock@0x426c10."""
    monkeypatch.setenv("SA_RB_FIX_SERIAL", serial)
    monkeypatch.setenv("SA_RB_SPEC_WG", spec_wg)   # (0: k_rb_spec's one grid; 2, the default: a counter)
    e = fq.Encoder(0)
    try:
        blocks = fq.blocks_from_fastq(_rblock_runs_fastq(31, 120, 30000), None, 2 << 20)
        assert len(blocks) >= 3
        for r in (1.05, 1.15, 1.6):
            _check(e, blocks, fq.Config(lossy=r))
        const = b"".join(b"@SIMRDc%d\n%s\n+\n%s\n" % (i, b"ACGT" * 5000, b"5" * 20000) for i in range(60))
        _check(e, fq.blocks_from_fastq(const), fq.Config(lossy=1.15))
    finally:
        e.close()


@pytest.mark.parametrize("chunk", ["4", "12", "1024"])
def test_front_read_counter_chunks(monkeypatch, chunk):
    """The front kernels' reads taken from the counter `chunk` at a time
    (SA_WQ_CHUNK; by default from the batch's mean read length: 64 for short
    reads, 4 for ONT-length ones) give the oracle's bytes: short PE reads,
    long reads with N / IUPAC bases and '#' runs, lossy long reads."""
    monkeypatch.setenv("SA_WQ_CHUNK", chunk)
    e = fq.Encoder(0)
    try:
        a, b = synth.generate(20_000, paired=True, seed=17)
        _check(e, fq.blocks_from_fastq(a, b, 2 << 20), fq.Config())
        _check(e, fq.blocks_from_fastq(_long_read_fastq(78, 500)), fq.Config(slevel=3, qlevel=3))
        t1, _ = synth.generate(40, paired=False, seed=14, read_len=20000)
        _check(e, fq.blocks_from_fastq(t1), fq.Config(lossy=1.15))
    finally:
        e.close()


def test_long_length_path(enc):
    """Reads > 65535 bp switch the block to compressLen_long@0x423710 (four length
    bytes); a block of short reads next to it keeps compressLen_short."""
    t_long, _ = synth.generate(12, paired=False, seed=5, read_len=70000)
    t_short, _ = synth.generate(300, paired=False, seed=6)
    blocks = fq.blocks_from_fastq(t_long) + fq.blocks_from_fastq(t_short)
    _check(enc, blocks, fq.Config())
    _check(enc, blocks, fq.Config(lossy=1.15, slevel=4))


def test_cli_archive(tmp_path, test_pair):
    """seqarc_amd -c (the SeqArc -c surface) writes the reference-sized archive:
    the GPU blocks inside the restated container, plain and gzip inputs."""
    import gzip
    import shutil
    import subprocess
    exe = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "fastqueeze_amd", "bin",
                       "seqarc_amd")
    names = ["ERR2755197_test_1.fq", "ERR2755197_test_2.fq"]
    paths = [str(tmp_path / n) for n in names]
    for p, t in zip(paths, test_pair):
        open(p, "wb").write(t)
    blocks = fq.blocks_from_fastq(*test_pair)
    tmpl = fq.analyze_ids(blocks[0], False)
    cfg = fq.Config(bin_mode=int(tmpl[0]))
    want = fq.arc_archive(_oracle_outs(blocks, cfg), blocks, names[0], names[1], tmpl, cfg)
    r = subprocess.run([exe, "-c", "-t", "1", "-1", paths[0], "-2", paths[1], "-o", str(tmp_path / "pe")],
                       capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr
    got = open(tmp_path / "pe.arc", "rb").read()
    assert len(got) == 821500 and got == want
    r = subprocess.run([exe, "-d", "-t", "4", str(tmp_path / "pe.arc"), str(tmp_path / "back")], capture_output=True,
                       text=True, timeout=120)
    assert r.returncode == 0, r.stderr
    assert (tmp_path / "back_1.fastq").read_bytes() == test_pair[0]
    assert (tmp_path / "back_2.fastq").read_bytes() == test_pair[1]
    for p in paths:
        with open(p, "rb") as f, gzip.open(p + ".gz", "wb") as g:
            shutil.copyfileobj(f, g)
    r = subprocess.run([exe, "-c", "-1", paths[0] + ".gz", "-2", paths[1] + ".gz", "-o", str(tmp_path / "gz")],
                       capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr
    gz = open(tmp_path / "gz.arc", "rb").read()
    assert len(gz) == len(want) and gz[:16 + len(got) - 700] == want[:16 + len(got) - 700]
    r = subprocess.run([exe, "-c", "-1", paths[0], "-o", str(tmp_path / "se")], capture_output=True, text=True,
                       timeout=120)
    assert r.returncode == 0 and os.path.getsize(tmp_path / "se.arc") == 379069, r.stderr


def test_cli_multi_device_gather(tmp_path, test_pair):
    """--devices: batches dealt to several encoder contexts (one host thread each)
    and gathered in input order -- the same archive as one context.  On the
    one-GPU test box the contexts share device 0 (--share-device)."""
    import subprocess
    exe = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "fastqueeze_amd", "bin",
                       "seqarc_amd")
    paths = [str(tmp_path / n) for n in ("m_1.fq", "m_2.fq")]
    for p, t in zip(paths, test_pair):
        open(p, "wb").write(t)
    base = [exe, "-c", "-1", paths[0], "-2", paths[1], "--block-size", "1", "--batch", "1"]
    r1 = subprocess.run(base + ["--contexts", "1", "-o", str(tmp_path / "one")], capture_output=True, text=True,
                        timeout=120)
    r3 = subprocess.run(base + ["--devices", "3", "--share-device", "-o", str(tmp_path / "three")],
                        capture_output=True, text=True, timeout=120)
    # the streaming pipeline with several contexts sharing a front, 2-block batches, 2 parser threads
    r4 = subprocess.run(base[:-1] + ["2", "--contexts", "3", "-t", "2", "-o", str(tmp_path / "four")],
                        capture_output=True, text=True, timeout=120)
    # the blocks parsed on host threads (--host-parse) instead of on the device
    r5 = subprocess.run(base[:-1] + ["2", "--contexts", "2", "--host-parse", "-t", "2", "-o", str(tmp_path / "five")],
                        capture_output=True, text=True, timeout=120)
    # the streamed uploads (SA_CLI_STREAM=1: every block's text to the device as
    # it is cut, the next batch into the other text arena) against the default
    # staging of whole batches; and the streamed path over a ring of 4 MiB
    # segments (every slot refilled while batches are in flight)
    env0 = dict(os.environ, SA_CLI_STREAM="1")
    r6 = subprocess.run(base[:-1] + ["2", "--contexts", "3", "-t", "2", "-o", str(tmp_path / "six")],
                        capture_output=True, text=True, timeout=120, env=env0)
    env7 = dict(os.environ, SA_CLI_SEG_SLICES="1", SA_CLI_STREAM="1")
    r7 = subprocess.run(base[:-1] + ["3", "--contexts", "2", "-o", str(tmp_path / "seven")],
                        capture_output=True, text=True, timeout=120, env=env7)
    assert r1.returncode == 0 and r3.returncode == 0 and r4.returncode == 0, (r1.stderr, r3.stderr, r4.stderr)
    assert r5.returncode == 0 and r6.returncode == 0 and r7.returncode == 0, (r5.stderr, r6.stderr, r7.stderr)
    one = open(tmp_path / "one.arc", "rb").read()
    assert one == open(tmp_path / "three.arc", "rb").read() == open(tmp_path / "four.arc", "rb").read()
    assert one == open(tmp_path / "five.arc", "rb").read()
    assert one == open(tmp_path / "six.arc", "rb").read() == open(tmp_path / "seven.arc", "rb").read()
    blocks = fq.blocks_from_fastq(*test_pair, 1 << 20)
    assert len(blocks) > 3
    tmpl = fq.analyze_ids(blocks[0], False)
    cfg = fq.Config(bin_mode=int(tmpl[0]))
    assert one == fq.arc_archive(_oracle_outs(blocks, cfg), blocks, "m_1.fq", "m_2.fq", tmpl, cfg)


@pytest.fixture(scope="module")
def pe_full():
    """Two full 50 MiB 150 bp PE blocks (~73k mate pairs each, Illumina headers:
    tokenizer path) plus a partial third: configs[2]'s unit of work."""
    a, b = synth.generate(150_000, paired=True, seed=31)
    blocks = fq.blocks_from_fastq(a, b)
    assert len(blocks) == 3 and blocks[0].text_bytes > 50_000_000 and blocks[0].nreads > 140_000
    tmpl = fq.analyze_ids(blocks[0], False)
    assert int(tmpl[0]) == 0   # Illumina-style mate IDs: the name tokenizer
    return blocks


def test_full_size_pe_block(enc, pe_full):
    """One full 50 MiB PE block, alone, equal to the oracle and decoding back."""
    got = _check(enc, pe_full[:1], fq.Config())
    b = pe_full[0]
    names, nl, seq, sl, qual, ok = oracle_py.decode_block(got[0], b.nreads, b.names.size, b.seq.size)
    assert ok and np.array_equal(names, b.names) and np.array_equal(seq, b.seq) and np.array_equal(qual, b.qual)


def test_two_block_pe_batch(enc, pe_full):
    """A 2-block PE batch (both full size) and the 3-block batch with its short tail."""
    _check(enc, pe_full[:2], fq.Config())
    _check(enc, pe_full, fq.Config())


@pytest.mark.parametrize("slevel", [5, 6, 8])
def test_high_order_seq_model(enc, slevel):
    """Slevel 5/6/8: k = 12/13/15 (2^24..2^30 contexts; 30-bit sort keys at k = 15),
    the README's "16-order" model as the binary builds it (ctor@0x42f63e)."""
    a, b = synth.generate(6000, paired=True, seed=40 + slevel)
    blocks = fq.blocks_from_fastq(a, b, 1_000_000)
    _check(enc, blocks, fq.Config(slevel=slevel))
    blocks = fq.blocks_from_fastq(_long_read_fastq(50 + slevel, 400))
    _check(enc, blocks, fq.Config(slevel=slevel, qlevel=3))


def test_full_size_block_slevel8(enc, pe_full):
    """A full 50 MiB PE block at Slevel 8 (k = 15: 4 GiB of BASE_MODEL tables in
    the oracle; context runs of ~1 symbol on the GPU)."""
    _check(enc, pe_full[:1], fq.Config(slevel=8))


@pytest.mark.parametrize("slevel", [8, 9])
def test_full_size_se_block_high_order(enc, slevel):
    """configs[1]'s unit of work: a full 50 MiB SE block of 150 bp reads at
    Slevel 8 / 9 (k = 15 / 16, the README's "16-order" model; ctor@0x42f63e)."""
    a, _ = synth.generate(150_000, seed=8)
    blocks = fq.blocks_from_fastq(a)
    assert blocks[0].text_bytes > 50_000_000
    _check(enc, blocks[:1], fq.Config(slevel=slevel))


@pytest.fixture(scope="module")
def ont_full():
    """configs[4]'s shape: 10/20/30/40/50 kbp SE reads with N / IUPAC bases
    (the bench's --ont generator), the first full 50 MiB block."""
    parts = [synth.generate(180, read_len=L, seed=700 + k, chunk=1000)[0]
             for k, L in enumerate((10_000, 20_000, 30_000, 40_000, 50_000))]
    blocks = fq.blocks_from_fastq(b"".join(parts))
    assert blocks[0].text_bytes > 50_000_000 and blocks[0].nreads > 500
    return blocks[:1]


@pytest.mark.parametrize("lossy", [0.0, 1.15])
def test_full_size_ont_block(enc, ont_full, lossy):
    """The ONT block lossless and at -l 1.15 (rblock@0x426c10; lengths through
    compressLen_short, every read < 65536 bp)."""
    _check(enc, ont_full, fq.Config(lossy=lossy))


def test_resident_inputs_concurrent_contexts(pe_full):
    """sa_input_create / sa_run_input: two resident batches encoded by two contexts
    sharing one front scratch (sa_create_shared) from two host threads at once
    (the bench's pipeline) == the oracle."""
    import threading
    a, b = synth.generate(20000, paired=True, seed=77)
    b1 = fq.blocks_from_fastq(a, b, 2_000_000)
    b2 = pe_full[2:]
    cfg = fq.Config()
    want = {0: _oracle_outs(b1, cfg), 1: _oracle_outs(b2, cfg)}
    inputs = [fq.Input(b1, 0), fq.Input(b2, 0)]
    e0 = fq.Encoder(0)
    encs = [e0, fq.Encoder(0, share_with=e0)]   # one front scratch, fronts one at a time
    got, errs = {}, []

    def work(i):
        try:
            for rep in range(3):
                encs[i].run_input(inputs[(i + rep) % 2], cfg)
                got[(i, rep)] = ((i + rep) % 2, encs[i].fetch())
        except Exception as e:
            errs.append(e)

    th = [threading.Thread(target=work, args=(i,)) for i in range(2)]
    for t in th:
        t.start()
    for t in th:
        t.join()
    for e in encs:
        e.close()
    for i in inputs:
        i.close()
    assert not errs, errs
    for (i, rep), (which, outs) in got.items():
        assert outs == want[which], (i, rep)


# ---- sa_stage_text: FASTQ text parsed on the device ------------------------------------------

def _texts(t1, t2=None, bs=fq.BLOCK_SIZE):
    a = fq._as_u8(t1)
    if t2 is None:
        return [(a[s:e], None) for s, e in fq.cut_se(a, bs)]
    b = fq._as_u8(t2)
    return [(a[s1:e1], b[s2:e2]) for (s1, e1), (s2, e2) in fq.cut_pe(a, b, bs)]


def _check_text(enc, t1, t2, cfg, bs=fq.BLOCK_SIZE):
    """Blocks staged as text (device parse) encode to the same bytes as the
    host-parsed blocks (getBlockRead[PE] restated in fastq_host.cpp)."""
    texts = _texts(t1, t2, bs)
    blocks = fq.blocks_from_fastq(t1, t2, bs)
    info = enc.stage_text(texts)
    enc.run(cfg)
    got = enc.fetch()
    assert [i["nreads"] for i in info] == [b.nreads for b in blocks]
    assert [i["name_bytes"] for i in info] == [b.names.size for b in blocks]
    assert [i["seq_bytes"] for i in info] == [b.seq.size for b in blocks]
    assert [i["len_long"] for i in info] == [int((b.seq_lens > 0xffff).any()) for b in blocks]
    want = enc.encode(blocks, cfg)
    for k, (g, w) in enumerate(zip(got, want)):
        assert g == w, f"block {k}: device-parsed {len(g)} B vs host-parsed {len(w)} B"
    return got


def test_stage_text_reference_pair(enc, test_pair):
    tmpl = fq.analyze_ids(fq.blocks_from_fastq(*test_pair)[0], False)
    _check_text(enc, *test_pair, fq.Config(bin_mode=int(tmpl[0])))
    _check_text(enc, *test_pair, fq.Config(bin_mode=int(tmpl[0])), bs=1 << 20)   # several blocks per batch
    _check_text(enc, test_pair[0], None, fq.Config(bin_mode=1), bs=300_000)


def test_stage_text_edge_cases(enc):
    _check_text(enc, synth.edge_cases(), None, fq.Config())
    _check_text(enc, _long_read_fastq(91, 120), None, fq.Config(qlevel=3))
    t_long, _ = synth.generate(6, seed=92, read_len=70000)             # len_long blocks
    _check_text(enc, t_long, None, fq.Config())
    a, _ = synth.generate(3000, paired=True, seed=93)
    _, short = synth.generate(3000, paired=True, seed=94, read_len=90)  # mates of unequal length
    _check_text(enc, a, short, fq.Config(), bs=400_000)
    # no newline at the end of the file: the partial last line is dropped by both parsers
    _check_text(enc, synth.edge_cases() + b"@tail", None, fq.Config())


def test_text_upload_streamed_equals_stage_text(enc, test_pair):
    """sa_text_upload block by block (each into its stride slot of either text
    arena) + sa_text_parse give the batch sa_stage_text gives: the encoded
    blocks equal, for PE with several blocks per batch, SE, mates of unequal
    length, a wider stride than the texts, and arena 1 after arena 0 (the
    command line alternates them)."""
    tmpl = fq.analyze_ids(fq.blocks_from_fastq(*test_pair)[0], False)
    a, _ = synth.generate(3000, paired=True, seed=95)
    _, short = synth.generate(3000, paired=True, seed=96, read_len=90)
    cases = [(test_pair[0], test_pair[1], fq.Config(bin_mode=int(tmpl[0])), 1 << 20),
             (test_pair[0], None, fq.Config(bin_mode=1), 300_000),
             (a, short, fq.Config(), 400_000),
             (synth.edge_cases(), None, fq.Config(qlevel=3), fq.BLOCK_SIZE)]
    for k, (t1, t2, cfg, bs) in enumerate(cases):
        texts = _texts(t1, t2, bs)
        enc.stage_text(texts)
        enc.run(cfg)
        want = enc.fetch()
        for slot, extra in ((0, 0), (1, 12345), (0, 4096)):
            stride = max(max(len(x), 0 if y is None else len(y)) for x, y in texts) + extra
            enc.stage_text_streamed(texts, slot=slot, stride=stride)
            enc.run(cfg)
            assert enc.fetch() == want, (k, slot, extra)
    with pytest.raises(fq.SeqArcError):   # a text longer than the stride is refused
        enc.stage_text_streamed(_texts(a, short, 400_000), stride=1000)


def test_stage_text_full_size_batch(enc):
    """Three 50 MiB PE blocks (the bench's unit of work), staged as text."""
    a, b = synth.generate(150_000, paired=True, seed=31)
    _check_text(enc, a, b, fq.Config())


@pytest.mark.parametrize("case", ["truncated_se", "qual_len_pe", "long_name", "qual_past_end"])
def test_stage_text_rejects_what_the_host_parser_rejects(enc, case):
    rec = b"@r\nACGT\n+\nIIII\n"
    if case == "truncated_se":
        t1, t2 = rec * 3 + b"@r\nACGT\n+\n", None
    elif case == "qual_len_pe":
        t1, t2 = rec * 2, rec + b"@r\nACGT\n+\nIII\n"
    elif case == "long_name":
        t1, t2 = rec + b"@" + b"n" * 70000 + b"\nACGT\n+\nIIII\n", None
    else:   # SE copies the sequence's length of qualities: past the end of the block
        t1, t2 = rec + b"@r\nACGTACGT\n+\nII\n", None
    with pytest.raises(fq.SeqArcError):
        fq.parse_se(t1) if t2 is None else fq.parse_pe(t1, t2)
    with pytest.raises(fq.SeqArcError):
        enc.stage_text([(t1, t2)])
    _check_text(enc, rec * 5, None, fq.Config())   # the context stays usable
