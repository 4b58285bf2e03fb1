"""GPU parity of the reference (HASH index) block path -- the encoder with an
index, configs[3]: AlignEncode{SE,PE}Job::doAlign
(@0x411910 / @0x413580: the aligner over the carried align_info chain, the 5 %
probe and bail-out, the PE insert window CaclInsertSize@0x413270) and
EncapFqzComp::doAlignEncode@0x42d4c0 (order / position / mismatch / strand /
PE-relation streams, the SEQ stream of the unaligned reads), every block byte
for byte against the CPU restatement (oracle/align_oracle.c +
oracle/hash_oracle.c + oracle/fqz_oracle.c).  Parity with SeqArc itself is
unpinned: the reference ships no index and no aligned archive."""
import numpy as np
import pytest

import fastqueeze_amd as fq
import oracle_py as orc
import synth

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def enc():
    e = fq.Encoder(0)
    yield e
    e.close()


@pytest.fixture(scope="module")
def ref():
    fa, g = synth.reference(3_000_000, 21)
    return fa, g


@pytest.fixture(scope="module")
def index(enc, ref):
    fa, _ = ref
    orc.hash_index(fa)               # the oracle keeps its index for encode_block_hash
    ix = fq.HashIndex(enc, fa)
    yield ix
    ix.close()


def oracle_blocks(blocks, paired, cfg, **kw):
    carry = [0, 0]
    return [orc.encode_block_hash(b, paired, carry, slevel=cfg.slevel, qlevel=cfg.qlevel, md5=cfg.md5,
                                  bin_mode=cfg.bin_mode, **kw) for b in blocks]


def check(enc, index, blocks, paired, cfg=None, **kw):
    cfg = cfg or fq.Config()
    got = enc.encode_aligned(blocks, cfg, index, paired, **kw)
    want = oracle_blocks(blocks, paired, cfg, **kw)
    assert len(got) == len(want)
    same(got, want)
    return got


def same(got, want):
    """Blocks equal (a failure names the first differing block and byte; pytest's
    own diff of two large byte strings takes minutes)."""
    if len(got) != len(want):
        pytest.fail(f"{len(got)} blocks vs {len(want)}")
    for i, (g, w) in enumerate(zip(got, want)):
        if g != w:
            k = next((k for k in range(min(len(g), len(w))) if g[k] != w[k]), min(len(g), len(w)))
            pytest.fail(f"block {i}: {len(g)} vs {len(w)} bytes, first difference at {k}")


@pytest.mark.parametrize("paired", [False, True])
def test_blocks_identical(enc, index, ref, paired):
    _, g = ref
    r1, r2 = synth.aligned_reads(g, 12000, 31, paired=paired, random_frac=0.08, far_frac=0.1, short_frac=0.2)
    blocks = fq.blocks_from_fastq(r1, r2, block_size=1_000_000)
    assert len(blocks) >= 3
    out = check(enc, index, blocks, paired)
    assert sum(map(len, out)) < sum(map(len, orc_noref(blocks)))   # aligned reads leave the SEQ stream


def orc_noref(blocks):
    return [orc.encode_block(b) for b in blocks]


@pytest.mark.parametrize("paired", [False, True])
def test_carried_state_and_short_reads(enc, index, ref, paired):
    """Short reads whose even-offset seeds are all broken: the search consults
    the carried align_info; both variants run on the GPU, the chain picks."""
    _, g = ref
    r1, r2 = synth.aligned_reads(g, 8000, 32, paired=paired, random_frac=0.1, short_frac=0.6)
    check(enc, index, fq.blocks_from_fastq(r1, r2, block_size=400_000), paired)


@pytest.mark.parametrize("paired", [False, True])
def test_bail_out(enc, index, ref, paired):
    """Blocks where fewer than half of the first 5 % of reads align: the rest of
    the block goes through the SEQ stream without order bytes."""
    _, g = ref
    r1, r2 = synth.aligned_reads(g, 6000, 33, paired=paired, random_frac=0.7, far_frac=0.3)
    check(enc, index, fq.blocks_from_fastq(r1, r2, block_size=300_000), paired)


def test_pe_insert_size_option(enc, index, ref):
    _, g = ref
    r1, r2 = synth.aligned_reads(g, 6000, 34, paired=True, far_frac=0.2)
    blocks = fq.blocks_from_fastq(r1, r2, block_size=600_000)
    check(enc, index, blocks, True, insert_size=500)
    check(enc, index, blocks, True, insert_size=50)


@pytest.mark.parametrize("maxmis", [0, 3, 8])
def test_maxmis(enc, index, ref, maxmis):
    """Mis stream model by maxmis (SIMPLE_MODEL<8> for 1..7, <9> for 8, no
    symbols otherwise; compressAlignInfo_Mis@0x425ff0)."""
    _, g = ref
    r1, _ = synth.aligned_reads(g, 4000, 35, short_frac=0.2)
    check(enc, index, fq.blocks_from_fastq(r1, None, block_size=400_000), False, maxmis=maxmis)


def test_chain_across_batches(enc, index, ref):
    """Two batches through one chain equal one oracle pass over all blocks."""
    _, g = ref
    r1, r2 = synth.aligned_reads(g, 8000, 36, paired=True, short_frac=0.4, random_frac=0.1)
    blocks = fq.blocks_from_fastq(r1, r2, block_size=500_000)
    cfg = fq.Config()
    chain = fq.AlignChain()
    got = []
    for k, part in enumerate((blocks[:2], blocks[2:])):
        enc.stage(part)
        enc.run_aligned(cfg, index, True, chain, batch=k)
        got += enc.fetch()
    chain.close()
    same(got, oracle_blocks(blocks, True, cfg))


def test_index_from_hash_file(enc, index, ref):
    """The `.hash` file loaded back (sa_hash_load) aligns as the built index."""
    _, g = ref
    ix2 = fq.HashIndex(enc, None, hash_file=index.file_bytes())
    try:
        r1, _ = synth.aligned_reads(g, 3000, 37)
        blocks = fq.blocks_from_fastq(r1, None, block_size=400_000)
        same(enc.encode_aligned(blocks, fq.Config(), ix2, False), enc.encode_aligned(blocks, fq.Config(), index, False))
    finally:
        ix2.close()


def test_full_block_pe(enc, index, ref):
    """A full 50 MiB block of 150 bp pairs (configs[3] shape, scaled genome)."""
    _, g = ref
    r1, r2 = synth.aligned_reads(g, 80_000, 38, paired=True, random_frac=0.02, far_frac=0.02)
    blocks = fq.blocks_from_fastq(r1, r2)
    assert blocks[0].nreads > 100_000
    check(enc, index, blocks[:1], True)


def test_other_configs(enc, index, ref):
    """Slevel 4 / Qlevel 3 / MD5 off / ID-bin names on the reference path."""
    _, g = ref
    r1, r2 = synth.aligned_reads(g, 3000, 39, paired=True)
    blocks = fq.blocks_from_fastq(r1, r2, block_size=400_000)
    tmpl = fq.analyze_ids(blocks[0], False)
    for cfg in (fq.Config(slevel=4), fq.Config(qlevel=3), fq.Config(md5=False), fq.Config(bin_mode=int(tmpl[0]))):
        check(enc, index, blocks, True, cfg)


def test_cli_reference_path(tmp_path):
    """seqarc_amd -i ref.fa / -c ref.fa / -d ref.fa (README.md:19-26, 55-93): the
    index files equal the restatement's, the archive equals the oracle's blocks
    in the restated container (the align_info chain through 1 MiB blocks in
    2-block batches over two contexts), with the index loaded from ref.fa.hash
    or built from ref.fa, -I, SE on the host parser; -d brings the reads back."""
    import hashlib
    import os
    import subprocess
    from fastqueeze_amd import build
    fa, g = synth.reference(1_500_000, 51, chroms=2)
    fa = fa.upper()   # (aligned bases come back from the genome in upper case)
    (tmp_path / "ref.fa").write_bytes(fa)
    run = lambda args: subprocess.run([build.CLI] + args, capture_output=True, cwd=tmp_path, timeout=300)
    r = run(["-i", "ref.fa"])
    assert r.returncode == 0, r.stderr
    hfile = orc.hash_index(fa)
    same([(tmp_path / "ref.fa.hash").read_bytes()], [hfile])
    assert (tmp_path / "ref.fa.md5").read_bytes() == hashlib.md5(fa).digest()
    r1, r2 = synth.aligned_reads(g, 14000, 52, paired=True, random_frac=0.1, far_frac=0.1, short_frac=0.2)
    (tmp_path / "a_1.fq").write_bytes(r1)
    (tmp_path / "a_2.fq").write_bytes(r2)
    (tmp_path / "s.fq").write_bytes(r1)

    def want(paired, ins=0):
        blocks = fq.blocks_from_fastq(r1, r2 if paired else None, 1 << 20)
        assert len(blocks) >= 3
        tmpl = fq.analyze_ids(blocks[0], not paired)
        cfg = fq.Config(bin_mode=int(tmpl[0]))
        carry = [0, 0]
        enc = [orc.encode_block_hash(b, paired, carry, bin_mode=cfg.bin_mode, insert_size=ins) for b in blocks]
        return fq.arc_archive(enc, blocks, "a_1.fq" if paired else "s.fq", "a_2.fq" if paired else None, tmpl, cfg,
                              plus_bare=fq.bare_plus(r1), ref_md5=hashlib.md5(fa).digest(), insert_size=ins)

    base = ["-c", "-f", "--block-size", "1", "--batch", "2"]
    r = run(base + ["--contexts", "2", "ref.fa", "-1", "a_1.fq", "-2", "a_2.fq", "pe"])
    assert r.returncode == 0, r.stderr
    same([(tmp_path / "pe.arc").read_bytes()], [want(True)])
    r = run(["-d", "ref.fa", "pe.arc", "back"])
    assert r.returncode == 0, r.stderr
    same([(tmp_path / "back_1.fastq").read_bytes(), (tmp_path / "back_2.fastq").read_bytes()], [r1, r2])
    r = run(base + ["--host-parse", "ref.fa", "-1", "s.fq", "se"])
    assert r.returncode == 0, r.stderr
    same([(tmp_path / "se.arc").read_bytes()], [want(False)])
    os.remove(tmp_path / "ref.fa.hash")   # the index built on the device from the FASTA
    r = run(base + ["-I", "300", "ref.fa", "-1", "a_1.fq", "-2", "a_2.fq", "pi"])
    assert r.returncode == 0, r.stderr
    same([(tmp_path / "pi.arc").read_bytes()], [want(True, 300)])
    r = run(["-d", "ref.fa", "pi.arc", "bi"])
    assert r.returncode == 0, r.stderr
    same([(tmp_path / "bi_1.fastq").read_bytes()], [r1])


def test_cli_reference_shm(tmp_path):
    """-i -s / -c -s (README.md:32): the index image goes to /dev/shm/<ref file
    name> (IHashRefIndex::createShm@0x41f280) and -c -s encodes from it with no
    ref.fa.hash on disk -- the same archive as from the file."""
    import hashlib
    import os
    import subprocess
    from fastqueeze_amd import build
    name = f"sa_shm_gpu_{os.getpid()}.fa"
    shm = os.path.join("/dev/shm", name)
    fa, g = synth.reference(800_000, 81, chroms=2)
    fa = fa.upper()
    (tmp_path / name).write_bytes(fa)
    run = lambda args: subprocess.run([build.CLI] + args, capture_output=True, cwd=tmp_path, timeout=300)
    r1, r2 = synth.aligned_reads(g, 6000, 82, paired=True, random_frac=0.1)
    (tmp_path / "a_1.fq").write_bytes(r1)
    (tmp_path / "a_2.fq").write_bytes(r2)
    base = ["-c", "-f", "--block-size", "1", "--batch", "2"]
    try:
        if os.path.exists(shm):
            os.remove(shm)
        r = run(["-s", "-i", name])
        assert r.returncode == 0, r.stderr
        assert open(shm, "rb").read() == (tmp_path / (name + ".hash")).read_bytes()
        r = run(base + [name, "-1", "a_1.fq", "-2", "a_2.fq", "file"])
        assert r.returncode == 0, r.stderr
        os.remove(tmp_path / (name + ".hash"))
        r = run(base + ["-s", "-v", name, "-1", "a_1.fq", "-2", "a_2.fq", "mem"])
        assert r.returncode == 0, r.stderr
        assert b"from /dev/shm/" in r.stderr
        assert (tmp_path / "mem.arc").read_bytes() == (tmp_path / "file.arc").read_bytes()
        r = run(["-d", "-s", name, "mem.arc", "back"])
        assert r.returncode == 0, r.stderr
        assert (tmp_path / "back_1.fastq").read_bytes() == r1
    finally:
        if os.path.exists(shm):
            os.remove(shm)


def test_cli_reference_maxmis_bailout_chain(tmp_path):
    """a non-default --maxmis is recorded in the archive (params field
    19) so -d rebuilds the same Mis model without the flag; blocks that bail out
    and -I across several batches per chain on two contexts; --maxmis 9 (no Mis
    model) is refused."""
    import hashlib
    import subprocess
    from fastqueeze_amd import build
    fa, g = synth.reference(1_200_000, 61, chroms=2)
    fa = fa.upper()
    (tmp_path / "ref.fa").write_bytes(fa)
    orc.hash_index(fa)   # (the oracle aligns against its last built index)
    run = lambda args: subprocess.run([build.CLI] + args, capture_output=True, cwd=tmp_path, timeout=300)
    # first half aligns, second half mostly random reads (later blocks bail out)
    a1, a2 = synth.aligned_reads(g, 6000, 62, paired=True, short_frac=0.2)
    b1, b2 = synth.aligned_reads(g, 6000, 63, paired=True, random_frac=0.8, far_frac=0.3)
    r1, r2 = a1 + b1, a2 + b2
    (tmp_path / "a_1.fq").write_bytes(r1)
    (tmp_path / "a_2.fq").write_bytes(r2)
    for maxmis, ins in ((3, 300), (0, 0), (8, 0)):
        blocks = fq.blocks_from_fastq(r1, r2, 1 << 20)
        assert len(blocks) >= 4
        tmpl = fq.analyze_ids(blocks[0], False)
        cfg = fq.Config(bin_mode=int(tmpl[0]))
        carry = [0, 0]
        enc = [orc.encode_block_hash(b, True, carry, bin_mode=cfg.bin_mode, insert_size=ins, maxmis=maxmis)
               for b in blocks]
        want = fq.arc_archive(enc, blocks, "a_1.fq", "a_2.fq", tmpl, cfg, plus_bare=fq.bare_plus(r1),
                              ref_md5=hashlib.md5(fa).digest(), insert_size=ins, maxmis=maxmis)
        args = ["-c", "-f", "--block-size", "1", "--batch", "1", "--contexts", "2", "--maxmis", str(maxmis)]
        args += (["-I", str(ins)] if ins else []) + ["ref.fa", "-1", "a_1.fq", "-2", "a_2.fq", f"m{maxmis}"]
        r = run(args)
        assert r.returncode == 0, r.stderr
        same([(tmp_path / f"m{maxmis}.arc").read_bytes()], [want])
        r = run(["-d", "ref.fa", f"m{maxmis}.arc", f"d{maxmis}"])   # (no --maxmis: from the archive)
        assert r.returncode == 0, r.stderr
        same([(tmp_path / f"d{maxmis}_1.fastq").read_bytes(), (tmp_path / f"d{maxmis}_2.fastq").read_bytes()],
             [r1, r2])
    r = run(["-c", "-f", "--maxmis", "9", "ref.fa", "-1", "a_1.fq", "-2", "a_2.fq", "bad"])
    assert r.returncode != 0 and b"0..8" in r.stderr


def test_aligned_maxmis_out_of_range_fails_chain(enc, index, ref):
    """maxmis 9 is refused by sa_run_input_aligned, and the chain is failed so a
    later batch waiting on it returns an error instead of hanging."""
    _, g = ref
    r1, _ = synth.aligned_reads(g, 2000, 64)
    blocks = fq.blocks_from_fastq(r1, None, block_size=200_000)
    chain = fq.AlignChain()
    try:
        enc.stage(blocks[:1])
        with pytest.raises(fq.SeqArcError):
            enc.run_aligned(fq.Config(), index, False, chain, batch=0, maxmis=9)
        enc.stage(blocks[1:2])
        with pytest.raises(fq.SeqArcError):   # batch 1 would wait for batch 0 forever
            enc.run_aligned(fq.Config(), index, False, chain, batch=1)
    finally:
        chain.close()
