"""HASH reference-index path on one MI355X.

Three legs, one JSON line:
  * index build (`SeqArc -i ref.fa`, buildRefIndex@0x410190) of a synthetic
    genome, GRCh38-sized with --genome-mb 3100 (seconds, FASTA in host memory);
  * gapless seed alignment (getHashAlignInfo@0x4113c0) of 150 bp reads drawn
    from it (reads/s, sa_hash_align incl. transfers);
  * the aligned block encode (AlignEncode{SE,PE}Job::doAlign + doAlignEncode
    @0x42d4c0, sa_run_input_aligned) of a batch of full 50 MiB PE blocks
    resident in HBM (FASTQ MB/s), with the no-reference encode of the same
    batch beside it.
CPU restatement (oracle/, one thread) on a sample where the genome is small
enough for its index (<= --cpu-max-mb), and its agreement with the GPU there.
usage: python scripts/bench_hash.py [--genome-mb 3100] [--reads 2000000] [--pairs 1200000]"""
import argparse
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))

import fastqueeze_amd as fq  # noqa: E402
import oracle_py as orc  # noqa: E402

ACGT = np.frombuffer(b"ACGT", dtype=np.uint8)
COMP = np.zeros(256, np.uint8)
COMP[list(b"ACGTN")] = list(b"TGCAN")


def log(msg):
    print(f"[hash] {msg}", file=sys.stderr, flush=True)


def genome_fasta(rng, glen, width=60):
    """A random ACGT genome as one FASTA record (60-column lines)."""
    g = ACGT[rng.integers(0, 4, glen, dtype=np.uint8)]
    full = glen // width
    body = np.empty((full, width + 1), np.uint8)
    body[:, :width] = g[:full * width].reshape(full, width)
    body[:, width] = 10
    tail = g[full * width:].tobytes()
    return b">chrS synthetic\n" + body.tobytes() + (tail + b"\n" if tail else b""), g


def fastq(seq, mate, first):
    """Fixed-width FASTQ records (Illumina-style headers) for an n x L base array."""
    n, L = seq.shape
    pre = b"@SYN:7:HXX3:1:"
    suf = b" %d:N:0:1" % mate
    digits = 10
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
    rng = np.random.default_rng(first + mate)
    a[:, o:o + L] = np.frombuffer(b"F:,F", np.uint8)[rng.integers(0, 4, (n, L), dtype=np.uint8)]
    a[:, o + L] = 10
    return a.tobytes()


def draw(rng, g, starts, rev, L, sub=0.004, random_frac=0.02):
    seq = g[starts[:, None] + np.arange(L)]
    m = rng.random(seq.shape) < sub
    seq[m] = ACGT[rng.integers(0, 4, int(m.sum()), dtype=np.uint8)]
    rnd = rng.random(len(starts)) < random_frac
    seq[rnd] = ACGT[rng.integers(0, 4, (int(rnd.sum()), L), dtype=np.uint8)]
    seq[rev] = COMP[seq[rev][:, ::-1]]
    return seq


def pe_reads(rng, g, pairs, L, first=0):
    glen = g.size
    s1 = rng.integers(0, glen - 1000 - L, pairs)
    rv = rng.random(pairs) < 0.5
    s2 = np.minimum(s1 + rng.integers(250, 450, pairs) - L, glen - L)
    far = rng.random(pairs) < 0.02
    s2[far] = rng.integers(0, glen - L, int(far.sum()))
    return fastq(draw(rng, g, s1, rv, L), 1, first), fastq(draw(rng, g, s2, ~rv, L), 2, first)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--genome-mb", type=float, default=3100)
    ap.add_argument("--reads", type=int, default=2_000_000)
    ap.add_argument("--read-len", type=int, default=150)
    ap.add_argument("--pairs", type=int, default=1_200_000, help="PE pairs of the aligned-encode batch")
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--cpu-reads", type=int, default=20_000)
    ap.add_argument("--cpu-max-mb", type=float, default=400)
    args = ap.parse_args()
    rng = np.random.default_rng(2024)
    glen = int(args.genome_mb * 1e6)
    L = args.read_len
    t0 = time.perf_counter()
    fa, g = genome_fasta(rng, glen)
    log(f"genome {glen / 1e6:.0f} Mb ({len(fa) / 1e9:.2f} GB FASTA) in {time.perf_counter() - t0:.1f} s")

    enc = fq.Encoder(0)
    t0 = time.perf_counter()
    ix = fq.HashIndex(enc, fa)
    t_build = time.perf_counter() - t0
    log(f"index built in {t_build:.2f} s")

    # ---- gapless seed alignment of single reads ----
    starts = rng.integers(0, glen - L, args.reads)
    rv = np.arange(args.reads) % 2 == 1
    seqs = draw(rng, g, starts, rv, L, sub=0.002, random_frac=0.0)
    raw = seqs.tobytes()
    reads = [raw[i * L:(i + 1) * L] for i in range(args.reads)]
    ix.align(reads[:10_000])   # warm-up
    t0 = time.perf_counter()
    ret, rev, pos, mp, mt = ix.align(reads)
    t_align = time.perf_counter() - t0
    n_chk = min(len(reads), 2000)
    ok = sum(int(ret[i] >= 0 and pos[i] == starts[i] + 1 and rev[i] == (i % 2)) for i in range(n_chk))
    log(f"{len(reads)} reads aligned in {t_align:.2f} s")

    # ---- the aligned block encode of a resident batch of 50 MiB PE blocks ----
    t1, t2 = pe_reads(rng, g, args.pairs, L)
    blocks = fq.blocks_from_fastq(t1, t2)
    text = sum(b.text_bytes for b in blocks)
    log(f"{len(blocks)} PE blocks, {text / 1e6:.0f} MB FASTQ")
    inp = fq.Input(blocks)
    tmpl = fq.analyze_ids(blocks[0], False)
    cfg = fq.Config(bin_mode=int(tmpl[0]))
    times, times_noref = [], []
    out_a = out_n = None
    for rep in range(args.reps + 1):
        chain = fq.AlignChain()
        torch.cuda.synchronize(0)
        t0 = time.perf_counter()
        enc.run_aligned(cfg, ix, True, chain, inp=inp)
        torch.cuda.synchronize(0)
        if rep:
            times.append(time.perf_counter() - t0)
        chain.close()
        if rep == args.reps:
            out_a = enc.fetch()
        t0 = time.perf_counter()
        enc.run_input(inp, cfg)
        torch.cuda.synchronize(0)
        if rep:
            times_noref.append(time.perf_counter() - t0)
        if rep == args.reps:
            out_n = enc.fetch()
    t_enc, t_noref = min(times), min(times_noref)
    ratio_a = text / sum(map(len, out_a))
    ratio_n = text / sum(map(len, out_n))
    log(f"aligned encode {text / t_enc / 1e6:.0f} MB/s (ratio {ratio_a:.2f}), "
        f"no reference {text / t_noref / 1e6:.0f} MB/s (ratio {ratio_n:.2f})")

    out = {
        "metric": "HASH reference path: aligned block encode, FASTQ MB/s (1 MI355X, batch resident in HBM)",
        "value": round(text / t_enc / 1e6, 1), "unit": "MB/s",
        "index_build_s": round(t_build, 3), "genome_bases": glen,
        "aligned_encode": {"blocks": len(blocks), "fastq_bytes": text, "s": round(t_enc, 4),
                           "ratio": round(ratio_a, 3)},
        "noref_encode_same_batch": {"MB/s": round(text / t_noref / 1e6, 1), "ratio": round(ratio_n, 3)},
        "align_reads_per_s": round(len(reads) / t_align, 1), "align_reads": len(reads), "read_len": L,
        "aligned_fraction": round(float((ret >= 0).mean()), 4),
        "true_position_fraction_first_2000": round(ok / n_chk, 4),
        "parity": "GPU == oracle/ restatement (tests/test_gpu_align.py); unpinned against SeqArc itself",
    }
    if glen <= args.cpu_max_mb * 1e6:
        orc.hash_index(fa)
        cs = reads[:args.cpu_reads]
        t0 = time.perf_counter()
        cret, crev, cpos, cmp_, cmt = orc.hash_align(cs)
        t_cpu = time.perf_counter() - t0
        out["cpu_align_baseline"] = {"value": round(len(cs) / t_cpu, 1), "unit": "reads/s", "cores": 1,
                                     "kind": "port", "sample": f"first {len(cs)} reads, oracle/hash_oracle.c"}
        out["gpu_align_equals_oracle_on_sample"] = bool(
            np.array_equal(cret, ret[:len(cs)]) and np.array_equal(cpos, pos[:len(cs)])
            and np.array_equal(cmp_, mp[:len(cs)]))
        b0 = blocks[0]
        t0 = time.perf_counter()
        want = orc.encode_block_hash(b0, True, [0, 0], bin_mode=cfg.bin_mode)
        t_cpu = time.perf_counter() - t0
        out["cpu_baseline"] = {"value": round(b0.text_bytes / t_cpu / 1e6, 2), "unit": "MB/s",
                               "cores": 1, "kind": "port", "sample": "block 0 (50 MiB PE), oracle/ doAlign + "
                                                                     "doAlignEncode restatement"}
        out["gpu_block0_equals_oracle"] = bool(out_a[0] == want)
    ix.close()
    enc.close()
    print(json.dumps(out))


if __name__ == "__main__":
    main()
