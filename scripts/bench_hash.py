"""HASH reference-index path on one MI355X: index
build time for a synthetic genome and gapless seed alignment throughput of
150 bp reads drawn from it (with substitutions, both strands), against the CPU
restatement (oracle/hash_oracle.c, one thread) on a sample.  One JSON line.
usage: python scripts/bench_hash.py [--genome-mb 100] [--reads 2000000]"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))

import fastqueeze_amd as fq  # noqa: E402
import oracle_py as orc  # noqa: E402

COMP = bytes.maketrans(b"ACGT", b"TGCA")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--genome-mb", type=float, default=100)
    ap.add_argument("--reads", type=int, default=2_000_000)
    ap.add_argument("--read-len", type=int, default=150)
    ap.add_argument("--cpu-reads", type=int, default=20_000)
    args = ap.parse_args()
    rng = np.random.default_rng(2024)
    glen = int(args.genome_mb * 1e6)
    g = np.frombuffer(b"ACGT", dtype=np.uint8)[rng.integers(0, 4, glen)]
    lines = g.tobytes()
    fa = b">chrS synthetic\n" + b"\n".join(lines[i:i + 60] for i in range(0, glen, 60)) + b"\n"
    L = args.read_len
    starts = rng.integers(0, glen - L, args.reads)
    win = np.lib.stride_tricks.sliding_window_view(g, L)[starts].copy()
    flat = win.reshape(-1)
    at = rng.integers(0, flat.size, int(flat.size * 0.002))
    flat[at] = np.frombuffer(b"ACGT", dtype=np.uint8)[rng.integers(0, 4, at.size)]
    raw = win.tobytes()
    reads = [raw[i * L:(i + 1) * L] for i in range(args.reads)]
    reads = [r.translate(COMP)[::-1] if i % 2 else r for i, r in enumerate(reads)]
    print(f"[hash] genome {glen / 1e6:.0f} Mb, {len(reads)} reads of {L} bp", file=sys.stderr, flush=True)

    enc = fq.Encoder(0)
    t0 = time.perf_counter()
    ix = fq.HashIndex(enc, fa)
    t_build = time.perf_counter() - t0
    ix.align(reads[:10_000])   # warm-up
    t0 = time.perf_counter()
    ret, rev, pos, mp, mt = ix.align(reads)
    t_align = time.perf_counter() - t0
    aligned = float((ret >= 0).mean())
    ok = 0
    n_chk = min(len(reads), 2000)
    for i in range(n_chk):
        ok += int(ret[i] >= 0 and pos[i] == starts[i] + 1 and rev[i] == (i % 2))
    # CPU restatement on a sample (and its agreement with the GPU there)
    orc.hash_index(fa)
    cs = reads[:args.cpu_reads]
    t0 = time.perf_counter()
    cret, crev, cpos, cmp_, cmt = orc.hash_align(cs)
    t_cpu = time.perf_counter() - t0
    same = bool(np.array_equal(cret, ret[:len(cs)]) and np.array_equal(cpos, pos[:len(cs)])
                and np.array_equal(cmp_, mp[:len(cs)]))
    out = {
        "metric": "HASH-index gapless seed alignment, reads/s (1 MI355X)",
        "value": round(len(reads) / t_align, 1), "unit": "reads/s",
        "index_build_s": round(t_build, 3), "genome_bases": glen, "reads": len(reads), "read_len": L,
        "aligned_fraction": round(aligned, 4), "true_position_fraction_first_2000": round(ok / n_chk, 4),
        "align_s_incl_transfers": round(t_align, 3),
        "cpu_baseline": {"value": round(len(cs) / t_cpu, 1), "unit": "reads/s", "cores": 1, "kind": "port",
                         "sample": f"first {len(cs)} reads, oracle/hash_oracle.c (-O2, 1 thread)"},
        "gpu_equals_oracle_on_sample": same,
        "parity": "unpinned against SeqArc (no reference index/alignments available)",
    }
    ix.close()
    enc.close()
    print(json.dumps(out))


if __name__ == "__main__":
    main()
