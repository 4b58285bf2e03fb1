"""bench.py -- MB/s of FASTQ compressed by the MI355X SeqArc block encoder.

Workload (BASELINE.json metric "150 bp PE"; configs[2]'s per-GPU shape):
synthetic 150 bp paired-end reads, no reference, default SeqArc parameters
(Slevel 3 -> order-10 base model, Qlevel 2, 50 MiB blocks, per-block MD5),
generated with the SURVEY.md 8(d) spec (tests/synth.py).  Every GPU holds
`--batches` distinct batches of `--pairs` mate pairs (5 M pairs = 3.57 GB of
FASTQ = 69 blocks) resident in HBM.  A step = one encode of one batch (all its
blocks, every stream, MD5, assembly; outputs left in HBM).  `--contexts` encoder
contexts per GPU run steps concurrently from their own host threads, so one
batch's throughput-bound front (symbol extraction, sorts, model replay) runs
while another batch's latency-bound range coder chains finish.

Multi-GPU: one process per GPU.  `--gpus N` without WORLD_SIZE in the
environment launches the N ranks itself (before any GPU call); under
torch.distributed.run the ranks come from the environment.  The global list of
batches is dealt to the ranks with fastqueeze_amd.shard.shard_indices (weak
scaling: each rank encodes its own batches, no data-path collective); the
barrier and the max-over-ranks time are the only collectives (gloo, host).
value = all ranks' FASTQ bytes of the timed steps / max-over-ranks time.

`--dry-run` runs the same launcher, sharding and gather on a tiny workload with
the CPU restatement as the encoder (no GPU; tests/test_shard.py).

Prints one JSON line (rank 0).
"""
from __future__ import annotations

import argparse
import hashlib
import shutil
import json
import os
import socket
import subprocess
import sys
import threading
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))

HBM_PEAK_GBS = 8000.0   # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec
# Dependency-chain bound of pass R: one wave issues at most one
# instruction per 4 cycles and a range-coder step's dependent chain is 8 SALU
# instructions (reciprocal multiply, correction multiply / compare / subtract,
# frequency multiply, leading zeros, mask, shift), so a stream of L symbols needs
# >= L * 32 cycles at 2.4 GHz.  (Rounds 1-3 priced 10 here: the record split,
# now in the VALU per segment.  The step issues 11: the 8 plus three readlanes.)
R_SALU_PER_SYMBOL = 8
R_ISSUED_PER_SYMBOL = 11
R_NS_PER_SYMBOL = R_SALU_PER_SYMBOL * 4 / 2.4
# reference per-block stream sizes of a 50 MiB 150 bp PE block
SURVEY_STREAMS = {"name": 58_700, "seq": 5_261_000, "qual": 1_552_000}
STREAM_IDS = {1: "count", 4: "len", 5: "name", 7: "qual", 23: "dege_tip", 14: "dege_ch", 24: "dege_maxq",
              25: "dege_ncnt", 26: "dege_npos", 6: "seq"}


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def parse_args(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=32,
                    help="timed batch encodes (the pipeline drain, ~1 batch latency, is amortised over them)")
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--contexts", type=int, default=5, help="encoder contexts (pipeline lanes) per GPU")
    ap.add_argument("--batches", type=int, default=0,
                    help="distinct resident batches per GPU (0: 4 at one rank, 2 with more ranks, whose generators "
                         "share the host's cores)")
    ap.add_argument("--no-share", action="store_true", help="contexts with their own front scratch (A/B)")
    ap.add_argument("--pairs", type=int, default=5_000_000, help="mate pairs per batch (reads with --se)")
    ap.add_argument("--se", action="store_true", help="single-end reads (configs[1] shape) instead of PE")
    ap.add_argument("--ont", action="store_true",
                    help="configs[4] shape: SE long reads of 10, 20, 30, 40 and 50 kbp (--pairs = reads per batch, "
                         "default 60000: ~3.6 GB of FASTQ); use with --lossy 1.15")
    ap.add_argument("--lossy", type=float, default=0.0, help="-l R: R-Block lossy qualities (rblock@0x426c10)")
    ap.add_argument("--read-len", type=int, default=150)
    ap.add_argument("--x-span", type=int, default=8,
                    help="header x coordinates drawn from this many values (8: ~60 kB name stream per block, "
                         "SURVEY 8's 58.7 kB; 0: uniform over 31000, ~195 kB)")
    ap.add_argument("--slevel", type=int, default=3)
    ap.add_argument("--qlevel", type=int, default=2)
    ap.add_argument("--block-size", type=int, default=50 << 20)
    ap.add_argument("--cpu-seconds", type=float, default=12.0, help="CPU baseline sample budget (each leg)")
    ap.add_argument("--gen-workers", type=int, default=0, help="generator processes (0: the CPU share)")
    ap.add_argument("--no-verify", action="store_true")
    ap.add_argument("--e2e-batches", type=int, default=-1,
                    help="batches written as FASTQ files for the end-to-end seqarc_amd -c run (-1: all at one "
                         "rank; rank 0's first with more ranks, run once through seqarc_amd --devices N; 0: skip)")
    ap.add_argument("--e2e-repeat", type=int, default=0,
                    help="the end-to-end files hold the e2e batches this many times over (a longer stream, so "
                         "pipeline fill and drain weigh less; 0: 3 at one rank, 2 x N with N ranks)")
    ap.add_argument("--e2e-batch", type=int, default=0, help="blocks per CLI batch in the e2e run (0: the bench's)")
    ap.add_argument("--e2e-gz-blocks", type=int, default=20,
                    help="the gzip end-to-end legs (BGZF, member-serial gzip) on this many blocks of batch 0 (0: skip)")
    ap.add_argument("--e2e-dir", default="/dev/shm" if os.path.isdir("/dev/shm") else os.environ.get("TMPDIR", "/tmp"))
    ap.add_argument("--e2e-log", default=None, help="write the CLI's stderr (-v stage lines, SA_TRACE) here")
    ap.add_argument("--e2e-settle", type=float, default=8.0,
                    help="seconds the device is left idle before each end-to-end run: the driver reclaims the "
                         "~200 GB the previous run released in the background, and allocations wait for it")
    ap.add_argument("--e2e-args", default="", help="extra seqarc_amd arguments for the end-to-end runs (A/B)")
    ap.add_argument("--dry-run", action="store_true", help="no GPU: CPU restatement, tiny batches (plumbing test)")
    ap.add_argument("--write-inputs", default=None, metavar="DIR",
                    help="generate this rank's batches as FASTQ files in DIR and exit (no GPU call): run it before a "
                         "profiled bench, whose process must not start generator processes under the profiler")
    ap.add_argument("--inputs", default=None, metavar="DIR",
                    help="read the batches from FASTQ files written by --write-inputs (no generator processes)")
    ap.add_argument("--no-legs", action="store_true",
                    help="only the in-HBM line (no e2e / gzip / ingest / ONT / HASH legs, no CPU baselines)")
    ap.add_argument("--ont-leg", type=int, default=1, help="configs[4] leg: ONT-shape SE long reads, -l 1.15 (0: skip)")
    ap.add_argument("--ont-reads", type=int, default=60_000, help="reads of the ONT leg's batch (10-50 kbp)")
    ap.add_argument("--se-leg", type=int, default=1,
                    help="configs[1] leg: 150 bp SE, default Slevel and Slevel 8 (0: skip)")
    ap.add_argument("--se-reads", type=int, default=10_000_000, help="reads of the SE leg's batch")
    ap.add_argument("--hash-leg", type=int, default=1, help="configs[3] leg: the HASH reference path (0: skip)")
    ap.add_argument("--hash-genome-mb", type=float, default=3100.0, help="synthetic genome of the HASH leg (GRCh38: 3100)")
    ap.add_argument("--hash-pairs", type=int, default=5_000_000,
                    help="PE pairs of the HASH leg's batch (5 M: 69 blocks, the headline's batch)")
    ap.add_argument("--hash-align-reads", type=int, default=4_000_000, help="single reads of the aligner leg")
    ap.add_argument("--leg-steps", type=int, default=10, help="timed steps of the ONT and HASH legs")
    ap.add_argument("--legs-fresh", type=int, default=1,
                    help="run the SE / ONT / HASH legs each in a process of its own (1) or in this one after "
                         "the headline (0: a second set of contexts in the process ran the ONT leg's front "
                         "~40 %% slower, r6s / r6v / r6w)")
    ap.add_argument("--leg-child", default=None, help=argparse.SUPPRESS)
    ap.add_argument("--text-leg", type=int, default=1,
                    help="staged-text leg: each step hands its batch over as FASTQ text in page-locked host "
                         "memory (sa_stage_text: H2D + device parse), encodes and fetches (0: skip)")
    ap.add_argument("--text-steps", type=int, default=15, help="timed steps of the staged-text leg")
    ap.add_argument("--decode-check", type=int, default=1,
                    help="decode the short e2e leg's archive with seqarc_amd -d and compare MD5s with the input")
    ap.add_argument("--ingest-devices", type=int, default=8,
                    help="the whole-node ingest leg: seqarc_amd --ingest-only --devices N over the long e2e files "
                         "(0: skip)")
    ap.add_argument("--step-gap-ms", type=float, default=0.0,
                    help="each context idles this long after each timed step (diagnostics: a bursty load like the "
                         "CLI's, whose contexts wait for the reader)")
    ap.add_argument("--traffic-json", default=os.path.join(ROOT, "profiles", "traffic_latest.json"),
                    help="per-launch HBM bytes per kernel from rocprofv3 --pmc passes of this bench "
                         "(scripts/pmc_traffic.py), committed under profiles/")
    a = ap.parse_args(argv)
    if a.ont:
        a.se = True
        if a.pairs == 5_000_000:
            a.pairs = 60_000
    if a.batches <= 0:
        a.batches = 4 if int(os.environ.get("WORLD_SIZE", "1")) == 1 and a.gpus == 1 else 2
    if a.e2e_batches < 0:   # (N ranks: rank 0's first batch, N x 2 times over, one seqarc_amd --devices N run)
        a.e2e_batches = a.batches if int(os.environ.get("WORLD_SIZE", "1")) == 1 and a.gpus == 1 else 1
    if a.no_legs:
        a.e2e_batches, a.cpu_seconds, a.ont_leg, a.hash_leg, a.ingest_devices, a.se_leg = 0, 0.0, 0, 0, 0, 0
    if a.dry_run:
        a.pairs = min(a.pairs, 3000)
        a.block_size = min(a.block_size, 300_000)
        a.steps = min(a.steps, 2)
        a.warmup = 0
        a.cpu_seconds = 0.0
    return a


def cpu_share() -> dict:
    """Host cores this process may use: affinity mask, capped by the cgroup quota."""
    aff = len(os.sched_getaffinity(0))
    quota = None
    try:
        q, p = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if q != "max":
            quota = max(1, int(int(q) / int(p)))
    except (OSError, ValueError):
        pass
    return {"nproc": os.cpu_count(), "affinity": aff, "cgroup_quota": quota,
            "usable": min(aff, quota) if quota else aff}


def free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def launch_ranks(argv: list[str], n: int) -> int:
    """--gpus N outside torch.distributed.run: one child process per GPU, started
    before this process touches a GPU; rank 0's stdout is the bench line."""
    port = free_port()
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + argv, env=env))
    rc = 0
    for p in procs:
        rc = p.wait() or rc
    return rc


INPUT_KEYS = ("pairs", "se", "ont", "read_len", "x_span")


def input_paths(d: str, gid: int, se: bool) -> list[str]:
    return [os.path.join(d, f"b{gid}_r1.fq")] + ([] if se else [os.path.join(d, f"b{gid}_r2.fq")])


def batch_text(gid: int, args, workers: int):
    """Global batch `gid`'s FASTQ text (seed 1000 + gid): (r1, r2 or None).
    With --inputs, the files --write-inputs made (their shape must match)."""
    if args.inputs:
        with open(os.path.join(args.inputs, "meta.json")) as f:
            meta = json.load(f)
        want = {k: getattr(args, k) for k in INPUT_KEYS}
        if {k: meta.get(k) for k in INPUT_KEYS} != want:
            raise SystemExit(f"--inputs {args.inputs}: written for {meta}, this run asks for {want}")
        texts = []
        for p in input_paths(args.inputs, gid, args.se):
            with open(p, "rb") as f:
                texts.append(f.read())
        return texts[0], (texts[1] if len(texts) > 1 else None)
    import synth
    paired = not args.se
    if args.ont:   # five read lengths, a fifth of the reads each, chunks small enough for the generator's arrays
        parts = [synth.generate(args.pairs // 5, read_len=L, seed=1000 + 10 * gid + k, workers=workers,
                                chunk=1000, x_span=args.x_span)[0]
                 for k, L in enumerate((10_000, 20_000, 30_000, 40_000, 50_000))]
        return b"".join(parts), None
    return synth.generate(args.pairs, read_len=args.read_len, paired=paired, seed=1000 + gid, workers=workers,
                          x_span=args.x_span)


def make_batch(gid: int, args, workers: int, files=None, texts=None):
    """Global batch `gid`, cut and parsed as the reference's reader does.
    Returns the parsed blocks; `files` (paths) get the FASTQ text appended (the
    end-to-end run's input), `texts` (a list) the text itself."""
    import fastqueeze_amd as fq
    t1, t2 = batch_text(gid, args, workers)
    if texts is not None:
        texts.append((t1, t2))
    if files:
        for path, t in zip(files, (t1, t2)):
            if t is not None:
                with open(path, "ab") as f:
                    f.write(t)
    return fq.blocks_from_fastq(t1, t2, args.block_size)


def end_to_end(args, files, contexts, expect: bytes, batch: int, threads: int, devices: int = 1,
               ingest_only: bool = False, keep_arc: bool = False):
    """`seqarc_amd -c` (the streaming reader / parser / encoder / writer
    pipeline) on the FASTQ files on disk: wall time of the whole process, and
    its own clock (device init to the closed .arc).  The archive's blocks must
    be the bench's blocks of the same input, byte for byte.  devices > 1: the
    whole node in one process (batches dealt over devices x contexts);
    ingest_only: the reader and the block cut alone (--dry-run: no device)."""
    from fastqueeze_amd import build
    out = os.path.join(os.path.dirname(files[0]), "e2e")
    cmd = [build.CLI, "-c", "-f", "-v", "-t", str(threads), "-1", files[0]] + (["-2", files[1]] if len(files) > 1 else []) \
        + ["-o", out, "--contexts", str(contexts), "--batch", str(batch), "--slevel", str(args.slevel),
           "--qlevel", str(args.qlevel), "--block-size", str(max(1, args.block_size >> 20))] \
        + (["--devices", str(devices)] if devices > 1 else []) + (["--ingest-only"] if ingest_only else []) \
        + args.e2e_args.split()
    if not ingest_only and args.e2e_settle > 0:
        time.sleep(args.e2e_settle)   # (outside the timed run: a fresh job starts on a settled device)
    t0, m0 = time.perf_counter(), time.monotonic()
    cmdline = " ".join(os.path.basename(c) if i == 0 else c for i, c in enumerate(cmd))
    try:
        r = subprocess.run(cmd, capture_output=True, text=True, timeout=900)
    except subprocess.TimeoutExpired:
        log(f"end-to-end run timed out: {cmdline}")
        return {"value": None, "unit": "MB/s", "error": "timed out after 900 s", "command": cmdline}
    wall, m1 = time.perf_counter() - t0, time.monotonic()
    if r.returncode != 0:   # (recorded, not fatal: the in-HBM line above is the bench's measurement)
        log(f"end-to-end run failed ({r.returncode}): {r.stderr[-2000:]}")
        return {"value": None, "unit": "MB/s", "error": f"exit {r.returncode}: {r.stderr[-500:]}", "command": cmdline}
    if args.e2e_log:
        with open(args.e2e_log, "a") as f:
            f.write(f"== {' '.join(os.path.basename(c) for c in cmd)}\n" + r.stderr)
    in_bytes = sum(os.path.getsize(f) for f in files)
    with open(out + ".arc", "rb") as f:
        arc = f.read()
    same = None if ingest_only else arc[16:16 + len(expect)] == expect   # (a batch's last, short block merges
    #                                                                          with the next batch's text)
    clock, stages, proc = None, None, None
    for ln in r.stderr.splitlines():
        if "MB/s" in ln:
            clock = float(ln.rsplit(",", 1)[1].split()[0])
        if "contexts ready" in ln:
            stages = ln.split(": ", 1)[1]
        if "monotonic clock: main" in ln:   # process start -> main, and exit -> reaped (dynamic loading; the
            mm, me = (float(x.split()[-1]) for x in ln.split(": ", 2)[2].split(", "))   # driver's teardown)
            proc = {"start_to_main_s": round(mm - m0, 3), "exit_to_reaped_s": round(m1 - me, 3)}
    if not keep_arc:
        os.remove(out + ".arc")
    return {"value": round(in_bytes / wall / 1e6, 1), "unit": "MB/s", "wall_s": round(wall, 3),
            "cli_clock_mb_s": clock, "cli_stages": stages, "process": proc, "fastq_bytes": in_bytes, "devices": devices,
            "contexts": contexts, "batch_blocks": batch, "device_settle_s": 0 if ingest_only else args.e2e_settle,
            "parse": "none (--ingest-only)" if ingest_only else "device (sa_stage_text from page-locked text windows)",
            "leading_blocks_identical_to_bench": same,
            "command": " ".join(os.path.basename(c) if i == 0 else c for i, c in enumerate(cmd)),
            **({"archive": out + ".arc", "archive_bytes": len(arc)} if keep_arc else {})}


def md5_files(paths, threads: int) -> list[str]:
    """MD5 of each file (hashlib releases the GIL: one thread per file, 64 MiB reads)."""
    from concurrent.futures import ThreadPoolExecutor

    def one(p):
        h = hashlib.md5()
        with open(p, "rb") as f:
            while True:
                b = f.read(64 << 20)
                if not b:
                    return h.hexdigest()
                h.update(b)
    with ThreadPoolExecutor(max(1, min(threads, len(paths)))) as ex:
        return list(ex.map(one, paths))


def decode_roundtrip(arc: str, inputs: list[str], threads: int) -> dict:
    """f1/f2: `seqarc_amd -d` of an e2e archive (host decoder, -t threads), and
    the decoded FASTQ's MD5 against the input files': the whole archive (every
    block, the block table, the trailer) comes back to the input."""
    from fastqueeze_amd import build
    prefix = os.path.join(os.path.dirname(arc), "rt")
    cmd = [build.CLI, "-d", "-f", "-t", str(threads), arc, prefix]
    t0 = time.perf_counter()
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=900)
    wall = time.perf_counter() - t0
    outs = [prefix + "_1.fastq", prefix + "_2.fastq"] if len(inputs) > 1 else [prefix + ".fastq"]
    try:
        if r.returncode != 0:
            return {"e2e_roundtrip_md5_ok": False, "error": f"exit {r.returncode}: {r.stderr[-500:]}"}
        t1 = time.perf_counter()
        got = md5_files(outs + list(inputs), 2 * len(inputs))
        md5_s = time.perf_counter() - t1
        n = len(inputs)
        in_bytes = sum(os.path.getsize(f) for f in inputs)
        return {"e2e_roundtrip_md5_ok": got[:n] == got[n:], "decoded_md5": got[:n], "input_md5": got[n:],
                "decode_wall_s": round(wall, 3), "decode_mb_s": round(in_bytes / wall / 1e6, 1),
                "decode_threads": threads, "md5_s": round(md5_s, 2), "fastq_bytes": in_bytes,
                "command": " ".join(["seqarc_amd"] + cmd[1:])}
    finally:
        for f in outs:
            if os.path.exists(f):
                os.remove(f)


def pipeline(encs, inputs, cfg, steps: int, warmup: int, local: int, runner=None):
    """The contexts' pipeline over resident inputs: warm (every context every
    input), W untimed steps, then K timed steps between device synchronisations.
    Returns (seconds, Workers)."""
    import torch
    W = Workers(encs, inputs, cfg, runner)
    W.warm_all()
    W.run(warmup, record=False)
    torch.cuda.synchronize(local)
    t0 = time.perf_counter()
    W.run(steps, record=True)
    torch.cuda.synchronize(local)
    return time.perf_counter() - t0, W


def phase_medians(W) -> dict:
    import numpy as np
    return {k: round(float(np.median([p[k] for p in W.phases])), 2) for k in W.phases[0]}


def make_contexts(local: int, n: int, share: bool = True):
    import fastqueeze_amd as fq
    encs = [fq.Encoder(local)]
    for _ in range(n - 1):
        encs.append(fq.Encoder(local, share_with=encs[0] if share else None))
    for e in encs:
        e.set_timing(True)
    return encs


def ont_leg(args, workers: int, local: int) -> dict:
    """configs[4]: ONT-shape SE long reads (10/20/30/40/50 kbp, 0.05 % N), -l
    1.15 R-Block lossy qualities (rblock@0x426c10), one batch resident in HBM,
    the contexts' pipeline as in the headline; first and last block checked
    against the CPU restatement (same -l)."""
    import copy
    import fastqueeze_amd as fq
    import oracle_py
    a = copy.copy(args)
    a.ont, a.se, a.pairs, a.lossy, a.inputs = True, True, args.ont_reads, 1.15, None
    t0 = time.perf_counter()
    blocks = make_batch(0, a, workers)
    gen_s = time.perf_counter() - t0
    tmpl = fq.analyze_ids(blocks[0], True)
    cfg = fq.Config(slevel=args.slevel, qlevel=args.qlevel, bin_mode=int(tmpl[0]), lossy=a.lossy)
    inp = fq.Input(blocks, local)
    encs = make_contexts(local, args.contexts)
    try:
        el, W = pipeline(encs, [inp], cfg, args.leg_steps, 2, local)
        encs[0].run_input(inp, cfg)
        outs = encs[0].fetch()
    finally:
        for e in encs:
            e.close()
        inp.close()
    for i in sorted({0, len(blocks) - 1}):
        b = blocks[i]
        if outs[i] != oracle_py.encode_block(b, cfg.slevel, cfg.qlevel, cfg.md5, cfg.bin_mode, cfg.lossy):
            raise SystemExit(f"ONT leg: block {i} differs from the CPU restatement")
    tb = inp.text_bytes
    return {"metric": "MB/s FASTQ compressed, ONT-shape SE long reads, -l 1.15 (configs[4], 1 MI355X)",
            "value": round(tb * args.leg_steps / el / 1e6, 1), "unit": "MB/s", "steps": args.leg_steps,
            "ms_per_step": round(el / args.leg_steps * 1e3, 2), "fastq_bytes_per_batch": tb, "blocks": len(blocks),
            "reads": a.pairs, "ratio": round(tb / sum(map(len, outs)), 3), "contexts": args.contexts,
            "phase_ms": phase_medians(W), "generate_s": round(gen_s, 1),
            "check": "first and last block bit-identical to oracle/fqz_oracle.c with -l 1.15",
            "data": "synthetic (tests/synth.py, 10/20/30/40/50 kbp SE, seed 1000 + k), inputs resident in HBM"}


def se_leg(args, workers: int, local: int) -> dict:
    """configs[1]: 10 M x 150 bp single-end reads, no reference, one batch
    resident in HBM (~70 blocks of 50 MiB), the contexts' pipeline as in the
    headline, at the default Slevel and at Slevel 8 (k = 15: the 2^30-context
    base model, the README's "16-order" path, compressSeq@0x4248a0 /
    BASE_MODEL ctor@0x42f63e); first and last block of each checked against
    the CPU restatement."""
    import copy
    import fastqueeze_amd as fq
    import oracle_py
    a = copy.copy(args)
    a.se, a.ont, a.pairs, a.inputs = True, False, args.se_reads, None
    t0 = time.perf_counter()
    blocks = make_batch(0, a, workers)
    gen_s = time.perf_counter() - t0
    tmpl = fq.analyze_ids(blocks[0], True)
    inp = fq.Input(blocks, local)
    tb = inp.text_bytes
    out = {"metric": "MB/s FASTQ compressed, 150 bp SE, no-ref (configs[1], 1 MI355X)", "unit": "MB/s",
           "reads": a.pairs, "fastq_bytes_per_batch": tb, "blocks": len(blocks), "contexts": args.contexts,
           "steps": args.leg_steps, "generate_s": round(gen_s, 1),
           "data": "synthetic (tests/synth.py, 150 bp SE, seed 1000), inputs resident in HBM", "slevels": {}}
    try:
        for sl in sorted({args.slevel, 8}):
            cfg = fq.Config(slevel=sl, qlevel=args.qlevel, bin_mode=int(tmpl[0]))
            encs = make_contexts(local, args.contexts)
            try:
                el, W = pipeline(encs, [inp], cfg, args.leg_steps, 2, local)
                encs[0].run_input(inp, cfg)
                outs = encs[0].fetch()
            finally:
                for e in encs:
                    e.close()
            for i in sorted({0, len(blocks) - 1}):
                if outs[i] != oracle_py.encode_block(blocks[i], cfg.slevel, cfg.qlevel, cfg.md5, cfg.bin_mode):
                    raise SystemExit(f"SE leg: Slevel {sl} block {i} differs from the CPU restatement")
            out["slevels"][str(sl)] = {
                "value": round(tb * args.leg_steps / el / 1e6, 1), "ms_per_step": round(el / args.leg_steps * 1e3, 2),
                "order_k": sl + 7 if sl < 9 else 0, "ratio": round(tb / sum(map(len, outs)), 3),
                "phase_ms": phase_medians(W),
                "check": f"first and last block bit-identical to oracle/fqz_oracle.c at Slevel {sl}"}
    finally:
        inp.close()
    out["value"] = out["slevels"][str(args.slevel)]["value"]
    return out


def hash_leg(args, local: int) -> dict:
    """configs[3]: the HASH reference path at GRCh38 size.  A synthetic genome
    of --hash-genome-mb Mb (3 records, N runs, one in lower case) indexed on the
    device (buildRefIndex@0x410190), single reads aligned
    (getHashAlignInfo@0x4113c0), and a batch of --hash-pairs PE pairs (69 x 50 MiB blocks) encoded
    through the aligned path (doAlign + doAlignEncode@0x42d4c0) by the contexts'
    pipeline, each step with its own align_info chain.  Checked by decoding the
    first and last blocks with the host decoder against the genome: the reads
    come back.  (The oracle's index of a 3 Gb genome takes minutes on the host:
    parity at this scale is tests/test_gpu_genome_scale.py's.)"""
    import numpy as np
    import torch
    import fastqueeze_amd as fq
    import synth
    t0 = time.perf_counter()
    glen = int(args.hash_genome_mb * 1e6)
    fa, g = synth.big_reference(glen, 2024)
    gen_s = time.perf_counter() - t0
    encs = make_contexts(local, args.contexts)
    ix = inp = None
    try:
        torch.cuda.synchronize(local)
        t0 = time.perf_counter()
        ix = fq.HashIndex(encs[0], fa)
        torch.cuda.synchronize(local)
        build_s = time.perf_counter() - t0
        fa_bytes = fa.size
        del fa
        # single reads: 150 bp, 0.2 % substitutions, either strand
        rng = np.random.default_rng(77)
        n = args.hash_align_reads
        starts = rng.integers(0, glen - 200, n)
        rv = np.arange(n) % 2 == 1
        raw = synth.draw_reads(rng, g, starts, rv, 150, sub=0.002, random_frac=0.0).reshape(-1)
        off = np.arange(n, dtype=np.uint64) * 150
        lens = np.full(n, 150, np.int32)
        ix.align_arrays(raw, off, lens, 20_000)
        t0 = time.perf_counter()
        ret, rev, pos, _, _ = ix.align_arrays(raw, off, lens, n)
        align_s = time.perf_counter() - t0
        align_kernel_ms = ix.last_kernel_ms
        del raw, off, lens
        good = int(((ret >= 0) & (pos == starts + 1) & (rev == rv)).sum())
        # the aligned encode of a PE batch (69 blocks by default)
        t1, t2 = synth.pe_reads_fast(g, args.hash_pairs, 78)
        del g
        blocks = fq.blocks_from_fastq(t1, t2)
        del t1, t2
        tmpl = fq.analyze_ids(blocks[0], False)
        cfg = fq.Config(slevel=args.slevel, qlevel=args.qlevel, bin_mode=int(tmpl[0]))
        inp = fq.Input(blocks, local)

        def aligned(enc, i, c):
            ch = fq.AlignChain()
            try:
                enc.run_aligned(c, ix, True, ch, inp=i)
            finally:
                ch.close()
        el, W = pipeline(encs, [inp], cfg, args.leg_steps, 2, local, aligned)
        aligned(encs[0], inp, cfg)
        outs = encs[0].fetch()
        encs[0].run_input(inp, cfg)
        noref = sum(map(len, encs[0].fetch()))
        words, bases = ix.packed()
        for i in sorted({0, len(blocks) - 1}):
            b = blocks[i]
            d, ok = fq.decode_block(outs[i], b.text_bytes, cfg, tmpl, ref=(words, bases, True, 7))
            if not (ok and np.array_equal(d.seq, b.seq) and np.array_equal(d.qual, b.qual)
                    and np.array_equal(d.names, b.names)):
                raise SystemExit(f"HASH leg: aligned block {i} does not decode back to its reads")
    finally:
        if ix is not None:
            ix.close()
        if inp is not None:
            inp.close()
        for e in encs:
            e.close()
    tb = sum(b.text_bytes for b in blocks)
    return {"metric": "MB/s FASTQ compressed, HASH reference path, 150 bp PE (configs[3] shape, 1 MI355X)",
            "value": round(tb * args.leg_steps / el / 1e6, 1), "unit": "MB/s", "steps": args.leg_steps,
            "ms_per_step": round(el / args.leg_steps * 1e3, 2), "fastq_bytes_per_batch": tb, "blocks": len(blocks),
            "ratio": round(tb / sum(map(len, outs)), 3), "ratio_noref_same_batch": round(tb / noref, 3),
            "contexts": args.contexts, "phase_ms": phase_medians(W),
            "genome_bases": glen, "fasta_bytes": fa_bytes, "genome_generate_s": round(gen_s, 1),
            "index_build_s": round(build_s, 3),
            "align": {"reads": n, "read_len": 150, "s": round(align_s, 3), "reads_per_s": round(n / align_s, 1),
                      "kernel_ms": round(align_kernel_ms, 3),
                      "kernel_reads_per_s": round(n / max(align_kernel_ms, 1e-6) * 1e3, 1),
                      "aligned_at_true_position": round(good / n, 5)},
            "check": "first and last aligned blocks decode back to their reads (sa_decode_block_ref, genome words)",
            "parity": "GPU == oracle/ restatement (tests/test_gpu_align.py, tests/test_gpu_genome_scale.py); "
                      "unpinned against SeqArc itself",
            "data": "synthetic genome (tests/synth.py big_reference, seed 2024) and reads (pe_reads_fast, seed 78)"}


def write_gz(src: str, dst: str, nbytes: int, kind: str, threads: int):
    """The first nbytes of src as gzip: kind "bgzf" (bgzip's <= 64 KiB members with
    the 'BC' size field, inflated in parallel by the reader) or "gzip" (one member
    per 16 MiB, inflated member after member).  Compressed on host threads (zlib
    releases the GIL)."""
    import struct
    import zlib
    from concurrent.futures import ThreadPoolExecutor

    def bgzf(part: bytes) -> bytes:
        out = bytearray()
        for i in range(0, len(part), 65280):
            chunk = part[i:i + 65280]
            c = zlib.compressobj(1, zlib.DEFLATED, -15)
            cd = c.compress(chunk) + c.flush()
            out += b"\x1f\x8b\x08\x04\x00\x00\x00\x00\x00\xff\x06\x00BC\x02\x00"
            out += struct.pack("<H", 25 + len(cd)) + cd + struct.pack("<II", zlib.crc32(chunk), len(chunk))
        return bytes(out)

    def member(part: bytes) -> bytes:
        c = zlib.compressobj(1, zlib.DEFLATED, 31)
        return c.compress(part) + c.flush()

    with open(src, "rb") as f:
        data = f.read(nbytes)
    step = 16 << 20 if kind == "gzip" else 65280 * 256
    parts = [data[i:i + step] for i in range(0, len(data), step)]
    with ThreadPoolExecutor(max(1, threads)) as ex:
        comp = list(ex.map(bgzf if kind == "bgzf" else member, parts))
    with open(dst, "wb") as f:
        for c in comp:
            f.write(c)
        if kind == "bgzf":
            f.write(bytes.fromhex("1f8b08040000000000ff0600424302001b0003000000000000000000"))


def replicate(files, times: int):
    """Append each file to itself until it holds its content `times` over."""
    for f in files:
        size0 = os.path.getsize(f)
        with open(f, "ab") as dst:
            for _ in range(times - 1):
                with open(f, "rb") as src:
                    left = size0
                    while left > 0:
                        chunk = src.read(min(left, 256 << 20))
                        dst.write(chunk)
                        left -= len(chunk)


def stream_sizes(block: bytes) -> dict:
    """Payload bytes of each encap of one encoded block (doFqzEncode@0x42d2d0 layout)."""
    def vint(i):
        b0 = block[i]
        w = 1
        while w <= 8 and not b0 & (0x80 >> (w - 1)):
            w += 1
        v = b0 & ((0x80 >> (w - 1)) - 1)
        for k in range(1, w):
            v = (v << 8) | block[i + k]
        return v, i + w
    _, i = vint(0)
    size, i = vint(i)
    end = i + size
    out = {}
    while i < end:
        sid, i = vint(i)
        sz, i = vint(i)
        out[STREAM_IDS.get(sid, str(sid))] = sz
        i += sz
    return out


def text_leg(args, encs, texts, cfg, want_digest: bytes, device_value: float) -> dict:
    """The bench's batches handed over as the reader cuts them: each block's
    FASTQ text in page-locked host memory (sa_host_alloc).  A step is one
    context's cycle in seqarc_amd -c without its file reader and writer:
    sa_stage_text (the text DMA'd to HBM and parsed there), sa_run, sa_fetch
    (the encoded blocks back to host memory).  Its MB/s is the PCIe-inclusive
    device rate; batch 0's blocks must equal the resident run's."""
    import numpy as np
    import fastqueeze_amd as fq
    t0 = time.perf_counter()
    bufs, batches = [], []
    for t1, t2 in texts:
        hb = []
        for t in (t1, t2):
            if t is not None:
                b = fq.HostBuffer(len(t))
                b.array[:] = np.frombuffer(t, np.uint8)
                hb.append(b)
        bufs += hb
        a = hb[0].array
        if len(hb) == 1:
            batches.append([(a[s:e], None) for s, e in fq.cut_se(a, args.block_size)])
        else:
            b2 = hb[1].array
            batches.append([(a[s1:e1], b2[s2:e2]) for (s1, e1), (s2, e2) in fq.cut_pe(a, b2, args.block_size)])
    pin_s = time.perf_counter() - t0
    nbytes = [sum(x.size + (0 if y is None else y.size) for x, y in bl) for bl in batches]
    lock = threading.Lock()
    phases, errs, stage_ms = [], [], []

    def one(enc, s, record):
        t = time.perf_counter()
        enc.stage_text(batches[s % len(batches)])
        st = time.perf_counter() - t
        enc.run(cfg)
        outs = enc.fetch()
        if record:
            ph = enc.phase_times()
            with lock:
                phases.append(ph)
                stage_ms.append(st * 1e3)
        return outs

    def drive(nsteps, record, per_enc=None):
        nxt = [0]

        def worker(enc):
            try:
                if per_enc is not None:
                    for s in range(per_enc):
                        one(enc, s, False)
                    return
                while True:
                    with lock:
                        s = nxt[0]
                        if s >= nsteps:
                            return
                        nxt[0] += 1
                    one(enc, s, record)
            except Exception as e:
                errs.append(e)

        th = [threading.Thread(target=worker, args=(e,)) for e in encs]
        for x in th:
            x.start()
        for x in th:
            x.join()
        if errs:
            raise errs[0]

    drive(0, False, per_enc=len(batches))   # every context every batch once: buffers at size
    outs = one(encs[0], 0, False)
    got = hashlib.sha256(b"".join(hashlib.sha256(o).digest() for o in outs)).digest()
    if got != want_digest:
        raise SystemExit("staged-text leg: batch 0 encoded from its text differs from the resident run")
    ts = time.perf_counter()
    drive(args.text_steps, True)
    el = time.perf_counter() - ts
    total = sum(nbytes[s % len(nbytes)] for s in range(args.text_steps))
    for b in bufs:
        b.close()
    med = {k: round(float(np.median([p[k] for p in phases])), 2) for k in phases[0]}
    v = total / el / 1e6
    return {"value": round(v, 1), "unit": "MB/s", "steps": args.text_steps, "ms_per_step": round(el / args.text_steps * 1e3, 2),
            "vs_device_encode": round(v / device_value, 3) if device_value else None,
            "stage_ms_median": round(float(np.median(stage_ms)), 1), "phase_ms": med,
            "pin_and_cut_s": round(pin_s, 1), "contexts": len(encs),
            "check": "batch 0's blocks from sa_stage_text identical to the resident run's",
            "what": "per step: sa_stage_text (FASTQ text in page-locked host memory -> HBM, device parse), "
                    "sa_run, sa_fetch (encoded blocks -> host); no file reader, no .arc writer"}


class Workers:
    """C encoder contexts on one GPU, each driven by its own host thread, taking
    steps (batch encodes) from a shared counter."""

    def __init__(self, encoders, inputs, cfg, runner=None, gap_s: float = 0.0):
        """runner(enc, inp, cfg): one step (default: the no-reference encode);
        gap_s: a pause after each recorded step (diagnostics)."""
        self.encs, self.inputs, self.cfg, self.gap_s = encoders, inputs, cfg, gap_s
        self.step = runner or (lambda enc, inp, c: enc.run_input(inp, c))
        self.phases, self.restarts, self.stats = [], 0, (0, 0)

    def warm_all(self):
        """Every context encodes every batch once (its buffers reach the size of
        the largest batch: no allocation, hence no device-wide hipFree, later)."""
        errs = []

        def worker(enc):
            try:
                for inp in self.inputs:
                    self.step(enc, inp, self.cfg)
            except Exception as e:
                errs.append(e)

        th = [threading.Thread(target=worker, args=(e,)) for e in self.encs]
        for t in th:
            t.start()
        for t in th:
            t.join()
        if errs:
            raise errs[0]

    def run(self, nsteps: int, record: bool):
        lock = threading.Lock()
        nxt = [0]
        errs = []

        def worker(enc):
            try:
                while True:
                    with lock:
                        s = nxt[0]
                        if s >= nsteps:
                            return
                        nxt[0] += 1
                    self.step(enc, self.inputs[s % len(self.inputs)], self.cfg)
                    if record and self.gap_s > 0:
                        time.sleep(self.gap_s)
                    if record:
                        ph = enc.phase_times()
                        with lock:
                            self.phases.append(ph)
                            self.restarts += enc.coder_restarts()
                            self.stats = max(self.stats, enc.stream_stats())
            except Exception as e:   # surfaced after join
                errs.append(e)

        th = [threading.Thread(target=worker, args=(e,)) for e in self.encs]
        for t in th:
            t.start()
        for t in th:
            t.join()
        if errs:
            raise errs[0]

    def verify_shared(self, probe=None):
        """Every batch encoded by the contexts together (sharing the front scratch,
        as in the timed region), outputs fetched per step; then each batch by
        context 0 alone.  Per-batch digests must agree.  probe(s, outs): an extra
        check on a batch's outputs from the shared run.  Returns {batch: context}."""
        lock = threading.Lock()
        nxt = [0]
        errs, shared, who = [], {}, {}

        def worker(k, enc):
            try:
                while True:
                    with lock:
                        s = nxt[0]
                        if s >= len(self.inputs):
                            return
                        nxt[0] += 1
                    enc.run_input(self.inputs[s], self.cfg)
                    outs = enc.fetch()
                    if probe:
                        probe(s, outs)
                    with lock:
                        shared[s] = hashlib.sha256(b"".join(hashlib.sha256(o).digest() for o in outs)).digest()
                        who[s] = k
            except Exception as e:
                errs.append(e)

        th = [threading.Thread(target=worker, args=(k, e)) for k, e in enumerate(self.encs)]
        for t in th:
            t.start()
        for t in th:
            t.join()
        if errs:
            raise errs[0]
        for s, inp in enumerate(self.inputs):
            self.encs[0].run_input(inp, self.cfg)
            outs = self.encs[0].fetch()
            if hashlib.sha256(b"".join(hashlib.sha256(o).digest() for o in outs)).digest() != shared[s]:
                raise SystemExit(f"batch {s}: the shared-front run (context {who[s]}) differs from context 0 alone")
        return who


def main():
    argv = sys.argv[1:]
    args = parse_args(argv)
    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        sys.exit(launch_ranks(argv, args.gpus))

    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        raise SystemExit(f"--gpus {args.gpus} but WORLD_SIZE {world}")
    # streams of several contexts each get a hardware queue: 4 streams per
    # context plus the runtime's own.  The GPU boxes preset 4 per process (HIP's
    # default), under which the contexts' streams share queues:
    # 13.45-13.48 GB/s with 8 / 24 queues against 13.0-13.3 with 4 (round 3 g4b)
    hwq0 = os.environ.get("GPU_MAX_HW_QUEUES")
    os.environ["GPU_MAX_HW_QUEUES"] = os.environ.get("SA_BENCH_HWQ") or str(min(32, 4 * args.contexts + 4))   # (A/B)

    import numpy as np
    import torch
    import torch.distributed as dist
    import fastqueeze_amd as fq
    from fastqueeze_amd.shard import gather_blocks, shard_indices

    if world > 1:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        dist.init_process_group("gloo", rank=rank, world_size=world)

    def barrier():
        if world > 1:
            dist.barrier()

    share = cpu_share()
    workers = args.gen_workers or max(1, min(16, share["usable"] // max(1, int(os.environ.get("LOCAL_WORLD_SIZE",
                                                                                               world)))))
    if args.leg_child:   # (--legs-fresh: one leg in this fresh process, its result as one JSON line)
        legs = {"se_leg": se_leg, "ont_lossy": ont_leg, "hash_path": hash_leg}
        leg = legs[args.leg_child]
        r = hash_leg(args, local) if leg is hash_leg else leg(args, workers, local)
        print(json.dumps(r), flush=True)
        return
    # ---- this rank's batches (global ids dealt round robin) ----
    gids = shard_indices(world * args.batches, rank, world)
    t0 = time.time()
    if args.write_inputs:   # (no GPU call in this mode)
        os.makedirs(args.write_inputs, exist_ok=True)
        for g in gids:
            for p, t in zip(input_paths(args.write_inputs, g, args.se), batch_text(g, args, workers)):
                with open(p, "wb") as f:
                    f.write(t)
            log(f"[rank {rank}] batch {g} written to {args.write_inputs} ({time.time() - t0:.1f}s)")
        with open(os.path.join(args.write_inputs, "meta.json"), "w") as f:
            json.dump({k: getattr(args, k) for k in INPUT_KEYS}, f)
        return
    batches = []
    e2e_files = None
    if args.e2e_batches > 0 and rank == 0:
        d = os.path.join(args.e2e_dir, f"seqarc_bench_{os.getpid()}")
        os.makedirs(d, exist_ok=True)
        e2e_files = [os.path.join(d, "r1.fq")] + ([] if args.se else [os.path.join(d, "r2.fq")])
        import atexit
        import shutil
        atexit.register(shutil.rmtree, d, True)   # /dev/shm is memory: never leave the files behind
        for f in e2e_files:
            open(f, "wb").close()
    texts = [] if args.text_leg and rank == 0 and world == 1 else None
    for k, g in enumerate(gids):
        batches.append(make_batch(g, args, workers, e2e_files if e2e_files and k < args.e2e_batches else None,
                                  texts))
        log(f"[rank {rank}] batch {g}: {len(batches[-1])} blocks, "
            f"{sum(b.text_bytes for b in batches[-1]) / 1e9:.2f} GB ({time.time() - t0:.1f}s)")
    tmpl = fq.analyze_ids(batches[0][0], args.se)
    cfg = fq.Config(slevel=args.slevel, qlevel=args.qlevel, bin_mode=int(tmpl[0]), lossy=args.lossy)
    batch_bytes = [sum(b.text_bytes for b in bl) for bl in batches]

    if args.dry_run:
        import oracle_py
        local_out = []
        for g, bl in zip(gids, batches):
            outs = [oracle_py.encode_block(b, cfg.slevel, cfg.qlevel, cfg.md5, cfg.bin_mode, cfg.lossy) for b in bl]
            local_out.append((g, b"".join(hashlib.sha256(o).digest() for o in outs)))
        allb = gather_blocks(local_out, world * args.batches) if world > 1 else [o for _, o in local_out]
        if rank == 0:
            line = {"dry_run": True, "n_gpus": world, "batches": len(allb),
                    "blocks_digest": hashlib.sha256(b"".join(allb)).hexdigest()}
            if e2e_files:   # the whole-node host path without a device: reader + cut dealt to N x C consumers
                try:
                    replicate(e2e_files, args.e2e_repeat or 2 * world)
                    line["end_to_end"] = end_to_end(args, e2e_files, args.contexts, b"", len(batches[0]), 1,
                                                    devices=world, ingest_only=True)
                finally:
                    shutil.rmtree(os.path.dirname(e2e_files[0]), True)
            print(json.dumps(line), flush=True)
        if world > 1:
            dist.destroy_process_group()
        return

    # ---- resident inputs, encoder contexts ----
    keep = {"verify": batches[0], "cpu": batches[0], "last": batches[-1]}
    inputs = [fq.Input(bl, local) for bl in batches]
    del batches
    encs = [fq.Encoder(local)]
    for _ in range(args.contexts - 1):   # one front scratch per GPU, fronts one at a time
        encs.append(fq.Encoder(local, share_with=None if args.no_share else encs[0]))
    for e in encs:
        e.set_timing(True)
    W = Workers(encs, inputs, cfg, gap_s=args.step_gap_ms / 1e3)
    W.warm_all()
    W.run(args.warmup, record=False)
    barrier()
    torch.cuda.synchronize(local)
    ts = time.perf_counter()
    W.run(args.steps, record=True)
    torch.cuda.synchronize(local)
    barrier()
    elapsed = time.perf_counter() - ts
    step_bytes = sum(inputs[s % len(inputs)].text_bytes for s in range(args.steps))
    if world > 1:
        t = torch.tensor([elapsed, float(step_bytes)], dtype=torch.float64)
        tm = t.clone()
        dist.all_reduce(tm, op=dist.ReduceOp.MAX)
        dist.all_reduce(t, op=dist.ReduceOp.SUM)
        elapsed, total_bytes = float(tm[0]), float(t[1])
    else:
        total_bytes = float(step_bytes)

    # ---- outputs of batch 0: spot-check against the oracle, stream sizes,
    #      checksum of the block checksums over all ranks ----
    encs[0].run_input(inputs[0], cfg)
    outs = encs[0].fetch()
    out_bytes = sum(len(o) for o in outs)
    vb = keep["verify"]
    if not args.no_verify and rank == 0:
        import oracle_py
        for i in sorted({0, len(vb) - 1}):
            b = vb[i]
            if outs[i] != oracle_py.encode_block(b, cfg.slevel, cfg.qlevel, cfg.md5, cfg.bin_mode, cfg.lossy):
                raise SystemExit(f"bench output of block {i} differs from the CPU restatement")
            if not cfg.bin_mode and not cfg.lossy:   # (lossy: the qualities do not come back)
                nm, nl, sq, sl, ql, ok = oracle_py.decode_block(outs[i], b.nreads, b.names.size, b.seq.size,
                                                               cfg.slevel, cfg.qlevel, cfg.md5)
                if not (ok and np.array_equal(sq, b.seq) and np.array_equal(ql, b.qual)
                        and np.array_equal(nm, b.names)):
                    raise SystemExit(f"bench output of block {i} does not decode back to its input")
        log("[rank 0] spot-check: first and last block of batch 0 bit-identical to the oracle, decode back")
    # every batch again with the contexts sharing the front (as timed) against
    # context 0 alone; the last block of the last batch against the oracle
    if not args.no_verify:
        import oracle_py
        lb = keep["last"]

        def probe(s, outs):
            if s == len(inputs) - 1 and outs[-1] != oracle_py.encode_block(lb[-1], cfg.slevel, cfg.qlevel, cfg.md5,
                                                                              cfg.bin_mode, cfg.lossy):
                raise SystemExit(f"bench output of the last block of batch {s} differs from the CPU restatement")
        who = W.verify_shared(probe)
        log(f"[rank {rank}] shared-front outputs of every batch identical to context 0 alone "
            f"(batch -> context {who}); last block of batch {len(inputs) - 1} bit-identical to the oracle")
    del keep["last"]
    digest = hashlib.sha256(b"".join(hashlib.sha256(o).digest() for o in outs)).digest()
    if world > 1:
        digs = gather_blocks([(rank, digest)], world)
    else:
        digs = [digest]
    streams = stream_sizes(outs[0])

    # ---- dominant kernel phase (device time from HIP events on its stream) ----
    ph = {k: float(np.median([p[k] for p in W.phases])) for k in W.phases[0]}
    kern = {k: v for k, v in ph.items() if k != "total"}
    dom = max(kern, key=kern.get)
    in0 = inputs[0].text_bytes
    algo_bytes = in0 + out_bytes          # FASTQ in + encoded out, per launch (one batch)
    achieved = algo_bytes / (kern[dom] / 1e3) / 1e9
    traffic = None
    if args.traffic_json and os.path.exists(args.traffic_json):
        with open(args.traffic_json) as f:
            traffic = json.load(f).get(dom)
    max_syms, all_syms = W.stats
    hbm_per_ctx = [e.device_bytes() for e in encs]
    hbm_front = sorted({e.front_bytes() for e in encs})

    cpu = cpu_mt = None
    if rank == 0 and args.cpu_seconds > 0:
        import oracle_py
        from concurrent.futures import ThreadPoolExecutor
        blocks = keep["cpu"]
        enc1 = lambda b: oracle_py.encode_block(b, cfg.slevel, cfg.qlevel, cfg.md5, cfg.bin_mode, cfg.lossy)  # noqa: E731
        t0 = time.perf_counter()
        nb = nbytes = 0
        for b in blocks:
            enc1(b)
            nb += 1
            nbytes += b.text_bytes
            if time.perf_counter() - t0 > args.cpu_seconds:
                break
        ct = time.perf_counter() - t0
        cpu = {"value": round(nbytes / ct / 1e6, 2), "unit": "MB/s", "cores": 1, "kind": "port",
               "sample": f"{nb} of the bench's 50 MiB PE blocks ({nbytes/1e6:.0f} MB FASTQ) encoded by "
                         f"oracle/fqz_oracle.c (-O2, 1 thread) on this host"}
        # the same restatement on every host core this process may use, one block
        # per thread (the reference's -t N shape; ctypes releases the GIL)
        nt = share["usable"]
        per_core = nb / ct
        count = min(len(blocks), max(nt, int(nt * per_core * args.cpu_seconds)))
        sample = [blocks[i % len(blocks)] for i in range(count)]
        t0 = time.perf_counter()
        with ThreadPoolExecutor(nt) as ex:
            list(ex.map(enc1, sample))
        ct2 = time.perf_counter() - t0
        sb = sum(b.text_bytes for b in sample)
        cpu_mt = {"value": round(sb / ct2 / 1e6, 2), "unit": "MB/s", "cores": nt, "kind": "port",
                  "host": share,
                  "sample": f"{len(sample)} 50 MiB PE blocks ({sb/1e6:.0f} MB FASTQ) encoded by "
                            f"oracle/fqz_oracle.c on {nt} host threads, one block per thread"}

    step_ms = elapsed / args.steps * 1e3
    value = total_bytes / elapsed / 1e6
    res = {
        "metric": "MB/s FASTQ compressed (whole node) + ratio, 150 bp PE, 1/2/4/8 MI355X",
        "value": round(value, 1),
        "unit": "MB/s",
        "value_kind": "device_encode: inputs parsed and resident in HBM before the timed region (FASTQ parse, "
                      "H2D and the .arc write are outside it; end_to_end_short / metric_end_to_end is the "
                      "metric-faithful seqarc_amd -c number)",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(step_ms, 2),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "u8",
        "data": "synthetic (SURVEY.md 8(d) generator, tests/synth.py, seed 1000 + global batch id), "
                "inputs resident in HBM",
        "config": {"workload": (f"synthetic {args.pairs} SE long reads of 10/20/30/40/50 kbp" if args.ont else
                                f"synthetic {args.pairs/1e6:g}M x {args.read_len} bp "
                                f"{'SE reads' if args.se else 'PE mate pairs (interleaved r1,r2)'}")
                               + f" per batch, {args.batches} distinct batches per GPU, no-ref, Slevel {args.slevel} "
                               f"(order-{args.slevel + 7}), Qlevel {args.qlevel}, 50 MiB blocks, MD5 on"
                               + (f", -l {args.lossy} (R-Block lossy qualities)" if args.lossy else ""),
                   "blocks_per_batch": len(keep["verify"]), "fastq_bytes_per_batch": in0,
                   "contexts_per_gpu": args.contexts, "batches_per_gpu": args.batches,
                   "parallelism": f"block-shard x{world} (batches dealt by shard_indices)"},
        "ratio": round(in0 / out_bytes, 3),
        "streams_block0": streams,
        "streams_survey_ref": SURVEY_STREAMS,
        "roofline": {"bound": "hbm", "kernel": dom, "achieved": round(achieved, 2), "peak": HBM_PEAK_GBS,
                     "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 5), "traffic": traffic,
                     "traffic_unit": "bytes per launch (rocprofv3 --pmc, profiles/traffic_latest.json)"},
        "chain_bound": {"kernel": "coder_r", "longest_stream_symbols": max_syms, "all_stream_symbols": all_syms,
                        "salu_per_symbol": R_SALU_PER_SYMBOL, "issued_per_symbol": R_ISSUED_PER_SYMBOL, "bound_ms": round(max_syms * R_NS_PER_SYMBOL / 1e6, 2),
                        "achieved_ms": round(ph.get("coder_r", 0.0), 2),
                        "frac": round(max_syms * R_NS_PER_SYMBOL / 1e6 / max(ph.get("coder_r", 1e-9), 1e-9), 3)},
        "phase_ms": {k: round(v, 2) for k, v in ph.items()},
        "coder_restarts": W.restarts,
        "hw_queues": {"set": int(os.environ["GPU_MAX_HW_QUEUES"]), "preset": hwq0},
        "hbm_bytes_per_context": hbm_per_ctx,
        "hbm_bytes_front_scratch": hbm_front,
        "checksum": hashlib.sha256(b"".join(digs)).hexdigest(),
        "cpu_baseline": cpu,
        "cpu_baseline_threads": cpu_mt,
    }
    for i in inputs:
        i.close()
    if texts:
        t0 = time.perf_counter()
        try:
            res["staged_text"] = text_leg(args, encs, texts, cfg, digest, value)
        except SystemExit:
            raise
        except Exception as e:   # (recorded: the headline line stands on its own)
            log(f"[rank 0] staged-text leg failed: {e!r}")
            res["staged_text"] = {"value": None, "error": repr(e)[:500]}
        res["staged_text"]["leg_wall_s"] = round(time.perf_counter() - t0, 1)
        log(f"[rank 0] staged_text: {res['staged_text'].get('value')} MB/s ({res['staged_text']['leg_wall_s']} s)")
        del texts
    for e in encs:
        e.close()
    # the whole host path: the CLI reads the FASTQ from disk (HBM of every rank's
    # contexts released above).  One rank: its batches, 3 times over.  N ranks:
    # rank 0's first batch 2 N times over through one seqarc_amd --devices N
    # (the whole node in one process, the reference's one reader feeding every
    # encoder); the other ranks wait
    barrier()
    if e2e_files:
        expect = b"".join(outs if args.e2e_batches == 1 else outs[:-1])
        blk = args.e2e_batch or len(keep["verify"])
        try:
            if world == 1 and args.e2e_batches != 1:
                # a short stream at configs[2]'s per-GPU share (143 GB / 8 GPUs ~ 18 GB, five
                # batches: the written batches plus batch 0 once more), where pipeline fill
                # and drain weigh most; the files are cut back to the written batches after it
                base = [os.path.getsize(f) for f in e2e_files]
                sizes = [sum(b.text1 or b.text_bytes for b in keep["verify"])] + \
                    ([sum(b.text2 for b in keep["verify"])] if len(e2e_files) > 1 else [])
                for f, n in zip(e2e_files, sizes):
                    with open(f, "rb") as src, open(f, "ab") as dst:
                        dst.write(src.read(n))
                short = end_to_end(args, e2e_files, args.contexts, expect, blk, share["usable"],
                                   keep_arc=args.decode_check > 0)
                arc = short.pop("archive", None)
                if arc:   # the whole archive back through seqarc_amd -d (f1 / f2), MD5 against the input
                    try:
                        short["roundtrip"] = decode_roundtrip(arc, e2e_files, share["usable"])
                        short["e2e_roundtrip_md5_ok"] = short["roundtrip"]["e2e_roundtrip_md5_ok"]
                    finally:
                        os.remove(arc)
                res["end_to_end_short"] = short
                if args.e2e_gz_blocks > 0:
                    # gzip inputs (the usual .fq.gz) at the short leg's size: BGZF (members
                    # inflated in parallel) and member-serial gzip (one inflate thread per
                    # file), through the inflate-ahead reader; the archive's leading blocks
                    # must be the bench's
                    gz = {}
                    sizes = [os.path.getsize(f) for f in e2e_files]
                    for kind in ("bgzf", "gzip"):
                        gzf = [f + "." + kind + ".gz" for f in e2e_files]
                        t0 = time.perf_counter()
                        for f, g, n in zip(e2e_files, gzf, sizes):
                            write_gz(f, g, n, kind, share["usable"])
                        gzb = sum(os.path.getsize(g) for g in gzf)
                        log(f"[rank 0] {kind} input: {gzb / 1e6:.0f} MB ({time.perf_counter() - t0:.1f}s)")
                        try:
                            r = end_to_end(args, gzf, args.contexts, expect, blk, share["usable"])
                        finally:
                            for g in gzf:
                                os.remove(g)
                        r["fastq_bytes"] = sum(sizes)
                        if r.get("wall_s"):
                            r["value"] = round(sum(sizes) / r["wall_s"] / 1e6, 1)
                        r["gz_bytes"] = gzb
                        if r.get("value") and short.get("value"):
                            r["vs_plain_short"] = round(r["value"] / short["value"], 3)
                        gz[kind] = r
                    res["end_to_end_gz"] = gz
                for f, n in zip(e2e_files, base):
                    os.truncate(f, n)
            replicate(e2e_files, args.e2e_repeat or (3 if world == 1 else 2 * world))
            # batches of the bench's size (69 blocks): pass R of a batch takes as long for 28 blocks as
            # for 69, so smaller batches lose the coder's parallelism
            res["end_to_end"] = end_to_end(args, e2e_files, args.contexts, expect, blk, share["usable"],
                                           devices=world)
            if args.ingest_devices > 0 and world == 1:
                # the whole node's ingest: the reader and the block cut dealt to N devices x C
                # contexts (no device work): the host ceiling an 8-GPU node meets
                ing = end_to_end(args, e2e_files, args.contexts, b"", blk, share["usable"],
                                 devices=args.ingest_devices, ingest_only=True)
                res["ingest_8way"] = ing
                res["ingest_8way_mb_s"] = ing.get("value")
        finally:
            shutil.rmtree(os.path.dirname(e2e_files[0]), True)
    def leg_in_child(name: str) -> dict:
        """One leg in a process of its own (this script, --leg-child NAME, the
        same arguments): a fresh process's contexts, like the headline's."""
        import subprocess
        cmd = [sys.executable, "-u", os.path.abspath(__file__)] + sys.argv[1:] + ["--leg-child", name]
        r = subprocess.run(cmd, capture_output=True, text=True, timeout=1200)
        sys.stderr.write(r.stderr)
        if r.returncode != 0:
            if r.returncode == 1 and "differs from the CPU restatement" in r.stderr:
                raise SystemExit(r.stderr.strip().splitlines()[-1])
            raise RuntimeError(f"leg process exit {r.returncode}: {r.stderr[-400:]}")
        out = r.stdout.strip().splitlines()
        leg_res = json.loads(out[-1])
        leg_res["process"] = "its own (--legs-fresh 1)"
        return leg_res

    if rank == 0 and world == 1:
        for name, leg, on in (("se_leg", se_leg, args.se_leg), ("ont_lossy", ont_leg, args.ont_leg),
                              ("hash_path", hash_leg, args.hash_leg)):
            if not on:
                continue
            t0 = time.perf_counter()
            try:
                if args.legs_fresh:
                    res[name] = leg_in_child(name)
                else:
                    res[name] = hash_leg(args, local) if leg is hash_leg else leg(args, workers, local)
            except SystemExit:
                raise
            except Exception as e:   # (recorded: the headline line stands on its own)
                log(f"[rank 0] {name} leg failed: {e!r}")
                res[name] = {"value": None, "error": repr(e)[:500]}
            res[name]["leg_wall_s"] = round(time.perf_counter() - t0, 1)
            log(f"[rank 0] {name}: {res[name].get('value')} MB/s ({res[name]['leg_wall_s']} s)")
    if "end_to_end_short" in res:   # the metric-faithful number (parse, H2D, .arc write included)
        res["metric_end_to_end"] = {k: res["end_to_end_short"].get(k) for k in ("value", "unit", "wall_s",
                                                                                  "fastq_bytes",
                                                                                  "e2e_roundtrip_md5_ok")}
    barrier()
    if rank == 0:
        print(json.dumps(res), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
