"""bench.py -- MB/s of FASTQ compressed by the MI355X SeqArc block encoder.

Workload (BASELINE.json configs[1]): synthetic 10M x 150 bp single-end reads,
no reference, default SeqArc parameters (Slevel 3 -> order-10 base model,
Qlevel 2, 50 MiB blocks, per-block MD5), generated with the SURVEY.md 8(d)
spec.  A step = one pass of the encoder over all blocks of the shard, inputs
resident in HBM (staged once), outputs left in HBM.  Multi-GPU: one process per
GPU, each encodes its own shard of blocks (weak scaling, no data-path
collective); value = all ranks' FASTQ bytes / max-over-ranks time.

Prints one JSON line (rank 0).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))

import numpy as np  # noqa: E402

import torch  # noqa: E402  (torch first: the library then binds to torch's HIP runtime)
import torch.distributed as dist  # noqa: E402

import fastqueeze_amd as fq  # noqa: E402

HBM_PEAK_GBS = 8000.0   # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec
# Dependency-chain bound of pass R: one wave issues at most one
# instruction per 4 cycles and a range-coder step is 10 SALU instructions, so a
# stream of L symbols needs >= L * 40 cycles at 2.4 GHz.
R_SALU_PER_SYMBOL = 10
R_NS_PER_SYMBOL = R_SALU_PER_SYMBOL * 4 / 2.4


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--reads", type=int, default=10_000_000, help="reads per GPU shard")
    ap.add_argument("--read-len", type=int, default=150)
    ap.add_argument("--paired", action="store_true",
                    help="150 bp PE (configs[2] shape): --reads/2 mate pairs, r2 the reverse complement of "
                         "the fragment end; same FASTQ volume per GPU as the SE default")
    ap.add_argument("--block-size", type=int, default=fq.BLOCK_SIZE)
    ap.add_argument("--cpu-seconds", type=float, default=15.0, help="CPU baseline sample budget")
    ap.add_argument("--no-verify", action="store_true")
    ap.add_argument("--traffic-json", default=os.path.join(ROOT, "profiles", "traffic_latest.json"),
                    help="per-launch HBM bytes per kernel from the two rocprofv3 --pmc passes "
                         "(FETCH_SIZE x2 + WRITE_SIZE; scripts/gpu_r2.sh + scripts/pmc_traffic.py) of this "
                         "tree's default bench, committed under profiles/")
    args = ap.parse_args()

    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        dist.init_process_group("gloo", rank=rank, world_size=world)

    def barrier():
        if world > 1:
            dist.barrier()

    def device_sync():
        torch.cuda.synchronize(local)

    t0 = time.time()
    n_gen = args.reads // 2 if args.paired else args.reads
    text, text2 = __import__("synth").generate(n_gen, read_len=args.read_len, paired=args.paired,
                                               seed=1000 + rank,
                                               progress=lambda k: log(f"[rank {rank}] generated {k} records"))
    t_gen = time.time() - t0
    t0 = time.time()
    blocks = fq.blocks_from_fastq(text, text2, args.block_size)
    t_parse = time.time() - t0
    in_bytes = sum(b.text_bytes for b in blocks)
    gen_bytes = len(text) + (len(text2) if text2 is not None else 0)
    del text, text2
    tmpl = fq.analyze_ids(blocks[0], not args.paired)
    cfg = fq.Config(bin_mode=int(tmpl[0]))
    log(f"[rank {rank}] generated {gen_bytes/1e9:.2f} GB in {t_gen:.1f}s, {len(blocks)} blocks parsed in "
        f"{t_parse:.1f}s, bin_mode={cfg.bin_mode}")

    enc = fq.Encoder(local)
    enc.set_timing(True)
    enc.stage(blocks)
    for _ in range(args.warmup):
        enc.run(cfg)
    barrier()
    device_sync()
    ts = time.perf_counter()
    phases = []
    for _ in range(args.steps):
        enc.run(cfg)
        phases.append(enc.phase_times())
    device_sync()
    barrier()
    elapsed = time.perf_counter() - ts
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
        tot_in = torch.tensor([float(in_bytes)], dtype=torch.float64)
        dist.all_reduce(tot_in, op=dist.ReduceOp.SUM)
        total_in = float(tot_in.item())
    else:
        total_in = float(in_bytes)

    max_syms, all_syms = enc.stream_stats()
    outs = enc.fetch()
    out_bytes = sum(len(o) for o in outs)
    if not args.no_verify and rank == 0:
        import oracle_py
        for i in sorted({0, len(blocks) - 1}):
            b = blocks[i]
            if outs[i] != oracle_py.encode_block(b, cfg.slevel, cfg.qlevel, cfg.md5, cfg.bin_mode):
                raise SystemExit(f"bench output of block {i} differs from the CPU restatement")
            if not cfg.bin_mode:   # round trip: decode (CPU) back to the block, MD5s verified
                nm, nl, sq, sl, ql, ok = oracle_py.decode_block(outs[i], b.nreads, b.names.size, b.seq.size,
                                                               cfg.slevel, cfg.qlevel, cfg.md5)
                if not (ok and np.array_equal(sq, b.seq) and np.array_equal(ql, b.qual)
                        and np.array_equal(nm, b.names)):
                    raise SystemExit(f"bench output of block {i} does not decode back to its input")
        log("[rank 0] spot-check: first and last block bit-identical to the oracle and decode back to the input")

    # dominant kernel phase (device time from HIP events on its own stream)
    ph = {k: float(np.median([p[k] for p in phases])) for k in phases[0]}
    kern = {k: v for k, v in ph.items() if k != "total"}
    dom = max(kern, key=kern.get)
    algo_bytes = in_bytes + out_bytes           # FASTQ in + encoded out
    achieved = algo_bytes / (kern[dom] / 1e3) / 1e9
    traffic = None
    if args.traffic_json and os.path.exists(args.traffic_json):
        with open(args.traffic_json) as f:
            traffic = json.load(f).get(dom)

    cpu = cpu_mt = None
    if rank == 0 and world == 1 and args.cpu_seconds > 0:
        import oracle_py
        t0 = time.perf_counter()
        nb, nbytes = 0, 0
        for b in blocks:
            oracle_py.encode_block(b, cfg.slevel, cfg.qlevel, cfg.md5, cfg.bin_mode)
            nb += 1
            nbytes += b.text_bytes
            if time.perf_counter() - t0 > args.cpu_seconds:
                break
        ct = time.perf_counter() - t0
        cpu = {"value": round(nbytes / ct / 1e6, 2), "unit": "MB/s", "cores": 1, "kind": "port",
               "sample": f"{nb} of the bench's 50 MiB blocks ({nbytes/1e6:.0f} MB FASTQ) encoded by "
                         f"oracle/fqz_oracle.c (-O2, 1 thread) on this host"}
        # the same restatement on the host cores this process may use, one block
        # per thread (the reference's -t N shape: independent blocks per thread;
        # ctypes releases the GIL during the C call)
        from concurrent.futures import ThreadPoolExecutor
        nt = max(1, min(16, len(os.sched_getaffinity(0))))
        sample = blocks[: min(len(blocks), max(nt, int(nt * (nb / ct) * args.cpu_seconds / 2)))]   # ~half the budget
        t0 = time.perf_counter()
        with ThreadPoolExecutor(nt) as ex:
            list(ex.map(lambda b: oracle_py.encode_block(b, cfg.slevel, cfg.qlevel, cfg.md5, cfg.bin_mode), sample))
        ct2 = time.perf_counter() - t0
        sb = sum(b.text_bytes for b in sample)
        cpu_mt = {"value": round(sb / ct2 / 1e6, 2), "unit": "MB/s", "cores": nt, "kind": "port",
                  "sample": f"{len(sample)} of the bench's 50 MiB blocks ({sb/1e6:.0f} MB FASTQ) encoded by "
                            f"oracle/fqz_oracle.c on {nt} host threads, one block per thread"}

    step_ms = elapsed / args.steps * 1e3
    value = total_in * args.steps / elapsed / 1e6
    res = {
        "metric": "MB/s FASTQ compressed (whole node) + ratio, 150 bp PE, 1/2/4/8 MI355X",
        "value": round(value, 1),
        "unit": "MB/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(step_ms, 2),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "u8",
        "data": "synthetic (SURVEY.md 8(d) generator, seed 1000+rank), inputs resident in HBM",
        "config": {"workload": f"synthetic {args.reads/1e6:g}M x {args.read_len} bp "
                               f"{'PE (interleaved mate pairs)' if args.paired else 'SE'} per GPU, no-ref, "
                               f"Slevel 3 (order-10), Qlevel 2, 50 MiB blocks, MD5 on",
                   "blocks_per_gpu": len(blocks), "fastq_bytes_per_gpu": in_bytes,
                   "parallelism": f"block-shard x{world}"},
        "ratio": round(in_bytes / out_bytes, 3),
        "roofline": {"bound": "hbm", "kernel": dom, "achieved": round(achieved, 2), "peak": HBM_PEAK_GBS,
                     "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 5), "traffic": traffic,
                     "traffic_unit": "bytes per launch (rocprofv3 --pmc, profiles/traffic_latest.json)"},
        "chain_bound": {"kernel": "coder_r", "longest_stream_symbols": max_syms, "all_stream_symbols": all_syms,
                        "salu_per_symbol": R_SALU_PER_SYMBOL, "bound_ms": round(max_syms * R_NS_PER_SYMBOL / 1e6, 2),
                        "achieved_ms": round(ph.get("coder_r", 0.0), 2),
                        "frac": round(max_syms * R_NS_PER_SYMBOL / 1e6 / max(ph.get("coder_r", 1e-9), 1e-9), 3)},
        "phase_ms": {k: round(v, 2) for k, v in ph.items()},
        "cpu_baseline": cpu,
        "cpu_baseline_threads": cpu_mt,
    }
    if rank == 0:
        print(json.dumps(res), flush=True)
    enc.close()
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
