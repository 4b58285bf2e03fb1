"""Step-by-step run of the reference path on the GPU with timestamps (debug aid:
SA_ALN_TRACE=1 adds the engine's host steps)."""
import os
import sys
import threading
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import fastqueeze_amd as fq  # noqa: E402
import oracle_py as orc  # noqa: E402
import synth  # noqa: E402

T0 = time.time()


def say(m):
    print(f"[{time.time() - T0:7.2f}] {m}", flush=True)


def beat():
    while True:
        time.sleep(20)
        say("...")


threading.Thread(target=beat, daemon=True).start()
paired = len(sys.argv) > 1 and sys.argv[1] == "pe"
fa, g = synth.reference(3_000_000, 21)
say("reference")
orc.hash_index(fa)
say("oracle index")
enc = fq.Encoder(0)
ix = fq.HashIndex(enc, fa)
say("gpu index")
r1, r2 = synth.aligned_reads(g, 12000, 31, paired=paired, random_frac=0.08, far_frac=0.1, short_frac=0.2)
blocks = fq.blocks_from_fastq(r1, r2, block_size=1_000_000)
say(f"{len(blocks)} blocks")
got = enc.encode_aligned(blocks[:1], fq.Config(), ix, paired)
say("gpu encode (1 block)")
want = [orc.encode_block_hash(b, paired, [0, 0]) for b in blocks[:1]]
say(f"oracle; equal {got == want}")
out = os.path.join(ROOT, "gpurun_out", "g3d")
os.makedirs(out, exist_ok=True)
tag = "pe" if paired else "se"
open(os.path.join(out, f"{tag}_got0.bin"), "wb").write(got[0])
open(os.path.join(out, f"{tag}_want0.bin"), "wb").write(want[0])
got = enc.encode_aligned(blocks, fq.Config(), ix, paired)
c = [0, 0]
want = [orc.encode_block_hash(b, paired, c) for b in blocks]
say(f"all blocks equal {got == want}")
ix.close()
enc.close()
