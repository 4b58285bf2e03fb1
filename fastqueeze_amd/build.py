"""Build the gfx950 shared library in-tree (fastqueeze_amd/lib/libseqarc_amd.so)."""
from __future__ import annotations

import os
import shutil
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(HERE, "csrc")
LIB_DIR = os.path.join(HERE, "lib")
LIB = os.path.join(LIB_DIR, "libseqarc_amd.so")
BIN_DIR = os.path.join(HERE, "bin")
CLI = os.path.join(BIN_DIR, "seqarc_amd")
SOURCES = ["sa_engine.hip", "fastq_host.cpp", "arc_file.cpp", "arc_decode.cpp"]
DEPS = SOURCES + ["seqarc_cli.cpp", "sa_kernels.hip", "sa_hash.hip", "sa_parse.hip", "sa_common.h", "sa_device.h", "sa_logic.h", "sa_plan.h",
                  "sa_align_host.h"]


def _hipcc() -> str:
    for cand in (shutil.which("hipcc"), "/opt/rocm/bin/hipcc"):
        if cand and os.path.exists(cand):
            return cand
    raise RuntimeError("hipcc not found: the gfx950 library cannot be built")


def needs_build() -> bool:
    if not os.path.exists(LIB):
        return True
    t = os.path.getmtime(LIB)
    inc = os.path.join(HERE, "..", "include", "seqarc_amd.h")
    if not os.path.exists(CLI):
        return True
    return any(os.path.getmtime(os.path.join(CSRC, f)) > t for f in DEPS) or os.path.getmtime(inc) > t


def build(force: bool = False, verbose: bool = False) -> str:
    if not force and not needs_build():
        return LIB
    os.makedirs(LIB_DIR, exist_ok=True)
    tmp = LIB + ".tmp"
    cmd = [_hipcc(), "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-shared", "-Wall",
           "-o", tmp] + [os.path.join(CSRC, s) for s in SOURCES]
    if verbose:
        print(" ".join(cmd), file=sys.stderr)
    subprocess.run(cmd, check=True)
    os.replace(tmp, LIB)
    # the SeqArc -c command line over the library (seqarc_cli.cpp)
    os.makedirs(BIN_DIR, exist_ok=True)
    cli = [_hipcc(), "-O2", "-std=c++17", "-Wall", "-o", CLI + ".tmp", os.path.join(CSRC, "seqarc_cli.cpp"),
           "-L" + LIB_DIR, "-lseqarc_amd", "-lz", "-Wl,-rpath,$ORIGIN/../lib"]
    if verbose:
        print(" ".join(cli), file=sys.stderr)
    subprocess.run(cli, check=True)
    os.replace(CLI + ".tmp", CLI)
    return LIB


if __name__ == "__main__":
    print(build(force="--force" in sys.argv, verbose=True))
