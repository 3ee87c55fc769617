"""In-tree build of the native library (hipcc, gfx950).  No JIT cache: the ``.so`` lives next
to the sources so that it travels with the repository snapshot to the GPU box."""
from __future__ import annotations

import os
import subprocess

PKG = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(PKG)
SRC = os.path.join(PKG, "csrc", "slgpu.hip")
SRCS = [SRC, os.path.join(PKG, "csrc", "png_device.hip"), os.path.join(PKG, "csrc", "png_gray.cpp"),
        os.path.join(PKG, "csrc", "gather.cpp")]
HDR = os.path.join(ROOT, "include", "slgpu.h")
OUT = os.path.join(PKG, "libslgpu.so")

HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
# -amdgpu-sched-strategy=max-ilp: the machine scheduler interleaves main3's independent fp64
# chains and loads more aggressively (243.8 vs 246.1 us per 12-view launch, bit-identical output,
# profiles/r3af); max-memory-clause was 1 % and iterative-minreg 5 % slower (profiles/r3ae)
FLAGS = ["-O3", "--offload-arch=gfx950", "-std=c++17", "-ffp-contract=off", "-mllvm",
         "-amdgpu-sched-strategy=max-ilp", "-fPIC", "-shared"]


def needs_build() -> bool:
    if not os.path.exists(OUT):
        return True
    t = os.path.getmtime(OUT)
    return any(os.path.getmtime(p) > t for p in (*SRCS, HDR, __file__))


def build_native(force: bool = False, verbose: bool = False) -> str:
    """Compile ``csrc/slgpu.hip`` (+ the host PNG fast path) into ``libslgpu.so`` (skipped when
    up to date)."""
    if force or needs_build():
        cmd = [HIPCC, *FLAGS, "-o", OUT + ".tmp", *SRCS, "-lz", "-ldl"]
        if verbose:
            print(" ".join(cmd))
        subprocess.run(cmd, check=True)
        os.replace(OUT + ".tmp", OUT)
        if verbose:
            print(f"built {OUT} for gfx950")
    elif verbose:
        print(f"{OUT} is newer than its sources ({', '.join(os.path.basename(p) for p in SRCS)}): not rebuilt")
    return OUT


if __name__ == "__main__":
    print(build_native(force=True, verbose=True))
