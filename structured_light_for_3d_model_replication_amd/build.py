"""In-tree build of the native library (hipcc, gfx950).  No JIT cache: the ``.so`` lives next
to the sources so that it travels with the repository snapshot to the GPU box.

Provenance: the library embeds ``slgbuild:<digest>`` (``slg_build_id()``), the sha256 of every
source, the header and the compile flags.  :func:`needs_build` rebuilds whenever the digest of the
sources present differs from the one in the library (content, not mtimes), and
``_native.lib()`` refuses a product library whose digest does not match them."""
from __future__ import annotations

import hashlib
import os
import re
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
BUILD_ID_PREFIX = b"slgbuild:"


def source_digest(srcs=None, flags=None) -> str:
    """sha256 (32 hex digits) of the sources (name + bytes), the header and the flags."""
    h = hashlib.sha256()
    for p in (*(srcs or SRCS), HDR):
        h.update(os.path.basename(p).encode() + b"\0")
        with open(p, "rb") as f:
            h.update(f.read())
        h.update(b"\0")
    h.update("\0".join(flags or FLAGS).encode())
    return h.hexdigest()[:32]


def built_digest(path: str = OUT) -> str | None:
    """The digest embedded in a built library (read from the file; nothing is loaded)."""
    try:
        with open(path, "rb") as f:
            data = f.read()
    except OSError:
        return None
    m = re.search(re.escape(BUILD_ID_PREFIX) + rb"([0-9a-f]{32})", data)
    return m.group(1).decode() if m else None


def needs_build() -> bool:
    return built_digest() != source_digest()


def build_native(force: bool = False, verbose: bool = False) -> str:
    """Compile ``csrc/slgpu.hip`` (+ the host PNG fast path) into ``libslgpu.so`` (skipped when
    the embedded digest matches the sources)."""
    if force or needs_build():
        digest = source_digest()
        cmd = [HIPCC, *FLAGS, f'-DSLG_BUILD_ID="{BUILD_ID_PREFIX.decode()}{digest}"', "-o", OUT + ".tmp", *SRCS,
               "-lz", "-ldl"]
        if verbose:
            print(" ".join(cmd))
        subprocess.run(cmd, check=True)
        os.replace(OUT + ".tmp", OUT)
        if verbose:
            print(f"built {OUT} for gfx950 (build id {digest})")
    elif verbose:
        print(f"{OUT} matches its sources (build id {built_digest()}): not rebuilt")
    return OUT


if __name__ == "__main__":
    print(build_native(force=True, verbose=True))
