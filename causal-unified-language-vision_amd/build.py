"""Build libcullavo_hip.so (every HIP kernel of the hot path) for gfx950 with hipcc.

The library is built in-tree next to this file so it travels to the GPU box with the repo
snapshot. Object files are cached under ``build/`` and rebuilt when a source or header is newer.
"""
from __future__ import annotations

import concurrent.futures as cf
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(HERE, "csrc")
REPO = os.path.dirname(HERE)
INCLUDE = os.path.join(REPO, "include")
BUILD = os.path.join(HERE, "build")
LIB_NAME = "libcullavo_hip.so"
LIB_PATH = os.path.join(HERE, LIB_NAME)
ARCH = os.environ.get("CULLAVO_ARCH", "gfx950")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")

CFLAGS = [
    f"--offload-arch={ARCH}",
    "-O3",
    "-std=c++17",
    "-fPIC",
    "-Wno-unused-result",
    f"-I{INCLUDE}",
]


def sources() -> list[str]:
    return sorted(os.path.join(CSRC, f) for f in os.listdir(CSRC) if f.endswith(".hip"))


def _headers_mtime() -> float:
    hs = [os.path.join(CSRC, f) for f in os.listdir(CSRC) if f.endswith(".h")]
    hs.append(os.path.join(INCLUDE, "cullavo_capi.h"))
    return max(os.path.getmtime(h) for h in hs)


def _compile(src: str, hdr_mtime: float, verbose: bool) -> str:
    obj = os.path.join(BUILD, os.path.basename(src) + ".o")
    if os.path.exists(obj) and os.path.getmtime(obj) >= max(os.path.getmtime(src), hdr_mtime):
        return obj
    cmd = [HIPCC, *CFLAGS, "-c", src, "-o", obj]
    if verbose:
        print(" ".join(cmd), flush=True)
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"hipcc failed for {src}:\n{r.stdout}\n{r.stderr}")
    return obj


def build(force: bool = False, verbose: bool = False, jobs: int | None = None) -> str:
    """Compile every csrc/*.hip for gfx950 and link libcullavo_hip.so; returns its path."""
    os.makedirs(BUILD, exist_ok=True)
    srcs = sources()
    hdr = _headers_mtime()
    if force:
        for f in os.listdir(BUILD):
            os.remove(os.path.join(BUILD, f))
    jobs = jobs or min(8, len(srcs))
    with cf.ThreadPoolExecutor(jobs) as ex:
        objs = list(ex.map(lambda s: _compile(s, hdr, verbose), srcs))
    newest = max(os.path.getmtime(o) for o in objs)
    if force or not os.path.exists(LIB_PATH) or os.path.getmtime(LIB_PATH) < newest:
        tmp = LIB_PATH + ".tmp"  # linked aside, then renamed: a reader never sees a half-written library
        cmd = [HIPCC, f"--offload-arch={ARCH}", "-shared", "-fPIC", "-o", tmp, *objs]
        if verbose:
            print(" ".join(cmd), flush=True)
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f"link failed:\n{r.stdout}\n{r.stderr}")
        os.replace(tmp, LIB_PATH)
    return LIB_PATH


if __name__ == "__main__":
    print(build(force="--force" in sys.argv, verbose=True))
