"""Build the gfx950 HIP library ``libd3rlpy_amd.so`` in-tree.

``python -m d3rlpy_amd._build`` (or ``__graft_entry__.build()``) compiles every
``csrc/*.hip`` with ``hipcc --offload-arch=gfx950`` and links one shared
object next to this file.  Incremental: an object is rebuilt only when its
source, a header, or the flags changed.
"""
from __future__ import annotations

import hashlib
import os
import shutil
import subprocess
import sys
from concurrent.futures import ThreadPoolExecutor
from pathlib import Path

PKG = Path(__file__).resolve().parent
CSRC = PKG / "csrc"
ROOT = PKG.parent
BUILD = PKG / "_objs"
LIB = PKG / "libd3rlpy_amd.so"
ARCH = os.environ.get("D3A_OFFLOAD_ARCH", "gfx950")
HIPCC = os.environ.get("HIPCC", shutil.which("hipcc") or "/opt/rocm/bin/hipcc")

CFLAGS = [
    f"--offload-arch={ARCH}",
    "-O3",
    "-fPIC",
    "-std=c++17",
    # no implicit a*b+c -> fma: elementwise stages round like the reference's
    # separate torch ops; fused multiply-adds are written as fmaf explicitly
    "-ffp-contract=off",
    "-Wall",
    "-Wno-unused-function",
    f"-I{ROOT / 'include'}",
]


def _headers_digest() -> str:
    h = hashlib.sha256()
    for p in sorted(list(CSRC.glob("*.hpp")) + list((ROOT / "include").glob("*.h"))):
        h.update(p.read_bytes())
    h.update(" ".join(CFLAGS).encode())
    return h.hexdigest()[:16]


def _compile(src: Path, hdr: str) -> Path:
    digest = hashlib.sha256(src.read_bytes() + hdr.encode()).hexdigest()[:16]
    obj = BUILD / f"{src.stem}.{digest}.o"
    if obj.exists():
        return obj
    for old in BUILD.glob(f"{src.stem}.*.o"):
        old.unlink()
    cmd = [HIPCC, *CFLAGS, "-c", str(src), "-o", str(obj) + ".tmp"]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"hipcc failed for {src.name}:\n{r.stdout}\n{r.stderr}")
    os.replace(str(obj) + ".tmp", obj)
    return obj


TORCH_LIB = PKG / "libd3rlpy_amd_torch.so"
TORCH_SRC = CSRC / "torch_ops.cpp"


def build_torch_ops(verbose: bool = False) -> Path:
    """libd3rlpy_amd_torch.so: the TORCH_LIBRARY registration of the C-ABI
    (csrc/torch_ops.cpp), host C++ against the installed torch, linked to
    libd3rlpy_amd.so (found next to it via $ORIGIN)."""
    import torch
    import torch.utils.cpp_extension as ce
    cxx = shutil.which("g++") or "g++"
    abi = int(torch._C._GLIBCXX_USE_CXX11_ABI)
    flags = ["-std=c++17", "-O2", "-fPIC", "-shared", "-D__HIP_PLATFORM_AMD__=1",
             "-DUSE_ROCM=1", f"-D_GLIBCXX_USE_CXX11_ABI={abi}",
             *[f"-I{p}" for p in ce.include_paths()], "-I/opt/rocm/include",
             f"-I{ROOT / 'include'}"]
    libs = [*[f"-L{p}" for p in ce.library_paths()], "-ltorch", "-ltorch_cpu", "-lc10",
            "-lc10_hip", "-ltorch_hip", f"-L{PKG}", "-ld3rlpy_amd", "-Wl,-rpath,$ORIGIN"]
    h = hashlib.sha256(TORCH_SRC.read_bytes() + (ROOT / "include" / "d3rlpy_amd.h").read_bytes()
                       + " ".join(flags + libs + [torch.__version__]).encode()).hexdigest()[:16]
    stamp = BUILD / "torch_ops.stamp"
    if TORCH_LIB.exists() and stamp.exists() and stamp.read_text() == h:
        return TORCH_LIB
    cmd = [cxx, *flags, str(TORCH_SRC), "-o", str(TORCH_LIB) + ".tmp", *libs]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"torch op library build failed:\n{r.stdout}\n{r.stderr}")
    os.replace(str(TORCH_LIB) + ".tmp", TORCH_LIB)
    stamp.write_text(h)
    if verbose:
        print(f"built {TORCH_LIB}")
    return TORCH_LIB


def build(verbose: bool = False) -> Path:
    lib = _build_hip(verbose)
    build_torch_ops(verbose)
    return lib


def _build_hip(verbose: bool = False) -> Path:
    BUILD.mkdir(exist_ok=True)
    hdr = _headers_digest()
    srcs = sorted(CSRC.glob("*.hip"))
    with ThreadPoolExecutor(max_workers=min(8, len(srcs))) as ex:
        objs = list(ex.map(lambda s: _compile(s, hdr), srcs))
    stamp = hashlib.sha256("|".join(o.name for o in objs).encode()).hexdigest()[:16]
    stamp_file = BUILD / "lib.stamp"
    if LIB.exists() and stamp_file.exists() and stamp_file.read_text() == stamp:
        return LIB
    cmd = [HIPCC, f"--offload-arch={ARCH}", "-shared", "-fPIC", *map(str, objs), "-o",
           str(LIB) + ".tmp"]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"link failed:\n{r.stdout}\n{r.stderr}")
    os.replace(str(LIB) + ".tmp", LIB)
    stamp_file.write_text(stamp)
    if verbose:
        print(f"built {LIB}")
    return LIB


if __name__ == "__main__":
    build(verbose=True)
    sys.exit(0)
