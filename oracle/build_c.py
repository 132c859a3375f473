"""Build the oracle's C restatements (gcc, host) — TEST INFRASTRUCTURE.

``python -m oracle.build_c`` (also run by ``__graft_entry__.build()``)
compiles ``oracle/c/*.c`` into ``oracle/_build/liboracle_c.so``; tests load it
with ctypes.  Never linked into the product library.
"""
from __future__ import annotations

import os
import subprocess
from pathlib import Path

HERE = Path(__file__).resolve().parent
OUT = HERE / "_build" / "liboracle_c.so"


def build() -> Path:
    srcs = sorted((HERE / "c").glob("*.c"))
    if OUT.exists() and all(OUT.stat().st_mtime >= s.stat().st_mtime for s in srcs):
        return OUT
    OUT.parent.mkdir(exist_ok=True)
    tmp = str(OUT) + f".{os.getpid()}.tmp"
    subprocess.run(["gcc", "-O2", "-fPIC", "-shared", "-ffp-contract=off", *map(str, srcs),
                    "-o", tmp, "-lm"], check=True)
    os.replace(tmp, OUT)
    return OUT


def load():
    import ctypes
    lib = ctypes.CDLL(str(build()))
    lib.d3a_oracle_nstep_return.restype = ctypes.c_float
    lib.d3a_oracle_nstep_return.argtypes = [ctypes.POINTER(ctypes.c_float), ctypes.c_int32,
                                            ctypes.c_int32, ctypes.c_float,
                                            ctypes.POINTER(ctypes.c_int32)]
    lib.d3a_oracle_powf.restype = ctypes.c_float
    lib.d3a_oracle_powf.argtypes = [ctypes.c_float, ctypes.c_int32]
    return lib


if __name__ == "__main__":
    print(build())
