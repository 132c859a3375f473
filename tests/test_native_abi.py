"""The C-ABI library loads and exports every symbol include/d3rlpy_amd.h declares
(CPU: no compute calls; the library cross-compiles for gfx950 here)."""
import ctypes
import re
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parents[1]
HEADER = ROOT / "include" / "d3rlpy_amd.h"


def declared_symbols():
    text = HEADER.read_text()
    return sorted(set(re.findall(r"^\s*(?:int|const char\*)\s+(d3a_\w+)\s*\(", text, re.M)))


def test_header_declares_entry_points():
    syms = declared_symbols()
    assert "d3a_gemm_f32" in syms and "d3a_gather_batch" in syms
    assert len(syms) >= 15


def test_library_exports_every_declared_symbol():
    from d3rlpy_amd import _build, _native
    if not _native.library_path().exists():
        _build.build()
    lib = _native.lib()
    for s in declared_symbols():
        assert hasattr(lib, s), s
    # the Python binding covers every declared symbol too
    assert set(declared_symbols()) <= set(_native.EXPORTED)
    assert lib.d3a_abi_version() == 1


def test_argument_errors_are_reported_without_a_gpu():
    """Argument validation happens before any HIP call: usable on CPU."""
    from d3rlpy_amd import _native as N
    lib = N.lib()
    d = N.GemmDesc()
    rc = lib.d3a_gemm_f32(ctypes.byref(d), None)  # null operands
    assert rc < 0
    assert b"null operand" in lib.d3a_last_error()
    with pytest.raises(RuntimeError, match="null operand"):
        N.check(rc, "d3a_gemm_f32")


def test_struct_layouts_match_header():
    """ctypes structure sizes equal the C sizes compiled into the library's view:
    field count of each typedef struct in the header == ctypes field count."""
    from d3rlpy_amd import _native as N
    text = HEADER.read_text()
    for cname, cls in (("d3a_gemm_desc", N.GemmDesc), ("d3a_adam_segment", N.AdamSegment),
                       ("d3a_cql_sample_desc", N.CqlSampleDesc),
                       ("d3a_cql_loss_desc", N.CqlLossDesc),
                       ("d3a_sac_actor_head_desc", N.SacActorHeadDesc),
                       ("d3a_gather_desc", N.GatherDesc)):
        m = re.search(r"typedef struct %s \{(.*?)\} %s;" % (cname, cname), text, re.S)
        assert m, cname
        body = re.sub(r"/\*.*?\*/", "", m.group(1), flags=re.S)
        n = 0
        for decl in body.split(";"):
            decl = decl.strip()
            if not decl:
                continue
            n += decl.count(",") + 1
        assert n == len(cls._fields_), (cname, n, len(cls._fields_))
