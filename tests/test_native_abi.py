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


import os

# the uint8 first-layer weight-gradient kernel switched off (A/B runs)
_U8S4_OFF = os.environ.get("D3A_CONV1_U8S4", "1") == "0"

STRUCTS = (("d3a_gemm_desc", "GemmDesc"), ("d3a_gemm_wnext", "GemmWnext"),
           ("d3a_adam_segment", "AdamSegment"), ("d3a_adam_desc", "AdamDesc"),
           ("d3a_head1_bwd_desc", "Head1BwdDesc"), ("d3a_head1_min_desc", "Head1MinDesc"),
           ("d3a_cql_sample_desc", "CqlSampleDesc"), ("d3a_cql_loss_desc", "CqlLossDesc"),
           ("d3a_sac_actor_head_desc", "SacActorHeadDesc"), ("d3a_gather_desc", "GatherDesc"),
           ("d3a_sac_actor_q_desc", "SacActorQDesc"),
           ("d3a_td3_prep_desc", "Td3PrepDesc"), ("d3a_td3_target_desc", "Td3TargetDesc"),
           ("d3a_td3_critic_loss_desc", "Td3CriticLossDesc"),
           ("d3a_td3bc_actor_desc", "Td3bcActorDesc"), ("d3a_mlp_fwd_desc", "MlpFwdDesc"), ("d3a_dqn_loss_desc", "DqnLossDesc"),
           ("d3a_mlp_bwd_desc", "MlpBwdDesc"), ("d3a_q2_bwd_desc", "Q2BwdDesc"),
           ("d3a_bcq_rows_desc", "BcqRowsDesc"),
           ("d3a_bcq_vae_desc", "BcqVaeDesc"), ("d3a_bcq_target_desc", "BcqTargetDesc"),
           ("d3a_bcq_qr_desc", "BcqQrDesc"), ("d3a_bcq_actor_desc", "BcqActorDesc"),
           ("d3a_im2col_desc", "Im2colDesc"), ("d3a_col2im_desc", "Col2imDesc"),
           ("d3a_transpose_desc", "TransposeDesc"), ("d3a_iqn_prior_desc", "IqnPriorDesc"),
           ("d3a_iqn_head_desc", "IqnHeadDesc"), ("d3a_iqn_loss_desc", "IqnLossDesc"),
           ("d3a_iqn_head_bwd_desc", "IqnHeadBwdDesc"), ("d3a_conv_desc", "ConvDesc"),
           ("d3a_iqn_embed_head_desc", "IqnEmbedHeadDesc"),
           ("d3a_iqn_head_bwd_fused_desc", "IqnHeadBwdFusedDesc"),
           ("d3a_mlp_bwd_small_desc", "MlpBwdSmallDesc"),
           ("d3a_x6_split_job", "X6SplitJob"), ("d3a_x6_split_desc", "X6SplitDesc"),
           ("d3a_philox_job", "PhiloxJob"), ("d3a_mlp_bwd_chain_desc", "MlpBwdChainDesc"))


def test_struct_layouts_match_header(tmp_path):
    """Every ctypes descriptor has the C struct's size and field offsets:
    a small C program compiled with gcc against include/d3rlpy_amd.h prints
    sizeof / offsetof, compared field by field with the ctypes layout."""
    import shutil
    import subprocess
    from d3rlpy_amd import _native as N
    cc = shutil.which("gcc") or shutil.which("cc")
    if cc is None:
        pytest.skip("no C compiler")
    lines = ["#include <stdio.h>", "#include <stddef.h>", f'#include "{HEADER}"', "int main(void){"]
    for cname, pyname in STRUCTS:
        cls = getattr(N, pyname)
        lines.append(f'printf("{cname} %zu\\n", sizeof({cname}));')
        for f, _ in cls._fields_:
            lines.append(f'printf("{cname}.{f} %zu\\n", offsetof({cname}, {f}));')
    lines.append("return 0;}")
    src = tmp_path / "layout.c"
    src.write_text("\n".join(lines))
    exe = tmp_path / "layout"
    subprocess.run([cc, str(src), "-o", str(exe)], check=True)
    out = dict(l.rsplit(" ", 1) for l in subprocess.run([str(exe)], capture_output=True,
                                                         text=True, check=True).stdout.split("\n")
               if l)
    for cname, pyname in STRUCTS:
        cls = getattr(N, pyname)
        assert int(out[cname]) == ctypes.sizeof(cls), cname
        for f, _ in cls._fields_:
            assert int(out[f"{cname}.{f}"]) == getattr(cls, f).offset, (cname, f)


def test_round4_entry_points_validate_and_size_without_a_gpu():
    """The round-4 entries check their arguments before any HIP call, and
    d3a_conv_bwd_w_splits is host arithmetic: the split counts K5 sizes its
    conv weight-gradient partials with (uint8 layer on the fp32 kernel: 32;
    fp32 layers: ~512 workgroups of the split-bf16 kernel)."""
    from d3rlpy_amd import _native as N
    lib = N.lib()

    def conv(B, C, H, W, CO, K, S):
        d = N.ConvDesc()
        d.B, d.C, d.H, d.W, d.KH, d.KW, d.S, d.CO = B, C, H, W, K, K, S, CO
        d.OH, d.OW = (H - K) // S + 1, (W - K) // S + 1
        return d

    u8 = conv(512, 4, 84, 84, 32, 8, 4)
    u8.x_u8 = 16
    # (256 splits on the uint8 first-layer kernel; D3A_CONV1_U8S4=0, the A/B
    # switch back to the generic fp32 kernel, keeps its 32)
    assert lib.d3a_conv_bwd_w_splits(ctypes.byref(u8)) == (32 if _U8S4_OFF else 256)
    l2, l3 = conv(512, 32, 20, 20, 64, 4, 2), conv(512, 64, 9, 9, 64, 3, 1)
    l2.x_f32 = l3.x_f32 = 16
    assert lib.d3a_conv_bwd_w_splits(ctypes.byref(l2)) == 32
    assert lib.d3a_conv_bwd_w_splits(ctypes.byref(l3)) == 29
    # input gradient: C must be 32 or 64
    bad = conv(2, 48, 20, 20, 64, 4, 2)
    bad.x_f32, bad.weight, bad.dy, bad.y = 16, 16, 16, 16
    assert lib.d3a_conv_bwd_x(ctypes.byref(bad), None) < 0
    assert b"C must be 32 or 64" in lib.d3a_last_error()
    # the one-launch weight copies: at most 8 layers
    descs = (N.ConvDesc * 9)()
    lays = (ctypes.c_int32 * 9)()
    assert lib.d3a_conv_pack_weights(descs, lays, 9, None) < 0
    # fused actor head + trunk backward: null descriptors
    assert lib.d3a_q2_bwd_actor_head(None, None, None) < 0
    # split-K epilogue: rows of N % 4 == 0 floats
    assert lib.d3a_splitk_epilogue_f32(16, 2, 12, 16, None, 4, 6, 1, None) < 0


def test_dcql_workspace_sizes_the_uint8_conv_like_its_launch():
    """the K5 workspace's partial count for the first (uint8) conv
    is the one d3a_conv_bwd_w uses for it (x_u8 set: the first-layer kernel's
    256 splits), not the split-bf16 count of an fp32 input of that shape."""
    from d3rlpy_amd.algos.discrete_cql_impl import _geometry, conv_wgrad_splits
    geom = _geometry((4, 84, 84))
    assert conv_wgrad_splits(geom, 0, 512) == (32 if _U8S4_OFF else 256)
    assert conv_wgrad_splits(geom, 1, 512) == 32
    assert conv_wgrad_splits(geom, 2, 512) == 29


def test_slice_backward_row_blocks():
    """d3a_q2_bwd_x6t_splits: about 256 workgroups (C P 16), >= 4 sub-blocks
    of 32 rows a row block."""
    from d3rlpy_amd import _native as N
    lib = N.lib()
    assert lib.d3a_q2_bwd_x6t_splits(7936, 2) == 8    # K2 critic backward
    assert lib.d3a_q2_bwd_x6t_splits(7936, 1) == 16
    assert lib.d3a_q2_bwd_x6t_splits(640, 10) == 1
    assert lib.d3a_q2_bwd_x6t_splits(256, 2) == 2
    assert lib.d3a_q2_bwd_x6t_splits(32, 2) == 1
    assert lib.d3a_q2_bwd_x6t_splits(100, 0) < 0


def test_presplit_forward_and_split_validate_without_a_gpu():
    """d3a_q2_fwd_x6 with weight images (wp) needs n_in <= 32 and aligned
    images for both layers; d3a_x6_split needs kpad % 16 == 0 and kpad >= k."""
    from d3rlpy_amd import _native as N
    lib = N.lib()
    d = N.MlpFwdDesc()
    d.n_in, d.n_hidden, d.H, d.n_out, d.C, d.rows, d.ldout = 40, 2, 256, 1, 1, 10, 1
    d.x = d.out = 16
    for l in range(3):
        d.W[l] = d.b[l] = 16
    d.wp[0], d.wp[1] = 16, 16
    assert lib.d3a_q2_fwd_x6(ctypes.byref(d), None) < 0
    assert b"wp needs" in lib.d3a_last_error()
    s = N.X6SplitDesc()
    s.n_jobs = 1
    s.job[0].src, s.job[0].dst, s.job[0].rows, s.job[0].k, s.job[0].kpad = 16, 16, 4, 14, 8
    assert lib.d3a_x6_split(ctypes.byref(s), None) < 0
    assert b"kpad % 16" in lib.d3a_last_error()


def test_wide_forward_validates_without_a_gpu():
    """d3a_mlp_fwd_x6 (round 6): up to three hidden layers; stream images only
    for n_in <= 32 and the three-layer Q-head / two-layer wide-head forms; an
    aux pass needs its inputs and excludes row_mean."""
    from d3rlpy_amd import _native as N
    lib = N.lib()

    def desc(n_hidden, n_in=14, n_out=1):
        d = N.MlpFwdDesc()
        d.n_in, d.n_hidden, d.H, d.n_out, d.C, d.rows, d.ldout = n_in, n_hidden, 256, n_out, 2, 64, n_out
        d.x = d.out = 16
        for l in range(n_hidden + 1):
            d.W[l] = d.b[l] = 16
            d.sW[l], d.sb[l] = 256 * 256, 256
        d.sh = 64 * 256
        return d
    d = desc(4)
    assert lib.d3a_mlp_fwd_x6(ctypes.byref(d), None) < 0
    assert b"256, 256 (, 256)" in lib.d3a_last_error()
    d = desc(3, n_in=40)
    d.wp[0], d.wp[1] = 16, 16
    assert lib.d3a_mlp_fwd_x6(ctypes.byref(d), None) < 0
    assert b"stream images" in lib.d3a_last_error()
    d = desc(2, n_out=1)  # two hidden layers with a one-output head: no image form
    d.wp[0], d.wp[1] = 16, 16
    assert lib.d3a_mlp_fwd_x6(ctypes.byref(d), None) < 0
    assert b"stream images" in lib.d3a_last_error()
    d = desc(3)
    d.aux_rows, d.aux_x, d.aux_out = 8, 16, 16
    mean = (ctypes.c_float * 1)()
    d.row_mean, d.s_mean = ctypes.addressof(mean), 64
    assert lib.d3a_mlp_fwd_x6(ctypes.byref(d), None) < 0
    assert b"aux pass" in lib.d3a_last_error()


def test_adam_thread_counts_mirror_the_kernel_rule():
    """nets._seg_threads is elementwise.hip's seg_threads: 16 lanes an element
    for >= 64 partials, four elements a thread for >= 2^18 elements (a multiple
    of 4), else one; AdamGroup.one_elem says no segment takes four."""
    from d3rlpy_amd.nets import _seg_threads
    assert _seg_threads(128, 33280) == 33280 * 16
    assert _seg_threads(4, 1605632) == 1605632 // 4
    assert _seg_threads(4, (1 << 18) - 4) == (1 << 18) - 4
    assert _seg_threads(1, (1 << 18) + 2) == (1 << 18) + 2
    assert _seg_threads(63, 1 << 20) == (1 << 20) // 4


def test_adam_one_elem_per_table():
    """AdamGroup.one_elem (the partials' table) and one_elem_reduced (the
    one-partial table of the data-parallel path) are decided separately: a
    segment of >= 2^18 elements with >= 64 partials runs 16 lanes an element in
    the first and four elements a thread in the second."""
    import torch
    from d3rlpy_amd.nets import AdamGroup, GradSpace, OptimState, ParamStore
    dev = torch.device("cpu")
    store = ParamStore()
    store.add("w", (1 << 18,))
    store.allocate(dev)
    gs = GradSpace(dev)
    gs.add("w", (1 << 18,), 64)
    opt = AdamGroup(OptimState(store, ["w"], lr=1e-3), gs, keep_grads=True)
    assert opt.one_elem and not opt.one_elem_reduced
