"""ctypes binding of the C-ABI in ``include/d3rlpy_amd.h``.

The library is loaded AFTER ``torch`` so that it binds to the HIP runtime
instance torch already loaded (both carry the soname ``libamdhip64.so.7``);
streams and device pointers handed over from torch are then valid here.

There is no fallback: if the library is missing or a call fails, a
``RuntimeError`` is raised.
"""
from __future__ import annotations

import ctypes as C
import os
from pathlib import Path

import torch  # noqa: F401  (must be loaded first: shares its HIP runtime)

_LIB_PATH = Path(__file__).resolve().parent / "libd3rlpy_amd.so"

c_f32p = C.POINTER(C.c_float)
c_i64p = C.POINTER(C.c_int64)
c_u32p = C.POINTER(C.c_uint32)
c_u8p = C.POINTER(C.c_uint8)
c_i32p = C.POINTER(C.c_int32)
vp = C.c_void_p


class GemmDesc(C.Structure):
    _fields_ = [
        ("A", vp), ("B", vp), ("C", vp), ("bias", vp), ("mask", vp), ("rowsum", vp),
        ("M", C.c_int64), ("N", C.c_int64), ("K", C.c_int64), ("batch", C.c_int64),
        ("sAb", C.c_int64), ("sAm", C.c_int64), ("sAk", C.c_int64),
        ("sBb", C.c_int64), ("sBk", C.c_int64), ("sBn", C.c_int64),
        ("sCb", C.c_int64), ("sCm", C.c_int64), ("sCn", C.c_int64),
        ("sbias_b", C.c_int64),
        ("sMb", C.c_int64), ("sMm", C.c_int64), ("sMn", C.c_int64),
        ("splits", C.c_int64), ("sCs", C.c_int64),
        ("sRb", C.c_int64), ("sRs", C.c_int64),
        ("alpha", C.c_float), ("relu", C.c_int32), ("accumulate", C.c_int32),
        ("variant", C.c_int32),
        ("batch2", C.c_int64), ("sAb2", C.c_int64), ("sBb2", C.c_int64), ("sCb2", C.c_int64),
        ("sbias_b2", C.c_int64), ("sMb2", C.c_int64),
        ("agen", vp), ("wnext", vp),
    ]


class GemmWnext(C.Structure):
    _fields_ = [
        ("x", vp), ("ldx", C.c_int64), ("sxb", C.c_int64), ("n_in", C.c_int64),
        ("dW", vp), ("db", vp),
    ]


class Head1MinDesc(C.Structure):
    _fields_ = [
        ("h", vp), ("shb", C.c_int64), ("ldh", C.c_int64),
        ("w", vp), ("swb", C.c_int64),
        ("b", vp), ("sbb", C.c_int64),
        ("q", vp), ("sqb", C.c_int64),
        ("scale", C.c_float),
        ("g_out", vp), ("sgb", C.c_int64),
        ("dz", vp), ("sdzb", C.c_int64), ("lddz", C.c_int64),
        ("rows", C.c_int64), ("n", C.c_int64),
        ("C", C.c_int32),
    ]


class Head1BwdDesc(C.Structure):
    _fields_ = [
        ("g", vp), ("sgb", C.c_int64),
        ("gscale", vp), ("n_scaled", C.c_int64),
        ("q_min", vp), ("sqb", C.c_int64),
        ("scale", C.c_float),
        ("g_out", vp),
        ("h", vp), ("shb", C.c_int64), ("ldh", C.c_int64),
        ("w", vp), ("swb", C.c_int64),
        ("dz", vp), ("sdzb", C.c_int64), ("lddz", C.c_int64),
        ("dW", vp), ("sWs", C.c_int64),
        ("db", vp), ("sbs", C.c_int64),
        ("rows", C.c_int64), ("n", C.c_int64), ("splits", C.c_int64),
        ("C", C.c_int32),
    ]


class AdamSegment(C.Structure):
    _fields_ = [
        ("param", vp), ("exp_avg", vp), ("exp_avg_sq", vp), ("grad", vp),
        ("numel", C.c_int64), ("n_partials", C.c_int64), ("partial_stride", C.c_int64),
        ("grad_out", vp),
    ]


class AdamDesc(C.Structure):
    _fields_ = [
        ("segs", vp), ("n_seg", C.c_int32), ("n_blocks", C.c_int64),
        ("step", vp), ("step_add", C.c_int32),
        ("lr", C.c_double), ("beta1", C.c_double), ("beta2", C.c_double), ("eps", C.c_double),
        ("grad_scale", C.c_double),
        ("soft", C.c_int32), ("targ_delta", C.c_int64), ("tau", C.c_double),
        ("counters", vp), ("inc_mask", C.c_uint32),
        ("metrics", vp), ("n_metrics", C.c_int32),
        ("ring", vp), ("ring_cap", C.c_int64), ("ring_ctr", vp), ("metric_scale", C.c_float),
        ("blocks", vp),
        ("commit_src", vp), ("commit_dst", vp * 8), ("n_commit", C.c_int32),
        ("commit_step", vp * 2), ("one_elem", C.c_int32),
    ]


class AdamBlock(C.Structure):
    _fields_ = [("seg", AdamSegment), ("first", C.c_int64)]


class X6SplitJob(C.Structure):
    _fields_ = [("src", vp), ("dst", vp), ("rows", C.c_int32), ("k", C.c_int32),
                ("kpad", C.c_int32), ("pad_", C.c_int32)]


X6_SPLIT_MAX_JOBS = 4


class PhiloxJob(C.Structure):
    _fields_ = [("out", vp), ("n_normal", C.c_int64), ("n_uniform", C.c_int64),
                ("lo", C.c_float), ("hi", C.c_float), ("seed", C.c_uint64),
                ("ctr", vp), ("ticket", vp)]


class MlpBwdChainDesc(C.Structure):
    _fields_ = [("dz_top", vp), ("dz_mid", vp), ("dz_bot", vp), ("h_mid", vp), ("h_bot", vp),
                ("Wa", vp), ("Wb", vp), ("sW", C.c_int64), ("ld", C.c_int64), ("sdz", C.c_int64),
                ("ldh", C.c_int64), ("sh", C.c_int64), ("rows", C.c_int64), ("C", C.c_int32)]


class X6SplitDesc(C.Structure):
    _fields_ = [("job", X6SplitJob * X6_SPLIT_MAX_JOBS), ("n_jobs", C.c_int32)]


class CqlSampleDesc(C.Structure):
    _fields_ = [
        ("head", vp), ("obs", vp), ("next_obs", vp), ("act", vp),
        ("eps_temp", vp), ("eps_pi", vp), ("u_rand", vp), ("eps_actor", vp),
        ("x_q", vp), ("x_targ", vp), ("x_actor", vp),
        ("logp_temp", vp), ("logp_is", vp), ("actor_u", vp), ("actor_logp", vp),
        ("B", C.c_int32), ("D", C.c_int32), ("A", C.c_int32), ("N", C.c_int32),
        ("ldx", C.c_int32),
        ("min_logstd", C.c_float), ("max_logstd", C.c_float),
        ("eps_targ", vp), ("logp_targ", vp), ("soft_target", C.c_int32),
        ("noise_base", vp), ("rng_ctr", vp), ("eps_actor_out", vp), ("seed", C.c_uint64),
        ("n_normal", C.c_int64), ("gen_noise", C.c_int32),
        ("head_parts", C.c_int32), ("s_head_part", C.c_int64),
        ("presplit", X6SplitDesc),
    ]


class CqlLossDesc(C.Structure):
    _fields_ = [
        ("q", vp), ("q_targ", vp), ("logp_temp", vp), ("logp_is", vp),
        ("rew", vp), ("term", vp), ("n_steps", vp),
        ("log_temp", vp), ("temp_m", vp), ("temp_v", vp), ("temp_step", vp),
        ("log_alpha", vp), ("alpha_m", vp), ("alpha_v", vp), ("alpha_step", vp),
        ("dq", vp), ("lse", vp), ("metrics", vp), ("scalars", vp),
        ("B", C.c_int32), ("A", C.c_int32), ("N", C.c_int32), ("C", C.c_int32),
        ("R", C.c_int64),
        ("gamma", C.c_float), ("temp_lr", C.c_double), ("alpha_lr", C.c_double),
        ("beta1", C.c_double), ("beta2", C.c_double), ("adam_eps", C.c_double),
        ("alpha_threshold", C.c_float), ("conservative_weight", C.c_float),
        ("update_temp", C.c_int32), ("update_alpha", C.c_int32), ("update_critic", C.c_int32),
        ("dp_phase", C.c_int32), ("scalar_grads", vp), ("grad_scale", C.c_float),
        ("logp_targ", vp), ("soft_target", C.c_int32), ("conservative", C.c_int32),
        ("ticket", vp),
        ("split", C.c_int32), ("td2", vp), ("bc", vp), ("stage", vp),
    ]


class SacActorHeadDesc(C.Structure):
    _fields_ = [
        ("head", vp), ("eps", vp), ("u", vp), ("logp", vp),
        ("dq_da", vp), ("ld_da", C.c_int64), ("da_off", C.c_int64), ("sda_c", C.c_int64),
        ("q", vp), ("sqc", C.c_int64), ("scalars", vp),
        ("dhead", vp), ("metrics", vp),
        ("B", C.c_int32), ("A", C.c_int32), ("C", C.c_int32),
        ("min_logstd", C.c_float), ("max_logstd", C.c_float),
        ("w_head", vp), ("h", vp), ("ldh", C.c_int64), ("dz", vp), ("lddz", C.c_int64),
        ("H", C.c_int32), ("dW_part", vp), ("db_part", vp),
        ("dq_dz", vp), ("lddqz", C.c_int64), ("sdz_c", C.c_int64),
        ("w0", vp), ("ldw0", C.c_int64), ("sw0_c", C.c_int64), ("H0", C.c_int32),
        ("dq_min", C.c_int32), ("dq_scale", C.c_float), ("n_part", C.c_int32),
        ("sq_part", C.c_int64), ("sda_part", C.c_int64),
        ("head_parts", C.c_int32), ("s_head_part", C.c_int64),
    ]


class SacActorQDesc(C.Structure):
    _fields_ = [
        ("x", vp), ("ldx", C.c_int64),
        ("W0", vp), ("b0", vp), ("W1", vp), ("b1", vp), ("wh", vp), ("bh", vp),
        ("q", vp), ("dq_da", vp),
        ("B", C.c_int32), ("C", C.c_int32), ("n_in", C.c_int32), ("A", C.c_int32),
        ("da_off", C.c_int32),
    ]


ACTOR_Q_PARTS = 4  # D3A_ACTOR_Q_PARTS


class GatherDesc(C.Structure):
    _fields_ = [
        ("obs", vp), ("frames", vp), ("act", vp), ("act_i", vp), ("rew", vp),
        ("t_row", vp), ("t_ep_start", vp), ("t_ep_last", vp), ("t_terminal", vp),
        ("n_trans", C.c_int64),
        ("D", C.c_int32), ("A", C.c_int32), ("frame_bytes", C.c_int32),
        ("n_frames", C.c_int32), ("n_steps", C.c_int32),
        ("gamma", C.c_float),
        ("idx", vp), ("idx_out", vp), ("seed", C.c_uint64), ("ctr", vp), ("ticket", vp),
        ("B", C.c_int32),
        ("o_obs", vp), ("o_frames", vp), ("o_act", vp), ("o_act_i", vp),
        ("o_rew", vp), ("o_next_obs", vp), ("o_next_frames", vp),
        ("o_term", vp), ("o_n_steps", vp), ("row_offset", C.c_int64),
        ("t_term_value", vp),
        ("gamma_pow", C.c_float * 64),
        ("ctr_value", C.c_int64),
    ]

    def set_gamma(self, gamma: float, n_steps: int) -> None:
        """gamma and the powf(gamma, i) table of the n-step return."""
        if not 1 <= n_steps <= 64:
            raise ValueError("n_steps must be in [1, 64]")
        self.gamma = gamma
        for i, v in enumerate(gamma_powers(gamma, n_steps)):
            self.gamma_pow[i] = v


_LIBM = None


def gamma_powers(gamma: float, n: int):
    """[powf(gamma, (float)i) for i < n] with the C library's powf — the
    arithmetic the reference's compiled n-step loop performs
    (dataset.pyx:1325 under Cython 0.29: float gamma ** int i -> powf)."""
    global _LIBM
    if _LIBM is None:
        import ctypes.util
        _LIBM = C.CDLL(ctypes.util.find_library("m"))
        _LIBM.powf.restype = C.c_float
        _LIBM.powf.argtypes = [C.c_float, C.c_float]
    return [_LIBM.powf(C.c_float(gamma), C.c_float(float(i))) for i in range(n)]


class Td3PrepDesc(C.Structure):
    _fields_ = [
        ("obs", vp), ("next_obs", vp), ("act", vp), ("mean", vp), ("std", vp),
        ("eps", C.c_float), ("x_q", vp), ("x_targ", vp),
        ("B", C.c_int32), ("D", C.c_int32), ("A", C.c_int32), ("ldx", C.c_int32),
    ]


class Td3TargetDesc(C.Structure):
    _fields_ = [
        ("head", vp), ("noise", vp), ("sigma", C.c_float), ("clip", C.c_float),
        ("x_targ", vp), ("ldx", C.c_int32), ("D", C.c_int32), ("B", C.c_int32),
        ("A", C.c_int32),
    ]


class Td3CriticLossDesc(C.Structure):
    _fields_ = [
        ("q", vp), ("q_targ", vp), ("rew", vp), ("term", vp), ("n_steps", vp),
        ("dq", vp), ("metrics", vp), ("B", C.c_int32), ("C", C.c_int32),
        ("gamma", C.c_float), ("actor_step", C.c_int32),
    ]


class Td3bcActorDesc(C.Structure):
    _fields_ = [
        ("head", vp), ("x_q", vp), ("x_actor", vp), ("pi_act", vp),
        ("q0", vp), ("g", vp), ("scalars", vp),
        ("dq_da", vp), ("ld_da", C.c_int32), ("da_off", C.c_int32),
        ("act", vp), ("dhead", vp), ("metrics", vp),
        ("alpha", C.c_float),
        ("B", C.c_int32), ("D", C.c_int32), ("A", C.c_int32), ("ldx", C.c_int32),
        ("bc", C.c_int32),
    ]


MLP_MAX_HIDDEN = 4


class MlpFwdDesc(C.Structure):
    _fields_ = [
        ("x", vp), ("ldx", C.c_int64), ("sxb", C.c_int64),
        ("n_in", C.c_int32), ("n_hidden", C.c_int32), ("H", C.c_int32), ("n_out", C.c_int32),
        ("W", vp * (MLP_MAX_HIDDEN + 1)), ("b", vp * (MLP_MAX_HIDDEN + 1)),
        ("sW", C.c_int64 * (MLP_MAX_HIDDEN + 1)), ("sb", C.c_int64 * (MLP_MAX_HIDDEN + 1)),
        ("h", vp * MLP_MAX_HIDDEN), ("sh", C.c_int64),
        ("out", vp), ("sout", C.c_int64), ("ldout", C.c_int64),
        ("r0", C.c_int64), ("rows", C.c_int64), ("h_from", C.c_int64),
        ("C", C.c_int32), ("block_rows", C.c_int32),
        ("aux_x", vp), ("aux_ldx", C.c_int64), ("aux_sxb", C.c_int64),
        ("aux_wdelta", C.c_int64), ("aux_out", vp), ("aux_sout", C.c_int64),
        ("aux_rows", C.c_int64),
        ("parts", C.c_int32), ("s_part", C.c_int64),
        ("row_mean", vp), ("s_mean", C.c_int64),
        ("xg_mode", C.c_int32), ("xg_D", C.c_int32), ("xg_rep", C.c_int32), ("xg_E", C.c_int32),
        ("xg_obs", vp), ("xg_a", vp), ("xg_lda", C.c_int64),
        ("xg_base", vp), ("xg_clip", C.c_float), ("xg_scale", C.c_float),
        ("hmask", vp), ("s_hmask", C.c_int64),
        ("hmaskT", vp), ("s_hmaskT", C.c_int64),
        ("xg_a_parts", C.c_int32), ("xg_s_apart", C.c_int64),
        ("xg_xout", vp), ("xg_ldxo", C.c_int64), ("xg_eout", vp),
        ("wp", vp * 2), ("aux_wp", vp * 2),
        ("presplit", X6SplitDesc), ("philox", PhiloxJob),
    ]


MLP_PARTS = 4  # D3A_MLP_PARTS


class MlpBwdDesc(C.Structure):
    _fields_ = [
        ("n_in", C.c_int32), ("n_hidden", C.c_int32), ("H", C.c_int32), ("n_out", C.c_int32),
        ("C", C.c_int32),
        ("W", vp * (MLP_MAX_HIDDEN + 1)), ("sW", C.c_int64 * (MLP_MAX_HIDDEN + 1)),
        ("h", vp * MLP_MAX_HIDDEN), ("sh", C.c_int64), ("ldh", C.c_int64),
        ("g", vp), ("sgb", C.c_int64), ("gscale", vp), ("n_scaled", C.c_int64),
        ("q_min", vp), ("sqb", C.c_int64), ("scale", C.c_float),
        ("g_eff", vp), ("sgeb", C.c_int64),
        ("dhead", vp), ("sdhb", C.c_int64), ("lddh", C.c_int64),
        ("dz", vp * MLP_MAX_HIDDEN), ("sdz", C.c_int64),
        ("dx", vp), ("sdxb", C.c_int64), ("lddx", C.c_int64),
        ("rows", C.c_int64), ("block_rows", C.c_int32),
    ]


class MlpBwdSmallDesc(C.Structure):
    _fields_ = [
        ("x", vp), ("ldx", C.c_int64), ("sxb", C.c_int64),
        ("h1", vp), ("h2", vp), ("sh", C.c_int64),
        ("dout", vp), ("ld_dout", C.c_int64), ("sdout", C.c_int64),
        ("W1", vp), ("W2", vp), ("W3", vp),
        ("sW1", C.c_int64), ("sW2", C.c_int64), ("sW3", C.c_int64),
        ("dW1", vp), ("db1", vp), ("dW2", vp), ("db2", vp), ("dW3", vp), ("db3", vp),
        ("dx", vp),
        ("scratch", vp), ("tickets", vp),
        ("rows", C.c_int32), ("n_in", C.c_int32), ("n_out", C.c_int32), ("C", C.c_int32),
    ]


class Q2BwdDesc(C.Structure):
    _fields_ = [
        ("x", vp), ("ldx", C.c_int64), ("sxb", C.c_int64),
        ("h1", vp), ("h2", vp), ("sh", C.c_int64), ("ldh", C.c_int64),
        ("g", vp), ("sgb", C.c_int64),
        ("gscale", vp), ("n_scaled", C.c_int64),
        ("W2", vp), ("sW2", C.c_int64),
        ("w3", vp), ("sw3", C.c_int64),
        ("dW1", vp), ("db1", vp), ("dW2", vp), ("db2", vp), ("dW3", vp), ("db3", vp),
        ("rows", C.c_int64),
        ("n_in", C.c_int32), ("C", C.c_int32),
        ("dz2", vp), ("sdz", C.c_int64),
        ("block_rows", C.c_int32),
        ("m2", vp), ("sm2", C.c_int64),
        ("m2t", vp), ("sm2t", C.c_int64),
        ("b2", vp), ("sb2", C.c_int64),
        ("row_splits", C.c_int32),
    ]


class BcqRowsDesc(C.Structure):
    _fields_ = [
        ("obs", vp), ("D", C.c_int32), ("rep", C.c_int32),
        ("a", vp), ("E", C.c_int32), ("lda", C.c_int64),
        ("base", vp), ("mode", C.c_int32), ("clip", C.c_float), ("scale", C.c_float),
        ("x", vp), ("ldx", C.c_int64), ("e_out", vp), ("rows", C.c_int64),
        ("a_parts", C.c_int32), ("s_a_part", C.c_int64),
    ]


class BcqVaeDesc(C.Structure):
    _fields_ = [
        ("obs", vp), ("act", vp), ("eps", vp),
        ("head_e", vp), ("std_out", vp), ("x_dec", vp), ("ldx", C.c_int64),
        ("head_d", vp), ("dhead_d", vp),
        ("dx_dec", vp), ("lddx", C.c_int64), ("dhead_e", vp),
        ("scalars", vp), ("metrics", vp),
        ("B", C.c_int32), ("D", C.c_int32), ("A", C.c_int32), ("L", C.c_int32),
        ("beta", C.c_float), ("min_logstd", C.c_float), ("max_logstd", C.c_float),
        ("head_parts", C.c_int32), ("s_e_part", C.c_int64), ("s_d_part", C.c_int64),
        ("kl", vp),
    ]


class BcqTargetDesc(C.Structure):
    _fields_ = [
        ("q", vp), ("target", vp),
        ("B", C.c_int32), ("N", C.c_int32), ("K", C.c_int32), ("C", C.c_int32),
        ("lam", C.c_float), ("means", vp),
    ]


class BcqQrDesc(C.Structure):
    _fields_ = [
        ("q", vp), ("target", vp), ("rew", vp), ("term", vp), ("n_steps", vp),
        ("dq", vp), ("loss_cb", vp),
        ("B", C.c_int32), ("K", C.c_int32), ("C", C.c_int32), ("gamma", C.c_float),
        ("tg_q", vp), ("tg_means", vp), ("tg_N", C.c_int32), ("tg_C", C.c_int32),
        ("tg_lam", C.c_float),
    ]


class BcqActorDesc(C.Structure):
    _fields_ = [
        ("head", vp), ("a_dec", vp), ("dq_da", vp), ("ld_da", C.c_int32),
        ("da_off", C.c_int32), ("dhead", vp), ("q0", vp), ("loss_cb", vp), ("metrics", vp),
        ("B", C.c_int32), ("A", C.c_int32), ("K", C.c_int32), ("C", C.c_int32),
        ("scale", C.c_float), ("head_parts", C.c_int32), ("s_head_part", C.c_int64),
    ]


IQN_MAX_ACTIONS = 18
IQN_MAX_GROUPS = 8


class Im2colDesc(C.Structure):
    _fields_ = [
        ("x_u8", vp), ("x_f32", vp),
        ("B", C.c_int32), ("C", C.c_int32), ("H", C.c_int32), ("W", C.c_int32),
        ("KH", C.c_int32), ("KW", C.c_int32), ("S", C.c_int32), ("OH", C.c_int32),
        ("OW", C.c_int32), ("col", vp), ("ldcol", C.c_int64),
    ]


class Col2imDesc(C.Structure):
    _fields_ = [
        ("dcol", vp), ("ldcol", C.c_int64), ("mask", vp), ("dx", vp),
        ("B", C.c_int32), ("C", C.c_int32), ("H", C.c_int32), ("W", C.c_int32),
        ("KH", C.c_int32), ("KW", C.c_int32), ("S", C.c_int32), ("OH", C.c_int32),
        ("OW", C.c_int32),
    ]


class ConvDesc(C.Structure):
    _fields_ = [
        ("x_u8", vp), ("x_f32", vp), ("weight", vp), ("bias", vp), ("y", vp), ("wpack", vp),
        ("dy", vp), ("dW", vp), ("db", vp),
        ("B", C.c_int32), ("C", C.c_int32), ("H", C.c_int32), ("W", C.c_int32),
        ("KH", C.c_int32), ("KW", C.c_int32), ("S", C.c_int32), ("OH", C.c_int32),
        ("OW", C.c_int32), ("CO", C.c_int32), ("relu", C.c_int32), ("splits", C.c_int32),
        ("wpack_ready", C.c_int32),
    ]


class TransposeDesc(C.Structure):
    _fields_ = [
        ("src", vp), ("dst", vp), ("mask", vp),
        ("B", C.c_int32), ("P", C.c_int32), ("C", C.c_int32), ("to_cp", C.c_int32),
    ]


class IqnPriorDesc(C.Structure):
    _fields_ = [("taus", vp), ("prior", vp), ("rows", C.c_int64), ("E", C.c_int32)]


class IqnHeadDesc(C.Structure):
    _fields_ = [
        ("h", vp * IQN_MAX_GROUPS), ("phi", vp), ("Wf", vp), ("bf", vp), ("q", vp),
        ("rows", C.c_int64), ("group_rows", C.c_int64),
        ("K", C.c_int32), ("F", C.c_int32), ("A", C.c_int32),
    ]


class DqnLossDesc(C.Structure):
    _fields_ = [
        ("q", vp), ("q_next", vp), ("q_targ", vp), ("act", vp), ("rew", vp), ("term", vp),
        ("n_steps", vp), ("dq", vp), ("metrics", vp),
        ("B", C.c_int32), ("A", C.c_int32), ("double_q", C.c_int32),
        ("gamma", C.c_float), ("alpha", C.c_float),
    ]


class IqnLossDesc(C.Structure):
    _fields_ = [
        ("q_loss", vp), ("q_next", vp), ("q_targ", vp),
        ("act", vp), ("rew", vp), ("term", vp), ("n_steps", vp), ("taus_loss", vp),
        ("dq", vp), ("loss_b", vp), ("cons_b", vp), ("metrics", vp),
        ("B", C.c_int32), ("K", C.c_int32), ("A", C.c_int32),
        ("gamma", C.c_float), ("alpha", C.c_float),
    ]


class IqnHeadBwdDesc(C.Structure):
    _fields_ = [
        ("h", vp), ("phi", vp), ("dq", vp), ("Wf", vp),
        ("dphi", vp), ("dh", vp), ("dWf_part", vp), ("dbf_part", vp),
        ("B", C.c_int32), ("K", C.c_int32), ("F", C.c_int32), ("A", C.c_int32),
        ("G", C.c_int32),
    ]


class IqnEmbedHeadDesc(C.Structure):
    _fields_ = [
        ("taus", vp), ("We", vp), ("be", vp), ("h", vp * IQN_MAX_GROUPS),
        ("Wf", vp), ("bf", vp), ("q", vp), ("prior_out", vp), ("phi_out", vp),
        ("rows", C.c_int64), ("group_rows", C.c_int64), ("n_keep", C.c_int64),
        ("K", C.c_int32), ("E", C.c_int32), ("F", C.c_int32), ("A", C.c_int32),
    ]


class IqnHeadBwdFusedDesc(C.Structure):
    _fields_ = [
        ("h", vp), ("phi", vp), ("prior", vp), ("dq", vp), ("Wf", vp),
        ("dh", vp), ("dWf_part", vp), ("dbf_part", vp), ("dWe_part", vp), ("dbe_part", vp),
        ("B", C.c_int32), ("K", C.c_int32), ("F", C.c_int32), ("E", C.c_int32),
        ("A", C.c_int32), ("G", C.c_int32), ("NB", C.c_int32),
        ("taus", vp), ("We", vp), ("be", vp), ("phi_dbg", vp),
    ]


# name -> (restype, argtypes)
_SIGNATURES = {
    "d3a_abi_version": (C.c_int, []),
    "d3a_last_error": (C.c_char_p, []),
    "d3a_device_count": (C.c_int, [C.POINTER(C.c_int)]),
    "d3a_gemm_f32": (C.c_int, [C.POINTER(GemmDesc), vp]),
    "d3a_gemm_f32_pair": (C.c_int, [C.POINTER(GemmDesc), C.POINTER(GemmDesc), vp]),
    "d3a_rowdot_f32": (C.c_int, [vp, C.c_int64, C.c_int64, vp, C.c_int64, vp, C.c_int64, vp,
                                 C.c_int64, C.c_int64, C.c_int64, C.c_int64, vp]),
    "d3a_rowdot2_f32": (C.c_int, [vp, C.c_int64, C.c_int64, vp, C.c_int64, vp, C.c_int64, vp,
                                  C.c_int64, C.c_int64, C.c_int64, C.c_int64, C.c_int32,
                                  C.c_int64,
                                  C.c_int64, C.c_int64, C.c_int64, C.c_int64, vp]),
    "d3a_colreduce_f32": (C.c_int, [vp, C.c_int64, C.c_int64, vp, C.c_int64, vp, C.c_int64,
                                    C.c_int64, C.c_int64, C.c_int64, C.c_int64, C.c_int64, vp]),
    "d3a_outer_mask_f32": (C.c_int, [vp, C.c_int64, vp, C.c_int64, vp, C.c_int64, vp,
                                     C.c_int64, C.c_int64, C.c_int64, C.c_int64, vp]),
    "d3a_adam_f32": (C.c_int, [vp, C.c_int32, C.c_int64, vp, C.c_double, C.c_double,
                               C.c_double, C.c_double, C.c_double, vp]),
    "d3a_adam_step": (C.c_int, [C.POINTER(AdamDesc), vp]),
    "d3a_logsumexp_f32": (C.c_int, [vp, C.c_int64, C.c_int64, C.c_int64, vp, vp]),
    "d3a_logsumexp_bwd_f32": (C.c_int, [vp, C.c_int64, C.c_int64, C.c_int64, vp, vp, vp,
                                        C.c_int64, vp]),
    "d3a_td_mse_f32": (C.c_int, [vp, vp, vp, vp, vp, C.c_int64, C.c_int64, vp, vp, vp]),
    "d3a_td_mse_bwd_f32": (C.c_int, [vp, vp, C.c_int64, C.c_int64, vp, vp]),
    "d3a_quantile_huber_f32": (C.c_int, [vp, C.c_int64, vp, C.c_int64, vp, C.c_int64, C.c_int64,
                                         C.c_int64, C.c_int64, vp, vp]),
    "d3a_quantile_huber_bwd_f32": (C.c_int, [vp, C.c_int64, vp, C.c_int64, vp, C.c_int64,
                                             C.c_int64, C.c_int64, C.c_int64, vp, vp, C.c_int64,
                                             vp]),
    "d3a_squashed_gauss_f32": (C.c_int, [vp, vp, vp, C.c_int64, C.c_int32, C.c_float, C.c_float,
                                         vp, vp, vp]),
    "d3a_squashed_gauss_bwd_f32": (C.c_int, [vp, vp, vp, C.c_int64, C.c_int32, C.c_float,
                                             C.c_float, vp, vp, vp, vp, vp]),
    "d3a_relu_mask_f32": (C.c_int, [vp, vp, C.c_int64, vp, vp]),
    "d3a_grad_reduce_f32": (C.c_int, [vp, C.c_int32, C.c_int64, vp]),
    "d3a_soft_update_f32": (C.c_int, [vp, vp, C.c_int64, C.c_double, vp]),
    "d3a_standardize_f32": (C.c_int, [vp, vp, C.c_int64, C.c_int32, C.c_int64, vp, vp, C.c_float,
                                      vp]),
    "d3a_step_end": (C.c_int, [vp, C.c_int32, vp, C.c_int64, vp, vp, C.c_uint32, vp, vp,
                               C.c_int64, C.c_double, C.c_float, vp]),
    "d3a_philox_fill": (C.c_int, [vp, C.c_int64, C.c_int64, C.c_float, C.c_float, C.c_uint64,
                                  vp, vp, vp]),
    "d3a_head1_bwd": (C.c_int, [C.POINTER(Head1BwdDesc), vp]),
    "d3a_head1_min": (C.c_int, [C.POINTER(Head1MinDesc), vp]),
    "d3a_cql_sample": (C.c_int, [C.POINTER(CqlSampleDesc), vp]),
    "d3a_x6_split": (C.c_int, [C.POINTER(X6SplitDesc), vp]),
    "d3a_cql_loss": (C.c_int, [C.POINTER(CqlLossDesc), vp]),
    "d3a_sac_actor_dq": (C.c_int, [vp, C.c_int64, C.c_int32, C.c_int32, vp, C.c_int64, vp]),
    "d3a_sac_actor_head": (C.c_int, [C.POINTER(SacActorHeadDesc), vp]),
    "d3a_sac_actor_q": (C.c_int, [C.POINTER(SacActorQDesc), vp]),
    "d3a_gather_batch": (C.c_int, [C.POINTER(GatherDesc), vp]),
    "d3a_mlp_fwd": (C.c_int, [C.POINTER(MlpFwdDesc), vp]),
    "d3a_gemm_sbf16": (C.c_int, [C.POINTER(GemmDesc), C.c_int32, vp]),
    "d3a_splitk_epilogue_f32": (C.c_int, [vp, C.c_int32, C.c_int64, vp, vp, C.c_int64, C.c_int64,
                                          C.c_int32, vp]),
    "d3a_im2col": (C.c_int, [C.POINTER(Im2colDesc), vp]),
    "d3a_col2im": (C.c_int, [C.POINTER(Col2imDesc), vp]),
    "d3a_iqn_transpose": (C.c_int, [C.POINTER(TransposeDesc), vp]),
    "d3a_conv_fwd": (C.c_int, [C.POINTER(ConvDesc), vp]),
    "d3a_conv_bwd_w": (C.c_int, [C.POINTER(ConvDesc), vp]),
    "d3a_conv_bwd_w_splits": (C.c_int32, [C.POINTER(ConvDesc)]),
    "d3a_q2_bwd_x6t_splits": (C.c_int32, [C.c_int64, C.c_int32]),
    "d3a_conv_bwd_x": (C.c_int, [C.POINTER(ConvDesc), vp]),
    "d3a_conv_pack_weights": (C.c_int, [C.POINTER(ConvDesc), C.POINTER(C.c_int32), C.c_int32, vp]),
    "d3a_conv_pack_weights_philox": (C.c_int, [C.POINTER(ConvDesc), C.POINTER(C.c_int32), C.c_int32,
                                               C.POINTER(PhiloxJob), vp]),
    "d3a_iqn_prior": (C.c_int, [C.POINTER(IqnPriorDesc), vp]),
    "d3a_iqn_head_fwd": (C.c_int, [C.POINTER(IqnHeadDesc), vp]),
    "d3a_iqn_loss": (C.c_int, [C.POINTER(IqnLossDesc), vp]),
    "d3a_dqn_loss": (C.c_int, [C.POINTER(DqnLossDesc), vp]),
    "d3a_iqn_head_bwd": (C.c_int, [C.POINTER(IqnHeadBwdDesc), vp]),
    "d3a_bcq_rows": (C.c_int, [C.POINTER(BcqRowsDesc), vp]),
    "d3a_bcq_vae_sample": (C.c_int, [C.POINTER(BcqVaeDesc), vp]),
    "d3a_bcq_vae_loss": (C.c_int, [C.POINTER(BcqVaeDesc), vp]),
    "d3a_bcq_vae_enc_grad": (C.c_int, [C.POINTER(BcqVaeDesc), vp]),
    "d3a_bcq_target": (C.c_int, [C.POINTER(BcqTargetDesc), vp]),
    "d3a_bcq_qr_loss": (C.c_int, [C.POINTER(BcqQrDesc), vp]),
    "d3a_bcq_actor_head": (C.c_int, [C.POINTER(BcqActorDesc), vp]),
    "d3a_mlp_bwd": (C.c_int, [C.POINTER(MlpBwdDesc), vp]),
    "d3a_mlp_bwd_small": (C.c_int, [C.POINTER(MlpBwdSmallDesc), vp]),
    "d3a_q2_bwd": (C.c_int, [C.POINTER(Q2BwdDesc), vp]),
    "d3a_q2_bwd_actor_head": (C.c_int, [C.POINTER(Q2BwdDesc), C.POINTER(SacActorHeadDesc), vp]),
    "d3a_q2_fwd_bf16": (C.c_int, [C.POINTER(MlpFwdDesc), vp]),
    "d3a_q2_bwd_bf16": (C.c_int, [C.POINTER(Q2BwdDesc), vp]),
    "d3a_q2_fwd_x6": (C.c_int, [C.POINTER(MlpFwdDesc), vp]),
    "d3a_q2_bwd_x6": (C.c_int, [C.POINTER(Q2BwdDesc), vp]),
    "d3a_q2_bwd_x6_cql": (C.c_int, [C.POINTER(Q2BwdDesc), C.POINTER(CqlLossDesc), vp]),
    "d3a_q2_fwd_x1": (C.c_int, [C.POINTER(MlpFwdDesc), vp]),
    "d3a_iqn_embed_head": (C.c_int, [C.POINTER(IqnEmbedHeadDesc), vp]),
    "d3a_iqn_head_bwd_fused": (C.c_int, [C.POINTER(IqnHeadBwdFusedDesc), vp]),
    "d3a_mlp_fwd_x6": (C.c_int, [C.POINTER(MlpFwdDesc), vp]),
    "d3a_mlp_bwd_chain": (C.c_int, [C.POINTER(MlpBwdChainDesc), vp]),
    "d3a_x6_stamps": (C.c_int, [C.POINTER(C.c_ulonglong), C.c_int]),
    "d3a_bwd_stamps": (C.c_int, [C.POINTER(C.c_ulonglong), C.c_int]),
    "d3a_wide_stamps": (C.c_int, [C.POINTER(C.c_ulonglong), C.c_int]),
    "d3a_wide_wave_stamps": (C.c_int, [C.POINTER(C.c_ulonglong), C.c_int]),
    "d3a_small_bwd_stamps": (C.c_int, [C.POINTER(C.c_ulonglong), C.c_int]),
    "d3a_td3_prep": (C.c_int, [C.POINTER(Td3PrepDesc), vp]),
    "d3a_td3_target": (C.c_int, [C.POINTER(Td3TargetDesc), vp]),
    "d3a_td3_critic_loss": (C.c_int, [C.POINTER(Td3CriticLossDesc), vp]),
    "d3a_td3bc_actor_input": (C.c_int, [C.POINTER(Td3bcActorDesc), vp]),
    "d3a_td3bc_actor_seed": (C.c_int, [C.POINTER(Td3bcActorDesc), vp]),
    "d3a_td3bc_actor_head": (C.c_int, [C.POINTER(Td3bcActorDesc), vp]),
}

EXPORTED = tuple(_SIGNATURES)

_lib = None


def lib() -> C.CDLL:
    """Load (once) and return the native library; raise if it is missing."""
    global _lib
    if _lib is None:
        if not _LIB_PATH.exists():
            raise RuntimeError(
                f"d3rlpy_amd native library not built: {_LIB_PATH} is missing "
                "(run `python -m d3rlpy_amd._build`). There is no CPU fallback."
            )
        mode = getattr(os, "RTLD_GLOBAL", 0) | getattr(os, "RTLD_NOW", 0)
        L = C.CDLL(str(_LIB_PATH), mode=mode)
        for name, (res, args) in _SIGNATURES.items():
            fn = getattr(L, name)
            fn.restype = res
            fn.argtypes = args
        _lib = L
    return _lib


def check(rc: int, what: str) -> None:
    if rc != 0:
        msg = lib().d3a_last_error().decode(errors="replace")
        raise RuntimeError(f"{what} failed ({rc}): {msg}")


def library_path() -> Path:
    return _LIB_PATH
