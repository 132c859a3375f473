"""DiscreteCQLImpl on HIP kernels on pixels — drop-in for
d3rlpy/algos/torch/cql_impl.py:246-302 (DiscreteCQLImpl) and what it inherits
(DoubleDQNImpl / DQNImpl, algos/torch/dqn_impl.py:27-171; the DQN and
DoubleDQN Impls of algos/dqn.py are this class with alpha = 0): Nature-DQN
PixelEncoder, n_critics 1, pixel scaler, and either the K5 configuration's
DiscreteIQNQFunction (n_quantiles 64, embed 64) or the reference's default
DiscreteMeanQFunction (a linear head, Huber TD loss in d3a_dqn_loss).

One ``update`` (dqn_impl.py:97-111) on the device:
  1  Philox taus for the five IQN evaluations of the step
     (next-online argmax, next-target, loss, logsumexp, data values)
  2  online encoder over [obs; next_obs] (2B samples), target encoder over
     next_obs: implicit-GEMM convs (uint8 -> /255 fused into the loads, no
     im2col matrix), NHWC -> NCHW flatten, fc
  3  IQN head: cos prior, embed GEMM + ReLU, (h * phi) . W_fc per row —
     online rows [loss | lse | data | next] in one pass, target rows in another
  4  d3a_iqn_loss: Double-DQN target, per-sample-tau quantile Huber loss,
     conservative logsumexp term, dL/dq
  5  head backward (d3a_iqn_head_bwd), embed weight gradient, encoder backward
     (fc; per conv an implicit-GEMM weight gradient; conv3 / conv2 input
     gradients via GEMM + col2im), Adam
  6  d3a_step_end: metrics ring, step counter, and on target-update steps the
     hard sync (tau = 1 copy, dqn_impl.py:146-149)
Encoder forwards on identical (params, input) are evaluated once: the three
online evaluations of obs share one encoder pass and its one backward.
"""
from __future__ import annotations

import ctypes as C
import contextlib
import os
from typing import Dict, List, Optional, Sequence, Tuple

import numpy as np
import torch
from torch import nn

from .. import _native as NAT
from .. import checkpoint as ckpt
from .. import mlp, ops
from ..nets import AdamGroup, GradSpace, OptimState, ParamStore
from .impl_base import DeviceBatch, ImplBase, as_device_batch

METRIC_NAMES = ("loss", "td_loss", "conservative_loss")
FILTERS = ((32, 8, 4), (64, 4, 2), (64, 3, 1))


def _geometry(obs_shape: Sequence[int]) -> List[Tuple[int, int, int, int, int, int, int]]:
    """Per conv: (C_in, H, W, C_out, K, S, OH) with square inputs/kernels."""
    c, h, w = obs_shape
    out = []
    for co, k, s in FILTERS:
        oh, ow = (h - k) // s + 1, (w - k) // s + 1
        out.append((c, h, w, co, k, s, oh, ow))
        c, h, w = co, oh, ow
    return out


class DiscreteCQLImpl(ImplBase):
    # DoubleDQN target (online argmax, dqn_impl.py:162-171); DQNImpl clears it
    _DOUBLE = True

    def __init__(
        self,
        observation_shape: Sequence[int],
        action_size: int,
        learning_rate: float,
        optim_factory,
        encoder_factory,
        q_func_factory,
        gamma: float,
        n_critics: int,
        alpha: float,
        use_gpu,
        scaler,
        reward_scaler,
    ):
        super().__init__(observation_shape, action_size, scaler, None, reward_scaler, use_gpu)
        self._q_type = q_func_factory.get_type()
        if self._q_type not in ("iqn", "mean"):
            raise NotImplementedError("the discrete HIP Impls implement the mean and IQN "
                                      "Q-functions")
        if self._q_type == "iqn" and not self._DOUBLE:
            raise NotImplementedError("DQN (target-network argmax) with the IQN Q-function is "
                                      "not implemented; DoubleDQN / DiscreteCQL are")
        if len(observation_shape) != 3:
            raise NotImplementedError("DiscreteCQL on HIP supports pixel observations")
        if scaler is None or scaler.get_type() != "pixel":
            raise NotImplementedError("DiscreteCQL on HIP expects the pixel scaler")
        if n_critics != 1 or reward_scaler is not None:
            raise NotImplementedError("n_critics = 1 and no reward scaler (K5)")
        if self._q_type == "iqn" and action_size > NAT.IQN_MAX_ACTIONS:
            raise NotImplementedError(f"at most {NAT.IQN_MAX_ACTIONS} actions")
        if getattr(encoder_factory, "TYPE", "pixel") != "pixel" or \
                [list(f) for f in encoder_factory.filters] != [list(f) for f in FILTERS] or \
                getattr(encoder_factory, "_use_batch_norm", False) or \
                getattr(encoder_factory, "_dropout_rate", None) is not None:
            raise NotImplementedError("the Nature-DQN PixelEncoder without batch norm / "
                                      "dropout (K5) is implemented")
        self._learning_rate = learning_rate
        self._optim_factory = optim_factory
        self._encoder_factory = encoder_factory
        self._q_func_factory = q_func_factory
        self._gamma = gamma
        self._n_critics = n_critics
        self._alpha = alpha
        iqn = self._q_type == "iqn"
        self._K = q_func_factory.n_quantiles if iqn else 1
        self._K_greedy = q_func_factory.n_greedy_quantiles if iqn else 1
        self._E = q_func_factory.embed_size if iqn else 0
        self._F = encoder_factory.feature_size
        self._ws: Dict[int, "_Workspace"] = {}

    # ------------------------------------------------------------------ build
    def build(self) -> None:
        dev = self.torch_device
        A, F, E = self._action_size, self._F, self._E
        self.geom = _geometry(self._observation_shape)
        st = ParamStore()
        self.conv_names = []
        for l, (ci, h, w, co, k, s, oh, ow) in enumerate(self.geom):
            st.add(f"enc.c{l}.W", (1, co, ci, k, k))
            st.add(f"enc.c{l}.b", (1, co))
            self.conv_names.append((f"enc.c{l}.W", f"enc.c{l}.b"))
        ci, h, w, co, k, s, oh, ow = self.geom[-1]
        self.flat = co * oh * ow
        st.add("enc.fc.W", (1, F, self.flat))
        st.add("enc.fc.b", (1, F))
        st.add("q.fc.W", (1, A, F))
        st.add("q.fc.b", (1, A))
        if self._q_type == "iqn":
            st.add("q.embed.W", (1, F, E))
            st.add("q.embed.b", (1, F))
        st.allocate(dev)
        self.store = st
        self._init_like_reference()
        self.targ = st.like()
        self.targ.data.copy_(st.data)
        self.counters = torch.zeros(8, dtype=torch.int64, device=dev)
        f = self._optim_factory
        self.names = list(st.specs)
        self.optim_state = OptimState(st, self.names, self._learning_rate, f.betas, f.eps,
                                      step=self.counters[0:1])

    def _init_like_reference(self) -> None:
        """nn.Conv2d / nn.Linear default init in the reference construction order
        (PixelEncoder convs, its fc, then the IQN _fc and _embed)."""
        st = self.store
        with torch.no_grad():
            for l, (ci, h, w, co, k, s, oh, ow) in enumerate(self.geom):
                conv = nn.Conv2d(ci, co, kernel_size=k, stride=s)
                st.view(f"enc.c{l}.W")[0].copy_(conv.weight)
                st.view(f"enc.c{l}.b")[0].copy_(conv.bias)
            layers = [("enc.fc", (self._F, self.flat)), ("q.fc", (self._action_size, self._F))]
            if self._q_type == "iqn":
                layers.append(("q.embed", (self._F, self._E)))
            for name, (o, i) in layers:
                lin = nn.Linear(i, o)
                st.view(f"{name}.W")[0].copy_(lin.weight)
                st.view(f"{name}.b")[0].copy_(lin.bias)

    # ---------------------------------------------------------- checkpoints
    def _refs(self):
        """EnsembleDiscreteQFunction(DiscreteIQN / DiscreteMeanQFunction).parameters() order."""
        p = "_q_funcs.0."
        refs = []
        for l in range(len(self.geom)):
            refs += [(f"{p}_encoder._convs.{l}.weight", f"enc.c{l}.W", 0, None),
                     (f"{p}_encoder._convs.{l}.bias", f"enc.c{l}.b", 0, None)]
        refs += [(f"{p}_encoder._fc.weight", "enc.fc.W", 0, None),
                 (f"{p}_encoder._fc.bias", "enc.fc.b", 0, None),
                 (f"{p}_fc.weight", "q.fc.W", 0, None), (f"{p}_fc.bias", "q.fc.b", 0, None)]
        if self._q_type == "iqn":
            refs += [(f"{p}_embed.weight", "q.embed.W", 0, None),
                     (f"{p}_embed.bias", "q.embed.b", 0, None)]
        return refs

    def get_state_dict(self) -> Dict[str, dict]:
        torch.cuda.synchronize()
        r = self._refs()
        return {"_q_func": ckpt.module_state(self.store, r),
                "_targ_q_func": ckpt.module_state(self.targ, r),
                "_optim": ckpt.adam_state(self.optim_state, r)}

    def set_state_dict(self, sd: Dict[str, dict]) -> None:
        r = self._refs()
        ckpt.load_module_state(self.store, r, sd["_q_func"])
        ckpt.load_module_state(self.targ, r, sd["_targ_q_func"])
        ckpt.load_adam_state(self.optim_state, r, sd["_optim"])
        torch.cuda.synchronize()

    def save_model(self, fname: str) -> None:
        torch.save(self.get_state_dict(), fname)

    def load_model(self, fname: str) -> None:
        self.set_state_dict(torch.load(fname, map_location="cpu", weights_only=True))

    # --------------------------------------------------------------- updates
    def _workspace(self, B: int) -> "_Workspace":
        ws = self._ws.get(B)
        if ws is None:
            if self._ws:
                raise NotImplementedError("one batch size per DiscreteCQLImpl is supported")
            ws = _Workspace(self, B)
            self._ws[B] = ws
        return ws

    def update_step(self, batch, update_target: bool = False,
                    taus: Optional[Dict[str, np.ndarray]] = None, sync: bool = True,
                    use_graph: bool = True):
        db = as_device_batch(batch, self.torch_device)
        ws = self._workspace(db.batch_size)
        ws.stage(db, taus)
        ws.execute((bool(update_target),), use_graph=use_graph and taus is None)
        if not sync:
            return None
        return {k: float(v) for k, v in zip(METRIC_NAMES, ws.metrics.cpu().numpy())}

    def update(self, batch) -> np.ndarray:
        """DQNImpl.update (dqn_impl.py:97-111): returns the loss."""
        return np.float32(self.update_step(batch)["loss"])

    def update_target(self) -> None:
        """hard_sync (torch_utility.py:36-41)."""
        self.targ.data.copy_(self.store.data)

    # ------------------------------------------------- device-side batches
    def staging_batch(self, batch_size: int) -> DeviceBatch:
        ws = self._workspace(batch_size)
        B = batch_size
        return DeviceBatch(ws.obs2[:B], ws.act, ws.rew, ws.obs2[B:], ws.term, ws.nsteps)

    def active_metric_names(self):
        return ["loss"]

    def metrics_ring(self, n_steps: int):
        for ws in self._ws.values():
            ws.ring_ctr.zero_()
        return n_steps

    def read_metrics_ring(self, handle):
        if not self._ws:
            return ["loss"], np.zeros((0, 1), dtype=np.float32)
        ws = next(iter(self._ws.values()))
        k = min(int(ws.ring_ctr.item()), ws.ring.shape[0])
        return ["loss"], ws.ring[:k, :1].cpu().numpy()

    # ------------------------------------------------------------- inference
    def _as_input(self, x) -> torch.Tensor:
        t = torch.as_tensor(np.asarray(x) if not isinstance(x, torch.Tensor) else x)
        assert t.ndim == 4, "Input must have batch dimension."
        return t.to(self.torch_device).to(torch.uint8).contiguous()

    def _q_values(self, x_u8: torch.Tensor) -> torch.Tensor:
        """DiscreteIQNQFunction.forward in eval mode (n_greedy_quantiles
        linspace taus, iqn_q_function.py:16-30): mean over quantiles, [B][A];
        DiscreteMeanQFunction.forward (mean_q_function.py:22-23)."""
        B = x_u8.shape[0]
        if self._q_type == "mean":
            enc = _EncoderPass(self, B, self.torch_device, keep=False)
            enc.forward(x_u8.data_ptr(), self.store)
            q = torch.zeros(B, self._action_size, device=x_u8.device)
            ops.linear_fwd(enc.h.data_ptr(), True, self._F, self.store.ptr("q.fc.W"),
                           self.store.ptr("q.fc.b"), q.data_ptr(), 1, B, self._F,
                           self._action_size, relu=False)
            return q
        Kg = self._K_greedy
        enc = _EncoderPass(self, B, self.torch_device, keep=False)
        enc.forward(x_u8.data_ptr(), self.store)
        taus = torch.linspace(0, 1, Kg, device=x_u8.device).repeat(B)
        head = _HeadPass(self, B * Kg, self.torch_device)
        q = head.forward(taus, [enc.h.data_ptr()], B * Kg, Kg, self.store)
        return q.view(B, Kg, -1).mean(dim=1)

    def _policy_module(self) -> nn.Module:
        from ..export import IQNGreedy, MeanQGreedy, conv_from, linear_from
        st = self.store
        convs = nn.ModuleList(
            conv_from(st.view(wn)[0], st.view(bn)[0], g[5])
            for (wn, bn), g in zip(self.conv_names, self.geom))
        if self._q_type == "mean":
            return MeanQGreedy(convs, linear_from(st.view("enc.fc.W")[0], st.view("enc.fc.b")[0]),
                               linear_from(st.view("q.fc.W")[0], st.view("q.fc.b")[0]))
        return IQNGreedy(convs, linear_from(st.view("enc.fc.W")[0], st.view("enc.fc.b")[0]),
                         linear_from(st.view("q.embed.W")[0], st.view("q.embed.b")[0]),
                         linear_from(st.view("q.fc.W")[0], st.view("q.fc.b")[0]),
                         self._K_greedy, self._E)

    def predict_best_action(self, x) -> np.ndarray:
        with torch.no_grad():
            return self._q_values(self._as_input(x)).argmax(dim=1).cpu().numpy()

    def sample_action(self, x) -> np.ndarray:
        return self.predict_best_action(x)

    def predict_value(self, x, action, with_std: bool = False):
        with torch.no_grad():
            q = self._q_values(self._as_input(x))
            a = torch.as_tensor(np.asarray(action), device=q.device).long().view(-1)
            v = q[torch.arange(q.shape[0], device=q.device), a].cpu().numpy()
            return (v, np.zeros_like(v)) if with_std else v

    # ------------------------------------------------------------ inspection
    def grad(self, name: str) -> torch.Tensor:
        ws = next(iter(self._ws.values()))
        if ws.opt_late is not None and name in ws.opt_late.names:
            return ws.opt_late.grad(name)
        return ws.opt.grad(name)


def conv_wgrad_splits(geom, l: int, B: int) -> int:
    """The split count d3a_conv_bwd_w fills the chip with for conv layer l of
    a B-sample backward (its kernel's choice, d3a_conv_bwd_w_splits): the
    first layer reads the uint8 frames (x_u8 set, as the backward launch sets
    it), which selects the first-layer kernel (conv1_bwd_w_u8s4_kernel, 256
    splits at K5's shape) -- not the split-bf16 kernel's count for an fp32
    input."""
    ci, h, w, co, k, s, oh, ow = geom[l]
    gd = NAT.ConvDesc()
    gd.B, gd.C, gd.H, gd.W, gd.KH, gd.KW, gd.S, gd.OH, gd.OW, gd.CO = B, ci, h, w, k, k, s, oh, ow, co
    if l == 0:
        gd.x_u8 = 16  # only its presence and 4-byte alignment are read by the query
    S = int(NAT.lib().d3a_conv_bwd_w_splits(C.byref(gd)))
    assert S >= 1
    return S


def _conv_desc(geom, l: int, n: int, store: ParamStore, names) -> "NAT.ConvDesc":
    ci, h, w, co, k, s, oh, ow = geom[l]
    d = NAT.ConvDesc()
    d.B, d.C, d.H, d.W, d.KH, d.KW, d.S, d.OH, d.OW, d.CO = n, ci, h, w, k, k, s, oh, ow, co
    Wn, bn = names[l]
    d.weight, d.bias = store.ptr(Wn), store.ptr(bn)
    d.relu = 1
    return d


class _EncoderPass:
    """Buffers + launches of one PixelEncoder forward over n samples (NHWC
    activations, NCHW flatten): implicit-GEMM convs (d3a_conv_fwd, the pixel
    scaler fused into the first layer's loads) — no im2col matrix."""

    def __init__(self, impl: DiscreteCQLImpl, n: int, dev, keep: bool = True):
        self.impl, self.n = impl, n
        z = lambda *s: torch.zeros(*s, dtype=torch.float32, device=dev)  # noqa: E731
        self.ys = [z(n * oh * ow, co) for (ci, h, w, co, k, s, oh, ow) in impl.geom]
        # walk-ordered weight scratch of the fp32-input convs (d3a_conv_fwd)
        self.wpack = [z(co * ci * k * k) for (ci, h, w, co, k, s, oh, ow) in impl.geom]
        self.yt = z(n, impl.flat)
        self.h = z(n, impl._F)
        # the fc as split-K split-bf16 GEMM: about one 128 x 128 tile x slice
        # per CU (d3a_gemm_sbf16 + d3a_splitk_epilogue_f32)
        tiles = ((n + 127) // 128) * ((impl._F + 127) // 128)
        self.fc_splits = max(1, min(32, 256 // tiles, impl.flat // 128))
        self.fc_part = (z(self.fc_splits, n, impl._F) if _FC_SPLITK and impl.flat % 4 == 0
                        and impl._F % 4 == 0 else None)

    def forward(self, x_u8: int, store: ParamStore, prepacked: bool = False) -> None:
        """``prepacked``: the fp32 layers' weight copies are already in
        self.wpack (d3a_conv_pack_weights earlier in the step)."""
        impl = self.impl
        n = self.n
        for l in range(len(impl.geom)):
            d = _conv_desc(impl.geom, l, n, store, impl.conv_names)
            if l == 0:
                d.x_u8 = x_u8
            else:
                d.x_f32 = self.ys[l - 1].data_ptr()
                d.wpack = self.wpack[l].data_ptr()
                d.wpack_ready = int(prepacked)
            d.y = self.ys[l].data_ptr()
            ops.call_desc("d3a_conv_fwd", d)
        ci, h, w, co, k, s, oh, ow = impl.geom[-1]
        t = NAT.TransposeDesc()
        t.src, t.dst = self.ys[-1].data_ptr(), self.yt.data_ptr()
        t.B, t.P, t.C, t.to_cp = n, oh * ow, co, 1
        ops.call_desc("d3a_iqn_transpose", t)
        # K = 3136, few output tiles: over 2B = 1024 rows the register-direct
        # 32x64 tile with K split over waves (tools/bench_gemm_k5.py: 98 us vs
        # 139 for 64x64 LDS); at 512 rows the library's 32x32 choice (58 vs 96)
        if self.fc_part is not None:
            ops.linear_fwd_splitk(self.yt.data_ptr(), impl.flat, store.ptr("enc.fc.W"),
                                  store.ptr("enc.fc.b"), self.h.data_ptr(), n, impl.flat,
                                  impl._F, True, self.fc_part, self.fc_splits)
            return
        ops.linear_fwd(self.yt.data_ptr(), True, impl.flat, store.ptr("enc.fc.W"),
                       store.ptr("enc.fc.b"), self.h.data_ptr(), 1, n, impl.flat, impl._F,
                       relu=True, variant=10 if n > 512 else -1)


# the encoder fc on the bf16 matrix cores with fp32-accurate split-bf16
# operands (d3a_gemm_sbf16, six products): the forward as split-K slices plus
# an in-order partial-sum epilogue, the weight and input gradients as one
# launch each; D3A_FC_SPLITK=0 for the fp32-MFMA GEMMs
_FC_SPLITK = os.environ.get("D3A_FC_SPLITK", "1") == "1"

# the conv input gradient as one implicit GEMM (d3a_conv_bwd_x) rather than
# the column-matrix GEMM + col2im pair; D3A_CONV_BWD_X=0 for the pair
_CONV_BWD_X = os.environ.get("D3A_CONV_BWD_X", "1") == "1"


# the step's conv weight copies in one d3a_conv_pack_weights launch (else each
# conv entry packs its own); D3A_CONV_PREPACK=0 for the per-entry packs
_CONV_PREPACK = os.environ.get("D3A_CONV_PREPACK", "1") == "1"
# the step's taus on the weight-copy launch's appended workgroups (round 6)
_PHILOX_IN_PACK = os.environ.get("D3A_K5_PHILOX_IN_PACK", "1") == "1"


def _conv_bwd_x(ci: int, co: int) -> bool:
    """d3a_conv_bwd_x takes this layer (input channels 32 / 64, CO % 16 == 0)."""
    return _CONV_BWD_X and ci in (32, 64) and co % 16 == 0

# the IQN head forward as one launch (d3a_iqn_embed_head); D3A_IQN_FUSED=0
# keeps d3a_iqn_prior + the embed GEMM + d3a_iqn_head_fwd (A/B)
_IQN_FUSED = os.environ.get("D3A_IQN_FUSED", "1") == "1"
_IQN_RECOMPUTE = os.environ.get("D3A_IQN_RECOMPUTE", "1") == "1"
# concurrent graph branches in the K5 update (target pass; weight gradients);
# D3A_K5_BRANCHES=0 keeps one stream (A/B)
_K5_BRANCHES = os.environ.get("D3A_K5_BRANCHES", "1") == "1"
# with branches, the head / encoder-fc Adam early on the weight-gradient
# branch (D3A_K5_EARLY_ADAM=1); off by default: measured slower, 1,071
# against 1,126 steps/s (round 5; the Adam's HBM streams compete with the conv
# input-gradient chain it was to hide behind)
_K5_EARLY_ADAM = os.environ.get("D3A_K5_EARLY_ADAM", "0") == "1"


class _HeadPass:
    """IQN head forward buffers over `rows` quantile rows."""

    def __init__(self, impl: DiscreteCQLImpl, rows: int, dev):
        self.impl = impl
        self.dev = dev
        # prior / phi ([rows][E] / [rows][F]) only once a launch keeps rows:
        # the update's backward recomputes them from tau (d3a_iqn_head_bwd_fused)
        self.prior = self.phi = None
        self.q = torch.zeros(rows, impl._action_size, dtype=torch.float32, device=dev)
        self.rows = rows

    def _keep_bufs(self) -> None:
        if self.phi is None:
            z = lambda *s: torch.zeros(*s, dtype=torch.float32, device=self.dev)  # noqa: E731
            self.prior, self.phi = z(self.rows, self.impl._E), z(self.rows, self.impl._F)

    def launch(self, taus_ptr: int, h_groups: List[int], group_rows: int, K: int,
               store: ParamStore, n_keep: Optional[int] = None) -> None:
        """q of every row; prior / phi of rows [0, n_keep) (all rows when
        None) are left in self.prior / self.phi for a backward."""
        impl = self.impl
        if (_IQN_FUSED and impl._E == 64 and impl._F % 64 == 0 and impl._F <= 512
                and impl._action_size <= 8 and K % 32 == 0 and group_rows % K == 0):
            # prior, embed + ReLU, product and head in one launch
            # (d3a_iqn_embed_head; phi never round-trips HBM)
            d = NAT.IqnEmbedHeadDesc()
            d.taus, d.We, d.be = taus_ptr, store.ptr("q.embed.W"), store.ptr("q.embed.b")
            for g, hp in enumerate(h_groups):
                d.h[g] = hp
            d.Wf, d.bf, d.q = store.ptr("q.fc.W"), store.ptr("q.fc.b"), self.q.data_ptr()
            keep = self.rows if n_keep is None else n_keep
            if keep:
                self._keep_bufs()
            d.prior_out = self.prior.data_ptr() if keep else None
            d.phi_out = self.phi.data_ptr() if keep else None
            d.rows, d.group_rows, d.n_keep = self.rows, group_rows, keep
            d.K, d.E, d.F, d.A = K, impl._E, impl._F, impl._action_size
            ops.call_desc("d3a_iqn_embed_head", d)
            return
        self._keep_bufs()
        p = NAT.IqnPriorDesc()
        p.taus, p.prior, p.rows, p.E = taus_ptr, self.prior.data_ptr(), self.rows, impl._E
        ops.call_desc("d3a_iqn_prior", p)
        ops.linear_fwd(self.prior.data_ptr(), True, impl._E, store.ptr("q.embed.W"),
                       store.ptr("q.embed.b"), self.phi.data_ptr(), 1, self.rows, impl._E,
                       impl._F, relu=True)
        d = NAT.IqnHeadDesc()
        for g, hp in enumerate(h_groups):
            d.h[g] = hp
        d.phi, d.Wf, d.bf, d.q = (self.phi.data_ptr(), store.ptr("q.fc.W"), store.ptr("q.fc.b"),
                                  self.q.data_ptr())
        d.rows, d.group_rows = self.rows, group_rows
        d.K, d.F, d.A = K, impl._F, impl._action_size
        ops.call_desc("d3a_iqn_head_fwd", d)

    def forward(self, taus: torch.Tensor, h_groups: List[int], group_rows: int, K: int,
                store: ParamStore) -> torch.Tensor:
        self.launch(taus.contiguous().data_ptr(), h_groups, group_rows, K, store)
        return self.q


class _Workspace:
    def __init__(self, impl: DiscreteCQLImpl, B: int):
        dev = impl.torch_device
        self.impl = impl
        self.B = B
        K, A, F, E = impl._K, impl._action_size, impl._F, impl._E
        BK = B * K
        obs_shape = impl._observation_shape
        self.obs2 = torch.zeros((2 * B,) + tuple(obs_shape), dtype=torch.uint8, device=dev)
        self.act = torch.zeros(B, dtype=torch.int32, device=dev)
        z = lambda *s: torch.zeros(*s, dtype=torch.float32, device=dev)  # noqa: E731
        self.rew, self.term, self.nsteps = z(B), z(B), z(B)
        # taus [5][B][K]: loss | cons_lse | cons_data | next_online | next_target
        self.taus = z(5, B, K)
        self.rng_ctr = torch.zeros(1, dtype=torch.int64, device=dev)
        self.rng_ticket = torch.zeros(1, dtype=torch.int32, device=dev)
        self.seed = int(torch.randint(0, 2**62, (1,)).item())
        self.enc = _EncoderPass(impl, 2 * B, dev)      # online: [obs; next_obs]
        self.enc_t = _EncoderPass(impl, B, dev)        # target: next_obs
        self.mean = impl._q_type == "mean"
        self.fused_bwd = False
        if self.mean:
            # linear head: online Q over [obs; next_obs], target Q over next_obs
            self.q_on, self.q_t = z(2 * B, A), z(B, A)
            self.dq = z(B, A)
        else:
            self.head = _HeadPass(impl, 4 * BK, dev)   # online rows [loss|lse|data|next]
            self.head_t = _HeadPass(impl, BK, dev)     # target rows
            self.dq = z(3 * BK, A)
            self.dphi = None   # dL/dphi rows: the two-launch backward only
        self.loss_b, self.cons_b = z(B), z(B)
        self.metrics = z(len(METRIC_NAMES))
        self.ring = z(1 << 16, len(METRIC_NAMES))
        self.ring_ctr = torch.zeros(1, dtype=torch.int64, device=dev)
        # backward buffers (obs samples only)
        self.dzfc = z(B, F)
        self.dyt = z(B, impl.flat)
        self.dys = [z(B * oh * ow, co) for (ci, h, w, co, k, s, oh, ow) in impl.geom]
        self.dcols = [None] + [None if _conv_bwd_x(ci, co) else z(B * oh * ow, ci * k * k)
                               for (ci, h, w, co, k, s, oh, ow) in impl.geom[1:]]
        # the input gradients' tap-major weight copies (d3a_conv_bwd_x)
        self.wtap = [None] + [z(co * ci * k * k) if _conv_bwd_x(ci, co) and co % 32 == 0 else None
                              for (ci, h, w, co, k, s, oh, ow) in impl.geom[1:]]
        # gradients: split-K partials for the GEMM weight gradients, per-row
        # partials (B) for the IQN fc
        self.grads = GradSpace(dev)
        self.splits = {}
        for l, (ci, h, w, co, k, s, oh, ow) in enumerate(impl.geom):
            S = conv_wgrad_splits(impl.geom, l, B)
            self.splits[l] = S
            self.grads.add(f"enc.c{l}.W", (1, co, ci, k, k), S)
            self.grads.add(f"enc.c{l}.b", (1, co), S)
        # weight-gradient splits / tiles from tools/bench_gemm_k5.py
        # (profiles/r01_gemm_sweep_k5.log): fc 4 splits (38 us vs 53 at 16),
        # embed 32 splits on the register-direct 32x64 tile (112 us vs 244)
        self.S_fc = min(4, mlp.n_splits(B))
        self.grads.add("enc.fc.W", (1, F, impl.flat), self.S_fc)
        self.grads.add("enc.fc.b", (1, F), self.S_fc)
        if self.mean:
            self.S_head = mlp.n_splits(B)
            self.grads.add("q.fc.W", (1, A, F), self.S_head)
            self.grads.add("q.fc.b", (1, A), self.S_head)
        else:
            # the head backward + embed weight gradient as one launch
            # (d3a_iqn_head_bwd_fused): one partial per workgroup of NB rows b
            self.fused_bwd = (_IQN_FUSED and F == 512 and E == 64 and A <= 8 and K % 32 == 0)
            # the fused backward recomputes prior / phi from tau (the forward
            # keeps nothing); D3A_IQN_RECOMPUTE=0 keeps the kept-rows path (A/B)
            self.recompute = self.fused_bwd and _IQN_RECOMPUTE
            if not self.recompute:
                self.head._keep_bufs()
            if not self.fused_bwd:
                self.dphi = z(3 * BK, F)
            # 4 rows b per workgroup pair (256 workgroups at B = 512, 128
            # partials) recomputing; 2 per workgroup keeping
            self.NB = int(os.environ.get("D3A_IQN_NB", "4" if self.recompute else "2"))
            P = (B + self.NB - 1) // self.NB
            self.grads.add("q.fc.W", (1, A, F), P if self.fused_bwd else B)
            self.grads.add("q.fc.b", (1, A), P if self.fused_bwd else B)
            self.S_emb = P if self.fused_bwd else mlp.n_splits(3 * BK)
            self.grads.add("q.embed.W", (1, F, E), self.S_emb)
            self.grads.add("q.embed.b", (1, F), self.S_emb)
        # with graph branches the optimiser runs as two launches: the head and
        # encoder-fc parameters on side stream 2 as soon as the fc weight
        # gradient is formed (beside the conv input-gradient chain), the conv
        # layers after the join
        self.opt = self.opt_late = None
        if _K5_BRANCHES and _K5_EARLY_ADAM:
            conv = [n for n in impl.optim_state.names if n.startswith("enc.c")]
            self.opt_late = AdamGroup(impl.optim_state, self.grads, names=conv)
            self.opt = AdamGroup(impl.optim_state, self.grads,
                                 names=[n for n in impl.optim_state.names if n not in conv])
        else:
            self.opt = AdamGroup(impl.optim_state, self.grads)
        self._graphs: Dict[tuple, torch.cuda.CUDAGraph] = {}
        self._op_state = None  # tensors the update-step op declares mutated
        self._ran_eager = set()
        self._external_taus = False
        self._build_descs()

    def _build_descs(self):
        impl = self.impl
        B, K, A, F = self.B, impl._K, impl._action_size, impl._F
        BK = B * K
        if self.mean:
            l = NAT.DqnLossDesc()
            l.q, l.q_next, l.q_targ = (self.q_on.data_ptr(), self.q_on.data_ptr() + 4 * B * A,
                                       self.q_t.data_ptr())
            l.act, l.rew, l.term, l.n_steps = (self.act.data_ptr(), self.rew.data_ptr(),
                                               self.term.data_ptr(), self.nsteps.data_ptr())
            l.dq, l.metrics = self.dq.data_ptr(), self.metrics.data_ptr()
            l.B, l.A, l.double_q = B, A, int(impl._DOUBLE)
            l.gamma, l.alpha = impl._gamma, impl._alpha
            self.loss_desc = l
            return
        l = NAT.IqnLossDesc()
        q = self.head.q
        l.q_loss = q.data_ptr()                       # rows [0, 3BK)
        l.q_next = q.data_ptr() + 4 * 3 * BK * A      # rows [3BK, 4BK)
        l.q_targ = self.head_t.q.data_ptr()
        l.act, l.rew, l.term, l.n_steps = (self.act.data_ptr(), self.rew.data_ptr(),
                                           self.term.data_ptr(), self.nsteps.data_ptr())
        l.taus_loss = self.taus.data_ptr()
        l.dq, l.loss_b, l.cons_b, l.metrics = (self.dq.data_ptr(), self.loss_b.data_ptr(),
                                               self.cons_b.data_ptr(), self.metrics.data_ptr())
        l.B, l.K, l.A, l.gamma, l.alpha = B, K, A, impl._gamma, impl._alpha
        self.loss_desc = l
        hb = NAT.IqnHeadBwdDesc()
        hb.h, hb.dq = self.enc.h.data_ptr(), self.dq.data_ptr()
        hb.phi = self.head.phi.data_ptr() if self.head.phi is not None else None
        hb.Wf = impl.store.ptr("q.fc.W")
        hb.dphi = self.dphi.data_ptr() if self.dphi is not None else None
        hb.dh = self.dzfc.data_ptr()
        hb.dWf_part = self.grads.get("q.fc.W").data_ptr()
        hb.dbf_part = self.grads.get("q.fc.b").data_ptr()
        hb.B, hb.K, hb.F, hb.A, hb.G = B, K, F, A, 3
        self.head_bwd_desc = hb
        if self.fused_bwd:
            fb = NAT.IqnHeadBwdFusedDesc()
            fb.h = self.enc.h.data_ptr()
            if self.recompute:
                fb.taus = self.taus.data_ptr()   # rows g B K + b K + k: the forward's rows
                fb.We, fb.be = impl.store.ptr("q.embed.W"), impl.store.ptr("q.embed.b")
            else:
                fb.phi, fb.prior = self.head.phi.data_ptr(), self.head.prior.data_ptr()
            fb.dq, fb.Wf = self.dq.data_ptr(), impl.store.ptr("q.fc.W")
            fb.dh = self.dzfc.data_ptr()
            fb.dWf_part = self.grads.get("q.fc.W").data_ptr()
            fb.dbf_part = self.grads.get("q.fc.b").data_ptr()
            fb.dWe_part = self.grads.get("q.embed.W").data_ptr()
            fb.dbe_part = self.grads.get("q.embed.b").data_ptr()
            fb.B, fb.K, fb.F, fb.E, fb.A, fb.G, fb.NB = B, K, F, impl._E, A, 3, self.NB
            self.head_bwd_fused_desc = fb

    def stage(self, db: DeviceBatch, taus) -> None:
        B = self.B
        if db.obs.data_ptr() != self.obs2.data_ptr():
            self.obs2[:B].copy_(db.obs.view_as(self.obs2[:B]), non_blocking=True)
            self.obs2[B:].copy_(db.next_obs.view_as(self.obs2[B:]), non_blocking=True)
            self.act.copy_(db.act.view(B).to(torch.int32), non_blocking=True)
            self.rew.copy_(db.rew.view(B), non_blocking=True)
            self.term.copy_(db.term.view(B), non_blocking=True)
            self.nsteps.copy_(db.n_steps.view(B), non_blocking=True)
        self._external_taus = taus is not None
        if taus is not None:
            order = ("loss", "cons_lse", "cons_data", "next_online", "next_target")
            for i, k in enumerate(order):
                self.taus[i].copy_(torch.as_tensor(np.asarray(taus[k]), dtype=torch.float32)
                                   .view(B, -1))

    def dominant_kernel(self):
        """The step's longest kernel: the fused IQN head backward over the G
        gradient passes (G B K rows x F units: dphi, dh, dWf, and the embed
        weight gradient dWe on split-bf16 MFMA) -- per row 2 F (2 A + 1 + E) + F
        flops, + 2 F E recomputing phi; else (mean head, or D3A_K5_DOMINANT=conv1) the first conv GEMM
        over [obs; next_obs] (2B x 400 positions x 32 filters x 256 taps)."""
        impl = self.impl
        if (not self.mean and self.fused_bwd
                and os.environ.get("D3A_K5_DOMINANT", "head_bwd") != "conv1"):
            fb = self.head_bwd_fused_desc
            rows = fb.G * fb.B * fb.K
            F, A, E = fb.F, fb.A, fb.E

            def launch_hb():
                ops.call_desc("d3a_iqn_head_bwd_fused", fb)
            if self.recompute:
                # + the phi recompute (2 F E per row: the forward's embed product)
                return launch_hb, rows * (2 * F * (2 * A + 1 + 2 * E) + F), (
                    f"d3a_iqn_head_bwd_fused (phi recomputed from tau and dWe on split-bf16 "
                    f"x6 MFMA, fp32 head backward): {rows} rows x {F} units, E {E}, A {A}; "
                    f"flops include the recompute")
            return launch_hb, rows * (2 * F * (2 * A + 1 + E) + F), (
                f"d3a_iqn_head_bwd_fused (dWe on split-bf16 x6 MFMA, fp32 head backward): "
                f"{rows} rows x {F} units, E {E}, A {A}")
        ci, h, w, co, k, s, oh, ow = impl.geom[0]
        rows = 2 * self.B * oh * ow
        d = _conv_desc(impl.geom, 0, 2 * self.B, impl.store, impl.conv_names)
        d.x_u8, d.y = self.obs2.data_ptr(), self.enc.ys[0].data_ptr()

        def launch():
            ops.call_desc("d3a_conv_fwd", d)
        x3 = os.environ.get("D3A_CONV_X6", "1") != "0"
        return launch, 2 * rows * ci * k * k * co, (
            f"d3a_conv_fwd conv1 (implicit GEMM, u8 input"
            f"{', split-bf16 x3: bytes exact, three bf16 products' if x3 else ''}): "
            f"[{rows}x{ci * k * k}]@[{ci * k * k}x{co}]")

    def execute(self, flags, use_graph: bool) -> None:
        key = tuple(flags) + (self._external_taus,)
        if not use_graph:
            self._enqueue(*flags)
            return
        g = self._graphs.get(key)
        if g is None:
            if key not in self._ran_eager:
                self._ran_eager.add(key)
                self._enqueue(*flags)
                return
            g = torch.cuda.CUDAGraph()
            torch.cuda.synchronize()
            with ops.graph_capture(g):
                self._enqueue(*flags)
            self._graphs[key] = g
        # the replay through the torch custom op (TORCH_LIBRARY d3rlpy_amd)
        if self._op_state is None:
            self._op_state = ops.update_state(self.impl, self)
        ops.replay_update(g, self._op_state)

    def _side(self, i: int) -> torch.cuda.Stream:
        if not hasattr(self, "_sides"):
            self._sides = [torch.cuda.Stream(device=self.obs2.device) for _ in range(2)]
        return self._sides[i]

    def _enqueue(self, sync_target: bool) -> None:
        impl = self.impl
        B, K, A, F, E = self.B, impl._K, impl._action_size, impl._F, impl._E
        BK = B * K
        st, tg = impl.store, impl.targ
        # every fp32 conv layer's weight copies for this step in one launch:
        # the online and target forwards' walk order, the input gradients'
        # tap-major order (the weights do not change before the step's Adam);
        # the step's taus drawn on that launch's appended workgroups (round 6;
        # D3A_K5_PHILOX_IN_PACK=0: their own d3a_philox_fill launch)
        pre = _CONV_PREPACK and len(impl.geom) > 1
        ph = None
        if not self._external_taus and not self.mean:
            if pre and _PHILOX_IN_PACK:
                ph = NAT.PhiloxJob()
                ph.out, ph.n_normal, ph.n_uniform = self.taus.data_ptr(), 0, self.taus.numel()
                ph.lo, ph.hi, ph.seed = 0.0, 1.0, self.seed
                ph.ctr, ph.ticket = self.rng_ctr.data_ptr(), self.rng_ticket.data_ptr()
            else:
                ops.philox_fill(self.taus, 0, self.taus.numel(), 0.0, 1.0, self.seed, self.rng_ctr,
                                self.rng_ticket)
        if pre:
            descs, lays = [], []
            for l in range(1, len(impl.geom)):
                for store_, buf, lay in ((st, self.enc.wpack[l], 0), (tg, self.enc_t.wpack[l], 0),
                                         (st, self.wtap[l], 1)):
                    if buf is None:
                        continue
                    d = _conv_desc(impl.geom, l, B, store_, impl.conv_names)
                    d.wpack = buf.data_ptr()
                    descs.append(d)
                    lays.append(lay)
            if descs:
                ops.conv_pack_weights(descs, lays, philox=ph)
            elif ph is not None:
                ops.philox_fill(self.taus, 0, self.taus.numel(), 0.0, 1.0, self.seed, self.rng_ctr,
                                self.rng_ticket)
        # graph branches: the target encoder + target head (own buffers, the
        # target parameters) run on side stream 1 beside the online encoder +
        # head, joined before the loss; in the backward each layer's weight
        # gradient runs on side stream 2 beside the input-gradient chain
        # (joined before Adam).  Nodes of the captured graph then overlap.
        main = torch.cuda.current_stream()
        br = _K5_BRANCHES
        if br:
            s1 = self._side(0)
            s1.wait_stream(main)
        # encoders
        self.enc.forward(self.obs2.data_ptr(), st, prepacked=pre)
        with torch.cuda.stream(s1) if br else contextlib.nullcontext():
            self.enc_t.forward(self.obs2.data_ptr() + self.obs2[0].numel() * B, tg, prepacked=pre)
            if not self.mean:
                self.head_t.launch(self.taus.data_ptr() + 4 * 4 * BK, [self.enc_t.h.data_ptr()],
                                   BK, K, tg, n_keep=0)
        h_obs = self.enc.h.data_ptr()
        h_next = h_obs + 4 * B * F
        g = self.grads
        if self.mean:
            if br:
                main.wait_stream(s1)
            # linear heads (mean_q_function.py:22-23), the TD (+ conservative)
            # loss with dL/dQ, then the head's weight and masked input gradients
            ops.linear_fwd(h_obs, True, F, st.ptr("q.fc.W"), st.ptr("q.fc.b"),
                           self.q_on.data_ptr(), 1, 2 * B, F, A, relu=False)
            ops.linear_fwd(self.enc_t.h.data_ptr(), True, F, tg.ptr("q.fc.W"), tg.ptr("q.fc.b"),
                           self.q_t.data_ptr(), 1, B, F, A, relu=False)
            ops.call_desc("d3a_dqn_loss", self.loss_desc)
            ops.linear_bwd_w(self.dq.data_ptr(), A, B * A, h_obs, F, B * F,
                             g.get("q.fc.W").data_ptr(), 1, B, F, A, self.S_head,
                             db=g.get("q.fc.b").data_ptr())
            ops.linear_bwd_x(self.dq.data_ptr(), A, B * A, st.ptr("q.fc.W"), self.dzfc.data_ptr(),
                             F, B * F, 1, B, F, A, mask=h_obs, ldm=F, smb=B * F)
        else:
            # IQN heads: online rows [loss | lse | data | next], target rows
            # (kept prior / phi of the three gradient passes only when the
            # backward does not recompute them)
            self.head.launch(self.taus.data_ptr(), [h_obs, h_obs, h_obs, h_next], BK, K, st,
                             n_keep=0 if self.recompute else 3 * BK)
            if br:
                main.wait_stream(s1)
            ops.call_desc("d3a_iqn_loss", self.loss_desc)
            # backward: head, embed, encoder (obs samples)
            if self.fused_bwd:
                ops.call_desc("d3a_iqn_head_bwd_fused", self.head_bwd_fused_desc)
            else:
                ops.call_desc("d3a_iqn_head_bwd", self.head_bwd_desc)
                ops.linear_bwd_w(self.dphi.data_ptr(), F, 3 * BK * F, self.head.prior.data_ptr(),
                                 E, 3 * BK * E, g.get("q.embed.W").data_ptr(), 1, 3 * BK, E, F,
                                 self.S_emb, db=g.get("q.embed.b").data_ptr(), variant=10)
        if br:
            s2 = self._side(1)

        def wgrad(fn):  # a weight gradient: on side stream 2 after main's work so far
            if br:
                s2.wait_stream(main)
                with torch.cuda.stream(s2):
                    fn()
            else:
                fn()
        wgrad(lambda: ops.linear_bwd_w(
            self.dzfc.data_ptr(), F, B * F, self.enc.yt.data_ptr(), impl.flat, B * impl.flat,
            g.get("enc.fc.W").data_ptr(), 1, B, impl.flat, F, self.S_fc,
            db=g.get("enc.fc.b").data_ptr(), sbf16=6 if _FC_SPLITK else 0))
        ops.linear_bwd_x(self.dzfc.data_ptr(), F, B * F, st.ptr("enc.fc.W"), self.dyt.data_ptr(),
                         impl.flat, B * impl.flat, 1, B, impl.flat, F, sbf16=6 if _FC_SPLITK else 0)
        if self.opt_late is not None:
            # the head / encoder-fc Adam on the weight-gradient branch, behind the
            # fc weight gradient there and (wait on main) the fc input gradient,
            # the last reader of those parameters in this step
            wgrad(self.opt.launch)
        ci, h, w, co, k, s, oh, ow = impl.geom[-1]
        t = NAT.TransposeDesc()
        t.src, t.dst, t.mask = self.dyt.data_ptr(), self.dys[-1].data_ptr(), \
            self.enc.ys[-1].data_ptr()
        t.B, t.P, t.C, t.to_cp = B, oh * ow, co, 0
        ops.call_desc("d3a_iqn_transpose", t)
        for l in range(len(impl.geom) - 1, -1, -1):
            ci, h, w, co, k, s, oh, ow = impl.geom[l]
            rows, Kc = B * oh * ow, ci * k * k
            Wn, bn = impl.conv_names[l]
            # weight gradient over the obs samples (the first B of the online pass)
            cd = _conv_desc(impl.geom, l, B, st, impl.conv_names)
            if l == 0:
                cd.x_u8 = self.obs2.data_ptr()
            else:
                cd.x_f32 = self.enc.ys[l - 1].data_ptr()
            cd.dy, cd.dW, cd.db = self.dys[l].data_ptr(), g.get(Wn).data_ptr(), \
                g.get(bn).data_ptr()
            cd.splits = self.splits[l]
            wgrad(lambda cd=cd: ops.call_desc("d3a_conv_bwd_w", cd))
            if l > 0 and _conv_bwd_x(ci, co):
                # the input gradient as one implicit GEMM through the ReLU of
                # the layer's input (no column matrix, no col2im)
                xd = _conv_desc(impl.geom, l, B, st, impl.conv_names)
                xd.x_f32, xd.dy, xd.y = (self.enc.ys[l - 1].data_ptr(), self.dys[l].data_ptr(),
                                         self.dys[l - 1].data_ptr())
                if self.wtap[l] is not None:
                    xd.wpack = self.wtap[l].data_ptr()  # tap-major weight copy
                    xd.wpack_ready = int(pre)
                ops.call_desc("d3a_conv_bwd_x", xd)
            elif l > 0:
                ops.linear_bwd_x(self.dys[l].data_ptr(), co, rows * co, st.ptr(Wn),
                                 self.dcols[l].data_ptr(), Kc, rows * Kc, 1, rows, Kc, co)
                c2 = NAT.Col2imDesc()
                c2.dcol, c2.ldcol = self.dcols[l].data_ptr(), Kc
                c2.mask = self.enc.ys[l - 1].data_ptr()
                c2.dx = self.dys[l - 1].data_ptr()
                c2.B, c2.C, c2.H, c2.W = B, ci, h, w
                c2.KH, c2.KW, c2.S, c2.OH, c2.OW = k, k, s, oh, ow
                ops.call_desc("d3a_col2im", c2)
        if br:
            main.wait_stream(s2)
        (self.opt_late or self.opt).launch()
        ops.step_end(impl.counters, 1, self.metrics, self.ring, self.ring_ctr,
                     tg.data if sync_target else None, st.data if sync_target else None,
                     1.0)
