"""Flat, HBM-resident parameter storage for the MLP ensembles of the update.

Layout (per network, one flat fp32 buffer shared by every network of an
Impl so that a single launch can soft-update all targets):

    for each layer l of an ensemble of C members:
        W_l  [C][out_l][in_l]   (nn.Linear weight layout, member-major)
        b_l  [C][out_l]

Segments start at 64-element (256 B) aligned offsets so that every row base
used by the kernels is 16-byte aligned.  ``nn.Parameter`` views of member c
(``W_l[c]``) are contiguous, so reference-shaped modules can alias the
buffer for checkpoints (``state_dict`` layout of d3rlpy/torch_utility.py:97-117).

Initialisation replays the reference construction order with torch's CPU
generator (nn.Linear defaults), so ``torch.manual_seed(s)`` gives the same
initial weights as the reference built under the same seed.
"""
from __future__ import annotations

import ctypes as C
from collections import OrderedDict
from typing import Dict, List, Optional, Sequence, Tuple

import torch
from torch import nn

from . import _native as N

_ALIGN = 64


def _align(n: int) -> int:
    return (n + _ALIGN - 1) // _ALIGN * _ALIGN


class ParamStore:
    """Named tensors packed in one flat fp32 buffer."""

    def __init__(self) -> None:
        self.specs: "OrderedDict[str, Tuple[Tuple[int, ...], int]]" = OrderedDict()
        self.size = 0
        self.data: Optional[torch.Tensor] = None

    def add(self, name: str, shape: Sequence[int]) -> int:
        assert self.data is None, "store already allocated"
        assert name not in self.specs, name
        off = self.size
        n = 1
        for s in shape:
            n *= int(s)
        self.specs[name] = (tuple(int(s) for s in shape), off)
        self.size = off + _align(n)
        return off

    def allocate(self, device: torch.device) -> "ParamStore":
        self.data = torch.zeros(max(self.size, 1), dtype=torch.float32, device=device)
        return self

    def like(self) -> "ParamStore":
        """A new store with the identical layout (zero-filled)."""
        o = ParamStore()
        o.specs = OrderedDict(self.specs)
        o.size = self.size
        assert self.data is not None
        o.data = torch.zeros_like(self.data)
        return o

    def offset(self, name: str) -> int:
        return self.specs[name][1]

    def numel(self, name: str) -> int:
        n = 1
        for s in self.specs[name][0]:
            n *= s
        return n

    def view(self, name: str) -> torch.Tensor:
        shape, off = self.specs[name]
        assert self.data is not None
        return self.data[off:off + self.numel(name)].view(shape)

    def ptr(self, name: str) -> int:
        assert self.data is not None
        return self.data.data_ptr() + 4 * self.offset(name)

    def span(self, names: Sequence[str]) -> Tuple[int, int]:
        """[start, end) element range covering the given segments."""
        offs = [self.offset(n) for n in names]
        ends = [self.offset(n) + self.numel(n) for n in names]
        return min(offs), max(ends)


class EnsembleMLP:
    """Registers an ensemble of C MLPs ``sizes[0] -> ... -> sizes[-1]`` in a store."""

    def __init__(self, store: ParamStore, prefix: str, n_members: int, sizes: Sequence[int]):
        self.store = store
        self.prefix = prefix
        self.C = n_members
        self.sizes = list(sizes)
        self.n_layers = len(sizes) - 1
        for l in range(self.n_layers):
            store.add(self.wname(l), (n_members, sizes[l + 1], sizes[l]))
            store.add(self.bname(l), (n_members, sizes[l + 1]))

    def wname(self, l: int) -> str:
        return f"{self.prefix}.W{l}"

    def bname(self, l: int) -> str:
        return f"{self.prefix}.b{l}"

    def names(self) -> List[str]:
        out = []
        for l in range(self.n_layers):
            out += [self.wname(l), self.bname(l)]
        return out

    def W(self, l: int, store: Optional[ParamStore] = None) -> int:
        return (store or self.store).ptr(self.wname(l))

    def b(self, l: int, store: Optional[ParamStore] = None) -> int:
        return (store or self.store).ptr(self.bname(l))

    def load_linear(self, l: int, member: int, lin: nn.Linear, store: Optional[ParamStore] = None):
        s = store or self.store
        with torch.no_grad():
            s.view(self.wname(l))[member].copy_(lin.weight.detach())
            s.view(self.bname(l))[member].copy_(lin.bias.detach())

    def export_linear(self, l: int, member: int, store: Optional[ParamStore] = None):
        s = store or self.store
        return s.view(self.wname(l))[member], s.view(self.bname(l))[member]


class GradSpace:
    """Split-K partial-gradient workspaces, one per parameter segment."""

    def __init__(self, device: torch.device):
        self.device = device
        self.parts: Dict[str, Tuple[torch.Tensor, int]] = {}

    def add(self, name: str, shape: Sequence[int], n_partials: int) -> torch.Tensor:
        t = torch.zeros((n_partials,) + tuple(shape), dtype=torch.float32, device=self.device)
        self.parts[name] = (t, n_partials)
        return t

    def get(self, name: str) -> torch.Tensor:
        return self.parts[name][0]


class OptimState:
    """torch.optim.Adam state of a set of segments: exp_avg / exp_avg_sq in
    store-shaped buffers plus the (device) step count of the optimiser."""

    def __init__(self, store: ParamStore, names: Sequence[str], lr: float,
                 betas=(0.9, 0.999), eps: float = 1e-8, step: Optional[torch.Tensor] = None):
        assert store.data is not None
        self.store = store
        self.names = list(names)
        self.lr, self.betas, self.eps = float(lr), (float(betas[0]), float(betas[1])), float(eps)
        dev = store.data.device
        self.exp_avg = store.like()
        self.exp_avg_sq = store.like()
        # completed steps (device int64, committed by d3a_step_end); may be a
        # view into an Impl-wide counter array
        self.step = torch.zeros(1, dtype=torch.int64, device=dev) if step is None else step


def _seg_threads(n_partials: int, numel: int) -> int:
    """Threads of one Adam / reduce segment (elementwise.hip seg_threads):
    16 lanes per element for >= 64 partials, else one lane per 4 elements when
    the size is a multiple of 4 and at least 2^18, else one per element."""
    if n_partials >= 64:
        return numel * 16
    return numel // 4 if (numel % 4 == 0 and numel >= 1 << 18) else numel


class AdamGroup:
    """A torch.optim.Adam equivalent over a set of segments of a ParamStore.

    Exposes the reduced gradient of the last step per segment (``grad(name)``)
    for parity tests; the optimiser state lives in an ``OptimState``.
    """

    def __init__(self, state: OptimState, grads: GradSpace, keep_grads: bool = True,
                 names: Optional[List[str]] = None):
        """``names``: a subset of the state's parameters (the optimiser split in
        launches whose gradients are ready at different times; the moments and
        the step counter are the state's, shared)."""
        store = state.store
        self.state = state
        self.store = store
        self.names = list(state.names) if names is None else [n for n in state.names if n in names]
        self.lr, self.eps = state.lr, state.eps
        self.beta1, self.beta2 = state.betas
        dev = store.data.device
        self.exp_avg = state.exp_avg
        self.exp_avg_sq = state.exp_avg_sq
        self.step = state.step
        self.grad_store = store.like() if keep_grads else None
        segs = (N.AdamSegment * len(self.names))()
        self.n_blocks = 0  # flat launch over the segments (d3a_adam_f32)
        self.n_blocks_reduced = 0
        # no segment takes four elements a thread (in the partials' table /
        # the reduced table, whose one-partial segments may)
        self.one_elem = True
        self.one_elem_reduced = True
        for i, n in enumerate(self.names):
            gt, parts = grads.parts[n]
            numel = store.numel(n)
            assert gt.numel() == parts * numel, (n, gt.shape, numel)
            if parts * numel * 4 >= 2 ** 32:  # elementwise.hip sum_partials_u: 32-bit offsets
                raise ValueError(f"AdamGroup: {n}'s partials exceed 4 GiB ({parts} x {numel})")
            segs[i].param = store.ptr(n)
            segs[i].exp_avg = self.exp_avg.ptr(n)
            segs[i].exp_avg_sq = self.exp_avg_sq.ptr(n)
            segs[i].grad = gt.data_ptr()
            segs[i].numel = numel
            segs[i].n_partials = parts
            segs[i].partial_stride = numel
            segs[i].grad_out = self.grad_store.ptr(n) if self.grad_store is not None else None
            self.n_blocks += (_seg_threads(parts, numel) + 255) // 256
            self.one_elem &= _seg_threads(parts, numel) == numel * (16 if parts >= 64 else 1)
            self.one_elem_reduced &= _seg_threads(1, numel) == numel
            self.n_blocks_reduced += (_seg_threads(1, numel) + 255) // 256
        raw = bytes(segs)
        self.seg_table = torch.frombuffer(bytearray(raw), dtype=torch.uint8).to(dev)
        self._segs = segs
        self.block_table = self._block_table(segs, True)
        self.seg_table_reduced = None
        self.block_table_reduced = None
        if self.grad_store is not None:
            # the same segments reading the already-reduced gradient (one
            # partial) from grad_store: the data-parallel path's Adam
            red = (N.AdamSegment * len(self.names))()
            for i, n in enumerate(self.names):
                red[i].param, red[i].exp_avg = segs[i].param, segs[i].exp_avg
                red[i].exp_avg_sq = segs[i].exp_avg_sq
                red[i].grad = self.grad_store.ptr(n)
                red[i].numel, red[i].n_partials = segs[i].numel, 1
                red[i].partial_stride = segs[i].numel
                red[i].grad_out = None
            self.seg_table_reduced = torch.frombuffer(bytearray(bytes(red)),
                                                      dtype=torch.uint8).to(dev)
            self.block_table_reduced = self._block_table(red, False)

    def _block_table(self, segs, partials: bool) -> torch.Tensor:
        """d3a_adam_block per flat block (the segment search done once here,
        in the kernel's block order: segment s owns ceil(threads_s / 256)
        blocks, _seg_threads)."""
        rows = []
        first = 0
        for sg in segs:
            nb = (_seg_threads(sg.n_partials if partials else 1, sg.numel) + 255) // 256
            for _ in range(nb):
                blk = N.AdamBlock()
                blk.seg, blk.first = sg, first
                rows.append(bytes(blk))
            first += nb
        raw = b"".join(rows)
        return torch.frombuffer(bytearray(raw), dtype=torch.uint8).to(self.store.data.device)

    def launch(self, reduced: bool = False, grad_scale: float = 1.0,
               tail: Optional[dict] = None) -> None:
        """Adam over every segment; ``reduced``: from grad_store (after
        ``reduce`` and an all-reduce) scaled by ``grad_scale``.  ``tail``:
        keyword arguments of ops.adam_step (soft target update through
        ``targ`` — a ParamStore of the same layout — and ``tau``, step_add,
        counters / metric ring) for the fused end-of-update launch."""
        from . import ops
        table = self.seg_table_reduced if reduced else self.seg_table
        assert table is not None
        nb = self.n_blocks_reduced if reduced else self.n_blocks
        if tail is None:
            ops.adam(table, len(self.names), nb, self.step, self.lr, self.beta1, self.beta2,
                     self.eps, grad_scale)
            return
        kw = dict(tail)
        targ = kw.pop("targ", None)
        if targ is not None:
            assert targ.size == self.store.size and list(targ.specs) == list(self.store.specs)
            kw["targ_delta"] = (targ.data.data_ptr() - self.store.data.data_ptr()) // 4
            assert kw["targ_delta"] != 0
        blocks = self.block_table_reduced if reduced else self.block_table
        # (the reduced table: one partial, the same four-a-thread segments)
        ops.adam_step(table, len(self.names), nb, self.step, self.lr, self.beta1, self.beta2,
                      self.eps, grad_scale, blocks=blocks,
                      one_elem=self.one_elem_reduced if reduced else self.one_elem, **kw)

    def reduce(self) -> None:
        """grad_store <- sum of the split-K partials (no parameter update)."""
        from . import ops
        assert self.grad_store is not None
        ops.grad_reduce(self.seg_table, len(self.names), self.n_blocks)

    def grad_span(self) -> torch.Tensor:
        """The contiguous slice of grad_store holding this group's gradients."""
        s, e = self.store.span(self.names)
        return self.grad_store.data[s:e]

    def grad(self, name: str) -> torch.Tensor:
        assert self.grad_store is not None
        return self.grad_store.view(name)
