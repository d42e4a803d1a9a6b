"""Multilayer perceptron classifier — bf16 MFMA training engine.

New capability (the reference has no MLP; BASELINE.json config 3 "WISDM 6-class
3-layer MLP bf16, DP all-reduce on 8xMI355X").  API modelled on Spark's
``MultilayerPerceptronClassifier(layers=[in, h1, ..., out], maxIter, blockSize,
stepSize, seed)``; hidden activations are ReLU and the solver is Adam.

Engine layout (MI355X-first):

* all parameters live in ONE flat fp32 master buffer (+ Adam m/v), with a bf16
  compute copy refreshed by the fused Adam kernel, and ONE flat fp32 gradient
  buffer — so data-parallel training issues exactly one RCCL all-reduce per step
  (the whole gradient is ~0.3 MB: latency-bound on xGMI, so one bucket);
* one training step = memset + L forward GEMMs (bias+ReLU fused) + fused
  softmax-CE head (loss, accuracy, dlogits, bias grad) + per layer one data-grad
  GEMM (ReLU mask + bias grad fused) and one split-K weight-grad GEMM
  + [all-reduce] + fused Adam.  No host synchronization inside a step; the loss
  and correct-count accumulators are read only when asked for;
* input rows are kept resident in HBM as padded bf16 ([N, F_pad]); a step reads a
  contiguous slice (zero-copy batches of a pre-shuffled resident dataset).

The CPU path (and test oracle) is the same network in PyTorch fp32.
"""
from __future__ import annotations

import math
import os
from dataclasses import dataclass
from typing import List, Optional, Sequence

import numpy as np
import torch

from ..data.table import Table
from ..ops import _native, rng
from ..ops.gemm import EPI_BIAS_RELU, EPI_F32_SLAB, EPI_RELU_GRAD, gemm_bf16, tile_counts
from .base import ClassificationModel, ClassifierParams, Estimator, dp_allreduce, dp_context, dp_owner, dp_rows, \
    features_tensor, labels_tensor, new_uid, resolve_device

HEAD_PAD = 32  # classes padded to 32 rows (two 16-wide MFMA column tiles)


def _pad(x: int, m: int) -> int:
    return (x + m - 1) // m * m


def n_splits_for(batch: int) -> int:
    """Batch slices of the split-K weight-gradient GEMMs (>= 1024-row slices, <= 64 slabs;
    ``HAR_MLP_SPLITS`` overrides the slab cap for tuning)."""
    cap = int(os.environ.get("HAR_MLP_SPLITS", "64"))
    return max(1, min(cap, batch // max(1, 65536 // cap)))


# Tile choices measured on MI355X with tools/gemm_bench.py (profiles/gemm_tile_sweep.md):
# ids index ops.gemm.TILES = (BM, BN, BK).
def fwd_tile(M: int, N: int, K: int) -> int:
    if K <= 64:
        return 12             # 64x128, BK 64
    return 6 if N >= 256 else 12  # 128x256 reads each activation row once


def dgrad_tile(M: int, N: int, K: int) -> int:
    return 18 if N >= 256 else 12    # 128x128 / 8 waves (24.0 us vs 24.8 for 128x256 at B = 65536)


def wgrad_tile(M: int, N: int) -> int:
    """Weight-gradient (split-K over the batch) tiles (profiles/gemm_tile_sweep_v2.md)."""
    if M <= 32:
        return 11 if N > 32 else 2   # 32x64, BK 128
    if N <= 64:
        return 20                    # 64x64, BK 128, 8 waves: 13.1 us vs 14.4 (4 waves)
    return 18                        # 128x128, BK 64, 8 waves: 23.4 us vs 30.0 (4 waves)


@dataclass
class Segment:
    name: str
    offset: int
    shape: tuple

    @property
    def numel(self):
        return int(np.prod(self.shape))


class FlatLayout:
    """Offsets of every weight/bias inside the flat buffers (16-element aligned)."""

    def __init__(self, layers: Sequence[int]):
        self.layers = list(layers)
        self.in_pad = _pad(layers[0], 32)
        self.hidden = list(layers[1:-1])
        for h in self.hidden:
            if h % 32:
                raise ValueError("hidden layer sizes must be multiples of 32")
        self.num_classes = layers[-1]
        if self.num_classes > HEAD_PAD:
            raise ValueError(f"at most {HEAD_PAD} classes")
        dims = [self.in_pad] + self.hidden
        self.segments: List[Segment] = []
        off = 0
        for i in range(len(self.hidden)):
            for name, shape in ((f"W{i}", (dims[i + 1], dims[i])), (f"b{i}", (dims[i + 1],))):
                self.segments.append(Segment(name, off, shape))
                off = _pad(off + int(np.prod(shape)), 64)
        last = dims[-1]
        for name, shape in (("Wout", (HEAD_PAD, last)), ("bout", (HEAD_PAD,))):
            self.segments.append(Segment(name, off, shape))
            off = _pad(off + int(np.prod(shape)), 64)
        self.total = off
        self.by_name = {s.name: s for s in self.segments}

    def view(self, flat: torch.Tensor, name: str) -> torch.Tensor:
        s = self.by_name[name]
        return flat[s.offset: s.offset + s.numel].view(s.shape)


def init_params(layout: FlatLayout, seed: int) -> torch.Tensor:
    """Kaiming-uniform weights from Philox (identical on every rank), zero biases."""
    flat = torch.zeros(layout.total, dtype=torch.float32)
    dims = [layout.in_pad] + layout.hidden
    fan_ins = {f"W{i}": layout.layers[0] if i == 0 else dims[i] for i in range(len(layout.hidden))}
    fan_ins["Wout"] = dims[-1]
    for s in layout.segments:
        if not s.name.startswith("W"):
            continue
        bound = math.sqrt(6.0 / fan_ins[s.name])
        u = rng.uniform(seed, rng.STREAM_INIT, np.arange(s.offset, s.offset + s.numel, dtype=np.uint64))
        w = torch.from_numpy(((2 * u - 1) * bound).astype(np.float32)).view(s.shape)
        if s.name == "W0":
            w[:, layout.layers[0]:] = 0  # padded input columns
        if s.name == "Wout":
            w[layout.num_classes:] = 0   # padded class rows
        flat[s.offset: s.offset + s.numel] = w.reshape(-1)
    return flat


class MLPEngine:
    """Device-resident training state + the fused native step."""

    def __init__(self, layers: Sequence[int], batch_size: int, device, lr=1e-3, betas=(0.9, 0.999), eps=1e-8,
                 weight_decay=0.0, seed=0, process_group=None, world_size: int = 1):
        self.layout = FlatLayout(layers)
        self.device = torch.device(device)
        self.B = int(batch_size)
        self.lr, self.betas, self.eps, self.wd = lr, betas, eps, weight_decay
        self.pg = process_group
        self.world = world_size
        L = self.layout
        dev = self.device
        self.P = init_params(L, seed).to(dev)
        self.G = torch.zeros_like(self.P)
        self.m = torch.zeros_like(self.P)
        self.v = torch.zeros_like(self.P)
        self.step_count = torch.zeros(1, dtype=torch.int32, device=dev)
        self.native = self.device.type == "cuda"
        if self.native:
            self.Pb = self.P.to(torch.bfloat16)
            dims = [L.in_pad] + L.hidden
            self.acts = [None] + [torch.empty(self.B, h, dtype=torch.bfloat16, device=dev) for h in L.hidden]
            hmax = max(L.hidden) if L.hidden else HEAD_PAD
            self.dbuf = [torch.empty(self.B * hmax, dtype=torch.bfloat16, device=dev) for _ in range(2)]
            self.dlogits = torch.zeros(self.B, HEAD_PAD, dtype=torch.bfloat16, device=dev)
            nblk = _native.kernels().head_fused_blocks(self.B)
            self.block_loss = torch.zeros(nblk, dtype=torch.float32, device=dev)
            self.block_correct = torch.zeros(nblk, dtype=torch.int32, device=dev)
            self.dims = dims
            # deterministic split-K: every weight-grad GEMM splits the batch into the same
            # <= n_splits slices and writes plain partial tiles into slab z of a
            # [n_splits, total] workspace laid out like the flat parameter buffer.
            self.n_splits = n_splits_for(self.B)
            self.slabs = torch.zeros(self.n_splits, L.total, dtype=torch.float32, device=dev)
            self.n_groups = min(8, self.n_splits)  # two-level reduction: splits -> groups -> 1
            self.partials = torch.zeros(self.n_groups, L.total, dtype=torch.float32, device=dev)
            # one-kernel forward + head + dWout (mlp_fused.hip) for the 2-hidden-layer shapes it covers
            self.fused_ok = (len(L.hidden) == 2 and L.hidden[0] == L.hidden[1] and L.hidden[0] in (128, 256)
                             and L.in_pad in (32, 64) and L.num_classes <= 16
                             and os.environ.get("HAR_MLP_FUSED", "1") != "0")
            if self.fused_ok:
                nwg = _native.kernels().mlp_fwd_head_grid(self.B)
                self.fslab = torch.zeros(nwg, 16 * L.hidden[-1] + 16, dtype=torch.float32, device=dev)
                self.fblock_loss = torch.zeros(nwg, dtype=torch.float32, device=dev)
                self.fblock_correct = torch.zeros(nwg, dtype=torch.int32, device=dev)
            self.last_fused = False
            # fused layer-1 backward (mlp_fused.hip mlp_bwd_l1): dgrad -> relu' -> dW0 / db0 in one
            # kernel, dact1 never reaches HBM (H = 256, batch % 32; HAR_MLP_BWD_FUSED=0 keeps the GEMMs)
            self.bwd_ok = (self.fused_ok and L.hidden[0] == 256
                           and os.environ.get("HAR_MLP_BWD_FUSED", "1") != "0")
            if self.bwd_ok:
                nbw = _native.kernels().mlp_bwd_l1_grid(self.B)
                self.bslab = torch.zeros(nbw, 256 * L.in_pad + 256, dtype=torch.float32, device=dev)
            self.last_bwd = False
            # optional: the two backward branches after the fused forward — dW1 (split-K over the
            # batch) and dgrad -> dW0 — are independent, so HAR_MLP_STREAMS=1 runs dW1 on a second
            # HIP stream (fork/join with events; graph-capturable).  Measured on MI355X at batch
            # 65536: 0.147 vs 0.141 ms/step — both branches already fill every CU — so it is off.
            self.side = torch.cuda.Stream(dev) if os.environ.get("HAR_MLP_STREAMS", "0") == "1" else None
            self.ev_fork = torch.cuda.Event() if self.side is not None else None
            self.ev_join = torch.cuda.Event() if self.side is not None else None
        else:
            self.t_step = 0

    # ---------------------------------------------------------------- native
    def _w(self, flat, name):
        return self.layout.view(flat, name)

    def _slab(self, name):
        s = self.layout.by_name[name]
        return self.slabs.view(-1)[s.offset:]

    def forward_backward_native(self, Xb: torch.Tensor, y32: torch.Tensor, scale: float, on_grad=None):
        """Xb: [B, in_pad] bf16 (contiguous slice), y32: [B] int32.  Leaves the split-K
        gradient partials in ``self.slabs[:self.active_splits]``; ``on_grad(name)`` is called
        as soon as layer ``name``'s weight/bias gradient slabs are enqueued (DP bucketing)."""
        L, mod, s = self.layout, _native.kernels(), _native.stream_ptr()
        B = Xb.shape[0]
        if Xb.shape[1] != L.in_pad or Xb.dtype != torch.bfloat16 or B > self.B or y32.dtype != torch.int32:
            raise ValueError("bad batch")
        ks = max(128, ((B + self.n_splits - 1) // self.n_splits + 127) // 128 * 128)  # multiple of every BK
        self.active_splits = (B + ks - 1) // ks
        total = L.total
        nh = len(L.hidden)
        acts = [Xb] + [a[:B] for a in self.acts[1:]]
        if self.fused_ok and B % 16 == 0:
            return self._forward_backward_fused(Xb, y32, scale, on_grad, ks, acts)
        self.last_fused = False
        self.last_bwd = False
        for i in range(nh):
            gemm_bf16(acts[i], self._w(self.Pb, f"W{i}"), acts[i + 1], M=B, N=self.dims[i + 1], K=self.dims[i],
                      layout=0, epi=EPI_BIAS_RELU, bias=self._w(self.P, f"b{i}"),
                      tile=fwd_tile(B, self.dims[i + 1], self.dims[i]))
        last = acts[nh]
        if nh == 0:
            raise ValueError("the native MLP step needs at least one hidden layer")
        # fused head: CE loss, dlogits, and dact of the last hidden layer = (dlogits . Wout) * relu'
        dact = self.dbuf[(nh - 1) % 2][: B * self.dims[-1]].view(B, self.dims[-1])
        mod.head_fused(last.data_ptr(), self._w(self.Pb, "Wout").data_ptr(), self._w(self.P, "bout").data_ptr(),
                       y32.data_ptr(), B, self.dims[-1], L.num_classes, float(scale), self.dlogits.data_ptr(),
                       dact.data_ptr(), self.block_loss.data_ptr(), self.block_correct.data_ptr(), s)
        self.last_batch = B
        dl = self.dlogits[:B]
        # dWout = dlogits^T . last  (+ dbout = row sums of dlogits^T)
        gemm_bf16(dl, last, self._slab("Wout"), M=HEAD_PAD, N=self.dims[-1], K=B, layout=3, epi=EPI_F32_SLAB,
                  k_split=ks, ldc=self.dims[-1], slab_stride=total, rowsum=self._slab("bout"),
                  slab_stride_rowsum=total, tile=wgrad_tile(HEAD_PAD, self.dims[-1]))
        if on_grad is not None:
            on_grad("Wout")
        for i in reversed(range(nh)):
            h = self.dims[i + 1]
            # dW_i = dact^T . acts[i]   (+ db_i = row sums of dact^T)
            gemm_bf16(dact, acts[i], self._slab(f"W{i}"), M=h, N=self.dims[i], K=B, layout=3, epi=EPI_F32_SLAB,
                      k_split=ks, ldc=self.dims[i], slab_stride=total, rowsum=self._slab(f"b{i}"),
                      slab_stride_rowsum=total, tile=wgrad_tile(h, self.dims[i]))
            if on_grad is not None:
                on_grad(f"W{i}")
            if i > 0:
                # dact_{i-1} = (dact . W_i) * relu'(acts[i])
                hp = self.dims[i]
                prev = self.dbuf[(i - 1) % 2][: B * hp].view(B, hp)
                gemm_bf16(dact, self._w(self.Pb, f"W{i}"), prev, M=B, N=hp, K=h, layout=2, epi=EPI_RELU_GRAD,
                          mask=acts[i], tile=dgrad_tile(B, hp, h))
                dact = prev

    def _forward_backward_fused(self, Xb, y32, scale, on_grad, ks, acts):
        """2-hidden-layer step: ONE kernel for fwd L1 + fwd L2 + head + dWout/dbout (h2 and the
        logit gradients stay on chip), then dW1, dgrad and dW0 as split-K MFMA GEMMs."""
        L, mod, s = self.layout, _native.kernels(), _native.stream_ptr()
        B, H, K0 = Xb.shape[0], self.dims[-1], L.in_pad
        total = L.total
        h1 = acts[1]
        dact = self.dbuf[1][: B * H].view(B, H)
        self.fused_nwg = mod.mlp_fwd_head_grid(B)
        mod.mlp_fwd_head(Xb.data_ptr(), K0, self._w(self.Pb, "W0").data_ptr(), self._w(self.P, "b0").data_ptr(),
                         self._w(self.Pb, "W1").data_ptr(), self._w(self.P, "b1").data_ptr(), H,
                         self._w(self.Pb, "Wout").data_ptr(), self._w(self.P, "bout").data_ptr(), y32.data_ptr(),
                         B, L.num_classes, float(scale), h1.data_ptr(), dact.data_ptr(), self.fslab.data_ptr(),
                         self.fblock_loss.data_ptr(), self.fblock_correct.data_ptr(), s)
        self.last_fused = True
        self.last_batch = B
        if on_grad is not None:
            on_grad("Wout")

        def dw1():
            gemm_bf16(dact, h1, self._slab("W1"), M=H, N=H, K=B, layout=3, epi=EPI_F32_SLAB, k_split=ks, ldc=H,
                      slab_stride=total, rowsum=self._slab("b1"), slab_stride_rowsum=total, tile=wgrad_tile(H, H))

        prev = self.dbuf[0][: B * H].view(B, H)
        main = torch.cuda.current_stream(self.device)
        if self.side is not None:  # fork: dW1 (+ its DP bucket) on the side stream, dgrad -> dW0 here
            self.ev_fork.record(main)
            self.side.wait_event(self.ev_fork)
            with torch.cuda.stream(self.side):
                dw1()
                if on_grad is not None:
                    on_grad("W1")  # DP: the W1 bucket's slab reduction + async all-reduce start here
                self.ev_join.record(self.side)
        else:
            dw1()
            if on_grad is not None:
                on_grad("W1")
        if self.bwd_ok and B % 32 == 0:  # dact1 stays on chip: dgrad + relu' + dW0 / db0 in one kernel
            self.bwd_nwg = mod.mlp_bwd_l1_grid(B)
            mod.mlp_bwd_l1(dact.data_ptr(), h1.data_ptr(), Xb.data_ptr(), K0, self._w(self.Pb, "W1").data_ptr(), H,
                           B, self.bslab.data_ptr(), s)
            self.last_bwd = True
        else:
            self.last_bwd = False
            gemm_bf16(dact, self._w(self.Pb, "W1"), prev, M=B, N=H, K=H, layout=2, epi=EPI_RELU_GRAD, mask=h1,
                      tile=dgrad_tile(B, H, H))
            gemm_bf16(prev, Xb, self._slab("W0"), M=H, N=K0, K=B, layout=3, epi=EPI_F32_SLAB, k_split=ks, ldc=K0,
                      slab_stride=total, rowsum=self._slab("b0"), slab_stride_rowsum=total, tile=wgrad_tile(H, K0))
        if on_grad is not None:
            on_grad("W0")
        if self.side is not None:  # join: the W1 slabs (and the next step's h1 / dact2 reuse) are ordered
            main.wait_event(self.ev_join)

    def _first_level(self, lo: int, hi: int, tick: bool):
        """First reduction level of G[lo:hi] into ``n_groups`` partials in ONE launch (one grid.z
        segment per source region): the split-K GEMM slabs, and after a fused step the fused
        kernels' per-workgroup slabs (dWout / dbout of the forward kernel, dW0 / db0 of the
        layer-1 backward kernel); optionally ticks the Adam step counter."""
        mod, st, L = _native.kernels(), _native.stream_ptr(), self.layout
        total = L.total
        regions = []  # (start, end, source pointer at start, #slabs, slab stride) in flat order
        start = 0
        if self.last_bwd:
            w0, b0 = L.by_name["W0"], L.by_name["b0"]
            bs, ldb = self.bslab.data_ptr(), self.bslab.shape[1]
            regions.append((w0.offset, w0.offset + w0.numel, bs, self.bwd_nwg, ldb))
            regions.append((b0.offset, b0.offset + b0.numel, bs + 4 * w0.numel, self.bwd_nwg, ldb))
            start = L.by_name["W1"].offset
        end = L.by_name["Wout"].offset if self.last_fused else total
        regions.append((start, end, self.slabs.data_ptr() + 4 * start, self.active_splits, total))
        if self.last_fused:
            H = self.dims[-1]
            fs, w = self.fslab.data_ptr(), self.fslab.shape[1]
            wo, bo = L.by_name["Wout"].offset, L.by_name["bout"].offset
            regions.append((wo, wo + 16 * H, fs, self.fused_nwg, w))
            regions.append((bo, bo + 16, fs + 4 * 16 * H, self.fused_nwg, w))
        pbase = self.partials.data_ptr()
        segs = []  # (slabs ptr, S, n, lds, dst ptr, ldd)
        for a, b, ptr, S, lds in regions:
            a2, b2 = max(a, lo), min(b, hi)
            if a2 < b2:
                segs.append((ptr + 4 * (a2 - a), S, b2 - a2, lds, pbase + 4 * a2, total))
        cols = list(zip(*segs))
        mod.reduce_slabs_multi(list(cols[0]), list(cols[1]), list(cols[2]), list(cols[3]), list(cols[4]),
                               list(cols[5]), self.n_groups, self.step_count.data_ptr() if tick else 0, st)

    def _reduce_to_partials(self):
        # the first reduction level also ticks the Adam step counter (one launch fewer per step)
        self._first_level(0, self.layout.total, True)

    def reduce_grads_native(self):
        """G = sum of the active gradient slabs (two deterministic levels; needed before a collective)."""
        self._reduce_to_partials()
        _native.kernels().reduce_slabs_grouped(self.partials.data_ptr(), self.n_groups, self.layout.total,
                                               self.G.data_ptr(), 1, _native.stream_ptr(), 0)

    def _layer_range(self, name):
        """[lo, hi) of layer ``name``'s weight + bias in the flat buffers."""
        L = self.layout
        k = L.segments.index(L.by_name[name])
        return L.segments[k].offset, (L.segments[k + 2].offset if k + 2 < len(L.segments) else L.total)

    def _reduce_range(self, lo: int, hi: int, tick: bool):
        """Two-level slab reduction of G[lo:hi] only (same summation order as the whole-buffer one)."""
        mod, st, total = _native.kernels(), _native.stream_ptr(), self.layout.total
        self._first_level(lo, hi, tick)
        mod.reduce_slabs_grouped(self.partials.data_ptr() + 4 * lo, self.n_groups, hi - lo, self.G.data_ptr() + 4 * lo,
                                 1, st, 0, lds=total, ldd=hi - lo)

    def train_step_overlapped(self, Xb: torch.Tensor, yb: torch.Tensor, global_batch: int,
                              bucket_bytes: int = 64 << 10):
        """DP step with the gradient all-reduce bucketed and overlapped with backward: as soon
        as the layers finished so far hold >= ``bucket_bytes`` of gradient, their slabs are
        reduced and an async RCCL all-reduce of that contiguous slice of G starts on the
        communicator's stream while the remaining dgrad/wgrad GEMMs run; Adam waits for all
        buckets.  Layers finish in reverse order, so every bucket is one contiguous range."""
        import torch.distributed as dist

        works, pend = [], []

        def flush():
            lo, hi = pend[-1][0], pend[0][1]
            self._reduce_range(lo, hi, tick=not works)
            works.append(dist.all_reduce(self.G[lo:hi], group=self.pg, async_op=True))
            pend.clear()

        def on_grad(name):
            pend.append(self._layer_range(name))
            if (pend[0][1] - pend[-1][0]) * 4 >= bucket_bytes or name == "W0":
                flush()

        self.forward_backward_native(Xb, yb, 1.0 / global_batch, on_grad=on_grad)
        for w in works:
            w.wait()  # stream-ordered: the compute stream waits on the RCCL stream, the host does not
        self.optimizer_step_native(from_slabs=False)

    def optimizer_step_native(self, from_slabs: bool):
        """Adam; with ``from_slabs`` the slabs are first reduced to ``n_groups`` partials and the
        last level of the reduction is fused into the Adam kernel."""
        b1, b2 = self.betas
        if from_slabs:
            self._reduce_to_partials()  # ticks the step counter
        _native.kernels().adam_step(self.P.data_ptr(), self.G.data_ptr(),
                                    self.partials.data_ptr() if from_slabs else 0, self.n_groups,
                                    self.m.data_ptr(), self.v.data_ptr(), self.Pb.data_ptr(), self.P.numel(),
                                    float(self.lr), b1, b2, float(self.eps), float(self.wd), 1.0,
                                    self.step_count.data_ptr(), _native.stream_ptr(), 0)

    def allreduce_grads(self):
        if self.world > 1:
            import torch.distributed as dist
            dist.all_reduce(self.G, group=self.pg)

    def grad_phase(self, Xb: torch.Tensor, yb: torch.Tensor, global_batch: int):
        """DP step, part 1 (graph-capturable): fwd + bwd + deterministic slab reduction into G."""
        self.forward_backward_native(Xb, yb, 1.0 / global_batch)
        self.reduce_grads_native()

    def apply_phase(self):
        """DP step, part 3 (graph-capturable): Adam from the all-reduced G (part 2 is the RCCL
        all-reduce, issued eagerly between the two graph replays)."""
        self.optimizer_step_native(from_slabs=False)

    def train_step(self, Xb: torch.Tensor, yb: torch.Tensor, global_batch: int):
        if self.native:
            if self.world > 1:
                self.train_step_overlapped(Xb, yb, global_batch)
            else:  # single GPU: the slab reduction is fused into Adam
                self.forward_backward_native(Xb, yb, 1.0 / global_batch)
                self.optimizer_step_native(from_slabs=True)
        else:
            self.train_step_torch(Xb, yb, global_batch)

    def state_tensors(self):
        """Everything needed to resume training bit-for-bit."""
        step = self.step_count.clone() if self.native else torch.tensor([self.t_step], dtype=torch.int32)
        return {"P": self.P, "m": self.m, "v": self.v, "step": step}

    def load_state(self, st):
        self.P.copy_(st["P"].to(self.P.device))
        self.m.copy_(st["m"].to(self.m.device))
        self.v.copy_(st["v"].to(self.v.device))
        if self.native:
            self.step_count.copy_(st["step"].to(self.step_count.device))
            self.Pb.copy_(self.P.to(torch.bfloat16))
        else:
            self.t_step = int(st["step"][0])

    def last_loss_and_correct(self):
        """(sum of CE, #correct) of the last native batch — one host sync."""
        if self.last_fused:
            n = self.fused_nwg
            return float(self.fblock_loss[:n].sum().item()), int(self.fblock_correct[:n].sum().item())
        return float(self.block_loss.sum().item()), int(self.block_correct.sum().item())

    # ---------------------------------------------------------------- torch
    def torch_forward(self, P: torch.Tensor, X: torch.Tensor):
        L = self.layout
        h = X
        if h.shape[1] < L.in_pad:
            h = torch.nn.functional.pad(h, (0, L.in_pad - h.shape[1]))
        for i in range(len(L.hidden)):
            h = torch.relu(h @ L.view(P, f"W{i}").T + L.view(P, f"b{i}"))
        z = h @ L.view(P, "Wout")[: L.num_classes].T + L.view(P, "bout")[: L.num_classes]
        return z

    def train_step_torch(self, X: torch.Tensor, y: torch.Tensor, global_batch: int):
        """fp32 reference step (CPU path / oracle); same Adam math as the kernel."""
        P = self.P.detach().requires_grad_(True)
        z = self.torch_forward(P, X.float())
        loss = torch.nn.functional.cross_entropy(z, y.long(), reduction="sum") / global_batch
        (g,) = torch.autograd.grad(loss, P)
        self.G.copy_(g)
        self.allreduce_grads()
        self.t_step += 1
        b1, b2 = self.betas
        with torch.no_grad():
            self.m.mul_(b1).add_((1 - b1) * self.G)
            self.v.mul_(b2).add_((1 - b2) * self.G * self.G)
            upd = (self.m / (1 - b1 ** self.t_step)) / ((self.v / (1 - b2 ** self.t_step)).sqrt() + self.eps)
            self.P.sub_(self.lr * (upd + self.wd * self.P))
        self.last_loss = float(loss.detach()) * global_batch / X.shape[0]

    # ---------------------------------------------------------------- inference
    def infer_fused(self, Xb: torch.Tensor):
        """Serving path: ONE fused kernel (mlp_fused.hip, INFER variant) per call — logits
        [B, C] fp32 and the argmax class [B] int32 from padded bf16 inputs."""
        L = self.layout
        B = Xb.shape[0]
        if not (self.fused_ok and B % 16 == 0 and Xb.dtype == torch.bfloat16 and Xb.shape[1] == L.in_pad):
            raise ValueError("infer_fused: unsupported shape")
        out = torch.empty(B, L.num_classes, dtype=torch.float32, device=Xb.device)
        pred = torch.empty(B, dtype=torch.int32, device=Xb.device)
        _native.kernels().mlp_fwd_infer(Xb.data_ptr(), L.in_pad, self._w(self.Pb, "W0").data_ptr(),
                                        self._w(self.P, "b0").data_ptr(), self._w(self.Pb, "W1").data_ptr(),
                                        self._w(self.P, "b1").data_ptr(), self.dims[-1],
                                        self._w(self.Pb, "Wout").data_ptr(), self._w(self.P, "bout").data_ptr(), B,
                                        L.num_classes, out.data_ptr(), pred.data_ptr(), _native.stream_ptr())
        return out, pred

    def infer_fused_f32(self, X: torch.Tensor):
        """Serving from raw fp32 features [B, F] (row stride >= F): ONE kernel, the bf16 cast
        and zero padding happen in its loads.  Returns (logits [B, C] fp32, argmax [B] int32)."""
        L = self.layout
        B, F = X.shape
        if not (self.fused_ok and B % 16 == 0 and X.dtype == torch.float32 and X.stride(1) == 1 and F <= L.in_pad):
            raise ValueError("infer_fused_f32: unsupported shape")
        out = torch.empty(B, L.num_classes, dtype=torch.float32, device=X.device)
        pred = torch.empty(B, dtype=torch.int32, device=X.device)
        _native.kernels().mlp_fwd_infer_f32(X.data_ptr(), X.stride(0), F, L.in_pad, self._w(self.Pb, "W0").data_ptr(),
                                            self._w(self.P, "b0").data_ptr(), self._w(self.Pb, "W1").data_ptr(),
                                            self._w(self.P, "b1").data_ptr(), self.dims[-1],
                                            self._w(self.Pb, "Wout").data_ptr(), self._w(self.P, "bout").data_ptr(),
                                            B, L.num_classes, out.data_ptr(), pred.data_ptr(), _native.stream_ptr())
        return out, pred

    def logits(self, X: torch.Tensor) -> torch.Tensor:
        L = self.layout
        if self.native and X.is_cuda:
            if self.fused_ok and X.shape[0] % 16 == 0 and X.dtype == torch.float32 and X.stride(1) == 1:
                return self.infer_fused_f32(X)[0]
            Xb = pad_input_bf16(X, L.in_pad)
            if self.fused_ok and X.shape[0] % 16 == 0:
                return self.infer_fused(Xb)[0]
            out = torch.empty(X.shape[0], L.num_classes, dtype=torch.float32, device=X.device)
            for r0 in range(0, X.shape[0], self.B):
                r1 = min(X.shape[0], r0 + self.B)
                B = r1 - r0
                acts = [Xb[r0:r1]] + [a[:B] for a in self.acts[1:]]
                for i in range(len(L.hidden)):
                    gemm_bf16(acts[i], self._w(self.Pb, f"W{i}"), acts[i + 1], M=B, N=self.dims[i + 1],
                              K=self.dims[i], layout=0, epi=EPI_BIAS_RELU, bias=self._w(self.P, f"b{i}"))
                _native.kernels().softmax_ce_head(acts[-1].data_ptr(), self._w(self.Pb, "Wout").data_ptr(),
                                                  self._w(self.P, "bout").data_ptr(), 0, B, self.dims[-1],
                                                  L.num_classes, 1.0, 0, 0, 0, out[r0:r1].data_ptr(),
                                                  _native.stream_ptr())
            return out
        Xp = torch.zeros(X.shape[0], L.in_pad, dtype=torch.float32, device=X.device)
        Xp[:, : X.shape[1]] = X
        with torch.no_grad():
            return self.torch_forward(self.P.to(X.device), Xp)


def pad_input_bf16(X: torch.Tensor, in_pad: int) -> torch.Tensor:
    """[N, F] fp32 -> [N, in_pad] bf16 (zero padded), on device via the HIP cast kernel."""
    X = X.contiguous().float()
    out = torch.empty(X.shape[0], in_pad, dtype=torch.bfloat16, device=X.device)
    if X.is_cuda:
        _native.kernels().cast_pad_bf16(X.data_ptr(), X.shape[0], X.shape[1], X.stride(0), out.data_ptr(), in_pad,
                                        _native.stream_ptr())
    else:
        out.zero_()
        out[:, : X.shape[1]] = X.to(torch.bfloat16)
    return out


class MultilayerPerceptronClassificationModel(ClassificationModel):
    def __init__(self, engine: MLPEngine, uid=None):
        super().__init__(uid or new_uid("MultilayerPerceptronClassifier"))
        self.engine = engine
        self.layers = engine.layout.layers
        self.num_classes = engine.layout.num_classes
        self.num_features = engine.layout.layers[0]
        self.device = engine.device
        self.mean = None
        self.inv_std = None

    def _prep(self, X):
        if self.mean is not None:
            X = (X - self.mean.to(X.device)) * self.inv_std.to(X.device)
        return X

    def predict_raw(self, X: torch.Tensor) -> torch.Tensor:
        return self.engine.logits(self._prep(X.to(self.device)))

    def raw_to_probability(self, raw):
        return torch.softmax(raw, dim=1)

    def __str__(self):
        return f"MultilayerPerceptronClassificationModel (uid={self.uid}) with {len(self.layers)} layers"

    def state(self):
        return {"layers": self.layers, "params": self.engine.P.cpu(), "mean": self.mean, "inv_std": self.inv_std}


class MultilayerPerceptronClassifier(Estimator, ClassifierParams):
    """``layers=[in, h1, ..., out]``; ``maxIter`` = epochs; ``blockSize`` = per-rank batch."""

    _param_names = ("layers", "maxIter", "blockSize", "stepSize", "seed", "standardize", "device", "weightDecay",
                    "checkpointDir", "checkpointInterval")

    def __init__(self, layers: Optional[Sequence[int]] = None, maxIter: int = 100, blockSize: int = 1024,
                 stepSize: float = 1e-3, seed: int = 0, standardize: bool = True, featuresCol="features",
                 labelCol="label", device=None, weightDecay: float = 0.0, checkpointDir: Optional[str] = None,
                 checkpointInterval: int = 0):
        super().__init__(new_uid("MultilayerPerceptronClassifier"))
        self.layers = list(layers) if layers else None
        self.maxIter, self.blockSize, self.stepSize, self.seed = maxIter, blockSize, stepSize, seed
        self.standardize, self.featuresCol, self.labelCol, self.device = standardize, featuresCol, labelCol, device
        self.weightDecay = weightDecay
        self.checkpointDir, self.checkpointInterval = checkpointDir, checkpointInterval

    def fit(self, table: Table) -> MultilayerPerceptronClassificationModel:
        dev = resolve_device(self.device)
        X = features_tensor(table, self.featuresCol, dev)
        y = labels_tensor(table, self.labelCol, dev)
        vocab = (table[self.labelCol].meta or {}).get("vocab")
        K = int(max(int(y.max()) + 1, len(vocab) if vocab else 0))
        ctx = dp_context()
        if ctx is None:
            return self.fit_tensors(X, y, num_classes=K)
        lo, hi = dp_rows(X.shape[0])  # data parallel: row shard, gradients all-reduced every step
        return self.fit_tensors(X[lo:hi], y[lo:hi], process_group=ctx.group, rank=ctx.rank,
                                world_size=ctx.world_size, num_classes=K)

    def fit_tensors(self, X: torch.Tensor, y: torch.Tensor, process_group=None, rank: int = 0,
                    world_size: int = 1, num_classes: Optional[int] = None) -> MultilayerPerceptronClassificationModel:
        """DP-ready fit: every rank passes its own shard (X, y); the standardization
        statistics, the class count and the steps per epoch are agreed over the group
        and the gradients are all-reduced every step."""
        dev = X.device
        K = int(num_classes) if num_classes else int(y.max()) + 1
        if world_size > 1 and not num_classes:
            import torch.distributed as dist
            kt = torch.tensor([K], device=dev)
            dist.all_reduce(kt, op=dist.ReduceOp.MAX, group=process_group)
            K = int(kt.item())
        layers = self.layers or [X.shape[1], 128, 128, K]
        if layers[0] != X.shape[1]:
            raise ValueError(f"layers[0]={layers[0]} but features have {X.shape[1]} columns")
        mean = inv_std = None
        if self.standardize:
            n = torch.tensor([float(X.shape[0])], device=dev, dtype=torch.float64)
            s1 = X.double().sum(0)
            s2 = (X.double() ** 2).sum(0)
            if world_size > 1:
                import torch.distributed as dist
                buf = torch.cat([n, s1, s2])
                dist.all_reduce(buf, group=process_group)
                n, s1, s2 = buf[:1], buf[1:1 + X.shape[1]], buf[1 + X.shape[1]:]
            mean = (s1 / n).float()
            var = (s2 / n - (s1 / n) ** 2).clamp_min(0).float()
            inv_std = torch.where(var > 0, 1.0 / var.sqrt(), torch.zeros_like(var))
            X = (X - mean) * inv_std
        B = min(self.blockSize, X.shape[0])
        if world_size > 1:  # every rank must run the same number of steps (collectives!)
            import torch.distributed as dist
            bt = torch.tensor([B], device=dev)
            dist.all_reduce(bt, op=dist.ReduceOp.MIN, group=process_group)
            B = int(bt.item())
        eng = MLPEngine(layers, B, dev, lr=self.stepSize, seed=self.seed, process_group=process_group,
                        world_size=world_size, weight_decay=self.weightDecay)
        N = X.shape[0]
        Xin = pad_input_bf16(X, eng.layout.in_pad) if eng.native else X
        y32 = y.to(torch.int32).contiguous()
        global_batch = B * world_size
        steps_per_epoch = max(1, N // B)
        if world_size > 1:
            import torch.distributed as dist
            st = torch.tensor([steps_per_epoch], device=dev)
            dist.all_reduce(st, op=dist.ReduceOp.MIN, group=process_group)
            steps_per_epoch = int(st.item())
        ckpt = None
        start_epoch, start_step = 0, 0
        if self.checkpointDir:
            from ..utils.checkpoint import Checkpointer

            ckpt = Checkpointer(self.checkpointDir, rank=rank)
            fp = {"layers": list(layers), "seed": self.seed, "batch": B, "world_size": world_size,
                  "stepSize": self.stepSize, "weightDecay": self.weightDecay, "rows": int(N),
                  "steps_per_epoch": steps_per_epoch, "standardize": bool(self.standardize)}
            last = ckpt.latest(fingerprint=fp)
            if last is not None:  # resume: parameters, Adam moments, step counter, data position
                state, meta = last
                eng.load_state(state)
                start_epoch, start_step = int(meta["epoch"]), int(meta["step_in_epoch"])
        from ..utils.checkpoint import maybe_inject_fault

        for epoch in range(start_epoch, self.maxIter):
            # data order is a pure function of (seed, rank, epoch): resumable without RNG state
            g = torch.Generator(device="cpu").manual_seed(self.seed + 7919 * rank + 104729 * epoch)
            perm = torch.randperm(N, generator=g).to(dev)
            Xe, ye = Xin[perm].contiguous(), y32[perm].contiguous()
            for s in range(start_step if epoch == start_epoch else 0, steps_per_epoch):
                gstep = epoch * steps_per_epoch + s
                maybe_inject_fault(gstep, rank)
                eng.train_step(Xe[s * B:(s + 1) * B], ye[s * B:(s + 1) * B], global_batch)
                if ckpt is not None and self.checkpointInterval and (gstep + 1) % self.checkpointInterval == 0:
                    nxt_e, nxt_s = (epoch, s + 1) if s + 1 < steps_per_epoch else (epoch + 1, 0)
                    ckpt.save(gstep + 1, eng.state_tensors(), {"epoch": nxt_e, "step_in_epoch": nxt_s},
                              fingerprint=fp)
        model = MultilayerPerceptronClassificationModel(eng, uid=self.uid)
        model.mean, model.inv_std = mean, inv_std
        return model
