"""Batched multinomial logistic-regression objective + device L-BFGS (kernels K8-K10).

For B models with effective weights ``W [B, K, F]`` and intercepts ``b [B, K]``
over one resident feature matrix ``X [N, F]``:

    Z   = X . W^T + b
    P   = softmax over each model's K columns
    R   = rw[b, i] / sum_i rw[b, i] * (P - onehot(y))
    loss[b] = sum_i rw[b,i] * CE_i / sum_i rw[b,i]
    dW  = R^T . X ,   db = sum_i R

``rw`` carries the per-model row weights (fold membership in CrossValidator,
Spark's instance weights otherwise), so 45 CV fits share one evaluation.

GPU path (gfx950, csrc/kernels/logreg_qn.hip + logreg_setup.hip): the features stay in
the HYBRID layout (one-hot index blocks + dense columns of any width, staged through LDS
in 32-column chunks); the summarizer, the standardization / masks / regularization
vectors, the CSC slice index of the gradient kernel and every L-BFGS / OWL-QN phase are
HIP kernels — a fit enqueues with no host synchronization.  Data parallel: ONE fp32
all-reduce per evaluation carries the gradient bucket and the exact (fixed-point) losses.
CPU path: the same math in PyTorch (test oracle).
"""
from __future__ import annotations

import os

from typing import Optional

import torch

from . import _native

SLICE_ROWS = int(os.environ.get("HAR_LR_SL", "16"))  # rows per CSC slice of the gradient / summary kernels (16: profiles/r5/lr_grad_blocks.md)


def logreg_loss_grad_torch(X, y, W, b, rw, inv_wsum):
    B, K, F = W.shape
    Z = X @ W.reshape(B * K, F).T + b.reshape(1, B * K)           # [N, B*K]
    Z = Z.view(-1, B, K)
    lse = torch.logsumexp(Z, dim=2)                                  # [N, B]
    zy = Z.gather(2, y.view(-1, 1, 1).expand(-1, B, 1)).squeeze(2)   # [N, B]
    wn = rw.T * inv_wsum.view(1, B)                                  # [N, B]
    loss = ((lse - zy) * wn).sum(dim=0)
    P = torch.softmax(Z, dim=2)
    P.scatter_add_(2, y.view(-1, 1, 1).expand(-1, B, 1), -torch.ones_like(P[:, :, :1]))
    R = P * wn.unsqueeze(2)                                          # [N, B, K]
    gW = (R.reshape(-1, B * K).T @ X).view(B, K, F)
    gb = R.sum(dim=0)
    return loss, gW, gb


# ------------------------------------------------------------------------------------------
# Hybrid-layout objective + device L-BFGS (csrc/kernels/logreg_qn.hip)
# ------------------------------------------------------------------------------------------
LOSS_FX = float(2 ** 40)


def pack_bucket(G: torch.Tensor, loss: torch.Tensor) -> torch.Tensor:
    """[gradients (fp32) | each loss as 2^-40 fixed point in four 16-bit pieces + a non-finite
    flag (fp32 integers)]: the data-parallel all-reduce bucket of one evaluation.  Summing the
    pieces in fp32 is exact (|sum| < 2^24), so ``unpack_bucket`` returns the exact sum of the
    ranks' fixed-point losses — the torch twin of logreg_qn.hip's loss_encode / loss_decode."""
    ld = loss.double()
    bad = ~(ld.abs() < 8388608.0)
    q = torch.round(torch.where(bad, torch.zeros_like(ld), ld) * LOSS_FX).to(torch.int64)
    pieces = [q & 0xffff, (q >> 16) & 0xffff, (q >> 32) & 0xffff, q >> 48, bad.to(torch.int64)]
    enc = torch.stack(pieces, 1).to(torch.float32)
    return torch.cat([G.reshape(-1).float(), enc.reshape(-1)])


def unpack_bucket(bucket: torch.Tensor, n_loss: int, g_shape):
    n = bucket.numel() - 5 * n_loss
    enc = bucket[n:].view(n_loss, 5).to(torch.int64)
    q = enc[:, 0] + (enc[:, 1] << 16) + (enc[:, 2] << 32) + (enc[:, 3] << 48)
    loss = q.double() / LOSS_FX
    loss = torch.where(enc[:, 4] != 0, torch.full_like(loss, float("nan")), loss)
    return bucket[:n].view(g_shape), loss


MAX_NATIVE_CLASSES = 16  # class rows of the logreg_qn.hip kernels (KP = 8 / 16)


def _kp(K: int) -> int:
    return 8 if K <= 8 else 16


def native_classes_ok(K: int) -> bool:
    """True when the device LR kernels take K classes; wider fits use the torch objective on the
    same device (dense GEMMs) with the same L-BFGS / OWL-QN algorithm (optim/lbfgs.py)."""
    return K <= MAX_NATIVE_CLASSES


def hybrid_index(hm):
    """(CSC offsets [F+2], CSC rows, column map [F+1]) of a hybrid matrix, cached on it: derived from
    the resident (immutable) features, so every fit / CV fold / evaluation over the same matrix
    reuses one index (one sort per dataset, not per fit)."""
    idx = getattr(hm, "_lr_index", None)
    if idx is None:
        off, rows = hm.csc()
        if rows.numel() == 0:
            rows = torch.zeros(1, dtype=torch.int32, device=hm.device)
        idx = (off, rows, hm.col_map())
        hm._lr_index = idx
    return idx


class LogregDesign:
    """Device data of one fit: the hybrid feature layout, labels, per-spec row weights, the
    one-hot CSC row lists (+ their row slices) and the column map of the gradient kernel."""

    def __init__(self, hm, y: torch.Tensor, rw, K: int, native: Optional[bool] = None):
        self.hm = hm
        # the HIP kernels serve this design (GPU, <= 16 classes); else the torch objective on its device
        self.native = (hm.device.type == "cuda" and native_classes_ok(K)) if native is None else bool(native)
        self.N, self.F = hm.n_rows, hm.n_features
        self.Fd, self.C = int(hm.dense.shape[1]), int(hm.cat.shape[1])
        self.K = K
        self.KP = _kp(K)
        self.y32 = y.to(torch.int32).contiguous()
        # [S, N] float32 row weights, or None (every spec unweighted: the kernels read 1)
        self.rw = None if rw is None else rw.float().contiguous()
        self.S = 1 if rw is None else int(rw.shape[0])
        self.csc_off, self.csc_rows, self.col_map = hybrid_index(hm)
        self.dense = hm.dense if self.Fd else torch.zeros(max(1, self.N), 1, device=hm.device)
        self.dense_cols = hm.dense_cols if self.Fd else torch.zeros(1, dtype=torch.int32, device=hm.device)
        self.cat = hm.cat if self.C else torch.zeros(max(1, self.N), 1, dtype=torch.int32, device=hm.device)
        self.SL = SLICE_ROWS
        self._col_slice = getattr(hm, "_lr_col_slice", None)  # cached on the (immutable) matrix

    @property
    def device(self):
        return self.hm.device

    def col_slice(self) -> torch.Tensor:
        """[F+2] int32: first CSC row slice (of SL rows) of every column — the work index of the
        gradient and summary kernels, built on the device (no host read)."""
        if self._col_slice is None:
            F = self.F
            if self.device.type == "cuda":
                cs = torch.empty(F + 2, dtype=torch.int32, device=self.device)
                _native.kernels().logreg_col_slices(self.csc_off.data_ptr(), F, self.SL, cs.data_ptr(),
                                                    _native.stream_ptr())
            else:
                L = (self.csc_off[1:].long() - self.csc_off[:-1].long())
                ns = (L + self.SL - 1) // self.SL
                cs = torch.zeros(F + 2, dtype=torch.int64)
                cs[1:] = torch.cumsum(ns, 0)
                cs = cs.to(torch.int32)
            self._col_slice = self.hm._lr_col_slice = cs
        return self._col_slice

    def col_blocks(self):
        """(blk, nblk, srow) of the gradient kernel: consecutive column blocks of at most 256 columns
        and 256 CSC row slices each (a lone column with more slices takes a block of its own) as
        [nblk][4] int32 (c0, c1, first slice, end slice), and srow [slices + 1] = the first CSC row of
        every slice (the row lists are contiguous across columns, so slice sl covers rows
        [srow[sl], srow[sl + 1])).  The kernel then loads everything a lane needs in one round at
        entry instead of searching the slice's column and reading its offsets (grad stamps,
        profiles/r5/lr_kernel_medians.md).  A column's slices are still summed in order by one lane:
        the gradient is bitwise the fixed-block one.  Built once per matrix (one host read of
        col_slice, cached on it); HAR_LR_COLBLK=0 keeps the fixed 256-column blocks."""
        if os.environ.get("HAR_LR_COLBLK", "1") == "0" or self.device.type != "cuda":
            return None, 0, None
        cached = getattr(self.hm, "_lr_col_blk", None)
        if cached is None or cached[3] != self.SL:
            F1 = self.F + 1
            cs = self.col_slice()[:F1 + 1].long()
            csh = cs.cpu().tolist()
            bounds, c0, sl = [0], 0, 0
            for c in range(F1):
                n = csh[c + 1] - csh[c]
                if c > c0 and (c - c0 == 256 or sl + n > 256):
                    bounds.append(c)
                    c0, sl = c, 0
                sl += n
            bounds.append(F1)
            blk = [(bounds[i], bounds[i + 1], csh[bounds[i]], csh[bounds[i + 1]]) for i in range(len(bounds) - 1)]
            blk_t = torch.tensor(blk, dtype=torch.int32, device=self.device).contiguous()
            total = csh[F1]
            off = self.csc_off.long()
            ns = cs[1:] - cs[:-1]
            col_of = torch.repeat_interleave(torch.arange(F1, device=self.device), ns)
            j = torch.arange(total, device=self.device) - cs[col_of]
            srow = torch.empty(total + 1, dtype=torch.int32, device=self.device)
            srow[:total] = (off[col_of] + j * self.SL).to(torch.int32)
            srow[total] = off[F1].to(torch.int32)
            cached = (blk_t, len(blk), srow, self.SL)
            self.hm._lr_col_blk = cached
        return cached[0], cached[1], cached[2]

    def rw_ptr(self) -> int:
        return 0 if self.rw is None else self.rw.data_ptr()

    def rw_rows(self) -> torch.Tensor:
        """[S, N] row weights (materialized ones when unweighted; CPU oracle only)."""
        if self.rw is None:
            return torch.ones(self.S, self.N, device=self.device)
        return self.rw

    def summary(self):
        """Weighted summarizer per spec (Spark MultivariateOnlineSummarizer + MultiClassSummarizer):
        [S, 1 + 2F + K] float64 = (sum w, sum w x, sum w x^2, class counts).  GPU: two HIP kernels
        (logreg_setup.hip: per-tile fp64 partials of the dense columns + class sums, then one lane
        per column: tile partials in order / w over the CSC row slices of a one-hot column).
        CPU: one-hot columns are segment sums over their CSC rows (fp64 scan), dense columns one
        fp64 product.  Every sum in a fixed order."""
        S_, N, F, K = self.S, self.N, self.F, self.K
        dev = self.device
        if self.native:
            mod, st = _native.kernels(), _native.stream_ptr()
            sb = getattr(self, "_summary_bufs", None)
            if sb is None:  # (a design reused by the solver cache keeps its summary buffers: no allocations)
                nt = mod.logreg_summary_tiles(N)
                sb = self._summary_bufs = (nt, torch.empty(S_, max(1, nt), 2 * self.Fd + K + 1, dtype=torch.float64,
                                                           device=dev))
            nt, part = sb
            # (a fresh output per call: callers keep it, e.g. expanded into the prepare kernel's input)
            out = torch.empty(S_, 1 + 2 * F + K, dtype=torch.float64, device=dev)
            cs = self.col_slice()
            srow = self.col_blocks()[2]
            for ph in (0, 1):
                mod.logreg_summary(ph, self.dense.data_ptr(), self.dense.stride(0), self.Fd, self.y32.data_ptr(),
                                   self.rw_ptr(), N, F, K, S_, self.col_map.data_ptr(), self.csc_rows.data_ptr(),
                                   self.csc_off.data_ptr(), cs.data_ptr(), self.SL, nt, part.data_ptr(),
                                   out.data_ptr(), 0 if srow is None else srow.data_ptr(), st)
            return out
        rwd = self.rw_rows().double()
        out = torch.zeros(S_, 1 + 2 * F + K, dtype=torch.float64, device=dev)
        out[:, 0] = rwd.sum(1)
        if self.C:
            off = self.csc_off.long()
            n = int(off[-1])
            cs = torch.zeros(S_, n + 1, dtype=torch.float64, device=dev)
            if n:
                cs[:, 1:] = torch.cumsum(rwd[:, self.csc_rows[:n].long()], dim=1)
            seg = cs[:, off[1:F + 1]] - cs[:, off[:F]]            # [S, F]
            out[:, 1:1 + F] += seg
            out[:, 1 + F:1 + 2 * F] += seg
        if self.Fd:
            Xd = self.hm.dense.double()
            cols = self.hm.dense_cols.long()
            out[:, 1 + cols] = rwd @ Xd
            out[:, 1 + F + cols] = rwd @ (Xd * Xd)
        out[:, 1 + 2 * F:] = rwd @ torch.nn.functional.one_hot(self.y32.long(), K).double()
        return out

    # ---- torch reference objective (CPU oracle and non-GPU path) ----
    def eval_torch(self, xt: torch.Tensor, T: int, inv_std: torch.Tensor, pmask: torch.Tensor,
                   inv_wsum: torch.Tensor):
        """xt [S*T, K, F+1] -> (data loss [S*T] float64, data grad [S*T, K*(F+1)] masked, scaled)."""
        BT = xt.shape[0]
        F, K = self.F, self.K
        spec = torch.arange(BT, device=xt.device) // T
        Weff = xt[:, :, :F] * inv_std[spec][:, None, :] * pmask[spec][:, :, :F]
        b = xt[:, :, F] * pmask[spec][:, :, F]
        if getattr(self, "_X", None) is None:
            self._X = self.hm.to_dense()
        X = self._X.to(xt.dtype)
        rw = self.rw_rows()[spec].to(xt.dtype)
        loss, gW, gb = logreg_loss_grad_torch(X, self.y32.long(), Weff, b, rw, inv_wsum[spec])
        G = torch.cat([gW * inv_std[spec][:, None, :], gb.unsqueeze(2)], dim=2) * pmask[spec]
        return loss.double(), G.reshape(BT, -1)


def _arena(specs, dev, into: dict) -> torch.Tensor:
    """One zero-filled device allocation carved into 256-byte aligned views ``(name, shape, dtype)``,
    stored into ``into``; returns the backing buffer."""
    offs, off = [], 0
    for _, shape, dt in specs:
        n = 1
        for v in shape:
            n *= int(v)
        nb = n * torch.empty((), dtype=dt).element_size()
        offs.append((off, nb))
        off = (off + nb + 255) // 256 * 256
    buf = torch.zeros(max(off, 256), dtype=torch.uint8, device=dev)
    for (name, shape, dt), (o, nb) in zip(specs, offs):
        into[name] = buf[o:o + nb].view(dt).view(shape)
    return buf


# how the last native solve ran: 1 = one persistent cooperative launch, 0 = the launch sequence, 3 = the
# persistent launch timed out in a grid barrier and the fit was rerun as the sequence (tests)
LAST_SOLVE_MODE = -1


class DeviceLogregSolver:
    """Runs ``optim.lbfgs.minimize_trials``' algorithm for the LR objective entirely with the
    logreg_qn.hip kernels: 4 launches per iteration (direction + trials, evaluate, gradient,
    pick + history + the next direction's dots, each model finalized on the device by its last
    chunk), no host synchronization unless ``poll`` asks for a convergence check."""

    def __init__(self, design: LogregDesign, B: int, T: int, m: int, inv_std, pmask, inv_wsum, l2v, l1v,
                 max_iter: int, tol: float, c1: float = 1e-4, allreduce=None):
        self.d = design
        dev = design.device
        K, F = design.K, design.F
        self.B, self.T, self.m = B, T, m
        self.D = K * (F + 1)
        D = self.D
        BT = B * T
        self.inv_std = inv_std.float().contiguous()
        self.pmask = pmask.float().reshape(B, D).contiguous()
        self.inv_wsum = inv_wsum.float().contiguous()
        self.l2v = l2v.float().contiguous()
        self.l1v = None if l1v is None else l1v.float().contiguous()
        self.max_iter, self.tol, self.c1 = max_iter, tol, c1
        self.allreduce = allreduce
        self.nch = _native.kernels().qn_chunks(D, B)
        self.ntiles = _native.kernels().logreg_eval_tiles(design.N)
        KP, N = design.KP, max(1, design.N)
        # trial models whose residual rows [N][KP] are held at once (the one-hot gradient reads them):
        # evaluations are launched in chunks of rchunk models so R stays within HAR_LR_R_BUDGET_MB
        budget = int(os.environ.get("HAR_LR_R_BUDGET_MB", "1024")) << 20
        self.rchunk = max(1, min(BT, budget // (N * KP * 4)))
        f32, f64, i32 = torch.float32, torch.float64, torch.int32
        # every buffer of the solve is a view of ONE zeroed arena (one allocation + one fill per fit
        # instead of ~30); the data-parallel bucket G is followed by the fixed-point losses so ONE
        # all-reduce carries both
        specs = [("x", (B, D), f32), ("g", (B, D), f32), ("fobj", (B,), f64), ("S", (m, B, D), f32),
                 ("Y", (m, B, D), f32), ("rho", (m, B), f64), ("SY", (B, m, m), f64), ("YY", (B, m, m), f64),
                 ("xtrial", (BT, D), f32), ("weff", (BT, F + 1, KP), f32), ("reg", (BT,), f64),
                 ("decr", (BT,), f64), ("bucket", (BT * D + 5 * BT,), f32), ("loss", (BT,), f64),
                 ("step_scale", (B,), f32), ("active", (B,), i32), ("fails", (B,), i32), ("iters", (B,), i32),
                 ("steep", (B,), i32), ("pick", (B,), i32), ("P1", (B, self.nch, 2 * 10 + 1), f64),
                 ("P2", (B, self.nch, 3 * 4 + 2), f64), ("P3", (B, self.nch, 5 + 3 * 10), f64),
                 ("hist", (max_iter + 1, B), f64), ("done", (B,), i32),
                 ("slab", (BT, max(1, self.ntiles), design.Fd * KP + KP + 1), f32)]
        if design.C:
            specs.append(("R", (self.rchunk, N, KP), f32))
        else:
            self.R = None
        self.arena = _arena(specs, dev, self.__dict__)
        self.G = self.bucket[: BT * D].view(BT, D)          # data gradient of every trial
        self.loss_fx = self.bucket[BT * D:].view(BT, 5)     # DP only: fixed-point loss pieces
        self.step_scale.fill_(1.0)
        self.active.fill_(1)
        self.n_evals = 0

    def reset(self):
        """Back to the state of a fresh solver (the zeroed arena, unit step scales, every model
        active) for another fit through the SAME buffers: a cached solver's pointers, argument
        blocks and solve plan stay valid, so a repeated fit skips their host-side construction."""
        self.arena.zero_()
        self.step_scale.fill_(1.0)
        self.active.fill_(1)
        self.n_evals = 0

    def _args(self, init: int = 0, head: int = 0, filled: int = 0, fin_it: int = 0):
        # the buffers never move during a solve: their pointers are read once (~40 data_ptr calls per
        # launch were most of the host time of a 20-iteration fit), only the iteration scalars change
        base = getattr(self, "_arg_base", None)
        if base is None:
            base = self._arg_base = self._pointer_args()
        a = dict(base)
        a.update(head=head, filled=filled, init=init, fin_it=fin_it)
        return a

    def _pointer_args(self):
        p = lambda t: 0 if t is None else t.data_ptr()  # noqa: E731
        return {"B": self.B, "T": self.T, "K": self.d.K, "F": self.d.F, "m": self.m, "head": 0,
                "filled": 0, "init": 0, "nch": self.nch, "fin_it": 0, "D": self.D, "x": p(self.x), "g": p(self.g),
                "fobj": p(self.fobj), "l1": p(self.l1v), "l2": p(self.l2v), "pmask": p(self.pmask),
                "inv_std": p(self.inv_std), "S": p(self.S), "Y": p(self.Y), "rho": p(self.rho),
                "SY": p(self.SY), "YY": p(self.YY), "P1": p(self.P1), "P2": p(self.P2), "P3": p(self.P3),
                "xtrial": p(self.xtrial), "weff": p(self.weff), "reg": p(self.reg), "decr": p(self.decr),
                "G": p(self.G), "loss": p(self.loss), "step_scale": p(self.step_scale), "active": p(self.active),
                "fails": p(self.fails), "iters": p(self.iters), "steep": p(self.steep), "pick": p(self.pick),
                "hist": p(self.hist), "done": p(self.done), "c1": float(self.c1), "tol": float(self.tol)}

    def _eval_args(self, tstride: int):
        """Per launch chunk: positional arguments (but the stream) of the evaluate + gradient
        launches, built once per tstride: the buffers never move during a solve."""
        cache = self.__dict__.setdefault("_eval_arg_cache", {})
        if tstride not in cache:
            d = self.d
            n_models = (self.B * self.T) // tstride
            R = 0 if self.R is None else self.R.data_ptr()
            cs = d.col_slice()
            cb, nblk, srow = d.col_blocks()
            dp = self.allreduce is not None
            launches = []
            for c0 in range(0, n_models, self.rchunk):
                n = min(self.rchunk, n_models - c0)
                m0 = c0 * tstride
                ev = (d.dense.data_ptr(), d.dense.stride(0), d.Fd, d.dense_cols.data_ptr(), d.cat.data_ptr(), d.C,
                      d.y32.data_ptr(), d.rw_ptr(), self.inv_wsum.data_ptr(), self.weff.data_ptr(), d.N, d.F,
                      d.K, self.T, tstride, m0, 0, R, self.slab.data_ptr(), d.KP, n)
                gr = (self.slab.data_ptr(), R, d.col_map.data_ptr(), d.csc_rows.data_ptr(), d.csc_off.data_ptr(),
                      cs.data_ptr(), d.SL, self.inv_std.data_ptr(), self.pmask.data_ptr(), d.N, d.F, d.Fd, d.K,
                      self.T, tstride, m0, self.ntiles, self.G.data_ptr(), self.loss.data_ptr(),
                      self.loss_fx.data_ptr() if dp else 0, d.KP, n, 0 if cb is None else cb.data_ptr(), nblk,
                      0 if srow is None else srow.data_ptr())
                launches.append((ev, gr))
            cache[tstride] = launches
        return cache[tstride]

    def _evaluate(self, tstride: int):
        mod = _native.kernels()
        s = _native.stream_ptr()
        for ev, gr in self._eval_args(tstride):
            mod.logreg_eval(*ev, s)
            mod.logreg_grad(*gr, s)
        if self.allreduce is not None:
            # data parallel: ONE fp32 all-reduce of [gradients | fixed-point losses], then the exact
            # loss sums back to fp64 (every rank then takes the identical optimizer step)
            self.allreduce(self.bucket)
            mod.logreg_loss_decode(self.loss_fx.data_ptr(), self.loss.data_ptr(), self.B * self.T, s)
        self.n_evals += 1

    def evaluate_at(self, x: torch.Tensor):
        """The data objective at arbitrary points ``x [B, D]`` through the evaluation kernels
        (T = 1 solvers: ``LogisticRegression(lineSearch="wolfe")``, whose line-search state machine
        runs as batched tensor ops in ``optim.lbfgs.minimize_wolfe``): W_eff = x * inv_std * mask in
        the evaluator's [F+1][KP] layout, then evaluate + gradient (+ the DP all-reduce).  Returns
        (loss [B] float64, G [B, D] float32) — views of the solver's buffers, overwritten by the next
        call."""
        if self.T != 1:
            raise ValueError("evaluate_at needs a one-trial solver")
        B, K, F = self.B, self.d.K, self.d.F
        xv = x.reshape(B, K, F + 1).float() * self.pmask.view(B, K, F + 1)
        sc = torch.cat([self.inv_std.view(B, F), torch.ones(B, 1, device=xv.device)], 1)
        self.weff[:, :, :K].copy_((xv * sc[:, None, :]).transpose(1, 2))
        self._evaluate(1)
        return self.loss, self.G

    def solve(self, x0: torch.Tensor, poll: int = 0):
        """Per iteration: phase 1 (direction + T trial points), evaluate + gradient of the B*T
        trials, phase 2 (pick + history + the next direction's dots; each model's last chunk
        finalizes it on the device).  The host polls ``active`` (one sync) every ``poll``
        iterations only."""
        mod, s, KP = _native.kernels(), _native.stream_ptr(), self.d.KP
        qa = getattr(self, "_qn_args", None)
        if qa is None:  # pointers / shapes converted once; a launch passes only the iteration scalars
            qa = self._qn_args = mod.qn_args(self._args())

        def phase(ph, head=0, filled=0, init=0, fin_it=0):
            mod.lbfgs_phase_h(qa, ph, head, filled, init, fin_it, KP, s)

        self.x.copy_(x0.reshape(self.B, self.D))
        self.hist_rows = self.max_iter + 1
        if not poll and self.allreduce is None and os.environ.get("HAR_LR_NATIVE_SOLVE", "1") != "0":
            # the fixed launch sequence below as ONE native call (bind.cpp logreg_solve): no
            # convergence poll and no collective, so nothing needs the host between launches
            plan = getattr(self, "_solve_plan", None)
            if plan is None:
                chunks = lambda ts: [mod.logreg_eval_chunk(ev, gr) for ev, gr in self._eval_args(ts)]  # noqa: E731
                plan = self._solve_plan = mod.logreg_solve_plan(qa, chunks(self.T), chunks(1), KP)
            # the launch sequence, or (HAR_LR_PERSISTENT=1) one cooperative launch for the whole solve
            # (logreg_solve_persistent_kernel, bitwise the same; measured slower); 1 = persistent ran
            global LAST_SOLVE_MODE
            self.solve_mode = LAST_SOLVE_MODE = mod.logreg_solve(plan, self.max_iter, self.m, s)
            if self.solve_mode == 2:
                # a grid barrier of the persistent solve timed out (its blocks went on unsynchronized):
                # the results are garbage — rerun the whole fit as the launch sequence, loudly
                import warnings

                warnings.warn("persistent LR solve: grid barrier timed out; rerunning as the launch sequence")
                self.reset()
                self.x.copy_(x0.reshape(self.B, self.D))
                old = mod.logreg_set_persistent(0)
                try:
                    mod.logreg_solve(plan, self.max_iter, self.m, s)
                finally:
                    mod.logreg_set_persistent(old)
                self.solve_mode = LAST_SOLVE_MODE = 3  # 3 = timed out, rerun as the sequence
            self.n_evals += 1 + self.max_iter
            return self.x, self.fobj, self.iters
        phase(1, init=1)
        self._evaluate(self.T)
        phase(2, init=1)
        head = filled = 0
        for it in range(self.max_iter):
            if poll and it and it % poll == 0 and not bool(self.active.any()):
                self.hist_rows = it + 1
                break
            phase(1, head, filled)
            self._evaluate(1)
            phase(2, head, filled, fin_it=it + 1)
            head = (head + 1) % self.m
            filled = min(filled + 1, self.m)
        return self.x, self.fobj, self.iters

    def history(self, b: int, hist_host=None):
        """Objective history of model ``b`` (a list like Spark's ``objectiveHistory``: the objective
        after each iteration, trailing repeats of the final value — iterations after convergence —
        dropped).  ``hist_host``: this solver's ``hist`` already on the host.  (Not cut by the
        iteration count: the solver writes a row every round, a rejected line-search round included —
        it repeats the objective — while ``iters`` counts accepted steps only, logreg_qn.hip:866/885.)"""
        h = (self.hist if hist_host is None else hist_host)[: self.hist_rows, b].tolist()
        while len(h) > 1 and h[-1] == h[-2]:
            h.pop()
        return h

    def histories(self, hist_host=None):
        """``history(b)`` of every model from ONE host list conversion (a per-model column slice +
        ``tolist`` was ~4 us each: ~0.2 ms of a 54-model CrossValidator fit)."""
        cols = (self.hist if hist_host is None else hist_host)[: self.hist_rows].T.tolist()
        for h in cols:
            while len(h) > 1 and h[-1] == h[-2]:
                h.pop()
        return cols

    def margins(self, W_models: torch.Tensor, hm, n_models: int) -> torch.Tensor:
        """Raw margins of ``n_models`` weight tables ``[n, F+1, KP]`` over ``hm`` rows: [n, N, KP]."""
        return logreg_margins_native(hm, W_models, self.d.K, n_models)


def logreg_margins_native(hm, W_models: torch.Tensor, K: int, n_models: int) -> torch.Tensor:
    """Margins of ``n_models`` LR weight tables ``W_models [n, F+1, KP]`` (row F = intercept) over a
    hybrid matrix, with the evaluation kernel in prediction mode: [n, N, KP] float32."""
    mod, s = _native.kernels(), _native.stream_ptr()
    KP = W_models.shape[2]
    N, F = hm.n_rows, hm.n_features
    dev = hm.device
    Fd, C = int(hm.dense.shape[1]), int(hm.cat.shape[1])
    dense = hm.dense if Fd else torch.zeros(max(1, N), 1, device=dev)
    dcols = hm.dense_cols if Fd else torch.zeros(1, dtype=torch.int32, device=dev)
    cat = hm.cat if C else torch.zeros(max(1, N), 1, dtype=torch.int32, device=dev)
    out = torch.empty(n_models, max(1, N), KP, device=dev)
    ones = torch.ones(1, device=dev)
    mod.logreg_eval(dense.data_ptr(), dense.stride(0), Fd, dcols.data_ptr(), cat.data_ptr(), C, 0, 0, ones.data_ptr(),
                    W_models.contiguous().data_ptr(), N, F, K, 1, 1, 0, 1, out.data_ptr(), 0, KP, n_models, s)
    return out[:, :N]


# Solver cache of repeated single-device fits on the same resident design (the suite's LR, the
# CrossValidator's batched fold fits on one table): the design, the solver's arena, its pointer /
# argument blocks and the native solve plan are built once; a later fit with the same key rewrites the
# per-fit inputs (row weights, standardization, masks, regularization, x0) in place and zeroes the arena.  Every
# kernel of the fit still runs; only the host-side construction (~0.15 ms of Python per fit, the GPU
# idle meanwhile) is skipped.  Entries hold the matrix and labels they were built for (identity
# checked, so a freed tensor's reused address can never alias a stale entry).
# Bounded twice: at most SOLVER_CACHE_MAX entries AND at most HAR_LR_CACHE_MB (default 1024) MB of
# device memory held by them (arena + design + per-fit inputs; least recently used evicted first);
# main.run / the reference suite clear it when they finish, so tables a caller has dropped do not
# stay resident for the life of the process.
SOLVER_CACHE_MAX = 4
SOLVER_CACHE_MAX_BYTES = int(os.environ.get("HAR_LR_CACHE_MB", "1024")) << 20
_SOLVER_CACHE: "dict" = {}


def _nbytes(*ts) -> int:
    return sum(t.numel() * t.element_size() for t in ts if isinstance(t, torch.Tensor))


class SolverCacheEntry:
    def __init__(self, hm, y, design, solver, bufs):
        self.hm, self.y, self.design, self.solver, self.bufs = hm, y, design, solver, bufs
        d = design
        self.nbytes = (_nbytes(solver.arena, getattr(solver, "R", None), d.rw, d.y32, d.csc_rows, d.csc_off)
                       + _nbytes(*[b for b in bufs if b is not None]))


def solver_cache_get(key, hm, y) -> Optional[SolverCacheEntry]:
    ent = _SOLVER_CACHE.get(key)
    # the labels may be a fresh view of the same storage (y[0:N]); the entry keeps its own reference,
    # so an equal pointer + layout is that same storage, never a reused address
    if (ent is None or ent.hm is not hm or ent.y.data_ptr() != y.data_ptr() or ent.y.shape != y.shape
            or ent.y.stride() != y.stride() or ent.y.dtype != y.dtype):
        return None
    _SOLVER_CACHE[key] = _SOLVER_CACHE.pop(key)  # most recently used last
    return ent


def solver_cache_put(key, ent: SolverCacheEntry):
    _SOLVER_CACHE.pop(key, None)
    if ent.nbytes > SOLVER_CACHE_MAX_BYTES:
        return  # larger than the whole budget: not cached
    while _SOLVER_CACHE and (len(_SOLVER_CACHE) >= SOLVER_CACHE_MAX or
                             sum(e.nbytes for e in _SOLVER_CACHE.values()) + ent.nbytes > SOLVER_CACHE_MAX_BYTES):
        _SOLVER_CACHE.pop(next(iter(_SOLVER_CACHE)))
    _SOLVER_CACHE[key] = ent


def solver_cache_bytes() -> int:
    return sum(e.nbytes for e in _SOLVER_CACHE.values())


def solver_cache_clear():
    _SOLVER_CACHE.clear()
