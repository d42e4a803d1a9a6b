"""Batched multinomial logistic-regression loss/gradient (kernel K9).

For B models with effective weights ``W [B, K, F]`` and intercepts ``b [B, K]``
over one resident feature matrix ``X [N, F]``:

    Z   = X . W^T + b                  (one GEMM for all B*K columns)
    P   = softmax over each model's K columns
    R   = rw[b, i] / sum_i rw[b, i] * (P - onehot(y))
    loss[b] = sum_i rw[b,i] * CE_i / sum_i rw[b,i]
    dW  = R^T . X ,   db = sum_i R

``rw`` carries the per-model row weights (fold membership in CrossValidator,
Spark's instance weights otherwise), so 45 CV fits share the two GEMMs.

GPU path (gfx950): ``har_gemm_f32`` (exact-fp32 ``v_mfma_f32_16x16x4_f32``,
bias fused in the epilogue) -> ``har_logreg_softmax_grad`` (fused softmax + CE +
residual + per-model loss reduction) -> ``har_gemm_f32`` split-K with fp32
atomics for ``R^T . X``.  CPU path: the same math in PyTorch (test oracle).
"""
from __future__ import annotations

import torch

from . import _native
from .gemm import EPI_BIAS_F32, EPI_F32_ATOMIC, gemm_f32


def _pad8(x: int) -> int:
    return (x + 7) // 8 * 8


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


class LogregWorkspace:
    """Device buffers reused across the ~30-60 objective evaluations of a fit."""

    def __init__(self, X: torch.Tensor, B: int, K: int):
        N, F = X.shape
        self.N, self.F, self.B, self.K = N, F, B, K
        self.cols = _pad8(B * K)
        dev = X.device
        self.Wflat = torch.zeros(self.cols, F, device=dev, dtype=torch.float32)
        self.bflat = torch.zeros(self.cols, device=dev, dtype=torch.float32)
        self.Z = torch.empty(N, self.cols, device=dev, dtype=torch.float32)
        self.R = torch.empty(N, self.cols, device=dev, dtype=torch.float32)
        self.G = torch.empty(self.cols, F, device=dev, dtype=torch.float32)
        self.loss = torch.empty(B, device=dev, dtype=torch.float64)


def logreg_loss_grad_native(X, y32, W, b, rw, inv_wsum, ws: LogregWorkspace):
    B, K, F = W.shape
    N = X.shape[0]
    if F % 4:
        raise ValueError("native logreg path needs F % 4 == 0 (pad the feature matrix)")
    mod = _native.kernels()
    s = _native.stream_ptr()
    ws.Wflat[: B * K].copy_(W.reshape(B * K, F))
    ws.bflat[: B * K].copy_(b.reshape(-1))
    # Z = X . W^T + b        (A = X K-major, B = W K-major)
    gemm_f32(X, ws.Wflat, ws.Z, M=N, N=ws.cols, K=F, layout=0, epi=EPI_BIAS_F32, bias=ws.bflat)
    ws.loss.zero_()
    mod.logreg_softmax_grad(ws.Z.data_ptr(), N, B, K, ws.cols, y32.data_ptr(), rw.data_ptr(),
                            inv_wsum.data_ptr(), ws.R.data_ptr(), ws.loss.data_ptr(), s)
    # G = R^T . X            (A = R M-major [N][cols], B = X N-major [N][F]); split-K over rows
    ws.G.zero_()
    gemm_f32(ws.R, X, ws.G, M=ws.cols, N=F, K=N, layout=3, epi=EPI_F32_ATOMIC,
             k_split=max(32, ((N + 63) // 64 + 31) // 32 * 32))
    gW = ws.G[: B * K].view(B, K, F)
    gb = ws.R[:, : B * K].sum(dim=0).view(B, K)
    return ws.loss.to(torch.float32), gW, gb


# ------------------------------------------------------------------------------------------
# Hybrid-layout objective + device L-BFGS (csrc/kernels/logreg_qn.hip)
# ------------------------------------------------------------------------------------------
def _kp(K: int) -> int:
    return 8 if K <= 8 else 16


class LogregDesign:
    """Device data of one fit: the hybrid feature layout, labels, per-spec row weights, the
    one-hot CSC row lists and the column map of the gradient kernel."""

    def __init__(self, hm, y: torch.Tensor, rw: torch.Tensor, K: int):
        self.hm = hm
        self.N, self.F = hm.n_rows, hm.n_features
        self.Fd, self.C = int(hm.dense.shape[1]), int(hm.cat.shape[1])
        self.K = K
        self.KP = _kp(K)
        self.y32 = y.to(torch.int32).contiguous()
        self.rw = rw.float().contiguous()                       # [S, N]
        self.csc_off, self.csc_rows = hm.csc()
        if self.csc_rows.numel() == 0:
            self.csc_rows = torch.zeros(1, dtype=torch.int32, device=hm.device)
        self.col_map = hm.col_map()
        self.dense = hm.dense if self.Fd else torch.zeros(max(1, self.N), 1, device=hm.device)
        self.dense_cols = hm.dense_cols if self.Fd else torch.zeros(1, dtype=torch.int32, device=hm.device)
        self.cat = hm.cat if self.C else torch.zeros(max(1, self.N), 1, dtype=torch.int32, device=hm.device)

    def grad_partition(self, cols_per_block: int = 128):
        """Work partition of the gradient kernel (one host read of the CSC offsets per fit):
        every one-hot column's row list is cut into slices of <= SL rows, SL chosen so no
        ``cols_per_block``-column window holds more than 256 slices; returns device int32
        (slice_lo [n_slices+1], col_slice [F+2], blk_col [nb+1], blk_slice [nb+1]) and nb."""
        if getattr(self, "_part", None) is not None:
            return self._part
        import numpy as np

        F = self.F
        off = self.csc_off.cpu().numpy().astype(np.int64)
        L = off[1:F + 2] - off[:F + 1]                                   # rows per column (F+1)
        starts = np.arange(0, F + 1, cols_per_block)
        win = np.add.reduceat(L, starts) if L.size else np.zeros(1, np.int64)
        SL = max(16, int(-(-int(win.max()) // cols_per_block)) if win.size else 16)
        ns = -(-L // SL)
        col_slice = np.zeros(F + 2, np.int64)
        col_slice[1:] = np.cumsum(ns)
        total = int(col_slice[-1])
        col_of = np.repeat(np.arange(F + 1), ns)
        within = np.arange(total) - col_slice[col_of]
        slice_lo = np.concatenate([off[col_of] + within * SL, [off[F + 1]]])
        blk_col = np.concatenate([starts, [F + 1]])
        blk_slice = col_slice[blk_col]
        assert int(np.max(np.diff(blk_slice), initial=0)) <= 256 and int(np.max(np.diff(blk_col))) <= 256
        dev = self.rw.device
        t = lambda a: torch.as_tensor(a.astype(np.int32)).to(dev)  # noqa: E731
        self._part = (t(slice_lo), t(col_slice), t(blk_col), t(blk_slice), len(starts))
        return self._part

    def summary(self):
        """Weighted summarizer per spec (Spark MultivariateOnlineSummarizer + MultiClassSummarizer):
        [S, 1 + 2F + K] float64 = (sum w, sum w x, sum w x^2, class counts).  One-hot columns are
        segment sums of the weights over their CSC row lists (fp64 scan), dense columns one fp64
        product — every sum in a fixed order."""
        S_, N, F, K = self.rw.shape[0], self.N, self.F, self.K
        dev = self.rw.device
        rwd = self.rw.double()
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
        rw = self.rw[spec].to(xt.dtype)
        loss, gW, gb = logreg_loss_grad_torch(X, self.y32.long(), Weff, b, rw, inv_wsum[spec])
        G = torch.cat([gW * inv_std[spec][:, None, :], gb.unsqueeze(2)], dim=2) * pmask[spec]
        return loss.double(), G.reshape(BT, -1)


class DeviceLogregSolver:
    """Runs ``optim.lbfgs.minimize_trials``' algorithm for the LR objective entirely with the
    logreg_qn.hip kernels: 4 launches per iteration (direction + trials, evaluate, gradient,
    pick + history), no host synchronization unless ``poll`` asks for a convergence check."""

    def __init__(self, design: LogregDesign, B: int, T: int, m: int, inv_std, pmask, inv_wsum, l2v, l1v,
                 max_iter: int, tol: float, c1: float = 1e-4, allreduce=None):
        self.d = design
        dev = design.rw.device
        K, F = design.K, design.F
        self.B, self.T, self.m = B, T, m
        self.D = K * (F + 1)
        D = self.D
        BT = B * T
        f32 = dict(dtype=torch.float32, device=dev)
        f64 = dict(dtype=torch.float64, device=dev)
        i32 = dict(dtype=torch.int32, device=dev)
        self.inv_std = inv_std.float().contiguous()
        self.pmask = pmask.float().reshape(B, D).contiguous()
        self.inv_wsum = inv_wsum.float().contiguous()
        self.l2v = l2v.float().contiguous()
        self.l1v = None if l1v is None else l1v.float().contiguous()
        self.max_iter, self.tol, self.c1 = max_iter, tol, c1
        self.allreduce = allreduce
        self.x = torch.zeros(B, D, **f32)
        self.g = torch.zeros(B, D, **f32)
        self.fobj = torch.zeros(B, **f64)
        self.S = torch.zeros(m, B, D, **f32)
        self.Y = torch.zeros(m, B, D, **f32)
        self.rho = torch.zeros(m, B, **f64)
        self.SY = torch.zeros(B, m, m, **f64)   # history Gram matrices (compact two-loop recursion)
        self.YY = torch.zeros(B, m, m, **f64)
        self.xtrial = torch.zeros(BT, D, **f32)
        self.weff = torch.zeros(BT, F + 1, design.KP, **f32)   # padded classes stay 0
        self.reg = torch.zeros(BT, **f64)
        self.decr = torch.zeros(BT, **f64)
        self.G = torch.zeros(BT, D, **f32)        # data gradient of every trial (the DP all-reduce bucket)
        self.loss = torch.zeros(BT, **f64)        # data loss of every trial (fp64, its own small all-reduce)
        self.step_scale = torch.ones(B, **f32)
        self.active = torch.ones(B, **i32)
        self.fails = torch.zeros(B, **i32)
        self.iters = torch.zeros(B, **i32)
        self.steep = torch.zeros(B, **i32)
        self.pick = torch.zeros(B, **i32)
        self.nch = _native.kernels().qn_chunks(D, B)
        self.P1 = torch.zeros(B, self.nch, 2 * 10 + 1, **f64)   # chunk partials (QN_MAX_M = 10)
        self.P2 = torch.zeros(B, self.nch, 3 * 4 + 2, **f64)    # (QN_MAX_TRIALS = 4)
        self.P3 = torch.zeros(B, self.nch, 5 + 3 * 10, **f64)
        self.hist = torch.zeros(max_iter + 1, B, **f64)
        self.ntiles = _native.kernels().logreg_eval_tiles(design.N)
        self.slab = torch.zeros(BT, max(1, self.ntiles), design.Fd * design.KP + design.KP + 1, **f32)
        self.R = torch.zeros(BT, max(1, design.N), design.KP, **f32) if design.C else None
        self.n_evals = 0

    def _args(self, init: int = 0, head: int = 0, filled: int = 0, fin: int = 0, fin_init: int = 0,
              fin_head: int = 0, fin_it: int = 0):
        # the buffers never move during a solve: their pointers are read once (~40 data_ptr calls per
        # launch were most of the host time of a 20-iteration fit), only the iteration scalars change
        base = getattr(self, "_arg_base", None)
        if base is None:
            base = self._arg_base = self._pointer_args()
        a = dict(base)
        a.update(head=head, filled=filled, init=init, fin=fin, fin_init=fin_init, fin_head=fin_head, fin_it=fin_it)
        return a

    def _pointer_args(self):
        p = lambda t: 0 if t is None else t.data_ptr()  # noqa: E731
        return {"B": self.B, "T": self.T, "K": self.d.K, "F": self.d.F, "m": self.m, "head": 0,
                "filled": 0, "init": 0, "nch": self.nch, "fin": 0, "fin_init": 0,
                "fin_head": 0, "fin_it": 0, "D": self.D, "x": p(self.x), "g": p(self.g),
                "fobj": p(self.fobj), "l1": p(self.l1v), "l2": p(self.l2v), "pmask": p(self.pmask),
                "inv_std": p(self.inv_std), "S": p(self.S), "Y": p(self.Y), "rho": p(self.rho),
                "SY": p(self.SY), "YY": p(self.YY), "P1": p(self.P1), "P2": p(self.P2), "P3": p(self.P3),
                "xtrial": p(self.xtrial), "weff": p(self.weff), "reg": p(self.reg), "decr": p(self.decr),
                "G": p(self.G), "loss": p(self.loss), "step_scale": p(self.step_scale), "active": p(self.active),
                "fails": p(self.fails), "iters": p(self.iters), "steep": p(self.steep), "pick": p(self.pick),
                "hist": p(self.hist), "c1": float(self.c1), "tol": float(self.tol)}

    def _eval_args(self, tstride: int):
        """Positional arguments (but the stream) of the evaluate + gradient launches, built once per
        tstride: the buffers never move during a solve."""
        cache = self.__dict__.setdefault("_eval_arg_cache", {})
        if tstride not in cache:
            d = self.d
            n_models = (self.B * self.T) // tstride
            R = 0 if self.R is None else self.R.data_ptr()
            ev = (d.dense.data_ptr(), d.dense.stride(0), d.Fd, d.dense_cols.data_ptr(), d.cat.data_ptr(), d.C,
                  d.y32.data_ptr(), d.rw.data_ptr(), self.inv_wsum.data_ptr(), self.weff.data_ptr(), d.N, d.F,
                  d.K, self.T, tstride, 0, R, self.slab.data_ptr(), d.KP, n_models)
            slice_lo, col_slice, blk_col, blk_slice, nb = d.grad_partition()
            gr = (self.slab.data_ptr(), R, d.col_map.data_ptr(), d.csc_rows.data_ptr(), slice_lo.data_ptr(),
                  col_slice.data_ptr(), blk_col.data_ptr(), blk_slice.data_ptr(), nb, self.inv_std.data_ptr(),
                  self.pmask.data_ptr(), d.N, d.F, d.Fd, d.K, self.T, tstride, self.ntiles, self.G.data_ptr(),
                  self.loss.data_ptr(), d.KP, n_models)
            cache[tstride] = (ev, gr)
        return cache[tstride]

    def _evaluate(self, tstride: int):
        mod = _native.kernels()
        ev, gr = self._eval_args(tstride)
        s = _native.stream_ptr()
        mod.logreg_eval(*ev, s)
        mod.logreg_grad(*gr, s)
        if self.allreduce is not None:  # data parallel: the flat fp32 gradient bucket + the fp64 losses
            self.allreduce(self.G)
            self.allreduce(self.loss)
        self.n_evals += 1

    def solve(self, x0: torch.Tensor, poll: int = 0):
        """Per iteration: phase 0 (finalize the previous update + history dots), phase 1 (direction
        + T trial points), evaluate + gradient of the B*T trials, phase 2 (pick + history).  The
        host polls ``active`` (one sync) every ``poll`` iterations only."""
        mod, s, KP = _native.kernels(), _native.stream_ptr(), self.d.KP
        qa = getattr(self, "_qn_args", None)
        if qa is None:  # pointers / shapes converted once; a launch passes only the iteration scalars
            qa = self._qn_args = mod.qn_args(self._args())

        def phase(ph, head=0, filled=0, init=0, fin=0, fin_init=0, fin_head=0, fin_it=0):
            mod.lbfgs_phase_h(qa, ph, head, filled, init, fin, fin_init, fin_head, fin_it, KP, s)

        self.x.copy_(x0.reshape(self.B, self.D))
        phase(1, init=1)
        self._evaluate(self.T)
        phase(2, init=1)
        head = filled = 0
        prev = -1  # history slot written by the previous phase 2 (-1: the init update)
        finalized = False
        for it in range(self.max_iter):
            phase(0, head, filled, fin=1, fin_init=int(prev < 0), fin_head=max(prev, 0), fin_it=it)
            if poll and it and it % poll == 0 and not bool(self.active.any()):
                finalized = True
                break
            phase(1, head, filled)
            self._evaluate(1)
            phase(2, head, filled)
            prev = head
            head = (head + 1) % self.m
            filled = min(filled + 1, self.m)
        if not finalized:
            phase(3, fin=1, fin_init=int(prev < 0), fin_head=max(prev, 0), fin_it=self.max_iter)
        return self.x, self.fobj, self.iters

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
                    W_models.contiguous().data_ptr(), N, F, K, 1, 1, 1, out.data_ptr(), 0, KP, n_models, s)
    return out[:, :N]
