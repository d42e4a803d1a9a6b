"""Numerics of every HIP kernel vs. a plain PyTorch fp32/fp64 reference (GPU only)."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def _bf(x):
    return x.to(torch.bfloat16)


LAYOUT_SHAPES = [(1000, 96, 160), (256, 256, 256), (77, 40, 64), (4096, 64, 512), (64, 32, 1024), (130, 520, 96)]


@pytest.mark.parametrize("M,N,K", LAYOUT_SHAPES)
@pytest.mark.parametrize("layout", [0, 2, 3])
def test_gemm_bf16_layouts(cuda, M, N, K, layout):
    from har.ops.gemm import EPI_F32, gemm_bf16

    if layout & 1 and M % 8:
        pytest.skip("M-major A needs M % 8 == 0 (16-byte vector rows)")
    g = torch.Generator(device=cuda).manual_seed(M * 7 + N * 3 + K + layout)
    A = torch.randn(M, K, device=cuda, generator=g)
    Bm = torch.randn(K, N, device=cuda, generator=g)
    ref = _bf(A).float() @ _bf(Bm).float()
    a_store = _bf(A.T.contiguous()) if layout & 1 else _bf(A)          # [K][M] or [M][K]
    b_store = _bf(Bm) if layout & 2 else _bf(Bm.T.contiguous())        # [K][N] or [N][K]
    C = torch.full((M, N), float("nan"), device=cuda)
    gemm_bf16(a_store, b_store, C, M=M, N=N, K=K, layout=layout, epi=EPI_F32)
    torch.testing.assert_close(C, ref, rtol=2e-3, atol=2e-3 * K ** 0.5)


@pytest.mark.parametrize("M,N,K", [(296, 64, 4096), (32, 256, 65536 // 8), (256, 48, 3000 // 8 * 8)])
def test_gemm_bf16_splitk_atomic(cuda, M, N, K):
    from har.ops.gemm import EPI_F32_ATOMIC, gemm_bf16

    g = torch.Generator(device=cuda).manual_seed(5)
    At = torch.randn(K, M, device=cuda, generator=g)   # stored [K][M]  (layout bit0)
    Bm = torch.randn(K, N, device=cuda, generator=g)   # stored [K][N]  (layout bit1)
    ref = _bf(At).float().T @ _bf(Bm).float()
    C = torch.zeros(M, N, device=cuda)
    gemm_bf16(_bf(At), _bf(Bm), C, M=M, N=N, K=K, layout=3, epi=EPI_F32_ATOMIC)
    torch.testing.assert_close(C, ref, rtol=2e-3, atol=3e-3 * K ** 0.5)


def test_gemm_bf16_epilogues(cuda):
    from har.ops.gemm import EPI_BIAS, EPI_BIAS_RELU, EPI_RELU_GRAD, gemm_bf16

    M, N, K = 517, 192, 96
    g = torch.Generator(device=cuda).manual_seed(11)
    A = _bf(torch.randn(M, K, device=cuda, generator=g))
    W = _bf(torch.randn(N, K, device=cuda, generator=g))
    bias = torch.randn(N, device=cuda, generator=g)
    ref = A.float() @ W.float().T + bias
    out = torch.empty(M, N, dtype=torch.bfloat16, device=cuda)
    gemm_bf16(A, W, out, M=M, N=N, K=K, layout=0, epi=EPI_BIAS_RELU, bias=bias)
    torch.testing.assert_close(out.float(), torch.relu(ref).to(torch.bfloat16).float(), rtol=1e-2, atol=2e-2)
    gemm_bf16(A, W, out, M=M, N=N, K=K, layout=0, epi=EPI_BIAS, bias=bias)
    torch.testing.assert_close(out.float(), ref.to(torch.bfloat16).float(), rtol=1e-2, atol=2e-2)
    # relu-grad: dX = (dY . W) * (mask > 0)
    dY = _bf(torch.randn(M, N, device=cuda, generator=g))
    mask = _bf(torch.randn(M, K, device=cuda, generator=g))
    dX = torch.empty(M, K, dtype=torch.bfloat16, device=cuda)
    gemm_bf16(dY, W, dX, M=M, N=K, K=N, layout=2, epi=EPI_RELU_GRAD, mask=mask)
    refd = (dY.float() @ W.float()) * (mask.float() > 0)
    torch.testing.assert_close(dX.float(), refd, rtol=1e-2, atol=5e-2)


@pytest.mark.parametrize("tile", [-1, 4, 5])
def test_gemm_bf16_slab_rowsum(cuda, tile):
    """Deterministic split-K slabs + fused A-row sums (bias gradient) vs torch."""
    from har.ops import _native
    from har.ops.gemm import EPI_F32_SLAB, gemm_bf16

    M, N, K = 96, 64, 5000 // 32 * 32
    g = torch.Generator(device=cuda).manual_seed(21)
    At = _bf(torch.randn(K, M, device=cuda, generator=g))   # [K][M]
    Bm = _bf(torch.randn(K, N, device=cuda, generator=g))   # [K][N]
    ks = 512
    splits = (K + ks - 1) // ks
    stride = M * N + M
    slabs = torch.full((splits, stride), float("nan"), device=cuda)
    gemm_bf16(At, Bm, slabs.view(-1), M=M, N=N, K=K, layout=3, epi=EPI_F32_SLAB, k_split=ks, ldc=N,
              slab_stride=stride, rowsum=slabs.view(-1)[M * N:], slab_stride_rowsum=stride, tile=tile)
    out = torch.empty(stride, device=cuda)
    _native.kernels().reduce_slabs_grouped(slabs.data_ptr(), splits, stride, out.data_ptr(), 1, _native.stream_ptr(), 0)
    ref = At.float().T @ Bm.float()
    torch.testing.assert_close(out[: M * N].view(M, N), ref, rtol=2e-3, atol=3e-3 * K ** 0.5)
    torch.testing.assert_close(out[M * N:], At.float().sum(0), rtol=1e-3, atol=1e-2)


@pytest.mark.parametrize("M,N,K", [(3793, 272, 3100), (100, 8, 12), (1625, 8, 3100)])
def test_gemm_f32_exact(cuda, M, N, K):
    from har.ops.gemm import EPI_BIAS_F32, EPI_F32_ATOMIC, gemm_f32

    g = torch.Generator(device=cuda).manual_seed(3)
    X = torch.randn(M, K, device=cuda, generator=g)
    W = torch.randn(N, K, device=cuda, generator=g)
    b = torch.randn(N, device=cuda, generator=g)
    Z = torch.empty(M, N, device=cuda)
    gemm_f32(X, W, Z, M=M, N=N, K=K, layout=0, epi=EPI_BIAS_F32, bias=b)
    ref = (X.double() @ W.double().T + b.double()).float()
    torch.testing.assert_close(Z, ref, rtol=1e-5, atol=2e-7 * K)
    # R^T X with R stored [M][N] (M-major for the transposed product)
    G = torch.zeros(N, K, device=cuda)
    gemm_f32(Z, X, G, M=N, N=K, K=M, layout=3, epi=EPI_F32_ATOMIC)
    refg = (Z.double().T @ X.double()).float()
    torch.testing.assert_close(G, refg, rtol=1e-4, atol=1e-3 * M ** 0.5)


def test_softmax_ce_head(cuda):
    from har.ops import _native

    B, D, C = 1000, 128, 6
    mod = _native.kernels()
    g = torch.Generator(device=cuda).manual_seed(1)
    H = _bf(torch.randn(B, D, device=cuda, generator=g))
    W = torch.zeros(32, D, device=cuda)
    W[:C] = torch.randn(C, D, device=cuda, generator=g) * 0.2
    Wb = _bf(W)
    b = torch.zeros(32, device=cuda)
    b[:C] = torch.randn(C, device=cuda, generator=g)
    y = torch.randint(0, C, (B,), device=cuda, generator=g).to(torch.int32)
    dl = torch.zeros(B, 32, dtype=torch.bfloat16, device=cuda)
    nb = mod.softmax_ce_head_blocks(B)
    loss = torch.zeros(nb, device=cuda)
    corr = torch.zeros(nb, dtype=torch.int32, device=cuda)
    logits = torch.empty(B, C, device=cuda)
    scale = 1.0 / B
    mod.softmax_ce_head(H.data_ptr(), Wb.data_ptr(), b.data_ptr(), y.data_ptr(), B, D, C, scale,
                        dl.data_ptr(), loss.data_ptr(), corr.data_ptr(), logits.data_ptr(), _native.stream_ptr())
    z = H.float() @ Wb.float()[:C].T + b[:C]
    torch.testing.assert_close(logits, z, rtol=1e-4, atol=1e-3)
    ref_loss = torch.nn.functional.cross_entropy(z, y.long(), reduction="sum")
    torch.testing.assert_close(loss.sum(), ref_loss, rtol=1e-4, atol=1e-2)
    p = torch.softmax(z, 1)
    p[torch.arange(B), y.long()] -= 1
    torch.testing.assert_close(dl[:, :C].float(), (p * scale).to(torch.bfloat16).float(), rtol=1e-2, atol=1e-5)
    assert dl[:, C:].float().abs().max() == 0
    assert int(corr.sum()) == int((z.argmax(1) == y.long()).sum())


def test_adam_step(cuda):
    from har.ops import _native

    n = 1040
    g = torch.Generator(device=cuda).manual_seed(2)
    p = torch.randn(n, device=cuda, generator=g)
    p0 = p.clone()
    grad = torch.randn(n, device=cuda, generator=g)
    m = torch.zeros(n, device=cuda)
    v = torch.zeros(n, device=cuda)
    pb = torch.empty(n, dtype=torch.bfloat16, device=cuda)
    step = torch.zeros(1, dtype=torch.int32, device=cuda)
    lr, b1, b2, eps, wd = 1e-2, 0.9, 0.999, 1e-8, 0.01
    for t in range(1, 4):
        _native.kernels().adam_step(p.data_ptr(), grad.data_ptr(), 0, 0, m.data_ptr(), v.data_ptr(), pb.data_ptr(),
                                    n, lr, b1, b2, eps, wd, 1.0, step.data_ptr(), _native.stream_ptr(), 1)
    # reference
    pr, mr, vr = p0.double(), torch.zeros(n, dtype=torch.float64, device=cuda), torch.zeros(n, dtype=torch.float64,
                                                                                           device=cuda)
    gd = grad.double()
    for t in range(1, 4):
        mr = b1 * mr + (1 - b1) * gd
        vr = b2 * vr + (1 - b2) * gd * gd
        upd = (mr / (1 - b1 ** t)) / ((vr / (1 - b2 ** t)).sqrt() + eps)
        pr = pr - lr * (upd + wd * pr)
    torch.testing.assert_close(p.double(), pr, rtol=1e-5, atol=1e-5)
    assert int(step[0]) == 3
    torch.testing.assert_close(pb.float(), p.to(torch.bfloat16).float())


def _bf_round(x):
    return x.to(torch.bfloat16).float()


@pytest.mark.parametrize("layers,B,path", [([43, 64, 96, 6], 512, "gemm"), ([43, 256, 256, 6], 4096, "step")])
def test_mlp_step_matches_torch(cuda, layers, B, path):
    """Native step gradients vs a manual fp32 backprop that rounds to bf16 at the same
    points as the kernels (activations, dlogits, data grads, weight copies): the generic GEMM
    path and the flagship three-kernel step."""
    from har.models.mlp import MLPEngine, pad_input_bf16

    eng = MLPEngine(layers, B, cuda, lr=1e-3, seed=3)
    g = torch.Generator(device=cuda).manual_seed(9)
    X = torch.randn(B, 43, device=cuda, generator=g)
    y = torch.randint(0, 6, (B,), device=cuda, generator=g)
    Xb = pad_input_bf16(X, eng.layout.in_pad)
    eng.forward_backward_native(Xb, y.to(torch.int32), 1.0 / B)
    eng.reduce_grads_native()
    assert eng.last_path == path
    L = eng.layout
    P = eng.P.double()
    W = {s.name: L.view(P, s.name) for s in L.segments}
    Wb = {k: _bf_round(v.float()).double() for k, v in W.items()}
    C = L.num_classes
    h0 = Xb.double()
    h1 = _bf_round((h0 @ Wb["W0"].T + W["b0"]).clamp_min(0).float()).double()
    h2 = _bf_round((h1 @ Wb["W1"].T + W["b1"]).clamp_min(0).float()).double()
    z = h2 @ Wb["Wout"][:C].T + W["bout"][:C]
    p = torch.softmax(z, 1)
    p[torch.arange(B), y] -= 1
    dl = _bf_round((p / B).float()).double()
    ref = {"Wout": dl.T @ h2, "bout": dl.sum(0)}
    dh2 = _bf_round(((dl @ Wb["Wout"][:C]) * (h2 > 0)).float()).double()
    ref["W1"], ref["b1"] = dh2.T @ h1, dh2.sum(0)
    dh1 = _bf_round(((dh2 @ Wb["W1"]) * (h1 > 0)).float()).double()
    ref["W0"], ref["b0"] = dh1.T @ h0, dh1.sum(0)
    G = eng.G.double()
    for name, r in ref.items():
        a = L.view(G, name)
        a = a[:C] if name in ("Wout", "bout") else a
        rel = (a - r).norm() / r.norm().clamp_min(1e-12)
        assert rel < 1e-2, f"{name}: rel err {rel:.3e}"
    # padded class rows / input columns receive exactly zero gradient
    assert L.view(G, "Wout")[C:].abs().max() == 0
    assert L.view(G, "W0")[:, 43:].abs().max() == 0
    lsum, _ = eng.last_loss_and_correct()
    ref_loss = torch.nn.functional.cross_entropy(z, y, reduction="sum")
    assert abs(lsum - float(ref_loss)) / float(ref_loss) < 1e-2


def test_logreg_wide_dense_eval_vs_torch(cuda):
    """The LR evaluation + gradient kernels on a wide all-dense design (124 columns: four LDS chunks,
    the last one partial) vs the fp64 torch objective, several row-weighted trial models."""
    from har.features.hybrid import from_dense
    from har.ops.logreg import DeviceLogregSolver, LogregDesign

    N, F, S, T, K = 777, 124, 2, 3, 6
    g = torch.Generator().manual_seed(4)
    X = torch.randn(N, F, generator=g)
    y = torch.randint(0, K, (N,), generator=g)
    hm = from_dense(X.to(cuda), [])
    rw = (torch.rand(S, N, generator=g) > 0.2).float().to(cuda)
    design = LogregDesign(hm, y.to(cuda), rw, K)
    inv_std = (torch.rand(S, F, generator=g) + 0.5).to(cuda)
    pmask = torch.ones(S, K, F + 1, device=cuda)
    inv_wsum = 1.0 / rw.sum(1)
    D = K * (F + 1)
    solver = DeviceLogregSolver(design, S, T, 4, inv_std, pmask, inv_wsum, torch.zeros(S, D, device=cuda), None, 1,
                                1e-6)
    xt = torch.randn(S * T, K, F + 1, generator=g).to(cuda) * 0.1
    spec = torch.arange(S * T, device=cuda) // T
    solver.weff.zero_()
    solver.weff[:, :F, :K] = (xt[:, :, :F] * inv_std[spec][:, None, :]).transpose(1, 2)
    solver.weff[:, F, :K] = xt[:, :, F]
    solver._evaluate(1)
    ref_loss, ref_G = LogregDesign(hm, y.to(cuda), rw.double(), K).eval_torch(
        xt.double(), T, inv_std.double(), pmask.double(), inv_wsum.double())
    torch.testing.assert_close(solver.loss, ref_loss, rtol=2e-5, atol=1e-6)
    torch.testing.assert_close(solver.G.double(), ref_G, rtol=2e-4, atol=2e-6)


def test_metrics_kernels(cuda):
    from har.ops.metrics import confusion_matrix, regression_moments

    g = torch.Generator(device=cuda).manual_seed(8)
    y = torch.randint(0, 6, (10001,), device=cuda, generator=g)
    p = torch.randint(0, 6, (10001,), device=cuda, generator=g)
    cm = confusion_matrix(y, p, 6)
    ref = torch.bincount((y * 6 + p).cpu(), minlength=36).view(6, 6)
    assert torch.equal(cm.cpu(), ref)
    n, se, ae, sy, syy = regression_moments(y.float(), p.float())
    d = (y - p).double().cpu()
    assert n == 10001
    assert abs(se - float((d * d).sum())) < 1e-6 and abs(ae - float(d.abs().sum())) < 1e-6
    assert abs(sy - float(y.double().sum())) < 1e-6


def test_roc_pr_kernel(cuda):
    """roc.hip (K19) vs the fp64 PyTorch curve: tie groups, ties straddling threads and chunks,
    a single row, and no-positive / no-negative label sets."""
    from har.evaluation import metrics as M
    from har.ops.metrics import roc_pr_auc

    g = torch.Generator().manual_seed(4)
    for n, levels in ((1625, 0), (10001, 37), (4096 * 3 + 5, 7), (5, 2), (1, 0)):
        s = torch.randn(n, generator=g)
        if levels:
            s = torch.round(s * levels) / levels
        y = torch.randint(0, 6, (n,), generator=g).float()
        ref = M.binary_metrics(s, y)  # CPU oracle
        auroc, aupr = roc_pr_auc(s.to(cuda), y.to(cuda))
        assert abs(auroc - ref["areaUnderROC"]) < 1e-9, (n, auroc, ref)
        assert abs(aupr - ref["areaUnderPR"]) < 1e-9, (n, aupr, ref)
    for yv in (0.0, 3.0):
        s = torch.randn(300, generator=g)
        y = torch.full((300,), yv)
        ref = M.binary_metrics(s, y)
        got = M.binary_metrics(s.to(cuda), y.to(cuda))  # evaluator entry point takes the kernel
        assert abs(got["areaUnderROC"] - ref["areaUnderROC"]) < 1e-12
        assert abs(got["areaUnderPR"] - ref["areaUnderPR"]) < 1e-12


def test_column_stats_and_binning(cuda):
    from har.ops import stats
    from har.ops import tree as T

    g = torch.Generator(device=cuda).manual_seed(12)
    X = torch.randn(3001, 37, device=cuda, generator=g)
    X[5, 3] = float("nan")
    w = (torch.rand(3001, device=cuda, generator=g) > 0.3).float()
    st = stats.column_stats(X, w)
    ref = stats.column_stats(X.cpu(), w.cpu())
    torch.testing.assert_close(st.cpu(), ref, rtol=1e-9, atol=1e-7)
    thr = T.find_thresholds(X.cpu().numpy(), 32)
    b = stats.bin_features(X, thr).cpu()
    assert torch.equal(b, torch.from_numpy(T.bin_features(X.cpu().numpy(), thr)))


@pytest.mark.parametrize("H,F", [(256, 43), (256, 20), (128, 20)])
def test_mlp_fused_fwd_head_matches_unfused(cuda, monkeypatch, H, F):
    """mlp_fused.hip (fwd L1 + fwd L2 + head + dWout/dbout in one kernel) against the unfused
    kernel chain: same h1 / dact2 / reduced gradients / loss up to bf16 summation-order noise
    (HAR_MLP_STEP=0: the fused forward + GEMM backward path, the one that writes h1 / dact2)."""
    from har.models.mlp import MLPEngine, pad_input_bf16

    monkeypatch.setenv("HAR_MLP_STEP", "0")

    B = 4096
    layers = [F, H, H, 6]
    a = MLPEngine(layers, B, cuda, lr=1e-3, seed=5)
    b = MLPEngine(layers, B, cuda, lr=1e-3, seed=5)
    b.fused_ok = False
    assert a.fused_ok
    g = torch.Generator(device=cuda).manual_seed(11)
    X = pad_input_bf16(torch.randn(B, F, device=cuda, generator=g), a.layout.in_pad)
    y = torch.randint(0, 6, (B,), device=cuda, generator=g).to(torch.int32)
    for e in (a, b):
        e.forward_backward_native(X, y, 1.0 / B)
        e.reduce_grads_native()
    torch.cuda.synchronize()
    assert a.last_fused and not b.last_fused
    torch.testing.assert_close(a.acts[1].float(), b.acts[1].float(), rtol=2e-2, atol=2e-2)
    da, db = a.dbuf[1][: B * H].float(), b.dbuf[1][: B * H].float()
    assert (da - db).norm() / db.norm() < 2e-2
    L = a.layout
    for s in L.segments:
        ga, gb = L.view(a.G, s.name), L.view(b.G, s.name)
        rel = float((ga - gb).norm() / gb.norm().clamp_min(1e-12))
        assert rel < 2e-2, f"{s.name}: {rel:.3e}"
    la, ca = a.last_loss_and_correct()
    lb, cb = b.last_loss_and_correct()
    assert abs(la - lb) / lb < 1e-3 and abs(ca - cb) <= 2
    # full steps: parameters track the unfused engine; a batch that is not a multiple of 16 falls back
    for _ in range(3):
        a.train_step(X, y, B)
        b.train_step(X, y, B)
    torch.testing.assert_close(a.P, b.P, rtol=0, atol=5e-4)
    a.forward_backward_native(X[:4090], y[:4090], 1.0 / 4090)
    assert not a.last_fused


@pytest.mark.parametrize("F,B", [(43, 4096), (20, 4160), (43, 8256), (43, 65536)])
def test_mlp_step_matches_gemm_path_and_is_deterministic(cuda, monkeypatch, F, B):
    """The three-kernel step (mlp_step.hip: forward -> dz + relu' mask, backward rebuilding dact2 and
    h1 on chip) against the fused forward + split-K GEMM backward on the same batch: reduced
    gradients, loss and #correct agree to bf16 summation-order noise; K0 = 64 and 32, a batch whose
    last row slices are short (8256), the flagship batch.  Two runs of the step are bit-identical."""
    from har.models.mlp import MLPEngine, pad_input_bf16

    g = torch.Generator(device=cuda).manual_seed(13)
    X = torch.randn(B, F, device=cuda, generator=g)
    y = torch.randint(0, 6, (B,), device=cuda, generator=g).to(torch.int32)
    runs = []
    for flag in ("1", "1", "0"):
        monkeypatch.setenv("HAR_MLP_STEP", flag)
        e = MLPEngine([F, 256, 256, 6], B, cuda, lr=1e-3, seed=7)
        Xb = pad_input_bf16(X, e.layout.in_pad)
        e.forward_backward_native(Xb, y, 1.0 / B)
        e.reduce_grads_native()
        torch.cuda.synchronize()
        assert (e.last_path == "step") == (flag == "1")
        runs.append((e.G.clone(), e.last_loss_and_correct(), e.layout))
    (g1, lc1, L), (g2, lc2, _), (gr, lcr, _) = runs
    assert torch.equal(g1, g2) and lc1 == lc2
    for s_ in L.segments:
        a, b = L.view(g1, s_.name), L.view(gr, s_.name)
        rel = float((a - b).norm() / b.norm().clamp_min(1e-12))
        assert rel < 1e-2, f"{s_.name}: {rel:.3e}"
    assert abs(lc1[0] - lcr[0]) / lcr[0] < 1e-3 and abs(lc1[1] - lcr[1]) <= 2


def test_mlp_step_prefetch_leaves_training_bitwise_unchanged(cuda):
    """train_step(prefetch=the next batch's rows): the reduction launch's extra workgroups only read
    those rows (bind.cpp MlpStepPlan, mlp.hip PrefetchSpec) — parameters, Adam moments and the bf16
    copy after six flagship-batch steps are bit-identical to plain steps."""
    from har.models.mlp import MLPEngine, pad_input_bf16

    B, F, nb = 65536, 43, 3
    g = torch.Generator(device=cuda).manual_seed(5)
    X = torch.randn(B * nb, F, device=cuda, generator=g)
    y = torch.randint(0, 6, (B * nb,), device=cuda, generator=g).to(torch.int32)
    outs = []
    for pf in (False, True):
        e = MLPEngine([F, 256, 256, 6], B, cuda, lr=1e-3, seed=7)
        Xb = pad_input_bf16(X, e.layout.in_pad)
        for i in range(2 * nb):
            j, k = i % nb, (i + 1) % nb
            e.train_step(Xb[j * B:(j + 1) * B], y[j * B:(j + 1) * B], B,
                         prefetch=(Xb[k * B:(k + 1) * B], y[k * B:(k + 1) * B]) if pf else None)
        torch.cuda.synchronize()
        assert e.last_path == "step"
        outs.append((e.P.clone(), e.m.clone(), e.v.clone(), e.Pb.clone()))
    for a, b in zip(*outs):
        assert torch.equal(a, b)


def test_mlp_step_outputs(cuda):
    """What the step forward hands the backward: dact2 = ((softmax - onehot) * scale) . Wout * relu'(h2)
    in bf16, in the backward's tile order (16-byte chunks of rows with bit 2 set swapped in pairs),
    against the fp32 PyTorch forward of the same (bf16-rounded) parameters."""
    from har.models.mlp import MLPEngine, pad_input_bf16

    B, F = 4096, 43
    e = MLPEngine([F, 256, 256, 6], B, cuda, lr=1e-3, seed=3)
    g = torch.Generator(device=cuda).manual_seed(5)
    X = pad_input_bf16(torch.randn(B, F, device=cuda, generator=g), 64)
    y = torch.randint(0, 6, (B,), device=cuda, generator=g).to(torch.int32)
    e.forward_backward_native(X, y, 1.0 / B)
    torch.cuda.synchronize()
    assert e.last_path == "step"
    P = e.Pb.float()
    L = e.layout
    h1 = torch.relu(X.float() @ L.view(P, "W0").T + L.view(e.P, "b0")).bfloat16().float()
    h2 = torch.relu(h1 @ L.view(P, "W1").T + L.view(e.P, "b1"))
    z = h2.bfloat16().float() @ L.view(P, "Wout")[:6].T + L.view(e.P, "bout")[:6]
    ref_dz = ((torch.softmax(z, 1) - torch.nn.functional.one_hot(y.long(), 6).float()) / B).bfloat16().float()
    ref = (ref_dz @ L.view(P, "Wout")[:6]) * (h2.bfloat16().float() > 0).float()     # [B][256]
    raw = e.dact2.view(B, 256).float()
    # undo the chunk swap: rows r with bit 2 set hold column c at c ^ 8
    cols = torch.arange(256, device=cuda)
    rows = torch.arange(B, device=cuda)
    swz = (cols[None, :] ^ (8 * ((rows[:, None] >> 2) & 1)))
    got = torch.gather(raw, 1, swz)
    assert float((got - ref).norm() / ref.norm()) < 2e-2
    # exact zeros where relu'(h2) = 0 (the mask is applied to the packed bf16 bits)
    zero = h2.bfloat16().float() == 0
    assert float(got[zero].abs().max()) == 0.0


@pytest.mark.parametrize("H,F", [(256, 43), (128, 20)])
def test_mlp_fused_infer_matches_fp32(cuda, H, F):
    """Serving variant of the fused kernel (logits + argmax only) vs the fp32 PyTorch forward
    of the same parameters (bf16 operands: relative logit error ~1e-2)."""
    from har.models.mlp import MLPEngine, pad_input_bf16

    B = 4096
    eng = MLPEngine([F, H, H, 6], B, cuda, lr=1e-3, seed=9)
    g = torch.Generator(device=cuda).manual_seed(3)
    X = torch.randn(B, F, device=cuda, generator=g)
    logits, pred = eng.infer_fused(pad_input_bf16(X, eng.layout.in_pad))
    Xp = torch.zeros(B, eng.layout.in_pad, device=cuda)
    Xp[:, :F] = X
    ref = eng.torch_forward(eng.P, Xp).float()
    assert logits.shape == (B, 6) and pred.dtype == torch.int32
    assert float((logits - ref).norm() / ref.norm()) < 2e-2
    assert torch.equal(pred.long(), torch.argmax(logits, 1))  # in-kernel argmax of its own logits
    agree = float((pred.long() == torch.argmax(ref, 1)).float().mean())
    assert agree > 0.97
    lf, pf = eng.infer_fused_f32(X)  # fp32 features (cast in the loads, or cast + the step's INFER pipeline)
    if H == 256:  # mlp_step.hip INFER: the training forward's pipeline, its own fp32 summation order
        assert float((lf - ref).norm() / ref.norm()) < 2e-2
        assert torch.equal(pf.long(), torch.argmax(lf, 1))
        assert float((pf == pred).float().mean()) > 0.99
        torch.testing.assert_close(lf, logits, rtol=2e-2, atol=2e-2)
    else:
        torch.testing.assert_close(lf, logits)
        assert torch.equal(pf, pred)
    torch.testing.assert_close(eng.logits(X), lf)  # logits() takes the fp32 serving path
    # after training steps the fragment copies the serving pipeline reads follow the new weights
    y = torch.randint(0, 6, (B,), device=cuda, generator=g).to(torch.int32)
    Xb = pad_input_bf16(X, eng.layout.in_pad)
    for _ in range(3):
        eng.train_step(Xb, y, B)
    lf2, pf2 = eng.infer_fused_f32(X)
    ref2 = eng.torch_forward(eng.P, Xp).float()
    assert float((lf2 - ref2).norm() / ref2.norm()) < 2e-2
    assert float((pf2.long() == torch.argmax(ref2, 1)).float().mean()) > 0.97


def test_find_thresholds_device_matches_numpy():
    """Device findSplits (HIP Philox sample mask + one sort) == the NumPy oracle on the host."""
    import numpy as np

    from har.ops import tree as T

    g = torch.Generator().manual_seed(3)
    X = torch.randn(60000, 13, generator=g)
    X[:, 1] = torch.round(X[:, 1] * 3)        # few distinct values
    X[torch.rand(60000, generator=g) < 0.2, 2] = float("nan")
    X[:, 3] = 2.0                             # constant column
    for row0, n_total in ((0, None), (120000, 480000)):
        a = T.find_thresholds(X.numpy(), 32, seed=5, row_offset=row0, n_total=n_total)
        b = T.find_thresholds_device(X.cuda(), 32, seed=5, row_offset=row0, n_total=n_total)
        for f in range(X.shape[1]):
            assert np.array_equal(a[f], b[f]), f


@pytest.mark.parametrize("n,F", [(10000, 43), (3853, 300), (1, 3), (16384, 5), (777, 1)])
def test_sort_columns_matches_torch_sort(cuda, n, F):
    """findSplits' per-feature LDS bitonic sort (tree.hip sort_columns) against torch.sort of the
    transposed sample: same ascending values, NaN last; ties, +-0 and constant columns included."""
    from har.ops import _native

    g = torch.Generator(device=cuda).manual_seed(n + F)
    X = torch.randn(n, F, device=cuda, generator=g)
    X[torch.rand(n, F, device=cuda, generator=g) < 0.1] = float("nan")
    X[:, 0] = torch.round(X[:, 0] * 2) / 2  # heavy ties
    if F > 1:
        X[:, 1] = 3.0  # constant column
    if F > 2:
        X[: n // 2, 2] = -0.0
    out = torch.empty(F, n, device=cuda)
    _native.kernels().sort_columns(X.data_ptr(), n, F, F, out.data_ptr(), _native.stream_ptr())
    ref = torch.sort(X.t().contiguous(), dim=1).values
    assert torch.equal(torch.isnan(out), torch.isnan(ref))
    assert torch.equal(torch.nan_to_num(out, nan=0.0), torch.nan_to_num(ref, nan=0.0))



def _frag_reference(M: torch.Tensor) -> torch.Tensor:
    """Independent construction of the fragment order of mlp.hip frag_pos: [R][C] -> blocks of 16 rows x
    32 k, one KB each, in MFMA lane order inside (lane l = 16 g + row reads the 16 bytes at 16 l: row,
    k = 8 g .. 8 g + 7)."""
    R, C = M.shape
    t = M.reshape(R // 16, 16, C // 32, 4, 8)        # (row block, row, k chunk, k group g, k)
    return t.permute(0, 2, 3, 1, 4).reshape(-1)      # (row block, k chunk, g, row, k)


@pytest.mark.parametrize("F", [43, 20])
def test_mlp_fragment_copies_track_pb(cuda, F):
    """The step's fragment-ordered weight copies (Pf = W0 | W1 | W1^T in MFMA fragment order): the W0 /
    W1 copies equal the flat bf16 copy Pb after the engine's init and after every fused Adam update;
    the W1^T copy is written by the step's forward from the W1 it ran with (the backward of the same
    step reads it), so after a step it holds the W1 from BEFORE that step's update."""
    from har.models.mlp import MLPEngine, pad_input_bf16

    B = 4096
    e = MLPEngine([F, 256, 256, 6], B, cuda, lr=1e-2, seed=11)
    assert e.step_ok
    g = torch.Generator(device=cuda).manual_seed(2)
    X = pad_input_bf16(torch.randn(B, F, device=cuda, generator=g), e.layout.in_pad)
    y = torch.randint(0, 6, (B,), device=cuda, generator=g).to(torch.int32)
    L = e.layout
    W1_used = L.view(e.Pb, "W1").clone()
    for step in range(3):
        if step:
            W1_used = L.view(e.Pb, "W1").clone()
            e.train_step(X, y, B)
        torch.cuda.synchronize()
        W0, W1 = L.view(e.Pb, "W0"), L.view(e.Pb, "W1")
        want = torch.cat([_frag_reference(W0), _frag_reference(W1), _frag_reference(W1_used.T.contiguous())])
        assert torch.equal(e.Pf, want), f"fragment copies differ from Pb after step {step}"
        if step:
            assert not torch.equal(W1, W1_used), "the update did not move W1"


@pytest.mark.parametrize("H,F,B", [(256, 43, 256), (128, 43, 256), (256, 20, 512), (128, 20, 64)])
def test_mlp_small_step_matches_other_paths(cuda, monkeypatch, H, F, B):
    """The small-batch step (mlp_small.hip: one workgroup per 32-row tile + the reduction / Adam kernel)
    against the engine's other native path on the same batches (the three-kernel step for H = 256, the
    fused forward + GEMM backward for H = 128): parameters after three Adam steps, loss and #correct;
    the fragment copies (W0, W1 and the W1^T copy the small path's Adam keeps current) equal Pb; two
    small-path engines are bit-identical."""
    from har.models.mlp import MLPEngine, pad_input_bf16

    g = torch.Generator(device=cuda).manual_seed(17)
    X = torch.randn(B, F, device=cuda, generator=g)
    y = torch.randint(0, 6, (B,), device=cuda, generator=g).to(torch.int32)
    engines = []
    for flag in ("1", "1", "0"):
        monkeypatch.setenv("HAR_MLP_SMALL", flag)
        e = MLPEngine([F, H, H, 6], B, cuda, lr=1e-3, seed=5)
        Xb = pad_input_bf16(X, e.layout.in_pad)
        for _ in range(3):
            e.train_step(Xb, y, B)
        torch.cuda.synchronize()
        assert (e.last_path == "small") == (flag == "1")
        engines.append((e, e.last_loss_and_correct()))
    (a, lca), (a2, lca2), (b, lcb) = engines
    assert torch.equal(a.P, a2.P) and lca == lca2
    torch.testing.assert_close(a.P, b.P, rtol=0, atol=5e-4)
    assert abs(lca[0] - lcb[0]) / lcb[0] < 2e-3 and abs(lca[1] - lcb[1]) <= 2
    L = a.layout
    W0, W1 = L.view(a.Pb, "W0"), L.view(a.Pb, "W1")
    want = torch.cat([_frag_reference(W0), _frag_reference(W1), _frag_reference(W1.T.contiguous())])
    assert torch.equal(a.Pf, want), "small-path fragment copies differ from Pb"


@pytest.mark.parametrize("metric", ["accuracy", "f1", "weightedPrecision", "areaUnderROC", "areaUnderPR", "mae"])
def test_batched_cv_metrics_gpu_match_cpu(cuda, metric):
    """CrossValidator scoring of B models at once: the batched confusion-matrix kernel and the
    segmented-sort + batched roc.hip pass give the CPU definitions (one-hot einsum, one sort per
    model) for every model / fold mask, ties in the scores included."""
    from har.evaluation.metrics import batched_metrics

    g = torch.Generator().manual_seed(21)
    B, N, K = 7, 3001, 6
    label = torch.randint(0, K, (N,), generator=g)
    pred = torch.randint(0, K, (B, N), generator=g)
    mask = torch.rand(B, N, generator=g) < 0.3
    raw = torch.round(torch.randn(B, N, K, generator=g) * 4) / 4  # coarse scores: many ties
    cpu = batched_metrics(metric, label, pred, mask, K, raw)
    gpu = batched_metrics(metric, label.to(cuda), pred.to(cuda), mask.to(cuda), K, raw.to(cuda))
    np.testing.assert_allclose(gpu, cpu, rtol=1e-9, atol=1e-12)


def test_batched_roc_with_minus_inf_scores_matches_cpu(cuda):
    """Selected rows whose score is -inf (a margin that overflowed) sort among the unselected rows
    under a -inf sentinel; the batched pass must still score exactly the selected rows."""
    from har.evaluation.metrics import batched_metrics

    g = torch.Generator().manual_seed(5)
    B, N, K = 5, 1201, 6
    label = torch.randint(0, K, (N,), generator=g)
    pred = torch.randint(0, K, (B, N), generator=g)
    mask = torch.rand(B, N, generator=g) < 0.4
    raw = torch.round(torch.randn(B, N, K, generator=g) * 4) / 4
    raw[:, ::7, 1] = float("-inf")  # selected and unselected rows alike
    for metric in ("areaUnderROC", "areaUnderPR"):
        cpu = batched_metrics(metric, label, pred, mask, K, raw)
        gpu = batched_metrics(metric, label.to(cuda), pred.to(cuda), mask.to(cuda), K, raw.to(cuda))
        np.testing.assert_allclose(gpu, cpu, rtol=1e-9, atol=1e-12)


def test_batched_confusion_rejects_out_of_range_labels_and_weights_rows(cuda):
    from har.evaluation.metrics import batched_metrics

    g = torch.Generator().manual_seed(6)
    B, N, K = 3, 500, 4
    label = torch.randint(0, K, (N,), generator=g)
    pred = torch.randint(0, K, (B, N), generator=g)
    w = torch.rand(B, N, generator=g)  # fractional row weights: the weighted definition, as on the CPU
    np.testing.assert_allclose(batched_metrics("accuracy", label.to(cuda), pred.to(cuda), w.to(cuda), K),
                               batched_metrics("accuracy", label, pred, w, K), rtol=1e-9)
    bad = label.clone()
    bad[3] = K
    with pytest.raises(ValueError):
        batched_metrics("accuracy", bad.to(cuda), pred.to(cuda), (w > 0.5).to(cuda), K)
