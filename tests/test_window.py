"""Window featurization (K22): definitions on a hand-made window, synthetic
streams, and the HIP kernel vs the PyTorch oracle."""
import math

import numpy as np
import pytest
import torch

from har.data.synth import StreamSpec, generate_stream
from har.features.window import WindowFeaturizer, feature_names, n_features, window_count, window_features_torch


def test_feature_layout():
    names = feature_names()
    assert len(names) == n_features(3) == 55
    assert names[:3] == ["X0", "X1", "X2"] and names[30:36] == ["XAVG", "YAVG", "ZAVG", "XPEAK", "YPEAK", "ZPEAK"]
    assert names[42] == "RESULTANT"  # the WISDM-43 block comes first
    assert len(feature_names(["AX", "AY", "AZ", "GX", "GY", "GZ", "MX", "MY", "MZ"])) == n_features(9) == 165


def test_definitions_on_one_window():
    W, hz = 40, 20.0
    t = torch.arange(W, dtype=torch.float64)
    x = torch.sin(2 * math.pi * t / 10)            # period 10 samples = 500 ms
    y = torch.full((W,), 9.81, dtype=torch.float64)
    z = torch.linspace(-1, 1, W, dtype=torch.float64)
    f = window_features_torch(torch.stack([x, y, z], 1), W, W, hz)[0].double()
    assert abs(f[30] - x.mean()) < 1e-6 and abs(f[31] - 9.81) < 1e-5
    assert abs(f[33] - 500.0) < 1e-3               # XPEAK: mean time between peaks (ms)
    assert math.isnan(float(f[34]))                 # constant axis: no peaks -> '?'
    assert abs(f[36] - (x - x.mean()).abs().mean()) < 1e-6
    assert abs(f[39] - x.std(unbiased=False)) < 1e-6
    assert abs(f[42] - torch.sqrt(x * x + y * y + z * z).mean()) < 1e-5
    assert abs(f[0:10].sum() - 1.0) < 1e-6 and abs(f[20:30].sum() - 1.0) < 1e-6
    assert abs(f[52] - float(np.corrcoef(x, y)[0, 1] if y.std() > 0 else 0.0)) < 1e-6  # y constant -> 0


def test_window_count_and_halo():
    assert window_count(1000, 200, 200) == 5 and window_count(1000, 200, 100) == 9
    fz = WindowFeaturizer(hz=50, seconds=10, overlap=0.5)
    assert fz.window == 500 and fz.stride == 250 and fz.halo() == 250


def test_wide_window_fallback_chunks_match_one_shot(monkeypatch):
    """The fallback for windows too wide for the kernel's LDS images computes the torch definition in
    chunks of windows (each chunk's sample range sliced from the stream): with tiny chunks (1 and 3
    windows) the rows equal the one-shot definition, and the warning is raised once per shape."""
    import warnings

    from har.features import window as wmod

    spec = StreamSpec(axes=6, window=300, seed=4)
    s, _ = generate_stream(6, spec)
    ref = window_features_torch(s, 300, 170, 50.0)
    for chunk_windows in (1, 3):
        monkeypatch.setattr(wmod, "_WIDE_CHUNK_BYTES", 6 * 300 * 8 * 6 * chunk_windows)
        monkeypatch.setattr(wmod, "_WIDE_WARNED", set())
        with warnings.catch_warnings(record=True) as rec:
            warnings.simplefilter("always")
            out = wmod._wide_windows(s, 300, 170, 50.0)
        assert len(rec) == 1 and "exceed the kernel" in str(rec[0].message)
        assert out.shape == ref.shape
        torch.testing.assert_close(out, ref, rtol=0, atol=0, equal_nan=True)


def test_synth_stream_shard_invariant():
    spec = StreamSpec(seed=3)
    s_all, y_all = generate_stream(12, spec)
    s_b, y_b = generate_stream(6, spec, first_window=6)
    assert torch.equal(y_all[6:], y_b)
    assert s_all.shape == (12 * 200, 3)


@pytest.mark.gpu
@pytest.mark.parametrize("axes,window,stride", [(3, 200, 200), (3, 500, 250), (9, 500, 500), (6, 97, 31), (3, 97, 40),
                                               (9, 37, 37), (3, 700, 350), (6, 1100, 1100),
                                               # fixed-length runs overhanging the window (8 x 25 / 16 x 13
                                               # groups, D = 1 .. 15 copies of sample W - 1)
                                               (3, 193, 97), (6, 199, 50), (9, 185, 100), (3, 195, 195),
                                               (3, 207, 207), (6, 193, 193)])
def test_window_kernel_matches_torch(cuda, axes, window, stride):
    from har.features.window import window_features

    spec = StreamSpec(axes=axes, window=window, seed=axes)
    s, _ = generate_stream(64, spec)
    s = s[: s.shape[0] - 13]  # ragged tail: last partial window dropped
    ref = window_features_torch(s, window, stride, 50.0)
    out = window_features(s.to(cuda), window, stride, 50.0).cpu()
    assert out.shape == ref.shape
    nb = 10 * axes
    # bins: float32 vs float64 bin edges may move a boundary sample by one bin
    assert (out[:, :nb] - ref[:, :nb]).abs().max() <= 1.0 / window + 1e-6
    torch.testing.assert_close(out[:, nb:], ref[:, nb:], rtol=2e-4, atol=2e-4, equal_nan=True)


@pytest.mark.gpu
@pytest.mark.parametrize("axes,window,stride", [(3, 200, 200), (9, 500, 500), (3, 128, 64)])
def test_window_kernel_mlp_output(cuda, axes, window, stride):
    """MLP-input mode of the window kernel: bf16 standardized, NaN-filled, zero-padded rows equal
    the fp32 features pushed through the same transform (bf16 rounding of the result only)."""
    from har.features.window import window_features, window_features_mlp

    spec = StreamSpec(axes=axes, window=window, seed=axes + 7)
    s, _ = generate_stream(48, spec, cuda)
    F = n_features(axes)
    mean = torch.randn(F, device=cuda)
    inv_std = torch.rand(F, device=cuda) + 0.5
    pad = (F + 31) // 32 * 32
    ref = (torch.nan_to_num(window_features(s, window, stride, 50.0), nan=-1.0) - mean) * inv_std
    out = window_features_mlp(s, window, stride, 50.0, mean, inv_std, pad)
    assert out.shape == (ref.shape[0], pad) and out.dtype == torch.bfloat16
    assert torch.count_nonzero(out[:, F:]) == 0
    torch.testing.assert_close(out[:, :F].float(), ref.to(torch.bfloat16).float(), rtol=0, atol=0)


@pytest.mark.gpu
@pytest.mark.parametrize("stride,nwin", [(200, 100_000), (100, 131_071)])
def test_window_kernel_large_counts_match_torch(cuda, stride, nwin):
    """The large-count dispatches of the window kernel at >= 100k windows — stride 200 (16-lane groups,
    padded per-window images) and stride 100 (8-lane groups on a shared span, the 1B-sample pass's shape)
    — against the PyTorch oracle (torch ops on the device), fp32 features and the MLP-input rows."""
    from har.features.window import window_features, window_features_mlp

    W = 200
    spec = StreamSpec(axes=3, window=W, seed=11 + stride)
    n_seg = ((nwin - 1) * stride + W + W - 1) // W
    s, _ = generate_stream(n_seg, spec, cuda)
    s = s[: (nwin - 1) * stride + W]
    assert window_count(s.shape[0], W, stride) == nwin
    ref = window_features_torch(s, W, stride, 50.0)
    out = window_features(s, W, stride, 50.0)
    assert out.shape == ref.shape == (nwin, n_features(3))
    nb = 30
    assert float((out[:, :nb] - ref[:, :nb]).abs().max()) <= 1.0 / W + 1e-6
    # (the oracle computes in float64 on the device; bins may move a boundary sample by one bin).  The
    # peak times: a sample within fp32 rounding of the threshold mean + (max - mean) / 2 counts as a peak
    # in one arithmetic and not the other — at this count a handful of windows (1 in 2.5M values seen)
    pk = slice(nb + 3, nb + 6)
    okp = torch.isclose(out[:, pk], ref[:, pk], rtol=2e-4, atol=2e-4, equal_nan=True)
    assert int((~okp).sum()) <= max(2, nwin // 20000), int((~okp).sum())
    rest = torch.cat([out[:, nb:nb + 3], out[:, nb + 6:]], 1)
    rest_ref = torch.cat([ref[:, nb:nb + 3], ref[:, nb + 6:]], 1)
    torch.testing.assert_close(rest, rest_ref, rtol=2e-4, atol=2e-4, equal_nan=True)
    F = n_features(3)
    g = torch.Generator(device=cuda).manual_seed(3)
    mean = torch.randn(F, device=cuda, generator=g)
    inv_std = torch.rand(F, device=cuda, generator=g) + 0.5
    mo = window_features_mlp(s, W, stride, 50.0, mean, inv_std, 64)
    assert mo.shape == (nwin, 64) and torch.count_nonzero(mo[:, F:]) == 0
    want = ((torch.nan_to_num(out, nan=-1.0) - mean) * inv_std).to(torch.bfloat16)
    # (the two instantiations may differ in a feature's last fp32 bit, which the bf16 rounding then
    # shows as one bf16 ulp in a few values; everything else bit-equal)
    torch.testing.assert_close(mo[:, :F].float(), want.float(), rtol=2 ** -7, atol=1e-6)
    assert int((mo[:, :F] != want).sum()) <= max(4, mo.numel() // 100000)



@pytest.mark.gpu
@pytest.mark.parametrize("stride", [200, 100])
def test_window_kernel_saturated_and_constant_runs(cuda, stride):
    """Clipped sensor data: runs where every sample of a lane's 25 (stride 100) or 13 (stride 200) sits
    at the window maximum — the unclamped bin-10 slot of the 5-bit packed histogram (window.hip SB = 5)
    full, then folded into bin 9 — and constant windows (range 0: every sample in bin 0, std 0,
    correlations 0), against the PyTorch oracle."""
    from har.features.window import window_features

    W = 200
    spec = StreamSpec(axes=3, window=W, seed=21)
    n_seg = 40
    s, _ = generate_stream(n_seg, spec, cuda)
    s = s.clone()
    hi = float(s.max()) * 0.25
    s = s.clamp(max=hi)                      # long runs at the clip value = the window max
    s[5 * W:7 * W] = 1.5                     # two constant windows (stride 200), more overlapping ones
    s[11 * W:11 * W + 60, 1] = 9.0           # a spike at the start of a window: max at t < 60 only
    nwin = (s.shape[0] - W) // stride + 1
    s = s[: (nwin - 1) * stride + W]
    ref = window_features_torch(s, W, stride, 50.0)
    out = window_features(s, W, stride, 50.0)
    assert out.shape == ref.shape
    nb = 30
    assert float((out[:, :nb] - ref[:, :nb]).abs().max()) <= 1.0 / W + 1e-6
    # every window's 10 bins of an axis sum to 1 (nothing lost in the packed slots)
    sums = out[:, :nb].reshape(-1, 3, 10).sum(-1)
    torch.testing.assert_close(sums, torch.ones_like(sums), rtol=0, atol=1e-5)
    torch.testing.assert_close(out[:, nb:], ref[:, nb:], rtol=2e-4, atol=2e-4, equal_nan=True)


@pytest.mark.gpu
@pytest.mark.parametrize("axes,window,stride", [(3, 3, 1), (3, 5, 2), (3, 8, 8), (6, 16, 3), (3, 17, 17), (9, 33, 11),
                                               (3, 64, 64), (3, 129, 64)])
def test_window_kernel_short_windows_match_torch(cuda, axes, window, stride):
    """Short windows: runs much longer than the window (up to LPW x 5 run slots for 3 samples), so most
    lanes hold only copies of sample W - 1 whose contributions the kernel subtracts (D = LPW C - W), and
    the peak masks cover almost every bit — against the PyTorch oracle."""
    from har.features.window import window_features

    spec = StreamSpec(axes=axes, window=max(window, 16), seed=window + axes)
    s, _ = generate_stream(24, spec)
    ref = window_features_torch(s, window, stride, 50.0)
    out = window_features(s.to(cuda), window, stride, 50.0).cpu()
    assert out.shape == ref.shape and out.shape[0] > 0
    nb = 10 * axes
    assert (out[:, :nb] - ref[:, :nb]).abs().max() <= 1.0 / window + 1e-6
    torch.testing.assert_close(out[:, nb:], ref[:, nb:], rtol=2e-4, atol=2e-4, equal_nan=True)


@pytest.mark.gpu
@pytest.mark.parametrize("axes,window,stride", [(3, 1984, 1984), (3, 1985, 1000), (9, 2600, 1300), (6, 4001, 4001)])
def test_window_kernel_long_windows_match_torch(cuda, axes, window, stride):
    """Long windows: 64-lane groups of 31-sample runs up to 1,984 samples, then the LDS-streaming kernel;
    windows whose images exceed the LDS (9 x 2,600, 6 x 4,001: kernel contract code -5) fall back to the
    torch definition on the device with a warning — all against the PyTorch oracle, fp32 features and
    the MLP-input rows."""
    import warnings

    from har.features.window import window_features, window_features_mlp

    spec = StreamSpec(axes=axes, window=window, seed=window % 97)
    s, _ = generate_stream(6, spec)
    ref = window_features_torch(s, window, stride, 50.0)
    with warnings.catch_warnings():
        warnings.simplefilter("ignore")
        out = window_features(s.to(cuda), window, stride, 50.0).cpu()
    assert out.shape == ref.shape and out.shape[0] > 0
    nb = 10 * axes
    assert (out[:, :nb] - ref[:, :nb]).abs().max() <= 1.0 / window + 1e-6
    torch.testing.assert_close(out[:, nb:], ref[:, nb:], rtol=2e-4, atol=2e-4, equal_nan=True)
    F = n_features(axes)
    mean = torch.zeros(F, device=cuda)
    inv_std = torch.ones(F, device=cuda)
    with warnings.catch_warnings():
        warnings.simplefilter("ignore")
        mo = window_features_mlp(s.to(cuda), window, stride, 50.0, mean, inv_std, (F + 31) // 32 * 32)
    assert mo.shape == (ref.shape[0], (F + 31) // 32 * 32) and torch.count_nonzero(mo[:, F:]) == 0
    want = torch.nan_to_num(out, nan=-1.0).to(torch.bfloat16)
    torch.testing.assert_close(mo[:, :F].float().cpu(), want.float(), rtol=2 ** -7, atol=1e-3)
