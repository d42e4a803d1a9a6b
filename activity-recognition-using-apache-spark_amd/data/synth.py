"""Synthetic accelerometer / IMU streams with class-conditional dynamics.

The reference only ships the pre-windowed WISDM table
(``Main/wisdm_main_ver_0.0/data/wisdm_data.csv``); the north-star configs in
BASELINE.json need *raw* streams ("Synthetic 1B-sample 3-axis stream",
"Synthetic 12-class / 9-axis IMU") that are featurized on the GPU by the window
kernel (``har.features.window``).  There is no network for
real datasets, so streams are generated here.

Model (per window of ``spec.window`` samples, one activity label per window):

* labels come in runs of ``spec.run_windows`` windows (people keep doing an
  activity for a while); for 6 classes the draw follows WISDM's class priors
  (Walking 2081, Jogging 1625, Upstairs 632, Downstairs 528, Sitting 306,
  Standing 246 — ``result.txt:36-41``), uniform otherwise;
* each class has a gravity orientation, a step frequency, per-axis amplitudes,
  a second-harmonic weight and a noise level.  The first six classes mimic the
  WISDM activities (two static postures, four periodic gaits of different
  cadence and intensity); further classes get random parameters;
* every activity run is one "session" with its own device orientation (the
  gravity direction is perturbed by ``spec.orientation_jitter``), cadence and
  intensity — so postures and gaits of different classes overlap the way they do
  across WISDM's 36 users (synthetic RandomForest accuracy ~0.9, not 1.0);
* every window further jitters frequency, amplitude and phase, then adds
  Gaussian sensor noise.

Every random number is a pure function of ``(spec.seed, global window id,
sample, axis)`` through a 32-bit integer hash, so a stream generated in shards
(``first_window=...``) is bit-identical to one generated whole — the same
world-size invariance the Philox split uses.  All
arithmetic is int64/fp32 torch ops, so the generator runs on whichever device
the caller names (chunks of 65,536 windows on an MI355X take a few ms).
"""
from __future__ import annotations

import math
from dataclasses import dataclass
from typing import Optional, Tuple

import torch

M32 = 0xFFFFFFFF
WISDM_PRIORS = (2081, 1625, 632, 528, 306, 246)

# field ids mixed into the per-window hash (fixed, so streams are reproducible)
_F_LABEL, _F_PHASE, _F_FREQ, _F_AMP, _F_ORI, _F_NOISE = 1, 2, 3, 4, 5, 6
_F_SFREQ, _F_SAMP, _F_SORI, _F_SPROF = 7, 8, 9, 10


@dataclass(frozen=True)
class StreamSpec:
    num_classes: int = 6
    axes: int = 3
    hz: float = 20.0          # WISDM v1.1 sampling rate
    window: int = 200         # 10 s at 20 Hz
    seed: int = 2018
    run_windows: int = 8      # windows per activity run
    noise_scale: float = 1.0  # multiplies every class's noise level (difficulty knob)
    orientation_jitter: float = 0.55  # per-session gravity-direction perturbation (difficulty knob)

    @property
    def seconds(self) -> float:
        return self.window / self.hz


def _mul32(x: torch.Tensor, c: int) -> torch.Tensor:
    """(x * c) mod 2^32 for x in [0, 2^32) held in int64, without int64 overflow."""
    lo, hi = c & 0xFFFF, c >> 16
    return (x * lo + (((x * hi) & 0xFFFF) << 16)) & M32


def hash32(x: torch.Tensor) -> torch.Tensor:
    """lowbias32 integer hash on int64 tensors holding uint32 values."""
    x = x & M32
    x = x ^ (x >> 16)
    x = _mul32(x, 0x7FEB352D)
    x = x ^ (x >> 15)
    x = _mul32(x, 0x846CA68B)
    return x ^ (x >> 16)


def _key(seed: int, field: int) -> int:
    h = hash32(torch.tensor([(seed * 0x9E3779B1 + field * 0x85EBCA77) & M32], dtype=torch.int64))
    return int(h[0])


def _uniform(idx: torch.Tensor, key: int) -> torch.Tensor:
    """U(0,1) float32 (never exactly 0) for int64 indices < 2^62."""
    h = hash32((idx & M32) ^ hash32((idx >> 32) ^ key))
    return ((h >> 8).float() + 0.5) * (1.0 / (1 << 24))


def _normal(idx: torch.Tensor, key: int) -> torch.Tensor:
    u1 = _uniform(idx, key)
    u2 = _uniform(idx, key ^ 0x5BD1E995)
    return torch.sqrt(-2.0 * torch.log(u1)) * torch.cos(2.0 * math.pi * u2)


def class_params(spec: StreamSpec) -> dict:
    """Per-class dynamics (host tensors): gravity unit vector per axis triad, step
    frequency (Hz), per-axis amplitude (m/s^2), harmonic weight, noise level."""
    K, A = spec.num_classes, spec.axes
    g = torch.Generator().manual_seed(spec.seed * 7919 + 17)
    ntri = max(1, (A + 2) // 3)
    # WISDM-like presets: (freq, amplitude scale, harmonic, noise, gravity dir)
    presets = [
        (1.9, 3.5, 0.35, 0.6, (0.05, 1.0, 0.15)),    # Walking
        (2.7, 8.0, 0.50, 1.2, (0.10, 1.0, 0.30)),    # Jogging
        (1.6, 3.0, 0.45, 0.7, (0.20, 1.0, 0.35)),    # Upstairs
        (1.8, 4.2, 0.55, 0.9, (0.15, 1.0, 0.05)),    # Downstairs
        (0.0, 0.15, 0.0, 0.25, (0.10, 0.35, 1.0)),   # Sitting
        (0.0, 0.20, 0.0, 0.25, (0.05, 1.0, 0.10)),   # Standing
    ]
    freq = torch.empty(K)
    amp = torch.empty(K, A)
    harm = torch.empty(K)
    noise = torch.empty(K)
    grav = torch.empty(K, A)
    for c in range(K):
        if c < len(presets):
            f, s, h, n, gd = presets[c]
            gvec = torch.tensor(gd)
        else:
            f = float(torch.rand(1, generator=g)) * 3.0
            f = 0.0 if f < 0.4 else f
            s = 0.2 + float(torch.rand(1, generator=g)) * 7.0
            h = float(torch.rand(1, generator=g)) * 0.6
            n = 0.2 + float(torch.rand(1, generator=g)) * 1.0
            gvec = torch.rand(3, generator=g) * 2 - 1
        gvec = gvec / gvec.norm()
        shape = 0.3 + torch.rand(A, generator=g) * 0.7          # per-axis amplitude profile
        freq[c], harm[c], noise[c] = f, h, n * spec.noise_scale
        amp[c] = s * shape
        for t in range(ntri):
            a0, a1 = 3 * t, min(A, 3 * t + 3)
            scale = 9.81 if t == 0 else (1.0 if t == 1 else 40.0)   # accel, gyro (rad/s), mag (uT)
            rot = torch.rand(3, generator=g) * 0.4 - 0.2 if t else torch.zeros(3)
            grav[c, a0:a1] = (gvec + rot)[: a1 - a0] * scale
    return {"freq": freq, "amp": amp, "harm": harm, "noise": noise, "grav": grav}


def window_labels(spec: StreamSpec, first_window: int, n_windows: int, device=None) -> torch.Tensor:
    """int64 labels of global windows ``[first_window, first_window + n_windows)``."""
    wid = torch.arange(first_window, first_window + n_windows, dtype=torch.int64, device=device)
    u = _uniform(wid // spec.run_windows, _key(spec.seed, _F_LABEL))
    K = spec.num_classes
    if K == len(WISDM_PRIORS):
        p = torch.tensor(WISDM_PRIORS, dtype=torch.float32, device=device)
        cdf = torch.cumsum(p / p.sum(), 0)
        return torch.searchsorted(cdf[:-1].contiguous(), u.contiguous(), right=True).to(torch.int64)
    return torch.clamp((u * K).to(torch.int64), max=K - 1)


def generate_stream(n_windows: int, spec: StreamSpec = StreamSpec(), device=None,
                    first_window: int = 0, dtype=torch.float32) -> Tuple[torch.Tensor, torch.Tensor]:
    """Return ``(stream [n_windows * window, axes], labels [n_windows])`` for the
    global windows starting at ``first_window``.  Shards concatenate exactly."""
    dev = torch.device(device) if device is not None else torch.device("cpu")
    W, A = spec.window, spec.axes
    y = window_labels(spec, first_window, n_windows, dev)
    P = {k: v.to(dev) for k, v in class_params(spec).items()}
    wid = torch.arange(first_window, first_window + n_windows, dtype=torch.int64, device=dev)
    run = wid // spec.run_windows
    ar = torch.arange(A, device=dev)[None, :]
    # per-session (activity run) cadence, intensity, device orientation and axis profile
    sf = 1.0 + 0.15 * _normal(run, _key(spec.seed, _F_SFREQ))                               # [n]
    sa = torch.exp(0.3 * _normal(run, _key(spec.seed, _F_SAMP)))                            # [n]
    sori = _normal(run[:, None] * A + ar, _key(spec.seed, _F_SORI))                           # [n, A]
    sprof = torch.exp(0.35 * _normal(run[:, None] * A + ar, _key(spec.seed, _F_SPROF)))      # [n, A]
    # per-window jitter
    phase = _uniform(wid, _key(spec.seed, _F_PHASE)) * (2 * math.pi)                        # [n]
    fj = sf * (1.0 + 0.05 * _normal(wid, _key(spec.seed, _F_FREQ)))                         # [n]
    aj = sa * torch.exp(0.1 * _normal(wid, _key(spec.seed, _F_AMP)))                         # [n]
    ori = 0.3 * _normal(wid[:, None] * A + ar, _key(spec.seed, _F_ORI))                      # [n, A]
    grav = P["grav"][y]
    ntri = (A + 2) // 3
    for t in range(ntri):  # rotate each sensor triad's reference direction per session
        a0, a1 = 3 * t, min(A, 3 * t + 3)
        gv = grav[:, a0:a1]
        mag = gv.norm(dim=1, keepdim=True).clamp_min(1e-6)
        d = gv / mag + spec.orientation_jitter * sori[:, a0:a1]
        grav = torch.cat([grav[:, :a0], d / d.norm(dim=1, keepdim=True).clamp_min(1e-6) * mag, grav[:, a1:]], 1)
    freq = P["freq"][y] * fj
    t = torch.arange(W, device=dev, dtype=torch.float32) / spec.hz                          # [W]
    ang = 2 * math.pi * freq[:, None] * t[None, :] + phase[:, None]                         # [n, W]
    base = torch.sin(ang) + P["harm"][y][:, None] * torch.sin(2 * ang + 0.7)                 # [n, W]
    # per-axis phase offsets so the axes are correlated but not identical
    axis_shift = torch.arange(A, device=dev, dtype=torch.float32) * 0.9
    wave = torch.sin(ang[:, :, None] + axis_shift[None, None, :]) * 0.35 + base[:, :, None] * 0.65
    amp = (P["amp"][y] * sprof * aj[:, None])[:, None, :]                                  # [n, 1, A]
    sig = grav[:, None, :] + ori[:, None, :] + amp * wave                                     # [n, W, A]
    sidx = (wid[:, None, None] * W + torch.arange(W, device=dev)[None, :, None]) * A \
        + torch.arange(A, device=dev)[None, None, :]
    sig = sig + P["noise"][y][:, None, None] * _normal(sidx, _key(spec.seed, _F_NOISE))
    return sig.reshape(n_windows * W, A).to(dtype), y
