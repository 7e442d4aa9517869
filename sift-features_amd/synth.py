"""Seeded synthetic grayscale frames for tests and bench.py.

Smooth procedural content: mid-grey 128 background, 10 000 small 2-D Gaussian
blobs per megapixel (sigma U[1, 8] px, amplitude U[-80, 80]) plus 60 large
ones per megapixel (sigma U[10, 60], amplitude U[-60, 60]) and U[-3, 3]
noise, rounded and clamped to u8.  A 1920x1080 frame yields ~8.6e3
keypoints with the reference algorithm (real photos of the reference's
images/ give 4e3-1e4 at that size); pure white noise would inflate counts.

The blob field is separable: one (H x K) @ (K x W) product per frame, so the
torch path generates a batch directly on the GPU (bench.py).  The two paths
draw identical parameters; their u8 outputs can differ in rare rounding ties,
which is why every parity test feeds the SAME u8 array to both sides.
"""
import numpy as np


def _params(width, height, seed):
    r = np.random.default_rng(seed)
    area = width * height / 1e6
    nb1, nb2 = int(10000 * area), int(60 * area)
    cx = r.uniform(0, width, nb1 + nb2)
    cy = r.uniform(0, height, nb1 + nb2)
    sig = np.concatenate([r.uniform(1, 8, nb1), r.uniform(10, 60, nb2)])
    amp = np.concatenate([r.uniform(-80, 80, nb1), r.uniform(-60, 60, nb2)])
    noise_seed = int(r.integers(0, 2**31 - 1))
    return cx, cy, sig, amp, noise_seed


def frame(width, height, seed):
    """One (height, width) u8 frame, numpy (CPU)."""
    cx, cy, sig, amp, ns = _params(width, height, seed)
    xs = np.arange(width, dtype=np.float64)
    ys = np.arange(height, dtype=np.float64)
    gx = np.exp(-((xs[None, :] - cx[:, None]) ** 2) / (2 * sig[:, None] ** 2))  # (K, W)
    gy = np.exp(-((ys[:, None] - cy[None, :]) ** 2) / (2 * sig[None, :] ** 2))  # (H, K)
    img = (gy * amp[None, :]) @ gx + 128.0
    img += np.random.default_rng(ns).uniform(-3.0, 3.0, (height, width))
    return np.clip(np.rint(img), 0, 255).astype(np.uint8)


def frames(n, width, height, seed0=0):
    out = np.empty((n, height, width), np.uint8)
    for i in range(n):
        out[i] = frame(width, height, seed0 + i)
    return out


def frames_torch(n, width, height, seed0=0, device="cuda"):
    """(n, height, width) torch.uint8 frames generated on `device`."""
    import torch

    out = torch.empty((n, height, width), dtype=torch.uint8, device=device)
    xs = torch.arange(width, dtype=torch.float64, device=device)
    ys = torch.arange(height, dtype=torch.float64, device=device)
    for i in range(n):
        cx, cy, sig, amp, ns = _params(width, height, seed0 + i)
        t = lambda a: torch.as_tensor(a, dtype=torch.float64, device=device)
        cx, cy, sig, amp = t(cx), t(cy), t(sig), t(amp)
        gx = torch.exp(-((xs[None, :] - cx[:, None]) ** 2) / (2 * sig[:, None] ** 2))
        gy = torch.exp(-((ys[:, None] - cy[None, :]) ** 2) / (2 * sig[None, :] ** 2))
        img = (gy * amp[None, :]) @ gx + 128.0
        g = torch.Generator(device=device)
        g.manual_seed(ns)
        img += torch.rand((height, width), generator=g, dtype=torch.float64, device=device) * 6.0 - 3.0
        out[i] = torch.clamp(torch.round(img), 0, 255).to(torch.uint8)
    return out
