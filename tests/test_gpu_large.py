"""Large and maximum frame sizes.

* 4096 x 4096: full parity against the C oracle (same contract as
  test_gpu_parity.assert_parity: identical keypoint count and emission order,
  |dx|,|dy| <= 1e-4, descriptors within +-1).  ~10 s of oracle time on the
  host.
* 8192 x 8192 (config #5, 13 octaves, ~16 GB of pyramid): full parity
  against the C oracle (~1 min and ~20 GB of host memory), plus the
  size-independent properties: determinism, emission order (keys strictly
  increasing), descriptor range, the single-frame and the batch entry points
  agreeing, and octave coverage.
* 16384 x 9000: octave 0 (32768 x 18000 f32) is a plane over 2^31 bytes, so
  every stage that addresses a plane must do it with offsets that do not
  wrap (k_orient's buffer resource spans only the patch's rows); full parity
  against the oracle (~2 min, ~40 GB of host memory).
* Over 8192 px on one side (the 2x seed is then wider than 16384, which needs
  the 15-bit x/y fields of the emission key): narrow strips 8200 x 48,
  48 x 8400 and 16384 x 24 against the oracle, plus a banded merge of the
  tall one.
* Above the 16384-pixel key field: rejected with an error, no launch.
Frames are tiled from a 2048 x 2048 synthetic frame (synth.frame generates
the blob field as one dense product, too large to form at 8192^2) plus
seeded noise, so the content has blobs at every scale and no repeats the
detector could merge.
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _tiled(n, seed):
    import synth
    base = synth.frame(2048, 2048, seed).astype(np.int16)
    img = np.tile(base, (n // 2048, n // 2048))
    noise = np.random.default_rng(seed).integers(-2, 3, img.shape, dtype=np.int16)
    return np.clip(img + noise, 0, 255).astype(np.uint8)


def _emission_sorted(keys):
    k = np.asarray(keys, dtype=np.uint64)
    return bool(np.all(k[1:] > k[:-1]))


def test_large_4096_parity(pkg, ctx, oracle):
    from test_gpu_parity import assert_parity
    img = _tiled(4096, 31)
    kp_o, desc_o, ext_o = oracle.sift(img, internal=True)
    res = ctx.sift(img)
    assert len(res) > 10000
    assert_parity(pkg, res, kp_o, desc_o, ext_o)


@pytest.mark.timeout(900)
def test_max_8192_parity(pkg, ctx, oracle):
    """Config #5 against the oracle (src/lib.rs:131-143 has no size limit)."""
    from test_gpu_parity import assert_parity
    img = _tiled(8192, 47)
    res = ctx.sift(img)
    kp_o, desc_o, ext_o = oracle.sift(img, internal=True)
    assert len(res) > 50000
    assert_parity(pkg, res, kp_o, desc_o, ext_o)


@pytest.mark.timeout(900)
def test_plane_over_2gb_parity(pkg, ctx, oracle):
    """Octave-0 planes above 2^31 bytes: 32-bit plane offsets would wrap
    (k_orient reads gradients through a buffer resource)."""
    from test_gpu_parity import assert_parity
    img = np.ascontiguousarray(_tiled(16384, 53)[:9000])
    res = ctx.sift(img)
    kp_o, desc_o, ext_o = oracle.sift(img, internal=True)
    assert len(res) > 50000
    # keypoints from the rows whose octave-0 byte offsets pass 2^31
    assert (res.keypoints_array[:, 1] * 2 * 32768 * 4 > 2 ** 31).sum() > 1000
    assert_parity(pkg, res, kp_o, desc_o, ext_o)


def test_max_8192_properties(pkg, ctx):
    img = _tiled(8192, 47)
    a = ctx.sift(img)
    b = ctx.sift(img)
    assert a == b  # deterministic, bit for bit
    n = len(a)
    assert n > 50000, n
    assert _emission_sorted(a.keys)  # the reference's lazy emission order
    f = pkg.key_fields(a.keys)
    assert np.all(f["frame"] == 0)
    # 13 octaves for 8192^2 (src/lib.rs:133-134); keypoints come from the
    # first several of them, none from beyond the last
    assert f["octave"].max() <= 12 and len(np.unique(f["octave"])) >= 6
    kp = a.keypoints_array
    assert np.all(np.isfinite(kp))
    assert kp[:, 0].min() >= 0 and kp[:, 0].max() < 8192 and kp[:, 1].min() >= 0 and kp[:, 1].max() < 8192
    d = a.descriptors.astype(np.int64)
    assert d.shape == (n, 128) and d.max() <= 255
    # normalised descriptors: every vector has energy (the 512 scale after
    # the 0.2 clamp puts |v| near 512; rounding and the 255 cap keep it below)
    nrm = np.sqrt((d * d).sum(1))
    assert nrm.min() > 200 and nrm.max() < 560, (nrm.min(), nrm.max())
    # the batch entry point gives the same result for the same frame
    (c,) = ctx.sift_batch(img[None])
    assert c == a


@pytest.mark.parametrize("w,h", [(8200, 48), (48, 8400), (16384, 24)])
def test_oversize_side_parity(pkg, ctx, oracle, w, h):
    """Octave-0 coordinates reach 2*side - 6 > 16383: the key's x/y fields
    must hold them (src/lib.rs:131-143 has no size limit)."""
    import synth
    from test_gpu_parity import assert_parity
    img = synth.frame(w, h, 5 + w % 7)
    kp_o, desc_o, ext_o = oracle.sift(img, internal=True)
    res = ctx.sift(img)
    assert len(res) > 100
    assert_parity(pkg, res, kp_o, desc_o, ext_o)
    f = pkg.key_fields(res.keys)
    big = f["x_init"] if w > h else f["y_init"]
    assert big.max() > 16383  # the case a 14-bit field could not hold
    assert _emission_sorted(res.keys)


def test_oversize_side_bands(pkg, ctx):
    import shard
    import synth
    img = synth.frame(48, 8400, 6)
    whole = ctx.sift(img)
    parts = []
    for r in range(3):
        b = shard.sift_row_bands(ctx, img, band=r, n_bands=3)
        parts.append((b.keypoints_array, b.descriptors, b.keys))
    k, d, y = shard.merge_bands(parts)
    assert np.array_equal(y, whole.keys)
    assert np.array_equal(k.view(np.uint32), whole.keypoints_array.view(np.uint32))
    assert np.array_equal(d, whole.descriptors)


def test_too_large_rejected(pkg, ctx):
    img = np.zeros((16, 16385), np.uint8)
    with pytest.raises(pkg.SiftMiError):
        ctx.sift(img)
