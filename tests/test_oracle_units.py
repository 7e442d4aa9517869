"""CPU unit tests of the oracle's building blocks (test infrastructure) and of
the package's host-side logic -- no GPU needed.

Expected values are the reference's own constants and formulas:
n_octaves (src/lib.rs:133-134), incremental octave sigmas (:220-229), the seed
sigma (:207), OpenCV's GaussianBlur kernel size cvRound(8*sigma+1)|1 and
BORDER_REFLECT_101, INTER_NEAREST picking (2x, 2y) and INTER_LINEAR's
half-pixel 0.25 / 0.75 weights for a 2x upsample (src/opencv_processing.rs).
"""
import numpy as np
import pytest


@pytest.mark.parametrize("w,h,n", [(320, 213, 8), (640, 480, 9), (1920, 1080, 10), (8192, 8192, 13),
                                   (16, 16, 4), (1, 1, 1)])
def test_n_octaves(oracle, w, h, n):
    assert oracle.n_octaves(w, h) == n


def test_octave_sigmas(oracle):
    s = oracle.octave_sigmas()
    np.testing.assert_allclose(s[1:], [1.226273, 1.545008, 1.946588, 2.452547, 3.090016], atol=2e-6)
    assert abs(oracle.seed_sigma() - 1.2489996) < 1e-6


def test_cv_kernel_sizes(oracle):
    sig = [oracle.seed_sigma()] + list(oracle.octave_sigmas()[1:])
    sizes = [len(oracle.cv_kernel(x)) for x in sig]
    assert sizes == [11, 11, 13, 17, 21, 27]
    for x in sig:
        k = oracle.cv_kernel(x)
        assert np.array_equal(k, k[::-1])
        assert abs(float(k.astype(np.float64).sum()) - 1.0) < 1e-6


def test_blur_constant_and_impulse(oracle):
    c = np.full((40, 50), 0.375, np.float32)
    np.testing.assert_allclose(oracle.gaussian_blur(c, 1.6), c, rtol=0, atol=1e-6)
    imp = np.zeros((41, 41), np.float32)
    imp[20, 20] = 1.0
    out = oracle.gaussian_blur(imp, 1.6)
    k = oracle.cv_kernel(1.6).astype(np.float64)
    r = len(k) // 2
    expect = np.outer(k, k)
    np.testing.assert_allclose(out[20 - r:21 + r, 20 - r:21 + r], expect, rtol=1e-5, atol=1e-8)
    # energy stays inside the kernel support
    assert np.abs(out).sum() - np.abs(out[20 - r:21 + r, 20 - r:21 + r]).sum() < 1e-7


def test_blur_reflect101_border(oracle):
    """Row 0 of a vertical ramp: BORDER_REFLECT_101 mirrors about row 0, so the
    blurred first row equals the kernel-weighted mirrored ramp."""
    h, w = 30, 8
    img = np.repeat(np.arange(h, dtype=np.float32)[:, None], w, axis=1) / h
    out = oracle.gaussian_blur(img, 1.2)
    k = oracle.cv_kernel(1.2).astype(np.float64)
    r = len(k) // 2
    col = img[:, 0].astype(np.float64)
    idx = np.abs(np.arange(-r, r + 1))  # reflect-101 about row 0
    assert abs(float(out[0, 3]) - float((k * col[idx]).sum())) < 1e-6


def test_resize_nearest_half(oracle):
    img = np.arange(12 * 10, dtype=np.float32).reshape(12, 10)
    out = oracle.resize_nearest(img, 5, 6)
    assert np.array_equal(out, img[0::2, 0::2][:6, :5])


def test_resize_linear_2x_weights(oracle):
    img = np.arange(4 * 6, dtype=np.float32).reshape(4, 6)
    out = oracle.resize_linear(img, 12, 8)
    # interior: dst x = 2k+1 -> 0.75*src[k] + 0.25*src[k+1] (half-pixel centres)
    assert abs(out[0, 3] - (0.75 * img[0, 1] + 0.25 * img[0, 2])) < 1e-6
    assert abs(out[0, 4] - (0.25 * img[0, 1] + 0.75 * img[0, 2])) < 1e-6
    # borders clamp
    assert out[0, 0] == img[0, 0] and out[0, 11] == img[0, 5]


def test_descriptor_normalised(oracle):
    rng = np.random.default_rng(3)
    img = rng.random((96, 96), dtype=np.float32)
    d = oracle.compute_descriptor(img, 48.0, 48.0, 2.0, 30.0)
    assert d.shape == (128,) and d.dtype == np.uint8
    n = np.sqrt((d.astype(np.float64) ** 2).sum())
    assert 480 < n < 530
    assert np.array_equal(d, oracle.compute_descriptor(img, 48.0, 48.0, 2.0, 30.0))


def test_features_limit_is_top_response(oracle):
    from conftest import load_golden
    img = load_golden("bird_small")["image"]
    kp, desc = oracle.sift(img)
    kl, dl = oracle.sift(img, features_limit=50)
    assert len(kl) == 50
    assert np.all(np.diff(kl[:, 4]) <= 0)  # response-descending
    assert np.isclose(kl[:, 4].min(), np.sort(kp[:, 4])[::-1][49])
    assert len(oracle.sift(img, features_limit=0)[0]) == 0
    k_all, _ = oracle.sift(img, features_limit=10 ** 6)
    assert len(k_all) == len(kp)


def test_flat_image_has_no_keypoints(oracle):
    kp, desc = oracle.sift(np.full((64, 80), 100, np.uint8))
    assert kp.shape == (0, 5) and desc.shape == (0, 128)


# ---- host-side package logic (no device calls) -----------------------------

def test_limit_argument(pkg):
    import sys
    S = sys.modules["sift_features_amd.sift"]
    assert S._limit(None) == -1 and S._limit(0) == 0 and S._limit(7) == 7
    with pytest.raises(ValueError):
        S._limit(-1)


def test_u8_image_validation(pkg):
    import sys
    S = sys.modules["sift_features_amd.sift"]
    with pytest.raises(TypeError):
        S._u8_image(np.zeros((4, 4), np.float32))
    with pytest.raises(TypeError):
        S._u8_image(np.zeros((4, 4, 3), np.uint8))
    a = np.zeros((8, 10), np.uint8)[:, ::2]  # non-unit column stride -> made contiguous
    assert S._u8_image(a).strides[1] == 1


def test_result_buffers_grow(pkg):
    rb = pkg.ResultBuffers(4)
    k, d, key = rb.views(3)
    assert k.shape == (3, 5) and d.shape == (3, 128) and key.shape == (3,)
    k, d, key = rb.views(100)
    assert k.shape == (100, 5) and len(rb.kps) >= 100


def test_key_fields_roundtrip(pkg):
    f, o, s, y, x, p = 37, 9, 2, 12345, 16000, 5
    key = (f << 42) | (o << 38) | (s << 36) | (y << 21) | (x << 6) | p
    d = pkg.key_fields(np.array([key], np.uint64))
    assert (d["frame"][0], d["octave"][0], d["s_init"][0], d["y_init"][0], d["x_init"][0], d["peak"][0]) == \
        (f, o, s, y, x, p)


def test_stable_sort_matches_snapshot_order(pkg):
    from conftest import load_golden
    g = load_golden("tree_small")["keypoints"]
    perm = np.random.default_rng(0).permutation(len(g))
    order = pkg.stable_sort_xy_size(g[perm])
    # same (x, y, size) sequence as the snapshot (rows tied on all three may swap)
    assert np.array_equal(g[perm][order][:, :3], g[:, :3])


# ---- ImageprocProcessing profile (restated third-party arithmetic; unpinned) --

def test_ip_kernel_sizes(oracle):
    import ctypes
    L = oracle.lib()
    L.oracle_ip_kernel.argtypes = [ctypes.c_float, ctypes.POINTER(ctypes.c_float)]
    k = (ctypes.c_float * 64)()
    sig = [oracle.seed_sigma()] + list(oracle.octave_sigmas()[1:])
    sizes = []
    for x in sig:
        n = L.oracle_ip_kernel(x, k)
        sizes.append(n)
        v = np.array(k[:n])
        assert np.array_equal(v, v[::-1]) and abs(float(v.astype(np.float64).sum()) - 1) < 1e-6
    assert sizes == [7, 7, 9, 9, 11, 15]  # radius ceil(2 sigma)


def test_ip_resize_semantics(oracle):
    img = np.arange(6 * 8, dtype=np.float32).reshape(6, 8) / 64.0
    near = oracle.resize_nearest(img, 4, 3, 1)
    assert np.array_equal(near, img[1::2, 1::2])  # image's Nearest halves at (2x+1, 2y+1)
    up = oracle.resize_linear(img, 16, 12, 1)
    # Triangle 2x: interior weights 0.25 / 0.75, clamped borders, vertical pass first
    col = 0.75 * img[:, 1] + 0.25 * img[:, 2]
    assert abs(up[0, 3] - np.float32(col[0])) < 1e-6
    assert up[0, 0] == img[0, 0]
    assert np.all((up >= 0) & (up <= 1))


def test_ip_blur_clamp_border(oracle):
    img = np.zeros((20, 20), np.float32)
    img[:, 0] = 1.0
    out = oracle.gaussian_blur(img, 1.0, 1)
    # clamp-to-edge: the edge column sees its own value in the outside taps
    assert out[10, 0] > 0.5 and out[10, 19] == 0.0
