"""Processing-trait ops (src/lib.rs:86-90) and compute_descriptor (src/lib.rs:785)
on the GPU vs the CPU oracle.  Blur / resize are bit-exact; compute_descriptor
within +-1 per component (LDS-atomic histogram order)."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("sigma", [0.6, 1.2489996, 1.2262735, 1.5450078, 1.9465878, 2.4525469, 3.0900155, 5.0])
@pytest.mark.parametrize("shape", [(61, 97), (480, 640), (7, 5)])
def test_gaussian_blur_bit_exact(ctx, oracle, sigma, shape):
    rng = np.random.default_rng(1)
    img = rng.random(shape, dtype=np.float32)
    assert np.array_equal(ctx.gaussian_blur(img, sigma), oracle.gaussian_blur(img, sigma))


@pytest.mark.parametrize("src,dst", [((13, 17), (26, 34)), ((213, 320), (426, 640)), ((10, 10), (37, 23)),
                                     ((50, 40), (20, 16))])
def test_resize_bit_exact(ctx, oracle, src, dst):
    rng = np.random.default_rng(2)
    img = rng.random(src, dtype=np.float32)
    h2, w2 = dst
    assert np.array_equal(ctx.resize_linear(img, w2, h2), oracle.resize_linear(img, w2, h2))
    assert np.array_equal(ctx.resize_nearest(img, w2, h2), oracle.resize_nearest(img, w2, h2))


def test_compute_descriptor(ctx, oracle):
    """benches/descriptor.rs: (100, 100), scale 2.1, 123 deg on bird.jpg / 255."""
    from conftest import load_golden
    img = load_golden("bird")["image"].astype(np.float32) / 255.0
    rng = np.random.default_rng(3)
    cases = [(100.0, 100.0, 2.1, 123.0)] + [
        (float(rng.uniform(0, 799)), float(rng.uniform(0, 533)), float(rng.uniform(1.8, 3.6)),
         float(rng.uniform(0, 360))) for _ in range(40)]
    same = 0
    for x, y, s, a in cases:
        g = ctx.compute_descriptor(img, x, y, s, a)
        o = oracle.compute_descriptor(img, x, y, s, a)
        d = np.abs(g.astype(int) - o.astype(int))
        assert d.max() <= 1, (x, y, s, a, d.max())
        same += (d == 0).sum()
    assert same == 128 * len(cases)  # sift_mi_compute_descriptor uses the exact accumulation order
