"""ImageprocProcessing profile (src/lib.rs:993-1007) on the GPU vs the CPU oracle.

The profile's arithmetic lives in imageproc 0.25.0 (gaussian_blur_f32) and
image 0.25.2 (imageops::resize Triangle / Nearest), which are not in
/root/reference and which no reference test runs: the oracle restates their
published algorithms and this profile's parity is UNPINNED against the
reference.  GPU vs oracle is held to the same bar as the OpenCV
profile: bit-exact ops and pyramid, identical keypoints, descriptors +-1.
"""
import numpy as np
import pytest
from test_gpu_parity import INPUTS, assert_parity

pytestmark = pytest.mark.gpu

PROFILE_IMAGEPROC = 1


@pytest.fixture(scope="module")
def ctx_ip(pkg):
    c = pkg.Context(0, pkg.ImageprocProcessing)
    yield c
    c.close()


@pytest.mark.parametrize("sigma", [0.6, 1.2489996, 1.2262735, 1.5450078, 1.9465878, 2.4525469, 3.0900155, 6.0])
@pytest.mark.parametrize("shape", [(61, 97), (480, 640), (7, 5)])
def test_ip_gaussian_blur_bit_exact(ctx_ip, oracle, sigma, shape):
    img = np.random.default_rng(4).random(shape, dtype=np.float32)
    assert np.array_equal(ctx_ip.gaussian_blur(img, sigma), oracle.gaussian_blur(img, sigma, PROFILE_IMAGEPROC))


@pytest.mark.parametrize("src,dst", [((13, 17), (26, 34)), ((213, 320), (426, 640)), ((10, 10), (37, 23)),
                                     ((50, 40), (20, 16)), ((9, 7), (4, 3)), ((64, 64), (64, 64))])
def test_ip_resize_bit_exact(ctx_ip, oracle, src, dst):
    img = np.random.default_rng(5).random(src, dtype=np.float32)
    h2, w2 = dst
    assert np.array_equal(ctx_ip.resize_linear(img, w2, h2), oracle.resize_linear(img, w2, h2, PROFILE_IMAGEPROC))
    assert np.array_equal(ctx_ip.resize_nearest(img, w2, h2), oracle.resize_nearest(img, w2, h2, PROFILE_IMAGEPROC))


@pytest.mark.parametrize("name", ["bird_small", "synth_301x207", "synth_97x61"])
def test_ip_pyramid_bit_exact(ctx_ip, oracle, name):
    img = INPUTS[name]
    pre = ctx_ip.precompute_images(img)
    opy = oracle.Pyramid(img, PROFILE_IMAGEPROC)
    assert pre.n_octaves == opy.n_octaves
    for o in range(opy.n_octaves):
        assert pre.dims(o) == opy.dims(o)
        g, go = pre.scale_space_octave(o), opy.scale_space(o)
        assert np.array_equal(g, go), (o, np.abs(g - go).max())
        d, do = pre.dog_octave(o), opy.dog(o)
        assert np.array_equal(d, do), (o, np.abs(d - do).max())


@pytest.mark.parametrize("name", list(INPUTS))
def test_ip_sift_parity(pkg, ctx_ip, oracle, name):
    img = INPUTS[name]
    kp_o, desc_o, ext_o = oracle.sift(img, profile=PROFILE_IMAGEPROC, internal=True)
    res = ctx_ip.sift(img)
    assert_parity(pkg, res, kp_o, desc_o, ext_o)


def test_ip_batch_and_limit(pkg, ctx_ip, oracle):
    import synth
    frames = synth.frames(3, 160, 120, seed0=40)
    out = ctx_ip.sift_batch(frames, features_limit=30)
    for f, res in zip(frames, out):
        kp_o, desc_o, ext_o = oracle.sift(f, features_limit=30, profile=PROFILE_IMAGEPROC, internal=True)
        assert_parity(pkg, res, kp_o, desc_o, ext_o)


@pytest.mark.parametrize("kernel", ["strip", "tile", "notail", "nopair", "noseedpair"])
@pytest.mark.parametrize("name", ["synth_640x480", "synth_301x207", "synth_1000x333", "synth_90x700",
                                  "synth_2000x40", "synth_97x61"])
def test_ip_pyramid_kernels(ctx_ip, oracle, kernel, name):
    """The imageproc profile's kernel families bit for bit against the oracle:
    "strip" (k_seed_pair<3, 3, imageproc>: the Triangle 2x upsample, vertical
    then horizontal, clamped, in the strip loader, then the seed blur and
    blur 1; the k_blur2_strip<4, 4> pair for G_2, G_3 and the next octave's
    base (image's Nearest: odd rows / columns) of octave 0 and the <3, 4>
    pair for G_1, G_2 of the others, whose border chunks read clamped rows;
    clamp-to-edge strip blurs and the tail kernel), "tile" (k_seed_ip and the
    tile blurs), "notail" (per-blur launches for the small octaves), "nopair"
    (single-blur strips for G_1, G_2), "noseedpair" (k_seed_strip, then
    octave 0 like the others)."""
    from test_gpu_parity import _KERNEL_OPTS, _extra
    img = INPUTS[name] if name in INPUTS else _extra(name)
    with ctx_ip.path_options(**_KERNEL_OPTS[kernel]):
        pre = ctx_ip.precompute_images(img)
        opy = oracle.Pyramid(img, PROFILE_IMAGEPROC)
        assert pre.n_octaves == opy.n_octaves
        for o in range(opy.n_octaves):
            g, go = pre.scale_space_octave(o), opy.scale_space(o)
            assert np.array_equal(g, go), (o, np.argwhere(g != go)[:5])


@pytest.mark.parametrize("kernel", ["strip", "tile", "notail", "nopair", "noseedpair"])
@pytest.mark.parametrize("shape", [(640, 480), (301, 207)])
def test_ip_saturated_next_octave_clamp(ctx_ip, oracle, kernel, shape):
    """Large saturated (255) regions: a blur of 1.0s can round a hair past 1,
    and image's resize clamps its f32 output to [0, 1] -- the next octave's
    base (Nearest 1/2 of G_3) is clamped in every kernel family (strip pair,
    strip blur, tile blur, tail)."""
    import synth
    from test_gpu_parity import _KERNEL_OPTS
    f = synth.frame(shape[0], shape[1], 9).astype(np.float32)
    img = np.clip(f * 2.0 - 60.0, 0, 255).astype(np.uint8)
    assert (img == 255).mean() > 0.1
    with ctx_ip.path_options(**_KERNEL_OPTS[kernel]):
        pre = ctx_ip.precompute_images(img)
        opy = oracle.Pyramid(img, PROFILE_IMAGEPROC)
        for o in range(opy.n_octaves):
            g, go = pre.scale_space_octave(o), opy.scale_space(o)
            assert np.array_equal(g, go), (o, np.argwhere(g != go)[:5])
