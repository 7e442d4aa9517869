"""GPU (HIP, gfx950) vs CPU oracle parity through the C ABI.

Parity contract:
  * pyramid (scale space + DoG): bit-identical f32 (np.array_equal);
  * keypoints: identical count and emission order -- every (octave, initial
    scale, initial y, initial x, orientation peak) key equal -- and
    |dx|,|dy|,|dsize| <= 1e-4 px, |dangle| <= 1e-2 deg, |dresponse| <= 1e-6
    (in practice bit-identical: same op order, -ffp-contract=off; the only
    possible deviations are 1-ulp differences of f64-evaluated exp/pow vs glibc);
  * descriptors: max |d| <= 1 per u8 component and >= 99 % of bytes identical
    (the default GPU mode sums the 6x6x8 histogram in lane-private LDS
    slices and uses hardware sqrt/exp and a polynomial atan2, so bin sums can
    differ from the sequential CPU order in the last f32 bits); the exact
    descriptor mode is byte-identical.
"""
import numpy as np
import pytest
from conftest import load_golden

pytestmark = pytest.mark.gpu

TOL_XY = 1e-4
TOL_ANGLE = 1e-2
TOL_RESP = 1e-6


def _inputs():
    import synth
    cases = {
        "bird_small": load_golden("bird_small")["image"],
        "tree_small": load_golden("tree_small")["image"],
        "bird": load_golden("bird")["image"],
        "synth_640x480": synth.frame(640, 480, 3),
        "synth_301x207": synth.frame(301, 207, 11),
        "synth_97x61": synth.frame(97, 61, 5),
    }
    return cases


INPUTS = _inputs()


def assert_parity(pkg, res, kp_o, desc_o, ext_o):
    assert len(res) == len(kp_o), (len(res), len(kp_o))
    if len(kp_o) == 0:
        return
    f = pkg.key_fields(res.keys)
    for col, name in [(0, "octave"), (2, "s_init"), (3, "y_init"), (4, "x_init"), (5, "peak")]:
        assert np.array_equal(f[name], ext_o[:, col]), name
    kp = res.keypoints_array
    d = np.abs(kp - kp_o)
    assert d[:, 0].max() <= TOL_XY and d[:, 1].max() <= TOL_XY and d[:, 2].max() <= TOL_XY, d.max(0)
    dang = np.abs(((kp[:, 3] - kp_o[:, 3]) + 180.0) % 360.0 - 180.0)
    assert dang.max() <= TOL_ANGLE, dang.max()
    assert d[:, 4].max() <= TOL_RESP, d[:, 4].max()
    dd = np.abs(res.descriptors.astype(np.int32) - desc_o.astype(np.int32))
    assert dd.max() <= 1, dd.max()
    assert (dd == 0).mean() >= 0.99, (dd == 0).mean()


@pytest.mark.parametrize("name", list(INPUTS))
def test_sift_parity(pkg, ctx, oracle, name):
    img = INPUTS[name]
    kp_o, desc_o, ext_o = oracle.sift(img, internal=True)
    res = ctx.sift(img)
    assert_parity(pkg, res, kp_o, desc_o, ext_o)


@pytest.mark.parametrize("name", ["bird_small", "synth_301x207", "synth_97x61"])
def test_pyramid_bit_exact(ctx, oracle, name):
    img = INPUTS[name]
    pre = ctx.precompute_images(img)
    opy = oracle.Pyramid(img)
    assert pre.n_octaves == opy.n_octaves
    for o in range(opy.n_octaves):
        assert pre.dims(o) == opy.dims(o)
        g, go = pre.scale_space_octave(o), opy.scale_space(o)
        assert np.array_equal(g, go), (o, np.abs(g - go).max())
        d, do = pre.dog_octave(o), opy.dog(o)
        assert np.array_equal(d, do), (o, np.abs(d - do).max())


_KERNEL_OPTS = {
    "strip": {},
    "tile": {"tile_blur": 1},
    "nopair": {"pair_blur": 0},
    "notail": {"tail": 0},
    "single": {"pair_blur": 0, "tail": 0},
    "noseedpair": {"seed_pair": 0},
}


@pytest.mark.parametrize("kernel", sorted(_KERNEL_OPTS))
@pytest.mark.parametrize("name", ["synth_640x480", "synth_301x207", "synth_97x61", "synth_1000x333",
                                  "synth_90x700", "synth_2000x40", "synth_33x17"])
def test_pyramid_blur_kernels(ctx, oracle, kernel, name):
    """Every blur kernel family against the oracle's blur chain, bit for bit:
    "strip" (the default: k_seed_pair for G_0, G_1 of octave 0 and the
    k_blur2_strip (6, 8) pair for its G_2, G_3 and the next octave's base,
    the (5, 6) pair for G_1, G_2 of the later octaves, k_blur_strip for the
    rest -- 128-column strips streamed down in row
    chunks, many row segments per octave at these sizes, partial strips,
    reflect-101 at every border -- and k_octave_tail from the first octave that
    fits LDS; the tile kernels where a strip does not apply: tiny octaves, W
    or H <= R), "tile" (path option tile_blur: one 64-column tile per
    workgroup everywhere), "nopair" / "notail" / "single" (pair_blur = 0,
    tail = 0: single-blur strips instead of the pair kernel, per-blur
    launches for the small octaves), "noseedpair" (seed_pair = 0:
    k_seed_strip, then octave 0 like the others)."""
    img = INPUTS[name] if name in INPUTS else _extra(name)
    with ctx.path_options(**_KERNEL_OPTS[kernel]):
        pre = ctx.precompute_images(img)
        opy = oracle.Pyramid(img)
        assert pre.n_octaves == opy.n_octaves
        for o in range(opy.n_octaves):
            g, go = pre.scale_space_octave(o), opy.scale_space(o)
            assert np.array_equal(g, go), (o, np.argwhere(g != go)[:5])
            d, do = pre.dog_octave(o), opy.dog(o)
            assert np.array_equal(d, do), (o, np.argwhere(d != do)[:5])


def _extra(name):
    import synth
    w, h = map(int, name.split("_")[1].split("x"))
    return synth.frame(w, h, 7)


@pytest.mark.parametrize("limit", [0, 1, 50, 100000])
def test_features_limit(pkg, ctx, oracle, limit):
    img = INPUTS["tree_small"]
    kp_o, desc_o, ext_o = oracle.sift(img, features_limit=limit, internal=True)
    res = ctx.sift(img, features_limit=limit)
    assert_parity(pkg, res, kp_o, desc_o, ext_o)
    if 0 < limit < 1000:
        assert np.all(np.diff(res.keypoints_array[:, 4]) <= 0)  # response descending


def test_precomputed_split(pkg, ctx, oracle):
    img = INPUTS["bird_small"]
    pre = ctx.precompute_images(img)
    res = ctx.sift_with_precomputed(pre)
    kp_o, desc_o, ext_o = oracle.sift(img, internal=True)
    assert_parity(pkg, res, kp_o, desc_o, ext_o)
    assert res == ctx.sift(img)


def test_module_level_api(pkg, oracle):
    """sift() is sift_with_processing::<ImageprocProcessing> (src/lib.rs:71-73)."""
    img = INPUTS["bird_small"]
    res = pkg.sift(img)
    assert res == pkg.sift_with_processing(pkg.ImageprocProcessing, img)
    kp_o, desc_o, ext_o = oracle.sift(img, profile=1, internal=True)
    assert_parity(pkg, res, kp_o, desc_o, ext_o)
    res_cv = pkg.sift_with_processing(pkg.OpenCVProcessing, img)
    kp_o, desc_o, ext_o = oracle.sift(img, internal=True)
    assert_parity(pkg, res_cv, kp_o, desc_o, ext_o)
    assert len(res.keypoints) == len(res)


def test_golden_snapshots_gpu(pkg, ctx, oracle):
    """GPU output vs the reference's snapshots: the oracle's agreement
    (tests/test_oracle_golden.py: exact counts, >= 99 % of rows within 1e-3 px,
    descriptor components within +-1).  The exact descriptor mode reproduces
    the oracle's identical-row fraction; the default mode adds its own +-1."""
    from test_oracle_golden import MIN_DESC_EQUAL, MIN_POS_EXACT, MIN_ROWS_CLOSE, golden_agreement
    ex = pkg.Context(0)
    ex.set_exact_descriptors(True)
    for name, count in [("tree_small", 1270), ("bird_small", 225)]:
        g = load_golden(name)
        # default mode: measured on MI355X (round 3) at the exact mode's max |d|
        # of 1 and 98.35 % / 97.33 % identical rows (tree / bird; exact mode
        # 98.35 / 97.78 %): its own +-1 does not stack on the oracle's here.
        # Bound 0.97 (bird: 219 / 225 rows measured = 0.9733; the round-4
        # pre-emptive 0.96 is withdrawn): a change of the fast path's
        # summation order that costs rows shows up.
        for c, min_desc, max_d in ((ctx, 0.97, 1), (ex, MIN_DESC_EQUAL, 1)):
            res = c.sift(g["image"])
            assert len(res) == count
            order = pkg.stable_sort_xy_size(res.keypoints_array)
            pos_exact, rows_close, desc_equal, desc_maxd = golden_agreement(res.keypoints_array[order],
                                                                             res.descriptors[order], g)
            print(f"golden {name} {'exact' if c is ex else 'default'}: pos_exact {pos_exact:.4f} "
                  f"rows_close {rows_close:.4f} desc_equal {desc_equal:.4f} desc_maxd {desc_maxd}")
            assert pos_exact >= MIN_POS_EXACT and rows_close >= MIN_ROWS_CLOSE, (name, pos_exact, rows_close)
            assert desc_equal >= min_desc, (name, desc_equal)
            assert desc_maxd <= max_d, (name, desc_maxd)
    ex.close()


@pytest.mark.parametrize("name", ["bird_small", "tree_small", "synth_640x480", "synth_97x61"])
def test_exact_descriptors_bit_identical(pkg, oracle, name):
    """sift_mi_set_exact_descriptors(1): bins accumulated in the reference's
    sequential sample order -> descriptors byte-identical to the CPU path."""
    img = INPUTS[name]
    kp_o, desc_o, ext_o = oracle.sift(img, internal=True)
    c = pkg.Context(0)
    c.set_exact_descriptors(True)
    res = c.sift(img)
    c.close()
    assert_parity(pkg, res, kp_o, desc_o, ext_o)
    assert np.array_equal(res.descriptors, desc_o), (res.descriptors != desc_o).sum()
    # keypoint fields: bit-identical except where an f64-evaluated pow / exp
    # rounds differently from glibc's f32 routine (1 ulp, rare)
    neq = res.keypoints_array != kp_o
    assert neq.sum() <= max(2, len(kp_o) // 200), (neq.sum(0), np.argwhere(neq)[:5])


@pytest.mark.parametrize("shape", [(24, 32), (64, 96)])
@pytest.mark.parametrize("profile", [0, 1])
def test_seed_all_byte_values(pkg, oracle, profile, shape):
    """Every u8 value goes through the seed's v / 255 (fma-corrected
    reciprocal, no table) and the 2x upsample: the first Gaussian of octave 0
    is bit-identical to the oracle's (which divides).  32x24: the tile seed
    kernels; 96x64: the strip seed (2x width >= 160)."""
    img = np.arange(shape[0] * shape[1], dtype=np.uint32).reshape(shape)
    img = ((img * 97 + 13) % 256).astype(np.uint8)  # all 256 values, scrambled
    c = pkg.Context(0, pkg.OpenCVProcessing if profile == 0 else pkg.ImageprocProcessing)
    pre = c.precompute_images(img)
    opy = oracle.Pyramid(img, profile)
    assert np.array_equal(pre.scale_space_octave(0), opy.scale_space(0))
    c.close()
