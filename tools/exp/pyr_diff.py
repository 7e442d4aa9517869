# Debug helper (GPU box): where the GPU pyramid differs from the oracle.
import os, sys
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "tests"))
from conftest import load_golden  # noqa: E402  (also sets sys.path)
import pkg_loader  # noqa: E402
import oracle as O  # noqa: E402
pkg = pkg_loader.load()
ctx = pkg.Context(0, pkg.OpenCVProcessing)
img = load_golden("bird_small")["image"]
pre = ctx.precompute_images(img)
opy = O.Pyramid(img)
for o in range(min(3, opy.n_octaves)):
    g, go = pre.scale_space_octave(o), opy.scale_space(o)
    d, do = pre.dog_octave(o), opy.dog(o)
    for nm, a, b in (("G", g, go), ("D", d, do)):
        for s in range(a.shape[0]):
            bad = np.argwhere(a[s] != b[s])
            if len(bad):
                ys, xs = bad[:, 0], bad[:, 1]
                print(f"oct {o} {nm}{s}: {len(bad)} bad of {a[s].size}; rows {ys.min()}..{ys.max()} "
                      f"cols {xs.min()}..{xs.max()}; uniq rows {np.unique(ys)[:20]} uniq cols {np.unique(xs)[:12]}")
                y, x = bad[0]
                print("   sample", y, x, a[s][y, x], b[s][y, x])
