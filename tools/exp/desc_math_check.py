"""Experiment: descriptor agreement with the oracle for the default build vs a
build with f32 per-sample transcendentals (tools/exp/libsift_mi_f32.so)."""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "oracle"), os.path.join(ROOT, "tests"), os.path.join(ROOT, "sift-features_amd")]
import numpy as np
variant = sys.argv[1]
import pkg_loader
pkg = pkg_loader.load()
from sift_features_amd import _lib
if variant == "f32":
    _lib.LIB_PATH = os.path.join(ROOT, "tools", "exp", "libsift_mi_f32.so")
import oracle, synth
from conftest import load_golden
ctx = pkg.Context(0)
tot_eq = tot = 0
worst = 0
for name, img in [("bird_small", load_golden("bird_small")["image"]), ("tree_small", load_golden("tree_small")["image"]),
                  ("bird", load_golden("bird")["image"]), ("synth", synth.frame(640, 480, 7))]:
    r = ctx.sift(img)
    kp, desc = oracle.sift(img)
    dd = np.abs(r.descriptors.astype(int) - desc.astype(int))
    print(variant, name, len(kp), "identical bytes %.5f" % (dd == 0).mean(), "max", dd.max(), "identical rows %.4f" % np.all(dd == 0, 1).mean())
