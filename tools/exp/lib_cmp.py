"""Bit-compare two library builds on the same synthetic frames (performance
experiments: a kernel change that should not move any output).

  python3 tools/exp/lib_cmp.py save NAME   # SIFT_MI_LIB picks the build
  python3 tools/exp/lib_cmp.py diff A B
"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "sift-features_amd")]

if sys.argv[1] == "save":
    import pkg_loader
    import synth
    sift = pkg_loader.load()

    fr = synth.frames(24, 1920, 1080, seed0=77)
    c = sift.Context(0, sift.OpenCVProcessing)
    res = c.sift_batch(fr)
    kp = np.concatenate([np.asarray(r.keypoints_array) for r in res])
    desc = np.concatenate([np.asarray(r.descriptors) for r in res])
    np.savez(os.path.join(ROOT, "gpurun_out", "cmp_%s.npz" % sys.argv[2]), kp=kp, desc=desc)
    print(sys.argv[2], "keypoints", len(desc))
else:
    a = np.load(os.path.join(ROOT, "gpurun_out", "cmp_%s.npz" % sys.argv[2]))
    b = np.load(os.path.join(ROOT, "gpurun_out", "cmp_%s.npz" % sys.argv[3]))
    same_kp = a["kp"].shape == b["kp"].shape and np.array_equal(a["kp"], b["kp"])
    same_d = a["desc"].shape == b["desc"].shape and np.array_equal(a["desc"], b["desc"])
    print("keypoints identical:", same_kp, "descriptors identical:", same_d)
    if not same_d and a["desc"].shape == b["desc"].shape:
        d = np.abs(a["desc"].astype(int) - b["desc"].astype(int))
        print("max |diff|", d.max(), "components differing", int((d > 0).sum()))
    sys.exit(0 if same_kp and same_d else 1)
