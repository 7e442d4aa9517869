#!/usr/bin/env python3
"""Which kernel path makes a batch-path pyramid plane differ from the
oracle: one frame through sift() (the batch arena, read back with
sift_mi_read_batch_scale_space) and through precompute_images, under
environment knobs, plane by plane.
    python3 tools/debug_pyr.py [--profile 1] [--size 640x480] [--seed 7]
"""
import argparse
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "sift-features_amd"))
sys.path.insert(0, os.path.join(ROOT, "oracle"))

KNOBS = [
    {},
    {"SIFT_MI_FUSED_DETECT": "0"},
    {"SIFT_MI_OCT_OVERLAP": "0"},
    {"SIFT_MI_SEED_PAIR": "0"},
    {"SIFT_MI_PAIR": "0"},
    {"SIFT_MI_TAIL": "0"},
    {"SIFT_MI_STAGE_OVERLAP": "0"},
]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--profile", type=int, default=1)
    ap.add_argument("--size", default="640x480")
    ap.add_argument("--seed", type=int, default=7)
    a = ap.parse_args()
    import oracle
    import pkg_loader
    import synth
    pkg = pkg_loader.load()
    w, h = map(int, a.size.split("x"))
    img = synth.frame(w, h, a.seed)
    opy = oracle.Pyramid(img, a.profile)
    prof = pkg.OpenCVProcessing if a.profile == 0 else pkg.ImageprocProcessing

    def report(tag, get):
        bad = []
        for o in range(opy.n_octaves):
            go = opy.scale_space(o)
            g = get(o, go)
            for s in range(6):
                d = np.argwhere(g[s] != go[s])
                if len(d):
                    bad.append(f"o{o}s{s}:{len(d)}@{d[0].tolist()}")
        print(f"{tag:40s} {'OK' if not bad else ' '.join(bad[:6])}", flush=True)

    for knob in KNOBS:
        for k, v in knob.items():
            os.environ[k] = v
        c = pkg.Context(0, prof)
        c.sift(img)
        report("sift " + str(knob), lambda o, go: c.read_batch_scale_space(0, o, (go.shape[2], go.shape[1])))
        pre = c.precompute_images(img)
        report("precompute " + str(knob), lambda o, go: pre.scale_space_octave(o))
        c.close()
        for k in knob:
            del os.environ[k]


if __name__ == "__main__":
    main()
