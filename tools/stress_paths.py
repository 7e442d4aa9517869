#!/usr/bin/env python3
"""Repeats the one-frame path comparisons (default, early off, large_first)
in one process, fresh contexts each round, and prints any mismatch: a check
for rare ordering races.  python tools/stress_paths.py [--rounds 8]"""
import argparse
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "sift-features_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=8)
    a = ap.parse_args()
    import pkg_loader
    import synth
    pkg = pkg_loader.load()
    frames = [synth.frame(640, 480, 3), synth.frame(1000, 333, 5), synth.frame(1920, 1080, 7)]
    bad = 0
    for r in range(a.rounds):
        for prof in (pkg.OpenCVProcessing, pkg.ImageprocProcessing):
            res = {}
            for knob, val in (("early", 1), ("early", 0), ("large_first", 0)):
                c = pkg.Context(0, prof)
                c.set_path_option(knob, val)
                res[(knob, val)] = [c.sift(f) for f in frames for _ in range(2)]
                c.close()
            ref = res[("early", 1)]
            for k, v in res.items():
                for i, (x, y) in enumerate(zip(v, ref)):
                    if not (x == y and np.array_equal(x.keys, y.keys)):
                        bad += 1
                        print(f"round {r} profile {prof} {k} call {i}: n {len(x)} vs {len(y)}", flush=True)
        print(f"round {r} done, mismatches so far {bad}", flush=True)
    print("STRESS", "FAIL" if bad else "OK", bad)
    sys.exit(1 if bad else 0)


if __name__ == "__main__":
    main()
