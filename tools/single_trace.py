#!/usr/bin/env python3
"""Timeline of single-frame calls from a rocprofv3 kernel trace
(tools/r04_measure.sh single): the kernels of the last calls, each with its
stream, start / end relative to the call's first kernel, and the idle gaps
on the critical path.
    python3 tools/single_trace.py <trace dir> [calls]
"""
import csv
import glob
import gzip
import io
import os
import re
import sys
from collections import defaultdict


def short(n):
    return re.sub(r"\(.*", "", n).replace("void ", "").replace("siftmi::", "")[:48]


def main():
    d = sys.argv[1]
    ncalls = int(sys.argv[2]) if len(sys.argv) > 2 else 3
    f = (glob.glob(os.path.join(d, "**/*kernel_trace.csv"), recursive=True) +
         glob.glob(os.path.join(d, "**/*kernel_trace.csv.gz"), recursive=True))[0]
    raw = gzip.open(f, "rt") if f.endswith(".gz") else open(f)
    rows = list(csv.DictReader(io.StringIO(raw.read())))
    ks = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Stream_Id"], short(r["Kernel_Name"]))
                for r in rows)
    # calls start at k_chunk_init
    starts = [i for i, k in enumerate(ks) if k[3].startswith("k_chunk_init")]
    calls = [ks[a:b] for a, b in zip(starts, starts[1:] + [len(ks)])]
    per = defaultdict(list)
    for c in calls[-ncalls:]:
        t0 = c[0][0]
        end = max(k[1] for k in c)
        print(f"--- call: {len(c)} kernels, first start -> last end {(end - t0) / 1e3:.1f} us")
        busy_end = t0
        for s, e, st, name in c:
            gap = (s - busy_end) / 1e3
            print(f"  {name:48s} st{st:>3s} {(s - t0) / 1e3:8.1f} {(e - t0) / 1e3:8.1f}  dur {(e - s) / 1e3:7.1f}"
                  f"  {'gap %.1f' % gap if gap > 0.5 else ''}")
            busy_end = max(busy_end, e)
            per[name].append((e - s) / 1e3)
    print("--- mean duration per kernel over the shown calls (us)")
    for k, v in sorted(per.items(), key=lambda kv: -sum(kv[1])):
        print(f"  {k:48s} n={len(v):3d} mean {sum(v) / len(v):7.1f}")
    spans = []
    for c in calls[1:]:
        spans.append((max(k[1] for k in c) - c[0][0]) / 1e3)
    if spans:
        spans.sort()
        print(f"--- GPU span per call over {len(spans)} calls: median {spans[len(spans) // 2]:.1f} us")
    gaps = [(calls[i + 1][0][0] - max(k[1] for k in calls[i])) / 1e3 for i in range(len(calls) - 1)]
    if gaps:
        gaps.sort()
        print(f"--- idle between calls: median {gaps[len(gaps) // 2]:.1f} us")


if __name__ == "__main__":
    main()
