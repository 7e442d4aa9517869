"""Per-call pyramid timeline from a rocprofv3 kernel trace of a probe that
synchronises after every call (tools/exp/single.py): calls are separated by
idle gaps; for each kernel position the average start offset (from the call's
first seed) and duration, per stream; the pyramid span = first seed start ->
last pyramid kernel end.
    python3 tools/exp/trace_calls.py <kernel_trace.csv[.gz]> [gap_us]"""
import csv, gzip, io, re, sys
from collections import defaultdict, Counter

path = sys.argv[1]
gap = float(sys.argv[2]) * 1e3 if len(sys.argv) > 2 else 30e3
raw = gzip.open(path, "rt") if path.endswith(".gz") else open(path)
rows = list(csv.DictReader(io.StringIO(raw.read())))
short = lambda n: re.sub(r"\(.*", "", n).replace("void ", "").replace("siftmi::", "")
import os
PYR = ("k_seed", "k_blur", "k_octave_tail") if not os.environ.get("ALL") else ("",)  # ALL=1: every kernel of the call
ks = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r.get("Stream_Id", r.get("Queue_Id")), short(r["Kernel_Name"]))
            for r in rows)
calls, cur, end = [], [], 0
for k in ks:
    if cur and k[0] - end > gap:
        calls.append(cur)
        cur = []
    cur.append(k)
    end = max(end, k[1])
calls.append(cur)
calls = [c for c in calls if any(k[3].startswith("k_seed") for k in c)]
sig = Counter(tuple(k[3] for k in c if k[3].startswith(PYR)) for c in calls)
common = sig.most_common(1)[0][0]
run = [c for c in calls if tuple(k[3] for k in c if k[3].startswith(PYR)) == common][2:]
print(f"{len(calls)} calls, {len(run)} with the common pyramid launch sequence ({len(common)} launches)")
spans, pos, other = [], defaultdict(list), defaultdict(float)
for c in run:
    pyr = [k for k in c if k[3].startswith(PYR)]
    t0 = min(k[0] for k in pyr)
    spans.append((max(k[1] for k in pyr) - t0) / 1e3)
    for j, k in enumerate(pyr):
        pos[(j, k[3], k[2])].append(((k[0] - t0) / 1e3, (k[1] - k[0]) / 1e3))
    for k in c:
        if not k[3].startswith(PYR):
            other[k[3][:50]] += (k[1] - k[0]) / 1e3
print(f"pyramid span per call: mean {sum(spans) / len(spans):.1f} us (min {min(spans):.1f}, max {max(spans):.1f})")
for (j, name, st), v in sorted(pos.items()):
    if len(v) < len(run) // 2:
        continue
    a = sum(x[0] for x in v) / len(v)
    d = sum(x[1] for x in v) / len(v)
    print(f"{j:3d} stream {st:>4} {name[:44]:44s} start {a:8.1f}  end {a + d:8.1f}  dur {d:7.1f} us")
for k, v in sorted(other.items(), key=lambda kv: -kv[1]):
    print(f"    {k:50s} {v / len(run):8.1f} us per call")
