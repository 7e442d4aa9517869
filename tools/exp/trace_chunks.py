"""Per-chunk pyramid timeline from a rocprofv3 kernel trace of bench.py: the
serialised (one-lane) chunks, their pyramid span (seed start -> last pyramid
kernel end, both streams) and each launch's average duration / start offset.
    python3 tools/exp/trace_chunks.py <kernel_trace.csv[.gz]>"""
import csv, gzip, io, re, sys
from collections import defaultdict

path = sys.argv[1]
raw = gzip.open(path, "rt") if path.endswith(".gz") else open(path)
rows = list(csv.DictReader(io.StringIO(raw.read())))
short = lambda n: re.sub(r"\(.*", "", n).replace("void ", "").replace("siftmi::", "")
PYR = ("k_seed", "k_blur", "k_octave_tail")
ks = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r.get("Stream_Id", r.get("Queue_Id")), short(r["Kernel_Name"]))
            for r in rows)
seeds = [i for i, k in enumerate(ks) if k[3].startswith("k_seed")]
chunks = []
for a, b in zip(seeds, seeds[1:] + [len(ks)]):
    seg = ks[a:b]
    pyr = [k for k in seg if k[3].startswith(PYR)]
    chunks.append((ks[a][0], max(k[1] for k in pyr), pyr, seg))
ser = []
for i, (t0, t1, pyr, seg) in enumerate(chunks):
    nxt = chunks[i + 1][0] if i + 1 < len(chunks) else 1 << 62
    prev_end = chunks[i - 1][1] if i else 0
    ser.append(prev_end <= t0 and nxt >= max(k[1] for k in seg))
# longest run of serialised chunks with the most common launch count
best, c0 = (0, 0), None
for i, s in enumerate(ser + [False]):
    if s and c0 is None:
        c0 = i
    if not s and c0 is not None:
        if i - c0 > best[1] - best[0]:
            best = (c0, i)
        c0 = None
run = chunks[best[0]:best[1]]
print(f"{len(chunks)} chunks, serialised run of {len(run)}")
spans = [(t1 - t0) / 1e3 for t0, t1, pyr, seg in run]
print(f"pyramid span per chunk: mean {sum(spans) / len(spans):.1f} us (min {min(spans):.1f}, max {max(spans):.1f}); "
      f"launches {len(run[0][2])}")
pos = defaultdict(list)
for t0, t1, pyr, seg in run:
    for j, k in enumerate(pyr):
        pos[(j, k[3], k[2])].append(((k[0] - t0) / 1e3, (k[1] - k[0]) / 1e3))
for (j, name, st), v in sorted(pos.items()):
    print(f"{j:3d} stream {st:>4} {name[:44]:44s} start {sum(x[0] for x in v) / len(v):8.1f} us  dur {sum(x[1] for x in v) / len(v):7.1f} us")
# non-pyramid kernels of the same chunks
other = defaultdict(float)
for t0, t1, pyr, seg in run:
    for k in seg:
        if not k[3].startswith(PYR):
            other[k[3][:50]] += (k[1] - k[0]) / 1e3
for k, v in sorted(other.items(), key=lambda kv: -kv[1]):
    print(f"    {k:50s} {v / len(run):8.1f} us per chunk")
