"""Per-launch-shape summary of a rocprofv3 kernel_trace.csv (sift kernels only by default)."""
import collections
import csv
import re
import sys

path = sys.argv[1]
pat = sys.argv[2] if len(sys.argv) > 2 else "siftmi::"
agg = collections.defaultdict(lambda: [0, 0.0])
for r in csv.DictReader(open(path)):
    if pat not in r["Kernel_Name"]:
        continue
    n = re.sub(r"\(.*", "", r["Kernel_Name"]).replace("void ", "").replace("siftmi::", "")
    key = (n, r["Grid_Size_X"], r["Grid_Size_Y"], r["Grid_Size_Z"])
    agg[key][0] += 1
    agg[key][1] += (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
tot = sum(v[1] for v in agg.values())
for k, v in sorted(agg.items(), key=lambda kv: -kv[1][1]):
    print(f"{v[1]:10.1f} us {100 * v[1] / tot:5.1f}%  n={v[0]:4d} avg={v[1] / v[0]:9.1f} us  {k[0]:28s} grid={k[1]}x{k[2]}x{k[3]}")
print(f"total {tot:.1f} us")
