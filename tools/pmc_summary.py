"""Average rocprofv3 --pmc counters per (kernel, grid) from counter_collection CSVs."""
import collections
import csv
import re
import sys

pat = sys.argv[1] if len(sys.argv) > 1 else ""
agg = collections.defaultdict(lambda: collections.defaultdict(list))
order = []
for f in sys.argv[2:]:
    for r in csv.DictReader(open(f)):
        if pat not in r["Kernel_Name"]:
            continue
        k = (re.sub(r"void |\(.*", "", r["Kernel_Name"]), r["Grid_Size"], "vgpr" + r["VGPR_Count"], "lds" + r["LDS_Block_Size"])
        if k not in agg:
            order.append(k)
        agg[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k in order:
    v = agg[k]
    print(" ".join(k))
    print("   ", " ".join(f"{c}={sum(x) / len(x):.4g}" for c, x in sorted(v.items())))
