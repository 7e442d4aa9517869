"""Summarise a round profile (tools/round_profile.sh) into profiles/.

Writes
  profiles/<round>_kernel_stats.csv   rocprofv3 --stats output (copied)
  profiles/<round>_summary.md         per-kernel table, the pyramid stage from
                                      the trace next to bench.py's own number,
                                      and HBM traffic from the PMC passes
  profiles/pmc_traffic.json           per-frame pyramid traffic, read by
                                      bench.py for roofline.traffic
HBM bytes follow MI355X_MICROARCH.md (HBM section): FETCH_SIZE and WRITE_SIZE
are in KiB; on gfx950 FETCH_SIZE counts half the bytes of 16-B-per-lane
streaming reads (doubled here); WRITE_SIZE is exact for 16-B stores.
"""
import csv
import glob
import json
import os
import re
import shutil
import sys
from collections import defaultdict

ROUND, OUT, FRAMES = sys.argv[1], sys.argv[2], int(sys.argv[3])
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PROF = os.path.join(ROOT, "profiles")
os.makedirs(PROF, exist_ok=True)
PYR = ("k_seed", "k_blur")


def short(n):
    return re.sub(r"\(.*", "", n).replace("void ", "").replace("siftmi::", "")


def one(pattern):
    f = glob.glob(os.path.join(OUT, pattern), recursive=True)
    return f[0] if f else None


def bench_line(log):
    for line in open(log):
        if line.startswith("{"):
            return json.loads(line)
    return None


trace = one("trace/**/run_kernel_trace.csv")
stats = one("trace/**/run_kernel_stats.csv")
shutil.copy(stats, os.path.join(PROF, f"{ROUND}_kernel_stats.csv"))
b = bench_line(os.path.join(OUT, "bench_trace.log"))

agg = defaultdict(lambda: [0, 0.0])
rows = list(csv.DictReader(open(trace)))
for r in rows:
    k = short(r["Kernel_Name"])
    agg[k][0] += 1
    agg[k][1] += (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
tot = sum(v[1] for k, v in agg.items() if "siftmi" in k or k.startswith("k_"))
pyr_us = sum(v[1] for k, v in agg.items() if k.startswith(PYR))
pyr_n = sum(v[0] for k, v in agg.items() if k.startswith(PYR))
n_chunks = agg["k_seed<5, 32>"][0] if "k_seed<5, 32>" in agg else max(1, sum(v[0] for k, v in agg.items() if k.startswith("k_seed")))

# The serialised stage-timing pass of bench.py (the roofline's HIP-event
# average): the longest run of consecutive sift kernels on a single stream.
# Its chunks start at k_seed; the last `steps` x chunks-per-call of them are
# the timed steps (one warmup step precedes them).
sk = sorted(((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Stream_Id"], short(r["Kernel_Name"]))
             for r in rows if short(r["Kernel_Name"]).startswith("k_") or "rocprim" in r["Kernel_Name"]))
best, cur = (0, 0), [0, 0]
for i in range(1, len(sk) + 1):
    if i == len(sk) or sk[i][2] != sk[cur[0]][2]:
        if i - cur[0] > best[1] - best[0]:
            best = (cur[0], i)
        cur = [i, i]
run = sk[best[0]:best[1]]
seeds = [i for i, x in enumerate(run) if x[3].startswith("k_seed")]
steps = b["steps"] if b else 3
chunks_per_call = max(1, len(seeds) // (steps + 1))
# complete chunks of the serialised pass: a seed and every blur after it up to
# the next seed (a group cut short at the run's end is dropped); the last
# steps * chunks_per_call complete groups are the timed steps
groups = []
for a, z in zip(seeds, seeds[1:] + [len(run)]):
    g = [x for x in run[a:z] if x[3].startswith(PYR)]
    groups.append(g)
full = max((len(g) for g in groups), default=0)
groups = [g for g in groups if len(g) == full]
timed = [x for g in groups[-steps * chunks_per_call:] for x in g]
iso = [(e - s0) / 1e3 for s0, e, _, k in timed]
iso_us, iso_n = sum(iso), len(iso)


def pmc(kind, name):
    f = one(f"{kind}/**/run_counter_collection.csv")
    v, n = 0.0, 0
    for r in csv.DictReader(open(f)):
        if r["Counter_Name"] == name and short(r["Kernel_Name"]).startswith(PYR):
            v += float(r["Counter_Value"])
            n += 1
    return v * 1024.0, n  # KiB -> bytes


fetch, n_f = pmc("fetch", "FETCH_SIZE")
fetch *= 2.0  # gfx950: half of 16-B streaming reads counted
write, n_w = pmc("write", "WRITE_SIZE")
W, H = 1920, 1080
sum_p, ow, oh = 0, 2 * W, 2 * H
for _ in range(int(round(__import__("math").log2(min(2 * W, 2 * H)) - 2)) + 1):
    sum_p += ow * oh
    ow //= 2
    oh //= 2
algo_pf = W * H + 44 * sum_p  # G_0..G_5 + D_0..D_4 written once (the batch path writes G only)
# host auto_chunk (host.cpp): <= 64 frames and ~32 GB of pyramid per chunk,
# balanced, at least two chunks per call
cmax = min(64, max(1, int(32e9 // (44.0 * sum_p))))
nck = max(-(-FRAMES // cmax), 2 if FRAMES >= 2 else 1)
chunk = -(-FRAMES // nck)
launches_per_chunk = pyr_n / max(1, n_chunks)
traffic_pl = fetch / max(1, n_f) + write / max(1, n_w)  # HBM bytes per pyramid launch
traffic_pf = traffic_pl * launches_per_chunk / chunk
json.dump({"round": ROUND, "frame": f"{W}x{H}", "frames_per_call": FRAMES, "frames_per_chunk": chunk,
           "pyramid_hbm_bytes_per_launch": traffic_pl, "pyramid_hbm_bytes_per_frame": traffic_pf,
           "fetch_bytes_per_launch": fetch / max(1, n_f), "write_bytes_per_launch": write / max(1, n_w),
           "algorithmic_bytes_per_frame": algo_pf,
           "source": f"profiles/{ROUND}_summary.md (rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes)"},
          open(os.path.join(PROF, "pmc_traffic.json"), "w"), indent=1)

with open(os.path.join(PROF, f"{ROUND}_summary.md"), "w") as f:
    f.write(f"# {ROUND} profile: `bench.py --frames {FRAMES} --steps 3 --warmup 1` on one MI355X\n\n")
    f.write("Command: `bash tools/round_profile.sh` (rocprofv3 --kernel-trace --stats; then separate "
            "--pmc FETCH_SIZE and --pmc WRITE_SIZE passes of the same command).\n\n")
    if b:
        f.write(f"bench line (traced run): value = {b['value']:.4g} keypoints/s, ms_per_step = "
                f"{b['ms_per_step']:.2f}, stage_ms_per_step = {json.dumps(b['stage_ms_per_step'])}\n\n")
    f.write("## Pyramid stage (the roofline kernel group: k_seed + k_blur<R>)\n\n")
    f.write(f"* trace, all passes: {pyr_n} launches, {pyr_us / 1e3:.3f} ms total, {pyr_us / max(1, pyr_n):.1f} us "
            f"per launch (two-lane passes overlap two chunks, which stretches each launch)\n")
    f.write(f"* trace, serialised stage-timing pass, timed steps: {iso_n} launches, "
            f"{iso_us / max(1, iso_n):.1f} us per launch (under the profiler)\n")
    if b:
        f.write(f"* bench.py (HIP events on the compute stream, serialised pass): pyramid_ms per step = "
                f"{b['stage_ms_per_step']['pyramid_ms']:.3f}, avg launch = {b['roofline']['avg_launch_ms'] * 1e3:.1f} us\n")
    f.write(f"* algorithmic bytes per frame (W*H + 44*sum P_o) = {algo_pf / 1e6:.1f} MB; per launch "
            f"{algo_pf * chunk / launches_per_chunk / 1e6:.1f} MB ({launches_per_chunk:.0f} launches per chunk of {chunk} frames)\n")
    f.write(f"* HBM traffic (PMC, FETCH_SIZE x2 + WRITE_SIZE, mean over {n_f} pyramid dispatches) = "
            f"{traffic_pl / 1e6:.1f} MB per launch = {traffic_pf / 1e6:.1f} MB per frame "
            f"(read {fetch / max(1, n_f) / 1e6:.1f} MB, write {write / max(1, n_w) / 1e6:.1f} MB per launch); "
            f"traffic / algorithmic = {traffic_pf / algo_pf:.2f}\n\n")
    f.write("## Kernels (trace, all calls)\n\n| kernel | launches | total ms | avg us | share |\n|---|---|---|---|---|\n")
    for k, (n, us) in sorted(agg.items(), key=lambda kv: -kv[1][1]):
        if not (k.startswith("k_") or "hipcub" in k or "rocprim" in k):
            continue
        f.write(f"| `{k}` | {n} | {us / 1e3:.3f} | {us / n:.1f} | {100 * us / tot:.1f}% |\n")
print(open(os.path.join(PROF, f"{ROUND}_summary.md")).read())
