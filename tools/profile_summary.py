"""Summarise a round profile (tools/round_profile.sh) into profiles/.

    python3 tools/profile_summary.py <round> <out dir> <frames per call> [W H]

Reads the passes under <out dir> (trace/, fetch/, write/, sq1/, sq2/; raw
CSVs, optionally gzipped) and writes
  profiles/<round>_kernel_stats.csv   rocprofv3 --stats output (copied)
  profiles/<round>_summary.md         per-kernel table; the pyramid stage from
                                      the trace next to bench.py's own number,
                                      per launch position (octave, blur) of the
                                      serialised pass; HBM traffic from the
                                      PMC passes; SQ counters per kernel
  profiles/pmc_traffic.json           pyramid traffic per launch, read by
                                      bench.py for roofline.traffic
and copies of them into <out dir>/profiles/ (gpurun merges only gpurun_out/).
HBM bytes follow MI355X_MICROARCH.md (HBM section): FETCH_SIZE and WRITE_SIZE
are in KiB; on gfx950 FETCH_SIZE counts half the bytes of 16-B-per-lane
streaming reads (doubled here); WRITE_SIZE is exact for 16-B stores.
SQ_* cycle counters count quad-cycles (x4 = cycles); GRBM_GUI_ACTIVE is summed
over the 8 XCDs.
"""
import csv
import glob
import gzip
import io
import json
import math
import os
import re
import shutil
import sys
from collections import defaultdict

ROUND, OUT, FRAMES = sys.argv[1], sys.argv[2], int(sys.argv[3])
W, H = (int(sys.argv[4]), int(sys.argv[5])) if len(sys.argv) > 5 else (1920, 1080)
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PROF = os.path.join(ROOT, "profiles")
os.makedirs(PROF, exist_ok=True)
PYR = ("k_seed", "k_blur", "k_octave_tail")
N_SIMD = 256 * 4


def short(n):
    return re.sub(r"\(.*", "", n).replace("void ", "").replace("siftmi::", "")


def one(pattern):
    f = sorted(glob.glob(os.path.join(OUT, pattern), recursive=True))
    f += sorted(glob.glob(os.path.join(OUT, pattern + ".gz"), recursive=True))
    return f[0] if f else None


def rows_of(path):
    if path is None:
        return []
    raw = gzip.open(path, "rt") if path.endswith(".gz") else open(path)
    with raw as fh:
        return list(csv.DictReader(io.StringIO(fh.read())))


def bench_line(log):
    if not os.path.exists(log):
        return None
    for line in open(log):
        if line.startswith("{"):
            return json.loads(line)
    return None


trace = one("trace/**/run_kernel_trace.csv")
stats = one("trace/**/run_kernel_stats.csv")
if stats:
    shutil.copy(stats, os.path.join(PROF, f"{ROUND}_kernel_stats.csv"))
b = bench_line(os.path.join(OUT, "bench_trace.log"))
steps = b["steps"] if b else 3

# ---- trace: per kernel totals -------------------------------------------------
agg = defaultdict(lambda: [0, 0.0])
rows = rows_of(trace)
for r in rows:
    k = short(r["Kernel_Name"])
    agg[k][0] += 1
    agg[k][1] += (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
tot = sum(v[1] for k, v in agg.items() if k.startswith("k_") or "rocprim" in k)

# ---- the serialised stage-timing pass of bench.py (the roofline's HIP-event
# figure): chunks start at k_seed*; a chunk is every kernel started between its
# seed and the next one, on any stream (the lane's stream and its aux stream:
# octave overlap, host.cpp run_pyramid).  A chunk is serialised when it starts
# after the previous chunk's kernels end and ends before the next seed (the
# one-lane pass; the two-lane pass overlaps neighbour chunks).  One warmup step
# precedes the timed steps.
sk = sorted(((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Stream_Id"], short(r["Kernel_Name"]),
              int(r.get("Dispatch_Id") or 0))
             for r in rows if short(r["Kernel_Name"]).startswith("k_") or "rocprim" in r["Kernel_Name"]))
seeds = [i for i, x in enumerate(sk) if x[3].startswith("k_seed")]
chunks = [sk[a:z] for a, z in zip(seeds, seeds[1:] + [len(sk)])]
ser = []
for i, g in enumerate(chunks):
    prev_end = max(x[1] for x in chunks[i - 1]) if i else 0
    nxt = chunks[i + 1][0][0] if i + 1 < len(chunks) else 1 << 62
    ser.append(prev_end <= g[0][0] and max(x[1] for x in g) <= nxt)
best, c0 = (0, 0), None
for i, sflag in enumerate(ser + [False]):
    if sflag and c0 is None:
        c0 = i
    if not sflag and c0 is not None:
        if i - c0 > best[1] - best[0]:
            best = (c0, i)
        c0 = None
groups = chunks[best[0]:best[1]]
full = max((sum(1 for x in g if x[3].startswith(PYR)) for g in groups), default=0)
groups = [g for g in groups if sum(1 for x in g if x[3].startswith(PYR)) == full]
chunks_per_call = max(1, len(groups) // (steps + 1))
timed = groups[-steps * chunks_per_call:]
n_oct = int(round(math.log2(min(2 * W, 2 * H)) - 2)) + 1
dims = [((2 * W) >> o, (2 * H) >> o) for o in range(n_oct)]
sum_p = sum(w * h for w, h in dims)
algo_pf = W * H + 44 * sum_p  # u8 read once, G_0..G_5 + D_0..D_4 written once
CHUNK_MODE = int(os.environ.get("CHUNK_MODE", "1"))  # host auto_chunk, path option chunk_mode
scale = 2.0 if CHUNK_MODE == 1 else 1.0
cmax = min(256, max(1, int(scale * 32e9 // (44.0 * sum_p))),
           max(1, int(scale * 64.0 * 3840 * 2160 // (4.0 * W * H))))
nck = max(-(-FRAMES // cmax), 2 if FRAMES >= 2 and CHUNK_MODE != 1 else 1)
chunk = -(-FRAMES // nck)

pos = defaultdict(list)     # launch position in the chunk (enqueue order) -> (start, duration) (us)
stage = defaultdict(float)  # non-pyramid kernels of the timed chunks (us)
spans = []                  # pyramid wall time per chunk: seed start -> last pyramid kernel end (us)
for g in timed:
    pyr = sorted((x for x in g if x[3].startswith(PYR)), key=lambda x: x[4])
    t0 = min(x[0] for x in pyr)
    spans.append((max(x[1] for x in pyr) - t0) / 1e3)
    for j, x in enumerate(pyr):
        pos[(j, x[3], x[2])].append(((x[0] - t0) / 1e3, (x[1] - x[0]) / 1e3))
    for x in g:
        if not x[3].startswith(PYR):
            stage[x[3]] += (x[1] - x[0]) / 1e3
iso_us = sum(spans)
iso_n = sum(len(v) for v in pos.values())
busy_us = sum(d for v in pos.values() for _, d in v)


def launch_blurs(k):
    """Blurs of the chain a pyramid launch performs (seed: 0; the seed pair:
    the seed and blur 1, counted as -1)."""
    if k.startswith("k_seed_pair"):
        return -1
    if k.startswith("k_seed"):
        return 0
    if k.startswith("k_blur2"):
        return 2
    if k.startswith("k_octave_tail"):
        return None  # every remaining octave
    return 1


def pos_info(seq):
    """(octave, blurs, actual HBM bytes) per launch of a chunk, from the
    kernel sequence in enqueue order: the seed reads the u8 frame and writes
    G_0; a blur reads G_{s-1} and writes G_s (8 B/px), a pair reads G_{s-1}
    and writes G_s, G_{s+1} (12 B/px); blur s = 3 also writes the next
    octave's G_0 (1 B/px); k_blur_detect (blur 5 + the scan) reads G_0..G_4
    and writes G_5 (24 B/px); the tail reads G_0 of its first octave and
    writes everything after it.  The first n octaves' blur 5 is a
    k_blur_detect launch, n = the number of those in the chunk; octave 0's is
    enqueued late (deferred until octave 1's G_3), so every launch is placed
    in the lowest octave with a blur it can perform pending."""
    n_fused = sum(1 for k in seq if k.startswith("k_blur_detect"))
    nxt = [1] * n_oct  # next blur (1..5; 6 = octave done) per octave
    out = []
    for k in seq:
        nb = launch_blurs(k)
        if nb == 0:
            out.append((0, "seed", chunk * (W * H + 4 * dims[0][0] * dims[0][1])))
            continue
        if nb == -1:  # k_seed_pair: u8 read, G_0 and G_1 written
            out.append((0, "seed,1", chunk * (W * H + 8 * dims[0][0] * dims[0][1])))
            nxt[0] = 2
            continue
        if nb is None:  # the tail: every octave not done
            o = next((i for i in range(n_oct) if nxt[i] <= 5), n_oct - 1)
            by = 4 * dims[o][0] * dims[o][1]
            for oo in range(o, n_oct):
                by += 4 * 5 * dims[oo][0] * dims[oo][1] + (4 * dims[oo + 1][0] * dims[oo + 1][1] if oo + 1 < n_oct else 0)
            out.append((o, f"{o}..{n_oct - 1}", chunk * by))
            for oo in range(o, n_oct):
                nxt[oo] = 6
            continue
        if k.startswith("k_blur_detect"):
            o = next(i for i in range(n_oct) if nxt[i] == 5)
            px = dims[o][0] * dims[o][1]
            out.append((o, "5+scan", chunk * 24 * px))
            nxt[o] = 6
            continue
        # a strip blur / pair: the lowest octave with such a blur pending (a
        # fused octave's blur 5 is left to its k_blur_detect)
        o = next(i for i in range(n_oct) if nxt[i] <= (4 if i < n_fused else 5))
        s = nxt[o]
        px = dims[o][0] * dims[o][1]
        by = (4 + 4 * nb) * px + (px if (s <= 3 < s + nb) and o + 1 < n_oct else 0)
        out.append((o, f"{s}" if nb == 1 else f"{s},{s + 1}", chunk * by))
        nxt[o] = s + nb
    return out


# ---- PMC passes ---------------------------------------------------------------
def pmc_rows(kind):
    return rows_of(one(f"{kind}/**/run_counter_collection.csv"))


def pmc_sum(rows_, name, pred):
    v, n = 0.0, 0
    for r in rows_:
        if r["Counter_Name"] == name and pred(short(r["Kernel_Name"])):
            v += float(r["Counter_Value"])
            n += 1
    return v, n


fr, wr = pmc_rows("fetch"), pmc_rows("write")
is_pyr = lambda k: k.startswith(PYR)
fetch, n_f = pmc_sum(fr, "FETCH_SIZE", is_pyr)
fetch *= 2.0 * 1024.0  # KiB -> bytes; gfx950: half of 16-B streaming reads counted
write, n_w = pmc_sum(wr, "WRITE_SIZE", is_pyr)
write *= 1024.0
launches_per_chunk = full
traffic_pl = fetch / max(1, n_f) + write / max(1, n_w)
traffic_pf = traffic_pl * launches_per_chunk / chunk
if n_f and n_w:
    tj = {"round": ROUND, "frame": f"{W}x{H}", "frames_per_call": FRAMES, "frames_per_chunk": chunk,
          "pyramid_hbm_bytes_per_launch": traffic_pl, "pyramid_hbm_bytes_per_frame": traffic_pf,
          "fetch_bytes_per_launch": fetch / max(1, n_f), "write_bytes_per_launch": write / max(1, n_w),
          "algorithmic_bytes_per_frame": algo_pf,
          "source": f"profiles/{ROUND}_summary.md (rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes)"}
    # bench.py reads pmc_traffic.json for its own (1080p) frame size
    TJ = "pmc_traffic.json" if (W, H) == (1920, 1080) else f"pmc_traffic_{W}x{H}.json"
    json.dump(tj, open(os.path.join(PROF, TJ), "w"), indent=1)

# per-kernel SQ counters (sums over every dispatch of the kernel in the pass)
sq = defaultdict(lambda: defaultdict(float))
sq_n = defaultdict(int)
for kind in ("sq1", "sq2", "fetch", "write"):
    seen = set()
    for r in pmc_rows(kind):
        k = short(r["Kernel_Name"])
        sq[k][r["Counter_Name"]] += float(r["Counter_Value"])
        if kind == "sq1" and (r.get("Dispatch_Id"), k) not in seen:
            seen.add((r.get("Dispatch_Id"), k))
            sq_n[k] += 1

out_md = os.path.join(PROF, f"{ROUND}_summary.md")
with open(out_md, "w") as f:
    f.write(f"# {ROUND} profile: `bench.py --frames {FRAMES} --width {W} --height {H} --steps {steps} --warmup 1 "
            f"--no-configs` on one MI355X\n\n")
    f.write("Command: `bash tools/round_profile.sh` (rocprofv3 --kernel-trace --stats; then separate "
            "--pmc passes: FETCH_SIZE; WRITE_SIZE; two SQ counter groups). Summarised by "
            "`tools/profile_summary.py`.\n\n")
    if b:
        f.write(f"bench line (traced run): value = {b['value']:.4g} keypoints/s, ms_per_step = "
                f"{b['ms_per_step']:.2f}, stage_ms_per_step = {json.dumps(b['stage_ms_per_step'])}\n\n")
    f.write("## Pyramid stage (the roofline kernel group: k_seed* + k_blur*)\n\n")
    f.write(f"* trace, serialised stage-timing pass, timed steps: {iso_n} launches "
            f"({len(timed)} chunks of {chunk} frames, {launches_per_chunk} launches each on two streams); "
            f"pyramid wall time (seed start -> last pyramid kernel end) {iso_us / max(1, len(timed)) / 1e3:.3f} ms "
            f"per chunk = {iso_us / max(1, iso_n):.1f} us per launch (wall / launches: the figure bench.py's "
            f"roofline divides by); summed kernel durations {busy_us / max(1, len(timed)) / 1e3:.3f} ms per chunk "
            f"(> wall: launches of the two streams overlap)\n")
    if b:
        f.write(f"* bench.py (HIP events on the compute stream, serialised pass): pyramid_ms per step = "
                f"{b['stage_ms_per_step']['pyramid_ms']:.3f}, avg launch = {b['roofline']['avg_launch_ms'] * 1e3:.1f} us\n")
    f.write(f"* algorithmic bytes per frame (W*H + 44*sum P_o) = {algo_pf / 1e6:.1f} MB; per launch "
            f"{algo_pf * chunk / max(1, launches_per_chunk) / 1e6:.1f} MB\n")
    if n_f and n_w:
        f.write(f"* HBM traffic (PMC, FETCH_SIZE x2 + WRITE_SIZE, mean over {n_f} pyramid dispatches) = "
                f"{traffic_pl / 1e6:.1f} MB per launch = {traffic_pf / 1e6:.1f} MB per frame "
                f"(read {fetch / max(1, n_f) / 1e6:.1f} MB, write {write / max(1, n_w) / 1e6:.1f} MB per launch); "
                f"traffic / algorithmic = {traffic_pf / algo_pf:.2f}\n")
    f.write("\n### Per launch position (serialised pass, enqueue order; start / end from the chunk's seed start; "
            "actual bytes = what the launch must read + write; TB/s over the launch's own duration, while "
            "it shares the chip with the other stream's launches)\n\n")
    f.write("| pos | octave | blur | kernel | stream | start us | end us | avg us | actual MB | TB/s |\n"
            "|---|---|---|---|---|---|---|---|---|---|\n")
    items = sorted(pos.items())
    info = pos_info([k for (j, k, st), v in items])
    for ((j, k, st), v), (o, sl, by) in zip(items, info):
        a0 = sum(x[0] for x in v) / len(v)
        us = sum(x[1] for x in v) / len(v)
        f.write(f"| {j} | {o} | {sl} | `{k}` | {st} | {a0:.1f} | {a0 + us:.1f} | {us:.1f} | {by / 1e6:.1f} | "
                f"{by / (us * 1e-6) / 1e12:.2f} |\n")
    if stage:
        f.write("\n### Other stages in the same serialised chunks (ms per chunk)\n\n| kernel | ms |\n|---|---|\n")
        for k, us in sorted(stage.items(), key=lambda kv: -kv[1]):
            f.write(f"| `{k[:60]}` | {us / max(1, len(timed)) / 1e3:.3f} |\n")
    if sq:
        f.write("\n## SQ counters per kernel (all dispatches of the profiled command)\n\n")
        f.write("Wave-cycle fractions are of SQ_WAVE_CYCLES (quad-cycles, summed over waves): `valu` = "
                "SQ_ACTIVE_INST_VALU, `lds` = SQ_ACTIVE_INST_LDS, `wait` = SQ_WAIT_ANY (parked at a waitcnt / "
                "barrier), `stall` = SQ_WAIT_INST_ANY (ready but not issued). `waves/SIMD` = SQ_WAVE_CYCLES / "
                "(1024 SIMDs x GRBM_GUI_ACTIVE / 8 XCDs / 4): mean resident waves per SIMD while the kernel "
                "ran, so `valu` x `waves/SIMD` approximates the SIMD's VALU issue share. `bank` = "
                "SQ_LDS_BANK_CONFLICT / SQ_ACTIVE_INST_LDS.\n\n")
        f.write("| kernel | dispatches | VALU insts / wave | valu | lds | wait | stall | waves/SIMD | bank |\n"
                "|---|---|---|---|---|---|---|---|---|\n")
        keys = sorted(sq, key=lambda k: -sq[k].get("SQ_WAVE_CYCLES", 0))
        for k in keys:
            c = sq[k]
            wc = c.get("SQ_WAVE_CYCLES", 0)
            if wc <= 0 or not (k.startswith("k_") or "rocprim" in k):
                continue
            waves = max(1.0, c.get("SQ_WAVES", 0))
            gui = c.get("GRBM_GUI_ACTIVE", 0) / 8
            vb = wc / (N_SIMD * gui / 4) if gui else float("nan")
            lds = c.get("SQ_ACTIVE_INST_LDS", 0)
            f.write(f"| `{k[:48]}` | {sq_n[k]} | {c.get('SQ_INSTS_VALU', 0) / waves:.0f} | "
                    f"{c.get('SQ_ACTIVE_INST_VALU', 0) / wc:.2f} | {lds / wc:.2f} | "
                    f"{c.get('SQ_WAIT_ANY', 0) / wc:.2f} | {c.get('SQ_WAIT_INST_ANY', 0) / wc:.2f} | "
                    f"{vb:.2f} | {c.get('SQ_LDS_BANK_CONFLICT', 0) / lds if lds else 0:.3f} |\n")
    f.write("\n## Kernels (trace, all calls)\n\n| kernel | launches | total ms | avg us | share |\n|---|---|---|---|---|\n")
    for k, (n, us) in sorted(agg.items(), key=lambda kv: -kv[1][1]):
        if not (k.startswith("k_") or "rocprim" in k):
            continue
        f.write(f"| `{k[:90]}` | {n} | {us / 1e3:.3f} | {us / n:.1f} | {100 * us / max(1e-9, tot):.1f}% |\n")

dst = os.path.join(OUT, "profiles")
os.makedirs(dst, exist_ok=True)
for name in (f"{ROUND}_summary.md", f"{ROUND}_kernel_stats.csv", "pmc_traffic.json", f"pmc_traffic_{W}x{H}.json"):
    p = os.path.join(PROF, name)
    if os.path.exists(p):
        shutil.copy(p, os.path.join(dst, name))
print(open(out_md).read())
