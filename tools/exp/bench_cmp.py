import json,sys
for f in sys.argv[1:]:
    try:
        d=json.loads(open(f).read().strip().splitlines()[-1]); print(f, round(d["value"]/1e6,2), round(d["roofline"]["frac"],3), {k:round(v,2) for k,v in d["stage_ms_per_step"].items()}, round(d["ms_per_step"],2))
    except Exception as e: print(f, "ERR", e)
