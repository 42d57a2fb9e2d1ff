import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
r = d["roofline"]
print(sys.argv[2], d["value"], d["ms_per_step"], r["kernel_ms"], r["grid"], r.get("vgprs"))
