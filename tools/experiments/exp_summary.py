import json, sys
for v in sys.argv[1:]:
    l = [x for x in open("gpurun_out/exp_%s.log" % v) if x.startswith("{")]
    d = json.loads(l[-1]) if l else None
    print(v, d and (d["value"], d["ms_per_step"], d["stage_ms_per_step"], d["roofline"] and d["roofline"]["frac"]))
