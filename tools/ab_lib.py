"""Interleaved A/B of library builds (OP_LIB_VARIANT) or environment settings with per-class times:
each variant runs in its own child process per round (a process loads one library).
usage: ab_lib.py ROUNDS base v1 NAME=VALUE[,NAME=VALUE] v1,NAME=VALUE ...  (NAME=VALUE parts set env
vars; a bare part picks the library variant, else the product library)
AB_BENCH_ARGS: extra bench.py arguments (e.g. "--precise --frame 720x1280 --steps 5")."""
import json
import os
import subprocess
import sys

rounds = int(sys.argv[1])
variants = sys.argv[2:]
here = os.path.dirname(os.path.abspath(__file__))
out = {v: [] for v in variants}
for r in range(rounds):
    for v in variants:
        # comma-separated parts: NAME=VALUE sets an env var, a bare name picks the library variant
        parts = v.split(",")
        libs = [x for x in parts if "=" not in x and x != "base"]
        env = dict(os.environ, OP_LIB_VARIANT=libs[0] if libs else "",
                   **dict(kv.split("=", 1) for kv in parts if "=" in kv))
        p = subprocess.run([sys.executable, os.path.join(here, "..", "bench.py"), "--no-cpu-baseline", "--no-variants", "--steps", "10",
                            "--warmup", "2"] + os.environ.get("AB_BENCH_ARGS", "").split(), env=env, capture_output=True,
                           text=True, timeout=300)
        if p.returncode:
            print(p.stdout[-2000:], p.stderr[-2000:])
            sys.exit(p.returncode)
        d = json.loads(p.stdout.strip().splitlines()[-1])
        out[v].append((d["value"], d["stage_ms_per_step"]))
        print(r, v, d["value"], d["stage_ms_per_step"], flush=True)
for v in variants:
    vals = sorted(x[0] for x in out[v])
    c3 = sorted(x[1]["conv3x3"] for x in out[v])
    c7 = sorted(x[1]["conv7x7"] for x in out[v])
    mr = sorted(x[1].get("map_resize", 0.0) for x in out[v])
    pp = sorted(x[1].get("postprocess", 0.0) for x in out[v])
    print("%-8s fps median %.1f | conv3x3 median %.3f | conv7x7 median %.3f | map_resize median %.3f | "
          "postprocess median %.3f" % (v, vals[len(vals) // 2], c3[len(c3) // 2], c7[len(c7) // 2], mr[len(mr) // 2],
                                       pp[len(pp) // 2]))
