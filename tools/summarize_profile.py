"""Summarise a tools/profile.sh run into profiles/<tag>.md + profiles/<tag>_traffic.json.

HBM (fabric) traffic per launch follows MI355X_MICROARCH.md §HBM: FETCH_SIZE and WRITE_SIZE come
from separate --pmc passes (KiB units), and FETCH_SIZE is doubled.  Round 3 measured why, per
kernel (tools/gpu_tcc_bytes.sh, profiles/r03/tcc_r03g_request_sizes.txt): every read request our
kernels and the calibration micro-benchmark send to the fabric is a 128-B request
(TCC_EA0_RDREQ_128B == TCC_EA0_RDREQ), and FETCH_SIZE's formula counts 128-B requests through
TCC_BUBBLE, which stays 0, i.e. at 64 B each.  Rounds 1-2 applied x0.98 / x1.12 to the conv halo
patterns from tools/micro/fetch_calib.hip, which compared FETCH_SIZE with the bytes the kernel USED;
a 64-B chunk of a 128-B line still moves the whole line, so those factors under-reported the conv
kernels' traffic by about 2x (profiles/fetch_calib_r03.md).
usage: python tools/summarize_profile.py gpurun_out/prof_<tag> <tag>
"""
import csv
import json
import os
import sys
from collections import defaultdict


def kernel_stats(d):
    return list(csv.DictReader(open(os.path.join(d, "stats", "run_kernel_stats.csv"))))


def pmc(d, sub, counter):
    p = os.path.join(d, sub, "run_counter_collection.csv")
    if not os.path.exists(p):
        return {}
    acc = defaultdict(list)
    for r in csv.DictReader(open(p)):
        if r["Counter_Name"] == counter:
            acc[r["Kernel_Name"]].append(float(r["Counter_Value"]))
    return acc


# FETCH_SIZE -> bytes: every read request is 128 B, tallied at 64 B (see the docstring)
def fetch_factor(name):
    return 2.0


def short(name):
    return name.split("(")[0].replace("void ", "")


def main():
    d, tag = sys.argv[1], sys.argv[2]
    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    stats = kernel_stats(d)
    fetch = pmc(d, "fetch", "FETCH_SIZE")
    write = pmc(d, "write", "WRITE_SIZE")
    bench = ""
    for line in open(os.path.join(d, "bench_stats.log")):
        if line.startswith("{"):
            bench = json.loads(line)
    lines = ["# rocprofv3 summary: %s" % tag, "",
             "Command: `rocprofv3 --kernel-trace --stats -- python3 bench.py --steps 5 --warmup 2 %s`; "
             "PMC: separate `--pmc FETCH_SIZE` / `--pmc WRITE_SIZE` passes with `--kernel-trace` only "
             "(bench `--steps 2 --warmup 1 --no-profile`)." % bench.get("config", {}).get("workload", ""), "",
             "Bench line of the stats pass: value %.1f frames/s, ms/step %.2f, dtype %s, batch %s." % (
                 bench.get("value", 0), bench.get("ms_per_step", 0), bench.get("dtype"),
                 bench.get("config", {}).get("frames_per_step_per_gpu")), "",
             "| kernel | calls | avg us | total % | HBM read MB/launch (FETCH_SIZE x 2: 128-B requests) | HBM write MB/launch |",
             "|---|---|---|---|---|---|"]
    traffic = {}
    for r in stats:
        name = r["Name"]
        f = fetch.get(name, [])
        w = write.get(name, [])
        fr = fetch_factor(name) * 1024 * sum(f) / len(f) / 1e6 if f else None
        wr = 1024 * sum(w) / len(w) / 1e6 if w else None
        if fr is not None and wr is not None:
            traffic[short(name)] = {"read_bytes": fr * 1e6, "write_bytes": wr * 1e6, "avg_ns": float(r["AverageNs"]),
                                   "calls": int(r["Calls"]), "fetch_factor": round(fetch_factor(name), 4)}
        lines.append("| `%s` | %s | %.1f | %.2f | %s | %s |" % (
            short(name)[:80], r["Calls"], float(r["AverageNs"]) / 1e3, float(r["Percentage"]),
            "%.1f" % fr if fr is not None else "-", "%.1f" % wr if wr is not None else "-"))
    os.makedirs(os.path.join(repo, "profiles"), exist_ok=True)
    open(os.path.join(repo, "profiles", tag + ".md"), "w").write("\n".join(lines) + "\n")
    json.dump({"tag": tag, "config": bench.get("config"), "dtype": bench.get("dtype"),
               "precision": "fp32" if bench.get("dtype") == "f32" else "bf16x3",
               "halo_mode": int(os.environ.get("OP_HALO_MODE", "4")), "kernels": traffic},
              open(os.path.join(repo, "profiles", tag + "_traffic.json"), "w"), indent=1)
    print("\n".join(lines[:30]))


if __name__ == "__main__":
    main()
