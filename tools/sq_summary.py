"""Per-kernel SQ counter ratios from tools/sq_counters.sh output: python tools/sq_summary.py <dir>"""
import csv
import os
import sys
from collections import defaultdict

d = sys.argv[1]
acc = defaultdict(lambda: defaultdict(float))
cnt = defaultdict(int)
for r in csv.DictReader(open(os.path.join(d, "run_counter_collection.csv"))):
    k = r["Kernel_Name"].split("(")[0].replace("void ", "")[:70]
    acc[k][r["Counter_Name"]] += float(r["Counter_Value"])
    if r["Counter_Name"] == "SQ_WAVE_CYCLES":
        cnt[k] += 1
dur = defaultdict(float)
for f in os.listdir(d):
    if f.endswith("kernel_trace.csv"):
        for r in csv.DictReader(open(os.path.join(d, f))):
            k = r["Kernel_Name"].split("(")[0].replace("void ", "")[:70]
            dur[k] += (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-9
print("%-70s %5s %8s %6s %6s %6s %7s %8s %7s" % ("kernel", "n", "ms", "wait", "winst", "activ", "mfma%", "ldsconf", "wlds"))
for k, c in sorted(acc.items(), key=lambda kv: -dur.get(kv[0], 0)):
    w = c["SQ_WAVE_CYCLES"] or 1
    t = dur.get(k, 0)
    mfma = c["SQ_VALU_MFMA_BUSY_CYCLES"] / (t * 2.4e9 * 1024) if t else 0
    print("%-70s %5d %8.3f %6.3f %6.3f %6.3f %7.3f %8.3f %7.3f" % (
        k, cnt[k], t * 1e3, c["SQ_WAIT_ANY"] / w, c["SQ_WAIT_INST_ANY"] / w, c["SQ_ACTIVE_INST_ANY"] / w, mfma,
        c["SQ_LDS_BANK_CONFLICT"] / max(c["SQ_INSTS_LDS"], 1), c["SQ_WAIT_INST_LDS"] / w))
