"""Average kernel times of tools/kstats.sh runs: python tools/kstats_sum.py PATTERN DIR [DIR ...]
(one line per run and matching kernel: tag, environment, calls, average us)"""
import csv
import os
import re
import sys

pat = re.compile(sys.argv[1])
for d in sys.argv[2:]:
    f = os.path.join(d, "run_kernel_stats.csv")
    if not os.path.exists(f):
        continue
    env = open(os.path.join(d, "env.txt")).read().strip() if os.path.exists(os.path.join(d, "env.txt")) else ""
    for r in csv.DictReader(open(f)):
        name = r["Name"].split("(")[0].replace("void ", "")
        if pat.search(name):
            print("%-24s %-40s %-60s %5s %10.1f" % (os.path.basename(d), env, name[:60], r["Calls"],
                                                    float(r["AverageNs"]) / 1e3))
