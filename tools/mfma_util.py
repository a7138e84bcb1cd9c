"""Per-kernel MFMA utilisation and clock from the tools/clk_counters.sh pass.

SQ_VALU_MFMA_BUSY_CYCLES counts MFMA pipe cycles summed over every SIMD (16 per
v_mfma_f32_16x16x32_bf16, 32 per 32x32x16: MI355X_MICROARCH.md cycle constants), GRBM_GUI_ACTIVE
counts GPU cycles summed over the 8 XCDs, so per kernel:
  clock       = GRBM_GUI_ACTIVE / 8 / duration
  MFMA busy   = SQ_VALU_MFMA_BUSY_CYCLES / (256 CUs x 4 SIMDs x GRBM_GUI_ACTIVE / 8)
usage: python tools/mfma_util.py gpurun_out/clk_<tag>
"""
import csv
import os
import sys
from collections import defaultdict


def main(d):
    acc = defaultdict(lambda: defaultdict(float))
    for r in csv.DictReader(open(os.path.join(d, "run_counter_collection.csv"))):
        k = r["Kernel_Name"].split("(")[0].replace("void ", "")[:60]
        acc[k][r["Counter_Name"]] += float(r["Counter_Value"])
    dur = defaultdict(float)
    for r in csv.DictReader(open(os.path.join(d, "run_kernel_trace.csv"))):
        k = r["Kernel_Name"].split("(")[0].replace("void ", "")[:60]
        dur[k] += (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-9
    print("| kernel | time share | clock GHz | MFMA busy (at that clock) |")
    print("|---|---|---|---|")
    tot = sum(dur[k] for k in acc)
    for k, c in sorted(acc.items(), key=lambda kv: -dur[kv[0]]):
        if not dur[k] or not c.get("GRBM_GUI_ACTIVE"):
            continue
        cyc = c["GRBM_GUI_ACTIVE"] / 8
        busy = c["SQ_VALU_MFMA_BUSY_CYCLES"] / (256 * 4 * cyc)
        if dur[k] / tot < 0.005:
            continue
        print("| `%s` | %.1f %% | %.2f | %.2f |" % (k, 100 * dur[k] / tot, cyc / dur[k] * 1e-9, busy))


if __name__ == "__main__":
    main(sys.argv[1])
