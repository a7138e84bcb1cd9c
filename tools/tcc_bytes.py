"""Per-kernel fabric read bytes from a tools/gpu_tcc_bytes.sh run: 32 x RDREQ_32B + 64 x RDREQ_64B +
128 x RDREQ_128B per dispatch (mean), next to what FETCH_SIZE's formula makes of the same requests
(128-B requests at 64 B) -- the ratio is the pattern's FETCH_SIZE factor.
usage: python tools/tcc_bytes.py gpurun_out/tcc_<tag>"""
import csv
import glob
import os
import sys
from collections import defaultdict


def load(d):
    per = defaultdict(lambda: defaultdict(float))  # (kernel, dispatch) -> counter -> value
    for p in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(p)):
            k = r["Kernel_Name"].split("(")[0].replace("void ", "")
            per[(k, r.get("Dispatch_Id", r.get("Correlation_Id", "")))][r["Counter_Name"]] += float(r["Counter_Value"])
    agg = defaultdict(list)
    for (k, _), c in per.items():
        agg[k].append(c)
    return agg


def main():
    root = sys.argv[1]
    for d in sorted(x for x in glob.glob(os.path.join(root, "*")) if os.path.isdir(x)):
        agg = load(d)
        rows = []
        for k, lst in agg.items():
            n = len(lst)
            m = {c: sum(x.get(c, 0.0) for x in lst) / n for c in
                 ("TCC_EA0_RDREQ_32B_sum", "TCC_EA0_RDREQ_64B_sum", "TCC_EA0_RDREQ_128B_sum", "TCC_EA0_RDREQ_sum")}
            b = 32 * m["TCC_EA0_RDREQ_32B_sum"] + 64 * m["TCC_EA0_RDREQ_64B_sum"] + 128 * m["TCC_EA0_RDREQ_128B_sum"]
            fetch = 32 * m["TCC_EA0_RDREQ_32B_sum"] + 64 * (m["TCC_EA0_RDREQ_sum"] - m["TCC_EA0_RDREQ_32B_sum"])
            rows.append((b * n, k, n, b, fetch, m))
        print("==", os.path.basename(d))
        for _, k, n, b, fetch, m in sorted(rows, reverse=True)[:12]:
            print(f"  {k:58s} n={n:4d} read={b / 1e6:9.1f} MB/launch  fetch_formula={fetch / 1e6:9.1f} MB"
                  f"  factor={b / fetch if fetch else 0:5.2f}  req32/64/128="
                  f"{m['TCC_EA0_RDREQ_32B_sum']:.3g}/{m['TCC_EA0_RDREQ_64B_sum']:.3g}/{m['TCC_EA0_RDREQ_128B_sum']:.3g}"
                  f" all={m['TCC_EA0_RDREQ_sum']:.3g}")


if __name__ == "__main__":
    main()
