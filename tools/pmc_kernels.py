"""Per-kernel PMC summary of rocprofv3 --pmc runs of bench.py (one counter set per run directory):
the average counter value per launch of each kernel, with its launch count.
  python tools/pmc_kernels.py <run_counter_collection.csv> [more csv ...]"""
import collections
import csv
import sys


def main(paths):
    agg = collections.defaultdict(lambda: collections.defaultdict(list))
    for p in paths:
        for r in csv.DictReader(open(p)):
            k = r["Kernel_Name"].split("(")[0].replace("void ", "").strip()
            agg[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
    names = sorted({c for k in agg for c in agg[k]})
    print("kernel".ljust(34) + "".join(n[:16].rjust(17) for n in names) + "  launches")
    rows = sorted(agg.items(), key=lambda kv: -sum(sum(v) / len(v) for v in kv[1].values()))
    for k, cs in rows:
        vals = [sum(cs[n]) / len(cs[n]) if n in cs else float("nan") for n in names]
        print(k[:34].ljust(34) + "".join(f"{v:17.0f}" for v in vals) + f"  {max(len(v) for v in cs.values())}")


if __name__ == "__main__":
    main(sys.argv[1:])
