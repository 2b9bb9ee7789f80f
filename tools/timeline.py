"""Timeline of the last batch of a rocprofv3 kernel trace (tools/trace_workload.sh): every
kernel's start / end relative to the batch's admission kernel, grouped by HW queue."""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
starts = [int(r["Start_Timestamp"]) for r in rows if r["Kernel_Name"].startswith("gome::k_adm(")]
t0 = max(starts)
lim = float(sys.argv[2]) if len(sys.argv) > 2 else 0.05
last = sorted((r for r in rows if int(r["Start_Timestamp"]) >= t0 - 20000), key=lambda r: int(r["Start_Timestamp"]))
for r in last:
    a0, a1 = (int(r["Start_Timestamp"]) - t0) / 1e6, (int(r["End_Timestamp"]) - t0) / 1e6
    if a1 - a0 >= lim:
        print(f"{r['Kernel_Name'].split('(')[0][:44]:44s} q{r['Queue_Id']:>3s} {a0:8.3f} {a1:8.3f} {a1 - a0:8.3f}")
