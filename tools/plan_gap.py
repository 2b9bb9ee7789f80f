"""What runs between two plans of the hottest book in a rocprofv3 kernel trace of bench.py
(run_kernel_trace.csv): every dispatch that overlaps the gap from one plan's end to the next one's
start, by queue, in microseconds from the plan's end.  usage:
  python tools/plan_gap.py <trace dir>/run_kernel_trace.csv [pair index from the end, default 2]"""
import csv
import sys

PLANS = ("k_flow_plan_head", "k_flow_plan_early", "k_flow_plan_deep")


def main(path, back=2):
    rows = list(csv.DictReader(open(path)))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    nm = lambda r: r["Kernel_Name"].split("(")[0].replace("void ", "").strip()
    plans = [r for r in rows if nm(r).split("<")[0] in PLANS and int(r["Grid_Size_X"]) <= 1024]
    gaps = [(int(b["Start_Timestamp"]) - int(a["End_Timestamp"])) / 1e3 for a, b in zip(plans, plans[1:])]
    print("plans", len(plans), "gaps us", [round(g, 1) for g in gaps])
    a, b = plans[-back - 1], plans[-back]
    te, ts = int(a["End_Timestamp"]), int(b["Start_Timestamp"])
    print(f"gap {(ts - te) / 1e3:.1f} us after {nm(a)} ({(te - int(a['Start_Timestamp'])) / 1e6:.3f} ms)")
    for r in rows:
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        if e >= te and s <= ts:
            print(f"  q{r['Queue_Id']:>2} {(s - te) / 1e3:9.1f} {(e - te) / 1e3:9.1f} {(e - s) / 1e3:8.1f}  "
                  f"{nm(r)[:48]}  g{r['Grid_Size_X']}x{r['Grid_Size_Y']}")


if __name__ == "__main__":
    main(sys.argv[1], int(sys.argv[2]) if len(sys.argv) > 2 else 2)
