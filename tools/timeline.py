"""Timeline of the last batch in a rocprofv3 kernel trace of bench.py (run_kernel_trace.csv):
every kernel with its stream, start and end relative to the batch's first kernel (k_adm opens
each batch on the flow stream, the radix sort on the main stream).  usage:
  python tools/timeline.py <trace dir>/run_kernel_trace.csv [batch index from the end, default 1]"""
import csv
import sys


def main(path, back=1):
    rows = list(csv.DictReader(open(path)))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    opens = [i for i, r in enumerate(rows) if r["Kernel_Name"].startswith("k_adm") and
             r["Kernel_Name"].split("(")[0].strip().endswith("k_adm")]
    a = opens[-back]
    b = opens[-back + 1] if back > 1 else len(rows)
    # the batch's first kernel may be a memset or the index rebuild just before k_adm
    t0 = min(int(r["Start_Timestamp"]) for r in rows[max(0, a - 8):a + 1])
    seg = [r for r in rows[max(0, a - 8):b] if int(r["Start_Timestamp"]) >= t0]
    tend = max(int(r["End_Timestamp"]) for r in seg)
    print(f"batch span {(tend - t0) / 1e3:.1f} us, {len(seg)} dispatches")
    for r in seg:
        s, e = int(r["Start_Timestamp"]) - t0, int(r["End_Timestamp"]) - t0
        name = r["Kernel_Name"].split("(")[0].replace("void ", "").strip()[:44]
        print(f"  q{r['Queue_Id']:>2} {s / 1e3:9.1f} {e / 1e3:9.1f} {(e - s) / 1e3:8.1f}  {name}  "
              f"grid {r['Grid_Size_X']}x{r['Grid_Size_Y']} wg {r['Workgroup_Size_X']}")


if __name__ == "__main__":
    main(sys.argv[1], int(sys.argv[2]) if len(sys.argv) > 2 else 1)
