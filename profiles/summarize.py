"""Summarise a rocprofv3 run of bench.py (profiles/run_rocprof.sh) into profiles/<tag>.md
and update profiles/traffic.json (PMC HBM bytes per launch of the bench line's roofline kernel,
keyed "<workload>:<kernel>_hbm_bytes_per_launch"; other entries are kept).

gfx950 corrections (MI355X_MICROARCH.md §HBM, cdna_hip_programming.md §7): FETCH_SIZE and
WRITE_SIZE are in KiB; FETCH_SIZE reads half the bytes of wide (16 B/lane) coalesced
streams.  k_flow_plan_head reads its records through the scalar cache (s_load_dwordx8) and
writes its touch log with per-lane dword stores, neither a calibrated width, so both the
raw and the x2 figure are reported and the raw one is used as the traffic estimate."""
import csv
import json
import os
import sys


def rows(path):
    with open(path) as f:
        return list(csv.DictReader(f))


def main(tag, src):
    st = rows(os.path.join(src, "trace", "run_kernel_stats.csv"))
    bench = None
    for line in open(os.path.join(src, "bench_trace.log")):
        if line.startswith("{"):
            bench = json.loads(line)
    KERNEL = bench["roofline"]["kernel"].split(" ")[0] if bench else "k_flow_plan_head"
    workload = bench["config"].get("name", "config3") if bench else "config3"
    def pmc(sub, name):
        vals = [float(r["Counter_Value"]) for r in rows(os.path.join(src, sub, "run_counter_collection.csv"))
                if r["Kernel_Name"].split("(")[0].replace("void ", "").strip() == KERNEL and r["Counter_Name"] == name]
        return sum(vals) / len(vals) if vals else None
    fetch_kib, write_kib = pmc("fetch", "FETCH_SIZE"), pmc("write", "WRITE_SIZE")
    out = [f"# rocprofv3 summary `{tag}`", "",
           "Command: `bash profiles/run_rocprof.sh` (bench.py under `rocprofv3 --kernel-trace --stats`,",
           "then separate `--pmc FETCH_SIZE` and `--pmc WRITE_SIZE` passes).", "",
           "| kernel | calls | avg ns | % |", "|---|---|---|---|"]
    for r in st[:16]:
        out.append(f"| {r['Name']} | {r['Calls']} | {float(r['AverageNs']):.0f} | {float(r['Percentage']):.3f} |")
    km = next(r for r in st if r["Name"].split("(")[0].replace("void ", "").strip() == KERNEL)
    out += ["", f"{KERNEL} average duration (rocprof, all launches incl. warmup): "
                f"{float(km['AverageNs'])/1e6:.3f} ms"]
    if bench:
        out.append(f"{KERNEL} average duration (bench.py HIP events on its stream, timed steps): "
                   f"{bench['roofline']['kernel_ms']} ms")
        out.append(f"algorithmic bytes per launch: {bench['roofline']['alg_bytes_per_launch']}")
    if fetch_kib is not None:
        fb, wb = fetch_kib * 1024, write_kib * 1024
        out += [f"FETCH_SIZE per {KERNEL} launch: {fetch_kib:.0f} KiB = {fb/1e6:.1f} MB (x2 wide-stream correction: {2*fb/1e6:.1f} MB)",
                f"WRITE_SIZE per {KERNEL} launch: {write_kib:.0f} KiB = {wb/1e6:.1f} MB",
                f"traffic estimate (FETCH+WRITE): {(fb+wb)/1e6:.1f} MB per launch"]
        tp = os.path.join(os.path.dirname(__file__), "traffic.json")
        tj = json.load(open(tp)) if os.path.exists(tp) else {}
        tj[f"{workload}:{KERNEL}_hbm_bytes_per_launch"] = int(fb + wb)
        tj[f"{workload}:{KERNEL}_detail"] = {"tag": tag, "fetch_bytes": int(fb), "write_bytes": int(wb),
                                             "note": "rocprofv3 PMC, separate passes, KiB->bytes; FETCH_SIZE not x2-corrected"}
        json.dump(tj, open(tp, "w"), indent=1)
    tr = rows(os.path.join(src, "trace", "run_kernel_trace.csv"))
    starts = [int(r["Start_Timestamp"]) for r in tr if r["Kernel_Name"].startswith("k_adm")]
    if starts:  # timeline of the last batch (k_adm and the radix sort open every batch)
        t0 = max(starts) - 20000
        last = sorted((r for r in tr if int(r["Start_Timestamp"]) >= t0), key=lambda r: int(r["Start_Timestamp"]))
        out += ["", "Timeline of the last batch (ms from its admission kernel - 20 us; queue = HIP stream's HW queue):", "",
                "| kernel | queue | start | end | dur |", "|---|---|---|---|---|"]
        for r in last:
            a0, a1 = (int(r["Start_Timestamp"]) - t0) / 1e6, (int(r["End_Timestamp"]) - t0) / 1e6
            out.append(f"| {r['Kernel_Name'].split('(')[0][:48]} | {r['Queue_Id']} | {a0:.3f} | {a1:.3f} | {a1 - a0:.3f} |")
    if bench:
        out += ["", "bench line of the traced run:", "", "```", json.dumps(bench), "```"]
    open(os.path.join(os.path.dirname(__file__), f"{tag}.md"), "w").write("\n".join(out) + "\n")
    print("\n".join(out))


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
