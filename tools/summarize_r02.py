"""Summarise a tools/r02_final.sh run (gpurun_out/<tag>/) into profiles/<tag>.md and refresh
profiles/traffic.json (the PMC HBM bytes per launch of the roofline kernel, read by bench.py).

gfx950 counter units (MI355X_MICROARCH.md, HBM / rocprofv3 section): FETCH_SIZE and WRITE_SIZE
are KiB per dispatch; FETCH_SIZE reads half the bytes of wide (16 B/lane) coalesced streams.
k_flow_plan_head reads its records through the scalar cache and writes its touch log with
per-lane dword stores (neither a calibrated width), so the raw figure is used as the estimate
and the x2 figure is listed beside it.

usage: python tools/summarize_r02.py <tag> [gpurun_out dir]"""
import csv
import json
import os
import sys
from collections import defaultdict

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
KERNELS = ("k_flow_plan_head", "k_match")


def rows(path):
    with open(path) as f:
        return list(csv.DictReader(f))


def short(name):
    return name.split("(")[0].replace("gome::", "").replace("void ", "")


def last_json(path):
    out = None
    for line in open(path):
        if line.startswith("{"):
            out = json.loads(line)
    return out


def pmc(src, sub):
    d = defaultdict(list)
    for r in rows(os.path.join(src, sub, "pmc_counter_collection.csv")):
        k = short(r["Kernel_Name"])
        if k in KERNELS:
            d[(k, r["Counter_Name"])].append(float(r["Counter_Value"]))
    return {key: sum(v) / len(v) for key, v in d.items()}


def main(tag, base):
    src = os.path.join(base, tag)
    bench = last_json(os.path.join(src, "bench_default.json"))
    tb = last_json(os.path.join(src, "trace_bench.json"))
    st = rows(os.path.join(src, "trace", "run_kernel_stats.csv"))
    c = {}
    for sub in ("p1", "p2", "p3"):
        c.update(pmc(src, sub))
    out = [f"# rocprofv3 summary `{tag}` (round 2, final tree)", "",
           "Command: `bash tools/r02_final.sh " + tag + "` on one MI355X: the default bench line, then "
           "`rocprofv3 --kernel-trace --stats -- python3 bench.py --steps 5 --warmup 2 --e2e-steps 0 "
           "--no-cpu-baseline` (config 3), then three separate `--pmc` passes of the same command "
           "(FETCH_SIZE / WRITE_SIZE / SQ block) restricted to `k_flow_plan_head` and `k_match`.", ""]
    if bench:
        out += ["## Default bench line (`python bench.py`)", "", "```", json.dumps(bench), "```", ""]
    out += ["## Kernel trace (config 3, all launches incl. warmup)", "",
            "| kernel | calls | avg µs | % |", "|---|---|---|---|"]
    for r in st[:18]:
        out.append(f"| {short(r['Name'])} | {r['Calls']} | {float(r['AverageNs']) / 1e3:.1f} | "
                   f"{float(r['Percentage']):.2f} |")
    km = next(r for r in st if short(r["Name"]) == "k_flow_plan_head")
    out += ["", f"`k_flow_plan_head`: {float(km['AverageNs']) / 1e6:.3f} ms rocprof average (all launches)"]
    if tb:
        out.append(f"vs {tb['roofline']['kernel_ms']} ms from bench.py's HIP events on its stream (timed "
                   f"launches of the traced run); algorithmic bytes per launch "
                   f"{tb['roofline']['alg_bytes_per_launch']}.")
    out += ["", "## PMC per launch (averaged over the launches of each pass)", "",
            "| counter | k_flow_plan_head | k_match |", "|---|---|---|"]
    names = sorted({n for (_, n) in c})
    for n in names:
        a, b = c.get(("k_flow_plan_head", n)), c.get(("k_match", n))
        fa = f"{a:,.0f}" if a is not None else "-"
        fb = f"{b:,.0f}" if b is not None else "-"
        out.append(f"| {n} | {fa} | {fb} |")
    fetch, write = c.get(("k_flow_plan_head", "FETCH_SIZE")), c.get(("k_flow_plan_head", "WRITE_SIZE"))
    if fetch is not None and write is not None:
        fb_, wb_ = fetch * 1024, write * 1024
        out += ["", f"`k_flow_plan_head` HBM traffic: FETCH {fb_ / 1e6:.2f} MB (x2 wide-stream correction "
                    f"{2 * fb_ / 1e6:.2f} MB) + WRITE {wb_ / 1e6:.2f} MB = {(fb_ + wb_) / 1e6:.2f} MB per launch"]
        if tb:
            out.append(f"vs {tb['roofline']['alg_bytes_per_launch'] / 1e6:.2f} MB algorithmic "
                       f"(8 B per order read + 16 B per touch written).")
        json.dump({"tag": tag, "kernel": "k_flow_plan_head",
                   "k_flow_plan_head_hbm_bytes_per_launch": int(fb_ + wb_),
                   "fetch_bytes": int(fb_), "write_bytes": int(wb_),
                   "note": "rocprofv3 PMC, separate passes, KiB->bytes; FETCH_SIZE not x2-corrected"},
                  open(os.path.join(ROOT, "profiles", "traffic.json"), "w"), indent=1)
    kf, kw = c.get(("k_match", "FETCH_SIZE")), c.get(("k_match", "WRITE_SIZE"))
    if kf is not None and kw is not None:
        out.append(f"`k_match` HBM traffic: FETCH {kf * 1024 / 1e6:.1f} MB + WRITE {kw * 1024 / 1e6:.1f} MB per launch.")
    path = os.path.join(ROOT, "profiles", f"{tag}.md")
    open(path, "w").write("\n".join(out) + "\n")
    print("\n".join(out))


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2] if len(sys.argv) > 2 else os.path.join(ROOT, "gpurun_out"))
