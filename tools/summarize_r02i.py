"""Summarise a tools/r02_prof.sh run (gpurun_out/<tag>/) into profiles/<tag>.md and refresh
profiles/traffic.json (PMC HBM bytes per launch of the roofline kernel, per workload; bench.py
reads the "<workload>:k_flow_plan_head_hbm_bytes_per_launch" keys).

gfx950 counter units (MI355X_MICROARCH.md, HBM / rocprofv3 section): FETCH_SIZE and WRITE_SIZE
are KiB per dispatch; FETCH_SIZE reads half the bytes of wide (16 B/lane) coalesced streams.
k_flow_plan_head reads its records through the scalar cache and writes its touch log with
per-lane dword stores (neither a calibrated width), so the raw figure is the estimate.

usage: python tools/summarize_r02i.py <tag> [gpurun_out dir]"""
import csv
import glob
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
K = "k_flow_plan_head"


def rows(pattern):
    files = sorted(glob.glob(pattern, recursive=True))
    if not files:
        return []
    with open(files[0]) as f:
        return list(csv.DictReader(f))


def short(name):
    return name.split("(")[0].replace("gome::", "").replace("void ", "")


def last_json(path):
    out = None
    if os.path.exists(path):
        for line in open(path):
            if line.startswith("{"):
                out = json.loads(line)
    return out


def pmc_avg(d, counter):
    v = [float(r["Counter_Value"]) for r in rows(os.path.join(d, "**", "*counter_collection.csv"))
         if short(r["Kernel_Name"]) == K and r["Counter_Name"] == counter]
    return sum(v) / len(v) if v else None


def union_len(iv):
    tot, cur_s, cur_e = 0, None, None
    for s, e in sorted(iv):
        if cur_e is None or s > cur_e:
            if cur_e is not None:
                tot += cur_e - cur_s
            cur_s, cur_e = s, e
        else:
            cur_e = max(cur_e, e)
    if cur_e is not None:
        tot += cur_e - cur_s
    return tot


def overlap(iv, kern):
    """Time of the intervals iv covered by the union of kern."""
    kern = sorted(kern)
    merged = []
    for s, e in kern:
        if merged and s <= merged[-1][1]:
            merged[-1][1] = max(merged[-1][1], e)
        else:
            merged.append([s, e])
    tot = 0
    for s, e in iv:
        for ks, ke in merged:
            if ke <= s:
                continue
            if ks >= e:
                break
            tot += min(e, ke) - max(s, ks)
    return tot


def main(tag, base):
    src = os.path.join(base, tag)
    tj_path = os.path.join(ROOT, "profiles", "traffic.json")
    tj = json.load(open(tj_path)) if os.path.exists(tj_path) else {}
    out = [f"# rocprofv3 summary `{tag}` (round 2, final tree)", "",
           f"Command: `bash tools/r02_prof.sh {tag}` on one MI355X. Per workload: `rocprofv3 --kernel-trace --stats -- "
           "python3 bench.py --workload W --steps 5 --warmup 2 --e2e-steps 0 --no-cpu-baseline`, then separate "
           "`--pmc FETCH_SIZE` and `--pmc WRITE_SIZE` passes of the same command restricted to `k_flow_plan_head`. "
           "Then `rocprofv3 --kernel-trace --memory-copy-trace --stats` of the pipelined e2e leg (config 3).", ""]
    for w in ("config3", "config4", "config5"):
        d = os.path.join(src, w)
        st = rows(os.path.join(d, "trace", "**", "*kernel_stats.csv"))
        tb = last_json(os.path.join(d, "trace_bench.json"))
        if not st:
            continue
        out += [f"## {w}", ""]
        if tb:
            out += [f"Bench line of the traced run: value {tb['value'] / 1e6:.1f}M orders/s, {tb['ms_per_step']} ms "
                    f"per step, hottest book {tb['hot_book']['ns_per_order']} ns/order.", ""]
        out += ["| kernel | calls | avg µs | % |", "|---|---|---|---|"]
        for r in st[:12]:
            out.append(f"| {short(r['Name'])} | {r['Calls']} | {float(r['AverageNs']) / 1e3:.1f} | "
                       f"{float(r['Percentage']):.2f} |")
        km = next((r for r in st if short(r["Name"]) == K), None)
        if km:
            out += ["", f"`{K}`: {float(km['AverageNs']) / 1e6:.3f} ms rocprof average (all launches)"
                    + (f" vs {tb['roofline']['kernel_ms']} ms from bench.py's HIP events on its stream "
                       f"(timed launches); algorithmic bytes per launch {tb['roofline']['alg_bytes_per_launch']}."
                       if tb else ".")]
        fetch, write = pmc_avg(os.path.join(d, "FETCH_SIZE"), "FETCH_SIZE"), pmc_avg(os.path.join(d, "WRITE_SIZE"), "WRITE_SIZE")
        if fetch is not None and write is not None:
            fb, wb = fetch * 1024, write * 1024
            line = (f"PMC: FETCH {fb / 1e6:.2f} MB (x2 wide-stream correction {2 * fb / 1e6:.2f} MB) + WRITE "
                    f"{wb / 1e6:.2f} MB = {(fb + wb) / 1e6:.2f} MB per launch")
            if tb:
                line += f" vs {tb['roofline']['alg_bytes_per_launch'] / 1e6:.2f} MB algorithmic (8 B per order + 16 B per touch)."
            out += ["", line]
            tj[f"{w}:{K}_hbm_bytes_per_launch"] = int(fb + wb)
            if w == "config3":
                tj.update({"tag": tag, "kernel": K, f"{K}_hbm_bytes_per_launch": int(fb + wb),
                           "fetch_bytes": int(fb), "write_bytes": int(wb)})
        out.append("")
    # e2e overlap
    kt = rows(os.path.join(src, "e2e", "**", "*kernel_trace.csv"))
    mc = rows(os.path.join(src, "e2e", "**", "*memory_copy_trace.csv"))
    eb = last_json(os.path.join(src, "e2e_bench.json"))
    if kt and mc:
        kern = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"])) for r in kt]
        big = [r for r in mc if int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) > 200_000]
        out += ["## e2e leg (config 3): copy / compute overlap", ""]
        by = {}
        for r in big:
            dname = r.get("Direction", r.get("Operation", "copy"))
            by.setdefault(dname, []).append((int(r["Start_Timestamp"]), int(r["End_Timestamp"])))
        out += ["Copies longer than 0.2 ms of the whole traced run (its non-pipelined device-resident steps included), "
                "and how much of their time kernels were running beside them:", "",
                "| direction | copies | total ms | ms overlapped by kernels | overlap |", "|---|---|---|---|---|"]
        for dname, iv in sorted(by.items()):
            tot = sum(e - s for s, e in iv)
            ov = overlap(iv, kern)
            out.append(f"| {dname} | {len(iv)} | {tot / 1e6:.2f} | {ov / 1e6:.2f} | {ov / max(tot, 1):.0%} |")
        if eb and "e2e" in eb:
            out += ["", f"e2e line of the traced run: {eb['e2e']['value'] / 1e6:.1f}M orders/s vs device-resident "
                        f"{eb['value'] / 1e6:.1f}M."]
        out.append("")
    tj["note"] = "rocprofv3 PMC, separate passes, KiB->bytes; FETCH_SIZE not x2-corrected"
    json.dump(tj, open(tj_path, "w"), indent=1)
    path = os.path.join(ROOT, "profiles", f"{tag}.md")
    open(path, "w").write("\n".join(out) + "\n")
    print("\n".join(out))


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2] if len(sys.argv) > 2 else os.path.join(ROOT, "gpurun_out"))
