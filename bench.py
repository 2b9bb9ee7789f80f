"""bench.py — matched orders/sec of the MI355X batch matching engine (BASELINE.json metric).

Workload (BASELINE.json configs[2], the config the metric is quoted on): 100k symbols,
symbol rank ~ Zipf(s=1.0), doorder.go price/volume distribution (2-dp prices in
(0, 1], 2-dp volumes), ADD-only, synthetic and seeded.  One step = one batch of
`--batch` orders per GPU applied end to end on the device (validate + radix sort by
symbol + admission + match_books + event compaction), records already resident in HBM.

Multi-GPU (one process per GPU, torchrun): symbols are sharded round-robin over Zipf
rank (rank r owns symbols whose Zipf rank % N == r), so every rank processes its own
symbols' orders with no data-path collective (weak scaling: the global stream has
N * batch orders per step).  The only collective is a per-step all_gather of a 32-word
per-GPU summary for the publisher (RCCL over xGMI).

Prints ONE JSON line on rank 0.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

from gome_amd import workload as wl  # noqa: E402

METRIC = "matched orders/sec (node) at 100k symbols; p99 batch match latency; HBM GB/s"
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md, chip-level parameters)


def algorithmic_bytes(st: dict) -> int:
    """Bytes match_books must move per launch:
    32 B per input record read, 64 B per event written, 24 B node write + 16 B index
    entry per resting order, 24 B node read per maker filled, 40 B (index probe + node)
    per cancel hit.  Level aggregates are not counted."""
    return (32 * st["n_orders"] + 64 * st["n_events"] + 40 * st["n_rests"]
            + 24 * st["n_fills"] + 40 * st["n_cancels"])


def hot_algorithmic_bytes(st: dict) -> int:
    """The same per-unit figures restricted to the work done inside k_match_hot."""
    ev = st["n_hot_fills"] + st["n_hot_cancels"]
    return (32 * st["n_hot_orders"] + 64 * ev + 40 * st["n_hot_rests"]
            + 24 * st["n_hot_fills"] + 40 * st["n_hot_cancels"])


def plan_algorithmic_bytes(st: dict) -> int:
    """Bytes k_flow_plan_head must move per launch: one 8-B packed record read
    per order of the head's flow books, one 16-B touch written per level an order visits."""
    return 8 * st["n_flow_head_orders"] + 16 * st["n_flow_head_touches"]


def shard_stream(n_symbols, zipf_s, rank, world, seed):
    """Generator of this rank's share of the global Zipf stream (conditional sampling
    over the ranks this GPU owns; equal in law to filtering the global stream)."""
    z = wl.ZipfSymbols(n_symbols, zipf_s)
    p = np.diff(np.concatenate([[0.0], z.cdf]))
    own = np.arange(rank, n_symbols, world)
    share = float(p[own].sum())
    cdf = np.cumsum(p[own] / share)
    cdf[-1] = 1.0
    rng = np.random.default_rng(seed + 1000 * rank)
    ids = z.rank_to_id[own]
    state = {"oid": 1}

    def batch(n):
        rec = np.zeros(n, wl.ORDER_DTYPE)
        rec["symbol_id"] = ids[np.searchsorted(cdf, rng.random(n), side="right")]
        rec["price_fx"] = wl.doorder_prices(rng, n)
        rec["volume_fx"] = wl.doorder_volumes(rng, n)
        rec["side"] = rng.integers(0, 2, n, dtype=np.uint8)
        rec["action"] = wl.ADD
        rec["uuid_id"] = 2
        rec["oid_id"] = np.arange(state["oid"], state["oid"] + n, dtype=np.uint64).astype(np.uint32)
        state["oid"] += n
        return rec

    return batch, share, float(p[0])


def combine_ranks(orders, fills, events, elapsed, lat, device):
    """Whole-job totals over ranks: sums of work, MAX of the timed region and of each
    step's latency (the slowest rank defines the job).  Works on any initialised process
    group (RCCL on the GPU box, gloo in tests/test_multirank.py)."""
    import torch
    import torch.distributed as dist
    t = torch.tensor([orders, fills, events], dtype=torch.float64, device=device)
    dist.all_reduce(t)
    e = torch.tensor([elapsed], dtype=torch.float64, device=device)
    dist.all_reduce(e, op=dist.ReduceOp.MAX)
    lt = torch.tensor(lat, dtype=torch.float64, device=device)
    dist.all_reduce(lt, op=dist.ReduceOp.MAX)
    o, f, ev = (float(x) for x in t.tolist())
    return o, f, ev, float(e.item()), lt.tolist()


def gather_summary(st, summary, gathered):
    """Per-GPU trade/depth summary to every rank (the publisher feed)."""
    import torch.distributed as dist
    summary.zero_()
    summary[0] = st["n_orders"]; summary[1] = st["n_fills"]; summary[2] = st["n_events"]
    summary[3] = st["n_resting"]; summary[4] = st["max_segment"]
    dist.all_gather_into_tensor(gathered, summary)
    return gathered


def cpu_baseline(batches, n_symbols, budget_s):
    """C oracle (oracle/gome_oracle.c, 1 thread) on the first batches of this rank's stream."""
    from oracle.pyoracle import Oracle
    orc = Oracle(n_symbols)
    done, t_cpu = 0, 0.0
    for b in batches:
        t = time.perf_counter()
        orc.submit(b)
        t_cpu += time.perf_counter() - t
        done += len(b)
        if t_cpu >= budget_s:
            break
    return done / t_cpu, done, t_cpu


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--batch", type=int, default=1 << 22, help="orders per GPU per step")
    ap.add_argument("--symbols", type=int, default=100000)
    ap.add_argument("--zipf", type=float, default=1.0)
    ap.add_argument("--seed", type=int, default=42)
    ap.add_argument("--cpu-budget", type=float, default=15.0, help="seconds of CPU-baseline work")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--traffic-json", default=os.path.join(ROOT, "profiles", "traffic.json"),
                    help="PMC-measured HBM bytes per match_books launch (optional)")
    args = ap.parse_args()

    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        if world == 1 and args.gpus > 1:
            print(f"--gpus {args.gpus} needs torchrun with {args.gpus} processes", file=sys.stderr)
            sys.exit(2)
    torch.cuda.set_device(local)
    if world > 1:
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))

    from gome_amd.abi import Engine

    steps, warm = args.steps, args.warmup
    gen, share, top_share = shard_stream(args.symbols, args.zipf, rank, world, args.seed)
    per_rank = int(round(args.batch * world * share))
    host_batches = [gen(per_rank) for _ in range(warm + steps)]
    dev_batches = [torch.from_numpy(b.view(np.uint8)).cuda() for b in host_batches]
    torch.cuda.synchronize()

    total_orders = per_rank * (warm + steps)
    eng = Engine(max_symbols=args.symbols, max_batch=per_rank,
                 max_nodes=max(1 << 20, int(total_orders * 0.3)),
                 max_levels=max(1 << 22, 256 * args.symbols), device=local)

    summary = torch.zeros(32, dtype=torch.int64, device="cuda")
    gathered = torch.zeros(32 * world, dtype=torch.int64, device="cuda")

    def step(i):
        b = dev_batches[i]
        eng.submit_device(b.data_ptr(), per_rank, seq_base=i * per_rank)
        st = eng.stats()
        if world > 1:  # per-GPU trade/depth summary to the publisher (RCCL all_gather)
            gather_summary(st, summary, gathered)
        return st

    for i in range(warm):
        step(i)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    lat, sts = [], []
    t0 = time.perf_counter()
    for i in range(warm, warm + steps):
        ts = time.perf_counter()
        sts.append(step(i))
        lat.append((time.perf_counter() - ts) * 1e3)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0

    orders = sum(s["n_orders"] for s in sts)
    fills = sum(s["n_fills"] for s in sts)
    events = sum(s["n_events"] for s in sts)
    ms_match = sum(s["ms_match"] for s in sts) / steps
    ms_total = sum(s["ms_total"] for s in sts) / steps
    balg = sum(algorithmic_bytes(s) for s in sts) / steps
    flow = sum(s["n_flow_books"] for s in sts) > 0
    if flow:  # the flow path's serial plan is the dominant kernel
        kname = "k_flow_plan_head (serial aggregate plan of the hottest book)"
        ms_hot = sum(s["ms_flow_plan"] for s in sts) / steps
        bhot = sum(plan_algorithmic_bytes(s) for s in sts) / steps
    else:
        kname = "k_match_hot (match_books, hot books)"
        ms_hot = sum(s["ms_hot"] for s in sts) / steps
        bhot = sum(hot_algorithmic_bytes(s) for s in sts) / steps
    max_seg = max(s["max_segment"] for s in sts)
    if world > 1:
        orders, fills, events, elapsed, lat = combine_ranks(orders, fills, events, elapsed, lat, "cuda")

    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        v, done, t_cpu = cpu_baseline(host_batches, args.symbols, args.cpu_budget)
        cpu = {"value": round(v, 1), "unit": "orders/s", "cores": 1, "kind": "port",
               "sample": f"oracle/gome_oracle.c (1 thread) on the first {done} orders "
                         f"({done // per_rank} batches) of the same rank-0 stream, {t_cpu:.1f} s"}

    traffic = None
    if os.path.exists(args.traffic_json):
        try:
            tj = json.load(open(args.traffic_json))
            traffic = tj.get("k_flow_plan_head_hbm_bytes_per_launch" if flow else "k_match_hot_hbm_bytes_per_launch")
        except (OSError, ValueError):
            traffic = None

    if rank == 0:
        achieved = bhot / (ms_hot * 1e-3) / 1e9 if ms_hot > 0 else 0.0
        lat_sorted = sorted(lat)
        p99 = lat_sorted[min(len(lat_sorted) - 1, int(np.ceil(0.99 * len(lat_sorted))) - 1)]
        p50 = lat_sorted[len(lat_sorted) // 2]
        out = {
            "metric": METRIC,
            "value": round(orders / elapsed, 1),
            "unit": "orders/s",
            "n_gpus": world,
            "steps": steps,
            "warmup": warm,
            "ms_per_step": round(elapsed / steps * 1e3, 3),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "int64",
            "data": "synthetic (seeded doorder.go distribution, Zipf symbols)",
            "config": {"workload": f"config3: {args.symbols} symbols, Zipf(s={args.zipf}) symbol rank, "
                                   "doorder 2-dp price/volume, ADD-only",
                       "symbols": args.symbols, "zipf_s": args.zipf,
                       "batch_per_gpu": per_rank, "global_batch": per_rank * world,
                       "parallelism": f"symbol-sharded x{world} (no data-path collective)"},
            "p50_batch_ms": round(p50, 3),
            "p99_batch_ms": round(p99, 3),
            "fills_per_s": round(fills / elapsed, 1),
            "events_per_s": round(events / elapsed, 1),
            "device_ms_per_batch": round(ms_total, 3),
            "match_books_ms": round(ms_match, 3),
            "hot_book": {"orders_per_batch": int(max_seg), "top_symbol_share": round(top_share, 5),
                         "ns_per_order": round(ms_hot * 1e6 / max(max_seg, 1), 1)},
            "roofline": {"bound": "hbm", "achieved": round(achieved, 3), "peak": HBM_PEAK_GBS,
                         "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 6),
                         "traffic": traffic, "kernel": kname,
                         "kernel_ms": round(ms_hot, 3), "alg_bytes_per_launch": int(bhot),
                         "match_phase_alg_bytes": int(balg)},
            "cpu_baseline": cpu,
        }
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.destroy_process_group()
    eng.close()


if __name__ == "__main__":
    main()
