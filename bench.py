"""bench.py — matched orders/sec of the MI355X batch matching engine (BASELINE.json metric).

Workloads (BASELINE.json configs; `--workload`):
  config2: 1k symbols, uniform symbol choice, doorder distribution, ADD-only (no hot symbol:
          every book is a flow candidate of ~4k orders per 4 Mi batch).
  config3 (default, the config the metric is quoted on): 100k symbols, symbol rank ~
          Zipf(s=1.0), doorder.go price/volume distribution (2-dp prices in (0, 1], 2-dp
          volumes), ADD-only.
  config4: config 3's symbols with the cancel-heavy mix: 50% DELs (each re-sends a uniformly
          chosen earlier ADD no DEL targeted yet, delorder.go), 10% of ADDs aggressive (BUY @
          1.00 / SALE @ 0.01, volume k * 10.00, k ~ U{1..16}).
  config5: 1M symbols, Zipf(1.0), 4-dp price grid (deep books, up to 10k levels), 2-dp volumes.
  config5c: config 5's grid with config 4's 50% DELs and 10% aggressive ADDs (cancels on deep books).
All synthetic and seeded.  One step = one batch of `--batch` orders per GPU applied end to end
on the device (validate + radix sort by symbol + admission + match_books + event compaction),
records already resident in HBM: that is `value`.  `e2e` then runs the same workload from
host memory through the pipelined path (gome_submit_batch_async / gome_collect: H2D of batch
k+1 and D2H of batch k-1's events overlap batch k's matching) — SURVEY §8d's primary metric.

Multi-GPU (one process per GPU, torchrun): symbols are sharded round-robin over Zipf rank
(rank r owns symbols whose Zipf rank % N == r), so every rank processes its own symbols'
orders with no data-path collective (weak scaling: the global stream has N * batch orders per
step).  The only collective is a per-step all_gather of a 32-word per-GPU summary consumed by
the rank-0 publisher (gome_amd/publisher.py; RCCL over xGMI).

Prints ONE JSON line on rank 0.
"""
from __future__ import annotations

import argparse
import json
from contextlib import nullcontext
import os
import sys
import threading
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

from gome_amd import workload as wl  # noqa: E402
from gome_amd.publisher import SUMMARY_WORDS, SummaryPublisher, pack_summary  # noqa: E402

METRIC = "matched orders/sec (node) at 100k symbols; p99 batch match latency; HBM GB/s"
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md, chip-level parameters)

WORKLOADS = {
    "config2": dict(symbols=1000, zipf=0.0, decimals=2, del_frac=0.0, aggr=0.0,
                    desc="config2: {symbols} symbols, uniform symbol choice, doorder 2-dp price/volume, ADD-only"),
    "config3": dict(symbols=100000, zipf=1.0, decimals=2, del_frac=0.0, aggr=0.0,
                    desc="config3: {symbols} symbols, Zipf(s={zipf}) symbol rank, doorder 2-dp price/volume, ADD-only"),
    "config4": dict(symbols=100000, zipf=1.0, decimals=2, del_frac=0.5, aggr=0.1,
                    desc="config4: {symbols} symbols, Zipf(s={zipf}), 50% DEL of earlier ADDs (delorder), "
                         "10% aggressive ADDs (BUY@1.00 / SALE@0.01, k*10.00), doorder 2-dp"),
    "config5": dict(symbols=1000000, zipf=1.0, decimals=4, del_frac=0.0, aggr=0.0,
                    desc="config5: {symbols} symbols, Zipf(s={zipf}), 4-dp price grid (deep books), "
                         "2-dp volumes, ADD-only"),
    "config5c": dict(symbols=1000000, zipf=1.0, decimals=4, del_frac=0.5, aggr=0.1,
                     desc="config5c: config 5's {symbols} symbols and 4-dp grid (deep books) with config 4's "
                          "cancel-heavy mix: 50% DEL of earlier ADDs, 10% aggressive ADDs"),
}


def algorithmic_bytes(st: dict) -> int:
    """Bytes match_books must move per launch:
    32 B per input record read, 48 B per event written, 24 B node write + 16 B index
    entry per resting order, 24 B node read per maker filled, 40 B (index probe + node)
    per cancel hit.  Level aggregates are not counted."""
    return (32 * st["n_orders"] + 48 * st["n_events"] + 40 * st["n_rests"]
            + 24 * st["n_fills"] + 40 * st["n_cancels"])


def hot_algorithmic_bytes(st: dict) -> int:
    """The same per-unit figures restricted to the work done inside k_match_hot / the flow path."""
    ev = st["n_hot_fills"] + st["n_hot_cancels"]
    return (32 * st["n_hot_orders"] + 48 * ev + 40 * st["n_hot_rests"]
            + 24 * st["n_hot_fills"] + 40 * st["n_hot_cancels"])


def cold_algorithmic_bytes(st: dict) -> int:
    """The same per-unit figures for k_match (every book neither hot path applied)."""
    o = st["n_orders"] - st["n_hot_orders"]
    f = st["n_fills"] - st["n_hot_fills"]
    c = st["n_cancels"] - st["n_hot_cancels"]
    r = st["n_rests"] - st["n_hot_rests"]
    return 32 * o + 48 * (f + c) + 40 * r + 24 * f + 40 * c


def plan_algorithmic_bytes(st: dict) -> int:
    """Bytes k_flow_plan_head must move per launch: one 8-B packed record read
    per order of the head's flow books, one 16-B touch written per level an order visits."""
    return 8 * st["n_flow_head_orders"] + 16 * st["n_flow_head_touches"]


# The pipeline's phases that can be the batch's longest (gome_stats.ms_phase, gome_abi.h GOME_PH_*):
# the kernel each is named after and its algorithmic bytes per launch (SURVEY §8d per-unit
# figures over the phase's units; tail = the flow books outside the head).
def phase_candidates(st: dict) -> dict:
    from gome_amd.abi import PHASES
    ms = dict(zip(PHASES, st["ms_phase"]))
    n = st["n_orders"]
    to = st["n_flow_orders"] - st["n_flow_head_orders"]      # tail orders / touches / fills
    tt = st["n_flow_touches"] - st["n_flow_head_touches"]
    tf = st["n_flow_tail_fills"]
    tr = st["n_rests"] * to // max(n, 1)
    return {
        "k_flow_plan_tail": (ms["tail_plan"], 8 * to + 16 * tt, "serial plans of the tail's flow books"),
        "k_flow_write_events": (ms["tail_write"], 48 * tf + 36 * tt + 4 * to + 32 * tt + 40 * tr,
                                "tail: FIFO appends and level arrays beside the events (binary searches) "
                                "into the arena"),
        "k_flow_level": (ms["tail_level"], 64 * tt + 24 * tf, "tail: per-level reconstruction"),
        "k_flow_sort": (ms["tail_sort"], 32 * tt, "tail: touches sorted by level"),
        "k_flow_prep": (ms["tail_prep"], 40 * to, "tail: books' prep"),
        "k_radix_scatter": (ms["sort"], 68 * n, "radix sort by symbol + segments"),
        "k_adm": (ms["admission"], 48 * n, "admission (Q4) and duplicate oids (Q7)"),
        "k_prep": (ms["records"], 68 * n, "symbol-sorted records"),
        "k_publish": (ms["publish"], 96 * st["n_events"] + 8 * n,
                      "publish-order scan, arena event scatter and the hottest book's events"),
    }


def shard_stream(n_symbols, zipf_s, rank, world, seed, price_decimals=2):
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
        rec["price_fx"] = wl.doorder_prices(rng, n, price_decimals)
        rec["volume_fx"] = wl.doorder_volumes(rng, n)
        rec["side"] = rng.integers(0, 2, n, dtype=np.uint8)
        rec["action"] = wl.ADD
        rec["uuid_id"] = 2
        rec["oid_id"] = np.arange(state["oid"], state["oid"] + n, dtype=np.uint64).astype(np.uint32)
        state["oid"] += n
        return rec

    return batch, share, float(p[0])


def note(msg):
    """Progress on stderr (a long bench line must keep writing: GPU runners treat a silent run as hung)."""
    print(f"[bench {time.strftime('%H:%M:%S')}] {msg}", file=sys.stderr, flush=True)


def make_stream(workload, rank, world, seed):
    """(batch(n) -> records, owned share, top-symbol share) of this rank's stream."""
    W = WORKLOADS[workload]
    if workload == "config3":  # the numpy stream round 1's headline was measured on
        return shard_stream(W["symbols"], W["zipf"], rank, world, seed)
    ns = wl.NativeStream(W["symbols"], W["zipf"], seed=seed, price_decimals=W["decimals"],
                         del_frac=W["del_frac"], aggressive_frac=W["aggr"], rank=rank, world=world)
    return ns.batch, ns.owned_share, ns.top_share


def hot_symbols(workload, rank, world, k=8):
    """Symbol ids of this rank's k hottest books (its lowest owned Zipf ranks): the books whose
    top-of-book digests go into the publisher summary."""
    W = WORKLOADS[workload]
    own = np.arange(rank, W["symbols"], world)[:k]
    if not W["zipf"]:
        return own.astype(np.uint32)
    return wl.ZipfSymbols(W["symbols"], W["zipf"]).rank_to_id[own]


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


def rank_batch(batch, world, share, scaling="weak"):
    """Records of one rank per step.  weak: `batch` orders per GPU (the global stream holds world x
    batch, each rank its symbols' share of it); strong: `batch` orders per step in all, split over
    the ranks by their symbols' share."""
    return int(round(batch * (world if scaling == "weak" else 1) * share))


def hottest_book_orders(rec) -> int:
    """Orders of the batch's hottest book (its longest symbol segment): the serial plan's length."""
    return int(np.bincount(rec["symbol_id"]).max()) if len(rec) else 0


def per_rank_values(x, rank, world, device):
    """Every rank's value of x, in rank order, on every rank (one all_reduce of a one-hot vector)."""
    import torch
    import torch.distributed as dist
    t = torch.zeros(world, dtype=torch.float64, device=device)
    t[rank] = float(x)
    dist.all_reduce(t)
    return [round(float(v), 3) for v in t.tolist()]


def gather_summary(st, summary, gathered, rank=0, step=0, digests=None):
    """Per-GPU trade/depth summary to every rank (the publisher feed)."""
    import torch.distributed as dist
    pack_summary(st, rank, step, summary, digests)
    dist.all_gather_into_tensor(gathered, summary)
    return gathered


def cpu_baseline(batches, n_symbols, budget_s, threads=1):
    """C oracle (oracle/gome_oracle.c) on the first batches of this rank's stream: 1 thread for
    up to budget_s, then the same batches symbol-sharded over `threads` threads (one oracle per
    thread; books never interact; ctypes calls release the GIL)."""
    from oracle.pyoracle import Oracle
    orc = Oracle(n_symbols)
    done, t_cpu, used = 0, 0.0, 0
    for b in batches:
        t = time.perf_counter()
        orc.submit(b)
        t_cpu += time.perf_counter() - t
        done += len(b)
        used += 1
        if t_cpu >= budget_s:
            break
    one = (done / t_cpu, done, t_cpu, used)
    if threads <= 1:
        return one, None
    parts = [[b[(b["symbol_id"] % threads) == k] for b in batches[:used]] for k in range(threads)]
    orcs = [Oracle(n_symbols) for _ in range(threads)]

    def run(k):
        for p in parts[k]:
            orcs[k].submit(p)

    ths = [threading.Thread(target=run, args=(k,)) for k in range(threads)]
    t = time.perf_counter()
    for th in ths:
        th.start()
    for th in ths:
        th.join()
    wall = time.perf_counter() - t
    return one, (done / wall, done, wall, used)


def consumer_leg(workload, n_symbols, n_msgs, seed, batch=1 << 15, threads=8, render_threads=None, warm_batches=4):
    """The drop-in boundary's own rate: n_msgs doOrder messages (the
    OrderNode JSON bodies the gRPC side enqueues, main.go:39-52 / ordernode.go:9-36, admission markers
    set) of the same workload through BatchingConsumer.process_stream -- native Go-Unmarshal decode on
    `threads` threads, fixed-point conversion, interning, admission (gome_consume_order_nodes), two
    batches in flight on the engine (gome_submit_batch_async / gome_collect), gome_render_events_mt
    into MatchResult lines on the sink (rabbitmq.go:116-125, engine.go:154-194); then the same
    messages through process() as Python objects (round 5's leg) and the renderer alone over the
    same events at 1 and `threads` threads.  Both consumers first take `warm_batches` batches of the
    same stream, untimed (as the main leg's warmup steps): the first batches of a process pay one-time
    costs -- the engine's second stream set is made when the first batch no book dominated is
    collected (46 ms on config 2's third submit, tools/consumer_submit_probe.py), the pools' threads
    start, the scratch is faulted in -- which that pass's own rate (`cold_messages_per_s`) shows."""
    import ctypes as C
    from gome_amd.abi import Engine
    from gome_amd.consumer import BatchingConsumer, MatchSink, Names, PrePool, _order_node_json
    gen, _, _ = make_stream(workload, 0, 1, seed + 7)
    n_warm = warm_batches * batch
    rec = gen(n_warm + n_msgs).copy()
    msgs = [_order_node_json(dict(symbol="s%d" % r["symbol_id"], uuid=str(int(r["uuid_id"])),
                                  oid=str(int(r["oid_id"])), transaction=int(r["side"])),
                             int(r["action"]), float(r["price_fx"]), float(r["volume_fx"]), 8).encode()
            for r in rec]  # (AMQP delivers bytes)
    pre, sink, names = PrePool(), MatchSink(), Names()
    for r in rec:
        if r["action"] == wl.ADD:
            pre.set("s%d" % r["symbol_id"], str(int(r["uuid_id"])), str(int(r["oid_id"])))
    eng = Engine(max_symbols=n_symbols, max_batch=batch, max_nodes=2 * (n_warm + n_msgs) + (1 << 20),
                 max_levels=(1 << 22) + 2 * (n_warm + n_msgs))
    cons = BatchingConsumer(eng, pre, sink, names, max_batch=batch, threads=threads, render_threads=render_threads)
    # the deliveries as one buffer of bodies + offsets (how an AMQP client reads them off its socket;
    # PackedQueue), two batches in flight (process_stream: decode and H2D of batch k+1 beside the
    # device's batch k, each batch rendered as it is collected)
    from gome_amd.consumer import PackedQueue
    t = time.perf_counter()
    lines_warm = cons.process_stream(PackedQueue(msgs[:n_warm]).batches(batch)) if n_warm else 0
    wall_warm = time.perf_counter() - t
    for k in cons.phase_s:
        cons.phase_s[k] = 0.0
    cons.queue_steps_s = [0.0] * len(cons.queue_steps_s)
    packed = PackedQueue(msgs[n_warm:])
    t = time.perf_counter()
    lines = cons.process_stream(packed.batches(batch))
    wall = time.perf_counter() - t
    phases = {k: round(v * 1e3, 2) for k, v in cons.phase_s.items()}
    # the same messages as Python bytes objects through process(), one synchronous batch at a time
    # (round 5's leg), on a fresh engine and pre-pool with the same markers
    pre2, sink2, names2 = PrePool(), MatchSink(), Names()
    for r in rec:
        if r["action"] == wl.ADD:
            pre2.set("s%d" % r["symbol_id"], str(int(r["uuid_id"])), str(int(r["oid_id"])))
    eng2 = Engine(max_symbols=n_symbols, max_batch=batch, max_nodes=2 * (n_warm + n_msgs) + (1 << 20),
                  max_levels=(1 << 22) + 2 * (n_warm + n_msgs))
    cons2 = BatchingConsumer(eng2, pre2, sink2, names2, max_batch=batch, threads=threads)
    evs, recs, bases = [], [], []
    orig_render = cons2.render_block

    def keep(ev, rc, base):  # (the events of each batch, for the render-only pass below)
        evs.append(ev.copy())
        recs.append(rc.copy())
        bases.append(base)
        return orig_render(ev, rc, base)
    lines2 = 0
    for k in range(0, n_warm, batch):
        lines2 += cons2.process(msgs[k:k + batch])
    cons2.render_block = keep
    t2 = time.perf_counter()
    for k in range(n_warm, n_warm + n_msgs, batch):
        lines2 += cons2.process(msgs[k:k + batch])
    wall2 = time.perf_counter() - t2
    same = lines2 == lines + lines_warm and sink2.q == sink.q
    eng2.close()
    lib = cons.lib
    N = names2
    nev = sum(len(e) for e in evs)
    out = {"messages": n_msgs, "batch": batch, "messages_per_s": round(n_msgs / wall, 1),
           "matchresults_per_s": round(lines / wall, 1), "matchresults": lines, "threads": threads,
           "warm_messages": n_warm, "cold_messages_per_s": round(n_warm / wall_warm, 1) if n_warm else None,
           "render_threads": cons.render_threads,
           "path": "OrderNode JSON deliveries (one buffer + offsets) -> BatchingConsumer.process_stream "
                   "(gome_consume_order_nodes: decode, convert, intern, admit into page-locked records; "
                   "gome_submit_batch_async, two batches in flight; gome_collect; gome_render_events_names "
                   "on a helper thread, beside the next batch's decode, straight into the sink's block) -> "
                   "MatchResult lines on the sink; host_ms.native_*: the consume call's own split",
           "host_ms": phases,
           "queue_steps_ms": [round(v * 1e3, 2) for v in cons.queue_steps_s],
           "list_messages_per_s": round(n_msgs / wall2, 1),
           "list_path": "the same messages as Python bytes objects through BatchingConsumer.process, one "
                        "synchronous batch at a time (packing included); sink bytes identical: " + str(same),
           "render_events_per_s": {}}
    cap = max(1 << 20, 1400 * max((len(e) for e in evs), default=0))
    rbuf = np.empty(cap, np.uint8)
    rbuf[::4096] = 0  # (its pages touched once, outside the timing)
    for th in (1, threads):
        nbytes = 0
        t = time.perf_counter()
        for ev, rc, base in zip(evs, recs, bases):
            k = lib.gome_render_events_mt(ev.ctypes.data, len(ev), rc.ctypes.data, len(rc), base, 8,
                                          N.table("sym"), N.count("sym"), N.table("uuid"), N.count("uuid"),
                                          N.table("oid"), N.count("oid"), N.tx_array().ctypes.data, th,
                                          rbuf.ctypes.data, cap)
            assert k >= 0
            nbytes += k
        dt = time.perf_counter() - t
        out["render_events_per_s"][str(th)] = round(nev / dt, 1)
        out["render_MB_per_s_" + str(th)] = round(nbytes / dt / 1e6, 1)
    eng.close()
    return out


def pcie_peak(nbytes=256 << 20, reps=3):
    """Measured PCIe copy rates of this GPU (page-locked host memory, one direction at a time
    and both at once on two streams), GB/s: the bound the e2e leg is compared with."""
    import torch
    h = torch.empty(nbytes, dtype=torch.uint8).pin_memory()
    h2 = torch.empty(nbytes, dtype=torch.uint8).pin_memory()
    d = torch.empty(nbytes, dtype=torch.uint8, device="cuda")
    d2 = torch.empty(nbytes, dtype=torch.uint8, device="cuda")
    s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()

    def timed(fn):
        best = 1e9
        for _ in range(reps):
            torch.cuda.synchronize()
            t = time.perf_counter()
            fn()
            torch.cuda.synchronize()
            best = min(best, time.perf_counter() - t)
        return best

    def both():
        with torch.cuda.stream(s1):
            d.copy_(h, non_blocking=True)
        with torch.cuda.stream(s2):
            h2.copy_(d2, non_blocking=True)
    th = timed(lambda: d.copy_(h, non_blocking=True))
    td = timed(lambda: h2.copy_(d2, non_blocking=True))
    tb = timed(both)
    return {"h2d_GBps": round(nbytes / th / 1e9, 2), "d2h_GBps": round(nbytes / td / 1e9, 2),
            "duplex_GBps_each": round(nbytes / tb / 1e9, 2)}


def pctl(xs, q):
    s = sorted(xs)
    return s[min(len(s) - 1, max(0, int(np.ceil(q * len(s))) - 1))]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--batch", type=int, default=1 << 22, help="orders per GPU per step")
    ap.add_argument("--workload", choices=sorted(WORKLOADS), default="config3")
    ap.add_argument("--seed", type=int, default=42)
    ap.add_argument("--e2e-depth", type=int, default=3, help="host batches in flight in the e2e leg (<= GOME_MAX_INFLIGHT)")
    ap.add_argument("--e2e-steps", type=int, default=-1,
                    help="timed steps of the host-to-host pipelined path (-1: = --steps, 0: off)")
    ap.add_argument("--cpu-budget", type=float, default=15.0, help="seconds of CPU-baseline work")
    ap.add_argument("--cpu-threads", type=int, default=8, help="threads of the sharded CPU baseline")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--backend", choices=("nccl", "gloo"), default="nccl",
                    help="process-group backend (nccl = RCCL over xGMI; gloo: CPU collectives, for tests)")
    ap.add_argument("--same-device", action="store_true",
                    help="every rank on device 0 (rehearsing the N-rank path on a one-GPU box)")
    ap.add_argument("--force-pg", action="store_true",
                    help="initialise the process group and run the summary gather, the publisher and the "
                         "digest check at N = 1 too (exercises the RCCL path on a one-GPU box)")
    ap.add_argument("--inject-quirks", choices=("none", "heal", "stuck", "q2heal", "q2stuck", "zero", "zeroheal", "zerodel"), default="none",
                    help="rewrite records of the hottest book in the first timed batch into wrong-side "
                         "cancels (Q2) of a bid level and a zero-volume ADD (Q6), or (zero) zero-volume "
                         "ADDs only (workload.inject_quirks); "
                         "the line's quirk_batch reports that batch's device time beside its neighbours'")
    ap.add_argument("--consumer-render-threads", type=int, default=0,
                    help="the consumer leg's render threads (0: as many as its 8 decode threads)")
    ap.add_argument("--consumer-msgs", type=int, default=1 << 18,
                    help="JSON OrderNode messages of the consumer leg, timed (0: off)")
    ap.add_argument("--consumer-warm-batches", type=int, default=4,
                    help="batches of the consumer leg's stream taken untimed first (one-time costs)")
    ap.add_argument("--pool-nodes", type=int, default=0, help="gome_config.max_nodes (0: sized from the run)")
    ap.add_argument("--pool-levels", type=int, default=0, help="gome_config.max_levels (0: sized from the run)")
    ap.add_argument("--scaling", choices=("weak", "strong"), default="strong",
                    help="strong (default): --batch orders per step in all, split over the GPUs by their "
                         "symbols' share, so rank 0's hottest book -- the batch's serial plan -- gets the same "
                         "orders per step at every N and the p99 batch latency stays that of one GPU; weak: "
                         "--batch orders per GPU per step (rank 0's hottest book N times longer; DESIGN 7)")
    ap.add_argument("--plan-cus", type=int, default=None,
                    help="gome_config.plan_cus (default: 0 = the engine's default, 8 plan CUs; -1: none)")
    ap.add_argument("--step-log", default="", help="write each timed step's engine counters (JSONL)")
    ap.add_argument("--sync", action="store_true",
                    help="one synchronous gome_submit_batch_device per step (default: two batches in "
                         "flight, gome_submit_batch_device_async + gome_collect_device)")
    ap.add_argument("--no-phase-pass", action="store_true",
                    help="skip the untimed replay with per-phase timing events (kernel_ms of the phases)")
    ap.add_argument("--traffic-json", default=os.path.join(ROOT, "profiles", "traffic.json"),
                    help="PMC-measured HBM bytes per launch of the dominant kernel (optional)")
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
    dev = 0 if args.same_device else local
    torch.cuda.set_device(dev)
    use_pg = world > 1 or args.force_pg  # (the summary gather, publisher and digest check)
    if use_pg:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        os.environ.setdefault("MASTER_PORT", "29517")
        os.environ.setdefault("RANK", "0")
        os.environ.setdefault("WORLD_SIZE", "1")
        if args.backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", dev))
        else:
            dist.init_process_group("gloo")
    cdev = "cuda" if args.backend == "nccl" else "cpu"  # where the collectives' tensors live

    from gome_amd.abi import GOME_MAX_INFLIGHT, Engine

    # gome_config.plan_cus: the engine's default (8 CUs reserved for the hottest book's plan) with or
    # without RCCL.  (Round 4 lost 5% per step with RCCL and plan CUs; round 5 found why: the CU-masked
    # streams (hipExtStreamCreateWithCUMask) are blocking streams, so the publisher's torch work on the
    # legacy default stream waited for every engine kernel enqueued before it, the next batch's
    # whole plan included.  The publisher now runs on a stream of its own; DESIGN 4.7, INTEGRATION.)
    plan_cus = args.plan_cus if args.plan_cus is not None else 0
    W = WORKLOADS[args.workload]
    n_symbols = W["symbols"]
    steps, warm = args.steps, args.warmup
    e2e_steps = steps if args.e2e_steps < 0 else args.e2e_steps
    # (every batch slot once, and once more: the first pass over a slot sizes its page-locked
    # event buffer, which two warm batches left for the third slot inside the timed region)
    e2e_warm = GOME_MAX_INFLIGHT + 1 if e2e_steps else 0
    gen, share, top_share = make_stream(args.workload, rank, world, args.seed)
    per_rank = rank_batch(args.batch, world, share, args.scaling)
    note(f"{args.workload}: generating {warm + steps} batches of {per_rank} records")
    host_batches = [gen(per_rank).copy() for _ in range(warm + steps)]
    injected = None
    dev_batches = [torch.from_numpy(b.view(np.uint8)).cuda() for b in host_batches]
    torch.cuda.synchronize()

    total_orders = per_rank * (warm + steps + e2e_warm + e2e_steps)
    # resting orders per order applied, with headroom (measured: config 3 ~0.16, config 5 0.23-0.24
    # over 13-60 steps, the cancel mixes far lower)
    keep = 0.3 if args.workload in ("config3", "config5") else 0.5
    # (+ GOME_MAX_INFLIGHT + 1 batches: the headroom a submit checks, in flight included, before
    # it is applied)
    head = (GOME_MAX_INFLIGHT + 1) * per_rank
    eng = Engine(max_symbols=n_symbols, max_batch=per_rank,
                 max_nodes=args.pool_nodes or max(1 << 20, int(total_orders * keep)) + head,
                 max_levels=args.pool_levels or max(1 << 22, (256 if n_symbols <= 100000 else 128) * n_symbols) + head,
                 device=dev, plan_cus=plan_cus)

    summary = torch.zeros(SUMMARY_WORDS, dtype=torch.int64, device=cdev)
    gathered = torch.zeros(SUMMARY_WORDS * world, dtype=torch.int64, device=cdev)
    # the publisher's torch work (summary packing, the all_gather, its readback) on a non-blocking
    # stream: never on the legacy default stream, which the engine's CU-masked (blocking) streams
    # synchronise with
    pub_stream = torch.cuda.Stream() if cdev == "cuda" else None
    pub = SummaryPublisher(world) if rank == 0 else None
    seq = [0]
    hot = hot_symbols(args.workload, rank, world)
    last_dg = [None]

    def publish(st, i, dg):
        if use_pg:  # per-GPU trade/depth summary to the publisher (RCCL all_gather)
            last_dg[0] = dg  # depth digests of this rank's hottest books after batch i
            with torch.cuda.stream(pub_stream) if pub_stream is not None else nullcontext():
                gather_summary(st, summary, gathered, rank, i, dg)
                if pub is not None:
                    pub.consume(gathered)

    def step(i):
        b = dev_batches[i]
        eng.submit_device(b.data_ptr(), per_rank, seq_base=seq[0])
        seq[0] += per_rank
        eng.release_device_events()  # events stay in HBM (a device-side consumer's input)
        st = eng.stats()
        publish(st, i, eng.top_of_book(hot) if use_pg else None)
        return st

    # pipelined steps (the default, any N): batch k+1 is enqueued before batch k is collected, so
    # the host's enqueue of one batch hides under the device's work on the other; the events stay
    # in HBM (a device-side consumer's input).  The publisher's depth digests of batch k are read
    # on the device behind batch k, before batch k+1 (gome_top_of_book_enqueue), and collected
    # after it: they never stall the pipeline.
    pipelined = not args.sync

    def run_steps(lo, hi, lat, sts, timed):
        tsub = {}

        def done(k, st):
            if lat is not None:
                lat.append((time.perf_counter() - tsub[k]) * 1e3)
                sts.append(st)
                if rank == 0 and timed:
                    note(f"step {k - lo + 1}/{hi - lo}: {lat[-1]:.1f} ms")
                if slog is not None and timed:  # (written as it goes: a failed run keeps its steps)
                    slog.write(json.dumps(dict(step=k - lo, wall_ms=round(lat[-1], 3), **st)) + "\n")
                    slog.flush()
            elif rank == 0:
                note(f"warmup step {k + 1}/{hi}")

        def collect(k):
            _, _, st = eng.collect_device()
            eng.release_device_events()
            publish(st, k, eng.top_of_book_collect() if use_pg else None)
            done(k, st)

        for k in range(lo, hi):
            tsub[k] = time.perf_counter()
            if not pipelined:
                done(k, step(k))
                continue
            if use_pg and k > lo:
                eng.top_of_book_enqueue(hot)  # (batch k-1's books, before batch k touches them)
            eng.submit_device_async(dev_batches[k].data_ptr(), per_rank, seq_base=seq[0])
            seq[0] += per_rank
            if k > lo:
                collect(k - 1)
        if pipelined and hi > lo:
            if use_pg:
                eng.top_of_book_enqueue(hot)
            collect(hi - 1)

    slog = None
    run_steps(0, warm, None, None, False)
    torch.cuda.synchronize()
    if args.inject_quirks != "none":
        # the FIRST TIMED batch's records of the hottest book rewritten from the engine's own
        # snapshot of that book after the warm-up (workload.inject_quirks), so the batch that
        # carries the quirks is timed; the line reports its own device time beside its neighbours'
        hs = int(hot[0])
        injected = wl.inject_quirks(host_batches[warm], hs, eng.levels(hs), lambda p: eng.fifo(hs, p),
                                    args.inject_quirks)
        dev_batches[warm].copy_(torch.from_numpy(host_batches[warm].view(np.uint8)))
        torch.cuda.synchronize()
        note(f"injected into batch {warm} (the first timed one): {injected['q2_cancels']} wrong-side cancels"
             + ("" if injected["q6_oid"] is None else f", {len(injected['records']) - injected['q2_cancels']} "
                "zero-volume ADDs"))
    if use_pg:
        dist.barrier()
    if pub is not None:
        pub = SummaryPublisher(world)  # the timed steps only
    lat, sts = [], []
    slog = open(args.step_log, "w") if args.step_log and rank == 0 else None
    t0 = time.perf_counter()
    run_steps(warm, warm + steps, lat, sts, True)
    torch.cuda.synchronize()
    if use_pg:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    if slog is not None:
        slog.close()

    dev_lat = [float(s["ms_total"]) for s in sts]
    p99_ranks = [round(pctl(dev_lat, 0.99), 3)]
    if use_pg:  # (each rank's own p99, then the slowest rank's device time per step)
        p99_ranks = per_rank_values(p99_ranks[0], rank, world, cdev)
        dev_lat = combine_ranks(0.0, 0.0, 0.0, 0.0, dev_lat, cdev)[4]
    orders = sum(s["n_orders"] for s in sts)
    fills = sum(s["n_fills"] for s in sts)
    events = sum(s["n_events"] for s in sts)
    cancels = sum(s["n_cancels"] for s in sts)
    ms_match = sum(s["ms_match"] for s in sts) / steps
    ms_total = sum(s["ms_total"] for s in sts) / steps
    balg = sum(algorithmic_bytes(s) for s in sts) / steps
    # the dominant kernel: the longest of the hottest book's plan, the legacy hot kernel and
    # the cold kernel (they run concurrently; the longest bounds the batch)
    # (the hottest book's plan: k_flow_plan_early when every timed batch planned it early, right
    # after the batch before's plan, match_early.h; k_flow_plan_head then launches and returns)
    plan_key = "k_flow_plan_early" if sum(int(s.get("n_early", 0)) for s in sts) == steps else "k_flow_plan_head"
    cands = {
        plan_key: (sum(s["ms_flow_plan"] for s in sts) / steps,
                             sum(plan_algorithmic_bytes(s) for s in sts) / steps,
                             "serial aggregate plan of the hottest book"),
        "k_match_hot": (sum(s["ms_hot"] for s in sts) / steps,
                        sum(hot_algorithmic_bytes(s) for s in sts) / steps,
                        "match_books, legacy hot books"),
        "k_match": (sum(s["ms_cold"] for s in sts) / steps,
                    sum(cold_algorithmic_bytes(s) for s in sts) / steps,
                    "match_books, cold books"),
    }
    if sum(s["n_flow_books"] for s in sts) == 0:
        cands.pop(plan_key)
    max_seg = max(s["max_segment"] for s in sts)
    # the hottest book's orders per step on each rank: the serial plan that bounds the rank's batch
    # (flat in N under strong scaling, N x under weak)
    hot_ranks = per_rank_values(max_seg, rank, world, cdev) if use_pg else [int(max_seg)]
    digest_check = None
    if use_pg:
        g_orders, g_fills, g_events, elapsed, lat = combine_ranks(orders, fills, events, elapsed, lat, cdev)
        # every rank checks the digests it published last against its books' snapshots
        # (gome_snapshot_levels); the publisher gets the mismatch count
        from gome_amd.publisher import digests_from_levels
        bad = 0
        for d in last_dg[0]:
            want = digests_from_levels(eng.levels(int(d["symbol_id"])))
            bad += int(any(int(d[k]) != v for k, v in want.items()))
        t = torch.tensor([bad, len(last_dg[0])], dtype=torch.int64, device=cdev)
        dist.all_reduce(t)
        digest_check = {"checked": int(t[1].item()), "mismatches": int(t[0].item())}
    else:
        g_orders, g_fills, g_events = orders, fills, events

    # ---- end to end from host memory (pipelined submit / collect)
    e2e = None
    if e2e_steps:
        bufs = [eng.host_buffer(per_rank) for _ in range(e2e_warm + e2e_steps)]
        for b in bufs:
            b[:] = gen(per_rank)
        done_ev = [0]

        # batches in flight on the host path (--e2e-depth)
        depth = max(1, min(args.e2e_depth, GOME_MAX_INFLIGHT))

        host_ms = {"submit": 0.0, "collect": 0.0}  # host time inside the two calls (timed steps)
        tdone = []  # host time of each collect's return (the steady-state interval: their median gap)
        edev = []   # each collected batch's device time (Status timing: first kernel to last)

        def run_pipe(lo, hi, lats):
            tsub = {}

            def coll(j):
                tc = time.perf_counter()
                ev, st = eng.collect(copy=False)
                host_ms["collect"] += (time.perf_counter() - tc) * 1e3
                tdone.append(time.perf_counter())
                edev.append(float(st["ms_total"]))
                done_ev[0] += len(ev)
                lats.append((time.perf_counter() - tsub[j]) * 1e3)
                if rank == 0:
                    note(f"e2e batch {j}: {lats[-1]:.1f} ms")
            for k in range(lo, hi):
                tsub[k] = time.perf_counter()
                eng.submit_async(bufs[k], seq_base=seq[0])
                host_ms["submit"] += (time.perf_counter() - tsub[k]) * 1e3
                seq[0] += per_rank
                if k - lo >= depth - 1:
                    coll(k - depth + 1)
            for j in range(max(lo, hi - depth + 1), hi):
                coll(j)

        run_pipe(0, e2e_warm, [])
        torch.cuda.synchronize()
        if use_pg:
            dist.barrier()
        elat = []
        done_ev[0] = 0
        host_ms["submit"] = host_ms["collect"] = 0.0
        tdone.clear()
        edev.clear()
        t1 = time.perf_counter()
        run_pipe(e2e_warm, e2e_warm + e2e_steps, elat)
        torch.cuda.synchronize()
        if use_pg:
            dist.barrier()
        e_el = time.perf_counter() - t1
        e_orders, e_events = per_rank * e2e_steps, done_ev[0]
        if use_pg:
            e_orders, _, e_events, e_el, elat = combine_ranks(e_orders, 0.0, e_events, e_el, elat, cdev)
        pk = pcie_peak() if rank == 0 else None
        in_b, out_b = 32 * per_rank, 48 * e_events / e2e_steps / max(world, 1)
        e2e = {"value": round(e_orders / e_el, 1), "unit": "orders/s", "steps": e2e_steps,
               "pcie_peak": pk,
               # the copies' time per step on this rank at the measured one-way rates: H2D and D2H
               # overlapped (PCIe is full duplex: the slower direction bounds the step) or serialised
               # (one after the other).  overlapped <= serial by construction; the measured rate with
               # both directions at once (pcie_peak.duplex_GBps_each) is reported beside them
               "pcie_bound_ms": None if pk is None else {
                   "overlapped": round(max(in_b / (pk["h2d_GBps"] * 1e9), out_b / (pk["d2h_GBps"] * 1e9)) * 1e3, 3),
                   "serial": round((in_b / (pk["h2d_GBps"] * 1e9) + out_b / (pk["d2h_GBps"] * 1e9)) * 1e3, 3),
                   "duplex_measured": round(max(in_b, out_b) / (pk["duplex_GBps_each"] * 1e9) * 1e3, 3)},
               "ms_per_step": round(e_el / e2e_steps * 1e3, 3),
               "host_ms_per_step": {k: round(v / e2e_steps, 3) for k, v in host_ms.items()},
               # the median gap between two batches' collects: the pipeline's steady-state step,
               # without the fill (the first H2D) and drain (the last D2H) that a K-step job adds
               "steady_ms_per_step": round(float(np.median(np.diff(tdone))) * 1e3, 3) if len(tdone) > 2 else None,
               "device_ms_per_batch_median": round(float(np.median(edev)), 3) if edev else None,
               "collect_gaps_ms": [round(x * 1e3, 2) for x in np.diff(tdone)],
               "p50_batch_ms": round(pctl(elat, 0.5), 3), "p99_batch_ms": round(pctl(elat, 0.99), 3),
               "events_per_s": round(e_events / e_el, 1),
               "pcie_bytes_per_step": int(32 * per_rank * world + 48 * e_events / e2e_steps),
               "path": "host records -> gome_submit_batch_async (H2D on a copy stream) -> device "
                       "pipeline -> gome_collect (events D2H into page-locked memory); batch k+1's "
                       "H2D and batch k-1's D2H overlap batch k"}

    # ---- the other phases of the pipeline (the tail's chain, the sort, admission, publishing):
    # with no hot symbol (config 2) one of them is the longest.  Their device times need ~24
    # timing-event records per batch (GOME_FLAG_PHASES, 0.12 ms of config 2's batch), so they
    # come from an untimed replay of the same batches on a fresh engine, never from the timed
    # steps above; rank 0 only (no collective inside).
    phase_src = None
    if rank == 0 and not args.no_phase_pass:
        from gome_amd.abi import GOME_FLAG_PHASES
        note("phase pass (untimed replay with per-phase timing events)")
        cfg = dict(eng.cfg_kwargs)
        eng.close()
        eng = Engine(**dict(cfg, flags=cfg.get("flags", 0) | GOME_FLAG_PHASES))
        sq, per = 0, []
        for i in range(warm + steps):
            eng.submit_device(dev_batches[i].data_ptr(), per_rank, seq_base=sq)
            sq += per_rank
            eng.release_device_events()
            if i >= warm:
                per.append(phase_candidates(eng.stats()))
        for k in per[0]:
            cands[k] = (sum(p[k][0] for p in per) / steps, sum(p[k][1] for p in per) / steps, per[0][k][2])
        phase_src = (f"k_flow_plan_head / k_match_hot / k_match: the timed steps; the other phases: an "
                     f"untimed replay of the same {warm + steps} batches with GOME_FLAG_PHASES")
    kname = max(cands, key=lambda k: cands[k][0])
    ms_dom, bdom, kdesc = cands[kname]

    consumer = None
    if rank == 0 and world == 1 and args.consumer_msgs > 0:
        note(f"consumer leg ({args.consumer_msgs} JSON messages)")
        consumer = consumer_leg(args.workload, n_symbols, args.consumer_msgs, args.seed,
                                render_threads=args.consumer_render_threads or None,
                                warm_batches=args.consumer_warm_batches)

    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        thr = max(1, min(args.cpu_threads, os.cpu_count() or 1))
        note("cpu baseline")
        one, many = cpu_baseline(host_batches, n_symbols, args.cpu_budget, thr)
        v1, done, t_cpu, used = one
        cpu = {"value": round(v1, 1), "unit": "orders/s", "cores": 1, "kind": "port",
               "sample": f"oracle/gome_oracle.c (1 thread) on the first {done} orders "
                         f"({used} batches) of the same rank-0 stream, {t_cpu:.1f} s",
               "reference": "not runnable here: no Go toolchain, Redis or RabbitMQ on the box "
                            "(BASELINE.md; the reference's CPU path is Go + Redis + RabbitMQ)"}
        if many is not None:
            cpu["sharded"] = {"value": round(many[0], 1), "unit": "orders/s", "cores": thr,
                              "sample": f"same {done} orders, symbol-sharded over {thr} threads "
                                        f"(one oracle per thread), {many[2]:.2f} s"}

    traffic = None
    if os.path.exists(args.traffic_json):
        try:
            tj = json.load(open(args.traffic_json))
            traffic = tj.get(f"{args.workload}:{kname}_hbm_bytes_per_launch",
                             tj.get(f"{kname}_hbm_bytes_per_launch") if args.workload == "config3" else None)
        except (OSError, ValueError):
            traffic = None

    if rank == 0:
        achieved = bdom / (ms_dom * 1e-3) / 1e9 if ms_dom > 0 else 0.0
        out = {
            "metric": METRIC,
            "value": round(g_orders / elapsed, 1),
            "unit": "orders/s",
            "n_gpus": world,
            "steps": steps,
            "warmup": warm,
            "ms_per_step": round(elapsed / steps * 1e3, 3),
            "higher_is_better": True,
            "scaling": args.scaling,
            "vs_baseline": None,
            "dtype": "int64",
            "data": "synthetic (seeded doorder.go distribution, Zipf symbols)",
            "config": {"workload": W["desc"].format(**W), "name": args.workload,
                       "symbols": n_symbols, "zipf_s": W["zipf"],
                       "batch_per_gpu": per_rank,
                       "global_batch": per_rank * world if args.scaling == "weak" else args.batch,
                       "parallelism": f"symbol-sharded x{world} (no data-path collective)"},
            "p50_batch_ms": round(pctl(lat, 0.5), 3),
            "p99_batch_ms": round(pctl(lat, 0.99), 3),
            # per-batch device latency (the batch's first to last kernel on the device; with two
            # batches in flight a batch starts when the one before it leaves the pipeline's stream)
            "p50_device_batch_ms": round(pctl(dev_lat, 0.5), 3),
            "p99_device_batch_ms": round(pctl(dev_lat, 0.99), 3),
            "p99_device_batch_ms_per_rank": p99_ranks,
            "hot_book_orders_per_rank": [int(x) for x in hot_ranks],
            "fills_per_s": round(g_fills / elapsed, 1),
            "events_per_s": round(g_events / elapsed, 1),
            "cancels_per_batch": int(cancels / steps),
            "device_ms_per_batch": round(ms_total, 3),
            "host_enqueue_ms": round(sum(s["ms_host_enqueue"] for s in sts) / steps, 3),
            "steps_mode": ("pipelined: two batches in flight (gome_submit_batch_device_async + "
                           "gome_collect_device); p50/p99_batch_ms are submit-to-collect times (two "
                           "batches), p50/p99_device_batch_ms each batch's own device time (from its "
                           "first kernel on the pipeline's stream; an early plan starts before it)") if pipelined
                          else "synchronous: one gome_submit_batch_device per step",
            # timed steps whose hottest book was planned early (match_early.h: right after the
            # previous batch's plan), and early plans not taken although ready (0 unless a bug)
            "early_plans": int(sum(s.get("n_early", 0) for s in sts)),
            "early_miss": int(sum(s.get("n_early_miss", 0) for s in sts)),
            "adm_ahead": int(sum(s.get("n_adm_ahead", 0) for s in sts)),
            "adm_redo": int(sum(s.get("n_adm_redo", 0) for s in sts)),
            "match_books_ms": round(ms_match, 3),
            "kernel_ms": {k: round(v[0], 3) for k, v in sorted(cands.items(), key=lambda kv: -kv[1][0])},
            "kernel_ms_source": phase_src,
            "hot_book": {"orders_per_batch": int(max_seg), "top_symbol_share": round(top_share, 5),
                         "ns_per_order": round(cands.get(plan_key, cands["k_match_hot"])[0] * 1e6
                                               / max(max_seg, 1), 1),
                         "path": "flow" if plan_key in cands else "legacy"},
            "roofline": {"bound": "hbm", "achieved": round(achieved, 3), "peak": HBM_PEAK_GBS,
                         "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 6),
                         "traffic": traffic, "kernel": f"{kname} ({kdesc})",
                         "kernel_ms": round(ms_dom, 3), "alg_bytes_per_launch": int(bdom),
                         "match_phase_alg_bytes": int(balg)},
            # SURVEY §8d's primary metric (host records in, H2D + pipeline + D2H, events back in host
            # memory) from the same run; `value` keeps the records resident in HBM (the bench contract:
            # a PCIe-inclusive rate is reported beside it, never as it)
            "value_e2e": e2e["value"] if e2e else None,
            "e2e": e2e,
            "consumer": consumer,
            "cpu_baseline": cpu,
        }
        if plan_key in cands and cands[plan_key][0] > 0:
            # the bound that matters: one wavefront's serial plan of the hottest book (rank 0's)
            plan_ms = cands[plan_key][0]
            bound = g_orders / steps / (plan_ms * 1e-3)
            out["critical_path"] = {"kernel": plan_key, "plan_ms": round(plan_ms, 3),
                                    "bound_orders_per_s": round(bound, 1),
                                    "frac": round(out["value"] / bound, 4),
                                    "note": "orders per step / the hottest book's plan time: the batch "
                                            "cannot end before that one wavefront does"}
        if injected is not None:
            out["config"]["injected"] = dict(injected, records=len(injected["records"]))
            clean = [float(s["ms_total"]) for s in sts[2:]]  # (the injected batch and the one after it aside)
            out["quirk_batch"] = {
                "injected_batch_device_ms": round(float(sts[0]["ms_total"]), 3),
                "next_batch_device_ms": round(float(sts[1]["ms_total"]), 3) if len(sts) > 1 else None,
                "clean_median_device_ms": round(float(np.median(clean)), 3) if clean else None,
                "ratio": round(float(sts[0]["ms_total"]) / float(np.median(clean)), 3) if clean else None,
                "legacy_hot_orders": [int(s["n_hot_orders"]) - int(s["n_flow_orders"]) for s in sts[:3]],
                "flow_head_orders": [int(s["n_flow_head_orders"]) for s in sts[:3]],
                "flow_wrong_zero_stale_bail": [[int(s[k]) for k in ("n_flow_wrong", "n_flow_zero", "n_flow_stale",
                                                                    "n_flow_bail")] for s in sts[:3]]}
        if consumer is not None:
            consumer["vs_value"] = round(consumer["messages_per_s"] / out["value"], 6)
        if pub is not None and use_pg:
            pub.check(int(g_orders), int(g_fills), int(g_events))
            out["publisher"] = pub.summary()
            out["publisher"]["digest_check"] = digest_check
            out["config"]["backend"] = args.backend + (" (all ranks on device 0)" if args.same_device else "")
        print(json.dumps(out), flush=True)
    if use_pg:
        dist.destroy_process_group()
    eng.close()


if __name__ == "__main__":
    main()
