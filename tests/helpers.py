"""Shared test utilities: string interning (the host's job at the boundary),
request -> gome_order conversion, event rendering, randomized request streams."""
from __future__ import annotations

import json

import numpy as np

from gome_amd.abi import fixed_from_double, render_match_result
from gome_amd.workload import ORDER_DTYPE

ADD, DEL = 1, 2


class Interner:
    def __init__(self):
        self.fwd: dict[str, dict[str, int]] = {"sym": {}, "uuid": {}, "oid": {}}
        self.rev: dict[str, list[str]] = {"sym": [], "uuid": [], "oid": []}
        self.tx_fwd = {0: 0, 1: 1}  # Transaction value -> code (gome_abi.h), 1 = SALE
        self.tx_rev = [0, 1]

    def tx_code(self, raw: int) -> int:
        raw = int(raw)
        if raw not in self.tx_fwd:
            if len(self.tx_rev) == 256:
                raise ValueError("more than 254 distinct Transaction values outside {0, 1}")
            self.tx_fwd[raw] = len(self.tx_rev)
            self.tx_rev.append(raw)
        return self.tx_fwd[raw]

    def tx_raw(self, code: int) -> int:
        return self.tx_rev[int(code)] if int(code) < len(self.tx_rev) else int(code)

    def tx_table(self):
        return self.tx_rev

    def id(self, kind: str, s: str) -> int:
        d = self.fwd[kind]
        if s not in d:
            d[s] = len(self.rev[kind])
            self.rev[kind].append(s)
        return d[s]

    def name(self, kind: str, i: int) -> str:
        return self.rev[kind][i]


def requests_to_records(batch, names: Interner, accuracy: int = 8) -> np.ndarray:
    """[(action, OrderRequest dict)] -> gome_order records (ordernode.go:38-54 conversion)."""
    rec = np.zeros(len(batch), ORDER_DTYPE)
    for i, (action, r) in enumerate(batch):
        rec[i]["price_fx"] = fixed_from_double(r["price"], accuracy)
        rec[i]["volume_fx"] = fixed_from_double(r["volume"], accuracy)
        rec[i]["symbol_id"] = names.id("sym", r["symbol"])
        rec[i]["oid_id"] = names.id("oid", r["oid"])
        rec[i]["uuid_id"] = names.id("uuid", r["uuid"])
        rec[i]["side"] = names.tx_code(r["transaction"])
        rec[i]["action"] = action
    return rec


def render_events(events: np.ndarray, records: np.ndarray, names: Interner,
                  accuracy: int = 8) -> list[str]:
    from gome_amd.workload import taker_remaining
    out = []
    rem = taker_remaining(events, records) if len(events) else []
    for e, tr in zip(events, rem):
        t = records[e["taker_seq"]]
        sym = names.name("sym", int(t["symbol_id"]))
        cancel = e["kind"] == 2
        out.append(render_match_result(
            e, t, int(tr), sym, names.name("uuid", int(t["uuid_id"])), names.name("oid", int(t["oid_id"])),
            None if cancel else names.name("uuid", int(e["maker_uuid_id"])),
            None if cancel else names.name("oid", int(e["maker_oid_id"])),
            None if (cancel or e["maker_is_last"]) else names.name("oid", int(e["maker_next_oid_id"])),
            accuracy, tx_table=names.tx_table()))
    return out


def random_batches(rng: np.random.Generator, n_batches: int, batch: int, symbols=("eth2usdt", "btc2usdt"),
                   del_frac: float = 0.3, quirks: bool = True, price_grid=None, oid_base: int = 1):
    """Randomized request streams exercising the reference quirks:
    wrong-side / wrong-price / wrong-uuid / unknown cancels (Q2, Q3), DEL before ADD and
    duplicate ADD in one batch (Q4), zero volumes (Q6), Transaction outside {0,1} (Q8),
    partial fills then cancel (Q9), ignored actions.  Oids are never reused across
    admitted ADDs (README.md:27; Q7 is outside the domain)."""
    price_grid = price_grid or [0.1, 0.2, 0.25, 0.3, 0.5, 0.55, 0.7, 0.9, 1.0]
    vol_grid = [0.01, 0.1, 0.25, 0.5, 1.0, 1.5, 3.0]
    added = []  # (sym, oid, uuid, side, price)
    next_oid = oid_base
    out = []
    for _ in range(n_batches):
        b = []
        pending_dup = []
        for _ in range(batch):
            u = rng.random()
            if u < del_frac and added:
                sym, oid, uuid, side, price = added[int(rng.integers(len(added)))]
                if quirks:
                    q = rng.random()
                    if q < 0.08:
                        side = 1 - side if side in (0, 1) else 0  # Q2 wrong side
                    elif q < 0.14:
                        price = float(rng.choice(price_grid))  # Q3 (maybe) wrong price
                    elif q < 0.18:
                        uuid = "u" + str(int(rng.integers(3)))  # uuid is not checked on cancel
                    elif q < 0.22:
                        oid = "nope" + str(int(rng.integers(1000)))  # unknown oid
                b.append((DEL, dict(uuid=uuid, oid=oid, symbol=sym, transaction=side,
                                    price=price, volume=float(rng.choice(vol_grid)))))
                continue
            if quirks and pending_dup and rng.random() < 0.05:
                b.append(pending_dup.pop())  # Q4 duplicate ADD in the same batch (same key)
                continue
            sym = str(rng.choice(symbols))
            side = int(rng.integers(2))
            if quirks and rng.random() < 0.03:
                side = int(rng.choice([2, 5]))  # Q8: treated as BUY
            price = float(rng.choice(price_grid))
            vol = float(rng.choice(vol_grid))
            if quirks and rng.random() < 0.03:
                vol = 0.0  # Q6
            uuid = "u" + str(int(rng.integers(3)))
            oid = str(next_oid)
            next_oid += 1
            req = dict(uuid=uuid, oid=oid, symbol=sym, transaction=side, price=price, volume=vol)
            if quirks and rng.random() < 0.04:
                # Q4: cancel placed before its ADD in the same batch -> ADD dropped
                b.append((DEL, dict(req)))
            if quirks and rng.random() < 0.02:
                b.append((7, dict(req)))  # unknown Action: consumed and ignored
            b.append((ADD, req))
            pending_dup.append((ADD, dict(req)))
            added.append((sym, oid, uuid, side, price))
        out.append(b)
    return out


def literal_state_to_levels(state: dict) -> dict:
    """literal.book_state -> {price_fx: (depth, in_buy, in_sale, [(oid, uuid, tx, vol)])}
    keeping only observable levels (as gome_snapshot_levels does)."""
    prices = set(state["depth"]) | set(state["BUY"]) | set(state["SALE"]) | set(state["fifo"])
    out = {}
    for p in prices:
        d = state["depth"].get(p, 0.0)
        fifo = state["fifo"].get(p, [])
        ib, isl = p in state["BUY"], p in state["SALE"]
        if not fifo and d == 0 and not ib and not isl:
            continue
        out[int(p)] = (int(d), ib, isl, [(o, u, int(t), int(v)) for o, u, t, v in fifo])
    return out


def engine_state_to_levels(eng, sym_id: int, names: Interner) -> dict:
    out = {}
    for lv in eng.levels(sym_id):
        p = int(lv["price_fx"])
        nodes = eng.fifo(sym_id, p)
        out[p] = (int(lv["depth_fx"]), bool(lv["in_buy"]), bool(lv["in_sale"]),
                  [(names.name("oid", int(n["oid_id"])), names.name("uuid", int(n["uuid_id"])),
                    names.tx_raw(int(n["side"])), int(n["volume_fx"])) for n in nodes])
    return out


def canon(js: str) -> str:
    """Stable re-serialisation (for readable diffs only; parity compares raw bytes)."""
    return json.dumps(json.loads(js), sort_keys=True)


def golden_names():
    return ["kat", "doorder_3k", "quirk_mix"]


def load_golden(name):
    from tests.golden.make_golden import load
    g = load(name)
    return g if isinstance(g, list) else [g]


def replay_fixture(fx, make_backend):
    """Replay a golden fixture through a backend (C oracle or HIP engine) and return
    (rendered MatchResult JSON list, state dict in the fixture's format).
    make_backend(n_symbols, max_batch) -> object with .submit(rec) -> events, .levels, .fifo"""
    names = Interner()
    batches = [[(a, r) for a, r in b] for b in fx["batches"]]
    syms = sorted({r["symbol"] for b in batches for _, r in b})
    for s in syms:
        names.id("sym", s)
    be = make_backend(len(syms), max(len(b) for b in batches))
    out = []
    for b in batches:
        rec = requests_to_records(b, names)
        out += render_events(be.submit(rec), rec, names)
    state = {}
    for s in syms:
        lv = engine_state_to_levels(be, names.id("sym", s), names)
        state[s] = {str(p): [d, ib, isl, [list(x) for x in fifo]] for p, (d, ib, isl, fifo) in sorted(lv.items())}
    return out, state
