"""The native OrderNode decoder (gome_decode_order_nodes / gome_consume_order_nodes, gome_host.h)
against the literal transliteration of Go's json.Unmarshal into an OrderNode
(oracle/literal.go_unmarshal_order_node; rabbitmq.go:118-121, ordernode.go:9-36), on CPU.

Corpus: the consumer tests' odd messages, hand-written edge cases (key folding, escapes and
surrogates, invalid UTF-8, number forms and widths, nesting, duplicates, trailing bytes), a
generated corpus of typed field variations and byte-level mutations of valid messages (mostly
syntax errors: the validator must agree byte for byte on what is JSON).  The seven fields the
engine reads are compared exactly (floats bit for bit).  Nesting deeper than Python's json can
parse is checked against Go's documented limit (maxNestingDepth 10000) alone: parity unpinned
there (the literal cannot parse it)."""
import json
import struct

import numpy as np
import pytest

from gome_amd.consumer import (BatchingConsumer, MatchSink, Names, PrePool, decode_order_nodes, pack_messages)
from oracle.literal import go_unmarshal_order_node
from tests.test_consumer import ODD_MESSAGES, _msg

FIELDS = ("Action", "Uuid", "Oid", "Symbol", "Transaction", "Price", "Volume")


def _lit(body):
    nd = go_unmarshal_order_node(body)
    return {k: getattr(nd, k) for k in FIELDS}


def _same(a, b):
    for k in FIELDS:
        x, y = a[k], b[k]
        if isinstance(x, float) or isinstance(y, float):
            if struct.pack("<d", float(x)) != struct.pack("<d", float(y)):
                return False
        elif x != y:
            return False
    return True


def _check(msgs, threads=0):
    got = decode_order_nodes(msgs, threads=threads)
    for m, g in zip(msgs, got):
        want = _lit(m)
        assert _same(g, want), f"{m!r}:\n native  {g}\n literal {want}"


EDGE = [
    # key folding: exact, ASCII case, U+017F / U+212A (Go folds them to S / K), ligatures (Go does not)
    '{"ſymbol":"x","action":1,"OID":"7"}'.encode(),
    '{"Symbol":"a","ſYMBOL":"b"}'.encode(),
    '{"AcKion":1}'.encode(), '{"Symbol":"s","Action":1,"Oid":"K"}'.encode(),
    '{"Isfirst":true,"Isﬁrst":false,"Action":2}'.encode(),
    '{"\\u0053ymbol":"esc-key","\\u0041ction":1}', '{"symbol ":"trailing space"}',
    # strings: escapes, pairs, lone surrogates, raw control bytes (syntax error), 0x7f, NUL
    r'{"Symbol":"a\"b\\c\/d\b\f\n\r\t","Action":1}', r'{"Symbol":"😀x","Oid":"\udc00\ud800"}',
    r'{"Symbol":"\ud800A","Uuid":"\ud800𐀀"}', r'{"Symbol":"\u0000z"}',
    b'{"Symbol":"a\x01b"}', b'{"Symbol":"a\x7fb"}', r'{"Symbol":"\x"}', r'{"Symbol":"\u12"}',
    b'{"Symbol":"\xc3\xa9\xe2\x82\xac\xf0\x9f\x98\x80"}', b'{"Symbol":"\xc0\xaf\xe0\x80\xaf\xf4\x90\x80\x80"}',
    b'{"Symbol":"\xf0\x9f\x98"}', b'{"Symbol":"x\xed\xbf\xbfy"}', b'\xef\xbb\xbf{"Action":1}',
    # numbers
    '{"Price":-0,"Volume":-0.0}', '{"Price":1e-400,"Volume":-1e-400}', '{"Price":1e308,"Volume":1.8e308}',
    '{"Price":4.9e-324,"Volume":2.2250738585072011e-308}', '{"Price":0.1,"Volume":123456789012345678901234567890}',
    '{"Price":01}', '{"Price":.5}', '{"Price":1.}', '{"Price":1e}', '{"Price":+1}', '{"Price":-}', '{"Price":1E+2}',
    '{"Action":127,"Transaction":-2147483648}', '{"Action":-128,"Transaction":2147483647}',
    '{"Action":128,"Transaction":2147483648}', '{"Action":-129,"Transaction":-2147483649}',
    '{"Action":1e0}', '{"Action":9223372036854775807}', '{"Action":9223372036854775808}',
    '{"Action":-9223372036854775808}', '{"Action":-0,"Transaction":-0}', '{"Action":"1"}',
    # types, null, duplicates
    '{"Action":1,"Action":null}', '{"Action":1,"Action":"x"}', '{"Action":1,"action":2}',
    '{"Symbol":1,"Uuid":true,"Oid":[1],"Price":"5","Volume":{"a":1}}', '{"Price":[1,{"Volume":2}],"Volume":3}',
    '{"IsFirst":"x","Accuracy":1.5,"NodeName":7,"Action":2}', '{"Symbol":null}',
    # structure
    '{}', ' {"Action":1} ', '{"Action":1}x', '{"Action":1,}', '{,"Action":1}', '{"Action" 1}', '{"Action":1 "x":2}',
    '', ' ', 'null', 'true', '1', '"s"', '[]', '[{"Action":1}]', '{"a":[[[[[[]]]]]],"Action":1}',
    '{"a":{"b":{"c":{}}},"Action":1}', '{"Action":1}\n\t\r ', '{"Action":1}\x00', '{"a":tru}', '{"a":nul}',
    '{"a":[1,2,]}', '{"a":[,1]}', '{"a":{"b"}}', '{"a":{"b":}}', '{"a" : [ 1 , { "c" : [ ] } ] , "Action" : 2 }',
    '{"Action":NaN}', '{"Action":Infinity}', '{"Action":-Infinity}', "{'Action':1}", '{"Action":1}}',
]


def test_odd_and_edge_messages_match_literal():
    _check(ODD_MESSAGES + EDGE)


def _typed_corpus(rng, n):
    vals = {
        "int": ["1", "2", "0", "-1", "127", "128", "300", "1.0", "1e2", '"1"', "null", "true", "[]", "{}",
                "2147483647", "2147483648", "-2147483649", "99999999999999999999", "-0", "7"],
        "float": ["50000000", "5e7", "1E8", "0.5", "-1", "1e400", "-1e400", "1e-400", '"abc"', "null", "false",
                  "[1]", "123456789.123456789", "0", "-0", "9007199254740993", "4.9e-324"],
        "str": ['"s"', '"a\\u0000b"', '"\\ud800"', '"\\ud83d\\ude00"', '"\\u212a"', "1", "null", '"<&>"',
                '"x\\/y"', '""', '"\\u00e9t\\u00e9"', '"long-' + "z" * 300 + '"'],
    }
    names = [("Action", "int"), ("Uuid", "str"), ("Oid", "str"), ("Symbol", "str"), ("Transaction", "int"),
             ("Price", "float"), ("Volume", "float"), ("Accuracy", "int"), ("NodeName", "str"),
             ("IsFirst", "str"), ("Extra", "str")]
    out = []
    for _ in range(n):
        parts = []
        for _ in range(int(rng.integers(0, 12))):
            nm, kind = names[int(rng.integers(len(names)))]
            r = rng.random()
            if r < 0.15:
                nm = nm.lower()
            elif r < 0.2:
                nm = nm.upper()
            elif r < 0.23:
                nm = nm.replace("s", "ſ").replace("k", "K")
            v = vals[kind][int(rng.integers(len(vals[kind])))]
            ws = " " if rng.random() < 0.1 else ""
            parts.append(f'{ws}"{nm}"{ws}:{ws}{v}{ws}')
        out.append(("{" + ",".join(parts) + "}").encode())
    return out


def _mutated(rng, n):
    base = [_msg(oid=str(k), tx=k % 2, price=str(40000000 + k), vol="100000000").encode() for k in range(64)]
    out = []
    for _ in range(n):
        b = bytearray(base[int(rng.integers(len(base)))])
        for _ in range(int(rng.integers(1, 4))):
            i = int(rng.integers(len(b) + 1))
            r = rng.random()
            if r < 0.35 and len(b):
                del b[min(i, len(b) - 1)]
            elif r < 0.7:
                b.insert(i, int(rng.choice(list(b'{}[]",:\\ 0123456789eE.-+tfnul') + [0x80, 0xff, 0x01, 0xc3])))
            elif len(b):
                b[min(i, len(b) - 1)] = int(rng.integers(256))
        out.append(bytes(b))
    return out


@pytest.mark.parametrize("seed", range(3))
def test_generated_corpus_matches_literal(seed):
    rng = np.random.default_rng(seed)
    _check(_typed_corpus(rng, 3000))


@pytest.mark.parametrize("seed", range(3))
def test_mutated_messages_match_literal(seed):
    rng = np.random.default_rng(100 + seed)
    msgs = _mutated(rng, 4000)
    _check(msgs)
    # (mutations leave both valid and invalid JSON behind)
    objs = sum(1 for m in msgs if go_unmarshal_order_node(m).Action != 0)
    assert 200 < objs < 3900


def test_threads_do_not_change_the_result():
    rng = np.random.default_rng(7)
    msgs = _typed_corpus(rng, 5000) + _mutated(rng, 5000)
    assert decode_order_nodes(msgs, threads=1) == decode_order_nodes(msgs, threads=8)


def test_nesting_depth_limit():
    """encoding/json rejects nesting deeper than 10000 (scanner maxNestingDepth); parity unpinned
    (Python's json cannot parse this deep)."""
    def deep(k):  # the top-level object is depth 1, then k - 1 arrays
        return ('{"Action":1,"x":' + "[" * (k - 1) + "]" * (k - 1) + "}").encode()
    ok, bad = decode_order_nodes([deep(10000), deep(10001)])
    assert ok["Action"] == 1 and bad["Action"] == 0


def test_consume_records_and_markers():
    """gome_consume_order_nodes: ignored actions keep a zero record, rejected ones are dropped,
    markers are consumed staged (commit / abort), ids in first-seen order."""
    lib_names, pre = Names(), PrePool()
    pre.set("s", "u", "1")
    pre.set("s", "u", "3")
    msgs = [_msg(oid="1"), "{bad", _msg(oid="2", vol="-5"), _msg(oid="3", action=2), _msg(oid="1"),
            _msg(sym="t", oid="4", price="0.5")]
    cons = BatchingConsumer(type("E", (), {"max_batch": 16, "max_symbols": 4})(), pre, MatchSink(), lib_names)
    rec = cons.records(msgs)
    assert len(rec) == 4 and cons.rejected == 2
    assert rec["action"].tolist() == [1, 0, 2, 1] and rec["oid_id"].tolist() == [0, 0, 1, 0]
    assert rec["flags"].tolist() == [3, 0, 1, 1]  # ADM_HOST | ADMITTED, zero, DEL, a repeated key
    assert len(pre) == 2
    pre.abort()
    assert len(pre) == 2
    cons.records(msgs)
    pre.commit()
    assert len(pre) == 0
    assert lib_names.count("sym") == 1 and lib_names.name("oid", 1) == "3"


def _queue_batch(rng, n, odd_tx=False):
    """A batch that exercises the queue-order rules: names new and seen (in and across batches),
    repeated keys (a DEL of a same-batch ADD, an ADD repeated), markers set once, twice or never,
    rejected and ignored messages."""
    out = []
    for k in range(n):
        r = rng.random()
        sym = f"S{int(rng.zipf(1.3)) % 300}"
        uuid = f"u{int(rng.integers(40))}"
        oid = str(int(rng.integers(3 * n)))  # (~1 in 6 repeats within the batch)
        tx = 5 if odd_tx and rng.random() < 0.01 else int(rng.integers(2))
        if r < 0.03:
            out.append(_msg(oid=oid, sym=sym, uuid=uuid, vol="-5"))             # rejected (volume)
        elif r < 0.05:
            out.append(_msg(oid=oid, sym=sym, uuid=uuid, price="0.5"))          # rejected (not scaled)
        elif r < 0.07:
            out.append(_msg(action=3, oid=oid, sym=sym, uuid=uuid))             # ignored action
        elif r < 0.08:
            out.append("{bad")
        else:
            out.append(_msg(action=2 if r < 0.35 else 1, oid=oid, sym=sym, uuid=uuid, tx=tx,
                            price=str(int(rng.integers(1, 100)) * 10**6)))
    return out


def _queue_run(batches, threads, marks, max_symbols=0):
    names, pre = Names(), PrePool()
    for s_, u_, o_ in marks:
        pre.set(s_, u_, o_)
    cons = BatchingConsumer(type("E", (), {"max_batch": 1 << 16, "max_symbols": max_symbols})(), pre, MatchSink(),
                            names, threads=threads)
    outs = []
    for i, b in enumerate(batches):
        rec = cons.records(b)
        outs.append((rec.copy(), cons.rejected, len(pre)))
        if i % 3 == 1:
            pre.abort()
            rec = cons.records(b)  # (the same batch again after a refusal: the same verdicts)
            outs.append((rec.copy(), cons.rejected, len(pre)))
        pre.commit()
        for s_, u_, o_ in marks[i::len(batches)]:  # (the gRPC side re-sets some markers between batches)
            pre.set(s_, u_, o_)
    tables = {k: [names.name(k, j) for j in range(names.count(k))] for k in ("sym", "uuid", "oid")}
    _queue_run.parallel = cons.parallel_batches
    _queue_run.steps = cons.queue_steps_s
    return outs, tables, len(pre)


@pytest.mark.parametrize("odd_tx,max_symbols", [(False, 0), (False, 280), (True, 0)])
def test_parallel_queue_pass_matches_the_serial_one(odd_tx, max_symbols):
    """Round 6: gome_consume_order_nodes interns a batch's new names shard by shard (numbered by
    their first message) and stages its markers shard by shard on its worker pool, instead of one
    message after another.  The records, admission verdicts, rejections, the name tables (id by id)
    and the markers left must be the serial pass's (threads = 1) exactly, over batches that repeat
    names and keys within and across batches, abort and re-consume, and re-set markers; with odd
    Transactions or a Symbol range that the batch could fill, the batch takes the serial pass."""
    rng = np.random.default_rng(11 + max_symbols + odd_tx)
    batches = [_queue_batch(rng, 6000, odd_tx) for _ in range(5)]
    adds = [json.loads(m) for b in batches for m in b if m.startswith('{"Action":1')]
    marks = [(a["Symbol"], a["Uuid"], a["Oid"]) for a in adds if rng.random() < 0.5]
    par = _queue_run(batches, 8, marks, max_symbols)
    npar, steps = _queue_run.parallel, _queue_run.steps
    ser = _queue_run(batches, 1, marks, max_symbols)
    assert _queue_run.parallel == 0
    assert npar == (0 if (odd_tx or max_symbols) else 7), npar  # (5 batches, 2 consumed twice)
    # (gome_consume_last_steps: the parallel path's step times; all zero where every batch was serial)
    assert (sum(steps) > 0) == (npar > 0) and sum(_queue_run.steps) == 0
    assert par[1] == ser[1] and par[2] == ser[2]
    for (ra, ja, pa), (rb, jb, pb) in zip(par[0], ser[0]):
        assert ja == jb and pa == pb
        assert np.array_equal(ra, rb)
    assert sum(int((r["flags"] == 3).sum()) for r, _, _ in par[0]) > 1000  # (admitted ADDs)


def test_pack_messages_offsets():
    buf, off = pack_messages(["ab", b"", "é"])
    assert buf == b"ab\xc3\xa9" and off.tolist() == [0, 2, 2, 4]


def test_staged_marker_set_again_survives_the_commit():
    """the gRPC side's SetPrePool of a key the consumer has staged (consumed by a batch not
    yet committed) leaves a live marker, as SetPrePool after DeletePrePool does in the reference
    (nodepool.go:14-28); abort keeps one marker; a take of the re-set marker consumes it."""
    names, pre = Names(), PrePool()
    cons = BatchingConsumer(type("E", (), {"max_batch": 16, "max_symbols": 4})(), pre, MatchSink(), names)
    pre.set("s", "u", "1")
    assert cons.records([_msg(oid="1")])["flags"].tolist() == [3]  # staged
    pre.set("s", "u", "1")                                          # set again before the commit
    pre.commit()
    assert len(pre) == 1
    assert cons.records([_msg(oid="1")])["flags"].tolist() == [3]  # the new marker admits it
    pre.set("s", "u", "1")
    pre.abort()
    assert len(pre) == 1
    cons.records([_msg(oid="1")])
    pre.set("s", "u", "1")
    assert pre.consume_add("s", "u", "1")                           # the re-set marker taken
    pre.commit()
    assert len(pre) == 0


# ---- Hypothesis: structured damage to valid OrderNode bodies (also the corpus of the sanitizer run,
# tests/test_host_sanitizers.py): truncated UTF-8 sequences, nesting, long escapes, duplicate keys
from hypothesis import HealthCheck, given, settings, strategies as hs  # noqa: E402

_UTF8 = [b"\xc3", b"\xe2\x82", b"\xf0\x9f\x98", b"\xed\xa0", b"\xf4\x90", b"\xc0", b"\xff", b"\x80\x80"]
_ESC = ["\\n", "\\\"", "\\\\", "\\/", "\\u0041", "\\ud83d\\ude00", "\\ud800", "\\udc00", "\\u00e9", "\\t"]


@hs.composite
def _damaged(draw):
    k = draw(hs.integers(0, 63))
    body = _msg(oid=str(k), tx=k % 2, price=str(40000000 + k), vol="100000000").encode()
    kind = draw(hs.sampled_from(["utf8", "nest", "escape", "dup", "cut"]))
    if kind == "utf8":  # a truncated or invalid UTF-8 sequence inside a string value
        at = body.index(b'"Symbol":"') + 10
        body = body[:at] + draw(hs.sampled_from(_UTF8)) * draw(hs.integers(1, 3)) + body[at:]
    elif kind == "nest":  # an extra member nested d deep (arrays and objects)
        d = draw(hs.integers(1, 400))
        o = draw(hs.sampled_from(["[", '{"n":']))
        c = "]" if o == "[" else "}"
        body = body[:-1] + b',"x":' + (o * d + "1" + c * d).encode() + b"}"
    elif kind == "escape":  # long runs of escapes in a string the engine reads
        s = "".join(draw(hs.lists(hs.sampled_from(_ESC), min_size=1, max_size=300)))
        body = body[:-1] + b',"Uuid":"' + s.encode() + b'"}'
    elif kind == "dup":  # duplicate and case-folded keys: the last one wins
        key = draw(hs.sampled_from(["Action", "action", "ACTION", "Price", "pRICE", "Symbol", "\\u0053ymbol"]))
        val = draw(hs.sampled_from(["1", "2", "null", '"s"', "1e3", "[]"]))
        body = body[:-1] + f',"{key}":{val}'.encode() * draw(hs.integers(1, 4)) + b"}"
    else:  # truncated anywhere
        body = body[:draw(hs.integers(0, len(body)))]
    return body


@settings(max_examples=300, deadline=None, suppress_health_check=[HealthCheck.too_slow])
@given(hs.lists(_damaged(), min_size=1, max_size=24))
def test_damaged_messages_match_literal(msgs):
    _check(msgs)
    _check(msgs, threads=3)
