"""Long single updates on the GPU (ylong.hip): the parallel parse -- a speculative block end at
every byte, pointer doubling per 8 KB chunk, the stitch along the true chain, the exact parse
of every block on it -- and the grid path for documents that are one long update
(merge_updates_v1 / diff_updates_v1 / encode_state_vector_from_update_v1 with a lane per block,
yrs/src/update.rs:107-114, 490-535, 537-704).  GPU == oracle byte for byte and status for
status.  The shapes cover both sides of every check: chunk-crossing and chunk-spanning blocks
(a 20 KB string), content kinds the speculative parse leaves to the exact parse (Any maps and
long lists, Doc, Move), multi-section updates, Skips, zero-length GC and Items, DeleteSets that
are unsorted / overlapping / adjacent / empty / of two clients, truncations, random bytes, and
more long documents than the grid path lists per batch."""
import numpy as np
import pytest

import corpus
import workloads
from test_gpu_diff import check_diff, check_sv
from test_gpu_parity import batch_of, check_batch, engine_with

pytestmark = pytest.mark.gpu


def _var(x):
    out = bytearray()
    while True:
        b, x = x & 0x7F, x >> 7
        if x:
            out.append(b | 0x80)
        else:
            out.append(b)
            return bytes(out)


def _ivar(v):  # lib0 signed varint (yrs/src/encoding/varint.rs:262-281)
    neg, v = v < 0, abs(v)
    out = bytearray([(0x80 if v > 63 else 0) | (0x40 if neg else 0) | (v & 63)])
    v >>= 6
    while v:
        out.append((0x80 if v > 127 else 0) | (v & 127))
        v >>= 7
    return bytes(out)


def _s(b):
    return _var(len(b)) + b


ROOT = _var(1) + _s(b"t")  # parent: named root "t"


def item(content, origin=None, right=None):
    """An Item (update.rs:433-488) with optional origins; without origins the parent is root "t"."""
    ref, body = content
    info = ref | (0x80 if origin else 0) | (0x40 if right else 0)
    b = bytes([info])
    if origin:
        b += _var(origin[0]) + _var(origin[1])
    if right:
        b += _var(right[0]) + _var(right[1])
    if not origin and not right:
        b += ROOT
    return b + body


def text(t):
    return (4, _s(t.encode()))


def deleted(n):
    return (1, _var(n))


def anys(vals):
    """ItemContent::Any (ref 8): ints (tag 125), strings (119), nulls, nested arrays (117)."""
    b = _var(len(vals))
    for v in vals:
        if v is None:
            b += bytes([126])
        elif isinstance(v, int):
            b += bytes([125]) + _ivar(v)
        elif isinstance(v, str):
            b += bytes([119]) + _s(v.encode())
        elif isinstance(v, list):
            b += bytes([117]) + _var(len(v)) + b"".join(bytes([125]) + _ivar(x) for x in v)
        elif isinstance(v, dict):
            b += bytes([118]) + _var(len(v)) + b"".join(_s(k.encode()) + bytes([125]) + _ivar(x) for k, x in v.items())
    return (8, b)


def gc(n):
    return bytes([0]) + _var(n)


def skip(n):
    return bytes([10]) + _var(n)


def content_len(c):
    ref, body = c
    if ref == 4:
        return len(body[len(_var(len(body))):].decode().encode("utf-16-le")) // 2 if body[0] else 0
    if ref in (1, 8):
        return _rv(body)
    return 1


def _rv(b):
    x = s = 0
    for c in b:
        x |= (c & 0x7F) << s
        s += 7
        if c < 0x80:
            return x
    return x


def section(client, clock, contents, chained=True):
    """A client section: `contents` are ItemContents (chained by origin when `chained`), raw
    block bytes, or ("skip", n) / ("gc", n)."""
    blocks, k = [], clock
    for c in contents:
        if isinstance(c, bytes):
            blocks.append(c)
            k += _rv(c[1:])
        elif c[0] == "skip":
            blocks.append(skip(c[1]))
            k += c[1]
        elif c[0] == "gc":
            blocks.append(gc(c[1]))
            k += c[1]
        else:
            n = content_len(c)
            blocks.append(item(c, origin=(client, k - 1) if chained and k > clock else None))
            k += n
    return client, clock, blocks


def update(sections, ds=()):
    b = bytearray(_var(len(sections)))
    for c, k, blocks in sections:
        b += _var(len(blocks)) + _var(c) + _var(k) + b"".join(blocks)
    b += _var(len(ds))
    for c, rs in ds:
        b += _var(c) + _var(len(rs))
        for s, n in rs:
            b += _var(s) + _var(n)
    return bytes(b)


def _rich(rng, n, client=7, big_client=False):
    """n blocks of mixed content: ASCII / non-ASCII text, deletions, Any lists (short, long,
    nested, maps), a few very long strings."""
    out = []
    words = ["alpha", "beta ", "γάμμα", "дельта", "ε", "日本語", "😀x", "z" * 40]
    for i in range(n):
        r = rng.random()
        if r < 0.45:
            out.append(text("".join(rng.choice(words) for _ in range(int(rng.integers(1, 6))))))
        elif r < 0.65:
            out.append(deleted(int(rng.integers(1, 30))))
        elif r < 0.8:
            out.append(anys([int(rng.integers(-1000, 1000)), "s" * int(rng.integers(0, 9)), None]))
        elif r < 0.85:
            out.append(anys(list(range(int(rng.integers(17, 40))))))  # > 16 values: exact parse
        elif r < 0.88:
            out.append(anys([[1, 2, 3], {"k": 1}]))  # nested: exact parse
        elif r < 0.9:
            out.append(text("q" * int(rng.integers(2000, 9000))))
        else:
            out.append(text("w" * int(rng.integers(50, 400))))
    return out


def _trace_merge(oracle, name, n, client=1):
    b, _ = workloads.trace_updates(name, client)
    ups = b.doc_updates(0)[:n]
    return oracle.merge_updates_v1([bytes(u) for u in ups], mode=1)


@pytest.fixture(scope="module")
def engine():
    # diff / SV grid path from 2 KB (default 64 KB); the single-update identity copy off, so the
    # grid paths see the canonical single-update documents (test_identity_copy covers it)
    e = engine_with(YMERGE_LS_MIN=2048, YMERGE_IDENTITY=0)
    yield e
    e.close()


@pytest.fixture(scope="module")
def longs(oracle):
    rng = np.random.default_rng(0x10C6)
    C = 0xB0B
    base = _rich(rng, 2600, C)  # > 1024 blocks: past the fast path's LDS capacity
    u = {}
    u["rich"] = update([section(C, 0, base)], ds=[(C, [(3, 2), (40, 10), (100, 1)])])
    u["rich_big_client"] = update([section(182476973021437, 5, base)], ds=[(182476973021437, [(6, 3)])])
    u["huge_string"] = update([section(C, 0, [text("a" * 20000), text("bc"), text("é" * 7000), deleted(3)])])
    u["skip"] = update([section(C, 0, base[:700] + [("skip", 5)] + base[700:1400])])
    u["zero_gc"] = update([section(C, 0, base[:400] + [("gc", 0)] + base[400:])])
    u["zero_item"] = update([section(C, 0, base[:200] + [text(""), deleted(0)] + base[200:1300])])
    u["gc_last"] = update([section(C, 0, base[:1500] + [("gc", 9)])])
    u["multi_section"] = update([section(C + 1, 0, base[:300]), section(C, 10, base[300:1700]),
                                 section(C + 2, 3, base[1700:])])
    u["repeated_client"] = update([section(C, 0, base[:1100]), section(C, 0, base[1100:2300])])
    u["ds_two_clients"] = update([section(C, 0, base[:1200])], ds=[(C, [(1, 2)]), (C + 9, [(0, 4)])])
    u["ds_unsorted"] = update([section(C, 0, base[:1200])], ds=[(C, [(50, 5), (10, 3), (70, 1)])])
    u["ds_overlap"] = update([section(C, 0, base[:1200])], ds=[(C, [(10, 5), (12, 8), (70, 1)])])
    u["ds_adjacent"] = update([section(C, 0, base[:1200])], ds=[(C, [(10, 5), (15, 8), (23, 1), (40, 2)])])
    u["ds_empty_range"] = update([section(C, 0, base[:1200])], ds=[(C, [(10, 0), (15, 8)])])
    u["ds_no_ranges"] = update([section(C, 0, base[:1200])], ds=[(C, [])])
    u["ds_many"] = update([section(C, 0, base[:1200])], ds=[(C, [(2 * k, 1) for k in range(3000)])])
    u["no_blocks"] = update([], ds=[(C, [(2 * k + 1, 1) for k in range(2000)])])
    u["trace"] = _trace_merge(oracle, "sveltecomponent", 900)
    u["trace2"] = _trace_merge(oracle, "friendsforever_flat", 1200)
    u["b4"] = corpus.b4_update()
    for k, v in u.items():
        assert len(v) >= 2048, k
    return u


def test_long_merge_single_update_docs(engine, oracle, longs):
    docs = [[v] for v in longs.values()]
    check_batch(engine, oracle, batch_of(docs))
    st = engine.stats()
    # rich, rich_big_client, zero_item, gc_last, ds_adjacent, ds_many, no_blocks, b4 (and the
    # DeleteSet shapes the grid path declines went on to the tiled kernel)
    assert st["docs_giant"] >= 7, (st["docs_giant"], st["docs_big"], st["docs_fast"], st["docs_exact"])


def test_identity_copy(oracle, longs):
    """With the identity copy on (the default), canonical single-update documents are copied by
    k_fast_merge: the same bytes as yrs' merge of the one update."""
    e = engine_with()
    try:
        docs = [[v] for v in longs.values()]
        check_batch(e, oracle, batch_of(docs))
    finally:
        e.close()


def test_long_merge_errors(engine, oracle, longs):
    u = longs["rich"]
    cuts = sorted({len(u) - k for k in (1, 2, 3, 7, 100, 5000)} | {2048 + 977 * k for k in range(12)})
    docs = [[u[:c]] for c in cuts if c >= 2048]
    rng = np.random.default_rng(7)
    docs.append([bytes(rng.integers(0, 256, 9000, dtype=np.uint8))])
    docs.append([bytes([1]) + u[1:5000]])
    docs.append([u[:3000] + bytes([0x80] * 12) + u[3012:]])
    check_batch(engine, oracle, batch_of(docs))


def test_long_merge_mixed_docs(engine, oracle, longs):
    """Long updates next to short ones and to each other (records consumed by the fast / tiled
    kernels), and more single-long-update documents than the grid path lists (LS_LIST)."""
    small = workloads.text_docs(4, 200, seed=3)
    docs = []
    for d in range(small.n_docs):
        ups = [bytes(x) for x in small.doc_updates(d)]
        docs.append(ups[:50] + [longs["trace"]] + ups[50:])
    docs.append([longs["rich"], longs["rich"]])
    docs.append([longs["trace"], longs["trace2"]])
    docs += [[longs["trace2"]]] * 20
    check_batch(engine, oracle, batch_of(docs))


def _cuts(clock):
    return sorted({0, 1, 2, 7, clock // 5, clock // 3, clock // 2 + 1, clock - 9, clock - 1, clock, clock + 4})


def test_long_state_vectors(engine, oracle, longs):
    check_sv(engine, oracle, list(longs.values()))


def test_long_diffs(engine, oracle, longs):
    us, ss = [], []
    for k, u in longs.items():
        st, sv = oracle.status_of(oracle.encode_state_vector_from_update_v1, u)
        pairs = oracle.parse_sv(sv) if st == 0 else []
        svs = [b"\x00", b"", bytes([0x80] * 3)]
        for c, clock in pairs[:1]:
            svs += [workloads.encode_sv([(c, x)]) for x in _cuts(clock)]
            svs.append(workloads.encode_sv([(c, 5), (c + 1, 3), (c, clock // 2)]))  # last insert wins
            svs.append(workloads.encode_sv([(c + (1 << 32), clock // 2)]))           # u64 id: no match
        us += [u] * len(svs)
        ss += svs
    check_diff(engine, oracle, us, ss)


def test_long_diffs_split_text(engine, oracle):
    """Remote clocks that cut non-ASCII strings (UTF-16 splits, surrogate pairs: yrs panics)."""
    C = 42
    u = update([section(C, 0, [text("ab" * 600), text("日本語" * 300), text("😀" * 500), text("xyz" * 400)])],
               ds=[(C, [(1, 1)])])
    svs = [workloads.encode_sv([(C, x)]) for x in (1199, 1200, 1201, 1650, 2100, 2101, 2102, 2103, 3000)]
    check_diff(engine, oracle, [u] * len(svs), svs)


def test_long_sync_frames(oracle, longs):
    """y-sync SyncStep1 / SyncStep2 replies (protocol.rs:62-69, 219-272) from the grid path."""
    e = engine_with(YMERGE_LS_MIN=2048)
    try:
        ups = [longs["trace"], longs["rich"], longs["b4"], longs["skip"]]
        msgs = []
        for u in ups:
            (c, k), = oracle.parse_sv(oracle.encode_state_vector_from_update_v1(u))[:1] or [(1, 0)]
            sv = workloads.encode_sv([(c, k // 2)])
            msgs.append(bytes([0, 0]) + _var(len(sv)) + sv)
        ub = np.frombuffer(b"".join(ups), np.uint8)
        uo = np.concatenate([[0], np.cumsum([len(u) for u in ups])]).astype(np.uint64)
        mb = np.frombuffer(b"".join(msgs), np.uint8)
        mo = np.concatenate([[0], np.cumsum([len(x) for x in msgs])]).astype(np.uint64)
        out, off, st = e.sync_step2_host(ub, uo, mb, mo)
        for d, (u, msg) in enumerate(zip(ups, msgs)):
            est, want = oracle.status_of(oracle.sync_step2_v1, u, msg)
            assert st[d] == est, d
            if not est:
                assert out[int(off[d]):int(off[d + 1])].tobytes() == want, d
        out, off, st = e.sync_step1_host(ub, uo)
        for d, u in enumerate(ups):
            assert st[d] == 0 and out[int(off[d]):int(off[d + 1])].tobytes() == oracle.sync_step1_v1(u), d
    finally:
        e.close()


@pytest.mark.parametrize("env", [{"YMERGE_LONG_GRID": 0}, {"YMERGE_LONG_PARSE": 0}])
def test_long_paths_off(oracle, longs, env):
    """The same documents with the grid path off (tiled kernel / planners) and with the parallel
    parse off (k_decode_huge's lockstep walk): same bytes."""
    e = engine_with(YMERGE_LS_MIN=2048, **env)
    try:
        vals = [longs[k] for k in ("rich", "huge_string", "multi_section", "ds_adjacent", "trace")]
        check_batch(e, oracle, batch_of([[v] for v in vals]))
        check_sv(e, oracle, vals)
    finally:
        e.close()


def _upd(sections, ds):
    """A v1 update: sections [(client, clock, [block bytes])], ds [(client, [(start, len)])]."""
    b = _var(len(sections))
    for client, clock, blocks in sections:
        b += _var(len(blocks)) + _var(client) + _var(clock) + b"".join(blocks)
    b += _var(len(ds))
    for client, ranges in ds:
        b += _var(client) + _var(len(ranges)) + b"".join(_var(s) + _var(n) for s, n in ranges)
    return b


def identity_reject_docs():
    """Single-update documents whose canonical-size check could pass although the merge writes
    other bytes: each must be merged, not copied.  The first ones are canonical
    (copied); the rest are shapes the identity copy must refuse."""
    t = item(text("abc"))
    o = item(text("xy"), origin=(7, 2))
    gc = bytes([0]) + _var(4)
    docs = {
        "canonical_one_block": [_upd([(7, 0, [t])], [])],
        "canonical_two_sections": [_upd([(9, 0, [t, o]), (7, 0, [t])], [(7, [(0, 2)])])],
        "canonical_ds_two_ranges": [_upd([], [(7, [(0, 2), (5, 1)])])],
        "ds_unsorted": [_upd([], [(7, [(5, 1), (0, 2)])])],
        "ds_adjacent": [_upd([], [(7, [(0, 2), (2, 3)])])],
        "ds_overlapping": [_upd([], [(7, [(0, 4), (2, 3)])])],
        "ds_unsorted_with_block": [_upd([(7, 0, [t])], [(7, [(2, 1), (0, 1)])])],
        "ds_adjacent_many": [_upd([(7, 0, [t, o])], [(7, [(0, 1), (1, 1), (3, 1), (4, 1)])])],
        "ds_two_entries": [_upd([], [(7, [(0, 2)]), (9, [(1, 1)])])],
        "ds_empty_entry": [_upd([(7, 0, [t])], [(7, [])])],
        "ds_zero_range": [_upd([(7, 0, [t])], [(7, [(1, 0)])])],
        "sections_ascending": [_upd([(7, 0, [t]), (9, 0, [t])], [])],
        "section_repeated_gap": [_upd([(7, 0, [t]), (7, 10, [t])], [])],
        "section_repeated_overlap": [_upd([(7, 0, [t, o]), (7, 2, [t])], [])],
        "section_repeated_contiguous": [_upd([(7, 0, [t]), (7, 3, [o])], [])],
        "skip_in_section": [_upd([(7, 0, [t, bytes([10]) + _var(3), o])], [])],
        "gc_blocks": [_upd([(7, 0, [gc, gc, t])], [])],
        "zero_length_item": [_upd([(7, 0, [t, item(text("")), o])], [])],
        "noncanonical_clock": [bytes([1, 1, 7, 0x80, 0x00]) + t + bytes([0])],  # clock 0 in two bytes
    }
    return docs


@pytest.mark.parametrize("env", [{}, {"YMERGE_LEAN": 0}, {"YMERGE_LEAN": 0, "YMERGE_IDENTITY": 0}],
                         ids=["default", "no_lean", "no_identity"])
def test_identity_copy_rejects(oracle, env):
    """Every identity-refused shape merges like yrs with the identity copy on and off, and the
    canonical ones are byte-identical to their input."""
    docs = identity_reject_docs()
    e = engine_with(**env)
    try:
        out, off, st = check_batch(e, oracle, batch_of(list(docs.values())))
        for k, name in enumerate(docs):
            if name.startswith("canonical"):
                assert st[k] == 0 and out[int(off[k]):int(off[k + 1])].tobytes() == docs[name][0], name
    finally:
        e.close()
