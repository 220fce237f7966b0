"""GPU parity of k_lean (ymerge_lean.hip: one wavefront per document) at the edges of the
shape it accepts, and of its hand-over to k_decode + k_fast_merge for everything else.
Every batch is checked byte for byte against the CPU oracle; the stats show which path
wrote the documents."""
import numpy as np
import pytest

from test_gpu_parity import batch_of, check_batch, engine, engine_with  # noqa: F401 (engine: fixture)

pytestmark = pytest.mark.gpu


def var(x):
    out = bytearray()
    while True:
        b, x = x & 0x7F, x >> 7
        if x:
            out.append(b | 0x80)
        else:
            out.append(b)
            return bytes(out)


def vstr(s):
    b = s.encode() if isinstance(s, str) else bytes(s)
    return var(len(b)) + b


def item(text=None, origin=None, right=None, root="t", parent=None, sub=None, deleted=None):
    """One Item block (yrs/src/update.rs:433-488 decode_block, block.rs:1363-1369 info)."""
    ref = 1 if deleted is not None else 4
    info = ref | (0x80 if origin else 0) | (0x40 if right else 0)
    body = b""
    if origin:
        body += var(origin[0]) + var(origin[1])
    if right:
        body += var(right[0]) + var(right[1])
    if not origin and not right:
        if sub is not None:
            info |= 0x20
        body += (var(1) + vstr(root)) if parent is None else (var(0) + var(parent[0]) + var(parent[1]))
        if sub is not None:
            body += vstr(sub)
    body += var(deleted) if deleted is not None else vstr(text)
    return bytes([info]) + body


def gc(n):
    return bytes([0]) + var(n)


def skip(n):
    return bytes([10]) + var(n)


def upd(client=None, clock=0, block=None, ds=()):
    """v1 update: <= 1 client section with <= 1 block, then the DeleteSet [(client, [(s, n)])]."""
    b = bytearray()
    if client is None:
        b += var(0)
    else:
        b += var(1) + var(1 if block is not None else 0) + var(client) + var(clock)
        if block is not None:
            b += block
    b += var(len(ds))
    for c, rs in ds:
        b += var(c) + var(len(rs))
        for s, n in rs:
            b += var(s) + var(n)
    return bytes(b)


def text_log(rng, clients, n, maxlen=8, del_frac=0.2, ds_clients=None):
    """A synced editing log: per client contiguous clocks, deletes of earlier content."""
    clocks = {c: 0 for c in clients}
    made = []
    ups = []
    for _ in range(n):
        if made and rng.random() < del_frac:
            k = int(rng.integers(1, 4))
            ents = {}
            for _ in range(k):
                c, s, ln = made[int(rng.integers(len(made)))]
                a = s + int(rng.integers(ln))
                ents.setdefault(c, []).append((a, int(rng.integers(1, s + ln - a + 1))))
            ups.append(upd(ds=list(ents.items())[:4]))
            continue
        c = clients[int(rng.integers(len(clients)))]
        t = "".join(chr(97 + int(x)) for x in rng.integers(0, 26, int(rng.integers(1, maxlen + 1))))
        blk = item(t, origin=(c, clocks[c] - 1) if clocks[c] else None) if clocks[c] else item(t)
        ups.append(upd(c, clocks[c], blk))
        made.append((c, clocks[c], len(t)))
        clocks[c] += len(t)
    return ups


def run(engine, oracle, docs):
    check_batch(engine, oracle, batch_of(docs))
    return engine.stats()


def test_lean_shapes_accepted(engine, oracle):
    """Documents k_lean must write itself (all lean, byte-exact)."""
    rng = np.random.default_rng(0x1EA4)
    docs = [
        [upd(7, 0, item("ab")), upd(7, 2, item("c", origin=(7, 1))), upd(3, 0, item("xyz"))],
        [upd(5, 0, gc(3)), upd(5, 3, gc(2)), upd(5, 5, item("q"))],                 # GC runs
        [upd(5, 0, item(deleted=4)), upd(5, 4, item(deleted=1))],                    # Deleted content
        [upd(9, 0, item("k", sub="key")), upd(9, 1, item("m", parent=(9, 0)))],      # parent_sub, ID parent
        [upd(4, 0, item("abcdef")), upd(8, 0, item("0123456789ab")),
         upd(ds=[(4, [(0, 3)])]), upd(ds=[(4, [(3, 2)]), (8, [(10, 1)])])],          # DeleteSets
        [upd(1, 0, item("a")), upd(ds=[(1, [(0, 1)])]), upd(ds=[(1, [(0, 1)])])],     # duplicate ranges
        [upd(2, 0, item("")), upd(2, 0, item("abc"))],                               # zero-length item dropped
        [upd(2, 0, skip(5)), upd(2, 0, item("abc"))],                                # Skip dropped
        [upd(2, 0, None), upd(2, 0, item("abc"))],                                   # empty section
        [upd(6, 0, item("x" * 1000))],                                              # block of ~1 KB
        [upd(c, 0, item("z")) for c in range(16)],                                   # 16 clients
        [upd(c, 0, item("xyzw" * 4)) for c in (11, 5, 1 << 31, 2)]
        + [upd(ds=[(c, [(c % 7, 1)]) for c in (11, 5, 1 << 31, 2)])],                # 4 entries, table order
        [upd(3, 0, item("a" * 600)), upd(3, 600, item("b" * 300)),
         upd(ds=[(3, [(10, 700)])]), upd(ds=[(3, [(2, 3), (5, 255), (260, 256)])])],  # ranges > 255 split
        [bytes([1, 1, 0x86, 0, 0, 0x04, 1, 1, ord("t"), 1, ord("a"), 0])],           # non-canonical client
        [upd(3, 0, item("abcdefgh" * 12))] + [upd(3, 96 + i, item("b")) for i in range(200)],
    ]
    for n in (1, 5, 63, 64, 65, 130, 700, 1000):
        docs.append(text_log(rng, [int(x) for x in rng.integers(0, 2 ** 32, int(rng.integers(1, 6)))], n))
    st = run(engine, oracle, docs)
    assert st["docs_lean"] == len(docs), st


def test_lean_shapes_handed_over(engine, oracle):
    """Documents outside the shape: k_lean hands every one over and the result is exact."""
    docs = [
        [upd(5, 0, item("ab")), upd(5, 3, item("c"))],                               # clock gap -> Skip
        [upd(5, 2, item("c")), upd(5, 0, item("ab"))],                               # out of order
        [upd(5, 0, item("ab")), upd(5, 0, item("ab"))],                              # duplicate update
        [upd(5, 0, item("ab")), upd(5, 1, item("bc"))],                              # overlap -> splice
        [upd(c, 0, item("z")) for c in range(17)],                                   # 17 clients
        [upd(ds=[(c, [(c, 1)]) for c in range(5)])],                                 # 5 entries
        [upd(ds=[(4, [(0, 1)]), (4, [(5, 1)])])],                                    # repeated client
        [upd(ds=[(4, [(0, 0)])])],                                                   # empty range
        [upd(ds=[(4, [])])],                                                         # entry without ranges
        [upd(6, 0, item("x" * 1030))],                                              # block > 1 KB
        [upd(6, 0, item("é"))],                                                      # non-ASCII string
        [upd(6, 0, gc(0))],                                                          # zero-length GC
        [upd(ds=[(4, [(0, 1)])]), upd(ds=[(4, [(3_000_000, 1)])])],                 # DS without blocks
        [upd(4, 5, item("abc")), upd(ds=[(4, [(0, 3)])])],                          # range below the blocks
        [upd(4, 0, item("abc")), upd(ds=[(4, [(0, 1)]), (9, [(0, 1)])])],           # client without blocks
        [b""],                                                                       # EOS
        [upd(6, 0, item("ab"))[:-2]],                                                # truncated
        [bytes([1, 1, 6, 0, 0x04, 1, 1, ord("t"), 0x81, 0, ord("a"), 0])],           # non-canonical length
        [],                                                                          # no updates
    ]
    st = run(engine, oracle, docs)
    assert st["docs_lean"] == 0, st


def test_lean_large_documents(engine, oracle):
    """Around the 64 KB document limit and the 2 KB round stage (updates of ~100 B: rounds
    shorter than 64 updates), plus the arena limit (many DeleteSet ranges)."""
    rng = np.random.default_rng(0xB16)
    docs = []
    for n in (600, 660):  # ~100 B per update: ~60 KB and ~66 KB
        ups, clock = [], 0
        for i in range(n):
            t = "".join(chr(97 + int(x)) for x in rng.integers(0, 26, 90))
            ups.append(upd(1, clock, item(t, origin=(1, clock - 1) if clock else None)))
            clock += len(t)
        docs.append(ups)
    ups = [upd(1, 0, item("x" * 500))]
    for i in range(400):  # 400 updates x 2 ranges: 1600 arena words > the arena
        ups.append(upd(ds=[(1, [(i, 1), (i + 100, 1)])]))
    docs.append(ups)
    docs.append(ups[:300])
    check_batch(engine, oracle, batch_of(docs))


def test_lean_matches_fast_path(oracle):
    """C2 and C3 batches: k_lean on and off give the same bytes (and the oracle's)."""
    import workloads
    for b in (workloads.text_docs(200, 1000, seed=3), workloads.zipf_docs(3000, seed=0x5EED + 1)):
        e0 = engine_with(YMERGE_LEAN=0)
        try:
            o0, f0, s0 = check_batch(e0, oracle, b)
        finally:
            e0.close()
        e1 = engine_with(YMERGE_LEAN=1)
        try:
            o1, f1, s1 = check_batch(e1, oracle, b)
            assert e1.stats()["docs_lean"] > 0
        finally:
            e1.close()
        assert o0.tobytes() == o1.tobytes() and np.array_equal(f0, f1) and np.array_equal(s0, s1)


def test_lean_big_documents(engine, oracle):
    """k_lean's BIG mode (documents above the LDS arena: > 1280 updates or >= 64 KB; tables
    in HBM scratch): multi-client editing logs of 1,281 - 12,000 updates, ~100 B updates
    past 64 KB, DeleteSet-heavy logs; all written by k_lean, byte-exact."""
    rng = np.random.default_rng(0xB1C)
    docs = []
    for n in (1281, 2000, 5000, 12000):
        cl = [int(x) for x in rng.integers(0, 2 ** 32, int(rng.integers(1, 6)))]
        docs.append(text_log(rng, cl, n))
    docs.append(text_log(rng, [7], 3000, del_frac=0.6))
    ups, clock = [], 0
    for i in range(700):  # ~100 B per update: ~70 KB with 700 updates
        t = "".join(chr(97 + int(x)) for x in rng.integers(0, 26, 90))
        ups.append(upd(1, clock, item(t, origin=(1, clock - 1) if clock else None)))
        clock += len(t)
    docs.append(ups)
    ups = [upd(1, 0, item("x" * 500))]
    for i in range(400):  # 400 updates x 2 ranges
        ups.append(upd(ds=[(1, [(i, 1), (i + 100, 1)])]))
    docs.append(ups)
    docs.append([upd(3, 0, item("a" * 600)), upd(3, 600, item("b" * 300))] +
                [upd(ds=[(3, [(2 * (i % 450), 1)])]) for i in range(1500)])  # 450 components
    # (a batch of <= 64 documents hands its documents of >= 4,096 updates to the grid path /
    # tiled kernel, ykernels.h GS_SMALL_DOCS: small documents make this a large batch)
    docs += [[upd(100 + k, 0, item("z"))] for k in range(64)]
    st = run(engine, oracle, docs)
    assert st["docs_lean"] == len(docs), st


def test_small_batch_long_documents(engine, oracle):
    """A batch of <= 64 documents: its documents of >= 4,096 updates skip k_lean (the grid path
    for one client, the tiled kernel otherwise), the others stay lean; byte-exact either way."""
    rng = np.random.default_rng(0x5B)
    docs = [text_log(rng, [11], 5000), text_log(rng, [12, 13], 4500), text_log(rng, [14], 4095),
            text_log(rng, [15, 16, 17], 300)]
    st = run(engine, oracle, docs)
    assert st["docs_lean"] == 2 and st["docs_giant"] == 1, st


def test_lean_c3_zipf(engine, oracle):
    """C3-shaped batch (Zipf update counts up to 10^4): every document lean, byte-exact."""
    import workloads
    b = workloads.zipf_docs(4000, seed=0x5EED)
    assert int((np.diff(b.doc_upd) > 1280).sum()) > 10
    check_batch(engine, oracle, b)
    st = engine.stats()
    assert st["docs_lean"] == b.n_docs and st["docs_exact"] == 0 and st["docs_big"] == 0, st



def test_lean_scratch_unavailable_degrades(oracle):
    """No k_lean BIG-mode scratch (env YMERGE_LEAN_SCR_MAX=0 stands in for a failed hipMalloc):
    the BIG documents are handed over to the fast/tiled path and the batch is still exact."""
    rng = np.random.default_rng(0x5C4)
    docs = [text_log(rng, [3, 9], 2000), text_log(rng, [5], 300), text_log(rng, [1, 2, 4], 1500)]
    e = engine_with(YMERGE_LEAN_SCR_MAX=0)
    try:
        check_batch(e, oracle, batch_of(docs))
        st = e.stats()
        assert st["docs_lean"] == 1, st  # the 300-update document fits LDS
    finally:
        e.close()


def test_stage_timing_off(engine, oracle):
    """ymerge_ctx_set_stage_timing(ctx, 0): a merge k_lean writes whole records no stage
    events (the stats' times read 0) and writes the same bytes; on again, the times return."""
    rng = np.random.default_rng(0x71)
    docs = [text_log(rng, [1, 2], 300) for _ in range(8)]
    try:
        engine.set_stage_timing(False)
        st = run(engine, oracle, docs)
        assert st["docs_lean"] == len(docs) and st["ms_lean"] == 0.0, st
    finally:
        engine.set_stage_timing(True)
    st = run(engine, oracle, docs)
    assert st["docs_lean"] == len(docs) and st["ms_lean"] > 0.0, st
