"""Long single updates (>= 2 KB, beyond k_decode's 16 KB stage once several share a workgroup):
k_decode_huge walks each with a whole wavefront over an LDS window and writes its record (and
overflow words) for every merge kernel.  GPU == oracle byte for byte on merged editing traces
taken as one update each (many blocks, DeleteSets), their truncations
(decode errors at every stage of the grammar), several long updates in one document, long
updates next to short ones, non-ASCII text, and the reference's b4-update.bin."""
import numpy as np
import pytest

import corpus
import workloads
from test_gpu_parity import batch_of, check_batch

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def engine():
    import ymerge
    e = ymerge.Engine(0)
    yield e
    e.close()


def _trace_merge(oracle, name, n, client=1):
    b, _ = workloads.trace_updates(name, client)
    ups = b.doc_updates(0)[:n]
    return oracle.merge_updates_v1([bytes(u) for u in ups], mode=1)


def test_long_updates_merged_traces(engine, oracle):
    longs = [_trace_merge(oracle, t, n, c) for t, n, c in
             (("sveltecomponent", 900, 1), ("rustcode", 400, 1), ("sveltecomponent", 500, 1),
              ("friendsforever_flat", 500, 1), ("friendsforever_flat", 1200, 1))]
    assert all(len(u) >= 2048 for u in longs)
    docs = [[u] for u in longs]
    docs.append(longs[:3])                       # several long updates in one document
    docs.append([longs[0], b"\x00\x00", longs[1][:100]])
    docs.append([u[: len(u) // 2] for u in longs[:2]])   # truncated: decode errors
    docs.append([longs[4][:-1]])
    check_batch(engine, oracle, batch_of(docs))


def test_long_update_truncations(engine, oracle):
    u = _trace_merge(oracle, "sveltecomponent", 700)
    cuts = sorted({len(u) - k for k in (1, 2, 3, 5, 8, 13, 40, 200)} | {2048 + k for k in range(0, 40, 3)})
    check_batch(engine, oracle, batch_of([[u[:c]] for c in cuts if c >= 2048]))


def test_long_updates_among_short(engine, oracle):
    long_ = _trace_merge(oracle, "friendsforever_flat", 800)
    small = workloads.text_docs(6, 300, seed=99)
    docs = []
    for d in range(small.n_docs):
        ups = [bytes(x) for x in small.doc_updates(d)]
        docs.append(ups[:100] + [long_] + ups[100:])
    check_batch(engine, oracle, batch_of(docs))


def test_b4_with_others(engine, oracle):
    u = corpus.b4_update()
    m = _trace_merge(oracle, "rustcode", 500)
    check_batch(engine, oracle, batch_of([[m], [u], [m, u], [u[:350_000]]]))
