"""GPU parity of the grid-wide path for long single-client documents (ygiant.hip): the
automerge-paper trace (C1) at the default threshold, and smaller documents forced onto it
(YMERGE_GIANT_MIN, with k_lean off so that they reach the tiled-kernel route), each byte for
byte against the oracle; documents outside the shape (several clients, gaps, duplicates,
empty ranges) must fall back to the tiled kernel and stay exact."""
import pytest

import workloads
from compact_cases import batch_of, var
from test_gpu_parity import check_batch, engine_with

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def forced():
    e = engine_with(YMERGE_LEAN=0, YMERGE_GIANT_MIN=1500)
    yield e
    e.close()


def test_c1_trace_grid_path(oracle):
    b, _ = workloads.trace_updates("automerge-paper")
    e = engine_with()
    check_batch(e, oracle, b)
    st = e.stats()
    assert st["docs_giant"] == 1, st
    e.close()


def test_single_client_documents(forced, oracle):
    b = workloads.text_docs(12, 3000, seed=31, min_clients=1, max_clients=1, del_frac=0.35)
    check_batch(forced, oracle, b)
    assert forced.stats()["docs_giant"] == 12


def test_traces_forced(forced, oracle):
    for name in workloads.TRACES:
        b, _ = workloads.trace_updates(name)
        check_batch(forced, oracle, b)


def test_fallbacks(forced, oracle):
    """Multi-client documents, a duplicated update (overlap), a gap, an empty deleted range:
    the tiled kernel writes them."""
    multi = workloads.text_docs(4, 2500, seed=32, min_clients=2, max_clients=3)
    one = workloads.text_docs(3, 2500, seed=33, min_clients=1, max_clients=1)
    docs = [multi.doc_updates(d) for d in range(multi.n_docs)]
    u = list(one.doc_updates(0))
    docs.append(u[:1200] + u[1100:1300] + u[1200:])      # duplicates
    u = list(one.doc_updates(1))
    docs.append(u[:1000] + u[1010:])                      # a clock gap
    u = list(one.doc_updates(2))
    docs.append(u + [var(0) + var(1) + var(one_client(u)) + var(1) + var(5) + var(0)])  # empty range
    b = batch_of(docs)
    check_batch(forced, oracle, b)
    assert forced.stats()["docs_giant"] == 0


def one_client(ups):
    """The client id of a single-client log (first section header of its first update)."""
    b = bytes(ups[0])
    i = 0

    def rv():
        nonlocal i
        x = s = 0
        while True:
            c = b[i]
            i += 1
            x |= (c & 0x7F) << s
            s += 7
            if c < 0x80:
                return x
    rv()  # sections
    rv()  # blocks
    return rv()


def test_mixed_batch(forced, oracle):
    """Long single-client documents among ordinary ones in one batch."""
    a = workloads.text_docs(3, 2000, seed=34, min_clients=1, max_clients=1)
    c = workloads.text_docs(50, 200, seed=35)
    docs = [a.doc_updates(0)] + [c.doc_updates(d) for d in range(25)] + [a.doc_updates(1)] + \
        [c.doc_updates(d) for d in range(25, 50)] + [a.doc_updates(2)]
    check_batch(forced, oracle, batch_of(docs))
    assert forced.stats()["docs_giant"] == 3


def test_single_document_fallbacks(forced, oracle):
    """One document alone in the batch (the grid lane: k_decode, then the grid kernels) that is
    not the grid shape -- several clients, a gap, duplicates -- must come out of the general
    route exact (the lane's rejection used to be retried on the same document)."""
    multi = workloads.text_docs(1, 2500, seed=34, min_clients=2, max_clients=3)
    one = workloads.text_docs(2, 2500, seed=35, min_clients=1, max_clients=1)
    u0, u1 = list(one.doc_updates(0)), list(one.doc_updates(1))
    for ups in ([bytes(x) for x in multi.doc_updates(0)], u0[:1000] + u0[1010:], u1[:1200] + u1[1100:1300] + u1[1200:]):
        check_batch(forced, oracle, batch_of([ups]))
        assert forced.stats()["docs_giant"] == 0


def test_high_clocks(forced, oracle):
    """A single-client log whose clocks start near 2^32 (the recent tail of a long-lived
    document): the deleted-clock bitmap starts at the smallest deleted clock."""
    from test_gpu_long import section, text, update
    c, k0 = 7777, 3_000_000_000
    ups = []
    for k in range(2400):
        ups.append(update([section(c, k0 + 2 * k, [text("ab")], chained=False)]))
        if k % 10 == 9:
            ups.append(update([], ds=[(c, [(k0 + 2 * k - 7, 3)])]))
    check_batch(forced, oracle, batch_of([ups]))
    assert forced.stats()["docs_giant"] == 1
