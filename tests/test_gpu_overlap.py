"""GPU parity on overlapping documents (snapshot + pending log shapes): partial overlaps,
same-clock blocks of different lengths, Item-vs-GC ties on both sides of the 20-decoder
insertion-sort threshold (tests/overlaps.py; policy in DESIGN.md §3), and full-size C4
documents.  Reference semantics: yrs/src/update.rs:537-704."""
import pytest

import workloads
from overlaps import overlap_docs
from test_gpu_parity import batch_of, check_batch

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def engine():
    import ymerge
    e = ymerge.Engine(0)
    yield e
    e.close()


@pytest.mark.parametrize("seed", [1, 2, 3])
def test_overlap_docs(engine, oracle, seed):
    check_batch(engine, oracle, batch_of(overlap_docs(seed)))
    print(engine.stats())


def test_c4_full_size_docs(engine, oracle):
    """C4 at its stated 5,000 ops per document (GC'd snapshot + log, withheld and
    duplicated updates)."""
    b = workloads.delete_heavy_docs(48, ops_per_doc=5000)
    check_batch(engine, oracle, b)
    st = engine.stats()
    print(st)
    assert st["docs_overlap"] >= 40, st  # run order + splices on the tiled kernel
    assert st["docs_exact"] <= 4, st     # only Item/GC ties in the insertion-sort tail
