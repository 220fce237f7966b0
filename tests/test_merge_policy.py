"""Oracle: the literal yrs loop (mode 0: a full re-sort of the live decoders every
iteration, update.rs:565-697) and the heap form (mode 1) agree on documents with
partial overlaps and Item-vs-GC same-clock ties, on both sides of the 20-decoder
insertion-sort threshold (yrs_oracle.c merge_blocks)."""
import numpy as np

from overlaps import overlap_docs, update


def test_literal_and_heap_agree(oracle):
    for seed in range(6):
        for k, ups in enumerate(overlap_docs(seed)):
            a = oracle.merge_updates_v1(ups, mode=0)
            b = oracle.merge_updates_v1(ups, mode=1)
            assert a == b, (seed, k)


def test_small_anomaly_is_literal_insertion_sort(oracle):
    """<= 20 live decoders: Rust's insertion_sort_shift_left with yrs' comparator.  Input
    order [GC@0 len 4, Item@0 len 2]: the Item is 'Less' than the GC (different types at
    one clock) and moves first, so the merge writes Item[0,2) then the GC spliced to [2,4)."""
    gc = update([(7, 0, [("g", 4)])])
    it = update([(7, 0, [("i", "ab")])])
    m = oracle.merge_updates_v1([gc, it], mode=0)
    assert m == oracle.merge_updates_v1([gc, it], mode=1)
    # clients 1, blocks 2, client 7 clock 0: Item "ab" then GC len 2; empty DeleteSet
    assert m == bytes([1, 2, 7, 0, 0x04, 1, 1]) + b"t" + bytes([2]) + b"ab" + bytes([0, 2, 0])
    # and the other input order flips it back: GC first (insertion sort moves the GC)
    m2 = oracle.merge_updates_v1([it, gc], mode=0)
    assert m2 == bytes([1, 1, 7, 0, 0, 4, 0])


def test_large_anomaly_policy(oracle):
    """> 20 live decoders: stable sort with the Item/GC tie read as Equal (policy), so the
    earlier input keeps its place: GC first -> one GC[0,4) covers the Item."""
    # 25 one-block updates of a LOWER client: still live when client 7's tie is sorted
    fill = [update([(3, 100 + 10 * i, [("i", "x")])]) for i in range(25)]
    gc = update([(7, 0, [("g", 4)])])
    it = update([(7, 0, [("i", "ab")])])
    m = oracle.merge_updates_v1([gc, it] + fill, mode=0)
    assert m == oracle.merge_updates_v1([gc, it] + fill, mode=1)
    # clients 2; client 7 first (descending): 1 block, clock 0, GC len 4
    assert m.startswith(bytes([2, 1, 7, 0, 0, 4]))
    # and with <= 20 decoders the same pair is spliced (literal insertion sort)
    assert oracle.merge_updates_v1([gc, it] + fill[:18], mode=1).startswith(bytes([2, 2, 7, 0, 0x04]))
