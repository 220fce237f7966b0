"""ContentMove (content ref 11) and TypeRef::WeakLink (type ref 7, the `weak` feature yffi
builds with) through merge / diff / state vector, oracle and GPU.

Vectors are built from the reference grammar — Move::decode/encode
(yrs/src/moving.rs:277-333: flags as a signed i32 varint, is_collapsed when start == end,
priority = flags >> 6) and TypeRef::decode/encode (yrs/src/types/mod.rs:118-200: u8
flags, is_single when start == end).  No Yjs emits either, so the expected bytes are
hand-derived from those functions; the GPU must equal the oracle on all of them."""
import numpy as np
import pytest

from test_gpu_parity import batch_of, check_batch


def var(x):
    o = bytearray()
    while True:
        b, x = x & 0x7F, x >> 7
        o.append(b | (0x80 if x else 0))
        if not x:
            return bytes(o)


def svar(v):  # lib0 signed varint (varint.rs:184-226 write_var_i64)
    neg = v < 0
    v = -v if neg else v
    o = bytearray([(0x80 if v > 63 else 0) | (0x40 if neg else 0) | (v & 63)])
    v >>= 6
    while v > 0:
        o.append((0x80 if v > 127 else 0) | (v & 127))
        v >>= 7
    return bytes(o)


def item_update(client, clock, ref, content, parent=b"arr"):
    body = bytes([ref]) + var(1) + var(len(parent)) + parent + content
    return var(1) + var(1) + var(client) + var(clock) + body + var(0)


def move(flags, sc, sk, ec=None, ek=None):
    c = svar(flags) + var(sc) + var(sk)
    if ec is not None:
        c += var(ec) + var(ek)
    return c


def weak(flags, sc, sk, ec=None, ek=None):
    c = bytes([7, flags]) + var(sc) + var(sk)
    if ec is not None:
        c += var(ec) + var(ek)
    return c


# (input update, expected merge_updates_v1 output or error code)
CASES = [
    (item_update(9, 0, 11, move(1, 5, 3)), item_update(9, 0, 11, move(1, 5, 3))),
    (item_update(9, 0, 11, move(0, 5, 3, 5, 3)), item_update(9, 0, 11, move(1, 5, 3))),  # start == end: collapsed
    (item_update(9, 0, 11, move(0, 5, 3, 6, 4)), item_update(9, 0, 11, move(0, 5, 3, 6, 4))),
    (item_update(9, 0, 11, move(2 | 4 | (3 << 6), 1 << 40, 7, 2, 2)),
     item_update(9, 0, 11, move(2 | 4 | (3 << 6), 1 << 40, 7, 2, 2))),
    (item_update(9, 0, 11, move(-64 | 1, 5, 3)), item_update(9, 0, 11, move(-64 | 1, 5, 3))),  # priority -1
    (item_update(9, 0, 11, move(8 | 1, 5, 3)), item_update(9, 0, 11, move(1, 5, 3))),  # bit 3 not re-emitted
    (item_update(9, 0, 11, svar(1 << 40) + var(5) + var(3)), 2),  # flags beyond i32: InvalidVarInt
    (item_update(9, 0, 11, move(0, 5, 3)), 3),  # end id missing: EndOfBuffer
    (item_update(9, 0, 7, weak(0, 5, 3)), item_update(9, 0, 7, weak(0, 5, 3))),
    (item_update(9, 0, 7, weak(1 | 2 | 4, 5, 3, 5, 9)), item_update(9, 0, 7, weak(1 | 2 | 4, 5, 3, 5, 9))),
    (item_update(9, 0, 7, weak(1 | 2, 5, 3, 5, 3)), item_update(9, 0, 7, weak(2, 5, 3))),  # start == end: single
    (item_update(9, 0, 7, weak(8, 5, 3)), item_update(9, 0, 7, weak(0, 5, 3))),  # flag bit 3 dropped
    (item_update(9, 0, 7, bytes([7, 1]) + var(5)), 3),
]


def test_oracle_move_weak(oracle):
    for u, want in CASES:
        st, m = oracle.status_of(oracle.merge_updates_v1, [u])
        if isinstance(want, int):
            assert st == want, u.hex()
        else:
            assert st == 0 and m == want, (u.hex(), m and m.hex(), want.hex())
            # merging with a neighbour block (a later clock of the same client) keeps the bytes
            nxt = item_update(9, 1, 4, var(2) + b"ab")
            m2 = oracle.merge_updates_v1([nxt, u])
            assert want[4:-1] in m2
            assert oracle.diff_updates_v1(m, b"\x00") == m
            assert oracle.encode_state_vector_from_update_v1(m) == var(1) + var(9) + var(1)


def _docs():
    docs = [[u] for u, _ in CASES]
    docs += [[item_update(9, 1, 4, var(2) + b"ab"), u] for u, w in CASES if not isinstance(w, int)]
    return docs


@pytest.mark.gpu
def test_gpu_move_weak_merge(oracle):
    import ymerge
    e = ymerge.Engine(0)
    try:
        check_batch(e, oracle, batch_of(_docs()))
    finally:
        e.close()


@pytest.mark.gpu
def test_gpu_move_weak_sv_diff(oracle):
    import ymerge
    e = ymerge.Engine(0)
    try:
        ups = [u for u, w in CASES]
        data = np.frombuffer(b"".join(ups), np.uint8)
        offs = np.concatenate([[0], np.cumsum([len(u) for u in ups])]).astype(np.uint64)
        sv, sv_off, st = e.state_vector_host(data, offs)
        esv, esv_off, est = oracle.sv_batch(data, offs, threads=2)
        assert np.array_equal(st, est) and sv.tobytes() == esv
        rsv = b"".join([b"\x00"] * len(ups))
        rsv_off = np.arange(len(ups) + 1, dtype=np.uint64)
        df, df_off, dst = e.diff_host(data, offs, np.frombuffer(rsv, np.uint8), rsv_off)
        edf, edf_off, edst = oracle.diff_batch(data, offs, np.frombuffer(rsv, np.uint8), rsv_off, threads=2)
        assert np.array_equal(dst, edst) and df.tobytes() == edf
    finally:
        e.close()
