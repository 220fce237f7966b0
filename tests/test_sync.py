"""y-sync SyncStep1 / SyncStep2 serving over the update algebra.

Message framing restated from yrs/src/sync/protocol.rs:219-272 (Message::Sync = tag 0,
SyncStep1 = 0 with varbuf(state vector), SyncStep2 = 1 with varbuf(update), tags written
with write_var::<u8>).  Pinned by the reference's own protocol_sync_steps test
(protocol.rs:409-444): client 1 pushes "hello" into text "test"; the reply to a
SyncStep1 with an empty state vector is SyncStep2 of exactly that document's update."""
import numpy as np
import pytest

from test_gpu_parity import _var

HELLO = bytes([1, 1, 1, 0, 4, 1, 4]) + b"test" + bytes([5]) + b"hello" + bytes([0])


def msg_step1(sv):
    return bytes([0, 0]) + _var(len(sv)) + sv


def test_protocol_sync_steps_kat(oracle):
    reply = oracle.sync_step2_v1(HELLO, msg_step1(b"\x00"))
    assert reply == bytes([0, 1]) + _var(len(HELLO)) + HELLO
    assert oracle.sync_step1_v1(HELLO) == bytes([0, 0, 3, 1, 1, 5])


def test_sync_messages(oracle):
    st, _ = oracle.status_of(oracle.sync_step2_v1, HELLO, bytes([1, 0]))  # awareness: not served
    assert st == 21
    st, _ = oracle.status_of(oracle.sync_step2_v1, HELLO, bytes([0, 1, 0]))  # SyncStep2 from the client
    assert st == 21
    st, _ = oracle.status_of(oracle.sync_step2_v1, HELLO, bytes([0, 7, 0]))
    assert st == 4  # SyncMessage::decode: unknown tag
    st, _ = oracle.status_of(oracle.sync_step2_v1, HELLO, bytes([0, 0, 5, 1]))
    assert st == 3  # varbuf past the end
    st, _ = oracle.status_of(oracle.sync_step2_v1, HELLO, bytes([0x80, 0x02]))
    assert st == 2  # tag 256: read_var::<u8> fails
    # a partial remote state vector: the reply carries the diff
    r = oracle.sync_step2_v1(HELLO, msg_step1(bytes([1, 1, 3])))
    assert r == bytes([0, 1]) + _var(len(oracle.diff_updates_v1(HELLO, bytes([1, 1, 3])))) + \
        oracle.diff_updates_v1(HELLO, bytes([1, 1, 3]))


def _sync_cases(oracle):
    import workloads
    b = workloads.text_docs(40, 300, seed=9)
    m, off, st = oracle.merge_batch(b.data, b.upd_off, b.doc_upd, mode=1, threads=4)
    ups = [m[int(off[d]):int(off[d + 1])] for d in range(b.n_docs)] + [HELLO] * 6
    svs = [oracle.encode_state_vector_from_update_v1(u) for u in ups[:40]]
    rsv, rsv_off = workloads.remote_svs(np.frombuffer(b"".join(svs), np.uint8),
                                        np.concatenate([[0], np.cumsum([len(s) for s in svs])]).astype(np.uint64))
    msgs = [msg_step1(rsv[int(rsv_off[d]):int(rsv_off[d + 1])].tobytes()) for d in range(40)]
    msgs += [msg_step1(b"\x00"), bytes([1, 0]), bytes([0, 1, 0]), bytes([0, 7, 0]), bytes([0, 0, 5, 1]),
             msg_step1(b"\x00") + b"trailing"]
    return ups, msgs


@pytest.mark.gpu
def test_gpu_sync_step2_and_step1(oracle):
    import ymerge
    ups, msgs = _sync_cases(oracle)
    e = ymerge.Engine(0)
    try:
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
            assert st[d] == 0 and out[int(off[d]):int(off[d + 1])].tobytes() == oracle.sync_step1_v1(u)
    finally:
        e.close()
