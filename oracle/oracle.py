"""TEST INFRASTRUCTURE ONLY — ctypes front-end of the CPU oracle (yrs_oracle.c).

Restates yrs 0.19.2 merge_updates_v1 / diff_updates_v1 /
encode_state_vector_from_update_v1 (yrs/src/alt.rs:15-81).  Only tests/,
__graft_entry__.smoke() and bench.py's cpu_baseline leg may import this.
"""
import ctypes
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB = os.path.join(_HERE, "libyrs_oracle.so")


def build():
    subprocess.check_call(["make", "-s", "-C", _HERE])


def _load():
    if not os.path.exists(_LIB):
        build()
    lib = ctypes.CDLL(_LIB)
    P = ctypes.POINTER
    u8p = P(ctypes.c_uint8)
    lib.yo_merge_updates_v1.argtypes = [P(u8p), P(ctypes.c_size_t), ctypes.c_size_t, ctypes.c_int,
                                        P(u8p), P(ctypes.c_size_t)]
    lib.yo_diff_updates_v1.argtypes = [u8p, ctypes.c_size_t, u8p, ctypes.c_size_t, P(u8p),
                                       P(ctypes.c_size_t)]
    lib.yo_encode_state_vector_from_update_v1.argtypes = [u8p, ctypes.c_size_t, P(u8p),
                                                          P(ctypes.c_size_t)]
    lib.yo_free.argtypes = [ctypes.c_void_p]
    vp = ctypes.c_void_p
    lib.yo_merge_batch.argtypes = [vp, vp, vp, ctypes.c_size_t, ctypes.c_int, ctypes.c_int,
                                   P(u8p), vp, vp]
    lib.yo_diff_batch.argtypes = [vp, vp, vp, vp, ctypes.c_size_t, ctypes.c_int, P(u8p), vp, vp]
    lib.yo_sv_batch.argtypes = [vp, vp, ctypes.c_size_t, ctypes.c_int, P(u8p), vp, vp]
    return lib


_lib = None


def lib():
    global _lib
    if _lib is None:
        _lib = _load()
    return _lib


class OracleError(Exception):
    def __init__(self, code):
        super().__init__(f"oracle status {code}")
        self.code = code


def _buf(b):
    b = bytes(b)
    arr = (ctypes.c_uint8 * max(1, len(b))).from_buffer_copy(b if b else b"\0")
    return arr, len(b)


def _take(out, n):
    res = ctypes.string_at(out, n.value) if n.value else b""
    lib().yo_free(out)
    return res


def merge_updates_v1(updates, mode=0):
    """mode 0: literal reference loop; mode 1: equivalent fast form."""
    bufs = [_buf(u) for u in updates]
    n = len(bufs)
    ptrs = (ctypes.POINTER(ctypes.c_uint8) * max(1, n))(*[ctypes.cast(b[0], ctypes.POINTER(ctypes.c_uint8)) for b in bufs])
    lens = (ctypes.c_size_t * max(1, n))(*[b[1] for b in bufs])
    out = ctypes.POINTER(ctypes.c_uint8)()
    olen = ctypes.c_size_t()
    st = lib().yo_merge_updates_v1(ptrs, lens, n, mode, ctypes.byref(out), ctypes.byref(olen))
    if st:
        raise OracleError(st)
    return _take(out, olen)


def compact_updates_v1(updates):
    """Store-based compaction (yrs_oracle_store.c): a Doc (GC on) applies the updates in order,
    one transaction each, then encode_state_as_update_v1 (yrs/src/transaction.rs:73-85)."""
    bufs = [_buf(u) for u in updates]
    n = len(bufs)
    ptrs = (ctypes.POINTER(ctypes.c_uint8) * max(1, n))(*[ctypes.cast(b[0], ctypes.POINTER(ctypes.c_uint8)) for b in bufs])
    lens = (ctypes.c_size_t * max(1, n))(*[b[1] for b in bufs])
    out = ctypes.POINTER(ctypes.c_uint8)()
    olen = ctypes.c_size_t()
    st = lib().yo_compact_updates_v1(ptrs, lens, n, ctypes.byref(out), ctypes.byref(olen))
    if st:
        raise OracleError(st)
    return _take(out, olen)


def diff_updates_v1(update, sv):
    a, an = _buf(update)
    b, bn = _buf(sv)
    out = ctypes.POINTER(ctypes.c_uint8)()
    olen = ctypes.c_size_t()
    st = lib().yo_diff_updates_v1(a, an, b, bn, ctypes.byref(out), ctypes.byref(olen))
    if st:
        raise OracleError(st)
    return _take(out, olen)


def encode_state_vector_from_update_v1(update):
    a, an = _buf(update)
    out = ctypes.POINTER(ctypes.c_uint8)()
    olen = ctypes.c_size_t()
    st = lib().yo_encode_state_vector_from_update_v1(a, an, ctypes.byref(out), ctypes.byref(olen))
    if st:
        raise OracleError(st)
    return _take(out, olen)


def merge_updates_v2(updates, mode=1, inputs_v1=False):
    """lib0 v2 merge (yrs/src/alt.rs:35-48).  inputs_v1: v1 inputs, the merged Update encoded
    with EncoderV2 (Update::merge_updates(decode_v1 each).encode_v2())."""
    bufs = [_buf(u) for u in updates]
    n = len(bufs)
    ptrs = (ctypes.POINTER(ctypes.c_uint8) * max(1, n))(*[ctypes.cast(b[0], ctypes.POINTER(ctypes.c_uint8)) for b in bufs])
    lens = (ctypes.c_size_t * max(1, n))(*[b[1] for b in bufs])
    out = ctypes.POINTER(ctypes.c_uint8)()
    olen = ctypes.c_size_t()
    L = lib()
    fn = L.yo_merge_updates_v1_to_v2 if inputs_v1 else L.yo_merge_updates_v2
    fn.argtypes = L.yo_merge_updates_v1.argtypes
    st = fn(ptrs, lens, n, mode, ctypes.byref(out), ctypes.byref(olen))
    if st:
        raise OracleError(st)
    return _take(out, olen)


def diff_updates_v2(update, sv):
    a, an = _buf(update)
    b, bn = _buf(sv)
    out = ctypes.POINTER(ctypes.c_uint8)()
    olen = ctypes.c_size_t()
    L = lib()
    L.yo_diff_updates_v2.argtypes = L.yo_diff_updates_v1.argtypes
    st = L.yo_diff_updates_v2(a, an, b, bn, ctypes.byref(out), ctypes.byref(olen))
    if st:
        raise OracleError(st)
    return _take(out, olen)


def encode_state_vector_from_update_v2(update):
    a, an = _buf(update)
    out = ctypes.POINTER(ctypes.c_uint8)()
    olen = ctypes.c_size_t()
    L = lib()
    L.yo_encode_state_vector_from_update_v2.argtypes = L.yo_encode_state_vector_from_update_v1.argtypes
    st = L.yo_encode_state_vector_from_update_v2(a, an, ctypes.byref(out), ctypes.byref(olen))
    if st:
        raise OracleError(st)
    return _take(out, olen)


def _convert(fn, update):
    a, an = _buf(update)
    out = ctypes.POINTER(ctypes.c_uint8)()
    olen = ctypes.c_size_t()
    f = getattr(lib(), fn)
    f.argtypes = lib().yo_encode_state_vector_from_update_v1.argtypes
    st = f(a, an, ctypes.byref(out), ctypes.byref(olen))
    if st:
        raise OracleError(st)
    return _take(out, olen)


def convert_update_v1_to_v2(update):
    """Update::decode_v1(u).encode_v2() (test helper)."""
    return _convert("yo_convert_update_v1_to_v2", update)


def convert_update_v2_to_v1(update):
    """Update::decode_v2(u).encode_v1() (test helper)."""
    return _convert("yo_convert_update_v2_to_v1", update)


def sync_step1_v1(update):
    a, an = _buf(update)
    L = lib()
    L.yo_sync_step1_v1.argtypes = [ctypes.POINTER(ctypes.c_uint8), ctypes.c_size_t,
                                   ctypes.POINTER(ctypes.POINTER(ctypes.c_uint8)), ctypes.POINTER(ctypes.c_size_t)]
    out = ctypes.POINTER(ctypes.c_uint8)()
    olen = ctypes.c_size_t()
    st = L.yo_sync_step1_v1(a, an, ctypes.byref(out), ctypes.byref(olen))
    if st:
        raise OracleError(st)
    return _take(out, olen)


def sync_step2_v1(update, msg):
    a, an = _buf(update)
    b, bn = _buf(msg)
    L = lib()
    P = ctypes.POINTER
    L.yo_sync_step2_v1.argtypes = [P(ctypes.c_uint8), ctypes.c_size_t, P(ctypes.c_uint8), ctypes.c_size_t,
                                   P(P(ctypes.c_uint8)), P(ctypes.c_size_t)]
    out = ctypes.POINTER(ctypes.c_uint8)()
    olen = ctypes.c_size_t()
    st = L.yo_sync_step2_v1(a, an, b, bn, ctypes.byref(out), ctypes.byref(olen))
    if st:
        raise OracleError(st)
    return _take(out, olen)


def status_of(fn, *args, **kw):
    try:
        return 0, fn(*args, **kw)
    except OracleError as e:
        return e.code, None


def merge_batch(data, upd_off, doc_upd, mode=0, threads=1, version=1):
    """Arena batch; returns (arena, offsets, status array).  version 2 = lib0 v2."""
    if version == 2:
        mode |= 4
    data = np.ascontiguousarray(data, dtype=np.uint8)
    upd_off = np.ascontiguousarray(upd_off, dtype=np.uint64)
    doc_upd = np.ascontiguousarray(doc_upd, dtype=np.uint64)
    n_docs = len(doc_upd) - 1
    out = ctypes.POINTER(ctypes.c_uint8)()
    out_off = np.zeros(n_docs + 1, dtype=np.uint64)
    status = np.zeros(max(1, n_docs), dtype=np.uint8)
    lib().yo_merge_batch(data.ctypes.data, upd_off.ctypes.data, doc_upd.ctypes.data, n_docs, mode,
                         threads, ctypes.byref(out), out_off.ctypes.data, status.ctypes.data)
    total = int(out_off[-1])
    arena = ctypes.string_at(out, total) if total else b""
    lib().yo_free(out)
    return arena, out_off, status[:n_docs]


def compact_batch(data, upd_off, doc_upd, threads=1):
    """compact_updates_v1 per document of an arena batch: (arena, offsets, status)."""
    return merge_batch(data, upd_off, doc_upd, mode=8, threads=threads)


def diff_batch(ubytes, u_off, svbytes, sv_off, threads=1, version=1):
    ubytes = np.ascontiguousarray(ubytes, dtype=np.uint8)
    u_off = np.ascontiguousarray(u_off, dtype=np.uint64)
    svbytes = np.ascontiguousarray(svbytes, dtype=np.uint8)
    sv_off = np.ascontiguousarray(sv_off, dtype=np.uint64)
    n_docs = len(u_off) - 1
    out = ctypes.POINTER(ctypes.c_uint8)()
    out_off = np.zeros(n_docs + 1, dtype=np.uint64)
    status = np.zeros(max(1, n_docs), dtype=np.uint8)
    L = lib()
    vp = ctypes.c_void_p
    L.yo_diff_batch2.argtypes = [vp, vp, vp, vp, ctypes.c_size_t, ctypes.c_int, ctypes.c_int,
                                 ctypes.POINTER(ctypes.POINTER(ctypes.c_uint8)), vp, vp]
    L.yo_diff_batch2(ubytes.ctypes.data, u_off.ctypes.data, svbytes.ctypes.data, sv_off.ctypes.data,
                     n_docs, version, threads, ctypes.byref(out), out_off.ctypes.data, status.ctypes.data)
    total = int(out_off[-1])
    arena = ctypes.string_at(out, total) if total else b""
    lib().yo_free(out)
    return arena, out_off, status[:n_docs]


def sv_batch(ubytes, u_off, threads=1, version=1):
    """encode_state_vector_from_update_v1 per document (one update each)."""
    ubytes = np.ascontiguousarray(ubytes, dtype=np.uint8)
    u_off = np.ascontiguousarray(u_off, dtype=np.uint64)
    n_docs = len(u_off) - 1
    out = ctypes.POINTER(ctypes.c_uint8)()
    out_off = np.zeros(n_docs + 1, dtype=np.uint64)
    status = np.zeros(max(1, n_docs), dtype=np.uint8)
    L = lib()
    vp = ctypes.c_void_p
    L.yo_sv_batch2.argtypes = [vp, vp, ctypes.c_size_t, ctypes.c_int, ctypes.c_int,
                               ctypes.POINTER(ctypes.POINTER(ctypes.c_uint8)), vp, vp]
    L.yo_sv_batch2(ubytes.ctypes.data, u_off.ctypes.data, n_docs, version, threads, ctypes.byref(out),
                   out_off.ctypes.data, status.ctypes.data)
    total = int(out_off[-1])
    arena = ctypes.string_at(out, total) if total else b""
    lib().yo_free(out)
    return arena, out_off, status[:n_docs]


def sv_roundtrip(sv):
    a, an = _buf(sv)
    L = lib()
    L.yo_sv_roundtrip.argtypes = [ctypes.POINTER(ctypes.c_uint8), ctypes.c_size_t,
                                  ctypes.POINTER(ctypes.POINTER(ctypes.c_uint8)), ctypes.POINTER(ctypes.c_size_t)]
    out = ctypes.POINTER(ctypes.c_uint8)()
    olen = ctypes.c_size_t()
    st = L.yo_sv_roundtrip(a, an, ctypes.byref(out), ctypes.byref(olen))
    if st:
        raise OracleError(st)
    return _take(out, olen)


def ds_offset(update):
    a, an = _buf(update)
    L = lib()
    L.yo_ds_offset.argtypes = [ctypes.POINTER(ctypes.c_uint8), ctypes.c_size_t, ctypes.POINTER(ctypes.c_size_t)]
    off = ctypes.c_size_t()
    st = L.yo_ds_offset(a, an, ctypes.byref(off))
    if st:
        raise OracleError(st)
    return off.value


def _rv(b, i):
    v = s = 0
    while True:
        x = b[i]
        i += 1
        v |= (x & 0x7F) << s
        s += 7
        if x < 0x80:
            return v, i


def parse_ds(b, i=0):
    """DeleteSet section -> (ordered list of (client, [(clock,len)...]), end)."""
    n, i = _rv(b, i)
    out = []
    for _ in range(n):
        c, i = _rv(b, i)
        k, i = _rv(b, i)
        rs = []
        for _ in range(k):
            s, i = _rv(b, i)
            ln, i = _rv(b, i)
            rs.append((s, ln))
        out.append((c, rs))
    return out, i


def parse_sv(b):
    n, i = _rv(b, 0)
    out = []
    for _ in range(n):
        c, i = _rv(b, i)
        k, i = _rv(b, i)
        out.append((c, k))
    return out


def normalized(update):
    """(blocks section bytes, DS as a client->ranges dict): equality modulo DS client order."""
    off = ds_offset(update)
    ds, _ = parse_ds(update, off)
    return update[:off], dict(ds)
