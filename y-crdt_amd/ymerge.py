"""Host-side mirror of yrs' binary-update API over the MI355X engine (C ABI).

Same names, argument meaning and error behaviour as yrs/src/alt.rs:
    merge_updates_v1(updates)                 -> bytes   (alt.rs:15-28)
    diff_updates_v1(update, state_vector)     -> bytes   (alt.rs:73-81)
    encode_state_vector_from_update_v1(update)-> bytes   (alt.rs:54-57)
and their lib0 v2 forms merge_updates_v2 / diff_updates_v2 /
encode_state_vector_from_update_v2 (alt.rs:35-48, 88-97, 63-66).
A decode failure raises YrsError carrying yffi's error code (yffi/src/lib.rs:1137-1174).

`Engine` is the batched, multi-tenant entry point (one HIP stream per device).
There is no CPU fallback: without the gfx950 library or a GPU, calls raise.
"""
import ctypes
import os

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("YMERGE_LIB") or os.path.join(_HERE, "lib", "libymerge.so")  # YMERGE_LIB: A/B experiments only

ERRORS = {2: "InvalidVarInt", 3: "EndOfBuffer", 4: "UnexpectedValue", 5: "InvalidJSON", 6: "Other",
          7: "NotEnoughMemory", 20: "ReferencePanic", 21: "Unsupported", 30: "DeviceError"}


class YrsError(Exception):
    def __init__(self, code):
        super().__init__(f"{ERRORS.get(code, 'error')} ({code})")
        self.code = code


class DeviceError(RuntimeError):
    """A HIP failure inside the engine.  The message carries the library's provenance of it
    (ymerge_last_error_message: the failing stage and the HIP error string)."""

    def __init__(self, msg):
        where = ""
        try:
            if _lib is not None:
                where = (_lib.ymerge_last_error_message() or b"").decode(errors="replace")
        except Exception:  # noqa: BLE001 -- the provenance is best effort
            where = ""
        super().__init__(f"{msg}: {where}" if where else msg)


class _Stats(ctypes.Structure):
    _fields_ = [("n_docs", ctypes.c_uint64), ("bytes_in", ctypes.c_uint64), ("bytes_out", ctypes.c_uint64),
                ("docs_fast", ctypes.c_uint64), ("docs_exact", ctypes.c_uint64), ("docs_error", ctypes.c_uint64),
                ("ms_total", ctypes.c_float), ("ms_fast", ctypes.c_float), ("ms_exact", ctypes.c_float),
                ("ms_tail", ctypes.c_float), ("ms_decode", ctypes.c_float), ("ms_big", ctypes.c_float),
                ("docs_overlap", ctypes.c_uint32), ("docs_big", ctypes.c_uint64), ("docs_tiny", ctypes.c_uint64),
                ("ms_tiny", ctypes.c_float), ("docs_lean", ctypes.c_uint64), ("ms_lean", ctypes.c_float),
                ("docs_giant", ctypes.c_uint64), ("ms_v2_decode", ctypes.c_float), ("ms_v2_merge", ctypes.c_float),
                ("ms_v2_encode", ctypes.c_float)]


class _DevRes(ctypes.Structure):
    _fields_ = [("d_out", ctypes.c_void_p), ("d_out_start", ctypes.c_void_p), ("d_out_len", ctypes.c_void_p),
                ("d_status", ctypes.c_void_p), ("arena_bytes", ctypes.c_uint64), ("out_bytes", ctypes.c_uint64)]


class _BatchRes(ctypes.Structure):
    _fields_ = [("out", ctypes.c_void_p), ("out_off", ctypes.c_void_p), ("status", ctypes.c_void_p),
                ("n_docs", ctypes.c_uint64), ("out_bytes", ctypes.c_uint64)]


# host-memory batch entries (include/ymerge.h, "batched, host memory"): name -> argument kinds
# (b = byte arena, o = u64 offsets, n = count); every one ends with (n_docs, result**)
HOST_BATCH = {
    "ymerge_updates_v1_batch": "bono", "ymerge_updates_v2_batch": "bono",
    "ydiff_updates_v1_batch": "bobo", "ydiff_updates_v2_batch": "bobo",
    "yencode_state_vector_from_update_v1_batch": "bo", "yencode_state_vector_from_update_v2_batch": "bo",
    "ysync_step1_v1_batch": "bo", "ysync_step2_v1_batch": "bobo",
    "ycompact_updates_v1_batch": "bono",
}

_lib = None


def lib():
    """Loads the in-tree gfx950 library; raises loudly if it is missing."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise DeviceError(f"HIP engine not built: {LIB_PATH} missing (run __graft_entry__.build())")
    # torch ships its own libamdhip64.so.7 (same soname as /opt/rocm's): load it first
    # so the engine and torch's allocator share ONE HIP runtime in this process.
    import torch  # noqa: F401
    L = ctypes.CDLL(LIB_PATH)
    c = ctypes
    vp, u64, u32 = c.c_void_p, c.c_uint64, c.c_uint32
    L.ymerge_ctx_create.restype = vp
    L.ymerge_ctx_create.argtypes = [c.c_int]
    L.ymerge_ctx_destroy.argtypes = [vp]
    L.ymerge_updates_v1_batch_device.argtypes = [vp, vp, u64, vp, u64, vp, u64, c.POINTER(_DevRes)]
    L.ydiff_updates_v1_batch_device.argtypes = [vp, vp, vp, vp, vp, u64, c.POINTER(_DevRes)]
    L.ysync_step2_v1_batch_device.argtypes = [vp, vp, vp, vp, vp, u64, c.POINTER(_DevRes)]
    L.ysync_step1_v1_batch_device.argtypes = [vp, vp, vp, u64, c.POINTER(_DevRes)]
    L.yencode_state_vector_from_update_v1_batch_device.argtypes = [vp, vp, vp, u64, c.POINTER(_DevRes)]
    L.ymerge_result_to_host.argtypes = [vp, c.POINTER(_DevRes), u64, vp, vp, vp]
    L.ymerge_last_stats.argtypes = [vp, c.POINTER(_Stats)]
    L.ymerge_ctx_set_stage_timing.argtypes = [vp, c.c_int]
    L.ymerge_ctx_set_stage_timing.restype = None
    L.ymerge_updates_v1.restype = vp
    L.ymerge_updates_v1.argtypes = [c.POINTER(c.c_char_p), c.POINTER(u32), u32, c.POINTER(u32)]
    L.ydiff_updates_v1.restype = vp
    L.ydiff_updates_v1.argtypes = [c.c_char_p, u32, c.c_char_p, u32, c.POINTER(u32)]
    L.yencode_state_vector_from_update_v1.restype = vp
    L.yencode_state_vector_from_update_v1.argtypes = [c.c_char_p, u32, c.POINTER(u32)]
    for v in ("v1", "v2"):
        getattr(L, f"ymerge_updates_{v}").restype = vp
        getattr(L, f"ymerge_updates_{v}").argtypes = [c.POINTER(c.c_char_p), c.POINTER(u32), u32, c.POINTER(u32)]
        getattr(L, f"ydiff_updates_{v}").restype = vp
        getattr(L, f"ydiff_updates_{v}").argtypes = [c.c_char_p, u32, c.c_char_p, u32, c.POINTER(u32)]
        getattr(L, f"yencode_state_vector_from_update_{v}").restype = vp
        getattr(L, f"yencode_state_vector_from_update_{v}").argtypes = [c.c_char_p, u32, c.POINTER(u32)]
    L.ymerge_updates_v2_batch_device.argtypes = [vp, vp, u64, vp, u64, vp, u64, c.POINTER(_DevRes)]
    L.ycompact_updates_v1_batch_device.argtypes = [vp, vp, u64, vp, u64, vp, u64, c.POINTER(_DevRes)]
    L.yconvert_updates_v1_to_v2_batch_device.argtypes = [vp, vp, u64, vp, u64, c.POINTER(_DevRes)]
    L.ydiff_updates_v2_batch_device.argtypes = [vp, vp, vp, vp, vp, u64, c.POINTER(_DevRes)]
    L.yencode_state_vector_from_update_v2_batch_device.argtypes = [vp, vp, vp, u64, c.POINTER(_DevRes)]
    L.ymerge_binary_destroy.argtypes = [vp, u32]
    L.ymerge_set_default_device.argtypes = [c.c_int]
    L.ymerge_last_error.restype = c.c_uint8
    L.ymerge_last_error_message.restype = c.c_char_p
    L.ydiff_updates_v1_batch.argtypes = [vp, vp, vp, vp, vp, u64, c.POINTER(c.c_void_p)]
    L.yencode_state_vector_from_update_v1_batch.argtypes = [vp, vp, vp, u64, c.POINTER(c.c_void_p)]
    L.ymerge_batch_result_destroy.argtypes = [vp]
    for name, kinds in HOST_BATCH.items():
        getattr(L, name).argtypes = [vp] + [u64 if k == "n" else vp for k in kinds] + [u64, c.POINTER(c.c_void_p)]
    _lib = L
    return L


def padded(a):
    """uint8 array + 16 zero bytes: the kernels read arenas in 16-byte words (include/ymerge.h)."""
    a = np.ascontiguousarray(a, dtype=np.uint8)
    return np.concatenate([a, np.zeros(16, np.uint8)])


def _take(ptr, n):
    if not ptr:
        code = lib().ymerge_last_error()
        if code == 30:
            raise DeviceError("no usable MI355X (HIP)")
        raise YrsError(code)
    data = ctypes.string_at(ptr, n.value)
    lib().ymerge_binary_destroy(ptr, n.value)
    return data


def merge_updates_v1(updates):
    """yrs::merge_updates_v1 (alt.rs:15)."""
    ups = [bytes(u) for u in updates]
    arr = (ctypes.c_char_p * max(1, len(ups)))(*ups)
    lens = (ctypes.c_uint32 * max(1, len(ups)))(*[len(u) for u in ups])
    n = ctypes.c_uint32()
    return _take(lib().ymerge_updates_v1(arr, lens, len(ups), ctypes.byref(n)), n)


def diff_updates_v1(update, state_vector):
    """yrs::diff_updates_v1 (alt.rs:73)."""
    n = ctypes.c_uint32()
    u, s = bytes(update), bytes(state_vector)
    return _take(lib().ydiff_updates_v1(u, len(u), s, len(s), ctypes.byref(n)), n)


def encode_state_vector_from_update_v1(update):
    """yrs::encode_state_vector_from_update_v1 (alt.rs:54)."""
    n = ctypes.c_uint32()
    u = bytes(update)
    return _take(lib().yencode_state_vector_from_update_v1(u, len(u), ctypes.byref(n)), n)


def merge_updates_v2(updates):
    """yrs::merge_updates_v2 (alt.rs:35)."""
    ups = [bytes(u) for u in updates]
    arr = (ctypes.c_char_p * max(1, len(ups)))(*ups)
    lens = (ctypes.c_uint32 * max(1, len(ups)))(*[len(u) for u in ups])
    n = ctypes.c_uint32()
    return _take(lib().ymerge_updates_v2(arr, lens, len(ups), ctypes.byref(n)), n)


def diff_updates_v2(update, state_vector):
    """yrs::diff_updates_v2 (alt.rs:88)."""
    n = ctypes.c_uint32()
    u, s = bytes(update), bytes(state_vector)
    return _take(lib().ydiff_updates_v2(u, len(u), s, len(s), ctypes.byref(n)), n)


def encode_state_vector_from_update_v2(update):
    """yrs::encode_state_vector_from_update_v2 (alt.rs:63)."""
    n = ctypes.c_uint32()
    u = bytes(update)
    return _take(lib().yencode_state_vector_from_update_v2(u, len(u), ctypes.byref(n)), n)


def _multi(fn_name, engines, arrays, doc_ids):
    L = lib()
    n_ctx = len(engines)
    ctxs = (ctypes.c_void_p * n_ctx)(*[e._ctx for e in engines])
    keep, args = [], []
    for k, a in arrays:
        if k == "n":
            args.append(ctypes.c_uint64(int(a)))
            continue
        a = np.ascontiguousarray(a, dtype=np.uint8 if k == "b" else np.uint64)
        if not len(a):
            a = np.zeros(1, a.dtype)
        keep.append(a)
        args.append(ctypes.c_void_p(a.ctypes.data))
    n_docs = len(arrays[-1][1]) - 1
    ids = None if doc_ids is None else np.ascontiguousarray(doc_ids, dtype=np.uint64)
    pres = ctypes.c_void_p()
    rc = getattr(L, fn_name)(ctxs, ctypes.c_uint32(n_ctx), *args, ctypes.c_uint64(n_docs),
                             ctypes.c_void_p(ids.ctypes.data if ids is not None else 0), ctypes.byref(pres))
    if rc:
        raise DeviceError(f"{fn_name} failed ({rc})")
    return _read_batch_result(pres, n_docs)


def merge_multi(engines, data, upd_off, doc_upd, doc_ids=None):
    """ymerge_updates_v1_batch_multi: the batch spread over several contexts (devices) by
    document hash; outputs in input order: (out, out_off, status)."""
    return _multi("ymerge_updates_v1_batch_multi", engines,
                  [("b", data), ("o", upd_off), ("n", len(upd_off) - 1), ("o", doc_upd)], doc_ids)


def diff_multi(engines, ubytes, u_off, svbytes, sv_off, doc_ids=None):
    """ydiff_updates_v1_batch_multi (one update + one remote state vector per document)."""
    return _multi("ydiff_updates_v1_batch_multi", engines,
                  [("b", ubytes), ("o", u_off), ("b", svbytes), ("o", sv_off)], doc_ids)


def _read_batch_result(pres, n_docs):
    try:
        r = _BatchRes.from_address(pres.value)
        nb = int(r.out_bytes)
        out = np.ctypeslib.as_array((ctypes.c_uint8 * max(1, nb)).from_address(r.out))[:nb].copy()
        off = np.ctypeslib.as_array((ctypes.c_uint64 * (n_docs + 1)).from_address(r.out_off)).copy()
        st = (np.ctypeslib.as_array((ctypes.c_uint8 * n_docs).from_address(r.status)).copy() if n_docs
              else np.zeros(0, np.uint8))
    finally:
        lib().ymerge_batch_result_destroy(pres)
    return out, off, st


class DeviceResult:
    def __init__(self, engine, res, n_docs):
        self.engine, self.res, self.n_docs = engine, res, n_docs

    @property
    def out_bytes(self):
        return int(self.res.out_bytes)

    def to_host(self):
        n = self.n_docs
        out = np.empty(max(1, self.out_bytes), dtype=np.uint8)
        off = np.empty(n + 1, dtype=np.uint64)
        st = np.empty(max(1, n), dtype=np.uint8)
        rc = lib().ymerge_result_to_host(self.engine._ctx, ctypes.byref(self.res), n, out.ctypes.data,
                                         off.ctypes.data, st.ctypes.data)
        if rc:
            raise DeviceError(f"result copy failed ({rc})")
        return out[: self.out_bytes], off, st[:n]


class Engine:
    """One HIP stream + HBM workspace on one GPU; batches of documents."""

    def __init__(self, device=0):
        self._ctx = lib().ymerge_ctx_create(device)
        if not self._ctx:
            raise DeviceError(f"cannot open HIP device {device}")
        self.device = device

    def close(self):
        if self._ctx:
            lib().ymerge_ctx_destroy(self._ctx)
            self._ctx = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def merge_device(self, d_bytes, n_bytes, d_upd_off, n_updates, d_doc_upd, n_docs, version=1):
        """Inputs are device pointers (ints) into HBM; returns a DeviceResult.  version 2 = lib0 v2.

        The byte arena must stay readable 16 bytes past n_bytes (the kernels stage whole
        16-byte groups): allocate it from `padded(data)`, as `merge_host` does."""
        res = _DevRes()
        fn = lib().ymerge_updates_v2_batch_device if version == 2 else lib().ymerge_updates_v1_batch_device
        rc = fn(self._ctx, d_bytes, n_bytes, d_upd_off, n_updates, d_doc_upd, n_docs, ctypes.byref(res))
        if rc:
            raise DeviceError(f"merge batch failed ({rc})")
        return DeviceResult(self, res, n_docs)

    def compact_device(self, d_bytes, n_bytes, d_upd_off, n_updates, d_doc_upd, n_docs):
        """Store-based compaction (ycompact_updates_v1_batch_device): each document's updates
        applied in order to a fresh Doc, then encode_state_as_update_v1.  Same argument
        layout as merge_device; documents outside the device shape get status 21."""
        res = _DevRes()
        rc = lib().ycompact_updates_v1_batch_device(self._ctx, d_bytes, n_bytes, d_upd_off, n_updates, d_doc_upd,
                                                     n_docs, ctypes.byref(res))
        if rc:
            raise DeviceError(f"compaction batch failed ({rc})")
        return DeviceResult(self, res, n_docs)

    def diff_device(self, d_bytes, d_upd_off, d_sv, d_sv_off, n_docs, version=1):
        """Device pointers in, DeviceResult out; the update arena must stay readable 16 bytes
        past its end (`padded`), as for merge_device."""
        res = _DevRes()
        fn = lib().ydiff_updates_v2_batch_device if version == 2 else lib().ydiff_updates_v1_batch_device
        rc = fn(self._ctx, d_bytes, d_upd_off, d_sv, d_sv_off, n_docs, ctypes.byref(res))
        if rc:
            raise DeviceError(f"diff batch failed ({rc})")
        return DeviceResult(self, res, n_docs)

    def sync_step2_device(self, d_bytes, d_upd_off, d_msg, d_msg_off, n_docs):
        """y-sync SyncStep2 replies to SyncStep1 client messages (yrs/src/sync/protocol.rs:62-69)."""
        res = _DevRes()
        rc = lib().ysync_step2_v1_batch_device(self._ctx, d_bytes, d_upd_off, d_msg, d_msg_off, n_docs,
                                               ctypes.byref(res))
        if rc:
            raise DeviceError(f"sync-step-2 batch failed ({rc})")
        return DeviceResult(self, res, n_docs)

    def sync_step1_device(self, d_bytes, d_upd_off, n_docs):
        res = _DevRes()
        rc = lib().ysync_step1_v1_batch_device(self._ctx, d_bytes, d_upd_off, n_docs, ctypes.byref(res))
        if rc:
            raise DeviceError(f"sync-step-1 batch failed ({rc})")
        return DeviceResult(self, res, n_docs)

    def sync_step2_host(self, ubytes, u_off, msg, msg_off):
        n = len(u_off) - 1
        ub = np.ascontiguousarray(ubytes, dtype=np.uint8)
        mb = np.ascontiguousarray(msg, dtype=np.uint8)
        args = [ub if len(ub) else np.zeros(1, np.uint8), np.asarray(u_off, np.uint64).view(np.int64),
                mb if len(mb) else np.zeros(1, np.uint8), np.asarray(msg_off, np.uint64).view(np.int64)]
        return self._host_batch(args, lambda a, b, c, d: self.sync_step2_device(a, b, c, d, n))

    def sync_step1_host(self, ubytes, u_off):
        n = len(u_off) - 1
        ub = np.ascontiguousarray(ubytes, dtype=np.uint8)
        args = [ub if len(ub) else np.zeros(1, np.uint8), np.asarray(u_off, np.uint64).view(np.int64)]
        return self._host_batch(args, lambda a, b: self.sync_step1_device(a, b, n))

    def state_vector_device(self, d_bytes, d_upd_off, n_docs, version=1):
        res = _DevRes()
        fn = (lib().yencode_state_vector_from_update_v2_batch_device if version == 2
              else lib().yencode_state_vector_from_update_v1_batch_device)
        rc = fn(self._ctx, d_bytes, d_upd_off, n_docs, ctypes.byref(res))
        if rc:
            raise DeviceError(f"state-vector batch failed ({rc})")
        return DeviceResult(self, res, n_docs)

    def set_stage_timing(self, on):
        """Stage timing events on / off (ymerge_ctx_set_stage_timing); off, the stats' ms_*
        of a merge k_lean writes whole read 0."""
        lib().ymerge_ctx_set_stage_timing(self._ctx, 1 if on else 0)

    def stats(self):
        s = _Stats()
        lib().ymerge_last_stats(self._ctx, ctypes.byref(s))
        return {k: getattr(s, k) for k, _ in _Stats._fields_}

    def host_batch(self, name, *arrays, copy=True):
        """Calls a host-memory batch entry of the C ABI (HOST_BATCH: the server-facing form,
        host pointers in, a library-owned ymerge_batch_result out) and copies the result:
        (out bytes, out_off[n_docs + 1], status[n_docs]).  Arrays are passed in the
        order of the C signature without the trailing n_docs, which is taken from the
        last offsets array."""
        kinds = HOST_BATCH[name]
        keep, args = [], []
        for k, a in zip(kinds, arrays):
            if k == "n":
                args.append(int(a))
                continue
            a = np.ascontiguousarray(a, dtype=np.uint8 if k == "b" else np.uint64)
            if not len(a):
                a = np.zeros(1, a.dtype)
            keep.append(a)
            args.append(a.ctypes.data)
        n_docs = len(arrays[-1]) - 1
        pres = ctypes.c_void_p()
        rc = getattr(lib(), name)(self._ctx, *args, n_docs, ctypes.byref(pres))
        if rc:
            raise DeviceError(f"{name} failed ({rc})")
        if not copy:  # timing: the library-owned result is released unread
            lib().ymerge_batch_result_destroy(pres)
            return None
        return _read_batch_result(pres, n_docs)

    def _host_batch(self, args_dev, fn):
        import torch
        dev = torch.device("cuda", self.device)
        ts = [torch.from_numpy(padded(a) if a.dtype == np.uint8 else np.ascontiguousarray(a)).to(dev)
              for a in args_dev]
        torch.cuda.synchronize(dev)
        r = fn(*[t.data_ptr() for t in ts])
        return r.to_host()

    def diff_host(self, ubytes, u_off, svbytes, sv_off, version=1):
        """Batched diff_updates_v1 (v2): document d = (update d, remote state vector d)."""
        n = len(u_off) - 1
        ub = np.ascontiguousarray(ubytes, dtype=np.uint8)
        sb = np.ascontiguousarray(svbytes, dtype=np.uint8)
        args = [ub if len(ub) else np.zeros(1, np.uint8), np.asarray(u_off, np.uint64).view(np.int64),
                sb if len(sb) else np.zeros(1, np.uint8), np.asarray(sv_off, np.uint64).view(np.int64)]
        return self._host_batch(args, lambda a, b, c, d: self.diff_device(a, b, c, d, n, version))

    def state_vector_host(self, ubytes, u_off, version=1):
        """Batched encode_state_vector_from_update_v1 (v2) (one update per document)."""
        n = len(u_off) - 1
        ub = np.ascontiguousarray(ubytes, dtype=np.uint8)
        args = [ub if len(ub) else np.zeros(1, np.uint8), np.asarray(u_off, np.uint64).view(np.int64)]
        return self._host_batch(args, lambda a, b: self.state_vector_device(a, b, n, version))

    # convenience: host arrays in, host arrays out (uses torch for HBM residency)
    def merge_host(self, data, upd_off, doc_upd, version=1):
        import torch
        dev = torch.device("cuda", self.device)
        t_b = torch.from_numpy(padded(data)).to(dev)
        t_u = torch.from_numpy(np.ascontiguousarray(upd_off, dtype=np.uint64).view(np.int64)).to(dev)
        t_d = torch.from_numpy(np.ascontiguousarray(doc_upd, dtype=np.uint64).view(np.int64)).to(dev)
        torch.cuda.synchronize(dev)
        r = self.merge_device(t_b.data_ptr(), int(upd_off[-1]), t_u.data_ptr(), len(upd_off) - 1, t_d.data_ptr(),
                              len(doc_upd) - 1, version)
        return r.to_host()

    def compact_host(self, data, upd_off, doc_upd):
        """compact_device over host arrays (torch for HBM residency)."""
        ub = np.ascontiguousarray(data, dtype=np.uint8)
        args = [ub if len(ub) else np.zeros(1, np.uint8), np.asarray(upd_off, np.uint64).view(np.int64),
                np.asarray(doc_upd, np.uint64).view(np.int64)]
        return self._host_batch(args, lambda a, b, c: self.compact_device(a, int(upd_off[-1]), b, len(upd_off) - 1,
                                                                          c, len(doc_upd) - 1))

    def convert_v1_to_v2_host(self, data, upd_off):
        """yconvert_updates_v1_to_v2_batch_device over host arrays: every v1 update re-encoded
        as lib0 v2 (out, out_off[n_updates + 1], status)."""
        n = len(upd_off) - 1
        ub = np.ascontiguousarray(data, dtype=np.uint8)
        args = [ub if len(ub) else np.zeros(1, np.uint8), np.asarray(upd_off, np.uint64).view(np.int64)]

        def run(a, b):
            res = _DevRes()
            rc = lib().yconvert_updates_v1_to_v2_batch_device(self._ctx, a, int(upd_off[-1]), b, n,
                                                               ctypes.byref(res))
            if rc:
                raise DeviceError(f"v1 -> v2 conversion failed ({rc})")
            return DeviceResult(self, res, n)
        return self._host_batch(args, run)
