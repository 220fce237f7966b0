"""CPU parity of the device compaction code (y-crdt_amd/csrc/ycompact.hip: k_compact_count +
k_compact's lane body) against the store-based oracle (oracle/yrs_oracle_store.c).

tools/hostemu compiles the same kernel source for the host, so the algorithm is checked
here on every CPU run; tests/test_gpu_compact.py then checks the gfx950 build against both.
Every document is either byte-identical to the oracle (same status) or outside the device
shape (status 21) for the reason the case names."""
import ctypes
import os
import subprocess

import numpy as np
import pytest

import workloads
from compact_cases import exhibits, CU, edge_docs, fixture_reason, fixtures, regrouped
from conftest import ROOT

EMU_DIR = os.path.join(ROOT, "tools", "hostemu")


@pytest.fixture(scope="module")
def emu():
    subprocess.check_call(["make", "-s", "-C", EMU_DIR])
    L = ctypes.CDLL(os.path.join(EMU_DIR, "libcompact_emu.so"))
    vp = ctypes.c_void_p
    L.emu_compact_batch.argtypes = [vp, vp, vp, ctypes.c_uint32, vp, vp, vp, vp, vp]

    def run(b):
        data = np.concatenate([np.ascontiguousarray(b.data, np.uint8), np.zeros(16, np.uint8)])
        uo = np.ascontiguousarray(b.upd_off, np.uint64)
        du = np.ascontiguousarray(b.doc_upd, np.uint64)
        n = len(du) - 1
        out = np.zeros(2 * int(uo[-1]) + 64 * n + 64, np.uint8)
        st, ln = np.zeros(n + 1, np.uint64), np.zeros(n + 1, np.uint64)
        status, why = np.zeros(n + 1, np.uint8), np.zeros(n + 1, np.uint8)
        L.emu_compact_batch(data.ctypes.data, uo.ctypes.data, du.ctypes.data, n, out.ctypes.data, st.ctypes.data,
                            ln.ctypes.data, status.ctypes.data, why.ctypes.data)
        return [out[int(a):int(a) + int(k)].tobytes() for a, k in zip(st[:n], ln[:n])], status[:n], why[:n]
    return run


def check(emu, oracle, b, reasons=None, min_device=1.0):
    """reasons[d]: 0 = the device must write document d, a CU code = it must refuse it for
    that reason, None = whatever the oracle says (status equal or 21)."""
    outs, st, why = emu(b)
    arena, off, est = oracle.compact_batch(b.data, b.upd_off, b.doc_upd, threads=8)
    done = 0
    for d in range(b.n_docs):
        r = None if reasons is None else reasons[d]
        if st[d] == 21 and est[d] != 21:
            assert r is None or r == why[d], f"doc {d}: refused ({why[d]}), expected reason {r}"
            assert reasons is not None or why[d] in (CU["GAP"], CU["PENDING"], CU["PENDING_DS"], CU["CLIENTS"]), \
                f"doc {d}: unexpected refusal {why[d]}"
            # the bytes show the refused shape (compact_cases.exhibits: an independent parse)
            assert exhibits(b.doc_updates(d), int(why[d])) is not False, f"doc {d}: reason {why[d]} not in its bytes"
            continue
        assert r in (0, None), f"doc {d}: written, expected refusal {r}"
        assert st[d] == est[d], f"doc {d}: status {st[d]} oracle {est[d]}"
        assert outs[d] == arena[int(off[d]):int(off[d + 1])], f"doc {d}: bytes differ"
        done += 1
    assert done >= min_device * b.n_docs - 1e-9, f"{done}/{b.n_docs} documents on the device"
    return st, why


def test_reference_corpus(emu, oracle):
    """The reference corpus (assets/bench-input/small-test-dataset.bin, 5,320 real Yjs documents):
    every document the device writes equals the oracle byte for byte; every refusal shows its
    shape in the document's bytes; the device share is pinned (round 6: every content kind but
    Doc / Move / WeakLink, maps and nested types on the device: all 5,320)."""
    b = workloads.dataset_docs()
    st, why = check(emu, oracle, b, reasons=[None] * b.n_docs, min_device=1.0)
    assert (st == 21).sum() == 0


def test_text_docs(emu, oracle):
    for seed, mc, df in ((1, 4, 0.2), (2, 8, 0.4), (3, 2, 0.05)):
        check(emu, oracle, workloads.text_docs(80, 300, seed=seed, max_clients=mc, del_frac=df))


def test_zipf_docs(emu, oracle):
    check(emu, oracle, workloads.zipf_docs(200))


def test_long_documents(emu, oracle):
    check(emu, oracle, workloads.text_docs(8, 4000, seed=11, max_clients=3, del_frac=0.3))


@pytest.mark.parametrize("name", workloads.TRACES)
def test_editing_traces(emu, oracle, name):
    b, _ = workloads.trace_updates(name)
    check(emu, oracle, b)


def test_many_clients(emu, oracle):
    """up to CP_MAXCL = 16 clients on the device; documents with more are refused (CU_CLIENTS)"""
    check(emu, oracle, workloads.text_docs(40, 400, seed=5, min_clients=9, max_clients=16))
    st, why = check(emu, oracle, workloads.text_docs(40, 400, seed=6, min_clients=9, max_clients=24), reasons=None,
                    min_device=0.2)
    assert set(why[st == 21].tolist()) <= {CU["CLIENTS"]}


@pytest.mark.parametrize("k", [2, 7, 31])
def test_merged_updates(emu, oracle, k):
    """Multi-client updates: blocks wait on the dependency stack (update.rs:183-262)."""
    check(emu, oracle, regrouped(oracle, workloads.text_docs(40, 300, seed=20 + k), k=k))


def test_snapshot_plus_log(emu, oracle):
    check(emu, oracle, regrouped(oracle, workloads.text_docs(40, 300, seed=40), head=200))


def test_yjs_fixtures(emu, oracle):
    names, b = fixtures()
    check(emu, oracle, b, reasons=[fixture_reason(n) for n in names], min_device=0.6)


def test_edge_documents(emu, oracle):
    b, reasons = edge_docs()
    check(emu, oracle, b, reasons=reasons, min_device=0.5)


def test_delete_heavy_pending(emu, oracle):
    """C4 withholds and duplicates updates: pending structs / delete sets are not on the
    device; every refusal must say so, every written document must be exact."""
    st, why = check(emu, oracle, workloads.delete_heavy_docs(10, 1000), min_device=0.0)
    assert set(why[st == 21].tolist()) <= {CU["GAP"], CU["PENDING"], CU["PENDING_DS"]}
