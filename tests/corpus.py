"""Readers for the reference's own corpora (copied under tests/golden/).

small-test-dataset.bin: the format test_data_set reads (yrs/src/tests/compatibility_tests.rs:437-476):
    var_u32 test_count, then per test: var_u32 updates_len, updates_len x read_buf (a v1 update),
    read_string (expected Y.Text "text"), read_any (expected Y.Map "map" JSON), read_any (Y.Array "array").
"""
import os
import struct

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def _rv(b, i):
    v = s = 0
    while True:
        x = b[i]
        i += 1
        v |= (x & 0x7F) << s
        s += 7
        if x < 0x80:
            return v, i


def _rvi(b, i):  # lib0 signed varint (yrs/src/encoding/varint.rs:262-281)
    x = b[i]
    i += 1
    v, neg, s = x & 0x3F, x & 0x40, 6
    while x & 0x80:
        x = b[i]
        i += 1
        v |= (x & 0x7F) << s
        s += 7
    return (-v if neg else v), i


def read_any(b, i):
    """lib0 Any (yrs/src/any.rs:37-83) -> Python value; buffers -> list of ints."""
    t = b[i]
    i += 1
    if t in (127, 126):
        return None, i
    if t == 125:
        return _rvi(b, i)
    if t == 124:
        return struct.unpack(">f", b[i:i + 4])[0], i + 4
    if t == 123:
        return struct.unpack(">d", b[i:i + 8])[0], i + 8
    if t == 122:
        return struct.unpack(">q", b[i:i + 8])[0], i + 8
    if t in (121, 120):
        return t == 120, i
    if t == 119:
        n, i = _rv(b, i)
        return b[i:i + n].decode("utf-8"), i + n
    if t == 118:
        n, i = _rv(b, i)
        d = {}
        for _ in range(n):
            k, i = _rv(b, i)
            key = b[i:i + k].decode("utf-8")
            i += k
            d[key], i = read_any(b, i)
        return d, i
    if t == 117:
        n, i = _rv(b, i)
        out = []
        for _ in range(n):
            v, i = read_any(b, i)
            out.append(v)
        return out, i
    if t == 116:
        n, i = _rv(b, i)
        return list(b[i:i + n]), i + n
    raise ValueError(f"bad Any tag {t}")


def small_dataset(path=None):
    """[(updates, expected_text, expected_map, expected_array)] for every test of the corpus."""
    data = open(path or os.path.join(GOLDEN, "small-test-dataset.bin"), "rb").read()
    n, i = _rv(data, 0)
    out = []
    for _ in range(n):
        k, i = _rv(data, i)
        ups = []
        for _ in range(k):
            ln, i = _rv(data, i)
            ups.append(data[i:i + ln])
            i += ln
        ln, i = _rv(data, i)
        text = data[i:i + ln].decode("utf-8")
        i += ln
        m, i = read_any(data, i)
        a, i = read_any(data, i)
        out.append((ups, text, m, a))
    assert i == len(data)
    return out


def b4_update():
    """assets/bench-input/b4-update.bin: one 400,972-byte v1 update (yrs/benches/benches.rs:456-473)."""
    return open(os.path.join(GOLDEN, "b4-update.bin"), "rb").read()
