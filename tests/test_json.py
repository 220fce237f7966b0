"""CPU pins of the JSON restatement behind ContentEmbed / ContentFormat (content refs 5/6).

yrs parses the JSON text with serde_json into an Any and writes it back with Any::to_json
(yrs/src/updates/decoder.rs:175-178, encoder.rs:170-174, any.rs:185-198,
encoding/serde/ser.rs:16-54).  No reference test holds re-serialised JSON bytes, so the
rules are restated from serde_json 1.0.116 / ryu 1.0.17 (Cargo.lock:725-726, 684-685) and
pinned here by: CPython's repr (an independent shortest round-trip float printer) for the
digit generator, hand-derived serde vectors for the parser and serializer, the offline
Yjs bundle on the reference's rich-text corpus (tests/golden/small_dataset_yjs_check.json).
Float text is "parity unpinned" against yrs itself: no reference vector holds one.
"""
import ctypes
import json
import math
import os
import random
import struct

import pytest

import corpus

HERE = os.path.dirname(os.path.abspath(__file__))


@pytest.fixture(scope="module")
def jlib(oracle):
    L = oracle.lib()
    P = ctypes.POINTER
    L.yo_json_canon.argtypes = [ctypes.c_char_p, ctypes.c_size_t, P(P(ctypes.c_uint8)), P(ctypes.c_size_t)]
    L.yo_f64_ryu.argtypes = [ctypes.c_double, ctypes.c_char_p, ctypes.c_size_t]
    return L


def canon(L, s):
    b = s.encode() if isinstance(s, str) else s
    o = ctypes.POINTER(ctypes.c_uint8)()
    n = ctypes.c_size_t()
    e = L.yo_json_canon(b, len(b), ctypes.byref(o), ctypes.byref(n))
    if e:
        return e
    r = ctypes.string_at(o, n.value)
    L.yo_free(o)
    return r


def ryu_layout(x):
    """ryu::Buffer::format_finite layout (ryu/src/pretty/mod.rs) over CPython's shortest digits."""
    if x == 0:
        return ("-" if math.copysign(1, x) < 0 else "") + "0.0"
    sign = "-" if x < 0 else ""
    r = repr(abs(x))
    m, e = (r.split("e") + ["0"])[:2]
    ip, fp = (m.split(".") + [""])[:2]
    digits, exp = (ip + fp).lstrip("0"), int(e) - len(fp)
    t = len(digits) - len(digits.rstrip("0"))
    digits, exp = digits.rstrip("0"), exp + t
    n = len(digits)
    kk = n + exp
    if 0 <= exp and kk <= 16:
        return sign + digits + "0" * (kk - n) + ".0"
    if 0 < kk <= 16:
        return sign + digits[:kk] + "." + digits[kk:]
    if -5 < kk <= 0:
        return sign + "0." + "0" * (-kk) + digits
    if n == 1:
        return sign + digits + "e" + str(kk - 1)
    return sign + digits[0] + "." + digits[1:] + "e" + str(kk - 1)


def test_shortest_digits_match_cpython(jlib):
    buf = ctypes.create_string_buffer(64)
    rnd = random.Random(7)
    xs = [0.1, 0.5, 1.5e-7, 1e21, 1e22, 123456.789, 5e-324, 2.2250738585072014e-308, 1.7976931348623157e308,
          1e16, 1e15, 0.3, 1 / 3, 1e-5, 1.2e-5, 0.001, 9.5367431640625e-07]
    xs += [2.0 ** e for e in range(-1074, 1024)]
    for i in range(60000):
        if i % 2:
            x = struct.unpack("<d", struct.pack("<Q", rnd.getrandbits(63)))[0]
        else:
            x = rnd.uniform(-1e6, 1e6) * 10.0 ** rnd.randint(-30, 30)
        if math.isfinite(x):
            xs.append(x)
    for x in xs:
        jlib.yo_f64_ryu(x, buf, 64)
        assert buf.value.decode() == ryu_layout(x), x


# (input, canonical output or InvalidJSON = 5), derived from serde_json's grammar and
# yrs' Any conversions (see the module docstring)
SERDE_VECTORS = [
    ('{"bold":true}', b'{"bold":true}'),
    (' { "a" : 1 , "b":[1,2.5,-0,1e2,1E-2,"x\\u0041\\n\\/"] } ', b'{"a":1,"b":[1,2.5,0,100,0.01,"xA\\n/"]}'),
    ('{"a":1,"a":2}', b'{"a":2}'),                     # HashMap insert: last value
    ('{"a":{"x":1},"b":2,"a":[3]}', b'{"b":2,"a":[3]}'),  # written at the last occurrence
    ('{"\\u0061":1,"a":2}', b'{"a":2}'),               # keys compare unescaped
    ('[1,]', 5), ('{"a":1,}', 5), ('01', 5), ('-', 5), ('1.', 5), ('.5', 5), ('1e', 5), ('+1', 5),
    ('"\\ud83d\\ude00"', '"\U0001F600"'.encode()), ('"\\ud83d"', 5), ('"\\ude00"', 5), ('"\\x"', 5),
    ('18446744073709551615', 5),                       # visit_u64 > i64::MAX: custom error
    ('9223372036854775807', b'9223372036854775807'),   # BigInt(v as f64 as i64) saturates
    ('9223372036854775808', 5),
    ('-9223372036854775808', b'-9223372036854775808'),
    ('-9223372036854775809', b'-9223372036854775808'),  # f64 path, then `as i64` saturates
    ('9007199254740993', b'9007199254740992'),         # u64 -> f64 rounding
    ('1e400', 5), ('1e-400', b'0'), ('-1e-400', b'0'),
    ('123456789012345678901234567890', b'1.2345678901234568e29'),
    ('0.1e1', b'1'), ('[[[]]]', b'[[[]]]'), ('"a\x01"', 5), ('"a\\u0001"', b'"a\\u0001"'),
    ('{"a":{"b":null}}', b'{"a":{"b":null}}'), ('1.5', b'1.5'), ('100000000000000000000.5', b'1e20'),
    ('"\\u00e9"', '"é"'.encode()), ('true ', b'true'), (' ', 5), ('', 5), ('{"k":1}x', 5),
    ('-0.0', b'0'), ('1e18', b'1000000000000000000'), ('1e19', b'1e19'), ('0.000001', b'1e-6'), ('0.00001', b'0.00001'),
    ('0.0000001', b'1e-7'), ('1.25e-7', b'1.25e-7'), ('[1e15]', b'[1000000000000000]'),
    ('{"a"}', 5), ('{1:2}', 5), ('nul', 5), ('[tru]', 5), ('"\t"', 5), ('"\x7f\xff"', b'"\x7f\xff"'),
]


@pytest.mark.parametrize("src,want", SERDE_VECTORS)
def test_serde_vectors(jlib, src, want):
    assert canon(jlib, src.encode("latin-1") if "\xff" in src else src) == want


def test_recursion_limit(jlib):
    assert canon(jlib, "[" * 127 + "]" * 127) == b"[" * 127 + b"]" * 127
    assert canon(jlib, "[" * 128 + "]" * 128) == 5
    assert canon(jlib, '{"a":' * 127 + "1" + "}" * 127).endswith(b"1" + b"}" * 127)
    assert canon(jlib, '{"a":' * 128 + "1" + "}" * 128) == 5


def _close(a, b):
    if isinstance(a, float) or isinstance(b, float):
        return math.isclose(a, b, rel_tol=1e-15, abs_tol=0)
    if isinstance(a, dict):
        return a.keys() == b.keys() and all(_close(a[k], b[k]) for k in a)
    if isinstance(a, list):
        return len(a) == len(b) and all(_close(x, y) for x, y in zip(a, b))
    return a == b


def test_python_json_roundtrip_agrees(jlib):
    """The canonical text re-parses to the same values; floats to within serde_json's
    non-float_roundtrip parse (significand * or / POW10, not correctly rounded)."""
    rnd = random.Random(3)
    for _ in range(2000):
        v = {"k%d" % j: rnd.choice([rnd.randint(-2**40, 2**40), rnd.random() * 10 ** rnd.randint(-8, 8), "s\n\"x",
                                     True, None, [1, 2.5]]) for j in range(rnd.randint(1, 4))}
        out = canon(jlib, json.dumps(v, indent=rnd.choice([None, 1])))
        assert isinstance(out, bytes)
        assert _close(json.loads(out), v), (v, out)


def _content_update(client, ref, payloads):
    """one update with one Item of content ref 5 (Embed) or 6 (Format) under root "text"."""
    def var(x):
        o = bytearray()
        while True:
            b, x = x & 0x7F, x >> 7
            o.append(b | (0x80 if x else 0))
            if not x:
                return bytes(o)
    def vs(b):
        return var(len(b)) + b
    body = bytes([ref]) + var(1) + vs(b"text") + b"".join(vs(p) for p in payloads)
    return var(1) + var(1) + var(client) + var(0) + body + var(0)


def test_embed_format_blocks_roundtrip(oracle):
    u = _content_update(7, 6, [b"bold", b' {"x" : 1.50, "x":true } '])
    m = oracle.merge_updates_v1([u])
    assert m == _content_update(7, 6, [b"bold", b'{"x":true}'])
    u = _content_update(7, 5, [b'{"image":"a.png"}'])
    assert oracle.merge_updates_v1([u]) == u
    st, _ = oracle.status_of(oracle.merge_updates_v1, [_content_update(7, 5, [b'{"image":'])])
    assert st == 5  # InvalidJSON at decode time
    st, _ = oracle.status_of(oracle.encode_state_vector_from_update_v1, _content_update(7, 6, [b"k", b"[1,]"]))
    assert st == 5


def test_any_map_duplicate_keys_collapse(oracle):
    """Any::decode inserts into a HashMap (any.rs:61-68): a repeated key keeps its last value."""
    def var(x):
        return bytes([x])
    def s(b):
        return var(len(b)) + b
    any_map = bytes([118, 3]) + s(b"a") + bytes([125, 1]) + s(b"b") + bytes([120]) + s(b"a") + bytes([125, 2])
    want_map = bytes([118, 2]) + s(b"b") + bytes([120]) + s(b"a") + bytes([125, 2])
    def upd(m):
        return bytes([1, 1, 9, 0, 0x08, 1]) + s(b"map") + bytes([1]) + m + bytes([0])
    assert oracle.merge_updates_v1([upd(any_map)]) == upd(want_map)


def test_small_dataset_oracle_pinned(oracle):
    """Every document of the reference's corpus merges with status 0, and the merge is the
    one the committed Yjs check validated (text/map/array values equal the corpus's)."""
    import hashlib
    fx = json.load(open(os.path.join(HERE, "golden", "small_dataset_yjs_check.json")))
    assert fx["docs"] == fx["text_equal"] == fx["map_equal"] == fx["array_equal"] == 5320
    docs = corpus.small_dataset()
    for k, (ups, _, _, _) in enumerate(docs):
        m = oracle.merge_updates_v1(ups, 1)
        assert hashlib.sha256(m).hexdigest()[:16] == fx["merge_sha256"][k], k
