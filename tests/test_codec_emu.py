"""CPU pins of the device fast paths for strings and JSON against the general walks they
short-cut (tools/hostemu/codec_emu.cpp builds ycodec.h / yjson.h for the host).

* `str_fast16` (SWAR UTF-16 length, 16-byte vector loads) replaces the serial
  `utf8_next` walk of `SplittableString::len(Utf16)` (yrs/src/block.rs:1391-1401) for strings of
  >= 64 bytes, and when it accepts a string the `split_str` check (block.rs:1718-1729) is skipped.
  So `str_info16` must give the serial walk's length, re-encode flag and panic flag on every
  input, valid UTF-8 or not (yrs decodes content strings unchecked).
* `json_plain` accepts the texts serde_json re-serialises byte for byte; `json_canon` then
  copies them.  Every accepted text must come out of the general walk (`json_canon_walk`, the
  serde_json 1.0.116 restatement) unchanged, and the walk must agree with the oracle's
  independent restatement (oracle/yrs_oracle.c `yo_json_canon`).
"""
import ctypes
import os
import random
import subprocess

import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
EMU = os.path.join(os.path.dirname(HERE), "tools", "hostemu")
PAD = 64


@pytest.fixture(scope="module")
def emu():
    subprocess.check_call(["make", "-s", "-C", EMU, "libcodec_emu.so"])
    L = ctypes.CDLL(os.path.join(EMU, "libcodec_emu.so"))
    P32 = ctypes.POINTER(ctypes.c_uint32)
    for f in ("emu_str_info16", "emu_str_serial"):
        getattr(L, f).argtypes = [ctypes.c_void_p, ctypes.c_uint32, P32]
    L.emu_str_fast16.argtypes = [ctypes.c_void_p, ctypes.c_uint32, P32]
    L.emu_bytes_ascii.argtypes = [ctypes.c_void_p, ctypes.c_uint32]
    L.emu_json_plain.argtypes = [ctypes.c_void_p, ctypes.c_uint32]
    L.emu_json.argtypes = [ctypes.c_void_p, ctypes.c_uint32, ctypes.c_int, ctypes.c_void_p, ctypes.c_uint64]
    L.emu_json.restype = ctypes.c_int64
    return L


class Placed:
    """bytes at a chosen 16-byte phase inside a buffer with PAD readable bytes on both sides
    (the device arena's padding), filled with `fill` around the string"""

    def __init__(self, s, phase=0, fill=0xFF):
        self.buf = (ctypes.c_uint8 * (len(s) + 2 * PAD + 16))()
        base = ctypes.addressof(self.buf)
        start = ((base + PAD + 15) & ~15) + phase - base
        for i in range(len(self.buf)):
            self.buf[i] = fill
        for i, x in enumerate(s):
            self.buf[start + i] = x
        self.ptr = base + start
        self.n = len(s)


def info(L, fn, s, phase=0, fill=0xFF):
    p = Placed(s, phase, fill)
    out = (ctypes.c_uint32 * 3)()
    getattr(L, fn)(p.ptr, p.n, out)
    return tuple(out)


CRAFTED = [
    b"\xc0\x80", b"\xc1\xbf", b"\xe0\x80\x80", b"\xe0\x9f\xbf", b"\xe0\xa0\x80", b"\xf0\x80\x80\x80",
    b"\xf0\x8f\xbf\xbf", b"\xf0\x90\x80\x80", b"\xf4\x8f\xbf\xbf", b"\xf4\x90\x80\x80", b"\xf5\x80\x80\x80",
    b"\xf8\x88\x80\x80\x80", b"\xfc\x84\x80\x80\x80\x80", b"\xfe", b"\xff", b"\xed\xa0\x80", b"\xed\xbf\xbf",
    b"\xed\x9f\xbf", b"\xee\x80\x80", b"\x80", b"\xbf", b"\xc2", b"\xe2\x82", b"\xf0\x9f\x98", b"\xc2\x80",
    b"\xdf\xbf", b"\xef\xbf\xbf", b"\xf0\x9f\x98\x80", "é".encode(), "€".encode(), "😀".encode(),
]


def crafted_strings(rng):
    out = []
    for c in CRAFTED:
        for pre in (0, 1, 3, 15, 16, 17, 63, 64, 70):
            for post in (0, 1, 5, 16):
                out.append(b"a" * pre + c + b"b" * post)
        # cut off at the end (every prefix of a multi-byte sequence as the last bytes)
        for k in range(1, len(c)):
            out.append(b"x" * 64 + c[:k])
            out.append(b"x" * 61 + c[:k])
    for _ in range(300):
        n = rng.randrange(60, 200)
        out.append(b"".join(rng.choice(CRAFTED)[:rng.randrange(1, 5)] if rng.random() < 0.2 else b"q"
                            for _ in range(n)))
    return out


def random_strings(rng):
    alphabet = ["a", "Z", " ", "é", "ß", "€", "中", "😀", "ࠀ", "￿", "\U0010ffff", "\x7f"]
    out = []
    for _ in range(400):
        n = rng.randrange(1, 120)
        out.append("".join(rng.choice(alphabet) for _ in range(n)).encode())
    for _ in range(400):  # random bytes, biased to the high half
        n = rng.randrange(1, 200)
        out.append(bytes(rng.randrange(0x80, 0x100) if rng.random() < 0.6 else rng.randrange(0, 0x80)
                         for _ in range(n)))
    return out


def test_str_info16_equals_serial_walk(emu):
    rng = random.Random(1234)
    strings = crafted_strings(rng) + random_strings(rng)
    fast_taken = 0
    for s in strings:
        for phase in (0, 1, 5, 15) if len(s) < 400 else (0, 7):
            want = info(emu, "emu_str_serial", s, phase)
            got = info(emu, "emu_str_info16", s, phase)
            assert got == want, (s, phase)
            p = Placed(s, phase)
            n16 = ctypes.c_uint32()
            if len(s) >= 64 and emu.emu_str_fast16(p.ptr, p.n, ctypes.byref(n16)):
                fast_taken += 1
                assert (n16.value, 0, 0) == want, (s, phase)
    assert fast_taken > 100  # the fast path really ran


def test_str_fast16_every_phase_and_length(emu):
    """start / end offsets on every 16-byte phase; the padding bytes around the string must not
    change the result (0x00, 0x80 and 0xFF fills)"""
    rng = random.Random(99)
    base = "aé€😀".encode() * 40
    for _ in range(200):
        a = rng.randrange(0, 40)
        b = a + rng.randrange(64, 200)
        s = base[a:b]
        for phase in range(16):
            ref = info(emu, "emu_str_serial", s, phase)
            for fill in (0x00, 0x80, 0xFF):
                assert info(emu, "emu_str_info16", s, phase, fill) == ref, (a, b, phase, fill)


def test_bytes_ascii(emu):
    rng = random.Random(5)
    for _ in range(500):
        n = rng.randrange(0, 300)
        s = bytearray(rng.randrange(0, 0x80) for _ in range(n))
        if n and rng.random() < 0.5:
            s[rng.randrange(n)] |= 0x80
        for phase in (0, 3, 15):
            p = Placed(bytes(s), phase, fill=0xFF)
            assert emu.emu_bytes_ascii(p.ptr, p.n) == (1 if all(x < 0x80 for x in s) else 0)


def jcall(L, s, mode):
    p = Placed(s, 0, fill=0x20)
    out = (ctypes.c_uint8 * (4 * len(s) + 256))()
    n = L.emu_json(p.ptr, p.n, mode, out, len(out))
    return None if n < 0 else bytes(out[:n])


def plain_json(rng, depth=0):
    r = rng.random()
    if depth < 6 and r < 0.25:
        return "[" + ",".join(plain_json(rng, depth + 1) for _ in range(rng.randrange(0, 4))) + "]"
    if depth < 6 and r < 0.45:
        if rng.random() < 0.3:
            return "{}"
        return "{" + json_str(rng) + ":" + plain_json(rng, depth + 1) + "}"
    if r < 0.8:
        return json_str(rng)
    return rng.choice(["true", "false", "null"])


def json_str(rng):
    alphabet = ["a", "b", " ", "é", "€", "😀", "/", "'", "\x7f", "~"]
    return '"' + "".join(rng.choice(alphabet) for _ in range(rng.randrange(0, 12))) + '"'


MUST_REJECT = [
    '{"a":1}', "[1]", "-0", "1.5", '[ "a"]', '["a" ]', '{"a" :"b"}', '"a\\"b"', '"a\\nb"', '"\\u0041"',
    '"a\x01b"', '"tab\there"', '{"a":"x","b":"y"}', '{"a":"x","a":"y"}', "[" * 64 + "]" * 64, "[]]", "[,]",
    '["a",]', "tru", "nul", '"unterminated', "", " ", "\n[]", "[]\n", '{"k":}', "{:}", '{"a"}',
]


def test_json_plain_accepts_only_canonical_texts(emu, oracle):
    rng = random.Random(77)
    L = oracle.lib()
    P = ctypes.POINTER
    L.yo_json_canon.argtypes = [ctypes.c_char_p, ctypes.c_size_t, P(P(ctypes.c_uint8)), P(ctypes.c_size_t)]
    accepted = 0
    texts = [plain_json(rng) for _ in range(1500)] + ["[" * 63 + "]" * 63, "{" + '"k":' * 0 + "}"]
    for t in texts:
        s = t.encode()
        p = Placed(s)
        if not emu.emu_json_plain(p.ptr, p.n):
            continue
        accepted += 1
        walk = jcall(emu, s, 1)
        assert walk == s, t  # its own canonical form, by the general walk
        assert jcall(emu, s, 0) == s
        o = P(ctypes.c_uint8)()
        n = ctypes.c_size_t()
        assert L.yo_json_canon(s, len(s), ctypes.byref(o), ctypes.byref(n)) == 0, t
        assert ctypes.string_at(o, n.value) == s, t  # and by the oracle's restatement
        L.yo_free(o)
    assert accepted > 1000
    for t in MUST_REJECT:
        s = t.encode()
        p = Placed(s)
        assert not emu.emu_json_plain(p.ptr, p.n), t
        assert jcall(emu, s, 0) == jcall(emu, s, 1), t  # the shortcut is not taken: same bytes


def test_json_canon_equals_walk_on_mutations(emu):
    """whatever json_plain decides, json_canon and the general walk write the same bytes"""
    rng = random.Random(3)
    for _ in range(1500):
        s = bytearray(plain_json(rng).encode())
        for _ in range(rng.randrange(0, 3)):
            if not s:
                break
            i = rng.randrange(len(s))
            s[i:i] = rng.choice([b" ", b"\\", b"1", b",", b":", b"\x01", b'"', b"]", b"}", b"{", b"["])
        s = bytes(s)
        assert jcall(emu, s, 0) == jcall(emu, s, 1), s
