// yjson.h — JSON text of ContentEmbed / ContentFormat (content refs 5/6) on gfx950.
//
// yrs decodes these through serde_json into an Any and re-serialises that Any when it
// encodes the block (read_json -> Any::from_json, write_json -> Any::to_json:
// yrs/src/updates/decoder.rs:175-178, yrs/src/updates/encoder.rs:170-174,
// yrs/src/any.rs:185-198).  This header restates, for device code, the same rules as
// the CPU oracle's JSON section (oracle/yrs_oracle.c):
//   serde_json 1.0.116 deserializer (default features): whitespace, literals, strings with
//     escapes and paired-surrogate validation, integers kept in u64 until they overflow,
//     f64_from_parts (significand as f64 times/divided by POW10[e]), recursion limit 128;
//   Deserialize for Any (yrs/src/encoding/serde/de.rs:17-211), From<i64> / TryFrom<u64>
//     (yrs/src/any.rs:243-318): unsafe integers become BigInt;
//   Serialize for Any (yrs/src/encoding/serde/ser.rs:16-54): `v as i64 as f64 == v` -> i64;
//   serde_json CompactFormatter escapes; ryu shortest f64 (format64 layout).
// Objects are HashMaps: duplicate keys collapse to the last value; an entry is written at
// the position of its key's last occurrence (the order of >= 2 distinct keys is random in
// yrs itself).  Any parse error is InvalidJSON (E_JSON).
#pragma once
// included by ycodec.h after its cursor/writer definitions (E_JSON, YM_TRY, Writer, Counter)

// (inside namespace ym)
__device__ __constant__ double kPow10[309] = {
    1e0, 1e1, 1e2, 1e3, 1e4, 1e5, 1e6, 1e7, 1e8, 1e9, 1e10, 1e11, 1e12, 1e13, 1e14, 1e15, 1e16, 1e17, 1e18, 1e19, 
    1e20, 1e21, 1e22, 1e23, 1e24, 1e25, 1e26, 1e27, 1e28, 1e29, 1e30, 1e31, 1e32, 1e33, 1e34, 1e35, 1e36, 1e37, 
    1e38, 1e39, 1e40, 1e41, 1e42, 1e43, 1e44, 1e45, 1e46, 1e47, 1e48, 1e49, 1e50, 1e51, 1e52, 1e53, 1e54, 1e55, 
    1e56, 1e57, 1e58, 1e59, 1e60, 1e61, 1e62, 1e63, 1e64, 1e65, 1e66, 1e67, 1e68, 1e69, 1e70, 1e71, 1e72, 1e73, 
    1e74, 1e75, 1e76, 1e77, 1e78, 1e79, 1e80, 1e81, 1e82, 1e83, 1e84, 1e85, 1e86, 1e87, 1e88, 1e89, 1e90, 1e91, 
    1e92, 1e93, 1e94, 1e95, 1e96, 1e97, 1e98, 1e99, 1e100, 1e101, 1e102, 1e103, 1e104, 1e105, 1e106, 1e107, 
    1e108, 1e109, 1e110, 1e111, 1e112, 1e113, 1e114, 1e115, 1e116, 1e117, 1e118, 1e119, 1e120, 1e121, 1e122, 
    1e123, 1e124, 1e125, 1e126, 1e127, 1e128, 1e129, 1e130, 1e131, 1e132, 1e133, 1e134, 1e135, 1e136, 1e137, 
    1e138, 1e139, 1e140, 1e141, 1e142, 1e143, 1e144, 1e145, 1e146, 1e147, 1e148, 1e149, 1e150, 1e151, 1e152, 
    1e153, 1e154, 1e155, 1e156, 1e157, 1e158, 1e159, 1e160, 1e161, 1e162, 1e163, 1e164, 1e165, 1e166, 1e167, 
    1e168, 1e169, 1e170, 1e171, 1e172, 1e173, 1e174, 1e175, 1e176, 1e177, 1e178, 1e179, 1e180, 1e181, 1e182, 
    1e183, 1e184, 1e185, 1e186, 1e187, 1e188, 1e189, 1e190, 1e191, 1e192, 1e193, 1e194, 1e195, 1e196, 1e197, 
    1e198, 1e199, 1e200, 1e201, 1e202, 1e203, 1e204, 1e205, 1e206, 1e207, 1e208, 1e209, 1e210, 1e211, 1e212, 
    1e213, 1e214, 1e215, 1e216, 1e217, 1e218, 1e219, 1e220, 1e221, 1e222, 1e223, 1e224, 1e225, 1e226, 1e227, 
    1e228, 1e229, 1e230, 1e231, 1e232, 1e233, 1e234, 1e235, 1e236, 1e237, 1e238, 1e239, 1e240, 1e241, 1e242, 
    1e243, 1e244, 1e245, 1e246, 1e247, 1e248, 1e249, 1e250, 1e251, 1e252, 1e253, 1e254, 1e255, 1e256, 1e257, 
    1e258, 1e259, 1e260, 1e261, 1e262, 1e263, 1e264, 1e265, 1e266, 1e267, 1e268, 1e269, 1e270, 1e271, 1e272, 
    1e273, 1e274, 1e275, 1e276, 1e277, 1e278, 1e279, 1e280, 1e281, 1e282, 1e283, 1e284, 1e285, 1e286, 1e287, 
    1e288, 1e289, 1e290, 1e291, 1e292, 1e293, 1e294, 1e295, 1e296, 1e297, 1e298, 1e299, 1e300, 1e301, 1e302, 
    1e303, 1e304, 1e305, 1e306, 1e307, 1e308};

// ---------------------------------------------------------------- sinks
// Output that can be muted: the value of a key that occurs again later in its object is
// validated but not written.
template <class W> struct JOut {
  W &w;
  bool mute;
  __device__ __forceinline__ void u8(uint8_t b) {
    if (!mute) w.u8(b);
  }
  __device__ __forceinline__ void lit(const char *s, uint32_t k) {
    if (!mute)
      for (uint32_t q = 0; q < k; q++) w.u8((uint8_t)s[q]);
  }
};

// ---------------------------------------------------------------- shortest f64 digits
// Burger & Dybvig free-format generation with exact big integers, ties to the even digit
// (ryu d2d).  x finite, > 0.  digits d1..dn, value = 0.d1..dn * 10^k.
constexpr int JBN = 40; // 1280 bits: r, s, m+, m- stay below 2^1140 for every double
struct JBig {
  uint32_t w[JBN];
};
// (the loops stay rolled: a fully unrolled JBig lives in registers, and f64_shortest's five of
// them took all 512 VGPRs, an allocation every kernel that can reach it inherited: one wave
// per SIMD; rolled, they live in scratch, touched only by the rare non-integral JSON number)
__device__ __forceinline__ void jb_set(JBig &a, uint64_t v) {
#pragma unroll 1
  for (int i = 0; i < JBN; i++) a.w[i] = 0;
  a.w[0] = (uint32_t)v;
  a.w[1] = (uint32_t)(v >> 32);
}
__device__ __forceinline__ void jb_mul10(JBig &a) {
  uint64_t c = 0;
#pragma unroll 1
  for (int i = 0; i < JBN; i++) {
    const uint64_t t = (uint64_t)a.w[i] * 10u + c;
    a.w[i] = (uint32_t)t;
    c = t >> 32;
  }
}
__device__ __forceinline__ void jb_shl(JBig &a, int k) {
  const int q = k >> 5, r = k & 31;
#pragma unroll 1
  for (int i = JBN - 1; i >= 0; i--) {
    const uint32_t hi = i - q >= 0 ? a.w[i - q] : 0;
    const uint32_t lo = i - q - 1 >= 0 ? a.w[i - q - 1] : 0;
    a.w[i] = r ? (hi << r) | (lo >> (32 - r)) : hi;
  }
}
__device__ __forceinline__ int jb_cmp(const JBig &a, const JBig &b) {
#pragma unroll 1
  for (int i = JBN - 1; i >= 0; i--)
    if (a.w[i] != b.w[i]) return a.w[i] < b.w[i] ? -1 : 1;
  return 0;
}
__device__ __forceinline__ void jb_add(JBig &r, const JBig &a, const JBig &b) {
  uint64_t c = 0;
#pragma unroll 1
  for (int i = 0; i < JBN; i++) {
    const uint64_t t = (uint64_t)a.w[i] + b.w[i] + c;
    r.w[i] = (uint32_t)t;
    c = t >> 32;
  }
}
__device__ __forceinline__ void jb_sub(JBig &a, const JBig &b) {
  uint64_t br = 0;
#pragma unroll 1
  for (int i = 0; i < JBN; i++) {
    const uint64_t t = (uint64_t)a.w[i] - b.w[i] - br;
    a.w[i] = (uint32_t)t;
    br = (t >> 32) & 1;
  }
}
__device__ __noinline__ int f64_shortest(double x, char *dg, int &k_out) {
  const uint64_t bits = (uint64_t)__double_as_longlong(x);
  const int be = (int)((bits >> 52) & 0x7FF);
  uint64_t f = bits & ((1ull << 52) - 1);
  int e;
  if (be == 0) {
    e = -1074;
  } else {
    f |= 1ull << 52;
    e = be - 1075;
  }
  const bool even = (f & 1) == 0;
  const bool unequal = be > 1 && f == (1ull << 52);
  JBig r, s, mp, mm, hi;
  jb_set(r, f);
  if (e >= 0) {
    jb_shl(r, e + (unequal ? 2 : 1));
    jb_set(s, unequal ? 4 : 2);
    jb_set(mp, 1);
    jb_shl(mp, e + (unequal ? 1 : 0));
    jb_set(mm, 1);
    jb_shl(mm, e);
  } else {
    jb_shl(r, unequal ? 2 : 1);
    jb_set(s, 1);
    jb_shl(s, -e + (unequal ? 2 : 1));
    jb_set(mp, unequal ? 2 : 1);
    jb_set(mm, 1);
  }
  int k = (int)ceil(log10(x) - 1e-10);
  if (k >= 0) {
    for (int q = 0; q < k; q++) jb_mul10(s);
  } else {
    for (int q = 0; q < -k; q++) {
      jb_mul10(r);
      jb_mul10(mp);
      jb_mul10(mm);
    }
  }
  for (;;) { // fixup: (r + m+) / s below 1 (at most 1 when the upper bound is inclusive)
    jb_add(hi, r, mp);
    int c = jb_cmp(hi, s);
    if (even ? c >= 0 : c > 0) {
      jb_mul10(s);
      k++;
      continue;
    }
    jb_mul10(hi);
    c = jb_cmp(hi, s);
    if (even ? c < 0 : c <= 0) {
      jb_mul10(r);
      jb_mul10(mp);
      jb_mul10(mm);
      k--;
      continue;
    }
    break;
  }
  int n = 0;
  for (;;) {
    jb_mul10(r);
    jb_mul10(mp);
    jb_mul10(mm);
    int d = 0;
    while (jb_cmp(r, s) >= 0) {
      jb_sub(r, s);
      d++;
    }
    const int cl = jb_cmp(r, mm);
    const bool tc1 = even ? cl <= 0 : cl < 0;
    jb_add(hi, r, mp);
    const int ch = jb_cmp(hi, s);
    const bool tc2 = even ? ch >= 0 : ch > 0;
    if (!tc1 && !tc2 && n < 24) {
      dg[n++] = (char)('0' + d);
      continue;
    }
    if (tc1 && tc2) {
      jb_add(hi, r, r);
      const int c2 = jb_cmp(hi, s);
      if (c2 > 0 || (c2 == 0 && (d & 1))) d++;
    } else if (tc2) {
      d++;
    }
    dg[n++] = (char)('0' + d);
    break;
  }
  for (int q = n - 1; q > 0 && dg[q] > '9'; q--) {
    dg[q] = '0';
    dg[q - 1]++;
  }
  if (dg[0] > '9') {
    dg[0] = '1';
    k++;
  }
  while (n > 1 && dg[n - 1] == '0') n--;
  k_out = k;
  return n;
}

template <class O> __device__ __forceinline__ void j_uint(O &o, uint64_t v) {
  char b[20];
  int n = 0;
  do {
    b[n++] = (char)('0' + v % 10);
    v /= 10;
  } while (v);
  while (n) o.u8((uint8_t)b[--n]);
}
template <class O> __device__ __forceinline__ void j_i64(O &o, int64_t v) { // itoa
  if (v < 0) {
    o.u8('-');
    j_uint(o, (uint64_t)0 - (uint64_t)v);
  } else {
    j_uint(o, (uint64_t)v);
  }
}
// ryu::Buffer::format_finite (format64)
template <class O> __device__ __noinline__ void j_ryu(O &o, double x) {
  if (signbit(x)) o.u8('-');
  if (x == 0.0) {
    o.lit("0.0", 3);
    return;
  }
  char dg[26];
  int kk;
  const int len = f64_shortest(fabs(x), dg, kk);
  const int k = kk - len;
  if (0 <= k && kk <= 16) {
    for (int i = 0; i < len; i++) o.u8((uint8_t)dg[i]);
    for (int i = len; i < kk; i++) o.u8('0');
    o.lit(".0", 2);
  } else if (0 < kk && kk <= 16) {
    for (int i = 0; i < kk; i++) o.u8((uint8_t)dg[i]);
    o.u8('.');
    for (int i = kk; i < len; i++) o.u8((uint8_t)dg[i]);
  } else if (-5 < kk && kk <= 0) {
    o.lit("0.", 2);
    for (int i = 0; i < -kk; i++) o.u8('0');
    for (int i = 0; i < len; i++) o.u8((uint8_t)dg[i]);
  } else {
    o.u8((uint8_t)dg[0]);
    if (len > 1) {
      o.u8('.');
      for (int i = 1; i < len; i++) o.u8((uint8_t)dg[i]);
    }
    o.u8('e');
    j_i64(o, kk - 1);
  }
}
// Serialize for Any, Any::Number (ser.rs:25-34)
template <class O> __device__ __forceinline__ void j_number(O &o, double x) {
  int64_t i;
  if (x != x) i = 0;
  else if (x >= 9223372036854775808.0) i = INT64_MAX; // Rust `as` saturates
  else if (x < -9223372036854775808.0) i = INT64_MIN;
  else i = (int64_t)x;
  if ((double)i == x) j_i64(o, i);
  else if (isfinite(x)) j_ryu(o, x);
  else o.lit("null", 4);
}

// ---------------------------------------------------------------- scanning helpers
__device__ __forceinline__ bool j_isws(uint8_t c) { return c == ' ' || c == '\n' || c == '\t' || c == '\r'; }
__device__ __forceinline__ uint32_t j_ws(const uint8_t *s, uint32_t n, uint32_t i) {
  while (i < n && j_isws(s[i])) i++;
  return i;
}
__device__ __forceinline__ int j_hex(uint8_t c) {
  if (c >= '0' && c <= '9') return c - '0';
  if (c >= 'a' && c <= 'f') return c - 'a' + 10;
  if (c >= 'A' && c <= 'F') return c - 'A' + 10;
  return -1;
}
__device__ __forceinline__ int j_hex4(const uint8_t *s, uint32_t n, uint32_t i, uint32_t &v) {
  if (n - i < 4 || i > n) return E_JSON;
  uint32_t x = 0;
  for (int q = 0; q < 4; q++) {
    const int h = j_hex(s[i + q]);
    if (h < 0) return E_JSON;
    x = x << 4 | (uint32_t)h;
  }
  v = x;
  return 0;
}
// Iterator over the unescaped bytes of the string literal whose opening quote is at i:
// next() returns the next byte, -1 at the closing quote, -2 on malformed input.
struct JStr {
  const uint8_t *s;
  uint32_t n, i;
  uint8_t b[4];
  int bl, bi;
  __device__ JStr(const uint8_t *s_, uint32_t n_, uint32_t i_) : s(s_), n(n_), i(i_ + 1), bl(0), bi(0) {}
  __device__ int next() {
    if (bi < bl) return b[bi++];
    if (i >= n) return -2;
    const uint8_t c = s[i++];
    if (c == '"') return -1;
    if (c < 0x20) return -2;
    if (c != '\\') return c;
    if (i >= n) return -2;
    const uint8_t e = s[i++];
    switch (e) {
    case '"': case '\\': case '/': return e;
    case 'b': return '\b';
    case 'f': return '\f';
    case 'n': return '\n';
    case 'r': return '\r';
    case 't': return '\t';
    case 'u': {
      uint32_t c1;
      if (j_hex4(s, n, i, c1)) return -2;
      i += 4;
      if (c1 >= 0xDC00 && c1 <= 0xDFFF) return -2;
      if (c1 >= 0xD800 && c1 <= 0xDBFF) {
        uint32_t c2;
        if (n - i < 2 || s[i] != '\\' || s[i + 1] != 'u' || j_hex4(s, n, i + 2, c2)) return -2;
        if (c2 < 0xDC00 || c2 > 0xDFFF) return -2;
        i += 6;
        c1 = (((c1 - 0xD800) << 10) | (c2 - 0xDC00)) + 0x10000;
      }
      bl = 0;
      bi = 0;
      if (c1 < 0x80) {
        b[bl++] = (uint8_t)c1;
      } else if (c1 < 0x800) {
        b[bl++] = (uint8_t)(0xC0 | c1 >> 6);
        b[bl++] = (uint8_t)(0x80 | (c1 & 63));
      } else if (c1 < 0x10000) {
        b[bl++] = (uint8_t)(0xE0 | c1 >> 12);
        b[bl++] = (uint8_t)(0x80 | ((c1 >> 6) & 63));
        b[bl++] = (uint8_t)(0x80 | (c1 & 63));
      } else {
        b[bl++] = (uint8_t)(0xF0 | c1 >> 18);
        b[bl++] = (uint8_t)(0x80 | ((c1 >> 12) & 63));
        b[bl++] = (uint8_t)(0x80 | ((c1 >> 6) & 63));
        b[bl++] = (uint8_t)(0x80 | (c1 & 63));
      }
      return b[bi++];
    }
    default: return -2;
    }
  }
};
// string literal at i -> escaped output (serde_json format_escaped_str); returns the index
// after the closing quote or ~0u on an error
template <class O> __device__ __forceinline__ uint32_t j_string(const uint8_t *s, uint32_t n, uint32_t i, O &o) {
  JStr it(s, n, i);
  o.u8('"');
  for (;;) {
    const int c = it.next();
    if (c == -1) break;
    if (c < 0) return ~0u;
    switch (c) {
    case '"': o.lit("\\\"", 2); break;
    case '\\': o.lit("\\\\", 2); break;
    case '\b': o.lit("\\b", 2); break;
    case '\f': o.lit("\\f", 2); break;
    case '\n': o.lit("\\n", 2); break;
    case '\r': o.lit("\\r", 2); break;
    case '\t': o.lit("\\t", 2); break;
    default:
      if (c < 0x20) {
        o.lit("\\u00", 4);
        o.u8((uint8_t)("0123456789abcdef"[c >> 4]));
        o.u8((uint8_t)("0123456789abcdef"[c & 15]));
      } else {
        o.u8((uint8_t)c);
      }
    }
  }
  o.u8('"');
  return it.i;
}
// index after the value starting at/after i (no validation: malformed input is rejected
// by the main parse); n on malformed input
__device__ __forceinline__ uint32_t j_skip(const uint8_t *s, uint32_t n, uint32_t i) {
  i = j_ws(s, n, i);
  int depth = 0;
  while (i < n) {
    const uint8_t c = s[i];
    if (c == '"') {
      i++;
      while (i < n && s[i] != '"') i += s[i] == '\\' ? 2 : 1;
      i++;
      if (depth == 0) return i < n ? i : n;
      continue;
    }
    if (c == '{' || c == '[') {
      depth++;
      i++;
      continue;
    }
    if (c == '}' || c == ']') {
      if (depth == 0) return i;
      depth--;
      i++;
      if (depth == 0) return i;
      continue;
    }
    if (depth == 0 && (c == ',' || j_isws(c))) return i;
    i++;
  }
  return n;
}
// does a later entry of the object being parsed repeat the key whose quote is at i?
__device__ __noinline__ bool j_key_repeats(const uint8_t *s, uint32_t n, uint32_t i) {
  JStr k0(s, n, i);
  while (k0.next() >= 0) {
  }
  uint32_t j = j_ws(s, n, k0.i);
  if (j >= n || s[j] != ':') return false;
  j = j_skip(s, n, j + 1);
  for (;;) {
    j = j_ws(s, n, j);
    if (j >= n || s[j] != ',') return false;
    j = j_ws(s, n, j + 1);
    if (j >= n || s[j] != '"') return false;
    JStr a(s, n, i), b(s, n, j);
    bool same = true;
    for (;;) {
      const int ca = a.next(), cb = b.next();
      if (ca != cb) {
        same = false;
        break;
      }
      if (ca < 0) break;
    }
    if (same) return true;
    while (b.next() >= 0) {
    }
    j = j_ws(s, n, b.i);
    if (j >= n || s[j] != ':') return false;
    j = j_skip(s, n, j + 1);
  }
}

// ---------------------------------------------------------------- numbers
__device__ __forceinline__ int j_from_parts(bool positive, uint64_t sig, int64_t exponent, double &out) {
  double f = (double)sig;
  for (;;) {
    const uint64_t ae = exponent < 0 ? (uint64_t)(-exponent) : (uint64_t)exponent;
    if (ae <= 308) {
      if (exponent >= 0) {
        f *= kPow10[ae];
        if (isinf(f)) return E_JSON;
      } else {
        f /= kPow10[ae];
      }
      break;
    }
    if (f == 0.0) break;
    if (exponent >= 0) return E_JSON;
    f /= 1e308;
    exponent += 308;
  }
  out = positive ? f : -f;
  return 0;
}
__device__ __forceinline__ bool j_ovf(uint64_t a, uint64_t b, uint64_t c) { return a >= c / 10 && (a > c / 10 || b > c % 10); }
__device__ __forceinline__ int j_exponent(const uint8_t *s, uint32_t n, uint32_t &i, bool positive, uint64_t sig,
                                          int64_t start, double &out) {
  i++;
  bool pos_exp = true;
  if (i < n && s[i] == '+') {
    i++;
  } else if (i < n && s[i] == '-') {
    i++;
    pos_exp = false;
  }
  if (i >= n || s[i] < '0' || s[i] > '9') return E_JSON;
  int32_t ex = s[i++] - '0';
  while (i < n && s[i] >= '0' && s[i] <= '9') {
    const int32_t dd = s[i++] - '0';
    if (j_ovf((uint64_t)ex, (uint64_t)dd, 0x7FFFFFFFu)) { // parse_exponent_overflow
      if (sig != 0 && pos_exp) return E_JSON;
      while (i < n && s[i] >= '0' && s[i] <= '9') i++;
      out = positive ? 0.0 : -0.0;
      return 0;
    }
    ex = ex * 10 + dd;
  }
  int64_t fe = pos_exp ? start + ex : start - ex; // i32 saturating_add / saturating_sub
  if (fe > INT32_MAX) fe = INT32_MAX;
  if (fe < INT32_MIN) fe = INT32_MIN;
  return j_from_parts(positive, sig, fe, out);
}
__device__ __forceinline__ int j_decimal(const uint8_t *s, uint32_t n, uint32_t &i, bool positive, uint64_t sig,
                                         int64_t before, double &out) {
  i++;
  int64_t after = 0;
  while (i < n && s[i] >= '0' && s[i] <= '9') {
    const uint64_t dd = s[i] - '0';
    if (j_ovf(sig, dd, ~0ull)) { // parse_decimal_overflow: ignore further digits
      while (i < n && s[i] >= '0' && s[i] <= '9') i++;
      if (i < n && (s[i] == 'e' || s[i] == 'E')) return j_exponent(s, n, i, positive, sig, before + after, out);
      return j_from_parts(positive, sig, before + after, out);
    }
    i++;
    sig = sig * 10 + dd;
    after--;
  }
  if (after == 0) return E_JSON;
  if (i < n && (s[i] == 'e' || s[i] == 'E')) return j_exponent(s, n, i, positive, sig, before + after, out);
  return j_from_parts(positive, sig, before + after, out);
}
// a number (the '-' consumed when !positive) -> Any -> text
template <class O> __device__ __noinline__ int j_num(const uint8_t *s, uint32_t n, uint32_t &i, bool positive, O &o) {
  if (i >= n || s[i] < '0' || s[i] > '9') return E_JSON;
  const uint8_t c0 = s[i++];
  uint64_t sig = c0 - '0';
  double f;
  if (c0 == '0') {
    if (i < n && s[i] >= '0' && s[i] <= '9') return E_JSON;
  } else {
    while (i < n && s[i] >= '0' && s[i] <= '9') {
      const uint64_t dd = s[i] - '0';
      if (j_ovf(sig, dd, ~0ull)) { // parse_long_integer
        int64_t ex = 0;
        while (i < n && s[i] >= '0' && s[i] <= '9') {
          i++;
          ex++;
        }
        int e;
        if (i < n && s[i] == '.') e = j_decimal(s, n, i, positive, sig, ex, f);
        else if (i < n && (s[i] == 'e' || s[i] == 'E')) e = j_exponent(s, n, i, positive, sig, ex, f);
        else e = j_from_parts(positive, sig, ex, f);
        if (e) return e;
        j_number(o, f);
        return 0;
      }
      i++;
      sig = sig * 10 + dd;
    }
  }
  if (i < n && s[i] == '.') {
    YM_TRY(j_decimal(s, n, i, positive, sig, 0, f));
    j_number(o, f);
    return 0;
  }
  if (i < n && (s[i] == 'e' || s[i] == 'E')) {
    YM_TRY(j_exponent(s, n, i, positive, sig, 0, f));
    j_number(o, f);
    return 0;
  }
  if (positive) { // visit_u64 -> TryFrom<u64> for Any
    if (sig > (uint64_t)INT64_MAX) return E_JSON;
    const double v = (double)sig;
    if (v <= 9007199254740991.0) j_number(o, v);
    else j_i64(o, v >= 9223372036854775808.0 ? INT64_MAX : (int64_t)v); // BigInt(v as f64 as i64)
    return 0;
  }
  const int64_t neg = (int64_t)(0 - sig);
  if (neg >= 0) { // -0, or below i64::MIN: visit_f64(-(significand as f64))
    j_number(o, -(double)sig);
    return 0;
  }
  const double v = (double)neg; // visit_i64 -> From<i64>
  if (v >= -9007199254740991.0) j_number(o, v);
  else j_i64(o, neg);
  return 0;
}

// ---------------------------------------------------------------- the walk
// Texts serde_json re-serialises byte for byte: well-formed, no whitespace, no numbers, strings
// without escapes or control bytes (j_string writes every other byte as is), objects of at most
// one key (no repeated-key question), <= 63 levels.  Read 16 bytes at a time (independent
// loads): the general walk below reads byte by byte over HBM and took ~370 k cycles for a
// 110-byte Embed of the corpus (tools/blockbench.hip).  true = the text is its own canonical form.
__device__ __forceinline__ bool json_plain(const uint8_t *s, uint32_t n) {
  enum : uint32_t { PV, PV0, PK0, PS, PC, PL, PA };
  uint32_t st = PV, litw = 0, litn = 0, depth = 0;
  uint64_t obj = 0, keyed = 0; // per level: an object / an object that has its key
  bool key = false;
  if (n == 0) return false;
  for (uint32_t i0 = 0; i0 < n; i0 += 16) {
    uint8_t t[16];
#pragma unroll
    for (uint32_t j = 0; j < 16; j++) t[j] = i0 + j < n ? s[i0 + j] : 0;
    const uint32_t jn = n - i0 < 16 ? n - i0 : 16;
    for (uint32_t j = 0; j < jn; j++) {
      uint32_t c = 0; // (t[j] through a select chain: t stays in registers)
#pragma unroll
      for (uint32_t q = 0; q < 16; q++) c = q == j ? t[q] : c;
      if (st == PS) {
        if (c == '"') st = key ? PC : PA;
        else if (c == '\\' || c < 0x20) return false;
        continue;
      }
      if (st == PL) {
        if (c != (litw & 0xFF)) return false;
        litw >>= 8;
        if (--litn == 0) st = PA;
        continue;
      }
      if (st == PC) {
        if (c != ':') return false;
        st = PV;
        continue;
      }
      if (st == PA) {
        if (depth == 0) return false;
        const uint64_t top = 1ull << (depth - 1);
        if (c == ',') {
          if (obj & top) return false; // a second key
          st = PV;
        } else if (c == (obj & top ? '}' : ']')) {
          depth--;
          obj &= ~top;
          keyed &= ~top;
        } else {
          return false;
        }
        continue;
      }
      if (st == PK0) {
        if (c == '}') {
          depth--;
          obj &= ~(1ull << depth);
          st = PA;
        } else if (c == '"') {
          keyed |= 1ull << (depth - 1);
          key = true;
          st = PS;
        } else {
          return false;
        }
        continue;
      }
      // a value (PV), or a value or ']' right after '[' (PV0)
      if (st == PV0 && c == ']') {
        depth--;
        st = PA;
      } else if (c == '{' || c == '[') {
        if (depth >= 63) return false;
        if (c == '{') obj |= 1ull << depth;
        depth++;
        st = c == '{' ? PK0 : PV0;
      } else if (c == '"') {
        key = false;
        st = PS;
      } else if (c == 't') {
        litw = 'r' | 'u' << 8 | 'e' << 16;
        litn = 3;
        st = PL;
      } else if (c == 'f') {
        litw = 'a' | 'l' << 8 | 's' << 16 | (uint32_t)'e' << 24;
        litn = 4;
        st = PL;
      } else if (c == 'n') {
        litw = 'u' | 'l' << 8 | 'l' << 16;
        litn = 3;
        st = PL;
      } else {
        return false; // numbers, whitespace, anything else: the general walk
      }
    }
  }
  (void)keyed;
  return st == PA && depth == 0;
}

// serde_json::from_str::<Any>(s[0..n]) then Any::to_json into w, by the general walk (every
// text; json_canon takes the json_plain shortcut first); 0 or E_JSON.
template <class W> __device__ __noinline__ int json_canon_walk(const uint8_t *s, uint32_t n, W &w) {
  JOut<W> o{w, false};
  uint32_t isobj[4] = {0, 0, 0, 0}, first[4] = {0, 0, 0, 0};
  int depth = 0;      // open containers (serde_json allows 127)
  int mute_from = 0;  // object depth whose current entry is muted (0: none)
  uint32_t i = j_ws(s, n, 0);
  bool want_value = true;
  auto bit = [](const uint32_t *m, int d) { return (m[d >> 5] >> (d & 31)) & 1u; };
  auto setb = [](uint32_t *m, int d, bool v) {
    if (v) m[d >> 5] |= 1u << (d & 31);
    else m[d >> 5] &= ~(1u << (d & 31));
  };
  // an object entry: key at i (after whitespace)
  auto entry = [&]() -> int {
    if (i >= n || s[i] != '"') return E_JSON;
    if (mute_from == 0 && j_key_repeats(s, n, i)) {
      mute_from = depth;
      o.mute = true;
    }
    if (!o.mute) {
      if (!bit(first, depth - 1)) o.u8(',');
      setb(first, depth - 1, false);
    }
    const uint32_t e = j_string(s, n, i, o);
    if (e == ~0u) return E_JSON;
    i = j_ws(s, n, e);
    if (i >= n || s[i] != ':') return E_JSON;
    o.u8(':');
    i = j_ws(s, n, i + 1);
    return 0;
  };
  for (;;) {
    if (want_value) {
      if (i >= n) return E_JSON;
      const uint8_t c = s[i];
      if (c == '{' || c == '[') {
        if (depth >= 127) return E_JSON; // RecursionLimitExceeded (remaining_depth 128)
        setb(isobj, depth, c == '{');
        setb(first, depth, true);
        depth++;
        o.u8(c);
        i = j_ws(s, n, i + 1);
        const uint8_t close = c == '{' ? '}' : ']';
        if (i < n && s[i] == close) {
          i++;
          depth--;
          o.u8(close);
          want_value = false;
        } else if (c == '{') {
          YM_TRY(entry());
        }
        continue;
      }
      if (c == '"') {
        const uint32_t e = j_string(s, n, i, o);
        if (e == ~0u) return E_JSON;
        i = e;
      } else if (c == 'n' || c == 't' || c == 'f') {
        const char *lit = c == 'n' ? "null" : c == 't' ? "true" : "false";
        const uint32_t ln = c == 'f' ? 5 : 4;
        if (n - i < ln) return E_JSON;
        for (uint32_t q = 0; q < ln; q++)
          if (s[i + q] != (uint8_t)lit[q]) return E_JSON;
        i += ln;
        o.lit(lit, ln);
      } else if (c == '-') {
        i++;
        YM_TRY(j_num(s, n, i, false, o));
      } else if (c >= '0' && c <= '9') {
        YM_TRY(j_num(s, n, i, true, o));
      } else {
        return E_JSON;
      }
      want_value = false;
      continue;
    }
    // after a value
    if (depth == 0) return j_ws(s, n, i) == n ? 0 : E_JSON; // TrailingCharacters
    const bool obj = bit(isobj, depth - 1);
    if (obj && mute_from == depth) { // the muted entry's value is complete
      mute_from = 0;
      o.mute = false;
    }
    i = j_ws(s, n, i);
    if (i >= n) return E_JSON;
    const uint8_t c = s[i];
    const uint8_t close = obj ? '}' : ']';
    if (c == close) {
      i++;
      depth--;
      o.u8(close);
      continue;
    }
    if (c != ',') return E_JSON;
    i = j_ws(s, n, i + 1);
    if (i < n && s[i] == close) return E_JSON; // trailing comma
    if (obj) {
      YM_TRY(entry());
    } else {
      o.u8(',');
    }
    want_value = true;
  }
}

// serde_json::from_str::<Any>(s[0..n]) then Any::to_json into w; 0 or E_JSON.  A text that is
// its own canonical form (json_plain) is copied; tests/test_codec_emu.py checks that every text
// json_plain accepts comes out of the general walk byte for byte.
template <class W> __device__ __noinline__ int json_canon(const uint8_t *s, uint32_t n, W &w) {
  if (json_plain(s, n)) {
    w.bytes(s, n);
    return 0;
  }
  return json_canon_walk(s, n, w);
}
