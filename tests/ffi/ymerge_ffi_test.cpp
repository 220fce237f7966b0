// ymerge_ffi_test.cpp — C++ harness for the C ABI (include/ymerge.h), linked against
// libymerge.so the way the reference's FFI suite links yffi (tests-ffi/main.cpp:38-50,
// 74-93: peers exchange state vectors and diffs through the C entry points and compare).
//
// Cases: the byte-exact KATs of yrs/src/alt.rs:103-160 through the single-document calls,
// error reporting (ymerge_last_error), the host-memory batch entries, an update exchange
// between two peers (state vector -> diff -> merge, both sides converge), and concurrent
// callers (the header's thread-safety contract).  Prints "N passed, M failed"; exit 1 on
// any failure.  Needs a GPU (run by tests/test_gpu_host_abi.py::test_ffi_binary).
#include "ymerge.h"

#include <cstdio>
#include <cstring>
#include <string>
#include <thread>
#include <vector>

using Bytes = std::vector<uint8_t>;
static int g_pass = 0, g_fail = 0;
#define CHECK(cond)                                                                                                   \
  do {                                                                                                                \
    if (cond) g_pass++;                                                                                               \
    else {                                                                                                            \
      g_fail++;                                                                                                       \
      printf("FAIL %s:%d: %s\n", __FILE__, __LINE__, #cond);                                                          \
    }                                                                                                                 \
  } while (0)

// yrs/src/alt.rs:103-160
static const Bytes MERGE1_A = {1, 1, 220, 240, 237, 172, 15, 0, 4, 1, 4, 116, 101, 115, 116, 3, 97, 98, 99, 0};
static const Bytes MERGE1_B = {1, 1, 201, 139, 250, 201, 1, 0, 4, 1, 4, 116, 101, 115, 116, 2, 100, 101, 0};
static const Bytes MERGE1_X = {2,   1,   220, 240, 237, 172, 15, 0, 4, 1, 4, 116, 101, 115, 116, 3,   97,  98, 99,
                               1,   201, 139, 250, 201, 1,   0,  4, 1, 4, 116, 101, 115, 116, 2,   100, 101, 0};
static const Bytes MERGE2_A = {1, 1, 129, 231, 135, 164, 7, 0, 4, 1, 4, 49, 50, 51, 52, 1, 97, 0};
static const Bytes MERGE2_B = {1, 1, 129, 231, 135, 164, 7, 1, 68, 129, 231, 135, 164, 7, 0, 1, 98, 0};
static const Bytes MERGE2_X = {1, 2,  129, 231, 135, 164, 7,   0,   4,   1,   4, 49, 50, 51,
                               52, 1, 97,  68,  129, 231, 135, 164, 7, 0, 1,  98, 0};
static const Bytes SV_U = MERGE1_X;
static const Bytes SV_X = {2, 220, 240, 237, 172, 15, 3, 201, 139, 250, 201, 1, 2};
static const Bytes DIFF_U = {1,  2, 148, 189, 145, 162, 9, 0,   4,   1,   4,   116, 101, 115, 116,
                             3, 97, 98,  99,  68,  148, 189, 145, 162, 9, 0, 2,   100, 101, 0};
static const Bytes DIFF_SV = {1, 148, 189, 145, 162, 9, 3};
static const Bytes DIFF_X = {1, 1, 148, 189, 145, 162, 9, 3, 68, 148, 189, 145, 162, 9, 0, 2, 100, 101, 0};

static Bytes take(char *p, uint32_t n) {
  Bytes r;
  if (p) {
    r.assign((uint8_t *)p, (uint8_t *)p + n);
    ymerge_binary_destroy(p, n);
  }
  return r;
}
static Bytes merge(const std::vector<Bytes> &ups) {
  std::vector<const char *> ptr;
  std::vector<uint32_t> len;
  for (auto &u : ups) {
    ptr.push_back((const char *)u.data());
    len.push_back((uint32_t)u.size());
  }
  uint32_t n = 0;
  char *r = ymerge_updates_v1(ptr.data(), len.data(), (uint32_t)ups.size(), &n);
  return r ? take(r, n) : Bytes{0xEE}; // 0xEE: "failed" marker (never a valid result)
}
static Bytes state_vector(const Bytes &u) {
  uint32_t n = 0;
  char *r = yencode_state_vector_from_update_v1((const char *)u.data(), (uint32_t)u.size(), &n);
  return r ? take(r, n) : Bytes{0xEE};
}
static Bytes diff(const Bytes &u, const Bytes &sv) {
  uint32_t n = 0;
  char *r = ydiff_updates_v1((const char *)u.data(), (uint32_t)u.size(), (const char *)sv.data(), (uint32_t)sv.size(),
                             &n);
  return r ? take(r, n) : Bytes{0xEE};
}

// A peer's text edit as one v1 update: one String item of `text` by `client` at `clock`,
// root type "test", no origins (what ytext_insert at position 0 of an empty text sends).
static Bytes insert_update(uint32_t client, uint32_t clock, const char *text) {
  Bytes u;
  auto var = [&](uint64_t v) {
    while (v >= 0x80) {
      u.push_back((uint8_t)(v | 0x80));
      v >>= 7;
    }
    u.push_back((uint8_t)v);
  };
  var(1);
  var(1);
  var(client);
  var(clock);
  u.push_back(4); // info: String content, no origins -> parent follows
  var(1);         // parent: named root type
  var(4);
  for (const char *c = "test"; *c; c++) u.push_back((uint8_t)*c);
  var(strlen(text));
  for (const char *c = text; *c; c++) u.push_back((uint8_t)*c);
  var(0); // empty DeleteSet
  return u;
}

static void test_alt_kats() {
  CHECK(merge({MERGE1_A, MERGE1_B}) == MERGE1_X);
  CHECK(merge({MERGE2_A, MERGE2_B}) == MERGE2_X);
  CHECK(state_vector(SV_U) == SV_X);
  CHECK(diff(DIFF_U, DIFF_SV) == DIFF_X);
  CHECK(ymerge_last_error() == 0);
}

static void test_errors() {
  uint32_t n = 7;
  const char *p = "";
  uint32_t l = 0;
  CHECK(ymerge_updates_v1(&p, &l, 1, &n) == nullptr);
  CHECK(ymerge_last_error() == YMERGE_ERR_EOS); // Update::decode on an empty buffer
  Bytes bad(12, 0x80);
  CHECK(yencode_state_vector_from_update_v1((const char *)bad.data(), (uint32_t)bad.size(), &n) == nullptr);
  CHECK(ymerge_last_error() == YMERGE_ERR_VAR_INT);
  CHECK(merge({MERGE1_A}) == MERGE1_A); // a success clears the error
  CHECK(ymerge_last_error() == 0);
}

// Two peers edit concurrently, then exchange SV -> diff -> merge (tests-ffi/main.cpp:74-93)
static void test_update_exchange() {
  const Bytes u1 = insert_update(1, 0, "world"), u2 = insert_update(2, 0, "hello ");
  Bytes sv1 = state_vector(u1), sv2 = state_vector(u2);
  Bytes d1 = diff(u1, sv2), d2 = diff(u2, sv1);
  CHECK(d1 == u1 && d2 == u2); // neither peer has seen the other's client
  Bytes p1 = merge({u1, d2}), p2 = merge({u2, d1});
  CHECK(p1 == p2); // both peers converge on the same compacted update
  CHECK(state_vector(p1) == state_vector(p2));
  CHECK(diff(p1, state_vector(p2)) == Bytes({0, 0})); // nothing left to send
  // a third edit by peer 1, delivered as a diff against peer 2's state vector
  const Bytes u3 = insert_update(1, 5, "!");
  Bytes p1b = merge({p1, u3});
  Bytes d3 = diff(p1b, state_vector(p2));
  CHECK(d3 == u3);
  CHECK(merge({p2, d3}) == p1b);
}

static void test_host_batch() {
  ymerge_ctx *c = ymerge_ctx_create(0);
  CHECK(c != nullptr);
  if (!c) return;
  // documents: KAT 1, KAT 2, an empty document, an empty update (EOS)
  std::vector<Bytes> ups = {MERGE1_A, MERGE1_B, MERGE2_A, MERGE2_B, Bytes{}};
  Bytes arena;
  std::vector<uint64_t> off = {0};
  for (auto &u : ups) {
    arena.insert(arena.end(), u.begin(), u.end());
    off.push_back(arena.size());
  }
  std::vector<uint64_t> doc = {0, 2, 4, 4, 5};
  ymerge_batch_result *r = nullptr;
  CHECK(ymerge_updates_v1_batch(c, arena.data(), off.data(), 5, doc.data(), 4, &r) == 0);
  if (r) {
    CHECK(r->n_docs == 4);
    CHECK(Bytes(r->out + r->out_off[0], r->out + r->out_off[1]) == MERGE1_X);
    CHECK(Bytes(r->out + r->out_off[1], r->out + r->out_off[2]) == MERGE2_X);
    CHECK(Bytes(r->out + r->out_off[2], r->out + r->out_off[3]) == Bytes({0, 0})); // merge of nothing
    CHECK(r->status[0] == 0 && r->status[1] == 0 && r->status[2] == 0 && r->status[3] == YMERGE_ERR_EOS);
    ymerge_batch_result_destroy(r);
  }
  // state vectors + diffs: one update per document
  Bytes ua;
  std::vector<uint64_t> uo = {0};
  for (const Bytes *u : {&SV_U, &DIFF_U}) {
    ua.insert(ua.end(), u->begin(), u->end());
    uo.push_back(ua.size());
  }
  r = nullptr;
  CHECK(yencode_state_vector_from_update_v1_batch(c, ua.data(), uo.data(), 2, &r) == 0);
  if (r) {
    CHECK(Bytes(r->out + r->out_off[0], r->out + r->out_off[1]) == SV_X);
    ymerge_batch_result_destroy(r);
  }
  Bytes sva = {0};
  sva.insert(sva.end(), DIFF_SV.begin(), DIFF_SV.end());
  std::vector<uint64_t> so = {0, 1, sva.size()};
  r = nullptr;
  CHECK(ydiff_updates_v1_batch(c, ua.data(), uo.data(), sva.data(), so.data(), 2, &r) == 0);
  if (r) {
    CHECK(Bytes(r->out + r->out_off[0], r->out + r->out_off[1]) == SV_U); // diff against {} = the update
    CHECK(Bytes(r->out + r->out_off[1], r->out + r->out_off[2]) == DIFF_X);
    ymerge_batch_result_destroy(r);
  }
  // y-sync: SyncStep1 greeting, then the SyncStep2 reply to a client's SyncStep1
  r = nullptr;
  CHECK(ysync_step1_v1_batch(c, ua.data(), uo.data(), 2, &r) == 0);
  if (r) {
    Bytes m(r->out + r->out_off[0], r->out + r->out_off[1]);
    Bytes want = {0, 0, (uint8_t)SV_X.size()};
    want.insert(want.end(), SV_X.begin(), SV_X.end());
    CHECK(m == want); // Message::Sync(SyncStep1(sv)) = [0, 0, varbuf(sv)]
    ymerge_batch_result_destroy(r);
  }
  Bytes msg = {0, 0, 1, 0, 0, 0, (uint8_t)DIFF_SV.size()};
  msg.insert(msg.end(), DIFF_SV.begin(), DIFF_SV.end());
  std::vector<uint64_t> mo = {0, 4, msg.size()};
  r = nullptr;
  CHECK(ysync_step2_v1_batch(c, ua.data(), uo.data(), msg.data(), mo.data(), 2, &r) == 0);
  if (r) {
    Bytes want = {0, 1, (uint8_t)DIFF_X.size()};
    want.insert(want.end(), DIFF_X.begin(), DIFF_X.end());
    CHECK(Bytes(r->out + r->out_off[1], r->out + r->out_off[2]) == want);
    ymerge_batch_result_destroy(r);
  }
  ymerge_stats st{};
  ymerge_last_stats(c, &st);
  CHECK(st.n_docs == 2);
  ymerge_ctx_destroy(c);
}

static void test_threads() {
  std::vector<std::thread> th;
  std::vector<int> ok(8, 0);
  for (int t = 0; t < 8; t++)
    th.emplace_back([&, t] {
      int good = 1;
      for (int i = 0; i < 20; i++) {
        good &= merge({MERGE1_A, MERGE1_B}) == MERGE1_X;
        good &= diff(DIFF_U, DIFF_SV) == DIFF_X;
      }
      ok[t] = good;
    });
  for (auto &x : th) x.join();
  for (int t = 0; t < 8; t++) CHECK(ok[t] == 1);
}

int main() {
  test_alt_kats();
  test_errors();
  test_update_exchange();
  test_host_batch();
  test_threads();
  printf("%d passed, %d failed\n", g_pass, g_fail);
  return g_fail ? 1 : 0;
}
