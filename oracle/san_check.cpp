// Sanitizer driver for the CPU oracle (TEST INFRASTRUCTURE ONLY; see rbref.h).
//
// `make -C oracle san` links this file with rbref.cpp under AddressSanitizer + UBSan
// (-fno-sanitize-recover: the first report aborts) and runs it: seeded random bitmaps of every
// container type go through each pairwise op (static, in-place, cardinality-only), every wide
// semantics, the serialize/deserialize round trip, and truncated / bit-flipped buffers that the
// decoder must reject or accept without touching memory out of bounds (the adversarial-input
// contract of TestAdversarialInputs.java:18-62).  Identities checked on the way:
// |A∪B| + |A∩B| = |A| + |B|, |A⊕B| = |A∪B| - |A∩B|, |A\B| = |A| - |A∩B|, and the single- and
// multi-threaded wide paths agree.  Exit status 0 = clean.
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
#include <vector>

#include "rbref.h"

namespace {
std::mt19937_64 rng;

// One bitmap over `nkeys` keys drawn from [0, 24): per key a sparse, dense or run-heavy container.
rbref_bitmap *random_bitmap(int nkeys) {
  std::vector<uint32_t> v;
  for (int k = 0; k < nkeys; ++k) {
    const uint32_t key = (uint32_t)(rng() % 24), base = key << 16;
    switch (rng() % 4) {
    case 0: { // sparse (Array)
      const int c = 1 + (int)(rng() % 300);
      for (int i = 0; i < c; ++i) v.push_back(base | (uint32_t)(rng() & 0xFFFF));
      break;
    }
    case 1: { // dense (Bitmap)
      const int c = 4097 + (int)(rng() % 20000);
      for (int i = 0; i < c; ++i) v.push_back(base | (uint32_t)(rng() & 0xFFFF));
      break;
    }
    case 2: { // runs
      uint32_t x = (uint32_t)(rng() % 512);
      const int nr = 1 + (int)(rng() % 200);
      for (int r = 0; r < nr && x < 65536; ++r) {
        const uint32_t len = 1 + (uint32_t)(rng() % 300);
        for (uint32_t i = 0; i < len && x + i < 65536; ++i) v.push_back(base | (x + i));
        x += len + 1 + (uint32_t)(rng() % 400);
      }
      break;
    }
    default: // full container
      for (uint32_t i = 0; i < 65536; ++i) v.push_back(base | i);
    }
  }
  rbref_bitmap *b = rbref_bitmap_of(v.data(), v.size());
  if (rng() % 2) rbref_run_optimize(b);
  return b;
}

int fails = 0;
void check(bool ok, const char *what, int it) {
  if (!ok) {
    std::fprintf(stderr, "san_check: %s failed (iteration %d)\n", what, it);
    ++fails;
  }
}

// no container of a result may be empty (RoaringArray never holds one; its serialized
// cardinality field would wrap to 65536)
bool no_empty(const rbref_bitmap *b) {
  for (uint32_t i = 0; i < rbref_container_count(b); ++i) {
    uint16_t k;
    uint8_t t;
    uint32_t c, r;
    rbref_container_info(b, i, &k, &t, &c, &r);
    if (c == 0) return false;
  }
  return true;
}

void round_trip(const rbref_bitmap *b, int it) {
  const uint64_t n = rbref_serialized_size(b);
  std::vector<uint8_t> buf(n);
  check(rbref_serialize(b, buf.data(), n) == RBREF_OK, "serialize", it);
  rbref_bitmap *d = nullptr;
  check(rbref_deserialize(buf.data(), n, &d) == RBREF_OK, "deserialize", it);
  if (d) {
    check(rbref_cardinality(d) == rbref_cardinality(b), "round-trip cardinality", it);
    rbref_free(d);
  }
  // truncations and bit flips: either rejected or decoded, never an out-of-bounds access
  for (int t = 0; t < 8 && n; ++t) {
    const size_t len = (size_t)(rng() % n);
    std::vector<uint8_t> cut(buf.begin(), buf.begin() + (long)len); // exact-size heap block
    rbref_bitmap *x = nullptr;
    if (rbref_deserialize(cut.data(), len, &x) == RBREF_OK && x) rbref_free(x);
    std::vector<uint8_t> flip(buf);
    flip[rng() % n] ^= (uint8_t)(1u << (rng() % 8));
    x = nullptr;
    if (rbref_deserialize(flip.data(), n, &x) == RBREF_OK && x) {
      (void)rbref_cardinality(x);
      rbref_free(x);
    }
  }
}
} // namespace

int main(int argc, char **argv) {
  const int iters = argc > 1 ? std::atoi(argv[1]) : 40;
  rng.seed(argc > 2 ? std::strtoull(argv[2], nullptr, 10) : 20261017ull);
  for (int it = 0; it < iters; ++it) {
    rbref_bitmap *a = random_bitmap((int)(rng() % 12)), *b = random_bitmap((int)(rng() % 12));
    const int64_t ca = (int64_t)rbref_cardinality(a), cb = (int64_t)rbref_cardinality(b);
    int64_t card[4];
    for (int op = 0; op < 4; ++op) {
      rbref_bitmap *r = rbref_op(op, a, b);
      card[op] = (int64_t)rbref_cardinality(r);
      check(rbref_op_cardinality(op, a, b) == card[op], "op cardinality", it);
      rbref_bitmap *ip = rbref_clone(a);
      check(rbref_op_inplace(op, ip, b) == RBREF_OK, "in-place op", it);
      check((int64_t)rbref_cardinality(ip) == card[op], "in-place cardinality", it);
      check(no_empty(r) && no_empty(ip), "no empty container (pairwise)", it);
      round_trip(r, it);
      rbref_free(ip);
      rbref_free(r);
    }
    check(card[RBREF_OR] + card[RBREF_AND] == ca + cb, "|A|B|+|A&B|", it);
    check(card[RBREF_XOR] == card[RBREF_OR] - card[RBREF_AND], "|A^B|", it);
    check(card[RBREF_ANDNOT] == ca - card[RBREF_AND], "|A\\B|", it);
    rbref_free(a);
    rbref_free(b);

    const int n = 2 + (int)(rng() % 6);
    std::vector<rbref_bitmap *> bs;
    for (int i = 0; i < n; ++i) bs.push_back(random_bitmap(1 + (int)(rng() % 8)));
    if (rng() % 3 == 0) bs.push_back(bs[0]); // pointer identity (naive_and)
    const rbref_bitmap *const *pb = bs.data();
    for (int sem = RBREF_FAST_OR; sem <= RBREF_PQ_XOR; ++sem) {
      rbref_bitmap *w = rbref_wide(sem, pb, bs.size());
      rbref_bitmap *m = rbref_wide_mt(sem, pb, bs.size(), 3);
      check(w && m && rbref_cardinality(w) == rbref_cardinality(m), "wide st == mt", it);
      // horizontal_xor appends a key's result even when empty (FastAggregation.java:278), whose
      // serialized card-1 then wraps; every other semantics drops empties
      const bool empties = w && !no_empty(w);
      if (empties && sem != RBREF_HORIZONTAL_XOR) {
        std::fprintf(stderr, "san_check: semantics %d left an empty container\n", sem);
        ++fails;
      }
      if (w && !empties) round_trip(w, it);
      rbref_free(w);
      rbref_free(m);
    }
    uint64_t tc = 0, tn = 0;
    check(rbref_pairwise_batch(RBREF_XOR, pb, pb + 1, bs.size() - 1, 2, &tc, &tn) == RBREF_OK, "pairwise batch", it);
    for (int i = 0; i < n; ++i) rbref_free(bs[i]);
  }
  std::printf("san_check: %d iterations, %d failures\n", iters, fails);
  return fails ? 1 : 0;
}
