// rbref.cpp — CPU restatement of the reference RoaringBitmap set-algebra path.
//
// TEST INFRASTRUCTURE ONLY (see rbref.h): the parity oracle and the timed CPU baseline.
// Never linked into the product library.
//
// The restatement follows the reference's *control flow* for every container operation
// (which container type each branch returns, how run lists are merged), because the
// serialized bytes are fixed by those type decisions.  All citations are relative to
// /root/reference/RoaringBitmap/src/main/java/org/roaringbitmap/.
#include "rbref.h"

#include <algorithm>
#include <atomic>
#include <cstring>
#include <map>
#include <memory>
#include <thread>
#include <vector>

namespace {

constexpr uint8_t kA = RBREF_ARRAY, kB = RBREF_BITMAP, kR = RBREF_RUN;
constexpr int kMaxArray = 4096;       // ArrayContainer.DEFAULT_MAX_SIZE (ArrayContainer.java:27)
constexpr int kArrayLazyLower = 1024; // ArrayContainer.ARRAY_LAZY_LOWERBOUND (ArrayContainer.java:25)
constexpr int kWords = 1024;          // BitmapContainer.MAX_CAPACITY / 64
constexpr int kSpan = 65536;
constexpr int kRunArrayThreshold = 32; // RunContainer.andNot/xor "arbitrary_threshold" (:576, :2412)

// One container.  Array: v = sorted values, card = v.size().  Bitmap: w = 1024 words,
// card = cardinality or -1 when "lazy" (BitmapContainer card -1 convention, :657-685).
// Run: v = interleaved (start, length-1) pairs (RunContainer.valueslength, :92-99).
struct Cont {
  uint8_t t = kA;
  int card = 0;
  std::vector<uint16_t> v;
  std::vector<uint64_t> w;
  int nruns() const { return (int)(v.size() / 2); }
  int rs(int i) const { return v[2 * i]; }
  int rl(int i) const { return v[2 * i + 1]; }
};

inline int popcnt(uint64_t x) { return __builtin_popcountll(x); }

// ---------------------------------------------------------------- Util.java word-range kernels
// Util.setBitmapRange (:616-631), resetBitmapRange (:505-522), flipBitmapRange (:366-377),
// ranges are [start, end).
void word_range(std::vector<uint64_t> &w, int start, int end, int mode) {
  if (start >= end) return;
  int fw = start >> 6, lw = (end - 1) >> 6;
  for (int i = fw; i <= lw; ++i) {
    uint64_t m = ~0ull;
    if (i == fw) m &= ~0ull << (start & 63);
    if (i == lw) m &= ~0ull >> (63 - ((end - 1) & 63));
    if (mode == 0) w[i] |= m;
    else if (mode == 1) w[i] &= ~m;
    else w[i] ^= m;
  }
}
inline bool bit(const std::vector<uint64_t> &w, int x) { return (w[x >> 6] >> (x & 63)) & 1; }
int words_card(const std::vector<uint64_t> &w) {
  int c = 0;
  for (uint64_t x : w) c += popcnt(x);
  return c;
}

// ---------------------------------------------------------------- constructors / conversions
Cont make_array(std::vector<uint16_t> vals) {
  Cont c;
  c.t = kA;
  c.card = (int)vals.size();
  c.v = std::move(vals);
  return c;
}
Cont make_bitmap(std::vector<uint64_t> w, int card) {
  Cont c;
  c.t = kB;
  c.card = card;
  c.w = std::move(w);
  return c;
}
Cont make_run(std::vector<uint16_t> vl) {
  Cont c;
  c.t = kR;
  c.v = std::move(vl);
  c.card = 0;
  return c;
}
Cont full_run() { return make_run({0, 0xFFFF}); } // RunContainer.full() (:1663-1665)

int run_card(const Cont &r) { // RunContainer.getCardinality (:1003-1009)
  int s = r.nruns();
  for (int i = 0; i < r.nruns(); ++i) s += r.rl(i);
  return s;
}
int cardinality(const Cont &c) { return c.t == kR ? run_card(c) : c.card; }
bool is_empty(const Cont &c) { // isEmpty of each container type
  if (c.t == kR) return c.nruns() == 0;
  return c.card == 0;
}
bool run_is_full(const Cont &r) { // RunContainer.isFull (:1659-1661)
  return r.nruns() == 1 && r.rs(0) == 0 && r.rl(0) == 0xFFFF;
}

Cont bitmap_to_array(const Cont &b) { // BitmapContainer.toArrayContainer (:1313-1322)
  std::vector<uint16_t> out;
  out.reserve(b.card > 0 ? b.card : 0);
  for (int i = 0; i < kWords; ++i) {
    uint64_t x = b.w[i];
    while (x) {
      out.push_back((uint16_t)(i * 64 + __builtin_ctzll(x)));
      x &= x - 1;
    }
  }
  return make_array(std::move(out));
}
std::vector<uint64_t> array_words(const std::vector<uint16_t> &vals) {
  std::vector<uint64_t> w(kWords, 0);
  for (uint16_t x : vals) w[x >> 6] |= 1ull << (x & 63);
  return w;
}
std::vector<uint64_t> run_words(const Cont &r) {
  std::vector<uint64_t> w(kWords, 0);
  for (int i = 0; i < r.nruns(); ++i) word_range(w, r.rs(i), r.rs(i) + r.rl(i) + 1, 0);
  return w;
}
// Container.toBitmapContainer: Array (ArrayContainer.java:1126-1130), Run (RunContainer.java:2634-2646),
// Bitmap returns itself (BitmapContainer.java:1676-1678).
Cont to_bitmap(const Cont &c) {
  if (c.t == kB) return c;
  if (c.t == kA) return make_bitmap(array_words(c.v), c.card);
  return make_bitmap(run_words(c), run_card(c));
}
std::vector<uint16_t> run_values(const Cont &r) {
  std::vector<uint16_t> out;
  for (int i = 0; i < r.nruns(); ++i)
    for (int x = r.rs(i); x <= r.rs(i) + r.rl(i); ++x) out.push_back((uint16_t)x);
  return out;
}
// RunContainer.toBitmapOrArrayContainer (:2300-2323)
Cont run_to_bitmap_or_array(const Cont &r, int card) {
  if (card <= kMaxArray) return make_array(run_values(r));
  return make_bitmap(run_words(r), card);
}
// RunContainer.toEfficientContainer (:2326-2335): stays Run iff 2+4r <= min(8192, 2c+2)
Cont run_eff(Cont r) {
  int size_run = 2 + 4 * r.nruns();
  int card = run_card(r);
  int size_arr = 2 * card + 2;
  if (size_run <= std::min(8192, size_arr)) return r;
  return run_to_bitmap_or_array(r, card);
}
// BitmapContainer.repairAfterLazy (:1214-1224)
Cont bitmap_repair(Cont b) {
  if (b.card < 0) {
    b.card = words_card(b.w);
    if (b.card <= kMaxArray) return bitmap_to_array(b);
    if (b.card == kSpan) return full_run();
  }
  return b;
}
// Container.repairAfterLazy per type: Array (ArrayContainer.java:1080), Bitmap, Run (RunContainer.java:2073)
Cont repair(Cont c) {
  if (c.t == kA) return c;
  if (c.t == kB) return bitmap_repair(std::move(c));
  return run_eff(std::move(c));
}
// maximal runs of a sorted array (RunContainer(ArrayContainer,int) :110-140)
std::vector<uint16_t> runs_of_array(const std::vector<uint16_t> &a) {
  std::vector<uint16_t> out;
  int prev = -2, len = 0;
  for (uint16_t x : a) {
    if (x == prev + 1) {
      ++len;
    } else {
      if (!out.empty()) out.back() = (uint16_t)len;
      out.push_back(x);
      out.push_back(0);
      len = 0;
    }
    prev = x;
  }
  if (!out.empty()) out.back() = (uint16_t)len;
  return out;
}
// maximal runs of a bitmap (RunContainer(BitmapContainer,int) :145-197)
std::vector<uint16_t> runs_of_words(const std::vector<uint64_t> &w) {
  std::vector<uint16_t> out;
  int x = 0;
  while (x < kSpan) {
    if (!bit(w, x)) {
      ++x;
      continue;
    }
    int s = x;
    while (x < kSpan && bit(w, x)) ++x;
    out.push_back((uint16_t)s);
    out.push_back((uint16_t)(x - s - 1));
  }
  return out;
}
int runs_count_words(const std::vector<uint64_t> &w) {
  int r = 0;
  uint64_t prev_top = 0;
  for (int i = 0; i < kWords; ++i) {
    uint64_t x = w[i];
    r += popcnt(x & ~((x << 1) | prev_top));
    prev_top = x >> 63;
  }
  return r;
}
int runs_count_array(const std::vector<uint16_t> &a) { // ArrayContainer.numberOfRuns (:932-946)
  if (a.empty()) return 0;
  int r = 1;
  for (size_t i = 1; i < a.size(); ++i)
    if (a[i - 1] + 1 != a[i]) ++r;
  return r;
}
// Container.runOptimize: Array (:1085-1099) → Run iff 2c > 2+4r; Bitmap (:1227-1246) → Run iff
// 8192 > 2+4r (the lower-bound early exit only fires when 2+4r >= 8192); Run → toEfficientContainer.
Cont run_optimize(Cont c) {
  if (c.t == kA) {
    int r = runs_count_array(c.v);
    if (2 * c.card > 2 + 4 * r) return make_run(runs_of_array(c.v));
    return c;
  }
  if (c.t == kB) {
    int r = runs_count_words(c.w);
    if (8192 > 2 + 4 * r) return make_run(runs_of_words(c.w));
    return c;
  }
  return run_eff(std::move(c));
}

// ---------------------------------------------------------------- sorted u16 set kernels (Util.java)
std::vector<uint16_t> arr_and(const std::vector<uint16_t> &a, const std::vector<uint16_t> &b) {
  std::vector<uint16_t> o; // Util.unsignedIntersect2by2 (:890-900)
  std::set_intersection(a.begin(), a.end(), b.begin(), b.end(), std::back_inserter(o));
  return o;
}
std::vector<uint16_t> arr_or(const std::vector<uint16_t> &a, const std::vector<uint16_t> &b) {
  std::vector<uint16_t> o; // Util.unsignedUnion2by2 (:1116-1168)
  std::set_union(a.begin(), a.end(), b.begin(), b.end(), std::back_inserter(o));
  return o;
}
std::vector<uint16_t> arr_xor(const std::vector<uint16_t> &a, const std::vector<uint16_t> &b) {
  std::vector<uint16_t> o; // Util.unsignedExclusiveUnion2by2 (:829-876)
  std::set_symmetric_difference(a.begin(), a.end(), b.begin(), b.end(), std::back_inserter(o));
  return o;
}
std::vector<uint16_t> arr_andnot(const std::vector<uint16_t> &a, const std::vector<uint16_t> &b) {
  std::vector<uint16_t> o; // Util.unsignedDifference (:717-816)
  std::set_difference(a.begin(), a.end(), b.begin(), b.end(), std::back_inserter(o));
  return o;
}

// ---------------------------------------------------------------- run-list builders
// A run list under construction, ints, (start, length-1) like RunContainer.valueslength.
struct RunList {
  std::vector<int> v;
  int n() const { return (int)(v.size() / 2); }
  int s(int i) const { return v[2 * i]; }
  int l(int i) const { return v[2 * i + 1]; }
  void push(int s, int l) {
    v.push_back(s);
    v.push_back(l);
  }
  // RunContainer.smartAppend(char start, char length) (:2191-2207)
  void smart_append(int start, int length) {
    int oldend;
    if (n() == 0 || start > (oldend = s(n() - 1) + l(n() - 1)) + 1) {
      push(start, length);
      return;
    }
    int newend = start + length + 1;
    if (newend > oldend) v[2 * (n() - 1) + 1] = newend - 1 - s(n() - 1);
  }
  void smart_append(int val) { smart_append(val, 0); } // (:2175-2189), identical effect for one value
  // RunContainer.smartAppendExclusive(char start, char length) (:2245-2292)
  void smart_append_excl(int start, int length) {
    int oldend;
    if (n() == 0 || start > (oldend = s(n() - 1) + l(n() - 1) + 1)) {
      push(start, length);
      return;
    }
    int last = n() - 1;
    if (oldend == start) {
      v[2 * last + 1] += length + 1;
      return;
    }
    int newend = start + length + 1;
    if (start == s(last)) {
      if (newend < oldend) {
        v[2 * last] = newend;
        v[2 * last + 1] = oldend - newend - 1;
      } else if (newend > oldend) {
        v[2 * last] = oldend;
        v[2 * last + 1] = newend - oldend - 1;
      } else {
        v.resize(v.size() - 2);
      }
      return;
    }
    v[2 * last + 1] = start - s(last) - 1;
    if (newend < oldend) push(newend, oldend - newend - 1);
    else if (newend > oldend) push(oldend, newend - oldend - 1);
  }
  void smart_append_excl(int val) { smart_append_excl(val, 0); } // (:2209-2243), same effect
  bool is_full() const { return n() == 1 && s(0) == 0 && l(0) == 0xFFFF; }
  Cont cont() const {
    std::vector<uint16_t> o(v.size());
    for (size_t i = 0; i < v.size(); ++i) o[i] = (uint16_t)v[i];
    return make_run(std::move(o));
  }
};

// RunContainer.and(RunContainer) (:381-456) — intersection list then toEfficientContainer.
Cont run_and_run(const Cont &x, const Cont &y) {
  RunList ans;
  if (x.nruns() == 0 || y.nruns() == 0) return ans.cont();
  int i = 0, j = 0;
  int s = x.rs(0), e = s + x.rl(0) + 1, ys = y.rs(0), ye = ys + y.rl(0) + 1;
  while (i < x.nruns() && j < y.nruns()) {
    if (e <= ys) {
      if (++i < x.nruns()) { s = x.rs(i); e = s + x.rl(i) + 1; }
    } else if (ye <= s) {
      if (++j < y.nruns()) { ys = y.rs(j); ye = ys + y.rl(j) + 1; }
    } else {
      int lo = std::max(s, ys), hi;
      if (e == ye) {
        hi = e;
        if (++i < x.nruns()) { s = x.rs(i); e = s + x.rl(i) + 1; }
        if (++j < y.nruns()) { ys = y.rs(j); ye = ys + y.rl(j) + 1; }
      } else if (e < ye) {
        hi = e;
        if (++i < x.nruns()) { s = x.rs(i); e = s + x.rl(i) + 1; }
      } else {
        hi = ye;
        if (++j < y.nruns()) { ys = y.rs(j); ye = ys + y.rl(j) + 1; }
      }
      ans.push(lo, hi - lo - 1);
    }
  }
  return run_eff(ans.cont());
}
// RunContainer.andNot(RunContainer) (:624-692)
Cont run_andnot_run(const Cont &x, const Cont &y) {
  RunList ans;
  if (x.nruns() == 0) return ans.cont();
  if (y.nruns() == 0) return run_eff(x);
  int i = 0, j = 0;
  int s = x.rs(0), e = s + x.rl(0) + 1, ys = y.rs(0), ye = ys + y.rl(0) + 1;
  while (i < x.nruns() && j < y.nruns()) {
    if (e <= ys) {
      ans.push(s, e - s - 1);
      if (++i < x.nruns()) { s = x.rs(i); e = s + x.rl(i) + 1; }
    } else if (ye <= s) {
      if (++j < y.nruns()) { ys = y.rs(j); ye = ys + y.rl(j) + 1; }
    } else {
      if (s < ys) ans.push(s, ys - s - 1);
      if (ye < e) {
        s = ye;
      } else if (++i < x.nruns()) {
        s = x.rs(i);
        e = s + x.rl(i) + 1;
      }
    }
  }
  if (i < x.nruns()) {
    ans.push(s, e - s - 1);
    for (++i; i < x.nruns(); ++i) ans.push(x.rs(i), x.rl(i));
  }
  return run_eff(ans.cont());
}
// RunContainer.lazyandNot(ArrayContainer) (:1707-1763), not yet made efficient.
Cont run_lazy_andnot_array(const Cont &x, const Cont &a) {
  if (a.card == 0) return x;
  RunList ans;
  if (x.nruns() == 0) return ans.cont();
  int i = 0, j = 0;
  int s = x.rs(0), e = s + x.rl(0) + 1, xs = a.v[0];
  while (i < x.nruns() && j < a.card) {
    if (e <= xs) {
      ans.push(s, e - s - 1);
      if (++i < x.nruns()) { s = x.rs(i); e = s + x.rl(i) + 1; }
    } else if (xs + 1 <= s) {
      if (++j < a.card) xs = a.v[j];
    } else {
      if (s < xs) ans.push(s, xs - s - 1);
      if (xs + 1 < e) {
        s = xs + 1;
      } else if (++i < x.nruns()) {
        s = x.rs(i);
        e = s + x.rl(i) + 1;
      }
    }
  }
  if (i < x.nruns()) {
    ans.push(s, e - s - 1);
    for (++i; i < x.nruns(); ++i) ans.push(x.rs(i), x.rl(i));
  }
  return ans.cont();
}
// RunContainer.lazyorToRun(ArrayContainer) (:1769-1813): Run, full Run, or lazy Bitmap when
// the merged list has more than 4096 runs (convertToLazyBitmapIfNeeded :861-875).
Cont run_lazy_or_array(const Cont &x, const Cont &a) {
  if (run_is_full(x)) return full_run();
  RunList ans;
  int i = 0, k = 0;
  while (k < a.card && i < x.nruns()) {
    if (x.rs(i) - (int)a.v[k] <= 0) {
      ans.smart_append(x.rs(i), x.rl(i));
      ++i;
    } else {
      ans.smart_append(a.v[k++]);
    }
  }
  if (k < a.card) {
    while (k < a.card) ans.smart_append(a.v[k++]);
  } else {
    while (i < x.nruns()) { ans.smart_append(x.rs(i), x.rl(i)); ++i; }
  }
  if (ans.is_full()) return full_run();
  Cont r = ans.cont();
  if (r.nruns() > kMaxArray) {
    Cont b = make_bitmap(run_words(r), -1);
    return b;
  }
  return r;
}
// RunContainer.lazyxor(ArrayContainer) (:1815-1852)
Cont run_lazy_xor_array(const Cont &x, const Cont &a) {
  if (a.card == 0) return x;
  if (x.nruns() == 0) return a;
  RunList ans;
  int i = 0, k = 0;
  int cv = a.v[k++];
  while (true) {
    if (x.rs(i) < cv) {
      ans.smart_append_excl(x.rs(i), x.rl(i));
      if (++i == x.nruns()) {
        ans.smart_append_excl(cv);
        while (k < a.card) ans.smart_append_excl(a.v[k++]);
        break;
      }
    } else {
      ans.smart_append_excl(cv);
      if (k == a.card) {
        while (i < x.nruns()) { ans.smart_append_excl(x.rs(i), x.rl(i)); ++i; }
        break;
      }
      cv = a.v[k++];
    }
  }
  return ans.cont();
}
// RunContainer.or(RunContainer) (:1948-1986)
Cont run_or_run(const Cont &x, const Cont &y) {
  if (run_is_full(x) || run_is_full(y)) return full_run();
  RunList ans;
  int i = 0, j = 0;
  while (j < y.nruns() && i < x.nruns()) {
    if (x.rs(i) - y.rs(j) <= 0) { ans.smart_append(x.rs(i), x.rl(i)); ++i; }
    else { ans.smart_append(y.rs(j), y.rl(j)); ++j; }
  }
  while (j < y.nruns()) { ans.smart_append(y.rs(j), y.rl(j)); ++j; }
  while (i < x.nruns()) { ans.smart_append(x.rs(i), x.rl(i)); ++i; }
  if (ans.is_full()) return full_run();
  return run_eff(ans.cont());
}
// RunContainer.xor(RunContainer) (:2448-2482)
Cont run_xor_run(const Cont &x, const Cont &y) {
  if (y.nruns() == 0) return x;
  if (x.nruns() == 0) return y;
  RunList ans;
  int i = 0, j = 0;
  while (true) {
    if (x.rs(i) < y.rs(j)) {
      ans.smart_append_excl(x.rs(i), x.rl(i));
      if (++i == x.nruns()) {
        while (j < y.nruns()) { ans.smart_append_excl(y.rs(j), y.rl(j)); ++j; }
        break;
      }
    } else {
      ans.smart_append_excl(y.rs(j), y.rl(j));
      if (++j == y.nruns()) {
        while (i < x.nruns()) { ans.smart_append_excl(x.rs(i), x.rl(i)); ++i; }
        break;
      }
    }
  }
  return run_eff(ans.cont());
}

// ---------------------------------------------------------------- Bitmap-side helpers
Cont ab_from_words(std::vector<uint64_t> w, int card) { // "card > 4096 ? Bitmap : Array"
  Cont b = make_bitmap(std::move(w), card);
  if (card > kMaxArray) return b;
  return bitmap_to_array(b);
}
std::vector<uint16_t> array_filter(const std::vector<uint16_t> &a, const std::vector<uint64_t> &w,
                                   bool keep_set) {
  std::vector<uint16_t> o;
  for (uint16_t x : a)
    if (bit(w, x) == keep_set) o.push_back(x);
  return o;
}
// BitmapContainer.or(ArrayContainer) (:1073-1094): Bitmap, or full Run.
Cont bitmap_or_array(const Cont &b, const Cont &a) {
  Cont r = b;
  for (uint16_t x : a.v) {
    uint64_t &wd = r.w[x >> 6];
    uint64_t aft = wd | (1ull << (x & 63));
    r.card += (wd != aft);
    wd = aft;
  }
  if (r.card == kSpan) return full_run();
  return r;
}
// BitmapContainer.xor(ArrayContainer) (:1381-1398) and ixor(ArrayContainer) (:837-852)
Cont bitmap_xor_array(const Cont &b, const Cont &a) {
  Cont r = b;
  for (uint16_t x : a.v) {
    uint64_t &wd = r.w[x >> 6];
    uint64_t m = 1ull << (x & 63);
    r.card += (wd & m) ? -1 : 1;
    wd ^= m;
  }
  if (r.card <= kMaxArray) return bitmap_to_array(r);
  return r;
}
// BitmapContainer.andNot(ArrayContainer) (:221-237)
Cont bitmap_andnot_array(const Cont &b, const Cont &a) {
  Cont r = b;
  for (uint16_t x : a.v) {
    uint64_t &wd = r.w[x >> 6];
    uint64_t m = 1ull << (x & 63);
    if (wd & m) --r.card;
    wd &= ~m;
  }
  if (r.card <= kMaxArray) return bitmap_to_array(r);
  return r;
}
// RunContainer.and(ArrayContainer) (:305-336): array values that fall inside a run.
std::vector<uint16_t> array_in_runs(const std::vector<uint16_t> &a, const Cont &r, bool inside) {
  std::vector<uint16_t> o;
  int i = 0;
  for (uint16_t x : a) {
    while (i < r.nruns() && r.rs(i) + r.rl(i) < x) ++i;
    bool in = i < r.nruns() && r.rs(i) <= x;
    if (in == inside) o.push_back(x);
  }
  return o;
}
// RunContainer.and(BitmapContainer) (:339-378)
Cont run_and_bitmap(const Cont &r, const Cont &b) {
  int card = run_card(r);
  if (card <= kMaxArray) return make_array(array_filter(run_values(r), b.w, true));
  std::vector<uint64_t> w = b.w, rw = run_words(r);
  for (int i = 0; i < kWords; ++i) w[i] &= rw[i];
  int c = words_card(w);
  return ab_from_words(std::move(w), c);
}
// RunContainer.andNot(BitmapContainer) (:586-622)
Cont run_andnot_bitmap(const Cont &r, const Cont &b) {
  int card = run_card(r);
  if (card <= kMaxArray) return make_array(array_filter(run_values(r), b.w, false));
  std::vector<uint64_t> w = run_words(r);
  for (int i = 0; i < kWords; ++i) w[i] &= ~b.w[i];
  int c = words_card(w);
  return ab_from_words(std::move(w), c);
}
// BitmapContainer.andNot(RunContainer) (:256-274)
Cont bitmap_andnot_run(const Cont &b, const Cont &r) {
  std::vector<uint64_t> w = b.w;
  for (int i = 0; i < r.nruns(); ++i) word_range(w, r.rs(i), r.rs(i) + r.rl(i) + 1, 1);
  int c = words_card(w);
  return ab_from_words(std::move(w), c);
}
// RunContainer.or(BitmapContainer) (:1932-1946): full Run or Bitmap.
Cont run_or_bitmap(const Cont &r, const Cont &b) {
  if (run_is_full(r)) return full_run();
  std::vector<uint64_t> w = b.w;
  for (int i = 0; i < r.nruns(); ++i) word_range(w, r.rs(i), r.rs(i) + r.rl(i) + 1, 0);
  int c = words_card(w);
  if (c == kSpan) return full_run();
  return make_bitmap(std::move(w), c);
}
// RunContainer.xor(BitmapContainer) (:2430-2446)
Cont run_xor_bitmap(const Cont &r, const Cont &b) {
  std::vector<uint64_t> w = b.w;
  for (int i = 0; i < r.nruns(); ++i) word_range(w, r.rs(i), r.rs(i) + r.rl(i) + 1, 2);
  int c = words_card(w);
  return ab_from_words(std::move(w), c);
}
// RunContainer.xor(ArrayContainer) (:2410-2428)
Cont run_xor_array(const Cont &r, const Cont &a) {
  if (a.card < kRunArrayThreshold) return repair(run_lazy_xor_array(r, a));
  int card = run_card(r);
  if (card <= kMaxArray) { // ArrayContainer.or(CharIterator, exclusive=true) (:982-1021)
    std::vector<uint16_t> o = arr_xor(a.v, run_values(r));
    int c = (int)o.size();
    if (c > kMaxArray) return make_bitmap(array_words(o), c);
    return make_array(std::move(o));
  }
  return bitmap_xor_array(run_to_bitmap_or_array(r, card), a);
}
// RunContainer.andNot(ArrayContainer) (:574-584)
Cont run_andnot_array(const Cont &r, const Cont &a) {
  if (a.card < kRunArrayThreshold) return run_eff(run_lazy_andnot_array(r, a));
  int card = run_card(r);
  if (card <= kMaxArray) return make_array(arr_andnot(run_values(r), a.v));
  return bitmap_andnot_array(run_to_bitmap_or_array(r, card), a);
}

// ---------------------------------------------------------------- static container ops
// Container.and dispatch (Container.java:81-88) and the 3x3 implementations.
Cont c_and(const Cont &x, const Cont &y) {
  switch (x.t * 3 + y.t) {
  case kA * 3 + kA: return make_array(arr_and(x.v, y.v));              // ArrayContainer.java:184
  case kA * 3 + kB: return make_array(array_filter(x.v, y.w, true));   // BitmapContainer.java:162
  case kA * 3 + kR: return make_array(array_in_runs(x.v, y, true));   // RunContainer.java:305
  case kB * 3 + kA: return make_array(array_filter(y.v, x.w, true));
  case kB * 3 + kB: {                                                   // BitmapContainer.java:174-188
    std::vector<uint64_t> w(kWords);
    for (int i = 0; i < kWords; ++i) w[i] = x.w[i] & y.w[i];
    int c = words_card(w);
    return ab_from_words(std::move(w), c);
  }
  case kB * 3 + kR: return run_and_bitmap(y, x);
  case kR * 3 + kA: return make_array(array_in_runs(y.v, x, true));
  case kR * 3 + kB: return run_and_bitmap(x, y);
  default: return run_and_run(x, y);
  }
}
Cont c_andnot(const Cont &x, const Cont &y) {
  switch (x.t * 3 + y.t) {
  case kA * 3 + kA: return make_array(arr_andnot(x.v, y.v));             // ArrayContainer.java:222
  case kA * 3 + kB: return make_array(array_filter(x.v, y.w, false));    // ArrayContainer.java:231
  case kA * 3 + kR:                                                       // ArrayContainer.java:243-271
    if (y.nruns() == 0) return x;
    if (run_is_full(y)) return make_array({});
    return make_array(array_in_runs(x.v, y, false));
  case kB * 3 + kA: return bitmap_andnot_array(x, y);                     // BitmapContainer.java:221
  case kB * 3 + kB: {                                                      // BitmapContainer.java:239-256
    std::vector<uint64_t> w(kWords);
    for (int i = 0; i < kWords; ++i) w[i] = x.w[i] & ~y.w[i];
    int c = words_card(w);
    return ab_from_words(std::move(w), c);
  }
  case kB * 3 + kR: return bitmap_andnot_run(x, y);
  case kR * 3 + kA: return run_andnot_array(x, y);
  case kR * 3 + kB: return run_andnot_bitmap(x, y);
  default: return run_andnot_run(x, y);
  }
}
Cont c_or(const Cont &x, const Cont &y) {
  switch (x.t * 3 + y.t) {
  case kA * 3 + kA: {                                                      // ArrayContainer.java:949-973
    if (x.card + y.card > kMaxArray) {
      Cont b = to_bitmap(x);
      for (uint16_t v : y.v) b.w[v >> 6] |= 1ull << (v & 63);
      b.card = -1;
      return bitmap_repair(std::move(b));
    }
    return make_array(arr_or(x.v, y.v));
  }
  case kA * 3 + kB: return bitmap_or_array(y, x);
  case kA * 3 + kR: return repair(run_lazy_or_array(y, x));               // RunContainer.java:1926-1930
  case kB * 3 + kA: return bitmap_or_array(x, y);
  case kB * 3 + kB: {                                                      // BitmapContainer.java:1102 + ior :769-778
    std::vector<uint64_t> w(kWords);
    for (int i = 0; i < kWords; ++i) w[i] = x.w[i] | y.w[i];
    int c = words_card(w);
    if (c == kSpan) return full_run();
    return make_bitmap(std::move(w), c);
  }
  case kB * 3 + kR: return run_or_bitmap(y, x);
  case kR * 3 + kA: return repair(run_lazy_or_array(x, y));
  case kR * 3 + kB: return run_or_bitmap(x, y);
  default: return run_or_run(x, y);
  }
}
Cont c_xor(const Cont &x, const Cont &y) {
  switch (x.t * 3 + y.t) {
  case kA * 3 + kA: {                                                      // ArrayContainer.java:1311-1322
    if (x.card + y.card > kMaxArray) return bitmap_xor_array(to_bitmap(x), y);
    return make_array(arr_xor(x.v, y.v));
  }
  case kA * 3 + kB: return bitmap_xor_array(y, x);
  case kA * 3 + kR: return run_xor_array(y, x);
  case kB * 3 + kA: return bitmap_xor_array(x, y);
  case kB * 3 + kB: {                                                      // BitmapContainer.java:1400-1417
    std::vector<uint64_t> w(kWords);
    for (int i = 0; i < kWords; ++i) w[i] = x.w[i] ^ y.w[i];
    int c = words_card(w);
    return ab_from_words(std::move(w), c);
  }
  case kB * 3 + kR: return run_xor_bitmap(y, x);
  case kR * 3 + kA: return run_xor_array(x, y);
  case kR * 3 + kB: return run_xor_bitmap(x, y);
  default: return run_xor_run(x, y);
  }
}
// In-place variants used by RoaringBitmap.and/xor/andNot(x2).  Their result types equal the
// static ones: ArrayContainer.iand/iandNot (:538-607), BitmapContainer.iand/iandNot/ixor
// non-lazy branches (:532-655, :837-885), RunContainer.iand/iandNot/ixor (:1166-1196, :1691-1705).
Cont c_iand(const Cont &x, const Cont &y) { return c_and(x, y); }
Cont c_iandnot(const Cont &x, const Cont &y) { return c_andnot(x, y); }
Cont c_ixor(const Cont &x, const Cont &y) { return c_xor(x, y); }
// ior (RoaringBitmap.or(x2) in place): differs from or() only for Bitmap.ior(Array), which never
// converts a full result (BitmapContainer.java:749-766), and Run.ior(*) which returns a full `this`.
Cont c_ior(const Cont &x, const Cont &y) {
  if (x.t == kB && y.t == kA) {
    Cont r = x;
    for (uint16_t v : y.v) {
      uint64_t &wd = r.w[v >> 6];
      uint64_t aft = wd | (1ull << (v & 63));
      r.card += (wd != aft);
      wd = aft;
    }
    return r;
  }
  if (x.t == kA && y.t == kA) return c_or(x, y);                         // ArrayContainer.java:726-756
  if (x.t == kR && run_is_full(x)) return x;                              // RunContainer.java:1462,1501,1508
  if (x.t == kR && y.t == kA) {                                           // RunContainer.java:1462-1499
    RunList ans;
    int i = 0, k = 0;
    while (k < y.card && i < x.nruns()) {
      if (x.rs(i) - (int)y.v[k] <= 0) { ans.smart_append(x.rs(i), x.rl(i)); ++i; }
      else ans.smart_append(y.v[k++]);
    }
    if (k < y.card) { while (k < y.card) ans.smart_append(y.v[k++]); }
    else { while (i < x.nruns()) { ans.smart_append(x.rs(i), x.rl(i)); ++i; } }
    return run_eff(ans.cont());
  }
  if (x.t == kR && y.t == kR) {                                           // RunContainer.java:1508-1550
    RunList ans;
    int i = 0, j = 0;
    while (i < x.nruns() && j < y.nruns()) {
      if (x.rs(i) - y.rs(j) <= 0) { ans.smart_append(x.rs(i), x.rl(i)); ++i; }
      else { ans.smart_append(y.rs(j), y.rl(j)); ++j; }
    }
    while (i < x.nruns()) { ans.smart_append(x.rs(i), x.rl(i)); ++i; }
    while (j < y.nruns()) { ans.smart_append(y.rs(j), y.rl(j)); ++j; }
    return run_eff(ans.cont());
  }
  return c_or(x, y);
}
// Container.lazyIOR (Container.java:717-740) — used by ParallelAggregation.or(List) chains.
Cont c_lazy_ior(const Cont &x, const Cont &y) {
  if (x.t == kA) {
    if (y.t == kA) { // ArrayContainer.lazyor (:1449-1464)
      if (x.card + y.card > kArrayLazyLower) {
        Cont b = to_bitmap(x);
        for (uint16_t v : y.v) b.w[v >> 6] |= 1ull << (v & 63);
        b.card = -1;
        return b;
      }
      return make_array(arr_or(x.v, y.v));
    }
    if (y.t == kB) return bitmap_or_array(y, x);  // ior(Bitmap) == x.or(this)
    return run_lazy_or_array(y, x);               // ((RunContainer) x).lazyor(this)
  }
  if (x.t == kR) {
    if (run_is_full(x)) return x; // ilazyor / ior return a full `this`
    if (y.t == kA) { // RunContainer.ilazyor -> ilazyorToRun (:1198-1236)
      Cont r = run_lazy_or_array(x, y);
      return r;
    }
    if (y.t == kB) return run_or_bitmap(x, y);
    return c_ior(x, y);
  }
  // BitmapContainer.ilazyor (:657-685): in place, cardinality invalidated
  Cont b = x;
  b.card = -1;
  if (y.t == kA) {
    for (uint16_t v : y.v) b.w[v >> 6] |= 1ull << (v & 63);
  } else if (y.t == kB) {
    for (int i = 0; i < kWords; ++i) b.w[i] |= y.w[i];
  } else {
    for (int i = 0; i < y.nruns(); ++i) word_range(b.w, y.rs(i), y.rs(i) + y.rl(i) + 1, 0);
  }
  return b;
}

int c_and_card(const Cont &x, const Cont &y) { // Container.andCardinality (Container.java:113-126)
  if (is_empty(x) || is_empty(y)) return 0;
  if (x.t == kB && y.t == kB) {
    int c = 0;
    for (int i = 0; i < kWords; ++i) c += popcnt(x.w[i] & y.w[i]);
    return c;
  }
  return cardinality(c_and(x, y));
}

} // namespace

// ---------------------------------------------------------------- bitmap (RoaringArray) level
struct rbref_bitmap {
  std::vector<uint16_t> keys; // RoaringArray.keys (:34)
  std::vector<Cont> vals;     // RoaringArray.values (:36)
  size_t size() const { return keys.size(); }
};

namespace {
using BM = rbref_bitmap;

// RoaringBitmap.and(x1, x2) (:377-401)
BM *bm_and(const BM &a, const BM &b) {
  BM *out = new BM;
  size_t i = 0, j = 0;
  while (i < a.size() && j < b.size()) {
    if (a.keys[i] == b.keys[j]) {
      Cont c = c_and(a.vals[i], b.vals[j]);
      if (!is_empty(c)) { out->keys.push_back(a.keys[i]); out->vals.push_back(std::move(c)); }
      ++i; ++j;
    } else if (a.keys[i] < b.keys[j]) {
      ++i;
    } else {
      ++j;
    }
  }
  return out;
}
// RoaringBitmap.or(x1, x2) (:860-902) / xor (:1071-1118): unmatched containers are cloned.
BM *bm_or_xor(const BM &a, const BM &b, bool is_xor) {
  BM *out = new BM;
  size_t i = 0, j = 0;
  while (i < a.size() && j < b.size()) {
    if (a.keys[i] == b.keys[j]) {
      Cont c = is_xor ? c_xor(a.vals[i], b.vals[j]) : c_or(a.vals[i], b.vals[j]);
      if (!is_xor || !is_empty(c)) { out->keys.push_back(a.keys[i]); out->vals.push_back(std::move(c)); }
      ++i; ++j;
    } else if (a.keys[i] < b.keys[j]) {
      out->keys.push_back(a.keys[i]); out->vals.push_back(a.vals[i]); ++i;
    } else {
      out->keys.push_back(b.keys[j]); out->vals.push_back(b.vals[j]); ++j;
    }
  }
  for (; i < a.size(); ++i) { out->keys.push_back(a.keys[i]); out->vals.push_back(a.vals[i]); }
  for (; j < b.size(); ++j) { out->keys.push_back(b.keys[j]); out->vals.push_back(b.vals[j]); }
  return out;
}
// Roaring64Bitmap.xor (longlong/Roaring64Bitmap.java:421-460 static, :392-419 in place) stores each
// matched key's xor result without an isEmpty check: an empty container stays under its key.
BM *bm_xor_keep_empty(const BM &a, const BM &b) {
  BM *out = new BM;
  size_t i = 0, j = 0;
  while (i < a.size() && j < b.size()) {
    if (a.keys[i] == b.keys[j]) {
      out->keys.push_back(a.keys[i]); out->vals.push_back(c_xor(a.vals[i], b.vals[j])); ++i; ++j;
    } else if (a.keys[i] < b.keys[j]) {
      out->keys.push_back(a.keys[i]); out->vals.push_back(a.vals[i]); ++i;
    } else {
      out->keys.push_back(b.keys[j]); out->vals.push_back(b.vals[j]); ++j;
    }
  }
  for (; i < a.size(); ++i) { out->keys.push_back(a.keys[i]); out->vals.push_back(a.vals[i]); }
  for (; j < b.size(); ++j) { out->keys.push_back(b.keys[j]); out->vals.push_back(b.vals[j]); }
  return out;
}
// RoaringBitmap.andNot(x1, x2) (:444-473)
BM *bm_andnot(const BM &a, const BM &b) {
  BM *out = new BM;
  size_t i = 0, j = 0;
  while (i < a.size() && j < b.size()) {
    if (a.keys[i] == b.keys[j]) {
      Cont c = c_andnot(a.vals[i], b.vals[j]);
      if (!is_empty(c)) { out->keys.push_back(a.keys[i]); out->vals.push_back(std::move(c)); }
      ++i; ++j;
    } else if (a.keys[i] < b.keys[j]) {
      out->keys.push_back(a.keys[i]); out->vals.push_back(a.vals[i]); ++i;
    } else {
      ++j;
    }
  }
  for (; i < a.size(); ++i) { out->keys.push_back(a.keys[i]); out->vals.push_back(a.vals[i]); }
  return out;
}
BM *bm_op(int op, const BM &a, const BM &b) {
  switch (op) {
  case RBREF_AND: return bm_and(a, b);
  case RBREF_OR: return bm_or_xor(a, b, false);
  case RBREF_XOR: return bm_or_xor(a, b, true);
  default: return bm_andnot(a, b);
  }
}
uint64_t bm_card(const BM &b) {
  uint64_t s = 0;
  for (const Cont &c : b.vals) s += (uint64_t)cardinality(c);
  return s;
}
// RoaringBitmap.andCardinality (:413-434)
int64_t bm_and_card(const BM &a, const BM &b) {
  int64_t s = 0;
  size_t i = 0, j = 0;
  while (i < a.size() && j < b.size()) {
    if (a.keys[i] == b.keys[j]) { s += c_and_card(a.vals[i], b.vals[j]); ++i; ++j; }
    else if (a.keys[i] < b.keys[j]) ++i;
    else ++j;
  }
  return s;
}

// In-place RoaringBitmap ops — and (:1272-1296), andNot (:1346-1382), or (:2481-2523), xor (:3296-3348).
void bm_iand(BM &a, const BM &b) {
  if (&a == &b) return;
  BM out;
  size_t i = 0, j = 0;
  while (i < a.size() && j < b.size()) {
    if (a.keys[i] == b.keys[j]) {
      Cont c = c_iand(a.vals[i], b.vals[j]);
      if (!is_empty(c)) { out.keys.push_back(a.keys[i]); out.vals.push_back(std::move(c)); }
      ++i; ++j;
    } else if (a.keys[i] < b.keys[j]) ++i;
    else ++j;
  }
  a = std::move(out);
}
void bm_iandnot(BM &a, const BM &b) {
  if (&a == &b) { a = BM(); return; }
  BM out;
  size_t i = 0, j = 0;
  while (i < a.size() && j < b.size()) {
    if (a.keys[i] == b.keys[j]) {
      Cont c = c_iandnot(a.vals[i], b.vals[j]);
      if (!is_empty(c)) { out.keys.push_back(a.keys[i]); out.vals.push_back(std::move(c)); }
      ++i; ++j;
    } else if (a.keys[i] < b.keys[j]) {
      out.keys.push_back(a.keys[i]); out.vals.push_back(std::move(a.vals[i])); ++i;
    } else ++j;
  }
  for (; i < a.size(); ++i) { out.keys.push_back(a.keys[i]); out.vals.push_back(std::move(a.vals[i])); }
  a = std::move(out);
}
void bm_ior_ixor(BM &a, const BM &b, bool is_xor) {
  if (&a == &b) { if (is_xor) a = BM(); return; }
  BM out;
  size_t i = 0, j = 0;
  while (i < a.size() && j < b.size()) {
    if (a.keys[i] == b.keys[j]) {
      Cont c = is_xor ? c_ixor(a.vals[i], b.vals[j]) : c_ior(a.vals[i], b.vals[j]);
      if (!is_xor || !is_empty(c)) { out.keys.push_back(a.keys[i]); out.vals.push_back(std::move(c)); }
      ++i; ++j;
    } else if (a.keys[i] < b.keys[j]) {
      out.keys.push_back(a.keys[i]); out.vals.push_back(std::move(a.vals[i])); ++i;
    } else {
      out.keys.push_back(b.keys[j]); out.vals.push_back(b.vals[j]); ++j;
    }
  }
  for (; i < a.size(); ++i) { out.keys.push_back(a.keys[i]); out.vals.push_back(std::move(a.vals[i])); }
  for (; j < b.size(); ++j) { out.keys.push_back(b.keys[j]); out.vals.push_back(b.vals[j]); }
  a = std::move(out);
}

// Accumulator indexed by key, for the wide aggregations (keeps the reference's key order
// because iteration is by ascending key).
struct KeyTable {
  std::vector<int> slot = std::vector<int>(kSpan, -1);
  std::vector<uint16_t> keys;
  std::vector<Cont> vals;
  bool has(int k) const { return slot[k] >= 0; }
  Cont &at(int k) { return vals[slot[k]]; }
  void put(int k, Cont c) {
    slot[k] = (int)vals.size();
    keys.push_back((uint16_t)k);
    vals.push_back(std::move(c));
  }
  BM *finish(bool drop_empty) {
    std::vector<uint16_t> ks = keys;
    std::sort(ks.begin(), ks.end());
    BM *out = new BM;
    for (uint16_t k : ks) {
      Cont &c = vals[slot[k]];
      if (drop_empty && is_empty(c)) continue;
      out->keys.push_back(k);
      out->vals.push_back(std::move(c));
    }
    return out;
  }
};

// FastAggregation.naive_or (:541-548) = naivelazyor (RoaringBitmap.java:2405-2448) + repairAfterLazy.
BM *wide_naive_or(const BM *const *bs, size_t n) {
  KeyTable t;
  for (size_t m = 0; m < n; ++m) {
    const BM &b = *bs[m];
    for (size_t i = 0; i < b.size(); ++i) {
      int k = b.keys[i];
      if (!t.has(k)) {
        t.put(k, b.vals[i]); // clone
      } else {
        Cont acc = to_bitmap(t.at(k));
        t.at(k) = c_lazy_ior(acc, b.vals[i]); // BitmapContainer.lazyIOR -> ilazyor
      }
    }
  }
  for (Cont &c : t.vals) c = repair(std::move(c));
  return t.finish(false);
}
// FastAggregation.workShyAnd (:356-396): intersect keys, lazy AND per key, repair, drop empty.
BM *wide_workshy_and(const BM *const *bs, size_t n) {
  BM *out = new BM;
  if (n == 0) return out;
  std::vector<int> cnt(kSpan, 0);
  for (size_t m = 0; m < n; ++m)
    for (uint16_t k : bs[m]->keys) cnt[k]++;
  std::vector<const Cont *> slice(n);
  for (int k = 0; k < kSpan; ++k) {
    if (cnt[k] != (int)n) continue; // Util.intersectKeys (Util.java:1244-1259)
    std::vector<uint64_t> w(kWords, ~0ull);
    for (size_t m = 0; m < n; ++m) {
      const BM &b = *bs[m];
      size_t idx = std::lower_bound(b.keys.begin(), b.keys.end(), (uint16_t)k) - b.keys.begin();
      const Cont &c = b.vals[idx];
      if (c.t == kA) { // BitmapContainer.iand(ArrayContainer) lazy: Util.intersectArrayIntoBitmap
        std::vector<uint64_t> aw = array_words(c.v);
        for (int i = 0; i < kWords; ++i) w[i] &= aw[i];
      } else if (c.t == kB) {
        for (int i = 0; i < kWords; ++i) w[i] &= c.w[i];
      } else { // BitmapContainer.iand(RunContainer) lazy branch (:566-590)
        std::vector<uint64_t> rw = run_words(c);
        for (int i = 0; i < kWords; ++i) w[i] &= rw[i];
      }
    }
    Cont r = bitmap_repair(make_bitmap(std::move(w), -1));
    if (!is_empty(r)) { out->keys.push_back((uint16_t)k); out->vals.push_back(std::move(r)); }
  }
  return out;
}
// FastAggregation.naive_and(RoaringBitmap...) (:328-346): clone the smallest (first on ties),
// then in-place and with every other bitmap (object identity) until empty.
BM *wide_naive_and(const BM *const *bs, size_t n) {
  if (n == 0) return new BM;
  const BM *smallest = bs[0];
  for (size_t i = 1; i < n; ++i)
    if (bs[i]->size() < smallest->size()) smallest = bs[i];
  BM *ans = new BM(*smallest);
  for (size_t k = 0; k < n && ans->size() > 0; ++k)
    if (bs[k] != smallest) bm_iand(*ans, *bs[k]);
  return ans;
}
// FastAggregation.naive_and(Iterator) (:304-313)
BM *wide_naive_and_iter(const BM *const *bs, size_t n) {
  if (n == 0) return new BM;
  BM *ans = new BM(*bs[0]);
  for (size_t k = 1; k < n && ans->size() > 0; ++k) bm_iand(*ans, *bs[k]);
  return ans;
}
// FastAggregation.naive_xor (:576-582)
BM *wide_naive_xor(const BM *const *bs, size_t n) {
  BM *ans = new BM;
  for (size_t k = 0; k < n; ++k) bm_ior_ixor(*ans, *bs[k], true);
  return ans;
}
// ParallelAggregation.groupByKey (:137-153): per key, containers in input order.
std::map<int, std::vector<const Cont *>> group_by_key(const BM *const *bs, size_t n) {
  std::map<int, std::vector<const Cont *>> g;
  for (size_t m = 0; m < n; ++m)
    for (size_t i = 0; i < bs[m]->size(); ++i) g[bs[m]->keys[i]].push_back(&bs[m]->vals[i]);
  return g;
}
// ParallelAggregation.or(List<Container>) (:197-223).  The >= 512 split with parallelism > 1
// (OrCollector) ends in the same lazy Bitmap + repair as the >= 16 branch.
Cont par_or_list(const std::vector<const Cont *> &cs) {
  if (cs.size() < 16) {
    Cont r = *cs[0];
    for (size_t i = 1; i < cs.size(); ++i) r = c_lazy_ior(r, *cs[i]);
    return repair(std::move(r));
  }
  Cont r = make_bitmap(std::vector<uint64_t>(kWords, 0), -1);
  for (const Cont *c : cs) r = c_lazy_ior(r, *c);
  return repair(std::move(r));
}
// ParallelAggregation.xor(List<Container>) (:189-195): clone + ixor fold, no intermediate removal.
Cont par_xor_list(const std::vector<const Cont *> &cs) {
  Cont r = *cs[0];
  for (size_t i = 1; i < cs.size(); ++i) r = c_ixor(r, *cs[i]);
  return r;
}
BM *wide_par(const BM *const *bs, size_t n, bool is_xor) {
  BM *out = new BM;
  for (auto &kv : group_by_key(bs, n)) {
    Cont c = is_xor ? par_xor_list(kv.second) : par_or_list(kv.second);
    if (is_xor && is_empty(c)) continue; // ContainerCollector.accumulator (:73-79)
    out->keys.push_back((uint16_t)kv.first);
    out->vals.push_back(std::move(c));
  }
  return out;
}

// ---- java.util.PriorityQueue (the OpenJDK binary heap the reference's horizontal_* / priorityqueue_*
// rely on, ties included): offer = append + siftUp, poll = root out, last element sifted down from
// the root; cmp(a, b) is compareTo / Comparator.compare (< 0, 0, > 0).
template <class T, class Cmp> struct JavaPQ {
  std::vector<T> q;
  Cmp cmp;
  explicit JavaPQ(Cmp c) : cmp(c) {}
  bool empty() const { return q.empty(); }
  size_t size() const { return q.size(); }
  const T &peek() const { return q[0]; }
  void offer(const T &x) { // PriorityQueue.siftUpComparable / siftUpUsingComparator
    size_t k = q.size();
    q.push_back(x);
    while (k > 0) {
      const size_t parent = (k - 1) >> 1;
      if (cmp(x, q[parent]) >= 0) break;
      q[k] = q[parent];
      k = parent;
    }
    q[k] = x;
  }
  T poll() { // PriorityQueue.poll + siftDownComparable / siftDownUsingComparator
    T result = q[0];
    T x = q.back();
    q.pop_back();
    const size_t n = q.size();
    if (n > 0) {
      size_t k = 0;
      const size_t half = n >> 1;
      while (k < half) {
        size_t child = 2 * k + 1;
        const size_t right = child + 1;
        if (right < n && cmp(q[child], q[right]) > 0) child = right;
        if (cmp(x, q[child]) <= 0) break;
        q[k] = q[child];
        k = child;
      }
      q[k] = x;
    }
    return result;
  }
};

// Container.lazyOR (Container.java:751-774): the non-in-place dispatch — Array with Bitmap and Run
// with Bitmap go to BitmapContainer.lazyor (a lazy Bitmap), Run with Run to RunContainer.or.
Cont c_lazy_or(const Cont &x, const Cont &y) {
  auto lazy_bitmap = [](const Cont &b, const Cont &o) { // BitmapContainer.lazyor (:887-918): clone, OR, card -1
    Cont r = b;
    r.card = -1;
    if (o.t == kA) {
      for (uint16_t v : o.v) r.w[v >> 6] |= 1ull << (v & 63);
    } else if (o.t == kB) {
      for (int i = 0; i < kWords; ++i) r.w[i] |= o.w[i];
    } else {
      for (int i = 0; i < o.nruns(); ++i) word_range(r.w, o.rs(i), o.rs(i) + o.rl(i) + 1, 0);
    }
    return r;
  };
  if (x.t == kA) {
    if (y.t == kA) return c_lazy_ior(x, y);   // ArrayContainer.lazyor (:1449-1464)
    if (y.t == kB) return lazy_bitmap(y, x);  // ((BitmapContainer) x).lazyor(this)
    return run_lazy_or_array(y, x);           // ((RunContainer) x).lazyor(this) -> lazyorToRun
  }
  if (x.t == kR) {
    if (y.t == kA) return run_lazy_or_array(x, y);
    if (y.t == kB) return lazy_bitmap(y, x);
    return run_or_run(x, y);
  }
  return lazy_bitmap(x, y);
}

// FastAggregation.horizontal_or / horizontal_xor (FastAggregation.java:124-289): a priority queue of
// ContainerPointers (RoaringArray.getContainerPointer, RoaringArray.java:688-746: ordered by key, then
// by cardinality descending); per key the first two polled containers are combined (lazyOR / xor), the
// rest of the key's pointers in poll order folded in place (lazyIOR / ixor); the OR is repaired, the
// XOR is appended as is (an empty result included).
struct CPtr {
  const BM *b;
  size_t k;
  bool valid() const { return k < b->size(); }
  int key() const { return b->keys[k]; }
  int card() const { return cardinality(b->vals[k]); }
  const Cont &c() const { return b->vals[k]; }
};
BM *wide_horizontal(const BM *const *bs, size_t n, bool is_xor) {
  BM *ans = new BM;
  if (n == 0) return ans;
  auto cmp = [](const CPtr &x, const CPtr &y) { return x.key() != y.key() ? x.key() - y.key() : y.card() - x.card(); };
  JavaPQ<CPtr, decltype(cmp)> pq(cmp);
  for (size_t k = 0; k < n; ++k) {
    CPtr x{bs[k], 0};
    if (x.valid()) pq.offer(x);
  }
  while (!pq.empty()) {
    CPtr x1 = pq.poll();
    if (pq.empty() || pq.peek().key() != x1.key()) {
      ans->keys.push_back((uint16_t)x1.key());
      ans->vals.push_back(x1.c());
      ++x1.k;
      if (x1.valid()) pq.offer(x1);
      continue;
    }
    CPtr x2 = pq.poll();
    Cont newc = is_xor ? c_xor(x1.c(), x2.c()) : c_lazy_or(x1.c(), x2.c());
    while (!pq.empty() && pq.peek().key() == x1.key()) {
      CPtr x = pq.poll();
      newc = is_xor ? c_ixor(newc, x.c()) : c_lazy_ior(newc, x.c());
      ++x.k;
      if (x.valid()) pq.offer(x);
      else if (pq.empty()) break;
    }
    if (!is_xor) newc = repair(std::move(newc));
    ans->keys.push_back((uint16_t)x1.key());
    ans->vals.push_back(std::move(newc));
    ++x1.k;
    if (x1.valid()) pq.offer(x1);
    ++x2.k;
    if (x2.valid()) pq.offer(x2);
  }
  return ans;
}

// RoaringBitmap.getLongSizeInBytes (RoaringBitmap.java:2212-2219) with the containers' getSizeInBytes:
// Array 2c + 4 (ArrayContainer.java:450), Bitmap 8192 (BitmapContainer.java:507), Run 4r + 4
// (RunContainer.java:1043) — a lazy Bitmap counts 8192 too.
int64_t bm_size_in_bytes(const BM &b) {
  int64_t s = 8;
  for (const Cont &c : b.vals) s += 2 + (c.t == kA ? 2 * (int64_t)c.card + 4 : c.t == kB ? 8192 : 4 * (int64_t)c.nruns() + 4);
  return s;
}
// RoaringBitmap.lazyor(x1, x2) static (RoaringBitmap.java:724-767): matched keys lazyOR, others cloned
BM bm_lazyor_static(const BM &a, const BM &b) {
  BM out;
  size_t i = 0, j = 0;
  while (i < a.size() && j < b.size()) {
    if (a.keys[i] == b.keys[j]) {
      out.keys.push_back(a.keys[i]);
      out.vals.push_back(c_lazy_or(a.vals[i], b.vals[j]));
      ++i;
      ++j;
    } else if (a.keys[i] < b.keys[j]) {
      out.keys.push_back(a.keys[i]);
      out.vals.push_back(a.vals[i++]);
    } else {
      out.keys.push_back(b.keys[j]);
      out.vals.push_back(b.vals[j++]);
    }
  }
  for (; i < a.size(); ++i) { out.keys.push_back(a.keys[i]); out.vals.push_back(a.vals[i]); }
  for (; j < b.size(); ++j) { out.keys.push_back(b.keys[j]); out.vals.push_back(b.vals[j]); }
  return out;
}
// this.lazyor(x2) in place (RoaringBitmap.java:2357-2402): matched keys lazyIOR, x2's other keys cloned
// in; lazyorfromlazyinputs(x1, x2) (:769-830): matched keys lazyIOR with a Bitmap (lazy or not) put
// first, the others taken over.  On value-semantics containers both are the same merge apart from
// that swap.
BM bm_lazyor_inplace(const BM &a, const BM &b, bool bitmap_first) {
  BM out;
  size_t i = 0, j = 0;
  while (i < a.size() && j < b.size()) {
    if (a.keys[i] == b.keys[j]) {
      const Cont *c1 = &a.vals[i], *c2 = &b.vals[j];
      if (bitmap_first && c2->t == kB && c1->t != kB) std::swap(c1, c2);
      out.keys.push_back(a.keys[i]);
      out.vals.push_back(c_lazy_ior(*c1, *c2));
      ++i;
      ++j;
    } else if (a.keys[i] < b.keys[j]) {
      out.keys.push_back(a.keys[i]);
      out.vals.push_back(a.vals[i++]);
    } else {
      out.keys.push_back(b.keys[j]);
      out.vals.push_back(b.vals[j++]);
    }
  }
  for (; i < a.size(); ++i) { out.keys.push_back(a.keys[i]); out.vals.push_back(a.vals[i]); }
  for (; j < b.size(); ++j) { out.keys.push_back(b.keys[j]); out.vals.push_back(b.vals[j]); }
  return out;
}
// FastAggregation.priorityqueue_or(RoaringBitmap...) (FastAggregation.java:675-721): the bitmaps by
// size in a priority queue of indices; the two smallest are lazily OR'd (which side is reused
// depends on which operands are temporaries), the result re-queued with its new size; the survivor
// is repaired.
BM *wide_pq_or(const BM *const *bs, size_t n) {
  if (n == 0) return new BM;
  std::vector<BM> buffer(n);
  for (size_t k = 0; k < n; ++k) buffer[k] = *bs[k];
  std::vector<int64_t> sizes(n);
  std::vector<char> istmp(n, 0);
  for (size_t k = 0; k < n; ++k) sizes[k] = bm_size_in_bytes(buffer[k]);
  auto cmp = [&](int a, int b) { return (int)(sizes[a] - sizes[b]); };
  JavaPQ<int, decltype(cmp)> pq(cmp);
  for (size_t k = 0; k < n; ++k) pq.offer((int)k);
  while (pq.size() > 1) {
    const int x1 = pq.poll(), x2 = pq.poll();
    if (istmp[x2] && istmp[x1]) {
      buffer[x1] = bm_lazyor_inplace(buffer[x1], buffer[x2], true);
      sizes[x1] = bm_size_in_bytes(buffer[x1]);
      istmp[x1] = 1;
      pq.offer(x1);
    } else if (istmp[x2]) {
      buffer[x2] = bm_lazyor_inplace(buffer[x2], buffer[x1], false);
      sizes[x2] = bm_size_in_bytes(buffer[x2]);
      pq.offer(x2);
    } else if (istmp[x1]) {
      buffer[x1] = bm_lazyor_inplace(buffer[x1], buffer[x2], false);
      sizes[x1] = bm_size_in_bytes(buffer[x1]);
      pq.offer(x1);
    } else {
      buffer[x1] = bm_lazyor_static(buffer[x1], buffer[x2]);
      sizes[x1] = bm_size_in_bytes(buffer[x1]);
      istmp[x1] = 1;
      pq.offer(x1);
    }
  }
  BM *ans = new BM(std::move(buffer[pq.poll()]));
  for (Cont &c : ans->vals) c = repair(std::move(c)); // RoaringBitmap.repairAfterLazy (:2752-2757)
  return ans;
}
// FastAggregation.priorityqueue_xor (FastAggregation.java:732-752): the two smallest bitmaps (by
// getLongSizeInBytes) replaced by their RoaringBitmap.xor until one is left
BM *wide_pq_xor(const BM *const *bs, size_t n) {
  if (n == 0) return new BM;
  std::vector<BM> pool;
  pool.reserve(2 * n);
  for (size_t k = 0; k < n; ++k) pool.push_back(*bs[k]);
  auto cmp = [&](int a, int b) { return (int)(bm_size_in_bytes(pool[a]) - bm_size_in_bytes(pool[b])); };
  JavaPQ<int, decltype(cmp)> pq(cmp);
  for (size_t k = 0; k < n; ++k) pq.offer((int)k); // Collections.addAll: add() in array order
  while (pq.size() > 1) {
    const int x1 = pq.poll(), x2 = pq.poll();
    std::unique_ptr<BM> r(bm_or_xor(pool[x1], pool[x2], true));
    pool.push_back(std::move(*r));
    pq.offer((int)pool.size() - 1);
  }
  return new BM(pool[pq.poll()]);
}

// ---- buffer/ (BufferFastAggregation over Immutable/MutableRoaringBitmap): the same container
// algebra (the Mappeable* containers restate the Container rules), three entry points that differ.
// ImmutableRoaringBitmap.getLongSizeInBytes (buffer/ImmutableRoaringBitmap.java:1508-1521) with
// BufferUtil.getSizeInBytesFromCardinalityEtc (buffer/BufferUtil.java:512-524): 4, then per container
// 4 + (Run: 2 + 4r; else getCardinality() > 4096 ? 8192 : 2 * getCardinality()).  A lazy Bitmap's
// getCardinality() is -1 (MappeableBitmapContainer.java:540-542), so it counts 4 - 2 bytes.
int64_t bm_size_immutable(const BM &b) {
  int64_t s = 4;
  for (const Cont &c : b.vals) {
    const int64_t card = c.t == kB && c.card < 0 ? -1 : (int64_t)cardinality(c);
    s += 4 + (c.t == kR ? 2 + 4 * (int64_t)c.nruns() : card > kMaxArray ? 8192 : 2 * card);
  }
  return s;
}
// ImmutableRoaringBitmap.serializedSizeInBytes = MutableRoaringArray.serializedSizeInBytes
// (buffer/MutableRoaringArray.java:756-764): headerSize + getArraySizeInBytes per container (a Bitmap
// 8192 whether lazy or not, MappeableBitmapContainer.java:533-535).
int64_t bm_serialized_size_lazy(const BM &b) {
  const uint64_t n = b.size();
  bool hr = false;
  int64_t s = 0;
  for (const Cont &c : b.vals) {
    hr |= c.t == kR;
    s += c.t == kA ? 2 * (int64_t)c.card : c.t == kB ? 8192 : 2 + 4 * (int64_t)c.nruns();
  }
  return s + (int64_t)(hr ? (n < 4 ? 4 + (n + 7) / 8 + 4 * n : 4 + (n + 7) / 8 + 8 * n) : 8 + 8 * n);
}
// BufferFastAggregation.naive_or(MutableRoaringBitmap...) / or(MutableRoaringBitmap...)
// (buffer/BufferFastAggregation.java:711-717, 797-799): an empty answer, answer.lazyor(b) per bitmap
// (MutableRoaringBitmap.lazyor, buffer/MutableRoaringBitmap.java:1309-1352: matched keys lazyIOR, new
// keys cloned in), then repairAfterLazy.  Per key: a clone of the first container, the lazyIOR chain
// over the rest — ParallelAggregation.or's short chain without its 16-container switch.
BM *wide_buffer_naive_or(const BM *const *bs, size_t n) {
  BM acc;
  for (size_t k = 0; k < n; ++k) acc = bm_lazyor_inplace(acc, *bs[k], false);
  BM *out = new BM(std::move(acc));
  for (Cont &c : out->vals) c = repair(std::move(c));
  return out;
}
// BufferFastAggregation.priorityqueue_or (buffer/BufferFastAggregation.java:810-866 varargs,
// :869-930 Iterator): FastAggregation.priorityqueue_or's lazy merges ordered by another size — the
// varargs form by serializedSizeInBytes (an int), the Iterator form by ImmutableRoaringBitmap.
// getLongSizeInBytes — and a single bitmap comes back as a copy (toMutableRoaringBitmap, no repair).
template <class Size> BM *wide_pq_or_sized(const BM *const *bs, size_t n, Size size, bool single_copy) {
  if (n == 0) return new BM;
  if (n == 1 && single_copy) return new BM(*bs[0]);
  std::vector<BM> buffer(n);
  for (size_t k = 0; k < n; ++k) buffer[k] = *bs[k];
  std::vector<int64_t> sizes(n);
  std::vector<char> istmp(n, 0);
  for (size_t k = 0; k < n; ++k) sizes[k] = size(buffer[k]);
  auto cmp = [&](int a, int b) { return (int)(sizes[a] - sizes[b]); };
  JavaPQ<int, decltype(cmp)> pq(cmp);
  for (size_t k = 0; k < n; ++k) pq.offer((int)k);
  while (pq.size() > 1) {
    const int x1 = pq.poll(), x2 = pq.poll();
    if (istmp[x1] && istmp[x2]) {        // MutableRoaringBitmap.lazyorfromlazyinputs (:522-570)
      buffer[x1] = bm_lazyor_inplace(buffer[x1], buffer[x2], true);
      sizes[x1] = size(buffer[x1]);
      pq.offer(x1);
    } else if (istmp[x2]) {              // ((MutableRoaringBitmap) x2).lazyor(x1)
      buffer[x2] = bm_lazyor_inplace(buffer[x2], buffer[x1], false);
      sizes[x2] = size(buffer[x2]);
      pq.offer(x2);
    } else if (istmp[x1]) {
      buffer[x1] = bm_lazyor_inplace(buffer[x1], buffer[x2], false);
      sizes[x1] = size(buffer[x1]);
      pq.offer(x1);
    } else {                             // ImmutableRoaringBitmap.lazyor (static)
      buffer[x1] = bm_lazyor_static(buffer[x1], buffer[x2]);
      sizes[x1] = size(buffer[x1]);
      istmp[x1] = 1;
      pq.offer(x1);
    }
  }
  BM *ans = new BM(std::move(buffer[pq.poll()]));
  for (Cont &c : ans->vals) c = repair(std::move(c)); // MutableRoaringBitmap.repairAfterLazy
  return ans;
}
// BufferFastAggregation.priorityqueue_xor (buffer/BufferFastAggregation.java:933-958): fewer than 2
// bitmaps throw IllegalArgumentException (nullptr here); the queue orders by ImmutableRoaringBitmap.
// getLongSizeInBytes.
BM *wide_buffer_pq_xor(const BM *const *bs, size_t n) {
  if (n < 2) return nullptr;
  std::vector<BM> pool;
  pool.reserve(2 * n);
  for (size_t k = 0; k < n; ++k) pool.push_back(*bs[k]);
  auto cmp = [&](int a, int b) { return (int)(bm_size_immutable(pool[a]) - bm_size_immutable(pool[b])); };
  JavaPQ<int, decltype(cmp)> pq(cmp);
  for (size_t k = 0; k < n; ++k) pq.offer((int)k); // Collections.addAll
  while (pq.size() > 1) {
    const int x1 = pq.poll(), x2 = pq.poll();
    std::unique_ptr<BM> r(bm_or_xor(pool[x1], pool[x2], true));
    pool.push_back(std::move(*r));
    pq.offer((int)pool.size() - 1);
  }
  return new BM(pool[pq.poll()]);
}

// ---- key-parallel restatements (the CPU baseline on all host cores).  Every wide semantics is
// per-key independent with the key's containers in member order, so each key's result is the
// single-threaded one; ParallelAggregation itself is key-parallel on the ForkJoin pool
// (ParallelAggregation.java:161-195, `IntStream.range(0, n).parallel()`).  Per key:
//   FAST_OR      naivelazyor chain + repairAfterLazy (wide_naive_or)
//   WORKSHY_AND  keys held by every member: lazy AND + repair, empty dropped (wide_workshy_and)
//   FAST_XOR     in-place xor chain: absent -> clone, empty -> removed (wide_naive_xor)
//   PAR_OR/XOR   par_or_list / par_xor_list (wide_par)
bool key_result(int sem, const std::vector<const Cont *> &cs, size_t n, Cont &out) {
  if (cs.empty()) return false;
  switch (sem) {
  case RBREF_FAST_OR: {
    Cont acc = *cs[0];
    for (size_t i = 1; i < cs.size(); ++i) acc = c_lazy_ior(to_bitmap(acc), *cs[i]);
    out = repair(std::move(acc));
    return true;
  }
  case RBREF_WORKSHY_AND: {
    if (cs.size() != n) return false;
    std::vector<uint64_t> w(kWords, ~0ull);
    for (const Cont *c : cs) {
      if (c->t == kA) {
        std::vector<uint64_t> aw = array_words(c->v);
        for (int i = 0; i < kWords; ++i) w[i] &= aw[i];
      } else if (c->t == kB) {
        for (int i = 0; i < kWords; ++i) w[i] &= c->w[i];
      } else {
        std::vector<uint64_t> rw = run_words(*c);
        for (int i = 0; i < kWords; ++i) w[i] &= rw[i];
      }
    }
    out = bitmap_repair(make_bitmap(std::move(w), -1));
    return !is_empty(out);
  }
  case RBREF_FAST_XOR: {
    bool present = false;
    Cont acc;
    for (const Cont *c : cs) {
      if (!present) {
        acc = *c;
        present = true;
      } else {
        acc = c_ixor(acc, *c);
        if (is_empty(acc)) present = false;
      }
    }
    if (present) out = std::move(acc);
    return present;
  }
  case RBREF_PAR_OR: out = par_or_list(cs); return true;
  case RBREF_PAR_XOR: out = par_xor_list(cs); return !is_empty(out);
  default: return false;
  }
}
BM *wide_key_parallel(int sem, const BM *const *bs, size_t n, int threads) {
  std::vector<std::vector<const Cont *>> g(kSpan); // ParallelAggregation.groupByKey (:137-153)
  for (size_t m = 0; m < n; ++m)
    for (size_t i = 0; i < bs[m]->size(); ++i) g[bs[m]->keys[i]].push_back(&bs[m]->vals[i]);
  std::vector<Cont> res(kSpan);
  std::vector<char> has(kSpan, 0);
  std::atomic<int> next{0};
  auto work = [&]() {
    for (int k0; (k0 = next.fetch_add(64)) < kSpan;)
      for (int k = k0; k < k0 + 64; ++k) has[k] = key_result(sem, g[k], n, res[k]);
  };
  if (threads <= 1) {
    work();
  } else {
    std::vector<std::thread> th;
    for (int t = 0; t < threads; ++t) th.emplace_back(work);
    for (auto &x : th) x.join();
  }
  BM *out = new BM;
  for (int k = 0; k < kSpan; ++k)
    if (has[k]) {
      out->keys.push_back((uint16_t)k);
      out->vals.push_back(std::move(res[k]));
    }
  return out;
}

// ---------------------------------------------------------------- serialization helpers
struct Reader {
  const uint8_t *p;
  size_t n, pos = 0;
  bool ok = true;
  bool need(size_t k) {
    if (pos + k > n) ok = false;
    return ok;
  }
  uint32_t u32() {
    if (!need(4)) return 0;
    uint32_t v;
    std::memcpy(&v, p + pos, 4);
    pos += 4;
    return v;
  }
  uint16_t u16() {
    if (!need(2)) return 0;
    uint16_t v;
    std::memcpy(&v, p + pos, 2);
    pos += 2;
    return v;
  }
};
constexpr uint32_t kCookie = 12347, kCookieNoRun = 12346; // RoaringArray.java:25-26
constexpr int kNoOffsetThreshold = 4;
} // namespace

// ============================================================== C ABI
extern "C" {

rbref_bitmap *rbref_new(void) { return new rbref_bitmap; }
void rbref_free(rbref_bitmap *b) { delete b; }
rbref_bitmap *rbref_clone(const rbref_bitmap *b) { return new rbref_bitmap(*b); }

rbref_bitmap *rbref_bitmap_of(const uint32_t *vals, size_t n) {
  // RoaringBitmap.bitmapOf -> addN (RoaringBitmap.java:498-560): per key an ArrayContainer that
  // turns into a BitmapContainer on the 4097th distinct value (ArrayContainer.add :139-170).
  std::map<int, std::vector<uint16_t>> g;
  for (size_t i = 0; i < n; ++i) g[vals[i] >> 16].push_back((uint16_t)(vals[i] & 0xFFFF));
  rbref_bitmap *b = new rbref_bitmap;
  for (auto &kv : g) {
    std::vector<uint16_t> &v = kv.second;
    std::sort(v.begin(), v.end());
    v.erase(std::unique(v.begin(), v.end()), v.end());
    b->keys.push_back((uint16_t)kv.first);
    if ((int)v.size() > kMaxArray) b->vals.push_back(make_bitmap(array_words(v), (int)v.size()));
    else b->vals.push_back(make_array(std::move(v)));
  }
  return b;
}

int rbref_run_optimize(rbref_bitmap *b) {
  int any = 0;
  for (Cont &c : b->vals) {
    c = run_optimize(std::move(c));
    any |= (c.t == kR);
  }
  return any;
}

uint64_t rbref_cardinality(const rbref_bitmap *b) { return bm_card(*b); }
uint32_t rbref_container_count(const rbref_bitmap *b) { return (uint32_t)b->size(); }
int rbref_container_info(const rbref_bitmap *b, uint32_t i, uint16_t *key, uint8_t *type,
                         uint32_t *card, uint32_t *nruns) {
  if (i >= b->size()) return RBREF_EINVAL;
  const Cont &c = b->vals[i];
  if (key) *key = b->keys[i];
  if (type) *type = c.t;
  if (card) *card = (uint32_t)cardinality(c);
  if (nruns) *nruns = (uint32_t)(c.t == kR ? c.nruns() : 0);
  return RBREF_OK;
}
uint64_t rbref_to_array(const rbref_bitmap *b, uint32_t *out, uint64_t cap) {
  uint64_t n = 0;
  for (size_t i = 0; i < b->size(); ++i) {
    uint32_t hi = (uint32_t)b->keys[i] << 16;
    const Cont &c = b->vals[i];
    std::vector<uint16_t> v = c.t == kA ? c.v : c.t == kR ? run_values(c) : bitmap_to_array(c).v;
    for (uint16_t x : v) {
      if (n < cap) out[n] = hi | x;
      ++n;
    }
  }
  return n;
}

int rbref_deserialize(const uint8_t *buf, size_t len, rbref_bitmap **out) {
  // RoaringArray.deserialize(DataInput) (RoaringArray.java:276-348); EOF / bad cookie / size
  // > 65536 are the IOException cases of TestAdversarialInputs.
  *out = nullptr;
  Reader r{buf, len};
  uint32_t cookie = r.u32();
  if (!r.ok) return RBREF_EFORMAT;
  if ((cookie & 0xFFFF) != kCookie && cookie != kCookieNoRun) return RBREF_EFORMAT;
  bool hasrun = (cookie & 0xFFFF) == kCookie;
  uint32_t size = hasrun ? (cookie >> 16) + 1 : r.u32();
  if (!r.ok) return RBREF_EFORMAT;
  if (size > (1u << 16)) return RBREF_EFORMAT;
  std::vector<uint8_t> runmark;
  if (hasrun) {
    size_t nb = (size + 7) / 8;
    if (!r.need(nb)) return RBREF_EFORMAT;
    runmark.assign(buf + r.pos, buf + r.pos + nb);
    r.pos += nb;
  }
  std::vector<uint16_t> keys(size);
  std::vector<int> cards(size);
  for (uint32_t k = 0; k < size; ++k) {
    keys[k] = r.u16();
    cards[k] = 1 + r.u16();
  }
  if (!r.ok) return RBREF_EFORMAT;
  if (!hasrun || size >= (uint32_t)kNoOffsetThreshold) {
    if (!r.need(4ull * size)) return RBREF_EFORMAT;
    r.pos += 4ull * size;
  }
  std::unique_ptr<rbref_bitmap> b(new rbref_bitmap);
  for (uint32_t k = 0; k < size; ++k) {
    bool is_run = hasrun && (runmark[k / 8] >> (k % 8)) & 1;
    bool is_bitmap = cards[k] > kMaxArray && !is_run;
    Cont c;
    if (is_bitmap) {
      if (!r.need(8192)) return RBREF_EFORMAT;
      std::vector<uint64_t> w(kWords);
      std::memcpy(w.data(), buf + r.pos, 8192);
      r.pos += 8192;
      c = make_bitmap(std::move(w), cards[k]);
    } else if (is_run) {
      int nr = r.u16();
      if (!r.ok || !r.need(4ull * nr)) return RBREF_EFORMAT;
      std::vector<uint16_t> vl(2 * nr);
      std::memcpy(vl.data(), buf + r.pos, 4ull * nr);
      r.pos += 4ull * nr;
      c = make_run(std::move(vl));
    } else {
      if (!r.need(2ull * cards[k])) return RBREF_EFORMAT;
      std::vector<uint16_t> v(cards[k]);
      std::memcpy(v.data(), buf + r.pos, 2ull * cards[k]);
      r.pos += 2ull * cards[k];
      c = make_array(std::move(v));
    }
    b->keys.push_back(keys[k]);
    b->vals.push_back(std::move(c));
  }
  *out = b.release();
  return RBREF_OK;
}

static uint64_t payload_bytes(const Cont &c) { // Container.getArraySizeInBytes
  if (c.t == kA) return 2ull * c.card;
  if (c.t == kB) return 8192;
  return 2 + 4ull * c.nruns();
}
static bool has_run(const rbref_bitmap *b) {
  for (const Cont &c : b->vals)
    if (c.t == kR) return true;
  return false;
}
uint64_t rbref_serialized_size(const rbref_bitmap *b) { // RoaringArray.serializedSizeInBytes (:947-953)
  uint64_t n = b->size();
  uint64_t h = has_run(b) ? (n < (uint64_t)kNoOffsetThreshold ? 4 + (n + 7) / 8 + 4 * n
                                                               : 4 + (n + 7) / 8 + 8 * n)
                          : 8 + 8 * n;
  for (const Cont &c : b->vals) h += payload_bytes(c);
  return h;
}
int rbref_serialize(const rbref_bitmap *b, uint8_t *dst, uint64_t cap) {
  // RoaringArray.serialize (:851-883) + Container.writeArray per type.
  uint64_t need = rbref_serialized_size(b);
  if (cap < need) return RBREF_EINVAL;
  uint8_t *p = dst;
  auto w32 = [&](uint32_t v) { std::memcpy(p, &v, 4); p += 4; };
  auto w16 = [&](uint16_t v) { std::memcpy(p, &v, 2); p += 2; };
  uint32_t n = (uint32_t)b->size();
  bool hr = has_run(b);
  uint32_t start;
  if (hr) {
    w32(kCookie | ((n - 1) << 16));
    uint32_t nb = (n + 7) / 8;
    std::memset(p, 0, nb);
    for (uint32_t i = 0; i < n; ++i)
      if (b->vals[i].t == kR) p[i / 8] |= (uint8_t)(1u << (i % 8));
    p += nb;
    start = n < (uint32_t)kNoOffsetThreshold ? 4 + 4 * n + nb : 4 + 8 * n + nb;
  } else {
    w32(kCookieNoRun);
    w32(n);
    start = 4 + 4 + 4 * n + 4 * n;
  }
  for (uint32_t i = 0; i < n; ++i) {
    w16(b->keys[i]);
    w16((uint16_t)(cardinality(b->vals[i]) - 1));
  }
  if (!hr || n >= (uint32_t)kNoOffsetThreshold) {
    for (uint32_t i = 0; i < n; ++i) {
      w32(start);
      start += (uint32_t)payload_bytes(b->vals[i]);
    }
  }
  for (const Cont &c : b->vals) {
    if (c.t == kA) {
      if (c.card) std::memcpy(p, c.v.data(), 2ull * c.card); // horizontal_xor may hold an empty one
      p += 2ull * c.card;
    } else if (c.t == kB) {
      std::memcpy(p, c.w.data(), 8192);
      p += 8192;
    } else {
      w16((uint16_t)c.nruns());
      std::memcpy(p, c.v.data(), 4ull * c.nruns());
      p += 4ull * c.nruns();
    }
  }
  return RBREF_OK;
}

int rbref_from_soa(uint32_t n, const uint16_t *keys, const uint8_t *types, const uint32_t *cards,
                   const uint16_t *nruns, const uint8_t *payload, const uint64_t *offsets,
                   rbref_bitmap **out) {
  std::unique_ptr<rbref_bitmap> b(new rbref_bitmap);
  for (uint32_t i = 0; i < n; ++i) {
    const uint8_t *pp = payload + offsets[i];
    Cont c;
    if (types[i] == kA) {
      std::vector<uint16_t> v(cards[i]);
      std::memcpy(v.data(), pp, 2ull * cards[i]);
      c = make_array(std::move(v));
    } else if (types[i] == kB) {
      std::vector<uint64_t> w(kWords);
      std::memcpy(w.data(), pp, 8192);
      c = make_bitmap(std::move(w), (int)cards[i]);
    } else if (types[i] == kR) {
      std::vector<uint16_t> vl(2ull * nruns[i]);
      std::memcpy(vl.data(), pp, 4ull * nruns[i]);
      c = make_run(std::move(vl));
    } else {
      return RBREF_EINVAL;
    }
    b->keys.push_back(keys[i]);
    b->vals.push_back(std::move(c));
  }
  *out = b.release();
  return RBREF_OK;
}

rbref_bitmap *rbref_op(int op, const rbref_bitmap *a, const rbref_bitmap *b) { return bm_op(op, *a, *b); }

int64_t rbref_op_cardinality(int op, const rbref_bitmap *a, const rbref_bitmap *b) {
  int64_t ca = (int64_t)bm_card(*a), cb = (int64_t)bm_card(*b), inter = bm_and_card(*a, *b);
  switch (op) {
  case RBREF_AND: return inter;                // RoaringBitmap.java:413-434
  case RBREF_OR: return ca + cb - inter;       // :916-920
  case RBREF_XOR: return ca + cb - 2 * inter;  // :931-933
  default: return ca - inter;                  // :944-985 (same value on both branches)
  }
}

rbref_bitmap *rbref_xor_keep_empty(const rbref_bitmap *a, const rbref_bitmap *b) {
  return bm_xor_keep_empty(*a, *b); // c_ixor == c_xor: the static and in-place forms agree
}

int rbref_op_inplace(int op, rbref_bitmap *a, const rbref_bitmap *b) {
  switch (op) {
  case RBREF_AND: bm_iand(*a, *b); break;
  case RBREF_OR: bm_ior_ixor(*a, *b, false); break;
  case RBREF_XOR: bm_ior_ixor(*a, *b, true); break;
  case RBREF_ANDNOT: bm_iandnot(*a, *b); break;
  default: return RBREF_EINVAL;
  }
  return RBREF_OK;
}

rbref_bitmap *rbref_wide(int sem, const rbref_bitmap *const *bs, size_t n) {
  switch (sem) {
  case RBREF_FAST_OR: return wide_naive_or(bs, n);
  case RBREF_FAST_AND: return n > 10 ? wide_workshy_and(bs, n) : wide_naive_and(bs, n);
  case RBREF_WORKSHY_AND: return wide_workshy_and(bs, n);
  case RBREF_NAIVE_AND: return wide_naive_and(bs, n);
  case RBREF_FAST_XOR: return wide_naive_xor(bs, n);
  case RBREF_PAR_OR: return wide_par(bs, n, false);
  case RBREF_PAR_XOR: return wide_par(bs, n, true);
  case RBREF_NAIVE_AND_ITER: return wide_naive_and_iter(bs, n);
  case RBREF_HORIZONTAL_OR: return wide_horizontal(bs, n, false);
  case RBREF_HORIZONTAL_XOR: return wide_horizontal(bs, n, true);
  case RBREF_PQ_OR: return wide_pq_or(bs, n);
  case RBREF_PQ_XOR: return wide_pq_xor(bs, n);
  case RBREF_BUFFER_NAIVE_OR: return wide_buffer_naive_or(bs, n);
  case RBREF_BUFFER_PQ_OR: return wide_pq_or_sized(bs, n, bm_serialized_size_lazy, true);
  case RBREF_BUFFER_PQ_OR_ITER: return wide_pq_or_sized(bs, n, bm_size_immutable, true);
  case RBREF_BUFFER_PQ_XOR: return wide_buffer_pq_xor(bs, n);
  default: return nullptr;
  }
}

rbref_bitmap *rbref_wide_mt(int sem, const rbref_bitmap *const *bs, size_t n, int threads) {
  if (sem == RBREF_FAST_AND) sem = n > 10 ? RBREF_WORKSHY_AND : RBREF_NAIVE_AND;
  // global-order semantics (the queue's tie order spans keys): single-threaded
  if (sem == RBREF_NAIVE_AND || sem == RBREF_NAIVE_AND_ITER || sem >= RBREF_HORIZONTAL_OR) return rbref_wide(sem, bs, n);
  if (n == 0) return new BM;
  return wide_key_parallel(sem, bs, n, threads);
}

int64_t rbref_wide_cardinality(int op, const rbref_bitmap *const *bs, size_t n) {
  // FastAggregation.andCardinality / orCardinality (:71-101): the values equal the cardinality of
  // the corresponding aggregate for every input.
  if (n == 0) return 0;
  std::unique_ptr<rbref_bitmap> r(op == RBREF_AND ? wide_workshy_and(bs, n) : wide_naive_or(bs, n));
  return (int64_t)bm_card(*r);
}

int rbref_pairwise_batch(int op, const rbref_bitmap *const *a, const rbref_bitmap *const *b,
                         size_t npairs, int threads, uint64_t *total_card, uint64_t *total_containers) {
  if (threads < 1) threads = 1;
  std::vector<uint64_t> cards(threads, 0), conts(threads, 0);
  auto work = [&](int t) {
    size_t lo = npairs * t / threads, hi = npairs * (t + 1) / threads;
    for (size_t i = lo; i < hi; ++i) {
      BM *r = bm_op(op, *a[i], *b[i]);
      cards[t] += bm_card(*r);
      conts[t] += r->size();
      delete r;
    }
  };
  if (threads == 1) {
    work(0);
  } else {
    std::vector<std::thread> th;
    for (int t = 0; t < threads; ++t) th.emplace_back(work, t);
    for (auto &x : th) x.join();
  }
  uint64_t c = 0, k = 0;
  for (int t = 0; t < threads; ++t) { c += cards[t]; k += conts[t]; }
  if (total_card) *total_card = c;
  if (total_containers) *total_containers = k;
  return RBREF_OK;
}

// compareUsingMinMax (bsi/src/main/java/org/roaringbitmap/bsi/buffer/... RoaringBitmapSliceIndex.java:505-577):
// 1 = all (ebM, or ebM AND foundSet), 0 = empty, -1 = evaluate
static int bsi_min_max(int op, uint64_t a, uint64_t b, uint64_t mn, uint64_t mx) {
  switch (op) {
  case RBREF_BSI_LT: return a > mx ? 1 : a <= mn ? 0 : -1;
  case RBREF_BSI_LE: return a >= mx ? 1 : a < mn ? 0 : -1;
  case RBREF_BSI_GT: return a < mn ? 1 : a >= mx ? 0 : -1;
  case RBREF_BSI_GE: return a <= mn ? 1 : a > mx ? 0 : -1;
  case RBREF_BSI_EQ: return (mn == mx && mn == a) ? 1 : (a < mn || a > mx) ? 0 : -1;
  case RBREF_BSI_NEQ: return mn == mx ? (mn == a ? 0 : 1) : -1;
  default: return (a <= mn && b >= mx) ? 1 : (a > mx || b < mn) ? 0 : -1;
  }
}
// oNeilCompare (RoaringBitmapSliceIndex.java:432-472): the slices top-down, GT / LT / EQ kept as bitmaps
static BM *bsi_oneil(const rbref_bitmap *const *sl, size_t ns, const BM &ebm, int op, uint64_t pred, const BM *found) {
  const BM &fixed = found ? *found : ebm;
  std::unique_ptr<BM> gt(new BM), lt(new BM), eq(new BM(ebm));
  for (size_t k = ns; k-- > 0;) {
    const BM &s = *sl[k];
    if ((pred >> k) & 1) {
      std::unique_ptr<BM> d(bm_op(RBREF_ANDNOT, *eq, s));
      lt.reset(bm_op(RBREF_OR, *lt, *d));
      eq.reset(bm_op(RBREF_AND, *eq, s));
    } else {
      std::unique_ptr<BM> d(bm_op(RBREF_AND, *eq, s));
      gt.reset(bm_op(RBREF_OR, *gt, *d));
      eq.reset(bm_op(RBREF_ANDNOT, *eq, s));
    }
  }
  eq.reset(bm_op(RBREF_AND, fixed, *eq));
  switch (op) {
  case RBREF_BSI_EQ: return eq.release();
  case RBREF_BSI_NEQ: return bm_op(RBREF_ANDNOT, fixed, *eq);
  case RBREF_BSI_GT: return bm_op(RBREF_AND, *gt, fixed);
  case RBREF_BSI_LT: return bm_op(RBREF_AND, *lt, fixed);
  case RBREF_BSI_LE: {
    std::unique_ptr<BM> u(bm_op(RBREF_OR, *lt, *eq));
    return bm_op(RBREF_AND, *u, fixed);
  }
  default: { // GE
    std::unique_ptr<BM> u(bm_op(RBREF_OR, *gt, *eq));
    return bm_op(RBREF_AND, *u, fixed);
  }
  }
}

rbref_bitmap *rbref_bsi_compare(const rbref_bitmap *const *sl, size_t ns, const rbref_bitmap *ebm, int op,
                                uint64_t start, uint64_t end, const rbref_bitmap *found, uint64_t vmin, uint64_t vmax) {
  // compare (RoaringBitmapSliceIndex.java:475-503)
  const int sc = bsi_min_max(op, start, end, vmin, vmax);
  if (sc == 1) return found ? bm_op(RBREF_AND, *ebm, *found) : new BM(*ebm);
  if (sc == 0) return new BM;
  if (op == RBREF_BSI_RANGE) {
    std::unique_ptr<BM> ge(bsi_oneil(sl, ns, *ebm, RBREF_BSI_GE, start, found)),
        le(bsi_oneil(sl, ns, *ebm, RBREF_BSI_LE, end, found));
    return bm_op(RBREF_AND, *ge, *le);
  }
  return bsi_oneil(sl, ns, *ebm, op, start, found);
}

uint64_t rbref_bsi_compare_keys(const rbref_bitmap *const *per_key, size_t nkeys, size_t ns, int op, uint64_t start,
                                uint64_t end, uint64_t vmin, uint64_t vmax, int threads) {
  if (threads < 1) threads = 1;
  std::vector<uint64_t> cards(threads, 0);
  auto work = [&](int t) {
    const size_t lo = nkeys * t / threads, hi = nkeys * (t + 1) / threads;
    for (size_t k = lo; k < hi; ++k) {
      const rbref_bitmap *const *key = per_key + k * (ns + 1);
      std::unique_ptr<BM> r(rbref_bsi_compare(key, ns, key[ns], op, start, end, nullptr, vmin, vmax));
      cards[t] += bm_card(*r);
    }
  };
  if (threads == 1) {
    work(0);
  } else {
    std::vector<std::thread> th;
    for (int t = 0; t < threads; ++t) th.emplace_back(work, t);
    for (auto &x : th) x.join();
  }
  uint64_t c = 0;
  for (uint64_t v : cards) c += v;
  return c;
}

} // extern "C"
