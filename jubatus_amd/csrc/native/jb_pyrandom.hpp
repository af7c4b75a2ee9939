// CPython's random.Random in C++: the Mersenne Twister (MT19937) seeded from
// an int the way _randommodule.c does it (init_by_array over the 32-bit words
// of |seed|), random() as 53-bit doubles, getrandbits / _randbelow, and the
// sample() / choices() / choice() algorithms of Lib/random.py (3.10). The
// native servers whose engines draw from Python's RNG in the Python servers
// (models/clustering.py: k-means++ draws, the simple compressor's sample)
// consume the identical stream, so both servers cluster alike.
#pragma once
#include <math.h>
#include <stdint.h>

#include <algorithm>
#include <stdexcept>
#include <unordered_set>
#include <vector>

namespace jb {

class PyRandom {
 public:
  explicit PyRandom(int64_t seed = 0) { seed_int(seed); }

  void seed_int(int64_t seed) {
    uint64_t n = seed < 0 ? (uint64_t)(-(seed + 1)) + 1 : (uint64_t)seed;
    std::vector<uint32_t> key;
    while (n) {
      key.push_back((uint32_t)(n & 0xffffffffu));
      n >>= 32;
    }
    if (key.empty()) key.push_back(0);
    init_by_array(key);
  }

  uint32_t genrand() {
    if (mti_ >= kN) {
      int kk;
      uint32_t y;
      for (kk = 0; kk < kN - kM; ++kk) {
        y = (mt_[kk] & kUpper) | (mt_[kk + 1] & kLower);
        mt_[kk] = mt_[kk + kM] ^ (y >> 1) ^ ((y & 1u) ? kMatrixA : 0u);
      }
      for (; kk < kN - 1; ++kk) {
        y = (mt_[kk] & kUpper) | (mt_[kk + 1] & kLower);
        mt_[kk] = mt_[kk + (kM - kN)] ^ (y >> 1) ^ ((y & 1u) ? kMatrixA : 0u);
      }
      y = (mt_[kN - 1] & kUpper) | (mt_[0] & kLower);
      mt_[kN - 1] = mt_[kM - 1] ^ (y >> 1) ^ ((y & 1u) ? kMatrixA : 0u);
      mti_ = 0;
    }
    uint32_t y = mt_[mti_++];
    y ^= (y >> 11);
    y ^= (y << 7) & 0x9d2c5680u;
    y ^= (y << 15) & 0xefc60000u;
    y ^= (y >> 18);
    return y;
  }

  // random.random()
  double random() {
    const uint32_t a = genrand() >> 5, b = genrand() >> 6;
    return ((double)a * 67108864.0 + (double)b) * (1.0 / 9007199254740992.0);
  }

  // getrandbits(k), 1 <= k <= 64
  uint64_t getrandbits(int k) {
    if (k <= 32) return genrand() >> (32 - k);
    const uint64_t lo = genrand();
    const uint64_t hi = genrand() >> (64 - k);
    return lo | (hi << 32);
  }

  // _randbelow_with_getrandbits(n)
  uint64_t randbelow(uint64_t n) {
    if (n == 0) return 0;
    int k = 0;
    for (uint64_t x = n; x; x >>= 1) ++k;          // n.bit_length()
    uint64_t r = getrandbits(k);
    while (r >= n) r = getrandbits(k);
    return r;
  }

  // sample(range(n), k)
  std::vector<int64_t> sample_range(int64_t n, int64_t k) {
    if (k < 0 || k > n) throw std::invalid_argument("Sample larger than population or is negative");
    std::vector<int64_t> out((size_t)k);
    int64_t setsize = 21;
    if (k > 5) setsize += (int64_t)pow(4.0, ceil(log((double)(k * 3)) / log(4.0)));
    if (n <= setsize) {
      std::vector<int64_t> pool((size_t)n);
      for (int64_t i = 0; i < n; ++i) pool[(size_t)i] = i;
      for (int64_t i = 0; i < k; ++i) {
        const int64_t j = (int64_t)randbelow((uint64_t)(n - i));
        out[(size_t)i] = pool[(size_t)j];
        pool[(size_t)j] = pool[(size_t)(n - i - 1)];
      }
    } else {
      std::unordered_set<int64_t> sel;
      for (int64_t i = 0; i < k; ++i) {
        int64_t j = (int64_t)randbelow((uint64_t)n);
        while (sel.count(j)) j = (int64_t)randbelow((uint64_t)n);
        sel.insert(j);
        out[(size_t)i] = j;
      }
    }
    return out;
  }

  // choices(range(n), weights=w, k=1)[0]; -1 when the total is not positive
  int64_t choice_weighted(const std::vector<double>& w) {
    const int64_t n = (int64_t)w.size();
    if (n == 0) return -1;
    std::vector<double> cum((size_t)n);
    double acc = 0.0;
    for (int64_t i = 0; i < n; ++i) cum[(size_t)i] = acc = acc + w[(size_t)i];
    const double total = cum.back() + 0.0;
    if (!(total > 0.0) || !std::isfinite(total)) return -1;
    const double x = random() * total;
    // bisect_right(cum, x, 0, n - 1)
    int64_t lo = 0, hi = n - 1;
    while (lo < hi) {
      const int64_t mid = (lo + hi) / 2;
      if (x < cum[(size_t)mid]) hi = mid;
      else lo = mid + 1;
    }
    return lo;
  }

  // choice(seq) index
  int64_t choice_index(int64_t n) { return (int64_t)randbelow((uint64_t)n); }

 private:
  static constexpr int kN = 624, kM = 397;
  static constexpr uint32_t kMatrixA = 0x9908b0dfu, kUpper = 0x80000000u, kLower = 0x7fffffffu;

  void init_genrand(uint32_t s) {
    mt_[0] = s;
    for (mti_ = 1; mti_ < kN; ++mti_)
      mt_[mti_] = 1812433253u * (mt_[mti_ - 1] ^ (mt_[mti_ - 1] >> 30)) + (uint32_t)mti_;
  }

  void init_by_array(const std::vector<uint32_t>& key) {
    init_genrand(19650218u);
    const int klen = (int)key.size();
    int i = 1, j = 0;
    for (int k = kN > klen ? kN : klen; k; --k) {
      mt_[i] = (mt_[i] ^ ((mt_[i - 1] ^ (mt_[i - 1] >> 30)) * 1664525u)) + key[(size_t)j] + (uint32_t)j;
      ++i;
      ++j;
      if (i >= kN) { mt_[0] = mt_[kN - 1]; i = 1; }
      if (j >= klen) j = 0;
    }
    for (int k = kN - 1; k; --k) {
      mt_[i] = (mt_[i] ^ ((mt_[i - 1] ^ (mt_[i - 1] >> 30)) * 1566083941u)) - (uint32_t)i;
      ++i;
      if (i >= kN) { mt_[0] = mt_[kN - 1]; i = 1; }
    }
    mt_[0] = 0x80000000u;
    mti_ = kN;
  }

  uint32_t mt_[kN];
  int mti_ = kN + 1;
};

}  // namespace jb
