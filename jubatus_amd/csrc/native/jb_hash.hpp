// Host hashing primitives: FNV-1a/64 feature hashing (twin of
// csrc/hip/jb_device.hpp), CRC-32 (model file container, reference
// jubatus/server/common/crc32.cpp:25-56) and MD5 (consistent hash ring,
// reference jubatus/server/common/cht.cpp:36-40).
#pragma once
#include <stdint.h>
#include <string.h>
#include <string>

namespace jb {

constexpr uint64_t kFnvOffset = 0xcbf29ce484222325ull;
constexpr uint64_t kFnvPrime = 0x100000001b3ull;

inline uint64_t fnv_bytes(uint64_t h, const uint8_t* p, size_t n) {
  for (size_t i = 0; i < n; ++i) {
    h ^= (uint64_t)p[i];
    h *= kFnvPrime;
  }
  return h;
}

inline int64_t hash_to_index(uint64_t h, uint64_t H) {
  h ^= h >> 29;
  h *= 0xbf58476d1ce4e5b9ull;
  h ^= h >> 32;
  return (int64_t)(((unsigned __int128)h * (unsigned __int128)H) >> 64);
}

// ------------------------------------------------------------------ CRC32 ---
struct Crc32Table {
  uint32_t t[256];
  Crc32Table() {
    for (uint32_t i = 0; i < 256; ++i) {
      uint32_t c = i;
      for (int k = 0; k < 8; ++k) c = (c & 1) ? (0xEDB88320u ^ (c >> 1)) : (c >> 1);
      t[i] = c;
    }
  }
};

inline uint32_t crc32_update(uint32_t crc, const uint8_t* p, size_t n) {
  static const Crc32Table tab;
  crc = ~crc;
  for (size_t i = 0; i < n; ++i) crc = tab.t[(crc ^ p[i]) & 0xff] ^ (crc >> 8);
  return ~crc;
}

// -------------------------------------------------------------------- MD5 ---
// RFC 1321, written from the specification.
class Md5 {
 public:
  Md5() { reset(); }
  void reset() {
    a_ = 0x67452301u; b_ = 0xefcdab89u; c_ = 0x98badcfeu; d_ = 0x10325476u;
    len_ = 0; fill_ = 0;
  }
  void update(const uint8_t* p, size_t n) {
    len_ += n;
    while (n > 0) {
      size_t take = 64 - fill_;
      if (take > n) take = n;
      memcpy(buf_ + fill_, p, take);
      fill_ += take; p += take; n -= take;
      if (fill_ == 64) { block(buf_); fill_ = 0; }
    }
  }
  void digest(uint8_t out[16]) {
    uint64_t bits = len_ * 8;
    uint8_t pad = 0x80;
    update(&pad, 1);
    uint8_t z = 0;
    while (fill_ != 56) update(&z, 1);
    uint8_t lb[8];
    for (int i = 0; i < 8; ++i) lb[i] = (uint8_t)(bits >> (8 * i));
    update(lb, 8);
    uint32_t v[4] = {a_, b_, c_, d_};
    for (int i = 0; i < 4; ++i)
      for (int k = 0; k < 4; ++k) out[4 * i + k] = (uint8_t)(v[i] >> (8 * k));
  }
  static std::string hex(const std::string& s) {
    Md5 m; m.update((const uint8_t*)s.data(), s.size());
    uint8_t d[16]; m.digest(d);
    static const char* hx = "0123456789abcdef";
    std::string r(32, '0');
    for (int i = 0; i < 16; ++i) { r[2 * i] = hx[d[i] >> 4]; r[2 * i + 1] = hx[d[i] & 15]; }
    return r;
  }

 private:
  static uint32_t rol(uint32_t x, int c) { return (x << c) | (x >> (32 - c)); }
  void block(const uint8_t* p) {
    static const uint32_t K[64] = {
        0xd76aa478, 0xe8c7b756, 0x242070db, 0xc1bdceee, 0xf57c0faf, 0x4787c62a, 0xa8304613,
        0xfd469501, 0x698098d8, 0x8b44f7af, 0xffff5bb1, 0x895cd7be, 0x6b901122, 0xfd987193,
        0xa679438e, 0x49b40821, 0xf61e2562, 0xc040b340, 0x265e5a51, 0xe9b6c7aa, 0xd62f105d,
        0x02441453, 0xd8a1e681, 0xe7d3fbc8, 0x21e1cde6, 0xc33707d6, 0xf4d50d87, 0x455a14ed,
        0xa9e3e905, 0xfcefa3f8, 0x676f02d9, 0x8d2a4c8a, 0xfffa3942, 0x8771f681, 0x6d9d6122,
        0xfde5380c, 0xa4beea44, 0x4bdecfa9, 0xf6bb4b60, 0xbebfbc70, 0x289b7ec6, 0xeaa127fa,
        0xd4ef3085, 0x04881d05, 0xd9d4d039, 0xe6db99e5, 0x1fa27cf8, 0xc4ac5665, 0xf4292244,
        0x432aff97, 0xab9423a7, 0xfc93a039, 0x655b59c3, 0x8f0ccc92, 0xffeff47d, 0x85845dd1,
        0x6fa87e4f, 0xfe2ce6e0, 0xa3014314, 0x4e0811a1, 0xf7537e82, 0xbd3af235, 0x2ad7d2bb,
        0xeb86d391};
    static const int R[64] = {7, 12, 17, 22, 7, 12, 17, 22, 7, 12, 17, 22, 7, 12, 17, 22,
                              5, 9,  14, 20, 5, 9,  14, 20, 5, 9,  14, 20, 5, 9,  14, 20,
                              4, 11, 16, 23, 4, 11, 16, 23, 4, 11, 16, 23, 4, 11, 16, 23,
                              6, 10, 15, 21, 6, 10, 15, 21, 6, 10, 15, 21, 6, 10, 15, 21};
    uint32_t M[16];
    for (int i = 0; i < 16; ++i)
      M[i] = (uint32_t)p[4 * i] | ((uint32_t)p[4 * i + 1] << 8) | ((uint32_t)p[4 * i + 2] << 16) |
             ((uint32_t)p[4 * i + 3] << 24);
    uint32_t a = a_, b = b_, c = c_, d = d_;
    for (int i = 0; i < 64; ++i) {
      uint32_t f; int g;
      if (i < 16) { f = (b & c) | (~b & d); g = i; }
      else if (i < 32) { f = (d & b) | (~d & c); g = (5 * i + 1) & 15; }
      else if (i < 48) { f = b ^ c ^ d; g = (3 * i + 5) & 15; }
      else { f = c ^ (b | ~d); g = (7 * i) & 15; }
      uint32_t tmp = d; d = c; c = b;
      b = b + rol(a + f + K[i] + M[g], R[i]);
      a = tmp;
    }
    a_ += a; b_ += b; c_ += c; d_ += d;
  }
  uint32_t a_, b_, c_, d_;
  uint64_t len_;
  size_t fill_;
  uint8_t buf_[64];
};

}  // namespace jb
