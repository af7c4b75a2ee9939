// Validating msgpack cursor used by the native request scanners.
// Accepts both the old spec (RAW only, what msgpack 0.5.9 / the reference
// clients emit: jubatus/tools/packaging/allinone/jubapkg_version:10) and the
// new spec (str8 / bin8-32).
#pragma once
#include <stdint.h>
#include <string.h>

namespace jb {

struct Cursor {
  const uint8_t* p;
  const uint8_t* end;

  bool need(uint64_t n) const { return (uint64_t)(end - p) >= n; }
  uint32_t be16() { uint32_t v = ((uint32_t)p[0] << 8) | p[1]; p += 2; return v; }
  uint32_t be32() {
    uint32_t v = ((uint32_t)p[0] << 24) | ((uint32_t)p[1] << 16) | ((uint32_t)p[2] << 8) | p[3];
    p += 4; return v;
  }
  uint64_t be64() { uint64_t hi = be32(); uint64_t lo = be32(); return (hi << 32) | lo; }

  bool array(uint32_t* n) {
    if (!need(1)) return false;
    uint8_t t = *p;
    if ((t & 0xf0) == 0x90) { ++p; *n = t & 0x0f; return true; }
    if (t == 0xdc) { if (!need(3)) return false; ++p; *n = be16(); return true; }
    if (t == 0xdd) { if (!need(5)) return false; ++p; *n = be32(); return true; }
    return false;
  }
  bool map(uint32_t* n) {
    if (!need(1)) return false;
    uint8_t t = *p;
    if ((t & 0xf0) == 0x80) { ++p; *n = t & 0x0f; return true; }
    if (t == 0xde) { if (!need(3)) return false; ++p; *n = be16(); return true; }
    if (t == 0xdf) { if (!need(5)) return false; ++p; *n = be32(); return true; }
    return false;
  }
  bool raw(const uint8_t** s, uint32_t* n) {
    if (!need(1)) return false;
    uint8_t t = *p;
    uint32_t len;
    const uint8_t* q = p + 1;
    if ((t & 0xe0) == 0xa0) len = t & 0x1f;
    else if (t == 0xd9 || t == 0xc4) { if (!need(2)) return false; len = q[0]; q += 1; }
    else if (t == 0xda || t == 0xc5) { if (!need(3)) return false; len = ((uint32_t)q[0] << 8) | q[1]; q += 2; }
    else if (t == 0xdb || t == 0xc6) {
      if (!need(5)) return false;
      len = ((uint32_t)q[0] << 24) | ((uint32_t)q[1] << 16) | ((uint32_t)q[2] << 8) | q[3]; q += 4;
    } else return false;
    if ((uint64_t)(end - q) < len) return false;
    *s = q; *n = len; p = q + len;
    return true;
  }
  bool number(double* out) {
    if (!need(1)) return false;
    uint8_t t = *p;
    if (t <= 0x7f) { ++p; *out = t; return true; }
    if (t >= 0xe0) { ++p; *out = (double)(int8_t)t; return true; }
    static const uint8_t sz[] = {1, 2, 4, 8};
    uint64_t n;
    switch (t) {
      case 0xcc: case 0xd0: n = 1; break;
      case 0xcd: case 0xd1: n = 2; break;
      case 0xce: case 0xd2: case 0xca: n = 4; break;
      case 0xcf: case 0xd3: case 0xcb: n = 8; break;
      default: return false;
    }
    (void)sz;
    if (!need(1 + n)) return false;
    ++p;
    switch (t) {
      case 0xcc: *out = *p++; return true;
      case 0xcd: *out = be16(); return true;
      case 0xce: *out = be32(); return true;
      case 0xcf: *out = (double)be64(); return true;
      case 0xd0: *out = (int8_t)*p++; return true;
      case 0xd1: *out = (int16_t)be16(); return true;
      case 0xd2: *out = (int32_t)be32(); return true;
      case 0xd3: *out = (double)(int64_t)be64(); return true;
      case 0xca: { uint32_t u = be32(); float f; memcpy(&f, &u, 4); *out = f; return true; }
      case 0xcb: { uint64_t u = be64(); double d; memcpy(&d, &u, 8); *out = d; return true; }
    }
    return false;
  }
  // skip one object of any type (bounded recursion)
  bool skip(int depth = 0) {
    if (depth > 64 || !need(1)) return false;
    uint8_t t = *p;
    if (t <= 0x7f || t >= 0xe0 || t == 0xc0 || t == 0xc2 || t == 0xc3) { ++p; return true; }
    if ((t & 0xe0) == 0xa0 || t == 0xd9 || t == 0xda || t == 0xdb || t == 0xc4 || t == 0xc5 || t == 0xc6) {
      const uint8_t* s; uint32_t n; return raw(&s, &n);
    }
    uint32_t n;
    if (array(&n)) { for (uint32_t i = 0; i < n; ++i) if (!skip(depth + 1)) return false; return true; }
    if (map(&n)) { for (uint32_t i = 0; i < 2 * n; ++i) if (!skip(depth + 1)) return false; return true; }
    double d;
    if (number(&d)) return true;
    // ext types
    uint64_t len = 0, hdr = 0;
    switch (t) {
      case 0xd4: len = 2; hdr = 1; break; case 0xd5: len = 3; hdr = 1; break;
      case 0xd6: len = 5; hdr = 1; break; case 0xd7: len = 9; hdr = 1; break;
      case 0xd8: len = 17; hdr = 1; break;
      case 0xc7: if (!need(2)) return false; len = 1 + p[1]; hdr = 2; break;
      case 0xc8: if (!need(3)) return false; len = 1 + (((uint32_t)p[1] << 8) | p[2]); hdr = 3; break;
      case 0xc9: if (!need(5)) return false;
        len = 1 + (((uint32_t)p[1] << 24) | ((uint32_t)p[2] << 16) | ((uint32_t)p[3] << 8) | p[4]); hdr = 5; break;
      default: return false;
    }
    if (!need(hdr + len)) return false;
    p += hdr + len;
    return true;
  }
};

}  // namespace jb
