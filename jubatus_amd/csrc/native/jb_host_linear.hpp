// Host linear classifier step: one sample of the online update, fp32, in
// the reference's order (jubatus/server/server/classifier_serv.cpp:138-144
// trains sample after sample). The same rules as csrc/hip/jb_linear.hpp
// step_coeffs / dprec and the fp64 oracle jubatus_amd/models/linear_oracle.py
// (P: the diagonal precision 1/S, additive updates).
//
// Users: the host serial trainer (jb_cpu_serial.cpp: the in-house CPU
// baseline of bench.py) and the native jubaclassifier's host backend
// (csrc/server/jubaclassifier.cpp HostClassifier: GPU-less hosts).
#pragma once
#include <algorithm>
#include <cmath>
#include <cstdint>
#include <vector>

namespace jb {
namespace hl {

enum { PERCEPTRON = 0, PA = 1, PA1 = 2, PA2 = 3, CW = 4, AROW = 5, NHERD = 6 };

// step sizes of one update (jb_linear.hpp step_coeffs); false: no update
inline bool coeffs(int method, float m, float var, float nrm, bool has_l, float C, float* tau,
                   float* beta) {
  switch (method) {
    case PERCEPTRON:
      if (m <= 0.f) { *tau = 1.f; *beta = 0.f; return true; }
      return false;
    case PA: case PA1: case PA2: {
      const float loss = 1.f - m;
      if (!(loss > 0.f && nrm > 0.f)) return false;
      const float sq = (has_l ? 2.f : 1.f) * nrm;
      *tau = method == PA ? loss / sq : method == PA1 ? std::fmin(C, loss / sq) : loss / (sq + 0.5f / C);
      *beta = 0.f;
      return true;
    }
    case CW: {
      if (!(var > 0.f)) return false;
      const float b = 1.f + 2.f * C * m;
      const float disc = b * b - 8.f * C * (m - C * var);
      const float g = (-b + std::sqrt(std::fmax(disc, 0.f))) / (4.f * C * var);
      if (!(g > 0.f)) return false;
      *tau = g; *beta = 2.f * g * C;
      return true;
    }
    case AROW:
      if (!(m < 1.f)) return false;
      *beta = 1.f / (var + 1.f / C);
      *tau = (1.f - m) * *beta;
      return true;
    case NHERD: {
      if (!(m < 1.f)) return false;
      *tau = (1.f - m) / (var + 1.f / C);
      const float cv = 1.f + C * var;
      *beta = (C * C * var + 2.f * C) / (cv * cv);
      return true;
    }
    default: return false;
  }
}

struct Trainer {
  int method, LC;
  float C;
  const uint8_t* active;
  float* W;
  float* P;          // precisions (CW / AROW / NHERD), else null
  std::vector<float> s, a, b;

  Trainer(int method_, float C_, int LC_, const uint8_t* act, float* W_, float* P_)
      : method(method_), LC(LC_), C(C_), active(act), W(W_), P(method_ >= CW ? P_ : nullptr),
        s((size_t)LC_), a(64), b(64) {}

  void prefetch(const int32_t* ix, int n) const {
    for (int f = 0; f < n; ++f)
      if (ix[f] >= 0) {
        __builtin_prefetch(W + (int64_t)ix[f] * LC);
        if (P != nullptr) __builtin_prefetch(P + (int64_t)ix[f] * LC);
      }
  }

  // one sample; mag (nullable): per slot max(|dW_y|, |dW_l*|) of the update
  bool step(const int32_t* ix, const float* x, int n, int y, float* mag) {
    if ((int)a.size() < n) { a.resize((size_t)n); b.resize((size_t)n); }
    std::fill(s.begin(), s.end(), 0.f);
    float nrm = 0.f;
    for (int f = 0; f < n; ++f) {
      nrm += x[f] * x[f];
      if (ix[f] < 0) continue;
      const float* w = W + (int64_t)ix[f] * LC;
      const float xf = x[f];
      for (int l = 0; l < LC; ++l) s[(size_t)l] += xf * w[l];
    }
    int ls = -1;
    float best = -INFINITY;
    for (int l = 0; l < LC; ++l)
      if (active[l] && l != y && s[(size_t)l] > best) { best = s[(size_t)l]; ls = l; }
    const float m = s[(size_t)y] - (ls >= 0 ? best : 0.f);
    float var = 0.f;
    if (P != nullptr) {
      for (int f = 0; f < n; ++f) {
        if (ix[f] < 0) { a[(size_t)f] = b[(size_t)f] = 0.f; continue; }
        const float* p = P + (int64_t)ix[f] * LC;
        a[(size_t)f] = 1.f / p[y];
        b[(size_t)f] = ls >= 0 ? 1.f / p[ls] : 0.f;
        var += x[f] * x[f] * (a[(size_t)f] + b[(size_t)f]);
      }
    }
    float tau = 0.f, beta = 0.f;
    if (!coeffs(method, m, var, nrm, ls >= 0, C, &tau, &beta)) {
      if (mag != nullptr) std::fill(mag, mag + n, 0.f);
      return false;
    }
    for (int f = 0; f < n; ++f) {
      if (ix[f] < 0) { if (mag != nullptr) mag[f] = 0.f; continue; }
      float* w = W + (int64_t)ix[f] * LC;
      const float xf = x[f];
      const float sa = P != nullptr ? a[(size_t)f] : 1.f;
      const float sb = P != nullptr ? b[(size_t)f] : 1.f;
      const float dy = tau * sa * xf;
      const float dl = ls >= 0 ? -tau * sb * xf : 0.f;
      w[y] += dy;
      if (ls >= 0) w[ls] += dl;
      if (mag != nullptr) mag[f] = std::fmax(std::fabs(dy), std::fabs(dl));
      if (P != nullptr) {
        float* p = P + (int64_t)ix[f] * LC;
        const float bx2 = beta * xf * xf;
        p[y] += method == CW ? bx2 : bx2 / (1.f - bx2 * sa);
        if (ls >= 0) p[ls] += method == CW ? bx2 : bx2 / (1.f - bx2 * sb);
      }
    }
    return true;
  }
};


// scores of every label column of one sample: out[LC]
inline void scores(const float* W, int LC, const int32_t* ix, const float* x, int n, float* out) {
  std::fill(out, out + LC, 0.f);
  for (int f = 0; f < n; ++f) {
    if (ix[f] < 0) continue;
    const float* w = W + (int64_t)ix[f] * LC;
    const float xf = x[f];
    for (int l = 0; l < LC; ++l) out[l] += xf * w[l];
  }
}

}  // namespace hl
}  // namespace jb
