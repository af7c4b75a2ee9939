// Squared euclidean distances points x centers on the matrix cores.
//
// Reference: the clustering engine's push / get_nearest_* paths
// (jubatus/server/server/clustering_serv.cpp:108-137) over jubatus_core's
// k-means / GMM on compressive coresets (EXTERNAL).
//
// D[i][j] = |x_i|^2 + |c_j|^2 - 2 x_i . c_j, with the Gram term X C^T on
// v_mfma_f32_16x16x4_f32 (fp32 in / fp32 accumulate: exact f32 products, the
// same numerics as an f32 fmaf chain). One wave computes a 16 x 16 tile
// (16 points x 16 centres) stepping K by 4; a 256-thread workgroup covers 64
// points. Fragment maps (gfx950, 16x16x4 f32):
//   A: lane l holds A[l & 15][k = l >> 4]     (X rows)
//   B: lane l holds B[k = l >> 4][l & 15]     (C^T, i.e. C[l & 15][k])
//   D: lane l, reg r -> row (l >> 4) * 4 + r, col l & 15
#include "jb_device.hpp"

namespace jb {

typedef float f32x4 __attribute__((ext_vector_type(4)));

__global__ __launch_bounds__(256) void sqdist_mfma_kernel(
    const float* __restrict__ X, int64_t n, const float* __restrict__ C, int k, int d,
    const float* __restrict__ xn2, const float* __restrict__ cn2, float* __restrict__ out) {
  const int lane = threadIdx.x & 63;
  const int wv = threadIdx.x >> 6;
  const int64_t row0 = ((int64_t)blockIdx.x * 4 + wv) * 16;
  const int col0 = blockIdx.y * 16;
  if (row0 >= n) return;
  const int ar = lane & 15;   // A row / B col inside the tile
  const int kq = lane >> 4;   // k offset 0..3
  const int64_t xi = row0 + ar;
  const int cj = col0 + ar;
  f32x4 acc = {0.f, 0.f, 0.f, 0.f};
  for (int kk = 0; kk < d; kk += 4) {
    const int kc = kk + kq;
    const float a = (xi < n && kc < d) ? X[xi * d + kc] : 0.f;
    const float b = (cj < k && kc < d) ? C[(int64_t)cj * d + kc] : 0.f;
    acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, acc, 0, 0, 0);
  }
  const int col = col0 + (lane & 15);
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const int64_t row = row0 + (lane >> 4) * 4 + r;
    if (row < n && col < k) out[row * k + col] = fmaxf(0.f, xn2[row] + cn2[col] - 2.f * acc[r]);
  }
}

}  // namespace jb

extern "C" int jb_sqdist_mfma(const float* X, int64_t n, const float* C, int k, int d,
                              const float* xn2, const float* cn2, float* out, hipStream_t stream) {
  if (n <= 0 || k <= 0) return 0;
  dim3 grid((unsigned)((n + 63) / 64), (unsigned)((k + 15) / 16));
  hipLaunchKernelGGL(jb::sqdist_mfma_kernel, grid, dim3(256), 0, stream, X, n, C, k, d, xn2, cn2, out);
  return (int)hipGetLastError();
}
