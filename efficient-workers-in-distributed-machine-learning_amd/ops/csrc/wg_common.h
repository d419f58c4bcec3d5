// Winograd transform constants and the weight-gradient output transform, shared by
// winograd_f32.hip and conv_f32.hip (where the transform of a deferred Winograd weight gradient
// rides in a direct conv's backward-data GEMM launch).
#pragma once
#include "common.h"

// channels per thread of the m = 2 input / weight / weight-gradient transforms.  2 (twice the
// threads) was measured on VGG-11: input transforms 132 -> 138 us/step (the 8x8-map passes
// already run at ~5 TB/s), output transforms 114 -> 101 -- so the output transform takes its own
// width (k_wg_output's VW: 2 where C_out <= 512) and these stay at 4.
#ifndef WG2_VW
#define WG2_VW 4
#endif

namespace {

// Transform matrices as constexpr functions: inside fully unrolled loops every coefficient is a
// compile-time constant, zero terms are skipped at the source (0 * x is not foldable in IEEE)
// and +-1 products fold to adds / subtracts.
template <int M>
__device__ constexpr float wg_bt(int i, int j) {
  if constexpr (M == 2) {
    constexpr float v[4][4] = {{1, 0, -1, 0}, {0, 1, 1, 0}, {0, -1, 1, 0}, {0, 1, 0, -1}};
    return v[i][j];
  } else {
    constexpr float v[6][6] = {{4, 0, -5, 0, 1, 0},  {0, -4, -4, 1, 1, 0}, {0, 4, -4, -1, 1, 0},
                               {0, -2, -1, 2, 1, 0}, {0, 2, -1, -2, 1, 0}, {0, 4, 0, -5, 0, 1}};
    return v[i][j];
  }
}

template <int M>
__device__ constexpr float wg_g(int i, int j) {
  if constexpr (M == 2) {
    constexpr float v[4][3] = {{1, 0, 0}, {.5f, .5f, .5f}, {.5f, -.5f, .5f}, {0, 0, 1}};
    return v[i][j];
  } else {
    constexpr float v[6][3] = {{1.f / 4, 0, 0},
                               {-1.f / 6, -1.f / 6, -1.f / 6},
                               {-1.f / 6, 1.f / 6, -1.f / 6},
                               {1.f / 24, 1.f / 12, 1.f / 6},
                               {1.f / 24, -1.f / 12, 1.f / 6},
                               {0, 0, 1}};
    return v[i][j];
  }
}

template <int M>
__device__ constexpr float wg_at(int i, int j) {
  if constexpr (M == 2) {
    constexpr float v[2][4] = {{1, 1, 1, 0}, {0, 1, -1, -1}};
    return v[i][j];
  } else {
    constexpr float v[4][6] = {
        {1, 1, 1, 1, 1, 0}, {0, 1, -1, 2, -2, 0}, {0, 1, 1, 4, 4, 0}, {0, 1, -1, 8, -8, 1}};
    return v[i][j];
  }
}

template <int M>
struct Wg {
  static constexpr int A = M + 2;             // patch / transform size
  static constexpr int VW = M == 2 ? WG2_VW : 2;   // channels per thread (registers: A*A vectors)
  typedef float V __attribute__((ext_vector_type(VW)));
};

// sum_k c(k) * x[k] over the nonzero constant coefficients (CF: coefficient function)
template <int N, typename T, typename CF>
__device__ __forceinline__ T wg_dot(CF cf, const T* x) {
  T acc{};
  bool first = true;
#pragma unroll
  for (int k = 0; k < N; ++k) {
    const float c = cf(k);
    if (c == 0.0f) continue;
    const T term = c == 1.0f ? x[k] : c == -1.0f ? -x[k] : c * x[k];
    acc = first ? term : acc + term;
    first = false;
  }
  return acc;
}

// Another layer's weight-gradient output transform riding along in an input launch (deferred by
// ops/conv.py: it only feeds the optimizer / codec, so it need not cost a launch of its own)
struct WgOut {
  const float* src;  // dU (nsplit 1) or the K-split slabs
  float* dw;
  int nsplit, Nc, C;
};


// dw[o][3][3][i..] = (G^T dU G) summed over the K-split slabs, for the thread's element group g
// (o, VW channels) of the Nc x C / VW groups
template <int M>
__device__ __forceinline__ void wg_wgrad_out(const float* __restrict__ src, int nsplit,
                                             float* __restrict__ dw, int Nc, int C, long long g) {
  using T = typename Wg<M>::V;
  constexpr int A = Wg<M>::A, VW = Wg<M>::VW;
  const int cq = C / VW;
  if (g >= (long long)Nc * cq) return;
  const int o = (int)(g / cq), i = (int)(g - (long long)o * cq) * VW;
  const long long xs = (long long)Nc * C;
  const float* p = src + (long long)o * C + i;
  T t[3][A];  // G^T dU, one column b at a time
#pragma unroll
  for (int b = 0; b < A; ++b) {
    T col[A];
#pragma unroll
    for (int a = 0; a < A; ++a) col[a] = *reinterpret_cast<const T*>(p + (a * A + b) * xs);
    for (int z = 1; z < nsplit; ++z) {  // fixed order
      const float* pz = p + (long long)z * A * A * xs;
#pragma unroll
      for (int a = 0; a < A; ++a) col[a] += *reinterpret_cast<const T*>(pz + (a * A + b) * xs);
    }
#pragma unroll
    for (int r = 0; r < 3; ++r) t[r][b] = wg_dot<A>([&](int a) { return wg_g<M>(a, r); }, col);
  }
  float* w = dw + (long long)o * 9 * C + i;
#pragma unroll
  for (int r = 0; r < 3; ++r)
#pragma unroll
    for (int s = 0; s < 3; ++s)  // (G^T dU) G
      *reinterpret_cast<T*>(w + (r * 3 + s) * C) =
          wg_dot<A>([&](int b) { return wg_g<M>(b, s); }, t[r]);
}

}  // namespace
