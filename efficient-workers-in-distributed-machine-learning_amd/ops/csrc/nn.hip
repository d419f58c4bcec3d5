// Model-side kernels for the CNNs of the reference (gfx950, wave64).
//
// MaxPool 2x2 / stride 2 (VGG's five pools, LeNet's two), NCHW, bf16 or fp32.  PyTorch's kernel
// stores an int64 argmax per output and its backward ran at 26 us per call on VGG-11 bs128
// (profiles/vgg11_bs128_topk1pct_qsgd8_graph_bf16params.txt); here the argmax is a 1-byte window
// position (0..3) and both directions are dense, coalesced streams: one thread per output reads
// two 2-element row pairs (4 B each in bf16) and writes the max + its code; backward writes the
// 2x2 window from dy and the code.  Tie / NaN semantics match PyTorch (first max in row-major
// window order; a NaN wins).
#include "bn_fin.h"
#include "common.h"
#include "ewdml_ops.h"

namespace {

template <typename T>
struct Pair;  // two consecutive elements loaded/stored as one word
template <>
struct Pair<uint16_t> {  // bf16
  using W = uint32_t;
  static __device__ __forceinline__ void split(W w, float& a, float& b) {
    a = __uint_as_float((w & 0xffffu) << 16);
    b = __uint_as_float(w & 0xffff0000u);
  }
  static __device__ __forceinline__ W join(float a, float b) {
    return (uint32_t)ew_f2bf(a) | ((uint32_t)ew_f2bf(b) << 16);
  }
  static __device__ __forceinline__ float one(uint16_t v) { return __uint_as_float((uint32_t)v << 16); }
  static __device__ __forceinline__ uint16_t make(float v) { return ew_f2bf(v); }
};
template <>
struct Pair<float> {
  using W = float2;
  static __device__ __forceinline__ void split(W w, float& a, float& b) { a = w.x; b = w.y; }
  static __device__ __forceinline__ W join(float a, float b) { return make_float2(a, b); }
  static __device__ __forceinline__ float one(float v) { return v; }
  static __device__ __forceinline__ float make(float v) { return v; }
};

template <typename T>
__global__ __launch_bounds__(EW_BLOCK) void k_maxpool2_fwd(const T* __restrict__ x,
                                                           T* __restrict__ y,
                                                           uint8_t* __restrict__ code,
                                                           long long total, int Wo, int W) {
  using P = Pair<T>;
  using Wd = typename P::W;
  for (long long o = blockIdx.x * (long long)EW_BLOCK + threadIdx.x; o < total;
       o += (long long)gridDim.x * EW_BLOCK) {
    const long long r = o / Wo;  // output row index over (n, c, ho)
    const int j = (int)(o - r * Wo);
    const long long base = (2 * r) * W + 2 * j;  // input (n, c, 2*ho, 2*j)
    float v[4];
    P::split(*reinterpret_cast<const Wd*>(x + base), v[0], v[1]);
    P::split(*reinterpret_cast<const Wd*>(x + base + W), v[2], v[3]);
    float m = v[0];
    int k = 0;
#pragma unroll
    for (int q = 1; q < 4; ++q) {
      if (v[q] > m || isnan(v[q])) {
        m = v[q];
        k = q;
      }
    }
    y[o] = P::make(m);
    code[o] = (uint8_t)k;
  }
}

template <typename T>
__global__ __launch_bounds__(EW_BLOCK) void k_maxpool2_bwd(const T* __restrict__ dy,
                                                           const uint8_t* __restrict__ code,
                                                           T* __restrict__ dx, long long total,
                                                           int Wo, int W) {
  using P = Pair<T>;
  using Wd = typename P::W;
  for (long long o = blockIdx.x * (long long)EW_BLOCK + threadIdx.x; o < total;
       o += (long long)gridDim.x * EW_BLOCK) {
    const long long r = o / Wo;
    const int j = (int)(o - r * Wo);
    const long long base = (2 * r) * W + 2 * j;
    const float g = P::one(dy[o]);
    const int k = code[o];
    *reinterpret_cast<Wd*>(dx + base) = P::join(k == 0 ? g : 0.0f, k == 1 ? g : 0.0f);
    *reinterpret_cast<Wd*>(dx + base + W) = P::join(k == 2 ? g : 0.0f, k == 3 ? g : 0.0f);
  }
}


// ================================================================================================
// NHWC (channels_last) BatchNorm(train/eval) + ReLU [+ MaxPool 2x2] for conv outputs.
//
// The activation is a row-major [M, C] matrix (M = N*H*W, C % 8 == 0).  A thread owns 8 channels
// (one 16-byte bf16 vector) of a row; tpr = C/8 threads cover a row, rpi = 256/tpr rows are in
// flight per block.  Per layer and direction three kernels run:
//   stats   : per-block partial sums (fp32 per thread, fixed-order LDS combine) -> part[s][blk][C]
//   finalize: one wave per channel sums the block partials in double in a fixed shuffle order
//             (deterministic), then writes the per-channel coefficients (+ running stats / dgamma,
//             dbeta, dbias)
//   apply   : elementwise, coefficients staged in LDS
// The conv bias preceding the BN is folded in: it cancels in training-mode normalisation, so it
// only enters the running mean (and eval-mode shift); its gradient is sum(dx), computed
// analytically from the backward sums.  The ReLU mask is recomputed in backward from the saved
// conv output with the forward's exact fp32 arithmetic (-ffp-contract=off), so y is never saved.
// With POOL the 2x2/2 max pool consumes the ReLU output inside the apply kernel (pre-pool
// activation never written) and backward routes dy through the 1-byte window code.
//
// stats layout [4][C] fp32: mean, invstd, scale = gamma*invstd, shift = beta - mean*scale.
// coef  layout [2][C] fp32 (backward): e = -scale*invstd*dgamma/M, f = -scale*dbeta/M,
//   dx = scale*dz + e*(h - mean) + f.
// ================================================================================================

template <typename T>
struct V8;
template <>
struct V8<uint16_t> {
  static __device__ __forceinline__ void ld(const uint16_t* p, float v[8]) {
    const uint4 w = *reinterpret_cast<const uint4*>(p);
    const uint32_t a[4] = {w.x, w.y, w.z, w.w};
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      v[2 * j] = __uint_as_float(a[j] << 16);
      v[2 * j + 1] = __uint_as_float(a[j] & 0xffff0000u);
    }
  }
  static __device__ __forceinline__ void st(uint16_t* p, const float v[8]) {
    uint4 w;
    w.x = (uint32_t)ew_f2bf(v[0]) | ((uint32_t)ew_f2bf(v[1]) << 16);
    w.y = (uint32_t)ew_f2bf(v[2]) | ((uint32_t)ew_f2bf(v[3]) << 16);
    w.z = (uint32_t)ew_f2bf(v[4]) | ((uint32_t)ew_f2bf(v[5]) << 16);
    w.w = (uint32_t)ew_f2bf(v[6]) | ((uint32_t)ew_f2bf(v[7]) << 16);
    *reinterpret_cast<uint4*>(p) = w;
  }
  static __device__ __forceinline__ float rnd(float v) {
    return __uint_as_float((uint32_t)ew_f2bf(v) << 16);
  }
};
template <>
struct V8<float> {
  static __device__ __forceinline__ void ld(const float* p, float v[8]) {
    const float4 a = *reinterpret_cast<const float4*>(p);
    const float4 b = *reinterpret_cast<const float4*>(p + 4);
    v[0] = a.x; v[1] = a.y; v[2] = a.z; v[3] = a.w;
    v[4] = b.x; v[5] = b.y; v[6] = b.z; v[7] = b.w;
  }
  static __device__ __forceinline__ void st(float* p, const float v[8]) {
    *reinterpret_cast<float4*>(p) = make_float4(v[0], v[1], v[2], v[3]);
    *reinterpret_cast<float4*>(p + 4) = make_float4(v[4], v[5], v[6], v[7]);
  }
  static __device__ __forceinline__ float rnd(float v) { return v; }
};

// 8 consecutive per-channel coefficients from LDS (p 32-B aligned: c0 % 8 == 0) as two b128 reads.
// Lanes hold c0 = 8 * lane: eight scalar reads put 8 lanes on each bank (8-way conflicts: the
// apply kernels ran ~20 conflict cycles per LDS instruction); a b128 read serves 8 lanes per pass
// over 64 distinct banks.
__device__ __forceinline__ void ew_lds8(const float* p, float v[8]) {
  const float4 a = *reinterpret_cast<const float4*>(p);
  const float4 b = *reinterpret_cast<const float4*>(p + 4);
  v[0] = a.x; v[1] = a.y; v[2] = a.z; v[3] = a.w;
  v[4] = b.x; v[5] = b.y; v[6] = b.z; v[7] = b.w;
}

__device__ __forceinline__ float ew_relu(float v) { return (v > 0.0f || v != v) ? v : 0.0f; }
__device__ __forceinline__ bool ew_relu_pass(float v) { return !(v <= 0.0f); }  // NaN passes

__device__ __forceinline__ void ew_ld_code8(const uint8_t* p, uint8_t c[8]) {
  const uint2 w = *reinterpret_cast<const uint2*>(p);
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    c[j] = (uint8_t)(w.x >> (8 * j));
    c[4 + j] = (uint8_t)(w.y >> (8 * j));
  }
}

// first input row (window position 0) of pooled row p; positions 1, 2, 3 are +1, +W, +W+1.
// 32-bit index math (the host guarantees rows * C < 2^31): 64-bit division is emulated.
__device__ __forceinline__ uint32_t ew_pool_base(uint32_t p, uint32_t HoWo, uint32_t Wo) {
  const uint32_t n = p / HoWo;
  const uint32_t rem = p - n * HoWo;
  const uint32_t ho = rem / Wo, wo = rem - ho * Wo;
  // input row = ((n * H) + 2 ho) * W + 2 wo with H = 2 Ho, W = 2 Wo; n * H * W = 4 n HoWo
  return 4 * n * HoWo + 4 * ho * Wo + 2 * wo;
}
__device__ __forceinline__ uint32_t ew_pool_off(int q, uint32_t Wo) {
  return (q >> 1) * (2 * Wo) + (q & 1);
}

// ---- forward statistics: sum(h), sum(h^2) per channel ----
template <typename T>
__global__ __launch_bounds__(EW_BLOCK) void k_bn_fwd_stats(const T* __restrict__ h, long long M,
                                                           int C, int rows_per_blk,
                                                           float* __restrict__ part) {
  __shared__ float ls[2048], lq[2048];
  const int tpr = C >> 3, rpi = EW_BLOCK / tpr;
  const int t = threadIdx.x, g = t % tpr, r = t / tpr;
  const long long row0 = (long long)blockIdx.x * rows_per_blk;
  const long long row1 = min(row0 + rows_per_blk, M);
  float s[8], q[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) s[j] = q[j] = 0.0f;
  if (r < rpi) {
    const T* hp = h + g * 8;
    long long row = row0 + r;
    for (; row + 3 * rpi < row1; row += 4 * rpi) {  // 4 independent loads in flight
      float v[4][8];
#pragma unroll
      for (int u = 0; u < 4; ++u) V8<T>::ld(hp + (row + u * rpi) * C, v[u]);
#pragma unroll
      for (int u = 0; u < 4; ++u) {
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          s[j] += v[u][j];
          q[j] += v[u][j] * v[u][j];
        }
      }
    }
    for (; row < row1; row += rpi) {
      float v[8];
      V8<T>::ld(hp + row * C, v);
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        s[j] += v[j];
        q[j] += v[j] * v[j];
      }
    }
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      ls[r * C + g * 8 + j] = s[j];
      lq[r * C + g * 8 + j] = q[j];
    }
  }
  __syncthreads();
  const long long nb = gridDim.x;
  for (int c = t; c < C; c += EW_BLOCK) {
    float a = 0.0f, b = 0.0f;
    for (int i = 0; i < rpi; ++i) {
      a += ls[i * C + c];
      b += lq[i * C + c];
    }
    part[(long long)blockIdx.x * C + c] = a;
    part[(nb + blockIdx.x) * C + c] = b;
  }
}

__device__ __forceinline__ double ew_wave_sum_d(double v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

// TH threads: 1024 (64 row slices) for the long partial lists of the large maps (1024 rows at
// VGG's 32x32 layers: one batch of loads per thread instead of four)
template <int TH>
__global__ __launch_bounds__(TH) void k_bn_fwd_finalize(
    const float* __restrict__ part, int nblk, int C, long long M, const float* __restrict__ gamma,
    const float* __restrict__ beta, const void* __restrict__ cbias, int cb_bf16,
    float* __restrict__ rmean, float* __restrict__ rvar, const long long* __restrict__ nbt,
    float momentum, float eps, float* __restrict__ stats) {
  const int c = blockIdx.x * EW_FIN_CH + (threadIdx.x % EW_FIN_CH);
  // the per-channel operands of the tail, loaded before the partial rows (their round trips
  // overlap the sums' instead of following them: a finalize is a short chain of L2 round trips)
  const int cc = c < C ? c : C - 1;
  const float g = gamma ? gamma[cc] : 1.0f;
  const float bb = beta ? beta[cc] : 0.0f;
  float rm0 = 0.0f, rv0 = 0.0f, cb = 0.0f;
  long long nb0 = 0;
  if (rmean) {
    rm0 = rmean[cc];
    rv0 = rvar[cc];
    if (momentum < 0.0f) nb0 = *nbt;
    if (cbias)
      cb = cb_bf16 ? ew_bf16f(reinterpret_cast<const uint16_t*>(cbias)[cc])
                   : reinterpret_cast<const float*>(cbias)[cc];
  }
  __shared__ double red[2 * (TH / 64) * EW_FIN_CH];
  double sums[2];
  if (!ew_sum_parts<2, 16, TH>(part, nblk, C, c, sums, red)) return;
  const double mean = sums[0] / (double)M;
  double var = sums[1] / (double)M - mean * mean;
  if (var < 0.0) var = 0.0;
  const float invstd = (float)(1.0 / sqrt(var + (double)eps));
  const float mf = (float)mean;
  const float scale = g * invstd;
  stats[c] = mf;
  stats[C + c] = invstd;
  stats[2 * C + c] = scale;
  stats[3 * C + c] = bb - mf * scale;
  if (rmean) {
    // momentum < 0: cumulative moving average (nn.BatchNorm2d(momentum=None)) over the batches
    // seen including this one; num_batches_tracked itself is incremented by the apply kernel
    const float f = momentum >= 0.0f ? momentum : 1.0f / (float)(nb0 + 1);
    const double unb = M > 1 ? var * (double)M / (double)(M - 1) : var;
    const float bm = mf + cb;
    rmean[c] = (1.0f - f) * rm0 + f * bm;
    rvar[c] = (1.0f - f) * rv0 + f * (float)unb;
  }
}

// ---- forward apply: y = act(h*scale + shift [+ res]) [-> 2x2 max pool + code] ----
enum { EW_BN_RELU = 0, EW_BN_RELU_POOL = 1, EW_BN_NONE = 2, EW_BN_ADD_RELU = 3 };

template <int MODE>
__device__ __forceinline__ float ew_act(float v) {
  if constexpr (MODE == EW_BN_NONE) return v;
  else return ew_relu(v);
}
template <int MODE>
__device__ __forceinline__ bool ew_act_pass(float v) {
  if constexpr (MODE == EW_BN_NONE) return true;
  else return ew_relu_pass(v);
}

template <typename T, int MODE, bool REGS = false>
__global__ __launch_bounds__(EW_BLOCK) void k_bn_fwd_apply(const T* __restrict__ h,
                                                           const T* __restrict__ res,
                                                           T* __restrict__ y,
                                                           uint8_t* __restrict__ code,
                                                           const float* __restrict__ stats,
                                                           long long rows, int C, int Ho, int Wo,
                                                           long long* __restrict__ nbt) {
  extern __shared__ float ew_dyn_lds[];  // 2*C floats (sized at launch: occupancy)
  float* lsc = ew_dyn_lds;
  float* lsh = ew_dyn_lds + C;
  if (nbt && blockIdx.x == 0 && threadIdx.x == 0) *nbt += 1;  // after the finalize read it
  const uint32_t tpr = C >> 3, HoWo = (uint32_t)Ho * Wo;
  const uint32_t nvec = (uint32_t)rows * tpr;
  // C / 8 dividing the block (every power-of-two C <= 2048): the grid stride is a multiple of
  // C / 8, so a thread keeps one 8-channel group -- its coefficients in registers, loaded once
  // (the LDS copy read per vector had 2-way bank conflicts on every read)
  const bool fixed = REGS && EW_BLOCK % tpr == 0;
  float rsc[8], rsh[8];
  if (fixed) {
    const int c0 = (int)(threadIdx.x % tpr) * 8;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      rsc[j] = stats[2 * C + c0 + j];
      rsh[j] = stats[3 * C + c0 + j];
    }
  } else {
    for (int c = threadIdx.x; c < C; c += EW_BLOCK) {
      lsc[c] = stats[2 * C + c];
      lsh[c] = stats[3 * C + c];
    }
    __syncthreads();
  }
  for (uint32_t v = blockIdx.x * EW_BLOCK + threadIdx.x; v < nvec; v += gridDim.x * EW_BLOCK) {
    const uint32_t row = v / tpr;
    const int c0 = (int)(v - row * tpr) * 8;
    float sc[8], sh[8];
    if (fixed) {
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        sc[j] = rsc[j];
        sh[j] = rsh[j];
      }
    } else {
      ew_lds8(lsc + c0, sc);
      ew_lds8(lsh + c0, sh);
    }
    if constexpr (MODE != EW_BN_RELU_POOL) {
      float x[8];
      V8<T>::ld(h + (long long)row * C + c0, x);
      if constexpr (MODE == EW_BN_ADD_RELU) {
        float r[8];
        V8<T>::ld(res + (long long)row * C + c0, r);
#pragma unroll
        for (int j = 0; j < 8; ++j) x[j] = ew_relu(x[j] * sc[j] + sh[j] + r[j]);
      } else {
#pragma unroll
        for (int j = 0; j < 8; ++j) x[j] = ew_act<MODE>(x[j] * sc[j] + sh[j]);
      }
      V8<T>::st(y + (long long)row * C + c0, x);
    } else {
      float m[8];
      uint32_t k[8];
      const uint32_t base = ew_pool_base(row, HoWo, Wo);
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        float x[8];
        V8<T>::ld(h + (long long)(base + ew_pool_off(q, Wo)) * C + c0, x);
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const float yv = V8<T>::rnd(ew_relu(x[j] * sc[j] + sh[j]));
          if (q == 0 || yv > m[j] || yv != yv) {
            m[j] = yv;
            k[j] = q;
          }
        }
      }
      V8<T>::st(y + (long long)row * C + c0, m);
      uint2 w;
      w.x = k[0] | (k[1] << 8) | (k[2] << 16) | (k[3] << 24);
      w.y = k[4] | (k[5] << 8) | (k[6] << 16) | (k[7] << 24);
      *reinterpret_cast<uint2*>(code + (long long)row * C + c0) = w;
    }
  }
}

// ---- backward statistics: sum(dz), sum(dz*(h-mean)), sum(h-mean), dz = act'(v) * dy ----
template <typename T, int MODE>
__global__ __launch_bounds__(EW_BLOCK) void k_bn_bwd_stats(
    const T* __restrict__ h, const T* __restrict__ res, const T* __restrict__ dy,
    const uint8_t* __restrict__ code,
    const float* __restrict__ stats, long long rows, int C, int Ho, int Wo, int rows_per_blk,
    float* __restrict__ part) {
  __shared__ float l1[2048], l2[2048], l3[2048];
  const int tpr = C >> 3, rpi = EW_BLOCK / tpr;
  const int t = threadIdx.x, g = t % tpr, r = t / tpr;
  const long long row0 = (long long)blockIdx.x * rows_per_blk;
  const long long row1 = min(row0 + rows_per_blk, rows);
  float s1[8], s2[8], s3[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) s1[j] = s2[j] = s3[j] = 0.0f;
  if (r < rpi) {
    const int c0 = g * 8;
    float mean[8], sc[8], sh[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      mean[j] = stats[c0 + j];
      sc[j] = stats[2 * C + c0 + j];
      sh[j] = stats[3 * C + c0 + j];
    }
    long long row = row0 + r;
    if constexpr (MODE != EW_BN_RELU_POOL) {  // 2 rows per iteration: 4-6 loads in flight
      for (; row + rpi < row1; row += 2 * rpi) {
        float d2[2][8], x2[2][8], r2[2][8];
#pragma unroll
        for (int u = 0; u < 2; ++u) {
          const long long o = (row + u * rpi) * C + c0;
          V8<T>::ld(dy + o, d2[u]);
          V8<T>::ld(h + o, x2[u]);
          if constexpr (MODE == EW_BN_ADD_RELU) V8<T>::ld(res + o, r2[u]);
        }
#pragma unroll
        for (int u = 0; u < 2; ++u) {
#pragma unroll
          for (int j = 0; j < 8; ++j) {
            float v = x2[u][j] * sc[j] + sh[j];
            if constexpr (MODE == EW_BN_ADD_RELU) v = v + r2[u][j];
            const float dz = ew_act_pass<MODE>(v) ? d2[u][j] : 0.0f;
            const float xc = x2[u][j] - mean[j];
            s1[j] += dz;
            s2[j] += dz * xc;
            s3[j] += xc;
          }
        }
      }
    }
    for (; row < row1; row += rpi) {
      float d[8];
      V8<T>::ld(dy + row * C + c0, d);
      if constexpr (MODE != EW_BN_RELU_POOL) {
        float x[8], rr[8];
        V8<T>::ld(h + row * C + c0, x);
        if constexpr (MODE == EW_BN_ADD_RELU) V8<T>::ld(res + row * C + c0, rr);
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          float v = x[j] * sc[j] + sh[j];
          if constexpr (MODE == EW_BN_ADD_RELU) v = v + rr[j];
          const float dz = ew_act_pass<MODE>(v) ? d[j] : 0.0f;
          const float xc = x[j] - mean[j];
          s1[j] += dz;
          s2[j] += dz * xc;
          s3[j] += xc;
        }
      } else {
        uint8_t k[8];
        ew_ld_code8(code + row * C + c0, k);
        const uint32_t base = ew_pool_base((uint32_t)row, (uint32_t)Ho * Wo, Wo);
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          float x[8];
          V8<T>::ld(h + (long long)(base + ew_pool_off(q, Wo)) * C + c0, x);
#pragma unroll
          for (int j = 0; j < 8; ++j) {
            const float dz = (k[j] == q && ew_relu_pass(x[j] * sc[j] + sh[j])) ? d[j] : 0.0f;
            const float xc = x[j] - mean[j];
            s1[j] += dz;
            s2[j] += dz * xc;
            s3[j] += xc;
          }
        }
      }
    }
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      l1[r * C + c0 + j] = s1[j];
      l2[r * C + c0 + j] = s2[j];
      l3[r * C + c0 + j] = s3[j];
    }
  }
  __syncthreads();
  const long long nb = gridDim.x;
  for (int c = t; c < C; c += EW_BLOCK) {
    float a = 0.0f, b = 0.0f, e = 0.0f;
    for (int i = 0; i < rpi; ++i) {
      a += l1[i * C + c];
      b += l2[i * C + c];
      e += l3[i * C + c];
    }
    part[(long long)blockIdx.x * C + c] = a;
    part[(nb + blockIdx.x) * C + c] = b;
    part[(2 * nb + blockIdx.x) * C + c] = e;
  }
}

// NS = 3: partials of k_bn_bwd_stats; NS = 2: of a backward-data conv epilogue (bn_fin.h)
template <int NS>
__global__ __launch_bounds__(EW_BLOCK) void k_bn_bwd_finalize(EwBnFin f) {
  __shared__ double red[NS * EW_WAVES * EW_FIN_CH];
  ew_bn_bwd_fin_group<NS>(f, blockIdx.x, red);
}

template <typename T, int MODE, bool REGS = false>
__global__ __launch_bounds__(EW_BLOCK) void k_bn_bwd_apply(
    const T* __restrict__ h, const T* __restrict__ res, const T* __restrict__ dy,
    const uint8_t* __restrict__ code, const float* __restrict__ stats,
    const float* __restrict__ coef, T* __restrict__ dx, T* __restrict__ dres, long long rows,
    int C, int Ho, int Wo) {
  extern __shared__ float ew_dyn_lds[];  // 5*C floats
  float* lm = ew_dyn_lds;
  float* lsc = lm + C;
  float* lsh = lsc + C;
  float* le = lsh + C;
  float* lf = le + C;
  const uint32_t tpr = C >> 3, HoWo = (uint32_t)Ho * Wo;
  const uint32_t nvec = (uint32_t)rows * tpr;
  // a thread keeps one 8-channel group when C / 8 divides the block (k_bn_fwd_apply): its five
  // coefficient vectors in registers instead of ten conflicting LDS reads per vector
  const bool fixed = REGS && EW_BLOCK % tpr == 0;
  float rmn[8], rsc[8], rsh[8], rce[8], rcf[8];
  if (fixed) {
    const int c0 = (int)(threadIdx.x % tpr) * 8;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      rmn[j] = stats[c0 + j];
      rsc[j] = stats[2 * C + c0 + j];
      rsh[j] = stats[3 * C + c0 + j];
      rce[j] = coef[c0 + j];
      rcf[j] = coef[C + c0 + j];
    }
  } else {
    for (int c = threadIdx.x; c < C; c += EW_BLOCK) {
      lm[c] = stats[c];
      lsc[c] = stats[2 * C + c];
      lsh[c] = stats[3 * C + c];
      le[c] = coef[c];
      lf[c] = coef[C + c];
    }
    __syncthreads();
  }
  for (uint32_t v = blockIdx.x * EW_BLOCK + threadIdx.x; v < nvec; v += gridDim.x * EW_BLOCK) {
    const uint32_t row = v / tpr;
    const int c0 = (int)(v - row * tpr) * 8;
    float d[8];
    V8<T>::ld(dy + (long long)row * C + c0, d);
    float mn[8], sc[8], sh[8], ce[8], cf[8];
    if (fixed) {
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        mn[j] = rmn[j];
        sc[j] = rsc[j];
        sh[j] = rsh[j];
        ce[j] = rce[j];
        cf[j] = rcf[j];
      }
    } else {
      ew_lds8(lm + c0, mn);
      ew_lds8(lsc + c0, sc);
      ew_lds8(lsh + c0, sh);
      ew_lds8(le + c0, ce);
      ew_lds8(lf + c0, cf);
    }
    if constexpr (MODE != EW_BN_RELU_POOL) {
      float x[8], o[8], rr[8], dzs[8];
      V8<T>::ld(h + (long long)row * C + c0, x);
      if constexpr (MODE == EW_BN_ADD_RELU) V8<T>::ld(res + (long long)row * C + c0, rr);
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        float vv = x[j] * sc[j] + sh[j];
        if constexpr (MODE == EW_BN_ADD_RELU) vv = vv + rr[j];
        const float dz = ew_act_pass<MODE>(vv) ? d[j] : 0.0f;
        dzs[j] = dz;
        o[j] = sc[j] * dz + ce[j] * (x[j] - mn[j]) + cf[j];
      }
      V8<T>::st(dx + (long long)row * C + c0, o);
      if constexpr (MODE == EW_BN_ADD_RELU) V8<T>::st(dres + (long long)row * C + c0, dzs);
    } else {
      uint8_t k[8];
      ew_ld_code8(code + (long long)row * C + c0, k);
      const uint32_t base = ew_pool_base(row, HoWo, Wo);
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const long long ir = base + ew_pool_off(q, Wo);
        float x[8], o[8];
        V8<T>::ld(h + ir * C + c0, x);
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const float dz = (k[j] == q && ew_relu_pass(x[j] * sc[j] + sh[j])) ? d[j] : 0.0f;
          o[j] = sc[j] * dz + ce[j] * (x[j] - mn[j]) + cf[j];
        }
        V8<T>::st(dx + ir * C + c0, o);
      }
    }
  }
}

// ---- standalone NHWC 2x2 max pool (no BN in front) ----
template <typename T>
__global__ __launch_bounds__(EW_BLOCK) void k_maxpool2_nhwc_fwd(const T* __restrict__ x,
                                                                T* __restrict__ y,
                                                                uint8_t* __restrict__ code,
                                                                long long rows, int C, int Ho,
                                                                int Wo) {
  const uint32_t tpr = C >> 3, HoWo = (uint32_t)Ho * Wo;
  const uint32_t nvec = (uint32_t)rows * tpr;
  for (uint32_t v = blockIdx.x * EW_BLOCK + threadIdx.x; v < nvec; v += gridDim.x * EW_BLOCK) {
    const uint32_t row = v / tpr;
    const int c0 = (int)(v - row * tpr) * 8;
    float m[8];
    uint32_t k[8];
    const uint32_t base = ew_pool_base(row, HoWo, Wo);
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      float a[8];
      V8<T>::ld(x + (long long)(base + ew_pool_off(q, Wo)) * C + c0, a);
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        if (q == 0 || a[j] > m[j] || a[j] != a[j]) {
          m[j] = a[j];
          k[j] = q;
        }
      }
    }
    V8<T>::st(y + (long long)row * C + c0, m);
    uint2 w;
    w.x = k[0] | (k[1] << 8) | (k[2] << 16) | (k[3] << 24);
    w.y = k[4] | (k[5] << 8) | (k[6] << 16) | (k[7] << 24);
    *reinterpret_cast<uint2*>(code + (long long)row * C + c0) = w;
  }
}

template <typename T>
__global__ __launch_bounds__(EW_BLOCK) void k_maxpool2_nhwc_bwd(const T* __restrict__ dy,
                                                                const uint8_t* __restrict__ code,
                                                                T* __restrict__ dx,
                                                                long long rows, int C, int Ho,
                                                                int Wo) {
  const uint32_t tpr = C >> 3, HoWo = (uint32_t)Ho * Wo;
  const uint32_t nvec = (uint32_t)rows * tpr;
  for (uint32_t v = blockIdx.x * EW_BLOCK + threadIdx.x; v < nvec; v += gridDim.x * EW_BLOCK) {
    const uint32_t row = v / tpr;
    const int c0 = (int)(v - row * tpr) * 8;
    float d[8];
    uint8_t k[8];
    V8<T>::ld(dy + (long long)row * C + c0, d);
    ew_ld_code8(code + (long long)row * C + c0, k);
    const uint32_t base = ew_pool_base(row, HoWo, Wo);
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      float o[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) o[j] = k[j] == q ? d[j] : 0.0f;
      V8<T>::st(dx + (long long)(base + ew_pool_off(q, Wo)) * C + c0, o);
    }
  }
}

// ---- standalone NHWC 3x3 / stride 2 / pad 1 max pool (the ImageNet ResNet stem) ----
// Forward: thread = (output pixel, 8 channels); the window's taps in (kh, kw) order, padding as
// -inf, a tap wins on > or NaN (F.max_pool2d's rule); the winning tap 0..8 is the 1-byte code.
// Backward as a gather (no atomics, deterministic): thread = (input pixel, 8 channels), summing in
// (oh, ow) order the dy of the (at most 2 x 2) windows whose code points at this pixel.
template <typename T>
__global__ __launch_bounds__(EW_BLOCK) void k_maxpool3s2_nhwc_fwd(const T* __restrict__ x,
                                                                  T* __restrict__ y,
                                                                  uint8_t* __restrict__ code,
                                                                  long long rows, int C, int H,
                                                                  int W, int Ho, int Wo) {
  const uint32_t tpr = C >> 3, HoWo = (uint32_t)Ho * Wo;
  const uint32_t nvec = (uint32_t)rows * tpr;
  for (uint32_t v = blockIdx.x * EW_BLOCK + threadIdx.x; v < nvec; v += gridDim.x * EW_BLOCK) {
    const uint32_t row = v / tpr;
    const int c0 = (int)(v - row * tpr) * 8;
    const uint32_t n = row / HoWo, rem = row - n * HoWo;
    const int oh = (int)(rem / (uint32_t)Wo), ow = (int)(rem - (uint32_t)oh * Wo);
    float m[8];
    uint32_t k[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      m[j] = -INFINITY;
      k[j] = 0;
    }
#pragma unroll
    for (int q = 0; q < 9; ++q) {
      const int h = 2 * oh - 1 + q / 3, w = 2 * ow - 1 + q % 3;
      if ((unsigned)h >= (unsigned)H || (unsigned)w >= (unsigned)W) continue;
      float a[8];
      V8<T>::ld(x + (((long long)n * H + h) * W + w) * C + c0, a);
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        if (a[j] > m[j] || a[j] != a[j]) {
          m[j] = a[j];
          k[j] = q;
        }
      }
    }
    V8<T>::st(y + (long long)row * C + c0, m);
    uint2 cw;
    cw.x = k[0] | (k[1] << 8) | (k[2] << 16) | (k[3] << 24);
    cw.y = k[4] | (k[5] << 8) | (k[6] << 16) | (k[7] << 24);
    *reinterpret_cast<uint2*>(code + (long long)row * C + c0) = cw;
  }
}

template <typename T>
__global__ __launch_bounds__(EW_BLOCK) void k_maxpool3s2_nhwc_bwd(const T* __restrict__ dy,
                                                                  const uint8_t* __restrict__ code,
                                                                  T* __restrict__ dx,
                                                                  long long rows, int C, int H,
                                                                  int W, int Ho, int Wo) {
  const uint32_t tpr = C >> 3, HW = (uint32_t)H * W;
  const uint32_t nvec = (uint32_t)rows * tpr;  // rows = N H W input pixels
  for (uint32_t v = blockIdx.x * EW_BLOCK + threadIdx.x; v < nvec; v += gridDim.x * EW_BLOCK) {
    const uint32_t row = v / tpr;
    const int c0 = (int)(v - row * tpr) * 8;
    const uint32_t n = row / HW, rem = row - n * HW;
    const int h = (int)(rem / (uint32_t)W), w = (int)(rem - (uint32_t)h * W);
    // windows oh with 2 oh - 1 <= h <= 2 oh + 1
    const int oh0 = h >> 1, oh1 = (h + 1) >> 1, ow0 = w >> 1, ow1 = (w + 1) >> 1;
    float o[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) o[j] = 0.0f;
#pragma unroll
    for (int a = 0; a < 2; ++a) {
      const int oh = a ? oh1 : oh0;
      if ((a && oh1 == oh0) || oh >= Ho) continue;
#pragma unroll
      for (int b = 0; b < 2; ++b) {
        const int ow = b ? ow1 : ow0;
        if ((b && ow1 == ow0) || ow >= Wo) continue;
        const uint32_t q = (uint32_t)((h - 2 * oh + 1) * 3 + (w - 2 * ow + 1));
        const long long r = ((long long)n * Ho + oh) * Wo + ow;
        float d[8];
        uint8_t kc[8];
        V8<T>::ld(dy + r * C + c0, d);
        ew_ld_code8(code + r * C + c0, kc);
#pragma unroll
        for (int j = 0; j < 8; ++j)
          if (kc[j] == q) o[j] += d[j];
      }
    }
    V8<T>::st(dx + (long long)row * C + c0, o);
  }
}

inline int ew_grid1(long long n) {
  long long b = (n + EW_BLOCK - 1) / EW_BLOCK;
  return (int)(b < 4096 ? (b > 0 ? b : 1) : 4096);
}

}  // namespace

void ew_maxpool2_fwd(uintptr_t x, uintptr_t y, uintptr_t code, long long rows, int W, int is_bf16,
                     uintptr_t stream) {
  // rows = N*C*H/2 output rows of Wo = W/2 outputs each
  const int Wo = W / 2;
  const long long total = rows * Wo;
  hipStream_t s = (hipStream_t)stream;
  if (is_bf16)
    hipLaunchKernelGGL(k_maxpool2_fwd<uint16_t>, dim3(ew_grid1(total)), dim3(EW_BLOCK), 0, s,
                       reinterpret_cast<const uint16_t*>(x), reinterpret_cast<uint16_t*>(y),
                       reinterpret_cast<uint8_t*>(code), total, Wo, W);
  else
    hipLaunchKernelGGL(k_maxpool2_fwd<float>, dim3(ew_grid1(total)), dim3(EW_BLOCK), 0, s,
                       reinterpret_cast<const float*>(x), reinterpret_cast<float*>(y),
                       reinterpret_cast<uint8_t*>(code), total, Wo, W);
  EW_CHECK_LAUNCH();
}

void ew_maxpool2_bwd(uintptr_t dy, uintptr_t code, uintptr_t dx, long long rows, int W,
                     int is_bf16, uintptr_t stream) {
  const int Wo = W / 2;
  const long long total = rows * Wo;
  hipStream_t s = (hipStream_t)stream;
  if (is_bf16)
    hipLaunchKernelGGL(k_maxpool2_bwd<uint16_t>, dim3(ew_grid1(total)), dim3(EW_BLOCK), 0, s,
                       reinterpret_cast<const uint16_t*>(dy), reinterpret_cast<const uint8_t*>(code),
                       reinterpret_cast<uint16_t*>(dx), total, Wo, W);
  else
    hipLaunchKernelGGL(k_maxpool2_bwd<float>, dim3(ew_grid1(total)), dim3(EW_BLOCK), 0, s,
                       reinterpret_cast<const float*>(dy), reinterpret_cast<const uint8_t*>(code),
                       reinterpret_cast<float*>(dx), total, Wo, W);
  EW_CHECK_LAUNCH();
}

// ---------------------------------------------------------------------------------------------
// host side of the NHWC BN kernels

// blocks / rows-per-block of a stats pass: per_thread row iterations per thread, <= 1024 blocks,
// nblk*C <= 256K partial floats per quantity (the workspace size the Python side allocates)
static void ew_bn_grid(long long rows, int C, int* nblk, int* rows_per_blk, int per_thread) {
  const int tpr = C / 8, rpi = EW_BLOCK / tpr;
  long long iters = (rows + rpi - 1) / rpi;
  long long nb = iters / per_thread;  // = the kernel's unroll: one unrolled iteration per thread
  long long cap = (1LL << 18) / C;
  if (cap > 1024) cap = 1024;
  if (nb > cap) nb = cap;
  if (nb < 1) nb = 1;
  long long rpb = (rows + nb - 1) / nb;
  rpb = (rpb + rpi - 1) / rpi * rpi;
  *rows_per_blk = (int)rpb;
  *nblk = (int)((rows + rpb - 1) / rpb);
}

int ew_bn_part_floats() { return 3 * (1 << 18); }

static int ew_grid_vec(long long nvec) {
  long long b = (nvec + EW_BLOCK - 1) / EW_BLOCK;
  const long long cap = 256LL * 16;  // 16 blocks per CU, grid-stride beyond
  return (int)(b < cap ? (b > 0 ? b : 1) : cap);
}


// The apply kernels keep each thread's channel coefficients in registers (k_bn_fwd_apply /
// k_bn_bwd_apply REGS) instead of reading the block's LDS copy (2-way bank conflicts) per vector:
// VGG-11 1.1454 -> 1.1410 ms, ResNet-50 CIFAR 13.16 -> 13.13 ms despite the lower occupancy
// (profiles/ab/README.md).  EWDML_BN_REGS=0: the LDS copy.
static bool ew_bn_regs() {
  static const bool on = [] {
    const char* e = getenv("EWDML_BN_REGS");
    return !(e && e[0] == '0');
  }();
  return on;
}

// EWDML_BN_FIN_WIDE=0: every forward finalize at EW_BLOCK threads (A/B)
static bool ew_fin_wide() {
  static const bool on = [] {
    const char* e = getenv("EWDML_BN_FIN_WIDE");
    return !(e && e[0] == '0');
  }();
  return on;
}

void ew_bn_relu_fwd(const BnFwdArgs& a) {
  hipStream_t s = (hipStream_t)a.stream;
  const long long M = a.N * (long long)a.H * a.W;
  const int Ho = a.H / 2, Wo = a.W / 2;
  const int C = a.C;
  if (a.training && a.phase != 2) {
    int nblk, rpb;
    ew_bn_grid(M, C, &nblk, &rpb, 4);
    float* part = reinterpret_cast<float*>(a.part);
    if (a.pre_nblk > 0)  // statistics computed by the producing conv's epilogue
      nblk = a.pre_nblk;
    else if (a.is_bf16)
      hipLaunchKernelGGL(k_bn_fwd_stats<uint16_t>, dim3(nblk), dim3(EW_BLOCK), 0, s,
                         reinterpret_cast<const uint16_t*>(a.h), M, C, rpb, part);
    else
      hipLaunchKernelGGL(k_bn_fwd_stats<float>, dim3(nblk), dim3(EW_BLOCK), 0, s,
                         reinterpret_cast<const float*>(a.h), M, C, rpb, part);
    EW_CHECK_LAUNCH();
#define EW_FF(TH)                                                                               \
  hipLaunchKernelGGL(k_bn_fwd_finalize<TH>, dim3((C + EW_FIN_CH - 1) / EW_FIN_CH), dim3(TH), 0, s, \
                     part, nblk, C, M, reinterpret_cast<const float*>(a.gamma),                    \
                     reinterpret_cast<const float*>(a.beta),                                       \
                     reinterpret_cast<const void*>(a.cbias), a.cb_bf16,                            \
                     reinterpret_cast<float*>(a.rmean), reinterpret_cast<float*>(a.rvar),          \
                     reinterpret_cast<const long long*>(a.nbt), a.momentum, a.eps,                 \
                     reinterpret_cast<float*>(a.stats))
    if (nblk > 256 && ew_fin_wide()) EW_FF(1024);
    else EW_FF(EW_BLOCK);
#undef EW_FF
    EW_CHECK_LAUNCH();
  }
  if (a.phase == 1) return;  // lazy: the consumer applies (winograd_f32.hip WgSrc KIND 1)
  const float* st = reinterpret_cast<const float*>(a.stats);
  uint8_t* code = reinterpret_cast<uint8_t*>(a.code);
  long long* nbt = a.training ? reinterpret_cast<long long*>(a.nbt) : nullptr;
  const size_t lds = 2 * sizeof(float) * C;
  const int mode = a.pool ? EW_BN_RELU_POOL : a.mode;
  const long long rows = a.pool ? a.N * (long long)Ho * Wo : M;
  const int grid = ew_grid_vec(rows * (C / 8));
#define EW_FA(T, MODE)                                                                          \
  if (ew_bn_regs())                                                                             \
    hipLaunchKernelGGL((k_bn_fwd_apply<T, MODE, true>), dim3(grid), dim3(EW_BLOCK), lds, s,     \
                       reinterpret_cast<const T*>(a.h), reinterpret_cast<const T*>(a.res),       \
                       reinterpret_cast<T*>(a.y), code, st, rows, C, Ho, Wo, nbt);              \
  else                                                                                          \
    hipLaunchKernelGGL((k_bn_fwd_apply<T, MODE>), dim3(grid), dim3(EW_BLOCK), lds, s,           \
                       reinterpret_cast<const T*>(a.h), reinterpret_cast<const T*>(a.res),       \
                       reinterpret_cast<T*>(a.y), code, st, rows, C, Ho, Wo, nbt)
#define EW_FA_MODES(T)                                                                          \
  switch (mode) {                                                                               \
    case EW_BN_RELU: EW_FA(T, EW_BN_RELU); break;                                               \
    case EW_BN_RELU_POOL: EW_FA(T, EW_BN_RELU_POOL); break;                                     \
    case EW_BN_NONE: EW_FA(T, EW_BN_NONE); break;                                               \
    default: EW_FA(T, EW_BN_ADD_RELU); break;                                                   \
  }
  if (a.is_bf16) {
    EW_FA_MODES(uint16_t)
  } else {
    EW_FA_MODES(float)
  }
#undef EW_FA_MODES
#undef EW_FA
  EW_CHECK_LAUNCH();
}

template <typename T, int MODE>
static void ew_bn_bwd_impl(const BnBwdArgs& a) {
  constexpr bool POOL = MODE == EW_BN_RELU_POOL;
  hipStream_t s = (hipStream_t)a.stream;
  const long long M = a.N * (long long)a.H * a.W;
  const int Ho = a.H / 2, Wo = a.W / 2;
  const int C = a.C;
  const long long rows = POOL ? a.N * (long long)Ho * Wo : M;
  int nblk, rpb;
  ew_bn_grid(rows, C, &nblk, &rpb, POOL ? 1 : 2);
  float* part = reinterpret_cast<float*>(a.part);
  const bool pre = a.pre_nblk > 0;  // sums from the producing conv (ops/csrc/conv.hip CvBnBwd)
  const T* h = reinterpret_cast<const T*>(a.h);
  const T* res = reinterpret_cast<const T*>(a.res);
  const T* dy = reinterpret_cast<const T*>(a.dy);
  const uint8_t* code = reinterpret_cast<const uint8_t*>(a.code);
  const float* st = reinterpret_cast<const float*>(a.stats);
  float* coef = reinterpret_cast<float*>(a.coef);
  EwBnFin fin{};
  fin.dgamma = reinterpret_cast<float*>(a.dgamma);
  fin.dbeta = reinterpret_cast<float*>(a.dbeta);
  fin.dcbias = reinterpret_cast<void*>(a.dcbias);
  fin.ngrp = (C + EW_FIN_CH - 1) / EW_FIN_CH;
  if (a.phase == 2) {
    // apply only (a lazy backward materialised after all): coef from the earlier phase-1 call
  } else if (pre) {
    hipLaunchKernelGGL(k_bn_bwd_finalize<2>, dim3(fin.ngrp), dim3(EW_BLOCK), 0, s,
                       EwBnFin{part, st, coef, fin.dgamma, fin.dbeta, fin.dcbias, M, (int)a.pre_nblk,
                               C, a.cb_bf16, fin.ngrp});
  } else {
    hipLaunchKernelGGL((k_bn_bwd_stats<T, MODE>), dim3(nblk), dim3(EW_BLOCK), 0, s, h, res, dy,
                       code, st, rows, C, Ho, Wo, rpb, part);
    EW_CHECK_LAUNCH();
    hipLaunchKernelGGL(k_bn_bwd_finalize<3>, dim3(fin.ngrp), dim3(EW_BLOCK), 0, s,
                       EwBnFin{part, st, coef, fin.dgamma, fin.dbeta, fin.dcbias, M, nblk, C,
                               a.cb_bf16, fin.ngrp});
  }
  EW_CHECK_LAUNCH();
  if (a.phase == 1) return;  // lazy: the producing conv's input transform forms dx (KIND 2)
  if (ew_bn_regs())
    hipLaunchKernelGGL((k_bn_bwd_apply<T, MODE, true>), dim3(ew_grid_vec(rows * (C / 8))),
                       dim3(EW_BLOCK), 5 * sizeof(float) * C, s, h, res, dy, code, st, coef,
                       reinterpret_cast<T*>(a.dx), reinterpret_cast<T*>(a.dres), rows, C, Ho, Wo);
  else
    hipLaunchKernelGGL((k_bn_bwd_apply<T, MODE>), dim3(ew_grid_vec(rows * (C / 8))),
                       dim3(EW_BLOCK), 5 * sizeof(float) * C, s, h, res, dy, code, st, coef,
                       reinterpret_cast<T*>(a.dx), reinterpret_cast<T*>(a.dres), rows, C, Ho, Wo);
  EW_CHECK_LAUNCH();
}

template <typename T>
static void ew_bn_bwd_modes(const BnBwdArgs& a) {
  switch (a.pool ? (int)EW_BN_RELU_POOL : a.mode) {
    case EW_BN_RELU: ew_bn_bwd_impl<T, EW_BN_RELU>(a); break;
    case EW_BN_RELU_POOL: ew_bn_bwd_impl<T, EW_BN_RELU_POOL>(a); break;
    case EW_BN_NONE: ew_bn_bwd_impl<T, EW_BN_NONE>(a); break;
    default: ew_bn_bwd_impl<T, EW_BN_ADD_RELU>(a); break;
  }
}

void ew_bn_relu_bwd(const BnBwdArgs& a) {
  if (a.is_bf16) ew_bn_bwd_modes<uint16_t>(a);
  else ew_bn_bwd_modes<float>(a);
}

void ew_maxpool2_nhwc(uintptr_t x, uintptr_t y, uintptr_t code, long long N, int H, int W, int C,
                      int is_bf16, int backward, uintptr_t stream) {
  hipStream_t s = (hipStream_t)stream;
  const int Ho = H / 2, Wo = W / 2;
  const long long rows = N * (long long)Ho * Wo;
  const int grid = ew_grid_vec(rows * (C / 8));
  uint8_t* cd = reinterpret_cast<uint8_t*>(code);
  if (!backward) {
    if (is_bf16)
      hipLaunchKernelGGL(k_maxpool2_nhwc_fwd<uint16_t>, dim3(grid), dim3(EW_BLOCK), 0, s,
                         reinterpret_cast<const uint16_t*>(x), reinterpret_cast<uint16_t*>(y), cd,
                         rows, C, Ho, Wo);
    else
      hipLaunchKernelGGL(k_maxpool2_nhwc_fwd<float>, dim3(grid), dim3(EW_BLOCK), 0, s,
                         reinterpret_cast<const float*>(x), reinterpret_cast<float*>(y), cd, rows,
                         C, Ho, Wo);
  } else {  // x = dy (pooled), y = dx (full)
    if (is_bf16)
      hipLaunchKernelGGL(k_maxpool2_nhwc_bwd<uint16_t>, dim3(grid), dim3(EW_BLOCK), 0, s,
                         reinterpret_cast<const uint16_t*>(x), cd, reinterpret_cast<uint16_t*>(y),
                         rows, C, Ho, Wo);
    else
      hipLaunchKernelGGL(k_maxpool2_nhwc_bwd<float>, dim3(grid), dim3(EW_BLOCK), 0, s,
                         reinterpret_cast<const float*>(x), cd, reinterpret_cast<float*>(y), rows,
                         C, Ho, Wo);
  }
  EW_CHECK_LAUNCH();
}

void ew_maxpool3s2_nhwc(uintptr_t x, uintptr_t y, uintptr_t code, long long N, int H, int W,
                        int C, int is_bf16, int backward, uintptr_t stream) {
  hipStream_t s = (hipStream_t)stream;
  const int Ho = (H - 1) / 2 + 1, Wo = (W - 1) / 2 + 1;  // kernel 3, stride 2, pad 1
  uint8_t* cd = reinterpret_cast<uint8_t*>(code);
  if (!backward) {
    const long long rows = N * (long long)Ho * Wo;
    const int grid = ew_grid_vec(rows * (C / 8));
    if (is_bf16)
      hipLaunchKernelGGL(k_maxpool3s2_nhwc_fwd<uint16_t>, dim3(grid), dim3(EW_BLOCK), 0, s,
                         reinterpret_cast<const uint16_t*>(x), reinterpret_cast<uint16_t*>(y), cd,
                         rows, C, H, W, Ho, Wo);
    else
      hipLaunchKernelGGL(k_maxpool3s2_nhwc_fwd<float>, dim3(grid), dim3(EW_BLOCK), 0, s,
                         reinterpret_cast<const float*>(x), reinterpret_cast<float*>(y), cd, rows,
                         C, H, W, Ho, Wo);
  } else {  // x = dy (pooled), y = dx (full)
    const long long rows = N * (long long)H * W;
    const int grid = ew_grid_vec(rows * (C / 8));
    if (is_bf16)
      hipLaunchKernelGGL(k_maxpool3s2_nhwc_bwd<uint16_t>, dim3(grid), dim3(EW_BLOCK), 0, s,
                         reinterpret_cast<const uint16_t*>(x), cd, reinterpret_cast<uint16_t*>(y),
                         rows, C, H, W, Ho, Wo);
    else
      hipLaunchKernelGGL(k_maxpool3s2_nhwc_bwd<float>, dim3(grid), dim3(EW_BLOCK), 0, s,
                         reinterpret_cast<const float*>(x), cd, reinterpret_cast<float*>(y), rows,
                         C, H, W, Ho, Wo);
  }
  EW_CHECK_LAUNCH();
}

// ---- global average pool over H x W (NHWC [N, HW, C] -> [N, C]; the ResNet head) ----
// Forward: one thread per (n, 8 channels), the HW rows summed in order in fp32, times 1 / HW.
// Backward: dx[n, hw, c] = dy[n, c] / HW, a vector store per (row, 8 channels).
template <typename T>
__global__ __launch_bounds__(EW_BLOCK) void k_gap_nhwc_fwd(const T* __restrict__ x,
                                                           T* __restrict__ y, int N, int HW, int C,
                                                           float inv) {
  const uint32_t tpr = C >> 3;
  const uint32_t v = blockIdx.x * EW_BLOCK + threadIdx.x;
  if (v >= (uint32_t)N * tpr) return;
  const uint32_t n = v / tpr;
  const int c0 = (int)(v - n * tpr) * 8;
  const T* src = x + (long long)n * HW * C + c0;
  float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  int r = 0;
  for (; r + 4 <= HW; r += 4) {  // 4 rows' loads in flight, added in row order
    float a[4][8];
#pragma unroll
    for (int u = 0; u < 4; ++u) V8<T>::ld(src + (long long)(r + u) * C, a[u]);
#pragma unroll
    for (int u = 0; u < 4; ++u)
#pragma unroll
      for (int j = 0; j < 8; ++j) acc[j] += a[u][j];
  }
  for (; r < HW; ++r) {
    float a[8];
    V8<T>::ld(src + (long long)r * C, a);
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[j] += a[j];
  }
#pragma unroll
  for (int j = 0; j < 8; ++j) acc[j] *= inv;
  V8<T>::st(y + (long long)n * C + c0, acc);
}

template <typename T>
__global__ __launch_bounds__(EW_BLOCK) void k_gap_nhwc_bwd(const T* __restrict__ dy,
                                                           T* __restrict__ dx, long long rows,
                                                           int HW, int C, float inv) {
  const uint32_t tpr = C >> 3;
  const uint32_t nvec = (uint32_t)rows * tpr;
  for (uint32_t v = blockIdx.x * EW_BLOCK + threadIdx.x; v < nvec; v += gridDim.x * EW_BLOCK) {
    const uint32_t row = v / tpr;
    const int c0 = (int)(v - row * tpr) * 8;
    float d[8];
    V8<T>::ld(dy + (long long)(row / HW) * C + c0, d);
#pragma unroll
    for (int j = 0; j < 8; ++j) d[j] *= inv;
    V8<T>::st(dx + (long long)row * C + c0, d);
  }
}

void ew_gap_nhwc(uintptr_t x, uintptr_t y, long long N, int HW, int C, int is_bf16, int backward,
                 uintptr_t stream) {
  hipStream_t s = (hipStream_t)stream;
  const float inv = 1.0f / (float)HW;
  if (!backward) {
    const int grid = (int)((N * (C / 8) + EW_BLOCK - 1) / EW_BLOCK);
    if (is_bf16)
      hipLaunchKernelGGL(k_gap_nhwc_fwd<uint16_t>, dim3(grid), dim3(EW_BLOCK), 0, s,
                         reinterpret_cast<const uint16_t*>(x), reinterpret_cast<uint16_t*>(y),
                         (int)N, HW, C, inv);
    else
      hipLaunchKernelGGL(k_gap_nhwc_fwd<float>, dim3(grid), dim3(EW_BLOCK), 0, s,
                         reinterpret_cast<const float*>(x), reinterpret_cast<float*>(y), (int)N,
                         HW, C, inv);
  } else {  // x = dy [N, C], y = dx [N, HW, C]
    const long long rows = N * HW;
    const int grid = ew_grid_vec(rows * (C / 8));
    if (is_bf16)
      hipLaunchKernelGGL(k_gap_nhwc_bwd<uint16_t>, dim3(grid), dim3(EW_BLOCK), 0, s,
                         reinterpret_cast<const uint16_t*>(x), reinterpret_cast<uint16_t*>(y), rows,
                         HW, C, inv);
    else
      hipLaunchKernelGGL(k_gap_nhwc_bwd<float>, dim3(grid), dim3(EW_BLOCK), 0, s,
                         reinterpret_cast<const float*>(x), reinterpret_cast<float*>(y), rows, HW,
                         C, inv);
  }
  EW_CHECK_LAUNCH();
}

// ================================================================================================
// Cross-entropy loss (mean over the batch) of [B, K] logits (bf16 or fp32) and int64 labels, as
// F.cross_entropy(logits.float(), y): forward = one block (one wave per row, fixed-order
// reductions: deterministic), writing the loss and each row's log-sum-exp; backward = one
// elementwise pass writing dlogits = (softmax - onehot) * grad / B in the logits' dtype.
// Replaces PyTorch's cast + log_softmax + nll_loss forward and the fill / nll / log_softmax
// backward / cast chain (9 launches per step).
// ================================================================================================
namespace {

template <typename T>
__device__ __forceinline__ float ew_ldf(const T* p, long long i);
template <>
__device__ __forceinline__ float ew_ldf<uint16_t>(const uint16_t* p, long long i) { return ew_bf16f(p[i]); }
template <>
__device__ __forceinline__ float ew_ldf<float>(const float* p, long long i) { return p[i]; }

template <typename T>
__global__ __launch_bounds__(1024) void k_ce_fwd(const T* __restrict__ x,
                                                 const long long* __restrict__ y, int B, int K,
                                                 float* __restrict__ loss,
                                                 float* __restrict__ lse, T* __restrict__ dx) {
  // dx (nullable): d(mean loss)/d logits for an upstream gradient of exactly 1, written here so
  // the backward needs no launch (k_ce_bwd's expressions with g = 1 / B: bit-identical)
  const float g1 = 1.0f / (float)B;
  __shared__ float lrow[16];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  float acc = 0.0f;  // this wave's sum of row losses (lane 0)
  if (K <= 32) {
    // few classes (CIFAR / MNIST: 10): one row per thread, no cross-lane reductions
    for (int r = threadIdx.x; r < B; r += 1024) {
      const T* xr = x + (long long)r * K;
      float m = -INFINITY;
      for (int k = 0; k < K; ++k) m = fmaxf(m, ew_ldf(xr, k));
      float s = 0.0f;
      for (int k = 0; k < K; ++k) s += expf(ew_ldf(xr, k) - m);
      const float l = m + logf(s);
      lse[r] = l;
      const long long t = y[r];
      acc += l - ((t >= 0 && t < K) ? ew_ldf(xr, t) : 0.0f);
      if (dx) {
        for (int k = 0; k < K; ++k) {
          float v = expf(ew_ldf(xr, k) - l);
          if ((long long)k == t) v -= 1.0f;
          v *= g1;
          if constexpr (sizeof(T) == 2) dx[(long long)r * K + k] = ew_f2bf(v);
          else dx[(long long)r * K + k] = v;
        }
      }
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) acc += __shfl_xor(acc, o, 64);  // fixed order
    if (lane != 0) acc = 0.0f;
  } else
  for (int r = wv; r < B; r += 16) {
    const T* xr = x + (long long)r * K;
    float m = -INFINITY;
    for (int k = lane; k < K; k += 64) m = fmaxf(m, ew_ldf(xr, k));
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) m = fmaxf(m, __shfl_xor(m, o, 64));
    float s = 0.0f;
    for (int k = lane; k < K; k += 64) s += expf(ew_ldf(xr, k) - m);
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) s += __shfl_xor(s, o, 64);
    const float l = m + logf(s);
    if (lane == 0) {
      lse[r] = l;
      const long long t = y[r];
      acc += l - ((t >= 0 && t < K) ? ew_ldf(xr, t) : 0.0f);
    }
    if (dx) {
      const long long t = y[r];
      for (int k = lane; k < K; k += 64) {
        float v = expf(ew_ldf(xr, k) - l);
        if ((long long)k == t) v -= 1.0f;
        v *= g1;
        if constexpr (sizeof(T) == 2) dx[(long long)r * K + k] = ew_f2bf(v);
        else dx[(long long)r * K + k] = v;
      }
    }
  }
  if (lane == 0) lrow[wv] = acc;
  __syncthreads();
  if (threadIdx.x == 0) {
    float tot = 0.0f;
    for (int i = 0; i < 16; ++i) tot += lrow[i];
    *loss = tot / (float)B;
  }
}

template <typename T>
__global__ __launch_bounds__(EW_BLOCK) void k_ce_bwd(const T* __restrict__ x,
                                                     const long long* __restrict__ y,
                                                     const float* __restrict__ lse,
                                                     const float* __restrict__ grad, int B, int K,
                                                     T* __restrict__ dx) {
  const float g = *grad / (float)B;
  const long long n = (long long)B * K;
  for (long long i = blockIdx.x * (long long)EW_BLOCK + threadIdx.x; i < n;
       i += (long long)gridDim.x * EW_BLOCK) {
    const int r = (int)(i / K), k = (int)(i - (long long)r * K);
    float v = expf(ew_ldf(x, i) - lse[r]);
    if ((long long)k == y[r]) v -= 1.0f;
    v *= g;
    if constexpr (sizeof(T) == 2) dx[i] = ew_f2bf(v);
    else dx[i] = v;
  }
}

}  // namespace

void ew_cross_entropy_fwd(uintptr_t x, uintptr_t y, int B, int K, int is_bf16, uintptr_t loss,
                          uintptr_t lse, uintptr_t stream, uintptr_t dx) {
  hipStream_t s = (hipStream_t)stream;
  if (is_bf16)
    hipLaunchKernelGGL(k_ce_fwd<uint16_t>, dim3(1), dim3(1024), 0, s,
                       reinterpret_cast<const uint16_t*>(x), reinterpret_cast<const long long*>(y),
                       B, K, reinterpret_cast<float*>(loss), reinterpret_cast<float*>(lse),
                       reinterpret_cast<uint16_t*>(dx));
  else
    hipLaunchKernelGGL(k_ce_fwd<float>, dim3(1), dim3(1024), 0, s,
                       reinterpret_cast<const float*>(x), reinterpret_cast<const long long*>(y), B,
                       K, reinterpret_cast<float*>(loss), reinterpret_cast<float*>(lse),
                       reinterpret_cast<float*>(dx));
  EW_CHECK_LAUNCH();
}

void ew_cross_entropy_bwd(uintptr_t x, uintptr_t y, uintptr_t lse, uintptr_t grad, int B, int K,
                          int is_bf16, uintptr_t dx, uintptr_t stream) {
  hipStream_t s = (hipStream_t)stream;
  const long long n = (long long)B * K;
  long long g = (n + EW_BLOCK - 1) / EW_BLOCK;
  if (g > 1024) g = 1024;
  if (g < 1) g = 1;
  if (is_bf16)
    hipLaunchKernelGGL(k_ce_bwd<uint16_t>, dim3((int)g), dim3(EW_BLOCK), 0, s,
                       reinterpret_cast<const uint16_t*>(x), reinterpret_cast<const long long*>(y),
                       reinterpret_cast<const float*>(lse), reinterpret_cast<const float*>(grad), B,
                       K, reinterpret_cast<uint16_t*>(dx));
  else
    hipLaunchKernelGGL(k_ce_bwd<float>, dim3((int)g), dim3(EW_BLOCK), 0, s,
                       reinterpret_cast<const float*>(x), reinterpret_cast<const long long*>(y),
                       reinterpret_cast<const float*>(lse), reinterpret_cast<const float*>(grad), B,
                       K, reinterpret_cast<float*>(dx));
  EW_CHECK_LAUNCH();
}

// ================================================================================================
// Classifier-head activations (VGG's Dropout / Linear-ReLU-Dropout / Linear-ReLU layers) on
// [rows, C] bf16 activations:
//   forward : z = act(y) * keep / (1 - p), keep = hash(key, i) >= p  (act = ReLU or identity)
//   backward: dy = dz * keep / (1 - p) * act'(y), and db[c] = sum over rows of dy (the bias
//             gradient of the Linear that produced y: no separate reduction kernel)
// The dropout key comes from a per-layer device counter ctr[0]: forward and backward read it,
// and the backward's last-arriving block (ticket ctr[1]) advances it -- a fresh mask every
// step, also under HIP-graph replay, without PyTorch's per-replay RNG offset fills.  Masks are
// recomputed, never stored.  Backward blocks own column strips, so the bias gradient needs no
// cross-block reduction.
// ================================================================================================
namespace {

__device__ __forceinline__ bool ew_keep(uint32_t i, uint32_t key, float p) {
  return ew_uniform(i, key) >= p;
}
__device__ __forceinline__ uint32_t ew_drop_key(int ctr, uint32_t salt) {
  return ew_mix32((uint32_t)ctr * 0x9E3779B9u + salt);
}

__global__ __launch_bounds__(EW_BLOCK) void k_act_dropout_fwd(const uint16_t* __restrict__ y,
                                                              uint16_t* __restrict__ z, int n,
                                                              float p, int relu,
                                                              const int* __restrict__ ctr,
                                                              uint32_t salt) {
  const uint32_t key = ew_drop_key(ctr[0], salt);
  const float scale = p > 0.0f ? 1.0f / (1.0f - p) : 1.0f;
  for (int v = blockIdx.x * EW_BLOCK + threadIdx.x; 8 * v < n; v += gridDim.x * EW_BLOCK) {
    const int i0 = 8 * v;  // n % 8 == 0 (host)
    float x[8];
    V8<uint16_t>::ld(y + i0, x);
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      if (relu) x[j] = ew_relu(x[j]);
      if (p > 0.0f) x[j] = ew_keep((uint32_t)(i0 + j), key, p) ? x[j] * scale : 0.0f;
    }
    V8<uint16_t>::st(z + i0, x);
  }
}

// block b: columns [16 b, 16 b + 16) over all rows, so its bias gradient is block-local (no
// cross-block partials).  Thread t: column octet t & 1 (8 columns as one 16-byte access), rows
// t >> 1, + 128, ...; the per-column sums are reduced across the wave's 32 row groups with
// shuffles and across the 4 waves through LDS, in a fixed order.
constexpr int EW_AD_TC = 2, EW_AD_RG = EW_BLOCK / EW_AD_TC;
__global__ __launch_bounds__(EW_BLOCK) void k_act_dropout_bwd(
    const uint16_t* __restrict__ dz, const uint16_t* __restrict__ y, uint16_t* __restrict__ dy,
    void* __restrict__ db, int db_bf16, int rows, int C, float p, int relu,
    int* __restrict__ ctr, uint32_t salt) {
  __shared__ float part[EW_WAVES][EW_AD_TC * 8];
  const uint32_t key = ew_drop_key(ctr[0], salt);
  const float scale = p > 0.0f ? 1.0f / (1.0f - p) : 1.0f;
  const int tc = threadIdx.x % EW_AD_TC, rg = threadIdx.x / EW_AD_TC;
  const int c0 = (blockIdx.x * EW_AD_TC + tc) * 8;
  float s[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) s[j] = 0.0f;
  if (c0 < C) {
    for (int r0 = rg; r0 < rows; r0 += 2 * EW_AD_RG) {  // two rows in flight per thread
      float g[2][8], yv[2][8];
      const bool two = r0 + EW_AD_RG < rows;
#pragma unroll
      for (int u = 0; u < 2; ++u) {
        const int r = two ? r0 + u * EW_AD_RG : r0;
        V8<uint16_t>::ld(dz + (long long)r * C + c0, g[u]);
        if (relu) V8<uint16_t>::ld(y + (long long)r * C + c0, yv[u]);
      }
#pragma unroll
      for (int u = 0; u < 2; ++u) {
        if (u == 1 && !two) break;
        const int r = r0 + u * EW_AD_RG;
        const uint32_t i0 = (uint32_t)r * (uint32_t)C + (uint32_t)c0;
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          float v = g[u][j];
          if (p > 0.0f) v = ew_keep(i0 + j, key, p) ? v * scale : 0.0f;
          if (relu && !ew_relu_pass(yv[u][j])) v = 0.0f;
          g[u][j] = V8<uint16_t>::rnd(v);
          s[j] += g[u][j];  // the bias gradient of the rounded dy the GEMMs consume
        }
        V8<uint16_t>::st(dy + (long long)r * C + c0, g[u]);
      }
    }
  }
  // sum over the wave's row groups (lanes with equal tc), then over the waves
#pragma unroll
  for (int o = EW_AD_TC; o < 64; o <<= 1) {
#pragma unroll
    for (int j = 0; j < 8; ++j) s[j] += __shfl_xor(s[j], o, 64);
  }
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  if (lane < EW_AD_TC) {
#pragma unroll
    for (int j = 0; j < 8; ++j) part[wave][lane * 8 + j] = s[j];
  }
  __syncthreads();
  if (db && threadIdx.x < EW_AD_TC * 8) {
    const int c = blockIdx.x * EW_AD_TC * 8 + threadIdx.x;
    if (c < C) {
      float a = 0.0f;
#pragma unroll
      for (int w = 0; w < EW_WAVES; ++w) a += part[w][threadIdx.x];  // fixed order
      if (db_bf16) reinterpret_cast<uint16_t*>(db)[c] = ew_f2bf(a);
      else reinterpret_cast<float*>(db)[c] = a;
    }
  }
  // advance the key counter once every block has read it: arrival ticket ctr[1] (each block's
  // read of ctr[0] completed before its ticket; the new value is seen by the next kernel)
  if (threadIdx.x == 0) {
    const int tk = __hip_atomic_fetch_add(&ctr[1], 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (tk == (int)gridDim.x - 1) {
      ctr[1] = 0;
      ctr[0] = ctr[0] + 1;
    }
  }
}

}  // namespace

void ew_act_dropout_fwd(uintptr_t y, uintptr_t z, int n, float p, int relu, uintptr_t ctr,
                        uint32_t salt, uintptr_t stream) {
  if (n % 8) throw std::runtime_error("ewdml act_dropout_fwd: n % 8 != 0");
  int g = (n / 8 + EW_BLOCK - 1) / EW_BLOCK;
  g = g < 1 ? 1 : (g > 1024 ? 1024 : g);
  hipLaunchKernelGGL(k_act_dropout_fwd, dim3(g), dim3(EW_BLOCK), 0, (hipStream_t)stream,
                     reinterpret_cast<const uint16_t*>(y), reinterpret_cast<uint16_t*>(z), n, p,
                     relu, reinterpret_cast<const int*>(ctr), salt);
  EW_CHECK_LAUNCH();
}

void ew_act_dropout_bwd(uintptr_t dz, uintptr_t y, uintptr_t dy, uintptr_t db, int db_bf16,
                        int rows, int C, float p, int relu, uintptr_t ctr, uint32_t salt,
                        uintptr_t stream) {
  if (C % 8) throw std::runtime_error("ewdml act_dropout_bwd: C % 8 != 0");
  const int g = (C + EW_AD_TC * 8 - 1) / (EW_AD_TC * 8);
  hipLaunchKernelGGL(k_act_dropout_bwd, dim3(g), dim3(EW_BLOCK), 0, (hipStream_t)stream,
                     reinterpret_cast<const uint16_t*>(dz), reinterpret_cast<const uint16_t*>(y),
                     reinterpret_cast<uint16_t*>(dy), reinterpret_cast<void*>(db), db_bf16, rows,
                     C, p, relu, reinterpret_cast<int*>(ctr), salt);
  EW_CHECK_LAUNCH();
}
