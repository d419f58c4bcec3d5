// fp32 3x3 (pad 1, stride 1) convolutions by Winograd F(m x m, 3x3), m = 2 or 4: forward,
// backward-data and weight-gradient.
//
// Each m x m output tile is A^T [ (G g G^T) .* (B^T d B) ] A over the a x a input patch d
// (a = m + 2), so the 9-tap implicit GEMM of conv_f32.hip (2*P*C*Nc*9 FLOPs) becomes a*a batched
// GEMMs over the tiles (2*(P/m^2)*a^2*C*Nc FLOPs: 2.25x fewer at m = 2, 4x at m = 4):
//
//   U[xi][Nc][C]    = (G g G^T)[xi]           weight transform, once per step
//   V[xi][tiles][C] = (B^T d B)[xi]           input transform (one launch for both: k_wg_input)
//   Mo[xi][tiles][Nc] = V[xi] U[xi]^T          a^2 fp32 MFMA GEMMs (conv_f32.hip k_cf_gemm, batched)
//   y = A^T Mo A                              output transform (k_wg_output), with the BatchNorm
//                                             partial sums (forward) or the producing BN layer's
//                                             backward sums + residual addend (backward data)
//
// Backward data is the same pipeline on dy with the 180-degree-rotated kernel and the channel
// roles swapped.  At m = 2, G J = P G (J: column reversal, P: rows 0 <-> 3), so its transformed
// weight is the forward U read transposed with positions (i, j) -> (p(i), p(j)) (CfGeom::b_flip:
// no second weight transform); at m = 4 the points (0, +-1, +-2) are not closed under p -> 1/p
// and the rotated kernel gets its own transform (in the backward input launch).
//
// Weight gradient, the transpose of the forward: dMo = A dy A^T per tile (made by the backward-
// data input pass from the same reads, or k_wg_dy), dU[xi][Nc][C] = sum over tiles of
// dMo[xi][tile][Nc] V[xi][tile][C] (the forward's V, kept; one K = tiles GEMM per position,
// K-split into slabs), then dw = G^T dU G summed over the splits in a fixed order.
//
// m = 2: B^T = [1 0 -1 0; 0 1 1 0; 0 -1 1 0; 0 1 0 -1], G = [1 0 0; .5 .5 .5; .5 -.5 .5; 0 0 1],
//        A^T = [1 1 1 0; 0 1 -1 -1].
// m = 4: points 0, 1, -1, 2, -2, inf (Lavin & Gray's F(4x4, 3x3)).
// All arithmetic fp32.  Relative error against float64 (tests/kernels/test_conv_f32.py, and
// tools/conv_f32_probe.py --err): direct ~2e-7, m = 2 ~5e-7, m = 4 ~3e-6 -- every form far inside
// fp32 training noise and 100x below tf32 / 1000x below bf16 operand rounding.
//
// Why unfused transforms: on the deep VGG / ResNet layers (C >= 128, maps <= 16x16) the GEMM
// dominates and V / Mo stay in the 256 MB MALL; ops/conv.py only routes a layer here where that
// holds (the per-layer choice is measured: tools/conv_f32_probe.py --wino).
#include <stdexcept>
#include <string>

#include "common.h"
#include "conv_f32.h"
#include "wg_common.h"
#include "ewdml_ops.h"

int ew_cf_gemm_tn_batched(const float* a, const float* b, float* out, float* ws,
                          long long ws_floats, int M, int N, int K, int batch, long long a_bs,
                          long long b_bs, hipStream_t s);
void ew_cf_gemm_batched(const float* a, const float* b, float* out, int M, int N, int K, int batch,
                        long long a_bs, long long b_bs, long long o_bs, bool nt, bool flip,
                        hipStream_t s);

namespace {

// U[xi][o][i..] = (G g G^T)[xi], g(r, s) = w[o][r][s][i..] (channels_last [Nc][3][3][C]);
// FLIP: the 180-degree-rotated kernel g(r, s) = w[o][2-r][2-s][i..] (backward data at m = 4)
template <int M, bool FLIP>
__device__ __forceinline__ void wg_weight(const float* __restrict__ w, float* __restrict__ U,
                                          int Nc, int C, long long g) {
  using T = typename Wg<M>::V;
  constexpr int A = Wg<M>::A, VW = Wg<M>::VW;
  const int cq = C / VW;
  if (g >= (long long)Nc * cq) return;
  const int o = (int)(g / cq), i = (int)(g - (long long)o * cq) * VW;
  T k[3][3];
#pragma unroll
  for (int r = 0; r < 3; ++r)
#pragma unroll
    for (int s = 0; s < 3; ++s) {
      const int tap = FLIP ? (2 - r) * 3 + (2 - s) : r * 3 + s;
      k[r][s] = *reinterpret_cast<const T*>(w + ((long long)o * 9 + tap) * C + i);
    }
  const long long xs = (long long)Nc * C;
  float* u = U + (long long)o * C + i;
#pragma unroll
  for (int a = 0; a < A; ++a) {
    T t[3];  // row a of G g
#pragma unroll
    for (int s = 0; s < 3; ++s) {
      const T col[3] = {k[0][s], k[1][s], k[2][s]};
      t[s] = wg_dot<3>([&](int r) { return wg_g<M>(a, r); }, col);
    }
#pragma unroll
    for (int b = 0; b < A; ++b)  // (G g) G^T
      *reinterpret_cast<T*>(u + (a * A + b) * xs) =
          wg_dot<3>([&](int s) { return wg_g<M>(b, s); }, t);
  }
}

// dMo = A dy A^T of one m x m dy tile (rows dy[i][j]), stored at o[xi * xs]
template <int M>
__device__ __forceinline__ void wg_dy_store(float* __restrict__ o, long long xs,
                                            const typename Wg<M>::V (&dy)[M][M]) {
  using T = typename Wg<M>::V;
  constexpr int A = Wg<M>::A;
#pragma unroll
  for (int a = 0; a < A; ++a) {
    T t[M];  // row a of A dy = sum_i AT[i][a] dy[i][.]
#pragma unroll
    for (int j = 0; j < M; ++j) {
      T col[M];
#pragma unroll
      for (int i = 0; i < M; ++i) col[i] = dy[i][j];
      t[j] = wg_dot<M>([&](int i) { return wg_at<M>(i, a); }, col);
    }
#pragma unroll
    for (int b = 0; b < A; ++b)
      *reinterpret_cast<T*>(o + (a * A + b) * xs) =
          wg_dot<M>([&](int j) { return wg_at<M>(j, b); }, t);
  }
}

// Where the input transform's operand comes from (KIND):
//  0: x itself (a materialised activation or gradient);
//  1: the forward of the BatchNorm(+ReLU)(+2x2 max pool) layer in front, applied on the fly:
//     x = maxpool?(relu(h * scale + shift)) with h that layer's BN input (2H x 2W when pooled);
//     the pool's window codes are written by the tile that owns the position (the patch's
//     inner m x m), num_batches_tracked incremented once -- the BN apply kernel and the x round
//     trip disappear (ops/nn.py lazy forward);
//  2: the backward of the BatchNorm(+ReLU)(+pool) layer whose input is this conv's output, on the
//     fly: dy = scale * dz + e * (h - mean) + f (nn.hip k_bn_bwd_apply's formula, coef = (e, f)),
//     dz = relu'(h * scale + shift) * (pool ? [code == q] dnext[pooled] : dnext), h this conv's
//     output -- the BN backward's apply kernel and the dh round trip disappear.
struct WgSrc {
  const float* h;       // KIND 1: the BN input in front; KIND 2: this conv's output
  const float* stats;   // [4][C]: mean, invstd, scale, shift
  uint8_t* code;        // pool window codes at the pooled resolution (KIND 1 writes, 2 reads)
  const float* coef;    // KIND 2: [2][C] (e, f)
  const float* dnext;   // KIND 2: gradient of the BN layer's (pooled) output
  long long* nbt;       // KIND 1: num_batches_tracked (incremented by thread 0 of block 0)
  int pool;
};

// V[xi][tile][c..] = (B^T d B)[xi], d = the a x a patch at (m ty - 1, m tx - 1) of x[N][H][W][C]
// (zero outside).  Thread: one tile x one channel vector; consecutive threads, consecutive
// vectors.  With D: also the weight gradient's dMo of the patch's inner m x m (the dy tile).
template <int M, int KIND>
__device__ __forceinline__ void wg_input(const float* __restrict__ x, float* __restrict__ V,
                                         int H, int W, int C, long long tiles, long long g,
                                         float* __restrict__ D, const WgSrc& src) {
  using T = typename Wg<M>::V;
  constexpr int A = Wg<M>::A, VW = Wg<M>::VW;
  const int cq = C / VW;
  if (KIND == 1 && src.nbt && g == 0) *src.nbt += 1;
  if (g >= tiles * cq) return;
  const long long tl = g / cq;
  const int c = (int)(g - tl * cq) * VW;
  const int tw = W / M, tpi = (H / M) * tw;
  const int n = (int)(tl / tpi), rem = (int)(tl - (long long)n * tpi);
  const int ty = rem / tw, tx = rem - ty * tw;
  const int h0 = M * ty - 1, w0 = M * tx - 1;
  T sc{}, sh{}, mean{}, ce{}, cf{};
  if constexpr (KIND != 0) {
#pragma unroll
    for (int q = 0; q < VW; ++q) {
      sc[q] = src.stats[2 * C + c + q];
      sh[q] = src.stats[3 * C + c + q];
      if constexpr (KIND == 2) {
        mean[q] = src.stats[c + q];
        ce[q] = src.coef[c + q];
        cf[q] = src.coef[C + c + q];
      }
    }
  }
  T d[A][A];
#pragma unroll
  for (int i = 0; i < A; ++i)
#pragma unroll
    for (int j = 0; j < A; ++j) {
      const int h = h0 + i, w = w0 + j;
      const bool ok = (unsigned)h < (unsigned)H && (unsigned)w < (unsigned)W;
      const long long r = ok ? ((long long)n * H + h) * W + w : 0;  // row at this resolution
      T v{};
      if constexpr (KIND == 0) {
        v = *reinterpret_cast<const T*>(x + r * C + c);
      } else if constexpr (KIND == 1) {
        if (!src.pool) {
          const T hv = *reinterpret_cast<const T*>(src.h + r * C + c);
#pragma unroll
          for (int q = 0; q < VW; ++q) {
            const float z = hv[q] * sc[q] + sh[q];  // as k_bn_fwd_apply writes it
            v[q] = (z > 0.0f || z != z) ? z : 0.0f;
          }
        } else {  // max over the 2x2 window of the 2H x 2W map, first max wins (k_bn_fwd_apply)
          const int W2 = 2 * W;
          const long long r0 = ((long long)n * 2 * H + 2 * h) * W2 + 2 * w;
          uint32_t k[VW];
#pragma unroll
          for (int qq = 0; qq < 4; ++qq) {
            const T hv = *reinterpret_cast<const T*>(
                src.h + (ok ? r0 + (qq >> 1) * W2 + (qq & 1) : 0) * C + c);
#pragma unroll
            for (int q = 0; q < VW; ++q) {
              const float z = hv[q] * sc[q] + sh[q];
              const float y = (z > 0.0f || z != z) ? z : 0.0f;
              if (qq == 0 || y > v[q] || y != y) {
                v[q] = y;
                k[q] = qq;
              }
            }
          }
          if (ok && i >= 1 && i <= M && j >= 1 && j <= M) {  // the owning tile writes the code
            uint32_t wd = 0;
#pragma unroll
            for (int q = 0; q < VW; ++q) wd |= k[q] << (8 * q);
            if constexpr (VW == 4)
              *reinterpret_cast<uint32_t*>(src.code + r * C + c) = wd;
            else
              *reinterpret_cast<uint16_t*>(src.code + r * C + c) = (uint16_t)wd;
          }
        }
      } else {  // KIND 2
        const T hv = *reinterpret_cast<const T*>(src.h + r * C + c);
        T dp;
        if (src.pool) {
          const int Wo = W / 2;
          // (h, w) may lie in the zero padding: index row 0 there (the value is masked below)
          const long long pr = ok ? ((long long)n * (H / 2) + (h >> 1)) * Wo + (w >> 1) : 0;
          const T dn = *reinterpret_cast<const T*>(src.dnext + pr * C + c);
          const uint32_t qq = (uint32_t)((h & 1) * 2 + (w & 1));
          uint32_t kw;
          if constexpr (VW == 4)
            kw = *reinterpret_cast<const uint32_t*>(src.code + pr * C + c);
          else
            kw = *reinterpret_cast<const uint16_t*>(src.code + pr * C + c);
#pragma unroll
          for (int q = 0; q < VW; ++q) dp[q] = ((kw >> (8 * q)) & 0xffu) == qq ? dn[q] : 0.0f;
        } else {
          dp = *reinterpret_cast<const T*>(src.dnext + r * C + c);
        }
#pragma unroll
        for (int q = 0; q < VW; ++q) {
          // the expressions of k_bn_bwd_apply: the same contraction, the same bits
          const float z = hv[q] * sc[q] + sh[q];
          const float dz = !(z <= 0.0f) ? dp[q] : 0.0f;
          v[q] = sc[q] * dz + ce[q] * (hv[q] - mean[q]) + cf[q];
        }
      }
      d[i][j] = ok ? v : T{};
    }
  if (D) {
    T dy[M][M];
#pragma unroll
    for (int i = 0; i < M; ++i)
#pragma unroll
      for (int j = 0; j < M; ++j) dy[i][j] = d[i + 1][j + 1];
    wg_dy_store<M>(D + tl * C + c, tiles * C, dy);
  }
  const long long xs = tiles * C;
  float* v = V + tl * C + c;
#pragma unroll
  for (int a = 0; a < A; ++a) {
    T t[A];  // row a of B^T d
#pragma unroll
    for (int j = 0; j < A; ++j) {
      T col[A];
#pragma unroll
      for (int i = 0; i < A; ++i) col[i] = d[i][j];
      t[j] = wg_dot<A>([&](int i) { return wg_bt<M>(a, i); }, col);
    }
#pragma unroll
    for (int b = 0; b < A; ++b)  // (B^T d) B
      *reinterpret_cast<T*>(v + (a * A + b) * xs) =
          wg_dot<A>([&](int j) { return wg_bt<M>(b, j); }, t);
  }
}

// the input transform over blocks [0, nbi), the weight transform (when w is given) over the next
// nbw and a riding weight-gradient output transform (wo.src) over the rest: one launch for all
// (each alone is a few-microsecond kernel)
template <int M, bool FLIP, int KIND>
__global__ __launch_bounds__(EW_BLOCK) void k_wg_input(const float* __restrict__ x,
                                                       float* __restrict__ V, int H, int W, int C,
                                                       long long tiles, int nbi,
                                                       const float* __restrict__ w,
                                                       float* __restrict__ U, int Nw, int Cw,
                                                       float* __restrict__ D, WgSrc src, int nbw,
                                                       WgOut wo) {
  const int b = (int)blockIdx.x;
  if (b < nbi)
    wg_input<M, KIND>(x, V, H, W, C, tiles, (long long)b * EW_BLOCK + threadIdx.x, D, src);
  else if (b < nbi + nbw)
    wg_weight<M, FLIP>(w, U, Nw, Cw, (long long)(b - nbi) * EW_BLOCK + threadIdx.x);
  else
    wg_wgrad_out<M>(wo.src, wo.nsplit, wo.dw, wo.Nc, wo.C,
                    (long long)(b - nbi - nbw) * EW_BLOCK + threadIdx.x);
}

template <int M>
__global__ __launch_bounds__(EW_BLOCK) void k_wg_weight(const float* __restrict__ w,
                                                        float* __restrict__ U, int Nc, int C) {
  wg_weight<M, false>(w, U, Nc, C, (long long)blockIdx.x * EW_BLOCK + threadIdx.x);
}

// dMo of dy alone (weight gradient without a Winograd backward-data pass before it)
template <int M>
__global__ __launch_bounds__(EW_BLOCK) void k_wg_dy(const float* __restrict__ dy,
                                                    float* __restrict__ D, int H, int W, int Nc,
                                                    long long tiles) {
  using T = typename Wg<M>::V;
  constexpr int VW = Wg<M>::VW;
  const int cq = Nc / VW;
  const long long g = (long long)blockIdx.x * EW_BLOCK + threadIdx.x;
  if (g >= tiles * cq) return;
  const long long tl = g / cq;
  const int c = (int)(g - tl * cq) * VW;
  const int tw = W / M, tpi = (H / M) * tw;
  const int n = (int)(tl / tpi), rem = (int)(tl - (long long)n * tpi);
  const int ty = rem / tw, tx = rem - ty * tw;
  const float* p = dy + (((long long)n * H + M * ty) * W + M * tx) * Nc + c;
  T t[M][M];
#pragma unroll
  for (int i = 0; i < M; ++i)
#pragma unroll
    for (int j = 0; j < M; ++j)
      t[i][j] = *reinterpret_cast<const T*>(p + ((long long)i * W + j) * Nc);
  wg_dy_store<M>(D + tl * Nc + c, tiles * Nc, t);
}

// y = A^T Mo A per tile (+ addend), with the BatchNorm partial sums of y (forward: sum, sum of
// squares; backward: CfBnBwd's sum dz, sum dz * (h - mean)) -> row blockIdx.x of bnpart[2][nb][Nc].
// Block: tiles [b * tpb, (b + 1) * tpb) x all Nc channels; thread: channel vector t % (Nc / VW),
// tiles t / (Nc / VW) + k * rpi (rpi = 256 / (Nc / VW) tiles per pass, Nc a power of two).
// VW channels per thread, independent of the other transforms' width: 2 where Nc <= 512 (twice
// the threads of 4: 114 -> 101 us/step of output transforms on VGG-11, profiles/ab/README.md)
template <int M, int VW>
__global__ __launch_bounds__(EW_BLOCK) void k_wg_output(const float* __restrict__ Mo,
                                                        float* __restrict__ y, int H, int W,
                                                        int Nc, long long tiles, int tpb,
                                                        float* __restrict__ bnpart, CfBnBwd bb,
                                                        const float* __restrict__ addend) {
  typedef float T __attribute__((ext_vector_type(VW)));
  constexpr int A = Wg<M>::A;
  __shared__ __attribute__((aligned(16))) float red[2][EW_BLOCK * 4];
  const int tpr = Nc / VW, rpi = EW_BLOCK / tpr;
  const int t = threadIdx.x, rg = t / tpr, c0 = (t - rg * tpr) * VW;
  const long long t0 = (long long)blockIdx.x * tpb;
  const long long t1 = t0 + tpb < tiles ? t0 + tpb : tiles;
  const int tw = W / M, tpi = (H / M) * tw;
  const long long xs = tiles * Nc;
  const uint32_t HoWo = (uint32_t)bb.Ho * bb.Wo;
  float s1[VW], s2[VW], mean[VW], sc[VW], sh[VW];
#pragma unroll
  for (int j = 0; j < VW; ++j) s1[j] = s2[j] = 0.0f;
  if (bnpart && bb.h) {
#pragma unroll
    for (int j = 0; j < VW; ++j) {
      mean[j] = bb.stats[c0 + j];
      sc[j] = bb.stats[2 * Nc + c0 + j];
      sh[j] = bb.stats[3 * Nc + c0 + j];
    }
  }
  for (long long tl = t0 + rg; tl < t1; tl += rpi) {
    const float* mp = Mo + tl * Nc + c0;
    T u[M][A];  // A^T Mo, one column b at a time
#pragma unroll
    for (int b = 0; b < A; ++b) {
      T col[A];
#pragma unroll
      for (int a = 0; a < A; ++a) col[a] = *reinterpret_cast<const T*>(mp + (a * A + b) * xs);
#pragma unroll
      for (int i = 0; i < M; ++i) u[i][b] = wg_dot<A>([&](int a) { return wg_at<M>(i, a); }, col);
    }
    const int n = (int)(tl / tpi), rem = (int)(tl - (long long)n * tpi);
    const int ty = rem / tw, tx = rem - ty * tw;
#pragma unroll
    for (int i = 0; i < M; ++i)
#pragma unroll
      for (int j = 0; j < M; ++j) {  // (A^T Mo) A
        T v = wg_dot<A>([&](int b) { return wg_at<M>(j, b); }, u[i]);
        const long long r = ((long long)n * H + M * ty + i) * W + M * tx + j;
        const long long off = r * Nc + c0;
        if (addend) v += *reinterpret_cast<const T*>(addend + off);
        *reinterpret_cast<T*>(y + off) = v;
        if (!bnpart) continue;
        if (!bb.h) {  // forward: this output's own statistics
#pragma unroll
          for (int q = 0; q < VW; ++q) {
            s1[q] += v[q];
            s2[q] += v[q] * v[q];
          }
          continue;
        }
        // backward sums of the BN layer whose (pooled) output this gradient is: its input h
        // (and residual) at the row the pool routed each channel from -- the window's four
        // candidate rows as vector loads, picked per channel by its code
        T xh, rr{};
        if (bb.code) {
          const uint32_t p = (uint32_t)r, nn = p / HoWo, rm = p - nn * HoWo;
          const uint32_t ho = rm / (uint32_t)bb.Wo, wo = rm - ho * (uint32_t)bb.Wo;
          const uint32_t base = 4 * nn * HoWo + 4 * ho * (uint32_t)bb.Wo + 2 * wo;
          uint32_t kw;
          if constexpr (VW == 4)
            kw = *reinterpret_cast<const uint32_t*>(bb.code + off);
          else
            kw = *reinterpret_cast<const uint16_t*>(bb.code + off);
          T hq[4], rq[4];
#pragma unroll
          for (int qq = 0; qq < 4; ++qq) {
            const size_t hr = base + (qq >> 1) * (2 * (uint32_t)bb.Wo) + (qq & 1);
            hq[qq] = *reinterpret_cast<const T*>(bb.h + hr * Nc + c0);
            if (bb.res) rq[qq] = *reinterpret_cast<const T*>(bb.res + hr * Nc + c0);
          }
#pragma unroll
          for (int q = 0; q < VW; ++q) {
            const uint32_t k = (kw >> (8 * q)) & 3u;
            xh[q] = k == 0 ? hq[0][q] : k == 1 ? hq[1][q] : k == 2 ? hq[2][q] : hq[3][q];
            if (bb.res) rr[q] = k == 0 ? rq[0][q] : k == 1 ? rq[1][q] : k == 2 ? rq[2][q] : rq[3][q];
          }
        } else {
          xh = *reinterpret_cast<const T*>(bb.h + (size_t)r * Nc + c0);
          if (bb.res) rr = *reinterpret_cast<const T*>(bb.res + (size_t)r * Nc + c0);
        }
#pragma unroll
        for (int q = 0; q < VW; ++q) {
          float z = xh[q] * sc[q] + sh[q];
          if (bb.res) z = z + rr[q];
          const float dz = (bb.relu == 0 || !(z <= 0.0f)) ? v[q] : 0.0f;
          s1[q] += dz;
          s2[q] += dz * (xh[q] - mean[q]);
        }
      }
  }
  if (!bnpart) return;
  // one VW-wide store per thread and array (lanes' vectors contiguous): scalar stores of
  // stride-VW addresses were VW-way bank conflicts (2.0 conflicts per LDS instruction, round-5
  // PMC table)
  {
    T a, b;
#pragma unroll
    for (int q = 0; q < VW; ++q) {
      a[q] = s1[q];
      b[q] = s2[q];
    }
    *reinterpret_cast<T*>(&red[0][rg * Nc + c0]) = a;
    *reinterpret_cast<T*>(&red[1][rg * Nc + c0]) = b;
  }
  __syncthreads();
  const int nb = gridDim.x;
  for (int c = t; c < Nc; c += EW_BLOCK) {
    float a = 0.0f, q = 0.0f;
    for (int i = 0; i < rpi; ++i) {  // fixed order
      a += red[0][i * Nc + c];
      q += red[1][i * Nc + c];
    }
    bnpart[(long long)blockIdx.x * Nc + c] = a;
    bnpart[(long long)(nb + blockIdx.x) * Nc + c] = q;
  }
}

// dw[o][r][s][i..] = (G^T (sum_z dU_z[xi]) G)[r][s], dU_z = src + z * A^2 * Nc * C

template <int M>
__global__ __launch_bounds__(EW_BLOCK) void k_wg_wgrad_out(const float* __restrict__ src,
                                                           int nsplit, float* __restrict__ dw,
                                                           int Nc, int C) {
  wg_wgrad_out<M>(src, nsplit, dw, Nc, C, (long long)blockIdx.x * EW_BLOCK + threadIdx.x);
}

long long wg_tiles(int m, long long N, int H, int W) { return N * (H / m) * (W / m); }

void wg_check(int m, long long N, int H, int W, int Cin, int Cout, const char* what) {
  const long long tiles = wg_tiles(m, N, H, W);
  const int vw = m == 2 ? WG2_VW : 2;
  const bool pow2 = Cout >= 64 && Cout <= 256 * vw && (Cout & (Cout - 1)) == 0;
  if ((m != 2 && m != 4) || H % m || W % m || tiles % 64 || Cin % 32 || !pow2 ||
      (long long)(m + 2) * (m + 2) * tiles * std::max(Cin, Cout) >= (1LL << 31))
    throw std::runtime_error(std::string("ewdml winograd f32 ") + what +
                             ": needs m in {2, 4}, H, W % m == 0, N*H*W/m^2 % 64 == 0, C_in % 32 "
                             "== 0, C_out a power of two in [64, 256 * (m == 2 ? 4 : 2)]");
}

// output transform launch: returns the BN partial rows written (0: none requested / no room)
template <int M>
int wg_output(const float* Mo, float* y, long long N, int H, int W, int Nc, float* bnpart,
              long long bnpart_floats, const CfBnBwd& bb, const float* addend, hipStream_t s) {
  const long long tiles = wg_tiles(M, N, H, W);
  const int ovw = Nc <= 2 * EW_BLOCK ? 2 : 4;
  const int rpi = EW_BLOCK / (Nc / ovw);
  long long tpb = rpi, nblk = (tiles + tpb - 1) / tpb;
  if (bnpart) {
    while (nblk > 1024) {
      tpb += rpi;
      nblk = (tiles + tpb - 1) / tpb;
    }
    if (2LL * nblk * Nc > bnpart_floats) bnpart = nullptr;
  }
  if (!bnpart) {
    tpb = rpi;
    nblk = (tiles + tpb - 1) / tpb;
  }
  if (ovw == 2)
    hipLaunchKernelGGL((k_wg_output<M, 2>), dim3((unsigned)nblk), dim3(EW_BLOCK), 0, s, Mo, y, H,
                       W, Nc, tiles, (int)tpb, bnpart, bb, addend);
  else
    hipLaunchKernelGGL((k_wg_output<M, 4>), dim3((unsigned)nblk), dim3(EW_BLOCK), 0, s, Mo, y, H,
                       W, Nc, tiles, (int)tpb, bnpart, bb, addend);
  EW_CHECK_LAUNCH();
  return bnpart ? (int)nblk : 0;
}

// input transform of x [N][H][W][C] into V (+ D); with w, also U from w [Nw][3][3][Cw] (FLIP:
// the rotated kernel)
template <int M, bool FLIP>
void wg_input(const float* x, float* V, long long N, int H, int W, int C, hipStream_t s,
              const float* w, float* U, int Nw, int Cw, float* D, const WgSrc* src = nullptr,
              int kind = 0, const WgOut* rider = nullptr) {
  constexpr int VW = Wg<M>::VW;
  const long long n = wg_tiles(M, N, H, W) * (C / VW);
  const int nbi = (int)((n + EW_BLOCK - 1) / EW_BLOCK);
  const int nbw = w ? (int)(((long long)Nw * (Cw / VW) + EW_BLOCK - 1) / EW_BLOCK) : 0;
  const WgOut no_out{nullptr, nullptr, 1, 0, 0};
  const WgOut& wo = rider && rider->src ? *rider : no_out;
  const int nbo = wo.src ? (int)(((long long)wo.Nc * (wo.C / VW) + EW_BLOCK - 1) / EW_BLOCK) : 0;
  const WgSrc none{nullptr, nullptr, nullptr, nullptr, nullptr, nullptr, 0};
  const WgSrc& sr = src ? *src : none;
#define WG_IN(K_)                                                                                \
  hipLaunchKernelGGL((k_wg_input<M, FLIP, K_>), dim3(nbi + nbw + nbo), dim3(EW_BLOCK), 0, s, x, V, \
                     H, W, C, wg_tiles(M, N, H, W), nbi, w, U, Nw, Cw, D, sr, nbw, wo)
  if (kind == 1) WG_IN(1);
  else if (kind == 2) WG_IN(2);
  else WG_IN(0);
#undef WG_IN
  EW_CHECK_LAUNCH();
}

template <int M>
int wino_fwd(const float* x, const float* w, float* U, float* y, float* v, float* mo, long long N,
             int H, int W, int C, int Nc, float* bnpart, long long bnpart_floats, hipStream_t s,
             const WgSrc* src) {
  constexpr int AA = Wg<M>::A * Wg<M>::A;
  const long long tiles = wg_tiles(M, N, H, W);
  wg_input<M, false>(x, v, N, H, W, C, s, w, U, Nc, C, nullptr, src, src ? 1 : 0);
  ew_cf_gemm_batched(v, U, mo, (int)tiles, Nc, C, AA, tiles * C, (long long)Nc * C, tiles * Nc,
                     true, false, s);
  const CfBnBwd none{nullptr, nullptr, nullptr, nullptr, 0, 0, 0};
  return wg_output<M>(mo, y, N, H, W, Nc, bnpart, bnpart_floats, none, nullptr, s);
}

template <int M>
int wino_bwd(const float* dy, const float* w, float* U, float* dx, float* v, float* mo,
             long long N, int H, int W, int C, int Nc, const CfBnBwd& bb, float* bnpart,
             long long bnpart_floats, const float* addend, float* D, hipStream_t s,
             const WgSrc* src, const WgOut* rider) {
  const int kind = src ? 2 : 0;
  constexpr int AA = Wg<M>::A * Wg<M>::A;
  const long long tiles = wg_tiles(M, N, H, W);
  // m = 4: U <- transform of the rotated kernel, in the input launch; m = 2: the forward's U,
  // read flipped.  Mo'[xi][tile][c] = sum_n V'[xi][tile][n] U'[xi][n][c]
  if constexpr (M == 4)
    wg_input<M, true>(dy, v, N, H, W, Nc, s, w, U, Nc, C, D, src, kind, rider);
  else
    wg_input<M, false>(dy, v, N, H, W, Nc, s, nullptr, nullptr, 0, 0, D, src, kind, rider);
  ew_cf_gemm_batched(v, U, mo, (int)tiles, C, Nc, AA, tiles * Nc, (long long)Nc * C, tiles * C,
                     false, M == 2, s);
  return wg_output<M>(mo, dx, N, H, W, C, bnpart, bnpart_floats, bb, addend, s);
}

template <int M>
int wino_wgrad(const float* dy, const float* V, float* dw, float* d, int d_ready, float* du,
               float* ws, long long ws_floats, long long N, int H, int W, int C, int Nc,
               int defer_out, hipStream_t s) {
  constexpr int A = Wg<M>::A, VW = Wg<M>::VW;
  const long long tiles = wg_tiles(M, N, H, W);
  if (!d_ready) {
    const long long n = tiles * (Nc / VW);
    hipLaunchKernelGGL(k_wg_dy<M>, dim3((unsigned)((n + EW_BLOCK - 1) / EW_BLOCK)),
                       dim3(EW_BLOCK), 0, s, dy, d, H, W, Nc, tiles);
    EW_CHECK_LAUNCH();
  }
  const int split = ew_cf_gemm_tn_batched(d, V, du, ws, ws_floats, Nc, C, (int)tiles, A * A,
                                          tiles * Nc, tiles * C, s);
  if (defer_out) return split;  // the caller runs the output transform (src: split > 1 ? ws : du)
  const long long m = (long long)Nc * (C / VW);
  hipLaunchKernelGGL(k_wg_wgrad_out<M>, dim3((unsigned)((m + EW_BLOCK - 1) / EW_BLOCK)),
                     dim3(EW_BLOCK), 0, s, split > 1 ? ws : du, split, dw, Nc, C);
  EW_CHECK_LAUNCH();
  return split;
}

}  // namespace

void ew_wino_f32_weight(uintptr_t w, uintptr_t U, int Nc, int C, int m, uintptr_t stream) {
  const int vw = m == 2 ? WG2_VW : 2;
  if ((m != 2 && m != 4) || C % vw || Nc <= 0)
    throw std::runtime_error("ewdml winograd f32: weight needs m in {2, 4}, C % 4 == 0");
  const long long n = (long long)Nc * (C / vw);
  const dim3 grid((unsigned)((n + EW_BLOCK - 1) / EW_BLOCK));
  const float* wp = reinterpret_cast<const float*>(w);
  float* up = reinterpret_cast<float*>(U);
  if (m == 2)
    hipLaunchKernelGGL(k_wg_weight<2>, grid, dim3(EW_BLOCK), 0, (hipStream_t)stream, wp, up, Nc, C);
  else
    hipLaunchKernelGGL(k_wg_weight<4>, grid, dim3(EW_BLOCK), 0, (hipStream_t)stream, wp, up, Nc, C);
  EW_CHECK_LAUNCH();
}

int ew_wino_f32_fwd(uintptr_t x, uintptr_t w, uintptr_t U, uintptr_t y, uintptr_t V, uintptr_t Mo,
                    long long N, int H, int W, int C, int Nc, int m, uintptr_t bnpart,
                    long long bnpart_floats, uintptr_t stream) {
  wg_check(m, N, H, W, C, Nc, "forward");
  auto* f = m == 2 ? wino_fwd<2> : wino_fwd<4>;
  return f(reinterpret_cast<const float*>(x), reinterpret_cast<const float*>(w),
           reinterpret_cast<float*>(U), reinterpret_cast<float*>(y), reinterpret_cast<float*>(V),
           reinterpret_cast<float*>(Mo), N, H, W, C, Nc, reinterpret_cast<float*>(bnpart),
           bnpart_floats, (hipStream_t)stream, nullptr);
}

// The forward whose input is the BatchNorm(+ReLU)(+pool) of bn_h, applied in the input transform
// (WgSrc KIND 1): bn_stats [4][C] of that layer, bn_code its pool codes (written here), nbt its
// num_batches_tracked (nullable).  H, W: this conv's (pooled) resolution.
int ew_wino_f32_fwd_bn(uintptr_t bn_h, uintptr_t bn_stats, uintptr_t bn_code, uintptr_t nbt,
                       int pool, uintptr_t w, uintptr_t U, uintptr_t y, uintptr_t V,
                       uintptr_t Mo, long long N, int H, int W, int C, int Nc, int m,
                       uintptr_t bnpart, long long bnpart_floats, uintptr_t stream) {
  wg_check(m, N, H, W, C, Nc, "forward");
  if (pool && !bn_code) throw std::runtime_error("ewdml winograd f32: pooled input needs codes");
  const WgSrc src{reinterpret_cast<const float*>(bn_h), reinterpret_cast<const float*>(bn_stats),
                  reinterpret_cast<uint8_t*>(bn_code), nullptr, nullptr,
                  reinterpret_cast<long long*>(nbt), pool};
  auto* f = m == 2 ? wino_fwd<2> : wino_fwd<4>;
  return f(nullptr, reinterpret_cast<const float*>(w), reinterpret_cast<float*>(U),
           reinterpret_cast<float*>(y), reinterpret_cast<float*>(V), reinterpret_cast<float*>(Mo),
           N, H, W, C, Nc, reinterpret_cast<float*>(bnpart), bnpart_floats, (hipStream_t)stream,
           &src);
}

// m = 2: U is the forward's transformed weight (read flipped; w unused); m = 4: U receives the
// rotated kernel's transform of w here
// wo_*: another layer's deferred weight-gradient output transform (ew_wino_f32_wgrad defer_out,
// same m) run in this call's input launch; wo_src 0 = none
static WgOut wg_rider(uintptr_t src, int split, uintptr_t dw, int Nc, int C, int m) {
  const int vw = m == 2 ? WG2_VW : 2;
  if (src && (!dw || split < 1 || Nc <= 0 || C % vw))
    throw std::runtime_error("ewdml winograd f32: bad riding weight-gradient output transform");
  return WgOut{reinterpret_cast<const float*>(src), reinterpret_cast<float*>(dw), split, Nc, C};
}

int ew_wino_f32_bwd_data(uintptr_t dy, uintptr_t w, uintptr_t U, uintptr_t dx, uintptr_t V,
                         uintptr_t Mo, long long N, int H, int W, int C, int Nc, int m,
                         uintptr_t bn_h, uintptr_t bn_res, uintptr_t bn_code, uintptr_t bn_stats,
                         int bn_relu, uintptr_t bnpart, long long bnpart_floats,
                         uintptr_t addend, uintptr_t D, uintptr_t wo_src, int wo_split,
                         uintptr_t wo_dw, int wo_Nc, int wo_C, uintptr_t stream) {
  const WgOut rider = wg_rider(wo_src, wo_split, wo_dw, wo_Nc, wo_C, m);
  wg_check(m, N, H, W, Nc, C, "backward data");
  if (m == 4 && !w) throw std::runtime_error("ewdml winograd f32: m = 4 backward needs w");
  const CfBnBwd bb{reinterpret_cast<const float*>(bn_h), reinterpret_cast<const float*>(bn_res),
                   reinterpret_cast<const uint8_t*>(bn_code),
                   reinterpret_cast<const float*>(bn_stats), bn_relu, H, W};
  auto* f = m == 2 ? wino_bwd<2> : wino_bwd<4>;
  // D != 0: the weight gradient's dMo from the same reads (ew_wino_f32_wgrad d_ready)
  return f(reinterpret_cast<const float*>(dy), reinterpret_cast<const float*>(w),
           reinterpret_cast<float*>(U), reinterpret_cast<float*>(dx), reinterpret_cast<float*>(V),
           reinterpret_cast<float*>(Mo), N, H, W, C, Nc, bb,
           bn_h ? reinterpret_cast<float*>(bnpart) : nullptr, bnpart_floats,
           reinterpret_cast<const float*>(addend), reinterpret_cast<float*>(D),
           (hipStream_t)stream, nullptr, &rider);
}

// Backward data whose dy is the BatchNorm(+ReLU)(+pool) backward of this conv's output, formed in
// the input transform (WgSrc KIND 2): out_h = this conv's output (that BN layer's input),
// out_dnext = the gradient of the BN layer's (pooled) output, out_code its pool codes,
// out_stats [4][Nc] / out_coef [2][Nc] (e, f) of that layer.  Otherwise ew_wino_f32_bwd_data.
int ew_wino_f32_bwd_data_bn(uintptr_t out_h, uintptr_t out_dnext, uintptr_t out_code,
                            uintptr_t out_stats, uintptr_t out_coef, int out_pool, uintptr_t w,
                            uintptr_t U, uintptr_t dx, uintptr_t V, uintptr_t Mo, long long N,
                            int H, int W, int C, int Nc, int m, uintptr_t bn_h, uintptr_t bn_res,
                            uintptr_t bn_code, uintptr_t bn_stats, int bn_relu, uintptr_t bnpart,
                            long long bnpart_floats, uintptr_t addend, uintptr_t D,
                            uintptr_t wo_src, int wo_split, uintptr_t wo_dw, int wo_Nc, int wo_C,
                            uintptr_t stream) {
  const WgOut rider = wg_rider(wo_src, wo_split, wo_dw, wo_Nc, wo_C, m);
  wg_check(m, N, H, W, Nc, C, "backward data");
  if (m == 4 && !w) throw std::runtime_error("ewdml winograd f32: m = 4 backward needs w");
  if (out_pool && (H % 2 || W % 2 || !out_code))
    throw std::runtime_error("ewdml winograd f32: pooled BN backward needs even maps and codes");
  const WgSrc src{reinterpret_cast<const float*>(out_h), reinterpret_cast<const float*>(out_stats),
                  reinterpret_cast<uint8_t*>(out_code), reinterpret_cast<const float*>(out_coef),
                  reinterpret_cast<const float*>(out_dnext), nullptr, out_pool};
  const CfBnBwd bb{reinterpret_cast<const float*>(bn_h), reinterpret_cast<const float*>(bn_res),
                   reinterpret_cast<const uint8_t*>(bn_code),
                   reinterpret_cast<const float*>(bn_stats), bn_relu, H, W};
  auto* f = m == 2 ? wino_bwd<2> : wino_bwd<4>;
  return f(nullptr, reinterpret_cast<const float*>(w), reinterpret_cast<float*>(U),
           reinterpret_cast<float*>(dx), reinterpret_cast<float*>(V), reinterpret_cast<float*>(Mo),
           N, H, W, C, Nc, bb, bn_h ? reinterpret_cast<float*>(bnpart) : nullptr, bnpart_floats,
           reinterpret_cast<const float*>(addend), reinterpret_cast<float*>(D),
           (hipStream_t)stream, &src, &rider);
}

// dw (channels_last [Nc][3][3][C]) from dy and the forward's V; D: a^2 * tiles * Nc floats;
// ws: K-split slabs (the plan uses what fits, ws_floats - 64 of it)
// defer_out: skip the output transform dw = G^T dU G and return the split count; the caller runs
// it later (ew_wino_f32_wgrad_out, or riding in a backward-data input launch) from
// split > 1 ? ws : U_scratch, which it keeps alive until then
int ew_wino_f32_wgrad(uintptr_t dy, uintptr_t V, uintptr_t dw, uintptr_t D, int d_ready,
                      uintptr_t U_scratch, uintptr_t ws, long long ws_floats, long long N, int H,
                      int W, int C, int Nc, int m, int defer_out, uintptr_t stream) {
  wg_check(m, N, H, W, C, Nc, "weight gradient");
  if (C % 64) throw std::runtime_error("ewdml winograd f32: weight gradient needs C % 64 == 0");
  auto* f = m == 2 ? wino_wgrad<2> : wino_wgrad<4>;
  return f(reinterpret_cast<const float*>(dy), reinterpret_cast<const float*>(V),
           reinterpret_cast<float*>(dw), reinterpret_cast<float*>(D), d_ready,
           reinterpret_cast<float*>(U_scratch), reinterpret_cast<float*>(ws), ws_floats, N, H, W,
           C, Nc, defer_out, (hipStream_t)stream);
}

void ew_wino_f32_wgrad_out(uintptr_t src, int split, uintptr_t dw, int Nc, int C, int m,
                           uintptr_t stream) {
  const WgOut wo = wg_rider(src, split, dw, Nc, C, m);
  if (!wo.src) return;
  const int vw = m == 2 ? WG2_VW : 2;
  const long long n = (long long)Nc * (C / vw);
  const dim3 grid((unsigned)((n + EW_BLOCK - 1) / EW_BLOCK));
  if (m == 2)
    hipLaunchKernelGGL(k_wg_wgrad_out<2>, grid, dim3(EW_BLOCK), 0, (hipStream_t)stream, wo.src,
                       wo.nsplit, wo.dw, Nc, C);
  else
    hipLaunchKernelGGL(k_wg_wgrad_out<4>, grid, dim3(EW_BLOCK), 0, (hipStream_t)stream, wo.src,
                       wo.nsplit, wo.dw, Nc, C);
  EW_CHECK_LAUNCH();
}
