// fp32 3x3 (pad 1, stride 1) convolutions by Winograd F(2x2, 3x3): forward and backward-data.
//
// Each 2x2 output tile is A^T [ (G g G^T) .* (B^T d B) ] A over the 4x4 input patch d, so the
// 9-tap implicit GEMM of conv_f32.hip (2*P*C*Nc*9 FLOPs) becomes 16 batched GEMMs over the
// tiles (2*(P/4)*16*C*Nc FLOPs, 2.25x fewer):
//
//   U[xi][Nc][C]    = (G g G^T)[xi]           weight transform, once per step
//   V[xi][tiles][C] = (B^T d B)[xi]           input transform (one launch for both: k_wg_input)
//   Mo[xi][tiles][Nc] = V[xi] U[xi]^T          16 fp32 MFMA GEMMs (conv_f32.hip k_cf_gemm, batched)
//   y = A^T Mo A                              output transform (k_wg_output), with the BatchNorm
//                                             partial sums (forward) or the producing BN layer's
//                                             backward sums + residual addend (backward data)
//
// Backward data is the same pipeline on dy with the 180-degree-rotated kernel and the channel
// roles swapped; since G J = P G (J: column reversal, P: rows 0 <-> 3), its transformed weight is
// the forward U read transposed with positions (i, j) -> (p(i), p(j)): no second weight
// transform, the GEMM reads U[p(xi)] as a [K = Nc][N = C] image (CfGeom::b_flip).
//
// B^T = [1 0 -1 0; 0 1 1 0; 0 -1 1 0; 0 1 0 -1], G = [1 0 0; .5 .5 .5; .5 -.5 .5; 0 0 1],
// A^T = [1 1 1 0; 0 1 -1 -1].  All arithmetic fp32 (the transforms add/subtract; G halves):
// the result differs from the direct convolution by rounding only (tests/kernels/test_conv_f32.py
// checks both against float64).
//
// Why unfused transforms: on the deep VGG / ResNet layers (C >= 128, maps <= 16x16) the GEMM
// dominates and V / Mo (4x the activations) stay in the 256 MB MALL; ops/conv.py only routes a
// layer here where that holds (the per-layer choice is measured: tools/conv_f32_probe.py --wino).
#include <stdexcept>

#include "common.h"
#include "conv_f32.h"
#include "ewdml_ops.h"

int ew_cf_gemm_tn_batched(const float* a, const float* b, float* out, float* ws,
                          long long ws_floats, int M, int N, int K, int batch, long long a_bs,
                          long long b_bs, hipStream_t s);
void ew_cf_gemm_batched(const float* a, const float* b, float* out, int M, int N, int K, int batch,
                        long long a_bs, long long b_bs, long long o_bs, bool nt, bool flip,
                        hipStream_t s);

namespace {

typedef float f32x4 __attribute__((ext_vector_type(4)));

// U[xi][o][i..i+3] = (G g G^T)[xi], g(r, s) = w[o][r][s][i..i+3] (channels_last [Nc][3][3][C])
__device__ __forceinline__ void wg_weight(const float* __restrict__ w, float* __restrict__ U,
                                          int Nc, int C, long long g) {
  const int cq = C >> 2;
  if (g >= (long long)Nc * cq) return;
  const int o = (int)(g / cq), i = (int)(g - (long long)o * cq) * 4;
  f32x4 k[3][3];
#pragma unroll
  for (int r = 0; r < 3; ++r)
#pragma unroll
    for (int s = 0; s < 3; ++s)
      k[r][s] = *reinterpret_cast<const f32x4*>(w + ((long long)o * 9 + r * 3 + s) * C + i);
  f32x4 t[4][3];  // G g
#pragma unroll
  for (int s = 0; s < 3; ++s) {
    t[0][s] = k[0][s];
    t[1][s] = 0.5f * (k[0][s] + k[1][s] + k[2][s]);
    t[2][s] = 0.5f * (k[0][s] - k[1][s] + k[2][s]);
    t[3][s] = k[2][s];
  }
  const long long xs = (long long)Nc * C;
  float* u = U + (long long)o * C + i;
#pragma unroll
  for (int r = 0; r < 4; ++r) {  // (G g) G^T
    *reinterpret_cast<f32x4*>(u + (r * 4 + 0) * xs) = t[r][0];
    *reinterpret_cast<f32x4*>(u + (r * 4 + 1) * xs) = 0.5f * (t[r][0] + t[r][1] + t[r][2]);
    *reinterpret_cast<f32x4*>(u + (r * 4 + 2) * xs) = 0.5f * (t[r][0] - t[r][1] + t[r][2]);
    *reinterpret_cast<f32x4*>(u + (r * 4 + 3) * xs) = t[r][2];
  }
}

// V[xi][tile][c..c+3] = (B^T d B)[xi], d = the 4x4 patch at (2 ty - 1, 2 tx - 1) of x[N][H][W][C]
// (zero outside).  Thread: one tile x one channel quad; consecutive threads, consecutive quads.
__device__ __forceinline__ void wg_dy_store(float* __restrict__ D, long long xs, f32x4 d00,
                                            f32x4 d01, f32x4 d10, f32x4 d11);

// (with D: also the weight-gradient transform A dy A^T of the patch's inner 2x2, see k_wg_dy)
__device__ __forceinline__ void wg_input(const float* __restrict__ x, float* __restrict__ V,
                                         int H, int W, int C, long long tiles, long long g,
                                         float* __restrict__ D = nullptr) {
  const int cq = C >> 2;
  if (g >= tiles * cq) return;
  const long long tl = g / cq;
  const int c = (int)(g - tl * cq) * 4;
  const int tw = W >> 1, tpi = (H >> 1) * tw;
  const int n = (int)(tl / tpi), rem = (int)(tl - (long long)n * tpi);
  const int ty = rem / tw, tx = rem - ty * tw;
  const int h0 = 2 * ty - 1, w0 = 2 * tx - 1;
  f32x4 d[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int h = h0 + i, w = w0 + j;
      const bool ok = (unsigned)h < (unsigned)H && (unsigned)w < (unsigned)W;
      const f32x4 v = *reinterpret_cast<const f32x4*>(
          x + (ok ? (((long long)n * H + h) * W + w) * C + c : c));
      d[i][j] = ok ? v : f32x4{0.0f, 0.0f, 0.0f, 0.0f};
    }
  if (D) wg_dy_store(D + tl * C + c, tiles * C, d[1][1], d[1][2], d[2][1], d[2][2]);
  f32x4 t[4][4];  // B^T d
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    t[0][j] = d[0][j] - d[2][j];
    t[1][j] = d[1][j] + d[2][j];
    t[2][j] = d[2][j] - d[1][j];
    t[3][j] = d[1][j] - d[3][j];
  }
  const long long xs = tiles * C;
  float* v = V + tl * C + c;
#pragma unroll
  for (int i = 0; i < 4; ++i) {  // (B^T d) B
    *reinterpret_cast<f32x4*>(v + (i * 4 + 0) * xs) = t[i][0] - t[i][2];
    *reinterpret_cast<f32x4*>(v + (i * 4 + 1) * xs) = t[i][1] + t[i][2];
    *reinterpret_cast<f32x4*>(v + (i * 4 + 2) * xs) = t[i][2] - t[i][1];
    *reinterpret_cast<f32x4*>(v + (i * 4 + 3) * xs) = t[i][1] - t[i][3];
  }
}

// the input transform over blocks [0, nbi) and, when w is given, the weight transform over the
// rest (one launch for both: each alone is a few-microsecond kernel)
__global__ __launch_bounds__(EW_BLOCK) void k_wg_input(const float* __restrict__ x,
                                                       float* __restrict__ V, int H, int W, int C,
                                                       long long tiles, int nbi,
                                                       const float* __restrict__ w,
                                                       float* __restrict__ U, int Nc,
                                                       float* __restrict__ D) {
  if ((int)blockIdx.x < nbi)
    wg_input(x, V, H, W, C, tiles, (long long)blockIdx.x * EW_BLOCK + threadIdx.x, D);
  else
    wg_weight(w, U, Nc, C, (long long)(blockIdx.x - nbi) * EW_BLOCK + threadIdx.x);
}

__global__ __launch_bounds__(EW_BLOCK) void k_wg_weight(const float* __restrict__ w,
                                                        float* __restrict__ U, int Nc, int C) {
  wg_weight(w, U, Nc, C, (long long)blockIdx.x * EW_BLOCK + threadIdx.x);
}

// y = A^T Mo A per tile (+ addend), with the BatchNorm partial sums of y (forward: sum, sum of
// squares; backward: CfBnBwd's sum dz, sum dz * (h - mean)) -> row blockIdx.x of bnpart[2][nb][Nc].
// Block: tiles [b * tpb, (b + 1) * tpb) x all Nc channels; thread: channel quad t % (Nc / 4),
// tiles t / (Nc / 4) + k * rpi (rpi = 256 / (Nc / 4) tiles per pass, Nc a power of two <= 1024).
__global__ __launch_bounds__(EW_BLOCK) void k_wg_output(const float* __restrict__ Mo,
                                                        float* __restrict__ y, int H, int W,
                                                        int Nc, long long tiles, int tpb,
                                                        float* __restrict__ bnpart, CfBnBwd bb,
                                                        const float* __restrict__ addend) {
  __shared__ float red[2][EW_BLOCK * 4];
  const int tpr = Nc >> 2, rpi = EW_BLOCK / tpr;
  const int t = threadIdx.x, rg = t / tpr, c0 = (t - rg * tpr) * 4;
  const long long t0 = (long long)blockIdx.x * tpb;
  const long long t1 = t0 + tpb < tiles ? t0 + tpb : tiles;
  const int tw = W >> 1, tpi = (H >> 1) * tw;
  const long long xs = tiles * Nc;
  const uint32_t HoWo = (uint32_t)bb.Ho * bb.Wo;
  float s1[4], s2[4], mean[4], sc[4], sh[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) s1[j] = s2[j] = 0.0f;
  if (bnpart && bb.h) {
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      mean[j] = bb.stats[c0 + j];
      sc[j] = bb.stats[2 * Nc + c0 + j];
      sh[j] = bb.stats[3 * Nc + c0 + j];
    }
  }
  for (long long tl = t0 + rg; tl < t1; tl += rpi) {
    const float* mp = Mo + tl * Nc + c0;
    f32x4 m[16];
#pragma unroll
    for (int q = 0; q < 16; ++q) m[q] = *reinterpret_cast<const f32x4*>(mp + q * xs);
    f32x4 u[2][4];  // A^T Mo
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      u[0][j] = m[j] + m[4 + j] + m[8 + j];
      u[1][j] = m[4 + j] - m[8 + j] - m[12 + j];
    }
    f32x4 o[2][2];  // (A^T Mo) A
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      o[i][0] = u[i][0] + u[i][1] + u[i][2];
      o[i][1] = u[i][1] - u[i][2] - u[i][3];
    }
    const int n = (int)(tl / tpi), rem = (int)(tl - (long long)n * tpi);
    const int ty = rem / tw, tx = rem - ty * tw;
#pragma unroll
    for (int a = 0; a < 2; ++a)
#pragma unroll
      for (int b = 0; b < 2; ++b) {
        const long long r = ((long long)n * H + 2 * ty + a) * W + 2 * tx + b;
        const long long off = r * Nc + c0;
        f32x4 v = o[a][b];
        if (addend) v += *reinterpret_cast<const f32x4*>(addend + off);
        *reinterpret_cast<f32x4*>(y + off) = v;
        if (!bnpart) continue;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const float dv = v[j];
          if (bb.h) {
            uint32_t hr = (uint32_t)r;
            if (bb.code) hr = cf_pool_row((uint32_t)r, HoWo, (uint32_t)bb.Wo, bb.code[off + j]);
            const float xh = bb.h[(size_t)hr * Nc + c0 + j];
            float z = xh * sc[j] + sh[j];
            if (bb.res) z = z + bb.res[(size_t)hr * Nc + c0 + j];
            const float dz = (bb.relu == 0 || !(z <= 0.0f)) ? dv : 0.0f;
            s1[j] += dz;
            s2[j] += dz * (xh - mean[j]);
          } else {
            s1[j] += dv;
            s2[j] += dv * dv;
          }
        }
      }
  }
  if (!bnpart) return;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    red[0][rg * Nc + c0 + j] = s1[j];
    red[1][rg * Nc + c0 + j] = s2[j];
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

// Weight gradient, the transpose of the forward: dMo = A dy A^T per tile and channel
// (k_wg_dy), dU[xi][Nc][C] = sum over tiles of dMo[xi][tile][Nc] V[xi][tile][C] (the forward's V,
// kept for the backward; one K = tiles GEMM per position, K-split into slabs), then
// dw = G^T dU G summed over the splits in a fixed order (k_wg_wgrad_out).
// A = [1 0; 1 1; 1 -1; 0 -1], G^T = [1 .5 .5 0; 0 .5 -.5 0; 0 .5 .5 1].
__global__ __launch_bounds__(EW_BLOCK) void k_wg_dy(const float* __restrict__ dy,
                                                    float* __restrict__ D, int H, int W, int Nc,
                                                    long long tiles) {
  const int cq = Nc >> 2;
  const long long g = (long long)blockIdx.x * EW_BLOCK + threadIdx.x;
  if (g >= tiles * cq) return;
  const long long tl = g / cq;
  const int c = (int)(g - tl * cq) * 4;
  const int tw = W >> 1, tpi = (H >> 1) * tw;
  const int n = (int)(tl / tpi), rem = (int)(tl - (long long)n * tpi);
  const int ty = rem / tw, tx = rem - ty * tw;
  const float* p = dy + (((long long)n * H + 2 * ty) * W + 2 * tx) * Nc + c;
  wg_dy_store(D + tl * Nc + c, tiles * Nc, *reinterpret_cast<const f32x4*>(p),
              *reinterpret_cast<const f32x4*>(p + Nc),
              *reinterpret_cast<const f32x4*>(p + (long long)W * Nc),
              *reinterpret_cast<const f32x4*>(p + (long long)W * Nc + Nc));
}

__device__ __forceinline__ void wg_dy_store(float* __restrict__ o, long long xs, f32x4 d00,
                                            f32x4 d01, f32x4 d10, f32x4 d11) {
  f32x4 t[4][2];  // A dy
  t[0][0] = d00;
  t[0][1] = d01;
  t[1][0] = d00 + d10;
  t[1][1] = d01 + d11;
  t[2][0] = d00 - d10;
  t[2][1] = d01 - d11;
  t[3][0] = -d10;
  t[3][1] = -d11;
#pragma unroll
  for (int i = 0; i < 4; ++i) {  // (A dy) A^T
    *reinterpret_cast<f32x4*>(o + (i * 4 + 0) * xs) = t[i][0];
    *reinterpret_cast<f32x4*>(o + (i * 4 + 1) * xs) = t[i][0] + t[i][1];
    *reinterpret_cast<f32x4*>(o + (i * 4 + 2) * xs) = t[i][0] - t[i][1];
    *reinterpret_cast<f32x4*>(o + (i * 4 + 3) * xs) = -t[i][1];
  }
}

// dw[o][r][s][i..i+3] = (G^T (sum_z dU_z[xi]) G)[r][s], dU_z = src + z * 16 * Nc * C
__global__ __launch_bounds__(EW_BLOCK) void k_wg_wgrad_out(const float* __restrict__ src,
                                                           int nsplit, float* __restrict__ dw,
                                                           int Nc, int C) {
  const int cq = C >> 2;
  const long long g = (long long)blockIdx.x * EW_BLOCK + threadIdx.x;
  if (g >= (long long)Nc * cq) return;
  const int o = (int)(g / cq), i = (int)(g - (long long)o * cq) * 4;
  const long long xs = (long long)Nc * C;
  const float* p = src + (long long)o * C + i;
  f32x4 u[16];
#pragma unroll
  for (int q = 0; q < 16; ++q) u[q] = *reinterpret_cast<const f32x4*>(p + q * xs);
  for (int z = 1; z < nsplit; ++z) {  // fixed order
    const float* pz = p + (long long)z * 16 * xs;
#pragma unroll
    for (int q = 0; q < 16; ++q) u[q] += *reinterpret_cast<const f32x4*>(pz + q * xs);
  }
  f32x4 t[3][4];  // G^T dU
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    t[0][j] = u[j] + 0.5f * (u[4 + j] + u[8 + j]);
    t[1][j] = 0.5f * (u[4 + j] - u[8 + j]);
    t[2][j] = 0.5f * (u[4 + j] + u[8 + j]) + u[12 + j];
  }
  float* w = dw + (long long)o * 9 * C + i;
#pragma unroll
  for (int r = 0; r < 3; ++r) {  // (G^T dU) G
    *reinterpret_cast<f32x4*>(w + (r * 3 + 0) * C) = t[r][0] + 0.5f * (t[r][1] + t[r][2]);
    *reinterpret_cast<f32x4*>(w + (r * 3 + 1) * C) = 0.5f * (t[r][1] - t[r][2]);
    *reinterpret_cast<f32x4*>(w + (r * 3 + 2) * C) = 0.5f * (t[r][1] + t[r][2]) + t[r][3];
  }
}

long long wg_tiles(long long N, int H, int W) { return N * (H / 2) * (W / 2); }

void wg_check(long long N, int H, int W, int Cin, int Cout, const char* what) {
  const long long tiles = wg_tiles(N, H, W);
  const bool pow2 = Cout >= 4 && Cout <= 1024 && (Cout & (Cout - 1)) == 0;
  if (H % 2 || W % 2 || tiles % 64 || Cin % 32 || Cout % 64 || !pow2 ||
      16 * tiles * (long long)std::max(Cin, Cout) >= (1LL << 31))
    throw std::runtime_error(std::string("ewdml winograd f32 ") + what +
                             ": needs even H, W, N*H*W/4 % 64 == 0, C_in % 32 == 0, C_out a "
                             "power of two in [64, 1024]");
}

// output transform launch: returns the BN partial rows written (0: none requested / no room)
int wg_output(const float* Mo, float* y, long long N, int H, int W, int Nc, float* bnpart,
              long long bnpart_floats, const CfBnBwd& bb, const float* addend, hipStream_t s) {
  const long long tiles = wg_tiles(N, H, W);
  const int rpi = EW_BLOCK / (Nc / 4);
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
  hipLaunchKernelGGL(k_wg_output, dim3((unsigned)nblk), dim3(EW_BLOCK), 0, s, Mo, y, H, W, Nc,
                     tiles, (int)tpb, bnpart, bb, addend);
  EW_CHECK_LAUNCH();
  return bnpart ? (int)nblk : 0;
}

// input transform of x [N][H][W][C] into V; with w, also U[16][Nc][C] from w [Nc][3][3][C]
void wg_input(const float* x, float* V, long long N, int H, int W, int C, hipStream_t s,
              const float* w = nullptr, float* U = nullptr, int Nc = 0, float* D = nullptr) {
  const long long n = wg_tiles(N, H, W) * (C / 4);
  const int nbi = (int)((n + EW_BLOCK - 1) / EW_BLOCK);
  const int nbw = w ? (int)(((long long)Nc * (C / 4) + EW_BLOCK - 1) / EW_BLOCK) : 0;
  hipLaunchKernelGGL(k_wg_input, dim3(nbi + nbw), dim3(EW_BLOCK), 0, s, x, V, H, W, C,
                     wg_tiles(N, H, W), nbi, w, U, Nc, D);
  EW_CHECK_LAUNCH();
}

}  // namespace

void ew_wino_f32_weight(uintptr_t w, uintptr_t U, int Nc, int C, uintptr_t stream) {
  if (C % 4 || Nc <= 0) throw std::runtime_error("ewdml winograd f32: weight needs C % 4 == 0");
  const long long n = (long long)Nc * (C / 4);
  hipLaunchKernelGGL(k_wg_weight, dim3((unsigned)((n + EW_BLOCK - 1) / EW_BLOCK)), dim3(EW_BLOCK),
                     0, (hipStream_t)stream, reinterpret_cast<const float*>(w),
                     reinterpret_cast<float*>(U), Nc, C);
  EW_CHECK_LAUNCH();
}

int ew_wino_f32_fwd(uintptr_t x, uintptr_t w, uintptr_t U, uintptr_t y, uintptr_t V, uintptr_t Mo,
                    long long N, int H, int W, int C, int Nc, uintptr_t bnpart,
                    long long bnpart_floats, uintptr_t stream) {
  wg_check(N, H, W, C, Nc, "forward");
  hipStream_t s = (hipStream_t)stream;
  const long long tiles = wg_tiles(N, H, W);
  float* v = reinterpret_cast<float*>(V);
  float* mo = reinterpret_cast<float*>(Mo);
  wg_input(reinterpret_cast<const float*>(x), v, N, H, W, C, s, reinterpret_cast<const float*>(w),
           reinterpret_cast<float*>(U), Nc);
  ew_cf_gemm_batched(v, reinterpret_cast<const float*>(U), mo, (int)tiles, Nc, C, 16, tiles * C,
                     (long long)Nc * C, tiles * Nc, true, false, s);
  const CfBnBwd none{nullptr, nullptr, nullptr, nullptr, 0, 0, 0};
  return wg_output(mo, reinterpret_cast<float*>(y), N, H, W, Nc, reinterpret_cast<float*>(bnpart),
                   bnpart_floats, none, nullptr, s);
}

int ew_wino_f32_bwd_data(uintptr_t dy, uintptr_t U, uintptr_t dx, uintptr_t V, uintptr_t Mo,
                         long long N, int H, int W, int C, int Nc, uintptr_t bn_h,
                         uintptr_t bn_res, uintptr_t bn_code, uintptr_t bn_stats, int bn_relu,
                         uintptr_t bnpart, long long bnpart_floats, uintptr_t addend,
                         uintptr_t D, uintptr_t stream) {
  wg_check(N, H, W, Nc, C, "backward data");
  hipStream_t s = (hipStream_t)stream;
  const long long tiles = wg_tiles(N, H, W);
  float* v = reinterpret_cast<float*>(V);
  float* mo = reinterpret_cast<float*>(Mo);
  // D != 0: the weight gradient's dy transform from the same reads (ew_wino_f32_wgrad d_ready)
  wg_input(reinterpret_cast<const float*>(dy), v, N, H, W, Nc, s, nullptr, nullptr, 0,
           reinterpret_cast<float*>(D));
  // Mo'[xi][tile][c] = sum_n V'[xi][tile][n] U[p(xi)][n][c]
  ew_cf_gemm_batched(v, reinterpret_cast<const float*>(U), mo, (int)tiles, C, Nc, 16, tiles * Nc,
                     (long long)Nc * C, tiles * C, false, true, s);
  const CfBnBwd bb{reinterpret_cast<const float*>(bn_h), reinterpret_cast<const float*>(bn_res),
                   reinterpret_cast<const uint8_t*>(bn_code),
                   reinterpret_cast<const float*>(bn_stats), bn_relu, H, W};
  return wg_output(mo, reinterpret_cast<float*>(dx), N, H, W, C,
                   bn_h ? reinterpret_cast<float*>(bnpart) : nullptr, bnpart_floats, bb,
                   reinterpret_cast<const float*>(addend), s);
}

// dw (channels_last [Nc][3][3][C]) from dy and the forward's V; D: 16 * tiles * Nc floats;
// ws: K-split slabs (the plan uses what fits, ws_floats - 64 of it)
void ew_wino_f32_wgrad(uintptr_t dy, uintptr_t V, uintptr_t dw, uintptr_t D, int d_ready,
                       uintptr_t U_scratch, uintptr_t ws, long long ws_floats, long long N, int H,
                       int W, int C, int Nc, uintptr_t stream) {
  wg_check(N, H, W, C, Nc, "weight gradient");
  if (C % 64) throw std::runtime_error("ewdml winograd f32: weight gradient needs C % 64 == 0");
  hipStream_t s = (hipStream_t)stream;
  const long long tiles = wg_tiles(N, H, W);
  float* d = reinterpret_cast<float*>(D);
  if (!d_ready) {
    const long long n = tiles * (Nc / 4);
    hipLaunchKernelGGL(k_wg_dy, dim3((unsigned)((n + EW_BLOCK - 1) / EW_BLOCK)), dim3(EW_BLOCK),
                       0, s, reinterpret_cast<const float*>(dy), d, H, W, Nc, tiles);
    EW_CHECK_LAUNCH();
  }
  float* du = reinterpret_cast<float*>(U_scratch);
  const int split = ew_cf_gemm_tn_batched(d, reinterpret_cast<const float*>(V), du,
                                          reinterpret_cast<float*>(ws), ws_floats, Nc, C,
                                          (int)tiles, 16, tiles * Nc, tiles * C, s);
  const long long m = (long long)Nc * (C / 4);
  hipLaunchKernelGGL(k_wg_wgrad_out, dim3((unsigned)((m + EW_BLOCK - 1) / EW_BLOCK)),
                     dim3(EW_BLOCK), 0, s, split > 1 ? reinterpret_cast<const float*>(ws) : du,
                     split, reinterpret_cast<float*>(dw), Nc, C);
  EW_CHECK_LAUNCH();
}
