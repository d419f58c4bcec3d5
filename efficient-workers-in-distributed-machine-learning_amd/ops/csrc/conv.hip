// 3x3 / stride 1 / pad 1 convolution as implicit GEMM on the gfx950 matrix cores (NHWC, bf16 in,
// fp32 accumulate), forward + backward-data + backward-weight.
//
// Why: VGG-11 on 32x32 inputs at batch 128 is a chain of small GEMM-shaped convolutions (M = N*H*W
// from 32768 down to 512 rows, K = 9*C up to 4608).  MIOpen runs them at 130-380 TF/s and its
// NHWC backward solvers add a zero-fill and an fp32->bf16 cast kernel per call (~115 us per
// training step, profiles/vgg11_bs128_fused_nhwc_graph.txt).  Here each direction is one MFMA
// kernel (+ one reduction kernel when the reduction is split to fill 256 CUs).
//
//   forward     y[m][n]  = sum_{k=(r,s,c)} X~[m][k] * w[n][k]        X~ = im2col(x), implicit
//   bwd data   dx[m][c]  = sum_{k=(r,s,n)} dY~[m][k] * w[n][2-r][2-s][c]
//   bwd weight dw[n][k]  = sum_m dy[m][n] * X~[m][k]
//
// The first two are "NT" GEMMs (both operands contiguous along the reduction): 16-byte chunks go
// global -> registers -> LDS (double buffered, one barrier per 64-deep k-step) and feed
// v_mfma_f32_16x16x32_bf16 through ds_read_b128.  The weight gradient reduces over m, which is
// the *slow* axis of both NHWC operands: each thread loads MR consecutive m rows x 8 channels,
// transposes them in registers (v_perm) and writes [row][m] images of the same layout, so the
// MFMA core is shared.  im2col is never materialised: a row's tap (r, s) is an offset of the
// pixel index, out-of-image taps load zeros.
//
// LDS image of an operand tile: [rows][64] bf16, 128-B rows, 16-B chunk c of row r at chunk
// c ^ ((r >> 1) & 7): the 16 rows a ds_read_b128 lane group fetches at one chunk land in 16
// distinct 16-B bank slots (conflict-free), and the 8 lanes of a ds_write_b128 group (one row)
// hit 8 distinct slots.
//
// Block = 256 threads = 4 waves in a 2 x 2 grid over the BM x BN output tile; wave tile
// (BM/2) x (BN/2) of 16 x 16 MFMA tiles.  C/D map of 16x16x32: col = lane & 15,
// row = 4 * (lane >> 4) + reg.
#include <cstdlib>

#include "common.h"
#include "ewdml_ops.h"

namespace {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

constexpr int CV_BK = 64;  // reduction depth of one k-step (one 128-B LDS row per operand row)

__device__ __forceinline__ int cv_off(int r, int c) {  // byte offset of chunk c of row r
  return r * 128 + ((c ^ ((r >> 1) & 7)) << 4);
}

// MFMA over one k-step: acc[i][j] += A[rows of wave][64] * B[cols of wave][64]^T
template <int MI, int NJ>
__device__ __forceinline__ void cv_mma(const char* __restrict__ As, const char* __restrict__ Bs,
                                       int arow0, int brow0, int lane, f32x4 (&acc)[MI][NJ]) {
#pragma unroll
  for (int kk = 0; kk < 2; ++kk) {
    const int ch = kk * 4 + (lane >> 4);
    bf16x8 a[MI], b[NJ];
#pragma unroll
    for (int i = 0; i < MI; ++i)
      a[i] = *reinterpret_cast<const bf16x8*>(As + cv_off(arow0 + i * 16 + (lane & 15), ch));
#pragma unroll
    for (int j = 0; j < NJ; ++j)
      b[j] = *reinterpret_cast<const bf16x8*>(Bs + cv_off(brow0 + j * 16 + (lane & 15), ch));
#pragma unroll
    for (int i = 0; i < MI; ++i)
#pragma unroll
      for (int j = 0; j < NJ; ++j)
        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[i], b[j], acc[i][j], 0, 0, 0);
  }
}

// Epilogue: bf16 output (ldo elements per row) or an fp32 split slab, straight from registers
// (16 consecutive columns = 32 B / 64 B per row segment).
template <int MI, int NJ>
__device__ __forceinline__ void cv_store(const f32x4 (&acc)[MI][NJ], int row0, int col0, int lane,
                                         uint16_t* __restrict__ out, float* __restrict__ slab,
                                         long long ldo) {
  const int c = col0 + (lane & 15);
#pragma unroll
  for (int i = 0; i < MI; ++i) {
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const long long r = row0 + i * 16 + 4 * (lane >> 4) + q;
#pragma unroll
      for (int j = 0; j < NJ; ++j) {
        if (slab) slab[r * ldo + c + j * 16] = acc[i][j][q];
        else out[r * ldo + c + j * 16] = ew_f2bf(acc[i][j][q]);
      }
    }
  }
}

// ---------------------------------------------------------------------------------------------
// Transposed-operand images (weight gradient, backward data): [64 k][64 cols], 128-B rows.
__device__ __forceinline__ int cv_trf(int r) { return (((r >> 1) & 1) << 1) | (((r >> 3) & 1) << 2); }
__device__ __forceinline__ int cv_toff(int r, int c) { return r * 128 + ((c ^ cv_trf(r)) << 4); }

typedef short cv_v4s __attribute__((ext_vector_type(4)));
typedef short cv_v8s __attribute__((ext_vector_type(8)));

__device__ __forceinline__ cv_v4s cv_tr_read(const char* p) {
  return __builtin_amdgcn_ds_read_tr16_b64_v4i16(
      (__attribute__((address_space(3))) cv_v4s*)(p));
}

// acc[i][j] += sum over the step's 64 m of A[m][acol0 + 16 i + .] * B[m][bcol0 + 16 j + .]
template <int MI, int NJ>
__device__ __forceinline__ void cv_mma_tr(const char* __restrict__ As, const char* __restrict__ Bs,
                                          int acol0, int bcol0, int lane,
                                          f32x4 (&acc)[MI][NJ]) {
  const int g = lane >> 4, li = lane & 15, q = li >> 2, p = li & 3;
#pragma unroll
  for (int kk = 0; kk < 2; ++kk) {
    const int r0 = kk * 32 + 8 * g + q;  // rows r0 (elements 0..3) and r0 + 4 (elements 4..7)
    bf16x8 a[MI], b[NJ];
#pragma unroll
    for (int i = 0; i < MI; ++i) {
      const int col = acol0 + i * 16 + 4 * p;
      const cv_v4s lo = cv_tr_read(As + cv_toff(r0, col >> 3) + (col & 7) * 2);
      const cv_v4s hi = cv_tr_read(As + cv_toff(r0 + 4, col >> 3) + (col & 7) * 2);
      a[i] = __builtin_bit_cast(bf16x8, __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7));
    }
#pragma unroll
    for (int j = 0; j < NJ; ++j) {
      const int col = bcol0 + j * 16 + 4 * p;
      const cv_v4s lo = cv_tr_read(Bs + cv_toff(r0, col >> 3) + (col & 7) * 2);
      const cv_v4s hi = cv_tr_read(Bs + cv_toff(r0 + 4, col >> 3) + (col & 7) * 2);
      b[j] = __builtin_bit_cast(bf16x8, __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7));
    }
#pragma unroll
    for (int i = 0; i < MI; ++i)
#pragma unroll
      for (int j = 0; j < NJ; ++j)
        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[i], b[j], acc[i][j], 0, 0, 0);
  }
}


// A fragments by ds_read_b128 from a [rows][64 k] image (cv_off), B fragments by transposed reads
// from a [64 k][cols] image (cv_toff): the backward-data GEMM, whose weight operand is stored
// with the reduction axis (the forward's output channel) slow.
template <int MI, int NJ>
__device__ __forceinline__ void cv_mma_mixed(const char* __restrict__ As,
                                             const char* __restrict__ Bs, int arow0, int bcol0,
                                             int lane, f32x4 (&acc)[MI][NJ]) {
  const int g = lane >> 4, li = lane & 15, q = li >> 2, p = li & 3;
#pragma unroll
  for (int kk = 0; kk < 2; ++kk) {
    const int ch = kk * 4 + g;
    const int r0 = kk * 32 + 8 * g + q;
    bf16x8 a[MI], b[NJ];
#pragma unroll
    for (int i = 0; i < MI; ++i)
      a[i] = *reinterpret_cast<const bf16x8*>(As + cv_off(arow0 + i * 16 + li, ch));
#pragma unroll
    for (int j = 0; j < NJ; ++j) {
      const int col = bcol0 + j * 16 + 4 * p;
      const cv_v4s lo = cv_tr_read(Bs + cv_toff(r0, col >> 3) + (col & 7) * 2);
      const cv_v4s hi = cv_tr_read(Bs + cv_toff(r0 + 4, col >> 3) + (col & 7) * 2);
      b[j] = __builtin_bit_cast(bf16x8, __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7));
    }
#pragma unroll
    for (int i = 0; i < MI; ++i)
#pragma unroll
      for (int j = 0; j < NJ; ++j)
        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[i], b[j], acc[i][j], 0, 0, 0);
  }
}

// Staging registers of one operand (2 or 4 rows x 16 B per thread), named members instead of an
// array: with arrays hipcc kept spilling the second staging set to scratch.
// (native vector type: HIP's uint4 struct copies lower to memcpy through a stack slot)
typedef unsigned cv_u4 __attribute__((ext_vector_type(4)));
template <int P>
struct CvRegs {
  static_assert(P == 2 || P == 4, "2 or 4 rows per thread");
  cv_u4 v0, v1, v2, v3;
};
#define CV_FOR_ROWS(P_, ...)                                                                    \
  do {                                                                                          \
    { constexpr int i = 0; cv_u4& v = R.v0; __VA_ARGS__; }                                      \
    { constexpr int i = 1; cv_u4& v = R.v1; __VA_ARGS__; }                                      \
    if constexpr (P_ > 2) {                                                                     \
      { constexpr int i = 2; cv_u4& v = R.v2; __VA_ARGS__; }                                    \
      { constexpr int i = 3; cv_u4& v = R.v3; __VA_ARGS__; }                                    \
    }                                                                                           \
  } while (0)

// ---------------------------------------------------------------------------------------------
// Both GEMM kernels run KG "k-groups" of 4 waves per block: group g takes the block's k-steps
// g, g + KG, g + 2 KG, ... into its own double-buffered LDS stages, all groups share one barrier
// per iteration, and at the end the groups' fp32 tiles are summed through LDS.  Small conv GEMMs
// are latency-bound (each k-step waits on one global-load round trip); KG groups put KG k-steps
// behind every round trip and KG x 4 waves on the CU, without the global traffic of a split-K
// reduction (which is used on top only when the output has fewer tiles than the chip has CUs).

// Sum the KG groups' accumulators into group 0's (LDS staging reused; call after a barrier).
template <int KG, int MI, int NJ>
__device__ __forceinline__ void cv_group_reduce(f32x4 (&acc)[MI][NJ], char* smem, int g, int wq,
                                                int lane) {
  if constexpr (KG > 1) {
    float* red = reinterpret_cast<float*>(smem);
    constexpr int PER = MI * NJ * 4 * 64;  // floats of one wave's accumulator
    if (g > 0) {
#pragma unroll
      for (int i = 0; i < MI; ++i)
#pragma unroll
        for (int j = 0; j < NJ; ++j)
#pragma unroll
          for (int q = 0; q < 4; ++q)
            red[((g - 1) * 4 + wq) * PER + ((i * NJ + j) * 4 + q) * 64 + lane] = acc[i][j][q];
    }
    __syncthreads();
    if (g == 0) {
#pragma unroll
      for (int gg = 1; gg < KG; ++gg)
#pragma unroll
        for (int i = 0; i < MI; ++i)
#pragma unroll
          for (int j = 0; j < NJ; ++j)
#pragma unroll
            for (int q = 0; q < 4; ++q)
              acc[i][j][q] += red[((gg - 1) * 4 + wq) * PER + ((i * NJ + j) * 4 + q) * 64 + lane];
    }
  }
}

// BatchNorm-backward statistics folded into a backward-data epilogue.  The launch produces the
// output gradient dy of a BN(+ReLU)(+2x2 max pool) layer L; with this set, the epilogue also sums,
// per channel c over its rows, dz = act'(h * scale + shift) * dy and dz * (h - mean) (the
// k_bn_bwd_stats quantities; sum(h - mean) is 0 up to rounding and is taken as 0), where h is
// layer L's BN input and, pooled, dy reaches the window position of the forward's argmax code.
// The BN backward then skips its statistics pass (ops/nn.py, ops/conv.py).
struct CvBnBwd {
  const uint16_t* h;      // layer L's BN input [rows (pre-pool)][C]; null: not requested
  const uint16_t* res;    // its residual input [rows][C] (BN + residual + ReLU), or null
  const uint8_t* code;    // pool window codes [rows][C] (null: no pool)
  const float* stats;     // [4][C]: mean, invstd, scale, shift
  int relu;               // 0: BN only
  int Ho, Wo;             // pooled map dims (pool)
};

// pre-pool row of window position q of pooled row p (nn.hip ew_pool_base / ew_pool_off)
__device__ __forceinline__ uint32_t cv_pool_row(uint32_t p, uint32_t HoWo, uint32_t Wo,
                                                uint32_t q) {
  const uint32_t n = p / HoWo, rem = p - n * HoWo;
  const uint32_t ho = rem / Wo, wo = rem - ho * Wo;
  return 4 * n * HoWo + 4 * ho * Wo + 2 * wo + (q >> 1) * (2 * Wo) + (q & 1);
}

// Epilogue of the NT kernels: fp32 split slab, or bf16 output + (optional) BatchNorm partial sums
// of the stored output (see k_conv_nt).  Every thread of the block calls it (barriers inside);
// only k-group 0 (g == 0) holds the reduced accumulators.
template <int BM, int BN, int MI, int NJ>
__device__ __forceinline__ void cv_nt_epilogue(f32x4 (&acc)[MI][NJ], char* smem, int g,
                                               int wm, int wn, int lane, int m0, int n0, int M,
                                               int Nc, uint16_t* __restrict__ out,
                                               float* __restrict__ slab,
                                               float* __restrict__ bnpart,
                                               const CvBnBwd& bb,
                                               const uint16_t* __restrict__ addend) {
  const int row0 = m0 + wm * (BM / 2), col0 = n0 + wn * (BN / 2);
  if (addend && !slab && g == 0) {
    // out = this GEMM + addend (a second gradient of the same tensor, e.g. the identity
    // residual's, so autograd does not add them in a separate kernel); loads first, then adds
    float av[MI][NJ][4];
#pragma unroll
    for (int i = 0; i < MI; ++i)
#pragma unroll
      for (int j = 0; j < NJ; ++j)
#pragma unroll
        for (int q = 0; q < 4; ++q)
          av[i][j][q] = __uint_as_float(
              (uint32_t)addend[(size_t)(row0 + i * 16 + 4 * (lane >> 4) + q) * Nc + col0 +
                               j * 16 + (lane & 15)] << 16);
#pragma unroll
    for (int i = 0; i < MI; ++i)
#pragma unroll
      for (int j = 0; j < NJ; ++j)
#pragma unroll
        for (int q = 0; q < 4; ++q) acc[i][j][q] += av[i][j][q];
  }
  if (slab) {
    if (g == 0)
      cv_store<MI, NJ>(acc, row0, col0, lane, nullptr, slab + (long long)blockIdx.z * M * Nc, Nc);
    return;
  }
  if (g == 0) cv_store<MI, NJ>(acc, row0, col0, lane, out, nullptr, Nc);
  if (bnpart) {  // every group keeps the barrier count; only group 0's values are used
    // BatchNorm statistics of the stored (bf16-rounded) output, fused into the epilogue: per
    // column, sum and sum of squares over the block's BM rows -> partial row blockIdx.x of
    // bnpart[2][M/BM][Nc] (the BN finalize kernel's layout).  The two waves sharing columns
    // (wm = 0, 1) combine through LDS.
    float* red = reinterpret_cast<float*>(smem);  // [wn][2][BN/2]
    const long long nrows = M / BM;
    float sm[NJ], sq[NJ];
    // BN-backward sums of layer L (see CvBnBwd), group 0 only: all window codes, then all h
    // values are loaded before any use (two load round trips, not one per element)
    float xv[NJ][MI][4], rv[NJ][MI][4];
    if (bb.h && g == 0) {
      const uint32_t HoWo = (uint32_t)bb.Ho * bb.Wo;
      uint32_t hr[NJ][MI][4];
#pragma unroll
      for (int j = 0; j < NJ; ++j)
#pragma unroll
        for (int i = 0; i < MI; ++i)
#pragma unroll
          for (int q = 0; q < 4; ++q) hr[j][i][q] = row0 + i * 16 + 4 * (lane >> 4) + q;
      if (bb.code) {
        uint8_t kc[NJ][MI][4];
#pragma unroll
        for (int j = 0; j < NJ; ++j)
#pragma unroll
          for (int i = 0; i < MI; ++i)
#pragma unroll
            for (int q = 0; q < 4; ++q)
              kc[j][i][q] = bb.code[(size_t)hr[j][i][q] * Nc + col0 + j * 16 + (lane & 15)];
#pragma unroll
        for (int j = 0; j < NJ; ++j)
#pragma unroll
          for (int i = 0; i < MI; ++i)
#pragma unroll
            for (int q = 0; q < 4; ++q)
              hr[j][i][q] = cv_pool_row(hr[j][i][q], HoWo, (uint32_t)bb.Wo, kc[j][i][q]);
      }
#pragma unroll
      for (int j = 0; j < NJ; ++j)
#pragma unroll
        for (int i = 0; i < MI; ++i)
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            const size_t o = (size_t)hr[j][i][q] * Nc + col0 + j * 16 + (lane & 15);
            xv[j][i][q] = __uint_as_float((uint32_t)bb.h[o] << 16);
            rv[j][i][q] = bb.res ? __uint_as_float((uint32_t)bb.res[o] << 16) : 0.0f;
          }
    }
#pragma unroll
    for (int j = 0; j < NJ; ++j) {
      sm[j] = sq[j] = 0.0f;
      if (bb.h) {
        if (g == 0) {
          const int c = col0 + j * 16 + (lane & 15);
          const float mean = bb.stats[c], sc = bb.stats[2 * Nc + c], sh = bb.stats[3 * Nc + c];
#pragma unroll
          for (int i = 0; i < MI; ++i)
#pragma unroll
            for (int q = 0; q < 4; ++q) {
              const float d = __uint_as_float((uint32_t)ew_f2bf(acc[i][j][q]) << 16);
              const float x = xv[j][i][q];
              float v = x * sc + sh;  // the BN kernels' exact arithmetic (no contraction)
              if (bb.res) v = v + rv[j][i][q];
              const float dz = (bb.relu == 0 || !(v <= 0.0f)) ? d : 0.0f;
              sm[j] += dz;
              sq[j] += dz * (x - mean);
            }
        }
      } else {
#pragma unroll
        for (int i = 0; i < MI; ++i)
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            const float v = __uint_as_float((uint32_t)ew_f2bf(acc[i][j][q]) << 16);
            sm[j] += v;
            sq[j] += v * v;
          }
      }
      sm[j] += __shfl_xor(sm[j], 16, 64);
      sq[j] += __shfl_xor(sq[j], 16, 64);
      sm[j] += __shfl_xor(sm[j], 32, 64);
      sq[j] += __shfl_xor(sq[j], 32, 64);
    }
    __syncthreads();  // group reduce / main loop finished reading smem
    if (g == 0 && wm == 1 && lane < 16) {
#pragma unroll
      for (int j = 0; j < NJ; ++j) {
        red[(wn * 2 + 0) * (BN / 2) + j * 16 + lane] = sm[j];
        red[(wn * 2 + 1) * (BN / 2) + j * 16 + lane] = sq[j];
      }
    }
    __syncthreads();
    if (g == 0 && wm == 0 && lane < 16) {
#pragma unroll
      for (int j = 0; j < NJ; ++j) {
        const int c = col0 + j * 16 + lane;
        bnpart[(long long)blockIdx.x * Nc + c] = sm[j] + red[(wn * 2 + 0) * (BN / 2) + j * 16 + lane];
        bnpart[(nrows + blockIdx.x) * Nc + c] = sq[j] + red[(wn * 2 + 1) * (BN / 2) + j * 16 + lane];
      }
    }
  }
}

// NT kernel (forward and backward-data).  x: [M][C] pixels of one NHWC tensor (M = N*H*W),
// w: [Nc][9*C] (tap-major, channel-minor), out: [M][Nc] bf16, or fp32 slabs [split][M][Nc].
// Split z covers k-steps [z*kps, min((z+1)*kps, ksteps)).  Requires C % 64 == 0, M % BM == 0,
// Nc % BN == 0 (checked on the host).
template <int BM, int BN, int KG, bool TRB>
__global__ __launch_bounds__(EW_BLOCK * KG) void k_conv_nt(const uint16_t* __restrict__ x,
                                                           const uint16_t* __restrict__ w,
                                                           uint16_t* __restrict__ out,
                                                           float* __restrict__ slab, int M, int H,
                                                           int W, int C, int Nc, int kps,
                                                           int taps, float* __restrict__ bnpart,
                                                           CvBnBwd bb,
                                                           const uint16_t* __restrict__ addend) {
  constexpr int PA = BM / 32, PB = BN / 32;   // 16-B vectors per thread per k-step
  constexpr int MI = BM / 32, NJ = BN / 32;   // 16x16 tiles per wave (wave tile BM/2 x BN/2)
  constexpr int STAGE = (BM + BN) * 128;      // bytes of one LDS stage (A then B)
  __shared__ __attribute__((aligned(16))) char smem[KG * 2 * STAGE];
  const int lane = threadIdx.x & 63, g = threadIdx.x >> 8, t = threadIdx.x & 255;
  const int wq = t >> 6, wm = wq >> 1, wn = wq & 1;
  const int m0 = blockIdx.x * BM, n0 = blockIdx.y * BN;
  const int CB = C / CV_BK, ksteps = taps * CB;  // taps: 9 (3x3) or 1 (1x1)
  const int kbeg = blockIdx.z * kps;
  const int kend = min(kbeg + kps, ksteps);
  const int chunk = t & 7;
  const long long K = (long long)taps * C;
  char* gsm = smem + g * 2 * STAGE;

  // per-thread A rows: pixel index and (h, w) (m = ((b*H)+h)*W + w)
  int am[PA], ah[PA], aw[PA];
#pragma unroll
  for (int i = 0; i < PA; ++i) {
    const int m = m0 + (t >> 3) + 32 * i;
    am[i] = m;
    const int hw = m % (H * W);
    ah[i] = hw / W;
    aw[i] = hw - ah[i] * W;
  }
  // B rows: weight rows n (forward: w[n][tap][c], contiguous along k) or, with TRB (backward
  // data, BN = 64), the rows (64 forward-output channels) of a [64 k][64 cols] image of the
  // forward weight w[k-channel][tap][out col], read transposed by the MFMA loop
  static_assert(!TRB || BN == 64, "transposed B images are 64 columns wide");
  // base of this thread's first B row; rows i are 32*i apart (row stride bstride elements)
  const uint16_t* wb = TRB ? w + (long long)(t >> 3) * taps * Nc + n0 + chunk * 8
                           : w + (long long)(n0 + (t >> 3)) * K + chunk * 8;
  const long long bstride = TRB ? 32LL * taps * Nc : 32LL * K;

  // two staging register sets: step s+2KG is loaded while step s computes and step s+KG (loaded
  // one iteration earlier) is written to LDS -- two k-group iterations to cover a global round trip
  CvRegs<PA> ra0, ra1;
  CvRegs<PB> rb0, rb1;
#define CV_NT_LOAD(S_, RA_, RB_)                                                                \
  do {                                                                                          \
    const int tap_ = (S_) / CB, cb_ = (S_) - tap_ * CB;                                         \
    const int dr_ = taps == 1 ? 0 : tap_ / 3 - 1;                                               \
    const int dc_ = taps == 1 ? 0 : tap_ - (tap_ / 3) * 3 - 1;                                  \
    {                                                                                           \
      auto& R = RA_;                                                                            \
      CV_FOR_ROWS(PA, {                                                                         \
        const int hh = ah[i] + dr_, ww = aw[i] + dc_;                                           \
        const bool ok = (unsigned)hh < (unsigned)H && (unsigned)ww < (unsigned)W;               \
        const cv_u4 x_ = *reinterpret_cast<const cv_u4*>(                                       \
            x + (long long)(ok ? am[i] + dr_ * W + dc_ : 0) * C + cb_ * CV_BK + chunk * 8);     \
        v = ok ? x_ : cv_u4{0u, 0u, 0u, 0u};                                                    \
      });                                                                                       \
    }                                                                                           \
    /* TRB: k-block cb_ of tap tap_ = forward channels cb_*64.. at the flipped tap */           \
    const long long bo_ = TRB ? ((long long)cb_ * CV_BK * taps + (taps - 1 - tap_)) * Nc          \
                              : (long long)(S_) * CV_BK;                                        \
    {                                                                                           \
      auto& R = RB_;                                                                            \
      CV_FOR_ROWS(PB, { v = *reinterpret_cast<const cv_u4*>(wb + i * bstride + bo_); });        \
    }                                                                                           \
  } while (0)
#define CV_NT_STORE(BUF_, RA_, RB_)                                                             \
  do {                                                                                          \
    char* As_ = gsm + (BUF_) * STAGE;                                                           \
    char* Bs_ = As_ + BM * 128;                                                                 \
    {                                                                                           \
      auto& R = RA_;                                                                            \
      CV_FOR_ROWS(PA, { *reinterpret_cast<cv_u4*>(As_ + cv_off((t >> 3) + 32 * i, chunk)) = v; }); \
    }                                                                                           \
    {                                                                                           \
      auto& R = RB_;                                                                            \
      CV_FOR_ROWS(PB, {                                                                         \
        *reinterpret_cast<cv_u4*>(Bs_ + (TRB ? cv_toff((t >> 3) + 32 * i, chunk)                \
                                             : cv_off((t >> 3) + 32 * i, chunk))) = v;          \
      });                                                                                       \
    }                                                                                           \
  } while (0)

  f32x4 acc[MI][NJ];
#pragma unroll
  for (int i = 0; i < MI; ++i)
#pragma unroll
    for (int j = 0; j < NJ; ++j) acc[i][j] = f32x4{0.0f, 0.0f, 0.0f, 0.0f};

  // group g: steps kbeg + g + KG*it; every group runs the same number of iterations (barriers)
  const int iters = (kend - kbeg + KG - 1) / KG;
  const int last = kend - 1;
  int s = kbeg + g;
#define CV_NT_MMA(BUF_)                                                                         \
  do {                                                                                          \
    const char* As_ = gsm + (BUF_) * STAGE;                                                     \
    if constexpr (TRB)                                                                          \
      cv_mma_mixed<MI, NJ>(As_, As_ + BM * 128, wm * (BM / 2), wn * (BN / 2), lane, acc);       \
    else                                                                                        \
      cv_mma<MI, NJ>(As_, As_ + BM * 128, wm * (BM / 2), wn * (BN / 2), lane, acc);             \
  } while (0)
  if (iters > 0) {
    CV_NT_LOAD(min(s, last), ra0, rb0);
    CV_NT_STORE(0, ra0, rb0);
    CV_NT_LOAD(min(s + KG, last), ra1, rb1);
    __syncthreads();
    // loads are clamped to the last step (dummy re-loads at the end: branch-free, keeps the
    // staging registers out of scratch); a group past the end only keeps the barrier count
    for (int it = 0; it < iters; it += 2, s += 2 * KG) {
      CV_NT_LOAD(min(s + 2 * KG, last), ra0, rb0);
      if (s <= last) CV_NT_MMA(0);
      CV_NT_STORE(1, ra1, rb1);  // buffer 1 last read one barrier ago
      __syncthreads();
      // second half unconditionally (an odd iteration count ends with an idle half: no MMA, one
      // barrier), so the loop has no branch around a barrier and the sets stay in registers
      CV_NT_LOAD(min(s + 3 * KG, last), ra1, rb1);
      if (s + KG <= last) CV_NT_MMA(1);
      CV_NT_STORE(0, ra0, rb0);
      __syncthreads();
    }
  }
#undef CV_NT_MMA
  cv_group_reduce<KG, MI, NJ>(acc, smem, g, wq, lane);
  cv_nt_epilogue<BM, BN, MI, NJ>(acc, smem, g, wm, wn, lane, m0, n0, M, Nc, out, slab, bnpart,
                                 bb, addend);
#undef CV_NT_LOAD
#undef CV_NT_STORE
}

// ---------------------------------------------------------------------------------------------
// LDS-DMA variant of the NT kernel (one k-group, NS-deep stage ring): operand tiles go global ->
// LDS directly with global_load_lds_dwordx4 (no staging registers, no ds_write), NS-1 k-steps in
// flight.  A wave instruction fills 8 consecutive 128-B rows lane-linearly (lane l -> row l/8,
// 16-B slot l%8), so each lane fetches the source chunk that the swizzled image stores at its
// slot (chunk = slot ^ swz(row)); out-of-image im2col rows read a zero page.  Ordering: a counted
// s_waitcnt vmcnt (the ring's younger stages stay in flight) + a raw s_barrier per k-step; the
// stage overwritten after the barrier was last read one step earlier (WAR-safe).
typedef __attribute__((address_space(3))) void* cv_lds_ptr;
typedef __attribute__((address_space(1))) void* cv_gbl_ptr;

__device__ __forceinline__ void cv_glds16(const void* src, char* lds_row_base) {
  __builtin_amdgcn_global_load_lds((cv_gbl_ptr)(src), (cv_lds_ptr)(lds_row_base), 16, 0, 0);
}

template <int N>
__device__ __forceinline__ void cv_wait_vm() {
  static_assert(N >= 0 && N < 64, "vmcnt range");
  // gfx9 s_waitcnt encoding: vmcnt[3:0] + vmcnt_hi[15:14], expcnt[6:4] = 7, lgkmcnt[11:8] = 15
  __builtin_amdgcn_s_waitcnt((N & 15) | ((N >> 4) << 14) | (7 << 4) | (15 << 8));
}

template <int BM, int BN, int NS, bool TRB>
__global__ __launch_bounds__(EW_BLOCK) void k_conv_nt_dma(const uint16_t* __restrict__ x,
                                                          const uint16_t* __restrict__ w,
                                                          uint16_t* __restrict__ out,
                                                          float* __restrict__ slab, int M, int H,
                                                          int W, int C, int Nc, int kps, int taps,
                                                          float* __restrict__ bnpart,
                                                          const uint16_t* __restrict__ zero,
                                                          CvBnBwd bb,
                                                          const uint16_t* __restrict__ addend) {
  constexpr int PA = BM / 32, PB = BN / 32;   // glds instructions per wave per k-step (8 rows each)
  constexpr int MI = BM / 32, NJ = BN / 32;
  constexpr int STAGE = (BM + BN) * 128;
  constexpr int LPW = PA + PB;
  static_assert(!TRB || BN == 64, "transposed B images are 64 columns wide");
  __shared__ __attribute__((aligned(16))) char smem[NS * STAGE];
  const int t = threadIdx.x, lane = t & 63, wq = t >> 6;
  const int wm = wq >> 1, wn = wq & 1;
  const int m0 = blockIdx.x * BM, n0 = blockIdx.y * BN;
  const int CB = C / CV_BK, ksteps = taps * CB;
  const int kbeg = blockIdx.z * kps;
  const int kend = min(kbeg + kps, ksteps);
  const long long K = (long long)taps * C;
  const int lr = lane >> 3, slot = lane & 7;

  // A rows of this lane: wave wq, instruction j -> tile row (wq*PA + j)*8 + lr
  int am[PA], ah[PA], aw[PA], ac[PA];
#pragma unroll
  for (int j = 0; j < PA; ++j) {
    const int row = (wq * PA + j) * 8 + lr;
    const int m = m0 + row;
    am[j] = m;
    const int hw = m % (H * W);
    ah[j] = hw / W;
    aw[j] = hw - ah[j] * W;
    ac[j] = slot ^ ((row >> 1) & 7);  // source chunk landing at this lane's slot
  }
  const uint16_t* bsrc[PB];
#pragma unroll
  for (int j = 0; j < PB; ++j) {
    const int row = (wq * PB + j) * 8 + lr;
    bsrc[j] = TRB ? w + (long long)row * taps * Nc + n0 + 8 * (slot ^ cv_trf(row))
                  : w + (long long)(n0 + row) * K + 8 * (slot ^ ((row >> 1) & 7));
  }

  auto issue = [&](int st, int buf) {
    const int tap = st / CB, cb = st - tap * CB;
    const int dr = taps == 1 ? 0 : tap / 3 - 1, dc = taps == 1 ? 0 : tap - (tap / 3) * 3 - 1;
    char* As = smem + buf * STAGE;
    char* Bs = As + BM * 128;
#pragma unroll
    for (int j = 0; j < PA; ++j) {
      const bool ok = (unsigned)(ah[j] + dr) < (unsigned)H && (unsigned)(aw[j] + dc) < (unsigned)W;
      const uint16_t* src =
          ok ? x + (long long)(am[j] + dr * W + dc) * C + cb * CV_BK + ac[j] * 8 : zero;
      cv_glds16(src, As + (wq * PA + j) * 8 * 128);
    }
    const long long bo = TRB ? ((long long)cb * CV_BK * taps + (taps - 1 - tap)) * Nc
                             : (long long)st * CV_BK;
#pragma unroll
    for (int j = 0; j < PB; ++j) cv_glds16(bsrc[j] + bo, Bs + (wq * PB + j) * 8 * 128);
  };

  f32x4 acc[MI][NJ];
#pragma unroll
  for (int i = 0; i < MI; ++i)
#pragma unroll
    for (int j = 0; j < NJ; ++j) acc[i][j] = f32x4{0.0f, 0.0f, 0.0f, 0.0f};

  const int n = kend - kbeg;
  if (n > 0) {
    const int last = kend - 1;
#pragma unroll
    for (int j = 0; j < NS - 1; ++j) issue(min(kbeg + j, last), j);  // clamped: dummy re-loads
    for (int i = 0; i < n; ++i) {
      cv_wait_vm<LPW * (NS - 2)>();  // this step's stage landed (younger NS-2 stages in flight)
      __builtin_amdgcn_s_barrier();  // ... for every wave; and step i-1's stage is free again
      issue(min(kbeg + i + NS - 1, last), (i + NS - 1) % NS);
      const char* As = smem + (i % NS) * STAGE;
      if constexpr (TRB)
        cv_mma_mixed<MI, NJ>(As, As + BM * 128, wm * (BM / 2), wn * (BN / 2), lane, acc);
      else
        cv_mma<MI, NJ>(As, As + BM * 128, wm * (BM / 2), wn * (BN / 2), lane, acc);
    }
    cv_wait_vm<0>();  // drain the dummy loads before the epilogue reuses the ring
  }
  __syncthreads();
  cv_nt_epilogue<BM, BN, MI, NJ>(acc, smem, 0, wm, wn, lane, m0, n0, M, Nc, out, slab, bnpart,
                                 bb, addend);
}

// ---------------------------------------------------------------------------------------------
// Weight-gradient kernel: dw[n][k] = sum_m dy[m][n] * X~[m][k], 64 rows of n x 64 columns of k
// (one tap: k0 = tap*C + c0), 64 m per k-step; split z covers m-steps
// [z*kps, min((z+1)*kps, msteps)).  dy: [M][Nc], x: [M][C].
// Both operands reduce over m, the slow axis of their NHWC tensors, so they are staged as they
// lie -- [64 m][64 cols] images, 8 lanes per 128-B row (coalesced loads, conflict-free
// ds_write_b128) -- and the MFMA fragments (8 consecutive m of one column) come from
// ds_read_b64_tr_b16 transposed reads: a 16-lane group reads a 4 (m) x 16 (col) block and lane i
// receives column i.  Image swizzle: chunk c of row r at c ^ cv_trf(r), which spreads the 8 rows
// {r0..r0+3, r0+8..r0+11} a 32-lane half reads at two adjacent chunks over 16 distinct bank slots
// and keeps each row's 8 chunks distinct for the writes.
template <int KG>
__global__ __launch_bounds__(EW_BLOCK * KG) void k_conv_wgrad(const uint16_t* __restrict__ dy,
                                                              const uint16_t* __restrict__ x,
                                                              uint16_t* __restrict__ dw,
                                                              float* __restrict__ slab, int M,
                                                              int H, int W, int C, int Nc,
                                                              int kps, int taps) {
  constexpr int BM = 64, BN = 64;
  constexpr int MI = BM / 32, NJ = BN / 32;
  constexpr int STAGE = (BM + BN) * 128;
  __shared__ __attribute__((aligned(16))) char smem[KG * 2 * STAGE];
  const int lane = threadIdx.x & 63, g = threadIdx.x >> 8, t = threadIdx.x & 255;
  const int wq = t >> 6, wm = wq >> 1, wn = wq & 1;
  const int n0 = blockIdx.x * BM;     // output rows (dy channels)
  const int k0 = blockIdx.y * BN;     // output columns (tap, channel)
  const int tap = k0 / C, c0 = k0 - tap * C;
  const int dr = taps == 1 ? 0 : tap / 3 - 1, dc = taps == 1 ? 0 : tap - (tap / 3) * 3 - 1;
  const int msteps = M / CV_BK;
  const int sbeg = blockIdx.z * kps;
  const int send = min(sbeg + kps, msteps);
  const int chunk = t & 7, r = t >> 3;  // this thread stages rows r and r + 32, chunk `chunk`
  const uint16_t* dyp = dy + n0 + chunk * 8;
  const uint16_t* xp = x + c0 + chunk * 8;
  char* gsm = smem + g * 2 * STAGE;

  const int iters = (send - sbeg + KG - 1) / KG;
  const int last = send - 1;
  int s = sbeg + g;
  // pixel (h, w) of rows r and r + 32 of the step being loaded, advanced by 64*KG pixels a step
  int m = min(s, last) * CV_BK + r;
  int h0, w0, h1, w1;
  {
    const int HW = H * W;
    int hw = m % HW;
    h0 = hw / W;
    w0 = hw - h0 * W;
    hw = (m + 32) % HW;
    h1 = hw / W;
    w1 = hw - h1 * W;
  }
  const int adv = CV_BK * KG, dH = (adv / W) % H, dW = adv % W;
  uint4 ra0, ra1, rb0, rb1, sa0, sa1, sb0, sb1;  // two staging sets (see k_conv_nt)
#define CV_WG_LOAD(ra0, ra1, rb0, rb1)                                                          \
  do {                                                                                          \
    ra0 = *reinterpret_cast<const uint4*>(dyp + (long long)m * Nc);                             \
    ra1 = *reinterpret_cast<const uint4*>(dyp + (long long)(m + 32) * Nc);                      \
    const bool ok0 = (unsigned)(h0 + dr) < (unsigned)H && (unsigned)(w0 + dc) < (unsigned)W;    \
    const bool ok1 = (unsigned)(h1 + dr) < (unsigned)H && (unsigned)(w1 + dc) < (unsigned)W;    \
    const uint4 x0_ = *reinterpret_cast<const uint4*>(                                          \
        xp + (ok0 ? (long long)(m + dr * W + dc) * C : 0));                                     \
    const uint4 x1_ = *reinterpret_cast<const uint4*>(                                          \
        xp + (ok1 ? (long long)(m + 32 + dr * W + dc) * C : 0));                                \
    rb0 = ok0 ? x0_ : make_uint4(0u, 0u, 0u, 0u);                                               \
    rb1 = ok1 ? x1_ : make_uint4(0u, 0u, 0u, 0u);                                               \
  } while (0)
#define CV_WG_STORE(BUF_, ra0, ra1, rb0, rb1)                                                   \
  do {                                                                                          \
    char* As_ = gsm + (BUF_) * STAGE;                                                           \
    char* Bs_ = As_ + BM * 128;                                                                 \
    *reinterpret_cast<uint4*>(As_ + cv_toff(r, chunk)) = ra0;                                   \
    *reinterpret_cast<uint4*>(As_ + cv_toff(r + 32, chunk)) = ra1;                              \
    *reinterpret_cast<uint4*>(Bs_ + cv_toff(r, chunk)) = rb0;                                   \
    *reinterpret_cast<uint4*>(Bs_ + cv_toff(r + 32, chunk)) = rb1;                              \
  } while (0)
  // advance (m, h, w) by one group step when the next step exists (else reload: a dummy)
#define CV_WG_ADVANCE(NEXT_)                                                                    \
  do {                                                                                          \
    if (NEXT_) {                                                                                \
      m += adv;                                                                                 \
      w0 += dW; h0 += dH; if (w0 >= W) { w0 -= W; ++h0; } if (h0 >= H) h0 -= H;                \
      w1 += dW; h1 += dH; if (w1 >= W) { w1 -= W; ++h1; } if (h1 >= H) h1 -= H;                \
    }                                                                                           \
  } while (0)

  f32x4 acc[MI][NJ];
#pragma unroll
  for (int i = 0; i < MI; ++i)
#pragma unroll
    for (int j = 0; j < NJ; ++j) acc[i][j] = f32x4{0.0f, 0.0f, 0.0f, 0.0f};

  if (iters > 0) {
    CV_WG_LOAD(ra0, ra1, rb0, rb1);
    CV_WG_STORE(0, ra0, ra1, rb0, rb1);
    CV_WG_ADVANCE(s + KG <= last);
    CV_WG_LOAD(sa0, sa1, sb0, sb1);
    __syncthreads();
    for (int it = 0; it < iters; it += 2, s += 2 * KG) {
      CV_WG_ADVANCE(s + 2 * KG <= last);
      CV_WG_LOAD(ra0, ra1, rb0, rb1);
      if (s <= last)
        cv_mma_tr<MI, NJ>(gsm, gsm + BM * 128, wm * (BM / 2), wn * (BN / 2), lane, acc);
      CV_WG_STORE(1, sa0, sa1, sb0, sb1);
      __syncthreads();
      CV_WG_ADVANCE(s + 3 * KG <= last);
      CV_WG_LOAD(sa0, sa1, sb0, sb1);
      if (s + KG <= last)
        cv_mma_tr<MI, NJ>(gsm + STAGE, gsm + STAGE + BM * 128, wm * (BM / 2), wn * (BN / 2),
                          lane, acc);
      CV_WG_STORE(0, ra0, ra1, rb0, rb1);
      __syncthreads();
    }
  }
#undef CV_WG_LOAD
#undef CV_WG_STORE
#undef CV_WG_ADVANCE
  cv_group_reduce<KG, MI, NJ>(acc, smem, g, wq, lane);
  if (g != 0) return;
  const long long K = (long long)taps * C;
  const int row0 = n0 + wm * (BM / 2), col0 = k0 + wn * (BN / 2);
  if (slab)
    cv_store<MI, NJ>(acc, row0, col0, lane, nullptr, slab + (long long)blockIdx.z * Nc * K, K);
  else
    cv_store<MI, NJ>(acc, row0, col0, lane, dw, nullptr, K);
}

// ---------------------------------------------------------------------------------------------
// out_bf16[i] = bf16(sum_z slab[z][i]), 8 elements per thread (n % 8 == 0)
__global__ __launch_bounds__(EW_BLOCK) void k_cv_slab_reduce(const float* __restrict__ slab,
                                                             int nsplit, long long n,
                                                             uint16_t* __restrict__ out,
                                                             const uint16_t* __restrict__ addend) {
  const long long nv = n / 8;
  for (long long v = blockIdx.x * (long long)EW_BLOCK + threadIdx.x; v < nv;
       v += (long long)gridDim.x * EW_BLOCK) {
    float a[8];
    const float4* p = reinterpret_cast<const float4*>(slab) + 2 * v;
    float4 lo = p[0], hi = p[1];
    a[0] = lo.x; a[1] = lo.y; a[2] = lo.z; a[3] = lo.w;
    a[4] = hi.x; a[5] = hi.y; a[6] = hi.z; a[7] = hi.w;
    for (int z = 1; z < nsplit; ++z) {
      p += n / 4;
      lo = p[0];
      hi = p[1];
      a[0] += lo.x; a[1] += lo.y; a[2] += lo.z; a[3] += lo.w;
      a[4] += hi.x; a[5] += hi.y; a[6] += hi.z; a[7] += hi.w;
    }
    if (addend) {  // see cv_nt_epilogue
      const uint4 w = reinterpret_cast<const uint4*>(addend)[v];
      const uint32_t aw[4] = {w.x, w.y, w.z, w.w};
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        a[2 * j] += __uint_as_float(aw[j] << 16);
        a[2 * j + 1] += __uint_as_float(aw[j] & 0xffff0000u);
      }
    }
    uint4 o;
    o.x = (uint32_t)ew_f2bf(a[0]) | ((uint32_t)ew_f2bf(a[1]) << 16);
    o.y = (uint32_t)ew_f2bf(a[2]) | ((uint32_t)ew_f2bf(a[3]) << 16);
    o.z = (uint32_t)ew_f2bf(a[4]) | ((uint32_t)ew_f2bf(a[5]) << 16);
    o.w = (uint32_t)ew_f2bf(a[6]) | ((uint32_t)ew_f2bf(a[7]) << 16);
    reinterpret_cast<uint4*>(out)[v] = o;
  }
}

// ---------------------------------------------------------------------------------------------
// Stem convolution: 3x3 / pad 1 / stride 1 over 3 input channels (VGG's first layer, the CIFAR
// ResNet stem).  The reduction K = 9 taps x 3 channels = 27, in the order of the channels_last
// weight [n][r][s][c], zero-padded to 32: one v_mfma_f32_16x16x32_bf16 step covers it, so the
// layer is bound by writing its output (forward) or reading its output gradient (weight
// gradient).  MIOpen runs it as a grouped-conv forward and, for the weight gradient, a zero-fill +
// igemm + cast chain (~42 us per VGG-11 step, profiles/vgg11_bs128_*).
typedef unsigned short cv_u16x8 __attribute__((ext_vector_type(8)));
constexpr int ST_K = 27;

constexpr int ST_WMAX = 256;  // image width bound of the LDS input patch

// The input pixels a block of PIX output pixels [m0, m0 + PIX) reads, [m0 - W - 1, m0 + PIX + W
// + 1) (clamped to the tensor), are one contiguous NHWC range: it goes to LDS as 16-B chunks and
// the im2col gathers read LDS.  Returns the element offset of patch[0].
template <int PIX>
__device__ __forceinline__ int st_patch(const uint16_t* __restrict__ x, int m0, int W, int M,
                                        uint16_t* patch, int t) {
  int lo = (m0 - W - 1) * 3;
  lo = lo < 0 ? 0 : (lo & ~7);
  int hi = ((m0 + PIX + W + 1) * 3 + 7) & ~7;
  hi = hi > 3 * M ? 3 * M : hi;
  const int nch = (hi - lo) >> 3;
  for (int c = t; c < nch; c += EW_BLOCK)
    *reinterpret_cast<cv_u4*>(patch + 8 * c) = *reinterpret_cast<const cv_u4*>(x + lo + 8 * c);
  return lo;
}
template <int PIX>
constexpr int st_patch_elems() { return (PIX + 2 * ST_WMAX + 2) * 3 + 16; }

// im2col element k (tap-major) of pixel m at (h, w) from the patch: 0 outside the image and for
// k >= 27
__device__ __forceinline__ uint16_t st_x(const uint16_t* patch, int lo, int m, int h, int w,
                                         int H, int W, int k) {
  const int tap = k / 3, c = k - 3 * tap;
  const int dr = tap / 3 - 1, dc = tap - 3 * (tap / 3) - 1;
  const bool ok = k < ST_K && (unsigned)(h + dr) < (unsigned)H && (unsigned)(w + dc) < (unsigned)W;
  return ok ? patch[(m + dr * W + dc) * 3 + c - lo] : (uint16_t)0;
}

// Forward: block = 4 waves over 128 pixels x 64 output channels; wave v owns pixels
// [32 v, 32 v + 32) (2 x 4 MFMA tiles).  A fragments are gathered from the LDS input patch
// (each im2col element is read by exactly one lane), the weight tile goes through LDS, the bf16
// tile is staged in LDS for 16-B coalesced stores, and the BatchNorm partial sums of the stored
// values (one row per block, the BN finalize layout) come from the registers.
__global__ __launch_bounds__(EW_BLOCK) void k_conv_stem_fwd(const uint16_t* __restrict__ x,
                                                            const uint16_t* __restrict__ w,
                                                            uint16_t* __restrict__ y, int H,
                                                            int W, int Nc, int M,
                                                            float* __restrict__ bnpart,
                                                            int nrows) {
  __shared__ __attribute__((aligned(16))) uint16_t patch[st_patch_elems<128>()];
  __shared__ __attribute__((aligned(16))) uint16_t wsm[64 * 32];
  __shared__ __attribute__((aligned(16))) uint16_t ysm[128 * 64];
  __shared__ float red[EW_WAVES][2][64];
  const int t = threadIdx.x, lane = t & 63, wv = t >> 6;
  const int m0 = blockIdx.x * 128, n0 = blockIdx.y * 64;
  for (int e = t; e < 64 * 32; e += EW_BLOCK) {
    const int n = e >> 5, k = e & 31;
    wsm[e] = k < ST_K ? w[(long long)(n0 + n) * ST_K + k] : (uint16_t)0;
  }
  const int lo = st_patch<128>(x, m0, W, M, patch, t);
  __syncthreads();
  const int kb = 8 * (lane >> 4), HW = H * W;
  bf16x8 a[2];
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int m = m0 + 32 * wv + 16 * i + (lane & 15);
    const int p = m % HW, h = p / W, ww = p - h * W;
    cv_u16x8 v;
#pragma unroll
    for (int e = 0; e < 8; ++e) v[e] = st_x(patch, lo, m, h, ww, H, W, kb + e);
    a[i] = __builtin_bit_cast(bf16x8, v);
  }
  f32x4 acc[2][4];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const bf16x8 b = *reinterpret_cast<const bf16x8*>(wsm + (16 * j + (lane & 15)) * 32 + kb);
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      acc[i][j] = f32x4{0.0f, 0.0f, 0.0f, 0.0f};
      acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[i], b, acc[i][j], 0, 0, 0);
    }
  }
  float sm[4], sq[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    sm[j] = sq[j] = 0.0f;
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const uint16_t hb = ew_f2bf(acc[i][j][q]);
        ysm[(32 * wv + 16 * i + 4 * (lane >> 4) + q) * 64 + 16 * j + (lane & 15)] = hb;
        const float v = __uint_as_float((uint32_t)hb << 16);
        sm[j] += v;
        sq[j] += v * v;
      }
  }
  if (bnpart) {
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      sm[j] += __shfl_xor(sm[j], 16, 64);
      sq[j] += __shfl_xor(sq[j], 16, 64);
      sm[j] += __shfl_xor(sm[j], 32, 64);
      sq[j] += __shfl_xor(sq[j], 32, 64);
    }
    if (lane < 16) {
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        red[wv][0][16 * j + lane] = sm[j];
        red[wv][1][16 * j + lane] = sq[j];
      }
    }
  }
  __syncthreads();
#pragma unroll
  for (int u = 0; u < 4; ++u) {
    const int e = t + EW_BLOCK * u, r = e >> 3, ch = e & 7;
    *reinterpret_cast<cv_u4*>(y + (long long)(m0 + r) * Nc + n0 + ch * 8) =
        *reinterpret_cast<const cv_u4*>(ysm + r * 64 + ch * 8);
  }
  if (bnpart && t < 64) {
    float s1 = 0.0f, s2 = 0.0f;
#pragma unroll
    for (int v = 0; v < EW_WAVES; ++v) {  // fixed order
      s1 += red[v][0][t];
      s2 += red[v][1][t];
    }
    bnpart[(long long)blockIdx.x * Nc + n0 + t] = s1;
    bnpart[(long long)(nrows + blockIdx.x) * Nc + n0 + t] = s2;
  }
}

// Weight gradient dw[n][k] = sum_m dy[m][n] x~[m][k]: block = 256 pixels x 64 output channels,
// staged as four [64 m][64 n] dy images and four [64 m][32 k] im2col images (transposed-read
// layout, cv_toff), wave v computes rows n0 + [16 v, 16 v + 16) x all 32 k; fp32 partial
// [64][27] per block into the slab, summed by k_conv_stem_reduce.
__global__ __launch_bounds__(EW_BLOCK) void k_conv_stem_wgrad(const uint16_t* __restrict__ dy,
                                                              const uint16_t* __restrict__ x,
                                                              float* __restrict__ slab, int H,
                                                              int W, int Nc, int M) {
  __shared__ __attribute__((aligned(16))) char As[4 * 8192];
  __shared__ __attribute__((aligned(16))) char Bs[4 * 8192];
  __shared__ __attribute__((aligned(16))) uint16_t patch[st_patch_elems<256>()];
  const int t = threadIdx.x, lane = t & 63, wv = t >> 6;
  const int m0 = blockIdx.x * 256, n0 = blockIdx.y * 64, HW = H * W;
  cv_u4 d[8];
#pragma unroll
  for (int u = 0; u < 8; ++u) {
    const int e = t + EW_BLOCK * u, r = e >> 3, ch = e & 7;
    d[u] = *reinterpret_cast<const cv_u4*>(dy + (long long)(m0 + r) * Nc + n0 + ch * 8);
  }
  const int lo = st_patch<256>(x, m0, W, M, patch, t);
  __syncthreads();
#pragma unroll
  for (int u = 0; u < 4; ++u) {
    const int e = t + EW_BLOCK * u, r = e >> 2, ch = e & 3;
    const int m = m0 + r, p = m % HW, h = p / W, ww = p - h * W;
    cv_u16x8 v;
#pragma unroll
    for (int e2 = 0; e2 < 8; ++e2) v[e2] = st_x(patch, lo, m, h, ww, H, W, 8 * ch + e2);
    *reinterpret_cast<cv_u16x8*>(Bs + (r >> 6) * 8192 + cv_toff(r & 63, ch)) = v;
  }
#pragma unroll
  for (int u = 0; u < 8; ++u) {
    const int e = t + EW_BLOCK * u, r = e >> 3, ch = e & 7;
    *reinterpret_cast<cv_u4*>(As + (r >> 6) * 8192 + cv_toff(r & 63, ch)) = d[u];
  }
  __syncthreads();
  f32x4 acc[1][2];
  acc[0][0] = acc[0][1] = f32x4{0.0f, 0.0f, 0.0f, 0.0f};
#pragma unroll
  for (int img = 0; img < 4; ++img)
    cv_mma_tr<1, 2>(As + img * 8192, Bs + img * 8192, 16 * wv, 0, lane, acc);
  float* sp = slab + (long long)blockIdx.x * Nc * ST_K;
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const int k = 16 * j + (lane & 15);
    if (k < ST_K) {
#pragma unroll
      for (int q = 0; q < 4; ++q)
        sp[(long long)(n0 + 16 * wv + 4 * (lane >> 4) + q) * ST_K + k] = acc[0][j][q];
    }
  }
}

// dw[o] = sum over the nb block partials slab[b][o] in a fixed order: block = 8 outputs x 32
// partial chunks, chunk sums combined through LDS pairwise.
__global__ __launch_bounds__(EW_BLOCK) void k_conv_stem_reduce(const float* __restrict__ slab,
                                                               int nb, int n,
                                                               uint16_t* __restrict__ dw) {
  __shared__ float red[32][8];
  const int t = threadIdx.x, o = blockIdx.x * 8 + (t & 7), ck = t >> 3;
  float s = 0.0f;
  if (o < n) {
    const int per = (nb + 31) / 32, b0 = ck * per, b1 = min(b0 + per, nb);
    int b = b0;
    for (; b + 3 < b1; b += 4) {
      const float v0 = slab[(long long)b * n + o], v1 = slab[(long long)(b + 1) * n + o];
      const float v2 = slab[(long long)(b + 2) * n + o], v3 = slab[(long long)(b + 3) * n + o];
      s += (v0 + v1) + (v2 + v3);
    }
    for (; b < b1; ++b) s += slab[(long long)b * n + o];
  }
  red[ck][t & 7] = s;
  __syncthreads();
#pragma unroll
  for (int h = 16; h > 0; h >>= 1) {
    if (ck < h) red[ck][t & 7] += red[ck + h][t & 7];
    __syncthreads();
  }
  if (ck == 0 && o < n) dw[o] = ew_f2bf(red[0][t & 7]);
}

// Split-K reduction that also writes the BatchNorm partial sums of its output (the epilogue's job
// when there is no split): forward sum / sum of squares of the bf16 output, or with bb.h the
// BN-backward sums of CvBnBwd.  Block b: rows [b * rpb, (b + 1) * rpb) x all Nc columns, thread:
// column octet t % tpr (tpr = Nc / 8), rows t / tpr + k * rpi; one partial row per block.
__global__ __launch_bounds__(EW_BLOCK) void k_cv_slab_reduce_bn(const float* __restrict__ slab,
                                                                int nsplit, int M, int Nc,
                                                                uint16_t* __restrict__ out,
                                                                float* __restrict__ bnpart,
                                                                int rpb, CvBnBwd bb,
                                                                const uint16_t* __restrict__ addend) {
  __shared__ float red[2][EW_BLOCK * 8];  // [2][rpi][Nc]: rpi * Nc = 8 * EW_BLOCK
  const int tpr = Nc >> 3, rpi = EW_BLOCK / tpr;
  const int t = threadIdx.x, g = t % tpr, rg = t / tpr;
  const int c0 = g * 8;
  const long long n = (long long)M * Nc;
  const int r0 = blockIdx.x * rpb, r1 = min(r0 + rpb, M);
  float s1[8], s2[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) s1[j] = s2[j] = 0.0f;
  float mean[8], sc[8], sh[8];
  if (bb.h && rg < rpi) {
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      mean[j] = bb.stats[c0 + j];
      sc[j] = bb.stats[2 * Nc + c0 + j];
      sh[j] = bb.stats[3 * Nc + c0 + j];
    }
  }
  const uint32_t HoWo = (uint32_t)bb.Ho * bb.Wo;
  if (rg < rpi) {
    for (int r = r0 + rg; r < r1; r += rpi) {
      const long long o = (long long)r * Nc + c0;
      float a[8];
      {
        const float4* p = reinterpret_cast<const float4*>(slab + o);
        float4 lo = p[0], hi = p[1];
        a[0] = lo.x; a[1] = lo.y; a[2] = lo.z; a[3] = lo.w;
        a[4] = hi.x; a[5] = hi.y; a[6] = hi.z; a[7] = hi.w;
        for (int z = 1; z < nsplit; ++z) {  // fixed order (as k_cv_slab_reduce)
          p += n / 4;
          lo = p[0];
          hi = p[1];
          a[0] += lo.x; a[1] += lo.y; a[2] += lo.z; a[3] += lo.w;
          a[4] += hi.x; a[5] += hi.y; a[6] += hi.z; a[7] += hi.w;
        }
        if (addend) {
          const uint4 w = *reinterpret_cast<const uint4*>(addend + o);
          const uint32_t aw[4] = {w.x, w.y, w.z, w.w};
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            a[2 * j] += __uint_as_float(aw[j] << 16);
            a[2 * j + 1] += __uint_as_float(aw[j] & 0xffff0000u);
          }
        }
      }
      uint16_t b[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) b[j] = ew_f2bf(a[j]);
      uint4 ov;
      ov.x = (uint32_t)b[0] | ((uint32_t)b[1] << 16);
      ov.y = (uint32_t)b[2] | ((uint32_t)b[3] << 16);
      ov.z = (uint32_t)b[4] | ((uint32_t)b[5] << 16);
      ov.w = (uint32_t)b[6] | ((uint32_t)b[7] << 16);
      *reinterpret_cast<uint4*>(out + o) = ov;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const float d = __uint_as_float((uint32_t)b[j] << 16);
        if (bb.h) {
          uint32_t hr = (uint32_t)r;
          if (bb.code) hr = cv_pool_row((uint32_t)r, HoWo, (uint32_t)bb.Wo, bb.code[o + j]);
          const float x = __uint_as_float((uint32_t)bb.h[(size_t)hr * Nc + c0 + j] << 16);
          float v = x * sc[j] + sh[j];
          if (bb.res) v = v + __uint_as_float((uint32_t)bb.res[(size_t)hr * Nc + c0 + j] << 16);
          const float dz = (bb.relu == 0 || !(v <= 0.0f)) ? d : 0.0f;
          s1[j] += dz;
          s2[j] += dz * (x - mean[j]);
        } else {
          s1[j] += d;
          s2[j] += d * d;
        }
      }
    }
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      red[0][rg * Nc + c0 + j] = s1[j];
      red[1][rg * Nc + c0 + j] = s2[j];
    }
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

// Launch shape of one conv GEMM: tiles, global split of the reduction, k-groups per block.
// Enough blocks for every CU (split-K slabs only below 128 tiles), then k-groups so that about
// 16 waves share each CU: resident blocks per CU r = ceil(blocks / 256), KG = 4 / r (<= kgmax).
struct CvPlan {
  int split, kg, kps;
};
CvPlan cv_plan(long long tiles, int ksteps, int kgmax, long long out_floats, long long ws_floats) {
  CvPlan p{1, 1, ksteps};
  if (tiles < 128) {
    while (tiles * p.split < 256 && ksteps / (p.split * 2) >= 8) p.split *= 2;
    while (p.split > 1 && (long long)p.split * out_floats > ws_floats) p.split /= 2;
  }
  const long long blocks = tiles * p.split;
  const long long r = (blocks + 255) / 256;
  p.kg = (int)(r >= 4 ? 1 : 4 / r);
  if (p.kg > kgmax) p.kg = kgmax;
  if (p.kg == 3) p.kg = 2;
  p.kps = (ksteps + p.split - 1) / p.split;
  while (p.kg > 1 && p.kps < 2 * p.kg) p.kg /= 2;  // keep >= 2 steps per group
  return p;
}

}  // namespace

// ------------------------------------------------------------------------------------------------
// host side

long long ew_conv_ws_floats() { return 8LL << 20; }  // 32 MiB of fp32 split slabs per workspace

#define CV_LAUNCH_NT(BM_, KG_, TRB_)                                                             \
  hipLaunchKernelGGL((k_conv_nt<BM_, BM_, KG_, TRB_>), grid, dim3(EW_BLOCK * KG_), 0, s, x, w,  \
                     out, slab, M, H, W, C, Nc, p.kps, taps, bnp, bbv, addend)

// NT GEMM (forward / backward-data): out[M][Nc] = sum X~[M][9C] w[Nc][9C]^T
// trb: w is the forward weight [C][9][Nc] of a backward-data GEMM (transposed B images, 64x64
// tiles); otherwise w is [Nc][9][C].
// bnpart (nullable, bnpart_floats capacity): BatchNorm partial sums of the output written by the
// epilogue when the launch has no split; returns the number of partial rows (0: not written).
static int ew_conv_nt(const uint16_t* x, const uint16_t* w, uint16_t* out, float* ws,
                      long long ws_floats, int M, int H, int W, int C, int Nc, int taps,
                      bool trb, hipStream_t s, float* bnpart = nullptr,
                      long long bnpart_floats = 0, const CvBnBwd* bnb = nullptr,
                      const uint16_t* addend = nullptr) {
  if (C % CV_BK || Nc % 64 || M % 64)
    throw std::runtime_error("ewdml conv: needs C % 64 == 0, Nc % 64 == 0, N*H*W % 64 == 0");
  const int ksteps = taps * (C / CV_BK);
  const bool big = !trb && (M % 128 == 0) && (Nc % 128 == 0) &&
                   (long long)(M / 128) * (Nc / 128) >= 256;
  const int BM = big ? 128 : 64;
  const long long tiles = (long long)(M / BM) * (Nc / BM);
  // EWDML_CONV_DMA=1: the LDS-DMA stage-ring kernels (one k-group per block)
  static const bool dma = [] {
    const char* e = getenv("EWDML_CONV_DMA");
    return e && e[0] == '1';
  }();
  // the last 64 floats of the workspace are a zero page (never part of a slab)
  ws_floats -= 64;
  const uint16_t* zero = reinterpret_cast<const uint16_t*>(ws + ws_floats);
  ws_floats -= 4096;  // conv_f32.hip's in-launch split-K tickets (CF_RED_TICKETS) precede the zero page
  const CvPlan p = cv_plan(tiles, ksteps, dma ? 1 : (big ? 2 : 4), (long long)M * Nc, ws_floats);
  dim3 grid(M / BM, Nc / BM, p.split);
  float* slab = p.split > 1 ? ws : nullptr;
  // epilogue BN partials: one row per M-tile; beyond 1024 rows the BN statistics pass (<= 1024
  // partial rows) leaves the finalize less to reduce
  const long long prow = M / BM;
  float* bnp = (bnpart && !slab && prow <= 1024 && 2 * prow * Nc <= bnpart_floats) ? bnpart
                                                                                  : nullptr;
  const CvBnBwd bbv = (bnp && bnb) ? *bnb : CvBnBwd{nullptr, nullptr, nullptr, nullptr, 0, 0, 0};
#define CV_LAUNCH_DMA(BM_, TRB_)                                                                 \
  hipLaunchKernelGGL((k_conv_nt_dma<BM_, BM_, 4, TRB_>), grid, dim3(EW_BLOCK), 0, s, x, w, out, \
                     slab, M, H, W, C, Nc, p.kps, taps, bnp, zero, bbv, addend)
  if (dma) {
    if (big) CV_LAUNCH_DMA(128, false);
    else if (trb) CV_LAUNCH_DMA(64, true);
    else CV_LAUNCH_DMA(64, false);
  } else if (big) {
    if (p.kg == 2) CV_LAUNCH_NT(128, 2, false);
    else CV_LAUNCH_NT(128, 1, false);
  } else if (trb) {
    if (p.kg == 4) CV_LAUNCH_NT(64, 4, true);
    else if (p.kg == 2) CV_LAUNCH_NT(64, 2, true);
    else CV_LAUNCH_NT(64, 1, true);
  } else {
    if (p.kg == 4) CV_LAUNCH_NT(64, 4, false);
    else if (p.kg == 2) CV_LAUNCH_NT(64, 2, false);
    else CV_LAUNCH_NT(64, 1, false);
  }
  EW_CHECK_LAUNCH();
  if (p.split > 1) {
    const long long n = (long long)M * Nc;
    // with BN partials requested: the reduction writes them (one partial row per block of rpb
    // rows, <= 1024 rows, as many blocks as possible)
    const int tpr = Nc / 8, rpi = tpr <= EW_BLOCK ? EW_BLOCK / tpr : 0;
    int rpb = rpi, nblk = 0;
    if (bnpart && rpi > 0 && Nc <= 2048 && EW_BLOCK % tpr == 0) {
      while ((M + rpb - 1) / rpb > 1024) rpb += rpi;
      nblk = (M + rpb - 1) / rpb;
      if (2LL * nblk * Nc > bnpart_floats) nblk = 0;
    }
    if (nblk > 0) {
      const CvBnBwd bbr = bnb ? *bnb : CvBnBwd{nullptr, nullptr, nullptr, nullptr, 0, 0, 0};
      hipLaunchKernelGGL(k_cv_slab_reduce_bn, dim3(nblk), dim3(EW_BLOCK), 0, s, ws, p.split, M,
                         Nc, out, bnpart, rpb, bbr, addend);
      EW_CHECK_LAUNCH();
      return nblk;
    }
    long long gr = (n / 8 + EW_BLOCK - 1) / EW_BLOCK;
    if (gr > 2048) gr = 2048;
    hipLaunchKernelGGL(k_cv_slab_reduce, dim3((int)gr), dim3(EW_BLOCK), 0, s, ws, p.split, n, out,
                       addend);
    EW_CHECK_LAUNCH();
  }
  return bnp ? (int)prow : 0;
}
#undef CV_LAUNCH_NT
#undef CV_LAUNCH_DMA

static int cv_taps(int ksize) {
  if (ksize != 1 && ksize != 3) throw std::runtime_error("ewdml conv: kernel size must be 1 or 3");
  return ksize * ksize;
}

int ew_conv_fwd(uintptr_t x, uintptr_t w, uintptr_t y, uintptr_t ws, long long ws_floats,
                long long N, int H, int W, int C, int Nc, int ksize, uintptr_t bnpart,
                long long bnpart_floats, uintptr_t stream) {
  return ew_conv_nt(reinterpret_cast<const uint16_t*>(x), reinterpret_cast<const uint16_t*>(w),
                    reinterpret_cast<uint16_t*>(y), reinterpret_cast<float*>(ws), ws_floats,
                    (int)(N * H * W), H, W, C, Nc, cv_taps(ksize), false, (hipStream_t)stream,
                    reinterpret_cast<float*>(bnpart), bnpart_floats);
}

int ew_conv_bwd_data(uintptr_t dy, uintptr_t w, uintptr_t dx, uintptr_t ws,
                     long long ws_floats, long long N, int H, int W, int C, int Nc, int ksize,
                     uintptr_t bn_h, uintptr_t bn_res, uintptr_t bn_code, uintptr_t bn_stats,
                     int bn_relu, uintptr_t bnpart, long long bnpart_floats, uintptr_t addend,
                     uintptr_t stream) {
  // the flipped / transposed weight is read in place through transposed B images (no copy)
  if (C % 64 || Nc % 64) throw std::runtime_error("ewdml conv: bwd-data needs C, Nc % 64 == 0");
  // optional BN-backward sums of the layer whose output gradient dx is (CvBnBwd); with a pool,
  // dx is at the pooled resolution H x W and bn_h at 2H x 2W
  const CvBnBwd bb{reinterpret_cast<const uint16_t*>(bn_h),
                   reinterpret_cast<const uint16_t*>(bn_res),
                   reinterpret_cast<const uint8_t*>(bn_code),
                   reinterpret_cast<const float*>(bn_stats), bn_relu, H, W};
  // dx[m][c] = sum over (tap', n) of dY~[m][(tap', n)] * w[n][8 - tap'][c]
  return ew_conv_nt(reinterpret_cast<const uint16_t*>(dy), reinterpret_cast<const uint16_t*>(w),
                    reinterpret_cast<uint16_t*>(dx), reinterpret_cast<float*>(ws), ws_floats,
                    (int)(N * H * W), H, W, Nc, C, cv_taps(ksize), true, (hipStream_t)stream,
                    bn_h ? reinterpret_cast<float*>(bnpart) : nullptr, bnpart_floats,
                    bn_h ? &bb : nullptr, reinterpret_cast<const uint16_t*>(addend));
}

void ew_conv_wgrad(uintptr_t dy, uintptr_t x, uintptr_t dw, uintptr_t ws, long long ws_floats,
                   long long N, int H, int W, int C, int Nc, int ksize, uintptr_t stream) {
  const int taps = cv_taps(ksize);
  hipStream_t s = (hipStream_t)stream;
  const long long M = N * H * W;
  if (C % 64 || Nc % 64 || M % CV_BK)
    throw std::runtime_error("ewdml conv: wgrad needs C, Nc % 64 == 0");
  const long long K = (long long)taps * C;
  const long long tiles = (long long)(Nc / 64) * (K / 64);
  const int msteps = (int)(M / CV_BK);
  CvPlan p{1, 1, msteps};
  ws_floats -= 64;  // zero page (see ew_conv_nt)
  // blocks for every CU through the m split (slabs are Nc x 9C, small next to the activations)
  while (tiles * p.split < 256 && msteps / (p.split * 2) >= 8) p.split *= 2;
  while (p.split > 1 && (long long)p.split * Nc * K > ws_floats) p.split /= 2;
  {
    const CvPlan q = cv_plan(tiles * p.split, msteps / p.split, 4, 0, 0);
    p.kg = q.kg;
  }
  p.kps = (msteps + p.split - 1) / p.split;
  while (p.kg > 1 && p.kps < 2 * p.kg) p.kg /= 2;
  dim3 grid(Nc / 64, (int)(K / 64), p.split);
  float* slab = p.split > 1 ? reinterpret_cast<float*>(ws) : nullptr;
  const uint16_t* dyp = reinterpret_cast<const uint16_t*>(dy);
  const uint16_t* xp = reinterpret_cast<const uint16_t*>(x);
  uint16_t* dwp = reinterpret_cast<uint16_t*>(dw);
  if (p.kg == 4)
    hipLaunchKernelGGL(k_conv_wgrad<4>, grid, dim3(EW_BLOCK * 4), 0, s, dyp, xp, dwp, slab,
                       (int)M, H, W, C, Nc, p.kps, taps);
  else if (p.kg == 2)
    hipLaunchKernelGGL(k_conv_wgrad<2>, grid, dim3(EW_BLOCK * 2), 0, s, dyp, xp, dwp, slab,
                       (int)M, H, W, C, Nc, p.kps, taps);
  else
    hipLaunchKernelGGL(k_conv_wgrad<1>, grid, dim3(EW_BLOCK), 0, s, dyp, xp, dwp, slab, (int)M,
                       H, W, C, Nc, p.kps, taps);
  EW_CHECK_LAUNCH();
  if (p.split > 1) {
    const long long n = (long long)Nc * K;
    long long g = (n / 8 + EW_BLOCK - 1) / EW_BLOCK;
    if (g > 2048) g = 2048;
    hipLaunchKernelGGL(k_cv_slab_reduce, dim3((int)g), dim3(EW_BLOCK), 0, s,
                       reinterpret_cast<const float*>(ws), p.split, n, reinterpret_cast<uint16_t*>(dw), nullptr);
    EW_CHECK_LAUNCH();
  }
}

// ---- stem convolution (3 input channels) ----
int ew_conv_stem_fwd(uintptr_t x, uintptr_t w, uintptr_t y, long long N, int H, int W, int Nc,
                     uintptr_t bnpart, long long bnpart_floats, uintptr_t stream) {
  const long long M = N * H * W;
  if (M % 128 || Nc % 64 || M >= (1LL << 31) / 3 || W > ST_WMAX)
    throw std::runtime_error("ewdml conv stem: needs N*H*W % 128 == 0, Nc % 64 == 0, W <= 256");
  const int nrows = (int)(M / 128);
  float* bnp = (bnpart && nrows <= 1024 && 2LL * nrows * Nc <= bnpart_floats)
                   ? reinterpret_cast<float*>(bnpart) : nullptr;
  hipLaunchKernelGGL(k_conv_stem_fwd, dim3(nrows, Nc / 64), dim3(EW_BLOCK), 0,
                     (hipStream_t)stream, reinterpret_cast<const uint16_t*>(x),
                     reinterpret_cast<const uint16_t*>(w), reinterpret_cast<uint16_t*>(y), H, W,
                     Nc, (int)M, bnp, nrows);
  EW_CHECK_LAUNCH();
  return bnp ? nrows : 0;
}

void ew_conv_stem_wgrad(uintptr_t dy, uintptr_t x, uintptr_t dw, uintptr_t ws,
                        long long ws_floats, long long N, int H, int W, int Nc,
                        uintptr_t stream) {
  const long long M = N * H * W;
  const long long nb = M / 256, n = (long long)Nc * ST_K;
  if (M % 256 || Nc % 64 || nb * n > ws_floats - 64 || W > ST_WMAX ||
      M >= (1LL << 31) / 3)
    throw std::runtime_error("ewdml conv stem: wgrad needs N*H*W % 256 == 0, Nc % 64 == 0, "
                             "W <= 256");
  hipStream_t s = (hipStream_t)stream;
  float* slab = reinterpret_cast<float*>(ws);
  hipLaunchKernelGGL(k_conv_stem_wgrad, dim3((int)nb, Nc / 64), dim3(EW_BLOCK), 0, s,
                     reinterpret_cast<const uint16_t*>(dy), reinterpret_cast<const uint16_t*>(x),
                     slab, H, W, Nc, (int)M);
  EW_CHECK_LAUNCH();
  hipLaunchKernelGGL(k_conv_stem_reduce, dim3((int)((n + 7) / 8)), dim3(EW_BLOCK), 0, s, slab,
                     (int)nb, (int)n, reinterpret_cast<uint16_t*>(dw));
  EW_CHECK_LAUNCH();
}
