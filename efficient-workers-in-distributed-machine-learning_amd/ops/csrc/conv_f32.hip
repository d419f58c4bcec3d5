// fp32 convolutions on the gfx950 matrix cores: 3x3 / stride 1 / pad 1 and 1x1 implicit GEMMs
// (NHWC, fp32 operands, fp32 accumulate, v_mfma_f32_16x16x4_f32) -- forward, backward-data and
// backward-weight -- plus the 3-input-channel stem.  This is the reference-precision path: the
// reference trains in plain fp32 (PyTorch-parameter-server/src/distributed_worker.py:249-251,
// src/optim/sgd.py:59-91), so these kernels do exact fp32 products (no bf16/xf32 splitting).
//
// Budget.  fp32 MFMA runs at 64 FLOP/clk/SIMD (157 TF/s on 256 CUs), 1/16 of the bf16 rate, so a
// fp32 conv GEMM is compute-bound as soon as a block keeps its matrix pipes fed: a 128x128 output
// tile (4 waves x 64x64) does 4096 MFMA cycles per 32-deep k-step against 32 KB of operand loads
// (~19 GB/s per CU, served by L2 / Infinity Cache).  MIOpen's fp32 NHWC solvers reach 100-123 TF/s
// on VGG-11's forward layers but need a zero-fill kernel before every backward call and run the
// backward passes at 60-100 TF/s (profiles/vgg11_fp32_miopen.txt).
//
//   forward     y[m][n]  = sum_{k=(tap,c)} X~[m][k] * w[n][k]          X~ = im2col(x), implicit
//   bwd data   dx[m][c]  = sum_{k=(tap,n)} dY~[m][k] * w[n][8-tap][c]
//   bwd weight dw[n][k]  = sum_m dy[m][n] * X~[m][k]
//
// Operand images in LDS, one 32-deep k-step per stage (double buffered, register staged):
//  * KC ("k contiguous": forward A and B, backward-data A): [rows][32 floats], 128-B rows, 16-B
//    chunk c of row r at c ^ ((r >> 1) & 7) (the bf16 kernels' swizzle: a ds_read_b128 lane group
//    reading 16 rows at one chunk hits 16 distinct bank slots).  A lane reads 4 consecutive k of
//    its row with one ds_read_b128.
//  * RC ("rows contiguous": backward-data B, both weight-gradient operands): [32 k][cols + 4]
//    floats as they lie in global memory; a lane reads one element per MFMA (ds_read_b32, the
//    +4 pad puts k and k + 4 -- the two halves of a 32-lane group -- 16 banks apart).
// The MFMA k order is permuted consistently in both operands: MFMA jj of half-step kk gives lane
// group g the reduction index kk*16 + 4g + jj, which is what a b128 read of chunk kk*4 + g yields.
//
// 16x16x4 f32 MFMA operand map: A lane l = A[l & 15][l >> 4], B lane l = B[l >> 4][l & 15];
// D lane l reg q = D[4 (l >> 4) + q][l & 15].
#include <cstdio>
#include <cstdlib>

#include "bn_fin.h"
#include "common.h"
#include "conv_f32.h"
#include "ewdml_ops.h"
#include "wg_common.h"

namespace {

typedef float f32x4 __attribute__((ext_vector_type(4)));

constexpr int CF_BK = 32;  // reduction depth of one k-step (floats)
enum { CF_FWD = 0, CF_BWD = 1, CF_WGRAD = 2 };
#ifndef CF_PRIO
#define CF_PRIO 0  // 1: s_setprio(1) around each MFMA cluster -- measured 3 % slower (profiles/ab/README.md)
#endif

__device__ __forceinline__ int cf_off(int r, int c) {  // byte offset of chunk c of row r (KC)
  return r * 128 + ((c ^ ((r >> 1) & 7)) << 4);
}

struct CfGeom {
  int M;      // GEMM rows (fwd/bwd: pixels N*H*W; wgrad: output channels Nc)
  int Ncol;   // GEMM columns (fwd: Nc; bwd: C; wgrad: taps*C)
  int P;      // pixels N*H*W
  int H, W;
  int C;      // fwd/wgrad: input channels of x; bwd: output channels of dx
  int Nc;     // fwd/wgrad: output channels; bwd: the reduction channels (forward's output)
  int taps;   // 9 or 1
  int ksteps, kps;
  // batched GEMMs (Winograd: one per transform position): blockIdx.z = batch * nsplit + split,
  // operand / output pointers advance by these strides (elements) per batch
  int nsplit;
  long long a_bs, b_bs, o_bs;
  // B batch index = the 4x4 position (i, j) of the A batch with 0 <-> 3 swapped on both axes (the
  // Winograd transform of the 180-degree-rotated kernel: G J = rows 0 and 3 of G exchanged)
  int b_flip;
  // stride-2 convolutions (k_cf_gemm<..., STR = 2>): Ho x Wo = the output map (H / 2, W / 2).
  // Forward / weight gradient: H, W = the input map, GEMM rows / reduction = output pixels.
  // Backward data: H, W = Ho, Wo = dy's map, blockIdx.z = the dx phase (ph, pw) = (z >> 1, z & 1)
  // -- dx pixels (2i + ph, 2j + pw) -- whose rows are dy's pixels (i, j): tap (kh, kw) of the
  // kernel reaches dy pixel (i + eh, j + ew) with eh = 1 for (ph, kh) = (1, 0), else 0.  A phase
  // has (1 + ph)(1 + pw) taps of a 3x3 kernel; only phase 0 has the 1x1 kernel's tap (the others
  // are written as zeros)
  int S, Ho, Wo;
};

// stride-2 backward data: taps of phase (ph, pw) and tap tp of it -> dy offset (eh, ew) on dy's
// map and the kernel tap kh * 3 + kw it multiplies (1x1: phase 0's single tap)
__host__ __device__ __forceinline__ int cf_s2_ntaps(int taps, int ph, int pw) {
  return taps == 1 ? ((ph | pw) ? 0 : 1) : (1 + ph) * (1 + pw);
}
__device__ __forceinline__ void cf_s2_tap(int taps, int ph, int pw, int tp, int& eh, int& ew,
                                          int& wtap) {
  if (taps == 1) {
    eh = ew = wtap = 0;
    return;
  }
  const int nc = 1 + pw, a = tp / nc, b = tp - a * nc;
  const int kh = ph ? 2 * a : 1, kw = pw ? 2 * b : 1;
  eh = (ph && a == 0) ? 1 : 0;
  ew = (pw && b == 0) ? 1 : 0;
  wtap = kh * 3 + kw;
}

__device__ __forceinline__ int cf_flip4(int z) {  // (i, j) -> (p(i), p(j)), p: 0 <-> 3
  const int i = z >> 2, j = z & 3;
  return (((i == 0 || i == 3) ? 3 - i : i) << 2) | ((j == 0 || j == 3) ? 3 - j : j);
}

// Stage images: A then B, KC or RC by mode.
template <int MODE, int BM, int BN>
struct CfLayout {
  static constexpr bool A_KC = MODE != CF_WGRAD;
  static constexpr bool B_KC = MODE == CF_FWD;
  static constexpr int PA = BM + 4, PB = BN + 4;  // RC row pitches (floats)
  static constexpr int A_BYTES = A_KC ? BM * 128 : CF_BK * PA * 4;
  static constexpr int B_BYTES = B_KC ? BN * 128 : CF_BK * PB * 4;
  static constexpr int STAGE = A_BYTES + B_BYTES;
};

// fp32 MFMA shapes.  16x16x4 (4 accumulator regs, 32-cycle issue): A lane l = A[l & 15][l >> 4],
// B lane l = B[l >> 4][l & 15], D lane l reg e = D[4 (l >> 4) + e][l & 15].  32x32x2 (16 regs,
// 64-cycle issue, half the instructions per FLOP): A lane l = A[l & 31][l >> 5], B lane l =
// B[l >> 5][l & 31], D lane l reg e = D[8 (e >> 2) + 4 (l >> 5) + (e & 3)][l & 31].
typedef float f32x16 __attribute__((ext_vector_type(16)));
template <int SH>
struct CfMfma;
template <>
struct CfMfma<16> {
  typedef f32x4 acc_t;
  static constexpr int E = 4, G = 4;  // accumulator regs; lane groups (k values per MFMA)
  __device__ static __forceinline__ int out_row(int lane, int e) { return 4 * (lane >> 4) + e; }
  __device__ static __forceinline__ acc_t mma(float a, float b, const acc_t& c) {
    return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
  }
};
template <>
struct CfMfma<32> {
  typedef f32x16 acc_t;
  static constexpr int E = 16, G = 2;
  __device__ static __forceinline__ int out_row(int lane, int e) {
    return 8 * (e >> 2) + 4 * (lane >> 5) + (e & 3);
  }
  __device__ static __forceinline__ acc_t mma(float a, float b, const acc_t& c) {
    return __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, c, 0, 0, 0);
  }
};

// One k-step's MFMA operand fragments of a wave, read from an LDS stage.  Lane group g
// (lane / SH) takes the 8/G 16-B chunks r*G + g (r < 8/G) of the 32-deep step: read r holds
// k = 4 (r G + g) + jj in element jj, and MFMA (r, jj) consumes element jj of both operands, so
// every k is used exactly once with the same permutation in A and B.
template <int SH, int MI, int NJ>
struct CfFrag {
  static constexpr int R = 8 / CfMfma<SH>::G;
  f32x4 a[R][MI], b[R][NJ];
};

template <int MODE, int BM, int BN, int SH, int MI, int NJ>
__device__ __forceinline__ void cf_frag_read(const char* __restrict__ As,
                                             const char* __restrict__ Bs, int arow0, int bcol0,
                                             int lane, CfFrag<SH, MI, NJ>& f) {
  using L = CfLayout<MODE, BM, BN>;
  constexpr int R = CfFrag<SH, MI, NJ>::R;
  const int g = lane / SH, li = lane % SH;
#pragma unroll
  for (int r = 0; r < R; ++r) {
    const int ch = r * CfMfma<SH>::G + g;
#pragma unroll
    for (int i = 0; i < MI; ++i) {
      if constexpr (L::A_KC) {
        f.a[r][i] = *reinterpret_cast<const f32x4*>(As + cf_off(arow0 + i * SH + li, ch));
      } else {
        const float* ap = reinterpret_cast<const float*>(As) + 4 * ch * L::PA + arow0 + i * SH + li;
#pragma unroll
        for (int jj = 0; jj < 4; ++jj) f.a[r][i][jj] = ap[jj * L::PA];
      }
    }
#pragma unroll
    for (int j = 0; j < NJ; ++j) {
      if constexpr (L::B_KC) {
        f.b[r][j] = *reinterpret_cast<const f32x4*>(Bs + cf_off(bcol0 + j * SH + li, ch));
      } else {
        const float* bp = reinterpret_cast<const float*>(Bs) + 4 * ch * L::PB + bcol0 + j * SH + li;
#pragma unroll
        for (int jj = 0; jj < 4; ++jj) f.b[r][j][jj] = bp[jj * L::PB];
      }
    }
  }
}

// MFMAs of fragment reads [R0, R1) of a step: acc[i][j] += A[rows] * B[cols]^T over those k
template <int SH, int MI, int NJ, int R0, int R1>
__device__ __forceinline__ void cf_mma(const CfFrag<SH, MI, NJ>& f,
                                       typename CfMfma<SH>::acc_t (&acc)[MI][NJ]) {
  using F = CfMfma<SH>;
  if (CF_PRIO) __builtin_amdgcn_s_setprio(1);
#pragma unroll
  for (int r = R0; r < R1; ++r)
#pragma unroll
    for (int jj = 0; jj < 4; ++jj)
#pragma unroll
      for (int i = 0; i < MI; ++i)
#pragma unroll
        for (int j = 0; j < NJ; ++j) acc[i][j] = F::mma(f.a[r][i][jj], f.b[r][j][jj], acc[i][j]);
  if (CF_PRIO) __builtin_amdgcn_s_setprio(0);
}

// Staging registers of one operand: R 16-B vectors per thread (named members: no scratch); sc /
// sh: the k-step's BatchNorm scale / shift of a lazily applied forward A operand (CfLz)
struct CfRegs {
  f32x4 v0, v1, v2, v3;
  f32x4 sc, sh;
};

// A lazily applied BatchNorm + ReLU operand (k_cf_gemm<..., LZ = true>; 1x1 stride-1 convs only:
// no padding taps, whose zeros the transform would not keep).  The conv's input relu(bn(h)) --
// ResNet bottleneck conv3's, models/resnet.py -- is never written: the forward's A rows and the
// weight gradient's x rows are read from h, and relu(h * scale + shift) is formed in the staging
// registers on their way to LDS, exactly as k_bn_fwd_apply writes it (bitwise the materialised
// operand).  stats [4][C]: mean, invstd, scale, shift; nbt: the BN layer's num_batches_tracked
// (the forward counts the batch, once) or null.
struct CfLz {
  const float* stats;
  long long* nbt;
};
__device__ __forceinline__ f32x4 cf_bn_relu4(const f32x4& v, const f32x4& sc, const f32x4& sh) {
  f32x4 r;
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const float z = v[q] * sc[q] + sh[q];  // as k_bn_fwd_apply writes it
    r[q] = (z > 0.0f || z != z) ? z : 0.0f;
  }
  return r;
}
#define CF_FOR(R_, ...)                                                                         \
  do {                                                                                          \
    { constexpr int i = 0; auto& v = RG.v0; __VA_ARGS__; }                                     \
    if constexpr (R_ > 1) { constexpr int i = 1; auto& v = RG.v1; __VA_ARGS__; }               \
    if constexpr (R_ > 2) { constexpr int i = 2; auto& v = RG.v2; __VA_ARGS__; }               \
    if constexpr (R_ > 3) { constexpr int i = 3; auto& v = RG.v3; __VA_ARGS__; }               \
  } while (0)

// Per-thread operand staging state (NT threads).  KC tiles: thread t stages chunk t & 7 of rows
// (t >> 3) + (NT / 8) i (i < 8 BM / NT).  RC tiles ([32 k][BN cols]): BN/4 chunks per k-row,
// thread t stages chunk t % (BN/4) of k-rows t / (BN/4) + (4 NT / BN) i (i < 8 BN / NT).
// 16 zero bytes in device memory (zero-initialised at module load), read by masked-out loads
__device__ __attribute__((aligned(16))) float cf_zero_page[4];

// Raw buffer descriptor over [p, p + bytes) (p and bytes wave-uniform) and a 16-B load through it;
// offsets past the range read zeros (CF_OOB: never in range, the host keeps operands < 4 GB - 16)
constexpr unsigned CF_OOB = 0xFFFFFFF0u;
__device__ __forceinline__ __amdgpu_buffer_rsrc_t cf_rsrc(const float* p, unsigned bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(p), (short)0, (int)bytes, 0x00020000);
}
__device__ __forceinline__ f32x4 cf_bload(__amdgpu_buffer_rsrc_t r, unsigned voff, int soff) {
  return __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(r, (int)voff, soff, 0));
}

template <int MODE, int BM, int BN, int NT, int STR = 1, bool LZ = false>
struct CfStager {
  using L = CfLayout<MODE, BM, BN>;
  static constexpr int RA = 8 * BM / NT, RB = 8 * BN / NT;    // 16-B vectors per thread
  static_assert(RA >= 1 && RA <= 4 && RB >= 1 && RB <= 4, "staging registers");
  static constexpr int RCA = BM / 4, RCB = BN / 4;            // RC chunks per k-row
  static constexpr int RPA = NT / RCA, RPB = NT / RCB;        // RC k-rows per pass
  // KC im2col rows (fwd, bwd A): pixel and its (h, w)
  int am[RA], ah[RA], aw[RA];
  // wgrad B: the thread's column chunk's tap offset and channel
  int bdr, bdc, bc;
  const float* xa;  // A source
  const float* xb;  // B source
  int t, m0, n0;
  int ph, pw;  // stride-2 backward data: this block's dx phase
  // Buffer loads (32-bit byte offsets from a wave-uniform descriptor; every operand < 4 GB, checked
  // on the host): the per-lane part of each offset is fixed at init and the per-step part is a
  // scalar, so a step's address work is a few 32-bit adds instead of 64-bit multiply-adds
  // (fwd / bwd A: an add, the padding test and a select per load; B and wgrad A: soffset only).
  __amdgpu_buffer_rsrc_t rsa, rsb;
  unsigned aoff[RA], boff[RB];
  // LZ: the forward's scale / shift rows (read per k-step into CfRegs); the weight gradient's
  // fixed 4 columns' scale / shift
  const float* lzs;
  f32x4 wsc, wsh;

  __device__ __forceinline__ void lz_init(const CfGeom& g, const CfLz& lz) {
    static_assert(STR == 1 && (MODE == CF_FWD || MODE == CF_WGRAD), "lazy BN operand");
    if constexpr (MODE == CF_FWD) {
      lzs = lz.stats;
    } else {
      wsc = *reinterpret_cast<const f32x4*>(lz.stats + 2 * g.C + bc);
      wsh = *reinterpret_cast<const f32x4*>(lz.stats + 3 * g.C + bc);
    }
  }

  __device__ __forceinline__ void init(const CfGeom& g, const float* a_src, const float* b_src,
                                       int t_, int m0_, int n0_, int zb = 0) {
    t = t_;
    m0 = m0_;
    n0 = n0_;
    xa = a_src;
    xb = b_src;
    ph = zb >> 1;
    pw = zb & 1;
    if constexpr (L::A_KC) {
#pragma unroll
      for (int i = 0; i < RA; ++i) {
        const int m = m0 + (t >> 3) + (NT / 8) * i;
        if constexpr (STR == 2 && MODE == CF_FWD) {
          // row m = output pixel (n, oh, ow); its taps start at input pixel (n, 2 oh, 2 ow)
          const int HoWo = g.Ho * g.Wo;
          const int n = m / HoWo, hw = m - n * HoWo, oh = hw / g.Wo;
          ah[i] = 2 * oh;
          aw[i] = 2 * (hw - oh * g.Wo);
          am[i] = n * g.H * g.W + ah[i] * g.W + aw[i];
        } else {
          am[i] = m;
          const int hw = m % (g.H * g.W);
          ah[i] = hw / g.W;
          aw[i] = hw - ah[i] * g.W;
        }
      }
    }
    if constexpr (MODE == CF_WGRAD) {
      const int k = n0 + (t % RCB) * 4;  // column (tap, c) of this thread's chunk
      const int tap = k / g.C;
      bc = k - tap * g.C;
      bdr = g.taps == 1 ? 0 : tap / 3 - 1;
      bdc = g.taps == 1 ? 0 : tap - (tap / 3) * 3 - 1;
    }
    if constexpr (MODE == CF_FWD || MODE == CF_BWD) {
      const unsigned CH = MODE == CF_FWD ? g.C : g.Nc;
      const unsigned rows = (STR == 2 && MODE == CF_FWD)
                                ? (unsigned)(g.M / (g.Ho * g.Wo)) * g.H * g.W
                                : (unsigned)g.M;
      rsa = cf_rsrc(xa, rows * CH * 4u);
#pragma unroll
      for (int i = 0; i < RA; ++i) aoff[i] = ((unsigned)am[i] * CH + (t & 7) * 4) * 4u;
      if constexpr (MODE == CF_FWD) {
        // w[n][taps*C]: row n's chunk t & 7, the step adds s * 128 B
        const unsigned K = (unsigned)g.taps * g.C;
        rsb = cf_rsrc(xb, (unsigned)g.Ncol * K * 4u);
#pragma unroll
        for (int i = 0; i < RB; ++i)
          boff[i] = ((unsigned)(n0 + (t >> 3) + (NT / 8) * i) * K + (t & 7) * 4) * 4u;
      } else {
        // w[Nc][taps][C]: k-row kr of the step's 32 channels; the step adds
        // ((cb * 32) * taps + tap) * C floats
        rsb = cf_rsrc(xb, (unsigned)g.Nc * g.taps * g.C * 4u);
#pragma unroll
        for (int i = 0; i < RB; ++i)
          boff[i] = ((unsigned)(t / RCB + RPB * i) * g.taps * g.C + n0 + (t % RCB) * 4) * 4u;
      }
    } else {
      // dy[m][Nc]: k-row kr of the step's 32 pixels, the step adds s * 32 * Nc floats
      rsa = cf_rsrc(xa, (unsigned)g.ksteps * CF_BK * g.Nc * 4u);
#pragma unroll
      for (int i = 0; i < RA; ++i) aoff[i] = ((unsigned)(t / RCA + RPA * i) * g.Nc + m0 + (t % RCA) * 4) * 4u;
      if constexpr (STR == 1) {
        // x[m][C] (stride 1: one input pixel per output pixel): k-row kr, channel bc
        rsb = cf_rsrc(xb, (unsigned)g.ksteps * CF_BK * g.C * 4u);
#pragma unroll
        for (int i = 0; i < RB; ++i) boff[i] = ((unsigned)(t / RCB + RPB * i) * g.C + bc) * 4u;
      }
    }
  }

  // global -> registers for k-step s
  __device__ __forceinline__ void load(const CfGeom& g, int s, CfRegs& ra, CfRegs& rb) const {
    if constexpr (MODE == CF_FWD || MODE == CF_BWD) {
      // A: im2col of x (fwd, channels C) or dy (bwd, channels Nc)
      const int CH = MODE == CF_FWD ? g.C : g.Nc;
      const int CB = CH / CF_BK;
      const int tap = s / CB, cb = s - tap * CB;
      int dr, dc, wtap;
      if constexpr (STR == 2 && MODE == CF_BWD) {
        cf_s2_tap(g.taps, ph, pw, tap, dr, dc, wtap);
      } else {
        // computed unconditionally and then selected: a conditional division became a scalar
        // branch, which split the k-step's scheduling region
        const int q = tap / 3, one = g.taps == 1;
        dr = one ? 0 : q - 1;
        dc = one ? 0 : tap - q * 3 - 1;
        wtap = g.taps - 1 - tap;  // backward data: the 180-degree-rotated kernel's tap
      }
      {
        // out-of-image taps load the zero page: a select on the loaded VALUE would make hipcc
        // wait for this step's loads before the step's MFMAs (s_waitcnt vmcnt ahead of the
        // masking), a select on the ADDRESS does not
        // the address is formed unconditionally and then selected (a select of a computed
        // value stays a v_cndmask; selecting between computing it or not became a branch,
        // which split the k-step and kept the address arithmetic out of the MFMA stream)
        CfRegs& RG = ra;
        const unsigned sa = (unsigned)(((dr * g.W + dc) * CH + cb * CF_BK) * 4);  // wave-uniform
        CF_FOR(RA, {
          const bool ok = (unsigned)(ah[i] + dr) < (unsigned)g.H &&
                          (unsigned)(aw[i] + dc) < (unsigned)g.W;
          // out-of-image taps: an offset past the descriptor's range reads zeros
          v = cf_bload(rsa, ok ? aoff[i] + sa : CF_OOB, 0);
        });
      }
      if constexpr (LZ && MODE == CF_FWD) {
        // this step's channels cb*32 + chunk*4 .. + 3 (1x1: tap 0)
        const int c = cb * CF_BK + (t & 7) * 4;
        ra.sc = *reinterpret_cast<const f32x4*>(lzs + 2 * g.C + c);
        ra.sh = *reinterpret_cast<const f32x4*>(lzs + 3 * g.C + c);
      }
      if constexpr (MODE == CF_FWD) {
        // B: w[n][taps*C], k index s*32 + chunk*4
        CfRegs& RG = rb;
        CF_FOR(RB, { v = cf_bload(rsb, boff[i], s * CF_BK * 4); });
      } else {
        // B (RC): k-row kr = reduction channel n = cb*32 + kr at the flipped tap; columns c
        CfRegs& RG = rb;
        const int sb = ((cb * CF_BK) * g.taps + wtap) * g.C * 4;
        CF_FOR(RB, { v = cf_bload(rsb, boff[i], sb); });
      }
    } else {
      // wgrad: k = pixel m = s*32 + kr.  A (RC): dy[m][rows m0..]; B (RC): im2col x[m][(tap,c)]
      {
        CfRegs& RG = ra;
        CF_FOR(RA, { v = cf_bload(rsa, aoff[i], (int)((unsigned)s * CF_BK * g.Nc * 4u)); });
      }
      {
        const int HW = g.H * g.W;
        CfRegs& RG = rb;
        if constexpr (STR == 2) {
          // reduction index m = output pixel (n, oh, ow); tap at input (2 oh + bdr, 2 ow + bdc)
          const int HoWo = g.Ho * g.Wo;
          CF_FOR(RB, {
            const int m = s * CF_BK + t / RCB + RPB * i;
            const int n = m / HoWo, hw = m - n * HoWo, oh = hw / g.Wo;
            const int h = 2 * oh + bdr, w = 2 * (hw - oh * g.Wo) + bdc;
            const bool ok = (unsigned)h < (unsigned)g.H && (unsigned)w < (unsigned)g.W;
            const float* src =
                ok ? xb + ((long long)n * HW + h * g.W + w) * g.C + bc : cf_zero_page;
            v = *reinterpret_cast<const f32x4*>(src);
          });
        } else if (g.taps == 1) {
          // 1x1: the im2col row is the pixel itself -- no (h, w), no padding
          CF_FOR(RB, { v = cf_bload(rsb, boff[i], (int)((unsigned)s * CF_BK * g.C * 4u)); });
        } else {
          CF_FOR(RB, {
            const int m = s * CF_BK + t / RCB + RPB * i;
            const int hw = m % HW, h = hw / g.W, w = hw - h * g.W;
            const bool ok =
                (unsigned)(h + bdr) < (unsigned)g.H && (unsigned)(w + bdc) < (unsigned)g.W;
            const unsigned off =
                boff[i] + (unsigned)((s * CF_BK + bdr * g.W + bdc) * g.C) * 4u;
            v = cf_bload(rsb, ok ? off : CF_OOB, 0);
          });
        }
      }
    }
  }

  // registers -> LDS stage
  __device__ __forceinline__ void store(char* stage, const CfRegs& ra, const CfRegs& rb) const {
    char* As = stage;
    char* Bs = stage + L::A_BYTES;
    {
      const CfRegs& RG = ra;
      if constexpr (L::A_KC) {
        if constexpr (LZ && MODE == CF_FWD) {
          CF_FOR(RA, {
            *reinterpret_cast<f32x4*>(As + cf_off((t >> 3) + (NT / 8) * i, t & 7)) =
                cf_bn_relu4(v, RG.sc, RG.sh);
          });
        } else {
          CF_FOR(RA, { *reinterpret_cast<f32x4*>(As + cf_off((t >> 3) + (NT / 8) * i, t & 7)) = v; });
        }
      } else {
        CF_FOR(RA, {
          *reinterpret_cast<f32x4*>(As + ((t / RCA + RPA * i) * L::PA + (t % RCA) * 4) * 4) = v;
        });
      }
    }
    {
      const CfRegs& RG = rb;
      if constexpr (L::B_KC) {
        CF_FOR(RB, { *reinterpret_cast<f32x4*>(Bs + cf_off((t >> 3) + (NT / 8) * i, t & 7)) = v; });
      } else if constexpr (LZ && MODE == CF_WGRAD) {
        CF_FOR(RB, {
          *reinterpret_cast<f32x4*>(Bs + ((t / RCB + RPB * i) * L::PB + (t % RCB) * 4) * 4) =
              cf_bn_relu4(v, wsc, wsh);
        });
      } else {
        CF_FOR(RB, {
          *reinterpret_cast<f32x4*>(Bs + ((t / RCB + RPB * i) * L::PB + (t % RCB) * 4) * 4) = v;
        });
      }
    }
  }
};

// Epilogue: fp32 output (or split slab) + optional addend, forward BN partial sums of the output
// (sum, sum of squares per column over the block's BM rows -> row blockIdx.x of
// bnpart[2][M/BM][Ncol]) or the backward sums of CfBnBwd.  Waves form a WM x WN grid of
// (BM/WM) x (BN/WN) tiles of MI x NJ SH x SH MFMA blocks.
// RMAP (stride-2 backward data): GEMM row r = dy pixel (n, i, j) of an rHo x rWo map is written
// to dx pixel (n, 2 i + rph, 2 j + rpw) (out and addend; no slab, no BN sums on this path)
// 16-B load through to L2 (agent scope): data another block of this launch wrote write-through
__device__ __forceinline__ f32x4 cf_ld4_sc1(const float* p) {
  f32x4 v;
#pragma unroll
  for (int k = 0; k < 4; ++k)
    v[k] = __hip_atomic_load(const_cast<float*>(p) + k, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  return v;
}

template <int BM, int BN, int WM, int WN, int SH, int MI, int NJ, bool RMAP = false>
__device__ __forceinline__ void cf_epilogue(typename CfMfma<SH>::acc_t (&acc)[MI][NJ], char* smem,
                                            int wm, int wn, int lane, int m0, int n0, int M,
                                            int Nc, float* __restrict__ out,
                                            float* __restrict__ slab, float* __restrict__ bnpart,
                                            const CfBnBwd& bb, const float* __restrict__ addend,
                                            int rHo = 0, int rWo = 0, int rph = 0, int rpw = 0,
                                            int* redtk = nullptr, int nsplit = 1, int zs = 0) {
  using F = CfMfma<SH>;
  constexpr int E = F::E;
  const int row0 = m0 + wm * (BM / WM), col0 = n0 + wn * (BN / WN);
  const int li = lane % SH;
  auto row_of = [&](int i, int e) { return row0 + i * SH + F::out_row(lane, e); };
  auto col_of = [&](int j) { return col0 + j * SH + li; };
  auto orow = [&](int r) -> long long {
    if constexpr (!RMAP) {
      return r;
    } else {
      const int HoWo = rHo * rWo;
      const int n = r / HoWo, hw = r - n * HoWo, i = hw / rWo, j = hw - i * rWo;
      return (long long)n * 4 * HoWo + (2 * i + rph) * (2 * rWo) + 2 * j + rpw;
    }
  };
  if (slab) {
    float* sp = slab;  // this block's split slab (k_cf_gemm offsets it)
    if (!RMAP && redtk) {
      // in-launch split-K reduction (no reduction launch): the slab is stored write-through, the
      // tile's last split (ticket red[tile]) sums the splits in k_cf_slab_reduce's order, reading
      // the others with agent-scope loads (cdna_hip_programming.md Guideline 16)
#pragma unroll
      for (int i = 0; i < MI; ++i)
#pragma unroll
        for (int e = 0; e < E; ++e)
#pragma unroll
          for (int j = 0; j < NJ; ++j)
            __hip_atomic_store(sp + (long long)row_of(i, e) * Nc + col_of(j), acc[i][j][e],
                               __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
      int* flag = reinterpret_cast<int*>(smem);
      if (threadIdx.x == 0) {
        int* tk = redtk + blockIdx.x + gridDim.x * blockIdx.y;
        const int last =
            __hip_atomic_fetch_add(tk, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == nsplit - 1;
        if (last) __hip_atomic_store(tk, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        *flag = last;
      }
      __syncthreads();
      if (!*flag) return;
      const long long zstride = (long long)M * Nc;
      const float* base = slab - (long long)zs * zstride;
      // the tile's BM x BN block of every split (the own one re-read: the same bits) summed in
      // split order as float4 rows, k_cf_slab_reduce's expression per element
      constexpr int NTH = 64 * WM * WN, Q = BN / 4, CH = BM * Q / NTH;
      static_assert(BM * Q % NTH == 0, "tile chunks");
      f32x4 a[CH];
#pragma unroll
      for (int u = 0; u < CH; ++u) {
        const int c = (int)threadIdx.x + u * NTH, r = c / Q, q = c - r * Q;
        a[u] = cf_ld4_sc1(base + (long long)(m0 + r) * Nc + n0 + 4 * q);
      }
      for (int z = 1; z < nsplit; ++z) {
        f32x4 v[CH];
#pragma unroll
        for (int u = 0; u < CH; ++u) {
          const int c = (int)threadIdx.x + u * NTH, r = c / Q, q = c - r * Q;
          v[u] = cf_ld4_sc1(base + z * zstride + (long long)(m0 + r) * Nc + n0 + 4 * q);
        }
#pragma unroll
        for (int u = 0; u < CH; ++u) a[u] += v[u];
      }
#pragma unroll
      for (int u = 0; u < CH; ++u) {
        const int c = (int)threadIdx.x + u * NTH, r = c / Q, q = c - r * Q;
        const long long o = (long long)(m0 + r) * Nc + n0 + 4 * q;
        f32x4 w = a[u];
        if (addend) w += *reinterpret_cast<const f32x4*>(addend + o);
        *reinterpret_cast<f32x4*>(out + o) = w;
      }
      return;
    }
#pragma unroll
    for (int i = 0; i < MI; ++i)
#pragma unroll
      for (int e = 0; e < E; ++e)
#pragma unroll
        for (int j = 0; j < NJ; ++j) sp[(long long)row_of(i, e) * Nc + col_of(j)] = acc[i][j][e];
    return;
  }
  if (addend) {
    float av[MI][NJ][E];
#pragma unroll
    for (int i = 0; i < MI; ++i)
#pragma unroll
      for (int j = 0; j < NJ; ++j)
#pragma unroll
        for (int e = 0; e < E; ++e)
          av[i][j][e] = addend[orow(row_of(i, e)) * Nc + col_of(j)];
#pragma unroll
    for (int i = 0; i < MI; ++i)
#pragma unroll
      for (int j = 0; j < NJ; ++j)
#pragma unroll
        for (int e = 0; e < E; ++e) acc[i][j][e] += av[i][j][e];
  }
#pragma unroll
  for (int i = 0; i < MI; ++i)
#pragma unroll
    for (int e = 0; e < E; ++e)
#pragma unroll
      for (int j = 0; j < NJ; ++j) out[orow(row_of(i, e)) * Nc + col_of(j)] = acc[i][j][e];
  if (RMAP || !bnpart) return;
  float* red = reinterpret_cast<float*>(smem);  // [wm][wn][2][BN/WN]
  const long long nrows = M / BM;
  float sm[NJ], sq[NJ];
#pragma unroll
  for (int j = 0; j < NJ; ++j) {
    sm[j] = sq[j] = 0.0f;
    const int c = col_of(j);
    if (bb.h) {
      const float mean = bb.stats[c], sc = bb.stats[2 * Nc + c], sh = bb.stats[3 * Nc + c];
      const uint32_t HoWo = (uint32_t)bb.Ho * bb.Wo;
#pragma unroll
      for (int i = 0; i < MI; ++i) {
        // all window codes, then all h values are loaded before any use (batched round trips)
        uint32_t hr[E];
#pragma unroll
        for (int e = 0; e < E; ++e) hr[e] = row_of(i, e);
        if (bb.code) {
          uint8_t kc[E];
#pragma unroll
          for (int e = 0; e < E; ++e) kc[e] = bb.code[(size_t)hr[e] * Nc + c];
#pragma unroll
          for (int e = 0; e < E; ++e) hr[e] = cf_pool_row(hr[e], HoWo, (uint32_t)bb.Wo, kc[e]);
        }
        float xv[E], rv[E];
#pragma unroll
        for (int e = 0; e < E; ++e) {
          xv[e] = bb.h[(size_t)hr[e] * Nc + c];
          rv[e] = bb.res ? bb.res[(size_t)hr[e] * Nc + c] : 0.0f;
        }
#pragma unroll
        for (int e = 0; e < E; ++e) {
          const float d = acc[i][j][e];
          float v = xv[e] * sc + sh;  // the BN kernels' arithmetic (no contraction)
          if (bb.res) v = v + rv[e];
          const float dz = (bb.relu == 0 || !(v <= 0.0f)) ? d : 0.0f;
          sm[j] += dz;
          sq[j] += dz * (xv[e] - mean);
        }
      }
    } else {
#pragma unroll
      for (int i = 0; i < MI; ++i)
#pragma unroll
        for (int e = 0; e < E; ++e) {
          const float v = acc[i][j][e];
          sm[j] += v;
          sq[j] += v * v;
        }
    }
    // lanes holding the same column: SH = 16 -> l, l^16, l^32, l^48; SH = 32 -> l, l^32
    if constexpr (SH == 16) {
      sm[j] += __shfl_xor(sm[j], 16, 64);
      sq[j] += __shfl_xor(sq[j], 16, 64);
    }
    sm[j] += __shfl_xor(sm[j], 32, 64);
    sq[j] += __shfl_xor(sq[j], 32, 64);
  }
  __syncthreads();  // main loop finished reading smem
  constexpr int CW = BN / WN;  // columns per wave
  if (wm > 0 && lane < SH) {
#pragma unroll
    for (int j = 0; j < NJ; ++j) {
      red[((wm * WN + wn) * 2 + 0) * CW + j * SH + lane] = sm[j];
      red[((wm * WN + wn) * 2 + 1) * CW + j * SH + lane] = sq[j];
    }
  }
  __syncthreads();
  if (wm == 0 && lane < SH) {
#pragma unroll
    for (int j = 0; j < NJ; ++j) {
      float a = sm[j], q = sq[j];
#pragma unroll
      for (int r = 1; r < WM; ++r) {  // fixed order
        a += red[((r * WN + wn) * 2 + 0) * CW + j * SH + lane];
        q += red[((r * WN + wn) * 2 + 1) * CW + j * SH + lane];
      }
      const int c = col0 + j * SH + lane;
      bnpart[(long long)blockIdx.x * Nc + c] = a;
      bnpart[(nrows + blockIdx.x) * Nc + c] = q;
    }
  }
}

// The GEMM kernel: block = 8 waves (two per SIMD) in a WM x (8/WM) grid over a BM x BN tile, one
// 32-deep k-step per iteration through two LDS stages and two staging register sets (step s+2 is
// loaded while s computes and s+1 is written), split z covers k-steps
// [z*kps, min((z+1)*kps, ksteps)).
// WPE: waves per SIMD the register allocation must allow (0: the compiler's choice)
// LZ: a lazily applied BatchNorm + ReLU operand (CfLz): forward A / weight-gradient B
template <int MODE, int BM, int BN, int WM, int WN, int SH, int STR = 1, int WPE = 0,
          bool LZ = false>
__global__ __launch_bounds__(64 * WM * WN, WPE) void k_cf_gemm(const float* __restrict__ a_src,
                                                   const float* __restrict__ b_src,
                                                   float* __restrict__ out,
                                                   float* __restrict__ slab, CfGeom geo,
                                                   float* __restrict__ bnpart, CfBnBwd bb,
                                                   const float* __restrict__ addend, EwBnFin fin,
                                                   WgOut wo, int* __restrict__ red, CfLz lz) {
  using L = CfLayout<MODE, BM, BN>;
  using acc_t = typename CfMfma<SH>::acc_t;
  constexpr int NT = 64 * WM * WN;
  constexpr int MI = BM / WM / SH, NJ = BN / WN / SH;
  static_assert(MI >= 1 && NJ >= 1 && MI * SH * WM == BM && NJ * SH * WN == BN, "wave tiling");
  static_assert(NT >= EW_BLOCK && 2 * L::STAGE >= 3 * EW_WAVES * EW_FIN_CH * 8, "finalize rider");
  __shared__ __attribute__((aligned(16))) char smem[2 * L::STAGE];
  int gz = gridDim.z;
  if constexpr (MODE != CF_FWD) {
    // riders (cf_gemm: extra z slices after the GEMM's, dispatched last): a BatchNorm backward
    // finalisation (weight-gradient launches; one channel group per block, bn_fin.h) and a
    // deferred Winograd weight-gradient output transform (backward-data launches; NT element
    // groups per block, wg_common.h)
    // (each kind compiled only into the mode it rides in: the other's registers stay out)
    if constexpr (MODE != CF_WGRAD) fin.ngrp = 0;
    // (the transform rides only in 128-row stride-1 tiles: in the 64x64 one it doubled the VGPRs)
    if constexpr (MODE != CF_BWD || BM != 128 || STR != 1) wo.src = nullptr;
    if (fin.ngrp || wo.src) {
      const int gxy = gridDim.x * gridDim.y;
      const int nwb = wo.src ? (wo.Nc * (wo.C / WG2_VW) + NT - 1) / NT : 0;
      const int zf = (fin.ngrp + gxy - 1) / gxy, zw = (nwb + gxy - 1) / gxy;
      gz -= zf + zw;
      if ((int)blockIdx.z >= gz) {
        const int rz = (int)blockIdx.z - gz, bxy = blockIdx.y * gridDim.x + blockIdx.x;
        if (rz < zf) {
          const int g = rz * gxy + bxy;
          // 8 rows in flight: no more registers than the GEMM's own (16 raised the 64x64 tile's)
          if constexpr (MODE == CF_WGRAD)
            if (g < fin.ngrp) ew_bn_bwd_fin_group<2, 8>(fin, g, reinterpret_cast<double*>(smem));
        } else {
          const int g = (rz - zf) * gxy + bxy;
          if constexpr (MODE == CF_BWD && BM == 128 && STR == 1)
            if (g < nwb)
              wg_wgrad_out<2>(wo.src, wo.nsplit, wo.dw, wo.Nc, wo.C,
                              (long long)g * NT + threadIdx.x);
        }
        return;
      }
    }
  }
  const int t = threadIdx.x, lane = t & 63, wq = t >> 6;
  const int wm = wq / WN, wn = wq % WN;
  const int m0 = blockIdx.x * BM, n0 = blockIdx.y * BN;
  const int zb = blockIdx.z / geo.nsplit, zs = blockIdx.z - zb * geo.nsplit;
  a_src += zb * geo.a_bs;
  b_src += (geo.b_flip ? cf_flip4(zb) : zb) * geo.b_bs;
  out += zb * geo.o_bs;
  // slabs [split][batch][M][Ncol]: the reduction sums the splits of a contiguous batch run
  if (slab) slab += (long long)(zs * (gz / geo.nsplit) + zb) * geo.M * geo.Ncol;
  // stride-2 backward data: z = dx phase, heaviest first (3x3: z 0 = phase (1, 1) with 4 taps
  // ... z 3 = phase (0, 0) with 1; blocks dispatch in z order, so the light phases backfill)
  constexpr bool S2B = STR == 2 && MODE == CF_BWD;
  const int phase = (S2B && geo.taps != 1) ? 3 - zb : zb;
  const int kbeg = zs * geo.kps;
  const int ksteps =
      S2B ? cf_s2_ntaps(geo.taps, phase >> 1, phase & 1) * (geo.Nc / CF_BK) : geo.ksteps;
  const int kend = min(kbeg + geo.kps, ksteps);
  CfStager<MODE, BM, BN, NT, STR, LZ> st;
  st.init(geo, a_src, b_src, t, m0, n0, phase);
  if constexpr (LZ) {
    st.lz_init(geo, lz);
    if constexpr (MODE == CF_FWD)
      if (lz.nbt && blockIdx.x == 0 && blockIdx.y == 0 && blockIdx.z == 0 && t == 0) *lz.nbt += 1;
  }

  acc_t acc[MI][NJ];
#pragma unroll
  for (int i = 0; i < MI; ++i)
#pragma unroll
    for (int j = 0; j < NJ; ++j) acc[i][j] = acc_t{};

  // Two LDS stages and two staging register sets: step s + 2 is loaded while step s computes
  // and step s + 1 (loaded one step earlier) is written; one barrier per step.  Loads past the
  // end are clamped re-loads of the last step.
  using Frag = CfFrag<SH, MI, NJ>;
  const int arow0 = wm * (BM / WM), bcol0 = wn * (BN / WN);
  const int n = kend - kbeg;
  if (n > 0) {
    const int last = kend - 1;
    CfRegs ra[2], rb[2];
    st.load(geo, kbeg, ra[0], rb[0]);
    st.store(smem, ra[0], rb[0]);
    st.load(geo, min(kbeg + 1, last), ra[1], rb[1]);
    __syncthreads();
    // pairs of steps without a guard (a branch around the MFMAs de-pipelines hipcc's waits)
    const int nfull = n - (n & 1);
    for (int i0 = 0; i0 < nfull; i0 += 2) {
#pragma unroll
      for (int u = 0; u < 2; ++u) {
        const char* cs = smem + u * L::STAGE;
        Frag fr;
        // fragment reads first: the loads' address arithmetic then runs under their latency
        cf_frag_read<MODE, BM, BN, SH, MI, NJ>(cs, cs + L::A_BYTES, arow0, bcol0, lane, fr);
        st.load(geo, min(kbeg + i0 + u + 2, last), ra[u], rb[u]);
        cf_mma<SH, MI, NJ, 0, Frag::R>(fr, acc);
        st.store(smem + (u ^ 1) * L::STAGE, ra[u ^ 1], rb[u ^ 1]);
        __syncthreads();
      }
    }
    if (n & 1) {  // the last step (stage 0)
      Frag fr;
      cf_frag_read<MODE, BM, BN, SH, MI, NJ>(smem, smem + L::A_BYTES, arow0, bcol0, lane, fr);
      cf_mma<SH, MI, NJ, 0, Frag::R>(fr, acc);
    }
  }
  __syncthreads();  // the epilogue reuses smem
  cf_epilogue<BM, BN, WM, WN, SH, MI, NJ, S2B>(acc, smem, wm, wn, lane, m0, n0, geo.M, geo.Ncol,
                                               out, slab, bnpart, bb, addend, geo.H, geo.W,
                                               phase >> 1, phase & 1, red, geo.nsplit, zs);
}

// ---------------------------------------------------------------------------------------------
// LDS-DMA staging (buffer_load_dwordx4 ... lds): the forward GEMM's KC operand tiles go from global
// memory straight into LDS, no staging registers and no ds_write pass.  One wave instruction fills
// 1 KB = 8 consecutive 128-B rows lane-linearly (lane l -> byte 16 l), so the KC swizzle moves to
// the SOURCE: lane l loads chunk (l & 7) ^ ((r >> 1) & 7) of its row r, which lands at slot l & 7 =
// the position cf_off(r, chunk) expects (the permutation is an involution; the fragment reads are
// unchanged).  Padding taps read zeros through an out-of-range buffer offset, as in CfStager.
// s_waitcnt on the vector-memory counter only (expcnt / lgkmcnt left at their maxima)
template <int N>
__device__ __forceinline__ void cf_wait_vm() {
  static_assert(N >= 0 && N < 64, "vmcnt range");
  __builtin_amdgcn_s_waitcnt((N & 15) | ((N >> 4) << 14) | (7 << 4) | (15 << 8));
}

typedef __attribute__((address_space(3))) void* cf_lds_ptr;

template <int BM, int BN, int NT>
struct CfGlds {
  static constexpr int RA = 8 * BM / NT, RB = 8 * BN / NT;  // wave instructions per operand
  static constexpr int LPS = RA + RB;                        // loads per k-step per thread
  static constexpr int A_BYTES = BM * 128;
  __amdgpu_buffer_rsrc_t rsa, rsb;
  unsigned aoff[RA], boff[RB];
  int ah[RA], aw[RA];
  int dst0;  // this wave's first 1-KB row group in a stage image (bytes)

  __device__ __forceinline__ void init(const CfGeom& g, const float* a_src, const float* b_src,
                                       int t, int m0, int n0) {
    dst0 = (t >> 6) * 8 * 128;
    const unsigned K = (unsigned)g.taps * g.C;
    rsa = cf_rsrc(a_src, (unsigned)g.M * g.C * 4u);
    rsb = cf_rsrc(b_src, (unsigned)g.Ncol * K * 4u);
#pragma unroll
    for (int i = 0; i < RA; ++i) {
      const int r = (t >> 3) + (NT / 8) * i;
      const int m = m0 + r;
      const int hw = m % (g.H * g.W);
      ah[i] = hw / g.W;
      aw[i] = hw - ah[i] * g.W;
      const unsigned c = (unsigned)((t & 7) ^ ((r >> 1) & 7));
      aoff[i] = ((unsigned)m * g.C + c * 4) * 4u;
    }
#pragma unroll
    for (int i = 0; i < RB; ++i) {
      const int r = (t >> 3) + (NT / 8) * i;
      const unsigned c = (unsigned)((t & 7) ^ ((r >> 1) & 7));
      boff[i] = ((unsigned)(n0 + r) * K + c * 4) * 4u;
    }
  }

  // DMA k-step s into the stage image at `stage`
  __device__ __forceinline__ void issue(const CfGeom& g, int s, char* stage) const {
    const int CB = g.C / CF_BK;
    const int tap = s / CB, cb = s - tap * CB;
    const int q = tap / 3, one = g.taps == 1;
    const int dr = one ? 0 : q - 1, dc = one ? 0 : tap - q * 3 - 1;
    const unsigned sa = (unsigned)(((dr * g.W + dc) * g.C + cb * CF_BK) * 4);
#pragma unroll
    for (int i = 0; i < RA; ++i) {
      const bool ok = (unsigned)(ah[i] + dr) < (unsigned)g.H && (unsigned)(aw[i] + dc) < (unsigned)g.W;
      __builtin_amdgcn_raw_ptr_buffer_load_lds(
          rsa, (cf_lds_ptr)(stage + dst0 + (NT / 8) * i * 128), 16, ok ? aoff[i] + sa : CF_OOB, 0,
          0, 0);
    }
#pragma unroll
    for (int i = 0; i < RB; ++i)
      __builtin_amdgcn_raw_ptr_buffer_load_lds(
          rsb, (cf_lds_ptr)(stage + A_BYTES + dst0 + (NT / 8) * i * 128), 16, boff[i],
          s * CF_BK * 4, 0, 0);
  }
};

// Forward GEMM (stride 1) with LDS-DMA staging through three stage images: step s + 2 is in flight
// while s computes; one counted vmcnt (step s landed, s + 1 may not have) and one raw barrier per
// step, never a vmcnt(0) inside the loop (a __syncthreads() would drain the DMA queue)
template <int BM, int BN, int WM, int WN, int SH, int WPE = 0>
__global__ __launch_bounds__(64 * WM * WN, WPE) void k_cf_gemm_gl(const float* __restrict__ a_src,
                                                      const float* __restrict__ b_src,
                                                      float* __restrict__ out,
                                                      float* __restrict__ slab, CfGeom geo,
                                                      float* __restrict__ bnpart, CfBnBwd bb,
                                                      const float* __restrict__ addend) {
  using L = CfLayout<CF_FWD, BM, BN>;
  using acc_t = typename CfMfma<SH>::acc_t;
  constexpr int NT = 64 * WM * WN;
  constexpr int MI = BM / WM / SH, NJ = BN / WN / SH;
  static_assert(MI >= 1 && NJ >= 1 && MI * SH * WM == BM && NJ * SH * WN == BN, "wave tiling");
  __shared__ __attribute__((aligned(16))) char smem[3 * L::STAGE];
  const int t = threadIdx.x, lane = t & 63, wq = t >> 6;
  const int wm = wq / WN, wn = wq % WN;
  const int m0 = blockIdx.x * BM, n0 = blockIdx.y * BN;
  const int zb = blockIdx.z / geo.nsplit, zs = blockIdx.z - zb * geo.nsplit;
  a_src += zb * geo.a_bs;
  b_src += (geo.b_flip ? cf_flip4(zb) : zb) * geo.b_bs;
  out += zb * geo.o_bs;
  if (slab) slab += (long long)(zs * (gridDim.z / geo.nsplit) + zb) * geo.M * geo.Ncol;
  const int kbeg = zs * geo.kps;
  const int kend = min(kbeg + geo.kps, geo.ksteps);
  CfGlds<BM, BN, NT> st;
  st.init(geo, a_src, b_src, t, m0, n0);

  acc_t acc[MI][NJ];
#pragma unroll
  for (int i = 0; i < MI; ++i)
#pragma unroll
    for (int j = 0; j < NJ; ++j) acc[i][j] = acc_t{};

  using Frag = CfFrag<SH, MI, NJ>;
  const int arow0 = wm * (BM / WM), bcol0 = wn * (BN / WN);
  const int n = kend - kbeg;
  if (n > 0) {
    const int last = kend - 1;
    st.issue(geo, kbeg, smem);
    st.issue(geo, min(kbeg + 1, last), smem + L::STAGE);
    int cur = 0;  // stage of step i; step i + 2 goes to the stage read at step i - 1
    for (int i = 0; i < n; ++i) {
      cf_wait_vm<CfGlds<BM, BN, NT>::LPS>();
      __builtin_amdgcn_s_barrier();
      const int nxt = cur == 0 ? 2 : cur - 1;
      st.issue(geo, min(kbeg + i + 2, last), smem + nxt * L::STAGE);
      const char* cs = smem + cur * L::STAGE;
      Frag fr;
      cf_frag_read<CF_FWD, BM, BN, SH, MI, NJ>(cs, cs + L::A_BYTES, arow0, bcol0, lane, fr);
      cf_mma<SH, MI, NJ, 0, Frag::R>(fr, acc);
      cur = cur == 2 ? 0 : cur + 1;
    }
  }
  cf_wait_vm<0>();
  __syncthreads();  // the epilogue reuses smem
  cf_epilogue<BM, BN, WM, WN, SH, MI, NJ, false>(acc, smem, wm, wn, lane, m0, n0, geo.M,
                                                 geo.Ncol, out, slab, bnpart, bb, addend);
}

// out[i] = sum_z slab[z][i] (+ addend), 8 elements per thread
__global__ __launch_bounds__(EW_BLOCK) void k_cf_slab_reduce(const float* __restrict__ slab,
                                                             int nsplit, long long n,
                                                             float* __restrict__ out,
                                                             const float* __restrict__ addend) {
  const long long nv = n / 4;
  for (long long v = blockIdx.x * (long long)EW_BLOCK + threadIdx.x; v < nv;
       v += (long long)gridDim.x * EW_BLOCK) {
    const f32x4* p = reinterpret_cast<const f32x4*>(slab) + v;
    f32x4 a = p[0];
    for (int z = 1; z < nsplit; ++z) a += p[(long long)z * (n / 4)];  // fixed order
    if (addend) a += reinterpret_cast<const f32x4*>(addend)[v];
    reinterpret_cast<f32x4*>(out)[v] = a;
  }
}

// Split-K reduction that also writes the BN partial sums of its output (forward sums or the
// backward sums of CfBnBwd).  Block b: rows [b * rpb, (b + 1) * rpb) x all Nc columns; thread:
// column quad t % tpr (tpr = Nc / 4), rows t / tpr + k * rpi; one partial row per block.
__global__ __launch_bounds__(EW_BLOCK) void k_cf_slab_reduce_bn(const float* __restrict__ slab,
                                                                int nsplit, int M, int Nc,
                                                                float* __restrict__ out,
                                                                float* __restrict__ bnpart,
                                                                int rpb, CfBnBwd bb,
                                                                const float* __restrict__ addend) {
  __shared__ float red[2][EW_BLOCK * 4];  // [2][rpi][Nc]: rpi * Nc = 4 * EW_BLOCK
  const int tpr = Nc >> 2, rpi = EW_BLOCK / tpr;
  const int t = threadIdx.x, gq = t % tpr, rg = t / tpr;
  const int c0 = gq * 4;
  const long long n = (long long)M * Nc;
  const int r0 = blockIdx.x * rpb, r1 = min(r0 + rpb, M);
  float s1[4], s2[4], mean[4], sc[4], sh[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) s1[j] = s2[j] = 0.0f;
  if (bb.h && rg < rpi) {
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      mean[j] = bb.stats[c0 + j];
      sc[j] = bb.stats[2 * Nc + c0 + j];
      sh[j] = bb.stats[3 * Nc + c0 + j];
    }
  }
  const uint32_t HoWo = (uint32_t)bb.Ho * bb.Wo;
  if (rg < rpi) {
    for (int r = r0 + rg; r < r1; r += rpi) {
      const long long o = (long long)r * Nc + c0;
      const f32x4* p = reinterpret_cast<const f32x4*>(slab + o);
      f32x4 a = p[0];
      for (int z = 1; z < nsplit; ++z) a += p[(long long)z * (n / 4)];
      if (addend) a += *reinterpret_cast<const f32x4*>(addend + o);
      *reinterpret_cast<f32x4*>(out + o) = a;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const float d = a[j];
        if (bb.h) {
          uint32_t hr = (uint32_t)r;
          if (bb.code) hr = cf_pool_row((uint32_t)r, HoWo, (uint32_t)bb.Wo, bb.code[o + j]);
          const float x = bb.h[(size_t)hr * Nc + c0 + j];
          float v = x * sc[j] + sh[j];
          if (bb.res) v = v + bb.res[(size_t)hr * Nc + c0 + j];
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
    for (int j = 0; j < 4; ++j) {
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

// ---------------------------------------------------------------------------------------------
// Stem (C = 3): K = 27 = 9 taps x 3 channels (the channels_last weight order), padded to 28 =
// seven 16x16x4 MFMA steps.  Forward block = 128 pixels x 64 channels (wave v: pixels 32v..32v+31
// = 2 x 4 tiles), im2col gathered from an LDS copy of the input rows the block touches, output
// staged in LDS for 16-B stores, BN partial sums from the registers.
constexpr int CS_K = 27, CS_KP = 28;
constexpr int CS_WMAX = 256;
template <int PIX>
constexpr int cs_patch_floats() { return (PIX + 2 * CS_WMAX + 2) * 3 + 8; }

template <int PIX, int NT = EW_BLOCK>
__device__ __forceinline__ int cs_patch(const float* __restrict__ x, int m0, int W, int M,
                                        float* patch, int t) {
  int lo = (m0 - W - 1) * 3;
  lo = lo < 0 ? 0 : (lo & ~3);
  int hi = ((m0 + PIX + W + 1) * 3 + 3) & ~3;
  hi = hi > 3 * M ? 3 * M : hi;
  const int nch = (hi - lo) >> 2;
  for (int c = t; c < nch; c += NT)
    *reinterpret_cast<f32x4*>(patch + 4 * c) = *reinterpret_cast<const f32x4*>(x + lo + 4 * c);
  return lo;
}

__device__ __forceinline__ float cs_x(const float* patch, int lo, int m, int h, int w, int H,
                                      int W, int k) {
  const int tap = k / 3, c = k - 3 * tap;
  const int dr = tap / 3 - 1, dc = tap - 3 * (tap / 3) - 1;
  const bool ok = k < CS_K && (unsigned)(h + dr) < (unsigned)H && (unsigned)(w + dc) < (unsigned)W;
  return ok ? patch[(m + dr * W + dc) * 3 + c - lo] : 0.0f;
}

__global__ __launch_bounds__(EW_BLOCK) void k_cf_stem_fwd(const float* __restrict__ x,
                                                          const float* __restrict__ w,
                                                          float* __restrict__ y, int H, int W,
                                                          int Nc, int M,
                                                          float* __restrict__ bnpart, int nrows) {
  // the output staging tile aliases the input patch and the weights (dead after the MFMAs): ~37
  // KB of LDS, 4 blocks per CU -- the grid's 4 blocks per CU in one round (53 KB: 3 + a tail of 1)
  constexpr int PF = (cs_patch_floats<128>() + 3) & ~3, WF = 64 * (CS_KP + 8), YF = 128 * 68;
  __shared__ __attribute__((aligned(16))) float smem[PF + WF > YF ? PF + WF : YF];
  __shared__ float red[EW_WAVES][2][64];
  float* patch = smem;
  float* wsm = smem + PF;
  float* ysm = smem;
  // wsm pitch: 36 floats puts the 16 channel rows x 4 k of a b read on 64 distinct banks (32 put
  // them on 8: 8-way conflicts on every weight read)
  constexpr int WP = CS_KP + 8;
  const int t = threadIdx.x, lane = t & 63, wv = t >> 6, li = lane & 15, g = lane >> 4;
  const int m0 = blockIdx.x * 128, n0 = blockIdx.y * 64;
  // the block's 64 x 27 weights: every load of the thread issued before its first LDS write (a
  // copy loop waited for each load in turn: 7 round trips at the head of every block)
  constexpr int WR = (64 * CS_KP + EW_BLOCK - 1) / EW_BLOCK;
  float wr[WR];
#pragma unroll
  for (int r = 0; r < WR; ++r) {
    const int e = min(t + r * EW_BLOCK, 64 * CS_KP - 1), nn = e / CS_KP, k = e - nn * CS_KP;
    wr[r] = w[(long long)(n0 + nn) * CS_K + min(k, CS_K - 1)];
  }
  const int lo = cs_patch<128>(x, m0, W, M, patch, t);
#pragma unroll
  for (int r = 0; r < WR; ++r) {
    const int e = t + r * EW_BLOCK, nn = e / CS_KP, k = e - nn * CS_KP;
    if (e < 64 * CS_KP) wsm[nn * WP + k] = k < CS_K ? wr[r] : 0.0f;
  }
  __syncthreads();
  const int HW = H * W;
  float a[2][7];
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int m = m0 + 32 * wv + 16 * i + li;
    const int p = m % HW, h = p / W, ww = p - h * W;
#pragma unroll
    for (int s = 0; s < 7; ++s) a[i][s] = cs_x(patch, lo, m, h, ww, H, W, 4 * s + g);
  }
  f32x4 acc[2][4];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
#pragma unroll
    for (int i = 0; i < 2; ++i) acc[i][j] = f32x4{0.0f, 0.0f, 0.0f, 0.0f};
#pragma unroll
    for (int s = 0; s < 7; ++s) {
      const float b = wsm[(16 * j + li) * WP + 4 * s + g];
#pragma unroll
      for (int i = 0; i < 2; ++i)
        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[i][s], b, acc[i][j], 0, 0, 0);
    }
  }
  float sm[4], sq[4];
  __syncthreads();  // every wave is done with patch / wsm before ysm overwrites them
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    sm[j] = sq[j] = 0.0f;
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const float v = acc[i][j][q];
        ysm[(32 * wv + 16 * i + 4 * g + q) * 68 + 16 * j + li] = v;
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
  for (int u = 0; u < 8; ++u) {  // 128 rows x 16 quads
    const int e = t + EW_BLOCK * u, r = e >> 4, ch = e & 15;
    *reinterpret_cast<f32x4*>(y + (long long)(m0 + r) * Nc + n0 + ch * 4) =
        *reinterpret_cast<const f32x4*>(ysm + r * 68 + ch * 4);
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

// Stem weight gradient dw[n][k] = sum_m dy[m][n] x~[m][k]: block = 256 pixels x 64 channels, 512
// threads (the ~116 KB of LDS allow one block per CU: 8 waves, not 4, keep its loads in flight).
// dy rows ([256 m][64 n], RC) and the im2col rows ([256 m][28 k], RC) go to LDS; wave v computes
// the 16 x 16 tile n0 + 16 (v & 3) x k 16 (v >> 2) over all 256 m (64 MFMA k-steps), fp32 partial
// [64][27] per block into the slab, summed by k_cf_stem_reduce.
// LAZY: dy is not materialised -- it is the BatchNorm(+ReLU)(+2x2 pool) backward of the stem's
// output, formed here from that layer's input h (= the stem output), the gradient of its
// (pooled) output, its pool codes, stats [4][Nc] and coef [2][Nc] with k_bn_bwd_apply's
// expressions (nn.hip: the same bits), so the BN backward's apply pass is not run at all.
struct CsLazy {
  const float* h;
  const float* dnext;
  const uint8_t* code;
  const float* stats;
  const float* coef;
  int pool;
};
constexpr int CS_WG_THREADS = 512;

template <bool LAZY>
__global__ __launch_bounds__(CS_WG_THREADS) void k_cf_stem_wgrad(const float* __restrict__ dy,
                                                                 const float* __restrict__ x,
                                                                 float* __restrict__ slab, int H,
                                                                 int W, int Nc, int M, CsLazy lz) {
  constexpr int NT = CS_WG_THREADS, NU = 256 * 16 / NT;  // f32x4 quads of dy per thread
  constexpr int DP = 64 + 4, XP = 32 + 4;  // pitches (floats): k and k + 4 16 banks apart
  __shared__ __attribute__((aligned(16))) float dsm[256 * DP];
  __shared__ __attribute__((aligned(16))) float xsm[256 * XP];
  __shared__ __attribute__((aligned(16))) float patch[cs_patch_floats<256>()];
  const int t = threadIdx.x, lane = t & 63, wv = t >> 6, li = lane & 15, g = lane >> 4;
  const int m0 = blockIdx.x * 256, n0 = blockIdx.y * 64, HW = H * W;
  f32x4 d[NU];
  if constexpr (!LAZY) {
#pragma unroll
    for (int u = 0; u < NU; ++u) {  // 256 rows x 16 quads
      const int e = t + NT * u, r = e >> 4, ch = e & 15;
      d[u] = *reinterpret_cast<const f32x4*>(dy + (long long)(m0 + r) * Nc + n0 + ch * 4);
    }
  } else {
    // thread t always holds channels c0 .. c0 + 3 (e & 15 == t & 15): their coefficients once
    const int c0 = n0 + (t & 15) * 4;
    const f32x4 mn = *reinterpret_cast<const f32x4*>(lz.stats + c0);
    const f32x4 sc = *reinterpret_cast<const f32x4*>(lz.stats + 2 * Nc + c0);
    const f32x4 sh = *reinterpret_cast<const f32x4*>(lz.stats + 3 * Nc + c0);
    const f32x4 ce = *reinterpret_cast<const f32x4*>(lz.coef + c0);
    const f32x4 cf = *reinterpret_cast<const f32x4*>(lz.coef + Nc + c0);
    const int Ho = H >> 1, Wo = W >> 1;
    f32x4 hv[NU], dn[NU];
    uint32_t kw[NU], qq[NU];
#pragma unroll
    for (int u = 0; u < NU; ++u) {  // every load of the thread in flight at once
      const int r = (t + NT * u) >> 4, m = m0 + r;
      hv[u] = *reinterpret_cast<const f32x4*>(lz.h + (long long)m * Nc + c0);
      if (lz.pool) {
        const int n = m / HW, p = m - n * HW, hh = p / W, ww = p - hh * W;
        const long long pr = ((long long)n * Ho + (hh >> 1)) * Wo + (ww >> 1);
        dn[u] = *reinterpret_cast<const f32x4*>(lz.dnext + pr * Nc + c0);
        kw[u] = *reinterpret_cast<const uint32_t*>(lz.code + pr * Nc + c0);
        qq[u] = (uint32_t)((hh & 1) * 2 + (ww & 1));
      } else {
        dn[u] = *reinterpret_cast<const f32x4*>(lz.dnext + (long long)m * Nc + c0);
        kw[u] = 0u;
        qq[u] = 0u;
      }
    }
#pragma unroll
    for (int u = 0; u < NU; ++u) {
      f32x4 o;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const float xv = hv[u][j];
        const bool route = !lz.pool || ((kw[u] >> (8 * j)) & 0xffu) == qq[u];
        const float z = xv * sc[j] + sh[j];  // k_bn_bwd_apply's expressions: the same bits
        const float dz = (route && !(z <= 0.0f)) ? dn[u][j] : 0.0f;
        o[j] = sc[j] * dz + ce[j] * (xv - mn[j]) + cf[j];
      }
      d[u] = o;
    }
  }
  const int lo = cs_patch<256, NT>(x, m0, W, M, patch, t);
#pragma unroll
  for (int u = 0; u < NU; ++u) {
    const int e = t + NT * u, r = e >> 4, ch = e & 15;
    *reinterpret_cast<f32x4*>(dsm + r * DP + ch * 4) = d[u];
  }
  __syncthreads();
  {
    // im2col row r = t & 255: k 16 (t >> 8) .. + 15 (k >= 27 zero)
    const int r = t & 255, kh = t >> 8;
    const int m = m0 + r, p = m % HW, h = p / W, ww = p - h * W;
#pragma unroll
    for (int k4 = 0; k4 < 4; ++k4) {
      f32x4 v;
#pragma unroll
      for (int e = 0; e < 4; ++e) v[e] = cs_x(patch, lo, m, h, ww, H, W, 16 * kh + 4 * k4 + e);
      *reinterpret_cast<f32x4*>(xsm + r * XP + 16 * kh + 4 * k4) = v;
    }
  }
  __syncthreads();
  const int nt = wv & 3, j = wv >> 2;
  f32x4 acc = {0.0f, 0.0f, 0.0f, 0.0f};
#pragma unroll 8
  for (int s = 0; s < 64; ++s) {
    // reduction row of MFMA step s for lane group g: the four groups read rows 4 apart (the +4
    // pitch pads put them 16 banks apart)
    const int mr = (s >> 2) * 16 + 4 * g + (s & 3);
    acc = __builtin_amdgcn_mfma_f32_16x16x4f32(dsm[mr * DP + 16 * nt + li],
                                               xsm[mr * XP + 16 * j + li], acc, 0, 0, 0);
  }
  float* sp = slab + (long long)blockIdx.x * Nc * CS_K;
  const int k = 16 * j + li;
  if (k < CS_K) {
#pragma unroll
    for (int q = 0; q < 4; ++q) sp[(long long)(n0 + 16 * nt + 4 * g + q) * CS_K + k] = acc[q];
  }
}

// dw[o] = sum over the nb block partials slab[b][o] in a fixed order
__global__ __launch_bounds__(EW_BLOCK) void k_cf_stem_reduce(const float* __restrict__ slab,
                                                             int nb, int n,
                                                             float* __restrict__ dw) {
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
  if (ck == 0 && o < n) dw[o] = red[0][t & 7];
}

// A split-K reduction left pending (ew_cf_defer_reduce) for the stem's reduction launch to run
// beside its own (k_cf_reduce2): its slabs stay in the workspace until then, and any GEMM launch
// that may write slabs, or a flush before a gradient is read, runs it on its own first.
struct CfPendRed {
  const float* slab;
  float* out;
  long long n;  // floats (multiple of 4)
  int split;
  hipStream_t s;
};
thread_local CfPendRed g_cf_pred{nullptr, nullptr, 0, 0, nullptr};
thread_local int g_cf_defer_red = 0;

// blocks [0, nb1): k_cf_stem_reduce's work; the rest k_cf_slab_reduce's (no addend), each
// element in its own kernel's order
__global__ __launch_bounds__(EW_BLOCK) void k_cf_reduce2(const float* __restrict__ sslab, int snb,
                                                         int sn, float* __restrict__ sdw, int nb1,
                                                         const float* __restrict__ slab,
                                                         int nsplit, long long n,
                                                         float* __restrict__ out) {
  if ((int)blockIdx.x < nb1) {
    __shared__ float red[32][8];
    const int t = threadIdx.x, o = blockIdx.x * 8 + (t & 7), ck = t >> 3;
    float sv = 0.0f;
    if (o < sn) {
      const int per = (snb + 31) / 32, b0 = ck * per, b1 = min(b0 + per, snb);
      int b = b0;
      for (; b + 3 < b1; b += 4) {
        const float v0 = sslab[(long long)b * sn + o], v1 = sslab[(long long)(b + 1) * sn + o];
        const float v2 = sslab[(long long)(b + 2) * sn + o], v3 = sslab[(long long)(b + 3) * sn + o];
        sv += (v0 + v1) + (v2 + v3);
      }
      for (; b < b1; ++b) sv += sslab[(long long)b * sn + o];
    }
    red[ck][t & 7] = sv;
    __syncthreads();
#pragma unroll
    for (int h = 16; h > 0; h >>= 1) {
      if (ck < h) red[ck][t & 7] += red[ck + h][t & 7];
      __syncthreads();
    }
    if (ck == 0 && o < sn) sdw[o] = red[0][t & 7];
    return;
  }
  const long long nv = n / 4;
  for (long long v = (blockIdx.x - nb1) * (long long)EW_BLOCK + threadIdx.x; v < nv;
       v += (long long)(gridDim.x - nb1) * EW_BLOCK) {
    const f32x4* p = reinterpret_cast<const f32x4*>(slab) + v;
    f32x4 a = p[0];
    for (int z = 1; z < nsplit; ++z) a += p[(long long)z * (n / 4)];  // fixed order
    reinterpret_cast<f32x4*>(out)[v] = a;
  }
}

long long cf_reduce_grid(long long n) {
  long long gr = (n / 4 + EW_BLOCK - 1) / EW_BLOCK;
  return gr > 2048 ? 2048 : gr;
}

void cf_flush_pred() {
  if (!g_cf_pred.slab) return;
  const CfPendRed j = g_cf_pred;
  g_cf_pred = CfPendRed{nullptr, nullptr, 0, 0, nullptr};
  hipLaunchKernelGGL(k_cf_slab_reduce, dim3((int)cf_reduce_grid(j.n)), dim3(EW_BLOCK), 0, j.s,
                     j.slab, j.split, j.n, j.out, nullptr);
  EW_CHECK_LAUNCH();
}

// Forward GEMMs through the LDS-DMA kernel (k_cf_gemm_gl): EWDML_CF_GLDS=1/0 at load, or
// ew_cf_set_glds at run time (tests compare both paths in one process)
int g_cf_glds = -1;
bool cf_glds_on() {
  if (g_cf_glds < 0) {
    const char* e = getenv("EWDML_CF_GLDS");
    g_cf_glds = (e && e[0] == '1') ? 1 : 0;
  }
  return g_cf_glds == 1;
}

// The BatchNorm backward finalisation armed for the next weight-gradient GEMM launch (host thread
// that enqueues a conv's backward; ew_cf_arm_bn_fin / ew_cf_flush_bn_fin)
thread_local EwBnFin g_cf_fin{};
// the deferred Winograd (m = 2) weight-gradient output transform armed for the next backward-data
// GEMM launch (ew_cf_arm_wgout / ew_cf_flush_wgout)
thread_local WgOut g_cf_wo{nullptr, nullptr, 1, 0, 0};

__global__ __launch_bounds__(EW_BLOCK) void k_cf_wgout(WgOut wo) {
  wg_wgrad_out<2>(wo.src, wo.nsplit, wo.dw, wo.Nc, wo.C,
                  (long long)blockIdx.x * EW_BLOCK + threadIdx.x);
}

__global__ __launch_bounds__(EW_BLOCK) void k_cf_bn_fin(EwBnFin f) {
  __shared__ double red[2 * EW_WAVES * EW_FIN_CH];
  ew_bn_bwd_fin_group<2>(f, blockIdx.x, red);
}

// Launch plan: tile shape and split of the reduction, from a small cost model (us): every block
// k-step costs its MFMA time (bm*bn*32*2 FLOP at 614 GFLOP/s per CU, derated for the narrower
// tiles' lower operand reuse), each block pays ~3 k-steps of prologue / epilogue, a CU runs
// ceil(blocks / 256) blocks' worth of work, and a split pays its slab round trip (write + read
// at ~4 TB/s) plus one reduction launch.
struct CfPlan {
  int bm, bn, split, kps;
};
// batch > 1: that many independent GEMMs share the grid (blockIdx.z); a split needs
// split * batch * M * Ncol slab floats
CfPlan cf_plan(int M, int Ncol, int ksteps, long long ws_floats, int batch) {
  const long long slab1 = (long long)batch * M * Ncol;  // slab floats per split
  // EWDML_CF_PLAN="bm,bn,split": forced plan (measurement only; invalid shapes fall through)
  static const char* force = getenv("EWDML_CF_PLAN");
  if (force) {
    int bm = 0, bn = 0, sp = 0;
    if (sscanf(force, "%d,%d,%d", &bm, &bn, &sp) == 3 && (bm == 64 || bm == 128) &&
        (bn == 64 || bn == 128) && sp >= 1 && M % bm == 0 && Ncol % bn == 0 &&
        (sp == 1 || sp * slab1 <= ws_floats)) {
      const int kps = (ksteps + sp - 1) / sp;
      return CfPlan{bm, bn, (ksteps + kps - 1) / kps, kps};
    }
  }
  // the reduction launch's fixed cost (us); EWDML_CF_RED_US overrides (A/B)
  static const double red_us = [] {
    const char* e = getenv("EWDML_CF_RED_US");
    return e ? atof(e) : 2.0;
  }();
  static const int shapes[4][2] = {{128, 128}, {128, 64}, {64, 128}, {64, 64}};
  static const double derate[4] = {1.0, 0.9, 0.9, 0.75};
  CfPlan best{64, 64, 1, ksteps};
  double best_t = 1e30;
  for (int sh = 0; sh < 4; ++sh) {
    const int bm = shapes[sh][0], bn = shapes[sh][1];
    if (M % bm || Ncol % bn) continue;
    const long long tiles = (long long)(M / bm) * (Ncol / bn) * batch;
    const double step_us = (double)bm * bn * CF_BK * 2 / 614e3 / derate[sh];
    for (int split = 1; split <= 64; ++split) {
      const int kps = (ksteps + split - 1) / split;
      if (split > 1 && (kps < 4 || split * slab1 > ws_floats)) break;
      const int sp = (ksteps + kps - 1) / kps;
      const long long blocks = tiles * sp;
      double t = (double)((blocks + 255) / 256) * step_us * (kps + 3);
      // operand traffic: every block streams (bm + bn) x K floats, ~6 TB/s from HBM / MALL
      // (small tiles over a long K -- the Winograd weight-gradient GEMMs -- are bound by it)
      t = std::max(t, (double)tiles * (bm + bn) * ksteps * CF_BK * 4 / 6e6);
      if (sp > 1) t += 8.0 * sp * slab1 / 4e6 + red_us;
      if (t < best_t * 0.999) {
        best_t = t;
        best = CfPlan{bm, bn, sp, kps};
      }
    }
  }
  return best;
}

// tickets of the in-launch split-K reduction (k_cf_gemm's epilogue) per workspace; conv.hip keeps
// its slabs clear of them
constexpr int CF_RED_TICKETS = 4096;
// EWDML_CF_INRED=1: the in-launch reduction instead of the k_cf_slab_reduce launch (opt-in,
// ew_cf_set_inred at run time).  Measured slower: VGG-11 1.153 -> 1.195 ms, ResNet-50 CIFAR 13.16
// -> 14.13 ms -- the write-through slabs and the reducing blocks' sc1 loads cost more than the
// launch they save (profiles/ab/README.md)
int g_cf_inred = -1;
bool cf_inred_on() {
  if (g_cf_inred < 0) {
    const char* e = getenv("EWDML_CF_INRED");
    g_cf_inred = (e && e[0] == '1') ? 1 : 0;
  }
  return g_cf_inred == 1;
}
// whether the split reduction would write BN partial rows (k_cf_slab_reduce_bn's condition)
bool Nc_bn_ok(const CfGeom& geo, long long bnpart_floats) {
  const int M = geo.M, Nc = geo.Ncol;
  const int tpr = Nc / 4, rpi = tpr <= EW_BLOCK ? EW_BLOCK / tpr : 0;
  if (rpi <= 0 || EW_BLOCK % tpr) return false;
  int rpb = rpi;
  while ((M + rpb - 1) / rpb > 1024) rpb += rpi;
  return 2LL * ((M + rpb - 1) / rpb) * Nc <= bnpart_floats;
}

#define CF_LAUNCH_W(MODE_, BM_, BN_, WM_, WN_, SH_, WPE_)                                   \
  hipLaunchKernelGGL((k_cf_gemm<MODE_, BM_, BN_, WM_, WN_, SH_, STR, WPE_, LZ>), grid,            \
                     dim3(64 * WM_ * WN_), 0, s, a, b, out, slab, geo, bnp, bbv, addend, fin, wo, \
                     red, lz)
#define CF_LAUNCH(MODE_, BM_, BN_, WM_, WN_, SH_) CF_LAUNCH_W(MODE_, BM_, BN_, WM_, WN_, SH_, 0)
#define CF_LAUNCH_GL(BM_, BN_, WM_, WN_, SH_, WPE_)                                           \
  hipLaunchKernelGGL((k_cf_gemm_gl<BM_, BN_, WM_, WN_, SH_, WPE_>), grid, dim3(64 * WM_ * WN_), 0, \
                     s, a, b, out, slab, geo, bnp, bbv, addend)

// the register-staged GEMM variant of a plan (LZ: with the lazy BatchNorm operand)
template <int MODE, int STR, bool LZ>
void cf_launch_staged(const CfPlan& p, bool w4, bool occ2, dim3 grid, hipStream_t s,
                      const float* a, const float* b, float* out, float* slab, const CfGeom& geo,
                      float* bnp, const CfBnBwd& bbv, const float* addend, const EwBnFin& fin,
                      const WgOut& wo, int* red, const CfLz& lz) {
  if (p.bm == 128 && p.bn == 128) {
    if (w4) CF_LAUNCH(MODE, 128, 128, 2, 2, 32);
    else CF_LAUNCH(MODE, 128, 128, 2, 4, 32);
  } else if (p.bm == 128) {
    if (occ2) CF_LAUNCH_W(MODE, 128, 64, 4, 2, 32, 4);
    else CF_LAUNCH(MODE, 128, 64, 4, 2, 32);
  } else if (p.bn == 128) {
    if (occ2) CF_LAUNCH_W(MODE, 64, 128, 2, 4, 32, 4);
    else CF_LAUNCH(MODE, 64, 128, 2, 4, 32);
  } else {
    CF_LAUNCH(MODE, 64, 64, 4, 2, 16);
  }
}

// lz (forward / weight gradient, stride 1): the lazily applied BatchNorm operand (CfLz)
template <int MODE, int STR = 1>
int cf_gemm(const float* a, const float* b, float* out, float* ws, long long ws_floats,
            CfGeom geo, hipStream_t s, float* bnpart, long long bnpart_floats,
            const CfBnBwd* bnb, const float* addend, int* split_out = nullptr,
            CfLz lz = CfLz{nullptr, nullptr}) {
  cf_flush_pred();  // this launch may write slabs over a pending reduction's
  const int defer_red = g_cf_defer_red;  // armed for this launch only
  g_cf_defer_red = 0;
  ws_floats -= 64;  // the workspace's last 64 floats are conv.hip's zero page (never a slab)
  // the shared per-stream workspace (not a caller's own slabs): the in-launch split-K tickets sit
  // before the zero page (zeroed with it, left zeroed)
  int* tick = nullptr;
  if (!split_out) {
    ws_floats -= CF_RED_TICKETS;
    tick = reinterpret_cast<int*>(ws + ws_floats);
  }
  const int batch = geo.nsplit;  // callers pass the batch count here (1: no batching)
  {
    // the buffer-load operands (per batch) must fit 32-bit byte offsets (CfStager)
    const long long K = (long long)geo.taps * geo.C;
    long long a_bytes, b_bytes = 0;
    if (MODE == CF_FWD) {
      const long long rows = STR == 2 ? (long long)(geo.M / (geo.Ho * geo.Wo)) * geo.H * geo.W
                                      : (long long)geo.M;
      a_bytes = rows * geo.C * 4;
      b_bytes = (long long)geo.Ncol * K * 4;
    } else if (MODE == CF_BWD) {
      a_bytes = (long long)geo.M * geo.Nc * 4;
      b_bytes = (long long)geo.Nc * K * 4;
    } else {
      a_bytes = (long long)geo.ksteps * CF_BK * geo.Nc * 4;
      if (STR == 1) b_bytes = (long long)geo.ksteps * CF_BK * geo.C * 4;
    }
    if (std::max(a_bytes, b_bytes) >= (long long)CF_OOB)
      throw std::runtime_error("ewdml conv f32: an operand of 4 GB or more");
  }
  const CfPlan p = cf_plan(geo.M, geo.Ncol, geo.ksteps, ws_floats, batch);
  geo.kps = p.kps;
  geo.nsplit = p.split;
  dim3 grid(geo.M / p.bm, geo.Ncol / p.bn, p.split * batch);
  // an armed BatchNorm backward finalisation (ew_cf_arm_bn_fin) rides in a weight-gradient GEMM
  EwBnFin fin{};
  if (MODE == CF_WGRAD && g_cf_fin.ngrp) {
    fin = g_cf_fin;
    g_cf_fin = EwBnFin{};
    grid.z += (fin.ngrp + grid.x * grid.y - 1) / (grid.x * grid.y);
  }
  static const int w4 = [] {  // EWDML_CF_WAVES=4: 4-wave 128x128 blocks (64x64 wave tiles)
    const char* e = getenv("EWDML_CF_WAVES");
    return e && e[0] == '4';
  }();
  // an armed deferred Winograd weight-gradient output transform rides in a backward-data GEMM
  WgOut wo{nullptr, nullptr, 1, 0, 0};
  if (MODE == CF_BWD && STR == 1 && p.bm == 128 && g_cf_wo.src) {
    wo = g_cf_wo;
    g_cf_wo = WgOut{nullptr, nullptr, 1, 0, 0};
    // the launched variant's threads (k_cf_gemm's NT): 8 waves but the 4-wave 128x128 option
    const int NTL = (p.bm == 128 && p.bn == 128 && w4) ? 256 : 512;
    const int nwb = (wo.Nc * (wo.C / WG2_VW) + NTL - 1) / NTL;
    grid.z += (nwb + grid.x * grid.y - 1) / (grid.x * grid.y);
  }
  float* slab = p.split > 1 ? ws : nullptr;
  const long long prow = geo.M / p.bm;
  // split-K reduced in-launch by each tile's last split (no k_cf_slab_reduce launch) when no BN
  // sums are due from the reduction (their partial rows come from k_cf_slab_reduce_bn)
  int* red = nullptr;
  if (slab && tick && batch == 1 && cf_inred_on() &&
      (long long)grid.x * grid.y <= CF_RED_TICKETS && !(bnpart && Nc_bn_ok(geo, bnpart_floats)) &&
      !(MODE == CF_FWD && STR == 1 && cf_glds_on() && !w4))  // (the LDS-DMA kernel: no tickets)
    red = tick;
  float* bnp = (bnpart && !slab && prow <= 1024 && 2 * prow * geo.Ncol <= bnpart_floats) ? bnpart
                                                                                      : nullptr;
  const CfBnBwd none{nullptr, nullptr, nullptr, nullptr, 0, 0, 0};
  const CfBnBwd bbv = (bnp && bnb) ? *bnb : none;
  // wave grids: 128x128 -> 2x4 waves of 64x32; 128x64 -> 4x2 of 32x32; 64x128 -> 2x4 of 32x32;
  // 64x64 -> 4x2 of 16x32
  // The 8-wave 128x64 / 64x128 kernels held to 128 VGPRs (4 waves per SIMD: two blocks per CU)
  // instead of the compiler's 130 (one block per CU), for grids of more than one block per CU:
  // ResNet-50 CIFAR +1.1 %, VGG-11 (one block per CU at these tiles) unchanged either way
  // (profiles/ab/README.md).  EWDML_CF_OCC=0: never, =2: always.
  static const int occ_env = [] {
    const char* e = getenv("EWDML_CF_OCC");
    return e ? e[0] - '0' : 1;
  }();
  // (rider slices count: with them a one-block-per-CU grid of 256 GEMM blocks leaves the riders
  // waiting for a CU -- VGG-11 conv2's backward data + transform 60 us held to one block per CU,
  // 54 us at two, profiles/ab/README.md)
  const bool occ2 = occ_env == 2 || (occ_env == 1 && (long long)grid.x * grid.y * grid.z > 256);
  bool launched = false;
  if constexpr ((MODE == CF_FWD || MODE == CF_WGRAD) && STR == 1) {
    if (lz.stats) {
      cf_launch_staged<MODE, STR, true>(p, w4, occ2, grid, s, a, b, out, slab, geo, bnp, bbv,
                                        addend, fin, wo, red, lz);
      launched = true;
    }
  }
  if constexpr (MODE == CF_FWD && STR == 1) {
    if (!launched && cf_glds_on() && !w4) {
      if (p.bm == 128 && p.bn == 128)
        CF_LAUNCH_GL(128, 128, 2, 4, 32, 0);
      else if (p.bm == 128)  // held to 128 VGPRs: two blocks per CU (72 KB of LDS each)
        CF_LAUNCH_GL(128, 64, 4, 2, 32, 4);
      else if (p.bn == 128)
        CF_LAUNCH_GL(64, 128, 2, 4, 32, 4);
      else
        CF_LAUNCH_GL(64, 64, 4, 2, 16, 0);
      launched = true;
    }
  }
  if (!launched)
    cf_launch_staged<MODE, STR, false>(p, w4, occ2, grid, s, a, b, out, slab, geo, bnp, bbv,
                                       addend, fin, wo, red, lz);
  EW_CHECK_LAUNCH();
  if (split_out) {  // the caller reduces the slabs (ws[split][batch][M][Ncol]) itself
    *split_out = p.split;
    return 0;
  }
  if (p.split > 1 && batch > 1)
    throw std::runtime_error("ewdml conv f32: a batched split GEMM needs the caller's reduction");
  if (p.split > 1 && red) return 0;  // reduced in the launch (no BN partial rows)
  if (p.split > 1) {
    const int M = geo.M, Nc = geo.Ncol;
    const long long n = (long long)M * Nc;
    const int tpr = Nc / 4, rpi = tpr <= EW_BLOCK ? EW_BLOCK / tpr : 0;
    int rpb = rpi, nblk = 0;
    if (bnpart && rpi > 0 && EW_BLOCK % tpr == 0) {
      while ((M + rpb - 1) / rpb > 1024) rpb += rpi;
      nblk = (M + rpb - 1) / rpb;
      if (2LL * nblk * Nc > bnpart_floats) nblk = 0;
    }
    if (nblk > 0) {
      const CfBnBwd bbr = bnb ? *bnb : none;
      hipLaunchKernelGGL(k_cf_slab_reduce_bn, dim3(nblk), dim3(EW_BLOCK), 0, s, ws, p.split, M,
                         Nc, out, bnpart, rpb, bbr, addend);
      EW_CHECK_LAUNCH();
      return nblk;
    }
    if (defer_red && !addend && n % 4 == 0) {  // left to the stem's reduction launch
      g_cf_pred = CfPendRed{ws, out, n, p.split, s};
      return 0;
    }
    hipLaunchKernelGGL(k_cf_slab_reduce, dim3((int)cf_reduce_grid(n)), dim3(EW_BLOCK), 0, s, ws,
                       p.split, n, out, addend);
    EW_CHECK_LAUNCH();
  }
  return bnp ? (int)prow : 0;
}
#undef CF_LAUNCH
#undef CF_LAUNCH_W
#undef CF_LAUNCH_GL

int cf_taps(int ksize) {
  if (ksize != 1 && ksize != 3) throw std::runtime_error("ewdml conv: kernel size must be 1 or 3");
  return ksize * ksize;
}

}  // namespace

// ------------------------------------------------------------------------------------------------
// host side (shapes validated here: the kernels assume them)

// Arm a BatchNorm backward finalisation (the partials of a backward-data epilogue, NS = 2; see
// bn_fin.h) for the next weight-gradient GEMM launched from this thread; ew_cf_flush_bn_fin
// launches it on its own if none took it (returns 1 then).
void ew_cf_arm_bn_fin(uintptr_t part, int nblk, int C, long long M, uintptr_t stats, uintptr_t coef,
                      uintptr_t dgamma, uintptr_t dbeta, uintptr_t dcbias, int cb_bf16) {
  if (!part || !stats || !coef || nblk <= 0 || C <= 0 || M <= 0)
    throw std::runtime_error("ewdml conv f32: bad BatchNorm finalisation job");
  if (g_cf_fin.ngrp) throw std::runtime_error("ewdml conv f32: a finalisation is already armed");
  g_cf_fin = EwBnFin{reinterpret_cast<const float*>(part), reinterpret_cast<const float*>(stats),
                     reinterpret_cast<float*>(coef), reinterpret_cast<float*>(dgamma),
                     reinterpret_cast<float*>(dbeta), reinterpret_cast<void*>(dcbias), M, nblk, C,
                     cb_bf16, (C + EW_FIN_CH - 1) / EW_FIN_CH};
}

void ew_cf_arm_wgout(uintptr_t src, int split, uintptr_t dw, int Nc, int C) {
  if (!src || !dw || split < 1 || Nc <= 0 || C % WG2_VW)
    throw std::runtime_error("ewdml conv f32: bad weight-gradient output transform job");
  if (g_cf_wo.src) throw std::runtime_error("ewdml conv f32: a transform is already armed");
  g_cf_wo = WgOut{reinterpret_cast<const float*>(src), reinterpret_cast<float*>(dw), split, Nc, C};
}

int ew_cf_flush_wgout(uintptr_t stream) {
  if (!g_cf_wo.src) return 0;
  const WgOut wo = g_cf_wo;
  g_cf_wo = WgOut{nullptr, nullptr, 1, 0, 0};
  const long long n = (long long)wo.Nc * (wo.C / WG2_VW);
  hipLaunchKernelGGL(k_cf_wgout, dim3((unsigned)((n + EW_BLOCK - 1) / EW_BLOCK)), dim3(EW_BLOCK),
                     0, (hipStream_t)stream, wo);
  EW_CHECK_LAUNCH();
  return 1;
}

int ew_cf_flush_bn_fin(uintptr_t stream) {
  if (!g_cf_fin.ngrp) return 0;
  const EwBnFin f = g_cf_fin;
  g_cf_fin = EwBnFin{};
  hipLaunchKernelGGL(k_cf_bn_fin, dim3(f.ngrp), dim3(EW_BLOCK), 0, (hipStream_t)stream, f);
  EW_CHECK_LAUNCH();
  return 1;
}

// Leave the next plain split-K reduction of an fp32 GEMM pending for the stem's reduction launch
// (ops/conv.py: the conv whose input comes from the stem's BN layer); ew_cf_flush_reduce runs a
// pending one (before any gradient is read).
void ew_cf_defer_reduce() { g_cf_defer_red = 1; }
void ew_cf_flush_reduce() {
  g_cf_defer_red = 0;
  cf_flush_pred();
}

int ew_cf_set_inred(int on) {
  const int prev = cf_inred_on() ? 1 : 0;
  if (on >= 0) g_cf_inred = on ? 1 : 0;
  return prev;
}

int ew_cf_set_glds(int on) {
  const int prev = cf_glds_on() ? 1 : 0;
  if (on >= 0) g_cf_glds = on ? 1 : 0;
  return prev;
}

// out[b][M][N] = A[b][M][K] * B[b][N][K]^T for b < batch (row-major, K contiguous): the forward
// GEMM as a 1x1 "convolution" over M pixels, batched over blockIdx.z (winograd_f32.hip).
// dU[z][M][N] = sum_k A[z][k][M] B[z][k][N] (both row-major over k; the weight-gradient GEMM),
// K-split into ws slabs [split][batch][M][N] that the caller reduces; returns the split count
// (1: written to out directly).
int ew_cf_gemm_tn_batched(const float* a, const float* b, float* out, float* ws,
                          long long ws_floats, int M, int N, int K, int batch, long long a_bs,
                          long long b_bs, hipStream_t s) {
  if (M % 64 || N % 64 || K % CF_BK || (long long)K * std::max(M, N) >= (1LL << 31))
    throw std::runtime_error("ewdml gemm f32: needs M, N % 64 == 0, K % 32 == 0");
  CfGeom g{M, N, K, 1, 1, N, M, 1, K / CF_BK, 0, batch, a_bs, b_bs, (long long)M * N, 0};
  int split = 1;
  cf_gemm<CF_WGRAD>(a, b, out, ws, ws_floats, g, s, nullptr, 0, nullptr, nullptr, &split);
  return split;
}

// out[z][M][N] = A[z][M][K] * op(B[z'])  for z < batch (row-major, K contiguous in A): the conv
// GEMMs as 1x1 "convolutions" over M pixels, batched over blockIdx.z (winograd_f32.hip).
// nt: B[z] is [N][K] (the forward's weight image); else B[z'] is [K][N] (backward data) with
// z' = cf_flip4(z) when flip.
void ew_cf_gemm_batched(const float* a, const float* b, float* out, int M, int N, int K, int batch,
                        long long a_bs, long long b_bs, long long o_bs, bool nt, bool flip,
                        hipStream_t s) {
  if (M % 64 || N % 64 || K % CF_BK || (long long)M * std::max(N, K) >= (1LL << 31) ||
      (flip && batch != 16))
    throw std::runtime_error("ewdml gemm f32: needs M, N % 64 == 0, K % 32 == 0");
  if (nt) {
    CfGeom g{M, N, M, 1, 1, K, N, 1, K / CF_BK, 0, batch, a_bs, b_bs, o_bs, 0};
    cf_gemm<CF_FWD>(a, b, out, nullptr, 64, g, s, nullptr, 0, nullptr, nullptr);
  } else {
    CfGeom g{M, N, M, 1, 1, N, K, 1, K / CF_BK, 0, batch, a_bs, b_bs, o_bs, flip ? 1 : 0};
    cf_gemm<CF_BWD>(a, b, out, nullptr, 64, g, s, nullptr, 0, nullptr, nullptr);
  }
}

int ew_conv_f32_fwd(uintptr_t x, uintptr_t w, uintptr_t y, uintptr_t ws, long long ws_floats,
                    long long N, int H, int W, int C, int Nc, int ksize, uintptr_t bnpart,
                    long long bnpart_floats, uintptr_t stream) {
  const long long P = N * H * W;
  if (C % CF_BK || Nc % 64 || P % 64 || P * (long long)std::max(C, Nc) >= (1LL << 31))
    throw std::runtime_error("ewdml conv f32: needs C % 32 == 0, Nc % 64 == 0, N*H*W % 64 == 0");
  const int taps = cf_taps(ksize);
  CfGeom g{(int)P, Nc, (int)P, H, W, C, Nc, taps, taps * C / CF_BK, 0, 1, 0, 0, 0};
  return cf_gemm<CF_FWD>(reinterpret_cast<const float*>(x), reinterpret_cast<const float*>(w),
                         reinterpret_cast<float*>(y), reinterpret_cast<float*>(ws), ws_floats, g,
                         (hipStream_t)stream, reinterpret_cast<float*>(bnpart), bnpart_floats,
                         nullptr, nullptr);
}

int ew_conv_f32_bwd_data(uintptr_t dy, uintptr_t w, uintptr_t dx, uintptr_t ws,
                         long long ws_floats, long long N, int H, int W, int C, int Nc, int ksize,
                         uintptr_t bn_h, uintptr_t bn_res, uintptr_t bn_code, uintptr_t bn_stats,
                         int bn_relu, uintptr_t bnpart, long long bnpart_floats, uintptr_t addend,
                         uintptr_t stream) {
  const long long P = N * H * W;
  if (C % 64 || Nc % CF_BK || P % 64 || P * (long long)std::max(C, Nc) >= (1LL << 31))
    throw std::runtime_error("ewdml conv f32: bwd-data needs C % 64 == 0, Nc % 32 == 0");
  const int taps = cf_taps(ksize);
  CfGeom g{(int)P, C, (int)P, H, W, C, Nc, taps, taps * Nc / CF_BK, 0, 1, 0, 0, 0};
  const CfBnBwd bb{reinterpret_cast<const float*>(bn_h), reinterpret_cast<const float*>(bn_res),
                   reinterpret_cast<const uint8_t*>(bn_code),
                   reinterpret_cast<const float*>(bn_stats), bn_relu, H, W};
  return cf_gemm<CF_BWD>(reinterpret_cast<const float*>(dy), reinterpret_cast<const float*>(w),
                         reinterpret_cast<float*>(dx), reinterpret_cast<float*>(ws), ws_floats, g,
                         (hipStream_t)stream, bn_h ? reinterpret_cast<float*>(bnpart) : nullptr,
                         bnpart_floats, bn_h ? &bb : nullptr,
                         reinterpret_cast<const float*>(addend));
}

void ew_conv_f32_wgrad(uintptr_t dy, uintptr_t x, uintptr_t dw, uintptr_t ws, long long ws_floats,
                       long long N, int H, int W, int C, int Nc, int ksize, uintptr_t stream) {
  const long long P = N * H * W;
  const int taps = cf_taps(ksize);
  if (C % 64 || Nc % 64 || P % CF_BK || P * (long long)std::max(C, Nc) >= (1LL << 31))
    throw std::runtime_error("ewdml conv f32: wgrad needs C, Nc % 64 == 0, N*H*W % 32 == 0");
  CfGeom g{Nc, taps * C, (int)P, H, W, C, Nc, taps, (int)(P / CF_BK), 0, 1, 0, 0, 0};
  cf_gemm<CF_WGRAD>(reinterpret_cast<const float*>(dy), reinterpret_cast<const float*>(x),
                    reinterpret_cast<float*>(dw), reinterpret_cast<float*>(ws), ws_floats, g,
                    (hipStream_t)stream, nullptr, 0, nullptr, nullptr);
}

// 1x1 convolutions of a lazily applied BatchNorm + ReLU input (CfLz): x = relu(h * scale + shift)
// is formed in the GEMM's operand staging from h [N][H][W][C] and the BN layer's stats [4][C];
// the forward counts the layer's batch in nbt (0: none)
int ew_conv_f32_fwd_lz(uintptr_t h, uintptr_t stats, uintptr_t nbt, uintptr_t w, uintptr_t y,
                       uintptr_t ws, long long ws_floats, long long N, int H, int W, int C, int Nc,
                       uintptr_t bnpart, long long bnpart_floats, uintptr_t stream) {
  const long long P = N * H * W;
  if (!h || !stats || (stats & 15) || C % 64 || Nc % 64 || P % 64 ||
      P * (long long)std::max(C, Nc) >= (1LL << 31))
    throw std::runtime_error("ewdml conv f32 lazy-BN 1x1: needs C, Nc, N*H*W % 64 == 0");
  CfGeom g{(int)P, Nc, (int)P, H, W, C, Nc, 1, C / CF_BK, 0, 1, 0, 0, 0};
  return cf_gemm<CF_FWD>(reinterpret_cast<const float*>(h), reinterpret_cast<const float*>(w),
                         reinterpret_cast<float*>(y), reinterpret_cast<float*>(ws), ws_floats, g,
                         (hipStream_t)stream, reinterpret_cast<float*>(bnpart), bnpart_floats,
                         nullptr, nullptr, nullptr,
                         CfLz{reinterpret_cast<const float*>(stats), reinterpret_cast<long long*>(nbt)});
}

void ew_conv_f32_wgrad_lz(uintptr_t dy, uintptr_t h, uintptr_t stats, uintptr_t dw, uintptr_t ws,
                          long long ws_floats, long long N, int H, int W, int C, int Nc,
                          uintptr_t stream) {
  const long long P = N * H * W;
  if (!h || !stats || (stats & 15) || C % 64 || Nc % 64 || P % CF_BK ||
      P * (long long)std::max(C, Nc) >= (1LL << 31))
    throw std::runtime_error("ewdml conv f32 lazy-BN 1x1 wgrad: needs C, Nc % 64 == 0");
  CfGeom g{Nc, C, (int)P, H, W, C, Nc, 1, (int)(P / CF_BK), 0, 1, 0, 0, 0};
  cf_gemm<CF_WGRAD>(reinterpret_cast<const float*>(dy), reinterpret_cast<const float*>(h),
                    reinterpret_cast<float*>(dw), reinterpret_cast<float*>(ws), ws_floats, g,
                    (hipStream_t)stream, nullptr, 0, nullptr, nullptr, nullptr,
                    CfLz{reinterpret_cast<const float*>(stats), nullptr});
}

// ---- stride-2 3x3 / pad 1 and 1x1 / pad 0 convolutions (the ResNet down-sampling convs):
// x [N][H][W][C] -> y [N][H/2][W/2][Nc], H and W even
static void cf_s2_check(long long N, int H, int W, int C, int Nc, const char* what) {
  const long long Po = N * (H / 2) * (W / 2);
  if (H % 2 || W % 2 || C % 64 || Nc % 64 || Po % 64 ||
      N * H * W * (long long)std::max(C, Nc) >= (1LL << 31))
    throw std::runtime_error(std::string("ewdml conv f32 stride 2: ") + what +
                             " needs even H, W, C % 64 == 0, Nc % 64 == 0, N*H*W/4 % 64 == 0");
}

int ew_conv_f32_fwd_s2(uintptr_t x, uintptr_t w, uintptr_t y, uintptr_t ws, long long ws_floats,
                       long long N, int H, int W, int C, int Nc, int ksize, uintptr_t bnpart,
                       long long bnpart_floats, uintptr_t stream) {
  cf_s2_check(N, H, W, C, Nc, "forward");
  const int taps = cf_taps(ksize), Ho = H / 2, Wo = W / 2;
  const long long M = N * Ho * Wo;
  CfGeom g{(int)M, Nc, (int)M, H, W, C, Nc, taps, taps * C / CF_BK, 0, 1, 0, 0, 0, 0, 2, Ho, Wo};
  return cf_gemm<CF_FWD, 2>(reinterpret_cast<const float*>(x), reinterpret_cast<const float*>(w),
                            reinterpret_cast<float*>(y), reinterpret_cast<float*>(ws), ws_floats,
                            g, (hipStream_t)stream, reinterpret_cast<float*>(bnpart),
                            bnpart_floats, nullptr, nullptr);
}

// dx [N][H][W][C] (every pixel written: the four phases, 1x1's empty ones as zeros (+ addend))
void ew_conv_f32_bwd_data_s2(uintptr_t dy, uintptr_t w, uintptr_t dx, long long N, int H, int W,
                             int C, int Nc, int ksize, uintptr_t addend, uintptr_t stream) {
  cf_s2_check(N, H, W, C, Nc, "backward data");
  const int taps = cf_taps(ksize), Ho = H / 2, Wo = W / 2;
  const long long M = N * Ho * Wo;
  const int kmax = cf_s2_ntaps(taps, 1, 1) > 1 ? 4 : 1;
  // batch 4 = the phases; no split-K (ws_floats 64: nothing beyond the zero page)
  CfGeom g{(int)M, C, (int)M, Ho, Wo, C, Nc, taps, kmax * Nc / CF_BK, 0, 4, 0, 0, 0, 0, 2, Ho, Wo};
  cf_gemm<CF_BWD, 2>(reinterpret_cast<const float*>(dy), reinterpret_cast<const float*>(w),
                     reinterpret_cast<float*>(dx), nullptr, 64, g, (hipStream_t)stream, nullptr, 0,
                     nullptr, reinterpret_cast<const float*>(addend));
}

void ew_conv_f32_wgrad_s2(uintptr_t dy, uintptr_t x, uintptr_t dw, uintptr_t ws,
                          long long ws_floats, long long N, int H, int W, int C, int Nc, int ksize,
                          uintptr_t stream) {
  cf_s2_check(N, H, W, C, Nc, "weight gradient");
  const int taps = cf_taps(ksize), Ho = H / 2, Wo = W / 2;
  const long long P = N * Ho * Wo;
  CfGeom g{Nc, taps * C, (int)P, H, W, C, Nc, taps, (int)(P / CF_BK), 0, 1, 0, 0, 0, 0, 2, Ho, Wo};
  cf_gemm<CF_WGRAD, 2>(reinterpret_cast<const float*>(dy), reinterpret_cast<const float*>(x),
                       reinterpret_cast<float*>(dw), reinterpret_cast<float*>(ws), ws_floats, g,
                       (hipStream_t)stream, nullptr, 0, nullptr, nullptr);
}

int ew_conv_f32_stem_fwd(uintptr_t x, uintptr_t w, uintptr_t y, long long N, int H, int W, int Nc,
                         uintptr_t bnpart, long long bnpart_floats, uintptr_t stream) {
  const long long M = N * H * W;
  if (M % 128 || Nc % 64 || M >= (1LL << 31) / 64 || W > CS_WMAX)
    throw std::runtime_error("ewdml conv f32 stem: needs N*H*W % 128 == 0, Nc % 64 == 0, W <= 256");
  const int nrows = (int)(M / 128);
  float* bnp = (bnpart && nrows <= 1024 && 2LL * nrows * Nc <= bnpart_floats)
                   ? reinterpret_cast<float*>(bnpart) : nullptr;
  hipLaunchKernelGGL(k_cf_stem_fwd, dim3(nrows, Nc / 64), dim3(EW_BLOCK), 0, (hipStream_t)stream,
                     reinterpret_cast<const float*>(x), reinterpret_cast<const float*>(w),
                     reinterpret_cast<float*>(y), H, W, Nc, (int)M, bnp, nrows);
  EW_CHECK_LAUNCH();
  return bnp ? nrows : 0;
}

static void cf_stem_wgrad(const float* dy, const CsLazy* lz, uintptr_t x, uintptr_t dw,
                          uintptr_t ws, long long ws_floats, long long N, int H, int W, int Nc,
                          uintptr_t stream) {
  const long long M = N * H * W;
  const long long nb = M / 256, n = (long long)Nc * CS_K;
  if (M % 256 || Nc % 64 || nb * n > ws_floats - 64 || W > CS_WMAX || M >= (1LL << 31) / 64)
    throw std::runtime_error("ewdml conv f32 stem: wgrad needs N*H*W % 256 == 0, Nc % 64 == 0, "
                             "W <= 256");
  if (lz && lz->pool && (H % 2 || W % 2 || !lz->code))
    throw std::runtime_error("ewdml conv f32 stem: a pooled BN backward needs even maps, codes");
  hipStream_t s = (hipStream_t)stream;
  float* slab = reinterpret_cast<float*>(ws);
  // a pending split-K reduction (its slabs at the workspace's start) runs in this reduction
  // launch: the stem's partials go behind them when they fit, else it runs now on its own
  CfPendRed pend = g_cf_pred;
  if (pend.slab) {
    const long long used = (long long)pend.split * pend.n;
    if (pend.slab == slab && pend.s == s && used + nb * n <= ws_floats - 64 - CF_RED_TICKETS) {
      slab += (used + 63) / 64 * 64;
      g_cf_pred = CfPendRed{nullptr, nullptr, 0, 0, nullptr};
    } else {
      cf_flush_pred();
      pend.slab = nullptr;
    }
  }
  const CsLazy none{nullptr, nullptr, nullptr, nullptr, nullptr, 0};
  if (lz)
    hipLaunchKernelGGL(k_cf_stem_wgrad<true>, dim3((int)nb, Nc / 64), dim3(CS_WG_THREADS), 0, s,
                       nullptr, reinterpret_cast<const float*>(x), slab, H, W, Nc, (int)M, *lz);
  else
    hipLaunchKernelGGL(k_cf_stem_wgrad<false>, dim3((int)nb, Nc / 64), dim3(CS_WG_THREADS), 0, s,
                       dy, reinterpret_cast<const float*>(x), slab, H, W, Nc, (int)M, none);
  EW_CHECK_LAUNCH();
  if (pend.slab) {
    const int nb1 = (int)((n + 7) / 8);
    hipLaunchKernelGGL(k_cf_reduce2, dim3(nb1 + (int)cf_reduce_grid(pend.n)), dim3(EW_BLOCK), 0,
                       s, slab, (int)nb, (int)n, reinterpret_cast<float*>(dw), nb1, pend.slab,
                       pend.split, pend.n, pend.out);
  } else {
    hipLaunchKernelGGL(k_cf_stem_reduce, dim3((int)((n + 7) / 8)), dim3(EW_BLOCK), 0, s, slab,
                       (int)nb, (int)n, reinterpret_cast<float*>(dw));
  }
  EW_CHECK_LAUNCH();
}

void ew_conv_f32_stem_wgrad(uintptr_t dy, uintptr_t x, uintptr_t dw, uintptr_t ws,
                            long long ws_floats, long long N, int H, int W, int Nc,
                            uintptr_t stream) {
  cf_stem_wgrad(reinterpret_cast<const float*>(dy), nullptr, x, dw, ws, ws_floats, N, H, W, Nc,
                stream);
}

// The weight gradient with dy formed from the BatchNorm(+ReLU)(+pool) backward of the stem's
// output (see k_cf_stem_wgrad LAZY): h = the stem output, dnext = the gradient of the BN layer's
// (pooled) output, code its pool codes, stats / coef that layer's [4][Nc] / [2][Nc].
void ew_conv_f32_stem_wgrad_bn(uintptr_t h, uintptr_t dnext, uintptr_t code, uintptr_t stats,
                               uintptr_t coef, int pool, uintptr_t x, uintptr_t dw, uintptr_t ws,
                               long long ws_floats, long long N, int H, int W, int Nc,
                               uintptr_t stream) {
  const CsLazy lz{reinterpret_cast<const float*>(h), reinterpret_cast<const float*>(dnext),
                  reinterpret_cast<const uint8_t*>(code), reinterpret_cast<const float*>(stats),
                  reinterpret_cast<const float*>(coef), pool};
  cf_stem_wgrad(nullptr, &lz, x, dw, ws, ws_floats, N, H, W, Nc, stream);
}
