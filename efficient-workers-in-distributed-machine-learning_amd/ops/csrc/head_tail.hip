// The VGG classifier's tail -- h2 = relu(h1 W2^T + b2), logits = h2 W3^T + b3, mean cross-entropy
// -- and its backward as two fp32 launches (the head's first Linear keeps head.hip's kernels, which
// own its dropout masks).  Replaces head.hip's fc2 / fc3 forward, the cross-entropy forward and the
// fc3 / fc2 backward launches (five -> two per step).
//
//   k_tail_fwd  grid (N2 / 16, ceil(B / 16)): a 16 x 16 tile of fc2 on v_mfma_f32_16x16x4_f32 (4
//               waves split K1), bias + ReLU, its share of the logits (partial sums over the
//               tile's 16 columns); the row tile's last arriving tile (ticket) sums the shares in
//               tile order -> logits, loss rows, d(logits) and dh2 = d(logits) W3 for its rows;
//               the last row tile sums the loss rows.  (models/lenet.py's fused step uses the same
//               scheme, ops/csrc/lenet_f32.hip.)
//   k_tail_bwd  dh1 = (dh2 * [h2 > 0]) W2 tiles (4 waves split N2), then one weight-gradient tile
//               per wave: dW2 = dz2^T h1 (db2 from the tiles' column sums), dW3 = dlogits^T h2
//               (db3 likewise).  Every gradient is scaled by the loss gradient read from memory.
// Hand-offs as in smallmap_f32.hip: agent-scope (sc1) stores drained before the ticket, sc1
// loads in the last arriver (cdna_hip_programming.md Guideline 16); sums in fixed orders.
// Parity: VGG's classifier (models/vgg.py, PyTorch-parameter-server/src/model_ops/vgg.py) with the
// reference's nn.CrossEntropyLoss (src/distributed_worker.py:249-251).
#include <cmath>
#include <stdexcept>
#include <string>

#include "common.h"
#include "ewdml_ops.h"

namespace {

typedef float f32x4 __attribute__((ext_vector_type(4)));

constexpr int TL_T = 256;   // 4 waves
constexpr int TL_FT = 16;   // tile
constexpr int TL_MAXK = 16; // classes
constexpr int TL_G = 8;     // loads per batch (all in flight before use)

#define TL_FENCE_SCHED() __builtin_amdgcn_sched_barrier(0)

__device__ __forceinline__ void tl_st(float* p, float v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ float tl_ld(const float* p) {
  return __hip_atomic_load(const_cast<float*>(p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ bool tl_ticket(int* cnt, int n, int* flag) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) {
    const int prev = __hip_atomic_fetch_add(cnt, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const int last = prev == n - 1;
    if (last) __hip_atomic_store(cnt, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    *flag = last;
  }
  __syncthreads();
  return *flag != 0;
}
__device__ __forceinline__ float tl_relu(float v) { return (v > 0.0f || v != v) ? v : 0.0f; }

// acc (16 rows x 16 cols) += A[rows][k0 ..) B[cols][k0 ..)^T over the chunks ch = w, w + 4, ... of
// 16 (A and B row-major with k contiguous, float4 per lane: lane group g takes k = 16 ch + 4 g +
// jj for MFMA jj in both operands); loads in batches of TL_G chunks
__device__ __forceinline__ f32x4 tl_kc_gemm(const float* ap, const float* bp, bool av, bool bv,
                                            int nch, int w) {
  f32x4 acc = {0.0f, 0.0f, 0.0f, 0.0f};
  for (int c0 = w; c0 < nch; c0 += 4 * TL_G) {
    f32x4 fa[TL_G], fb[TL_G];
#pragma unroll
    for (int i = 0; i < TL_G; ++i) {
      const int ch = min(c0 + 4 * i, nch - 1);
      fa[i] = *reinterpret_cast<const f32x4*>(ap + ch * 16);
      fb[i] = *reinterpret_cast<const f32x4*>(bp + ch * 16);
    }
    TL_FENCE_SCHED();
#pragma unroll
    for (int i = 0; i < TL_G; ++i) {
      if (c0 + 4 * i >= nch) break;
      const f32x4 a = av ? fa[i] : f32x4{0.0f, 0.0f, 0.0f, 0.0f};
      const f32x4 b = bv ? fb[i] : f32x4{0.0f, 0.0f, 0.0f, 0.0f};
#pragma unroll
      for (int jj = 0; jj < 4; ++jj) acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a[jj], b[jj], acc, 0, 0, 0);
    }
  }
  return acc;
}

// the 4 waves' accumulators summed in wave order into wave 0's
__device__ __forceinline__ f32x4 tl_wave_sum(f32x4 acc, f32x4 (*red)[64], int w, int l) {
  red[w][l] = acc;
  __syncthreads();
  f32x4 s = red[0][l];
#pragma unroll
  for (int r = 1; r < 4; ++r) s += red[r][l];
  return s;
}

__global__ __launch_bounds__(TL_T) void k_tail_fwd(
    const float* __restrict__ h1, const float* __restrict__ w2, const float* __restrict__ b2,
    const float* __restrict__ w3, const float* __restrict__ b3, const long long* __restrict__ y,
    int B, int K1, int N2, int K, float* __restrict__ h2, float* __restrict__ slab,
    int* __restrict__ cnt, float* __restrict__ lossrow, float* __restrict__ logits,
    float* __restrict__ dlogits, float* __restrict__ dh2, float* __restrict__ loss) {
  __shared__ f32x4 red[4][64];
  __shared__ float s_lg[TL_FT][TL_MAXK];
  __shared__ int s_flag;
  const int t = threadIdx.x, w = t >> 6, l = t & 63, g = l >> 4, li = l & 15;
  const int ct = blockIdx.x, rt = blockIdx.y, nct = gridDim.x, nrt = gridDim.y;
  const int Bp = nrt * TL_FT;
  {
    const int arow = rt * TL_FT + li, bcol = ct * TL_FT + li;
    // the epilogue's fc3 column and bias, loaded ahead of the GEMM (off its critical path)
    float wk[TL_MAXK];
#pragma unroll
    for (int k = 0; k < TL_MAXK; ++k) wk[k] = w3[(long long)min(k, K - 1) * N2 + bcol];
    const float bias = b2[bcol];
    const f32x4 acc = tl_kc_gemm(h1 + (long long)min(arow, B - 1) * K1 + 4 * g,
                                 w2 + (long long)bcol * K1 + 4 * g, arow < B, true, K1 / 16, w);
    const f32x4 s = tl_wave_sum(acc, red, w, l);
    if (w == 0) {
      const int col = bcol;
      float h[4];
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int row = rt * TL_FT + 4 * g + e;
        h[e] = tl_relu(s[e] + bias);
        if (row < B) h2[(long long)row * N2 + col] = h[e];
      }
      // this tile's share of the logits: sums over its 16 columns (lanes li of group g)
#pragma unroll
      for (int k = 0; k < TL_MAXK; ++k) {
        if (k >= K) break;
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          float p = h[e] * wk[k];
          p += __shfl_xor(p, 8, 64);
          p += __shfl_xor(p, 4, 64);
          p += __shfl_xor(p, 2, 64);
          p += __shfl_xor(p, 1, 64);
          if (li == 0) tl_st(slab + ((long long)ct * Bp + rt * TL_FT + 4 * g + e) * TL_MAXK + k, p);
        }
      }
    }
  }
  if (!tl_ticket(cnt + rt, nct, &s_flag)) return;
  // the row tile's logits (tile shares in tile order), loss rows, d(logits)
  for (int u = t; u < TL_FT * K; u += TL_T) {
    const int r = u / K, k = u - r * K;
    float s = 0.0f;
    for (int c0 = 0; c0 < nct; c0 += 16) {
      float v[16];
#pragma unroll
      for (int i = 0; i < 16; ++i)
        v[i] = tl_ld(slab + ((long long)min(c0 + i, nct - 1) * Bp + rt * TL_FT + r) * TL_MAXK + k);
      TL_FENCE_SCHED();
#pragma unroll
      for (int i = 0; i < 16; ++i)
        if (c0 + i < nct) s += v[i];
    }
    s_lg[r][k] = s + b3[k];
  }
  __syncthreads();
  if (t < TL_FT) {
    const int row = rt * TL_FT + t;
    if (row < B) {
      float m = s_lg[t][0];
      for (int k = 1; k < K; ++k) m = fmaxf(m, s_lg[t][k]);
      float se = 0.0f;
      for (int k = 0; k < K; ++k) se += expf(s_lg[t][k] - m);
      const float lse = m + logf(se);
      const int yy = min(max((int)y[row], 0), K - 1);
      tl_st(lossrow + row, lse - s_lg[t][yy]);
      const float inv = 1.0f / (float)B;
      for (int k = 0; k < K; ++k) {
        const float z = s_lg[t][k];
        logits[(long long)row * K + k] = z;
        const float d = (expf(z - m) / se - (k == yy ? 1.0f : 0.0f)) * inv;
        dlogits[(long long)row * K + k] = d;
        s_lg[t][k] = d;
      }
    }
  }
  // the loss ticket right after the loss rows (not behind the dh2 stores); the last row tile
  // sums them after its dh2
  const bool last_rt = tl_ticket(cnt + nrt, nrt, &s_flag);
  {
    // dh2 = d(logits) W3 for the 16 rows (k = classes, 4 steps of 4, masked past K); wave w takes
    // the column tiles w, w + 4, ...
    const int row = rt * TL_FT + li;
    float fa[TL_MAXK / 4];
#pragma unroll
    for (int s2 = 0; s2 < TL_MAXK / 4; ++s2) {
      const int k = 4 * s2 + g;
      fa[s2] = (k < K && row < B) ? s_lg[li][k] : 0.0f;
    }
    for (int tc0 = w; tc0 < nct; tc0 += 4 * TL_G) {  // TL_G column tiles' W3 loads in flight
      float fb[TL_G][TL_MAXK / 4];
#pragma unroll
      for (int i = 0; i < TL_G; ++i)
#pragma unroll
        for (int s2 = 0; s2 < TL_MAXK / 4; ++s2)
          fb[i][s2] = w3[(long long)min(4 * s2 + g, K - 1) * N2 +
                         min(tc0 + 4 * i, nct - 1) * TL_FT + li];
      TL_FENCE_SCHED();
#pragma unroll
      for (int i = 0; i < TL_G; ++i) {
        const int tc = tc0 + 4 * i;
        if (tc >= nct) break;
        f32x4 acc = {0.0f, 0.0f, 0.0f, 0.0f};
#pragma unroll
        for (int s2 = 0; s2 < TL_MAXK / 4; ++s2)
          acc = __builtin_amdgcn_mfma_f32_16x16x4f32(fa[s2], fb[i][s2], acc, 0, 0, 0);
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const int r2 = rt * TL_FT + 4 * g + e;
          if (r2 < B) dh2[(long long)r2 * N2 + tc * TL_FT + li] = acc[e];
        }
      }
    }
  }
  if (!last_rt) return;
  if (w == 0) {  // the mean loss: lane-strided partial sums, then a fixed shuffle tree
    float s = 0.0f;
    for (int r = l; r < B; r += 64) s += tl_ld(lossrow + r);
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) s += __shfl_xor(s, o, 64);
    if (l == 0) loss[0] = s / (float)B;
  }
}

// ---- backward: [0, nda) dh1 tiles; then one weight-gradient tile per wave: dW2 (N2/16 x K1/16
// tiles), dW3 (N2/16 tiles) ----
__global__ __launch_bounds__(TL_T) void k_tail_bwd(
    const float* __restrict__ h1, const float* __restrict__ h2, const float* __restrict__ dh2,
    const float* __restrict__ dlogits, const float* __restrict__ w2,
    const float* __restrict__ gscale, int B, int K1, int N2, int K, int nda,
    float* __restrict__ dh1, float* __restrict__ dw2, float* __restrict__ db2,
    float* __restrict__ dw3, float* __restrict__ db3) {
  __shared__ f32x4 red[4][64];
  const int t = threadIdx.x, w = t >> 6, l = t & 63, g = l >> 4, li = l & 15;
  const float gs = *gscale;
  const int b = blockIdx.x;
  const int ct1 = K1 / TL_FT, ct2 = N2 / TL_FT;
  if (b < nda) {
    // dh1[r][n] = sum_k dz2[r][k] w2[k][n], dz2 = dh2 * [h2 > 0], k < N2 in chunks of 16
    const int ct = b % ct1, rt = b / ct1;
    const int arow = rt * TL_FT + li, bcol = ct * TL_FT + li;
    const bool av = arow < B;
    const long long ao = (long long)min(arow, B - 1) * N2 + 4 * g;
    const int nch = N2 / 16;
    f32x4 acc = {0.0f, 0.0f, 0.0f, 0.0f};
    for (int c0 = w; c0 < nch; c0 += 4 * TL_G) {
      f32x4 fd[TL_G], fh[TL_G], fb[TL_G];
#pragma unroll
      for (int i = 0; i < TL_G; ++i) {
        const int ch = min(c0 + 4 * i, nch - 1);
        fd[i] = *reinterpret_cast<const f32x4*>(dh2 + ao + ch * 16);
        fh[i] = *reinterpret_cast<const f32x4*>(h2 + ao + ch * 16);
#pragma unroll
        for (int jj = 0; jj < 4; ++jj) fb[i][jj] = w2[(long long)(ch * 16 + 4 * g + jj) * K1 + bcol];
      }
      TL_FENCE_SCHED();
#pragma unroll
      for (int i = 0; i < TL_G; ++i) {
        if (c0 + 4 * i >= nch) break;
#pragma unroll
        for (int jj = 0; jj < 4; ++jj) {
          const float a = (av && fh[i][jj] > 0.0f) ? fd[i][jj] : 0.0f;  // ReLU backward
          acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a, fb[i][jj], acc, 0, 0, 0);
        }
      }
    }
    const f32x4 s = tl_wave_sum(acc, red, w, l);
    if (w == 0) {
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int row = rt * TL_FT + 4 * g + e;
        if (row < B) dh1[(long long)row * K1 + bcol] = gs * s[e];
      }
    }
    return;
  }
  const int tile = (b - nda) * 4 + w;
  const bool fc3 = tile >= ct2 * ct1;
  if (tile >= ct2 * ct1 + ct2) return;
  // out[m][n] = sum_r A[r][m] Bm[r][n] (k = batch rows, 4 per MFMA); the tile's bias gradient is
  // the column sum of A
  const int mt = fc3 ? 0 : tile / ct1, nt = fc3 ? tile - ct2 * ct1 : tile - (tile / ct1) * ct1;
  const int am = fc3 ? li : mt * TL_FT + li;              // A column: output row
  const int bn = nt * TL_FT + li;                         // B column: output column
  const bool amv = fc3 ? li < K : true;
  f32x4 acc = {0.0f, 0.0f, 0.0f, 0.0f};
  float asum = 0.0f;
  for (int r0 = 0; r0 < B; r0 += 4 * TL_G * 2) {
    float fa[2 * TL_G], fb[2 * TL_G], fm[2 * TL_G];
#pragma unroll
    for (int s2 = 0; s2 < 2 * TL_G; ++s2) {
      const long long r = min(r0 + 4 * s2 + g, B - 1);
      if (fc3) {
        fa[s2] = dlogits[r * K + min(am, K - 1)];
        fm[s2] = 1.0f;
        fb[s2] = h2[r * N2 + bn];
      } else {
        fa[s2] = dh2[r * N2 + am];
        fm[s2] = h2[r * N2 + am];
        fb[s2] = h1[r * K1 + bn];
      }
    }
    TL_FENCE_SCHED();
#pragma unroll
    for (int s2 = 0; s2 < 2 * TL_G; ++s2) {
      const bool rv = r0 + 4 * s2 + g < B;
      const float a = (rv && amv && fm[s2] > 0.0f) ? fa[s2] : 0.0f;  // dz2: ReLU backward
      const float bq = rv ? fb[s2] : 0.0f;
      acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a, bq, acc, 0, 0, 0);
      asum += a;
    }
  }
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    const int m = 4 * g + e;
    if (fc3) {
      if (m < K) dw3[(long long)m * N2 + bn] = gs * acc[e];
    } else {
      dw2[(long long)(mt * TL_FT + m) * K1 + bn] = gs * acc[e];
    }
  }
  asum += __shfl_xor(asum, 16, 64);
  asum += __shfl_xor(asum, 32, 64);
  if (g == 0 && amv) {
    if (!fc3 && nt == 0) db2[am] = gs * asum;
    if (fc3 && nt == 0) db3[am] = gs * asum;
  }
}

void tl_check(int B, int K1, int N2, int K) {
  if (B <= 0 || K1 <= 0 || N2 <= 0 || K1 % 16 || N2 % 16 || K <= 0 || K > TL_MAXK ||
      (long long)B * std::max(K1, N2) >= (1LL << 31))
    throw std::runtime_error("ewdml head tail: needs K1, N2 % 16 == 0 and 0 < classes <= 16");
}
void tl_aligned(uintptr_t p, const char* what) {
  if (p % 16) throw std::runtime_error(std::string("ewdml head tail: ") + what + " not 16-B aligned");
}

}  // namespace

// workspace floats (logit shares [N2/16][B16][16]) and ticket ints (row tiles + loss)
long long ew_tail_ws_floats(int B, int N2) {
  return (long long)(N2 / TL_FT) * ((B + TL_FT - 1) / TL_FT * TL_FT) * TL_MAXK;
}
int ew_tail_counters(int B) { return (B + TL_FT - 1) / TL_FT + 1; }

void ew_tail_fwd(uintptr_t h1, uintptr_t w2, uintptr_t b2, uintptr_t w3, uintptr_t b3, uintptr_t y,
                 int B, int K1, int N2, int K, uintptr_t h2, uintptr_t logits, uintptr_t dlogits,
                 uintptr_t dh2, uintptr_t lossrow, uintptr_t loss, uintptr_t ws,
                 long long ws_floats, uintptr_t cnt, int cnt_ints, uintptr_t stream) {
  tl_check(B, K1, N2, K);
  if (ws_floats < ew_tail_ws_floats(B, N2) || cnt_ints < ew_tail_counters(B))
    throw std::runtime_error("ewdml head tail: workspace too small");
  tl_aligned(h1, "h1");
  tl_aligned(w2, "fc2 weight");
  const int nrt = (B + TL_FT - 1) / TL_FT;
  hipLaunchKernelGGL(k_tail_fwd, dim3(N2 / TL_FT, nrt), dim3(TL_T), 0,
                     reinterpret_cast<hipStream_t>(stream), reinterpret_cast<const float*>(h1),
                     reinterpret_cast<const float*>(w2), reinterpret_cast<const float*>(b2),
                     reinterpret_cast<const float*>(w3), reinterpret_cast<const float*>(b3),
                     reinterpret_cast<const long long*>(y), B, K1, N2, K,
                     reinterpret_cast<float*>(h2), reinterpret_cast<float*>(ws),
                     reinterpret_cast<int*>(cnt), reinterpret_cast<float*>(lossrow),
                     reinterpret_cast<float*>(logits), reinterpret_cast<float*>(dlogits),
                     reinterpret_cast<float*>(dh2), reinterpret_cast<float*>(loss));
  EW_CHECK_LAUNCH();
}

void ew_tail_bwd(uintptr_t h1, uintptr_t h2, uintptr_t dh2, uintptr_t dlogits, uintptr_t w2,
                 uintptr_t gscale, int B, int K1, int N2, int K, uintptr_t dh1, uintptr_t dw2,
                 uintptr_t db2, uintptr_t dw3, uintptr_t db3, uintptr_t stream) {
  tl_check(B, K1, N2, K);
  tl_aligned(h2, "h2");
  tl_aligned(dh2, "dh2");
  const int nrt = (B + TL_FT - 1) / TL_FT;
  const int nda = nrt * (K1 / TL_FT);
  const int nwt = ((N2 / TL_FT) * (K1 / TL_FT) + N2 / TL_FT + 3) / 4;
  hipLaunchKernelGGL(k_tail_bwd, dim3(nda + nwt), dim3(TL_T), 0,
                     reinterpret_cast<hipStream_t>(stream), reinterpret_cast<const float*>(h1),
                     reinterpret_cast<const float*>(h2), reinterpret_cast<const float*>(dh2),
                     reinterpret_cast<const float*>(dlogits), reinterpret_cast<const float*>(w2),
                     reinterpret_cast<const float*>(gscale), B, K1, N2, K, nda,
                     reinterpret_cast<float*>(dh1), reinterpret_cast<float*>(dw2),
                     reinterpret_cast<float*>(db2), reinterpret_cast<float*>(dw3),
                     reinterpret_cast<float*>(db3));
  EW_CHECK_LAUNCH();
}
