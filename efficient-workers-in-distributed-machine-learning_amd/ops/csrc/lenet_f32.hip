// LeNet's training step in four fp32 launches (BASELINE config #2: LeNet / MNIST, batch 64).
//
// The network (models/lenet.py, PyTorch-parameter-server/src/model_ops/lenet.py:15-36):
//   x [1x28x28] -> conv1 20 k5 (+b) -> 2x2 max pool -> relu -> a1 [20x12x12]
//   -> conv2 50 k5 (+b) -> 2x2 max pool -> relu -> a2 [800] -> fc1 500 (+b) -> h1 -> fc2 K (+b)
//   -> mean cross-entropy.
// At batch 64 the whole step is ~0.9 GFLOP: every layer is far below the size at which a
// library GEMM / conv fills 256 CUs, and the module composition (MIOpen convs, hipBLASLt, pool /
// relu / bias / reduce kernels, transposes) spends the step in ~37 launch floors.  Here:
//
//   k_ln_conv_fwd  grid (4, B): block (q, n) = image n's conv1 + pool + relu for the a1 rows its
//                  conv2 output row pair needs (in LDS), then conv2 + pool + relu of pooled row q
//                  (thread = (out channel, column, conv row): the 2x2 window's two rows meet by a
//                  lane shuffle).  Writes a1 / a2 and the pool window codes (backward routing).
//   k_ln_fc_fwd    grid (32, B / 16): a 16x16 tile of fc1 on v_mfma_f32_16x16x4_f32 (4 waves
//                  split K = 800), its share of fc2's logits (partial sums per column tile); the
//                  last tile of a row tile to finish (ticket) sums the partials in tile order ->
//                  logits, cross-entropy, dlogits and dh1 = dlogits W_fc2 for its 16 rows; the
//                  last row tile sums the per-row losses -> the mean loss.
//   k_ln_fc_bwd    da2 = dh1 W_fc1 tiles (relu mask applied: dp2, the pooled conv2 gradient),
//                  dW_fc1 = dh1^T a2 tiles (one wave each), db_fc1 / dW_fc2 / db_fc2.
//   k_ln_conv_bwd  (2B blocks) image halves: da1 = conv2^T(dy2) gathered from the sparse unpooled
//                  dy2 (one non-zero per window, at its code), relu mask -> dp1 in LDS, the block's
//                  partial dW_conv1 / db_conv1; the last of the 2B blocks sums the partials in
//                  block order.  (10 * ceil(B / 8) blocks) dW_conv2 / db_conv2 partials per
//                  (5 output channels, 8 images) over a1 staged in LDS; the last image group of
//                  each channel group sums them in group order.
//
// Cross-block hand-offs (the tickets) follow smallmap_f32.hip: agent-scope relaxed (sc1) stores,
// every wave drains its stores before the block's barrier, one lane draws the ticket, the last
// arriver reads with agent-scope loads and re-arms the counter (cdna_hip_programming.md
// Guideline 16).  Every sum runs in a fixed order: the step is bitwise reproducible.
// The backward scales every gradient by the loss gradient g read from device memory (1 for the
// trainer's persistent seed: exact).
#include <cmath>
#include <cstdlib>
#include <stdexcept>
#include <string>

#include "common.h"
#include "ewdml_ops.h"

namespace {

typedef float f32x4 __attribute__((ext_vector_type(4)));

constexpr int LN_T = 512;                  // conv kernels' block
constexpr int LN_FT = 256;                 // fc kernels' block (4 waves)
constexpr int C1 = 20, C2 = 50, KS = 5, TAPS = 25;
constexpr int IN = 28, P1 = 12, P2 = 4;
constexpr int A1N = C1 * P1 * P1;          // 2880: a1 per image
constexpr int A2N = C2 * P2 * P2;          // 800: a2 per image (fc1's input)
constexpr int F1 = 500;                    // fc1 outputs
constexpr int W1N = C1 * TAPS;             // 500
constexpr int W2N = C2 * C1 * TAPS;        // 25000
constexpr int MAXK = 16;                   // classes
constexpr int FT = 16;                     // fc tile
constexpr int F1T = (F1 + FT - 1) / FT;    // 32 column tiles of fc1 / row tiles of dW_fc1
constexpr int A2T = A2N / FT;              // 50 column tiles of da2 / dW_fc1
constexpr int W2P = C1 * TAPS + 1;         // dW_conv2 partial row per out channel: 500 + bias
constexpr int OG = 5, NOG = C2 / OG;       // dW_conv2: out channels per block, groups
constexpr int IG = 2;                      // dW_conv2: images per block

__device__ __forceinline__ void sc1_store(float* p, float v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ float sc1_load(const float* p) {
  return __hip_atomic_load(const_cast<float*>(p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// Block-wide ticket over n arrivals: every wave's sc1 stores drained, one lane draws; true in
// the last arriver (which re-arms the counter)
__device__ __forceinline__ bool ln_ticket(int* cnt, int n, int* flag) {
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

// 2x2 max in window order (0,0) (0,1) (1,0) (1,1): the first maximum wins and a NaN sticks
// (max_pool2d's rule); code = the winner's position dy * 2 + dx
__device__ __forceinline__ float ln_pool4(float v0, float v1, float v2, float v3, int& code) {
  float m = v0;
  int c = 0;
  if (v1 > m || v1 != v1) { m = v1; c = 1; }
  if (v2 > m || v2 != v2) { m = v2; c = 2; }
  if (v3 > m || v3 != v3) { m = v3; c = 3; }
  code = c;
  return m;
}
__device__ __forceinline__ float ln_relu(float v) { return (v > 0.0f || v != v) ? v : 0.0f; }

// Keeps the scheduler from sinking a batch of loads down to their uses (it otherwise interleaves
// them 2-3 deep with the consumers, one memory round trip per few loads)
#define LN_FENCE_SCHED() __builtin_amdgcn_sched_barrier(0)

// LDS <- global, n4 (<= N4) float4s by LN_T threads: every load of a thread is issued before its
// first LDS write (a plain copy loop waits for each load in turn: ~one L2 round trip per float4)
template <int N4>
__device__ __forceinline__ void ln_stage(float* dst, const float* src, int n4, int t) {
  constexpr int R = (N4 + LN_T - 1) / LN_T;
  f32x4 v[R];
#pragma unroll
  for (int i = 0; i < R; ++i)
    v[i] = reinterpret_cast<const f32x4*>(src)[min(t + i * LN_T, n4 - 1)];
  LN_FENCE_SCHED();
#pragma unroll
  for (int i = 0; i < R; ++i)
    if (t + i * LN_T < n4) reinterpret_cast<f32x4*>(dst)[t + i * LN_T] = v[i];
}

// ---- forward convolutions: block (q, n), q = conv2's pooled output row ----
constexpr int LN_CT = 256;  // conv forward block (4 waves)

// The batch formed in the conv launch instead of its own (data/loader.py DeviceLoader, the
// k_make_batch arithmetic of data.hip without augmentation, 1 channel): every block normalises
// image n from the uint8 source at its slot of the permutation, the q = 0 blocks write it (for
// the backward) and its label, and the launch's last block advances the batch position -- as
// k_make_batch does, bit for bit.  src == nullptr: x is an ordinary input.
struct LnBatch {
  const uint8_t* src;
  const long long* labels;
  const long long* perm;
  long long* state;  // {position, epoch}
  int* done;         // arrival ticket (zeroed, left zeroed)
  long long perm_len;
  float mean, inv_std;
  long long* y_out;
};

__global__ __launch_bounds__(LN_CT) void k_ln_conv_fwd(const float* __restrict__ x,
                                                       const float* __restrict__ w1,
                                                       const float* __restrict__ b1,
                                                       const float* __restrict__ w2,
                                                       const float* __restrict__ b2,
                                                       float* __restrict__ a1,
                                                       uint8_t* __restrict__ code1,
                                                       float* __restrict__ a2,
                                                       uint8_t* __restrict__ code2,
                                                       LnBatch bt) {
  __shared__ __attribute__((aligned(16))) float s_x[IN * IN];
  __shared__ __attribute__((aligned(16))) float s_w1[W1N];
  __shared__ float s_b1[C1];
  __shared__ float s_a1[C1 * 6 * P1];  // a1 rows 2q .. 2q + 5 (conv2 rows 2q, 2q + 1 read them)
  __shared__ short s_ko[W1N];          // conv2 reduction index (c, ky, kx) -> s_a1 offset
  const int t = threadIdx.x, q = blockIdx.x, n = blockIdx.y;
  const int w = t >> 6, l = t & 63, g = l >> 4, li = l & 15;
  const int r0 = 2 * q;
  long long bpos = 0;
  {
    f32x4 xv;
    if (bt.src) {
      bpos = bt.state[0];
      long long slot = bpos * gridDim.y + n;
      if (slot >= bt.perm_len) slot %= bt.perm_len;  // never read past the permutation
      const long long sample = bt.perm[slot];
      const uint32_t px = reinterpret_cast<const uint32_t*>(
          bt.src + sample * (IN * IN))[min(t, IN * IN / 4 - 1)];
#pragma unroll
      for (int k = 0; k < 4; ++k)
        xv[k] = ((float)((px >> (8 * k)) & 0xffu) * (1.0f / 255.0f) - bt.mean) * bt.inv_std;
      if (q == 0) {
        if (t < IN * IN / 4)
          reinterpret_cast<f32x4*>(const_cast<float*>(x) + (long long)n * IN * IN)[t] = xv;
        if (t == 0) bt.y_out[n] = bt.labels[sample];
      }
    } else {
      const f32x4* xs = reinterpret_cast<const f32x4*>(x + (long long)n * IN * IN);
      xv = xs[min(t, IN * IN / 4 - 1)];
    }
    const f32x4 wv = reinterpret_cast<const f32x4*>(w1)[min(t, W1N / 4 - 1)];
    const float bv = b1[min(t, C1 - 1)];
    if (t < IN * IN / 4) reinterpret_cast<f32x4*>(s_x)[t] = xv;
    if (t < W1N / 4) reinterpret_cast<f32x4*>(s_w1)[t] = wv;
    if (t < C1) s_b1[t] = bv;
    for (int k = t; k < W1N; k += LN_CT) {
      const int c = k / TAPS, r = k - c * TAPS, ky = r / KS;
      s_ko[k] = (short)(c * 6 * P1 + ky * P1 + r - ky * KS);
    }
  }
  __syncthreads();
  // conv1 + bias + pool + relu; block q writes a1 rows 2q, 2q + 1 (q = 3: rows 6 .. 11)
  for (int u = t; u < C1 * 6 * P1; u += LN_CT) {
    const int c = u / (6 * P1), rem = u - c * 6 * P1, rr = rem / P1, j = rem - rr * P1;
    const int R = r0 + rr;
    const float* wc = s_w1 + c * TAPS;
    const float* xp = s_x + 2 * R * IN + 2 * j;
    float v[4] = {0.0f, 0.0f, 0.0f, 0.0f};
#pragma unroll
    for (int ky = 0; ky < KS + 1; ++ky) {
      float xr[6];
#pragma unroll
      for (int z = 0; z < 6; ++z) xr[z] = xp[ky * IN + z];
#pragma unroll
      for (int kx = 0; kx < KS; ++kx) {
        // input row ky serves conv row 2R (tap ky) and conv row 2R + 1 (tap ky - 1)
        if (ky < KS) {
          const float wv = wc[ky * KS + kx];
          v[0] = fmaf(xr[kx], wv, v[0]);
          v[1] = fmaf(xr[kx + 1], wv, v[1]);
        }
        if (ky > 0) {
          const float wv = wc[(ky - 1) * KS + kx];
          v[2] = fmaf(xr[kx], wv, v[2]);
          v[3] = fmaf(xr[kx + 1], wv, v[3]);
        }
      }
    }
    int code;
    const float bb = s_b1[c];
    const float a = ln_relu(ln_pool4(v[0] + bb, v[1] + bb, v[2] + bb, v[3] + bb, code));
    s_a1[u] = a;
    if (q == 3 || rr < 2) {
      const long long o = (long long)n * A1N + c * P1 * P1 + R * P1 + j;
      a1[o] = a;
      code1[o] = (uint8_t)code;
    }
  }
  __syncthreads();
  // conv2 on v_mfma_f32_16x16x4_f32: M = the 16 conv positions (dy, col) of rows 2q, 2q + 1,
  // N = out channels (wave w: 16 w .. 16 w + 15), K = (c, ky, kx) = 500 in 32 chunks of 16 (lane
  // group g takes k = 16 ch + 4 g + jj for MFMA jj in both operands).  B rows are W_conv2 rows,
  // read as float4s straight from global memory (all 32 in flight before the first MFMA).
  {
    const int oc = min(16 * w + li, C2 - 1);
    const float* wrow = w2 + (long long)oc * (C1 * TAPS);
    constexpr int NCH = (C1 * TAPS + 15) / 16;  // 32 (the last chunk 4 deep)
    f32x4 fb[NCH];
#pragma unroll
    for (int ch = 0; ch < NCH; ++ch)
      fb[ch] = *reinterpret_cast<const f32x4*>(wrow + min(16 * ch + 4 * g, C1 * TAPS - 4));
    LN_FENCE_SCHED();
    const int abase = (li >> 3) * P1 + (li & 7);
    f32x4 acc = {0.0f, 0.0f, 0.0f, 0.0f};
#pragma unroll
    for (int ch = 0; ch < NCH; ++ch) {
      const int k0 = 16 * ch + 4 * g;
      const bool kv = k0 < C1 * TAPS;  // 500 is a multiple of 4: all 4 k or none
      f32x4 fa;
#pragma unroll
      for (int jj = 0; jj < 4; ++jj) fa[jj] = kv ? s_a1[abase + s_ko[min(k0 + jj, C1 * TAPS - 1)]] : 0.0f;
#pragma unroll
      for (int jj = 0; jj < 4; ++jj) acc = __builtin_amdgcn_mfma_f32_16x16x4f32(fa[jj], fb[ch][jj], acc, 0, 0, 0);
    }
    // D lane (g, li) reg e = position 4 g + e (dy = g >> 1, column 4 (g & 1) + e), channel li;
    // the window's second row sits in lane l ^ 32
    const float bb = b2[oc];
    float v[4], u[4];
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      v[e] = acc[e] + bb;
      u[e] = __shfl_xor(v[e], 32, 64);
    }
    const int o = 16 * w + li;
    if (g < 2 && o < C2) {
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        int code;
        const float m = ln_pool4(v[2 * h], v[2 * h + 1], u[2 * h], u[2 * h + 1], code);
        const int j = 2 * g + h;
        const long long i = (long long)n * A2N + o * P2 * P2 + q * P2 + j;
        a2[i] = ln_relu(m);
        code2[i] = (uint8_t)code;
      }
    }
  }
  if (bt.src) {
    // the launch's last block advances the batch position (k_make_batch's rule: every block read
    // it before its barrier, hence before its arrival)
    __syncthreads();
    if (t == 0 && ew_grid_last(bt.done)) bt.state[0] = bpos + 1;
  }
}

// ---- fc1 + fc2 + cross-entropy: block (ct, rt) = fc1 tile (16 rows x 16 columns) ----
__global__ __launch_bounds__(LN_FT) void k_ln_fc_fwd(
    const float* __restrict__ a2, const float* __restrict__ wf1, const float* __restrict__ bf1,
    const float* __restrict__ wf2, const float* __restrict__ bf2, const long long* __restrict__ y,
    int B, int K, float* __restrict__ h1, float* __restrict__ slab, int* __restrict__ cnt,
    float* __restrict__ lossrow, float* __restrict__ logits, float* __restrict__ dlogits,
    float* __restrict__ dh1, float* __restrict__ loss) {
  __shared__ f32x4 s_acc[4][64];
  __shared__ float s_lg[FT][MAXK];
  __shared__ int s_flag;
  const int t = threadIdx.x, w = t >> 6, l = t & 63, g = l >> 4, li = l & 15;
  const int ct = blockIdx.x, rt = blockIdx.y, nrt = gridDim.y;
  const int Bp = nrt * FT;
  {
    // A lane l = a2[row li][k], B lane l = wf1[col li][k]: lane group g takes k = 16 ch + 4 g + jj
    // for MFMA jj of chunk ch (the same permutation in both operands)
    const int arow = rt * FT + li, bcol = ct * FT + li;
    const bool av = arow < B, bv = bcol < F1;
    const float* ap = a2 + (long long)min(arow, B - 1) * A2N + 4 * g;
    const float* bp = wf1 + (long long)min(bcol, F1 - 1) * A2N + 4 * g;
    // wave w: chunks w, w + 4, ... (13 or 12 of the 50), every load in flight before the MFMAs
    constexpr int NCH = (A2N / 16 + 3) / 4;
    f32x4 fa[NCH], fb[NCH];
#pragma unroll
    for (int i = 0; i < NCH; ++i) {
      const int ch = min(w + 4 * i, A2N / 16 - 1);
      fa[i] = *reinterpret_cast<const f32x4*>(ap + ch * 16);
      fb[i] = *reinterpret_cast<const f32x4*>(bp + ch * 16);
    }
    LN_FENCE_SCHED();
    f32x4 acc = {0.0f, 0.0f, 0.0f, 0.0f};
#pragma unroll
    for (int i = 0; i < NCH; ++i) {
      if (w + 4 * i >= A2N / 16) continue;
      const f32x4 a = av ? fa[i] : f32x4{0.0f, 0.0f, 0.0f, 0.0f};
      const f32x4 bq = bv ? fb[i] : f32x4{0.0f, 0.0f, 0.0f, 0.0f};
#pragma unroll
      for (int jj = 0; jj < 4; ++jj) acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a[jj], bq[jj], acc, 0, 0, 0);
    }
    s_acc[w][l] = acc;
  }
  __syncthreads();
  if (w == 0) {
    f32x4 s = s_acc[0][l];
#pragma unroll
    for (int r = 1; r < 4; ++r) s += s_acc[r][l];  // fixed order
    const int col = ct * FT + li;
    const bool cv = col < F1;
    const float bias = cv ? bf1[col] : 0.0f;
    float h[4];
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const int row = rt * FT + 4 * g + e;
      h[e] = cv ? s[e] + bias : 0.0f;
      if (cv && row < B) h1[(long long)row * F1 + col] = h[e];
    }
    // this column tile's share of the logits: sum over its 16 columns (lanes li of group g)
    float wks[MAXK];
#pragma unroll
    for (int k = 0; k < MAXK; ++k) wks[k] = wf2[min(k, K - 1) * F1 + min(col, F1 - 1)];
    LN_FENCE_SCHED();
#pragma unroll
    for (int k = 0; k < MAXK; ++k) {
      if (k >= K) break;
      const float wk = cv ? wks[k] : 0.0f;
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        float p = h[e] * wk;
        p += __shfl_xor(p, 8, 64);
        p += __shfl_xor(p, 4, 64);
        p += __shfl_xor(p, 2, 64);
        p += __shfl_xor(p, 1, 64);
        if (li == 0) sc1_store(slab + ((long long)ct * Bp + rt * FT + 4 * g + e) * MAXK + k, p);
      }
    }
  }
  if (!ln_ticket(cnt + rt, gridDim.x, &s_flag)) return;
  // last column tile of row tile rt: logits, loss, dlogits, dh1 for rows rt * 16 ..
  for (int u = t; u < FT * K; u += LN_FT) {  // the 32 partials of (row, class): all in flight
    const int r = u / K, k = u - r * K;
    float v[F1T];
#pragma unroll
    for (int c2 = 0; c2 < F1T; ++c2) v[c2] = sc1_load(slab + ((long long)c2 * Bp + rt * FT + r) * MAXK + k);
    LN_FENCE_SCHED();
    float s = 0.0f;
#pragma unroll
    for (int c2 = 0; c2 < F1T; ++c2) s += v[c2];
    s_lg[r][k] = s + bf2[k];
  }
  __syncthreads();
  if (t < FT) {
    const int row = rt * FT + t;
    if (row < B) {
      float m = s_lg[t][0];
      for (int k = 1; k < K; ++k) m = fmaxf(m, s_lg[t][k]);
      float se = 0.0f;
      for (int k = 0; k < K; ++k) se += expf(s_lg[t][k] - m);
      const float lse = m + logf(se);
      const int yy = min(max((int)y[row], 0), K - 1);
      sc1_store(lossrow + row, lse - s_lg[t][yy]);
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
  __syncthreads();
  {
    // dh1 = dlogits W_fc2 for the 16 rows: 32 column tiles of 16 (wave w: tiles w + 4 i), k =
    // classes in 4 steps of 4 (masked past K); every W_fc2 load in flight before the MFMAs
    const int row = rt * FT + li;
    float fa[MAXK / 4];
#pragma unroll
    for (int s2 = 0; s2 < MAXK / 4; ++s2) {
      const int k = 4 * s2 + g;
      fa[s2] = (k < K && row < B) ? s_lg[li][k] : 0.0f;
    }
    constexpr int NT = F1T / 4;
    float fb[NT][MAXK / 4];
#pragma unroll
    for (int i = 0; i < NT; ++i)
#pragma unroll
      for (int s2 = 0; s2 < MAXK / 4; ++s2) {
        const int k = min(4 * s2 + g, K - 1), col = min((w + 4 * i) * FT + li, F1 - 1);
        fb[i][s2] = wf2[k * F1 + col];
      }
    LN_FENCE_SCHED();
#pragma unroll
    for (int i = 0; i < NT; ++i) {
      f32x4 acc = {0.0f, 0.0f, 0.0f, 0.0f};
#pragma unroll
      for (int s2 = 0; s2 < MAXK / 4; ++s2)
        acc = __builtin_amdgcn_mfma_f32_16x16x4f32(fa[s2], fb[i][s2], acc, 0, 0, 0);
      const int col = (w + 4 * i) * FT + li;
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int r2 = rt * FT + 4 * g + e;
        if (r2 < B && col < F1) dh1[(long long)r2 * F1 + col] = acc[e];
      }
    }
  }
  if (!ln_ticket(cnt + nrt, nrt, &s_flag)) return;
  if (w == 0) {  // the mean loss: lane-strided partial sums, then a fixed shuffle tree
    float s = 0.0f;
    for (int r = l; r < B; r += 64) s += sc1_load(lossrow + r);
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) s += __shfl_xor(s, o, 64);
    if (l == 0) loss[0] = s / (float)B;
  }
}

// ---- fc backward: [0, nda) da2 tiles (4 waves split K = 500); then one weight-gradient tile per
// wave: dW_fc1 (32 x 50 tiles, db_fc1 folded into the nt = 0 column) and dW_fc2 (32 tiles,
// db_fc2 folded into tile 0) ----
constexpr int LN_WT = F1T * A2T + F1T;  // weight-gradient tiles

__global__ __launch_bounds__(LN_FT) void k_ln_fc_bwd(
    const float* __restrict__ a2, const float* __restrict__ h1, const float* __restrict__ dlogits,
    const float* __restrict__ dh1, const float* __restrict__ wf1, const float* __restrict__ gscale,
    int B, int K, int nda, float* __restrict__ dp2, float* __restrict__ dwf1,
    float* __restrict__ dbf1, float* __restrict__ dwf2, float* __restrict__ dbf2) {
  __shared__ f32x4 s_acc[4][64];
  const int t = threadIdx.x, w = t >> 6, l = t & 63, g = l >> 4, li = l & 15;
  const float gs = *gscale;
  const int b = blockIdx.x;
  if (b < nda) {
    // da2[r][n] = sum_k dh1[r][k] wf1[k][n] over k < 500 (32 chunks of 16, the last 4 deep; wave
    // w takes chunks w + 4 i, every load in flight before the MFMAs)
    const int ct = b % A2T, rt = b / A2T;
    const int arow = rt * FT + li, bcol = ct * FT + li;
    const bool av = arow < B;
    const float* ap = dh1 + (long long)min(arow, B - 1) * F1;
    constexpr int NCH = F1T / 4;
    f32x4 fa[NCH], fb[NCH];
#pragma unroll
    for (int i = 0; i < NCH; ++i) {
      const int k = (w + 4 * i) * 16 + 4 * g;
      fa[i] = *reinterpret_cast<const f32x4*>(ap + min(k, F1 - 4));
#pragma unroll
      for (int jj = 0; jj < 4; ++jj) fb[i][jj] = wf1[(long long)min(k + jj, F1 - 1) * A2N + bcol];
    }
    LN_FENCE_SCHED();
    f32x4 acc = {0.0f, 0.0f, 0.0f, 0.0f};
#pragma unroll
    for (int i = 0; i < NCH; ++i) {
      // k is a multiple of 4 and so is F1: a lane's 4 k are all in range or all out
      const bool ok = av && (w + 4 * i) * 16 + 4 * g < F1;
      const f32x4 a = ok ? fa[i] : f32x4{0.0f, 0.0f, 0.0f, 0.0f};
#pragma unroll
      for (int jj = 0; jj < 4; ++jj) acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a[jj], fb[i][jj], acc, 0, 0, 0);
    }
    s_acc[w][l] = acc;
    __syncthreads();
    if (w == 0) {
      f32x4 s = s_acc[0][l];
#pragma unroll
      for (int r = 1; r < 4; ++r) s += s_acc[r][l];
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int row = rt * FT + 4 * g + e;
        if (row < B) {
          const long long i = (long long)row * A2N + bcol;
          const float d = gs * s[e];
          dp2[i] = a2[i] > 0.0f ? d : 0.0f;  // relu backward
        }
      }
    }
    return;
  }
  // weight-gradient tile: out[m][n] = sum_r A[r][m] Bm[r][n] (k = batch rows, 4 per MFMA); the
  // bias gradient of the tile's rows is the column sum of A (lane sums, then over lane groups)
  const int tile = (b - nda) * 4 + w;
  if (tile >= LN_WT) return;
  const bool fc2 = tile >= F1T * A2T;
  const int jt = fc2 ? tile - F1T * A2T : tile / A2T, nt = fc2 ? 0 : tile - jt * A2T;
  const float* pa = fc2 ? dlogits : dh1;
  const float* pb = fc2 ? h1 : a2;
  const int lda = fc2 ? K : F1, ldb = fc2 ? F1 : A2N;
  const int am = fc2 ? li : jt * FT + li;             // A column (output row m)
  const int bn = fc2 ? jt * FT + li : nt * FT + li;   // B column (output column n)
  const bool amv = am < (fc2 ? K : F1), bnv = bn < (fc2 ? F1 : A2N);
  const int amc = min(am, lda - 1), bnc = min(bn, ldb - 1);
  f32x4 acc = {0.0f, 0.0f, 0.0f, 0.0f};
  float asum = 0.0f;
  for (int r0 = 0; r0 < B; r0 += 64) {
    float fa[16], fb[16];
#pragma unroll
    for (int s2 = 0; s2 < 16; ++s2) {
      const int r = min(r0 + 4 * s2 + g, B - 1);
      fa[s2] = pa[(long long)r * lda + amc];
      fb[s2] = pb[(long long)r * ldb + bnc];
    }
    LN_FENCE_SCHED();
#pragma unroll
    for (int s2 = 0; s2 < 16; ++s2) {
      const bool rv = r0 + 4 * s2 + g < B;
      const float a = (rv && amv) ? fa[s2] : 0.0f;
      const float bq = (rv && bnv) ? fb[s2] : 0.0f;
      acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a, bq, acc, 0, 0, 0);
      asum += a;
    }
  }
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    const int m = 4 * g + e;
    if (fc2) {
      if (m < K && bn < F1) dwf2[(long long)m * F1 + bn] = gs * acc[e];
    } else {
      const int j = jt * FT + m;
      if (j < F1) dwf1[(long long)j * A2N + bn] = gs * acc[e];
    }
  }
  asum += __shfl_xor(asum, 16, 64);
  asum += __shfl_xor(asum, 32, 64);
  if (g == 0 && amv) {
    if (!fc2 && nt == 0) dbf1[am] = gs * asum;
    if (fc2 && jt == 0) dbf2[am] = gs * asum;
  }
}

// ---- conv backward.  [0, 4B): block (n, cq) = image n, conv1 channels 5 cq .. 5 cq + 4:
// d(a1) as a transposed convolution on the matrix cores -- S[(p, q)][(c, ky, kx)] =
// sum_o dy2[o][p][q] W_conv2[o][c][ky][kx] (M = the 64 conv2 positions, N = the group's 125
// weight columns, K = 50 out channels), then d(a1)[c][y][x] = sum_(ky, kx) S[(y - ky, x - kx)]
// [(c, ky, kx)] -- the relu mask (dp1), and the block's dW_conv1 / db_conv1 partial for its 5
// channels; per channel group the partials of 16 images, then of the image groups, are summed in
// order by the last arrivals.  [4B, 4B + NOG * ngr): dW_conv2 block (out-channel group og, image
// group ig) ----
constexpr int LN_CQ = 5;                       // conv1 channels per d(a1) block
constexpr int LN_SN = LN_CQ * TAPS;            // 125 S columns per block
constexpr int LN_AP = 52;                      // A (dy2^T) row pitch: 50 out channels + pad
constexpr int LN_SP = 129;                     // S row pitch
constexpr int LN_W1Q = LN_SN + LN_CQ;          // dW_conv1 partial row: 125 weights + 5 biases
constexpr int LN_GA = 16;                      // images per first-level dW_conv1 group
constexpr int LN_A_LDS = 64 * LN_AP + 64 * LN_SP + IN * IN + LN_CQ * P1 * P1 + LN_CQ * P1 * P1 / 4 +
                         3 * LN_W1Q;           // floats
constexpr int LN_B_LDS = IG * A1N + 2 * IG * OG * 16;
constexpr int LN_BWD_LDS = LN_A_LDS > LN_B_LDS ? LN_A_LDS : LN_B_LDS;
static_assert(W2P - 1 + OG <= LN_T && LN_CQ * P1 * P1 <= 2 * LN_T && 3 * LN_W1Q <= LN_T &&
                  IG * OG * 16 <= LN_T,
              "thread maps");

__global__ __launch_bounds__(LN_T) void k_ln_conv_bwd(
    const float* __restrict__ x, const float* __restrict__ w2, const float* __restrict__ a1,
    const uint8_t* __restrict__ code1, const uint8_t* __restrict__ code2,
    const float* __restrict__ dp2, int B, float* __restrict__ part1, float* __restrict__ part1g,
    float* __restrict__ part2, int* __restrict__ cnt, float* __restrict__ dw1,
    float* __restrict__ db1, float* __restrict__ dw2, float* __restrict__ db2, int boff,
    long long* __restrict__ prof) {
  __shared__ __attribute__((aligned(16))) float smem[LN_BWD_LDS];
  __shared__ int s_flag;
  const int t = threadIdx.x;
  const int na = 4 * B, ngi = (B + LN_GA - 1) / LN_GA;
  const int bid = (int)blockIdx.x + boff;  // boff / a shorter grid: one part alone (probes)
  // prof (probes): thread 0 stamps wall_clock64() at the phase boundaries, 8 per block
#define LN_STAMP(i) \
  if (prof && t == 0) prof[(long long)blockIdx.x * 8 + (i)] = wall_clock64()
  LN_STAMP(0);
  if (bid < na) {
    float* s_A = smem;                               // [64 (p, q)][52]: dy2^T
    float* s_S = s_A + 64 * LN_AP;                   // [64 (p, q)][129]
    float* s_x = s_S + 64 * LN_SP;                   // [28][28]
    float* s_dp1 = s_x + IN * IN;                    // [5][144]
    uint8_t* s_c1 = reinterpret_cast<uint8_t*>(s_dp1 + LN_CQ * P1 * P1);  // [5][144]
    float* s_red = s_dp1 + LN_CQ * P1 * P1 + LN_CQ * P1 * P1 / 4;         // [3][130]
    const int n = bid >> 2, cq = bid & 3;
    const int w = t >> 6, l = t & 63, g = l >> 4, li = l & 15;
    // B operand (W_conv2 rows o, the group's 125 columns): wave w = S columns 16 w .. 16 w + 15,
    // k = o = 4 s + g; all 13 loads in flight while the staging below runs
    const int bcol = 16 * w + li;
    float fb[13];
#pragma unroll
    for (int s2 = 0; s2 < 13; ++s2)
      fb[s2] = w2[(long long)min(4 * s2 + g, C2 - 1) * (C1 * TAPS) + cq * LN_SN + min(bcol, LN_SN - 1)];
    {
      // dy2^T: window (o, i, j) puts its value at its maximum's position, zeros at the other three
      const long long o2 = (long long)n * A2N;
      float dv[2];
      int ev[2];
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const int v = min(t + h * LN_T, A2N - 1);
        dv[h] = dp2[o2 + v];
        ev[h] = code2[o2 + v];
      }
      const float xv0 = x[(long long)n * IN * IN + t];
      const float xv1 = x[(long long)n * IN * IN + min(t + LN_T, IN * IN - 1)];
      uint8_t kc[2];
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const int v = min(t + h * LN_T, LN_CQ * P1 * P1 - 1);
        kc[h] = code1[(long long)n * A1N + (cq * LN_CQ) * P1 * P1 + v];
      }
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const int v = t + h * LN_T;
        if (v < A2N) {
          const int o = v >> 4, i = (v >> 2) & 3, j = v & 3;
#pragma unroll
          for (int d = 0; d < 4; ++d) {
            const int pq = (2 * i + (d >> 1)) * 8 + 2 * j + (d & 1);
            s_A[pq * LN_AP + o] = d == ev[h] ? dv[h] : 0.0f;
          }
        }
      }
      if (t < 64 * (LN_AP - C2)) s_A[(t >> 1) * LN_AP + C2 + (t & 1)] = 0.0f;  // pad columns
      s_x[t] = xv0;
      if (t + LN_T < IN * IN) s_x[t + LN_T] = xv1;
      s_c1[t] = kc[0];
      if (t + LN_T < LN_CQ * P1 * P1) s_c1[t + LN_T] = kc[1];
    }
    __syncthreads();
    LN_STAMP(1);
    {
      f32x4 acc[4];
#pragma unroll
      for (int mt = 0; mt < 4; ++mt) acc[mt] = f32x4{0.0f, 0.0f, 0.0f, 0.0f};
#pragma unroll
      for (int s2 = 0; s2 < 13; ++s2) {
        const bool kv = 4 * s2 + g < C2 && bcol < LN_SN;
        const float bq = kv ? fb[s2] : 0.0f;
#pragma unroll
        for (int mt = 0; mt < 4; ++mt) {
          const float a = s_A[(mt * 16 + li) * LN_AP + 4 * s2 + g];
          acc[mt] = __builtin_amdgcn_mfma_f32_16x16x4f32(a, bq, acc[mt], 0, 0, 0);
        }
      }
#pragma unroll
      for (int mt = 0; mt < 4; ++mt)
#pragma unroll
        for (int e = 0; e < 4; ++e) s_S[(mt * 16 + 4 * g + e) * LN_SP + bcol] = acc[mt][e];
    }
    __syncthreads();
    // col2im + relu mask: dp1[c][y][x] for the group's 5 channels
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int u = t + h * LN_T;
      if (u < LN_CQ * P1 * P1) {
        const int cc = u / (P1 * P1), pos = u - cc * P1 * P1, yy = pos / P1, xq = pos - yy * P1;
        const float av = a1[(long long)n * A1N + (cq * LN_CQ + cc) * P1 * P1 + pos];
        float s = 0.0f;
#pragma unroll
        for (int ky = 0; ky < KS; ++ky)
#pragma unroll
          for (int kx = 0; kx < KS; ++kx) {
            const int p = yy - ky, q = xq - kx;
            const bool ok = (unsigned)p < 8u && (unsigned)q < 8u;
            const float v = s_S[(ok ? p * 8 + q : 0) * LN_SP + cc * TAPS + ky * KS + kx];
            s += ok ? v : 0.0f;
          }
        s_dp1[u] = av > 0.0f ? s : 0.0f;
      }
    }
    __syncthreads();
    LN_STAMP(2);
    // the block's dW_conv1 (125) / db_conv1 (5) partial: 3 position slices per entry, combined in
    // slice order
    if (t < 3 * LN_W1Q) {
      const int u = t % LN_W1Q, sl = t / LN_W1Q;
      float s = 0.0f;
      if (u < LN_SN) {
        const int cc = u / TAPS, k = u - cc * TAPS, ky = k / KS, kx = k - ky * KS;
        for (int pos = sl * 48; pos < sl * 48 + 48; ++pos) {
          const int e = s_c1[cc * P1 * P1 + pos];
          const int oy = 2 * (pos / P1) + (e >> 1), ox = 2 * (pos % P1) + (e & 1);
          s = fmaf(s_dp1[cc * P1 * P1 + pos], s_x[(oy + ky) * IN + ox + kx], s);
        }
      } else {
        const int cc = u - LN_SN;
        for (int pos = sl * 48; pos < sl * 48 + 48; ++pos) s += s_dp1[cc * P1 * P1 + pos];
      }
      s_red[sl * LN_W1Q + u] = s;
    }
    __syncthreads();
    if (t < LN_W1Q)
      sc1_store(part1 + ((long long)cq * B + n) * LN_W1Q + t,
                s_red[t] + s_red[LN_W1Q + t] + s_red[2 * LN_W1Q + t]);
    // first level: per channel group, the last of each group of 16 images sums them in order
    const int gi = n / LN_GA, n0 = gi * LN_GA, gn = min(LN_GA, B - n0);
    LN_STAMP(3);
    if (!ln_ticket(cnt + cq * ngi + gi, gn, &s_flag)) return;
    LN_STAMP(4);
    if (t < LN_W1Q) {
      float v[LN_GA];
#pragma unroll
      for (int i = 0; i < LN_GA; ++i)
        v[i] = sc1_load(part1 + ((long long)cq * B + n0 + min(i, gn - 1)) * LN_W1Q + t);
      LN_FENCE_SCHED();
      float s = 0.0f;
#pragma unroll
      for (int i = 0; i < LN_GA; ++i)
        if (i < gn) s += v[i];
      sc1_store(part1g + ((long long)cq * ngi + gi) * LN_W1Q + t, s);
    }
    // second level: the last image group of the channel group sums the groups in order
    LN_STAMP(5);
    if (!ln_ticket(cnt + 4 * ngi + cq, ngi, &s_flag)) return;
    LN_STAMP(6);
    if (t < LN_W1Q) {
      float s = 0.0f;
      for (int g0 = 0; g0 < ngi; g0 += 8) {
        float v[8];
#pragma unroll
        for (int i = 0; i < 8; ++i)
          v[i] = sc1_load(part1g + ((long long)cq * ngi + min(g0 + i, ngi - 1)) * LN_W1Q + t);
        LN_FENCE_SCHED();
#pragma unroll
        for (int i = 0; i < 8; ++i)
          if (g0 + i < ngi) s += v[i];
      }
      if (t < LN_SN) dw1[cq * LN_SN + t] = s;  // [20][1][5][5]: channel 5 cq + t / 25
      else db1[cq * LN_CQ + t - LN_SN] = s;
    }
    LN_STAMP(7);
    return;
  }
  // dW_conv2[o][c][ky][kx] = sum_n sum_windows dp2[n][o][win] * a1[n][c][p + ky][q + kx]
  const int bi = bid - na;
  const int og = bi % NOG, ig = bi / NOG, ngr = (B + IG - 1) / IG;
  float* s_a1 = smem;  // [IG][2880]
  const int n0 = ig * IG, nimg = min(IG, B - n0);
  ln_stage<IG * A1N / 4>(s_a1, a1 + (long long)n0 * A1N, nimg * A1N / 4, t);
  // this block's (image, out channel, window) entries, 80 per image: lane l of every wave holds
  // entries l (and 64 + l): dp2 and the a1 offset p * 12 + q of the window's maximum; the loop
  // below takes them with v_readlane (no LDS traffic for block-uniform operands)
  // this block's (image, out channel, window) entries, 80 per image, in LDS: dp2 and the a1
  // offset p * 12 + q of the window's maximum (read back as block-wide broadcasts)
  float* s_ed = s_a1 + IG * A1N;                                // [IG][80]
  int* s_eo = reinterpret_cast<int*>(s_ed + IG * OG * 16);      // [IG][80]
  if (t < IG * OG * 16) {
    const int nn = t / (OG * 16), v = t - nn * OG * 16, oo = v >> 4, wi = v & 15;
    const long long gi = (long long)(n0 + min(nn, nimg - 1)) * A2N + (og * OG + oo) * 16 + wi;
    const int e = code2[gi];
    const float d = dp2[gi];
    s_ed[t] = nn < nimg ? d : 0.0f;
    s_eo[t] = (2 * (wi >> 2) + (e >> 1)) * P1 + 2 * (wi & 3) + (e & 1);
  }
  __syncthreads();
  LN_STAMP(1);
  if (t < W2P - 1) {
    const int c = t / TAPS, k = t - c * TAPS, ky = k / KS, kx = k - ky * KS;
    const int tap = c * P1 * P1 + ky * P1 + kx;
    float s[OG];
#pragma unroll
    for (int oo = 0; oo < OG; ++oo) s[oo] = 0.0f;
    for (int nn = 0; nn < IG; ++nn) {
      const float* ai = s_a1 + nn * A1N + tap;
#pragma unroll
      for (int oo = 0; oo < OG; ++oo) {
        // the channel's 16 entries (4 broadcast b128 reads each), its 16 a1 reads issued together
        const f32x4* dq = reinterpret_cast<const f32x4*>(s_ed + (nn * OG + oo) * 16);
        const int4* oq = reinterpret_cast<const int4*>(s_eo + (nn * OG + oo) * 16);
        f32x4 dv[4];
        int4 ov[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          dv[i] = dq[i];
          ov[i] = oq[i];
        }
        float av[16];
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          av[4 * i + 0] = ai[ov[i].x];
          av[4 * i + 1] = ai[ov[i].y];
          av[4 * i + 2] = ai[ov[i].z];
          av[4 * i + 3] = ai[ov[i].w];
        }
        LN_FENCE_SCHED();
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int jj = 0; jj < 4; ++jj) s[oo] = fmaf(dv[i][jj], av[4 * i + jj], s[oo]);
      }
    }
#pragma unroll
    for (int oo = 0; oo < OG; ++oo)
      sc1_store(part2 + ((long long)ig * C2 + og * OG + oo) * W2P + t, s[oo]);
  } else if (t < W2P - 1 + OG) {  // db_conv2 partials: thread 500 + oo sums channel oo's entries
    const int oo = t - (W2P - 1);
    float s = 0.0f;
    for (int nn = 0; nn < IG; ++nn)
#pragma unroll
      for (int wi = 0; wi < 16; ++wi) s += s_ed[(nn * OG + oo) * 16 + wi];
    sc1_store(part2 + ((long long)ig * C2 + og * OG + oo) * W2P + (W2P - 1), s);
  }
  if (prof) __syncthreads();  // probes: stamp 2 = the whole block's compute done
  LN_STAMP(2);
  if (!ln_ticket(cnt + 4 * ngi + 4 + og, ngr, &s_flag)) return;
  LN_STAMP(3);
  if (t < W2P) {
    float s[OG];
#pragma unroll
    for (int oo = 0; oo < OG; ++oo) s[oo] = 0.0f;
    for (int g0 = 0; g0 < ngr; g0 += 16) {  // 16 image groups x 5 channels of loads in flight
      float v[OG][16];
#pragma unroll
      for (int oo = 0; oo < OG; ++oo)
#pragma unroll
        for (int i = 0; i < 16; ++i)
          v[oo][i] = sc1_load(part2 + ((long long)min(g0 + i, ngr - 1) * C2 + og * OG + oo) * W2P + t);
      LN_FENCE_SCHED();
#pragma unroll
      for (int oo = 0; oo < OG; ++oo)
#pragma unroll
        for (int i = 0; i < 16; ++i)
          if (g0 + i < ngr) s[oo] += v[oo][i];
    }
#pragma unroll
    for (int oo = 0; oo < OG; ++oo) {
      const int o = og * OG + oo;
      if (t < W2P - 1) dw2[o * (C1 * TAPS) + t] = s[oo];
      else db2[o] = s[oo];
    }
  }
  LN_STAMP(4);
#undef LN_STAMP
}

long long* g_ln_prof = nullptr;  // probes: per-block phase stamps of k_ln_conv_bwd (8 per block)

void ln_check(int B, int K) {
  if (B <= 0 || B > (1 << 20) || K <= 0 || K > MAXK)
    throw std::runtime_error("ewdml lenet: needs 0 < batch and 0 < classes <= 16");
}
void ln_aligned(uintptr_t p, const char* what) {
  if (p % 16)
    throw std::runtime_error(std::string("ewdml lenet: ") + what + " is not 16-byte aligned");
}

}  // namespace

// Persistent workspace (floats): fc2 logit partials [32][B16][16], dW_conv1 partials [4][B][130]
// and their image-group sums [4][ceil(B/16)][130], dW_conv2 partials [ceil(B/4)][50][501]; ticket
// ints (zeroed once, left zero by the kernels): fc row tiles + loss, dW_conv1 image groups per
// channel group + one per channel group, dW_conv2 channel groups
static long long ln_ngi(int B) { return (B + LN_GA - 1) / LN_GA; }
long long ew_lenet_ws_floats(int B) {
  const long long Bp = (B + FT - 1) / FT * FT;
  return (long long)F1T * Bp * MAXK + 4LL * (B + ln_ngi(B)) * LN_W1Q +
         (long long)((B + IG - 1) / IG) * C2 * W2P;
}
int ew_lenet_counters(int B) { return (int)((B + FT - 1) / FT + 1 + 4 * ln_ngi(B) + 4 + NOG); }

void ew_lenet_fwd(uintptr_t x, uintptr_t w1, uintptr_t b1, uintptr_t w2, uintptr_t b2,
                  uintptr_t wf1, uintptr_t bf1, uintptr_t wf2, uintptr_t bf2, uintptr_t y, int B,
                  int K, uintptr_t a1, uintptr_t code1, uintptr_t a2, uintptr_t code2,
                  uintptr_t h1, uintptr_t logits, uintptr_t dlogits, uintptr_t dh1,
                  uintptr_t lossrow, uintptr_t loss, uintptr_t ws, long long ws_floats,
                  uintptr_t cnt, int cnt_ints, uintptr_t stream, uintptr_t bsrc,
                  uintptr_t blabels, uintptr_t bperm, long long bperm_len, uintptr_t bstate,
                  uintptr_t bdone, float bmean, float binv_std) {
  ln_check(B, K);
  if (ws_floats < ew_lenet_ws_floats(B) || cnt_ints < ew_lenet_counters(B))
    throw std::runtime_error("ewdml lenet: workspace too small");
  // bsrc: form the batch in the conv launch (LnBatch) into x and y
  if (bsrc && (!blabels || !bperm || !bstate || !bdone || bperm_len < B || (bsrc & 3)))
    throw std::runtime_error("ewdml lenet: bad batch source");
  const LnBatch bt{reinterpret_cast<const uint8_t*>(bsrc),
                   reinterpret_cast<const long long*>(blabels),
                   reinterpret_cast<const long long*>(bperm), reinterpret_cast<long long*>(bstate),
                   reinterpret_cast<int*>(bdone), bperm_len, bmean, binv_std,
                   reinterpret_cast<long long*>(y)};
  ln_aligned(x, "x");
  ln_aligned(w1, "conv1 weight");
  ln_aligned(w2, "conv2 weight");
  ln_aligned(a2, "a2");
  ln_aligned(wf1, "fc1 weight");
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  hipLaunchKernelGGL(k_ln_conv_fwd, dim3(4, B), dim3(LN_CT), 0, s,
                     reinterpret_cast<const float*>(x), reinterpret_cast<const float*>(w1),
                     reinterpret_cast<const float*>(b1), reinterpret_cast<const float*>(w2),
                     reinterpret_cast<const float*>(b2), reinterpret_cast<float*>(a1),
                     reinterpret_cast<uint8_t*>(code1), reinterpret_cast<float*>(a2),
                     reinterpret_cast<uint8_t*>(code2), bt);
  EW_CHECK_LAUNCH();
  const int nrt = (B + FT - 1) / FT;
  hipLaunchKernelGGL(k_ln_fc_fwd, dim3(F1T, nrt), dim3(LN_FT), 0, s,
                     reinterpret_cast<const float*>(a2), reinterpret_cast<const float*>(wf1),
                     reinterpret_cast<const float*>(bf1), reinterpret_cast<const float*>(wf2),
                     reinterpret_cast<const float*>(bf2), reinterpret_cast<const long long*>(y),
                     B, K, reinterpret_cast<float*>(h1), reinterpret_cast<float*>(ws),
                     reinterpret_cast<int*>(cnt), reinterpret_cast<float*>(lossrow),
                     reinterpret_cast<float*>(logits), reinterpret_cast<float*>(dlogits),
                     reinterpret_cast<float*>(dh1), reinterpret_cast<float*>(loss));
  EW_CHECK_LAUNCH();
}

void ew_lenet_bwd(uintptr_t x, uintptr_t w2, uintptr_t wf1, uintptr_t a1, uintptr_t code1,
                  uintptr_t a2, uintptr_t code2, uintptr_t h1, uintptr_t dlogits, uintptr_t dh1,
                  uintptr_t gscale, int B, int K, uintptr_t dp2, uintptr_t dw1, uintptr_t db1,
                  uintptr_t dw2, uintptr_t db2, uintptr_t dwf1, uintptr_t dbf1, uintptr_t dwf2,
                  uintptr_t dbf2, uintptr_t ws, long long ws_floats, uintptr_t cnt, int cnt_ints,
                  uintptr_t stream) {
  ln_check(B, K);
  if (ws_floats < ew_lenet_ws_floats(B) || cnt_ints < ew_lenet_counters(B))
    throw std::runtime_error("ewdml lenet: workspace too small");
  ln_aligned(w2, "conv2 weight");
  ln_aligned(a1, "a1");
  ln_aligned(dh1, "dh1");
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  const int nrt = (B + FT - 1) / FT;
  const int nda = nrt * A2T, nwt = (LN_WT + 3) / 4;
  hipLaunchKernelGGL(k_ln_fc_bwd, dim3(nda + nwt), dim3(LN_FT), 0, s,
                     reinterpret_cast<const float*>(a2), reinterpret_cast<const float*>(h1),
                     reinterpret_cast<const float*>(dlogits), reinterpret_cast<const float*>(dh1),
                     reinterpret_cast<const float*>(wf1), reinterpret_cast<const float*>(gscale),
                     B, K, nda, reinterpret_cast<float*>(dp2), reinterpret_cast<float*>(dwf1),
                     reinterpret_cast<float*>(dbf1), reinterpret_cast<float*>(dwf2),
                     reinterpret_cast<float*>(dbf2));
  EW_CHECK_LAUNCH();
  const long long Bp = (long long)nrt * FT;
  float* part1 = reinterpret_cast<float*>(ws) + (long long)F1T * Bp * MAXK;
  float* part1g = part1 + 4LL * B * LN_W1Q;
  float* part2 = part1g + 4 * ln_ngi(B) * LN_W1Q;
  const int ngr = (B + IG - 1) / IG;
  // EWDML_LN_PART=1 / 2: launch only the d(a1) + dW_conv1 blocks / only the dW_conv2 blocks
  // (timing probes; the other part's gradients are left unwritten)
  static const int part = [] {
    const char* e = std::getenv("EWDML_LN_PART");
    return e ? std::atoi(e) : 0;
  }();
  const int nblk = part == 1 ? 4 * B : part == 2 ? NOG * ngr : 4 * B + NOG * ngr;
  const int boff = part == 2 ? 4 * B : 0;
  hipLaunchKernelGGL(k_ln_conv_bwd, dim3(nblk), dim3(LN_T), 0, s,
                     reinterpret_cast<const float*>(x), reinterpret_cast<const float*>(w2),
                     reinterpret_cast<const float*>(a1), reinterpret_cast<const uint8_t*>(code1),
                     reinterpret_cast<const uint8_t*>(code2), reinterpret_cast<const float*>(dp2),
                     B, part1, part1g, part2, reinterpret_cast<int*>(cnt) + nrt + 1,
                     reinterpret_cast<float*>(dw1), reinterpret_cast<float*>(db1),
                     reinterpret_cast<float*>(dw2), reinterpret_cast<float*>(db2), boff,
                     g_ln_prof);
  EW_CHECK_LAUNCH();
}

void ew_lenet_set_prof(uintptr_t buf) { g_ln_prof = reinterpret_cast<long long*>(buf); }
