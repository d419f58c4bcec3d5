// Classifier-head Linear layers (VGG: Dropout, Linear, ReLU, Dropout, Linear, ReLU, Linear) as
// small MFMA GEMMs with the elementwise work folded into their operand loads and epilogues.
//
// Why: at batch 128 every head GEMM is ~128 x 512 x 512 -- a few microseconds of work each -- and
// PyTorch (hipBLASLt + separate ReLU / dropout / bias-gradient kernels) runs the head as 22
// launches per step (~114 us, profiles/vgg11_*: more than 10% of the VGG-11 step).  Here one
// kernel per Linear and direction (6 per step):
//   forward   z = drop_out(act(drop_in(x) W^T + b))     drop_in applied to the A operand on load,
//             bias / ReLU / dropout in the epilogue (pre-activation y stored for the backward)
//   backward  dy = bf16(dz * act'(y) * keep_out / (1 - p_out)) recomputed on load, and one grid
//             of two block roles: dW = dy^T drop_in(x) (+ db = sum over rows of dy) and
//             dx = (dy W) * keep_in / (1 - p_in)
// Masks come from the counter hash of ops/csrc/nn.hip (key from a per-layer device counter,
// element index r * width + c); the backward's last block advances the counters (arrival
// ticket, no fences: every block read them before arriving).
//
// Element types: bf16 (v_mfma_f32_16x16x32_bf16, one MFMA per 32-deep step) or fp32 (the reference
// precision: eight v_mfma_f32_16x16x4_f32 per 32-deep step, MFMA e taking element e of each lane's
// 8 consecutive k -- the same k permutation in both operands; no rounding of intermediates).
//
// Tiles: one 16 x 16 output tile per block, the reduction split over
// the block's 4 waves (every wave issues all its loads before its first MFMA; partial tiles summed
// through LDS): a 128 x 512 x 512 GEMM is 256 blocks with ~4 loads in flight per lane instead of
// a few long dependent k-loops.  Operands go straight from L2 into the fragment registers (each
// fragment element is used by one lane; the whole head's operands are ~1.5 MB).
#include "common.h"
#include "ewdml_ops.h"

namespace {

typedef __bf16 hd_bf16x8 __attribute__((ext_vector_type(8)));
typedef float hd_f32x4 __attribute__((ext_vector_type(4)));
typedef unsigned short hd_u16x8 __attribute__((ext_vector_type(8)));

// device counter: ctr[0] = mask step, ctr[HD_TICKET ...] = the backward's arrival tickets
// (EW_TICKET_INTS), HD_CTR_INTS ints in all
constexpr int HD_TICKET = 32;
struct HdDrop {
  const int* ctr;
  uint32_t salt;
  float p;  // 0: no dropout
};

__device__ __forceinline__ uint32_t hd_key(const HdDrop& d) {
  return d.p > 0.0f ? ew_mix32((uint32_t)d.ctr[0] * 0x9E3779B9u + d.salt) : 0u;
}
__device__ __forceinline__ float hd_scale(const HdDrop& d) {
  return d.p > 0.0f ? 1.0f / (1.0f - d.p) : 1.0f;
}
// keep * 1/(1-p) of element i (the forward's mask)
__device__ __forceinline__ float hd_mask(uint32_t i, uint32_t key, float p, float scale) {
  return ew_uniform(i, key) >= p ? scale : 0.0f;
}
__device__ __forceinline__ float hd_f(uint16_t v) { return ew_bf16f(v); }
// torch ReLU semantics (NaN propagates), as the NHWC BN kernels
__device__ __forceinline__ float hd_relu(float v) { return (v > 0.0f || v != v) ? v : 0.0f; }
__device__ __forceinline__ bool hd_relu_pass(float v) { return !(v <= 0.0f); }
__device__ __forceinline__ float hd_rnd(float v) { return hd_f(ew_f2bf(v)); }

// Element-type traits: 8-wide operand vector, load / store / rounding, one 32-deep MFMA step
typedef float hd_f32x8 __attribute__((ext_vector_type(8)));
template <typename T>
struct HdT;
template <>
struct HdT<uint16_t> {
  typedef hd_u16x8 v8;
  __device__ static __forceinline__ float f(uint16_t v) { return hd_f(v); }
  __device__ static __forceinline__ uint16_t st(float v) { return ew_f2bf(v); }
  __device__ static __forceinline__ float rnd(float v) { return hd_rnd(v); }
  __device__ static __forceinline__ hd_f32x4 mma(const v8& a, const v8& b, hd_f32x4 acc) {
    return __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(hd_bf16x8, a),
                                                   __builtin_bit_cast(hd_bf16x8, b), acc, 0, 0, 0);
  }
};
template <>
struct HdT<float> {
  typedef hd_f32x8 v8;
  __device__ static __forceinline__ float f(float v) { return v; }
  __device__ static __forceinline__ float st(float v) { return v; }
  __device__ static __forceinline__ float rnd(float v) { return v; }
  __device__ static __forceinline__ hd_f32x4 mma(const v8& a, const v8& b, hd_f32x4 acc) {
#pragma unroll
    for (int e = 0; e < 8; ++e) acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a[e], b[e], acc, 0, 0, 0);
    return acc;
  }
};

// Sum the 4 waves' 16 x 16 accumulators (each wave took a quarter of the reduction) into wave 0's,
// in a fixed order.
__device__ __forceinline__ void hd_wave_reduce(hd_f32x4& acc, float* red, int wv, int lane) {
#pragma unroll
  for (int q = 0; q < 4; ++q) red[(wv * 4 + q) * 64 + lane] = acc[q];
  __syncthreads();
  if (wv == 0) {
#pragma unroll
    for (int q = 0; q < 4; ++q)
      acc[q] = (red[q * 64 + lane] + red[(4 + q) * 64 + lane]) +
               (red[(8 + q) * 64 + lane] + red[(12 + q) * 64 + lane]);
  }
}

// Cross-entropy riding in the last Linear's forward (N <= 16 classes: a block's tile holds whole
// rows): per row log-sum-exp, loss and d(loss)/d(logits) for an upstream 1 (k_ce_fwd's expressions,
// bit for bit), the per-row losses summed by the grid's last block in k_ce_fwd's order.
template <typename T>
struct HdCe {
  const long long* y;  // labels; null: no cross-entropy
  float* lossrow;      // [B] scratch
  float* loss;         // mean loss
  float* lse;          // [B]
  T* dlog;             // [B][N] (nullable)
  int* tick;           // zeroed grid ticket (left zeroed)
};

// wave 0 of a forward block (16 rows x N <= 16 logits in zq, lane = column li of row group
// lane >> 4); the grid's last block (a wave-level ticket: the other waves have exited) sums
// the row losses.
template <typename T>
__device__ __forceinline__ void hd_ce_tail(const HdCe<T>& ce, const float (&zq)[4], int B, int N,
                                           int lane, int n) {
  const float g1 = 1.0f / (float)B;
  const int base = lane & ~15;
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const int rr = blockIdx.x * 16 + 4 * (lane >> 4) + q;
    const bool valid = rr < B;
    const float xv = zq[q];
    float m = -INFINITY;
    for (int k = 0; k < N; ++k) m = fmaxf(m, __shfl(xv, base + k, 64));
    float sum = 0.0f;
    for (int k = 0; k < N; ++k) sum += expf(__shfl(xv, base + k, 64) - m);
    const float l = m + logf(sum);
    const long long t = valid ? ce.y[rr] : -1;
    const bool tin = t >= 0 && t < N;
    const float xt = __shfl(xv, base + (tin ? (int)t : 0), 64);
    if (!valid) continue;
    if (n < N && ce.dlog) {
      float v = expf(xv - l);
      if ((long long)n == t) v -= 1.0f;
      v *= g1;
      ce.dlog[(long long)rr * N + n] = HdT<T>::st(v);
    }
    if ((lane & 15) == 0) {
      ce.lse[rr] = l;
      // write-through: the grid's last block reads the row losses in this launch
      __hip_atomic_store(ce.lossrow + rr, l - (tin ? xt : 0.0f), __ATOMIC_RELAXED,
                         __HIP_MEMORY_SCOPE_AGENT);
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  int last = 0;
  if (lane == 0) {
    const int G = (int)(gridDim.x * gridDim.y);
    last = __hip_atomic_fetch_add(ce.tick, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == G - 1;
    if (last) __hip_atomic_store(ce.tick, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  if (!__shfl(last, 0, 64)) return;
  // k_ce_fwd's sum: its wave w (of 16) lane l held rows w * 64 + l + 1024 j; butterfly per wave,
  // then the 16 wave sums in order
  float tot = 0.0f;
  for (int w = 0; w < 16; ++w) {
    float a = 0.0f;
    for (int r = w * 64 + lane; r < B; r += 1024)
      a += __hip_atomic_load(ce.lossrow + r, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) a += __shfl_xor(a, o, 64);
    tot += __shfl(a, 0, 64);
  }
  if (lane == 0) *ce.loss = tot / (float)B;
}

// ---- forward: z[B][N] = drop_out(act(drop_in(x) w^T + b)), y = pre-activation (optional) ----
// Block: one 16 x 16 output tile; wave v takes the k-steps v, v + 4, ... (all its loads issued
// before the first MFMA), the 4 partial tiles are summed through LDS.
template <typename T, bool RELU>
__global__ __launch_bounds__(EW_BLOCK) void k_head_fwd(const T* __restrict__ x,
                                                       const T* __restrict__ w,
                                                       const T* __restrict__ b,
                                                       T* __restrict__ z, T* __restrict__ y, int B,
                                                       int N, int K, HdDrop din, HdDrop dout,
                                                       HdCe<T> ce) {
  using H = HdT<T>;
  typedef typename H::v8 v8;
  __shared__ float red[16 * 64];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6, li = lane & 15;
  const int r = blockIdx.x * 16 + li;  // A row (batch row) of this lane
  const int n = blockIdx.y * 16 + li;  // B row (output feature) of this lane
  const int kq = 8 * (lane >> 4);
  const bool rok = r < B, nok = n < N;
  const T* xp = x + (long long)(rok ? r : 0) * K + kq;
  const T* wp = w + (long long)(nok ? n : 0) * K + kq;
  const uint32_t kin = hd_key(din);
  const float sin = hd_scale(din);
  const v8 zero = {};
  const int nsteps = K / 32;
  hd_f32x4 acc = {0.0f, 0.0f, 0.0f, 0.0f};
  for (int s0 = wv; s0 < nsteps; s0 += 16) {  // up to 4 steps of this wave in flight
    v8 av[4], bv[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int s = s0 + 4 * u;
      const bool ok = s < nsteps;
      av[u] = (ok && rok) ? *reinterpret_cast<const v8*>(xp + 32 * s) : zero;
      bv[u] = (ok && nok) ? *reinterpret_cast<const v8*>(wp + 32 * s) : zero;
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int s = s0 + 4 * u;
      if (s >= nsteps) break;
      v8 a = av[u];
      if (din.p > 0.0f) {  // the head's input Dropout, on the A operand (rounded like a stored z)
        const uint32_t i0 = (uint32_t)r * (uint32_t)K + (uint32_t)(32 * s + kq);
#pragma unroll
        for (int e = 0; e < 8; ++e)
          a[e] = H::st(H::f(a[e]) * hd_mask(i0 + e, kin, din.p, sin));
      }
      acc = H::mma(a, bv[u], acc);
    }
  }
  hd_wave_reduce(acc, red, wv, lane);
  // C/D layout: column li (output feature), rows 4 (lane >> 4) + q (batch rows)
  if (wv != 0) return;
  const float bias = (b && nok) ? H::f(b[n]) : 0.0f;
  const uint32_t kout = hd_key(dout);
  const float sout = hd_scale(dout);
  float zq[4];  // the stored outputs (the cross-entropy reads them as k_ce_fwd reads the logits)
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const int rr = blockIdx.x * 16 + 4 * (lane >> 4) + q;
    const long long o = (long long)rr * N + n;
    const T yb = H::st(acc[q] + bias);  // the GEMM's output (bias in fp32)
    float v = H::f(yb);
    if (RELU) v = hd_relu(v);
    if (dout.p > 0.0f) v = v * hd_mask((uint32_t)o, kout, dout.p, sout);
    zq[q] = H::f(H::st(v));
    if (rr >= B || !nok) continue;
    if (y) y[o] = yb;
    z[o] = H::st(v);
  }
  if constexpr (!RELU) {
    if (ce.y) hd_ce_tail<T>(ce, zq, B, N, lane, n);
  }
}

// dy = bf16(dz * act'(y) * keep_out / (1 - p_out)) of element o (the value the GEMMs consume)
template <typename T, bool RELU>
__device__ __forceinline__ float hd_dyv(T dzv, T yv, uint32_t o, uint32_t kout,
                                        const HdDrop& dout, float sout) {
  float v = HdT<T>::f(dzv);
  if (RELU && !hd_relu_pass(HdT<T>::f(yv))) v = 0.0f;
  if (dout.p > 0.0f) v = v * hd_mask(o, kout, dout.p, sout);
  return HdT<T>::rnd(v);
}

// The backward statistics and finalisation of the BatchNorm + ReLU + 2x2 max pool layer (2x2 maps
// pooled to 1x1: VGG's last conv block) whose flattened output is this Linear's input, riding in
// the input-gradient blocks: each channel tile's last row tile (a ticket per tile) sums, for its
// 16 channels over all rows, dz = dx at the pool's argmax where its ReLU passed, dz * (h - mean)
// and h - mean (the three sums of nn.hip k_bn_bwd_stats), then forms k_bn_bwd_finalize's outputs.
// fp32 only.
struct HdBnB {
  const float* h;        // [B][2][2][K] BN input (null: none)
  const uint8_t* code;   // [B][K] pool window codes
  const float* stats;    // [4][K] mean, invstd, scale, shift
  float* coef;           // [2][K]
  float* dgamma;         // nullable
  float* dbeta;          // nullable
  void* dcbias;          // nullable
  int cb_bf16;
  int* tick;             // [K / 16] zeroed tickets (left zeroed)
};

__device__ __forceinline__ void hd_bn_tile(const HdBnB& bn, const float* dx, int B, int K, int tk,
                                           double* red) {
  const int t = threadIdx.x, li = t & 15, sl = t >> 4, lane = t & 63, wv = t >> 6;
  const int c = tk * 16 + li;
  const bool cok = c < K;
  const int cc = cok ? c : K - 1;
  const float mean = bn.stats[cc], sc = bn.stats[2 * K + cc], sh = bn.stats[3 * K + cc];
  float s1 = 0.0f, s2 = 0.0f, s3 = 0.0f;
  for (int r0 = sl; r0 < B; r0 += 16 * 4) {  // 4 rows in flight per thread
    float d[4], x[4][4];
    uint8_t k[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int r = min(r0 + 16 * u, B - 1);
      d[u] = __hip_atomic_load(const_cast<float*>(dx) + (long long)r * K + cc, __ATOMIC_RELAXED,
                               __HIP_MEMORY_SCOPE_AGENT);
      k[u] = bn.code[(long long)r * K + cc];
#pragma unroll
      for (int q = 0; q < 4; ++q) x[u][q] = bn.h[((long long)r * 4 + q) * K + cc];
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      if (r0 + 16 * u >= B) continue;
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const float dz = (k[u] == q && hd_relu_pass(x[u][q] * sc + sh)) ? d[u] : 0.0f;
        const float xc = x[u][q] - mean;
        s1 += dz;
        s2 += dz * xc;
        s3 += xc;
      }
    }
  }
  double a[3] = {s1, s2, s3};
#pragma unroll
  for (int i = 0; i < 3; ++i) {
    a[i] += __shfl_xor(a[i], 16, 64);
    a[i] += __shfl_xor(a[i], 32, 64);
    if (lane < 16) red[(i * 4 + wv) * 16 + lane] = a[i];
  }
  __syncthreads();
  if (t >= 16 || !cok) return;
  double sum[3];
#pragma unroll
  for (int i = 0; i < 3; ++i)
    sum[i] = (red[(i * 4) * 16 + t] + red[(i * 4 + 1) * 16 + t]) +
             (red[(i * 4 + 2) * 16 + t] + red[(i * 4 + 3) * 16 + t]);
  const double M = 4.0 * B;
  const double invstd = bn.stats[K + c], scale = sc;
  const double db = sum[0], dg = sum[1] * invstd;
  const double e = -scale * invstd * dg / M;
  bn.coef[c] = (float)e;
  bn.coef[K + c] = (float)(-scale * db / M);
  if (bn.dgamma) bn.dgamma[c] = (float)dg;
  if (bn.dbeta) bn.dbeta[c] = (float)db;
  if (bn.dcbias) {
    const float v = (float)(e * sum[2]);
    if (bn.cb_bf16) reinterpret_cast<uint16_t*>(bn.dcbias)[c] = ew_f2bf(v);
    else reinterpret_cast<float*>(bn.dcbias)[c] = v;
  }
}

// ---- backward: blocks [0, nbw) 16 x 16 weight-gradient tiles (+ bias gradient), the rest
// 16 x 16 input-gradient tiles; in both, wave v takes a quarter of the reduction ----
template <typename T, bool RELU>
__global__ __launch_bounds__(EW_BLOCK) void k_head_bwd(
    const T* __restrict__ dz, const T* __restrict__ y, const T* __restrict__ x,
    const T* __restrict__ w, T* __restrict__ dx, T* __restrict__ dw, void* __restrict__ db,
    int db_bf16, int B, int N, int K, HdDrop dout, HdDrop din, int nbw, int* __restrict__ adv0,
    int* __restrict__ adv1, HdBnB bn) {
  using H = HdT<T>;
  typedef typename H::v8 v8;
  __shared__ float red[16 * 64];
  __shared__ float dbr[4][16];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int g = lane >> 4, li = lane & 15;
  const uint32_t kout = hd_key(dout), kin = hd_key(din);
  const float sout = hd_scale(dout), sin = hd_scale(din);
  hd_f32x4 acc = {0.0f, 0.0f, 0.0f, 0.0f};
  const int n16 = (N + 15) / 16, b16 = (B + 15) / 16;
  if ((int)blockIdx.x < nbw) {
    // dW[n][k] = sum_r dy[r][n] x~[r][k]: A = dy^T (rows n), B = x~^T (rows k), reduction over
    // the batch rows in 32-row steps; wave v: steps v, v + 4, ...
    const int tn = blockIdx.x % n16, tk = blockIdx.x / n16;
    const int n = tn * 16 + li, k = tk * 16 + li;
    const bool nok = n < N, kok = k < K;
    const int nc = nok ? n : 0, kc = kok ? k : 0;
    float dbs = 0.0f;
    for (int r0 = 32 * wv; r0 < B; r0 += 128) {
      T dv[8], yv[8], xv[8];
#pragma unroll
      for (int e = 0; e < 8; ++e) {  // clamped rows: loads issued unconditionally, masked below
        const int rc = min(r0 + 8 * g + e, B - 1);
        dv[e] = dz[(long long)rc * N + nc];
        yv[e] = RELU ? y[(long long)rc * N + nc] : (T)0;
        xv[e] = x[(long long)rc * K + kc];
      }
      v8 a, bb;
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const int rr = r0 + 8 * g + e;
        const bool ok = rr < B;
        const float d = (ok && nok)
                            ? hd_dyv<T, RELU>(dv[e], yv[e],
                                              (uint32_t)rr * (uint32_t)N + (uint32_t)n, kout,
                                              dout, sout)
                            : 0.0f;
        dbs += d;
        a[e] = H::st(d);
        float xf = 0.0f;
        if (ok && kok) {
          xf = H::f(xv[e]);
          if (din.p > 0.0f)
            xf = H::rnd(xf * hd_mask((uint32_t)rr * (uint32_t)K + (uint32_t)k, kin, din.p, sin));
        }
        bb[e] = H::st(xf);
      }
      acc = H::mma(a, bb, acc);
    }
    // bias gradient (tiles of column block 0): the A operand's sums over the rows
    dbs += __shfl_xor(dbs, 16, 64);
    dbs += __shfl_xor(dbs, 32, 64);
    if (g == 0) dbr[wv][li] = dbs;
    hd_wave_reduce(acc, red, wv, lane);  // (its barrier also publishes dbr)
    if (wv == 0) {
      // C/D: column li -> k, rows 4 g + q -> n
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int nn = tn * 16 + 4 * g + q;
        if (nn < N && kok) dw[(long long)nn * K + k] = H::st(acc[q]);
      }
      if (db && tk == 0 && g == 0 && nok) {
        const float t = (dbr[0][li] + dbr[1][li]) + (dbr[2][li] + dbr[3][li]);
        if (db_bf16) reinterpret_cast<uint16_t*>(db)[n] = ew_f2bf(t);
        else reinterpret_cast<float*>(db)[n] = t;
      }
    }
  } else if (dx) {
    // dx[r][k] = (sum_n dy[r][n] w[n][k]) * keep_in: A = dy (rows r), B = w^T (rows k),
    // reduction over the output features in 32-wide steps; wave v: steps v, v + 4, ...
    const int bx = blockIdx.x - nbw, tr = bx % b16, tk = bx / b16;
    const int r = tr * 16 + li, k = tk * 16 + li;
    const bool rok = r < B, kok = k < K;
    const int rc = rok ? r : 0, kc = kok ? k : 0;
    const bool vec = (N % 8) == 0;
    const int nsteps = (N + 31) / 32;
    for (int s = wv; s < nsteps; s += 4) {
      const int nb = 32 * s + 8 * g;
      T dv[8], yv[8], wv8[8];
      if (vec && nb < N) {  // vector loads of this row's dz / y (N % 8 == 0: nb + 8 <= N)
        const long long o = (long long)rc * N + nb;
        const v8 d8 = *reinterpret_cast<const v8*>(dz + o);
        v8 y8 = {};
        if (RELU) y8 = *reinterpret_cast<const v8*>(y + o);
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          dv[e] = d8[e];
          yv[e] = y8[e];
        }
      } else {
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          const int nn = min(nb + e, N - 1);
          dv[e] = dz[(long long)rc * N + nn];
          yv[e] = RELU ? y[(long long)rc * N + nn] : (T)0;
        }
      }
#pragma unroll
      for (int e = 0; e < 8; ++e) wv8[e] = w[(long long)min(nb + e, N - 1) * K + kc];
      v8 a, bb;
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const int nn = nb + e;
        const bool ok = nn < N;
        a[e] = (ok && rok) ? H::st(hd_dyv<T, RELU>(dv[e], yv[e],
                                                   (uint32_t)r * (uint32_t)N + (uint32_t)nn,
                                                   kout, dout, sout))
                           : (T)0;
        bb[e] = (ok && kok) ? wv8[e] : (T)0;
      }
      acc = H::mma(a, bb, acc);
    }
    hd_wave_reduce(acc, red, wv, lane);
    if (wv == 0 && kok) {
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int rr = tr * 16 + 4 * g + q;
        if (rr >= B) continue;
        const long long o = (long long)rr * K + k;
        float v = acc[q];
        if (din.p > 0.0f) v = v * hd_mask((uint32_t)o, kin, din.p, sin);
        if constexpr (sizeof(T) == 4) {
          if (bn.h) {  // write-through: the tile's last row block reads it in this launch
            __hip_atomic_store(reinterpret_cast<float*>(dx) + o, v, __ATOMIC_RELAXED,
                               __HIP_MEMORY_SCOPE_AGENT);
            continue;
          }
        }
        dx[o] = H::st(v);
      }
    }
    if constexpr (sizeof(T) == 4) {
      if (bn.h) {
        __shared__ int last;
        __shared__ double bred[3 * 4 * 16];
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        if (threadIdx.x == 0) {
          const int prev =
              __hip_atomic_fetch_add(bn.tick + tk, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          last = prev == b16 - 1;
          if (last) __hip_atomic_store(bn.tick + tk, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
        __syncthreads();
        if (last) hd_bn_tile(bn, reinterpret_cast<const float*>(dx), B, K, tk, bred);
      }
    }
  }
  // advance the dropout counters once every block has read them (grid arrival ticket in adv0;
  // each block's counter reads completed before its barrier, hence before its ticket)
  if (adv0) {
    __syncthreads();
    if (threadIdx.x == 0 && ew_grid_last(adv0 + HD_TICKET)) {
      adv0[0] = adv0[0] + 1;
      if (adv1) adv1[0] = adv1[0] + 1;
    }
  }
}

}  // namespace

// ------------------------------------------------------------------------------------------------
// host side

static HdDrop hd_drop(uintptr_t ctr, uint32_t salt, float p) {
  HdDrop d{reinterpret_cast<const int*>(ctr), salt, ctr ? p : 0.0f};
  if (!(d.p >= 0.0f && d.p < 1.0f)) throw std::runtime_error("ewdml head: dropout p out of [0, 1)");
  return d;
}

void ew_head_fwd(uintptr_t x, uintptr_t w, uintptr_t b, uintptr_t z, uintptr_t y, int B, int N,
                 int K, int relu, uintptr_t ctr_in, uint32_t salt_in, float p_in,
                 uintptr_t ctr_out, uint32_t salt_out, float p_out, uintptr_t stream, int is_f32) {
  if (B <= 0 || N <= 0 || K % 32)
    throw std::runtime_error("ewdml head: needs B, N > 0 and K % 32 == 0");
  const HdDrop din = hd_drop(ctr_in, salt_in, p_in), dout = hd_drop(ctr_out, salt_out, p_out);
  const dim3 grid((B + 15) / 16, (N + 15) / 16);
#define HD_FWD(T, R)                                                                            \
  hipLaunchKernelGGL((k_head_fwd<T, R>), grid, dim3(EW_BLOCK), 0, (hipStream_t)stream,         \
                     reinterpret_cast<const T*>(x), reinterpret_cast<const T*>(w),               \
                     reinterpret_cast<const T*>(b), reinterpret_cast<T*>(z),                     \
                     reinterpret_cast<T*>(y), B, N, K, din, dout, HdCe<T>{})
  if (is_f32) {
    if (relu) HD_FWD(float, true);
    else HD_FWD(float, false);
  } else {
    if (relu) HD_FWD(uint16_t, true);
    else HD_FWD(uint16_t, false);
  }
#undef HD_FWD
  EW_CHECK_LAUNCH();
}

// The last Linear (no activation, no dropout) with the cross-entropy against labels yl riding in
// it (HdCe): z = logits, loss, lse [B], dlog [B][N] (nullable), lossrow [B] scratch, tick one
// zeroed int (left zeroed).  N <= 16.
void ew_head_fwd_ce(uintptr_t x, uintptr_t w, uintptr_t b, uintptr_t z, int B, int N, int K,
                    uintptr_t yl, uintptr_t lossrow, uintptr_t loss, uintptr_t lse, uintptr_t dlog,
                    uintptr_t tick, uintptr_t stream, int is_f32) {
  if (B <= 0 || N <= 0 || N > 16 || K % 32 || !yl || !lossrow || !loss || !lse || !tick)
    throw std::runtime_error("ewdml head: the cross-entropy head needs 0 < N <= 16, K % 32 == 0");
  const HdDrop none{nullptr, 0u, 0.0f};
  const dim3 grid((B + 15) / 16, 1);
#define HD_FWD_CE(T)                                                                            \
  hipLaunchKernelGGL((k_head_fwd<T, false>), grid, dim3(EW_BLOCK), 0, (hipStream_t)stream,      \
                     reinterpret_cast<const T*>(x), reinterpret_cast<const T*>(w),               \
                     reinterpret_cast<const T*>(b), reinterpret_cast<T*>(z), nullptr, B, N, K,   \
                     none, none,                                                                 \
                     HdCe<T>{reinterpret_cast<const long long*>(yl),                             \
                             reinterpret_cast<float*>(lossrow), reinterpret_cast<float*>(loss),  \
                             reinterpret_cast<float*>(lse), reinterpret_cast<T*>(dlog),          \
                             reinterpret_cast<int*>(tick)})
  if (is_f32) HD_FWD_CE(float);
  else HD_FWD_CE(uint16_t);
#undef HD_FWD_CE
  EW_CHECK_LAUNCH();
}

static void hd_bwd(uintptr_t dz, uintptr_t y, uintptr_t x, uintptr_t w, uintptr_t dx, uintptr_t dw,
                   uintptr_t db, int db_bf16, int B, int N, int K, int relu, uintptr_t ctr_out,
                   uint32_t salt_out, float p_out, uintptr_t ctr_in, uint32_t salt_in, float p_in,
                   int advance, uintptr_t stream, int is_f32, const HdBnB& bn) {
  if (B <= 0 || N <= 0 || K % 32)
    throw std::runtime_error("ewdml head: needs B, N > 0 and K % 32 == 0");
  if (relu && !y) throw std::runtime_error("ewdml head: ReLU backward needs the pre-activation");
  const HdDrop dout = hd_drop(ctr_out, salt_out, p_out), din = hd_drop(ctr_in, salt_in, p_in);
  const int nbw = ((N + 15) / 16) * ((K + 15) / 16);
  const int nbx = dx ? ((B + 15) / 16) * ((K + 15) / 16) : 0;
  // counters to advance: the masks this launch recomputed (forward and backward read one step)
  int* a0 = nullptr;
  int* a1 = nullptr;
  if (advance) {
    int* c_in = din.p > 0.0f ? reinterpret_cast<int*>(ctr_in) : nullptr;
    int* c_out = dout.p > 0.0f ? reinterpret_cast<int*>(ctr_out) : nullptr;
    a0 = c_in ? c_in : c_out;
    a1 = (c_in && c_out && c_out != c_in) ? c_out : nullptr;
  }
#define HD_BWD(T, R)                                                                            \
  hipLaunchKernelGGL((k_head_bwd<T, R>), dim3(nbw + nbx), dim3(EW_BLOCK), 0, (hipStream_t)stream, \
                     reinterpret_cast<const T*>(dz), reinterpret_cast<const T*>(y),              \
                     reinterpret_cast<const T*>(x), reinterpret_cast<const T*>(w),               \
                     reinterpret_cast<T*>(dx), reinterpret_cast<T*>(dw),                         \
                     reinterpret_cast<void*>(db), db_bf16, B, N, K, dout, din, nbw, a0, a1, bn)
  if (is_f32) {
    if (relu) HD_BWD(float, true);
    else HD_BWD(float, false);
  } else {
    if (relu) HD_BWD(uint16_t, true);
    else HD_BWD(uint16_t, false);
  }
#undef HD_BWD
  EW_CHECK_LAUNCH();
}

void ew_head_bwd(uintptr_t dz, uintptr_t y, uintptr_t x, uintptr_t w, uintptr_t dx, uintptr_t dw,
                 uintptr_t db, int db_bf16, int B, int N, int K, int relu, uintptr_t ctr_out,
                 uint32_t salt_out, float p_out, uintptr_t ctr_in, uint32_t salt_in, float p_in,
                 int advance, uintptr_t stream, int is_f32) {
  hd_bwd(dz, y, x, w, dx, dw, db, db_bf16, B, N, K, relu, ctr_out, salt_out, p_out, ctr_in, salt_in,
         p_in, advance, stream, is_f32, HdBnB{});
}

// ew_head_bwd (fp32) whose input x is the flattened output of a BatchNorm + ReLU + 2x2 max pool
// layer over 2x2 maps (bn_h [B][2][2][K], bn_code [B][K], bn_stats [4][K]): that layer's backward
// statistics and finalisation (coef [2][K], dgamma, dbeta, dcbias: k_bn_bwd_finalize's outputs)
// ride in the input-gradient blocks (HdBnB); bn_tick: K / 16 zeroed ints (left zeroed).
void ew_head_bwd_bn(uintptr_t dz, uintptr_t y, uintptr_t x, uintptr_t w, uintptr_t dx,
                    uintptr_t dw, uintptr_t db, int B, int N, int K, int relu, uintptr_t ctr_out,
                    uint32_t salt_out, float p_out, uintptr_t ctr_in, uint32_t salt_in,
                    float p_in, int advance, uintptr_t bn_h, uintptr_t bn_code,
                    uintptr_t bn_stats, uintptr_t bn_coef, uintptr_t bn_dgamma,
                    uintptr_t bn_dbeta, uintptr_t bn_dcbias, int bn_cb_bf16, uintptr_t bn_tick,
                    uintptr_t stream) {
  if (!dx || !bn_h || !bn_code || !bn_stats || !bn_coef || !bn_tick || K % 16)
    throw std::runtime_error("ewdml head: the BN backward rider needs dx, h, code, stats, coef");
  const HdBnB bn{reinterpret_cast<const float*>(bn_h), reinterpret_cast<const uint8_t*>(bn_code),
                 reinterpret_cast<const float*>(bn_stats), reinterpret_cast<float*>(bn_coef),
                 reinterpret_cast<float*>(bn_dgamma), reinterpret_cast<float*>(bn_dbeta),
                 reinterpret_cast<void*>(bn_dcbias), bn_cb_bf16, reinterpret_cast<int*>(bn_tick)};
  hd_bwd(dz, y, x, w, dx, dw, db, 0, B, N, K, relu, ctr_out, salt_out, p_out, ctr_in, salt_in, p_in,
         advance, stream, 1, bn);
}
