// Shared device helpers for the ewdml CDNA4 (gfx950) kernels.
//
// Conventions used by every kernel in this directory:
//   * a block is 256 threads = 4 wave64s (EW_BLOCK); lane = threadIdx.x & 63;
//   * a *chunk* is EW_CHUNK = 8192 consecutive elements of one parameter tensor inside the flat
//     gradient bucket; one block owns one chunk (compress/plan.py builds the tables);
//   * reductions use a fixed shuffle tree so results are bitwise reproducible run to run;
//   * the file set is compiled with -ffp-contract=off so results match the torch oracle
//     (compress/oracle.py) bit for bit.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <stdexcept>
#include <string>

// Host-side error check: turn a HIP error into a C++ exception (surfaces as a Python RuntimeError).
#define EW_CHECK(expr)                                                                       \
  do {                                                                                       \
    hipError_t _e = (expr);                                                                  \
    if (_e != hipSuccess)                                                                    \
      throw std::runtime_error(std::string("ewdml HIP error: ") + hipGetErrorString(_e) +   \
                               " at " __FILE__ ":" + std::to_string(__LINE__));             \
  } while (0)
#define EW_CHECK_LAUNCH() EW_CHECK(hipGetLastError())

#define EW_CHUNK 8192
#define EW_BLOCK 256
#define EW_WAVES (EW_BLOCK / 64)
#define EW_MAX_RANKS 64

struct TensorRow {  // mirrors BucketPlan.tensor_table()
  // idx0: position in the u16 index list (-1: bitmap-indexed); bm0: word offset of the tensor's
  // bitmap (-1: index list).  code0: dense QSGD code offset.  cap0 / cap / ncb: the predictive
  // top-k encode's candidate list offset, capacity and candidate-pass blocks.
  int off, numel, k, chunk0, nchunks, entry0, code0, idx0, bm0, cap0, cap, ncb;
};
struct CBlockRow {  // mirrors BucketPlan.cblock_table()
  int tensor, j;
};
#define EW_BM_WORDS (EW_CHUNK / 32)  // bitmap words per chunk
struct ChunkRow {  // mirrors BucketPlan.chunk_table()
  int tensor, start, len, local;
};

// Per-tensor gradient base pointers of one bucket, passed by value as a kernel argument so a
// captured HIP graph keeps them (autograd's own gradient tensors are read in place: no copy into
// a flat buffer, no accumulate-add).  Buckets hold at most EW_MAX_T tensors.
#define EW_MAX_T 128
struct GradPtrs {
  const void* p[EW_MAX_T];         // gradient base pointer of each tensor of the bucket
  uint32_t bf16[EW_MAX_T / 32];    // bit t set: tensor t's gradient is bf16 (else fp32)
};
inline void ew_fill_ptrs(GradPtrs& g, const uintptr_t* ptrs, int n, int T, const uint32_t* mask,
                         int nmask) {
  if (n != T || T > EW_MAX_T)
    throw std::runtime_error("ewdml: gradient pointer table has " + std::to_string(n) +
                             " entries, bucket has " + std::to_string(T) + " tensors (max " +
                             std::to_string(EW_MAX_T) + ")");
  for (int i = 0; i < EW_MAX_T; ++i) g.p[i] = i < T ? reinterpret_cast<const void*>(ptrs[i]) : nullptr;
  for (int i = 0; i < EW_MAX_T / 32; ++i) g.bf16[i] = (mask && i < nmask) ? mask[i] : 0u;
}

__device__ __forceinline__ float ew_bf16f(uint32_t v) { return __uint_as_float((v & 0xffffu) << 16); }
__device__ __forceinline__ uint16_t ew_f2bf(float x) {  // round-to-nearest-even, quiet NaN
  uint32_t u = __float_as_uint(x);
  if ((u & 0x7fffffffu) > 0x7f800000u) return (uint16_t)((u >> 16) | 0x40u);
  u += 0x7fffu + ((u >> 16) & 1u);
  return (uint16_t)(u >> 16);
}

// Gradient source of a chunk: the per-tensor table (fp32 or bf16 per tensor), or -- when `flat`
// is set -- a flat fp32 buffer indexed by the chunk's bucket offset (error-feedback passes read
// the staged g + residual from there).  The branch is uniform per block.
__device__ __forceinline__ float4 ew_ld4(const GradPtrs& gp, const float* flat, const ChunkRow& c,
                                         int i) {
  if (flat) return *reinterpret_cast<const float4*>(flat + c.start + i);
  const size_t off = (size_t)c.local * EW_CHUNK + i;
  if ((gp.bf16[c.tensor >> 5] >> (c.tensor & 31)) & 1u) {
    const uint2 v = *reinterpret_cast<const uint2*>(reinterpret_cast<const uint16_t*>(gp.p[c.tensor]) + off);
    return make_float4(ew_bf16f(v.x), ew_bf16f(v.x >> 16), ew_bf16f(v.y), ew_bf16f(v.y >> 16));
  }
  return *reinterpret_cast<const float4*>(reinterpret_cast<const float*>(gp.p[c.tensor]) + off);
}
__device__ __forceinline__ float ew_ld1(const GradPtrs& gp, const float* flat, const ChunkRow& c,
                                       int i) {
  if (flat) return flat[c.start + i];
  const size_t off = (size_t)c.local * EW_CHUNK + i;
  if ((gp.bf16[c.tensor >> 5] >> (c.tensor & 31)) & 1u)
    return ew_bf16f(reinterpret_cast<const uint16_t*>(gp.p[c.tensor])[off]);
  return reinterpret_cast<const float*>(gp.p[c.tensor])[off];
}
// 4 consecutive elements (i % 4 == 0) with tail handling
__device__ __forceinline__ void ew_ld4t(const GradPtrs& gp, const float* flat, const ChunkRow& c,
                                       int i, float xs[4]) {
  if (i + 3 < c.len) {
    const float4 v = ew_ld4(gp, flat, c, i);
    xs[0] = v.x; xs[1] = v.y; xs[2] = v.z; xs[3] = v.w;
  } else {
#pragma unroll
    for (int j = 0; j < 4; ++j) xs[j] = (i + j < c.len) ? ew_ld1(gp, flat, c, i + j) : 0.0f;
  }
}
// A chunk is EW_CU slabs of 4 * EW_BLOCK elements; thread t owns elements [4t, 4t + 4) of each.
// The whole chunk is loaded into registers with every load issued before any is used (a loop of
// load -> use left one round trip per slab exposed: the codec passes ran at ~3 TB/s).  Elements
// past c.len read as 0; callers mask them with ew_chunk_valid.
#define EW_CU (EW_CHUNK / (4 * EW_BLOCK))
__device__ __forceinline__ int ew_chunk_idx(int u) { return 4 * (int)threadIdx.x + u * 4 * EW_BLOCK; }
__device__ __forceinline__ void ew_ld_chunk(const GradPtrs& gp, const float* flat, const ChunkRow& c,
                                            float4 (&v)[EW_CU]) {
  // source and type resolved once (uniform), so each case below is straight-line code
  const size_t off = (size_t)c.local * EW_CHUNK;
  const bool bf = !flat && ((gp.bf16[c.tensor >> 5] >> (c.tensor & 31)) & 1u);
  const float* src = flat ? flat + c.start : reinterpret_cast<const float*>(gp.p[c.tensor]) + off;
  if (c.len == EW_CHUNK && !bf) {
#pragma unroll
    for (int u = 0; u < EW_CU; ++u) v[u] = *reinterpret_cast<const float4*>(src + ew_chunk_idx(u));
  } else if (c.len == EW_CHUNK) {
    const uint16_t* s16 = reinterpret_cast<const uint16_t*>(gp.p[c.tensor]) + off;
    uint2 r[EW_CU];
#pragma unroll
    for (int u = 0; u < EW_CU; ++u) r[u] = *reinterpret_cast<const uint2*>(s16 + ew_chunk_idx(u));
#pragma unroll
    for (int u = 0; u < EW_CU; ++u)
      v[u] = make_float4(ew_bf16f(r[u].x), ew_bf16f(r[u].x >> 16), ew_bf16f(r[u].y),
                         ew_bf16f(r[u].y >> 16));
  } else {  // a tensor's last chunk
#pragma unroll
    for (int u = 0; u < EW_CU; ++u) {
      float xs[4] = {0.0f, 0.0f, 0.0f, 0.0f};
      if (ew_chunk_idx(u) < c.len) ew_ld4t(gp, flat, c, ew_chunk_idx(u), xs);
      v[u] = make_float4(xs[0], xs[1], xs[2], xs[3]);
    }
  }
}
__device__ __forceinline__ float ew_f4(const float4& v, int j) {
  return j == 0 ? v.x : j == 1 ? v.y : j == 2 ? v.z : v.w;
}
// store back a chunk held as by ew_ld_chunk into a flat fp32 buffer (dst = chunk start)
__device__ __forceinline__ void ew_st_chunk(float* dst, int len, const float4 (&v)[EW_CU]) {
#pragma unroll
  for (int u = 0; u < EW_CU; ++u) {
    const int i = ew_chunk_idx(u);
    if (i + 3 < len) {
      *reinterpret_cast<float4*>(dst + i) = v[u];
    } else {
#pragma unroll
      for (int j = 0; j < 4; ++j)
        if (i + j < len) dst[i + j] = ew_f4(v[u], j);
    }
  }
}
// store 4 fp32 values as bf16 (8-byte store when whole)
__device__ __forceinline__ void ew_st4_bf16(uint16_t* dst, int n, const float v[4]) {
  if (n >= 4) {
    uint2 o;
    o.x = (uint32_t)ew_f2bf(v[0]) | ((uint32_t)ew_f2bf(v[1]) << 16);
    o.y = (uint32_t)ew_f2bf(v[2]) | ((uint32_t)ew_f2bf(v[3]) << 16);
    *reinterpret_cast<uint2*>(dst) = o;
  } else {
    for (int j = 0; j < n; ++j) dst[j] = ew_f2bf(v[j]);
  }
}

struct SgdArgs {
  float lr, momentum, dampening, weight_decay, grad_scale;
  int nesterov, first;
  // HIP-graph RNG key advance (nullable): key_state = {step, key} of the QSGD stream; the decode
  // kernel of a step's last bucket moves it to the next step (no host->device key copy per step)
  uint32_t* key_state;
  uint32_t key_seed, key_rank;
  // device learning rate (nullable): read at run time, so an lr schedule needs no graph
  // re-capture (the host value is frozen into a captured kernel's arguments)
  const float* lr_ptr;
};
__device__ __forceinline__ void ew_sgd_resolve(SgdArgs& a) {
  if (a.lr_ptr) a.lr = *a.lr_ptr;
}

// ---- counter-based RNG (must equal compress/rng.py) -------------------------------------------
__device__ __forceinline__ uint32_t ew_mix32(uint32_t x) {
  x ^= x >> 16;
  x *= 0x7feb352dU;
  x ^= x >> 15;
  x *= 0x846ca68bU;
  x ^= x >> 16;
  return x;
}
__device__ __forceinline__ float ew_uniform(uint32_t idx, uint32_t key) {
  return (float)(ew_mix32(idx ^ key) >> 8) * (1.0f / 16777216.0f);
}

// compress/rng.py::stream_key
__device__ __forceinline__ uint32_t ew_stream_key(uint32_t seed, uint32_t step, uint32_t rank) {
  const uint32_t k = ew_mix32(step * 0x9E3779B9u + rank * 0x85EBCA6Bu + 0x632BE59Bu);
  return ew_mix32(seed ^ k);
}

// One thread of the step's last decode kernel advances the device RNG key to the next step.  The
// step's encode kernels (the only readers) ran before this kernel; the next step's run after it.
__device__ __forceinline__ void ew_key_advance(const SgdArgs& sa) {
  if (sa.key_state && blockIdx.x == 0 && threadIdx.x == 0) {
    const uint32_t s = sa.key_state[0] + 1u;
    sa.key_state[0] = s;
    sa.key_state[1] = ew_stream_key(sa.key_seed, s, sa.key_rank);
  }
}

// Grid arrival ticket: called by thread 0 of every block (after the block's last read of the data
// the winner will update); returns true in exactly one of them, the last block to arrive.  The
// arrivals are spread over 8 sub-counters 128 B apart plus one top counter: a single counter
// serialises one atomic per block on one L2 line (~10 us at ~1000 blocks).  `tk` holds
// EW_TICKET_INTS (ewdml_ops.h) zero-initialised ints and is left zeroed.  No fences: the winner's
// writes are consumed by later kernels (kernel boundary), and every block read before it arrived.
__device__ __forceinline__ bool ew_grid_last(int* tk) {
  const int G = (int)(gridDim.x * gridDim.y * gridDim.z);
  const int b = (int)(blockIdx.x + gridDim.x * (blockIdx.y + gridDim.y * blockIdx.z));
  const int s = b & 7, members = (G - s + 7) >> 3, groups = G < 8 ? G : 8;
  int* sub = tk + 32 * s;
  if (__hip_atomic_fetch_add(sub, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != members - 1)
    return false;
  *sub = 0;
  int* top = tk + 32 * 8;
  if (__hip_atomic_fetch_add(top, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != groups - 1)
    return false;
  *top = 0;
  return true;
}

// QSGD stochastic rounding of one value (compress/oracle.py::quantize).
__device__ __forceinline__ int ew_quantize(float x, float inv, float levels, uint32_t gidx,
                                           uint32_t key) {
  float lvl = fabsf(x) * inv;
  float fl = floorf(lvl);
  float u = ew_uniform(gidx, key);
  float q = fl + ((u < (lvl - fl)) ? 1.0f : 0.0f);
  q = fminf(q, levels);
  return (int)(x < 0.0f ? -q : q);
}

__device__ __forceinline__ uint32_t ew_key(float x) { return __float_as_uint(x) & 0x7fffffffu; }

// ---- wave / block scans and reductions ----------------------------------------------------------
__device__ __forceinline__ uint32_t ew_wave_incl_scan(uint32_t v) {
  const int lane = threadIdx.x & 63;
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    uint32_t t = __shfl_up(v, d, 64);
    if (lane >= d) v += t;
  }
  return v;
}

// Exclusive scan over the block in thread order; `ws` is EW_WAVES words of LDS.
__device__ __forceinline__ uint32_t ew_block_excl_scan(uint32_t v, uint32_t* ws, uint32_t& total) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  uint32_t inc = ew_wave_incl_scan(v);
  if (lane == 63) ws[w] = inc;
  __syncthreads();
  uint32_t base = 0, tot = 0;
#pragma unroll
  for (int i = 0; i < EW_WAVES; ++i) {
    uint32_t x = ws[i];
    base += (i < w) ? x : 0u;
    tot += x;
  }
  __syncthreads();
  total = tot;
  return base + inc - v;
}

__device__ __forceinline__ float ew_wave_sum(float v) {
#pragma unroll
  for (int d = 32; d > 0; d >>= 1) v += __shfl_down(v, d, 64);
  return v;  // valid in lane 0
}
__device__ __forceinline__ uint32_t ew_wave_sum_u(uint32_t v) {
#pragma unroll
  for (int d = 32; d > 0; d >>= 1) v += __shfl_down(v, d, 64);
  return v;
}
__device__ __forceinline__ uint32_t ew_wave_max_u(uint32_t v) {
#pragma unroll
  for (int d = 32; d > 0; d >>= 1) v = max(v, (uint32_t)__shfl_down(v, d, 64));
  return v;
}

// Block sum in a fixed order (wave trees, then waves 0..3); result valid in thread 0.
__device__ __forceinline__ float ew_block_sum(float v, float* wsf) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  v = ew_wave_sum(v);
  if (lane == 0) wsf[w] = v;
  __syncthreads();
  float s = 0.0f;
  if (threadIdx.x == 0) {
#pragma unroll
    for (int i = 0; i < EW_WAVES; ++i) s += wsf[i];
  }
  __syncthreads();
  return s;
}

// ---- optimizer element updates (reference optim/sgd.py:75-91) ----------------------------------
__device__ __forceinline__ void ew_sgd(float& p, float& b, float g, const SgdArgs& a) {
  float d = g;
  if (a.weight_decay != 0.0f) d = d + a.weight_decay * p;
  if (a.momentum != 0.0f) {
    b = a.first ? d : (b * a.momentum + (1.0f - a.dampening) * d);
    d = a.nesterov ? (d + a.momentum * b) : b;
  }
  p = p - a.lr * d;
}
