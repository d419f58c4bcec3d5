// Top-k sparsification + QSGD quantisation of a flat gradient bucket, and the fused
// decode -> average -> SGD step on the receive side.  CDNA4 / gfx950, wave64.
//
// Replaces the reference's per-tensor torch chains:
//   TopK.py:5-10   flatten/abs/topk/gather       -> radix select + ordered compaction below
//   qsgd.py:17-28  norm/abs/floor/uniform/sign   -> fused into the compaction (ew_quantize)
//   TopK.py:13-17  zeros().scatter_()            -> LDS scatter in k_topk_decode_apply
//   sync_replicas_master_nn.py:189,216  sum/avg  -> fused (rank-ordered LDS sum * 1/N)
//   optim/sgd.py:75-91 per-tensor SGD           -> fused into the same kernel (ew_sgd)
//
// Exact top-k by a 3-pass MSD radix select over the 31-bit |g| key (11 + 10 + 10 bits).  Per
// pass: every chunk block builds an LDS histogram of the current digit over the elements that
// match the prefix selected so far and merges it into a per-tensor global histogram; a one-block-
// per-tensor kernel then finds the digit holding the k-th largest key.  After 3 passes the exact
// threshold key and the number of threshold ties to keep are known; ties are kept lowest index
// first, so every rank emits exactly k entries per tensor (fixed-size all-gather).
//
// Encode launches per bucket: hist0, hist1, hist2, write (max-norm scale) or hist0, hist1, hist2,
// count, write (L2 scale, which needs the selected values' sum of squares before quantising).
// The per-tensor steps between them (digit select after each histogram pass, tie allocation /
// offsets / scale after the count) run in the tensor's last-arriving chunk block
// (topk_tensor_last), not as separate launches.  hist1 also compacts the keys that match the
// selected top digit into a per-tensor candidate list, so hist2 reads a few % of the bucket instead
// of all of it; with the max-norm scale the write pass finds its chunk's entry offset and tie
// share by a decoupled look-back over the tensor's earlier chunks instead of a count pass.
// The global state lives in one scratch block: zero-initialised once, histograms re-cleared by
// k_topk_write after use, everything else fully rewritten per encode (no per-step memset).
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "common.h"
#include "ewdml_ops.h"

namespace {

constexpr int NB0 = 2048;  // pass-0 digit: key bits [30:20]
constexpr int NB1 = 1024;  // pass-1 digit: key bits [19:10]
constexpr int NB2 = 1024;  // pass-2 digit: key bits [9:0]
// Global histograms (and the max key) are replicated NREP times, chosen by block index: the
// chunks of a large tensor all hit the same few dozen bins (gradients cluster in a few exponent
// bins), and one copy serialised ~300 global atomics per bin; the select kernel sums the copies.
constexpr int NREP = 8;
constexpr int TICK_STRIDE = 32;  // ints per ticket (one 128-B line)
// the first PK_MISS_T tensors' full-path (missed prediction) counts, after the fast / full totals
// on the look-back error counter's line
constexpr int PK_MISS_T = TICK_STRIDE - 4;

// Per-tensor hand-off from the chunk blocks of a pass to the tensor's last-arriving block, which
// then runs the pass's per-tensor step itself (select / scan) instead of a one-block-per-tensor
// launch.  Everything handed off is written by device-scope atomics (histograms, max key) or
// agent-scope (sc1, write-through) stores (the count pass's per-chunk words), so no release fence
// (a per-block L2 write-back): every wave drains them (vmcnt), lane 0 draws the ticket, and only
// the last drawer acquires (cdna_hip_programming.md Guideline 16, sc1 form).  Tickets are zero at
// allocation and re-zeroed by the last drawer.
__device__ __forceinline__ bool topk_tensor_last(int* tick, int nchunks, int* flag) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) {
    const int prev = __hip_atomic_fetch_add(tick, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const int last = prev == nchunks - 1;
    if (last) {
      __hip_atomic_store(tick, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    *flag = last;
  }
  __syncthreads();
  return *flag != 0;
}

// Tensor t's digit (scanning from the top) holding its k_rem-th largest key, run by one block.
template <int NB, int SHIFT, bool FIRST>
__device__ __forceinline__ void topk_select(const uint32_t* __restrict__ hist,
                                            const TensorRow* __restrict__ tensors,
                                            uint32_t* __restrict__ state,
                                            const uint32_t* __restrict__ kmaxr, int T, int t);

// Momentum-corrected error feedback (DGC): velocity, parameters (weight decay) and hyper-
// parameters, by value.
struct DgcArgs {
  float* vel;
  const float* param;
  float momentum, damp1, wd;
  int nesterov;
  int mask;              // momentum factor masking (DGC) | keep the velocity (--ef-mode local)
  const float* lr_ptr;   // nullable: accumulate lr-scaled updates (--ef-mode local)
  // nullable, one word per tensor: 1 = the gradient's producer already staged this tensor
  // (dgc_stage.h: e in the residual, the velocity updated, the gradient never stored); the encode
  // reads e and clears the word (its write pass)
  uint32_t* stamps;
};

// error-feedback mode of the encode: none, plain (e = g + r), momentum-corrected (DGC)
enum EfMode { EF_NONE = 0, EF_PLAIN = 1, EF_DGC = 2 };

// Error-feedback staging of one chunk held in registers (v = the gradient on entry, the vector to
// compress on exit): plain e = g + r, or DGC's momentum correction; e (and DGC's velocity) are
// written back, so later passes read e from the residual.
// slabs [u0, u0 + N) of a chunk of a flat fp32 buffer (src / dst = the chunk's start), as
// ew_ld_chunk / ew_st_chunk hold them
template <int N>
__device__ __forceinline__ void ew_ld_slabs(const float* src, int len, int u0, float4 (&v)[N]) {
#pragma unroll
  for (int q = 0; q < N; ++q) {
    const int i = ew_chunk_idx(u0 + q);
    if (len == EW_CHUNK) {
      v[q] = *reinterpret_cast<const float4*>(src + i);
    } else {
      float xs[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) xs[j] = i + j < len ? src[i + j] : 0.0f;
      v[q] = make_float4(xs[0], xs[1], xs[2], xs[3]);
    }
  }
}
template <int N>
__device__ __forceinline__ void ew_st_slabs(float* dst, int len, int u0, const float4* v) {
#pragma unroll
  for (int q = 0; q < N; ++q) {
    const int i = ew_chunk_idx(u0 + q);
    if (i + 3 < len) {
      *reinterpret_cast<float4*>(dst + i) = v[q];
    } else {
#pragma unroll
      for (int j = 0; j < 4; ++j)
        if (i + j < len) dst[i + j] = ew_f4(v[q], j);
    }
  }
}

template <int EFM, bool HALVES = false>
__device__ __forceinline__ void topk_ef_stage(const GradPtrs& gp, const DgcArgs& dg,
                                              float* __restrict__ resid, const ChunkRow& c,
                                              float4 (&v)[EW_CU]) {
  if (EFM == EF_PLAIN) {  // error feedback: compress e = g + residual, staged in the residual
    float4 r[EW_CU];
    ew_ld_chunk(gp, resid, c, r);
#pragma unroll
    for (int u = 0; u < EW_CU; ++u)
      v[u] = make_float4(v[u].x + r[u].x, v[u].y + r[u].y, v[u].z + r[u].z, v[u].w + r[u].w);
    ew_st_chunk(resid + c.start, c.len, v);
  } else if (EFM == EF_DGC && HALVES) {
    // the same in two halves of the chunk: the residual / velocity / parameter registers of one
    // half at a time (k_pk_hist0: 150 -> fewer VGPRs, more chunks resident at once)
    const float lr = dg.lr_ptr ? *dg.lr_ptr : 1.0f;
    constexpr int H = EW_CU / 2;
#pragma unroll
    for (int hh = 0; hh < 2; ++hh) {
      float4 r[H], uv[H], pv[H];
      ew_ld_slabs<H>(resid + c.start, c.len, hh * H, r);
      ew_ld_slabs<H>(dg.vel + c.start, c.len, hh * H, uv);
      if (dg.wd != 0.0f) ew_ld_slabs<H>(dg.param + c.start, c.len, hh * H, pv);
#pragma unroll
      for (int q = 0; q < H; ++q) {
        const int u = hh * H + q;
        float g4[4] = {v[u].x, v[u].y, v[u].z, v[u].w};
        float u4[4] = {uv[q].x, uv[q].y, uv[q].z, uv[q].w};
        const float r4[4] = {r[q].x, r[q].y, r[q].z, r[q].w};
        float e4[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          float g = g4[j];
          if (dg.wd != 0.0f) g = g + ew_f4(pv[q], j) * dg.wd;
          const float a = u4[j] * dg.momentum;
          const float b = g * dg.damp1;
          u4[j] = a + b;
          float d = u4[j];
          if (dg.nesterov) {
            const float mu = u4[j] * dg.momentum;
            d = g + mu;
          }
          if (dg.lr_ptr) d = d * lr;
          e4[j] = r4[j] + d;
        }
        uv[q] = make_float4(u4[0], u4[1], u4[2], u4[3]);
        v[u] = make_float4(e4[0], e4[1], e4[2], e4[3]);
      }
      ew_st_slabs<H>(dg.vel + c.start, c.len, hh * H, uv);
      ew_st_slabs<H>(resid + c.start, c.len, hh * H, v + hh * H);
      __builtin_amdgcn_sched_barrier(0);  // the second half's loads after the first half's stores
    }
  } else if (EFM == EF_DGC) {
    // momentum correction (oracle.dgc_accumulate, every product / sum rounded on its own):
    // g' = g + wd p ; u = m u + (1 - d) g' ; d = g' + m u (Nesterov) | u ; e = r + d
    float4 r[EW_CU], uv[EW_CU], pv[EW_CU];
    const float lr = dg.lr_ptr ? *dg.lr_ptr : 1.0f;
    ew_ld_chunk(gp, resid, c, r);
    ew_ld_chunk(gp, dg.vel, c, uv);
    if (dg.wd != 0.0f) ew_ld_chunk(gp, dg.param, c, pv);  // uniform branch
#pragma unroll
    for (int u = 0; u < EW_CU; ++u) {
      float g4[4] = {v[u].x, v[u].y, v[u].z, v[u].w};
      float u4[4] = {uv[u].x, uv[u].y, uv[u].z, uv[u].w};
      const float r4[4] = {r[u].x, r[u].y, r[u].z, r[u].w};
      float e4[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        float g = g4[j];
        if (dg.wd != 0.0f) g = g + ew_f4(pv[u], j) * dg.wd;
        const float a = u4[j] * dg.momentum;
        const float b = g * dg.damp1;
        u4[j] = a + b;
        float d = u4[j];
        if (dg.nesterov) {
          const float mu = u4[j] * dg.momentum;
          d = g + mu;
        }
        if (dg.lr_ptr) d = d * lr;
        e4[j] = r4[j] + d;
      }
      uv[u] = make_float4(u4[0], u4[1], u4[2], u4[3]);
      v[u] = make_float4(e4[0], e4[1], e4[2], e4[3]);
    }
    ew_st_chunk(dg.vel + c.start, c.len, uv);
    ew_st_chunk(resid + c.start, c.len, v);
  }
}

// The chunk to compress into registers: the gradient, staged (topk_ef_stage) -- or, for a tensor
// its producer already staged this step (DgcArgs.stamps, dgc_stage.h), e straight from the
// residual: neither the gradient nor the velocity is read, nothing is written.
template <int EFM, bool HALVES = false>
__device__ __forceinline__ void topk_load_stage(const GradPtrs& gp, const DgcArgs& dg,
                                                float* __restrict__ resid, const ChunkRow& c,
                                                float4 (&v)[EW_CU]) {
  if (EFM == EF_DGC && dg.stamps && dg.stamps[c.tensor]) {
    ew_ld_chunk(gp, resid, c, v);
    return;
  }
  ew_ld_chunk(gp, nullptr, c, v);
  topk_ef_stage<EFM, HALVES>(gp, dg, resid, c, v);
}

// state[t] = {prefix, k_rem, max_key, pad}
template <int EFM>
__global__ __launch_bounds__(EW_BLOCK) void k_topk_hist0(GradPtrs gp, DgcArgs dg,
                                                         unsigned long long* __restrict__ lb,
                                                         float* __restrict__ resid,
                                                         const ChunkRow* __restrict__ chunks,
                                                         uint32_t* __restrict__ hist,
                                                         uint32_t* __restrict__ kmaxr, int T,
                                                         const TensorRow* __restrict__ tensors,
                                                         uint32_t* __restrict__ state,
                                                         int* __restrict__ tick) {
  // Gradients cluster in a few exponent bins, so most lanes of a wave add to the same bin and an
  // LDS atomic serialises per conflicting lane.  HSUB copies per bin in consecutive words (banks),
  // chosen by lane: a shared bin splits into HSUB bank groups; the copies are summed at the flush.
  constexpr int HSUB = 4;
  __shared__ uint32_t hs[NB0 * HSUB];
  for (int i = threadIdx.x; i < NB0 * HSUB; i += EW_BLOCK) hs[i] = 0;
  __syncthreads();
  uint32_t* h = hs + (threadIdx.x & (HSUB - 1));
  const ChunkRow c = chunks[blockIdx.x];
  // the write pass's look-back word of this chunk, from the previous encode (stream-ordered)
  if (threadIdx.x == 0) lb[blockIdx.x] = 0ull;
  float4 v[EW_CU];
  topk_load_stage<EFM>(gp, dg, resid, c, v);
  uint32_t kmax = 0;
#pragma unroll
  for (int u = 0; u < EW_CU; ++u) {
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      if (ew_chunk_idx(u) + j < c.len) {
        const uint32_t k = ew_key(ew_f4(v[u], j));
        atomicAdd(&h[(k >> 20) * HSUB], 1u);
        kmax = max(kmax, k);
      }
    }
  }
  __shared__ uint32_t wmax[EW_WAVES];
  kmax = ew_wave_max_u(kmax);
  if ((threadIdx.x & 63) == 0) wmax[threadIdx.x >> 6] = kmax;
  __syncthreads();
  const int rep = blockIdx.x & (NREP - 1);
  if (threadIdx.x == 0) {
    uint32_t m = wmax[0];
    for (int w = 1; w < EW_WAVES; ++w) m = max(m, wmax[w]);
    atomicMax(&kmaxr[rep * T + c.tensor], m);
  }
  uint32_t* dst = hist + ((size_t)rep * T + c.tensor) * NB0;
  for (int i = threadIdx.x; i < NB0; i += EW_BLOCK) {
    uint32_t v = 0;
#pragma unroll
    for (int j = 0; j < HSUB; ++j) v += hs[i * HSUB + j];
    if (v) atomicAdd(&dst[i], v);
  }
  if (topk_tensor_last(tick + TICK_STRIDE * c.tensor, tensors[c.tensor].nchunks, reinterpret_cast<int*>(wmax)))
    topk_select<NB0, 20, true>(hist, tensors, state, kmaxr, T, c.tensor);
}

// Histogram of key bits [19:10] over the elements whose top 11 bits equal the selected digit; those
// keys (the candidates of the last pass) are appended to the tensor's candidate list
// cand[tensor.off + 0 .. cand_n), at most numel of them, in no particular order.
__global__ __launch_bounds__(EW_BLOCK) void k_topk_hist1(GradPtrs gp, const float* __restrict__ flat,
                                                         const ChunkRow* __restrict__ chunks,
                                                         uint32_t* __restrict__ state,
                                                         uint32_t* __restrict__ hist, int T,
                                                         const TensorRow* __restrict__ tensors,
                                                         const uint32_t* __restrict__ kmaxr,
                                                         int* __restrict__ tick,
                                                         uint32_t* __restrict__ cand,
                                                         int* __restrict__ cand_n) {
  __shared__ uint32_t h[NB1];
  __shared__ uint32_t ws[EW_WAVES];
  __shared__ uint32_t s_base;
  for (int i = threadIdx.x; i < NB1; i += EW_BLOCK) h[i] = 0;
  __syncthreads();
  const ChunkRow c = chunks[blockIdx.x];
  const uint32_t want = state[c.tensor * 4] >> 20;
  float4 v[EW_CU];
  ew_ld_chunk(gp, flat, c, v);
  uint32_t nm = 0;
#pragma unroll
  for (int u = 0; u < EW_CU; ++u) {
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const uint32_t k = ew_key(ew_f4(v[u], j));
      if (ew_chunk_idx(u) + j < c.len && (k >> 20) == want) {
        atomicAdd(&h[(k >> 10) & (NB1 - 1)], 1u);
        ++nm;
      }
    }
  }
  uint32_t tot;
  const uint32_t ex = ew_block_excl_scan(nm, ws, tot);  // contains __syncthreads
  if (threadIdx.x == 0 && tot)
    s_base = (uint32_t)atomicAdd(cand_n + TICK_STRIDE * c.tensor, (int)tot);
  __syncthreads();
  if (nm) {
    uint32_t* dst = cand + tensors[c.tensor].off + s_base + ex;
#pragma unroll
    for (int u = 0; u < EW_CU; ++u) {
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const uint32_t k = ew_key(ew_f4(v[u], j));
        if (ew_chunk_idx(u) + j < c.len && (k >> 20) == want) *dst++ = k;
      }
    }
  }
  uint32_t* dst = hist + ((size_t)(blockIdx.x & (NREP - 1)) * T + c.tensor) * NB1;
  for (int i = threadIdx.x; i < NB1; i += EW_BLOCK)
    if (h[i]) atomicAdd(&dst[i], h[i]);
  if (topk_tensor_last(tick + TICK_STRIDE * c.tensor, tensors[c.tensor].nchunks, reinterpret_cast<int*>(h)))
    topk_select<NB1, 10, false>(hist, tensors, state, kmaxr, T, c.tensor);
}

// Histogram of key bits [9:0] over the tensor's candidates matching the 21-bit prefix: the block of
// chunk j reads candidates [8192 j, 8192 (j + 1)) of its tensor's list (most blocks have none and
// return at once).
// The tensor's last block selects the threshold and resets the candidate count for the next encode.
__global__ __launch_bounds__(EW_BLOCK) void k_topk_hist2(const ChunkRow* __restrict__ chunks,
                                                         uint32_t* __restrict__ state,
                                                         uint32_t* __restrict__ hist, int T,
                                                         const TensorRow* __restrict__ tensors,
                                                         const uint32_t* __restrict__ kmaxr,
                                                         int* __restrict__ tick,
                                                         const uint32_t* __restrict__ cand,
                                                         int* __restrict__ cand_n) {
  __shared__ uint32_t h[NB2];
  const ChunkRow c = chunks[blockIdx.x];
  const int n = __hip_atomic_load(cand_n + TICK_STRIDE * c.tensor, __ATOMIC_RELAXED,
                                  __HIP_MEMORY_SCOPE_AGENT);
  // only the first ceil(n / EW_CHUNK) chunk blocks of a tensor have candidates to read: the rest
  // leave at once (no histogram, no ticket), so the tensor's ticket counts just the readers.  A
  // reader reads n before it arrives and the count is reset only after the last arrival, so every
  // reader sees the same n; a block that sees the reset value is not a reader either way.
  const int readers = max(1, (n + EW_CHUNK - 1) / EW_CHUNK);  // chunk 0 always runs the select
  if (c.local >= readers) return;
  for (int i = threadIdx.x; i < NB2; i += EW_BLOCK) h[i] = 0;
  __syncthreads();
  const uint32_t want = state[c.tensor * 4] >> 10;
  const uint32_t* src = cand + tensors[c.tensor].off;
  const int i1 = min(n, (c.local + 1) * EW_CHUNK);
  for (int i = c.local * EW_CHUNK + (int)threadIdx.x; i < i1; i += EW_BLOCK) {
    const uint32_t k = src[i];
    if ((k >> 10) == want) atomicAdd(&h[k & (NB2 - 1)], 1u);
  }
  __syncthreads();
  uint32_t* dst = hist + ((size_t)(blockIdx.x & (NREP - 1)) * T + c.tensor) * NB2;
  for (int i = threadIdx.x; i < NB2; i += EW_BLOCK)
    if (h[i]) atomicAdd(&dst[i], h[i]);
  if (topk_tensor_last(tick + TICK_STRIDE * c.tensor, readers, reinterpret_cast<int*>(h))) {
    topk_select<NB2, 0, false>(hist, tensors, state, kmaxr, T, c.tensor);
    if (threadIdx.x == 0) cand_n[TICK_STRIDE * c.tensor] = 0;  // every reader read it before arriving
  }
}

template <int NB, int SHIFT, bool FIRST>
__device__ __forceinline__ void topk_select(const uint32_t* __restrict__ hist,
                                            const TensorRow* __restrict__ tensors,
                                            uint32_t* __restrict__ state,
                                            const uint32_t* __restrict__ kmaxr, int T, int t) {
  constexpr int PER = NB / EW_BLOCK;
  __shared__ uint32_t ws[EW_WAVES];
  const uint32_t k_rem = FIRST ? (uint32_t)tensors[t].k : state[t * 4 + 1];
  uint32_t prefix = FIRST ? 0u : state[t * 4 + 0];
  uint32_t cnt[PER];
  uint32_t tsum = 0;
#pragma unroll
  for (int j = 0; j < PER; ++j) cnt[j] = 0;
#pragma unroll
  for (int r = 0; r < NREP; ++r) {
    const uint32_t* ht = hist + ((size_t)r * T + t) * NB;
#pragma unroll
    for (int j = 0; j < PER; ++j) cnt[j] += ht[NB - 1 - (threadIdx.x * PER + j)];
  }
#pragma unroll
  for (int j = 0; j < PER; ++j) tsum += cnt[j];
  if (FIRST && threadIdx.x == 0) {
    uint32_t m = 0;
    for (int r = 0; r < NREP; ++r) m = max(m, kmaxr[r * T + t]);
    state[t * 4 + 2] = m;
  }
  uint32_t total;
  const uint32_t excl = ew_block_excl_scan(tsum, ws, total);
  if (excl < k_rem && k_rem <= excl + tsum) {
    uint32_t run = excl;
#pragma unroll
    for (int j = 0; j < PER; ++j) {
      if (run + cnt[j] >= k_rem) {
        const uint32_t bin = NB - 1 - (threadIdx.x * PER + j);
        state[t * 4 + 0] = prefix | (bin << SHIFT);
        state[t * 4 + 1] = k_rem - run;
        break;
      }
      run += cnt[j];
    }
  }
}

// Per chunk: #(key > thr), #(key == thr) and sum of squares of the key > thr values.
__device__ __forceinline__ void topk_scan(
    const TensorRow* __restrict__ tensors, const uint32_t* __restrict__ state,
    const uint32_t* __restrict__ cnt_gt, const uint32_t* __restrict__ cnt_eq,
    const float* __restrict__ chunk_sq, uint32_t* __restrict__ chunk_off,
    uint32_t* __restrict__ chunk_ties, float* __restrict__ inv_out, uint8_t* __restrict__ payload,
    int scales_off, int counts_off, float levels, int norm_l2, int t);

__global__ __launch_bounds__(EW_BLOCK) void k_topk_count(
    GradPtrs gp, const float* __restrict__ flat, const ChunkRow* __restrict__ chunks,
    const uint32_t* __restrict__ state, uint32_t* __restrict__ cnt_gt,
    uint32_t* __restrict__ cnt_eq, float* __restrict__ chunk_sq,
    const TensorRow* __restrict__ tensors, int* __restrict__ tick,
    uint32_t* __restrict__ chunk_off, uint32_t* __restrict__ chunk_ties,
    float* __restrict__ inv_out, uint8_t* __restrict__ payload, int scales_off, int counts_off,
    float levels, int norm_l2) {
  __shared__ float wsf[EW_WAVES];
  __shared__ uint32_t wsu[2 * EW_WAVES];
  const ChunkRow c = chunks[blockIdx.x];
  const uint32_t thr = state[c.tensor * 4];
  uint32_t gt = 0, eq = 0;
  float sq = 0.0f;
  float4 v[EW_CU];
  ew_ld_chunk(gp, flat, c, v);
#pragma unroll
  for (int u = 0; u < EW_CU; ++u) {
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      if (ew_chunk_idx(u) + j < c.len) {
        const float x = ew_f4(v[u], j);
        const uint32_t k = ew_key(x);
        if (k > thr) {
          ++gt;
          sq = sq + x * x;
        }
        eq += (k == thr);
      }
    }
  }
  gt = ew_wave_sum_u(gt);
  eq = ew_wave_sum_u(eq);
  if ((threadIdx.x & 63) == 0) {
    wsu[threadIdx.x >> 6] = gt;
    wsu[EW_WAVES + (threadIdx.x >> 6)] = eq;
  }
  const float s = ew_block_sum(sq, wsf);  // contains a __syncthreads
  if (threadIdx.x == 0) {
    uint32_t a = 0, b = 0;
    for (int i = 0; i < EW_WAVES; ++i) {
      a += wsu[i];
      b += wsu[EW_WAVES + i];
    }
    // sc1 stores: read by the tensor's last block in this launch
    __hip_atomic_store(cnt_gt + blockIdx.x, a, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_store(cnt_eq + blockIdx.x, b, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_store(chunk_sq + blockIdx.x, s, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  if (topk_tensor_last(tick + TICK_STRIDE * c.tensor, tensors[c.tensor].nchunks, reinterpret_cast<int*>(wsu)))
    topk_scan(tensors, state, cnt_gt, cnt_eq, chunk_sq, chunk_off, chunk_ties, inv_out, payload,
              scales_off, counts_off, levels, norm_l2, c.tensor);
}

// Tensor t, one block: allocate threshold ties to chunks (lowest index first), chunk entry
// offsets, the per-chunk uint16 counts of the payload, and the tensor's QSGD scale.
__device__ __forceinline__ void topk_scan(
    const TensorRow* __restrict__ tensors, const uint32_t* __restrict__ state,
    const uint32_t* __restrict__ cnt_gt, const uint32_t* __restrict__ cnt_eq,
    const float* __restrict__ chunk_sq, uint32_t* __restrict__ chunk_off,
    uint32_t* __restrict__ chunk_ties, float* __restrict__ inv_out, uint8_t* __restrict__ payload,
    int scales_off, int counts_off, float levels, int norm_l2, int t) {
  __shared__ uint32_t ws[EW_WAVES];
  __shared__ float wsf[EW_WAVES];
  const TensorRow tr = tensors[t];
  const uint32_t need = state[t * 4 + 1];
  const uint32_t thr = state[t * 4 + 0];
  uint16_t* counts = reinterpret_cast<uint16_t*>(payload + counts_off);
  uint32_t carry_eq = 0, carry_cnt = 0;
  float sq = 0.0f;
  for (int base = 0; base < tr.nchunks; base += EW_BLOCK) {
    const int lc = base + threadIdx.x;
    const bool ok = lc < tr.nchunks;
    const int c = tr.chunk0 + lc;
    const uint32_t gt = ok ? cnt_gt[c] : 0u, eq = ok ? cnt_eq[c] : 0u;
    uint32_t tot_eq, tot_cnt;
    const uint32_t eq_before = carry_eq + ew_block_excl_scan(eq, ws, tot_eq);
    const uint32_t ties = need > eq_before ? min(need - eq_before, eq) : 0u;
    const uint32_t cnt = gt + ties;
    const uint32_t off = carry_cnt + ew_block_excl_scan(cnt, ws, tot_cnt);
    if (ok) {
      counts[c] = (uint16_t)cnt;
      chunk_off[c] = off;
      chunk_ties[c] = ties;
      sq = sq + chunk_sq[c];
    }
    carry_eq += tot_eq;
    carry_cnt += tot_cnt;
  }
  const float total_sq = ew_block_sum(sq, wsf);
  if (threadIdx.x == 0) {
    const float tv = __uint_as_float(thr);
    float scale;
    if (norm_l2) {
      scale = sqrtf(total_sq + (float)need * (tv * tv));
    } else {
      scale = __uint_as_float(state[t * 4 + 2]);
    }
    reinterpret_cast<float*>(payload + scales_off)[t] = scale;
    inv_out[t] = scale > 0.0f ? levels / scale : 0.0f;
  }
}

enum ValueKind { VK_Q8 = 0, VK_Q4 = 1, VK_F32 = 2 };


// Ordered stream compaction of the selected entries of one chunk + fused quantisation.
// Decoupled look-back word of a chunk: status (1 = its own counts, 2 = inclusive prefix over the
// tensor's chunks up to it) | #(key > thr) | #(key == thr), 31 bits each.
constexpr unsigned long long LB_AGG = 1ull << 62, LB_INC = 2ull << 62;
// Look-back spin bound, counted in polls (each ~1 us of s_sleep): never hang, and time a wave spends
// descheduled (CWSR time-slicing between processes sharing the GPU) does not count against it, as
// it would with a wall-clock bound.  A predecessor is an earlier block of the same launch (resident
// or done), so a healthy wait is a few polls; reaching the bound bumps the error counter, which the
// trainer checks (GradientExchange.check_codec_health) and turns into a loud failure.
constexpr uint32_t LB_MAX_POLLS = 1u << 18;
__device__ __forceinline__ unsigned long long lb_pack(uint32_t gt, uint32_t eq) {
  return ((unsigned long long)gt << 31) | (unsigned long long)eq;
}

// Decoupled look-back over a tensor's chunks (consecutive blocks of one launch, dispatched in
// order): publish this chunk's per-thread counts gt (#key > thr) and eq (#key == thr) summed over
// the block, then sum the words of the earlier chunks (64 per poll) until an inclusive one.
// Leaves {gt before, eq before, gt, eq} of this chunk in s_lb[0..3] (after a __syncthreads).
__device__ __forceinline__ void topk_lookback(uint32_t gt, uint32_t eq, const ChunkRow& c,
                                              const TensorRow& tr,
                                              unsigned long long* __restrict__ lb,
                                              int* __restrict__ lb_err, uint32_t* s_lb,
                                              int lb_fault) {
  gt = ew_wave_sum_u(gt);
  eq = ew_wave_sum_u(eq);
  if ((threadIdx.x & 63) == 0) {
    s_lb[threadIdx.x >> 6] = gt;
    s_lb[EW_WAVES + (threadIdx.x >> 6)] = eq;
  }
  __syncthreads();
  if (threadIdx.x < 64) {  // wave 0: publish, then look back 64 predecessors at a time
    const int lane = threadIdx.x;
    gt = eq = 0;
    for (int w = 0; w < EW_WAVES; ++w) {
      gt += s_lb[w];
      eq += s_lb[EW_WAVES + w];
    }
    unsigned long long* my = lb + blockIdx.x;
    uint32_t gb = 0, eb = 0;
    // lb_fault (test hook): a tensor's first chunk never publishes, so its successors reach the
    // poll bound and report through lb_err
    if (lane == 0 && !(lb_fault && c.local == 0))
      __hip_atomic_store(my, (c.local == 0 ? LB_INC : LB_AGG) | lb_pack(gt, eq),
                         __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (c.local > 0) {
      // predecessors are earlier blocks of this launch (chunk rows of a tensor are consecutive
      // and dispatched in order), so they are resident or done; the spin is still bounded
      int p = (int)blockIdx.x - 1;
      uint32_t polls = 0;
      while (true) {
        const int q = p - lane;  // lane 0: the nearest predecessor
        // the tensor's first chunk always publishes an inclusive word: nothing before it
        const unsigned long long w = q >= tr.chunk0
            ? __hip_atomic_load(lb + q, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)
            : LB_INC;
        const unsigned long long st = w & (3ull << 62);
        const unsigned long long inc = __ballot(st == LB_INC);
        const unsigned long long none = __ballot(st == 0);
        const int last = inc ? __ffsll((long long)inc) - 1 : 63;  // lanes 0..last contribute
        const unsigned long long need_mask = last == 63 ? ~0ull : ((2ull << last) - 1ull);
        if (none & need_mask) {  // a predecessor not published yet: read the window again
          if (++polls > LB_MAX_POLLS) {
            if (lane == 0) atomicAdd(lb_err, 1);
            break;
          }
          __builtin_amdgcn_s_sleep(16);
          continue;
        }
        const bool use = lane <= last;
        const uint32_t wg = use ? ((uint32_t)(w >> 31) & 0x7fffffffu) : 0u;
        const uint32_t we = use ? ((uint32_t)w & 0x7fffffffu) : 0u;
        gb += ew_wave_sum_u(wg);  // valid in lane 0
        eb += ew_wave_sum_u(we);
        if (inc) break;
        p -= 64;
      }
      if (lane == 0)
        __hip_atomic_store(my, LB_INC | lb_pack(gb + gt, eb + eq), __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_AGENT);
    }
    if (lane == 0) {
      s_lb[0] = gb;
      s_lb[1] = eb;
      s_lb[2] = gt;
      s_lb[3] = eq;
    }
  }
  __syncthreads();
}

// World of one: the update the decode of this rank's own payload would apply, done by the write
// pass at each sent coordinate (k_topk_decode_sparse's arithmetic for one rank: acc = 0 + sent,
// skipped where it is 0, p = p - lr * (acc * scale)); param null = off.
struct TkApply {
  float* param;
  uint16_t* shadow;
  SgdArgs sa;  // lr / lr_ptr (resolved on entry), grad_scale; momentum, decay 0 (sparse)
  int* ticket;  // grid arrival ticket of the key advance (sa.key_state)
  // dense (receiver-side momentum: no-EF / plain-EF top-k, k_pk_one only): the momentum buffer
  // and the chunk's LDS accumulator the write fills; the step then runs over the whole chunk
  // (k_topk_decode_apply's dense pass for one rank)
  float* mom;
  float* acc;
};
__device__ __forceinline__ void tk_apply_one(const TkApply& ap, size_t i, float sent) {
  if (ap.acc) {  // dense: the decode's one-rank accumulator, 0 + sent
    ap.acc[i - 0] = 0.0f + sent;
    return;
  }
  if (sent == 0.0f) return;  // the decode's zero accumulator: p - lr * 0 is p, bit for bit
  float pv = ap.param[i], bz = 0.0f;
  ew_sgd(pv, bz, sent * ap.sa.grad_scale, ap.sa);
  ap.param[i] = pv;
  if (ap.shadow) ap.shadow[i] = ew_f2bf(pv);
}
// after the block's last read of the key: the last block of the launch advances the key state
__device__ __forceinline__ void tk_apply_done(const TkApply& ap) {
  if (!ap.param || !ap.sa.key_state) return;
  __syncthreads();
  if (threadIdx.x == 0 && ew_grid_last(ap.ticket)) {
    const uint32_t st = ap.sa.key_state[0] + 1u;
    ap.sa.key_state[0] = st;
    ap.sa.key_state[1] = ew_stream_key(ap.sa.key_seed, st, ap.sa.key_rank);
  }
}

// Predictive encode, write pass of a tensor on the fast path: the chunk's candidates (every
// element at or above the predicted threshold, which the fast path guarantees is <= the exact
// one) were compacted by k_pk_hist0 in index order, so this block reads only them -- ~3 % of the
// chunk -- instead of the chunk.  Same selection, positions, codes, bitmap words and residual /
// velocity updates as the full pass below, bit for bit.
// The tensor scale a payload publishes: NaN once any encode of this bucket counted a failure
// (a look-back or a fused-select barrier that gave up: its offsets / thresholds are stale), so a
// corrupted exchange poisons every rank's decoded update at once -- a non-finite loss at the next
// step -- instead of training on silently until the next health check (codec_health raises too).
__device__ __forceinline__ float topk_pub_scale(float scale, const int* lb_err) {
  return (lb_err && __hip_atomic_load(lb_err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0)
             ? __uint_as_float(0x7fc00000u)
             : scale;
}

template <int VK, bool EF>
__device__ __forceinline__ void topk_write_cands(
    const ChunkRow& c, const TensorRow& tr, float* __restrict__ resid, float* __restrict__ vel,
    const uint32_t* __restrict__ state, uint8_t* __restrict__ payload, int scales_off,
    int idx_off, int codes_off, int bitmap_off, int counts_off, float levels, float inv_levels,
    uint32_t key, uint32_t bucket_offset, unsigned long long* __restrict__ lb,
    int* __restrict__ lb_err, uint32_t n, const uint2* __restrict__ cs, uint32_t* ws,
    uint32_t* s_lb, int lb_fault, uint32_t thr, uint32_t need, float scale, const TkApply& ap,
    bool have0 = false, uint2 e0 = uint2{0u, 0u}) {
  // have0: the thread's first candidate (index threadIdx.x < n) already loaded as e0 (ahead of
  // the wait for the select); otherwise it is loaded once here for both loops
  __shared__ uint32_t bm[EW_BM_WORDS];
  const uint32_t eend = (uint32_t)(tr.entry0 + tr.k);
  const bool bitmap = tr.bm0 >= 0;
  if (bitmap)
    for (int i = threadIdx.x; i < EW_BM_WORDS; i += EW_BLOCK) bm[i] = 0u;
  if (!have0 && threadIdx.x < n) e0 = cs[threadIdx.x];
  uint32_t gt = 0, eq = 0;
  for (uint32_t i = threadIdx.x; i < n; i += EW_BLOCK) {
    const uint32_t k = (i == threadIdx.x ? e0 : cs[i]).x & 0x7fffffffu;
    gt += k > thr;
    eq += k == thr;
  }
  topk_lookback(gt, eq, c, tr, lb, lb_err, s_lb, lb_fault);  // ends with __syncthreads
  const uint32_t gb = s_lb[0], eb = s_lb[1], gtc = s_lb[2], eqc = s_lb[3];
  const uint32_t left_ties = need > eb ? need - eb : 0u;
  const uint32_t ties = left_ties < eqc ? left_ties : eqc;
  const uint32_t ebase = (uint32_t)tr.entry0 + gb + (need < eb ? need : eb);
  if (threadIdx.x == 0)
    reinterpret_cast<uint16_t*>(payload + counts_off)[blockIdx.x] = (uint16_t)(gtc + ties);
  const float inv = scale > 0.0f ? levels / scale : 0.0f;
  const float step = VK != VK_F32 ? scale * inv_levels : 0.0f;
  if (threadIdx.x == 0 && c.local == 0)
    reinterpret_cast<float*>(payload + scales_off)[c.tensor] = topk_pub_scale(scale, lb_err);
  uint16_t* idx_out = reinterpret_cast<uint16_t*>(payload + idx_off) + (bitmap ? 0 : tr.idx0) -
                      tr.entry0;
  const uint32_t gbase = bucket_offset + (uint32_t)c.start;
  const int ibase = c.local * EW_CHUNK;
  uint32_t carry_gt = 0, carry_eq = 0;
  for (uint32_t r0 = 0; r0 < n; r0 += EW_BLOCK) {  // uniform: n is the block's
    const uint32_t i = r0 + threadIdx.x;
    const bool valid = i < n;
    const uint2 e = valid ? (r0 == 0 ? e0 : cs[i]) : make_uint2(0u, 0u);
    const float x = __uint_as_float(e.x);
    const uint32_t k = e.x & 0x7fffffffu;
    const bool isgt = valid && k > thr, iseq = valid && k == thr;
    uint32_t tot;
    const uint32_t ex = ew_block_excl_scan((uint32_t)isgt | ((uint32_t)iseq << 16), ws, tot);
    const uint32_t eqr = carry_eq + (ex >> 16);
    const uint32_t pos = ebase + carry_gt + (ex & 0xffffu) + min(ties, eqr);
    if ((isgt || (iseq && eqr < ties)) && pos < eend) {
      const int li = (int)e.y - ibase;  // chunk-local index
      if (bitmap) atomicOr(&bm[li >> 5], 1u << (li & 31));
      else idx_out[pos] = (uint16_t)li;
      float sent;
      if (VK == VK_F32) {
        reinterpret_cast<float*>(payload + codes_off)[pos] = x;
        sent = x;
      } else {
        const int q = ew_quantize(x, inv, levels, gbase + (uint32_t)li, key);
        if (VK == VK_Q8) {
          reinterpret_cast<int8_t*>(payload + codes_off)[pos] = (int8_t)q;
        } else {
          atomicOr(reinterpret_cast<uint32_t*>(payload + codes_off) + (pos >> 3),
                   ((uint32_t)q & 0xfu) << ((pos & 7u) * 4u));
        }
        sent = (float)q * step;
      }
      if (vel) vel[c.start + li] = 0.0f;
      if (EF) resid[c.start + li] = x - sent;
      if (ap.param) tk_apply_one(ap, ap.acc ? (size_t)li : (size_t)c.start + li, sent);
    }
    carry_gt += tot & 0xffffu;
    carry_eq += tot >> 16;
  }
  if (bitmap) {
    __syncthreads();
    uint32_t* bm_out = reinterpret_cast<uint32_t*>(payload + bitmap_off) + tr.bm0 +
                       c.local * EW_BM_WORDS;
    for (int w = threadIdx.x; w * 32 < c.len; w += EW_BLOCK) bm_out[w] = bm[w];
  }
}

// The ordered write of one chunk held in registers (v: the vector to compress, e under error
// feedback), given its tensor's threshold key, this chunk's share of the threshold ties, its first
// entry and the quantiser's scale factors: indices or bitmap words, codes, residual and velocity.
template <int VK, bool EF>
__device__ __forceinline__ void topk_write_chunk(
    const ChunkRow& c, const TensorRow& tr, const float4 (&v)[EW_CU], float* __restrict__ resid,
    float* __restrict__ vel, uint8_t* __restrict__ payload, int idx_off, int codes_off,
    int bitmap_off, float levels, uint32_t key, uint32_t bucket_offset, uint32_t thr,
    uint32_t ties, uint32_t ebase, uint32_t eend, float inv, float step, uint32_t* ws,
    const TkApply& ap) {
  // entries' indices: the tensor's u16 list (chunk-local offsets), or its bitmap (one bit per
  // element; a wave's 256 elements of a slab are 8 whole words)
  const bool bitmap = tr.bm0 >= 0;
  uint16_t* idx_out = reinterpret_cast<uint16_t*>(payload + idx_off) + (bitmap ? 0 : tr.idx0) -
                      tr.entry0;
  uint32_t* bm_out = reinterpret_cast<uint32_t*>(payload + bitmap_off) +
                     (bitmap ? tr.bm0 + c.local * EW_BM_WORDS : 0);
  const uint32_t gbase = bucket_offset + (uint32_t)c.start;
  uint32_t carry_gt = 0, carry_eq = 0;
#pragma unroll
  for (int u = 0; u < EW_CU; ++u) {
    if (u * 4 * EW_BLOCK >= c.len) break;  // uniform
    const int i0 = ew_chunk_idx(u);
    const float xs[4] = {v[u].x, v[u].y, v[u].z, v[u].w};
    bool valid[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) valid[j] = (i0 + j) < c.len;
    uint32_t ngt = 0, neq = 0;
    bool isgt[4], iseq[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const uint32_t k = ew_key(xs[j]);
      isgt[j] = valid[j] && k > thr;
      iseq[j] = valid[j] && k == thr;
      ngt += isgt[j];
      neq += iseq[j];
    }
    uint32_t tot;
    const uint32_t ex = ew_block_excl_scan(ngt | (neq << 16), ws, tot);
    const uint32_t gt_before = carry_gt + (ex & 0xffffu);
    uint32_t eqr = carry_eq + (ex >> 16);
    uint32_t pos = ebase + gt_before + min(ties, eqr);
    uint32_t nib = 0;  // bitmap bits of this thread's 4 elements
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const bool sel = isgt[j] || (iseq[j] && eqr < ties);
      eqr += iseq[j];
      float sent = 0.0f;
      if (sel && pos < eend) {
        if (!bitmap) idx_out[pos] = (uint16_t)(i0 + j);
        nib |= 1u << j;
        if (VK == VK_F32) {
          reinterpret_cast<float*>(payload + codes_off)[pos] = xs[j];
          sent = xs[j];
        } else {
          const int q = ew_quantize(xs[j], inv, levels, gbase + (uint32_t)(i0 + j), key);
          if (VK == VK_Q8) {
            reinterpret_cast<int8_t*>(payload + codes_off)[pos] = (int8_t)q;
          } else {
            atomicOr(reinterpret_cast<uint32_t*>(payload + codes_off) + (pos >> 3),
                     ((uint32_t)q & 0xfu) << ((pos & 7u) * 4u));
          }
          sent = (float)q * step;
        }
        if (vel) vel[c.start + i0 + j] = 0.0f;  // DGC momentum factor masking: sent coordinates
        // EF residual: what this rank did not send.  hist0 staged e in the residual, and e - 0
        // is e bit for bit, so only the sent coordinates are rewritten (a sparse store instead
        // of rewriting the whole bucket)
        if (EF) resid[c.start + i0 + j] = xs[j] - sent;
        if (ap.param) tk_apply_one(ap, ap.acc ? (size_t)(i0 + j) : (size_t)c.start + i0 + j, sent);
        ++pos;
      }
    }
    if (bitmap) {  // uniform per block: 8 lanes' nibbles make one word; every word is written
      uint32_t w = nib << (4 * (threadIdx.x & 7));
      w |= __shfl_xor(w, 1, 64);
      w |= __shfl_xor(w, 2, 64);
      w |= __shfl_xor(w, 4, 64);
      const int wi = i0 >> 5;
      if ((threadIdx.x & 7) == 0 && wi * 32 < c.len) bm_out[wi] = w;
    }
    carry_gt += tot & 0xffffu;
    carry_eq += tot >> 16;
  }
}

// The look-back write of one chunk held in registers (max-norm scale): this chunk's #(key > thr)
// and #(key == thr), then the exclusive prefix over the tensor's earlier chunks by decoupled
// look-back -- the entry offset and the chunk's share of the threshold ties (lowest index first)
// without a counting pass -- then the ordered write.  need: the tensor's ties to keep; scale: its
// max |e|.
template <int VK, bool EF>
__device__ __forceinline__ void topk_write_lb(
    const ChunkRow& c, const TensorRow& tr, const float4 (&v)[EW_CU], float* __restrict__ resid,
    float* __restrict__ vel, uint8_t* __restrict__ payload, int scales_off, int idx_off,
    int codes_off, int bitmap_off, int counts_off, float levels, float inv_levels, uint32_t key,
    uint32_t bucket_offset, unsigned long long* __restrict__ lb, int* __restrict__ lb_err,
    uint32_t* s_lb, uint32_t* ws, int lb_fault, uint32_t thr, uint32_t need, float scale,
    const TkApply& ap) {
  const uint32_t eend = (uint32_t)(tr.entry0 + tr.k);  // never write past this tensor's entries
  uint32_t gt = 0, eq = 0;
#pragma unroll
  for (int u = 0; u < EW_CU; ++u) {
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const uint32_t k = ew_key(ew_f4(v[u], j));
      const bool ok = ew_chunk_idx(u) + j < c.len;
      gt += ok && k > thr;
      eq += ok && k == thr;
    }
  }
  topk_lookback(gt, eq, c, tr, lb, lb_err, s_lb, lb_fault);
  // ties go to the lowest-index chunks: this chunk keeps what the earlier ones left of `need`
  const uint32_t gb = s_lb[0], eb = s_lb[1], gtc = s_lb[2], eqc = s_lb[3];
  const uint32_t left_ties = need > eb ? need - eb : 0u;
  const uint32_t ties = left_ties < eqc ? left_ties : eqc;
  const uint32_t ebase = (uint32_t)tr.entry0 + gb + (need < eb ? need : eb);
  if (threadIdx.x == 0)
    reinterpret_cast<uint16_t*>(payload + counts_off)[blockIdx.x] = (uint16_t)(gtc + ties);
  // max-norm scale: the largest selected |e| is the tensor's max key (hist0)
  const float inv = scale > 0.0f ? levels / scale : 0.0f;
  const float step = VK != VK_F32 ? scale * inv_levels : 0.0f;
  if (threadIdx.x == 0 && c.local == 0)
    reinterpret_cast<float*>(payload + scales_off)[c.tensor] = topk_pub_scale(scale, lb_err);
  topk_write_chunk<VK, EF>(c, tr, v, resid, vel, payload, idx_off, codes_off, bitmap_off, levels,
                           key, bucket_offset, thr, ties, ebase, eend, inv, step, ws, ap);
}

// A chunk with more candidates than this writes from its staged values instead of its candidate
// list (the same entries, bit for bit: the candidates are every element at or above the bound,
// which the threshold is not below, in index order): the list's write runs one round of L2 loads
// and a block scan per 256 candidates, the register write a fixed EW_CU scans
constexpr uint32_t PK_WRITE_CANDS_MAX = 2048;

template <int VK, bool EF, bool LB, bool PK>
__global__ __launch_bounds__(EW_BLOCK) void k_topk_write(
    GradPtrs gp, float* __restrict__ resid, const ChunkRow* __restrict__ chunks,
    const TensorRow* __restrict__ tensors, const uint32_t* __restrict__ state,
    const uint32_t* __restrict__ chunk_off, const uint32_t* __restrict__ chunk_ties,
    const float* __restrict__ inv_arr, uint8_t* __restrict__ payload, int scales_off, int idx_off,
    int codes_off, int bitmap_off, float levels, float inv_levels, uint32_t key_arg,
    const uint32_t* __restrict__ keyp,
    uint32_t bucket_offset, uint32_t* __restrict__ rezero, uint32_t rezero_words,
    float* __restrict__ vel, unsigned long long* __restrict__ lb, int counts_off,
    int* __restrict__ lb_err, const uint32_t* __restrict__ pst,
    const uint32_t* __restrict__ cbase, const uint32_t* __restrict__ ccnt,
    const uint2* __restrict__ pcand, int lb_fault, uint32_t* __restrict__ rz1, uint32_t rz1_words,
    uint32_t* __restrict__ rz2, uint32_t rz2_words, TkApply ap, uint32_t* __restrict__ stamps) {
  __shared__ uint32_t ws[EW_WAVES];
  ew_sgd_resolve(ap.sa);
  __shared__ uint32_t s_lb[2 * EW_WAVES];
  // loads that depend on the block index alone first: the chunk row and (predictive encode) this
  // chunk's candidate segment, in flight together; then the tensor's rows
  const ChunkRow c = chunks[blockIdx.x];
  const uint32_t pk_n = PK ? ccnt[blockIdx.x] : 0u, pk_b = PK ? cbase[blockIdx.x] : 0u;
  // the histograms / max-key replicas are dead once the thresholds are selected: clear them here
  // for the next encode of this bucket (replaces a per-step memset node; first use: zero-alloc).
  // The predictive path uses one histogram copy per pass: three short ranges (rz1, rz2 too).
  for (uint32_t i = blockIdx.x * EW_BLOCK + threadIdx.x; i < rezero_words; i += gridDim.x * EW_BLOCK)
    rezero[i] = 0u;
  if (PK) {
    for (uint32_t i = blockIdx.x * EW_BLOCK + threadIdx.x; i < rz1_words; i += gridDim.x * EW_BLOCK)
      rz1[i] = 0u;
    for (uint32_t i = blockIdx.x * EW_BLOCK + threadIdx.x; i < rz2_words; i += gridDim.x * EW_BLOCK)
      rz2[i] = 0u;
  }
  const uint32_t key = keyp ? *keyp : key_arg;  // device key: fresh per replay of a captured graph
  const TensorRow tr = tensors[c.tensor];
  // the producer-staging stamps were read by the staging pass (an earlier launch): re-arm
  if (stamps && c.local == 0 && threadIdx.x == 0) stamps[c.tensor] = 0u;
  if (PK && pst[c.tensor * 8 + 3] && pk_n <= PK_WRITE_CANDS_MAX) {
    // predictive fast path: the chunk's candidates only
    // the tensor's selection state, loaded together before the look-back's barriers
    topk_write_cands<VK, EF>(c, tr, resid, vel, state, payload, scales_off, idx_off, codes_off,
                             bitmap_off, counts_off, levels, inv_levels, key, bucket_offset, lb,
                             lb_err, pk_n, pcand + tr.cap0 + pk_b, ws, s_lb, lb_fault,
                             state[c.tensor * 4], state[c.tensor * 4 + 1],
                             __uint_as_float(state[c.tensor * 4 + 2]), ap);
    tk_apply_done(ap);
    return;
  }
  const float* flat = EF ? resid : nullptr;  // EF: hist0 staged e = g + r in the residual
  const uint32_t thr = state[c.tensor * 4];
  const uint32_t eend = (uint32_t)(tr.entry0 + tr.k);  // never write past this tensor's entries
  float4 v[EW_CU];
  ew_ld_chunk(gp, flat, c, v);
  if (LB) {
    topk_write_lb<VK, EF>(c, tr, v, resid, vel, payload, scales_off, idx_off, codes_off,
                          bitmap_off, counts_off, levels, inv_levels, key, bucket_offset, lb,
                          lb_err, s_lb, ws, lb_fault, thr, state[c.tensor * 4 + 1],
                          __uint_as_float(state[c.tensor * 4 + 2]), ap);
    tk_apply_done(ap);
    return;
  }
  uint32_t ties, ebase;
  float inv, step = 0.0f;
  {
    ties = chunk_ties[blockIdx.x];
    ebase = (uint32_t)tr.entry0 + chunk_off[blockIdx.x];
    inv = inv_arr[c.tensor];
    if (VK != VK_F32) step = reinterpret_cast<const float*>(payload + scales_off)[c.tensor] * inv_levels;
  }
  topk_write_chunk<VK, EF>(c, tr, v, resid, vel, payload, idx_off, codes_off, bitmap_off, levels,
                           key, bucket_offset, thr, ties, ebase, eend, inv, step, ws, ap);
  tk_apply_done(ap);
}

// =============================================================================================
// Predictive encode (max-norm scale).  Under error feedback the vector to compress changes little
// from one step to the next, so the exact threshold of the previous encode predicts this one's.
// k_pk_hist0 stages e (error feedback) and, in the same pass over the bucket, compacts every
// element whose key is >= P = key(beta * previous threshold) into a per-tensor candidate list
// (value, index; chunk segments in index order).  If a tensor's candidates number at least k (so
// its exact threshold is >= P and every element the selection can take is a candidate) and fit
// the list, the three radix passes and the write pass read only the candidates (~3 % of the
// bucket) instead of re-reading the bucket twice; otherwise that tensor takes the full passes for
// this step.  Either way the selection is exact: same entries, codes, ties, residual and
// velocity as the full path, bit for bit.  beta adapts per tensor (k_pk_pass2's tail).
//
// pst[8 t + ...]: 0 P (key used by this encode), 1 beta (float bits; 0 = not yet set), 2 M (this
// encode's candidates), 3 fast flag, 4 P valid (a previous encode set it).
// =============================================================================================
constexpr float PK_BETA0 = 0.85f;

// block-exclusive scan of two packed u64 words (4 x 16-bit fields each) in thread order
__device__ __forceinline__ void pk_scan2(unsigned long long& a, unsigned long long& b,
                                         unsigned long long* ws, unsigned long long& ta,
                                         unsigned long long& tb) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  unsigned long long ia = a, ib = b;
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    const unsigned long long xa = __shfl_up(ia, d, 64), xb = __shfl_up(ib, d, 64);
    if (lane >= d) {
      ia += xa;
      ib += xb;
    }
  }
  if (lane == 63) {
    ws[w] = ia;
    ws[EW_WAVES + w] = ib;
  }
  __syncthreads();
  unsigned long long ba = 0, bb = 0, sa = 0, sb = 0;
#pragma unroll
  for (int i = 0; i < EW_WAVES; ++i) {
    const unsigned long long xa = ws[i], xb = ws[EW_WAVES + i];
    ba += i < w ? xa : 0ull;
    bb += i < w ? xb : 0ull;
    sa += xa;
    sb += xb;
  }
  __syncthreads();
  ta = sa;
  tb = sb;
  a = ba + ia - a;
  b = bb + ib - b;
}

// Calls f(key) (f(key, value) not needed) for this candidate-pass block's share of tensor t: its
// candidates [8192 j, 8192 (j + 1)) on the fast path, else every ncb-th chunk from j of the tensor
// (the full pass, read from the staged e or the gradients).
template <typename F>
__device__ __forceinline__ void pk_visit(const GradPtrs& gp, const float* flat,
                                         const ChunkRow* __restrict__ chunks, const TensorRow& tr,
                                         int j, bool fast, uint32_t M,
                                         const uint2* __restrict__ pcand, F&& f) {
  if (fast) {
    // all of this thread's candidate loads in flight before the first use (a load -> atomic
    // loop leaves one round trip per iteration exposed)
    constexpr int R = EW_CHUNK / EW_BLOCK;
    const uint32_t* src = reinterpret_cast<const uint32_t*>(pcand + tr.cap0);
    const uint32_t i0 = (uint32_t)j * EW_CHUNK + threadIdx.x;
    const uint32_t i1 = min(M, (uint32_t)(j + 1) * EW_CHUNK);
    uint32_t kv[R];
#pragma unroll
    for (int r = 0; r < R; ++r) {
      const uint32_t i = i0 + r * EW_BLOCK;
      kv[r] = i < i1 ? src[2 * i] : 0u;
    }
#pragma unroll
    for (int r = 0; r < R; ++r)
      if (i0 + r * EW_BLOCK < i1) f(kv[r] & 0x7fffffffu);
    return;
  }
  for (int lc = j; lc < tr.nchunks; lc += tr.ncb) {
    const ChunkRow c = chunks[tr.chunk0 + lc];
    float4 v[EW_CU];
    ew_ld_chunk(gp, flat, c, v);
#pragma unroll
    for (int u = 0; u < EW_CU; ++u)
#pragma unroll
      for (int jj = 0; jj < 4; ++jj)
        if (ew_chunk_idx(u) + jj < c.len) f(ew_key(ew_f4(v[u], jj)));
  }
}

// wave-aggregated append: one atomic per wave per call (order within the list does not matter)
__device__ __forceinline__ void pk_append(bool pred, uint32_t key, int* counter, uint32_t* dst) {
  const unsigned long long m = __ballot(pred);
  if (!m) return;
  const int lane = threadIdx.x & 63;
  const int leader = __ffsll((long long)m) - 1;
  uint32_t base = 0;
  if (lane == leader) base = (uint32_t)atomicAdd(counter, __popcll(m));
  base = __shfl(base, leader, 64);
  if (pred)  // agent scope: read by other blocks of the fused select kernel
    __hip_atomic_store(dst + base + __popcll(m & ((1ull << lane) - 1ull)), key, __ATOMIC_RELAXED,
                       __HIP_MEMORY_SCOPE_AGENT);
}

// Radix select over a tensor's keys in *relative* digits: rel = key - B, digit 0 = rel >> s0
// (< 2048), digit 1 = the next s0 - s1 bits, digit 2 = the last s1 bits (s0 <= 20, s1 <= 10).  The
// full passes use B = 0, s0 = 20, s1 = 10 (the key's bits [30:20], [19:10], [9:0]); the candidate
// passes use B = the predicted bound P and s0 = bit length of (max key - P) - 11, so the keys
// between P and the max spread over all 2048 pass-0 bins instead of the few bins of their
// exponent (an LDS-atomic hot spot).  pst[8 t + 5..7] = B, s0, s1 (set by k_pk_hist0).
// Tensor t's digit holding its k_rem-th largest key (run by one block); state[4 t] holds the
// relative prefix until pass 2 turns it into the absolute threshold key.
template <int NB, bool FIRST>
__device__ __forceinline__ void pk_select(const uint32_t* __restrict__ hist,
                                          const TensorRow* __restrict__ tensors,
                                          uint32_t* __restrict__ state,
                                          const uint32_t* __restrict__ kmaxr, int T, int t,
                                          uint32_t shift, size_t hstride = NB) {
  constexpr int PER = NB / EW_BLOCK;
  __shared__ uint32_t ws[EW_WAVES];
  // state is handed between the blocks of the fused select kernel (other XCDs): agent-scope
  // (L2-coherent) loads and stores
  const uint32_t k_rem = FIRST ? (uint32_t)tensors[t].k
                               : __hip_atomic_load(state + t * 4 + 1, __ATOMIC_RELAXED,
                                                   __HIP_MEMORY_SCOPE_AGENT);
  const uint32_t prefix = FIRST ? 0u
                                : __hip_atomic_load(state + t * 4, __ATOMIC_RELAXED,
                                                    __HIP_MEMORY_SCOPE_AGENT);
  uint32_t cnt[PER];
  uint32_t tsum = 0;
#pragma unroll
  for (int j = 0; j < PER; ++j) cnt[j] = 0;
  {  // the candidate passes use one histogram copy (<= ncb blocks per tensor add to it)
    const uint32_t* ht = hist + (size_t)t * hstride;  // hstride 0: this block's LDS histogram
#pragma unroll
    for (int j = 0; j < PER; ++j) cnt[j] = ht[NB - 1 - (threadIdx.x * PER + j)];
  }
#pragma unroll
  for (int j = 0; j < PER; ++j) tsum += cnt[j];
  if (FIRST && threadIdx.x == 0) {
    uint32_t m = 0;
    for (int r = 0; r < NREP; ++r) m = max(m, kmaxr[r * T + t]);
    __hip_atomic_store(state + t * 4 + 2, m, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  uint32_t total;
  const uint32_t excl = ew_block_excl_scan(tsum, ws, total);
  if (excl < k_rem && k_rem <= excl + tsum) {
    uint32_t run = excl;
#pragma unroll
    for (int j = 0; j < PER; ++j) {
      if (run + cnt[j] >= k_rem) {
        const uint32_t bin = NB - 1 - (threadIdx.x * PER + j);
        __hip_atomic_store(state + t * 4, prefix | (bin << shift), __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_store(state + t * 4 + 1, k_rem - run, __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_AGENT);
        // the digit-0 bin's key count: few keys are ranked directly (k_pk_select pass 1)
        if (FIRST)
          __hip_atomic_store(state + t * 4 + 3, cnt[j], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        break;
      }
      run += cnt[j];
    }
  }
}

// Tensor t's pass-2 tail (one thread): the exact threshold as an absolute key, the reset of the
// pass-1 key count, and the next encode's candidate bound: beta x this threshold, beta steered so
// the candidates stay between ~2k and 3/4 of the list.
// (beta_bits, had: pst[8 t + 1], pst[8 t + 4] as this encode found them, loaded by the caller)
__device__ __forceinline__ void pk_predict_thr(const TensorRow& tr, int t, uint32_t thr,
                                               uint32_t* __restrict__ pst,
                                               int* __restrict__ cand_n, uint32_t M,
                                               uint32_t fast, uint32_t beta_bits, uint32_t had,
                                               uint32_t hi = 0xffffffffu, uint32_t lo = 0u) {
  cand_n[TICK_STRIDE * t] = 0;  // every block read n before it arrived
  // next encode's candidate bound: beta x this exact threshold, beta steered so the
  // candidates stay between ~2k and 3/4 of the list
  float beta = __uint_as_float(beta_bits);
  if (!(beta > 0.0f)) beta = PK_BETA0;
  const uint32_t k = (uint32_t)tr.k, cap = (uint32_t)tr.cap;
  if (had) {
    if (!fast && M > cap) beta = beta + (1.0f - beta) * 0.5f;  // too many: tighter
    else if (!fast) beta = beta * 0.8f;                        // too few: the bound was above
    else if (M > min(cap - cap / 4, hi)) beta = beta + (1.0f - beta) * 0.25f;
    else if (M < (lo ? lo : 2u * k)) beta = beta * 0.95f;
  }
  beta = fminf(fmaxf(beta, 0.25f), 0.99f);
  pst[t * 8 + 1] = __float_as_uint(beta);
  // a tensor whose every element fits the candidate list (biases, small layers) takes them all:
  // bound 0, always the fast path -- without error feedback such tensors' thresholds jump from
  // step to step and a predicted bound above the k-th key sent the whole select launch through
  // the full passes (LeNet no-EF: 1 tensor-encode in 11)
  pst[t * 8 + 0] = cap >= (uint32_t)tr.numel ? 0u : ew_key(__uint_as_float(thr) * beta);
  pst[t * 8 + 4] = 1u;
}

// The candidate band of the three-launch encode in quarters of k ({lo, hi}; hi 0: 3/4 of the
// list): EWDML_PK_BAND="lo,hi" (ew_topk_encode sets it once)
__device__ uint32_t g_pk_band_q[2] = {8u, 0u};

// the same after a select whose state holds the threshold relative to B (made absolute here)
__device__ __forceinline__ void pk_predict_mf(const TensorRow& tr, int t, uint32_t B,
                                              uint32_t* __restrict__ state,
                                              uint32_t* __restrict__ pst,
                                              int* __restrict__ cand_n, uint32_t M,
                                              uint32_t fast) {
  // written by this block's select just now (agent-scope load: not a stale L1 line)
  const uint32_t thr = B + __hip_atomic_load(state + t * 4, __ATOMIC_RELAXED,
                                             __HIP_MEMORY_SCOPE_AGENT);
  __hip_atomic_store(state + t * 4, thr, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  const uint32_t k = (uint32_t)tr.k, lq = g_pk_band_q[0], hq = g_pk_band_q[1];
  pk_predict_thr(tr, t, thr, pst, cand_n, M, fast, pst[t * 8 + 1], pst[t * 8 + 4],
                 hq ? (uint32_t)(((unsigned long long)k * hq) / 4u) : 0xffffffffu,
                 (uint32_t)(((unsigned long long)k * lq) / 4u));
}

// the same, M and the fast flag from pst (set by k_pk_hist0's tensor-last block: an earlier launch,
// or this block)
__device__ __forceinline__ void pk_predict(const TensorRow& tr, int t, uint32_t B,
                                           uint32_t* __restrict__ state, uint32_t* __restrict__ pst,
                                           int* __restrict__ cand_n) {
  pk_predict_mf(tr, t, B, state, pst, cand_n, pst[t * 8 + 2], pst[t * 8 + 3]);
}

// Tensor t's three radix passes over its M <= PK_INLINE_MAX candidates in one block (LDS
// histograms), run by k_pk_hist0's tensor-last block: the same digits and selects as the
// candidate-pass kernels, so the same threshold and tie count, without their per-tensor barriers
// (each a chain of L2 round trips).  The candidates were written by other blocks of this launch
// with sc1 stores; read here with sc1 loads (cdna_hip_programming.md Guideline 16).
constexpr uint32_t PK_INLINE_MAX = 16384;  // EWDML_TOPK_INLINE: another bound, 0 = off

__device__ __forceinline__ void pk_inline_select(const uint2* __restrict__ cands, uint32_t M,
                                                 uint32_t B, uint32_t s0, uint32_t s1,
                                                 const TensorRow* __restrict__ tensors,
                                                 uint32_t* __restrict__ state,
                                                 const uint32_t* __restrict__ kmaxr, int T, int t) {
  __shared__ uint32_t h[NB0];
  constexpr int R = 16;
  const uint32_t* src = reinterpret_cast<const uint32_t*>(cands);
  // pass p: histogram of the digit of the keys whose higher digits match `want`
  auto pass = [&](int p, uint32_t want) {
    const int nb = p == 0 ? NB0 : NB1;
    for (int i = threadIdx.x; i < nb; i += EW_BLOCK) h[i] = 0;
    __syncthreads();
    for (uint32_t b0 = 0; b0 < M; b0 += EW_BLOCK * R) {
      uint32_t kv[R];
#pragma unroll
      for (int r = 0; r < R; ++r) {
        const uint32_t i = min(b0 + r * EW_BLOCK + threadIdx.x, M - 1);
        kv[r] = __hip_atomic_load(src + 2 * i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
#pragma unroll
      for (int r = 0; r < R; ++r) {
        if (b0 + r * EW_BLOCK + threadIdx.x >= M) continue;
        const uint32_t rel = (kv[r] & 0x7fffffffu) - B;
        if (p == 0) atomicAdd(&h[rel >> s0], 1u);
        else if (p == 1) {
          if ((rel >> s0) == want) atomicAdd(&h[(rel >> s1) & ((1u << (s0 - s1)) - 1u)], 1u);
        } else if ((rel >> s1) == want) {
          atomicAdd(&h[rel & ((1u << s1) - 1u)], 1u);
        }
      }
    }
    __syncthreads();
  };
  // the select's state stores (one thread) drained before the block reads them back
  auto sync_state = [&]() {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    return __hip_atomic_load(state + t * 4, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  };
  pass(0, 0u);
  pk_select<NB0, true>(h, tensors, state, kmaxr, T, t, s0, 0);
  uint32_t pre = sync_state();
  pass(1, pre >> s0);
  pk_select<NB1, false>(h, tensors, state, kmaxr, T, t, s1, 0);
  pre = sync_state();
  pass(2, pre >> s1);
  pk_select<NB2, false>(h, tensors, state, kmaxr, T, t, 0u, 0);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
}

// WPE: waves per SIMD the register allocation must allow (0: the compiler's choice, 150 VGPRs with
// DGC staging = 3 blocks per CU, so VGG-11's 1190 chunks ran in two rounds)
template <int EFM, int WPE = 0>
__global__ __launch_bounds__(EW_BLOCK, WPE) void k_pk_hist0(
    GradPtrs gp, DgcArgs dg, unsigned long long* __restrict__ lb, float* __restrict__ resid,
    const ChunkRow* __restrict__ chunks, uint32_t* __restrict__ kmaxr, int T,
    const TensorRow* __restrict__ tensors, uint32_t* __restrict__ pst, int* __restrict__ tick,
    int* __restrict__ ccount, uint32_t* __restrict__ cbase, uint32_t* __restrict__ ccnt,
    uint2* __restrict__ pcand, int* __restrict__ stats, uint32_t* __restrict__ state,
    int* __restrict__ cand_n, uint32_t inline_max) {
  __shared__ unsigned long long ws2[2 * EW_WAVES];
  __shared__ uint32_t wmax[EW_WAVES];
  __shared__ uint32_t s_base;
  __shared__ uint32_t s_sel[4];  // tensor-last block: inline flag, B, s0, s1
  const ChunkRow c = chunks[blockIdx.x];
  const TensorRow tr = tensors[c.tensor];
  if (threadIdx.x == 0) lb[blockIdx.x] = 0ull;  // the write pass's look-back word
  // the candidate passes' per-tensor arrival counts start from zero every encode: a fused select
  // whose barrier gave up (pk_wait's poll bound) can leave one behind, which would desynchronise
  // every later encode's barriers (the generation words are read relative to their value)
  if (blockIdx.x == 0)
    for (int t = threadIdx.x; t < T; t += EW_BLOCK) tick[TICK_STRIDE * (T + t)] = 0;
  float4 v[EW_CU];
  topk_load_stage<EFM, (WPE > 0)>(gp, dg, resid, c, v);
  const uint32_t P = pst[c.tensor * 8];
  uint32_t kmax = 0;
  unsigned long long pa = 0, pb = 0;  // candidates per slab, 16-bit fields (slabs 0-3, 4-7)
#pragma unroll
  for (int u = 0; u < EW_CU; ++u) {
    uint32_t n = 0;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      if (ew_chunk_idx(u) + j < c.len) {
        const uint32_t k = ew_key(ew_f4(v[u], j));
        kmax = max(kmax, k);
        n += k >= P;
      }
    }
    if (u < 4) pa |= (unsigned long long)n << (16 * u);
    else pb |= (unsigned long long)n << (16 * (u - 4));
  }
  kmax = ew_wave_max_u(kmax);
  if ((threadIdx.x & 63) == 0) wmax[threadIdx.x >> 6] = kmax;
  unsigned long long ta, tb;
  pk_scan2(pa, pb, ws2, ta, tb);  // contains __syncthreads: wmax visible
  // slab starts within the chunk's candidate segment (index order: slab, then thread, then j)
  uint32_t start[EW_CU];
  uint32_t run = 0;
#pragma unroll
  for (int u = 0; u < EW_CU; ++u) {
    start[u] = run;
    run += (uint32_t)(((u < 4 ? ta : tb) >> (16 * (u & 3))) & 0xffffull);
  }
  const uint32_t tot = run;
  if (threadIdx.x == 0) {
    uint32_t m = wmax[0];
    for (int w = 1; w < EW_WAVES; ++w) m = max(m, wmax[w]);
    atomicMax(&kmaxr[(blockIdx.x & (NREP - 1)) * T + c.tensor], m);
    const uint32_t base = tot ? (uint32_t)atomicAdd(ccount + TICK_STRIDE * c.tensor, (int)tot) : 0u;
    s_base = base;
    cbase[blockIdx.x] = base;
    ccnt[blockIdx.x] = tot;
  }
  __syncthreads();
  if (tot) {
    uint2* dst = pcand + tr.cap0;
    const uint32_t cap = (uint32_t)tr.cap, base = s_base;
#pragma unroll
    for (int u = 0; u < EW_CU; ++u) {
      uint32_t pos = base + start[u] +
                     (uint32_t)(((u < 4 ? pa : pb) >> (16 * (u & 3))) & 0xffffull);
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int i = ew_chunk_idx(u) + j;
        const float x = ew_f4(v[u], j);
        if (i < c.len && ew_key(x) >= P) {
          // write-through (sc1): the tensor's last block may select over the list in this launch
          if (pos < cap)
            __hip_atomic_store(reinterpret_cast<unsigned long long*>(dst + pos),
                               (unsigned long long)__float_as_uint(x) |
                                   ((unsigned long long)(c.local * EW_CHUNK + i) << 32),
                               __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          ++pos;
        }
      }
    }
  }
  if (!topk_tensor_last(tick + TICK_STRIDE * c.tensor, tr.nchunks, reinterpret_cast<int*>(wmax)))
    return;
  if (threadIdx.x == 0) {
    int* cc = ccount + TICK_STRIDE * c.tensor;
    const uint32_t M = (uint32_t)__hip_atomic_load(cc, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_store(cc, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const uint32_t fast = M >= (uint32_t)tr.k && M <= (uint32_t)tr.cap;
    pst[c.tensor * 8 + 2] = M;
    pst[c.tensor * 8 + 3] = fast;
    // digit geometry of the radix passes (pk_select): relative to P over the candidates, the
    // key's own bits on the full passes
    uint32_t B = 0u, s0 = 20u, s1 = 10u;
    if (fast) {
      uint32_t kmax = 0;
      for (int r = 0; r < NREP; ++r)
        kmax = max(kmax, __hip_atomic_load(kmaxr + r * T + c.tensor, __ATOMIC_RELAXED,
                                           __HIP_MEMORY_SCOPE_AGENT));
      B = P;
      const uint32_t span = kmax - P;  // >= 0: M >= k >= 1 candidates are >= P
      const int bl = span ? 32 - __clz(span) : 0;
      s0 = bl > 11 ? (uint32_t)(bl - 11) : 0u;
      s1 = s0 > 10 ? s0 - 10 : 0u;
    }
    pst[c.tensor * 8 + 5] = B;
    pst[c.tensor * 8 + 6] = s0;
    pst[c.tensor * 8 + 7] = s1;
    atomicAdd(stats + (fast ? 0 : 1), 1);
    if (!fast && c.tensor < PK_MISS_T)  // per-tensor misses: too few candidates (1) / too many (2^16)
      atomicAdd(stats + 2 + c.tensor, M < (uint32_t)tr.k ? 1 : 65536);
    s_sel[0] = fast && M <= inline_max;
    s_sel[1] = B;
    s_sel[2] = s0;
    s_sel[3] = s1;
  }
  __syncthreads();
  if (!s_sel[0]) return;
  // few candidates: this block runs the three radix passes over them itself (the select launch's
  // blocks of this tensor then exit at once: pst fast flag 2)
  pk_inline_select(pcand + tr.cap0, pst[c.tensor * 8 + 2], s_sel[1], s_sel[2], s_sel[3], tensors,
                   state, kmaxr, T, c.tensor);
  if (threadIdx.x == 0) {
    pk_predict(tr, c.tensor, s_sel[1], state, pst, cand_n);
    pst[c.tensor * 8 + 3] = 2u;
  }
}

// Radix pass 0 over the candidates (fast) or the tensor (full).
__global__ __launch_bounds__(EW_BLOCK) void k_pk_pass0(
    GradPtrs gp, const float* __restrict__ flat, const ChunkRow* __restrict__ chunks,
    const CBlockRow* __restrict__ cblocks, const TensorRow* __restrict__ tensors,
    const uint32_t* __restrict__ pst, const uint2* __restrict__ pcand, uint32_t* __restrict__ hist,
    const uint32_t* __restrict__ kmaxr, uint32_t* __restrict__ state, int T, int* __restrict__ tick) {
  constexpr int HSUB = 4;
  __shared__ uint32_t hs[NB0 * HSUB];
  for (int i = threadIdx.x; i < NB0 * HSUB; i += EW_BLOCK) hs[i] = 0;
  __syncthreads();
  uint32_t* h = hs + (threadIdx.x & (HSUB - 1));
  const CBlockRow cb = cblocks[blockIdx.x];
  const int t = cb.tensor;
  if (pst[t * 8 + 3] == 2u) return;  // selected inline by k_pk_hist0
  const TensorRow tr = tensors[t];
  const uint32_t B = pst[t * 8 + 5], s0 = pst[t * 8 + 6];
  pk_visit(gp, flat, chunks, tr, cb.j, pst[t * 8 + 3] != 0, pst[t * 8 + 2], pcand,
           [&](uint32_t k) { atomicAdd(&h[((k - B) >> s0) * HSUB], 1u); });
  __syncthreads();
  uint32_t* dst = hist + (size_t)t * NB0;
  for (int i = threadIdx.x; i < NB0; i += EW_BLOCK) {
    uint32_t x = 0;
#pragma unroll
    for (int q = 0; q < HSUB; ++q) x += hs[i * HSUB + q];
    if (x) atomicAdd(&dst[i], x);
  }
  if (topk_tensor_last(tick + TICK_STRIDE * t, tr.ncb, reinterpret_cast<int*>(hs)))
    pk_select<NB0, true>(hist, tensors, state, kmaxr, T, t, s0);
}

// Radix pass 1 over the keys in the selected digit 0; they are also appended to the tensor's key
// list cand[tensor.off ..) for pass 2 (fast path: one atomic per block, order within a block
// kept; full path: one per wave).
__global__ __launch_bounds__(EW_BLOCK) void k_pk_pass1(
    GradPtrs gp, const float* __restrict__ flat, const ChunkRow* __restrict__ chunks,
    const CBlockRow* __restrict__ cblocks, const TensorRow* __restrict__ tensors,
    const uint32_t* __restrict__ pst, const uint2* __restrict__ pcand, uint32_t* __restrict__ hist,
    const uint32_t* __restrict__ kmaxr, uint32_t* __restrict__ state, int T, int* __restrict__ tick,
    uint32_t* __restrict__ cand, int* __restrict__ cand_n) {
  __shared__ uint32_t h[NB1];
  __shared__ uint32_t ws[EW_WAVES];
  __shared__ uint32_t s_base;
  for (int i = threadIdx.x; i < NB1; i += EW_BLOCK) h[i] = 0;
  __syncthreads();
  const CBlockRow cb = cblocks[blockIdx.x];
  const int t = cb.tensor;
  if (pst[t * 8 + 3] == 2u) return;  // selected inline by k_pk_hist0
  const TensorRow tr = tensors[t];
  const uint32_t B = pst[t * 8 + 5], s0 = pst[t * 8 + 6], s1 = pst[t * 8 + 7];
  const uint32_t want = state[t * 4] >> s0;
  const uint32_t dmask = (1u << (s0 - s1)) - 1u;
  int* cn = cand_n + TICK_STRIDE * t;
  uint32_t* cdst = cand + tr.off;
  const bool fast = pst[t * 8 + 3] != 0;
  if (fast) {
    constexpr int R = EW_CHUNK / EW_BLOCK;
    const uint32_t* src = reinterpret_cast<const uint32_t*>(pcand + tr.cap0);
    const uint32_t M = pst[t * 8 + 2];
    const uint32_t i0 = (uint32_t)cb.j * EW_CHUNK + threadIdx.x;
    const uint32_t i1 = min(M, (uint32_t)cb.j * EW_CHUNK + EW_CHUNK);
    uint32_t kv[R];
#pragma unroll
    for (int r = 0; r < R; ++r) {
      const uint32_t i = i0 + r * EW_BLOCK;
      kv[r] = i < i1 ? (src[2 * i] & 0x7fffffffu) : 0u;
    }
    uint32_t nm = 0, mbits = 0;  // matches of this thread (bit r: kv[r] matched)
#pragma unroll
    for (int r = 0; r < R; ++r) {
      const uint32_t rel = kv[r] - B;
      if (i0 + r * EW_BLOCK < i1 && (rel >> s0) == want) {
        atomicAdd(&h[(rel >> s1) & dmask], 1u);
        ++nm;
        mbits |= 1u << r;
      }
    }
    uint32_t tot;
    const uint32_t ex = ew_block_excl_scan(nm, ws, tot);
    if (threadIdx.x == 0) s_base = tot ? (uint32_t)atomicAdd(cn, (int)tot) : 0u;
    __syncthreads();
    if (nm) {
      uint32_t pos = s_base + ex;
#pragma unroll
      for (int r = 0; r < R; ++r)
        if ((mbits >> r) & 1u) cdst[pos++] = kv[r];
    }
  } else {
    pk_visit(gp, flat, chunks, tr, cb.j, false, 0u, pcand, [&](uint32_t k) {
      const uint32_t rel = k - B;
      const bool m = (rel >> s0) == want;
      if (m) atomicAdd(&h[(rel >> s1) & dmask], 1u);
      pk_append(m, k, cn, cdst);
    });
  }
  __syncthreads();
  uint32_t* dst = hist + (size_t)t * NB1;
  for (int i = threadIdx.x; i < NB1; i += EW_BLOCK)
    if (h[i]) atomicAdd(&dst[i], h[i]);
  if (topk_tensor_last(tick + TICK_STRIDE * t, tr.ncb, reinterpret_cast<int*>(h)))
    pk_select<NB1, false>(hist, tensors, state, kmaxr, T, t, s1);
}

// Radix pass 2 over the pass-1 keys; the tensor's last block fixes the exact threshold (absolute
// key) and the ties, then predicts the next encode's candidate bound.
__global__ __launch_bounds__(EW_BLOCK) void k_pk_pass2(
    const CBlockRow* __restrict__ cblocks, const TensorRow* __restrict__ tensors,
    uint32_t* __restrict__ pst, uint32_t* __restrict__ hist, const uint32_t* __restrict__ kmaxr,
    uint32_t* __restrict__ state, int T, int* __restrict__ tick, const uint32_t* __restrict__ cand,
    int* __restrict__ cand_n) {
  __shared__ uint32_t h[NB2];
  for (int i = threadIdx.x; i < NB2; i += EW_BLOCK) h[i] = 0;
  __syncthreads();
  const CBlockRow cb = cblocks[blockIdx.x];
  const int t = cb.tensor;
  if (pst[t * 8 + 3] == 2u) return;  // selected inline by k_pk_hist0
  const TensorRow tr = tensors[t];
  const uint32_t n = (uint32_t)__hip_atomic_load(cand_n + TICK_STRIDE * t, __ATOMIC_RELAXED,
                                                 __HIP_MEMORY_SCOPE_AGENT);
  const uint32_t B = pst[t * 8 + 5], s1 = pst[t * 8 + 7];
  const uint32_t want = state[t * 4] >> s1;
  const uint32_t dmask = (1u << s1) - 1u;
  const uint32_t* src = cand + tr.off;
  const uint32_t stride = (uint32_t)tr.ncb * EW_CHUNK;
  constexpr int R = EW_CHUNK / EW_BLOCK;
  for (uint32_t b0 = (uint32_t)cb.j * EW_CHUNK; b0 < n; b0 += stride) {
    const uint32_t i0 = b0 + threadIdx.x, i1 = min(n, b0 + EW_CHUNK);
    uint32_t kv[R];
#pragma unroll
    for (int r = 0; r < R; ++r) {
      const uint32_t i = i0 + r * EW_BLOCK;
      kv[r] = i < i1 ? src[i] : 0u;
    }
#pragma unroll
    for (int r = 0; r < R; ++r) {
      const uint32_t rel = kv[r] - B;
      if (i0 + r * EW_BLOCK < i1 && (rel >> s1) == want) atomicAdd(&h[rel & dmask], 1u);
    }
  }
  __syncthreads();
  uint32_t* dst = hist + (size_t)t * NB2;
  for (int i = threadIdx.x; i < NB2; i += EW_BLOCK)
    if (h[i]) atomicAdd(&dst[i], h[i]);
  if (topk_tensor_last(tick + TICK_STRIDE * t, tr.ncb, reinterpret_cast<int*>(h))) {
    pk_select<NB2, false>(hist, tensors, state, kmaxr, T, t, 0u);
    __syncthreads();
    if (threadIdx.x == 0) {
      pk_predict(tr, t, B, state, pst, cand_n);
    }
  }
}

// ---------------------------------------------------------------------------------------------
// The three radix passes as ONE launch: a tensor's candidate-pass blocks (<= 24 for VGG-11's
// largest) meet at a per-tensor barrier between passes instead of at kernel boundaries -- each
// pass kernel cost ~8-15 us of which little was work (a chain of dependent round trips: block
// row, tensor row, data, histogram flush, ticket, select).  Valid only when every block of the
// grid is resident at once (the host launches it when the grid is at most one block per CU;
// otherwise the three kernels above).  The barrier: the pass's last arriver runs the select and
// then publishes a per-tensor generation word the others wait on (bounded poll; a timeout bumps
// the look-back error counter, which the health check turns into a failure).
// ---------------------------------------------------------------------------------------------
constexpr uint32_t PK_MAX_POLLS = 1u << 22;  // ~2 s of polls: only a broken launch gets there
constexpr uint32_t PK_LOCAL_MAX = 4 * EW_CHUNK;  // pass-1 keys one block takes pass 2 over
constexpr uint32_t PK_RANK_MAX = EW_BLOCK;  // digit-0 keys the pass-1 last block ranks directly
// ... as set for this process (EWDML_PK_RANK=0: never, the digit-1 / digit-2 histograms; A/B)
__device__ uint32_t g_pk_rank_max = PK_RANK_MAX;

// Everything handed across the barrier is written with device-coherent operations (histogram
// atomics, agent-scope stores of the select state and the pass-1 keys) and every wave drains its
// memory operations (vmcnt) before the block arrives, so no release fence (a write-back of the
// XCD's L2) is needed; a block that proceeds past a barrier takes an agent acquire (cdna
// guideline 16, as topk_tensor_last).
// block-uniform: true in the pass's last-arriving block of tensor t
__device__ __forceinline__ bool pk_arrive(int* arrive, int ncb, int* flag) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this wave's flushes and appends landed
  __syncthreads();
  if (threadIdx.x == 0) {
    const int prev = __hip_atomic_fetch_add(arrive, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const int last = prev == ncb - 1;
    if (last) __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
    *flag = last;
  }
  __syncthreads();
  return *flag != 0;
}

// the last arriver, after its select: reset the arrive count, publish generation `g`
__device__ __forceinline__ void pk_publish(int* arrive, uint32_t* gen, uint32_t g) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // every wave's select stores landed
  __syncthreads();
  if (threadIdx.x == 0) {
    __hip_atomic_store(arrive, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_store(gen, g, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
}

// everyone else: wait for generation g, block-uniform; returns the generation seen
__device__ __forceinline__ uint32_t pk_wait(const uint32_t* gen, uint32_t g, int* err,
                                            uint32_t* s_gen) {
  if (threadIdx.x == 0) {
    uint32_t polls = 0, v;
    while ((int)((v = __hip_atomic_load(gen, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) - g) < 0) {
      if (++polls > PK_MAX_POLLS) {
        atomicAdd(err, 1);
        break;
      }
      __builtin_amdgcn_s_sleep(2);
    }
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
    *s_gen = v;
  }
  __syncthreads();
  return *s_gen;
}

__global__ __launch_bounds__(EW_BLOCK) void k_pk_select(
    GradPtrs gp, const float* __restrict__ flat, const ChunkRow* __restrict__ chunks,
    const CBlockRow* __restrict__ cblocks, const TensorRow* __restrict__ tensors,
    uint32_t* __restrict__ pst, const uint2* __restrict__ pcand, uint32_t* __restrict__ hist0,
    uint32_t* __restrict__ hist1, uint32_t* __restrict__ hist2, const uint32_t* __restrict__ kmaxr,
    uint32_t* __restrict__ state, int T, int* __restrict__ arrive, uint32_t* __restrict__ gen,
    uint32_t* __restrict__ cand, int* __restrict__ cand_n, int* __restrict__ err) {
  constexpr int HSUB = 4;
  constexpr int R = EW_CHUNK / EW_BLOCK;
  __shared__ uint32_t hs[NB0 * HSUB];
  __shared__ uint32_t ws[EW_WAVES];
  __shared__ uint32_t s_base, s_gen;
  __shared__ int s_flag;
  const CBlockRow cb = cblocks[blockIdx.x];
  const int t = cb.tensor;
  if (pst[t * 8 + 3] == 2u) return;  // selected inline by k_pk_hist0: no barrier to join
  const TensorRow tr = tensors[t];
  int* arr = arrive + TICK_STRIDE * t;
  uint32_t* gn = gen + TICK_STRIDE * t;
  // every block reads the generation before its first arrival; it moves only after all arrived
  const uint32_t g0 = __hip_atomic_load(gn, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  const bool fast = pst[t * 8 + 3] != 0;
  const uint32_t M = pst[t * 8 + 2];
  const uint32_t B = pst[t * 8 + 5], s0 = pst[t * 8 + 6], s1 = pst[t * 8 + 7];
  // this block's candidates (fast path), loaded once for passes 0 and 1
  const uint32_t i0 = (uint32_t)cb.j * EW_CHUNK + threadIdx.x;
  const uint32_t i1 = min(M, (uint32_t)cb.j * EW_CHUNK + EW_CHUNK);
  uint32_t kv[R];
  if (fast) {
    const uint32_t* src = reinterpret_cast<const uint32_t*>(pcand + tr.cap0);
#pragma unroll
    for (int r = 0; r < R; ++r) {
      const uint32_t i = i0 + r * EW_BLOCK;
      kv[r] = i < i1 ? (src[2 * i] & 0x7fffffffu) : 0u;
    }
  }
  // ---- pass 0: digit (key - B) >> s0 ----
  for (int i = threadIdx.x; i < NB0 * HSUB; i += EW_BLOCK) hs[i] = 0;
  __syncthreads();
  {
    uint32_t* h = hs + (threadIdx.x & (HSUB - 1));
    if (fast) {
#pragma unroll
      for (int r = 0; r < R; ++r)
        if (i0 + r * EW_BLOCK < i1) atomicAdd(&h[((kv[r] - B) >> s0) * HSUB], 1u);
    } else {
      pk_visit(gp, flat, chunks, tr, cb.j, false, 0u, pcand,
               [&](uint32_t k) { atomicAdd(&h[((k - B) >> s0) * HSUB], 1u); });
    }
  }
  __syncthreads();
  {
    uint32_t* dst = hist0 + (size_t)t * NB0;
    for (int i = threadIdx.x; i < NB0; i += EW_BLOCK) {
      uint32_t x = 0;
#pragma unroll
      for (int q = 0; q < HSUB; ++q) x += hs[i * HSUB + q];
      if (x) atomicAdd(&dst[i], x);
    }
  }
  if (pk_arrive(arr, tr.ncb, &s_flag)) {
    pk_select<NB0, true>(hist0, tensors, state, kmaxr, T, t, s0);
    pk_publish(arr, gn, g0 + 1u);
  } else {
    pk_wait(gn, g0 + 1u, err, &s_gen);
  }
  // ---- pass 1: next s0 - s1 bits of the keys in the selected digit 0; those keys -> cand ----
  // (fast path with at most PK_RANK_MAX keys in that digit: no digit-1 histogram -- the last
  // block ranks the compacted keys directly)
  const bool ranked = fast && __hip_atomic_load(state + t * 4 + 3, __ATOMIC_RELAXED,
                                                __HIP_MEMORY_SCOPE_AGENT) <= g_pk_rank_max;
  {
    const uint32_t want = __hip_atomic_load(state + t * 4, __ATOMIC_RELAXED,
                                            __HIP_MEMORY_SCOPE_AGENT) >> s0;
    const uint32_t dmask = (1u << (s0 - s1)) - 1u;
    int* cn = cand_n + TICK_STRIDE * t;
    uint32_t* cdst = cand + tr.off;
    uint32_t* h = hs;
    if (!ranked) {
      for (int i = threadIdx.x; i < NB1; i += EW_BLOCK) h[i] = 0;
      __syncthreads();
    }
    if (fast) {
      uint32_t nm = 0, mbits = 0;
#pragma unroll
      for (int r = 0; r < R; ++r) {
        const uint32_t rel = kv[r] - B;
        if (i0 + r * EW_BLOCK < i1 && (rel >> s0) == want) {
          if (!ranked) atomicAdd(&h[(rel >> s1) & dmask], 1u);
          ++nm;
          mbits |= 1u << r;
        }
      }
      uint32_t tot;
      const uint32_t ex = ew_block_excl_scan(nm, ws, tot);
      if (threadIdx.x == 0) s_base = tot ? (uint32_t)atomicAdd(cn, (int)tot) : 0u;
      __syncthreads();
      if (nm) {
        uint32_t pos = s_base + ex;
#pragma unroll
        for (int r = 0; r < R; ++r)
          if ((mbits >> r) & 1u)
            __hip_atomic_store(cdst + pos++, kv[r], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
    } else {
      pk_visit(gp, flat, chunks, tr, cb.j, false, 0u, pcand, [&](uint32_t k) {
        const uint32_t rel = k - B;
        const bool m = (rel >> s0) == want;
        if (m) atomicAdd(&h[(rel >> s1) & dmask], 1u);
        pk_append(m, k, cn, cdst);
      });
    }
    if (!ranked) {
      __syncthreads();
      uint32_t* dst = hist1 + (size_t)t * NB1;
      for (int i = threadIdx.x; i < NB1; i += EW_BLOCK)
        if (h[i]) atomicAdd(&dst[i], h[i]);
    }
  }
  if (pk_arrive(arr, tr.ncb, &s_flag)) {
    if (ranked) {
      // the n compacted keys (absolute), one per thread: the k_rem-th largest is the threshold,
      // k_rem minus the keys above it the ties to keep (what digits 1 and 2 give)
      const uint32_t n = (uint32_t)__hip_atomic_load(cand_n + TICK_STRIDE * t, __ATOMIC_RELAXED,
                                                     __HIP_MEMORY_SCOPE_AGENT);
      const uint32_t k_rem = __hip_atomic_load(state + t * 4 + 1, __ATOMIC_RELAXED,
                                               __HIP_MEMORY_SCOPE_AGENT);
      const uint32_t* src = cand + tr.off;
      // n is the digit-0 bin's count (<= PK_RANK_MAX): the same keys, the same predicate
      if (threadIdx.x == 0 && n > (uint32_t)EW_BLOCK) atomicAdd(err, 1);
      if (threadIdx.x < n)
        hs[threadIdx.x] = __hip_atomic_load(src + threadIdx.x, __ATOMIC_RELAXED,
                                            __HIP_MEMORY_SCOPE_AGENT);
      __syncthreads();
      if (threadIdx.x < n) {
        const uint32_t mine = hs[threadIdx.x];
        uint32_t gt = 0, eq = 0;
        for (uint32_t j = 0; j < n; ++j) {
          const uint32_t x = hs[j];
          gt += x > mine;
          eq += x == mine;
        }
        if (gt < k_rem && k_rem <= gt + eq) {  // (equal keys: the same two words)
          __hip_atomic_store(state + t * 4, mine - B, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          __hip_atomic_store(state + t * 4 + 1, k_rem - gt, __ATOMIC_RELAXED,
                             __HIP_MEMORY_SCOPE_AGENT);
        }
      }
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the state stores before pk_predict's loads
      __syncthreads();
      if (threadIdx.x == 0) pk_predict(tr, t, B, state, pst, cand_n);
      pk_publish(arr, gn, g0 + 3u);
      return;
    }
    pk_select<NB1, false>(hist1, tensors, state, kmaxr, T, t, s1);
    // few pass-1 keys (the usual case): this block runs pass 2 over them alone, in LDS, and the
    // tensor is done without a third barrier (generation g0 + 3 tells the waiting blocks)
    const uint32_t n = (uint32_t)__hip_atomic_load(cand_n + TICK_STRIDE * t, __ATOMIC_RELAXED,
                                                   __HIP_MEMORY_SCOPE_AGENT);
    if (n <= PK_LOCAL_MAX) {
      __syncthreads();  // the select's state stores issued; hs free
      const uint32_t want = __hip_atomic_load(state + t * 4, __ATOMIC_RELAXED,
                                              __HIP_MEMORY_SCOPE_AGENT) >> s1;
      const uint32_t dmask = (1u << s1) - 1u;
      const uint32_t* src = cand + tr.off;
      uint32_t* h = hs;
      for (int i = threadIdx.x; i < NB2; i += EW_BLOCK) h[i] = 0;
      __syncthreads();
      for (uint32_t b0 = 0; b0 < n; b0 += EW_CHUNK) {
        const uint32_t j0 = b0 + threadIdx.x, j1 = min(n, b0 + EW_CHUNK);
        uint32_t kk[R];
#pragma unroll
        for (int r = 0; r < R; ++r) {
          const uint32_t i = j0 + r * EW_BLOCK;
          kk[r] = i < j1 ? __hip_atomic_load(src + i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)
                         : 0u;
        }
#pragma unroll
        for (int r = 0; r < R; ++r) {
          const uint32_t rel = kk[r] - B;
          if (j0 + r * EW_BLOCK < j1 && (rel >> s1) == want) atomicAdd(&h[rel & dmask], 1u);
        }
      }
      __syncthreads();
      pk_select<NB2, false>(h, tensors, state, kmaxr, T, t, 0u, 0);
      __syncthreads();
      if (threadIdx.x == 0) pk_predict(tr, t, B, state, pst, cand_n);
      pk_publish(arr, gn, g0 + 3u);
      return;
    }
    pk_publish(arr, gn, g0 + 2u);
  } else if (pk_wait(gn, g0 + 2u, err, &s_gen) == g0 + 3u) {
    return;  // pass 2 ran in the last block of pass 1
  }
  // ---- pass 2: the last s1 bits over the pass-1 keys ----
  {
    const uint32_t n = (uint32_t)__hip_atomic_load(cand_n + TICK_STRIDE * t, __ATOMIC_RELAXED,
                                                   __HIP_MEMORY_SCOPE_AGENT);
    const uint32_t want = __hip_atomic_load(state + t * 4, __ATOMIC_RELAXED,
                                            __HIP_MEMORY_SCOPE_AGENT) >> s1;
    const uint32_t dmask = (1u << s1) - 1u;
    const uint32_t* src = cand + tr.off;
    const uint32_t stride = (uint32_t)tr.ncb * EW_CHUNK;
    uint32_t* h = hs;
    for (int i = threadIdx.x; i < NB2; i += EW_BLOCK) h[i] = 0;
    __syncthreads();
    for (uint32_t b0 = (uint32_t)cb.j * EW_CHUNK; b0 < n; b0 += stride) {
      const uint32_t j0 = b0 + threadIdx.x, j1 = min(n, b0 + EW_CHUNK);
      uint32_t kk[R];
#pragma unroll
      for (int r = 0; r < R; ++r) {
        const uint32_t i = j0 + r * EW_BLOCK;
        kk[r] = i < j1 ? __hip_atomic_load(src + i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)
                       : 0u;
      }
#pragma unroll
      for (int r = 0; r < R; ++r) {
        const uint32_t rel = kk[r] - B;
        if (j0 + r * EW_BLOCK < j1 && (rel >> s1) == want) atomicAdd(&h[rel & dmask], 1u);
      }
    }
    __syncthreads();
    uint32_t* dst = hist2 + (size_t)t * NB2;
    for (int i = threadIdx.x; i < NB2; i += EW_BLOCK)
      if (h[i]) atomicAdd(&dst[i], h[i]);
  }
  if (pk_arrive(arr, tr.ncb, &s_flag)) {
    pk_select<NB2, false>(hist2, tensors, state, kmaxr, T, t, 0u);
    __syncthreads();
    if (threadIdx.x == 0) pk_predict(tr, t, B, state, pst, cand_n);
    pk_publish(arr, gn, g0 + 3u);
  }
}

// ---------------------------------------------------------------------------------------------
// Small buckets (every chunk block resident at once): the whole predictive encode as ONE launch.
// The bucket's three launches (k_pk_hist0 -> k_pk_select -> k_topk_write) were each a chain of
// dependent round trips over a few dozen blocks (LeNet: 53 chunks; ~40 us of encode for 1.7 MB):
//   1. stage + compact candidates (k_pk_hist0's body; the staged chunk stays in registers);
//   2. the tensor's last-arriving block selects the exact threshold over the candidates, staged
//      in LDS (fast path), and publishes the tensor's generation word; when the prediction missed
//      (the first encode, a jump), every block of the tensor joins three histogram passes over
//      its own registers with a per-tensor barrier between them (k_pk_select's full path);
//   3. each block writes its chunk (k_topk_write: candidates or registers, decoupled look-back
//      over its tensor's earlier chunks, all resident).
// Same selection, codes, ties, residual and velocity as the three launches, bit for bit.
// Hand-offs (cdna_hip_programming.md Guideline 16; MI355X_MICROARCH.md's table, row 1): every
// word another block reads -- candidates, select state, mode and generation words, look-back
// words, histogram rows -- is written by agent-scope atomics or sc1 stores after the writer's
// vmcnt drain and read by agent-scope (sc1) loads after the poll, plus an agent acquire.
// ---------------------------------------------------------------------------------------------
constexpr int PK1_NSTAMP = 16;  // probe stamps per block (EWDML_PK1_STAMPS)
// the candidate band's floor for few-k tensors without error feedback (k_pk_one's prediction;
// EWDML_PK1_LO: another, 0 = none; A/B)
__device__ uint32_t g_pk1_lo_keys = 2048u;
constexpr int PK1_LDS_KEYS = 10240;  // candidate keys the selecting block stages in LDS (40 KB):
                                     // with the histograms ~73 KB, two blocks per CU
constexpr int PK1_HSUB = 4;  // pass-0 sub-histograms (lanes t % 4): the candidates crowd the low
                             // bins (just above the predicted bound), a same-address LDS atomic hot
                             // spot

// One digit select over an LDS histogram of NB bins, scanned from the top, state in LDS: the bin
// holding the k_rem-th largest key (st[0] |= bin << shift; st[1] = what is left of k_rem).  The
// same arithmetic as pk_select without its global state round trips.
// SUB: bin b's count is the sum of h[b * SUB .. b * SUB + SUB - 1] (pass 0's sub-histograms)
template <int NB, int SUB = 1>
__device__ __forceinline__ void pk1_digit(const uint32_t* h, uint32_t* st, uint32_t shift,
                                          uint32_t* ws) {
  constexpr int PER = NB / EW_BLOCK;
  const uint32_t k_rem = st[1], prefix = st[0];
  uint32_t cnt[PER], tsum = 0;
#pragma unroll
  for (int j = 0; j < PER; ++j) {
    const int b = NB - 1 - (threadIdx.x * PER + j);
    if constexpr (SUB == 4) {
      const uint4 q = *reinterpret_cast<const uint4*>(h + b * 4);
      cnt[j] = q.x + q.y + q.z + q.w;
    } else {
      cnt[j] = 0;
#pragma unroll
      for (int q = 0; q < SUB; ++q) cnt[j] += h[b * SUB + q];
    }
    tsum += cnt[j];
  }
  uint32_t total;
  const uint32_t excl = ew_block_excl_scan(tsum, ws, total);  // (its barriers: k_rem read by all)
  if (excl < k_rem && k_rem <= excl + tsum) {
    uint32_t run = excl;
#pragma unroll
    for (int j = 0; j < PER; ++j) {
      if (run + cnt[j] >= k_rem) {
        st[0] = prefix | ((uint32_t)(NB - 1 - (threadIdx.x * PER + j)) << shift);
        st[1] = k_rem - run;
        break;
      }
      run += cnt[j];
    }
  }
  __syncthreads();
}

// Tensor t's three radix passes over its M candidates (keys in .x of pcand) in one block: keys
// [0, nl) from LDS (staged there first), the rest from the list (sc1 loads); histograms and the
// select state in LDS; the same digits and selects as pk_inline_select / the candidate-pass
// kernels.  Leaves the absolute threshold key in st[0] and the ties to keep in st[1], and stores
// the tensor's select state {threshold, ties, max key} once.
__device__ __forceinline__ void pk1_select_cands(const uint2* __restrict__ cands, uint32_t M,
                                                 uint32_t B, uint32_t s0, uint32_t s1,
                                                 uint32_t kmax, uint32_t k, uint32_t* keys,
                                                 uint32_t nl, uint32_t* h, uint32_t* st,
                                                 uint32_t* ws, uint32_t* __restrict__ state,
                                                 int t, unsigned long long* stamp = nullptr) {
  // probe stamps (k_pk_one's row, slots 8..12): pass 0 (keys staged), fold, digit 0, the
  // selected bin's keys ranked (or passes 1 and 2)
#define PK1_SSTAMP(i) \
  if (stamp && threadIdx.x == 0) stamp[i] = wall_clock64()
  constexpr int R = 16;  // loads in flight per thread (each an L2 round trip)
  const uint32_t* src = reinterpret_cast<const uint32_t*>(cands);
  uint32_t* h0 = h + (threadIdx.x & (PK1_HSUB - 1));
  auto add = [&](int p, uint32_t want, uint32_t key) {
    const uint32_t rel = key - B;
    if (p == 0) atomicAdd(&h0[(rel >> s0) * PK1_HSUB], 1u);
    else if (p == 1) {
      if ((rel >> s0) == want) atomicAdd(&h[(rel >> s1) & ((1u << (s0 - s1)) - 1u)], 1u);
    } else if ((rel >> s1) == want) {
      atomicAdd(&h[rel & ((1u << s1) - 1u)], 1u);
    }
  };
  // the keys beyond the LDS copy: batched sc1 loads from the list
  auto beyond = [&](auto&& f) {
    for (uint32_t b0 = nl; b0 < M; b0 += EW_BLOCK * R) {
      uint32_t kv[R];
#pragma unroll
      for (int r = 0; r < R; ++r) {
        const uint32_t i = min(b0 + r * EW_BLOCK + threadIdx.x, M - 1);
        kv[r] = __hip_atomic_load(src + 2 * i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
#pragma unroll
      for (int r = 0; r < R; ++r)
        if (b0 + r * EW_BLOCK + threadIdx.x < M) f(kv[r] & 0x7fffffffu);
    }
  };
  auto pass = [&](int p, uint32_t want) {
    const int nb = p == 0 ? NB0 * PK1_HSUB : NB1;
    for (int i = threadIdx.x; i < nb; i += EW_BLOCK) h[i] = 0;
    __syncthreads();
    for (uint32_t i = threadIdx.x; i < nl; i += EW_BLOCK) add(p, want, keys[i]);
    beyond([&](uint32_t key) { add(p, want, key); });
    __syncthreads();
  };
  if (threadIdx.x == 0) {
    st[0] = 0u;
    st[1] = k;
  }
  // pass 0 while the keys are staged into LDS: each key counted as it arrives (h: its
  // NB0 x PK1_HSUB sub-histograms, zeroed by every block at the kernel's start)
  for (uint32_t b0 = 0; b0 < nl; b0 += EW_BLOCK * R) {
    uint32_t kv[R];
#pragma unroll
    for (int r = 0; r < R; ++r) {
      const uint32_t i = min(b0 + r * EW_BLOCK + threadIdx.x, nl - 1);
      kv[r] = __hip_atomic_load(src + 2 * i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
#pragma unroll
    for (int r = 0; r < R; ++r) {
      const uint32_t i = b0 + r * EW_BLOCK + threadIdx.x;
      if (i < nl) {
        const uint32_t key = kv[r] & 0x7fffffffu;
        keys[i] = key;
        add(0, 0u, key);
      }
    }
  }
  beyond([&](uint32_t key) { add(0, 0u, key); });
  __syncthreads();
  PK1_SSTAMP(8);
  PK1_SSTAMP(9);
  pk1_digit<NB0, PK1_HSUB>(h, st, s0, ws);  // (ends with a barrier: h is free)
  PK1_SSTAMP(10);
  // the keys of the selected digit-0 bin (a small share of the candidates) compacted into LDS
  // (h[0] their count, h[1..] the keys relative to B) and ranked directly: the k_rem-th largest
  // of them is the threshold, k_rem minus the keys above it the ties to keep -- the threshold
  // and tie count digits 1 and 2 would give, without two more passes over every candidate
  const uint32_t rank_max = min((uint32_t)EW_BLOCK, g_pk_rank_max);
  uint32_t* lst = h + 4;  // (16-B aligned: read four keys at a time when ranking)
  uint32_t nbin = 0xffffffffu;
  const uint32_t k_rem = st[1];
  if (rank_max) {
    // count, scan, place: no atomics (a per-match atomic made each step a dependent round trip)
    const uint32_t want = st[0] >> s0;
    constexpr uint32_t CAP = NB0 * PK1_HSUB - 4;
    const uint4* k4 = reinterpret_cast<const uint4*>(keys);
    const uint32_t nq = (nl + 3u) >> 2;
    auto hit = [&](uint32_t key, uint32_t idx) -> uint32_t {
      return (idx < nl && ((key - B) >> s0) == want) ? 1u : 0u;
    };
    uint32_t cnt = 0;
    for (uint32_t q = threadIdx.x; q < nq; q += EW_BLOCK) {
      const uint4 x = k4[q];
      cnt += hit(x.x, 4 * q) + hit(x.y, 4 * q + 1) + hit(x.z, 4 * q + 2) + hit(x.w, 4 * q + 3);
    }
    uint32_t total;
    uint32_t pos = ew_block_excl_scan(cnt, ws, total);  // (its barriers: st read by all first)
    if (cnt) {
      for (uint32_t q = threadIdx.x; q < nq; q += EW_BLOCK) {
        const uint4 x = k4[q];
        const uint32_t kk[4] = {x.x, x.y, x.z, x.w};
#pragma unroll
        for (int e = 0; e < 4; ++e)
          if (hit(kk[e], 4 * q + e)) {
            if (pos < CAP) lst[pos] = kk[e] - B;
            ++pos;
          }
      }
    }
    nbin = total;
    if (M > nl) {  // (rare: the band keeps the candidates within the LDS copy)
      if (threadIdx.x == 0) h[0] = total;
      __syncthreads();
      beyond([&](uint32_t key) {
        const uint32_t rel = key - B;
        if ((rel >> s0) == want) {
          const uint32_t p = atomicAdd(&h[0], 1u);
          if (p < CAP) lst[p] = rel;
        }
      });
      __syncthreads();
      nbin = h[0];
    }
  }
  __syncthreads();  // the list complete; every thread holds k_rem before st is rewritten
  PK1_SSTAMP(12);
  if (stamp && threadIdx.x == 0) {  // (probe: the candidate count and the ranked bin's)
    stamp[14] = M;
    stamp[15] = nbin;
  }
  if (nbin <= rank_max) {
    if (threadIdx.x < nbin) {
      const uint32_t mine = lst[threadIdx.x];
      uint32_t gt = 0, eq = 0, j = 0;
      for (; j + 4 <= nbin; j += 4) {
        const uint4 x = *reinterpret_cast<const uint4*>(lst + j);
        gt += (uint32_t)(x.x > mine) + (uint32_t)(x.y > mine) + (uint32_t)(x.z > mine) +
              (uint32_t)(x.w > mine);
        eq += (uint32_t)(x.x == mine) + (uint32_t)(x.y == mine) + (uint32_t)(x.z == mine) +
              (uint32_t)(x.w == mine);
      }
      for (; j < nbin; ++j) {
        const uint32_t x = lst[j];
        gt += x > mine;
        eq += x == mine;
      }
      // (threads holding an equal key write the same two words)
      if (gt < k_rem && k_rem <= gt + eq) {
        st[0] = mine;
        st[1] = k_rem - gt;
      }
    }
    __syncthreads();
  } else {  // a crowded bin: the two remaining radix digits
    pass(1, st[0] >> s0);
    pk1_digit<NB1>(h, st, s1, ws);
    pass(2, st[0] >> s1);
    pk1_digit<NB2>(h, st, 0u, ws);
  }
  PK1_SSTAMP(11);
#undef PK1_SSTAMP
  if (threadIdx.x == 0) {
    st[0] += B;  // absolute threshold key
    __hip_atomic_store(state + t * 4, st[0], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_store(state + t * 4 + 1, st[1], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_store(state + t * 4 + 2, kmax, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
}

// the tensor's generation word moved to >= g (block-uniform; bounded poll, then an acquire)
__device__ __forceinline__ void pk1_wait(const uint32_t* gen, uint32_t g, int* err, uint32_t* s_gen) {
  pk_wait(gen, g, err, s_gen);
}

template <int EFM, int VK, bool EF>
__global__ __launch_bounds__(EW_BLOCK) void k_pk_one(
    GradPtrs gp, DgcArgs dg, unsigned long long* __restrict__ lb, float* __restrict__ resid,
    const ChunkRow* __restrict__ chunks, uint32_t* __restrict__ kmaxr, int T,
    const TensorRow* __restrict__ tensors, uint32_t* __restrict__ pst, int* __restrict__ tick,
    int* __restrict__ ccount, uint2* __restrict__ pcand, int* __restrict__ stats,
    uint32_t* __restrict__ state, int* __restrict__ cand_n, uint32_t* __restrict__ gen,
    uint32_t* __restrict__ mode, uint32_t* __restrict__ hist0, uint32_t* __restrict__ hist1,
    uint32_t* __restrict__ hist2, int* __restrict__ lb_err, uint8_t* __restrict__ payload,
    int scales_off, int idx_off, int codes_off, int bitmap_off, int counts_off, float levels,
    float inv_levels, uint32_t key_arg, const uint32_t* __restrict__ keyp, uint32_t bucket_offset,
    int lb_fault, uint32_t lds_keys, unsigned long long* __restrict__ stamps, TkApply ap) {
  extern __shared__ __attribute__((aligned(16))) uint32_t s_dyn[];  // select: histogram + staged
  // keys; full passes: histograms
  // stamps (probes, EWDML_PK1_STAMPS=1): thread 0 stamps wall_clock64() at the phase boundaries
#define PK1_STAMP(i) \
  if (stamps && threadIdx.x == 0) stamps[(size_t)blockIdx.x * PK1_NSTAMP + (i)] = wall_clock64()
  PK1_STAMP(0);
  __shared__ unsigned long long ws2[2 * EW_WAVES];
  __shared__ uint32_t wmax[EW_WAVES];
  __shared__ uint32_t ws[EW_WAVES];
  __shared__ uint32_t s_lb[2 * EW_WAVES];
  __shared__ uint32_t s_u[7];  // base of this chunk's candidates; tensor-last: fast, B, s0, s1, M,
                              // max key
  __shared__ uint32_t s_st[2];  // the select's {prefix, k_rem}
  __shared__ int s_flag;
  __shared__ uint32_t s_gen;
  const ChunkRow c = chunks[blockIdx.x];
  const int t = c.tensor;
  const TensorRow tr = tensors[t];
  uint32_t* gn = gen + TICK_STRIDE * t;
  int* arr = tick + TICK_STRIDE * (T + t);  // the full passes' arrival count
  // the generation moves only after every block of the tensor arrived: read before arriving
  const uint32_t g0 = __hip_atomic_load(gn, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  // this chunk's look-back word starts unpublished; its successors read it after the tensor's
  // select (they wait for the generation, which moves after this block arrived)
  if (threadIdx.x == 0)
    __hip_atomic_store(lb + blockIdx.x, 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  const uint32_t key = keyp ? *keyp : key_arg;
  ew_sgd_resolve(ap.sa);
  // the select's pass-0 sub-histograms zeroed while this block's staging loads are in flight
  // (any block may turn out to be its tensor's last; the barriers before the select order it)
  for (int i = threadIdx.x; i < NB0 * PK1_HSUB / 4; i += EW_BLOCK)
    reinterpret_cast<uint4*>(s_dyn)[i] = uint4{0u, 0u, 0u, 0u};
  // ---- 1. stage (error feedback) and compact the candidates (k_pk_hist0) ----
  float4 v[EW_CU];
  topk_load_stage<EFM>(gp, dg, resid, c, v);
  // the previous launch's prediction (and its steering state, for the tensor-last block)
  const uint32_t P = pst[t * 8], pbeta = pst[t * 8 + 1], phad = pst[t * 8 + 4];
  PK1_STAMP(1);
  uint32_t kmax = 0;
  unsigned long long pa = 0, pb = 0;
#pragma unroll
  for (int u = 0; u < EW_CU; ++u) {
    uint32_t n = 0;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      if (ew_chunk_idx(u) + j < c.len) {
        const uint32_t k = ew_key(ew_f4(v[u], j));
        kmax = max(kmax, k);
        n += k >= P;
      }
    }
    if (u < 4) pa |= (unsigned long long)n << (16 * u);
    else pb |= (unsigned long long)n << (16 * (u - 4));
  }
  kmax = ew_wave_max_u(kmax);
  if ((threadIdx.x & 63) == 0) wmax[threadIdx.x >> 6] = kmax;
  unsigned long long ta, tb;
  pk_scan2(pa, pb, ws2, ta, tb);
  uint32_t start[EW_CU];
  uint32_t run = 0;
#pragma unroll
  for (int u = 0; u < EW_CU; ++u) {
    start[u] = run;
    run += (uint32_t)(((u < 4 ? ta : tb) >> (16 * (u & 3))) & 0xffffull);
  }
  const uint32_t tot = run;
  if (threadIdx.x == 0) {
    uint32_t m = wmax[0];
    for (int w = 1; w < EW_WAVES; ++w) m = max(m, wmax[w]);
    atomicMax(&kmaxr[(blockIdx.x & (NREP - 1)) * T + t], m);
    s_u[0] = tot ? (uint32_t)atomicAdd(ccount + TICK_STRIDE * t, (int)tot) : 0u;
  }
  __syncthreads();
  const uint32_t cbase0 = s_u[0];
  if (tot) {
    uint2* dst = pcand + tr.cap0;
    const uint32_t cap = (uint32_t)tr.cap;
#pragma unroll
    for (int u = 0; u < EW_CU; ++u) {
      uint32_t pos = cbase0 + start[u] +
                     (uint32_t)(((u < 4 ? pa : pb) >> (16 * (u & 3))) & 0xffffull);
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int i = ew_chunk_idx(u) + j;
        const float x = ew_f4(v[u], j);
        if (i < c.len && ew_key(x) >= P) {
          if (pos < cap)
            __hip_atomic_store(reinterpret_cast<unsigned long long*>(dst + pos),
                               (unsigned long long)__float_as_uint(x) |
                                   ((unsigned long long)(c.local * EW_CHUNK + i) << 32),
                               __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          ++pos;
        }
      }
    }
  }
  // ---- 2. the tensor's select ----
  PK1_STAMP(2);
  unsigned long long pre0 = 0ull;  // (non-last blocks: the first candidate, loaded before the wait)
  bool have_pre = false;
  if (topk_tensor_last(tick + TICK_STRIDE * t, tr.nchunks, reinterpret_cast<int*>(wmax))) {
    PK1_STAMP(6);
    // every block of the tensor read its producer-staging stamp before arriving: re-arm it
    if (dg.stamps && threadIdx.x == 0) dg.stamps[t] = 0u;
    if (threadIdx.x == 0) {
      int* cc = ccount + TICK_STRIDE * t;
      // the candidate count and the max-key replicas: all loads in flight together
      uint32_t kr[NREP];
#pragma unroll
      for (int r = 0; r < NREP; ++r)
        kr[r] = __hip_atomic_load(kmaxr + r * T + t, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      const uint32_t M = (uint32_t)__hip_atomic_load(cc, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(cc, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      const uint32_t fast = M >= (uint32_t)tr.k && M <= (uint32_t)tr.cap;
      uint32_t B = 0u, s0 = 20u, s1 = 10u;
      if (fast) {
        uint32_t km = 0;
#pragma unroll
        for (int r = 0; r < NREP; ++r) km = max(km, kr[r]);
        s_u[6] = km;
        B = P;
        const uint32_t span = km - P;
        const int bl = span ? 32 - __clz(span) : 0;
        s0 = bl > 11 ? (uint32_t)(bl - 11) : 0u;
        s1 = s0 > 10 ? s0 - 10 : 0u;
      }
      // M is read back by the full passes' last block (maybe another block): agent-scope
      __hip_atomic_store(pst + t * 8 + 2, M, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      pst[t * 8 + 3] = fast;
      pst[t * 8 + 5] = B;
      pst[t * 8 + 6] = s0;
      pst[t * 8 + 7] = s1;
      atomicAdd(stats + (fast ? 0 : 1), 1);
      if (!fast && t < PK_MISS_T)  // per-tensor misses: too few candidates (1) / too many (2^16)
        atomicAdd(stats + 2 + t, M < (uint32_t)tr.k ? 1 : 65536);
      s_u[1] = fast;
      s_u[2] = B;
      s_u[3] = s0;
      s_u[4] = s1;
      s_u[5] = M;
    }
    __syncthreads();
    const uint32_t fast = s_u[1], M = s_u[5];
    if (fast) {
      pk1_select_cands(pcand + tr.cap0, M, s_u[2], s_u[3], s_u[4], s_u[6], (uint32_t)tr.k,
                       s_dyn + NB0 * PK1_HSUB, min(M, lds_keys), s_dyn, s_st, ws, state, t,
                       stamps ? stamps + (size_t)blockIdx.x * PK1_NSTAMP : nullptr);
    }
    if (threadIdx.x == 0)
      __hip_atomic_store(mode + TICK_STRIDE * t, fast, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    PK1_STAMP(7);
    pk_publish(arr, gn, g0 + 1u);  // (arr: zero already; rewritten to zero)
    if (fast && threadIdx.x == 0) {
      // the next launch's prediction, after the publish: no block of this launch reads these
      // words again (P, beta and had were read before the tensor's ticket; n before arriving;
      // the write takes the scale from the select state).  Candidates steered to 1.5 k ..
      // min(2.5 k, 7/8 of the LDS copy): the select's time grows with them, and its single
      // block is this launch's critical path.  Few-k tensors keep at least g_pk1_lo_keys (their
      // thresholds jump the most -- without error feedback LeNet's conv2 and fc2 missed ~1 step
      // in 4 -- and a few thousand keys cost their select next to nothing)
      // (without error feedback only: under EF the thresholds move smoothly, and the floor's
      // extra candidates cost the write ~2 us, profiles/ab/README.md)
      const uint32_t kk = (uint32_t)tr.k, lo_keys = EF ? 0u : g_pk1_lo_keys;
      const uint32_t hi = min(lds_keys - lds_keys / 8, max(kk * 2u + kk / 2u, 2u * lo_keys));
      pk_predict_thr(tr, t, s_st[0], pst, cand_n, M, 1u, pbeta, phad, hi,
                     max(kk + kk / 2u, min(lo_keys, hi / 2u)));
      for (int r = 0; r < NREP; ++r)  // dead once the max is in the select state
        __hip_atomic_store(kmaxr + r * T + t, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      PK1_STAMP(13);
    }
  } else {
    // this block's first candidates (written by it before the ticket), in flight during the wait
    have_pre = tot <= PK_WRITE_CANDS_MAX;  // (block-uniform)
    // (only entries inside the tensor's list: past its capacity -- a prediction that let too many
    // in -- nothing was stored, and the address may lie past the scratch)
    if (threadIdx.x < tot && have_pre && cbase0 + threadIdx.x < (uint32_t)tr.cap)
      pre0 = __hip_atomic_load(reinterpret_cast<const unsigned long long*>(
                                   pcand + tr.cap0 + cbase0 + threadIdx.x),
                               __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    pk1_wait(gn, g0 + 1u, lb_err, &s_gen);
  }
  __syncthreads();
  const bool fast = __hip_atomic_load(mode + TICK_STRIDE * t, __ATOMIC_RELAXED,
                                      __HIP_MEMORY_SCOPE_AGENT) != 0u;
  if (!fast) {
    // ---- 2'. the prediction missed: three radix passes over the tensor, every block over its
    // own registers (k_pk_select's full path: key bits [30:20], [19:10], [9:0]) ----
    constexpr int HSUB = 4;
    uint32_t* hs = s_dyn;
    auto flush = [&](uint32_t* dstrow, int nb, int sub) {
      __syncthreads();
      for (int i = threadIdx.x; i < nb; i += EW_BLOCK) {
        uint32_t x = 0;
        for (int q = 0; q < sub; ++q) x += hs[i * sub + q];
        if (x) atomicAdd(&dstrow[i], x);
      }
    };
    // pass 0
    for (int i = threadIdx.x; i < NB0 * HSUB; i += EW_BLOCK) hs[i] = 0;
    __syncthreads();
    {
      uint32_t* h = hs + (threadIdx.x & (HSUB - 1));
#pragma unroll
      for (int u = 0; u < EW_CU; ++u)
#pragma unroll
        for (int j = 0; j < 4; ++j)
          if (ew_chunk_idx(u) + j < c.len) atomicAdd(&h[(ew_key(ew_f4(v[u], j)) >> 20) * HSUB], 1u);
    }
    flush(hist0 + (size_t)t * NB0, NB0, HSUB);
    if (pk_arrive(arr, tr.nchunks, &s_flag)) {
      pk_select<NB0, true>(hist0, tensors, state, kmaxr, T, t, 20u);
      __syncthreads();
      for (int i = threadIdx.x; i < NB0; i += EW_BLOCK) hist0[(size_t)t * NB0 + i] = 0u;
      if (threadIdx.x < NREP)
        __hip_atomic_store(kmaxr + threadIdx.x * T + t, 0u, __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_AGENT);
      pk_publish(arr, gn, g0 + 2u);
    } else {
      pk1_wait(gn, g0 + 2u, lb_err, &s_gen);
    }
    // pass 1
    __syncthreads();
    uint32_t want = __hip_atomic_load(state + t * 4, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) >> 20;
    for (int i = threadIdx.x; i < NB1; i += EW_BLOCK) hs[i] = 0;
    __syncthreads();
#pragma unroll
    for (int u = 0; u < EW_CU; ++u)
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const uint32_t k = ew_key(ew_f4(v[u], j));
        if (ew_chunk_idx(u) + j < c.len && (k >> 20) == want) atomicAdd(&hs[(k >> 10) & 1023u], 1u);
      }
    flush(hist1 + (size_t)t * NB1, NB1, 1);
    if (pk_arrive(arr, tr.nchunks, &s_flag)) {
      pk_select<NB1, false>(hist1, tensors, state, kmaxr, T, t, 10u);
      __syncthreads();
      for (int i = threadIdx.x; i < NB1; i += EW_BLOCK) hist1[(size_t)t * NB1 + i] = 0u;
      pk_publish(arr, gn, g0 + 3u);
    } else {
      pk1_wait(gn, g0 + 3u, lb_err, &s_gen);
    }
    // pass 2
    __syncthreads();
    want = __hip_atomic_load(state + t * 4, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) >> 10;
    for (int i = threadIdx.x; i < NB2; i += EW_BLOCK) hs[i] = 0;
    __syncthreads();
#pragma unroll
    for (int u = 0; u < EW_CU; ++u)
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const uint32_t k = ew_key(ew_f4(v[u], j));
        if (ew_chunk_idx(u) + j < c.len && (k >> 10) == want) atomicAdd(&hs[k & 1023u], 1u);
      }
    flush(hist2 + (size_t)t * NB2, NB2, 1);
    if (pk_arrive(arr, tr.nchunks, &s_flag)) {
      pk_select<NB2, false>(hist2, tensors, state, kmaxr, T, t, 0u);
      __syncthreads();
      for (int i = threadIdx.x; i < NB2; i += EW_BLOCK) hist2[(size_t)t * NB2 + i] = 0u;
      if (threadIdx.x == 0) {
        const uint32_t M = __hip_atomic_load(pst + t * 8 + 2, __ATOMIC_RELAXED,
                                             __HIP_MEMORY_SCOPE_AGENT);
        const uint32_t thr = __hip_atomic_load(state + t * 4, __ATOMIC_RELAXED,
                                               __HIP_MEMORY_SCOPE_AGENT);  // (B = 0: absolute)
        pk_predict_thr(tr, t, thr, pst, cand_n, M, 0u, pbeta, phad);
      }
      pk_publish(arr, gn, g0 + 4u);
    } else {
      pk1_wait(gn, g0 + 4u, lb_err, &s_gen);
    }
    __syncthreads();
  }
  PK1_STAMP(3);
  if (ap.param && ap.mom) {  // dense apply: the chunk's accumulator in the (free) dynamic LDS
    ap.acc = reinterpret_cast<float*>(s_dyn);
    for (int i = threadIdx.x; i < EW_CHUNK; i += EW_BLOCK) ap.acc[i] = 0.0f;
    __syncthreads();
  }
  // ---- 3. the ordered write of this chunk ----
  const uint32_t thr = __hip_atomic_load(state + t * 4, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  const uint32_t need = __hip_atomic_load(state + t * 4 + 1, __ATOMIC_RELAXED,
                                          __HIP_MEMORY_SCOPE_AGENT);
  const float scale = __uint_as_float(__hip_atomic_load(state + t * 4 + 2, __ATOMIC_RELAXED,
                                                        __HIP_MEMORY_SCOPE_AGENT));
  float* velm = dg.mask ? dg.vel : nullptr;
  if (fast && tot <= PK_WRITE_CANDS_MAX) {
    topk_write_cands<VK, EF>(c, tr, resid, velm, state, payload, scales_off, idx_off, codes_off,
                             bitmap_off, counts_off, levels, inv_levels, key, bucket_offset, lb,
                             lb_err, tot, pcand + tr.cap0 + cbase0, ws, s_lb, lb_fault, thr, need,
                             scale, ap, have_pre,
                             make_uint2((uint32_t)pre0, (uint32_t)(pre0 >> 32)));
  } else {
    topk_write_lb<VK, EF>(c, tr, v, resid, velm, payload, scales_off, idx_off, codes_off,
                          bitmap_off, counts_off, levels, inv_levels, key, bucket_offset, lb,
                          lb_err, s_lb, ws, lb_fault, thr, need, scale, ap);
  }
  if (ap.acc) {  // dense apply over the chunk (its accumulator holds the sent values)
    __syncthreads();
    const float inv_n = ap.sa.grad_scale;
    float* p = ap.param + c.start;
    float* b = ap.mom + c.start;
    const int n4 = c.len >> 2;
    const float4* acc4 = reinterpret_cast<const float4*>(ap.acc);
    // every load of the thread's vectors in flight before the first step (k_topk_decode_apply's
    // dense pass: the same per-element arithmetic)
    float4 pv[EW_CU], bv[EW_CU];
#pragma unroll
    for (int u = 0; u < EW_CU; ++u) {
      const int i = threadIdx.x + u * EW_BLOCK;
      if (i < n4) {
        pv[u] = reinterpret_cast<const float4*>(p)[i];
        bv[u] = reinterpret_cast<const float4*>(b)[i];
      }
    }
#pragma unroll
    for (int u = 0; u < EW_CU; ++u) {
      const int i = threadIdx.x + u * EW_BLOCK;
      if (i >= n4) break;
      const float4 a = acc4[i];
      float4 pu = pv[u], bu = bv[u];
      ew_sgd(pu.x, bu.x, a.x * inv_n, ap.sa);
      ew_sgd(pu.y, bu.y, a.y * inv_n, ap.sa);
      ew_sgd(pu.z, bu.z, a.z * inv_n, ap.sa);
      ew_sgd(pu.w, bu.w, a.w * inv_n, ap.sa);
      reinterpret_cast<float4*>(p)[i] = pu;
      reinterpret_cast<float4*>(b)[i] = bu;
      if (ap.shadow) {
        const float v4[4] = {pu.x, pu.y, pu.z, pu.w};
        ew_st4_bf16(ap.shadow + c.start + 4 * i, 4, v4);
      }
    }
    for (int i = (n4 << 2) + threadIdx.x; i < c.len; i += EW_BLOCK) {
      float pq = p[i], bq = b[i];
      ew_sgd(pq, bq, ap.acc[i] * inv_n, ap.sa);
      p[i] = pq;
      b[i] = bq;
      if (ap.shadow) ap.shadow[c.start + i] = ew_f2bf(pq);
    }
  }
  tk_apply_done(ap);
  PK1_STAMP(4);
#undef PK1_STAMP
}

// Value of payload entry `pe` (fp32 value, or the int8 / int4 QSGD code as a float).
template <int VK>
__device__ __forceinline__ float ew_topk_code(const uint8_t* pay, int codes_off, uint32_t pe) {
  if (VK == VK_F32) return reinterpret_cast<const float*>(pay + codes_off)[pe];
  if (VK == VK_Q8) return (float)reinterpret_cast<const int8_t*>(pay + codes_off)[pe];
  const uint32_t b = pay[codes_off + (pe >> 1)];
  const int q = (int)((pe & 1u) ? (b >> 4) : (b & 0xfu));
  return (float)(q >= 8 ? q - 16 : q);
}

// Entry offset of this chunk inside each rank's payload: entry0 + the sum of the tensor's earlier
// chunk counts (a few hundred for the last chunks of a large tensor).  A wave takes ranks w and
// w + EW_WAVES together, every count load of both in flight before any is summed: one round trip
// for up to 2 * EW_WAVES = 8 ranks instead of one per group of 4.
__device__ __forceinline__ void topk_chunk_offsets(const uint8_t* __restrict__ recv, int nranks,
                                                   long long stride, int counts_off,
                                                   const ChunkRow& c, const TensorRow& tr,
                                                   uint32_t* s_off, int lane, int w) {
  for (int r = w; r < nranks; r += 2 * EW_WAVES) {
    const int r2 = r + EW_WAVES;
    const bool two = r2 < nranks;  // wave-uniform
    const uint16_t* cn1 = reinterpret_cast<const uint16_t*>(recv + r * stride + counts_off) + tr.chunk0;
    const uint16_t* cn2 = reinterpret_cast<const uint16_t*>(recv + (two ? r2 : r) * stride +
                                                            counts_off) + tr.chunk0;
    uint32_t s1 = 0, s2 = 0;
    for (int j0 = 0; j0 < c.local; j0 += 8 * 64) {
      uint32_t v1[8], v2[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        const int j = j0 + u * 64 + lane;
        v1[u] = j < c.local ? (uint32_t)cn1[j] : 0u;
        v2[u] = j < c.local ? (uint32_t)cn2[j] : 0u;
      }
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        s1 += v1[u];
        s2 += v2[u];
      }
    }
    s1 = ew_wave_sum_u(s1);
    s2 = ew_wave_sum_u(s2);
    if (lane == 0) {
      s_off[r] = (uint32_t)tr.entry0 + s1;
      if (two) s_off[r2] = (uint32_t)tr.entry0 + s2;
    }
  }
}

// Every rank's first list entry of this thread (e = thread index: all of a chunk's entries at
// <= 2.5 % density) for the first PR ranks, loaded before any is summed -- one round trip for all
// of them instead of one per rank -- plus each of those ranks' count and scale (any tensor kind),
// kept in registers for the rank-ordered sum.  Loads are clamped into the tensor's entry range and
// masked, not branched around (a branch makes the compiler wait for every load at its merge).
template <int VK, int PR>
__device__ __forceinline__ void topk_decode_prefetch(
    const uint8_t* __restrict__ recv, int nranks, long long stride, const ChunkRow& c,
    const TensorRow& tr, int scales_off, int counts_off, int idx_off, int codes_off,
    float inv_levels, const uint32_t* s_off, uint32_t eend, bool list, float (&pre_v)[PR],
    int (&pre_i)[PR], uint32_t (&pre_c)[PR], float (&pre_s)[PR]) {
#pragma unroll
  for (int r = 0; r < PR; ++r) {
    pre_i[r] = -1;
    pre_v[r] = 0.0f;
    pre_c[r] = 0u;
    pre_s[r] = 1.0f;
    if (r < nranks) {
      const uint8_t* pay = recv + r * stride;
      const uint32_t off = s_off[r];
      uint32_t cnt = reinterpret_cast<const uint16_t*>(pay + counts_off)[blockIdx.x];
      cnt = off >= eend ? 0u : min(cnt, eend - off);
      const float step = VK != VK_F32
          ? reinterpret_cast<const float*>(pay + scales_off)[c.tensor] * inv_levels : 1.0f;
      pre_c[r] = cnt;
      pre_s[r] = step;
      if (list) {
        const uint32_t e = threadIdx.x;
        const uint32_t pe = min(off + min(e, cnt ? cnt - 1u : 0u), eend - 1u);
        const float prod = ew_topk_code<VK>(pay, codes_off, pe) * step;
        const int i = reinterpret_cast<const uint16_t*>(pay + idx_off)[tr.idx0 + (pe - (uint32_t)tr.entry0)];
        if (e < cnt) {
          pre_v[r] = prod;
          pre_i[r] = i;
        }
      }
    }
  }
}

// Rank r's entry count in this chunk (clamped) and value step: from the prefetch registers for
// the first PR ranks, loaded otherwise.
template <int VK, int PR>
__device__ __forceinline__ void topk_decode_rank_cs(const uint8_t* pay, int r, const ChunkRow& c,
                                                    int counts_off, int scales_off,
                                                    float inv_levels, uint32_t off, uint32_t eend,
                                                    const uint32_t (&pre_c)[PR],
                                                    const float (&pre_s)[PR], uint32_t& cnt,
                                                    float& step) {
  if (r < PR) {
    cnt = 0u;
    step = 1.0f;
#pragma unroll
    for (int q = 0; q < PR; ++q)
      if (q == r) {
        cnt = pre_c[q];
        step = pre_s[q];
      }
    return;
  }
  cnt = reinterpret_cast<const uint16_t*>(pay + counts_off)[blockIdx.x];
  cnt = off >= eend ? 0u : min(cnt, eend - off);
  step = VK != VK_F32
      ? reinterpret_cast<const float*>(pay + scales_off)[c.tensor] * inv_levels : 1.0f;
}

// Receive side: one block per chunk.  Sum the N ranks' entries for this chunk in rank order in an
// LDS accumulator (indices are unique within a rank, so no atomics), scale by 1/N, then either
// write the averaged gradient and/or apply the SGD update to the chunk's parameters.
template <int VK>
__global__ __launch_bounds__(EW_BLOCK) void k_topk_decode_apply(
    const uint8_t* __restrict__ recv, int nranks, long long stride,
    const ChunkRow* __restrict__ chunks, const TensorRow* __restrict__ tensors, int scales_off,
    int counts_off, int idx_off, int codes_off, int bitmap_off, float inv_levels,
    float* __restrict__ param,
    float* __restrict__ mom, float* __restrict__ grad_out, uint16_t* __restrict__ shadow,
    SgdArgs sa, int apply) {
  __shared__ float4 acc4[EW_CHUNK / 4];
  ew_sgd_resolve(sa);
  __shared__ uint32_t s_off[EW_MAX_RANKS];
  __shared__ uint32_t ws[EW_WAVES];
  float* acc = reinterpret_cast<float*>(acc4);
  const ChunkRow c = chunks[blockIdx.x];
  const TensorRow tr = tensors[c.tensor];
  float* p = param + c.start;
  float* b = mom ? mom + c.start : nullptr;
  // chunk starts are 64-element aligned: float4 body + scalar tail.  The body's parameters and
  // momenta are loaded here, before the scatter, so their latency hides behind it.
  const int n4 = c.len >> 2;
  float4 pv[EW_CU], bv[EW_CU];
  // mom == nullptr: a step without momentum buffer (momentum-corrected error feedback ran the
  // momentum on the sender; the host passes momentum = 0)
  const bool has_mom = mom != nullptr;
  // SPARSE: a step with neither momentum nor weight decay (momentum-corrected error feedback ran
  // both on the sender) changes a parameter only where the averaged gradient is non-zero -- p -
  // lr * (+0) is p bit for bit -- so only the touched float4s are read and written (~1 % of the
  // elements at top-1 %: a fraction of the bucket's cache lines instead of all of them)
  const bool sparse = apply && !has_mom && sa.momentum == 0.0f && sa.weight_decay == 0.0f &&
                      grad_out == nullptr;
  if (apply && !sparse) {
#pragma unroll
    for (int u = 0; u < EW_CU; ++u) {
      const int i = threadIdx.x + u * EW_BLOCK;
      if (i < n4) {
        pv[u] = reinterpret_cast<const float4*>(p)[i];
        bv[u] = has_mom ? reinterpret_cast<const float4*>(b)[i] : make_float4(0.f, 0.f, 0.f, 0.f);
      }
    }
  }
  ew_key_advance(sa);
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  for (int i = threadIdx.x; i < (c.len + 3) / 4; i += EW_BLOCK) acc4[i] = make_float4(0.f, 0.f, 0.f, 0.f);
  // entry offset of this chunk inside each rank's payload: entry0 + sum of earlier chunk counts
  // (a wave per rank; each lane's loads of up to 8 counts are all in flight before the sum: the
  // tensor's last chunks sum a few hundred counts, a dependent round trip per 64 otherwise)
  topk_chunk_offsets(recv, nranks, stride, counts_off, c, tr, s_off, lane, w);
  __syncthreads();
  // Index-list tensors: every rank's first entry of this thread (e = thread index: all of a chunk's
  // entries at <= 2.5 % density) is loaded for the first PR ranks before any is summed -- one
  // round trip for all ranks instead of one per rank -- then the rank-ordered LDS sum below
  // consumes them (same order, same bits).  Loads are clamped into the tensor's entry range and
  // masked, not branched around (a branch makes the compiler wait for every load at its merge).
  constexpr int PR = 8;
  const uint32_t eend = (uint32_t)(tr.entry0 + tr.k);  // never read past the tensor's entries
  float pre_v[PR], pre_s[PR];
  int pre_i[PR];
  uint32_t pre_c[PR];
  const bool list = tr.bm0 < 0;
  topk_decode_prefetch<VK, PR>(recv, nranks, stride, c, tr, scales_off, counts_off, idx_off,
                               codes_off, inv_levels, s_off, eend, list, pre_v, pre_i, pre_c,
                               pre_s);
  for (int r = 0; r < nranks; ++r) {
    const uint8_t* pay = recv + r * stride;
    const uint32_t off = s_off[r];
    // clamped to the tensor's entry range (a corrupted payload must not read out of bounds);
    // the first PR ranks' count and scale were loaded with the prefetch
    uint32_t cnt;
    float step;
    topk_decode_rank_cs<VK, PR>(pay, r, c, counts_off, scales_off, inv_levels, off, eend, pre_c,
                                pre_s, cnt, step);
    if (list && r < PR) {  // the prefetched first entry, then any beyond the block's width
#pragma unroll
      for (int q = 0; q < PR; ++q)
        if (q == r && pre_i[q] >= 0 && pre_i[q] < c.len) acc[pre_i[q]] = acc[pre_i[q]] + pre_v[q];
      if (cnt > (uint32_t)EW_BLOCK) {
        const uint16_t* idx = reinterpret_cast<const uint16_t*>(pay + idx_off) + tr.idx0 +
                              (off - (uint32_t)tr.entry0);
        for (uint32_t e = threadIdx.x + EW_BLOCK; e < cnt; e += EW_BLOCK) {
          const float prod = ew_topk_code<VK>(pay, codes_off, off + e) * step;
          const int i = idx[e];
          if (i < c.len) acc[i] = acc[i] + prod;
        }
      }
    } else if (tr.bm0 >= 0) {
      // bitmap-indexed tensor: thread t owns word t of the chunk (256 words = 8192 elements);
      // a block scan of the popcounts gives each word's first entry
      const uint32_t* bw = reinterpret_cast<const uint32_t*>(pay + bitmap_off) + tr.bm0 +
                           c.local * EW_BM_WORDS;
      uint32_t word = (int)threadIdx.x * 32 < c.len ? bw[threadIdx.x] : 0u;
      uint32_t tot;
      uint32_t e = ew_block_excl_scan((uint32_t)__popc(word), ws, tot);
      while (word) {
        const int b = __ffs(word) - 1;
        word &= word - 1u;
        const int i = (int)threadIdx.x * 32 + b;
        if (e < cnt && i < c.len) acc[i] = acc[i] + ew_topk_code<VK>(pay, codes_off, off + e) * step;
        ++e;
      }
    } else {
      const uint16_t* idx = reinterpret_cast<const uint16_t*>(pay + idx_off) + tr.idx0 +
                            (off - (uint32_t)tr.entry0);
      for (uint32_t e = threadIdx.x; e < cnt; e += EW_BLOCK) {
        const float prod = ew_topk_code<VK>(pay, codes_off, off + e) * step;
        const int i = idx[e];
        if (i < c.len) acc[i] = acc[i] + prod;
      }
    }
    __syncthreads();
  }
  const float inv_n = sa.grad_scale;
  float* go = grad_out ? grad_out + c.start : nullptr;
#pragma unroll
  for (int u = 0; u < EW_CU; ++u) {
    const int i = threadIdx.x + u * EW_BLOCK;
    if (i >= n4) break;
    const float4 a = acc4[i];
    const float4 gv = make_float4(a.x * inv_n, a.y * inv_n, a.z * inv_n, a.w * inv_n);
    if (go) reinterpret_cast<float4*>(go)[i] = gv;
    if (sparse && a.x == 0.0f && a.y == 0.0f && a.z == 0.0f && a.w == 0.0f) continue;
    if (apply) {
      float4 pu = sparse ? reinterpret_cast<const float4*>(p)[i] : pv[u];
      float4 bu = sparse ? make_float4(0.f, 0.f, 0.f, 0.f) : bv[u];
      ew_sgd(pu.x, bu.x, gv.x, sa);
      ew_sgd(pu.y, bu.y, gv.y, sa);
      ew_sgd(pu.z, bu.z, gv.z, sa);
      ew_sgd(pu.w, bu.w, gv.w, sa);
      reinterpret_cast<float4*>(p)[i] = pu;
      if (has_mom) reinterpret_cast<float4*>(b)[i] = bu;
      if (shadow) {  // bf16 compute copy of the updated master weights
        const float v4[4] = {pu.x, pu.y, pu.z, pu.w};
        ew_st4_bf16(shadow + c.start + 4 * i, 4, v4);
      }
    }
  }
  for (int i = (n4 << 2) + threadIdx.x; i < c.len; i += EW_BLOCK) {
    const float gv = acc[i] * inv_n;
    if (go) go[i] = gv;
    if (apply && !(sparse && acc[i] == 0.0f)) {
      float pv = p[i], bv = has_mom ? b[i] : 0.0f;
      ew_sgd(pv, bv, gv, sa);
      p[i] = pv;
      if (has_mom) b[i] = bv;
      if (shadow) shadow[c.start + i] = ew_f2bf(pv);
    }
  }
}

// The SPARSE step of k_topk_decode_apply (no momentum buffer, no weight decay, no averaged
// gradient out: only touched float4s change) in its own kernel sized for one round of blocks: no
// parameter / momentum prefetch registers, and the LDS accumulator holds half a chunk -- the
// chunk's two halves are summed and applied one after the other from the same entry loads (the
// index-list entries are prefetched once and filtered per half).  16 KB of LDS and no prefetch:
// >= 5 blocks per CU instead of 4, so a VGG-11 bucket's ~1200 chunk blocks run in one round.
// Sums are per element in rank order from +0, as in k_topk_decode_apply: the same bits.
template <int VK>
__global__ __launch_bounds__(EW_BLOCK) void k_topk_decode_sparse(
    const uint8_t* __restrict__ recv, int nranks, long long stride,
    const ChunkRow* __restrict__ chunks, const TensorRow* __restrict__ tensors, int scales_off,
    int counts_off, int idx_off, int codes_off, int bitmap_off, float inv_levels,
    float* __restrict__ param, uint16_t* __restrict__ shadow, SgdArgs sa) {
  constexpr int HALF = EW_CHUNK / 2;
  __shared__ float4 acc4[HALF / 4];
  __shared__ uint32_t s_off[EW_MAX_RANKS];
  __shared__ uint32_t ws[EW_WAVES];
  float* acc = reinterpret_cast<float*>(acc4);
  ew_sgd_resolve(sa);
  ew_key_advance(sa);
  const ChunkRow c = chunks[blockIdx.x];
  const TensorRow tr = tensors[c.tensor];
  float* p = param + c.start;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  topk_chunk_offsets(recv, nranks, stride, counts_off, c, tr, s_off, lane, w);
  __syncthreads();
  constexpr int PR = 8;
  const uint32_t eend = (uint32_t)(tr.entry0 + tr.k);  // never read past the tensor's entries
  float pre_v[PR], pre_s[PR];
  int pre_i[PR];
  uint32_t pre_c[PR];
  const bool list = tr.bm0 < 0;
  topk_decode_prefetch<VK, PR>(recv, nranks, stride, c, tr, scales_off, counts_off, idx_off,
                               codes_off, inv_levels, s_off, eend, list, pre_v, pre_i, pre_c,
                               pre_s);
  for (int lo = 0; lo < c.len; lo += HALF) {  // block-uniform
    const int hl = min(c.len - lo, HALF);
    if (lo) __syncthreads();  // the previous half's apply has read the accumulator
    for (int i = threadIdx.x; i < (hl + 3) / 4; i += EW_BLOCK) acc4[i] = make_float4(0.f, 0.f, 0.f, 0.f);
    __syncthreads();
    for (int r = 0; r < nranks; ++r) {
      const uint8_t* pay = recv + r * stride;
      const uint32_t off = s_off[r];
      uint32_t cnt;
      float step;
      topk_decode_rank_cs<VK, PR>(pay, r, c, counts_off, scales_off, inv_levels, off, eend, pre_c,
                                  pre_s, cnt, step);
      if (list && r < PR) {
#pragma unroll
        for (int q = 0; q < PR; ++q) {
          const int i = pre_i[q] - lo;
          if (q == r && pre_i[q] >= 0 && i >= 0 && i < hl) acc[i] = acc[i] + pre_v[q];
        }
        if (cnt > (uint32_t)EW_BLOCK) {
          const uint16_t* idx = reinterpret_cast<const uint16_t*>(pay + idx_off) + tr.idx0 +
                                (off - (uint32_t)tr.entry0);
          for (uint32_t e = threadIdx.x + EW_BLOCK; e < cnt; e += EW_BLOCK) {
            const int i = (int)idx[e] - lo;
            if (i >= 0 && i < hl) acc[i] = acc[i] + ew_topk_code<VK>(pay, codes_off, off + e) * step;
          }
        }
      } else if (!list) {
        // bitmap: thread t owns word t (elements 32t..32t+31); the scan runs over the whole chunk
        // (it gives each word's first entry), the adds only for the words of this half
        const uint32_t* bw = reinterpret_cast<const uint32_t*>(pay + bitmap_off) + tr.bm0 +
                             c.local * EW_BM_WORDS;
        uint32_t word = (int)threadIdx.x * 32 < c.len ? bw[threadIdx.x] : 0u;
        uint32_t tot;
        uint32_t e = ew_block_excl_scan((uint32_t)__popc(word), ws, tot);
        if ((int)threadIdx.x * 32 < lo || (int)threadIdx.x * 32 >= lo + hl) word = 0u;
        while (word) {
          const int b = __ffs(word) - 1;
          word &= word - 1u;
          const int i = (int)threadIdx.x * 32 + b - lo;
          if (e < cnt && i < hl) acc[i] = acc[i] + ew_topk_code<VK>(pay, codes_off, off + e) * step;
          ++e;
        }
      } else {
        const uint16_t* idx = reinterpret_cast<const uint16_t*>(pay + idx_off) + tr.idx0 +
                              (off - (uint32_t)tr.entry0);
        for (uint32_t e = threadIdx.x; e < cnt; e += EW_BLOCK) {
          const int i = (int)idx[e] - lo;
          if (i >= 0 && i < hl) acc[i] = acc[i] + ew_topk_code<VK>(pay, codes_off, off + e) * step;
        }
      }
      __syncthreads();
    }
    const float inv_n = sa.grad_scale;
    float* ph = p + lo;
    const int n4 = hl >> 2;
    for (int i = threadIdx.x; i < n4; i += EW_BLOCK) {
      const float4 a = acc4[i];
      if (a.x == 0.0f && a.y == 0.0f && a.z == 0.0f && a.w == 0.0f) continue;
      float4 pu = reinterpret_cast<const float4*>(ph)[i];
      float bz = 0.0f;
      ew_sgd(pu.x, bz, a.x * inv_n, sa);
      bz = 0.0f;
      ew_sgd(pu.y, bz, a.y * inv_n, sa);
      bz = 0.0f;
      ew_sgd(pu.z, bz, a.z * inv_n, sa);
      bz = 0.0f;
      ew_sgd(pu.w, bz, a.w * inv_n, sa);
      reinterpret_cast<float4*>(ph)[i] = pu;
      if (shadow) {
        const float v4[4] = {pu.x, pu.y, pu.z, pu.w};
        ew_st4_bf16(shadow + c.start + lo + 4 * i, 4, v4);
      }
    }
    for (int i = (n4 << 2) + threadIdx.x; i < hl; i += EW_BLOCK) {
      if (acc[i] == 0.0f) continue;
      float pv = ph[i], bz = 0.0f;
      ew_sgd(pv, bz, acc[i] * inv_n, sa);
      ph[i] = pv;
      if (shadow) shadow[c.start + lo + i] = ew_f2bf(pv);
    }
  }
}

}  // namespace

// ---------------------------------------------------------------------------------------------
// host launchers
// ---------------------------------------------------------------------------------------------
#define EW_LAUNCH(kern, grid, stream, ...) \
  hipLaunchKernelGGL(kern, dim3(grid), dim3(EW_BLOCK), 0, (hipStream_t)(stream), __VA_ARGS__)

// Largest candidate-pass grid launched as the fused select kernel (its per-tensor barriers wait
// for peers of the same launch, so every block must become resident).  One block per CU, and only
// when the occupancy API reports room for at least two per CU: the API can read one block per CU
// high for some SGPR counts (MI355X_MICROARCH.md, correctness boundaries), so two leave the one
// we use even then.  Kernels sharing the GPU (a concurrent graph branch) delay blocks, they cannot
// strand them: they do not wait on this launch, so they drain and free their CUs
// (tests/kernels/test_hip_codecs.py::test_fused_select_beside_a_long_gemm); a barrier that still
// gives up counts a failure, which codec_health raises and the next payload's NaN scale makes
// visible on every rank (topk_pub_scale).  No cooperative launch: the step graph captures this
// kernel, and the graph path does not enforce co-residency either.  EWDML_TOPK_FUSED_SELECT=0:
// always the three pass kernels.
static int ew_pk_fused_max_blocks() {
  static int n = -1;
  if (n < 0) {
    const char* e = std::getenv("EWDML_TOPK_FUSED_SELECT");
    int dev = 0, cus = 0, occ = 0;
    EW_CHECK(hipGetDevice(&dev));
    EW_CHECK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
    EW_CHECK(hipOccupancyMaxActiveBlocksPerMultiprocessor(
        &occ, reinterpret_cast<const void*>(&k_pk_select), EW_BLOCK, 0));
    n = ((e && e[0] == '0') || occ < 2) ? 0 : cus;
  }
  return n;
}

int ew_topk_fused_select_max_blocks() { return ew_pk_fused_max_blocks(); }

// dynamic LDS of k_pk_one: the select's histogram + staged keys, or the full passes' histograms
constexpr size_t PK1_DYN_BYTES = 4 * (size_t)(NB0 * PK1_HSUB + PK1_LDS_KEYS);

// Largest bucket (in chunks) encoded by the one-launch kernel k_pk_one: its per-tensor waits and
// look-backs wait for peers of the same launch, so every block must be resident -- one block per
// CU, and only when the occupancy API reports room for two (as ew_pk_fused_max_blocks).
// EWDML_TOPK_ONE=0: never (the three launches).
static int ew_pk_one_max_blocks() {
  static int n = -1;
  if (n < 0) {
    const char* e = std::getenv("EWDML_TOPK_ONE");
    int dev = 0, cus = 0, occ = 0;
    EW_CHECK(hipGetDevice(&dev));
    EW_CHECK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
    EW_CHECK(hipOccupancyMaxActiveBlocksPerMultiprocessor(
        &occ, reinterpret_cast<const void*>(&k_pk_one<EF_DGC, VK_Q8, true>), EW_BLOCK,
        PK1_DYN_BYTES));
    n = ((e && e[0] == '0') || occ < 2) ? 0 : cus;
  }
  return n;
}

int ew_topk_one_max_blocks() { return ew_pk_one_max_blocks(); }

// EWDML_PK1_STAMPS=1 (probes): k_pk_one's per-block phase stamps, 16 u64 per block, of the last
// launch (tools/probes/encode_probe.py reads them with topk_one_stamps)
static unsigned long long* g_pk1_stamps = nullptr;
static int g_pk1_stamp_blocks = 0;
static unsigned long long* ew_pk1_stamps(int C) {
  static const bool on = [] {
    const char* e = std::getenv("EWDML_PK1_STAMPS");
    return e && e[0] == '1';
  }();
  if (!on) return nullptr;
  if (C > g_pk1_stamp_blocks) {
    if (g_pk1_stamps) EW_CHECK(hipFree(g_pk1_stamps));
    EW_CHECK(hipMalloc(&g_pk1_stamps, (size_t)C * PK1_NSTAMP * sizeof(unsigned long long)));
    EW_CHECK(hipMemset(g_pk1_stamps, 0, (size_t)C * PK1_NSTAMP * sizeof(unsigned long long)));
    g_pk1_stamp_blocks = C;
  }
  return g_pk1_stamps;
}

std::vector<unsigned long long> ew_topk_one_stamps() {
  std::vector<unsigned long long> out((size_t)g_pk1_stamp_blocks * PK1_NSTAMP);
  if (g_pk1_stamps) {
    EW_CHECK(hipDeviceSynchronize());
    EW_CHECK(hipMemcpy(out.data(), g_pk1_stamps, out.size() * 8, hipMemcpyDeviceToHost));
  }
  return out;
}

// Most candidates a tensor may have for k_pk_hist0's tensor-last block to select over them itself
static uint32_t ew_pk_inline_max() {
  static long long n = -1;
  if (n < 0) {
    const char* e = std::getenv("EWDML_TOPK_INLINE");
    n = e ? std::atoll(e) : (long long)PK_INLINE_MAX;
    if (n < 0) n = 0;
  }
  return (uint32_t)n;
}

static void ew_pk_band_init() {
  static bool done = false;
  if (done) return;
  done = true;
  const char* e = std::getenv("EWDML_PK_BAND");
  if (!e) return;
  uint32_t q[2] = {8u, 0u};
  if (std::sscanf(e, "%u,%u", &q[0], &q[1]) < 1) return;
  EW_CHECK(hipMemcpyToSymbol(HIP_SYMBOL(g_pk_band_q), q, sizeof(q)));
}

static void ew_pk1_lo_init() {
  static bool done = false;
  if (done) return;
  done = true;
  const char* e = std::getenv("EWDML_PK1_LO");
  if (!e) return;
  const uint32_t v = (uint32_t)std::atol(e);
  EW_CHECK(hipMemcpyToSymbol(HIP_SYMBOL(g_pk1_lo_keys), &v, sizeof(v)));
}

static void ew_pk_rank_init() {
  static bool done = false;
  if (done) return;
  done = true;
  const char* e = std::getenv("EWDML_PK_RANK");
  if (!e || e[0] != '0') return;
  const uint32_t z = 0u;
  EW_CHECK(hipMemcpyToSymbol(HIP_SYMBOL(g_pk_rank_max), &z, sizeof(z)));
}

void ew_topk_encode(const TopkEncodeArgs& a) {
  ew_pk_band_init();
  ew_pk_rank_init();
  ew_pk1_lo_init();
  auto* chunks = reinterpret_cast<const ChunkRow*>(a.chunks);
  auto* tensors = reinterpret_cast<const TensorRow*>(a.tensors);
  auto* scratch = reinterpret_cast<uint8_t*>(a.scratch);
  const int T = a.num_tensors, C = a.num_chunks;
  // scratch layout (all zeroed at once): state[T*4] | kmaxr[NREP*T] | hist0[NREP*T*NB0]
  // | hist1[NREP*T*NB1] | hist2[NREP*T*NB2] | cnt_gt[C] | cnt_eq[C] | chunk_off[C]
  // | chunk_ties[C] | chunk_sq[C] | inv[T] | tickets[4*T]
  uint32_t* state = reinterpret_cast<uint32_t*>(scratch);
  uint32_t* kmaxr = state + 4 * T;
  uint32_t* hist0 = kmaxr + NREP * T;
  uint32_t* hist1 = hist0 + (size_t)NREP * T * NB0;
  uint32_t* hist2 = hist1 + (size_t)NREP * T * NB1;
  uint32_t* cnt_gt = hist2 + (size_t)NREP * T * NB2;
  uint32_t* cnt_eq = cnt_gt + C;
  uint32_t* chunk_off = cnt_eq + C;
  uint32_t* chunk_ties = chunk_off + C;
  float* chunk_sq = reinterpret_cast<float*>(chunk_ties + C);
  float* inv = chunk_sq + C;
  // [4][T] per-pass tensor tickets, one 128-B line each (blocks of different tensors must not
  // serialise on one line's atomics), then [T] candidate counts (same stride), the look-back error
  // counter, the look-back words u64[C] and the candidate keys u32[L]
  int* tick = reinterpret_cast<int*>(
      (reinterpret_cast<uintptr_t>(inv + T) + TICK_STRIDE * 4 - 1) & ~(uintptr_t)(TICK_STRIDE * 4 - 1));
  int* cand_n = tick + 4 * TICK_STRIDE * T;
  int* lb_err = cand_n + TICK_STRIDE * T;
  int* pk_stats = lb_err + 2;  // predictive encode: tensor-encodes on the fast / full path
  // the write-pass apply's grid arrival ticket (ew_grid_last: 9 lines, left zeroed)
  int* apply_ticket = lb_err + TICK_STRIDE;
  auto* lb = reinterpret_cast<unsigned long long*>(apply_ticket + 9 * TICK_STRIDE);
  uint32_t* cand = reinterpret_cast<uint32_t*>(lb + C);
  if (a.bucket_len <= 0) throw std::runtime_error("ewdml topk: bucket length missing");
  // predictive encode state after the candidate keys: pstate u32[8 T] | chunk candidate base and
  // count u32[C] each | candidate counters [T] (one line each) | candidate list u64[total_cap]
  uint32_t* pst = cand + a.bucket_len;
  uint32_t* cbase = pst + 8 * T;
  uint32_t* ccnt = cbase + C;
  int* ccount = reinterpret_cast<int*>(ccnt + C);
  auto* pcand = reinterpret_cast<uint2*>(
      (reinterpret_cast<uintptr_t>(ccount + TICK_STRIDE * T) + 15) & ~(uintptr_t)15);
  hipStream_t s = (hipStream_t)a.stream;
  // no scratch memset: state / count sections are fully rewritten each encode, and the histogram
  // replicas are cleared by k_topk_write for the next one (zero-initialised at allocation)
  const uint32_t rezero_words = (uint32_t)((size_t)NREP * T * (1 + NB0 + NB1 + NB2));
  if (a.value_kind == VK_Q4)  // nibbles are OR-ed in; every other section is fully overwritten
    EW_CHECK(hipMemsetAsync(reinterpret_cast<void*>(a.payload), 0, a.payload_bytes, s));
  GradPtrs g;
  ew_fill_ptrs(g, a.grad_ptrs, a.n_grad_ptrs, T, a.bf16_mask, a.n_bf16_mask);
  float* resid = reinterpret_cast<float*>(a.resid);
  const float* src_flat = resid;  // passes after hist0 read the staged e = g + r under EF
  // each pass's per-tensor step (select / scan) runs in the tensor's last-arriving chunk block
  DgcArgs dg{reinterpret_cast<float*>(a.vel), reinterpret_cast<const float*>(a.param),
             a.dgc_momentum, a.dgc_damp1, a.dgc_wd, a.dgc_nesterov, a.dgc_mask,
             reinterpret_cast<const float*>(a.dgc_lr_ptr),
             reinterpret_cast<uint32_t*>(a.dgc_stamps)};
  if (dg.stamps && !dg.vel)
    throw std::runtime_error("ewdml topk: producer-staging stamps need momentum correction");
  if (dg.vel && !resid) throw std::runtime_error("ewdml topk: momentum correction needs a residual");
  if (dg.vel && dg.wd != 0.0f && !dg.param)
    throw std::runtime_error("ewdml topk: weight decay in the momentum correction needs params");
  auto* pay = reinterpret_cast<uint8_t*>(a.payload);
  const bool pk = a.predict && !a.norm_l2 && a.cblocks && a.num_cblocks > 0;
  TkApply ap{};
  if (a.apply_param) {
    if (!pk) throw std::runtime_error("ewdml topk: the write-pass apply needs the predictive encode");
    ap.param = reinterpret_cast<float*>(a.apply_param);
    ap.shadow = reinterpret_cast<uint16_t*>(a.apply_shadow);
    ap.sa.lr = a.apply_lr;
    ap.sa.lr_ptr = reinterpret_cast<const float*>(a.apply_lr_ptr);
    ap.sa.grad_scale = a.apply_scale;
    ap.sa.key_state = reinterpret_cast<uint32_t*>(a.apply_key_state);
    ap.sa.key_seed = a.apply_key_seed;
    ap.sa.key_rank = a.apply_key_rank;
    ap.ticket = apply_ticket;
    if (a.apply_mom_set) {  // receiver-side momentum SGD: the dense pass (k_pk_one only)
      ap.mom = reinterpret_cast<float*>(a.apply_mom);
      ap.sa.momentum = a.apply_momentum;
      ap.sa.dampening = a.apply_dampening;
      ap.sa.weight_decay = a.apply_wd;
      ap.sa.nesterov = a.apply_nesterov;
      ap.sa.first = a.apply_first;
      if (!ap.mom) throw std::runtime_error("ewdml topk: dense apply needs the momentum buffer");
      if (!(pk && C <= ew_pk_one_max_blocks()))
        throw std::runtime_error("ewdml topk: the dense write-pass apply runs in k_pk_one only");
    }
  }
  if (pk) {
    // predictive path: hist0 (+ candidates) -> 3 radix passes over the candidates -> write.
    // Its passes use histogram copy 0 only: kmaxr + hist0's copy 0 are one range, hist1's and
    // hist2's copies 0 two more (0.6 MB for VGG-11 instead of 5 MB of zeroing per encode)
    const uint32_t pk_rz0 = (uint32_t)(NREP * T + T * NB0);
    // in-hist0 selects only when every tensor's candidates can fit one block (the encode steers
    // them to ~2-3 k): then the select launch's blocks all exit at once.  With any larger tensor
    // the select launch keeps its barriers anyway, and inline selects would only lengthen hist0.
    const uint32_t inline_max =
        (a.max_k > 0 && 4LL * a.max_k <= (long long)ew_pk_inline_max()) ? ew_pk_inline_max() : 0u;
    auto* cbl = reinterpret_cast<const CBlockRow*>(a.cblocks);
    const int G = a.num_cblocks;
    if (C <= ew_pk_one_max_blocks()) {
      // small bucket: stage, select and write in ONE launch (k_pk_one)
      uint32_t* gen1 = reinterpret_cast<uint32_t*>(tick + 2 * TICK_STRIDE * T);
      uint32_t* mode1 = reinterpret_cast<uint32_t*>(tick + 3 * TICK_STRIDE * T);
#define EW_PK1(EFM, VK, EFV)                                                                     \
  hipLaunchKernelGGL((k_pk_one<EFM, VK, EFV>), dim3(C), dim3(EW_BLOCK), PK1_DYN_BYTES, s, g, dg,  \
                     lb, resid, chunks, kmaxr, T, tensors, pst, tick, ccount, pcand, pk_stats,    \
                     state, cand_n, gen1, mode1, hist0, hist1, hist2, lb_err, pay, a.scales_off,   \
                     a.idx_off, a.codes_off, a.bitmap_off, a.counts_off, a.levels, a.inv_levels,  \
                     a.key, reinterpret_cast<const uint32_t*>(a.key_ptr), a.bucket_offset,         \
                     a.lb_fault, (uint32_t)PK1_LDS_KEYS, ew_pk1_stamps(C), ap)
#define EW_PK1_VK(EFM, EFV)                                                                      \
  if (a.value_kind == VK_Q8) EW_PK1(EFM, VK_Q8, EFV);                                            \
  else if (a.value_kind == VK_Q4) EW_PK1(EFM, VK_Q4, EFV);                                       \
  else EW_PK1(EFM, VK_F32, EFV)
      if (dg.vel) { EW_PK1_VK(EF_DGC, true); }
      else if (resid) { EW_PK1_VK(EF_PLAIN, true); }
      else { EW_PK1_VK(EF_NONE, false); }
#undef EW_PK1_VK
#undef EW_PK1
      EW_CHECK_LAUNCH();
      return;
    }
#define EW_PKH(EFM)                                                                              \
  EW_LAUNCH(k_pk_hist0<EFM>, C, s, g, dg, lb, resid, chunks, kmaxr, T, tensors, pst, tick, ccount, \
            cbase, ccnt, pcand, pk_stats, state, cand_n, inline_max)
#define EW_PKH_W(EFM, WPE)                                                                       \
  EW_LAUNCH((k_pk_hist0<EFM, WPE>), C, s, g, dg, lb, resid, chunks, kmaxr, T, tensors, pst, tick,  \
            ccount, cbase, ccnt, pcand, pk_stats, state, cand_n, inline_max)
    static const int h0_wpe = [] {  // EWDML_PK_H0_WPE=4|5: DGC hist0 held to that occupancy (A/B)
      const char* e = getenv("EWDML_PK_H0_WPE");
      return e ? atoi(e) : 0;
    }();
    if (dg.vel && h0_wpe == 5) EW_PKH_W(EF_DGC, 5);
    else if (dg.vel && h0_wpe == 4) EW_PKH_W(EF_DGC, 4);
    else if (dg.vel) EW_PKH(EF_DGC);
    else if (resid) EW_PKH(EF_PLAIN);
    else EW_PKH(EF_NONE);
#undef EW_PKH
#undef EW_PKH_W
    if (G <= ew_pk_fused_max_blocks()) {
      // one launch for the three passes (per-tensor barriers; every block resident at once)
      EW_LAUNCH(k_pk_select, G, s, g, src_flat, chunks, cbl, tensors, pst, pcand, hist0, hist1,
                hist2, kmaxr, state, T, tick + TICK_STRIDE * T,
                reinterpret_cast<uint32_t*>(tick + 2 * TICK_STRIDE * T), cand, cand_n, lb_err);
    } else {
      EW_LAUNCH(k_pk_pass0, G, s, g, src_flat, chunks, cbl, tensors, pst, pcand, hist0, kmaxr,
                state, T, tick + TICK_STRIDE * T);
      EW_LAUNCH(k_pk_pass1, G, s, g, src_flat, chunks, cbl, tensors, pst, pcand, hist1, kmaxr,
                state, T, tick + 2 * TICK_STRIDE * T, cand, cand_n);
      EW_LAUNCH(k_pk_pass2, G, s, cbl, tensors, pst, hist2, kmaxr, state, T,
                tick + 3 * TICK_STRIDE * T, cand, cand_n);
    }
#define EW_PKW(VK, EFV)                                                                          \
  EW_LAUNCH((k_topk_write<VK, EFV, true, true>), C, s, g, resid, chunks, tensors, state, chunk_off, \
            chunk_ties, inv, pay, a.scales_off, a.idx_off, a.codes_off, a.bitmap_off, a.levels,   \
            a.inv_levels, a.key, reinterpret_cast<const uint32_t*>(a.key_ptr), a.bucket_offset,   \
            kmaxr, pk_rz0, dg.mask ? dg.vel : nullptr, lb, a.counts_off, lb_err, pst, cbase,      \
            ccnt, pcand, a.lb_fault, hist1, (uint32_t)(T * NB1), hist2, (uint32_t)(T * NB2), ap, \
            dg.stamps)
    if (a.value_kind == VK_Q8) {
      if (resid) EW_PKW(VK_Q8, true); else EW_PKW(VK_Q8, false);
    } else if (a.value_kind == VK_Q4) {
      if (resid) EW_PKW(VK_Q4, true); else EW_PKW(VK_Q4, false);
    } else {
      if (resid) EW_PKW(VK_F32, true); else EW_PKW(VK_F32, false);
    }
#undef EW_PKW
    EW_CHECK_LAUNCH();
    return;
  }
  if (dg.vel)
    EW_LAUNCH(k_topk_hist0<EF_DGC>, C, s, g, dg, lb, resid, chunks, hist0, kmaxr, T, tensors, state,
              tick);
  else if (resid)
    EW_LAUNCH(k_topk_hist0<EF_PLAIN>, C, s, g, dg, lb, resid, chunks, hist0, kmaxr, T, tensors,
              state, tick);
  else
    EW_LAUNCH(k_topk_hist0<EF_NONE>, C, s, g, dg, lb, resid, chunks, hist0, kmaxr, T, tensors, state,
              tick);
  EW_LAUNCH(k_topk_hist1, C, s, g, src_flat, chunks, state, hist1, T, tensors, kmaxr,
            tick + TICK_STRIDE * T, cand, cand_n);
  EW_LAUNCH(k_topk_hist2, C, s, chunks, state, hist2, T, tensors, kmaxr, tick + 2 * TICK_STRIDE * T,
            cand, cand_n);
  // the L2 scale needs the selected values' sum of squares before any code is written: a count
  // pass; the max-norm scale is hist0's max key and the write pass looks back for its offsets
  const bool lbk = !a.norm_l2;
  if (!lbk)
    EW_LAUNCH(k_topk_count, C, s, g, src_flat, chunks, state, cnt_gt, cnt_eq, chunk_sq, tensors,
              tick + 3 * TICK_STRIDE * T, chunk_off, chunk_ties, inv, pay, a.scales_off, a.counts_off,
              a.levels, a.norm_l2);
#define EW_WRITE(VK, EFV, LBV)                                                                     \
  EW_LAUNCH((k_topk_write<VK, EFV, LBV, false>), C, s, g, resid, chunks, tensors, state, chunk_off, \
            chunk_ties, inv, pay, a.scales_off, a.idx_off, a.codes_off, a.bitmap_off, a.levels,     \
            a.inv_levels, a.key, reinterpret_cast<const uint32_t*>(a.key_ptr), a.bucket_offset,     \
            kmaxr, rezero_words, dg.mask ? dg.vel : nullptr, lb, a.counts_off, lb_err, nullptr,     \
            nullptr, nullptr, nullptr, a.lb_fault, nullptr, 0u, nullptr, 0u, TkApply{}, dg.stamps)
#define EW_WRITE2(VK, EFV) \
  do { if (lbk) EW_WRITE(VK, EFV, true); else EW_WRITE(VK, EFV, false); } while (0)
  if (a.value_kind == VK_Q8) {
    if (resid) EW_WRITE2(VK_Q8, true); else EW_WRITE2(VK_Q8, false);
  } else if (a.value_kind == VK_Q4) {
    if (resid) EW_WRITE2(VK_Q4, true); else EW_WRITE2(VK_Q4, false);
  } else {
    if (resid) EW_WRITE2(VK_F32, true); else EW_WRITE2(VK_F32, false);
  }
#undef EW_WRITE2
#undef EW_WRITE
  EW_CHECK_LAUNCH();
}

size_t ew_topk_scratch_bytes(int T, int C, long long L, long long total_cap) {
  // state .. inv, alignment slack + tickets + candidate counts + error counter, look-back words,
  // candidate keys; predictive state, chunk candidate tables, counters, candidate list
  return sizeof(uint32_t) *
             ((size_t)4 * T + (size_t)NREP * T * (1 + NB0 + NB1 + NB2) + 5 * (size_t)C + T +
              (5 * (size_t)T + 2 + 9) * TICK_STRIDE + (size_t)L) +
         sizeof(unsigned long long) * (size_t)C + 128 +
         sizeof(uint32_t) * (8 * (size_t)T + 2 * (size_t)C + (size_t)TICK_STRIDE * T) + 16 +
         sizeof(uint2) * (size_t)total_cap;
}

std::vector<int> ew_topk_stats(uintptr_t scratch, int T, int C) {
  // same carving as ew_topk_encode: {look-back errors, fast tensor-encodes, full tensor-encodes}
  uint32_t* state = reinterpret_cast<uint32_t*>(scratch);
  uint32_t* kmaxr = state + 4 * T;
  uint32_t* hist2 = kmaxr + NREP * T + (size_t)NREP * T * NB0 + (size_t)NREP * T * NB1;
  float* inv = reinterpret_cast<float*>(hist2 + (size_t)NREP * T * NB2 + 5 * (size_t)C);
  int* tick = reinterpret_cast<int*>(
      (reinterpret_cast<uintptr_t>(inv + T) + TICK_STRIDE * 4 - 1) & ~(uintptr_t)(TICK_STRIDE * 4 - 1));
  int* lb_err = tick + 5 * TICK_STRIDE * T;
  // {look-back errors, fast, full, full per tensor (the first PK_MISS_T tensors)}
  std::vector<int> v(3 + PK_MISS_T, 0);
  EW_CHECK(hipMemcpy(v.data(), lb_err, sizeof(int), hipMemcpyDeviceToHost));
  EW_CHECK(hipMemcpy(v.data() + 1, lb_err + 2, (2 + PK_MISS_T) * sizeof(int),
                     hipMemcpyDeviceToHost));
  return v;
}

int ew_topk_lookback_errors(uintptr_t scratch, int T, int C) {
  // same carving as ew_topk_encode
  uint32_t* state = reinterpret_cast<uint32_t*>(scratch);
  uint32_t* kmaxr = state + 4 * T;
  uint32_t* hist2 = kmaxr + NREP * T + (size_t)NREP * T * NB0 + (size_t)NREP * T * NB1;
  float* inv = reinterpret_cast<float*>(hist2 + (size_t)NREP * T * NB2 + 5 * (size_t)C);
  int* tick = reinterpret_cast<int*>(
      (reinterpret_cast<uintptr_t>(inv + T) + TICK_STRIDE * 4 - 1) & ~(uintptr_t)(TICK_STRIDE * 4 - 1));
  int* lb_err = tick + 5 * TICK_STRIDE * T;
  int v = 0;
  EW_CHECK(hipMemcpy(&v, lb_err, sizeof(int), hipMemcpyDeviceToHost));
  return v;
}

void ew_topk_decode_apply(const TopkDecodeArgs& a) {
  auto* chunks = reinterpret_cast<const ChunkRow*>(a.chunks);
  auto* tensors = reinterpret_cast<const TensorRow*>(a.tensors);
  if (a.apply && !a.mom && (a.momentum != 0.0f || a.nesterov))
    throw std::runtime_error("ewdml topk decode: a momentum step needs the momentum buffer");
  SgdArgs sa{a.lr, a.momentum, a.dampening, a.weight_decay, a.grad_scale, a.nesterov, a.first,
             reinterpret_cast<uint32_t*>(a.key_state), a.key_seed, a.key_rank};
  sa.lr_ptr = reinterpret_cast<const float*>(a.lr_ptr);
  auto* recv = reinterpret_cast<const uint8_t*>(a.recv);
  auto* p = reinterpret_cast<float*>(a.param);
  auto* m = reinterpret_cast<float*>(a.mom);
  auto* go = reinterpret_cast<float*>(a.grad_out);
  auto* sh = reinterpret_cast<uint16_t*>(a.shadow);
  const int C = a.num_chunks;
  // neither momentum nor weight decay nor an averaged-gradient output: the sparse kernel
  const bool sparse = a.apply && !m && a.momentum == 0.0f && a.weight_decay == 0.0f && !go;
#define EW_DEC(VK)                                                                                   \
  if (sparse)                                                                                       \
    EW_LAUNCH(k_topk_decode_sparse<VK>, C, a.stream, recv, a.nranks, a.stride, chunks, tensors,      \
              a.scales_off, a.counts_off, a.idx_off, a.codes_off, a.bitmap_off, a.inv_levels, p, sh, \
              sa);                                                                                   \
  else                                                                                              \
    EW_LAUNCH(k_topk_decode_apply<VK>, C, a.stream, recv, a.nranks, a.stride, chunks, tensors,         \
            a.scales_off, a.counts_off, a.idx_off, a.codes_off, a.bitmap_off, a.inv_levels, p, m, go, \
            sh, sa,                                                                                  \
            a.apply)
  if (a.value_kind == VK_Q8) EW_DEC(VK_Q8);
  else if (a.value_kind == VK_Q4) EW_DEC(VK_Q4);
  else EW_DEC(VK_F32);
#undef EW_DEC
  EW_CHECK_LAUNCH();
}
