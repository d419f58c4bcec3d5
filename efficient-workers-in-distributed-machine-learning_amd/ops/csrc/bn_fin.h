// BatchNorm statistics finalisation shared by nn.hip (its own launches) and conv_f32.hip (the
// backward finalisation riding in a weight-gradient GEMM launch as extra blocks: the partial sums
// come from the backward-data launch before it, and nothing in the GEMM reads or writes them, so
// the ~5 us finalize launch runs under the GEMM instead of after it).
#pragma once
#include "common.h"

// Sum the nblk partial rows of NS quantities per channel in a fixed order.  16 channels (t & 15) x
// 16 row slices (t >> 4) of the first EW_BLOCK threads: a wave's load covers 4 rows x 16
// consecutive channels (64-B segments; 4 channels x 64 slices -- 16-B segments, 16 lines per load --
// was slower, 5.7 -> 7.2 us), each thread issues the loads of 16 of its rows for every quantity
// before adding any (was 4: ~8 dependent round trips for VGG's 512-row partials).  Slices combine
// by a fixed shuffle tree within each wave (lanes with the same channel: xor 16, 32) and then over
// the 4 waves in order through `red` (LDS, NS * EW_WAVES * EW_FIN_CH doubles).  Threads past
// EW_BLOCK (a larger block running this as a side task) only take part in the barrier, so the sums
// are bitwise those of an EW_BLOCK launch.  Returns true (for threads 0-15, c < C) with out[]
// holding the sums.
constexpr int EW_FIN_CH = 16;
// U: rows in flight per thread (the sums' order does not depend on it); TH: the threads that sum
// (TH / 16 row slices, TH / 64 waves; the order does depend on it)
template <int NS, int U = 16, int TH = EW_BLOCK>
__device__ __forceinline__ bool ew_sum_parts(const float* __restrict__ part, int nblk, int C,
                                             int c, double out[NS], double* red) {
  constexpr int NW = TH / 64;
  const int t = threadIdx.x, rs = t / EW_FIN_CH, lane = t & 63, w = t >> 6;
  const bool act = t < TH;
  constexpr int RS = TH / EW_FIN_CH;  // row slices
  double acc[NS];
#pragma unroll
  for (int s = 0; s < NS; ++s) acc[s] = 0.0;
  if (act && c < C) {
    for (int b0 = rs; b0 < nblk; b0 += U * RS) {
      // unconditional loads of a clamped row, masked when added: a guarded load is a branch,
      // and hipcc waits for every load at each branch merge (one round trip per row)
      float v[NS][U];
#pragma unroll
      for (int s = 0; s < NS; ++s)
#pragma unroll
        for (int u = 0; u < U; ++u) {
          const int b = min(b0 + u * RS, nblk - 1);
          v[s][u] = part[((long long)s * nblk + b) * C + c];
        }
#pragma unroll
      for (int s = 0; s < NS; ++s)
#pragma unroll
        for (int u = 0; u < U; ++u)
          if (b0 + u * RS < nblk) acc[s] += (double)v[s][u];
    }
  }
#pragma unroll
  for (int s = 0; s < NS; ++s) {
#pragma unroll
    for (int o = EW_FIN_CH; o < 64; o <<= 1) acc[s] += __shfl_xor(acc[s], o, 64);
    if (act && lane < EW_FIN_CH) red[(s * NW + w) * EW_FIN_CH + lane] = acc[s];
  }
  __syncthreads();
  if (t >= EW_FIN_CH || c >= C) return false;
#pragma unroll
  for (int s = 0; s < NS; ++s) {
    double a = red[s * NW * EW_FIN_CH + t];
#pragma unroll
    for (int r = 1; r < NW; ++r) a += red[(s * NW + r) * EW_FIN_CH + t];
    out[s] = a;
  }
  return true;
}

// One BatchNorm backward finalisation: from the partial sums (NS = 3: k_bn_bwd_stats'; NS = 2: a
// backward-data conv epilogue's, whose sum(h - mean) -- 0 up to rounding -- is taken as 0) the
// apply coefficients coef [2][C] (e, f: dx = e * (h - mean) + f + scale * dz), dgamma, dbeta and
// the conv bias gradient.  ngrp = ceil(C / EW_FIN_CH) channel groups, one per block.
struct EwBnFin {
  const float* part;
  const float* stats;  // [4][C] of the forward: mean, invstd, scale, shift
  float* coef;
  float* dgamma;
  float* dbeta;
  void* dcbias;
  long long M;  // rows the statistics cover (pre-pool)
  int nblk;     // partial rows
  int C;
  int cb_bf16;
  int ngrp;     // 0: no job
};

template <int NS, int U = 16>
__device__ __forceinline__ void ew_bn_bwd_fin_group(const EwBnFin& f, int grp, double* red) {
  const int C = f.C;
  const int c = grp * EW_FIN_CH + (threadIdx.x % EW_FIN_CH);
  const int cc = c < C ? c : C - 1;
  const double invstd = f.stats[C + cc], scale = f.stats[2 * C + cc];  // ahead of the sums' loads
  double sums[3];
  if (!ew_sum_parts<NS, U>(f.part, f.nblk, C, c, sums, red)) return;
  if (NS == 2) sums[2] = 0.0;
  const double db = sums[0];           // sum dz
  const double dg = sums[1] * invstd;  // sum dz * xhat
  const double e = -scale * invstd * dg / (double)f.M;
  f.coef[c] = (float)e;
  f.coef[C + c] = (float)(-scale * db / (double)f.M);
  if (f.dgamma) f.dgamma[c] = (float)dg;
  if (f.dbeta) f.dbeta[c] = (float)db;
  if (f.dcbias) {  // sum over rows of dx = e * sum(h - mean)
    const float v = (float)(e * sums[2]);
    if (f.cb_bf16) reinterpret_cast<uint16_t*>(f.dcbias)[c] = ew_f2bf(v);
    else reinterpret_cast<float*>(f.dcbias)[c] = v;
  }
}

// ew_bn_bwd_fin_group's sums for one channel c in one thread, in exactly the group's order (the
// 16 row slices' sums in row order, the xor-16 / xor-32 pairs of each wave, then the 4 waves in
// order): bitwise the same outputs, for a producer whose last block finalises a few channels
// itself.  SC1: the partials were written in this launch by other blocks (write-through), read
// with agent-scope loads.
template <bool SC1>
__device__ __forceinline__ float ew_fin_ld(const float* p) {
  return SC1 ? __hip_atomic_load(const_cast<float*>(p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)
             : *p;
}

template <int NS, bool SC1>
__device__ __forceinline__ void ew_bn_bwd_fin_chan(const EwBnFin& f, int c) {
  const int C = f.C;
  double sums[3] = {0.0, 0.0, 0.0};
  // up to 16 partial rows (one per row slice): every load issued before the first add
  float r16[NS][16];
  if (f.nblk <= 16) {
#pragma unroll
    for (int s = 0; s < NS; ++s)
#pragma unroll
      for (int b = 0; b < 16; ++b)
        r16[s][b] = ew_fin_ld<SC1>(f.part + ((long long)s * f.nblk + min(b, f.nblk - 1)) * C + c);
  }
#pragma unroll
  for (int s = 0; s < NS; ++s) {
    double w4[4];
#pragma unroll
    for (int w = 0; w < 4; ++w) {
      double x[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        double a = 0.0;
        if (f.nblk <= 16) {
          if (4 * w + i < f.nblk) a += (double)r16[s][4 * w + i];
        } else {
          for (int b = 4 * w + i; b < f.nblk; b += 16)
            a += (double)ew_fin_ld<SC1>(f.part + ((long long)s * f.nblk + b) * C + c);
        }
        x[i] = a;
      }
      w4[w] = (x[0] + x[1]) + (x[2] + x[3]);
    }
    double a = w4[0];
#pragma unroll
    for (int w = 1; w < 4; ++w) a += w4[w];
    sums[s] = a;
  }
  const double invstd = f.stats[C + c], scale = f.stats[2 * C + c];
  if (NS == 2) sums[2] = 0.0;
  const double db = sums[0];
  const double dg = sums[1] * invstd;
  const double e = -scale * invstd * dg / (double)f.M;
  f.coef[c] = (float)e;
  f.coef[C + c] = (float)(-scale * db / (double)f.M);
  if (f.dgamma) f.dgamma[c] = (float)dg;
  if (f.dbeta) f.dbeta[c] = (float)db;
  if (f.dcbias) {
    const float v = (float)(e * sums[2]);
    if (f.cb_bf16) reinterpret_cast<uint16_t*>(f.dcbias)[c] = ew_f2bf(v);
    else reinterpret_cast<float*>(f.dcbias)[c] = v;
  }
}
