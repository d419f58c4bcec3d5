// fp32 3x3 / pad 1 / stride 1 convolutions over 2x2 maps (VGG-11's conv7 / conv8 on CIFAR) as
// dense position GEMMs -- forward, backward data and weight gradient, no transforms.
//
// On a 2x2 map every (input position ip, output position op) pair is joined by exactly one tap of
// the kernel, tap(ip, op) = (ih - oh + 1) * 3 + (iw - ow + 1), so the layer is the dense GEMM
//
//   y[n][op][o]  = sum_{ip, c} x[n][ip][c] * w[o][tap(ip, op)][c]      M = N, N' = 4 Nc, K = 4 C
//   dx[n][ip][c] = sum_{op, o} dy[n][op][o] * w[o][tap(ip, op)][c]     M = N, N' = 4 C,  K = 4 Nc
//   dw[o][t][c]  = sum_{(ip, op): tap = t} sum_n dy[n][op][o] x[n][ip][c]    (16 pairs over 9 taps)
//
// with 4/9 of the implicit GEMM's 9-tap work (5 of a pixel's 9 taps are padding) and the FLOPs of
// Winograd F(2x2) (whose 4x4 patch of a 2x2 map is mostly zeros) without its input / weight /
// output transforms: on VGG-11 the two 2x2 layers took ~156 us of a 1.26 ms step as 14 kernels
// (Winograd input + GEMM + output transform per pass, profiles/vgg11_bs128_fp32_current_graph.txt);
// here the forward is one launch and the whole backward (data and weight gradient) another.
//
// GEMM: 64 x 64 tiles, 8 waves (two per SIMD) as 4 x 2 sub-tiles of 16 x 32, v_mfma_f32_16x16x4_f32
// (exact fp32 products and sums, as conv_f32.hip), 32-deep k-steps through two LDS stages and two
// staging register sets (step s + 2 loads while s computes and s + 1 is written; a lazily formed
// operand is formed when written, so its loads never stall the loop).
// Forward and backward data split K over the four positions (a tile is 64 rows x 64 channels of
// one position, K = C (or Nc) per split: 4 x tiles = 256 blocks on VGG-11) and reduce in the launch:
// every split writes its fp32 slab, takes a ticket, and the last arriver sums the four slabs in
// split order (deterministic whatever the arrival order) and runs the epilogue: the output, the
// BatchNorm partial sums of the output (forward) or the producing BN layer's backward sums
// (backward data), one partial row per (64 rows, position) -- 8 rows at batch 128 instead of
// 128-1024, so the finalize is one round trip.  The slab hand-off is cdna_hip_programming.md's
// in-launch split-K recipe in its write-through form (sc1 stores and loads, no fences); the four
// splits of a tile are dispatched to one XCD.
//
// Operands may be formed on the fly (the lazy BatchNorm of ops/nn.py, winograd_f32.hip WgSrc):
// x as relu(h * scale + shift) of the BN layer in front (KIND 1), dy as the backward of the
// BN(+ReLU)(+2x2 pool to 1x1) layer this conv feeds (KIND 2: dy = scale * dz + e * (h - mean) + f,
// k_bn_bwd_apply's expressions), so neither activation is ever written.
//
// Parity: the layers are the reference's nn.Conv2d(512, 512, 3, padding=1) of VGG-11's last block
// (src/model_ops/vgg.py:46-59, cfg "A"); only the execution differs.
#include <algorithm>
#include <cstdlib>
#include <stdexcept>
#include <type_traits>
#include <string>

#include "bn_fin.h"
#include "common.h"
#include "dgc_stage.h"
#include "conv_f32.h"
#include "ewdml_ops.h"

namespace {

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));

constexpr int SM_T = 512;  // threads per block (8 waves, two per SIMD)
constexpr int SM_BM = 64, SM_BN = 64, SM_BK = 64;
constexpr int SM_RC_PITCH = SM_BN + 4;                 // RC image row pitch (floats)
constexpr int SM_KC_BYTES = SM_BM * SM_BK * 4;         // 16 KB
constexpr int SM_RC_BYTES = SM_BK * SM_RC_PITCH * 4;   // 17 KB
constexpr int SM_STAGE = 2 * SM_RC_BYTES;              // A + B image, any layouts
// the A image's size (B follows it): an RC image is larger than a KC one
template <int AL>
constexpr int sm_abytes() { return AL == 0 ? SM_KC_BYTES : SM_RC_BYTES; }
constexpr int SM_TILE = SM_BM * SM_BN;                 // slab floats per (tile, split)
struct F2 {  // two plain operand vectors
  f32x4 v[2];
};

enum { SM_KC = 0, SM_RC = 1 };

// KC image: [64 rows][64 k], 256-B rows (one full pass over the 64 banks), 16-B chunk c of row r at
// c ^ (r & 15): a ds_read_b128 lane group reading 16 rows at one chunk hits 16 distinct 4-bank
// slots, and the 16 lanes writing one row's chunks fill the row
__device__ __forceinline__ int sm_kc(int r, int c) { return r * 256 + ((c ^ (r & 15)) << 4); }

// tap joining input position ip and output position op of a 2x2 map (positions p = h * 2 + w)
__device__ __forceinline__ int sm_tap(int ip, int op) {
  return ((ip >> 1) - (op >> 1) + 1) * 3 + ((ip & 1) - (op & 1) + 1);
}

// pair p (op ascending) of the pairs (ip, op) joined by tap t: op = (oh, ow) over the output rows /
// columns the tap reaches (dh = t / 3 - 1: oh = 0..1 when dh = 0, oh = 0 for dh = 1, oh = 1 for
// dh = -1; the same for w), ip = (oh + dh, ow + dw)
__device__ __forceinline__ int sm_npairs(int t) {
  return ((t / 3) == 1 ? 2 : 1) * ((t % 3) == 1 ? 2 : 1);
}
__device__ __forceinline__ void sm_pair(int t, int p, int& ip, int& op) {
  const int dh = t / 3 - 1, dw = t % 3 - 1;
  const int nw = dw == 0 ? 2 : 1;
  const int ph = p / nw, pw = p - ph * nw;
  const int oh = dh == 0 ? ph : (dh > 0 ? 0 : 1);
  const int ow = dw == 0 ? pw : (dw > 0 ? 0 : 1);
  ip = (oh + dh) * 2 + ow + dw;
  op = oh * 2 + ow;
}

// split-K block -> (tile, split): with a tile count that is a multiple of 8, the four splits of a
// tile are blocks b, b + 8, b + 16, b + 24 (one XCD: blocks go round-robin to the 8 XCDs)
__device__ __forceinline__ void sm_split_map(int b, int tiles, int& tile, int& split) {
  if ((tiles & 7) == 0) {
    const int xcd = b & 7, l = b >> 3;
    split = l & 3;
    tile = (l >> 2) * 8 + xcd;
  } else {
    split = b & 3;
    tile = b >> 2;
  }
}

// the conv input x[N][2][2][C]: materialised (KIND 0) or relu(h * scale + shift) of the BN layer
// in front (KIND 1, stats [4][C]: mean, invstd, scale, shift)
struct SmX {
  const float* x;
  const float* h;
  const float* stats;
  long long* nbt;  // KIND 1: that layer's num_batches_tracked (incremented once, forward only)
};
// dy[N][2][2][Nc]: materialised (KIND 0) or the backward of the BN(+ReLU)(+2x2 pool) layer whose
// input is this conv's output h (KIND 2): pooled, dnext / code are [N][Nc] (the 1x1 map)
struct SmDy {
  const float* dy;
  const float* h;
  const float* dnext;
  const uint8_t* code;
  const float* stats;  // [4][Nc]
  const float* coef;   // [2][Nc]: e, f
  int pool;
};

// per-channel coefficients of 4 consecutive dy channels (KIND 2)
struct SmDyCoef {
  f32x4 mean, sc, sh, e, f;
};
__device__ __forceinline__ void sm_dy_coef(const SmDy& s, int Nc, int o, SmDyCoef& k) {
  k.mean = *reinterpret_cast<const f32x4*>(s.stats + o);
  k.sc = *reinterpret_cast<const f32x4*>(s.stats + 2 * Nc + o);
  k.sh = *reinterpret_cast<const f32x4*>(s.stats + 3 * Nc + o);
  k.e = *reinterpret_cast<const f32x4*>(s.coef + o);
  k.f = *reinterpret_cast<const f32x4*>(s.coef + Nc + o);
}

// Operand staging is split in two: the k-loop issues a step's raw loads two steps ahead (RawX /
// RawDy, no arithmetic on them) and forms the operand only when it writes the step to LDS one step
// later, so a lazily formed operand (KIND 1 / 2) never makes the loop wait for its loads.
// A thread stages two vectors of each operand per step: rows (or k-rows) r and r + 32, the same
// four channels.
struct RawX {  // x: the values (KIND 0) or the BN inputs and their scale / shift (KIND 1)
  f32x4 v[2], sc, sh;
};
// rows at off and off + rs
template <int XK>
__device__ __forceinline__ void sm_raw_x(const SmX& s, long long off, long long rs,
                                         const float* stats_c, int C, RawX& r) {
  const float* src = XK == 0 ? s.x : s.h;
  r.v[0] = *reinterpret_cast<const f32x4*>(src + off);
  r.v[1] = *reinterpret_cast<const f32x4*>(src + off + rs);
  if constexpr (XK == 1) {
    if (stats_c) {  // per-step channels (else hoisted by the caller)
      r.sc = *reinterpret_cast<const f32x4*>(stats_c + 2 * C);
      r.sh = *reinterpret_cast<const f32x4*>(stats_c + 3 * C);
    }
  }
}
template <int XK>
__device__ __forceinline__ f32x4 sm_make_x(const RawX& r, int i) {
  if constexpr (XK == 0) {
    return r.v[i];
  } else {
    f32x4 v;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const float z = r.v[i][q] * r.sc[q] + r.sh[q];  // as k_bn_fwd_apply writes it
      v[q] = (z > 0.0f || z != z) ? z : 0.0f;
    }
    return v;
  }
}

struct RawDy {  // dy (KIND 0) or this conv's output h, the BN layer's output gradient, its codes
  f32x4 v[2], dn[2];
  uint32_t code[2];
  SmDyCoef k;
};
// dy at images n and n + 32, output position op, channels o..o+3; coef: load the channels'
// coefficients (per-step channels) or leave them to the caller (hoisted)
template <int DK>
__device__ __forceinline__ void sm_raw_dy(const SmDy& s, int Nc, int n, int op, int o, bool coef,
                                          RawDy& r) {
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const long long m = n + 32 * i;
    const long long off = (m * 4 + op) * Nc + o;
    if constexpr (DK == 0) {
      r.v[i] = *reinterpret_cast<const f32x4*>(s.dy + off);
    } else {
      r.v[i] = *reinterpret_cast<const f32x4*>(s.h + off);
      if constexpr (DK == 3) {  // 2x2 -> 1x1 pool: the window is the whole map, op's code is op
        r.dn[i] = *reinterpret_cast<const f32x4*>(s.dnext + m * Nc + o);
        r.code[i] = *reinterpret_cast<const uint32_t*>(s.code + m * Nc + o);
      } else {
        r.dn[i] = *reinterpret_cast<const f32x4*>(s.dnext + off);
        r.code[i] = 0u;
      }
    }
  }
  if constexpr (DK != 0) {
    if (coef) sm_dy_coef(s, Nc, o, r.k);
  }
}
template <int DK>
__device__ __forceinline__ f32x4 sm_make_dy(const SmDy& s, int op, const RawDy& r,
                                            const SmDyCoef& k, int i) {
  if constexpr (DK == 0) {
    return r.v[i];
  } else {
    f32x4 v;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const float dp =
          (DK != 3 || ((r.code[i] >> (8 * q)) & 0xffu) == (uint32_t)op) ? r.dn[i][q] : 0.0f;
      // the expressions of k_bn_bwd_apply: the same contraction, the same bits
      const float z = r.v[i][q] * k.sc[q] + k.sh[q];
      const float dz = !(z <= 0.0f) ? dp : 0.0f;
      v[q] = k.sc[q] * dz + k.e[q] * (r.v[i][q] - k.mean[q]) + k.f[q];
    }
    return v;
  }
}

// ---- the GEMM core: 8 waves (two per SIMD) as 4 x 2 tiles of 16 rows x 32 columns over a
// 64 x 64 tile, v_mfma_f32_16x16x4_f32 (A lane l = A[l & 15][k], B lane l = B[k][l & 15], D lane
// l reg e = D[4 (l >> 4) + e][l & 15]), a 64-deep k-step per iteration through two LDS stages.
// Lane group g = lane >> 4 takes k = 4 (4 r + g) + jj for MFMA (r, jj), r < 4, in both operands.
constexpr int SM_WM = 4, SM_WN = 2;        // wave grid
constexpr int SM_NJ = SM_BN / SM_WN / 16;  // 16-column accumulators per wave (2)

struct SmAcc {
  f32x4 a[SM_NJ];
};
// tile row / column of accumulator j, element e of lane `lane` of wave (wm, wn)
__device__ __forceinline__ int sm_row(int wm, int lane, int e) {
  return wm * 16 + 4 * (lane >> 4) + e;
}
__device__ __forceinline__ int sm_col(int wn, int lane, int j) {
  return wn * 32 + j * 16 + (lane & 15);
}

template <int AL, int BL>
__device__ __forceinline__ void sm_mma_step(const char* __restrict__ st, int wm, int wn, int lane,
                                            SmAcc& acc) {
  const char* As = st;
  const char* Bs = st + sm_abytes<AL>();
  const int g = lane >> 4, li = lane & 15;
  constexpr int R = SM_BK / 16;
  f32x4 fa[R], fb[R][SM_NJ];
#pragma unroll
  for (int r = 0; r < R; ++r) {
    const int ch = r * 4 + g;
    if constexpr (AL == SM_KC) {
      fa[r] = *reinterpret_cast<const f32x4*>(As + sm_kc(wm * 16 + li, ch));
    } else {
      const float* ap = reinterpret_cast<const float*>(As) + 4 * ch * SM_RC_PITCH + wm * 16 + li;
#pragma unroll
      for (int jj = 0; jj < 4; ++jj) fa[r][jj] = ap[jj * SM_RC_PITCH];
    }
#pragma unroll
    for (int j = 0; j < SM_NJ; ++j) {
      const int col = wn * 32 + j * 16 + li;
      if constexpr (BL == SM_KC) {
        fb[r][j] = *reinterpret_cast<const f32x4*>(Bs + sm_kc(col, ch));
      } else {
        const float* bp = reinterpret_cast<const float*>(Bs) + 4 * ch * SM_RC_PITCH + col;
#pragma unroll
        for (int jj = 0; jj < 4; ++jj) fb[r][j][jj] = bp[jj * SM_RC_PITCH];
      }
    }
  }
#pragma unroll
  for (int r = 0; r < R; ++r)
#pragma unroll
    for (int jj = 0; jj < 4; ++jj)
#pragma unroll
      for (int j = 0; j < SM_NJ; ++j)
        acc.a[j] = __builtin_amdgcn_mfma_f32_16x16x4f32(fa[r][jj], fb[r][j][jj], acc.a[j], 0, 0, 0);
}

// operand vector i of thread t -> LDS stage: chunk t & 15 of row (KC, [64 rows][64 k]) or k-row
// (RC, [64 k][64 cols]) (t >> 4) + 32 i
template <int L>
__device__ __forceinline__ void sm_put(char* img, int t, int i, const f32x4& v) {
  const int r = (t >> 4) + 32 * i;
  if constexpr (L == SM_KC)
    *reinterpret_cast<f32x4*>(img + sm_kc(r, t & 15)) = v;
  else
    *reinterpret_cast<f32x4*>(img + (r * SM_RC_PITCH + (t & 15) * 4) * 4) = v;
}

// The pipelined k-loop over ksteps steps, SM_NS register stages deep: step s + SM_NS is loaded
// while s computes and s + 1 is written to the other LDS stage (the loads have SM_NS - 1 steps to
// land: a 64x64 step is only ~1k SIMD cycles of MFMA, shorter than a miss to HBM under load, so two
// stages -- conv_f32.hip's depth for its 4x longer steps -- left the loop waiting on memory).
// LA(s, RA&) / LB(s, RB&) issue step s's raw loads, MA(const RA&, i) / MB(const RB&, i) form the
// thread's operand vector i (i < 2) at LDS-write time.  Loads past the last step are clamped re-loads of it.
constexpr int SM_NS = 2;
template <int AL, int BL, typename RA, typename RB, typename LA, typename LB, typename MA,
          typename MB>
__device__ __forceinline__ void sm_gemm(char* smem, int ksteps, LA&& la, LB&& lb, MA&& ma,
                                        MB&& mb, SmAcc& acc) {
  const int t = threadIdx.x, lane = t & 63, wq = t >> 6;
  const int wm = wq / SM_WN, wn = wq % SM_WN;
#pragma unroll
  for (int j = 0; j < SM_NJ; ++j) acc.a[j] = f32x4{};
  if (ksteps <= 0) return;
  const int last = ksteps - 1;
  RA ra[SM_NS];
  RB rb[SM_NS];
#pragma unroll
  for (int i = 0; i < SM_NS; ++i) {
    la(min(i, last), ra[i]);
    lb(min(i, last), rb[i]);
  }
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    sm_put<AL>(smem, t, i, ma(ra[0], i));
    sm_put<BL>(smem + sm_abytes<AL>(), t, i, mb(rb[0], i));
  }
  __syncthreads();
  // iteration s: compute LDS stage s % 2, reload register slot s % SM_NS with step s + SM_NS,
  // write step s + 1 (slot (s + 1) % SM_NS) to the other stage
  auto body = [&](int s, auto uc) {
    constexpr int u = decltype(uc)::value;
    la(min(s + SM_NS, last), ra[u]);
    lb(min(s + SM_NS, last), rb[u]);
    sm_mma_step<AL, BL>(smem + (u & 1) * SM_STAGE, wm, wn, lane, acc);
    char* ns = smem + ((u + 1) & 1) * SM_STAGE;
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      sm_put<AL>(ns, t, i, ma(ra[(u + 1) % SM_NS], i));
      sm_put<BL>(ns + sm_abytes<AL>(), t, i, mb(rb[(u + 1) % SM_NS], i));
    }
    __syncthreads();
  };
  static_assert(SM_NS == 2 || SM_NS == 4, "register stages");
  const int nfull = ksteps - ksteps % SM_NS;
  for (int s0 = 0; s0 < nfull; s0 += SM_NS) {
    body(s0 + 0, std::integral_constant<int, 0>{});
    body(s0 + 1, std::integral_constant<int, 1>{});
    if constexpr (SM_NS == 4) {
      body(s0 + 2, std::integral_constant<int, 2 % SM_NS>{});
      body(s0 + 3, std::integral_constant<int, 3 % SM_NS>{});
    }
  }
  const int rem = ksteps - nfull;  // block-uniform
  if (rem > 0) body(nfull + 0, std::integral_constant<int, 0>{});
  if (SM_NS == 4 && rem > 1) body(nfull + 1, std::integral_constant<int, 1>{});
  if (SM_NS == 4 && rem > 2) body(nfull + 2, std::integral_constant<int, 2 % SM_NS>{});
}

// In-launch split-K over the four positions: every split stores its slab, the tile's last arriver
// (ticket) sums the four slabs in split order into acc.  Returns true in the reducer.
// Hand-off (cdna_hip_programming.md Guideline 16, R1 with sc1 loads): the slab is stored
// write-through (agent-scope relaxed stores: global_store sc1), every wave drains its stores
// before the block's barrier and one lane draws the ticket; the reducer reads the other slabs
// with agent-scope (sc1) loads only, so neither a release (an L2 write-back of the XCD) nor an
// acquire (an L1 invalidate) is needed, wherever the four splits ran.
//
// The contract, cell by cell against MI355X_MICROARCH.md's table of measured hand-offs (row 1):
//   who signals   -- ONE lane per storing workgroup (t == 0), an agent-scope atomic add (the
//                    ticket), after EVERY storing wave's `s_waitcnt vmcnt(0)` and a workgroup
//                    barrier (so the add comes after all four waves' slab stores landed);
//   how learned   -- the workgroup whose add came last, told by the value its add returned;
//   before loads  -- the reducer's waves load only after the block barrier that publishes the
//                    flag the ticket-drawing lane set;
//   memory        -- hipMalloc'd slabs (the torch caching allocator), one block per CU or more;
//   stores/loads  -- every slab byte stored by a 4-B sc1 store, read by a 4-B sc1 load.
// That table records hardware behaviour measured on gfx950 / ROCm 7.2, not a guarantee of the
// HIP memory model: with relaxed atomics and no release / acquire pair the language does not
// order the slab stores before the ticket.  The fenced form (fence = 1: plain stores, lane 0's
// agent release fence + vmcnt before the ticket, the last arriver's agent acquire) is the memory
// model's own release/acquire pairing; tests/kernels/test_conv_f32.py::
// test_conv_f32_smallmap_fenced_handoff_bitwise keeps it bitwise equal to the default, so a
// compiler or firmware change that broke the measured form can be answered by EWDML_SM_FENCE=1.
int g_sm_fence = -1;  // EWDML_SM_FENCE=1: plain stores + release / acquire fences (A/B, tests)

__device__ __forceinline__ bool sm_reduce(SmAcc& acc, float* __restrict__ slab, int* cnt, int tile,
                                          int split, int* flag, int fence) {
  const int t = threadIdx.x, lane = t & 63, wq = t >> 6;
  const int wm = wq / SM_WN, wn = wq % SM_WN;
  float* mine = slab + ((size_t)tile * 4 + split) * SM_TILE;
  if (fence) {
#pragma unroll
    for (int j = 0; j < SM_NJ; ++j)
#pragma unroll
      for (int e = 0; e < 4; ++e)
        mine[sm_row(wm, lane, e) * SM_BN + sm_col(wn, lane, j)] = acc.a[j][e];
  } else {
#pragma unroll
    for (int j = 0; j < SM_NJ; ++j)
#pragma unroll
      for (int e = 0; e < 4; ++e)
        __hip_atomic_store(mine + sm_row(wm, lane, e) * SM_BN + sm_col(wn, lane, j), acc.a[j][e],
                           __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (t == 0) {
    if (fence) {
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    const int prev = __hip_atomic_fetch_add(cnt + tile, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const int last = prev == 3;
    if (last) {
      __hip_atomic_store(cnt + tile, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (fence) {
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      }
    }
    *flag = last;
  }
  __syncthreads();
  if (!*flag) return false;
  float v[4][SM_NJ][4];
#pragma unroll
  for (int z = 0; z < 4; ++z) {
    if (z == split) continue;
    const float* p = slab + ((size_t)tile * 4 + z) * SM_TILE;
#pragma unroll
    for (int j = 0; j < SM_NJ; ++j)
#pragma unroll
      for (int e = 0; e < 4; ++e)
        v[z][j][e] = __hip_atomic_load(p + sm_row(wm, lane, e) * SM_BN + sm_col(wn, lane, j),
                                       __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
#pragma unroll
  for (int j = 0; j < SM_NJ; ++j)
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      float s = split == 0 ? acc.a[j][e] : v[0][j][e];
#pragma unroll
      for (int z = 1; z < 4; ++z) s += split == z ? acc.a[j][e] : v[z][j][e];  // fixed order
      acc.a[j][e] = s;
    }
  return true;
}

// Column sums of the tile (two quantities) over its 64 rows: a lane's 4 rows, the 4 lanes of a
// column (xor 16, 32), then the 4 row waves through LDS in a fixed order -> bnpart[2][nrows][ld]
// at row prow, columns col0..+63
// wt: write-through stores (a BN finalisation riding in this launch reads them)
__device__ __forceinline__ void sm_colsums(const float (&s1)[SM_NJ][4],
                                           const float (&s2)[SM_NJ][4], char* smem, float* bnpart,
                                           int nrows, int prow, int ld, int col0, bool wt = false) {
  const int t = threadIdx.x, lane = t & 63, wq = t >> 6;
  const int wm = wq / SM_WN, wn = wq % SM_WN;
  float* red = reinterpret_cast<float*>(smem);  // [SM_WM][2][64]
  __syncthreads();
#pragma unroll
  for (int j = 0; j < SM_NJ; ++j) {
    float a = 0.0f, q = 0.0f;
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      a += s1[j][e];
      q += s2[j][e];
    }
    a += __shfl_xor(a, 16, 64);
    q += __shfl_xor(q, 16, 64);
    a += __shfl_xor(a, 32, 64);
    q += __shfl_xor(q, 32, 64);
    if (lane < 16) {
      red[(wm * 2 + 0) * 64 + sm_col(wn, lane, j)] = a;
      red[(wm * 2 + 1) * 64 + sm_col(wn, lane, j)] = q;
    }
  }
  __syncthreads();
  if (t < 64) {
    float sa = red[t], sq = red[64 + t];
#pragma unroll
    for (int r = 1; r < SM_WM; ++r) {
      sa += red[(r * 2 + 0) * 64 + t];
      sq += red[(r * 2 + 1) * 64 + t];
    }
    float* pa = bnpart + (long long)prow * ld + col0 + t;
    float* pq = bnpart + (long long)(nrows + prow) * ld + col0 + t;
    if (wt) {
      __hip_atomic_store(pa, sa, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(pq, sq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    } else {
      *pa = sa;
      *pq = sq;
    }
  }
}

// ---- forward: tile = (mt, op, ot) of y's [N rows][4 positions x Nc] map, split = ip ----
template <int XK>
__global__ __launch_bounds__(SM_T) void k_sm_fwd(SmX xs, const float* __restrict__ w,
                                                 float* __restrict__ y, float* __restrict__ slab,
                                                 int* __restrict__ cnt, int N, int C, int Nc,
                                                 float* __restrict__ bnpart, int fence) {
  __shared__ __attribute__((aligned(16))) char smem[2 * SM_STAGE + 16];
  int& flag = *reinterpret_cast<int*>(smem + 2 * SM_STAGE);
  const int t = threadIdx.x;
  if (XK == 1 && xs.nbt && blockIdx.x == 0 && t == 0) *xs.nbt += 1;
  int tile, split;
  sm_split_map(blockIdx.x, gridDim.x / 4, tile, split);
  const int ots = Nc / SM_BN;
  const int ot = tile % ots, op = (tile / ots) & 3, mt = tile / (ots * 4);
  const int ip = split, tap = sm_tap(ip, op);
  const int n0 = mt * SM_BM, o0 = ot * SM_BN;
  const int q = t & 15, r0 = t >> 4;  // KC: chunk q of rows r0, r0 + 32
  const long long arow = ((long long)(n0 + r0) * 4 + ip) * C + q * 4;
  const float* wr = w + ((long long)(o0 + r0) * 9 + tap) * C + q * 4;
  SmAcc acc;
  sm_gemm<SM_KC, SM_KC, RawX, F2>(
      smem, C / SM_BK,
      [&](int s, RawX& r) {
        sm_raw_x<XK>(xs, arow + s * SM_BK, 32LL * 4 * C,
                     XK == 1 ? xs.stats + s * SM_BK + q * 4 : nullptr, C, r);
      },
      [&](int s, F2& r) {
        r.v[0] = *reinterpret_cast<const f32x4*>(wr + s * SM_BK);
        r.v[1] = *reinterpret_cast<const f32x4*>(wr + 32LL * 9 * C + s * SM_BK);
      },
      [&](const RawX& r, int i) { return sm_make_x<XK>(r, i); },
      [&](const F2& r, int i) { return r.v[i]; }, acc);
  __syncthreads();
  if (!sm_reduce(acc, slab, cnt, tile, split, &flag, fence)) return;
  const int lane = t & 63, wq = t >> 6, wm = wq / SM_WN, wn = wq % SM_WN;
  float s1[SM_NJ][4], s2[SM_NJ][4];
#pragma unroll
  for (int j = 0; j < SM_NJ; ++j) {
    const int o = o0 + sm_col(wn, lane, j);
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const int n = n0 + sm_row(wm, lane, e);
      const float v = acc.a[j][e];
      y[((long long)n * 4 + op) * Nc + o] = v;
      s1[j][e] = v;
      s2[j][e] = v * v;
    }
  }
  if (bnpart) sm_colsums(s1, s2, smem, bnpart, (N / SM_BM) * 4, mt * 4 + op, Nc, o0);
}

// ---- backward: blocks [0, nbd) backward-data tiles (mt, ip, ct) of dx with split = op,
// [nbd, nbd + nbw) weight-gradient tiles (tap, ot, ct) ----
template <int XK, int DK>
__global__ __launch_bounds__(SM_T) void k_sm_bwd(SmX xs, SmDy ds, const float* __restrict__ w,
                                                 float* __restrict__ dx, float* __restrict__ dw,
                                                 float* __restrict__ slab, int* __restrict__ cnt,
                                                 int N, int C, int Nc, int nbd, CfBnBwd bb,
                                                 float* __restrict__ bnpart, int fence,
                                                 EwBnFin fin, int* __restrict__ fcnt,
                                                 DgcStage st) {
  __shared__ __attribute__((aligned(16))) char smem[2 * SM_STAGE + 16];
  int& flag = *reinterpret_cast<int*>(smem + 2 * SM_STAGE);
  const int t = threadIdx.x;
  const int lane = t & 63, wq = t >> 6, wm = wq / SM_WN, wn = wq % SM_WN;
  if ((int)blockIdx.x < nbd) {
    int tile, split;
    sm_split_map(blockIdx.x, nbd / 4, tile, split);
    const int cts = C / SM_BN;
    const int ct = tile % cts, ip = (tile / cts) & 3, mt = tile / (cts * 4);
    const int op = split, tap = sm_tap(ip, op);
    const int n0 = mt * SM_BM, c0 = ct * SM_BN;
    const int q = t & 15, r0 = t >> 4;           // A (KC): rows n0 + r0 (+ 32), channels 4 q..
    const int kr = t >> 4, cq = (t & 15) * 4;    // B (RC): k-rows o = kr (+ 32), columns c0 + cq
    const float* wb = w + ((long long)kr * 9 + tap) * C + c0 + cq;
    SmAcc acc;
    sm_gemm<SM_KC, SM_RC, RawDy, F2>(
        smem, Nc / SM_BK,
        [&](int s, RawDy& r) { sm_raw_dy<DK>(ds, Nc, n0 + r0, op, s * SM_BK + q * 4, true, r); },
        [&](int s, F2& r) {
          const float* p = wb + (long long)s * SM_BK * 9 * C;
          r.v[0] = *reinterpret_cast<const f32x4*>(p);
          r.v[1] = *reinterpret_cast<const f32x4*>(p + 32LL * 9 * C);
        },
        [&](const RawDy& r, int i) { return sm_make_dy<DK>(ds, op, r, r.k, i); },
        [&](const F2& r, int i) { return r.v[i]; }, acc);
    __syncthreads();
    if (!sm_reduce(acc, slab, cnt, tile, split, &flag, fence)) return;
    float s1[SM_NJ][4], s2[SM_NJ][4];
#pragma unroll
    for (int j = 0; j < SM_NJ; ++j) {
      const int c = c0 + sm_col(wn, lane, j);
      float mean = 0.0f, sc = 0.0f, sh = 0.0f;
      if (bb.h) {
        mean = bb.stats[c];
        sc = bb.stats[2 * C + c];
        sh = bb.stats[3 * C + c];
      }
      // the producing BN layer's input row of each dx element (routed by its pool code)
      uint32_t hr[4];
#pragma unroll
      for (int e = 0; e < 4; ++e) hr[e] = (uint32_t)((n0 + sm_row(wm, lane, e)) * 4 + ip);
      if (bb.h && bb.code) {
        uint8_t kc[4];
#pragma unroll
        for (int e = 0; e < 4; ++e) kc[e] = bb.code[(size_t)hr[e] * C + c];
#pragma unroll
        for (int e = 0; e < 4; ++e) hr[e] = cf_pool_row(hr[e], 4u, 2u, kc[e]);
      }
      float xv[4] = {0.0f, 0.0f, 0.0f, 0.0f}, rv[4] = {0.0f, 0.0f, 0.0f, 0.0f};
      if (bb.h) {
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          xv[e] = bb.h[(size_t)hr[e] * C + c];
          if (bb.res) rv[e] = bb.res[(size_t)hr[e] * C + c];
        }
      }
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int n = n0 + sm_row(wm, lane, e);
        const float d = acc.a[j][e];
        dx[((long long)n * 4 + ip) * C + c] = d;
        s1[j][e] = s2[j][e] = 0.0f;
        if (bb.h) {
          float v = xv[e] * sc + sh;  // the BN kernels' arithmetic (no contraction)
          if (bb.res) v = v + rv[e];
          const float dz = (bb.relu == 0 || !(v <= 0.0f)) ? d : 0.0f;
          s1[j][e] = dz;
          s2[j][e] = dz * (xv[e] - mean);
        }
      }
    }
    if (bb.h && bnpart) {
      const int nrows = (N / SM_BM) * 4;
      sm_colsums(s1, s2, smem, bnpart, nrows, mt * 4 + ip, C, c0, fin.ngrp != 0);
      if (fin.ngrp) {
        // the BN backward finalisation of this channel tile, by its last row tile (the weight-
        // gradient blocks of the launch keep running beside it)
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        if (t == 0) {
          const int prev = __hip_atomic_fetch_add(fcnt + ct, 1, __ATOMIC_RELAXED,
                                                  __HIP_MEMORY_SCOPE_AGENT);
          const int last = prev == nrows - 1;
          if (last) __hip_atomic_store(fcnt + ct, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          flag = last;
        }
        __syncthreads();
        if (flag && t < SM_BN) ew_bn_bwd_fin_chan<2, true>(fin, c0 + t);
      }
    }
    return;
  }
  // weight gradient: dw[o][tap][c] = sum over the tap's pairs and the batch
  const int b = (int)blockIdx.x - nbd;
  const int ots = Nc / SM_BN, cts = C / SM_BN, per = ots * cts;
  // centre tap (4 pairs) first, then the edges 1, 3, 5, 7 (2), then the corners 0, 2, 6, 8 (1)
  const int ti = b / per, rem = b % per;
  const int tap = ti == 0 ? 4 : ti <= 4 ? 2 * ti - 1 : 2 * (ti - 5) + (ti >= 7 ? 2 : 0);
  const int ot = rem / cts, ct = rem % cts;
  const int o0 = ot * SM_BN, c0 = ct * SM_BN;
  const int np = sm_npairs(tap);
  const int kr = t >> 4, cq = (t & 15) * 4;  // both RC: k-rows n = kr (+ 32), columns +cq
  SmDyCoef k;
  if constexpr (DK >= 2) sm_dy_coef(ds, Nc, o0 + cq, k);
  RawX xc;  // hoisted BN scale / shift of the thread's 4 x channels
  if constexpr (XK == 1) {
    xc.sc = *reinterpret_cast<const f32x4*>(xs.stats + 2 * C + c0 + cq);
    xc.sh = *reinterpret_cast<const f32x4*>(xs.stats + 3 * C + c0 + cq);
  }
  const int spp = N / SM_BK;  // k-steps per pair
  struct RawDyOp {
    RawDy r;
    int op;
  };
  // producer staging (dgc_stage.h): the tile's velocity / residual (/ parameter) loads issued
  // here, ahead of the k-loop, so they are in registers by the epilogue
  float su[SM_NJ][4], sr[SM_NJ][4], sp[SM_NJ][4];
  if (st.vel) {
#pragma unroll
    for (int j = 0; j < SM_NJ; ++j)
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const long long i =
            ((long long)(o0 + sm_row(wm, lane, e)) * 9 + tap) * C + c0 + sm_col(wn, lane, j);
        su[j][e] = st.vel[i];
        sr[j][e] = st.resid[i];
        sp[j][e] = st.wd != 0.0f ? st.param[i] : 0.0f;
      }
  }
  SmAcc acc;
  sm_gemm<SM_RC, SM_RC, RawDyOp, RawX>(
      smem, np * spp,
      [&](int s, RawDyOp& r) {
        const int p = s / spp, n = (s - p * spp) * SM_BK + kr;
        int ip, op;
        sm_pair(tap, p, ip, op);
        r.op = op;
        sm_raw_dy<DK>(ds, Nc, n, op, o0 + cq, false, r.r);
      },
      [&](int s, RawX& r) {
        const int p = s / spp, n = (s - p * spp) * SM_BK + kr;
        int ip, op;
        sm_pair(tap, p, ip, op);
        sm_raw_x<XK>(xs, ((long long)n * 4 + ip) * C + c0 + cq, 32LL * 4 * C, nullptr, C, r);
        if constexpr (XK == 1) {
          r.sc = xc.sc;
          r.sh = xc.sh;
        }
      },
      [&](const RawDyOp& r, int i) { return sm_make_dy<DK>(ds, r.op, r.r, k, i); },
      [&](const RawX& r, int i) { return sm_make_x<XK>(r, i); }, acc);
  if (st.vel) {  // the encode's error-feedback staging here (dgc_stage.h): dw is never stored
    const float lr = st.lr_ptr ? *st.lr_ptr : 1.0f;
#pragma unroll
    for (int j = 0; j < SM_NJ; ++j)
#pragma unroll
      for (int e = 0; e < 4; ++e)
        dgc_stage_loaded(st, lr,
                         ((long long)(o0 + sm_row(wm, lane, e)) * 9 + tap) * C + c0 +
                             sm_col(wn, lane, j),
                         acc.a[j][e], su[j][e], sr[j][e], sp[j][e]);
    if (b == 0 && t == 0) *st.stamp = 1u;  // read by the encode, a later kernel
    return;
  }
#pragma unroll
  for (int j = 0; j < SM_NJ; ++j)
#pragma unroll
    for (int e = 0; e < 4; ++e)
      dw[((long long)(o0 + sm_row(wm, lane, e)) * 9 + tap) * C + c0 + sm_col(wn, lane, j)] =
          acc.a[j][e];
}

void sm_check(long long N, int C, int Nc) {
  if (N <= 0 || N % SM_BM || C % SM_BN || Nc % SM_BN ||
      N * 4 * (long long)std::max(C, Nc) >= (1LL << 31) || (long long)Nc * 9 * C >= (1LL << 31))
    throw std::runtime_error("ewdml small-map conv: needs N % 64 == 0, C_in and C_out % 64 == 0");
}

}  // namespace

static int sm_fence() {
  if (g_sm_fence < 0) {
    const char* e = std::getenv("EWDML_SM_FENCE");
    g_sm_fence = (e && e[0] == '1') ? 1 : 0;
  }
  return g_sm_fence;
}

int ew_sm_set_fence(int on) {
  const int prev = sm_fence();
  g_sm_fence = on ? 1 : 0;
  return prev;
}

long long ew_sm_f32_ws_floats(long long N, int C, int Nc) {
  return 4LL * N * 4 * std::max(C, Nc);
}
long long ew_sm_f32_counters(long long N, int C, int Nc) {
  // the tile tickets, then one finalisation ticket per 64-channel tile (k_sm_bwd)
  return (N / SM_BM) * 4 * (std::max(C, Nc) / SM_BN) + std::max(C, Nc) / SM_BN;
}

// y [N][2][2][Nc] = conv(x) with x materialised (bn_h == 0) or relu(bn_h * scale + shift) of the
// BN layer in front (bn_stats [4][C], nbt its num_batches_tracked or 0).  bnpart [2][rows][Nc]:
// the output's BN partial sums; returns the rows written (0: none requested / no room).
int ew_sm_f32_fwd(uintptr_t x, uintptr_t bn_h, uintptr_t bn_stats, uintptr_t nbt, uintptr_t w,
                  uintptr_t y, uintptr_t slab, long long slab_floats, uintptr_t cnt,
                  long long cnt_ints, long long N, int C, int Nc, uintptr_t bnpart,
                  long long bnpart_floats, uintptr_t stream) {
  sm_check(N, C, Nc);
  const long long tiles = (N / SM_BM) * 4 * (Nc / SM_BN);
  if (slab_floats < 4 * tiles * SM_TILE || cnt_ints < tiles)
    throw std::runtime_error("ewdml small-map conv: workspace too small");
  const int rows = (int)((N / SM_BM) * 4);
  float* bp = reinterpret_cast<float*>(bnpart);
  if (bp && 2LL * rows * Nc > bnpart_floats) bp = nullptr;
  const SmX xs{reinterpret_cast<const float*>(x), reinterpret_cast<const float*>(bn_h),
               reinterpret_cast<const float*>(bn_stats), reinterpret_cast<long long*>(nbt)};
  const dim3 grid((unsigned)(4 * tiles));
  auto* sp = reinterpret_cast<float*>(slab);
  auto* cp = reinterpret_cast<int*>(cnt);
  const float* wp = reinterpret_cast<const float*>(w);
  float* yp = reinterpret_cast<float*>(y);
  if (bn_h)
    hipLaunchKernelGGL(k_sm_fwd<1>, grid, dim3(SM_T), 0, (hipStream_t)stream, xs, wp, yp, sp, cp,
                       (int)N, C, Nc, bp, sm_fence());
  else
    hipLaunchKernelGGL(k_sm_fwd<0>, grid, dim3(SM_T), 0, (hipStream_t)stream, xs, wp, yp, sp, cp,
                       (int)N, C, Nc, bp, sm_fence());
  EW_CHECK_LAUNCH();
  return bp ? rows : 0;
}

// Backward data (dx != 0) and weight gradient (dw != 0) in one launch.  x: as the forward's
// (x or bn_h / bn_stats); dy: materialised (dy != 0) or the backward of the BN layer this conv
// feeds (out_h = this conv's output, out_dnext, out_code (pool 2x2 -> 1x1), out_stats, out_coef).
// pb_*: the BN(+ReLU)(+pool)(+residual) layer that produced x, whose backward sums (sum dz,
// sum dz * (h - mean)) go to bnpart [2][rows][C]; returns the rows written.
int ew_sm_f32_bwd(uintptr_t x, uintptr_t bn_h, uintptr_t bn_stats, uintptr_t dy,
                  uintptr_t out_h, uintptr_t out_dnext, uintptr_t out_code, uintptr_t out_stats,
                  uintptr_t out_coef, int out_pool, uintptr_t w, uintptr_t dx, uintptr_t dw,
                  uintptr_t slab, long long slab_floats, uintptr_t cnt, long long cnt_ints,
                  long long N, int C, int Nc, uintptr_t pb_h, uintptr_t pb_res, uintptr_t pb_code,
                  uintptr_t pb_stats, int pb_relu, uintptr_t bnpart, long long bnpart_floats,
                  uintptr_t fin_coef, uintptr_t fin_dgamma, uintptr_t fin_dbeta,
                  uintptr_t fin_dcbias, int fin_cb_bf16, long long fin_M, uintptr_t stream,
                  uintptr_t st_vel, uintptr_t st_resid, uintptr_t st_param, float st_momentum,
                  float st_damp1, float st_wd, int st_nesterov, uintptr_t st_lr,
                  uintptr_t st_stamp) {
  sm_check(N, C, Nc);
  const DgcStage st{reinterpret_cast<float*>(st_vel), reinterpret_cast<float*>(st_resid),
                    reinterpret_cast<const float*>(st_param), st_momentum, st_damp1, st_wd,
                    st_nesterov, reinterpret_cast<const float*>(st_lr),
                    reinterpret_cast<uint32_t*>(st_stamp)};
  if (st.vel && !(dw && st.resid && st.stamp && (st.wd == 0.0f || st.param)))
    throw std::runtime_error("ewdml small-map conv: error-feedback staging arguments missing");
  if (!dy && !(out_h && out_dnext && out_stats && out_coef))
    throw std::runtime_error("ewdml small-map conv: backward needs dy or its BN source");
  if (out_h && out_pool && !out_code)
    throw std::runtime_error("ewdml small-map conv: pooled BN source needs its codes");
  const long long tiles = (N / SM_BM) * 4 * (C / SM_BN);
  if (dx && (slab_floats < 4 * tiles * SM_TILE || cnt_ints < tiles))
    throw std::runtime_error("ewdml small-map conv: workspace too small");
  const int nbd = dx ? (int)(4 * tiles) : 0;
  const int nbw = dw ? 9 * (Nc / SM_BN) * (C / SM_BN) : 0;
  if (nbd + nbw == 0) return 0;
  const int rows = (int)((N / SM_BM) * 4);
  float* bp = reinterpret_cast<float*>(bnpart);
  if (!pb_h || (bp && 2LL * rows * C > bnpart_floats)) bp = nullptr;
  const SmX xs{reinterpret_cast<const float*>(x), reinterpret_cast<const float*>(bn_h),
               reinterpret_cast<const float*>(bn_stats), nullptr};
  const SmDy ds{reinterpret_cast<const float*>(dy), reinterpret_cast<const float*>(out_h),
                reinterpret_cast<const float*>(out_dnext),
                reinterpret_cast<const uint8_t*>(out_code),
                reinterpret_cast<const float*>(out_stats), reinterpret_cast<const float*>(out_coef),
                out_pool};
  // the dx map is the producing BN layer's (pooled) output: 2 x 2
  const CfBnBwd bb{bp ? reinterpret_cast<const float*>(pb_h) : nullptr,
                   reinterpret_cast<const float*>(pb_res), reinterpret_cast<const uint8_t*>(pb_code),
                   reinterpret_cast<const float*>(pb_stats), pb_relu, 2, 2};
  const dim3 grid((unsigned)(nbd + nbw));
  auto* sp = reinterpret_cast<float*>(slab);
  auto* cp = reinterpret_cast<int*>(cnt);
  // fin_coef: that layer's backward finalisation rides here (coef [2][C], dgamma, dbeta, dcbias
  // as k_bn_bwd_finalize<2> forms them from bnpart, bitwise), one ticket per 64-channel tile in
  // cnt[tiles ..)
  EwBnFin fin{};
  if (fin_coef && bp) {
    if (cnt_ints < tiles + C / SM_BN || fin_M <= 0)
      throw std::runtime_error("ewdml small-map conv: finalisation tickets / rows missing");
    fin = EwBnFin{bp, reinterpret_cast<const float*>(pb_stats), reinterpret_cast<float*>(fin_coef),
                  reinterpret_cast<float*>(fin_dgamma), reinterpret_cast<float*>(fin_dbeta),
                  reinterpret_cast<void*>(fin_dcbias), fin_M, rows, C, fin_cb_bf16,
                  (C + EW_FIN_CH - 1) / EW_FIN_CH};
  }
  const float* wp = reinterpret_cast<const float*>(w);
  float* dxp = reinterpret_cast<float*>(dx);
  float* dwp = reinterpret_cast<float*>(dw);
#define SM_BWD(XK_, DK_)                                                                         \
  hipLaunchKernelGGL((k_sm_bwd<XK_, DK_>), grid, dim3(SM_T), 0, (hipStream_t)stream, xs, ds, wp, \
                     dxp, dwp, sp, cp, (int)N, C, Nc, nbd, bb, bp, sm_fence(), fin, cp + tiles, \
                     st)
  // DK: dy materialised (0), formed from the BN layer it feeds (2), that layer pooled 2x2 -> 1x1 (3)
  const int dk = dy ? 0 : out_pool ? 3 : 2;
  if (bn_h) {
    if (dk == 0) SM_BWD(1, 0);
    else if (dk == 2) SM_BWD(1, 2);
    else SM_BWD(1, 3);
  } else {
    if (dk == 0) SM_BWD(0, 0);
    else if (dk == 2) SM_BWD(0, 2);
    else SM_BWD(0, 3);
  }
#undef SM_BWD
  EW_CHECK_LAUNCH();
  return bp ? rows : 0;
}
