// Momentum-corrected error-feedback staging (DGC; compress/oracle.py dgc_accumulate) done by a
// gradient's PRODUCER instead of the top-k encode's first pass: the kernel that forms a weight
// gradient element writes the velocity and the vector to compress,
//   g' = g + p wd ; u = m u + (1 - dampening) g' ; d = g' + m u (Nesterov) | u ; (d *= lr) ;
//   e = r + d        (u -> vel, e -> resid; the gradient itself is never stored)
// and stamps the tensor; the encode (topk_codec.hip topk_ef_stage) then reads e from the residual
// for a stamped tensor instead of reading gradient, residual and velocity and writing the last
// two (and clears the stamp).  The expressions are topk_ef_stage's, one for one: with
// -ffp-contract=off every product and sum rounds on its own, so both give the same bits.
#pragma once
#include <stdint.h>

struct DgcStage {
  float* vel;          // the bucket's velocity at this tensor's first element (null: off)
  float* resid;        // its residual (the staged e)
  const float* param;  // its parameters (read when wd != 0)
  float momentum, damp1, wd;
  int nesterov;
  const float* lr_ptr;  // nullable: lr-scaled accumulation (--ef-mode local)
  uint32_t* stamp;      // the tensor's word in the encode's stamp array (set to 1)
};

// element i with its velocity u0, residual r0 and parameter p0 already loaded (a producer issues
// those loads before its own k-loop, so they land while it computes)
__device__ __forceinline__ void dgc_stage_loaded(const DgcStage& d, float lr, long long i, float g,
                                                 float u0, float r0, float p0) {
  if (d.wd != 0.0f) g = g + p0 * d.wd;
  const float a = u0 * d.momentum;
  const float b = g * d.damp1;
  const float u = a + b;
  float dd = u;
  if (d.nesterov) {
    const float mu = u * d.momentum;
    dd = g + mu;
  }
  if (d.lr_ptr) dd = dd * lr;
  d.vel[i] = u;
  d.resid[i] = r0 + dd;
}

__device__ __forceinline__ void dgc_stage_elem(const DgcStage& d, float lr, long long i, float g) {
  if (d.wd != 0.0f) g = g + d.param[i] * d.wd;
  const float u0 = d.vel[i];
  const float a = u0 * d.momentum;
  const float b = g * d.damp1;
  const float u = a + b;
  float dd = u;
  if (d.nesterov) {
    const float mu = u * d.momentum;
    dd = g + mu;
  }
  if (d.lr_ptr) dd = dd * lr;
  d.vel[i] = u;
  d.resid[i] = d.resid[i] + dd;
}
