// Device-side optimizer updates with the TF 1.x formulas of rocfm/optim/tf_optim.py
// (reference: PS:292-307 / HVD:281-297).  One element at a time; callers vectorise.
#pragma once
#include "../common.h"

namespace rocfm {

enum OptType : int { kAdam = 0, kAdagrad = 1, kMomentum = 2, kFtrl = 3, kGD = 4 };

struct OptParams {
  int type = kAdam;
  float lr = 5e-4f;
  float beta1 = 0.9f, beta2 = 0.999f, eps = 1e-8f;
  float momentum = 0.95f;
  float ftrl_lr_power = -0.5f, ftrl_l1 = 0.f, ftrl_l2 = 0.f;
  const float* lrt = nullptr;  // precomputed step-dependent lr_t (written by fetch_batch), or null
};

// Halted step: the side chain's batch preparation sets this bit in a step's device global_step when
// the input pipeline has flagged an error (a malformed record parsed on the GPU, decode.hip): every
// optimizer update of that step is skipped, so a bad batch never reaches the parameters, the slots or
// a checkpoint (tf.data's parse_example fails before the batch is used, PS:117-132).  The low 32 bits
// (dropout keys, tags) are unchanged.
constexpr int64_t kHaltStepBit = 1ll << 62;

// Step-dependent scalars, computed once per thread from the device step counter (t = step+1).
struct OptStep {
  float lr_t;  // Adam: lr·√(1−β2ᵗ)/(1−β1ᵗ); others: lr
  bool skip;   // halted step (kHaltStepBit): no update
};

__host__ __device__ inline float adam_lr_t(float lr, float beta1, float beta2, int64_t step) {
  const double t = (double)(step + 1);
  return (float)((double)lr * sqrt(1.0 - pow((double)beta2, t)) / (1.0 - pow((double)beta1, t)));
}

__device__ __forceinline__ OptStep opt_step(const OptParams& o, int64_t step) {
  OptStep s;
  s.skip = (step & kHaltStepBit) != 0;
  if (o.lrt) {
    s.lr_t = *o.lrt;
  } else if (o.type == kAdam) {
    s.lr_t = adam_lr_t(o.lr, o.beta1, o.beta2, step);
  } else {
    s.lr_t = o.lr;
  }
  return s;
}

// The gradient every embedding-row update feeds opt_apply: g + λ·w as ONE explicit fused
// multiply-add, so every kernel that applies it (step tail, merges, dense update) rounds it the same
// way whatever the surrounding code lets the compiler contract.
__device__ __forceinline__ float l2_grad(float g, float l2, float w) { return __fmaf_rn(l2, w, g); }

// In-place update of param p and slots s0/s1 with gradient g.
__device__ __forceinline__ void opt_apply(const OptParams& o, const OptStep& st, float& p, float g, float& s0,
                                          float& s1) {
  // the fused multiply-adds are explicit (__fmaf_rn) and nothing else may be contracted: the update
  // is then the same bits in every kernel that inlines it, with the FMAs kept (round 5 had turned
  // contraction off altogether)
#pragma clang fp contract(off)
  if (st.skip) return;
  switch (o.type) {
    case kAdam: {
      s0 = __fmaf_rn(o.beta1, s0, (1.f - o.beta1) * g);
      s1 = __fmaf_rn(o.beta2, s1, ((1.f - o.beta2) * g) * g);
      p -= (st.lr_t * s0) / (sqrtf(s1) + o.eps);
      break;
    }
    case kAdagrad: {
      s0 = __fmaf_rn(g, g, s0);
      p = __fmaf_rn(-(o.lr * g), rsqrtf(s0), p);
      break;
    }
    case kMomentum: {
      s0 = __fmaf_rn(o.momentum, s0, g);
      p = __fmaf_rn(-o.lr, s0, p);
      break;
    }
    case kFtrl: {
      const float acc_new = __fmaf_rn(g, g, s0);
      // TF's ApplyFtrl special-cases the default lr_power = -0.5 with sqrt; powf otherwise
      float pn, po;
      if (o.ftrl_lr_power == -0.5f) {
        pn = sqrtf(acc_new);
        po = sqrtf(s0);
      } else {
        pn = powf(acc_new, -o.ftrl_lr_power);
        po = powf(s0, -o.ftrl_lr_power);
      }
      const float sigma = (pn - po) / o.lr;
      s1 += __fmaf_rn(-sigma, p, g);
      const float quad = __fmaf_rn(2.f, o.ftrl_l2, pn / o.lr);
      p = fabsf(s1) > o.ftrl_l1 ? (copysignf(o.ftrl_l1, s1) - s1) / quad : 0.f;
      s0 = acc_new;
      break;
    }
    default:
      p = __fmaf_rn(-o.lr, g, p);
  }
}

}  // namespace rocfm
