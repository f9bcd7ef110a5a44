// Native updaters + learning-rate schedules (reference C13,
// src/utils/updater.cc:11-182) for host-resident fp32 parameters: the CppCPU
// device's optimiser step and the native parameter server's server-side
// update (ps.cc).  The GPU path runs the same math in optim.hip.
//
// Semantics are the INTENDED ones: grad_scale
// multiplies the gradient before every use (the reference's SGD ignored it
// and AdaGrad/RMSProp/AdaDelta applied it inside the history term only),
// Nesterov's momentum is initialised.  Kinds match singa_amd.opt._KIND.
//
// Large buffers are split over the CppCPU worker pool (the reference's
// mshadow CPU loops were single-threaded SSE2); every element's update is
// independent, so the result does not depend on the split.
#include <algorithm>
#include <cmath>
#include <stdexcept>
#include <string>
#include <thread>
#include <vector>

#include "cpu_ops.h"
#include "runtime.h"

namespace sgrt {

namespace {

// the CppCPU device's persistent worker pool (cpu_ops.cc): no thread start-up
// per step, inline when called from inside another parallel region
template <typename F>
void parallel_for(int64_t n, int64_t grain, F&& f) {
  cpu::ParallelFor(n, grain, [&f](int64_t b, int64_t e) { f(b, e); });
}

}  // namespace

int UpdaterKind(const std::string& name) {
  // codes shared with singa_amd.opt._KIND and optim.hip
  static const char* names[] = {"sgd", "nesterov_ref", "adagrad", "rmsprop", "adadelta", "adam", "sgd_ref"};
  for (int i = 0; i < 7; ++i)
    if (name == names[i]) return i;
  throw std::invalid_argument("unknown updater kind: " + name);
}

namespace {

// One kind's update over [b, e).  The kind, the presence of the per-element
// lr / wd / mask vectors and momentum != 0 are compile-time, so every inner
// loop is branch-free and auto-vectorises (AVX2 at -O3); masked elements keep
// their old weight and state through selects.
template <int K, bool VEC, bool MOM>
void UpdateRange(const UpdateArgs& a, float* __restrict w, const float* __restrict g, float* __restrict s1,
                 float* __restrict s2, const float* __restrict lr_vec, const float* __restrict wd_vec,
                 const uint8_t* __restrict mask, float bc1, float bc2, int64_t b, int64_t e) {
  const float gs = a.grad_scale, mom = a.momentum, damp1 = 1.f - a.dampening, rho = a.rho, rho1 = 1.f - a.rho;
  const float b1 = a.beta1, b1c = 1.f - a.beta1, b2 = a.beta2, b2c = 1.f - a.beta2, eps = a.eps;
  const bool nest = a.nesterov, adamw = a.adamw;
#pragma GCC ivdep
  for (int64_t i = b; i < e; ++i) {
    const bool on = VEC ? mask == nullptr || mask[i] != 0 : true;
    const float lr = VEC && lr_vec ? a.lr * lr_vec[i] : a.lr;
    const float wd = VEC && wd_vec ? a.wd * wd_vec[i] : a.wd;
    const float wi = w[i];
    float gv = g[i] * gs;
    if (!(K == kAdam && adamw)) gv += wd * wi;
    float upd = 0.f, n1 = 0.f, n2 = 0.f;
    if constexpr (K == kSGD) {
      if constexpr (MOM) {
        n1 = mom * s1[i] + damp1 * gv;
        gv = nest ? gv + mom * n1 : n1;
      }
      upd = lr * gv;
    } else if constexpr (K == kSGDRef) {  // h = m*h + lr*g; w -= h  (src/utils/updater.cc:62-80)
      if constexpr (MOM) {
        n1 = mom * s1[i] + lr * gv;
        upd = n1;
      } else {
        upd = lr * gv;
      }
    } else if constexpr (K == kNesterovRef) {  // h0 = h; h = m*h + lr*g; w -= (1+m)*h - m*h0  (:89-105)
      const float h0 = s1[i];
      n1 = mom * h0 + lr * gv;
      upd = (1.f + mom) * n1 - mom * h0;
    } else if constexpr (K == kAdaGrad) {  // h += g^2; w -= lr*g/sqrt(h+delta)  (:115-128)
      n1 = s1[i] + gv * gv;
      upd = lr * gv / std::sqrt(n1 + eps);
    } else if constexpr (K == kRMSProp) {  // h = rho*h + (1-rho)*g^2  (:140-153)
      n1 = rho * s1[i] + rho1 * gv * gv;
      upd = lr * gv / std::sqrt(n1 + eps);
    } else if constexpr (K == kAdaDelta) {  // (:163-182)
      n1 = rho * s1[i] + rho1 * gv * gv;
      const float d = gv * std::sqrt(s2[i] + eps) / std::sqrt(n1 + eps);
      n2 = rho * s2[i] + rho1 * d * d;
      upd = lr * d;
    } else if constexpr (K == kAdam) {
      n1 = b1 * s1[i] + b1c * gv;
      n2 = b2 * s2[i] + b2c * gv * gv;
      upd = lr * (n1 / bc1 / (std::sqrt(n2 / bc2) + eps) + (adamw ? wd * wi : 0.f));
    }
    constexpr bool S1 = K != kSGD && K != kSGDRef ? true : MOM;
    constexpr bool S2 = K == kAdaDelta || K == kAdam;
    if constexpr (S1) s1[i] = on ? n1 : s1[i];
    if constexpr (S2) s2[i] = on ? n2 : s2[i];
    w[i] = on ? wi - upd : wi;
  }
}

template <int K, bool MOM>
void Dispatch(const UpdateArgs& a, float* w, const float* g, float* s1, float* s2, int64_t n, const float* lr_vec,
              const float* wd_vec, const uint8_t* mask, float bc1, float bc2) {
  const bool vec = lr_vec || wd_vec || mask;
  parallel_for(n, 1 << 15, [&](int64_t b, int64_t e) {
    if (vec)
      UpdateRange<K, true, MOM>(a, w, g, s1, s2, lr_vec, wd_vec, mask, bc1, bc2, b, e);
    else
      UpdateRange<K, false, MOM>(a, w, g, s1, s2, lr_vec, wd_vec, mask, bc1, bc2, b, e);
  });
}

}  // namespace

void OptUpdate(const UpdateArgs& a, float* w, const float* g, float* s1, float* s2, int64_t n, const float* lr_vec,
               const float* wd_vec, const uint8_t* mask) {
  if (n <= 0) return;
  const bool need_s1 = a.kind != kSGD || a.momentum != 0.f;
  if (need_s1 && !s1) throw std::invalid_argument("OptUpdate: slot 1 required");
  if ((a.kind == kAdaDelta || a.kind == kAdam) && !s2) throw std::invalid_argument("OptUpdate: slot 2 required");
  const float bc1 = a.kind == kAdam ? 1.f - std::pow(a.beta1, a.t) : 1.f;
  const float bc2 = a.kind == kAdam ? 1.f - std::pow(a.beta2, a.t) : 1.f;
  const bool mom = a.momentum != 0.f;
#define SG_UPD(K)                                                              \
  (mom ? Dispatch<K, true>(a, w, g, s1, s2, n, lr_vec, wd_vec, mask, bc1, bc2) \
       : Dispatch<K, false>(a, w, g, s1, s2, n, lr_vec, wd_vec, mask, bc1, bc2))
  switch (a.kind) {
    case kSGD: SG_UPD(kSGD); break;
    case kSGDRef: SG_UPD(kSGDRef); break;
    case kNesterovRef: SG_UPD(kNesterovRef); break;
    case kAdaGrad: SG_UPD(kAdaGrad); break;
    case kRMSProp: SG_UPD(kRMSProp); break;
    case kAdaDelta: SG_UPD(kAdaDelta); break;
    case kAdam: SG_UPD(kAdam); break;
    default: break;
  }
#undef SG_UPD
}

// reference GetLearningRate (src/utils/updater.cc:11-51); kLinear clamps at
// the final rate instead of extrapolating past freq steps
double LearningRate(const std::string& method, double base, double final_lr, int freq, double gamma, double pw,
                    int64_t step) {
  const double f = std::max(1, freq);
  if (method == "kFixed") return base;
  if (method == "kLinear") {
    const double r = step / f;
    return r < 1.0 ? (1.0 - r) * base + r * final_lr : final_lr;
  }
  if (method == "kExponential") return base / std::pow(2.0, step / f);
  if (method == "kInverse_t") return base / (1.0 + step / final_lr);
  if (method == "kInverse") return base * std::pow(1.0 + gamma * step, -pw);
  if (method == "kStep") return base * std::pow(gamma, (double)(step / (int64_t)f));
  throw std::invalid_argument("unknown learning-rate change method: " + method);
}

}  // namespace sgrt
