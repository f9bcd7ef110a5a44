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
// Large buffers are split over a small pool of std::threads (the reference's
// mshadow CPU loops were single-threaded SSE2); every element's update is
// independent, so the result does not depend on the split.
#include <algorithm>
#include <cmath>
#include <stdexcept>
#include <string>
#include <thread>
#include <vector>

#include "runtime.h"

namespace sgrt {

namespace {

template <typename F>
void parallel_for(int64_t n, int64_t grain, F&& f) {
  const unsigned hw = std::max(1u, std::thread::hardware_concurrency());
  const int64_t chunks = std::min<int64_t>(hw, (n + grain - 1) / grain);
  if (chunks <= 1) {
    f(0, n);
    return;
  }
  std::vector<std::thread> th;
  const int64_t step = (n + chunks - 1) / chunks;
  for (int64_t c = 1; c < chunks; ++c) {
    const int64_t b = c * step, e = std::min(n, b + step);
    if (b < e) th.emplace_back([&f, b, e] { f(b, e); });
  }
  f(0, std::min(n, step));
  for (auto& t : th) t.join();
}

}  // namespace

int UpdaterKind(const std::string& name) {
  // codes shared with singa_amd.opt._KIND and optim.hip
  static const char* names[] = {"sgd", "nesterov_ref", "adagrad", "rmsprop", "adadelta", "adam", "sgd_ref"};
  for (int i = 0; i < 7; ++i)
    if (name == names[i]) return i;
  throw std::invalid_argument("unknown updater kind: " + name);
}

void OptUpdate(const UpdateArgs& a, float* w, const float* g, float* s1, float* s2, int64_t n, const float* lr_vec,
               const float* wd_vec, const uint8_t* mask) {
  if (n <= 0) return;
  const bool need_s1 = a.kind != kSGD || a.momentum != 0.f;
  if (need_s1 && !s1) throw std::invalid_argument("OptUpdate: slot 1 required");
  if ((a.kind == kAdaDelta || a.kind == kAdam) && !s2) throw std::invalid_argument("OptUpdate: slot 2 required");
  const float bc1 = a.kind == kAdam ? 1.f - std::pow(a.beta1, a.t) : 1.f;
  const float bc2 = a.kind == kAdam ? 1.f - std::pow(a.beta2, a.t) : 1.f;
  parallel_for(n, 1 << 16, [&](int64_t b, int64_t e) {
    for (int64_t i = b; i < e; ++i) {
      if (mask && !mask[i]) continue;
      const float lr = lr_vec ? a.lr * lr_vec[i] : a.lr;
      const float wd = wd_vec ? a.wd * wd_vec[i] : a.wd;
      float gv = g[i] * a.grad_scale;
      if (!(a.kind == kAdam && a.adamw)) gv += wd * w[i];
      float upd;
      switch (a.kind) {
        case kSGD:
          if (a.momentum != 0.f) {
            s1[i] = a.momentum * s1[i] + (1.f - a.dampening) * gv;
            gv = a.nesterov ? gv + a.momentum * s1[i] : s1[i];
          }
          upd = lr * gv;
          break;
        case kSGDRef:  // h = m*h + lr*g; w -= h  (src/utils/updater.cc:62-80)
          if (a.momentum > 0.f) {
            s1[i] = a.momentum * s1[i] + lr * gv;
            upd = s1[i];
          } else {
            upd = lr * gv;
          }
          break;
        case kNesterovRef: {  // h0 = h; h = m*h + lr*g; w -= (1+m)*h - m*h0  (:89-105)
          const float h0 = s1[i];
          s1[i] = a.momentum * h0 + lr * gv;
          upd = (1.f + a.momentum) * s1[i] - a.momentum * h0;
          break;
        }
        case kAdaGrad:  // h += g^2; w -= lr*g/sqrt(h+delta)  (:115-128)
          s1[i] += gv * gv;
          upd = lr * gv / std::sqrt(s1[i] + a.eps);
          break;
        case kRMSProp:  // h = rho*h + (1-rho)*g^2  (:140-153)
          s1[i] = a.rho * s1[i] + (1.f - a.rho) * gv * gv;
          upd = lr * gv / std::sqrt(s1[i] + a.eps);
          break;
        case kAdaDelta: {  // (:163-182)
          s1[i] = a.rho * s1[i] + (1.f - a.rho) * gv * gv;
          const float d = gv * std::sqrt(s2[i] + a.eps) / std::sqrt(s1[i] + a.eps);
          s2[i] = a.rho * s2[i] + (1.f - a.rho) * d * d;
          upd = lr * d;
          break;
        }
        case kAdam: {
          s1[i] = a.beta1 * s1[i] + (1.f - a.beta1) * gv;
          s2[i] = a.beta2 * s2[i] + (1.f - a.beta2) * gv * gv;
          const float mh = s1[i] / bc1, vh = s2[i] / bc2;
          upd = lr * (mh / (std::sqrt(vh) + a.eps) + (a.adamw ? wd * w[i] : 0.f));
          break;
        }
        default:
          upd = 0.f;
      }
      w[i] -= upd;
    }
  });
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
