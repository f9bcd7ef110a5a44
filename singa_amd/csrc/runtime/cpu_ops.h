// CppCPU compute backend of the host runtime: the reference's CPU math
// (mshadow's CPU evaluation loops + CBLAS sgemm, include/mshadow/tensor_cpu-inl.hpp:52-165,
// include/mshadow/tensor_expr_engine-inl.hpp:272-298; the layers of
// src/worker/layer.cc:18-764) as native C++ over raw host pointers, run on a
// persistent worker pool.  Layouts: activations NCHW fp32 (the CppCPU
// device's layout), weights [K][C/g][R][S].  Op codes and semantics are those
// of the GPU kernels (csrc/kernels/*.hip), so one Python dispatch layer
// (singa_amd/ops) drives both devices.
#pragma once
#include <stdint.h>

#include <functional>

namespace sgrt {
namespace cpu {

// Persistent pool: f(begin, end) over [0, n) in chunks of >= grain.  A call
// made while the pool is busy (another thread's op, or from inside a task)
// runs inline on the calling thread.
void ParallelFor(int64_t n, int64_t grain, const std::function<void(int64_t, int64_t)>& f);
int NumThreads();

// C = alpha * op(A) op(B) (+ beta C) (+ bias[n]) (ReLU); op(A) [M][K] (ta: A stored [K][M]),
// op(B) [K][N] (tb: B stored [N][K]); row-major with leading dims.
void Gemm(bool ta, bool tb, int64_t M, int64_t N, int64_t K, float alpha, const float* A, int64_t lda, const float* B,
          int64_t ldb, float beta, float* C, int64_t ldc, const float* bias, bool relu);

// unary op codes of csrc/kernels/elementwise.hip
void UnaryFwd(int op, const float* x, float* y, int64_t n, float a);
void UnaryBwd(int op, const float* x, const float* y, const float* dy, float* dx, int64_t n, float a);

// dtype codes of singa_amd/ops/native.py: 0 f32, 1 bf16, 2 f16(raw), 3 i32, 4 i64, 5 u8
void CopyNd(const void* src, int dti, void* dst, int dto, int nd, const int64_t* size, const int64_t* dst_st,
            const int64_t* src_st);
void BinaryNd(int op, const float* a, const float* b, float* out, int nd, const int64_t* size, const int64_t* os,
              const int64_t* as, const int64_t* bs, float alpha);
void Fill(void* p, int64_t n, int dt, double v);
// out = c ? a : b (c: bytes, non-zero = true), broadcasting strides like BinaryNd
void WhereNd(const uint8_t* c, const float* a, const float* b, float* out, int nd, const int64_t* size,
             const int64_t* os, const int64_t* as, const int64_t* bs, const int64_t* cs);
// y = clamp(a x + b, lo, hi); with dy: dx = dy * a inside (lo, hi), else 0
void ClampAffine(const float* x, const float* dy, float* y, int64_t n, float a, float b, float lo, float hi);
void EasgdDiff(float* w, const float* c, float* d, int64_t n, float alpha);
void AffineElasticSample(const float* img, const float* theta, const float* disp, float* out, int B, int H, int W);
void GaussBlur2D(const float* in, float* out, int N, int H, int W, const float* g, int k);
void ResizeBilinear(const float* in, float* out, int B, int H, int W, int h, int w);
void RsyncGather(const float* w, const float* snap, float* buf, int64_t m, int64_t n, int64_t a, int64_t b);
void RsyncScatter(float* w, float* snap, const float* buf, int64_t m, int64_t n, int64_t a, int64_t b);
// y[outer][inner] = op over j of x[outer][j][inner]; ops: 0 sum 1 mean 2 max 3 min 4 sumsq
void Reduce(const float* x, float* y, int64_t outer, int64_t red, int64_t inner, int op);

void SoftmaxRows(const float* x, float* y, int64_t rows, int64_t C);
void SoftmaxRowsBwd(const float* y, const float* dy, float* dx, int64_t rows, int64_t C);
// labels (int32 / int64 by lab64) or soft targets t[B][C]; loss / correct [B]; dx optional
void SoftmaxXent(const float* x, const void* lab, int lab64, const float* t, float* loss, float* correct, float* dx,
                 int64_t B, int64_t C, int topk, float gs);

// convolution, NCHW; w [K][C/g][R][S]; dw accumulated (+=)
void ConvFwd(const float* x, const float* w, const float* bias, float* y, int N, int C, int H, int W, int K, int R,
             int S, int Ho, int Wo, int sh, int sw, int ph, int pw, int dh, int dw, int groups);
void ConvBwd(const float* x, const float* w, const float* dy, float* dx, float* dwt, float* db, int N, int C, int H,
             int W, int K, int R, int S, int Ho, int Wo, int sh, int sw, int ph, int pw, int dh, int dw, int groups);

// pooling, NCHW; arg = int32 flat index into the H*W plane (max)
void PoolFwd(const float* x, float* y, int32_t* arg, int N, int C, int H, int W, int Ho, int Wo, int kh, int kw,
             int sh, int sw, int ph, int pw, int is_max, int count_include_pad);
void PoolBwd(const float* dy, const int32_t* arg, float* dx, int N, int C, int H, int W, int Ho, int Wo, int kh,
             int kw, int sh, int sw, int ph, int pw, int is_max, int count_include_pad);

// across-channel LRN, NCHW (reference kLRN, src/worker/layer.cc:331-378)
void LrnFwd(const float* x, float* y, int N, int C, int HW, int size, float alpha, float beta, float k);
void LrnBwd(const float* x, const float* dy, float* dx, int N, int C, int HW, int size, float alpha, float beta,
            float k);

// inverted dropout with the GPU kernels' Philox stream (bit-identical masks)
void DropoutFwd(const float* x, float* y, uint8_t* mask, int64_t n, float pkeep, uint64_t seed, uint64_t offset);
void DropoutBwd(const float* dy, const uint8_t* mask, float* dx, int64_t n, float pkeep);
void RandFill(float* y, int64_t n, int dist, float a, float b, uint64_t seed, uint64_t offset);

// batch norm over NCHW (or [B][C] with HW = 1); running stats updated in training
void BatchNormFwd(const float* x, const float* gamma, const float* beta, float* rm, float* rv, float* y, float* mean,
                  float* invstd, int N, int C, int64_t HW, int training, float momentum, float eps, int relu,
                  const float* residual);
// ReLU mask: y_for_mask > 0, or (relu_x) x * scale + shift > 0; dres (optional) = the masked dy
void BatchNormBwd(const float* x, const float* dy, const float* gamma, const float* mean, const float* invstd,
                  const float* y_for_mask, int relu_x, const float* scale, const float* shift, float* dx, float* dg,
                  float* db, float* dres, int N, int C, int64_t HW);
void LayerNormFwd(const float* x, const float* g, const float* b, float* y, float* mean, float* rstd, int64_t R,
                  int64_t D, float eps);
void LayerNormBwd(const float* x, const float* dy, const float* g, const float* mean, const float* rstd, float* dx,
                  float* dg, float* db, int64_t R, int64_t D);

void IndexSelect(const void* src, const void* idx, int idx64, void* dst, int64_t outer, int64_t nsrc, int64_t inner,
                 int64_t nidx, int esize);
void IndexAdd(float* dst, const void* idx, int idx64, const float* src, int64_t outer, int64_t ndst, int64_t inner,
              int64_t nidx, float alpha);

}  // namespace cpu
}  // namespace sgrt
