// pybind11 entry point of the singa_amd gfx950 kernel library (_C).
//
// Every launcher takes raw device pointers (uintptr_t from torch's caching
// allocator) and the hipStream_t of the caller's current stream, so kernels
// are stream-ordered with everything else and capture into HIP graphs.
// Shape / dtype validation happens on the Python side (singa_amd/ops/native.py)
// before anything is launched.
#include <hip/hip_runtime.h>
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>
#include <stdint.h>
#include <stdexcept>
#include <string>
#include <vector>

namespace py = pybind11;
typedef uintptr_t P;
#define V(x) ((void*)(x))
#define CV(x) ((const void*)(x))
#define S(x) ((hipStream_t)(x))

extern "C" {
void sg_unary_fwd(int, const void*, void*, int64_t, int, float, hipStream_t);
void sg_unary_bwd(int, const void*, const void*, const void*, void*, int64_t, int, float, hipStream_t);
void sg_add_act(const void*, const void*, void*, int64_t, int, float, float, int, hipStream_t);
void sg_relu_bwd_from_y(const void*, const void*, void*, int64_t, int, hipStream_t);
void sg_mask_bits_apply(const void*, const void*, void*, int64_t, hipStream_t);
void sg_zero_ranges(void*, const void*, int, hipStream_t);
void sg_cast(const void*, int, void*, int, int64_t, hipStream_t);
void sg_dropout_fwd(const void*, void*, void*, int64_t, int, float, uint64_t, uint64_t, const void*, hipStream_t);
void sg_dropout_bwd(const void*, const void*, void*, int64_t, int, float, hipStream_t);
void sg_rand_fill(void*, int64_t, int, int, float, float, uint64_t, uint64_t, hipStream_t);
void sg_nchw_to_nhwc_pad(const void*, void*, int, int, int, int, int, hipStream_t);
void sg_nchw_to_nhwc_pad_bf16(const void*, void*, int, int, int, int, int, hipStream_t);
void sg_bn_relu_maxpool(const void*, const void*, const void*, void*, void*, int, int, int, int, int, int, int, int, int,
                        int, int, int, hipStream_t);
void sg_nchw_to_pairs(const void*, void*, int, int, int, int, hipStream_t);
void sg_softmax_fwd(const void*, void*, int64_t, int, int, int, hipStream_t);
void sg_softmax_bwd(const void*, const void*, void*, int64_t, int, int, hipStream_t);
void sg_softmax_xent(const void*, const void*, const void*, void*, void*, void*, int64_t, int, int, int, float,
                     hipStream_t);
void sg_layernorm_fwd(const void*, const void*, const void*, void*, void*, void*, int64_t, int, int, float,
                      hipStream_t);
void sg_softmax_rows(const void*, void*, int64_t, int, int, int, hipStream_t);
void sg_gemm_heads(const void*, int64_t, int, const void*, int64_t, int, void*, int64_t, int, int, int, float, float,
                   const void*, int, int, int, int, int64_t, int64_t, int64_t, int, int64_t, int64_t, int64_t,
                   hipStream_t);
void sg_lrn_rows(const void*, const void*, void*, int64_t, int, int, float, float, float, int, int, hipStream_t);
int64_t sg_layernorm_bwd_ws(int64_t, int);
void sg_drop_add_ln_fwd(const void*, const void*, const void*, const void*, void*, void*, void*, void*, void*, int64_t,
                        int, int, float, float, uint64_t, uint64_t, const void*, hipStream_t);
void sg_drop_add_ln_bwd(const void*, const void*, const void*, const void*, const void*, const void*, float, void*,
                        void*, void*, void*, void*, void*, int64_t, int, int, hipStream_t);
void sg_layernorm_bwd_v2(const void*, const void*, const void*, const void*, const void*, void*, void*, void*, void*,
                         int64_t, int, int, hipStream_t);
void sg_layernorm_bwd(const void*, const void*, const void*, const void*, const void*, void*, void*, void*, int64_t,
                      int, int, hipStream_t);
int sg_colreduce_bands(int64_t, int);
int64_t sg_colreduce_ws(int64_t, int);
int sg_conv_stats_rows(int, int);
void sg_bn_set_deterministic(int);
int sg_bn_deterministic();
void sg_colsum(const void*, void*, void*, void*, int64_t, int, int, int, hipStream_t);
void sg_bn_fwd_stats(const void*, void*, const void*, const void*, void*, void*, void*, void*, void*, void*, int64_t,
                     int, float, float, int, hipStream_t);
void sg_bn_infer_params(const void*, const void*, const void*, const void*, void*, void*, void*, void*, int, float,
                        hipStream_t);
void sg_bn_apply(const void*, const void*, const void*, const void*, void*, void*, int64_t, int, int, int, hipStream_t);
void sg_set_wt_ready(int);
void sg_wt_transpose_batched(const void*, int, int, hipStream_t);
void sg_bn_apply2(const void*, const void*, const void*, const void*, const void*, const void*, void*, void*, int64_t,
                  int, int, int, hipStream_t);
void sg_bn_bwd2(const void*, const void*, const void*, const void*, const void*, const void*, const void*, const void*,
                const void*, const void*, void*, void*, void*, void*, void*, void*, void*, void*, void*, void*, int64_t,
                int, int, hipStream_t);
void sg_bn_bwd(const void*, const void*, const void*, const void*, const void*, const void*, const void*, const void*,
               void*, void*, void*, void*, void*, void*, int64_t, int, int, int, hipStream_t);
void sg_bn_bwd_pool(const void*, const void*, const void*, const void*, const void*, const void*, const void*,
                    const void*, void*, void*, void*, void*, void*, int, int, int, int, int, int, int, int, int, int,
                    int, int, hipStream_t);
void sg_pool_fwd(const void*, void*, void*, int, int, int, int, int, int, int, int, int, int, int, int, int, int, int,
                 hipStream_t);
void sg_pool_bwd(const void*, const void*, void*, int, int, int, int, int, int, int, int, int, int, int, int, int, int,
                 int, hipStream_t);
void sg_gap_fwd(const void*, void*, int, int, int, int, hipStream_t);
void sg_gap_bwd(const void*, void*, int, int, int, int, hipStream_t);
void sg_lrn_fwd(const void*, void*, void*, int64_t, int, int, float, float, float, int, hipStream_t);
void sg_lrn_bwd(const void*, const void*, const void*, void*, int64_t, int, int, float, float, int, hipStream_t);
void sg_opt_update(int, void*, const void*, void*, void*, void*, const void*, const void*, const void*, const void*,
                   const void*, const void*, int, float, float, float, float, float, float, float, float, int, int,
                   hipStream_t);
void sg_sqnorm(const void*, int64_t, void*, hipStream_t);
void sg_easgd_diff(void*, const void*, void*, int64_t, float, hipStream_t);
void sg_axpy(void*, const void*, int64_t, float, hipStream_t);
void sg_rsync_gather(const void*, const void*, void*, int64_t, int64_t, int64_t, int64_t, hipStream_t);
void sg_rsync_scatter(void*, void*, const void*, int64_t, int64_t, int64_t, int64_t, hipStream_t);
void sg_gemm(const void*, int64_t, int, const void*, int64_t, int, void*, int64_t, int, int, int, float, float,
             const void*, int, int, int, int, int64_t, int64_t, int64_t, hipStream_t);
void sg_conv_fwd(const void*, const void*, void*, const void*, int, int, int, int, int, int, int, int, int, int, int,
                 int, int, int, int, int, int, void*, hipStream_t);
void sg_bn_fwd_from_ws(const void*, int, const void*, const void*, void*, void*, void*, void*, void*, void*, int64_t,
                       int, float, float, hipStream_t);
void sg_set_ws_prezeroed(int);
void sg_zero(void*, int64_t, hipStream_t);
void sg_conv_dgrad_bn(const void*, const void*, void*, int, int, int, int, int, int, int, int, int, int, int, int,
                      int, int, int, int, float, void*, void*, const void*, const void*, const void*, const void*,
                      const void*, hipStream_t);
void sg_conv_dgrad_bn_ex(const void*, const void*, void*, int, int, int, int, int, int, int, int, int, int, int, int,
                         int, int, int, int, float, void*, void*, const void*, const void*, const void*, const void*,
                         const void*, const void*, hipStream_t);
void sg_bn_bwd_from_ws(const void*, const void*, const void*, const void*, const void*, const void*, const void*,
                       const void*, const void*, int, void*, void*, void*, void*, void*, int64_t, int, int, int,
                       hipStream_t);
int sg_conv_dgrad_res(const void*, const void*, void*, int, int, int, int, int, int, int, int, int, int, int, int, int,
                      int, int, void*, const void*, const void*, hipStream_t);
void sg_conv_dgrad(const void*, const void*, void*, int, int, int, int, int, int, int, int, int, int, int, int, int,
                   int, int, int, float, void*, hipStream_t);
void sg_conv_wgrad(const void*, const void*, void*, int, int, int, int, int, int, int, int, int, int, int, int, int,
                   int, int, int, hipStream_t);
void sg_wdot_colsum(const void*, const void*, int, int, float, void*, int, const void*, const void*, float,
                    hipStream_t);
void sg_bn_bwd_wdot(const void*, const void*, const void*, const void*, const void*, const void*, const void*,
                    const void*, const void*, const void*, const void*, void*, void*, void*, void*, void*, void*,
                    int64_t, int, float, hipStream_t);
void sg_ggemm(int, const void*, int64_t, int, int64_t, const void*, int64_t, int, int64_t, void*, int64_t, int64_t,
              int, int, int, float, float, const void*, int, int, int, int, float*, int, const void*, void*,
              hipStream_t);
void sg_ggemm_tune(int, int);
int sg_ggemm_last_dma();
void sg_bnres_tune(int, int);
int sg_stem_fwd(const void*, const void*, void*, void*, int, int, int, int, int, hipStream_t);
void sg_conv3x3_set(int);
int sg_conv3x3_enabled();
void sg_bnres_wgrad(const void*, const void*, void*, int, int, int, hipStream_t);
void sg_bnres_dgrad(const void*, const void*, const void*, const void*, void*, int, int, int, void*, const void*,
                    hipStream_t);
void sg_bnres_coef(const void*, const void*, const void*, const void*, const void*, const void*, int, int, int, void*,
                   void*, void*, void*, void*, hipStream_t);
void sg_bnres_combine(const void*, const void*, const void*, const void*, int, const void*, const void*, int, int,
                      void*, void*, void*, void*, const void*, const void*, float, hipStream_t);
void sg_bnres_masksum(const void*, const void*, void*, void*, int64_t, int, hipStream_t);
void sg_set_dgrad_mask_out(int);
void sg_bn_apply_cs(const void*, const void*, const void*, void*, void*, void*, int64_t, int, int, hipStream_t);
void sg_conv_dgrad_gsum(const void*, const void*, void*, int, int, int, int, int, int, int, int, int, int, int, int,
                        int, int, int, void*, const void*, void*, const void*, int, int, int, hipStream_t);
int sg_sk_tail_ok(int, int, int);
void sg_bnres_gram_stats(const void*, const void*, const void*, int, int, int, void*, hipStream_t);
int sg_sk_tail2(const void*, const void*, const void*, const void*, const void*, void*, void*, int, int, int, int,
                hipStream_t);
void sg_bnres_fold(const void*, const void*, const void*, const void*, const void*, const void*, int, int, int, void*,
                   void*, void*, hipStream_t);
void sg_strided_pick(const void*, void*, int, int, int, int, int, int, int, int, hipStream_t);
int sg_sk_tail(const void*, const void*, void*, void*, const void*, const void*, const void*, void*, int, int, int, int,
               hipStream_t);
void sg_workq_set(int);
int sg_workq_enabled();
int sg_cu_count();
void sg_cu_hog(int, double, int, int*, hipStream_t);
int sg_fattn_ok(int, int);
int sg_fattn_fwd(const void*, void*, float*, const float*, int64_t, int, int, int, int, float, hipStream_t);
int sg_fattn_bwd(const void*, const void*, const void*, const float*, const float*, int64_t, void*, float*, int, int,
                 int, int, float, hipStream_t);
int sg_loop_allreduce(const void* const*, void* const*, int, int64_t, int, int, hipStream_t);
void* sg_workq_arena_begin();
void sg_workq_arena_end();
void sg_workq_arena_free(void*);
int sg_workq_arena_slots(void*);
int sg_gemm_act(const void*, int64_t, int, const void*, int64_t, int, void*, int64_t, int, int, int, float, const void*,
                int, int64_t, int64_t, int64_t, int, void*, int, const void*, float*, hipStream_t);
void sg_gconv_fwd(int, const void*, const void*, void*, const void*, int, int, int, int, int, int, int, int, int, int,
                  int, int, int, int, int, int, int, int, hipStream_t);
void sg_gconv_dgrad(int, const void*, const void*, void*, int, int, int, int, int, int, int, int, int, int, int, int,
                    int, int, int, int, int, float, hipStream_t);
void sg_gconv_wgrad(int, const void*, const void*, void*, int, int, int, int, int, int, int, int, int, int, int, int,
                    int, int, int, int, int, hipStream_t);
void sg_copy_nd(const void*, int, void*, int, int, const int64_t*, const int64_t*, const int64_t*, hipStream_t);
void sg_binary_nd(int, const void*, const void*, void*, int, int, const int64_t*, const int64_t*, const int64_t*,
                  const int64_t*, float, hipStream_t);
void sg_where_nd(const void*, const void*, const void*, void*, int, int, const int64_t*, const int64_t*,
                 const int64_t*, const int64_t*, const int64_t*, hipStream_t);
void sg_reduce(const void*, int, void*, int, int64_t, int64_t, int64_t, int, hipStream_t);
void sg_index_select(const void*, const void*, int, void*, int64_t, int64_t, int64_t, int64_t, int, hipStream_t);
void sg_index_add(void*, const void*, int, const void*, int, int64_t, int64_t, int64_t, int64_t, float, hipStream_t);
void sg_gather_el(const void*, const void*, int, void*, int, int64_t, int64_t, int64_t, int64_t, hipStream_t);
void sg_scatter_el(void*, const void*, int, const void*, int, int64_t, int64_t, int64_t, int64_t, int, hipStream_t);
void sg_pad_nd(const void*, void*, int, int, const int64_t*, const int64_t*, const int64_t*, const int64_t*, int, float,
               hipStream_t);
void sg_pad_bwd(const void*, void*, int, int, const int64_t*, const int64_t*, const int64_t*, const int64_t*, int,
                hipStream_t);
void sg_fill(void*, int64_t, int, double, hipStream_t);
void sg_iadd_i64(void*, int64_t, int64_t, hipStream_t);
void sg_kth_largest_abs(const void*, int64_t, int64_t, void*, void*, hipStream_t);
void sg_clamp_affine(const void*, const void*, void*, int64_t, int, float, float, float, float, hipStream_t);
void sg_set_tuning(int key, int value);
int sg_get_tuning(int key);
void sg_bn_set_unroll(int);
void sg_bn_set_rows_per_thread(int);
}

void register_rccl(py::module& m);  // csrc/comm/rccl_comm.cpp
void register_mem(py::module& m);   // csrc/mem/pool.cpp
void register_loop(py::module& m);  // csrc/comm/loop_comm.cpp
void register_stream_graph(py::module& m);  // csrc/mem/stream_graph.cpp

static void check_launch(const char* what) {
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) throw std::runtime_error(std::string(what) + ": " + hipGetErrorString(e));
}
#define CHK(name) check_launch(name)

PYBIND11_MODULE(_C, m) {
  m.doc() = "singa_amd gfx950 HIP kernel library";
  register_rccl(m);
  register_mem(m);
  register_loop(m);
  register_stream_graph(m);

  m.def("device_info", []() {
    py::dict d;
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess) n = 0;
    d["count"] = n;
    if (n > 0) {
      hipDeviceProp_t pr;
      if (hipGetDeviceProperties(&pr, 0) == hipSuccess) {
        d["name"] = std::string(pr.name);
        d["gcnArchName"] = std::string(pr.gcnArchName);
        d["multiProcessorCount"] = pr.multiProcessorCount;
        d["sharedMemPerBlock"] = (int64_t)pr.sharedMemPerBlock;
        d["maxSharedMemoryPerMultiProcessor"] = (int64_t)pr.maxSharedMemoryPerMultiProcessor;
        d["warpSize"] = pr.warpSize;
        d["totalGlobalMem"] = (int64_t)pr.totalGlobalMem;
      }
    }
    return d;
  });

  m.def("unary_fwd", [](int op, P x, P y, int64_t n, int dt, float a, P s) {
    sg_unary_fwd(op, CV(x), V(y), n, dt, a, S(s)); CHK("unary_fwd");
  });
  m.def("unary_bwd", [](int op, P x, P y, P dy, P dx, int64_t n, int dt, float a, P s) {
    sg_unary_bwd(op, CV(x), CV(y), CV(dy), V(dx), n, dt, a, S(s)); CHK("unary_bwd");
  });
  m.def("add_act", [](P a, P b, P y, int64_t n, int dt, float al, float be, int relu, P s) {
    sg_add_act(CV(a), CV(b), V(y), n, dt, al, be, relu, S(s)); CHK("add_act");
  });
  m.def("zero_ranges", [](P base, P ranges, int nr, P s) {
    sg_zero_ranges(V(base), CV(ranges), nr, S(s));
    CHK("zero_ranges");
  });
  m.def("mask_bits_apply", [](P g, P mask, P out, int64_t n, P s) {
    sg_mask_bits_apply(CV(g), CV(mask), V(out), n, S(s)); CHK("mask_bits_apply");
  });
  m.def("relu_bwd_from_y", [](P y, P dy, P dx, int64_t n, int dt, P s) {
    sg_relu_bwd_from_y(CV(y), CV(dy), V(dx), n, dt, S(s)); CHK("relu_bwd_from_y");
  });
  m.def("cast", [](P x, int dtx, P y, int dty, int64_t n, P s) {
    sg_cast(CV(x), dtx, V(y), dty, n, S(s)); CHK("cast");
  });
  m.def("dropout_fwd", [](P x, P y, P mask, int64_t n, int dt, float pk, uint64_t seed, uint64_t off, P epoch, P s) {
    sg_dropout_fwd(CV(x), V(y), V(mask), n, dt, pk, seed, off, CV(epoch), S(s)); CHK("dropout_fwd");
  });
  m.def("dropout_bwd", [](P dy, P mask, P dx, int64_t n, int dt, float pk, P s) {
    sg_dropout_bwd(CV(dy), CV(mask), V(dx), n, dt, pk, S(s)); CHK("dropout_bwd");
  });
  m.def("rand_fill", [](P y, int64_t n, int dt, int dist, float a, float b, uint64_t seed, uint64_t off, P s) {
    sg_rand_fill(V(y), n, dt, dist, a, b, seed, off, S(s)); CHK("rand_fill");
  });
  m.def("bn_relu_maxpool", [](P x, P scale, P shift, P y, P arg, int N, int H, int W, int C, int Ho, int Wo, int kh,
                              int kw, int sh, int sw, int ph, int pw, P s) {
    sg_bn_relu_maxpool(CV(x), CV(scale), CV(shift), V(y), V(arg), N, H, W, C, Ho, Wo, kh, kw, sh, sw, ph, pw, S(s));
    CHK("bn_relu_maxpool");
  });
  m.def("nchw_to_pairs", [](P x, P y, int N, int C, int H, int W, P s) {
    sg_nchw_to_pairs(CV(x), V(y), N, C, H, W, S(s)); CHK("nchw_to_pairs");
  });
  m.def("nchw_to_nhwc_pad_bf16", [](P x, P y, int N, int C, int H, int W, int Cp, P s) {
    sg_nchw_to_nhwc_pad_bf16(CV(x), V(y), N, C, H, W, Cp, S(s));
    CHK("nchw_to_nhwc_pad_bf16");
  });
  m.def("nchw_to_nhwc_pad", [](P x, P y, int N, int C, int H, int W, int Cp, P s) {
    sg_nchw_to_nhwc_pad(CV(x), V(y), N, C, H, W, Cp, S(s)); CHK("nchw_to_nhwc_pad");
  });
  m.def("softmax_fwd", [](P x, P y, int64_t R, int C, int dt, int out_f32, P s) {
    sg_softmax_fwd(CV(x), V(y), R, C, dt, out_f32, S(s)); CHK("softmax_fwd");
  });
  m.def("softmax_bwd", [](P y, P dy, P dx, int64_t R, int C, int dt, P s) {
    sg_softmax_bwd(CV(y), CV(dy), V(dx), R, C, dt, S(s)); CHK("softmax_bwd");
  });
  m.def("softmax_xent", [](P x, P lab, P soft, P loss, P correct, P dx, int64_t R, int C, int dt, int topk,
                           float gs, P s) {
    sg_softmax_xent(CV(x), CV(lab), CV(soft), V(loss), V(correct), V(dx), R, C, dt, topk, gs, S(s));
    CHK("softmax_xent");
  });
  m.def("layernorm_fwd", [](P x, P g, P b, P y, P mean, P rstd, int64_t R, int D, int dt, float eps, P s) {
    sg_layernorm_fwd(CV(x), CV(g), CV(b), V(y), V(mean), V(rstd), R, D, dt, eps, S(s)); CHK("layernorm_fwd");
  });
  m.def("softmax_rows", [](P x, P y, int64_t R, int C, int idt, int odt, P s) {
    sg_softmax_rows(CV(x), V(y), R, C, idt, odt, S(s));
    CHK("softmax_rows");
  });
  m.def("layernorm_bwd", [](P x, P dy, P g, P mean, P rstd, P dx, P dg, P db, int64_t R, int D, int dt, P s) {
    sg_layernorm_bwd(CV(x), CV(dy), CV(g), CV(mean), CV(rstd), V(dx), V(dg), V(db), R, D, dt, S(s));
    CHK("layernorm_bwd");
  });
  m.def("layernorm_bwd_ws", [](int64_t R, int D) { return sg_layernorm_bwd_ws(R, D); });
  m.def("drop_add_ln_fwd", [](P x, P a, P g, P b, P s_out, P mask, P y, P mean, P rstd, int64_t R, int D, int dt,
                              float eps, float pkeep, uint64_t seed, uint64_t offset, P epoch, P s) {
    sg_drop_add_ln_fwd(CV(x), CV(a), CV(g), CV(b), V(s_out), V(mask), V(y), V(mean), V(rstd), R, D, dt, eps, pkeep,
                       seed, offset, CV(epoch), S(s));
    CHK("drop_add_ln_fwd");
  });
  m.def("drop_add_ln_bwd", [](P x, P dy, P g, P mean, P rstd, P mask, float pkeep, P dx, P da, P dg, P db, P cs, P ws,
                              int64_t R, int D, int dt, P s) {
    sg_drop_add_ln_bwd(CV(x), CV(dy), CV(g), CV(mean), CV(rstd), CV(mask), pkeep, V(dx), V(da), V(dg), V(db), V(cs),
                       V(ws), R, D, dt, S(s));
    CHK("drop_add_ln_bwd");
  });
  m.def("layernorm_bwd_v2", [](P x, P dy, P g, P mean, P rstd, P dx, P dg, P db, P ws, int64_t R, int D, int dt, P s) {
    sg_layernorm_bwd_v2(CV(x), CV(dy), CV(g), CV(mean), CV(rstd), V(dx), V(dg), V(db), V(ws), R, D, dt, S(s));
    CHK("layernorm_bwd_v2");
  });
  m.def("colreduce_bands", [](int64_t R, int C) { return sg_colreduce_bands(R, C); });
  m.def("colreduce_ws", [](int64_t R, int C) { return sg_colreduce_ws(R, C); });
  m.def("conv_stats_rows", [](int M, int N) { return sg_conv_stats_rows(M, N); });
  m.def("set_deterministic", [](int on) { sg_bn_set_deterministic(on); });
  m.def("deterministic", []() { return sg_bn_deterministic(); });
  m.def("colsum", [](P x, P ws, P o0, P o1, int64_t R, int C, int dt, int acc, P s) {
    sg_colsum(CV(x), V(ws), V(o0), V(o1), R, C, dt, acc, S(s)); CHK("colsum");
  });
  m.def("bn_fwd_stats", [](P x, P ws, P gamma, P beta, P rm, P rv, P mean, P invstd, P scale, P shift, int64_t R,
                           int C, float mom, float eps, int dt, P s) {
    sg_bn_fwd_stats(CV(x), V(ws), CV(gamma), CV(beta), V(rm), V(rv), V(mean), V(invstd), V(scale), V(shift), R, C,
                    mom, eps, dt, S(s));
    CHK("bn_fwd_stats");
  });
  m.def("bn_infer_params", [](P g, P b, P rm, P rv, P scale, P shift, P mean, P invstd, int C, float eps, P s) {
    sg_bn_infer_params(CV(g), CV(b), CV(rm), CV(rv), V(scale), V(shift), V(mean), V(invstd), C, eps, S(s));
    CHK("bn_infer_params");
  });
  m.def("bn_apply", [](P x, P scale, P shift, P res, P y, int64_t R, int C, int relu, int dt, P s, P mask) {
    sg_bn_apply(CV(x), CV(scale), CV(shift), CV(res), V(y), V(mask), R, C, relu, dt, S(s)); CHK("bn_apply");
  });
  m.def("bn_bwd", [](P x, P dy, P y, P scale, P shift, P mean, P invstd, P gamma, P ws, P coef, P dg, P db, P dx,
                     P dres, int64_t R, int C, int mask_mode, int dt, P s) {
    sg_bn_bwd(CV(x), CV(dy), CV(y), CV(scale), CV(shift), CV(mean), CV(invstd), CV(gamma), V(ws), V(coef), V(dg),
              V(db), V(dx), V(dres), R, C, mask_mode, dt, S(s));
    CHK("bn_bwd");
  });
  m.def("bn_bwd_pool", [](P x, P dyp, P arg, P scale, P shift, P mean, P invstd, P gamma, P ws, P coef, P dg, P db,
                          P dx, int N, int H, int W, int C, int Ho, int Wo, int kh, int kw, int sh, int sw, int ph,
                          int pw, P s) {
    sg_bn_bwd_pool(CV(x), CV(dyp), CV(arg), CV(scale), CV(shift), CV(mean), CV(invstd), CV(gamma), V(ws), V(coef),
                   V(dg), V(db), V(dx), N, H, W, C, Ho, Wo, kh, kw, sh, sw, ph, pw, S(s));
    CHK("bn_bwd_pool");
  });
  m.def("set_wt_ready", [](int on) { sg_set_wt_ready(on); });
  m.def("wt_transpose_batched", [](P desc, int n, int total, P s) {
    sg_wt_transpose_batched(CV(desc), n, total, S(s));
    CHK("wt_transpose_batched");
  });
  m.def("bn_apply2", [](P x, P scale, P shift, P x2, P scale2, P shift2, P y, P mask, int64_t R, int C, int relu,
                        int dt, P s) {
    sg_bn_apply2(CV(x), CV(scale), CV(shift), CV(x2), CV(scale2), CV(shift2), V(y), V(mask), R, C, relu, dt, S(s));
    CHK("bn_apply2");
  });
  m.def("bn_bwd2", [](P x, P dy, P mask, P mean, P invstd, P gamma, P x2, P mean2, P invstd2, P gamma2, P ws, P ws2,
                      P coef, P coef2, P dg, P db, P dg2, P db2, P dx, P dx2, int64_t R, int C, int dt, P s) {
    sg_bn_bwd2(CV(x), CV(dy), CV(mask), CV(mean), CV(invstd), CV(gamma), CV(x2), CV(mean2), CV(invstd2), CV(gamma2),
               V(ws), V(ws2), V(coef), V(coef2), V(dg), V(db), V(dg2), V(db2), V(dx), V(dx2), R, C, dt, S(s));
    CHK("bn_bwd2");
  });
  m.def("pool_fwd", [](P x, P y, P arg, int N, int H, int W, int C, int Ho, int Wo, int kh, int kw, int sh, int sw,
                       int ph, int pw, int is_max, int cp, int dt, P s) {
    sg_pool_fwd(CV(x), V(y), V(arg), N, H, W, C, Ho, Wo, kh, kw, sh, sw, ph, pw, is_max, cp, dt, S(s));
    CHK("pool_fwd");
  });
  m.def("pool_bwd", [](P dy, P arg, P dx, int N, int H, int W, int C, int Ho, int Wo, int kh, int kw, int sh, int sw,
                       int ph, int pw, int is_max, int cp, int dt, P s) {
    sg_pool_bwd(CV(dy), CV(arg), V(dx), N, H, W, C, Ho, Wo, kh, kw, sh, sw, ph, pw, is_max, cp, dt, S(s));
    CHK("pool_bwd");
  });
  m.def("gap_fwd", [](P x, P y, int N, int HW, int C, int dt, P s) {
    sg_gap_fwd(CV(x), V(y), N, HW, C, dt, S(s)); CHK("gap_fwd");
  });
  m.def("gap_bwd", [](P dy, P dx, int N, int HW, int C, int dt, P s) {
    sg_gap_bwd(CV(dy), V(dx), N, HW, C, dt, S(s)); CHK("gap_bwd");
  });
  m.def("lrn_fwd", [](P x, P y, P norm, int64_t R, int C, int size, float al, float be, float k, int dt, P s) {
    sg_lrn_fwd(CV(x), V(y), V(norm), R, C, size, al, be, k, dt, S(s)); CHK("lrn_fwd");
  });
  m.def("lrn_bwd", [](P x, P dy, P norm, P dx, int64_t R, int C, int size, float al, float be, int dt, P s) {
    sg_lrn_bwd(CV(x), CV(dy), CV(norm), V(dx), R, C, size, al, be, dt, S(s)); CHK("lrn_bwd");
  });
  m.def("opt_update", [](int kind, P w, P g, P s1, P s2, P wlow, P cstart, P clen, P cseg, P seg_lr, P seg_wd, P hp,
                         int nchunks, float mom, float damp, float wd, float gs, float b1, float b2, float eps,
                         float rho, int nesterov, int adamw, P s) {
    sg_opt_update(kind, V(w), CV(g), V(s1), V(s2), V(wlow), CV(cstart), CV(clen), CV(cseg), CV(seg_lr), CV(seg_wd),
                  CV(hp), nchunks, mom, damp, wd, gs, b1, b2, eps, rho, nesterov, adamw, S(s));
    CHK("opt_update");
  });
  m.def("sqnorm", [](P x, int64_t n, P out, P s) { sg_sqnorm(CV(x), n, V(out), S(s)); CHK("sqnorm"); });
  m.def("easgd_diff", [](P w, P c, P d, int64_t n, float alpha, P s) {
    sg_easgd_diff(V(w), CV(c), V(d), n, alpha, S(s)); CHK("easgd_diff");
  });
  m.def("axpy", [](P y, P x, int64_t n, float a, P s) { sg_axpy(V(y), CV(x), n, a, S(s)); CHK("axpy"); });
  m.def("rsync_gather", [](P w, P snap, P out, int64_t mm, int64_t n, int64_t a, int64_t b, P s) {
    sg_rsync_gather(CV(w), CV(snap), V(out), mm, n, a, b, S(s)); CHK("rsync_gather");
  });
  m.def("rsync_scatter", [](P w, P snap, P dsum, int64_t mm, int64_t n, int64_t a, int64_t b, P s) {
    sg_rsync_scatter(V(w), V(snap), CV(dsum), mm, n, a, b, S(s)); CHK("rsync_scatter");
  });
  m.def("gemm", [](P a, int64_t lda, int ako, P b, int64_t ldb, int bko, P c, int64_t ldc, int M, int N, int K,
                   float alpha, float beta, P bias, int relu, int out_mode, int splits, int batch, int64_t sa,
                   int64_t sb, int64_t sc, P s) {
    sg_gemm(CV(a), lda, ako, CV(b), ldb, bko, V(c), ldc, M, N, K, alpha, beta, CV(bias), relu, out_mode, splits,
            batch, sa, sb, sc, S(s));
    CHK("gemm");
  });
  m.def("gemm_heads", [](P a, int64_t lda, int ako, P b, int64_t ldb, int bko, P c, int64_t ldc, int M, int N, int K,
                         float alpha, float beta, int out_mode, int batch, int64_t sa, int64_t sb, int64_t sc, int bh,
                         int64_t sa2, int64_t sb2, int64_t sc2, P s) {
    sg_gemm_heads(CV(a), lda, ako, CV(b), ldb, bko, V(c), ldc, M, N, K, alpha, beta, nullptr, 0, out_mode, 1, batch,
                  sa, sb, sc, bh, sa2, sb2, sc2, S(s));
    CHK("gemm_heads");
  });
  // fused multi-head attention over the in-place [B][S][3][H][D] projection (fattn.hip)
  m.def("fattn_ok", [](int S, int D) { return sg_fattn_ok(S, D); });
  m.def("fattn_fwd", [](P qkv, P o, P lse, P mask, int64_t mstride, int B, int S, int H, int D, float scale, P s) {
    const int rc = sg_fattn_fwd(CV(qkv), V(o), (float*)V(lse), (const float*)CV(mask), mstride, B, S, H, D, scale, S(s));
    if (rc != 0) throw std::runtime_error("fattn_fwd: unsupported shape or launch failure (" + std::to_string(rc) + ")");
    CHK("fattn_fwd");
  });
  m.def("fattn_bwd", [](P qkv, P o, P dout, P lse, P mask, int64_t mstride, P dqkv, P dbias, int B, int S, int H,
                        int D, float scale, P s) {
    const int rc = sg_fattn_bwd(CV(qkv), CV(o), CV(dout), (const float*)CV(lse), (const float*)CV(mask), mstride,
                                V(dqkv), (float*)V(dbias), B, S, H, D, scale, S(s));
    if (rc != 0) throw std::runtime_error("fattn_bwd: unsupported shape or launch failure (" + std::to_string(rc) + ")");
    CHK("fattn_bwd");
  });
  m.def("lrn_rows", [](P x, P dy, P out, int64_t R, int C, int size, float alpha, float beta, float k, int bwd, int dt,
                       P s) {
    sg_lrn_rows(CV(x), CV(dy), V(out), R, C, size, alpha, beta, k, bwd, dt, S(s));
    CHK("lrn_rows");
  });
  m.def("conv_fwd", [](P x, P w, P y, P bias, int N, int H, int W, int C, int K, int R, int Sd, int Ho, int Wo,
                       int sh, int sw, int ph, int pw, int dh, int dw, int relu, int out_mode, P s, P stats) {
    sg_conv_fwd(CV(x), CV(w), V(y), CV(bias), N, H, W, C, K, R, Sd, Ho, Wo, sh, sw, ph, pw, dh, dw, relu, out_mode,
                V(stats), S(s));
    CHK("conv_fwd");
  }, py::arg("x"), py::arg("w"), py::arg("y"), py::arg("bias"), py::arg("N"), py::arg("H"), py::arg("W"), py::arg("C"),
     py::arg("K"), py::arg("R"), py::arg("S"), py::arg("Ho"), py::arg("Wo"), py::arg("sh"), py::arg("sw"),
     py::arg("ph"), py::arg("pw"), py::arg("dh"), py::arg("dw"), py::arg("relu"), py::arg("out_mode"),
     py::arg("stream"), py::arg("stats") = 0);
  m.def("bn_fwd_from_ws", [](P ws, int nb, P gamma, P beta, P rm, P rv, P mean, P invstd, P scale, P shift, int64_t R,
                             int C, float mom, float eps, P s) {
    sg_bn_fwd_from_ws(CV(ws), nb, CV(gamma), CV(beta), V(rm), V(rv), V(mean), V(invstd), V(scale), V(shift), R, C, mom,
                      eps, S(s));
    CHK("bn_fwd_from_ws");
  });
  m.def("conv_dgrad", [](P dy, P wt, P dx, int N, int H, int W, int C, int K, int R, int Sd, int Ho, int Wo, int sh,
                         int sw, int ph, int pw, int dh, int dw, int out_mode, P s) {
    sg_conv_dgrad(CV(dy), CV(wt), V(dx), N, H, W, C, K, R, Sd, Ho, Wo, sh, sw, ph, pw, dh, dw, out_mode, 0.f, nullptr,
                  S(s));
    CHK("conv_dgrad");
  });
  // dx = dgrad + beta * dx (accumulate into an existing gradient, bf16 out)
  // dx = dgrad + beta * dx; wtbuf (0 or K*R*S*C bf16 scratch): K-major transposed-weight path
  m.def("conv_dgrad_acc", [](P dy, P wt, P dx, int N, int H, int W, int C, int K, int R, int Sd, int Ho, int Wo,
                             int sh, int sw, int ph, int pw, int dh, int dw, int out_mode, float beta, P s, P wtbuf) {
    sg_conv_dgrad(CV(dy), CV(wt), V(dx), N, H, W, C, K, R, Sd, Ho, Wo, sh, sw, ph, pw, dh, dw, out_mode, beta,
                  V(wtbuf), S(s));
    CHK("conv_dgrad_acc");
  });
  // dx = dgrad + res_g * bit(res_mask) (bf16; returns 0 when the shape needs the caller to materialise)
  m.def("conv_dgrad_res", [](P dy, P wt, P dx, int N, int H, int W, int C, int K, int R, int Sd, int Ho, int Wo,
                             int sh, int sw, int ph, int pw, int dh, int dw, P wtbuf, P res_g, P res_mask, P s) {
    const int r = sg_conv_dgrad_res(CV(dy), CV(wt), V(dx), N, H, W, C, K, R, Sd, Ho, Wo, sh, sw, ph, pw, dh, dw,
                                    V(wtbuf), CV(res_g), CV(res_mask), S(s));
    CHK("conv_dgrad_res");
    return r;
  });
  m.def("conv_wgrad", [](P x, P dy, P dw_out, int N, int H, int W, int C, int K, int R, int Sd, int Ho, int Wo,
                         int sh, int sw, int ph, int pw, int dh, int dw, int splits, P s) {
    sg_conv_wgrad(CV(x), CV(dy), V(dw_out), N, H, W, C, K, R, Sd, Ho, Wo, sh, sw, ph, pw, dh, dw, splits, S(s));
    CHK("conv_wgrad");
  });
  // dgrad whose epilogue also sums the producer BN(+ReLU)'s backward partials into bn_ws [32][2][C]
  m.def("conv_dgrad_bn", [](P dy, P wt, P dx, int N, int H, int W, int C, int K, int R, int Sd, int Ho, int Wo,
                            int sh, int sw, int ph, int pw, int dh, int dw, P wtbuf, P bn_ws, P bn_x, P mean,
                            P invstd, P scale, P shift, P s, float beta, P bn_mask) {
    sg_conv_dgrad_bn_ex(CV(dy), CV(wt), V(dx), N, H, W, C, K, R, Sd, Ho, Wo, sh, sw, ph, pw, dh, dw, 0, beta,
                        V(wtbuf), V(bn_ws), CV(bn_x), CV(mean), CV(invstd), CV(scale), CV(shift), CV(bn_mask), S(s));
    CHK("conv_dgrad_bn");
  }, py::arg("dy"), py::arg("wt"), py::arg("dx"), py::arg("N"), py::arg("H"), py::arg("W"), py::arg("C"),
     py::arg("K"), py::arg("R"), py::arg("S"), py::arg("Ho"), py::arg("Wo"), py::arg("sh"), py::arg("sw"),
     py::arg("ph"), py::arg("pw"), py::arg("dh"), py::arg("dw"), py::arg("wtbuf"), py::arg("bn_ws"), py::arg("bn_x"),
     py::arg("mean"), py::arg("invstd"), py::arg("scale"), py::arg("shift"), py::arg("s"), py::arg("beta") = 0.f,
     py::arg("bn_mask") = 0);
  m.def("bn_bwd_from_ws", [](P x, P dy, P y, P scale, P shift, P mean, P invstd, P gamma, P ws, int nb, P coef, P dg,
                             P db, P dx, P dres, int64_t R, int C, int mask_mode, int dt, P s) {
    sg_bn_bwd_from_ws(CV(x), CV(dy), CV(y), CV(scale), CV(shift), CV(mean), CV(invstd), CV(gamma), CV(ws), nb, V(coef),
                      V(dg), V(db), V(dx), V(dres), R, C, mask_mode, dt, S(s));
    CHK("bn_bwd_from_ws");
  });
  // wdot[c] += sign * sum_rows W[row][c] * dW[row][c] (KRSC filter as [rows][C])
  m.def("wdot_colsum", [](P w, P dw, int rows, int C, float sign, P wdot, int zero_first, P gamma, P beta,
                          float tau, P s) {
    sg_wdot_colsum(CV(w), CV(dw), rows, C, sign, V(wdot), zero_first, CV(gamma), CV(beta), tau, S(s));
    CHK("wdot_colsum");
  });
  // BN(+ReLU) backward from the consuming conv's masked-gradient sums and <W, dW> (bf16, mask bits)
  m.def("bn_bwd_wdot", [](P x, P dy, P mask, P scale, P shift, P mean, P invstd, P gamma, P beta, P ws1, P wdot,
                          P ws2, P flag, P coef, P dg, P db, P dx, int64_t R, int C, float tau, P s) {
    sg_bn_bwd_wdot(CV(x), CV(dy), CV(mask), CV(scale), CV(shift), CV(mean), CV(invstd), CV(gamma), CV(beta), CV(ws1),
                   CV(wdot), V(ws2), V(flag), V(coef), V(dg), V(db), V(dx), R, C, tau, S(s));
    CHK("bn_bwd_wdot");
  });
  m.def("set_ws_prezeroed", [](int on) { sg_set_ws_prezeroed(on); });
  m.def("zero", [](P p, int64_t bytes, P s) { sg_zero(V(p), bytes, S(s)); CHK("zero"); });
  // generic MFMA GEMM / conv (csrc/kernels/ggemm.hip): dt 0 = fp32 operands (exact f32 MFMA), 1 = bf16
  m.def("ggemm", [](int dt, P a, int64_t lda, int ako, int64_t sa, P b, int64_t ldb, int bko, int64_t sb, P c,
                    int64_t ldc, int64_t sc, int M, int N, int K, float alpha, float beta, P bias, int relu,
                    int out_mode, int splits, int batch, P csum, int act_bwd, P act_x, P aux, P s) {
    sg_ggemm(dt, CV(a), lda, ako, sa, CV(b), ldb, bko, sb, V(c), ldc, sc, M, N, K, alpha, beta, CV(bias), relu,
             out_mode, splits, batch, (float*)V(csum), act_bwd, CV(act_x), V(aux), S(s));
    CHK("ggemm");
  });
  m.def("ggemm_tune", [](int key, int value) { sg_ggemm_tune(key, value); });
  m.def("ggemm_last_dma", []() { return sg_ggemm_last_dma(); });
  m.def("bnres_tune", [](int key, int v) { sg_bnres_tune(key, v); });
  // persistent 3x3 64-channel stage-1 conv (csrc/kernels/conv3x3.hip): A/B switch
  m.def("conv3x3_set", [](int on) { sg_conv3x3_set(on); });
  m.def("conv3x3_enabled", []() { return sg_conv3x3_enabled(); });
  // algebraic residual-BN backward (csrc/kernels/bnres.hip)
  m.def("bnres_wgrad", [](P g, P y, P out, int Pn, int K4, int C, P s) {
    sg_bnres_wgrad(CV(g), CV(y), V(out), Pn, K4, C, S(s));
    CHK("bnres_wgrad");
  });
  m.def("bnres_dgrad", [](P g, P y, P bd, P bias, P dx, int Pn, int K4, int C, P stats, P mask, P s) {
    sg_bnres_dgrad(CV(g), CV(y), CV(bd), CV(bias), V(dx), Pn, K4, C, V(stats), CV(mask), S(s));
    CHK("bnres_dgrad");
  });
  m.def("bnres_coef", [](P G, P w, P gws, P mean, P invstd, P gamma, int Pn, int K4, int C, P coef, P wf, P wu,
                         P dg, P db, P s) {
    sg_bnres_coef(CV(G), CV(w), CV(gws), CV(mean), CV(invstd), CV(gamma), Pn, K4, C, V(coef), V(wf), V(wu), V(dg),
                  V(db), S(s));
    CHK("bnres_coef");
  });
  m.def("bnres_combine", [](P G, P T, P M, P cs, int cs_rows, P coef, P w, int K4, int C, P dw, P bd, P bias,
                            P wdot, P gamma2, P beta2, float tau, P s) {
    sg_bnres_combine(CV(G), CV(T), CV(M), CV(cs), cs_rows, CV(coef), CV(w), K4, C, V(dw), V(bd), V(bias), V(wdot),
                     CV(gamma2), CV(beta2), tau, S(s));
    CHK("bnres_combine");
  });
  m.def("bnres_masksum", [](P dy, P mask, P g, P ws, int64_t R, int C, P s) {
    sg_bnres_masksum(CV(dy), CV(mask), V(g), V(ws), R, C, S(s));
    CHK("bnres_masksum");
  });
  // dgrad completing a fused residual tail's output gradient: (dgrad + acc) * bit, summed (stats_mode 4)
  m.def("conv_dgrad_gsum", [](P dy, P w, P dx, int N, int H, int W, int C, int K, int R, int Sd, int Ho, int Wo,
                              int sh, int sw, int ph, int pw, int dh, int dw, P wt, P acc, P bn_ws, P mask, int acc_s,
                              int acc_Ho, int acc_Wo, P s) {
    sg_conv_dgrad_gsum(CV(dy), CV(w), V(dx), N, H, W, C, K, R, Sd, Ho, Wo, sh, sw, ph, pw, dh, dw, V(wt), CV(acc),
                       V(bn_ws), CV(mask), acc_s, acc_Ho, acc_Wo, S(s));
    CHK("conv_dgrad_gsum");
  });
  // fused residual tail forward with the 1x1-conv output recomputed (pass 0: BN sums; pass 1: apply + mask)
  m.def("strided_pick", [](P x, P y, int N, int H, int W, int C, int Ho, int Wo, int st, int place, P s) {
    sg_strided_pick(CV(x), V(y), N, H, W, C, Ho, Wo, st, place, S(s));
    CHK("strided_pick");
  });
  m.def("sk_tail_ok", [](int M, int N, int K) { return sg_sk_tail_ok(M, N, K); });
  m.def("bnres_gram_stats", [](P w, P gram, P cs, int cs_rows, int K4, int C, P ws, P s) {
    sg_bnres_gram_stats(CV(w), CV(gram), CV(cs), cs_rows, K4, C, V(ws), S(s));
    CHK("bnres_gram_stats");
  });
  m.def("sk_tail2", [](P y, P x, P wf, P shift, P ones, P out, P mask, int M, int N, int K1, int K2, P s) {
    const int r = sg_sk_tail2(CV(y), CV(x), CV(wf), CV(shift), CV(ones), V(out), V(mask), M, N, K1, K2, S(s));
    CHK("sk_tail2");
    return r;
  });
  m.def("bnres_fold", [](P w3, P wd, P s3, P f3, P sd, P fd, int N, int K1, int K2, P wf, P shift, P ones, P s) {
    sg_bnres_fold(CV(w3), CV(wd), CV(s3), CV(f3), CV(sd), CV(fd), N, K1, K2, V(wf), V(shift), V(ones), S(s));
    CHK("bnres_fold");
  });
  m.def("sk_tail", [](P a, P w, P out, P stats, P scale, P shift, P res, P mask, int M, int N, int K, int pass, P s) {
    const int r = sg_sk_tail(CV(a), CV(w), V(out), V(stats), CV(scale), CV(shift), CV(res), V(mask), M, N, K, pass,
                             S(s));
    CHK("sk_tail");
    return r;
  });
  m.def("bn_apply_cs", [](P x, P scale, P shift, P y, P mask, P colsum, int64_t R, int C, int relu, P s) {
    sg_bn_apply_cs(CV(x), CV(scale), CV(shift), V(y), V(mask), V(colsum), R, C, relu, S(s));
    CHK("bn_apply_cs");
  });
  // one-shot: the next mask-only BN-producer dgrad writes its output masked (stats_mode 4)
  m.def("set_dgrad_mask_out", [](int on) { sg_set_dgrad_mask_out(on); });
  // persistent kernels' dynamic work queues (csrc/kernels/workq.hip): A/B switch
  m.def("workq_set", [](int on) { sg_workq_set(on); });
  m.def("workq_enabled", []() { return sg_workq_enabled(); });
  // per-capture slot arenas (a captured graph never shares a slot with other work)
  m.def("workq_arena_begin", []() { return (P)sg_workq_arena_begin(); });
  m.def("workq_arena_end", []() { sg_workq_arena_end(); });
  m.def("workq_arena_free", [](P h) { sg_workq_arena_free(V(h)); });
  m.def("workq_arena_slots", [](P h) { return sg_workq_arena_slots(V(h)); });
  m.def("cu_count", []() { return sg_cu_count(); });
  // interference rehearsal: occupy ncu CUs for `us` microseconds on stream s
  m.def("cu_hog", [](int ncu, double us, int lds_bytes, P started, P s) {
    sg_cu_hog(ncu, us, lds_bytes, (int*)V(started), S(s));
    CHK("cu_hog");
  });
  // ImageNet stem forward (csrc/kernels/stem.hip): 1 if taken, 0 = use conv_fwd
  m.def("stem_fwd", [](P x, P w, P y, P stats, int N, int H, int W, int Ho, int Wo, P s) {
    const int r = sg_stem_fwd(CV(x), CV(w), V(y), V(stats), N, H, W, Ho, Wo, S(s));
    CHK("stem_fwd");
    return r;
  });
  m.def("gemm_act", [](P a, int64_t lda, int ako, P b, int64_t ldb, int bko, P c, int64_t ldc, int M, int N, int K,
                       float alpha, P bias, int batch, int64_t sa, int64_t sb, int64_t sc, int act, P aux, int act_bwd,
                       P act_x, P colsum, P s) {
    const int r = sg_gemm_act(CV(a), lda, ako, CV(b), ldb, bko, V(c), ldc, M, N, K, alpha, CV(bias), batch, sa, sb, sc,
                              act, V(aux), act_bwd, CV(act_x), (float*)V(colsum), S(s));
    CHK("gemm_act");
    return r;
  });
  m.def("gconv_fwd", [](int dt, P x, P w, P y, P bias, int N, int H, int W, int C, int K, int R, int Sd, int Ho,
                        int Wo, int sh, int sw, int ph, int pw, int dh, int dw, int groups, int relu, int out_mode,
                        P s) {
    sg_gconv_fwd(dt, CV(x), CV(w), V(y), CV(bias), N, H, W, C, K, R, Sd, Ho, Wo, sh, sw, ph, pw, dh, dw, groups, relu,
                 out_mode, S(s));
    CHK("gconv_fwd");
  });
  m.def("gconv_dgrad", [](int dt, P dy, P w, P dx, int N, int H, int W, int C, int K, int R, int Sd, int Ho, int Wo,
                          int sh, int sw, int ph, int pw, int dh, int dw, int groups, int out_mode, float beta, P s) {
    sg_gconv_dgrad(dt, CV(dy), CV(w), V(dx), N, H, W, C, K, R, Sd, Ho, Wo, sh, sw, ph, pw, dh, dw, groups, out_mode,
                   beta, S(s));
    CHK("gconv_dgrad");
  });
  m.def("gconv_wgrad", [](int dt, P x, P dy, P dw_out, int N, int H, int W, int C, int K, int R, int Sd, int Ho,
                          int Wo, int sh, int sw, int ph, int pw, int dh, int dw, int groups, int splits, P s) {
    sg_gconv_wgrad(dt, CV(x), CV(dy), V(dw_out), N, H, W, C, K, R, Sd, Ho, Wo, sh, sw, ph, pw, dh, dw, groups, splits,
                   S(s));
    CHK("gconv_wgrad");
  });
  // glue kernels (csrc/kernels/glue.hip); shapes / strides as int64 lists, already coalesced
  typedef std::vector<int64_t> VI;
  m.def("copy_nd", [](P src, int dti, P dst, int dto, const VI& size, const VI& dst_st, const VI& src_st, P s) {
    sg_copy_nd(CV(src), dti, V(dst), dto, (int)size.size(), size.data(), dst_st.data(), src_st.data(), S(s));
    CHK("copy_nd");
  });
  m.def("binary_nd", [](int op, P a, P b, P out, int dt, const VI& size, const VI& os, const VI& as, const VI& bs,
                        float alpha, P s) {
    sg_binary_nd(op, CV(a), CV(b), V(out), dt, (int)size.size(), size.data(), os.data(), as.data(), bs.data(), alpha,
                 S(s));
    CHK("binary_nd");
  });
  m.def("where_nd", [](P c, P a, P b, P out, int dt, const VI& size, const VI& os, const VI& as, const VI& bs,
                       const VI& cs, P s) {
    sg_where_nd(CV(c), CV(a), CV(b), V(out), dt, (int)size.size(), size.data(), os.data(), as.data(), bs.data(),
                cs.data(), S(s));
    CHK("where_nd");
  });
  m.def("reduce", [](P x, int dti, P y, int dto, int64_t outer, int64_t red, int64_t inner, int op, P s) {
    sg_reduce(CV(x), dti, V(y), dto, outer, red, inner, op, S(s)); CHK("reduce");
  });
  m.def("index_select", [](P src, P idx, int idx64, P dst, int64_t outer, int64_t nsrc, int64_t inner, int64_t nidx,
                           int esize, P s) {
    sg_index_select(CV(src), CV(idx), idx64, V(dst), outer, nsrc, inner, nidx, esize, S(s)); CHK("index_select");
  });
  m.def("index_add", [](P dst, P idx, int idx64, P src, int dts, int64_t outer, int64_t ndst, int64_t inner,
                        int64_t nidx, float alpha, P s) {
    sg_index_add(V(dst), CV(idx), idx64, CV(src), dts, outer, ndst, inner, nidx, alpha, S(s)); CHK("index_add");
  });
  m.def("gather_el", [](P src, P idx, int idx64, P out, int dt, int64_t outer, int64_t nsrc, int64_t nidx,
                        int64_t inner, P s) {
    sg_gather_el(CV(src), CV(idx), idx64, V(out), dt, outer, nsrc, nidx, inner, S(s)); CHK("gather_el");
  });
  m.def("scatter_el", [](P dst, P idx, int idx64, P upd, int dt, int64_t outer, int64_t ndst, int64_t nidx,
                         int64_t inner, int add, P s) {
    sg_scatter_el(V(dst), CV(idx), idx64, CV(upd), dt, outer, ndst, nidx, inner, add, S(s)); CHK("scatter_el");
  });
  m.def("pad_nd", [](P x, P y, int dt, const VI& osz, const VI& isz, const VI& ist, const VI& before, int mode,
                     float value, P s) {
    sg_pad_nd(CV(x), V(y), dt, (int)osz.size(), osz.data(), isz.data(), ist.data(), before.data(), mode, value, S(s));
    CHK("pad_nd");
  });
  m.def("pad_bwd", [](P dy, P dx, int dt, const VI& osz, const VI& isz, const VI& ist, const VI& before, int mode,
                      P s) {
    sg_pad_bwd(CV(dy), V(dx), dt, (int)osz.size(), osz.data(), isz.data(), ist.data(), before.data(), mode, S(s));
    CHK("pad_bwd");
  });
  m.def("fill", [](P p, int64_t n, int dt, double v, P s) { sg_fill(V(p), n, dt, v, S(s)); CHK("fill"); });
  m.def("iadd_i64", [](P p, int64_t n, int64_t v, P s) { sg_iadd_i64(V(p), n, v, S(s)); CHK("iadd_i64"); });
  m.def("kth_largest_abs", [](P x, int64_t n, int64_t k, P out, P ws, P s) {
    sg_kth_largest_abs(CV(x), n, k, V(out), V(ws), S(s)); CHK("kth_largest_abs");
  });
  m.def("clamp_affine", [](P x, P dy, P out, int64_t n, int dt, float a, float b, float lo, float hi, P s) {
    sg_clamp_affine(CV(x), CV(dy), V(out), n, dt, a, b, lo, hi, S(s)); CHK("clamp_affine");
  });
  m.def("set_tuning", [](int key, int value) { sg_set_tuning(key, value); });
  m.def("get_tuning", [](int key) { return sg_get_tuning(key); });
  m.def("bn_set_unroll", [](int ur) { sg_bn_set_unroll(ur); });
  m.def("bn_set_rows_per_thread", [](int rpt) { sg_bn_set_rows_per_thread(rpt); });
}
