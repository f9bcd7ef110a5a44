// pybind11 bindings of the host runtime (_core).
#include <pybind11/numpy.h>
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include "cpu_ops.h"
#include "runtime.h"

namespace py = pybind11;
using namespace sgrt;

PYBIND11_MODULE(_core, m) {
  m.doc() = "singa_amd host runtime: Shard, Record codec, Prefetcher, Graph, updaters, parameter server";

  py::class_<Shard>(m, "Shard")
      .def(py::init<const std::string&, int, int64_t>(), py::arg("folder"), py::arg("mode"),
           py::arg("capacity") = 104857600)
      .def("next",
           [](Shard& s) -> py::object {
             std::string k, v;
             if (!s.Next(&k, &v)) return py::none();
             return py::make_tuple(py::bytes(k), py::bytes(v));
           })
      .def("insert", [](Shard& s, py::bytes k, py::bytes v) { return s.Insert(std::string(k), std::string(v)); })
      .def("flush", &Shard::Flush)
      .def("seek_to_first", &Shard::SeekToFirst)
      .def("count", &Shard::Count)
      .def_property_readonly("path", &Shard::path);
  m.attr("kRead") = (int)Shard::kRead;
  m.attr("kCreate") = (int)Shard::kCreate;
  m.attr("kAppend") = (int)Shard::kAppend;

  m.def("encode_record", [](std::vector<int32_t> shape, int32_t label, py::bytes pixel, std::vector<float> data) {
    ImageRecord r;
    r.shape = std::move(shape);
    r.label = label;
    r.pixel = std::string(pixel);
    r.data = std::move(data);
    return py::bytes(EncodeRecord(r));
  }, py::arg("shape"), py::arg("label"), py::arg("pixel") = py::bytes(""), py::arg("data") = std::vector<float>());
  m.def("decode_record", [](py::bytes b) -> py::object {
    ImageRecord r;
    if (!DecodeRecord(std::string(b), &r)) return py::none();
    py::dict d;
    d["shape"] = r.shape;
    d["label"] = r.label;
    d["pixel"] = py::bytes(r.pixel);
    d["data"] = r.data;
    return d;
  });

  py::class_<Prefetcher>(m, "Prefetcher")
      .def(py::init<const std::string&, int, int64_t, float, float, bool>(), py::arg("folder"), py::arg("batch"),
           py::arg("dim"), py::arg("scale") = 1.f, py::arg("bias") = 0.f, py::arg("loop") = true)
      .def("next", [](Prefetcher& p, py::array_t<float, py::array::c_style> img,
                      py::array_t<int32_t, py::array::c_style> lab) {
        int n;
        {
          py::gil_scoped_release rel;
          n = p.Next(img.mutable_data(), lab.mutable_data());
        }
        return n;
      });

  m.def("load_mnist", &LoadMnist, py::arg("imagefile"), py::arg("labelfile"), py::arg("folder"),
        py::arg("limit") = 0, py::call_guard<py::gil_scoped_release>());
  m.def("split_shard", &SplitShard, py::arg("num"), py::arg("input"), py::arg("prefix"),
        py::call_guard<py::gil_scoped_release>());
  m.def("split_shard_n", &SplitShardN, py::arg("n"), py::arg("input"), py::arg("prefix"),
        py::call_guard<py::gil_scoped_release>());
  py::class_<Graph>(m, "Graph")
      .def(py::init<>())
      .def("add_node", &Graph::AddNode)
      .def("add_edge", &Graph::AddEdge)
      .def("sort", &Graph::Sort)
      .def("to_json", &Graph::ToJson, py::arg("color") = std::vector<int>())
      .def_readonly("names", &Graph::names);

  // ---- native updaters (C13) -------------------------------------------
  using F32 = py::array_t<float, py::array::c_style>;
  auto fptr = [](py::object o) -> float* {
    if (o.is_none()) return nullptr;
    auto a = o.cast<F32>();
    return a.mutable_data();
  };
  m.def("updater_kind", &UpdaterKind);
  m.def("learning_rate", &LearningRate, py::arg("method"), py::arg("base"), py::arg("final"), py::arg("freq"),
        py::arg("gamma"), py::arg("pow"), py::arg("step"));
  m.def("opt_update",
        [fptr](int kind, F32 w, F32 g, py::object s1, py::object s2, float lr, float wd, float grad_scale, float t,
               float momentum, float dampening, float beta1, float beta2, float eps, float rho, bool nesterov,
               bool adamw, py::object lr_vec, py::object wd_vec, py::object mask) {
          UpdateArgs a;
          a.kind = kind; a.lr = lr; a.wd = wd; a.grad_scale = grad_scale; a.t = t; a.momentum = momentum;
          a.dampening = dampening; a.beta1 = beta1; a.beta2 = beta2; a.eps = eps; a.rho = rho;
          a.nesterov = nesterov; a.adamw = adamw;
          const int64_t n = w.size();
          if (g.size() != n) throw std::invalid_argument("opt_update: w/g size mismatch");
          float *p1 = fptr(s1), *p2 = fptr(s2), *lv = fptr(lr_vec), *wv = fptr(wd_vec);
          const uint8_t* mk = nullptr;
          py::array_t<uint8_t, py::array::c_style> mka;
          if (!mask.is_none()) {
            mka = mask.cast<py::array_t<uint8_t, py::array::c_style>>();
            mk = mka.data();
          }
          float* pw = w.mutable_data();
          const float* pg = g.data();
          py::gil_scoped_release rel;
          OptUpdate(a, pw, pg, p1, p2, n, lv, wv, mk);
        },
        py::arg("kind"), py::arg("w"), py::arg("g"), py::arg("s1"), py::arg("s2"), py::arg("lr"), py::arg("wd"),
        py::arg("grad_scale"), py::arg("t"), py::arg("momentum") = 0.f, py::arg("dampening") = 0.f,
        py::arg("beta1") = 0.9f, py::arg("beta2") = 0.999f, py::arg("eps") = 1e-8f, py::arg("rho") = 0.9f,
        py::arg("nesterov") = false, py::arg("adamw") = false, py::arg("lr_vec") = py::none(),
        py::arg("wd_vec") = py::none(), py::arg("mask") = py::none());

  // ---- native parameter server (C25 / C26 / C12 / C15) --------------------
  py::class_<PServer>(m, "PServer")
      .def(py::init<int, int>(), py::arg("port") = 0, py::arg("nworkers") = 1)
      .def_property_readonly("port", &PServer::port)
      .def_property_readonly("messages", &PServer::messages)
      .def("set_updater",
           [](PServer& s, int kind, float momentum, float wd, float eps, float rho, float beta1, float beta2,
              const std::string& method, double base, double final_lr, int freq, double gamma, double pw) {
             UpdateArgs a;
             a.kind = kind; a.momentum = momentum; a.wd = wd; a.eps = eps; a.rho = rho; a.beta1 = beta1;
             a.beta2 = beta2;
             s.SetUpdater(a, method, base, final_lr, freq, gamma, pw);
           },
           py::arg("kind"), py::arg("momentum") = 0.f, py::arg("weight_decay") = 0.f, py::arg("eps") = 1e-8f,
           py::arg("rho") = 0.9f, py::arg("beta1") = 0.9f, py::arg("beta2") = 0.999f, py::arg("method") = "kFixed",
           py::arg("base") = 0.01, py::arg("final") = 0.0, py::arg("freq") = 1, py::arg("gamma") = 1.0,
           py::arg("pow") = 0.0)
      .def("wait_stop", &PServer::WaitStop, py::arg("timeout_s") = -1.0, py::call_guard<py::gil_scoped_release>())
      .def("value", [](PServer& s, int id) {
        auto v = s.Value(id);
        F32 a((py::ssize_t)v.size());
        std::copy(v.begin(), v.end(), a.mutable_data());
        return a;
      })
      .def("close", &PServer::Close, py::call_guard<py::gil_scoped_release>());

  py::class_<PSClient>(m, "PSClient")
      .def(py::init<const std::vector<std::string>&, int, double>(), py::arg("endpoints"), py::arg("retries") = 10,
           py::arg("retry_s") = 1.0, py::call_guard<py::gil_scoped_release>())
      .def_property_readonly("nservers", &PSClient::nservers)
      .def("server_of", &PSClient::server_of)
      .def("put", [](PSClient& c, int id, F32 w) {
        const float* p = w.data();
        const uint64_t n = w.size();
        py::gil_scoped_release rel;
        c.Put(id, p, n);
      })
      .def("get", [](PSClient& c, int id, F32 out) {
        float* p = out.mutable_data();
        const uint64_t n = out.size();
        py::gil_scoped_release rel;
        return c.Get(id, p, n);
      })
      .def("update", [](PSClient& c, int id, F32 grad, F32 w_out, int step, float gs) {
        const float* g = grad.data();
        float* w = w_out.mutable_data();
        const uint64_t n = grad.size();
        if ((uint64_t)w_out.size() != n) throw std::invalid_argument("update: size mismatch");
        py::gil_scoped_release rel;
        c.Update(id, g, w, n, step, gs);
      }, py::arg("id"), py::arg("grad"), py::arg("w_out"), py::arg("step") = -1, py::arg("grad_scale") = 0.f)
      .def("elastic", [](PSClient& c, int id, F32 w, float alpha) {
        float* p = w.mutable_data();
        const uint64_t n = w.size();
        py::gil_scoped_release rel;
        c.Elastic(id, p, n, alpha);
      })
      .def("random_sync", [](PSClient& c, int id, F32 delta, F32 old_out, int64_t a, int64_t b) {
        const float* d = delta.data();
        float* o = old_out.mutable_data();
        const uint64_t m = delta.size();
        if ((uint64_t)old_out.size() != m) throw std::invalid_argument("random_sync: size mismatch");
        py::gil_scoped_release rel;
        c.RandomSync(id, d, o, m, a, b);
      })
      .def("push_replace", [](PSClient& c, int id, F32 w) {
        const float* p = w.data();
        const uint64_t n = w.size();
        py::gil_scoped_release rel;
        c.PushReplace(id, p, n);
      })
      .def("push_update", [](PSClient& c, int id, F32 grad, int step, float gs) {
        const float* p = grad.data();
        const uint64_t n = grad.size();
        py::gil_scoped_release rel;
        c.PushUpdate(id, p, n, step, gs);
      }, py::arg("id"), py::arg("grad"), py::arg("step") = -1, py::arg("grad_scale") = 0.f)
      .def("collect", [](PSClient& c, std::vector<int> ids, std::vector<F32> outs) {
        std::vector<float*> ps;
        std::vector<uint64_t> caps;
        for (auto& o : outs) {
          ps.push_back(o.mutable_data());
          caps.push_back(o.size());
        }
        py::gil_scoped_release rel;
        return c.Collect(ps, caps, ids);
      })
      .def("stop", &PSClient::Stop, py::call_guard<py::gil_scoped_release>());

  // ---- LMDB (kLMDBData without liblmdb / the lmdb module) -----------------
  py::class_<LmdbReader>(m, "LmdbReader")
      .def(py::init<const std::string&>())
      .def("count", &LmdbReader::Count)
      .def("seek_to_first", &LmdbReader::SeekToFirst)
      .def("next", [](LmdbReader& r) -> py::object {
        std::string k, v;
        if (!r.Next(&k, &v)) return py::none();
        return py::make_tuple(py::bytes(k), py::bytes(v));
      });
  m.def("decode_datum", [](py::bytes b) -> py::object {
    ImageRecord r;
    bool enc = false;
    if (!DecodeDatum(std::string(b), &r, &enc)) return py::none();
    py::dict d;
    d["shape"] = r.shape;
    d["label"] = r.label;
    d["pixel"] = py::bytes(r.pixel);
    d["data"] = r.data;
    d["encoded"] = enc;
    return d;
  });

  // ---- CppCPU compute backend (cpu_ops.cc): raw host pointers, GIL released --
  {
    namespace C = sgrt::cpu;
    typedef uintptr_t P;
    auto fp = [](P p) { return (float*)p; };
    auto cfp = [](P p) { return (const float*)p; };
    auto ng = py::call_guard<py::gil_scoped_release>();
    py::module_ c = m.def_submodule("cpu", "CppCPU compute kernels (host pointers)");
    c.def("num_threads", &C::NumThreads);
    c.def("gemm", [=](bool ta, bool tb, int64_t M, int64_t N, int64_t K, float alpha, P a, int64_t lda, P b,
                      int64_t ldb, float beta, P cc, int64_t ldc, P bias, bool relu) {
      C::Gemm(ta, tb, M, N, K, alpha, cfp(a), lda, cfp(b), ldb, beta, fp(cc), ldc, cfp(bias), relu);
    }, ng);
    c.def("gemm_batched", [=](bool ta, bool tb, int64_t M, int64_t N, int64_t K, float alpha, P a, int64_t lda,
                              int64_t sa, P b, int64_t ldb, int64_t sb, float beta, P cc, int64_t ldc, int64_t sc,
                              int64_t batch) {
      // batch-parallel: each GEMM of the batch runs on one worker
      C::ParallelFor(batch, 1, [&](int64_t b0, int64_t b1) {
        for (int64_t i = b0; i < b1; ++i)
          C::Gemm(ta, tb, M, N, K, alpha, cfp(a) + i * sa, lda, cfp(b) + i * sb, ldb, beta, fp(cc) + i * sc, ldc,
                  nullptr, false);
      });
    }, ng);
    c.def("unary_fwd", [=](int op, P x, P y, int64_t n, float a) { C::UnaryFwd(op, cfp(x), fp(y), n, a); }, ng);
    c.def("unary_bwd", [=](int op, P x, P y, P dy, P dx, int64_t n, float a) {
      C::UnaryBwd(op, cfp(x), cfp(y), cfp(dy), fp(dx), n, a);
    }, ng);
    c.def("copy_nd", [](P src, int dti, P dst, int dto, std::vector<int64_t> size, std::vector<int64_t> dst_st,
                        std::vector<int64_t> src_st) {
      if (size.size() > 8 || dst_st.size() != size.size() || src_st.size() != size.size())
        throw std::invalid_argument("copy_nd: bad rank");
      py::gil_scoped_release rel;
      C::CopyNd((const void*)src, dti, (void*)dst, dto, (int)size.size(), size.data(), dst_st.data(), src_st.data());
    });
    c.def("binary_nd", [=](int op, P a, P b, P out, std::vector<int64_t> size, std::vector<int64_t> os,
                           std::vector<int64_t> as, std::vector<int64_t> bs, float alpha) {
      if (size.size() > 8 || os.size() != size.size() || as.size() != size.size() || bs.size() != size.size())
        throw std::invalid_argument("binary_nd: bad rank");
      py::gil_scoped_release rel;
      C::BinaryNd(op, cfp(a), cfp(b), fp(out), (int)size.size(), size.data(), os.data(), as.data(), bs.data(), alpha);
    });
    c.def("fill", [](P p, int64_t n, int dt, double v) { C::Fill((void*)p, n, dt, v); }, ng);
    c.def("reduce", [=](P x, P y, int64_t outer, int64_t red, int64_t inner, int op) {
      C::Reduce(cfp(x), fp(y), outer, red, inner, op);
    }, ng);
    c.def("softmax", [=](P x, P y, int64_t rows, int64_t n) { C::SoftmaxRows(cfp(x), fp(y), rows, n); }, ng);
    c.def("softmax_bwd", [=](P y, P dy, P dx, int64_t rows, int64_t n) {
      C::SoftmaxRowsBwd(cfp(y), cfp(dy), fp(dx), rows, n);
    }, ng);
    c.def("softmax_xent", [=](P x, P lab, int lab64, P t, P loss, P correct, P dx, int64_t B, int64_t n, int topk,
                              float gs) {
      C::SoftmaxXent(cfp(x), (const void*)lab, lab64, cfp(t), fp(loss), fp(correct), fp(dx), B, n, topk, gs);
    }, ng);
    c.def("conv_fwd", [=](P x, P w, P bias, P y, int N, int Ci, int H, int W, int K, int R, int S, int Ho, int Wo,
                          int sh, int sw, int ph, int pw, int dh, int dw, int groups) {
      C::ConvFwd(cfp(x), cfp(w), cfp(bias), fp(y), N, Ci, H, W, K, R, S, Ho, Wo, sh, sw, ph, pw, dh, dw, groups);
    }, ng);
    c.def("conv_bwd", [=](P x, P w, P dy, P dx, P dwt, P db, int N, int Ci, int H, int W, int K, int R, int S, int Ho,
                          int Wo, int sh, int sw, int ph, int pw, int dh, int dw, int groups) {
      C::ConvBwd(cfp(x), cfp(w), cfp(dy), fp(dx), fp(dwt), fp(db), N, Ci, H, W, K, R, S, Ho, Wo, sh, sw, ph, pw, dh,
                 dw, groups);
    }, ng);
    c.def("pool_fwd", [=](P x, P y, P arg, int N, int Ci, int H, int W, int Ho, int Wo, int kh, int kw, int sh,
                          int sw, int ph, int pw, int is_max, int cip) {
      C::PoolFwd(cfp(x), fp(y), (int32_t*)arg, N, Ci, H, W, Ho, Wo, kh, kw, sh, sw, ph, pw, is_max, cip);
    }, ng);
    c.def("pool_bwd", [=](P dy, P arg, P dx, int N, int Ci, int H, int W, int Ho, int Wo, int kh, int kw, int sh,
                          int sw, int ph, int pw, int is_max, int cip) {
      C::PoolBwd(cfp(dy), (const int32_t*)arg, fp(dx), N, Ci, H, W, Ho, Wo, kh, kw, sh, sw, ph, pw, is_max, cip);
    }, ng);
    c.def("lrn_fwd", [=](P x, P y, int N, int Ci, int HW, int size, float alpha, float beta, float k) {
      C::LrnFwd(cfp(x), fp(y), N, Ci, HW, size, alpha, beta, k);
    }, ng);
    c.def("lrn_bwd", [=](P x, P dy, P dx, int N, int Ci, int HW, int size, float alpha, float beta, float k) {
      C::LrnBwd(cfp(x), cfp(dy), fp(dx), N, Ci, HW, size, alpha, beta, k);
    }, ng);
    c.def("dropout_fwd", [=](P x, P y, P mask, int64_t n, float pkeep, uint64_t seed, uint64_t offset) {
      C::DropoutFwd(cfp(x), fp(y), (uint8_t*)mask, n, pkeep, seed, offset);
    }, ng);
    c.def("dropout_bwd", [=](P dy, P mask, P dx, int64_t n, float pkeep) {
      C::DropoutBwd(cfp(dy), (const uint8_t*)mask, fp(dx), n, pkeep);
    }, ng);
    c.def("rand_fill", [=](P y, int64_t n, int dist, float a, float b, uint64_t seed, uint64_t offset) {
      C::RandFill(fp(y), n, dist, a, b, seed, offset);
    }, ng);
    c.def("bn_fwd", [=](P x, P g, P b, P rm, P rv, P y, P mean, P invstd, int N, int Ci, int64_t HW, int training,
                        float momentum, float eps, int relu, P res) {
      C::BatchNormFwd(cfp(x), cfp(g), cfp(b), fp(rm), fp(rv), fp(y), fp(mean), fp(invstd), N, Ci, HW, training,
                      momentum, eps, relu, cfp(res));
    }, ng);
    c.def("bn_bwd", [=](P x, P dy, P g, P mean, P invstd, P ym, int relu_x, P scale, P shift, P dx, P dg, P db,
                        P dres, int N, int Ci, int64_t HW) {
      C::BatchNormBwd(cfp(x), cfp(dy), cfp(g), cfp(mean), cfp(invstd), cfp(ym), relu_x, cfp(scale), cfp(shift), fp(dx),
                      fp(dg), fp(db), fp(dres), N, Ci, HW);
    }, ng);
    c.def("where_nd", [=](P cond, P a, P b, P out, std::vector<int64_t> size, std::vector<int64_t> os,
                          std::vector<int64_t> as, std::vector<int64_t> bs, std::vector<int64_t> cs) {
      if (size.size() > 8 || os.size() != size.size() || as.size() != size.size() || bs.size() != size.size() ||
          cs.size() != size.size())
        throw std::invalid_argument("where_nd: bad rank");
      py::gil_scoped_release rel;
      C::WhereNd((const uint8_t*)cond, cfp(a), cfp(b), fp(out), (int)size.size(), size.data(), os.data(), as.data(),
                 bs.data(), cs.data());
    });
    c.def("clamp_affine", [=](P x, P dy, P y, int64_t n, float a, float b, float lo, float hi) {
      C::ClampAffine(cfp(x), cfp(dy), fp(y), n, a, b, lo, hi);
    }, ng);
    c.def("affine_elastic_sample", [=](P img, P theta, P disp, P out, int B, int H, int W) {
      C::AffineElasticSample(cfp(img), cfp(theta), cfp(disp), fp(out), B, H, W);
    }, ng);
    c.def("gauss_blur2d", [=](P in, P out, int N, int H, int W, P g, int k) {
      C::GaussBlur2D(cfp(in), fp(out), N, H, W, cfp(g), k);
    }, ng);
    c.def("resize_bilinear", [=](P in, P out, int B, int H, int W, int h, int w) {
      C::ResizeBilinear(cfp(in), fp(out), B, H, W, h, w);
    }, ng);
    c.def("easgd_diff", [=](P w, P c_, P d, int64_t n, float alpha) { C::EasgdDiff(fp(w), cfp(c_), fp(d), n, alpha); },
          ng);
    c.def("rsync_gather", [=](P w, P snap, P buf, int64_t m, int64_t n, int64_t a, int64_t b) {
      C::RsyncGather(cfp(w), cfp(snap), fp(buf), m, n, a, b);
    }, ng);
    c.def("rsync_scatter", [=](P w, P snap, P buf, int64_t m, int64_t n, int64_t a, int64_t b) {
      C::RsyncScatter(fp(w), fp(snap), cfp(buf), m, n, a, b);
    }, ng);
    c.def("layernorm_fwd", [=](P x, P g, P b, P y, P mean, P rstd, int64_t R, int64_t D, float eps) {
      C::LayerNormFwd(cfp(x), cfp(g), cfp(b), fp(y), fp(mean), fp(rstd), R, D, eps);
    }, ng);
    c.def("layernorm_bwd", [=](P x, P dy, P g, P mean, P rstd, P dx, P dg, P db, int64_t R, int64_t D) {
      C::LayerNormBwd(cfp(x), cfp(dy), cfp(g), cfp(mean), cfp(rstd), fp(dx), fp(dg), fp(db), R, D);
    }, ng);
    c.def("index_select", [](P src, P idx, int idx64, P dst, int64_t outer, int64_t nsrc, int64_t inner,
                             int64_t nidx, int esize) {
      C::IndexSelect((const void*)src, (const void*)idx, idx64, (void*)dst, outer, nsrc, inner, nidx, esize);
    }, ng);
    c.def("index_add", [=](P dst, P idx, int idx64, P src, int64_t outer, int64_t ndst, int64_t inner, int64_t nidx,
                           float alpha) {
      C::IndexAdd(fp(dst), (const void*)idx, idx64, cfp(src), outer, ndst, inner, nidx, alpha);
    }, ng);
  }
}
