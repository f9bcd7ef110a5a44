// pybind11 bindings of the host runtime (_core).
#include <pybind11/numpy.h>
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

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
}
