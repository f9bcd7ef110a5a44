// pybind11 bindings of the host runtime (_core).
#include <pybind11/numpy.h>
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include "runtime.h"

namespace py = pybind11;
using namespace sgrt;

PYBIND11_MODULE(_core, m) {
  m.doc() = "singa_amd host runtime: Shard, Record codec, Prefetcher, Graph";

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
}
