// pybind11 bindings of the native runtime (config language, graph config,
// checkpoint PODs, data IO, metrics). No torch / HIP dependency, so this module
// builds and runs identically on the CPU container and on the GPU box.
#include <pybind11/numpy.h>
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include <fstream>
#include <sstream>

#include "config_reader.h"
#include "data_io.h"
#include "jpeg_decode.h"
#include "layer_param.h"
#include "layer_types.h"
#include "metric.h"
#include "netconfig.h"

namespace py = pybind11;
using namespace cxxnet_rt;

static KVList ParseConfigFile(const std::string &path) {
  std::ifstream fi(path, std::ios::binary);
  if (!fi) throw std::runtime_error("cannot open file " + path);
  std::stringstream ss;
  ss << fi.rdbuf();
  return ConfigTokenizer(ss.str()).ParseAll();
}

// (out_h, out_w, channels, rand_crop, rand_mirror, mirror, crop_y_start, crop_x_start,
//  max_random_contrast, max_random_illumination, mean_mode)
static CropConfig ParseCropConfig(py::tuple cfg) {
  CropConfig c;
  c.out_h = cfg[0].cast<int>();
  c.out_w = cfg[1].cast<int>();
  c.channels = cfg[2].cast<int>();
  c.rand_crop = cfg[3].cast<int>();
  c.rand_mirror = cfg[4].cast<int>();
  c.mirror = cfg[5].cast<int>();
  c.crop_y_start = cfg[6].cast<int>();
  c.crop_x_start = cfg[7].cast<int>();
  c.max_random_contrast = cfg[8].cast<float>();
  c.max_random_illumination = cfg[9].cast<float>();
  c.mean_mode = cfg[10].cast<int>();
  if (c.channels < 1 || c.channels > 3) throw std::runtime_error("JpegDecodePool: 1-3 channels");
  return c;
}

static void CheckPrmCm(py::array_t<int32_t> &prm, py::array_t<float> &cm, long B) {
  if (prm.ndim() != 2 || prm.shape(0) != B || prm.shape(1) != 4 || cm.ndim() != 2 || cm.shape(0) != B ||
      cm.shape(1) != 2 || !(prm.flags() & py::array::c_style) || !(cm.flags() & py::array::c_style))
    throw std::runtime_error("JpegDecodePool: prm [B][4] int32 / cm [B][2] float32 expected");
}

// items: [(row, payload bytes-like or path str, seed)]
static std::vector<DecodeItem> ParseItems(py::list items, long B, std::vector<py::buffer_info> &keep) {
  std::vector<DecodeItem> its;
  its.reserve(items.size());
  keep.reserve(items.size());
  for (auto h : items) {
    py::tuple t = h.cast<py::tuple>();
    DecodeItem d;
    d.row = t[0].cast<int>();
    if (d.row < 0 || d.row >= B) throw std::runtime_error("JpegDecodePool: row out of range");
    d.seed = t[2].cast<uint64_t>();
    py::handle pl = t[1];
    if (py::isinstance<py::str>(pl)) {
      d.data = nullptr;
      d.size = 0;
      d.path = pl.cast<std::string>();
    } else {
      keep.push_back(py::reinterpret_borrow<py::buffer>(pl).request());
      d.data = static_cast<const unsigned char *>(keep.back().ptr);
      d.size = static_cast<size_t>(keep.back().size * keep.back().itemsize);
    }
    its.push_back(std::move(d));
  }
  return its;
}

PYBIND11_MODULE(_cxxnet_rt, m) {
  m.doc() = "cxxnet_amd native runtime: config parser, NetConfig, checkpoint PODs, IO, metrics";

  m.def("parse_config", [](const std::string &text) { return ConfigTokenizer(text).ParseAll(); },
        "Tokenize .conf text into an ordered list of (name, value) pairs");
  m.def("parse_config_file", &ParseConfigFile);
  m.def("get_layer_type", &GetLayerType);

  py::class_<LayerInfo>(m, "LayerInfo")
      .def(py::init<>())
      .def_readwrite("type", &LayerInfo::type)
      .def_readwrite("primary_layer_index", &LayerInfo::primary_layer_index)
      .def_readwrite("name", &LayerInfo::name)
      .def_readwrite("nindex_in", &LayerInfo::nindex_in)
      .def_readwrite("nindex_out", &LayerInfo::nindex_out);

  py::class_<NetConfig>(m, "NetConfig")
      .def(py::init<>())
      .def("configure", &NetConfig::Configure)
      .def("save_net", [](const NetConfig &c) { return py::bytes(c.SaveNet()); })
      .def("load_net",
           [](NetConfig &c, py::bytes b) {
             std::string s = b;
             return c.LoadNet(s.data(), s.size());
           },
           "Load structure from bytes; returns bytes consumed")
      .def("get_layer_index", &NetConfig::GetLayerIndex)
      .def_property_readonly("num_nodes", [](const NetConfig &c) { return c.param.num_nodes; })
      .def_property_readonly("num_layers", [](const NetConfig &c) { return c.param.num_layers; })
      .def_property_readonly("init_end", [](const NetConfig &c) { return c.param.init_end; })
      .def_property_readonly("extra_data_num", [](const NetConfig &c) { return c.param.extra_data_num; })
      .def_property_readonly("input_shape",
                             [](const NetConfig &c) {
                               return std::vector<uint32_t>{c.param.input_shape[0], c.param.input_shape[1],
                                                            c.param.input_shape[2]};
                             })
      .def_readonly("layers", &NetConfig::layers)
      .def_readonly("node_names", &NetConfig::node_names)
      .def_readonly("node_name_map", &NetConfig::node_name_map)
      .def_readonly("layer_name_map", &NetConfig::layer_name_map)
      .def_readonly("updater_type", &NetConfig::updater_type)
      .def_readonly("sync_type", &NetConfig::sync_type)
      .def_readonly("label_name_map", &NetConfig::label_name_map)
      .def_readonly("label_range", &NetConfig::label_range)
      .def_readonly("defcfg", &NetConfig::defcfg)
      .def_readonly("layercfg", &NetConfig::layercfg)
      .def_readonly("extra_shape", &NetConfig::extra_shape);

  py::class_<LayerParam>(m, "LayerParam")
      .def(py::init<>())
      .def("set_param", &LayerParam::SetParam)
      .def("to_bytes",
           [](const LayerParam &p) { return py::bytes(reinterpret_cast<const char *>(&p), sizeof(LayerParam)); })
      .def_static("from_bytes",
                  [](py::bytes b) {
                    std::string s = b;
                    if (s.size() < sizeof(LayerParam)) throw std::runtime_error("LayerParam: short buffer");
                    LayerParam p;
                    std::memcpy(&p, s.data(), sizeof(LayerParam));
                    return p;
                  })
      .def_property_readonly_static("nbytes", [](py::object) { return sizeof(LayerParam); })
      .def_readwrite("num_hidden", &LayerParam::num_hidden)
      .def_readwrite("init_sigma", &LayerParam::init_sigma)
      .def_readwrite("init_sparse", &LayerParam::init_sparse)
      .def_readwrite("init_uniform", &LayerParam::init_uniform)
      .def_readwrite("init_bias", &LayerParam::init_bias)
      .def_readwrite("num_channel", &LayerParam::num_channel)
      .def_readwrite("random_type", &LayerParam::random_type)
      .def_readwrite("num_group", &LayerParam::num_group)
      .def_readwrite("kernel_height", &LayerParam::kernel_height)
      .def_readwrite("kernel_width", &LayerParam::kernel_width)
      .def_readwrite("stride", &LayerParam::stride)
      .def_readwrite("pad_y", &LayerParam::pad_y)
      .def_readwrite("pad_x", &LayerParam::pad_x)
      .def_readwrite("no_bias", &LayerParam::no_bias)
      .def_readwrite("temp_col_max", &LayerParam::temp_col_max)
      .def_readwrite("silent", &LayerParam::silent)
      .def_readwrite("num_input_channel", &LayerParam::num_input_channel)
      .def_readwrite("num_input_node", &LayerParam::num_input_node);

  m.def("load_mnist", [](const std::string &img, const std::string &lab) {
    MNISTData d = LoadMNIST(img, lab);
    py::array_t<float> imgs({d.count, d.rows, d.cols});
    std::memcpy(imgs.mutable_data(), d.images.data(), d.images.size() * sizeof(float));
    py::array_t<float> labels(static_cast<py::ssize_t>(d.labels.size()));
    std::memcpy(labels.mutable_data(), d.labels.data(), d.labels.size() * sizeof(float));
    return py::make_tuple(imgs, labels);
  });

  py::class_<BinaryPage>(m, "BinaryPage")
      .def(py::init<>())
      .def("size", &BinaryPage::Size)
      .def("clear", &BinaryPage::Clear)
      .def("push",
           [](BinaryPage &p, py::bytes b) {
             std::string s = b;
             return p.Push(s.data(), s.size());
           })
      .def("get", [](const BinaryPage &p, int r) { return py::bytes(p.Get(r)); })
      .def("to_bytes", [](const BinaryPage &p) { return py::bytes(p.raw(), BinaryPage::kPageBytes); })
      .def_property_readonly_static("page_bytes", [](py::object) { return BinaryPage::kPageBytes; });
  m.def("pack_image_bin", &PackImageBin, "Pack files into 64MB BinaryPages (im2bin)");

  py::class_<ImageBinReader>(m, "ImageBinReader")
      .def(py::init<std::vector<std::string>, int>(), py::arg("paths"), py::arg("prefetch") = 2)
      .def("before_first", &ImageBinReader::BeforeFirst, py::call_guard<py::gil_scoped_release>())
      .def("next", [](ImageBinReader &r) -> py::object {
        std::string s;
        bool ok;
        if (r.Ready()) {  // no wait: keep the GIL (a release per record costs two thread handoffs)
          ok = r.Next(&s);
        } else {
          py::gil_scoped_release rel;
          ok = r.Next(&s);
        }
        if (!ok) {
          std::string err = r.Error();
          if (!err.empty()) throw std::runtime_error("ImageBinReader: " + err);
          return py::none();
        }
        return py::bytes(s);
      })
      .def("next_run",
           [](ImageBinReader &r, int n) -> py::object {
             // up to n consecutive objects of one page: (bytes blob, [(offset, length)]) -- one copy
             // for the run; None at the end of the files
             std::string blob;
             std::vector<std::pair<long, long>> spans;
             bool ok;
             if (r.Ready()) {
               ok = r.NextRun(n, &blob, &spans);
             } else {
               py::gil_scoped_release rel;
               ok = r.NextRun(n, &blob, &spans);
             }
             if (!ok) {
               std::string err = r.Error();
               if (!err.empty()) throw std::runtime_error("ImageBinReader: " + err);
               return py::none();
             }
             return py::make_tuple(py::bytes(blob), spans);
           })
      .def("next_n",
           [](ImageBinReader &r, int n) -> py::list {
             // up to n objects (fewer at the end of the files), one call per chunk of records
             py::list out;
             std::string s;
             for (int k = 0; k < n; ++k) {
               bool ok;
               if (r.Ready()) {
                 ok = r.Next(&s);
               } else {
                 py::gil_scoped_release rel;
                 ok = r.Next(&s);
               }
               if (!ok) {
                 std::string err = r.Error();
                 if (!err.empty()) throw std::runtime_error("ImageBinReader: " + err);
                 break;
               }
               out.append(py::bytes(s));
             }
             return out;
           })
      .def("next_page", [](ImageBinReader &r) -> py::object {
        std::vector<std::string> objs;
        bool ok;
        {
          py::gil_scoped_release rel;
          ok = r.NextPage(&objs);
        }
        if (!ok) {
          std::string err = r.Error();
          if (!err.empty()) throw std::runtime_error("ImageBinReader: " + err);
          return py::none();
        }
        py::list out;
        for (auto &o : objs) out.append(py::bytes(o));
        return out;
      });

  py::class_<JpegDecodePool>(m, "JpegDecodePool")
      .def(py::init<int>(), py::arg("threads"))
      .def_property_readonly("threads", &JpegDecodePool::threads)
      .def_static("available", [] { return jpg::api().ok; })
      .def_static("error", [] { return jpg::api().error; })
      .def(
          "decode",
          [](JpegDecodePool &pool, py::list items, py::tuple cfg, py::array_t<uint8_t> out, py::array_t<int32_t> prm,
             py::array_t<float> cm) {
            // items: [(row, payload bytes-like or path str, seed)]; cfg: (out_h, out_w, channels,
            // rand_crop, rand_mirror, mirror, crop_y_start, crop_x_start, max_random_contrast,
            // max_random_illumination, mean_mode)
            CropConfig c = ParseCropConfig(cfg);
            if (out.ndim() != 4 || out.shape(1) != c.out_h || out.shape(2) != c.out_w || out.shape(3) != c.channels ||
                !(out.flags() & py::array::c_style))
              throw std::runtime_error("JpegDecodePool: out must be a C-contiguous [B][h][w][C] uint8 array");
            const long B = out.shape(0);
            CheckPrmCm(prm, cm, B);
            std::vector<py::buffer_info> keep;  // buffer views stay valid while the GIL is released
            std::vector<DecodeItem> its = ParseItems(items, B, keep);
            uint8_t *o = out.mutable_data();
            int32_t *pp = prm.mutable_data();
            float *cp = cm.mutable_data();
            std::vector<int> failed;
            {
              py::gil_scoped_release rel;
              failed = pool.Run(its, c, o, pp, cp);
            }
            return failed;
          },
          "Decode + crop/mirror every (row, payload, seed) into out[row]; returns the rows it could not "
          "decode (non-JPEG or unsupported JPEG: use the Pillow path for those)")
      .def(
          "decode_coef",
          [](JpegDecodePool &pool, py::list items, py::tuple cfg, py::array_t<int16_t> coef, py::array_t<int32_t> bwin,
             py::array_t<int32_t> meta, py::array_t<int32_t> prm, py::array_t<float> cm) {
            CropConfig c = ParseCropConfig(cfg);
            const long B = meta.ndim() == 3 ? meta.shape(0) : -1;
            if (B < 0 || meta.shape(1) != 3 || meta.shape(2) != kCoefMeta || !(meta.flags() & py::array::c_style))
              throw std::runtime_error("JpegDecodePool.decode_coef: meta must be a C-contiguous [B][3][80] int32 array");
            if (coef.ndim() != 2 || coef.shape(1) != 64 || bwin.ndim() != 1 || bwin.shape(0) != coef.shape(0) ||
                !(coef.flags() & py::array::c_style) || !(bwin.flags() & py::array::c_style))
              throw std::runtime_error("JpegDecodePool.decode_coef: coef [cap][64] int16 / bwin [cap] int32 expected");
            CheckPrmCm(prm, cm, B);
            std::vector<py::buffer_info> keep;
            std::vector<DecodeItem> its = ParseItems(items, B, keep);
            CoefStage st;
            st.coef = coef.mutable_data();
            st.bwin = bwin.mutable_data();
            st.meta = meta.mutable_data();
            st.cap_blocks = coef.shape(0);
            int32_t *pp = prm.mutable_data();
            float *cp = cm.mutable_data();
            std::pair<std::vector<int>, long> r;
            {
              py::gil_scoped_release rel;
              r = pool.RunCoef(its, c, st, pp, cp);
            }
            return py::make_tuple(r.first, r.second);
          },
          "Entropy-decode every (row, payload, seed) into the GPU decode stage (coef blocks, their window "
          "ids, per-row window tables; ops.jpeg_decode finishes on the GPU); returns (rows left to "
          "decode(), blocks used)");

  py::class_<ImageListEntry>(m, "ImageListEntry")
      .def_readonly("index", &ImageListEntry::index)
      .def_readonly("labels", &ImageListEntry::labels)
      .def_readonly("path", &ImageListEntry::path);
  m.def("parse_image_list", &ParseImageList);

  py::class_<Metric>(m, "Metric")
      .def(py::init<const std::string &>())
      .def("clear", &Metric::Clear)
      .def("add_eval",
           [](Metric &mt, py::array_t<float, py::array::c_style | py::array::forcecast> pred,
              py::array_t<float, py::array::c_style | py::array::forcecast> label) {
             if (pred.ndim() != 2 || label.ndim() != 2) throw std::runtime_error("add_eval expects 2-D arrays");
             if (pred.shape(0) != label.shape(0)) throw std::runtime_error("add_eval: batch mismatch");
             mt.AddEval(pred.data(), static_cast<int>(pred.shape(0)), static_cast<int>(pred.shape(1)),
                        label.data(), static_cast<int>(label.shape(1)));
           })
      .def("get", &Metric::Get)
      .def_property_readonly("name", &Metric::name);
}
