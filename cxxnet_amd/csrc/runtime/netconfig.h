// Network-graph configuration: parses the `netconfig=start ... netconfig=end`
// section of a .conf stream into nodes and connections, and (de)serializes the
// structure in the checkpoint layout.
//
// Behavioural parity with reference src/nnet/nnet_config.h:
//   NetParam POD (152 B)              :28-50
//   SaveNet / LoadNet                 :126-191
//   SetGlobalParam (updater, label_vec):192-203
//   Configure                         :207-289
//   GetLayerInfo (layer[a->b], +1, +0, :name, share[tag]) :303-360
#pragma once
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <map>
#include <stdexcept>
#include <string>
#include <utility>
#include <vector>

#include "config_reader.h"
#include "layer_types.h"
#include "stream.h"

namespace cxxnet_rt {

struct NetParam {
  int32_t num_nodes = 0;
  int32_t num_layers = 0;
  uint32_t input_shape[3] = {0, 0, 0};  // (c, h, w)
  int32_t init_end = 0;
  int32_t extra_data_num = 0;
  int32_t reserved[31] = {0};
};
static_assert(sizeof(NetParam) == 152, "NetParam must stay 152 bytes (checkpoint layout)");

struct LayerInfo {
  int32_t type = 0;
  int32_t primary_layer_index = -1;
  std::string name;
  std::vector<int32_t> nindex_in;
  std::vector<int32_t> nindex_out;
  bool operator==(const LayerInfo &b) const {
    return type == b.type && primary_layer_index == b.primary_layer_index && name == b.name &&
           nindex_in == b.nindex_in && nindex_out == b.nindex_out;
  }
};

class NetConfig {
 public:
  NetParam param;
  std::vector<LayerInfo> layers;
  std::vector<std::string> node_names;
  std::map<std::string, int> node_name_map;
  std::map<std::string, int> layer_name_map;
  std::string updater_type = "sgd";
  std::string sync_type = "simple";
  std::map<std::string, int> label_name_map;
  std::vector<std::pair<int, int>> label_range;
  KVList defcfg;
  std::vector<KVList> layercfg;
  std::vector<int32_t> extra_shape;

  NetConfig() {
    label_name_map["label"] = 0;
    label_range.emplace_back(0, 1);
  }

  std::string SaveNet() const {
    ByteWriter fo;
    SaveNet(&fo);
    return fo.str();
  }
  void SaveNet(ByteWriter *fo) const {
    fo->WritePOD(param);
    if (param.extra_data_num != 0) fo->WriteVec(extra_shape);
    if (param.num_layers != static_cast<int>(layers.size())) throw std::runtime_error("model inconsistent");
    if (param.num_nodes != static_cast<int>(node_names.size()))
      throw std::runtime_error("num_nodes is inconsistent with node_names");
    for (const auto &n : node_names) fo->WriteStr(n);
    for (const auto &l : layers) {
      fo->WritePOD(l.type);
      fo->WritePOD(l.primary_layer_index);
      fo->WriteStr(l.name);
      fo->WriteVec(l.nindex_in);
      fo->WriteVec(l.nindex_out);
    }
  }
  // Reads the structure; returns number of bytes consumed.
  size_t LoadNet(const char *data, size_t size) {
    ByteReader fi(data, size);
    LoadNet(&fi);
    return fi.tell();
  }
  void LoadNet(ByteReader *fi) {
    param = fi->ReadPOD<NetParam>();
    if (param.num_nodes < 0 || param.num_layers < 0 || param.num_nodes > (1 << 20) ||
        param.num_layers > (1 << 20))
      throw std::runtime_error("NetConfig: invalid model file");
    if (param.extra_data_num != 0) extra_shape = fi->ReadVec<int32_t>();
    node_names.resize(param.num_nodes);
    for (auto &n : node_names) n = fi->ReadStr();
    node_name_map.clear();
    for (size_t i = 0; i < node_names.size(); ++i) node_name_map[node_names[i]] = static_cast<int>(i);
    layers.assign(param.num_layers, LayerInfo());
    layercfg.assign(param.num_layers, KVList());
    layer_name_map.clear();
    for (int i = 0; i < param.num_layers; ++i) {
      LayerInfo &l = layers[i];
      l.type = fi->ReadPOD<int32_t>();
      l.primary_layer_index = fi->ReadPOD<int32_t>();
      l.name = fi->ReadStr();
      l.nindex_in = fi->ReadVec<int32_t>();
      l.nindex_out = fi->ReadVec<int32_t>();
      if (l.type == kSharedLayer) {
        if (!l.name.empty()) throw std::runtime_error("SharedLayer must not have name");
      } else if (!l.name.empty()) {
        if (layer_name_map.count(l.name))
          throw std::runtime_error("NetConfig: invalid model file, duplicated layer name: " + l.name);
        layer_name_map[l.name] = i;
      }
    }
    ClearConfig();
  }

  void SetGlobalParam(const std::string &name, const std::string &val) {
    if (name == "updater") updater_type = val;
    if (name == "sync") sync_type = val;
    unsigned a, b;
    if (sscanf(name.c_str(), "label_vec[%u,%u)", &a, &b) == 2) {
      label_range.emplace_back(static_cast<int>(a), static_cast<int>(b));
      label_name_map[val] = static_cast<int>(label_range.size()) - 1;
    }
  }

  void Configure(const KVList &cfg) {
    ClearConfig();
    if (node_names.empty() && node_name_map.empty()) {
      node_names.push_back("in");
      node_name_map["in"] = 0;
    }
    node_name_map["0"] = 0;
    int netcfg_mode = 0;
    int cfg_top_node = 0;
    int cfg_layer_index = 0;
    for (const auto &kv : cfg) {
      const std::string &name = kv.first;
      const std::string &val = kv.second;
      if (name == "extra_data_num") {
        int num = atoi(val.c_str());
        for (int i = 0; i < num; ++i) {
          std::string nm = "in_" + std::to_string(i + 1);
          if (!node_name_map.count(nm)) {
            node_names.push_back(nm);
            node_name_map[nm] = i + 1;
          }
        }
        param.extra_data_num = num;
      }
      if (!strncmp(name.c_str(), "extra_data_shape[", 17)) {
        int x, y, z;
        if (sscanf(val.c_str(), "%d,%d,%d", &x, &y, &z) != 3)
          throw std::runtime_error("extra data shape config incorrect");
        extra_shape.push_back(x);
        extra_shape.push_back(y);
        extra_shape.push_back(z);
      }
      if (param.init_end == 0 && name == "input_shape") {
        unsigned x, y, z;
        if (sscanf(val.c_str(), "%u,%u,%u", &z, &y, &x) != 3)
          throw std::runtime_error(
              "input_shape must be three consecutive integers without space example: 1,1,200");
        param.input_shape[0] = z;
        param.input_shape[1] = y;
        param.input_shape[2] = x;
      }
      if (netcfg_mode != 2) SetGlobalParam(name, val);
      if (name == "netconfig" && val == "start") netcfg_mode = 1;
      if (name == "netconfig" && val == "end") netcfg_mode = 0;
      if (!strncmp(name.c_str(), "layer[", 6)) {
        LayerInfo info = GetLayerInfo(name, val, cfg_top_node, cfg_layer_index);
        netcfg_mode = 2;
        if (param.init_end == 0) {
          if (static_cast<int>(layers.size()) != cfg_layer_index)
            throw std::runtime_error("NetConfig inconsistent");
          layers.push_back(info);
          layercfg.resize(layers.size());
        } else {
          if (cfg_layer_index >= static_cast<int>(layers.size()))
            throw std::runtime_error("config layer index exceed bound");
          if (!(info == layers[cfg_layer_index]))
            throw std::runtime_error("config setting does not match existing network structure");
        }
        cfg_top_node = info.nindex_out.size() == 1 ? info.nindex_out[0] : -1;
        cfg_layer_index += 1;
        continue;
      }
      if (netcfg_mode == 2) {
        if (layers[cfg_layer_index - 1].type == kSharedLayer)
          throw std::runtime_error(
              "please do not set parameters in shared layer, set them in primary layer");
        layercfg[cfg_layer_index - 1].emplace_back(name, val);
      } else {
        defcfg.emplace_back(name, val);
      }
    }
    if (param.init_end == 0) InitNet();
  }

  int GetLayerIndex(const std::string &name) const {
    auto it = layer_name_map.find(name);
    if (it == layer_name_map.end()) throw std::runtime_error("unknown layer name " + name);
    return it->second;
  }

 private:
  LayerInfo GetLayerInfo(const std::string &sname, const std::string &sval, int top_node,
                         int cfg_layer_index) {
    LayerInfo inf;
    int inc;
    char ltype[256] = {0}, tag[256] = {0}, src[256] = {0}, dst[256] = {0};
    const char *name = sname.c_str();
    if (sscanf(name, "layer[+%d", &inc) == 1) {
      if (top_node < 0)
        throw std::runtime_error(
            "ConfigError: layer[+1] is used, but last layer have more than one output; "
            "use layer[input-name->output-name] instead");
      inf.nindex_in.push_back(top_node);
      if (sscanf(name, "layer[+1:%255[^]]]", tag) == 1) {
        inf.nindex_out.push_back(GetNodeIndex(tag, true));
      } else if (inc == 0) {
        inf.nindex_out.push_back(top_node);
      } else {
        std::string t = "!node-after-" + std::to_string(top_node);
        inf.nindex_out.push_back(GetNodeIndex(t, true));
      }
    } else if (sscanf(name, "layer[%255[^-]->%255[^]]]", src, dst) == 2) {
      ParseNodeIndex(src, &inf.nindex_in, false);
      ParseNodeIndex(dst, &inf.nindex_out, true);
    } else {
      throw std::runtime_error(std::string("ConfigError: invalid layer format ") + name);
    }
    std::string layer_name;
    if (sscanf(sval.c_str(), "%255[^:]:%255s", ltype, tag) == 2) {
      inf.type = GetLayerType(ltype);
      layer_name = tag;
    } else {
      snprintf(ltype, sizeof(ltype), "%s", sval.c_str());
      inf.type = GetLayerType(sval);
    }
    if (inf.type == kSharedLayer) {
      const char *start = strchr(ltype, '[');
      if (start == nullptr)
        throw std::runtime_error("ConfigError: shared layer must specify tag of layer to share with");
      std::string s_tag = start + 1;
      s_tag = s_tag.substr(0, s_tag.size() - 1);
      if (!layer_name_map.count(s_tag))
        throw std::runtime_error("ConfigError: shared layer tag " + s_tag + " is not defined before");
      inf.primary_layer_index = layer_name_map[s_tag];
    } else if (!layer_name.empty()) {
      auto it = layer_name_map.find(layer_name);
      if (it != layer_name_map.end()) {
        if (it->second != cfg_layer_index)
          throw std::runtime_error(
              "ConfigError: layer name in the configuration file do not match the name stored in model");
      } else {
        layer_name_map[layer_name] = cfg_layer_index;
      }
      inf.name = layer_name;
    }
    return inf;
  }
  void ParseNodeIndex(char *nodes, std::vector<int32_t> *out, bool alloc_unknown) {
    char *save = nullptr;
    for (char *p = strtok_r(nodes, ",", &save); p != nullptr; p = strtok_r(nullptr, ",", &save)) {
      out->push_back(GetNodeIndex(p, alloc_unknown));
    }
  }
  int GetNodeIndex(const std::string &key, bool alloc_unknown) {
    auto it = node_name_map.find(key);
    if (it != node_name_map.end()) return it->second;
    if (!alloc_unknown)
      throw std::runtime_error("ConfigError: undefined node name " + key +
                               ", input node of a layer must be specified as output of another "
                               "layer presented before the layer declaration");
    int value = static_cast<int>(node_names.size());
    node_name_map[key] = value;
    node_names.push_back(key);
    return value;
  }
  void InitNet() {
    param.num_nodes = 0;
    param.num_layers = static_cast<int>(layers.size());
    for (const auto &info : layers) {
      for (int j : info.nindex_in) param.num_nodes = std::max(j + 1, param.num_nodes);
      for (int j : info.nindex_out) param.num_nodes = std::max(j + 1, param.num_nodes);
    }
    if (param.num_nodes != static_cast<int>(node_names.size()))
      throw std::runtime_error("num_nodes is inconsistent with node_names");
    param.init_end = 1;
  }
  void ClearConfig() {
    defcfg.clear();
    for (auto &c : layercfg) c.clear();
  }
};

}  // namespace cxxnet_rt
