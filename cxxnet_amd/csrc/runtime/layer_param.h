// Common per-layer POD parameters. Serialized raw (328 bytes) at the head of
// every parameterised layer's blob, so the field order and defaults follow the
// reference LayerParam (src/layer/param.h:15-111) exactly.
#pragma once
#include <cstdint>
#include <cstdlib>
#include <cstring>
#include <stdexcept>
#include <string>

namespace cxxnet_rt {

struct LayerParam {
  int32_t num_hidden = 0;
  float init_sigma = 0.01f;
  int32_t init_sparse = 10;
  float init_uniform = -1.0f;
  float init_bias = 0.0f;
  int32_t num_channel = 0;
  int32_t random_type = 0;
  int32_t num_group = 1;
  int32_t kernel_height = 0;
  int32_t kernel_width = 0;
  int32_t stride = 1;
  int32_t pad_y = 0;
  int32_t pad_x = 0;
  int32_t no_bias = 0;
  int32_t temp_col_max = 64 << 18;
  int32_t silent = 0;
  int32_t num_input_channel = 0;
  int32_t num_input_node = 0;
  int32_t reserved[64] = {0};

  void SetParam(const std::string &n, const std::string &v) {
    const char *name = n.c_str();
    const char *val = v.c_str();
    if (!strcmp(name, "init_sigma")) init_sigma = static_cast<float>(atof(val));
    if (!strcmp(name, "init_uniform")) init_uniform = static_cast<float>(atof(val));
    if (!strcmp(name, "init_bias")) init_bias = static_cast<float>(atof(val));
    if (!strcmp(name, "init_sparse")) init_sparse = atoi(val);
    if (!strcmp(name, "random_type")) {
      if (!strcmp(val, "gaussian")) random_type = 0;
      else if (!strcmp(val, "uniform")) random_type = 1;
      else if (!strcmp(val, "xavier")) random_type = 1;
      else if (!strcmp(val, "kaiming")) random_type = 2;
      else throw std::runtime_error(std::string("invalid random_type ") + val);
    }
    if (!strcmp(name, "nhidden")) num_hidden = atoi(val);
    if (!strcmp(name, "nchannel")) num_channel = atoi(val);
    if (!strcmp(name, "ngroup")) num_group = atoi(val);
    if (!strcmp(name, "kernel_size")) kernel_width = kernel_height = atoi(val);
    if (!strcmp(name, "kernel_height")) kernel_height = atoi(val);
    if (!strcmp(name, "kernel_width")) kernel_width = atoi(val);
    if (!strcmp(name, "stride")) stride = atoi(val);
    if (!strcmp(name, "pad")) pad_y = pad_x = atoi(val);
    if (!strcmp(name, "pad_y")) pad_y = atoi(val);
    if (!strcmp(name, "pad_x")) pad_x = atoi(val);
    if (!strcmp(name, "no_bias")) no_bias = atoi(val);
    if (!strcmp(name, "silent")) silent = atoi(val);
    if (!strcmp(name, "temp_col_max")) temp_col_max = atoi(val) << 18;
  }
};
static_assert(sizeof(LayerParam) == 328, "LayerParam must stay 328 bytes (checkpoint layout)");

}  // namespace cxxnet_rt
