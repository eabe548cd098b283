// Layer type ids. The integer values are part of the checkpoint format, so they
// are kept identical to the reference enumeration (src/layer/layer.h:284-315)
// and the string -> id mapping follows GetLayerType (src/layer/layer.h:322-361).
#pragma once
#include <cstdio>
#include <cstring>
#include <stdexcept>
#include <string>

namespace cxxnet_rt {

enum : int {
  kSharedLayer = 0,
  kFullConnect = 1,
  kSoftmax = 2,
  kRectifiedLinear = 3,
  kSigmoid = 4,
  kTanh = 5,
  kSoftplus = 6,
  kFlatten = 7,
  kDropout = 8,
  kConv = 10,
  kMaxPooling = 11,
  kSumPooling = 12,
  kAvgPooling = 13,
  kLRN = 15,
  kBias = 17,
  kConcat = 18,
  kXelu = 19,
  kCaffe = 20,
  kReluMaxPooling = 21,
  kMaxout = 22,
  kSplit = 23,
  kInsanity = 24,
  kInsanityPooling = 25,
  kL2Loss = 26,
  kMultiLogistic = 27,
  kChConcat = 28,
  kPRelu = 29,
  kBatchNorm = 30,
  kFixConnect = 31,
  kPairTestGap = 1024,
};

inline int GetLayerType(const std::string &t) {
  const char *type = t.c_str();
  if (!strncmp(type, "share", 5)) return kSharedLayer;
  struct E { const char *n; int v; };
  static const E table[] = {
      {"fullc", kFullConnect}, {"fixconn", kFixConnect}, {"bias", kBias},
      {"softmax", kSoftmax}, {"relu", kRectifiedLinear}, {"sigmoid", kSigmoid},
      {"tanh", kTanh}, {"softplus", kSoftplus}, {"flatten", kFlatten},
      {"dropout", kDropout}, {"conv", kConv}, {"relu_max_pooling", kReluMaxPooling},
      {"max_pooling", kMaxPooling}, {"sum_pooling", kSumPooling},
      {"avg_pooling", kAvgPooling}, {"lrn", kLRN}, {"concat", kConcat},
      {"xelu", kXelu}, {"maxout", kMaxout}, {"split", kSplit},
      {"insanity", kInsanity}, {"insanity_max_pooling", kInsanityPooling},
      {"l2_loss", kL2Loss}, {"multi_logistic", kMultiLogistic},
      {"ch_concat", kChConcat}, {"prelu", kPRelu}, {"batch_norm", kBatchNorm},
      {"caffe", kCaffe},
  };
  for (const auto &e : table) {
    if (!strcmp(type, e.n)) return e.v;
  }
  if (!strncmp(type, "pairtest-", 9)) {
    char tmaster[256] = {0}, tslave[256] = {0};
    if (sscanf(type + 9, "%255[^-]-%255[^:]", tmaster, tslave) != 2) {
      throw std::runtime_error(std::string("invalid pairtest layer type: ") + type);
    }
    return kPairTestGap * GetLayerType(tmaster) + GetLayerType(tslave);
  }
  throw std::runtime_error(std::string("unknown layer type: \"") + type + "\"");
}

}  // namespace cxxnet_rt
