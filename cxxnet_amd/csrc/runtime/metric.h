// Evaluation metrics: error, rmse, logloss, rec@n, bound to a label field.
// Semantics and print format follow reference src/utils/metric.h:20-236:
//   "\t<evname>-<metric>[field]:<value>"  (field omitted when "label").
#pragma once
#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <memory>
#include <sstream>
#include <stdexcept>
#include <string>
#include <utility>
#include <vector>

namespace cxxnet_rt {

// rand_r-based sampler, identical stream to reference src/utils/random.h:16-52.
class RandomSampler {
 public:
  explicit RandomSampler(unsigned seed = 0) : rseed_(seed) {}
  void Seed(unsigned s) { rseed_ = s; }
  double NextDouble() { return static_cast<double>(rand_r(&rseed_)) / (static_cast<double>(RAND_MAX) + 1.0); }
  uint32_t NextUInt32(uint32_t n) { return static_cast<uint32_t>(std::floor(NextDouble() * n)); }
  template <typename T>
  void Shuffle(std::vector<T> &d) {
    if (d.empty()) return;
    for (uint32_t i = static_cast<uint32_t>(d.size()) - 1; i > 0; i--) std::swap(d[i], d[NextUInt32(i + 1)]);
  }

 private:
  unsigned rseed_;
};

class Metric {
 public:
  explicit Metric(const std::string &name) : name_(name) {
    if (name == "rmse") kind_ = 0;
    else if (name == "error") kind_ = 1;
    else if (name == "logloss") kind_ = 2;
    else if (!strncmp(name.c_str(), "rec@", 4)) {
      kind_ = 3;
      if (sscanf(name.c_str(), "rec@%d", &topn_) != 1) throw std::runtime_error("must specify n for rec@n");
    } else {
      throw std::runtime_error("Metric: Unknown metric name: " + name);
    }
    Clear();
  }
  void Clear() { sum_ = 0.0; cnt_ = 0; }
  // pred: [n, k] row-major; label: [n, w] row-major.
  void AddEval(const float *pred, int n, int k, const float *label, int w) {
    for (int i = 0; i < n; ++i) {
      sum_ += Calc(pred + static_cast<size_t>(i) * k, k, label + static_cast<size_t>(i) * w, w);
      cnt_ += 1;
    }
  }
  double Get() const { return cnt_ == 0 ? 0.0 : sum_ / cnt_; }
  const std::string &name() const { return name_; }

 private:
  float Calc(const float *p, int k, const float *y, int w) {
    switch (kind_) {
      case 0: {
        if (k != w) throw std::runtime_error("Metric: In RMSE metric, the size of prediction and label must be same.");
        float d = 0;
        for (int i = 0; i < w; ++i) d += (p[i] - y[i]) * (p[i] - y[i]);
        return d;
      }
      case 1: {
        int maxidx = 0;
        if (k != 1) {
          for (int i = 1; i < k; ++i)
            if (p[i] > p[maxidx]) maxidx = i;
        } else {
          maxidx = p[0] > 0.0f ? 1 : 0;
        }
        return maxidx != static_cast<int>(y[0]);
      }
      case 2: {
        if (k != 1) {
          int t = static_cast<int>(y[0]);
          return -std::log(std::max(std::min(p[t], 1.0f - 1e-15f), 1e-15f));
        }
        const float py = std::max(std::min(p[0], 1.0f - 1e-15f), 1e-15f);
        const float res = -(y[0] * std::log(py) + (1.0f - y[0]) * std::log(1 - py));
        if (res != res) throw std::runtime_error("NaN detected!");
        return res;
      }
      default: {
        if (k < topn_) throw std::runtime_error("it is meaningless to take rec@n for list shorter than n");
        vec_.resize(k);
        for (int i = 0; i < k; ++i) vec_[i] = std::make_pair(p[i], i);
        rnd_.Shuffle(vec_);
        std::sort(vec_.begin(), vec_.end(),
                  [](const std::pair<float, int> &a, const std::pair<float, int> &b) { return a.first > b.first; });
        int hit = 0;
        for (int i = 0; i < topn_; ++i) {
          for (int j = 0; j < w; ++j) {
            if (vec_[i].second == static_cast<int>(y[j])) {
              ++hit;
              break;
            }
          }
        }
        return static_cast<float>(hit) / w;
      }
    }
  }
  std::string name_;
  int kind_ = 1;
  int topn_ = 1;
  double sum_ = 0.0;
  long cnt_ = 0;
  std::vector<std::pair<float, int>> vec_;
  RandomSampler rnd_;
};

}  // namespace cxxnet_rt
