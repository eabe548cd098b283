// Native data-IO primitives:
//  * MNIST idx(.gz) loader                      (reference src/io/iter_mnist-inl.hpp:77-108)
//  * BinaryPage 64 MB paged object container    (reference src/utils/io.h:254-326)
//  * ImageBinReader: threaded page prefetcher over a .bin file
//                                               (reference src/io/iter_thread_imbin-inl.hpp)
//  * image list (.lst) parser                   (`index \t label... \t path`)
#pragma once
#include <zlib.h>

#include <atomic>
#include <condition_variable>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <deque>
#include <fstream>
#include <memory>
#include <mutex>
#include <sstream>
#include <stdexcept>
#include <string>
#include <thread>
#include <vector>

namespace cxxnet_rt {

// ---------------------------------------------------------------- gz / raw reader
inline std::string ReadMaybeGz(const std::string &path) {
  gzFile f = gzopen(path.c_str(), "rb");  // zlib reads plain files transparently
  if (f == nullptr) throw std::runtime_error("cannot open file " + path);
  std::string out;
  char buf[1 << 16];
  int n;
  while ((n = gzread(f, buf, sizeof(buf))) > 0) out.append(buf, n);
  gzclose(f);
  if (n < 0) throw std::runtime_error("gz read error on " + path);
  return out;
}

inline int32_t ReadBE32(const std::string &s, size_t off) {
  if (off + 4 > s.size()) throw std::runtime_error("Failed to read an int");
  const unsigned char *b = reinterpret_cast<const unsigned char *>(s.data() + off);
  return static_cast<int32_t>(b[0] << 24 | b[1] << 16 | b[2] << 8 | b[3]);
}

// Returns images as float32 [count, rows, cols] scaled by 1/256 and labels.
struct MNISTData {
  int count = 0, rows = 0, cols = 0;
  std::vector<float> images;
  std::vector<float> labels;
};

inline MNISTData LoadMNIST(const std::string &path_img, const std::string &path_label) {
  MNISTData d;
  std::string img = ReadMaybeGz(path_img);
  ReadBE32(img, 0);
  d.count = ReadBE32(img, 4);
  d.rows = ReadBE32(img, 8);
  d.cols = ReadBE32(img, 12);
  size_t n = static_cast<size_t>(d.count) * d.rows * d.cols;
  if (img.size() < 16 + n) throw std::runtime_error("MNIST image file truncated");
  d.images.resize(n);
  const unsigned char *p = reinterpret_cast<const unsigned char *>(img.data() + 16);
  for (size_t i = 0; i < n; ++i) d.images[i] = p[i] * (1.0f / 256.0f);
  std::string lab = ReadMaybeGz(path_label);
  ReadBE32(lab, 0);
  int nl = ReadBE32(lab, 4);
  if (lab.size() < 8 + static_cast<size_t>(nl)) throw std::runtime_error("MNIST label file truncated");
  d.labels.resize(nl);
  const unsigned char *q = reinterpret_cast<const unsigned char *>(lab.data() + 8);
  for (int i = 0; i < nl; ++i) d.labels[i] = q[i];
  return d;
}

// ---------------------------------------------------------------- BinaryPage
class BinaryPage {
 public:
  static constexpr size_t kPageInts = 64 << 18;  // 64 MB page
  static constexpr size_t kPageBytes = kPageInts * sizeof(int32_t);
  // zero = false: contents left undefined (a page about to be overwritten by a file read)
  explicit BinaryPage(bool zero = true) : data_(new int32_t[kPageInts]) {
    if (zero) Clear();
  }
  int32_t Size() const { return data_[0]; }
  void Clear() { std::fill(data_.get(), data_.get() + kPageInts, 0); }
  bool Push(const void *p, size_t sz) {
    if (FreeBytes() < sz + sizeof(int32_t)) return false;
    int32_t s = Size();
    data_[s + 2] = data_[s + 1] + static_cast<int32_t>(sz);
    std::memcpy(Offset(data_[s + 2]), p, sz);
    ++data_[0];
    return true;
  }
  // object r's byte range [*a, *b) within the page
  void Span(int r, long *a, long *b) const {
    if (r < 0 || r >= Size()) throw std::runtime_error("BinaryPage: index exceed bound");
    *a = static_cast<long>(kPageBytes) - data_[r + 2];
    *b = static_cast<long>(kPageBytes) - data_[r + 1];
  }
  std::string Get(int r) const {
    if (r < 0 || r >= Size()) throw std::runtime_error("BinaryPage: index exceed bound");
    int32_t end = data_[r + 2], beg = data_[r + 1];
    return std::string(Offset(end), static_cast<size_t>(end - beg));
  }
  char *raw() { return reinterpret_cast<char *>(data_.get()); }
  const char *raw() const { return reinterpret_cast<const char *>(data_.get()); }
  bool Valid() const {
    int32_t s = Size();
    if (s < 0 || static_cast<size_t>(s) + 2 > kPageInts) return false;
    for (int r = 0; r < s; ++r) {
      if (data_[r + 2] < data_[r + 1] || static_cast<size_t>(data_[r + 2]) > kPageBytes) return false;
    }
    return true;
  }

 private:
  size_t FreeBytes() const {
    int32_t s = Size();
    return (kPageInts - (s + 2)) * sizeof(int32_t) - static_cast<size_t>(data_[s + 1]);
  }
  char *Offset(int32_t pos) { return raw() + (kPageBytes - pos); }
  const char *Offset(int32_t pos) const { return raw() + (kPageBytes - pos); }
  std::unique_ptr<int32_t[]> data_;
};

// Packs a list of files into BinaryPages (the im2bin tool; reference tools/im2bin.cpp:6-67).
inline size_t PackImageBin(const std::vector<std::string> &files, const std::string &out_path) {
  std::ofstream fo(out_path, std::ios::binary);
  if (!fo) throw std::runtime_error("cannot open " + out_path);
  BinaryPage page;
  size_t npages = 0;
  for (const auto &f : files) {
    std::ifstream fi(f, std::ios::binary);
    if (!fi) throw std::runtime_error("cannot open image " + f);
    std::string buf((std::istreambuf_iterator<char>(fi)), std::istreambuf_iterator<char>());
    if (!page.Push(buf.data(), buf.size())) {
      fo.write(page.raw(), BinaryPage::kPageBytes);
      ++npages;
      page.Clear();
      if (!page.Push(buf.data(), buf.size())) throw std::runtime_error("image larger than a page: " + f);
    }
  }
  if (page.Size() != 0) {
    fo.write(page.raw(), BinaryPage::kPageBytes);
    ++npages;
  }
  return npages;
}

// Threaded reader over one or more .bin files: a background thread loads
// pages ahead (double buffer) so decoding never waits on disk.
class ImageBinReader {
 public:
  ImageBinReader(std::vector<std::string> paths, int prefetch)
      : paths_(std::move(paths)), prefetch_(prefetch < 1 ? 1 : prefetch) {
    Start();
  }
  ~ImageBinReader() { Stop(); }
  // Rewind to the first page.
  void BeforeFirst() {
    Stop();
    Start();
  }
  // Next object bytes; returns false at end of all files.
  bool Next(std::string *out) {
    while (cur_ == nullptr || cur_idx_ >= cur_->Size()) {
      std::unique_lock<std::mutex> lk(mu_);
      if (cur_ != nullptr) free_.push_back(std::move(cur_));  // recycled by the loader
      cv_.wait(lk, [&] { return !queue_.empty() || done_; });
      if (queue_.empty()) return false;
      cur_ = std::move(queue_.front());
      queue_.pop_front();
      cur_idx_ = 0;
      cv_.notify_all();
    }
    *out = cur_->Get(cur_idx_++);
    return true;
  }
  // True when Next() will not wait (the current page still has objects): callers holding an
  // interpreter lock then need not drop it per record.
  bool Ready() const { return cur_ != nullptr && cur_idx_ < cur_->Size(); }
  // Up to n consecutive objects of one page as ONE contiguous byte range: (*blob, object k at
  // [spans[k].first, +spans[k].second) of it).  Objects are packed backward from the page end,
  // so a run of them is one span of the page (copied once instead of once per object).  False
  // at the end of all files.
  bool NextRun(int n, std::string *blob, std::vector<std::pair<long, long>> *spans) {
    spans->clear();
    blob->clear();
    std::string first;
    if (n <= 0) return true;
    if (!Ready()) {  // move to the next page (Next() waits for it), then un-take its first object
      if (!Next(&first)) return false;
      --cur_idx_;
    }
    const int r0 = cur_idx_, r1 = std::min(cur_->Size(), r0 + n);
    long lo = 0, hi = 0;
    cur_->Span(r1 - 1, &lo, &hi);  // the run's lowest address: its last object
    long a = 0, b = 0;
    cur_->Span(r0, &a, &b);
    const long base = lo, top = b;
    blob->assign(cur_->raw() + base, static_cast<size_t>(top - base));
    for (int r = r0; r < r1; ++r) {
      cur_->Span(r, &a, &b);
      spans->emplace_back(a - base, b - a);
    }
    cur_idx_ = r1;
    return true;
  }
  // All remaining objects of the current page (or of the next page when the current
  // one is exhausted); false at end of all files.  Used by the page-shuffling reader.
  bool NextPage(std::vector<std::string> *out) {
    out->clear();
    std::string s;
    if (!Next(&s)) return false;
    out->push_back(std::move(s));
    while (cur_idx_ < cur_->Size()) out->push_back(cur_->Get(cur_idx_++));
    return true;
  }
  // Non-empty when a file could not be opened by the loader thread.
  std::string Error() {
    std::lock_guard<std::mutex> lk(mu_);
    return error_;
  }

 private:
  void Start() {
    done_ = false;
    stop_ = false;
    cur_.reset();
    cur_idx_ = 0;
    queue_.clear();
    worker_ = std::thread([this] { Run(); });
  }
  void Stop() {
    {
      std::lock_guard<std::mutex> lk(mu_);
      stop_ = true;
    }
    cv_.notify_all();
    if (worker_.joinable()) worker_.join();
  }
  void Run() {
    for (const auto &p : paths_) {
      std::ifstream fi(p, std::ios::binary);
      if (!fi) {
        std::lock_guard<std::mutex> lk(mu_);
        error_ = "cannot open " + p;
        break;
      }
      while (true) {
        // a recycled page when there is one: a fresh 64 MB page costs its page faults, which
        // made the loader (not the decoders) the limit of the whole pipeline
        std::unique_ptr<BinaryPage> page;
        {
          std::lock_guard<std::mutex> lk(mu_);
          if (!free_.empty()) {
            page = std::move(free_.back());
            free_.pop_back();
          }
        }
        if (page == nullptr) page = std::make_unique<BinaryPage>(false);
        fi.read(page->raw(), BinaryPage::kPageBytes);
        if (fi.gcount() != static_cast<std::streamsize>(BinaryPage::kPageBytes)) break;
        if (!page->Valid()) break;
        std::unique_lock<std::mutex> lk(mu_);
        cv_.wait(lk, [&] { return static_cast<int>(queue_.size()) < prefetch_ || stop_; });
        if (stop_) return;
        queue_.push_back(std::move(page));
        cv_.notify_all();
      }
    }
    std::lock_guard<std::mutex> lk(mu_);
    done_ = true;
    cv_.notify_all();
  }

  std::vector<std::string> paths_;
  int prefetch_;
  std::thread worker_;
  std::mutex mu_;
  std::condition_variable cv_;
  std::deque<std::unique_ptr<BinaryPage>> queue_;
  std::vector<std::unique_ptr<BinaryPage>> free_;
  std::unique_ptr<BinaryPage> cur_;
  int cur_idx_ = 0;
  bool done_ = false, stop_ = false;
  std::string error_;
};

// Parses an image list: `index \t label_1 ... label_w \t path` per line.
struct ImageListEntry {
  uint32_t index;
  std::vector<float> labels;
  std::string path;
};

inline std::vector<ImageListEntry> ParseImageList(const std::string &path, int label_width) {
  std::ifstream fi(path);
  if (!fi) throw std::runtime_error("cannot open image list " + path);
  std::vector<ImageListEntry> out;
  std::string line;
  while (std::getline(fi, line)) {
    if (line.empty() || line == "\r") continue;
    std::istringstream ss(line);
    ImageListEntry e;
    if (!(ss >> e.index)) continue;
    e.labels.resize(label_width);
    for (int i = 0; i < label_width; ++i) ss >> e.labels[i];
    std::string rest;
    std::getline(ss, rest);
    size_t b = rest.find_first_not_of(" \t");
    size_t en = rest.find_last_not_of(" \t\r\n");
    e.path = (b == std::string::npos) ? "" : rest.substr(b, en - b + 1);
    out.push_back(std::move(e));
  }
  return out;
}

}  // namespace cxxnet_rt
