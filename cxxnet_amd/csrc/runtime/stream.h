// Binary serialization streams used for checkpoints and dataset pages.
// Encoding matches the reference IStream helpers (src/utils/io.h:19-103):
// vectors and strings carry a uint64 little-endian length prefix.
#pragma once
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <stdexcept>
#include <string>
#include <vector>

namespace cxxnet_rt {

class ByteWriter {
 public:
  void Write(const void *p, size_t n) {
    const char *c = static_cast<const char *>(p);
    buf_.append(c, n);
  }
  template <typename T>
  void WritePOD(const T &v) { Write(&v, sizeof(T)); }
  template <typename T>
  void WriteVec(const std::vector<T> &v) {
    uint64_t sz = v.size();
    WritePOD(sz);
    if (sz) Write(v.data(), sizeof(T) * sz);
  }
  void WriteStr(const std::string &s) {
    uint64_t sz = s.size();
    WritePOD(sz);
    if (sz) Write(s.data(), sz);
  }
  const std::string &str() const { return buf_; }
  std::string &str() { return buf_; }

 private:
  std::string buf_;
};

class ByteReader {
 public:
  ByteReader(const char *data, size_t size) : d_(data), n_(size), pos_(0) {}
  void Read(void *p, size_t n) {
    if (pos_ + n > n_) throw std::runtime_error("ByteReader: unexpected end of stream (invalid model file)");
    std::memcpy(p, d_ + pos_, n);
    pos_ += n;
  }
  template <typename T>
  T ReadPOD() { T v; Read(&v, sizeof(T)); return v; }
  template <typename T>
  std::vector<T> ReadVec() {
    uint64_t sz = ReadPOD<uint64_t>();
    if (sz * sizeof(T) > n_ - pos_) throw std::runtime_error("ByteReader: vector length exceeds stream");
    std::vector<T> v(sz);
    if (sz) Read(v.data(), sizeof(T) * sz);
    return v;
  }
  std::string ReadStr() {
    uint64_t sz = ReadPOD<uint64_t>();
    if (sz > n_ - pos_) throw std::runtime_error("ByteReader: string length exceeds stream");
    std::string s(sz, '\0');
    if (sz) Read(&s[0], sz);
    return s;
  }
  size_t tell() const { return pos_; }
  size_t remaining() const { return n_ - pos_; }

 private:
  const char *d_;
  size_t n_;
  size_t pos_;
};

}  // namespace cxxnet_rt
