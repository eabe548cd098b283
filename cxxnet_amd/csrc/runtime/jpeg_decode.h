// Native threaded JPEG decode + crop/mirror augmentation into a uint8 HWC batch.
//
// Reference: src/io/iter_thread_imbin_x-inl.hpp:150-388 (page thread -> decode thread ->
// batch), src/utils/decoder.h:21-125 (libjpeg decode of one record), and the geometric part
// of src/io/iter_augment_proc-inl.hpp:98-162 (crop, mirror; mean / contrast / illumination
// are applied on the GPU by the image kernel, so only their random draws happen here).
//
// MI355X-first shape of it:
//   * a persistent pool of std::threads (no interpreter, no per-image Python work): one call
//     decodes a whole batch, records handed out by an atomic counter, the GIL released;
//   * libjpeg-turbo is loaded at run time (dlopen of the system libjpeg.so.8 -- the image has
//     the library but not its headers, so the v8 ABI structs used are declared below and
//     the struct size is checked by jpeg_CreateDecompress itself);
//   * only the crop window is decoded: jpeg_crop_scanline narrows the IDCT to the iMCU
//     columns around the crop and jpeg_skip_scanlines skips the rows above it;
//   * every record's crop / mirror / contrast / illumination draws come from its own
//     generator seeded by the per-record seed the iterator draws, so a batch does not depend
//     on the thread count or on which thread decoded which record;
//   * a record libjpeg cannot decode to RGB (PNG, CMYK JPEG, corrupt data) is reported back
//     and decoded by the Pillow path instead.
#pragma once
#include <dlfcn.h>

#include <algorithm>
#include <atomic>
#include <condition_variable>
#include <csetjmp>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <fstream>
#include <functional>
#include <mutex>
#include <stdexcept>
#include <string>
#include <thread>
#include <vector>

namespace cxxnet_rt {
namespace jpg {

// ---- libjpeg v8 ABI (jpeglib.h / jmorecfg.h of libjpeg-turbo, JPEG_LIB_VERSION 80) --------
typedef int boolean_t;
typedef unsigned int JDIMENSION;
typedef unsigned char JSAMPLE;
typedef JSAMPLE *JSAMPROW;
typedef JSAMPROW *JSAMPARRAY;
enum { JCS_RGB = 2, JDCT_ISLOW = 0, JPEG_LIB_VERSION = 80 };
struct jpeg_common_struct;
typedef jpeg_common_struct *j_common_ptr;

struct jpeg_error_mgr {
  void (*error_exit)(j_common_ptr);
  void (*emit_message)(j_common_ptr, int);
  void (*output_message)(j_common_ptr);
  void (*format_message)(j_common_ptr, char *);
  void (*reset_error_mgr)(j_common_ptr);
  int msg_code;
  union {
    int i[8];
    char s[80];
  } msg_parm;
  int trace_level;
  long num_warnings;
  const char *const *jpeg_message_table;
  int last_jpeg_message;
  const char *const *addon_message_table;
  int first_addon_message;
  int last_addon_message;
};

struct jpeg_decompress_struct {
  jpeg_error_mgr *err;
  void *mem, *progress, *client_data;
  boolean_t is_decompressor;
  int global_state;
  void *src;
  JDIMENSION image_width, image_height;
  int num_components;
  int jpeg_color_space, out_color_space;
  unsigned int scale_num, scale_denom;
  double output_gamma;
  boolean_t buffered_image, raw_data_out;
  int dct_method;
  boolean_t do_fancy_upsampling, do_block_smoothing, quantize_colors;
  int dither_mode;
  boolean_t two_pass_quantize;
  int desired_number_of_colors;
  boolean_t enable_1pass_quant, enable_external_quant, enable_2pass_quant;
  JDIMENSION output_width, output_height;
  int out_color_components, output_components, rec_outbuf_height;
  int actual_number_of_colors;
  JSAMPARRAY colormap;
  JDIMENSION output_scanline;
  int input_scan_number;
  JDIMENSION input_iMCU_row;
  int output_scan_number;
  JDIMENSION output_iMCU_row;
  void *coef_bits;
  void *quant_tbl_ptrs[4], *dc_huff_tbl_ptrs[4], *ac_huff_tbl_ptrs[4];
  int data_precision;
  void *comp_info;
  boolean_t is_baseline, progressive_mode, arith_code;
  unsigned char arith_dc_L[16], arith_dc_U[16], arith_ac_K[16];
  unsigned int restart_interval;
  boolean_t saw_JFIF_marker;
  unsigned char JFIF_major_version, JFIF_minor_version, density_unit;
  unsigned short X_density, Y_density;
  boolean_t saw_Adobe_marker;
  unsigned char Adobe_transform;
  boolean_t CCIR601_sampling;
  void *marker_list;
  int max_h_samp_factor, max_v_samp_factor;
  int min_DCT_h_scaled_size, min_DCT_v_scaled_size;
  JDIMENSION total_iMCU_rows;
  JSAMPLE *sample_range_limit;
  int comps_in_scan;
  void *cur_comp_info[4];
  JDIMENSION MCUs_per_row, MCU_rows_in_scan;
  int blocks_in_MCU;
  int MCU_membership[10];
  int Ss, Se, Ah, Al;
  int block_size;
  const int *natural_order;
  int lim_Se;
  int unread_marker;
  void *master, *main, *coef, *post, *inputctl, *marker, *entropy, *idct, *upsample, *cconvert, *cquantize;
};
static_assert(sizeof(jpeg_decompress_struct) == 656, "libjpeg v8 jpeg_decompress_struct layout");

struct Api {
  jpeg_error_mgr *(*std_error)(jpeg_error_mgr *) = nullptr;
  void (*create_decompress)(jpeg_decompress_struct *, int, size_t) = nullptr;
  void (*destroy_decompress)(jpeg_decompress_struct *) = nullptr;
  void (*mem_src)(jpeg_decompress_struct *, const unsigned char *, unsigned long) = nullptr;
  int (*read_header)(jpeg_decompress_struct *, boolean_t) = nullptr;
  boolean_t (*start_decompress)(jpeg_decompress_struct *) = nullptr;
  JDIMENSION (*read_scanlines)(jpeg_decompress_struct *, JSAMPARRAY, JDIMENSION) = nullptr;
  JDIMENSION (*skip_scanlines)(jpeg_decompress_struct *, JDIMENSION) = nullptr;
  void (*crop_scanline)(jpeg_decompress_struct *, JDIMENSION *, JDIMENSION *) = nullptr;
  void (*abort_decompress)(jpeg_decompress_struct *) = nullptr;
  std::string error;
  bool ok = false;

  Api() {
    const char *names[] = {"libjpeg.so.8", "libjpeg.so"};
    void *h = nullptr;
    for (const char *n : names)
      if ((h = dlopen(n, RTLD_NOW | RTLD_LOCAL)) != nullptr) break;
    if (h == nullptr) {
      error = "libjpeg.so.8 not found";
      return;
    }
    bool all = true;
    auto sym = [&](auto &fn, const char *name) {
      fn = reinterpret_cast<std::remove_reference_t<decltype(fn)>>(dlsym(h, name));
      all = all && fn != nullptr;
    };
    sym(std_error, "jpeg_std_error");
    sym(create_decompress, "jpeg_CreateDecompress");
    sym(destroy_decompress, "jpeg_destroy_decompress");
    sym(mem_src, "jpeg_mem_src");
    sym(read_header, "jpeg_read_header");
    sym(start_decompress, "jpeg_start_decompress");
    sym(read_scanlines, "jpeg_read_scanlines");
    sym(skip_scanlines, "jpeg_skip_scanlines");
    sym(crop_scanline, "jpeg_crop_scanline");
    sym(abort_decompress, "jpeg_abort_decompress");
    ok = all;
    if (!ok) error = "libjpeg lacks the libjpeg-turbo partial-decode entry points";
  }
};

inline const Api &api() {
  static Api a;
  return a;
}

// error manager with a jump target: libjpeg's error_exit must not return
struct ErrMgr {
  jpeg_error_mgr pub;
  char pad[256];  // slack in case the library's manager is larger than declared
  std::jmp_buf jb;
  int code;
};
inline void on_error(j_common_ptr c) {
  ErrMgr *e = reinterpret_cast<ErrMgr *>(*reinterpret_cast<jpeg_error_mgr **>(c));
  e->code = e->pub.msg_code;
  std::longjmp(e->jb, 1);
}
inline void on_message(j_common_ptr, int) {}  // corrupt-data warnings: decode what is there

// splitmix64 -> uniform draws; one generator per record
struct Rng {
  uint64_t s;
  explicit Rng(uint64_t seed) : s(seed) {}
  uint64_t next() {
    uint64_t z = (s += 0x9E3779B97F4A7C15ull);
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
  }
  double uniform() { return static_cast<double>(next() >> 11) * (1.0 / 9007199254740992.0); }  // [0, 1)
  uint32_t below(uint32_t n) { return n ? static_cast<uint32_t>((static_cast<unsigned __int128>(next()) * n) >> 64) : 0; }
};

}  // namespace jpg

// Per-batch augmentation settings (the geometric subset of AugmentParam, io/augment.py)
struct CropConfig {
  int out_h = 0, out_w = 0, channels = 3;
  int rand_crop = 0, rand_mirror = 0, mirror = 0, crop_y_start = -1, crop_x_start = -1;
  float max_random_contrast = 0.f, max_random_illumination = 0.f;
  int mean_mode = 0;
};

struct DecodeItem {
  int row;
  const unsigned char *data;  // encoded bytes (nullptr: read `path`)
  size_t size;
  std::string path;
  uint64_t seed;
};

// Decodes one record's crop into out (out_h x out_w x channels, row-major), params (y, x,
// mirrored), (contrast, illumination).  Returns 0, or a libjpeg message code / -1 / -2.
inline int DecodeCrop(const jpg::Api &J, const unsigned char *buf, size_t len, const CropConfig &c, uint64_t seed,
                      unsigned char *out, int *prm, float *cm, std::vector<unsigned char> &row) {
  using namespace jpg;
  jpeg_decompress_struct cinfo;
  ErrMgr err;
  std::memset(&cinfo, 0, sizeof(cinfo));
  cinfo.err = J.std_error(&err.pub);
  err.pub.error_exit = on_error;
  err.pub.emit_message = on_message;
  err.code = 0;
  volatile bool created = false;  // read after a longjmp
  if (setjmp(err.jb)) {
    if (created) J.destroy_decompress(&cinfo);
    return err.code > 0 ? err.code : -1;
  }
  J.create_decompress(&cinfo, JPEG_LIB_VERSION, sizeof(cinfo));
  created = true;
  J.mem_src(&cinfo, buf, static_cast<unsigned long>(len));
  J.read_header(&cinfo, 1);
  cinfo.out_color_space = JCS_RGB;
  cinfo.dct_method = JDCT_ISLOW;
  const int H = static_cast<int>(cinfo.image_height), W = static_cast<int>(cinfo.image_width);
  const int ch = c.out_h, cw = c.out_w;
  if (H < ch || W < cw) {
    J.destroy_decompress(&cinfo);
    return -2;  // the Pillow path raises the reference's message
  }
  // the draws of io/augment.py _augment_one, in its order
  Rng rng(seed);
  int yy = H - ch, xx = W - cw;
  if (c.rand_crop && (yy || xx)) {
    yy = static_cast<int>(rng.below(static_cast<uint32_t>(yy + 1)));
    xx = static_cast<int>(rng.below(static_cast<uint32_t>(xx + 1)));
  } else {
    yy /= 2;
    xx /= 2;
  }
  if (H != ch && c.crop_y_start != -1) yy = c.crop_y_start;
  if (W != cw && c.crop_x_start != -1) xx = c.crop_x_start;
  if (yy < 0 || xx < 0 || yy + ch > H || xx + cw > W) {
    J.destroy_decompress(&cinfo);
    return -2;
  }
  float contrast = static_cast<float>(rng.uniform() * c.max_random_contrast * 2 - c.max_random_contrast + 1);
  float illum = static_cast<float>(rng.uniform() * c.max_random_illumination * 2 - c.max_random_illumination);
  bool mirror;
  if (c.mean_mode == 0) {
    mirror = c.rand_mirror && rng.uniform() < 0.5;
    contrast = 1.f;
    illum = 0.f;
  } else {
    mirror = (c.rand_mirror && rng.uniform() < 0.5) || c.mirror == 1;
  }
  J.start_decompress(&cinfo);
  if (cinfo.output_components != 3) {
    J.abort_decompress(&cinfo);
    J.destroy_decompress(&cinfo);
    return -1;
  }
  // crop_scanline aligns the window's left edge down to an iMCU boundary but keeps its right
  // edge where asked, and the fancy upsampler treats that edge as the image border: ask for
  // up to 16 more columns so the crop's last column keeps its right-hand chroma context
  // (bit-identical to a full decode then; without the margin the edge column differs by a few
  // levels on 4:2:0 images)
  JDIMENSION x0 = static_cast<JDIMENSION>(xx), wd = static_cast<JDIMENSION>(std::min(cw + 16, W - xx));
  J.crop_scanline(&cinfo, &x0, &wd);  // x0 <= xx, x0 + wd >= xx + cw
  const int dx = xx - static_cast<int>(x0);
  row.resize(static_cast<size_t>(cinfo.output_width) * 3 + 64);
  if (yy > 0) J.skip_scanlines(&cinfo, static_cast<JDIMENSION>(yy));
  const int C = c.channels;
  for (int y = 0; y < ch; ++y) {
    JSAMPROW rp = row.data();
    if (J.read_scanlines(&cinfo, &rp, 1) != 1) {
      J.abort_decompress(&cinfo);
      J.destroy_decompress(&cinfo);
      return -1;
    }
    const unsigned char *src = row.data() + static_cast<size_t>(dx) * 3;
    unsigned char *dst = out + static_cast<size_t>(y) * cw * C;
    if (!mirror) {
      if (C == 3) {
        std::memcpy(dst, src, static_cast<size_t>(cw) * 3);
      } else {
        for (int x = 0; x < cw; ++x)
          for (int k = 0; k < C; ++k) dst[x * C + k] = src[x * 3 + k];
      }
    } else {
      for (int x = 0; x < cw; ++x) {
        const unsigned char *s = src + static_cast<size_t>(cw - 1 - x) * 3;
        for (int k = 0; k < C; ++k) dst[x * C + k] = s[k];
      }
    }
  }
  // the rows below the crop are never decoded
  J.abort_decompress(&cinfo);
  J.destroy_decompress(&cinfo);
  prm[0] = yy;
  prm[1] = xx;
  prm[2] = mirror ? 1 : 0;
  cm[0] = contrast;
  cm[1] = illum;
  return 0;
}

// Persistent decode thread pool.  Run() hands a batch of records to every thread and
// returns when all are done (the caller's thread works too).
class JpegDecodePool {
 public:
  explicit JpegDecodePool(int nthreads) {
    if (nthreads < 1) nthreads = 1;
    for (int t = 1; t < nthreads; ++t) threads_.emplace_back([this] { Loop(); });
  }
  ~JpegDecodePool() {
    {
      std::lock_guard<std::mutex> lk(mu_);
      stop_ = true;
    }
    cv_.notify_all();
    for (auto &t : threads_) t.join();
  }
  int threads() const { return static_cast<int>(threads_.size()) + 1; }

  // out: [B][out_h][out_w][channels] uint8, prm: [B][4] int32, cm: [B][2] float.  Returns the
  // rows that were not decoded (caller falls back to Pillow for them).
  std::vector<int> Run(const std::vector<DecodeItem> &items, const CropConfig &cfg, unsigned char *out, int32_t *prm,
                       float *cm) {
    const jpg::Api &J = jpg::api();
    if (!J.ok) throw std::runtime_error("native JPEG decoder unavailable: " + J.error);
    std::vector<int> failed_flag(items.size(), 0);
    const size_t img_bytes = static_cast<size_t>(cfg.out_h) * cfg.out_w * cfg.channels;
    auto work = [&, img_bytes](size_t i, std::vector<unsigned char> &rowbuf, std::string &filebuf) {
      const DecodeItem &it = items[i];
      const unsigned char *p = it.data;
      size_t n = it.size;
      if (p == nullptr) {
        std::ifstream f(it.path, std::ios::binary);
        if (!f) {
          failed_flag[i] = 1;
          return;
        }
        filebuf.assign(std::istreambuf_iterator<char>(f), std::istreambuf_iterator<char>());
        p = reinterpret_cast<const unsigned char *>(filebuf.data());
        n = filebuf.size();
      }
      if (n < 4 || p[0] != 0xFF || p[1] != 0xD8) {  // not a JPEG (PNG, ...): Pillow path
        failed_flag[i] = 1;
        return;
      }
      const int r = it.row;
      int rc = DecodeCrop(J, p, n, cfg, it.seed, out + static_cast<size_t>(r) * img_bytes, prm + 4 * r, cm + 2 * r,
                          rowbuf);
      if (rc != 0) failed_flag[i] = 1;
    };
    {
      std::lock_guard<std::mutex> lk(mu_);
      job_ = work;
      njobs_ = items.size();
      next_.store(0);
      active_ = static_cast<int>(threads_.size());
      ++gen_;
    }
    cv_.notify_all();
    Drain();
    {
      std::unique_lock<std::mutex> lk(mu_);
      done_cv_.wait(lk, [this] { return active_ == 0; });
      job_ = nullptr;
    }
    std::vector<int> failed;
    for (size_t i = 0; i < items.size(); ++i)
      if (failed_flag[i]) failed.push_back(items[i].row);
    return failed;
  }

 private:
  void Drain() {
    std::vector<unsigned char> rowbuf;
    std::string filebuf;
    for (;;) {
      const size_t i = next_.fetch_add(1);
      if (i >= njobs_) break;
      job_(i, rowbuf, filebuf);
    }
  }
  void Loop() {
    uint64_t seen = 0;
    for (;;) {
      {
        std::unique_lock<std::mutex> lk(mu_);
        cv_.wait(lk, [&] { return stop_ || gen_ != seen; });
        if (stop_) return;
        seen = gen_;
      }
      Drain();
      {
        std::lock_guard<std::mutex> lk(mu_);
        if (--active_ == 0) done_cv_.notify_all();
      }
    }
  }

  std::vector<std::thread> threads_;
  std::mutex mu_;
  std::condition_variable cv_, done_cv_;
  std::function<void(size_t, std::vector<unsigned char> &, std::string &)> job_;
  size_t njobs_ = 0;
  std::atomic<size_t> next_{0};
  int active_ = 0;
  uint64_t gen_ = 0;
  bool stop_ = false;
};

}  // namespace cxxnet_rt
