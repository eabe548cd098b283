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
#include <utility>
#include <vector>

namespace cxxnet_rt {
namespace jpg {

// ---- libjpeg v8 ABI (jpeglib.h / jmorecfg.h of libjpeg-turbo, JPEG_LIB_VERSION 80) --------
typedef int boolean_t;
typedef unsigned int JDIMENSION;
typedef unsigned char JSAMPLE;
typedef JSAMPLE *JSAMPROW;
typedef JSAMPROW *JSAMPARRAY;
enum { JCS_GRAYSCALE = 1, JCS_RGB = 2, JCS_YCbCr = 3, JDCT_ISLOW = 0, JPEG_LIB_VERSION = 80 };
struct jpeg_common_struct;
typedef jpeg_common_struct *j_common_ptr;
typedef short JCOEF;
typedef JCOEF JBLOCK[64];  // one 8x8 block of quantised coefficients, natural (row-major) order
typedef JBLOCK *JBLOCKROW;
typedef JBLOCKROW *JBLOCKARRAY;
struct jvirt_barray_control;
typedef jvirt_barray_control *jvirt_barray_ptr;

// the memory manager's method table (only access_virt_barray is called)
struct jpeg_memory_mgr {
  void *alloc_small, *alloc_large, *alloc_sarray, *alloc_barray, *request_virt_sarray, *request_virt_barray,
      *realize_virt_arrays, *access_virt_sarray;
  JBLOCKARRAY (*access_virt_barray)(j_common_ptr, jvirt_barray_ptr, JDIMENSION start_row, JDIMENSION num_rows,
                                    int writable);
};

struct JQUANT_TBL {
  unsigned short quantval[64];  // natural order
  int sent_table;
};

struct jpeg_component_info {
  int component_id, component_index, h_samp_factor, v_samp_factor, quant_tbl_no, dc_tbl_no, ac_tbl_no;
  JDIMENSION width_in_blocks, height_in_blocks;
  int DCT_h_scaled_size, DCT_v_scaled_size;
  JDIMENSION downsampled_width, downsampled_height;
  int component_needed;
  int MCU_width, MCU_height, MCU_blocks, MCU_sample_width, last_col_width, last_row_height;
  JQUANT_TBL *quant_table;
  void *dct_table;
};
static_assert(sizeof(jpeg_component_info) == 96, "libjpeg v8 jpeg_component_info layout");

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
  jvirt_barray_ptr *(*read_coefficients)(jpeg_decompress_struct *) = nullptr;
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
    sym(read_coefficients, "jpeg_read_coefficients");
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

// The crop / mirror / contrast / illumination draws of io/augment.py _augment_one, in its order,
// from the record's own generator.  False if the crop does not fit the H x W image.
inline bool DrawCrop(int H, int W, const CropConfig &c, uint64_t seed, int *py, int *px, bool *pmirror,
                     float *pcontrast, float *pillum) {
  using namespace jpg;
  const int ch = c.out_h, cw = c.out_w;
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
  if (yy < 0 || xx < 0 || yy + ch > H || xx + cw > W) return false;
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
  *py = yy;
  *px = xx;
  *pmirror = mirror;
  *pcontrast = contrast;
  *pillum = illum;
  return true;
}

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
  int yy, xx;
  bool mirror;
  float contrast, illum;
  if (!DrawCrop(H, W, c, seed, &yy, &xx, &mirror, &contrast, &illum)) {
    J.destroy_decompress(&cinfo);
    return -2;
  }
  J.start_decompress(&cinfo);
  if (cinfo.output_components != 3) {
    J.abort_decompress(&cinfo);
    J.destroy_decompress(&cinfo);
    return -1;
  }
  // crop_scanline aligns the window's left edge down to an iMCU boundary but keeps its right
  // edge where asked, and the fancy upsampler treats both window edges as the image border:
  // ask for one column more on the left (a crop starting on an iMCU boundary then starts one
  // iMCU earlier) and up to 16 more on the right, so the crop's edge columns keep their
  // chroma context (bit-identical to a full decode then; without the margins an edge column
  // differs by a few levels on subsampled images)
  JDIMENSION x0 = static_cast<JDIMENSION>(xx > 0 ? xx - 1 : 0);
  JDIMENSION wd = static_cast<JDIMENSION>(std::min(xx + cw + 16, W)) - x0;
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

// ---- GPU decode stage: entropy decode here, everything after it on the GPU ------------------
//
// The host keeps only the serial part of JPEG decoding (Huffman / arithmetic decoding of the
// coefficients: jpeg_read_coefficients); dequantisation, the islow IDCT, the fancy chroma
// upsampling, YCbCr->RGB, crop and mirror run in ops/jpeg_kernels.hip over the whole batch.
// Per record only the coefficient blocks of the crop window (plus the one chroma sample of
// upsampling context on each side) are staged, so a large photo costs what a 256px one does.
//
// Staging layout (one batch): coef int16 [cap][64] blocks packed by an atomic cursor (the
// order between records depends on the threads; every record finds its blocks through its
// window table, so the decoded batch does not), bwin int32 [cap] window id of each block
// (row * 3 + component), meta int32 [B][3][kCoefMeta] window tables (layout below).
constexpr int kCoefMeta = 80;
enum CoefMetaField {
  kBlk0 = 0,    // first block of the window in coef
  kBw = 1,      // window width / height in blocks
  kBh = 2,
  kBy0 = 3,     // window origin in the component's block grid
  kBx0 = 4,
  kDw = 5,      // component's real sample width / height (libjpeg downsampled_width / _height)
  kDh = 6,
  kRh = 7,      // horizontal / vertical expansion to the luma grid (1 or 2)
  kRv = 8,
  kNcomp = 9,   // 1 (grayscale) or 3 (YCbCr); same in the three windows of a record
  kValid = 10,  // 1: decoded here; 0: not this stage's row (padding / fallback / other rank)
  kQuant = 16,  // 64 dequantisation steps, natural order
};

struct CoefStage {
  int16_t *coef = nullptr;
  int32_t *bwin = nullptr;
  int32_t *meta = nullptr;
  long cap_blocks = 0;
  std::atomic<long> cursor{0};
};

// Entropy-decodes one record into the stage.  Returns 0, or -1 (not a layout the GPU stage
// handles: 12-bit, CMYK / RGB-coded, 4:4:0 or exotic sampling -> the CPU decoder), -2 (crop
// does not fit), -3 (stage full), or a libjpeg message code.
inline int ReadCoefCrop(const jpg::Api &J, const unsigned char *buf, size_t len, const CropConfig &c, uint64_t seed,
                        int row, CoefStage &st, int *prm, float *cm) {
  using namespace jpg;
  jpeg_decompress_struct cinfo;
  ErrMgr err;
  std::memset(&cinfo, 0, sizeof(cinfo));
  cinfo.err = J.std_error(&err.pub);
  err.pub.error_exit = on_error;
  err.pub.emit_message = on_message;
  err.code = 0;
  volatile bool created = false;
  if (setjmp(err.jb)) {
    if (created) J.destroy_decompress(&cinfo);
    return err.code > 0 ? err.code : -1;
  }
  J.create_decompress(&cinfo, JPEG_LIB_VERSION, sizeof(cinfo));
  created = true;
  J.mem_src(&cinfo, buf, static_cast<unsigned long>(len));
  J.read_header(&cinfo, 1);
  const int nc = cinfo.num_components;
  const jpeg_component_info *ci = static_cast<const jpeg_component_info *>(cinfo.comp_info);
  bool ok = cinfo.data_precision == 8 && ((nc == 3 && cinfo.jpeg_color_space == JCS_YCbCr) ||
                                          (nc == 1 && cinfo.jpeg_color_space == JCS_GRAYSCALE));
  const int mh = cinfo.max_h_samp_factor, mv = cinfo.max_v_samp_factor;
  for (int k = 0; ok && k < nc; ++k) {
    const int rh = mh / ci[k].h_samp_factor, rv = mv / ci[k].v_samp_factor;
    ok = ci[k].h_samp_factor * rh == mh && ci[k].v_samp_factor * rv == mv && rh <= 2 && rv <= rh &&
         (k > 0 || (rh == 1 && rv == 1));  // luma at full rate; chroma 4:4:4, 4:2:2 or 4:2:0
  }
  const int H = static_cast<int>(cinfo.image_height), W = static_cast<int>(cinfo.image_width);
  if (!ok) {
    J.destroy_decompress(&cinfo);
    return -1;
  }
  if (H < c.out_h || W < c.out_w) {
    J.destroy_decompress(&cinfo);
    return -2;
  }
  int yy, xx;
  bool mirror;
  float contrast, illum;
  if (!DrawCrop(H, W, c, seed, &yy, &xx, &mirror, &contrast, &illum)) {
    J.destroy_decompress(&cinfo);
    return -2;
  }
  jvirt_barray_ptr *arrays = J.read_coefficients(&cinfo);
  ci = static_cast<const jpeg_component_info *>(cinfo.comp_info);
  int win[3][6];  // by0, bx0, bw, bh, rh, rv
  long total = 0;
  for (int k = 0; k < nc; ++k) {
    const int rh = mh / ci[k].h_samp_factor, rv = mv / ci[k].v_samp_factor;
    const int dw = static_cast<int>(ci[k].downsampled_width), dh = static_cast<int>(ci[k].downsampled_height);
    // samples of this component the crop reads: the covered range, widened by the one
    // neighbour the triangle upsampling filter takes on each side
    int r0 = yy / rv, r1 = (yy + c.out_h - 1) / rv, c0 = xx / rh, c1 = (xx + c.out_w - 1) / rh;
    if (rv == 2) --r0, ++r1;
    if (rh == 2) --c0, ++c1;
    r0 = std::max(r0, 0), c0 = std::max(c0, 0), r1 = std::min(r1, dh - 1), c1 = std::min(c1, dw - 1);
    win[k][0] = r0 / 8, win[k][1] = c0 / 8, win[k][2] = c1 / 8 - c0 / 8 + 1, win[k][3] = r1 / 8 - r0 / 8 + 1;
    win[k][4] = rh, win[k][5] = rv;
    total += static_cast<long>(win[k][2]) * win[k][3];
  }
  const long blk0 = st.cursor.fetch_add(total);
  // the reserved blocks get a valid window id before anything can fail (stage full below, or a
  // libjpeg longjmp from access_virt_barray): a failed row keeps meta VALID = 0 and falls back
  // to the host decoder, but its blocks stay in the uploaded range and the IDCT reads their ids
  if (blk0 < st.cap_blocks) std::fill(st.bwin + blk0, st.bwin + std::min(blk0 + total, st.cap_blocks), row * 3);
  if (blk0 + total > st.cap_blocks) {
    J.abort_decompress(&cinfo);
    J.destroy_decompress(&cinfo);
    return -3;
  }
  jpeg_memory_mgr *mem = static_cast<jpeg_memory_mgr *>(cinfo.mem);
  long b = blk0;
  for (int k = 0; k < nc; ++k) {
    int32_t *m = st.meta + (static_cast<long>(row) * 3 + k) * kCoefMeta;
    m[kBlk0] = static_cast<int32_t>(b);
    m[kBw] = win[k][2], m[kBh] = win[k][3], m[kBy0] = win[k][0], m[kBx0] = win[k][1];
    m[kDw] = static_cast<int32_t>(ci[k].downsampled_width), m[kDh] = static_cast<int32_t>(ci[k].downsampled_height);
    m[kRh] = win[k][4], m[kRv] = win[k][5], m[kNcomp] = nc, m[kValid] = 1;
    for (int q = 0; q < 64; ++q) m[kQuant + q] = ci[k].quant_table->quantval[q];
    const size_t row_bytes = static_cast<size_t>(win[k][2]) * sizeof(JBLOCK);
    for (int by = 0; by < win[k][3]; ++by) {
      JBLOCKARRAY a = mem->access_virt_barray(reinterpret_cast<j_common_ptr>(&cinfo), arrays[k],
                                              static_cast<JDIMENSION>(win[k][0] + by), 1, 0);
      std::memcpy(st.coef + b * 64, a[0][win[k][1]], row_bytes);
      std::fill(st.bwin + b, st.bwin + b + win[k][2], row * 3 + k);
      b += win[k][2];
    }
  }
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
    Dispatch(items.size(), work);
    std::vector<int> failed;
    for (size_t i = 0; i < items.size(); ++i)
      if (failed_flag[i]) failed.push_back(items[i].row);
    return failed;
  }

  // The GPU stage's host half: every record's crop-window coefficients into the stage (see
  // ReadCoefCrop).  Rows it reports back (non-JPEG, layouts the GPU stage does not take, a full
  // stage) go through Run() instead.  Returns (failed rows, blocks used).
  std::pair<std::vector<int>, long> RunCoef(const std::vector<DecodeItem> &items, const CropConfig &cfg,
                                            CoefStage &st, int32_t *prm, float *cm) {
    const jpg::Api &J = jpg::api();
    if (!J.ok) throw std::runtime_error("native JPEG decoder unavailable: " + J.error);
    std::vector<int> failed_flag(items.size(), 0);
    st.cursor.store(0);
    auto work = [&](size_t i, std::vector<unsigned char> &, std::string &filebuf) {
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
      if (n < 4 || p[0] != 0xFF || p[1] != 0xD8) {
        failed_flag[i] = 1;
        return;
      }
      const int r = it.row;
      if (ReadCoefCrop(J, p, n, cfg, it.seed, r, st, prm + 4 * r, cm + 2 * r) != 0) {
        for (int k = 0; k < 3; ++k) st.meta[(static_cast<long>(r) * 3 + k) * kCoefMeta + kValid] = 0;
        failed_flag[i] = 1;
      }
    };
    Dispatch(items.size(), work);
    std::vector<int> failed;
    for (size_t i = 0; i < items.size(); ++i)
      if (failed_flag[i]) failed.push_back(items[i].row);
    return {failed, std::min(st.cursor.load(), st.cap_blocks)};
  }

 private:
  void Dispatch(size_t n, std::function<void(size_t, std::vector<unsigned char> &, std::string &)> work) {
    {
      std::lock_guard<std::mutex> lk(mu_);
      job_ = std::move(work);
      njobs_ = n;
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
  }

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
