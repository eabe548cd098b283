// im2bin: pack the images named by a list file into 64 MB BinaryPages -- a native executable with
// the reference tool's command line and output (tools/im2bin.cpp:6-67):
//
//   im2bin image.lst image_root_dir output.bin
//
// Every list line is `index <tab> label... <tab> path`; the file at image_root_dir + path is
// appended, as its raw encoded bytes, to the current page, and a full page is flushed
// (cxxnet_rt::PackImageBin, csrc/runtime/data_io.h, the same packer the Python tool and the
// pybind11 module use).  Built by cxxnet_amd/build.py into cxxnet_amd/_native/im2bin.
#include <chrono>
#include <cstdio>

#include "../runtime/data_io.h"

int main(int argc, char *argv[]) {
  if (argc != 4) {
    std::fprintf(stderr, "Usage: im2bin image.lst image_root_dir output_file\n");
    return 255;
  }
  const auto t0 = std::chrono::steady_clock::now();
  std::printf("create image binary pack from %s, this will take some time...\n", argv[1]);
  try {
    const std::vector<cxxnet_rt::ImageListEntry> entries = cxxnet_rt::ParseImageList(argv[1], 1);
    std::vector<std::string> files;
    files.reserve(entries.size());
    const std::string root = argv[2];
    for (const auto &e : entries) files.push_back(root + e.path);
    const size_t npages = cxxnet_rt::PackImageBin(files, argv[3]);
    const double sec = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    std::printf("finished [%8zu] images processed to %zu pages, %d sec elapsed\n", files.size(), npages,
                static_cast<int>(sec));
  } catch (const std::exception &ex) {
    std::fprintf(stderr, "im2bin: %s\n", ex.what());
    return 1;
  }
  return 0;
}
