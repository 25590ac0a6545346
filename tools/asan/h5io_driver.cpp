// AddressSanitizer / UBSan driver for the native HDF5 layer (csrc/h5ad/h5io.cpp).
// The executable itself links the sanitizer runtimes and embeds Python, so the
// sanitized _h5io module can be exercised by an ordinary Python round-trip script
// without preloading anything (host code only: GPU sanitizers are not used here).
#include <pybind11/embed.h>

#include <cstdio>
#include <string>

namespace py = pybind11;

int main(int argc, char** argv) {
  if (argc < 3) {
    std::fprintf(stderr, "usage: %s <module_dir> <script.py>\n", argv[0]);
    return 2;
  }
  py::scoped_interpreter guard{};
  try {
    py::module_::import("sys").attr("path").attr("insert")(0, std::string(argv[1]));
    py::eval_file(argv[2]);
  } catch (const std::exception& e) {
    std::fprintf(stderr, "driver: %s\n", e.what());
    return 1;
  }
  return 0;
}
