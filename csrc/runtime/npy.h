// npy.h - .npy parser into float32 (reference: NumpyArrayLoader,
// libVeles/inc/veles/numpy_array_loader.h; header parse, f16/f64/int
// conversion, Fortran-order transpose by cycle following).
#pragma once
#include <cstdint>
#include <string>
#include <vector>

#include "archive.h"

namespace veles_rt {

struct NpyArray {
  std::vector<size_t> shape;
  std::vector<float> data;
  size_t size() const {
    size_t n = 1;
    for (auto s : shape) n *= s;
    return n;
  }
};

NpyArray ParseNpy(const Bytes& bytes);
Bytes WriteNpy(const NpyArray& a);  // float32, C order
float HalfToFloat(uint16_t h);

}  // namespace veles_rt
