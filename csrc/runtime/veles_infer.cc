// veles_infer - command-line front end of the native runtime:
//   veles_infer <package.zip|.tgz> <input.npy> <output.npy> [--gpu]
// (reference: libVeles has no CLI; this stands in for its sample driver).
#include <cstdio>
#include <cstring>
#include <fstream>
#include <iostream>

#include "npy.h"
#include "runtime.h"

namespace veles_rt {
extern int veles_rt_units_anchor;
}

int main(int argc, char** argv) {
  if (argc < 4) {
    std::fprintf(stderr, "usage: %s package input.npy output.npy [--gpu]\n",
                 argv[0]);
    return 2;
  }
  (void)veles_rt::veles_rt_units_anchor;
  bool gpu = argc > 4 && std::strcmp(argv[4], "--gpu") == 0;
  try {
    auto wf = veles_rt::LoadWorkflow(argv[1]);
    auto in = veles_rt::ParseNpy(veles_rt::ReadFile(argv[2]));
    wf->Initialize(in.shape, gpu);
    auto out = wf->Run(in.data);
    veles_rt::NpyArray o;
    o.shape = wf->OutputShape();
    o.data = std::move(out);
    auto bytes = veles_rt::WriteNpy(o);
    std::ofstream f(argv[3], std::ios::binary);
    f.write((const char*)bytes.data(), bytes.size());
    std::cout << wf->name << ": " << wf->units.size() << " units, arena "
              << wf->ArenaBytes() << " bytes, output";
    for (auto s : o.shape) std::cout << " " << s;
    std::cout << std::endl;
  } catch (const std::exception& e) {
    std::fprintf(stderr, "error: %s\n", e.what());
    return 1;
  }
  return 0;
}
