// veles_infer - command-line front end of the native runtime:
//   veles_infer <package.zip|.tgz> <input.npy> <output.npy> [--gpu]
//               [--threads N] [--graph] [--repeat R]
// (reference: libVeles has no CLI; this stands in for its sample driver).
#include <algorithm>
#include <cstdio>
#include <cstdlib>
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
    std::fprintf(stderr,
                 "usage: %s package input.npy output.npy [--gpu] "
                 "[--threads N] [--graph] [--repeat R]\n",
                 argv[0]);
    return 2;
  }
  (void)veles_rt::veles_rt_units_anchor;
  bool gpu = false, graph = false;
  int threads = 0, repeat = 1;
  for (int i = 4; i < argc; ++i) {
    if (!std::strcmp(argv[i], "--gpu")) gpu = true;
    else if (!std::strcmp(argv[i], "--graph")) graph = true;
    else if (!std::strcmp(argv[i], "--threads") && i + 1 < argc)
      threads = std::atoi(argv[++i]);
    else if (!std::strcmp(argv[i], "--repeat") && i + 1 < argc)
      repeat = std::max(1, std::atoi(argv[++i]));
  }
  try {
    auto wf = veles_rt::LoadWorkflow(argv[1]);
    auto in = veles_rt::ParseNpy(veles_rt::ReadFile(argv[2]));
    if (threads > 0) wf->SetEngine(veles_rt::MakeThreadPoolEngine(threads));
    wf->EnableGraph(graph);
    wf->Initialize(in.shape, gpu);
    std::vector<float> out;
    for (int r = 0; r < repeat; ++r) out = wf->Run(in.data);
    veles_rt::NpyArray o;
    o.shape = wf->OutputShape();
    o.data = std::move(out);
    auto bytes = veles_rt::WriteNpy(o);
    std::ofstream f(argv[3], std::ios::binary);
    f.write((const char*)bytes.data(), bytes.size());
    std::cout << wf->name << ": " << wf->units.size() << " units, arena "
              << wf->ArenaBytes() << " bytes, " << wf->NumStreams()
              << " stream(s)" << (wf->GraphActive() ? ", hipGraph" : "")
              << ", output";
    for (auto s : o.shape) std::cout << " " << s;
    std::cout << std::endl;
  } catch (const std::exception& e) {
    std::fprintf(stderr, "error: %s\n", e.what());
    return 1;
  }
  return 0;
}
