// capi.cc - C ABI of the native runtime (loaded by veles_amd.runtime via
// ctypes, and by C/C++ serving code).  Errors are reported through
// vr_last_error(); every call returns 0 on success.
#include <cstring>
#include <sstream>
#include <string>

#include "memory_optimizer.h"
#include "runtime.h"

namespace veles_rt {
extern int veles_rt_units_anchor;
}

namespace {
thread_local std::string g_err;
}

#define VR_TRY(body)                 \
  try {                              \
    body;                            \
    return 0;                        \
  } catch (const std::exception& e) { \
    g_err = e.what();                \
    return -1;                       \
  }

extern "C" {

const char* vr_last_error() { return g_err.c_str(); }

int vr_gpu_available() { return veles_rt::GpuAvailable() ? 1 : 0; }

int vr_load(const char* path, void** handle) {
  (void)veles_rt::veles_rt_units_anchor;
  VR_TRY(*handle = veles_rt::LoadWorkflow(path).release());
}

void vr_free(void* h) { delete static_cast<veles_rt::Workflow*>(h); }

int vr_num_units(void* h) {
  return (int)static_cast<veles_rt::Workflow*>(h)->units.size();
}

const char* vr_unit_class(void* h, int i) {
  static thread_local std::string s;
  auto& u = static_cast<veles_rt::Workflow*>(h)->units[i];
  s = u->registered_name.empty() ? u->Class() : u->registered_name;
  return s.c_str();
}

// threads > 0: a thread-pool Engine (independent branches enqueue from
// several host threads); 0: the serial engine
int vr_set_engine(void* h, int threads) {
  VR_TRY({
    auto* wf = static_cast<veles_rt::Workflow*>(h);
    wf->SetEngine(threads > 0 ? veles_rt::MakeThreadPoolEngine(threads)
                              : veles_rt::MakeSerialEngine());
  });
}

// 1: capture the GPU pass into a hipGraph (2nd run) and replay it
int vr_enable_graph(void* h, int on) {
  VR_TRY(static_cast<veles_rt::Workflow*>(h)->EnableGraph(on != 0));
}

int vr_graph_active(void* h) {
  return static_cast<veles_rt::Workflow*>(h)->GraphActive() ? 1 : 0;
}

int vr_num_streams(void* h) {
  return static_cast<veles_rt::Workflow*>(h)->NumStreams();
}

// input_shape: ndim sizes (batch first); gpu: 1 = run through libhvk
int vr_initialize(void* h, const long long* shape, int ndim, int gpu) {
  VR_TRY({
    veles_rt::Shape s(shape, shape + ndim);
    static_cast<veles_rt::Workflow*>(h)->Initialize(s, gpu != 0);
  });
}

int vr_output_shape(void* h, long long* shape, int* ndim) {
  auto& s = static_cast<veles_rt::Workflow*>(h)->OutputShape();
  *ndim = (int)s.size();
  for (size_t i = 0; i < s.size(); ++i) shape[i] = (long long)s[i];
  return 0;
}

long long vr_arena_bytes(void* h) {
  return (long long)static_cast<veles_rt::Workflow*>(h)->ArenaBytes();
}

int vr_run(void* h, const float* input, long long n_in, float* output,
           long long n_out) {
  VR_TRY({
    auto* wf = static_cast<veles_rt::Workflow*>(h);
    std::vector<float> in(input, input + n_in);
    auto out = wf->Run(in);
    if ((long long)out.size() != n_out)
      throw std::runtime_error("output size mismatch");
    std::memcpy(output, out.data(), out.size() * 4);
  });
}

// MemoryOptimizer exposed for tests: nodes = [start, finish, size] * n
long long vr_optimize_memory(const long long* nodes, int n,
                             long long* positions) {
  std::vector<veles_rt::MemoryNode> v(n);
  for (int i = 0; i < n; ++i) {
    v[i].time_start = (int)nodes[3 * i];
    v[i].time_finish = (int)nodes[3 * i + 1];
    v[i].value = (size_t)nodes[3 * i + 2];
  }
  size_t h = veles_rt::MemoryOptimizer().Optimize(&v);
  for (int i = 0; i < n; ++i) positions[i] = (long long)v[i].position;
  return (long long)h;
}

}  // extern "C"
