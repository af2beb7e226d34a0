// runtime.h - veles_amd native inference runtime (the libVeles equivalent).
//
// Reference: libVeles/inc/veles/{unit,workflow,engine,unit_factory,
// workflow_loader}.h and src/*.cc.  A package written by
// Workflow.package_export() (contents.json + NNNN_AxB.npy in a zip / tgz) is
// loaded into a DAG of units; outputs live in ONE arena planned by
// MemoryOptimizer; units execute on the CPU (float32 reference loops) or on
// an MI355X through the same hand-written HIP kernels as training
// (libhvk.so: MFMA GEMM / implicit-GEMM conv, pooling, LRN, softmax).
#pragma once
#include <hip/hip_runtime.h>

#include <functional>
#include <map>
#include <memory>
#include <mutex>
#include <condition_variable>
#include <string>
#include <vector>

#include "json.h"
#include "npy.h"

namespace veles_rt {

using Shape = std::vector<size_t>;
inline size_t numel(const Shape& s) {
  size_t n = 1;
  for (auto v : s) n *= v;
  return n;
}

struct ExecContext {
  bool gpu = false;
  hipStream_t stream = nullptr;
  // scratch (device): reused between units
  void* scratch = nullptr;
  size_t scratch_bytes = 0;
  void* Scratch(size_t bytes);
};

// A unit output / input: float32 host pointer (CPU) or bf16 device pointer
struct Tensor {
  Shape shape;
  void* data = nullptr;
};

class Unit {
 public:
  explicit Unit(const std::string& name) : name_(name) {}
  virtual ~Unit() = default;
  const std::string& Name() const { return name_; }
  virtual std::string Class() const = 0;
  // parameters from contents.json "data" (arrays resolved by the loader)
  virtual void SetParameter(const std::string& key, const Json& value,
                            const std::map<std::string, NpyArray>& arrays) {}
  virtual Shape OutputShape(const Shape& in) const = 0;
  virtual void Initialize(ExecContext& ctx) {}
  virtual void Execute(const Tensor& in, Tensor& out, ExecContext& ctx) = 0;

  std::vector<Unit*> children;
  std::vector<Unit*> parents;
  std::string registered_name;  // the package's class name

 protected:
  std::string name_;
};

using UnitFactoryFn = std::function<std::unique_ptr<Unit>(const std::string&)>;

// Meyers-singleton registry name -> constructor (libVeles unit_factory.h)
class UnitFactory {
 public:
  static UnitFactory& Instance();
  void Register(const std::string& cls, UnitFactoryFn fn) { map_[cls] = fn; }
  std::unique_ptr<Unit> Create(const std::string& cls,
                               const std::string& name) const;
  bool Has(const std::string& cls) const { return map_.count(cls) > 0; }
  std::vector<std::string> Names() const;

 private:
  std::map<std::string, UnitFactoryFn> map_;
};

struct RegisterUnit {
  RegisterUnit(const std::string& cls, UnitFactoryFn fn) {
    UnitFactory::Instance().Register(cls, fn);
  }
};
#define VELES_RT_CAT2(a, b) a##b
#define VELES_RT_CAT(a, b) VELES_RT_CAT2(a, b)
#define VELES_REGISTER_UNIT(CLS, NAME)                                   \
  static ::veles_rt::RegisterUnit VELES_RT_CAT(veles_reg_, __LINE__)(    \
      NAME, [](const std::string& n) {                                   \
        return std::unique_ptr<::veles_rt::Unit>(new CLS(n));            \
      })

// Scheduling (libVeles engine.h:43-60): Schedule() runs a callable,
// Finish() signals the end of one workflow pass.
class Engine {
 public:
  virtual ~Engine() = default;
  virtual void Schedule(std::function<void()> fn) = 0;
  virtual void Wait() = 0;
};
std::unique_ptr<Engine> MakeSerialEngine();
std::unique_ptr<Engine> MakeThreadPoolEngine(size_t threads);

class Workflow {
 public:
  Workflow() = default;
  ~Workflow();
  std::string name, checksum;
  std::vector<std::unique_ptr<Unit>> units;  // topological order
  // plan the arena for a batch and initialise every unit
  void Initialize(const Shape& input_shape, bool gpu);
  // input: host float32 [batch, ...]; output copied to host float32
  std::vector<float> Run(const std::vector<float>& input);
  const Shape& OutputShape() const { return out_shape_; }
  size_t ArenaBytes() const { return arena_bytes_; }
  bool gpu() const { return ctx_.gpu; }

 private:
  ExecContext ctx_;
  std::vector<Shape> shapes_;    // per unit output
  std::vector<size_t> offsets_;  // per unit output (bytes) in the arena
  size_t arena_bytes_ = 0;
  void* arena_ = nullptr;        // host or device
  void* in_dev_ = nullptr;
  Shape in_shape_, out_shape_;
  std::vector<float> host_arena_;
};

// Build a workflow from a package (zip / tar / tar.gz)
std::unique_ptr<Workflow> LoadWorkflow(const std::string& path);
std::unique_ptr<Workflow> LoadWorkflowFromMemory(const Bytes& data);

bool GpuAvailable();

}  // namespace veles_rt
