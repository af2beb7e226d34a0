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

#include <atomic>
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
  // several parents (in ``parents`` order): units that join branches
  // override these; single-input units see their first parent only
  virtual Shape OutputShapeN(const std::vector<Shape>& ins) const {
    return OutputShape(ins.at(0));
  }
  virtual void Initialize(ExecContext& ctx) {}
  virtual void Execute(const Tensor& in, Tensor& out, ExecContext& ctx) = 0;
  virtual void ExecuteN(const std::vector<const Tensor*>& ins, Tensor& out,
                        ExecContext& ctx) {
    Execute(*ins.at(0), out, ctx);
  }

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

// A DAG of units with one planned arena.  Run() drives the units through
// an Engine the way libVeles does (unit.cc:60-76, workflow.cc:91-107): the
// heads are scheduled, each finished unit schedules every child whose
// parents have all finished, and the pass ends when every unit ran.  On an
// MI355X each branch of the graph enqueues on its own HIP stream (a child
// continues its first parent's stream if it is that parent's first child,
// else it starts a new one) and waits on its other parents' events, so
// independent branches overlap on the device; optionally the whole pass is
// captured once into a hipGraph and replayed (EnableGraph).
class Workflow {
 public:
  Workflow();
  ~Workflow();
  std::string name, checksum;
  std::vector<std::unique_ptr<Unit>> units;  // topological order
  // the scheduler (default: serial); MakeThreadPoolEngine(n) enqueues
  // independent branches from n host threads
  void SetEngine(std::unique_ptr<Engine> e) { engine_ = std::move(e); }
  // capture the unit pass into a hipGraph on the 2nd Run and replay it
  // from the 3rd (GPU only; the 1st run is eager: lazy allocations)
  void EnableGraph(bool on) { use_graph_ = on; graph_runs_ = 0; }
  bool GraphActive() const { return graph_exec_ != nullptr; }
  // plan the arena for a batch and initialise every unit
  void Initialize(const Shape& input_shape, bool gpu);
  // input: host float32 [batch, ...]; output (the sink unit's) on the host
  std::vector<float> Run(const std::vector<float>& input);
  const Shape& OutputShape() const { return out_shape_; }
  size_t ArenaBytes() const { return arena_bytes_; }
  bool gpu() const { return ctx_.gpu; }
  int NumStreams() const { return (int)streams_.size(); }
  int StreamOf(size_t unit) const { return stream_of_[unit]; }
  // execution order of the last Run (unit indices, as units finished)
  std::vector<int> LastOrder() const;
  // [start, finish) of unit i's output in the planning timeline
  std::pair<int, int> Lifetime(size_t i) const { return life_[i]; }
  size_t Offset(size_t i) const { return offsets_[i]; }

 private:
  void Enqueue(size_t i, const Tensor& in);
  void RunPass(const Tensor& in);
  void ReleaseGraph();
  ExecContext ctx_;
  std::unique_ptr<Engine> engine_;
  std::vector<Shape> shapes_;    // per unit output
  std::vector<size_t> offsets_;  // per unit output (bytes) in the arena
  std::vector<std::pair<int, int>> life_;
  std::vector<std::vector<size_t>> parent_idx_, child_idx_;
  std::vector<int> stream_of_;
  std::vector<hipStream_t> streams_;      // [0] = ctx_.stream
  std::vector<ExecContext> stream_ctx_;   // per stream: own scratch
  std::vector<hipEvent_t> done_;          // per unit (GPU)
  hipEvent_t start_ev_ = nullptr;
  std::vector<Tensor> outs_;
  std::vector<std::atomic<int>*> pending_;
  std::mutex order_mu_;
  std::vector<int> order_;
  size_t arena_bytes_ = 0;
  void* arena_ = nullptr;        // host or device
  void* in_dev_ = nullptr;
  Shape in_shape_, out_shape_;
  std::vector<float> host_arena_;
  bool use_graph_ = false;
  int graph_runs_ = 0;
  hipGraphExec_t graph_exec_ = nullptr;
  const void* graph_in_ = nullptr;
};

// Build a workflow from a package (zip / tar / tar.gz)
std::unique_ptr<Workflow> LoadWorkflow(const std::string& path);
std::unique_ptr<Workflow> LoadWorkflowFromMemory(const Bytes& data);

bool GpuAvailable();

}  // namespace veles_rt
