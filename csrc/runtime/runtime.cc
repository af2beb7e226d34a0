#include "runtime.h"

#include <algorithm>
#include <cstring>
#include <stdexcept>

#include "../kernels/hvk_api.h"
#include "memory_optimizer.h"
#include "thread_pool.h"

namespace veles_rt {

#define HIPCHECK(x)                                                     \
  do {                                                                  \
    hipError_t e_ = (x);                                                \
    if (e_ != hipSuccess)                                               \
      throw std::runtime_error(std::string("HIP: ") + hipGetErrorString(e_)); \
  } while (0)

bool GpuAvailable() {
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess) return false;
  return n > 0;
}

void* ExecContext::Scratch(size_t bytes) {
  if (bytes > scratch_bytes) {
    if (scratch) {
      if (gpu) (void)hipFree(scratch);
      else std::free(scratch);
    }
    if (gpu) HIPCHECK(hipMalloc(&scratch, bytes));
    else scratch = std::malloc(bytes);
    scratch_bytes = bytes;
  }
  return scratch;
}

UnitFactory& UnitFactory::Instance() {
  static UnitFactory f;
  return f;
}

std::unique_ptr<Unit> UnitFactory::Create(const std::string& cls,
                                          const std::string& name) const {
  auto it = map_.find(cls);
  if (it == map_.end()) throw std::runtime_error("no unit class " + cls);
  return it->second(name);
}

std::vector<std::string> UnitFactory::Names() const {
  std::vector<std::string> v;
  for (auto& kv : map_) v.push_back(kv.first);
  return v;
}

namespace {
class SerialEngine : public Engine {
 public:
  void Schedule(std::function<void()> fn) override { fn(); }
  void Wait() override {}
};
class PoolEngine : public Engine {
 public:
  explicit PoolEngine(size_t n) : pool_(n) {}
  void Schedule(std::function<void()> fn) override {
    std::lock_guard<std::mutex> lk(mu_);
    futs_.push_back(pool_.Enqueue(std::move(fn)));
  }
  // Tasks may schedule children (a unit fires its successors): drain until
  // no task scheduled while waiting is left, or Wait() could return while a
  // child is still queued.
  void Wait() override {
    while (true) {
      std::vector<std::future<void>> f;
      {
        std::lock_guard<std::mutex> lk(mu_);
        f.swap(futs_);
      }
      if (f.empty()) return;
      for (auto& x : f) x.get();
    }
  }

 private:
  ThreadPool pool_;
  std::mutex mu_;
  std::vector<std::future<void>> futs_;
};
}  // namespace

std::unique_ptr<Engine> MakeSerialEngine() {
  return std::unique_ptr<Engine>(new SerialEngine());
}
std::unique_ptr<Engine> MakeThreadPoolEngine(size_t n) {
  return std::unique_ptr<Engine>(new PoolEngine(n));
}

Workflow::~Workflow() {
  if (ctx_.gpu) {
    if (arena_) (void)hipFree(arena_);
    if (in_dev_) (void)hipFree(in_dev_);
    if (ctx_.scratch) (void)hipFree(ctx_.scratch);
    if (ctx_.stream) (void)hipStreamDestroy(ctx_.stream);
  } else if (ctx_.scratch) {
    std::free(ctx_.scratch);
  }
}

void Workflow::Initialize(const Shape& input_shape, bool gpu) {
  if (arena_ && ctx_.gpu) HIPCHECK(hipFree(arena_));
  if (in_dev_) HIPCHECK(hipFree(in_dev_));
  arena_ = in_dev_ = nullptr;
  ctx_.gpu = gpu && GpuAvailable();
  if (ctx_.gpu && !ctx_.stream) HIPCHECK(hipStreamCreate(&ctx_.stream));
  in_shape_ = input_shape;
  const size_t esz = ctx_.gpu ? 2 : 4;  // bf16 on the device, f32 on host
  shapes_.clear();
  Shape s = input_shape;
  std::vector<MemoryNode> nodes(units.size());
  // unit i runs at time i; its output lives until its last consumer runs
  std::map<Unit*, int> index;
  for (size_t i = 0; i < units.size(); ++i) index[units[i].get()] = (int)i;
  for (size_t i = 0; i < units.size(); ++i) {
    Unit* u = units[i].get();
    Shape in = u->parents.empty() ? input_shape
                                  : shapes_[index[u->parents.front()]];
    s = u->OutputShape(in);
    shapes_.push_back(s);
    int last = (int)i + 1;
    for (Unit* c : u->children) last = std::max(last, index[c] + 1);
    if (u->children.empty()) last = (int)units.size() + 1;  // the output
    nodes[i].time_start = (int)i;
    nodes[i].time_finish = last;
    nodes[i].value = (numel(s) * esz + 255) / 256 * 256;
  }
  out_shape_ = shapes_.empty() ? input_shape : shapes_.back();
  arena_bytes_ = MemoryOptimizer().Optimize(&nodes);
  offsets_.resize(units.size());
  for (size_t i = 0; i < units.size(); ++i) offsets_[i] = nodes[i].position;
  if (ctx_.gpu) {
    HIPCHECK(hipMalloc(&arena_, std::max<size_t>(arena_bytes_, 256)));
    HIPCHECK(hipMalloc(&in_dev_, numel(input_shape) * 6 + 256));
  } else {
    host_arena_.assign(arena_bytes_ / 4 + 64, 0.f);
    arena_ = host_arena_.data();
  }
  for (auto& u : units) u->Initialize(ctx_);
}

std::vector<float> Workflow::Run(const std::vector<float>& input) {
  if (input.size() != numel(in_shape_))
    throw std::runtime_error("input size mismatch");
  Tensor in;
  in.shape = in_shape_;
  if (ctx_.gpu) {
    float* f32 = (float*)in_dev_;
    uint16_t* bf = (uint16_t*)((char*)in_dev_ + numel(in_shape_) * 4);
    HIPCHECK(hipMemcpyAsync(f32, input.data(), input.size() * 4,
                            hipMemcpyHostToDevice, ctx_.stream));
    hvk_cast(f32, HVK_F32, bf, HVK_BF16, (long long)input.size(), 1.f,
             ctx_.stream);
    in.data = bf;
  } else {
    in.data = const_cast<float*>(input.data());
  }
  std::map<Unit*, size_t> index;
  for (size_t i = 0; i < units.size(); ++i) index[units[i].get()] = i;
  std::vector<Tensor> outs(units.size());
  for (size_t i = 0; i < units.size(); ++i) {
    Unit* u = units[i].get();
    const Tensor& src = u->parents.empty() ? in : outs[index[u->parents.front()]];
    outs[i].shape = shapes_[i];
    outs[i].data = (char*)arena_ + offsets_[i];
    u->Execute(src, outs[i], ctx_);
  }
  const Tensor& last = outs.empty() ? in : outs.back();
  std::vector<float> result(numel(last.shape));
  if (ctx_.gpu) {
    float* tmp = (float*)ctx_.Scratch(result.size() * 4 + 256);
    hvk_cast(last.data, HVK_BF16, tmp, HVK_F32, (long long)result.size(), 1.f,
             ctx_.stream);
    HIPCHECK(hipMemcpyAsync(result.data(), tmp, result.size() * 4,
                            hipMemcpyDeviceToHost, ctx_.stream));
    HIPCHECK(hipStreamSynchronize(ctx_.stream));
  } else {
    std::memcpy(result.data(), last.data, result.size() * 4);
  }
  return result;
}

// ------------------------------------------------------------------ loader
static std::unique_ptr<Workflow> Build(const WorkflowArchive& ar) {
  Json c = Json::parse(ar.Text("contents.json"));
  auto wf = std::unique_ptr<Workflow>(new Workflow());
  wf->name = c.has("workflow") ? c["workflow"].str : "";
  wf->checksum = c.has("checksum") ? c["checksum"].str : "";
  std::map<std::string, NpyArray> arrays;
  for (auto& n : ar.Names()) {
    if (n.size() > 4 && n.substr(n.size() - 4) == ".npy")
      arrays["@" + n.substr(0, n.size() - 4)] = ParseNpy(ar.Get(n));
  }
  const Json& us = c["units"];
  std::vector<std::unique_ptr<Unit>> created;
  for (size_t i = 0; i < us.size(); ++i) {
    const Json& u = us[i];
    std::string cls = u["class"]["name"].str;
    auto unit = UnitFactory::Instance().Create(cls, cls + "_" + std::to_string(i));
    unit->registered_name = cls;
    if (u.has("data"))
      for (auto& kv : u["data"].obj) unit->SetParameter(kv.first, kv.second, arrays);
    created.push_back(std::move(unit));
  }
  for (size_t i = 0; i < us.size(); ++i) {
    const Json& links = us[i]["links"];
    for (size_t j = 0; j < links.size(); ++j) {
      size_t dst = (size_t)links[j].num;
      created[i]->children.push_back(created.at(dst).get());
      created[dst]->parents.push_back(created[i].get());
    }
  }
  // topological order (Kahn), the head is the unit without parents
  std::map<Unit*, int> indeg;
  for (auto& u : created) indeg[u.get()] = (int)u->parents.size();
  std::vector<Unit*> order, ready;
  for (auto& u : created)
    if (u->parents.empty()) ready.push_back(u.get());
  while (!ready.empty()) {
    Unit* u = ready.front();
    ready.erase(ready.begin());
    order.push_back(u);
    for (Unit* c2 : u->children)
      if (--indeg[c2] == 0) ready.push_back(c2);
  }
  if (order.size() != created.size())
    throw std::runtime_error("package graph has a cycle");
  for (Unit* u : order)
    for (auto& p : created)
      if (p.get() == u) wf->units.push_back(std::move(p));
  return wf;
}

std::unique_ptr<Workflow> LoadWorkflow(const std::string& path) {
  return Build(WorkflowArchive::Load(path));
}

std::unique_ptr<Workflow> LoadWorkflowFromMemory(const Bytes& data) {
  return Build(WorkflowArchive::FromMemory(data, ""));
}

}  // namespace veles_rt
