#include <exception>
#include "runtime.h"

#include <algorithm>
#include <cstring>
#include <stdexcept>

#include "../kernels/hvk_api.h"
#include "logger.h"
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
  // child is still queued.  A task that throws does not stop the drain: the
  // remaining tasks reference the caller's stack (Run's input) and outputs,
  // so every one of them finishes before the first exception is rethrown.
  void Wait() override {
    std::exception_ptr first;
    while (true) {
      std::vector<std::future<void>> f;
      {
        std::lock_guard<std::mutex> lk(mu_);
        f.swap(futs_);
      }
      if (f.empty()) break;
      for (auto& x : f) {
        try {
          x.get();
        } catch (...) {
          if (!first) first = std::current_exception();
        }
      }
    }
    if (first) std::rethrow_exception(first);
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

namespace {
Logger g_log("workflow");
}

Workflow::Workflow() : engine_(MakeSerialEngine()) {}

void Workflow::ReleaseGraph() {
  if (graph_exec_) (void)hipGraphExecDestroy(graph_exec_);
  graph_exec_ = nullptr;
  graph_runs_ = 0;
}

static void FreeStreams(std::vector<hipStream_t>* streams,
                        std::vector<ExecContext>* ctxs) {
  for (size_t i = 0; i < ctxs->size(); ++i) {
    ExecContext& c = (*ctxs)[i];
    if (c.scratch) {
      if (c.gpu) (void)hipFree(c.scratch);
      else std::free(c.scratch);
    }
    if (i > 0 && i < streams->size()) (void)hipStreamDestroy((*streams)[i]);
  }
  ctxs->clear();
  streams->clear();
}

Workflow::~Workflow() {
  for (auto* p : pending_) delete p;
  FreeStreams(&streams_, &stream_ctx_);
  if (ctx_.gpu) {
    ReleaseGraph();
    for (auto e : done_) (void)hipEventDestroy(e);
    if (start_ev_) (void)hipEventDestroy(start_ev_);
    if (arena_) (void)hipFree(arena_);
    if (in_dev_) (void)hipFree(in_dev_);
    if (ctx_.scratch) (void)hipFree(ctx_.scratch);
    if (ctx_.stream) (void)hipStreamDestroy(ctx_.stream);
  } else if (ctx_.scratch) {
    std::free(ctx_.scratch);
  }
}

void Workflow::Initialize(const Shape& input_shape, bool gpu) {
  ReleaseGraph();
  if (arena_ && ctx_.gpu) HIPCHECK(hipFree(arena_));
  if (in_dev_) HIPCHECK(hipFree(in_dev_));
  arena_ = in_dev_ = nullptr;
  ctx_.gpu = gpu && GpuAvailable();
  if (ctx_.gpu && !ctx_.stream) HIPCHECK(hipStreamCreate(&ctx_.stream));
  in_shape_ = input_shape;
  const size_t n = units.size();
  const size_t esz = ctx_.gpu ? 2 : 4;  // bf16 on the device, f32 on host
  std::map<Unit*, size_t> index;
  for (size_t i = 0; i < n; ++i) index[units[i].get()] = i;
  parent_idx_.assign(n, {});
  child_idx_.assign(n, {});
  for (size_t i = 0; i < n; ++i) {
    for (Unit* p : units[i]->parents) parent_idx_[i].push_back(index.at(p));
    for (Unit* c : units[i]->children) child_idx_[i].push_back(index.at(c));
  }
  // ancestors / descendants (n is a few dozen units: bitsets by vectors)
  std::vector<std::vector<char>> anc(n, std::vector<char>(n, 0));
  for (size_t i = 0; i < n; ++i)
    for (size_t p : parent_idx_[i]) {
      anc[i][p] = 1;
      for (size_t k = 0; k < n; ++k) anc[i][k] |= anc[p][k];
    }
  std::vector<int> nanc(n, 0), ndesc(n, 0);
  for (size_t i = 0; i < n; ++i)
    for (size_t k = 0; k < n; ++k)
      if (anc[i][k]) { ++nanc[i]; ++ndesc[k]; }
  // output shapes (multi-parent units get every parent's shape)
  shapes_.assign(n, {});
  for (size_t i = 0; i < n; ++i) {
    std::vector<Shape> ins;
    for (size_t p : parent_idx_[i]) ins.push_back(shapes_[p]);
    if (ins.empty()) ins.push_back(input_shape);
    shapes_[i] = units[i]->OutputShapeN(ins);
  }
  // Lifetimes valid for ANY schedule the engine and the streams may take:
  // unit u runs no earlier than position |anc(u)| and no later than
  // n-1-|desc(u)|; an output is born at its producer's earliest position
  // and dies after its consumers' latest.  Two outputs whose intervals
  // are disjoint are ordered by the dependencies in every schedule, so they
  // may share arena bytes even with branches running concurrently.  For a
  // chain this is exactly [i, i+2).
  std::vector<MemoryNode> nodes(n);
  life_.assign(n, {0, 0});
  for (size_t i = 0; i < n; ++i) {
    int fin = nanc[i] + 1;
    for (size_t c : child_idx_[i]) fin = std::max(fin, (int)n - ndesc[c]);
    if (child_idx_[i].empty()) fin = (int)n + 1;  // a sink: the output
    nodes[i].time_start = nanc[i];
    nodes[i].time_finish = fin;
    nodes[i].value = (numel(shapes_[i]) * esz + 255) / 256 * 256;
    life_[i] = {nanc[i], fin};
  }
  out_shape_ = n ? shapes_.back() : input_shape;
  arena_bytes_ = MemoryOptimizer().Optimize(&nodes);
  offsets_.resize(n);
  for (size_t i = 0; i < n; ++i) offsets_[i] = nodes[i].position;
  // streams: a unit continues its first parent's stream when it is that
  // parent's first child; every other branch (and every extra head) opens
  // a stream of its own
  stream_of_.assign(n, 0);
  int nstreams = 0;
  for (size_t i = 0; i < n; ++i) {
    if (parent_idx_[i].empty()) {
      stream_of_[i] = nstreams++;
    } else {
      size_t p = parent_idx_[i][0];
      stream_of_[i] = child_idx_[p][0] == i ? stream_of_[p] : nstreams++;
    }
  }
  nstreams = std::max(nstreams, 1);
  FreeStreams(&streams_, &stream_ctx_);
  for (auto e : done_) (void)hipEventDestroy(e);
  done_.clear();
  streams_.assign(1, ctx_.stream);
  stream_ctx_.assign(1, ExecContext());
  stream_ctx_[0].gpu = ctx_.gpu;
  stream_ctx_[0].stream = ctx_.stream;
  if (ctx_.gpu) {
    for (int k = 1; k < nstreams; ++k) {
      hipStream_t st;
      HIPCHECK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
      streams_.push_back(st);
      ExecContext c;
      c.gpu = true;
      c.stream = st;
      stream_ctx_.push_back(c);
    }
    done_.resize(n);
    for (auto& e : done_)
      HIPCHECK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
    if (!start_ev_)
      HIPCHECK(hipEventCreateWithFlags(&start_ev_, hipEventDisableTiming));
  } else {
    // host branches run on the engine's threads; each unit gets the
    // stream-0 context but scratch must not be shared between threads
    for (int k = 1; k < nstreams; ++k) {
      ExecContext c;
      stream_ctx_.push_back(c);
    }
  }
  for (auto* p : pending_) delete p;
  pending_.clear();
  for (size_t i = 0; i < n; ++i) pending_.push_back(new std::atomic<int>(0));
  if (ctx_.gpu) {
    HIPCHECK(hipMalloc(&arena_, std::max<size_t>(arena_bytes_, 256)));
    HIPCHECK(hipMalloc(&in_dev_, numel(input_shape) * 6 + 256));
  } else {
    host_arena_.assign(arena_bytes_ / 4 + 64, 0.f);
    arena_ = host_arena_.data();
  }
  for (auto& u : units) u->Initialize(ctx_);
  VR_INF(g_log, "%s: %zu units, %d stream(s), arena %zu bytes (%s)",
         name.c_str(), n, nstreams, arena_bytes_, ctx_.gpu ? "gpu" : "cpu");
}

std::vector<int> Workflow::LastOrder() const {
  auto* self = const_cast<Workflow*>(this);
  std::lock_guard<std::mutex> lk(self->order_mu_);
  return order_;
}

// Run unit i (its parents are done, or enqueued earlier on the device),
// then schedule every child whose last parent this was.
void Workflow::Enqueue(size_t i, const Tensor& in) {
  Unit* u = units[i].get();
  const int sid = stream_of_[i];
  ExecContext& c = stream_ctx_[sid];
  std::vector<const Tensor*> ins;
  for (size_t p : parent_idx_[i]) ins.push_back(&outs_[p]);
  if (ins.empty()) ins.push_back(&in);
  if (ctx_.gpu) {
    if (parent_idx_[i].empty() && sid != 0)
      HIPCHECK(hipStreamWaitEvent(c.stream, start_ev_, 0));
    for (size_t p : parent_idx_[i])
      if (stream_of_[p] != sid)
        HIPCHECK(hipStreamWaitEvent(c.stream, done_[p], 0));
  }
  u->ExecuteN(ins, outs_[i], c);
  if (ctx_.gpu) HIPCHECK(hipEventRecord(done_[i], c.stream));
  {
    std::lock_guard<std::mutex> lk(order_mu_);
    order_.push_back((int)i);
  }
  for (size_t ch : child_idx_[i]) {
    if (pending_[ch]->fetch_sub(1) == 1) {
      Engine* e = engine_.get();
      e->Schedule([this, ch, &in] { Enqueue(ch, in); });
    }
  }
}

void Workflow::RunPass(const Tensor& in) {
  const size_t n = units.size();
  for (size_t i = 0; i < n; ++i)
    pending_[i]->store((int)parent_idx_[i].size());
  {
    std::lock_guard<std::mutex> lk(order_mu_);
    order_.clear();
  }
  if (ctx_.gpu) HIPCHECK(hipEventRecord(start_ev_, ctx_.stream));
  for (size_t i = 0; i < n; ++i)
    if (parent_idx_[i].empty())
      engine_->Schedule([this, i, &in] { Enqueue(i, in); });
  engine_->Wait();
  if (order_.size() != n)
    throw std::runtime_error("workflow pass did not reach every unit");
  if (ctx_.gpu)  // the main stream joins every branch
    for (size_t i = 0; i < n; ++i)
      if (stream_of_[i] != 0)
        HIPCHECK(hipStreamWaitEvent(ctx_.stream, done_[i], 0));
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
  const size_t n = units.size();
  outs_.assign(n, Tensor());
  for (size_t i = 0; i < n; ++i) {
    outs_[i].shape = shapes_[i];
    outs_[i].data = (char*)arena_ + offsets_[i];
  }
  if (ctx_.gpu && graph_exec_ && graph_in_ == in.data) {
    HIPCHECK(hipGraphLaunch(graph_exec_, ctx_.stream));
  } else if (ctx_.gpu && use_graph_ && graph_runs_ >= 1) {
    // capture this pass (every branch stream joins through the events)
    ReleaseGraph();
    // the captured pass is enqueued by ONE host thread: appending to one
    // capture graph from several pool threads at once is not safe in the
    // HIP runtime (a rare crash in the --gpu-branch test); the branch
    // streams and their events keep the parallelism inside the graph
    std::unique_ptr<Engine> pool = std::move(engine_);
    engine_ = MakeSerialEngine();
    HIPCHECK(hipStreamBeginCapture(ctx_.stream, hipStreamCaptureModeRelaxed));
    hipGraph_t g = nullptr;
    try {
      RunPass(in);
    } catch (...) {
      engine_ = std::move(pool);
      (void)hipStreamEndCapture(ctx_.stream, &g);
      if (g) (void)hipGraphDestroy(g);
      throw;
    }
    engine_ = std::move(pool);
    HIPCHECK(hipStreamEndCapture(ctx_.stream, &g));
    HIPCHECK(hipGraphInstantiate(&graph_exec_, g, nullptr, nullptr, 0));
    (void)hipGraphDestroy(g);
    graph_in_ = in.data;
    VR_INF(g_log, "%s: inference pass captured into a hipGraph",
           name.c_str());
    HIPCHECK(hipGraphLaunch(graph_exec_, ctx_.stream));
  } else {
    RunPass(in);
    ++graph_runs_;
  }
  const Tensor& last = n ? outs_.back() : in;
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
