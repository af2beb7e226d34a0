// tests.cc - self-test binary of the native runtime (the reference's
// libVeles/tests/ gtest suite: memory_optimizer, workflow_loader, units).
//   veles_rt_tests [package.zip input.npy expected.npy [--gpu]]
//   veles_rt_tests --gpu-branch   (branch streams + hipGraph on an MI355X)
#include <atomic>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <iostream>

#include <sstream>
#include <unistd.h>

#include "../kernels/hvk_api.h"
#include "json.h"
#include "logger.h"
#include "memory_optimizer.h"
#include "npy.h"
#include "runtime.h"

namespace veles_rt {
extern int veles_rt_units_anchor;
}
using namespace veles_rt;

static int g_fail = 0;
#define EXPECT(c)                                                    \
  do {                                                               \
    if (!(c)) {                                                      \
      std::fprintf(stderr, "%s:%d: EXPECT(%s) failed\n", __FILE__,   \
                   __LINE__, #c);                                    \
      ++g_fail;                                                      \
    }                                                                \
  } while (0)

static bool Overlaps(const MemoryNode& a, const MemoryNode& b) {
  bool t = a.time_start < b.time_finish && b.time_start < a.time_finish;
  bool m = a.position < b.position + b.value && b.position < a.position + a.value;
  return t && m;
}

static void TestMemoryOptimizer() {
  MemoryOptimizer opt;
  // libVeles/tests/memory_optimizer.cc:43-56 (Linear): five buffers, each
  // alive for two steps -> height 2, buffer i at offset i % 2
  std::vector<MemoryNode> lin(5);
  for (int i = 0; i < 5; ++i) lin[i] = {i, i + 2, 1, 0};
  EXPECT(opt.Optimize(&lin) == 2);
  for (int i = 0; i < 5; ++i) EXPECT(lin[i].position == (size_t)(i % 2));
  // libVeles/tests/memory_optimizer.cc:58-93 (Twisted): height exactly 6
  std::vector<MemoryNode> tw = {{0, 5, 2, 0}, {1, 6, 1, 0}, {1, 4, 1, 0},
                                {1, 4, 1, 0}, {1, 7, 1, 0}, {4, 7, 2, 0},
                                {6, 7, 3, 0}};
  EXPECT(opt.Optimize(&tw) == 6);
  for (size_t i = 0; i < tw.size(); ++i)
    for (size_t j = i + 1; j < tw.size(); ++j) EXPECT(!Overlaps(tw[i], tw[j]));
  std::ostringstream os;
  opt.Print(tw, &os);
  EXPECT(!os.str().empty());
  // random lifetimes: never overlap, and the height is at least the peak
  unsigned seed = 12345;
  auto rnd = [&seed](int m) {
    seed = seed * 1103515245u + 12345u;
    return (int)((seed >> 16) % (unsigned)m);
  };
  for (int rep = 0; rep < 50; ++rep) {
    std::vector<MemoryNode> v(12);
    for (auto& n : v) {
      n.time_start = rnd(10);
      n.time_finish = n.time_start + 1 + rnd(5);
      n.value = 1 + (size_t)rnd(8);
    }
    size_t h = opt.Optimize(&v);
    size_t peak = 0;
    for (int t = 0; t < 16; ++t) {
      size_t live = 0;
      for (auto& n : v)
        if (n.time_start <= t && t < n.time_finish) live += n.value;
      peak = std::max(peak, live);
    }
    EXPECT(h >= peak);
    for (size_t i = 0; i < v.size(); ++i) {
      EXPECT(v[i].position + v[i].value <= h);
      for (size_t j = i + 1; j < v.size(); ++j) EXPECT(!Overlaps(v[i], v[j]));
    }
  }
}

// ------------------------------------------------- branching-graph units
// out = k * in, on the host or (GPU) through hvk_cast's scale
class TScale : public Unit {
 public:
  TScale(const std::string& n, float k) : Unit(n), k_(k) {}
  std::string Class() const override { return "TScale"; }
  Shape OutputShape(const Shape& in) const override { return in; }
  void Execute(const Tensor& in, Tensor& out, ExecContext& ctx) override {
    const size_t n = numel(in.shape);
    if (ctx.gpu) {
      hvk_cast(in.data, HVK_BF16, out.data, HVK_BF16, (long long)n, k_,
               ctx.stream);
      return;
    }
    for (size_t i = 0; i < n; ++i)
      ((float*)out.data)[i] = k_ * ((const float*)in.data)[i];
  }

 private:
  float k_;
};

// concatenation of every parent along the last axis (per sample row)
class TJoin : public Unit {
 public:
  explicit TJoin(const std::string& n) : Unit(n) {}
  std::string Class() const override { return "TJoin"; }
  Shape OutputShape(const Shape& in) const override { return in; }
  Shape OutputShapeN(const std::vector<Shape>& ins) const override {
    Shape s = ins.at(0);
    s.back() = 0;
    for (auto& x : ins) s.back() += x.back();
    return s;
  }
  void Execute(const Tensor&, Tensor&, ExecContext&) override {}
  void ExecuteN(const std::vector<const Tensor*>& ins, Tensor& out,
                ExecContext& ctx) override {
    const size_t rows = numel(out.shape) / out.shape.back();
    const size_t es = ctx.gpu ? 2 : 4;
    size_t col = 0;
    for (auto* t : ins) {
      const size_t w = t->shape.back();
      if (ctx.gpu) {
        (void)hipMemcpy2DAsync((char*)out.data + col * es,
                               out.shape.back() * es, t->data, w * es, w * es,
                               rows, hipMemcpyDeviceToDevice, ctx.stream);
      } else {
        for (size_t r = 0; r < rows; ++r)
          std::memcpy((char*)out.data + (r * out.shape.back() + col) * es,
                      (const char*)t->data + r * w * es, w * es);
      }
      col += w;
    }
  }
};

static void Link(Unit* from, Unit* to) {
  from->children.push_back(to);
  to->parents.push_back(from);
}

// head -> {a = 2x, b = 3x, c = 5x}; a -> a2 = -1 * a; join(a2, b, c) -> tail
static std::unique_ptr<Workflow> Diamond() {
  auto wf = std::unique_ptr<Workflow>(new Workflow());
  wf->name = "diamond";
  std::vector<Unit*> u;
  auto add = [&](Unit* x) {
    wf->units.emplace_back(x);
    u.push_back(x);
    return x;
  };
  Unit* head = add(new TScale("head", 1.f));
  Unit* a = add(new TScale("a", 2.f));
  Unit* b = add(new TScale("b", 3.f));
  Unit* c = add(new TScale("c", 5.f));
  Unit* a2 = add(new TScale("a2", -1.f));
  Unit* j = add(new TJoin("join"));
  Unit* tail = add(new TScale("tail", 0.5f));
  Link(head, a);
  Link(head, b);
  Link(head, c);
  Link(a, a2);
  Link(a2, j);
  Link(b, j);
  Link(c, j);
  Link(j, tail);
  return wf;
}

static bool Reaches(Unit* from, Unit* to) {
  if (from == to) return true;
  for (Unit* c : from->children)
    if (Reaches(c, to)) return true;
  return false;
}

// Multi-parent readiness through the Engine (libVeles unit.cc:60-76): every
// unit runs once, after all of its parents; outputs of units that may run
// concurrently never share arena bytes; serial, pooled and (GPU) streamed /
// graph-replayed passes give the same result.
static void TestBranchingEngine(bool gpu) {
  const Shape shape = {3, 4};
  std::vector<float> x(12);
  for (int i = 0; i < 12; ++i) x[i] = (float)(i - 5) * 0.25f;
  std::vector<float> expect;
  for (int r = 0; r < 3; ++r) {
    for (int k : {-2, 3, 5})
      for (int q = 0; q < 4; ++q) expect.push_back(0.5f * k * x[r * 4 + q]);
  }
  for (int mode = 0; mode < 3; ++mode) {
    auto wf = Diamond();
    if (mode >= 1) wf->SetEngine(MakeThreadPoolEngine(4));
    if (mode == 2) wf->EnableGraph(true);
    wf->Initialize(shape, gpu);
    if (gpu && wf->gpu()) EXPECT(wf->NumStreams() == 3);
    for (int run = 0; run < 4; ++run) {
      auto y = wf->Run(x);
      EXPECT(y.size() == expect.size());
      for (size_t i = 0; i < y.size() && i < expect.size(); ++i)
        EXPECT(std::fabs(y[i] - expect[i]) <= (gpu ? 0.02f : 1e-6f) *
                                                  (1 + std::fabs(expect[i])));
      auto order = wf->LastOrder();
      if (!(mode == 2 && wf->GraphActive() && run >= 2)) {
        EXPECT(order.size() == wf->units.size());
        std::vector<int> pos(wf->units.size(), -1);
        for (size_t k = 0; k < order.size(); ++k) pos[order[k]] = (int)k;
        for (size_t i = 0; i < wf->units.size(); ++i)
          for (Unit* p : wf->units[i]->parents)
            for (size_t k = 0; k < wf->units.size(); ++k)
              if (wf->units[k].get() == p) EXPECT(pos[k] < pos[i]);
      }
    }
    if (mode == 2 && gpu && wf->gpu()) EXPECT(wf->GraphActive());
    // arena: two outputs whose producers are unordered (may run at once)
    // never overlap in bytes while both are alive
    const size_t n = wf->units.size();
    for (size_t i = 0; i < n; ++i)
      for (size_t k = i + 1; k < n; ++k) {
        Unit* ui = wf->units[i].get();
        Unit* uk = wf->units[k].get();
        if (Reaches(ui, uk) || Reaches(uk, ui)) continue;
        auto li = wf->Lifetime(i), lk = wf->Lifetime(k);
        EXPECT(li.first < lk.second && lk.first < li.second);
      }
  }
  // a chain keeps the tight libVeles lifetimes [i, i + 2)
  auto chain = std::unique_ptr<Workflow>(new Workflow());
  Unit* prev = nullptr;
  for (int i = 0; i < 5; ++i) {
    Unit* u = new TScale("s" + std::to_string(i), 1.f);
    chain->units.emplace_back(u);
    if (prev) Link(prev, u);
    prev = u;
  }
  chain->Initialize(shape, false);
  for (int i = 0; i < 4; ++i)
    EXPECT(chain->Lifetime(i) == std::make_pair(i, i + 2));
}

static void TestLogger() {
  char path[] = "/tmp/veles_rt_logXXXXXX";
  int fd = mkstemp(path);
  FILE* f = fdopen(fd, "w+");
  Logger::Sink() = f;
  LogLevel old = Logger::Threshold();
  Logger::Threshold() = LogLevel::Info;
  Logger lg("tests");
  VR_DBG(lg, "hidden %d", 1);
  VR_INF(lg, "shown %d", 2);
  VR_ERR(lg, "error %s", "x");
  Logger::Threshold() = old;
  Logger::Sink() = nullptr;
  std::fflush(f);
  std::rewind(f);
  char buf[512] = {0};
  size_t got = std::fread(buf, 1, sizeof(buf) - 1, f);
  std::fclose(f);
  std::remove(path);
  std::string text(buf, got);
  EXPECT(text.find("hidden") == std::string::npos);
  EXPECT(text.find("INFO tests: shown 2") != std::string::npos);
  EXPECT(text.find("ERROR tests: error x") != std::string::npos);
  EXPECT(ParseLogLevel("debug") == LogLevel::Debug);
  EXPECT(ParseLogLevel("bogus") == LogLevel::Warning);
}

static void TestJson() {
  Json j = Json::parse(
      R"({"a": [1, 2.5, -3e2], "b": {"c": "x\"y"}, "d": true, "e": null})");
  EXPECT(j["a"].size() == 3);
  EXPECT(std::fabs(j["a"][2].num + 300) < 1e-9);
  EXPECT(j["b"]["c"].str == "x\"y");
  EXPECT(j["d"].b);
  EXPECT(j["e"].type == Json::Null);
}

static void TestNpy() {
  NpyArray a;
  a.shape = {2, 3};
  a.data = {1, 2, 3, 4, 5, 6};
  NpyArray b = ParseNpy(WriteNpy(a));
  EXPECT(b.shape == a.shape);
  EXPECT(b.data == a.data);
  EXPECT(HalfToFloat(0x3c00) == 1.0f);
  EXPECT(HalfToFloat(0xc000) == -2.0f);
}

static void TestFactory() {
  auto& f = UnitFactory::Instance();
  const char* need[] = {"All2AllTanh", "All2AllSoftmax", "ConvStrictRELU",
                        "MaxPooling", "LRNormalizerForward", "DropoutForward"};
  for (auto n : need) EXPECT(f.Has(n));
}

static int TestPackage(const char* pkg, const char* in, const char* exp,
                       bool gpu) {
  auto wf = LoadWorkflow(pkg);
  NpyArray x = ParseNpy(ReadFile(in));
  NpyArray e = ParseNpy(ReadFile(exp));
  wf->Initialize(x.shape, gpu);
  auto y = wf->Run(x.data);
  EXPECT(y.size() == e.data.size());
  double maxerr = 0, maxref = 0;
  for (size_t i = 0; i < y.size() && i < e.data.size(); ++i) {
    maxerr = std::max(maxerr, (double)std::fabs(y[i] - e.data[i]));
    maxref = std::max(maxref, (double)std::fabs(e.data[i]));
  }
  std::cout << "package " << pkg << " (" << (wf->gpu() ? "gpu" : "cpu")
            << "): max|err| " << maxerr << " max|ref| " << maxref
            << " arena " << wf->ArenaBytes() << std::endl;
  double tol = wf->gpu() ? 3e-2 * std::max(1.0, maxref) : 1e-4 * std::max(1.0, maxref);
  EXPECT(maxerr <= tol);
  return 0;
}

// Engine contract under concurrency (run under -fsanitize=thread by
// tests/test_native_runtime.py): tasks that schedule children, Wait()
// returning only after every descendant ran.
static void TestEngines() {
  for (int rep = 0; rep < 20; ++rep) {
    auto eng = MakeThreadPoolEngine(4);
    std::atomic<int> ran{0};
    std::function<void(int)> fan;
    Engine* e = eng.get();
    fan = [&](int depth) {
      ran.fetch_add(1);
      if (depth < 4)
        for (int c = 0; c < 3; ++c) e->Schedule([&fan, depth] { fan(depth + 1); });
    };
    e->Schedule([&fan] { fan(0); });
    e->Wait();
    EXPECT(ran.load() == 1 + 3 + 9 + 27 + 81);
  }
  auto ser = MakeSerialEngine();
  int n = 0;
  ser->Schedule([&n] { ++n; });
  ser->Wait();
  EXPECT(n == 1);
}

int main(int argc, char** argv) {
  (void)veles_rt_units_anchor;
  try {
    TestMemoryOptimizer();
    TestJson();
    TestNpy();
    TestFactory();
    TestEngines();
    TestLogger();
    TestBranchingEngine(false);
    if (argc >= 2 && std::strcmp(argv[1], "--gpu-branch") == 0)
      TestBranchingEngine(true);
    else if (argc >= 4)
      TestPackage(argv[1], argv[2], argv[3],
                  argc > 4 && std::strcmp(argv[4], "--gpu") == 0);
  } catch (const std::exception& ex) {
    std::fprintf(stderr, "exception: %s\n", ex.what());
    return 1;
  }
  std::cout << (g_fail ? "FAILED " : "OK ") << g_fail << std::endl;
  return g_fail ? 1 : 0;
}
