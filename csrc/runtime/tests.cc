// tests.cc - self-test binary of the native runtime (the reference's
// libVeles/tests/ gtest suite: memory_optimizer, workflow_loader, units).
//   veles_rt_tests [package.zip input.npy expected.npy [--gpu]]
#include <atomic>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <iostream>

#include "json.h"
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
  // a chain: each buffer lives for two steps -> two slots suffice
  std::vector<MemoryNode> lin(6);
  for (int i = 0; i < 6; ++i) lin[i] = {i, i + 2, 1, 0};
  EXPECT(opt.Optimize(&lin) == 2);
  // twisted lifetimes of varying sizes: never overlap, bound by the peak
  std::vector<MemoryNode> tw = {{0, 3, 3, 0}, {1, 2, 2, 0}, {2, 5, 1, 0},
                                {3, 6, 2, 0}, {0, 6, 1, 0}, {4, 6, 3, 0}};
  size_t h = opt.Optimize(&tw);
  size_t peak = 0;
  for (int t = 0; t < 6; ++t) {
    size_t live = 0;
    for (auto& n : tw)
      if (n.time_start <= t && t < n.time_finish) live += n.value;
    peak = std::max(peak, live);
  }
  EXPECT(h >= peak);
  EXPECT(h <= peak + 2);
  for (size_t i = 0; i < tw.size(); ++i)
    for (size_t j = i + 1; j < tw.size(); ++j) EXPECT(!Overlaps(tw[i], tw[j]));
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
    if (argc >= 4)
      TestPackage(argv[1], argv[2], argv[3],
                  argc > 4 && std::strcmp(argv[4], "--gpu") == 0);
  } catch (const std::exception& ex) {
    std::fprintf(stderr, "exception: %s\n", ex.what());
    return 1;
  }
  std::cout << (g_fail ? "FAILED " : "OK ") << g_fail << std::endl;
  return g_fail ? 1 : 0;
}
