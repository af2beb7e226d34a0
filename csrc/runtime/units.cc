// units.cc - NN units of the native runtime (inference): all2all*,
// softmax, conv*, pooling, LRN, dropout (identity), activations.
// CPU: float32 reference loops.  GPU: the libhvk kernels on bf16 tensors.
#include <cmath>
#include <cstring>
#include <stdexcept>

#include "../kernels/hvk_api.h"
#include "runtime.h"

namespace veles_rt {
namespace {

#define HIPCHECK(x)                                                     \
  do {                                                                  \
    hipError_t e_ = (x);                                                \
    if (e_ != hipSuccess)                                               \
      throw std::runtime_error(std::string("HIP: ") + hipGetErrorString(e_)); \
  } while (0)
#define HVKCHECK(x)                                                     \
  do {                                                                  \
    int r_ = (x);                                                       \
    if (r_ != 0) throw std::runtime_error("hvk call failed: " #x);      \
  } while (0)

int ActCode(const std::string& m) {
  if (m == "ACTIVATION_TANH") return 1;
  if (m == "ACTIVATION_RELU") return 2;
  if (m == "ACTIVATION_STRICT_RELU") return 3;
  if (m == "ACTIVATION_SIGMOID") return 4;
  return 0;
}

float Act(float x, int a) {
  switch (a) {
    case 1: return 1.7159f * std::tanh(0.6666f * x);
    case 2: return x > 15.f ? x : std::log1p(std::exp(x));
    case 3: return x > 0.f ? x : 0.f;
    case 4: return 1.f / (1.f + std::exp(-x));
    default: return x;
  }
}

uint16_t F2Bf(float f) {
  uint32_t u;
  std::memcpy(&u, &f, 4);
  if ((u & 0x7fffffff) > 0x7f800000) return (uint16_t)((u >> 16) | 0x40);
  u += 0x7fff + ((u >> 16) & 1);
  return (uint16_t)(u >> 16);
}

void* UploadBf16(const std::vector<float>& v) {
  std::vector<uint16_t> h(v.size());
  for (size_t i = 0; i < v.size(); ++i) h[i] = F2Bf(v[i]);
  void* d = nullptr;
  HIPCHECK(hipMalloc(&d, h.size() * 2 + 16));
  HIPCHECK(hipMemcpy(d, h.data(), h.size() * 2, hipMemcpyHostToDevice));
  return d;
}
void* UploadF32(const std::vector<float>& v) {
  void* d = nullptr;
  HIPCHECK(hipMalloc(&d, v.size() * 4 + 16));
  HIPCHECK(hipMemcpy(d, v.data(), v.size() * 4, hipMemcpyHostToDevice));
  return d;
}

const NpyArray& Arr(const Json& v, const std::map<std::string, NpyArray>& a) {
  auto it = a.find(v.str);
  if (it == a.end()) throw std::runtime_error("missing array " + v.str);
  return it->second;
}

std::vector<int> Ints(const Json& v) {
  std::vector<int> r;
  if (v.type == Json::Array)
    for (auto& x : v.arr) r.push_back((int)x.num);
  else
    r.push_back((int)v.num);
  return r;
}

// ------------------------------------------------------------- parametric
class ParamUnit : public Unit {
 public:
  using Unit::Unit;
  ~ParamUnit() override {
    if (dw_) (void)hipFree(dw_);
    if (db_) (void)hipFree(db_);
  }
  void SetParameter(const std::string& k, const Json& v,
                    const std::map<std::string, NpyArray>& a) override {
    if (k == "weights") w_ = Arr(v, a);
    else if (k == "bias") b_ = Arr(v, a);
    else if (k == "include_bias") include_bias_ = v.b;
    else if (k == "weights_transposed") transposed_ = v.b;
    else if (k == "activation_mode") act_ = ActCode(v.str);
    else Other(k, v);
  }
  virtual void Other(const std::string& k, const Json& v) {}

 protected:
  NpyArray w_, b_;
  bool include_bias_ = true, transposed_ = false;
  int act_ = 0;
  void* dw_ = nullptr;
  void* db_ = nullptr;
};

class All2All : public ParamUnit {
 public:
  using ParamUnit::ParamUnit;
  std::string Class() const override { return "All2All"; }
  size_t Out() const { return transposed_ ? w_.shape[1] : w_.shape[0]; }
  size_t In() const { return transposed_ ? w_.shape[0] : w_.shape[1]; }
  Shape OutputShape(const Shape& in) const override { return {in[0], Out()}; }
  void Initialize(ExecContext& ctx) override {
    if (ctx.gpu && !dw_) {
      dw_ = UploadBf16(w_.data);
      if (include_bias_ && b_.size()) db_ = UploadF32(b_.data);
    }
  }
  virtual bool Softmax() const { return false; }
  void Execute(const Tensor& in, Tensor& out, ExecContext& ctx) override {
    size_t B = in.shape[0], I = In(), O = Out();
    if (numel(in.shape) != B * I) throw std::runtime_error(name_ + ": input");
    if (ctx.gpu) {
      if (!Softmax()) {
        HVKCHECK(hvk_gemm(0, transposed_ ? 0 : 1, (int)B, (int)O, (int)I,
                          in.data, (int)I, dw_, transposed_ ? (int)O : (int)I,
                          out.data, (int)O, 0, 0, 1.f, 0.f, (const float*)db_,
                          1, act_, nullptr, 0, 0, 1, nullptr, ctx.stream));
      } else {
        float* lg = (float*)ctx.Scratch(B * O * 8 + 256);
        float* pr = lg + B * O;
        HVKCHECK(hvk_gemm(0, transposed_ ? 0 : 1, (int)B, (int)O, (int)I,
                          in.data, (int)I, dw_, transposed_ ? (int)O : (int)I,
                          lg, (int)O, 1, 0, 1.f, 0.f, (const float*)db_, 1, 0,
                          nullptr, 0, 0, 1, nullptr, ctx.stream));
        HVKCHECK(hvk_softmax_ce(lg, HVK_F32, (int)B, (int)O, nullptr, 1.f,
                                nullptr, 0, pr, nullptr, nullptr, nullptr,
                                ctx.stream));
        HVKCHECK(hvk_cast(pr, HVK_F32, out.data, HVK_BF16, (long long)(B * O),
                          1.f, ctx.stream));
      }
      return;
    }
    const float* x = (const float*)in.data;
    float* y = (float*)out.data;
    for (size_t b = 0; b < B; ++b) {
      for (size_t o = 0; o < O; ++o) {
        double s = (include_bias_ && b_.size()) ? b_.data[o] : 0.0;
        for (size_t i = 0; i < I; ++i)
          s += (double)x[b * I + i] *
               (transposed_ ? w_.data[i * O + o] : w_.data[o * I + i]);
        y[b * O + o] = Softmax() ? (float)s : Act((float)s, act_);
      }
      if (Softmax()) {
        float m = y[b * O];
        for (size_t o = 1; o < O; ++o) m = std::max(m, y[b * O + o]);
        double z = 0;
        for (size_t o = 0; o < O; ++o) {
          y[b * O + o] = std::exp(y[b * O + o] - m);
          z += y[b * O + o];
        }
        for (size_t o = 0; o < O; ++o) y[b * O + o] = (float)(y[b * O + o] / z);
      }
    }
  }
};
class All2AllSoftmax : public All2All {
 public:
  using All2All::All2All;
  std::string Class() const override { return "All2AllSoftmax"; }
  bool Softmax() const override { return true; }
};

class Conv : public ParamUnit {
 public:
  using ParamUnit::ParamUnit;
  std::string Class() const override { return "Conv"; }
  void Other(const std::string& k, const Json& v) override {
    if (k == "padding") {
      auto p = Ints(v);
      if (p.size() == 4) { pl_ = p[0]; pt_ = p[1]; pr_ = p[2]; pb_ = p[3]; }
    } else if (k == "sliding") {
      auto s = Ints(v);
      sx_ = s[0];
      sy_ = s.size() > 1 ? s[1] : s[0];
    } else if (k == "grouping") {
      groups_ = (int)v.num;
    }
  }
  int OC() const { return (int)w_.shape[0]; }
  int KH() const { return (int)w_.shape[1]; }
  int KW() const { return (int)w_.shape[2]; }
  int Cg() const { return (int)w_.shape[3]; }
  Shape OutputShape(const Shape& in) const override {
    size_t H = in[1], W = in[2];
    size_t OH = (H + pt_ + pb_ - KH()) / sy_ + 1;
    size_t OW = (W + pl_ + pr_ - KW()) / sx_ + 1;
    return {in[0], OH, OW, (size_t)OC()};
  }
  void Initialize(ExecContext& ctx) override {
    if (!ctx.gpu || dw_) return;
    int C = Cg() * groups_;
    run_ = (groups_ == 1 && C % 8 != 0);
    if (run_) {  // repack to [OC][KH][RUNP] zero padded runs
      int run = KW() * C, runp = (run + 7) / 8 * 8;
      std::vector<float> p((size_t)OC() * KH() * runp, 0.f);
      for (int o = 0; o < OC(); ++o)
        for (int h = 0; h < KH(); ++h)
          for (int j = 0; j < run; ++j)
            p[((size_t)o * KH() + h) * runp + j] =
                w_.data[((size_t)o * KH() + h) * run + j];
      dw_ = UploadBf16(p);
    } else {
      dw_ = UploadBf16(w_.data);
    }
    if (include_bias_ && b_.size()) db_ = UploadF32(b_.data);
  }
  void Execute(const Tensor& in, Tensor& out, ExecContext& ctx) override {
    int N = (int)in.shape[0], H = (int)in.shape[1], W = (int)in.shape[2],
        C = (int)in.shape[3];
    int OH = (int)out.shape[1], OW = (int)out.shape[2], OCn = OC();
    if (ctx.gpu) {
      if (run_)
        HVKCHECK(hvk_conv_fwd_run(in.data, dw_, (const float*)db_, out.data,
                                  N, H, W, C, OCn, KH(), KW(), sy_, sx_, pt_,
                                  pl_, OH, OW, act_, ctx.stream));
      else
        HVKCHECK(hvk_conv_fwd(in.data, dw_, (const float*)db_, out.data, N, H,
                              W, C, OCn, KH(), KW(), sy_, sx_, pt_, pl_, OH,
                              OW, groups_, act_, ctx.stream));
      return;
    }
    const float* x = (const float*)in.data;
    float* y = (float*)out.data;
    int cg = Cg(), ocg = OCn / groups_;
    for (int n = 0; n < N; ++n)
      for (int oh = 0; oh < OH; ++oh)
        for (int ow = 0; ow < OW; ++ow)
          for (int o = 0; o < OCn; ++o) {
            int g = o / ocg;
            double s = (include_bias_ && b_.size()) ? b_.data[o] : 0.0;
            for (int kh = 0; kh < KH(); ++kh) {
              int ih = oh * sy_ - pt_ + kh;
              if (ih < 0 || ih >= H) continue;
              for (int kw = 0; kw < KW(); ++kw) {
                int iw = ow * sx_ - pl_ + kw;
                if (iw < 0 || iw >= W) continue;
                const float* xp = x + (((size_t)n * H + ih) * W + iw) * C + g * cg;
                const float* wp =
                    w_.data.data() + (((size_t)o * KH() + kh) * KW() + kw) * cg;
                for (int c = 0; c < cg; ++c) s += (double)xp[c] * wp[c];
              }
            }
            y[(((size_t)n * OH + oh) * OW + ow) * OCn + o] = Act((float)s, act_);
          }
  }

 private:
  int pl_ = 0, pt_ = 0, pr_ = 0, pb_ = 0, sx_ = 1, sy_ = 1, groups_ = 1;
  bool run_ = false;
};

class Pooling : public Unit {
 public:
  Pooling(const std::string& n, int mode) : Unit(n), mode_(mode) {}
  std::string Class() const override { return "Pooling"; }
  void SetParameter(const std::string& k, const Json& v,
                    const std::map<std::string, NpyArray>&) override {
    if (k == "kx") kx_ = (int)v.num;
    else if (k == "ky") ky_ = (int)v.num;
    else if (k == "sliding") {
      auto s = Ints(v);
      sx_ = s[0];
      sy_ = s.size() > 1 ? s[1] : s[0];
    }
  }
  Shape OutputShape(const Shape& in) const override {
    int H = (int)in[1], W = (int)in[2];
    size_t OH = H > ky_ ? (H - ky_ + sy_ - 1) / sy_ + 1 : 1;
    size_t OW = W > kx_ ? (W - kx_ + sx_ - 1) / sx_ + 1 : 1;
    return {in[0], OH, OW, in[3]};
  }
  void Execute(const Tensor& in, Tensor& out, ExecContext& ctx) override {
    int N = (int)in.shape[0], H = (int)in.shape[1], W = (int)in.shape[2],
        C = (int)in.shape[3], OH = (int)out.shape[1], OW = (int)out.shape[2];
    if (ctx.gpu) {
      HVKCHECK(hvk_pool_fwd(in.data, out.data, nullptr, N, H, W, C, OH, OW,
                            ky_, kx_, sy_, sx_, 0, 0, mode_, ctx.stream));
      return;
    }
    const float* x = (const float*)in.data;
    float* y = (float*)out.data;
    for (int n = 0; n < N; ++n)
      for (int oh = 0; oh < OH; ++oh)
        for (int ow = 0; ow < OW; ++ow)
          for (int c = 0; c < C; ++c) {
            float best = 0, sum = 0;
            int cnt = 0;
            bool first = true;
            for (int h = oh * sy_; h < std::min(oh * sy_ + ky_, H); ++h)
              for (int w = ow * sx_; w < std::min(ow * sx_ + kx_, W); ++w) {
                float v = x[(((size_t)n * H + h) * W + w) * C + c];
                sum += v;
                ++cnt;
                float key = mode_ == 2 ? std::fabs(v) : v;
                float bk = mode_ == 2 ? std::fabs(best) : best;
                if (first || key > bk) { best = v; first = false; }
              }
            y[(((size_t)n * OH + oh) * OW + ow) * C + c] =
                mode_ == 1 ? sum / std::max(cnt, 1) : best;
          }
  }

 private:
  int mode_, kx_ = 2, ky_ = 2, sx_ = 2, sy_ = 2;
};
struct MaxPooling : Pooling { MaxPooling(const std::string& n) : Pooling(n, 0) {} };
struct AvgPooling : Pooling { AvgPooling(const std::string& n) : Pooling(n, 1) {} };
struct MaxAbsPooling : Pooling { MaxAbsPooling(const std::string& n) : Pooling(n, 2) {} };

class LRN : public Unit {
 public:
  using Unit::Unit;
  std::string Class() const override { return "LRNormalizerForward"; }
  void SetParameter(const std::string& k, const Json& v,
                    const std::map<std::string, NpyArray>&) override {
    if (k == "alpha") alpha_ = (float)v.num;
    else if (k == "beta") beta_ = (float)v.num;
    else if (k == "k") k_ = (float)v.num;
    else if (k == "n") n_ = (int)v.num;
  }
  Shape OutputShape(const Shape& in) const override { return in; }
  void Execute(const Tensor& in, Tensor& out, ExecContext& ctx) override {
    size_t C = in.shape.back(), P = numel(in.shape) / C;
    if (ctx.gpu) {
      HVKCHECK(hvk_lrn_fwd(in.data, out.data, (long long)P, (int)C, n_, alpha_,
                           beta_, k_, ctx.stream));
      return;
    }
    const float* x = (const float*)in.data;
    float* y = (float*)out.data;
    int half = n_ / 2;
    for (size_t p = 0; p < P; ++p)
      for (size_t c = 0; c < C; ++c) {
        double s = 0;
        for (int j = std::max<int>(0, (int)c - half);
             j <= std::min<int>((int)C - 1, (int)c + half); ++j)
          s += (double)x[p * C + j] * x[p * C + j];
        y[p * C + c] = x[p * C + c] * std::pow(k_ + alpha_ * s, -beta_);
      }
  }

 private:
  float alpha_ = 1e-4f, beta_ = 0.75f, k_ = 2.f;
  int n_ = 5;
};

class Identity : public Unit {
 public:
  using Unit::Unit;
  std::string Class() const override { return "Identity"; }
  Shape OutputShape(const Shape& in) const override { return in; }
  void Execute(const Tensor& in, Tensor& out, ExecContext& ctx) override {
    size_t n = numel(in.shape);
    if (ctx.gpu)
      HIPCHECK(hipMemcpyAsync(out.data, in.data, n * 2,
                              hipMemcpyDeviceToDevice, ctx.stream));
    else
      std::memcpy(out.data, in.data, n * 4);
  }
};

class Activation : public Unit {
 public:
  Activation(const std::string& n, int act) : Unit(n), act_(act) {}
  std::string Class() const override { return "Activation"; }
  Shape OutputShape(const Shape& in) const override { return in; }
  void Execute(const Tensor& in, Tensor& out, ExecContext& ctx) override {
    size_t n = numel(in.shape);
    if (ctx.gpu) {
      HVKCHECK(hvk_act_fwd(in.data, HVK_BF16, out.data, HVK_BF16,
                           (long long)n, act_, ctx.stream));
      return;
    }
    const float* x = (const float*)in.data;
    float* y = (float*)out.data;
    for (size_t i = 0; i < n; ++i) y[i] = Act(x[i], act_);
  }

 private:
  int act_;
};

template <int A>
struct ActN : Activation { ActN(const std::string& n) : Activation(n, A) {} };

}  // namespace

// registrations (class names written by Workflow.package_export)
VELES_REGISTER_UNIT(All2All, "All2All");
VELES_REGISTER_UNIT(All2All, "All2AllTanh");
VELES_REGISTER_UNIT(All2All, "All2AllRELU");
VELES_REGISTER_UNIT(All2All, "All2AllStrictRELU");
VELES_REGISTER_UNIT(All2All, "All2AllSigmoid");
VELES_REGISTER_UNIT(All2All, "ResizableAll2All");
VELES_REGISTER_UNIT(All2AllSoftmax, "All2AllSoftmax");
VELES_REGISTER_UNIT(Conv, "Conv");
VELES_REGISTER_UNIT(Conv, "ConvTanh");
VELES_REGISTER_UNIT(Conv, "ConvRELU");
VELES_REGISTER_UNIT(Conv, "ConvStrictRELU");
VELES_REGISTER_UNIT(Conv, "ConvSigmoid");
VELES_REGISTER_UNIT(MaxPooling, "MaxPooling");
VELES_REGISTER_UNIT(AvgPooling, "AvgPooling");
VELES_REGISTER_UNIT(MaxAbsPooling, "MaxAbsPooling");
VELES_REGISTER_UNIT(LRN, "LRNormalizerForward");
VELES_REGISTER_UNIT(Identity, "DropoutForward");
VELES_REGISTER_UNIT(ActN<1>, "ForwardTanh");
VELES_REGISTER_UNIT(ActN<2>, "ForwardRELU");
VELES_REGISTER_UNIT(ActN<3>, "ForwardStrictRELU");
VELES_REGISTER_UNIT(ActN<4>, "ForwardSigmoid");

// force-link anchor
int veles_rt_units_anchor = 0;

}  // namespace veles_rt
