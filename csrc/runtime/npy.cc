#include "npy.h"

#include <cstring>
#include <sstream>
#include <stdexcept>

namespace veles_rt {

float HalfToFloat(uint16_t h) {
  uint32_t sign = (h & 0x8000) << 16, exp = (h >> 10) & 0x1f,
           man = h & 0x3ff, f;
  if (exp == 0) {
    if (man == 0) {
      f = sign;
    } else {  // subnormal
      exp = 127 - 15 + 1;
      while (!(man & 0x400)) { man <<= 1; --exp; }
      man &= 0x3ff;
      f = sign | (exp << 23) | (man << 13);
    }
  } else if (exp == 31) {
    f = sign | 0x7f800000 | (man << 13);
  } else {
    f = sign | ((exp - 15 + 127) << 23) | (man << 13);
  }
  float out;
  std::memcpy(&out, &f, 4);
  return out;
}

static std::string field(const std::string& hdr, const std::string& key) {
  size_t p = hdr.find("'" + key + "'");
  if (p == std::string::npos) throw std::runtime_error("npy: no " + key);
  p = hdr.find(':', p) + 1;
  while (hdr[p] == ' ') ++p;
  size_t e;
  if (hdr[p] == '\'') {
    e = hdr.find('\'', p + 1);
    return hdr.substr(p + 1, e - p - 1);
  }
  if (hdr[p] == '(') {
    e = hdr.find(')', p);
    return hdr.substr(p + 1, e - p - 1);
  }
  e = hdr.find_first_of(",}", p);
  return hdr.substr(p, e - p);
}

NpyArray ParseNpy(const Bytes& b) {
  if (b.size() < 10 || std::memcmp(b.data(), "\x93NUMPY", 6) != 0)
    throw std::runtime_error("npy: bad magic");
  int major = b[6];
  size_t hlen, off;
  if (major == 1) {
    hlen = b[8] | (b[9] << 8);
    off = 10;
  } else {
    hlen = b[8] | (b[9] << 8) | (b[10] << 16) | ((size_t)b[11] << 24);
    off = 12;
  }
  std::string hdr((const char*)&b[off], hlen);
  off += hlen;
  std::string descr = field(hdr, "descr");
  bool fortran = field(hdr, "fortran_order").find("True") != std::string::npos;
  NpyArray a;
  std::stringstream ss(field(hdr, "shape"));
  std::string tok;
  while (std::getline(ss, tok, ',')) {
    size_t s = tok.find_first_not_of(' ');
    if (s == std::string::npos) continue;
    a.shape.push_back(std::stoull(tok.substr(s)));
  }
  size_t n = a.size();
  a.data.resize(n);
  const uint8_t* src = &b[off];
  char kind = descr[1];
  int w = std::stoi(descr.substr(2));
  if (descr[0] == '>') throw std::runtime_error("npy: big endian");
  for (size_t i = 0; i < n; ++i) {
    float v = 0;
    if (kind == 'f' && w == 4) std::memcpy(&v, src + 4 * i, 4);
    else if (kind == 'f' && w == 8) { double d; std::memcpy(&d, src + 8 * i, 8); v = (float)d; }
    else if (kind == 'f' && w == 2) { uint16_t h; std::memcpy(&h, src + 2 * i, 2); v = HalfToFloat(h); }
    else if (kind == 'i' && w == 4) { int32_t x; std::memcpy(&x, src + 4 * i, 4); v = (float)x; }
    else if (kind == 'i' && w == 2) { int16_t x; std::memcpy(&x, src + 2 * i, 2); v = (float)x; }
    else if (kind == 'i' && w == 8) { int64_t x; std::memcpy(&x, src + 8 * i, 8); v = (float)x; }
    else if (kind == 'u' && w == 1) v = (float)src[i];
    else throw std::runtime_error("npy: unsupported dtype " + descr);
    a.data[i] = v;
  }
  if (fortran && a.shape.size() >= 2) {
    // reverse-axes transpose into C order
    std::vector<float> c(n);
    size_t nd = a.shape.size();
    std::vector<size_t> idx(nd, 0);
    for (size_t i = 0; i < n; ++i) {
      // i is the Fortran-linear index; compute C-linear index
      size_t rem = i, cidx = 0;
      for (size_t d = 0; d < nd; ++d) {
        idx[d] = rem % a.shape[d];
        rem /= a.shape[d];
      }
      for (size_t d = 0; d < nd; ++d) cidx = cidx * a.shape[d] + idx[d];
      c[cidx] = a.data[i];
    }
    a.data.swap(c);
  }
  return a;
}

Bytes WriteNpy(const NpyArray& a) {
  std::string shape = "(";
  for (size_t i = 0; i < a.shape.size(); ++i) {
    shape += std::to_string(a.shape[i]);
    shape += (a.shape.size() == 1 || i + 1 < a.shape.size()) ? "," : "";
  }
  shape += ")";
  std::string hdr = "{'descr': '<f4', 'fortran_order': False, 'shape': " +
                    shape + ", }";
  while ((10 + hdr.size() + 1) % 64) hdr += ' ';
  hdr += '\n';
  Bytes out = {0x93, 'N', 'U', 'M', 'P', 'Y', 1, 0,
               (uint8_t)(hdr.size() & 0xff), (uint8_t)(hdr.size() >> 8)};
  out.insert(out.end(), hdr.begin(), hdr.end());
  const uint8_t* p = (const uint8_t*)a.data.data();
  out.insert(out.end(), p, p + a.data.size() * 4);
  return out;
}

}  // namespace veles_rt
