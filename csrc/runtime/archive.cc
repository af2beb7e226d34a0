#include "archive.h"

#include <zlib.h>

#include <cstring>
#include <fstream>
#include <stdexcept>

namespace veles_rt {

Bytes ReadFile(const std::string& path) {
  std::ifstream f(path, std::ios::binary);
  if (!f) throw std::runtime_error("cannot open " + path);
  return Bytes((std::istreambuf_iterator<char>(f)),
               std::istreambuf_iterator<char>());
}

static uint32_t rd32(const uint8_t* p) {
  return p[0] | (p[1] << 8) | (p[2] << 16) | ((uint32_t)p[3] << 24);
}
static uint16_t rd16(const uint8_t* p) { return p[0] | (p[1] << 8); }

Bytes InflateRaw(const uint8_t* data, size_t n, size_t out_size) {
  Bytes out(out_size);
  z_stream zs;
  std::memset(&zs, 0, sizeof(zs));
  if (inflateInit2(&zs, -MAX_WBITS) != Z_OK)
    throw std::runtime_error("inflateInit2 failed");
  zs.next_in = const_cast<uint8_t*>(data);
  zs.avail_in = (uInt)n;
  zs.next_out = out.data();
  zs.avail_out = (uInt)out.size();
  int r = inflate(&zs, Z_FINISH);
  inflateEnd(&zs);
  if (r != Z_STREAM_END) throw std::runtime_error("zip: inflate failed");
  return out;
}

Bytes Gunzip(const Bytes& in) {
  z_stream zs;
  std::memset(&zs, 0, sizeof(zs));
  if (inflateInit2(&zs, 16 + MAX_WBITS) != Z_OK)
    throw std::runtime_error("gunzip init failed");
  Bytes out;
  zs.next_in = const_cast<uint8_t*>(in.data());
  zs.avail_in = (uInt)in.size();
  uint8_t buf[1 << 16];
  int r;
  do {
    zs.next_out = buf;
    zs.avail_out = sizeof(buf);
    r = inflate(&zs, Z_NO_FLUSH);
    if (r != Z_OK && r != Z_STREAM_END) {
      inflateEnd(&zs);
      throw std::runtime_error("gunzip failed");
    }
    out.insert(out.end(), buf, buf + (sizeof(buf) - zs.avail_out));
  } while (r != Z_STREAM_END);
  inflateEnd(&zs);
  return out;
}

void WorkflowArchive::ParseZip(const Bytes& d) {
  // end of central directory record
  if (d.size() < 22) throw std::runtime_error("zip: too small");
  size_t e = d.size() - 22;
  while (true) {
    if (rd32(&d[e]) == 0x06054b50) break;
    if (e == 0) throw std::runtime_error("zip: no EOCD");
    --e;
  }
  uint16_t n = rd16(&d[e + 10]);
  size_t cd = rd32(&d[e + 16]);
  for (uint16_t i = 0; i < n; ++i) {
    if (rd32(&d[cd]) != 0x02014b50) throw std::runtime_error("zip: bad CD");
    uint16_t method = rd16(&d[cd + 10]);
    uint32_t csize = rd32(&d[cd + 20]), usize = rd32(&d[cd + 24]);
    uint16_t fnl = rd16(&d[cd + 28]), exl = rd16(&d[cd + 30]),
             cml = rd16(&d[cd + 32]);
    uint32_t lho = rd32(&d[cd + 42]);
    std::string name((const char*)&d[cd + 46], fnl);
    cd += 46 + fnl + exl + cml;
    if (rd32(&d[lho]) != 0x04034b50) throw std::runtime_error("zip: bad LH");
    size_t data = lho + 30 + rd16(&d[lho + 26]) + rd16(&d[lho + 28]);
    if (!name.empty() && name.back() == '/') continue;
    if (method == 0) {
      files_[name] = Bytes(d.begin() + data, d.begin() + data + usize);
    } else if (method == 8) {
      files_[name] = InflateRaw(&d[data], csize, usize);
    } else {
      throw std::runtime_error("zip: unsupported method for " + name);
    }
  }
}

void WorkflowArchive::ParseTar(const Bytes& d) {
  size_t p = 0;
  while (p + 512 <= d.size()) {
    const char* h = (const char*)&d[p];
    if (h[0] == 0) break;
    std::string name(h, strnlen(h, 100));
    std::string prefix(h + 345, strnlen(h + 345, 155));
    if (!prefix.empty()) name = prefix + "/" + name;
    size_t size = std::strtoull(std::string(h + 124, 12).c_str(), nullptr, 8);
    char type = h[156];
    p += 512;
    if (type == '0' || type == 0) {
      if (name.rfind("./", 0) == 0) name = name.substr(2);
      files_[name] = Bytes(d.begin() + p, d.begin() + p + size);
    }
    p += (size + 511) / 512 * 512;
  }
}

WorkflowArchive WorkflowArchive::FromMemory(const Bytes& data,
                                            const std::string& hint) {
  WorkflowArchive a;
  if (data.size() >= 4 && rd32(data.data()) == 0x04034b50) {
    a.ParseZip(data);
  } else if (data.size() >= 2 && data[0] == 0x1f && data[1] == 0x8b) {
    a.ParseTar(Gunzip(data));
  } else {
    a.ParseTar(data);
  }
  (void)hint;
  return a;
}

WorkflowArchive WorkflowArchive::Load(const std::string& path) {
  return FromMemory(ReadFile(path), path);
}

const Bytes& WorkflowArchive::Get(const std::string& name) const {
  auto it = files_.find(name);
  if (it == files_.end()) throw std::runtime_error("archive: no " + name);
  return it->second;
}

std::vector<std::string> WorkflowArchive::Names() const {
  std::vector<std::string> v;
  for (auto& kv : files_) v.push_back(kv.first);
  return v;
}

}  // namespace veles_rt
