// archive.h - in-memory reader for workflow packages: zip (stored/deflate)
// and tar / tar.gz, via zlib (the reference uses libarchive:
// libVeles/src/workflow_archive.cc:54-171).
#pragma once
#include <cstdint>
#include <map>
#include <string>
#include <vector>

namespace veles_rt {

using Bytes = std::vector<uint8_t>;

class WorkflowArchive {
 public:
  // Loads every entry of a .zip, .tar or .tar.gz/.tgz file.
  static WorkflowArchive Load(const std::string& path);
  static WorkflowArchive FromMemory(const Bytes& data, const std::string& hint);
  bool Has(const std::string& name) const { return files_.count(name) > 0; }
  const Bytes& Get(const std::string& name) const;
  std::vector<std::string> Names() const;
  std::string Text(const std::string& name) const {
    const Bytes& b = Get(name);
    return std::string(b.begin(), b.end());
  }

 private:
  void ParseZip(const Bytes& d);
  void ParseTar(const Bytes& d);
  std::map<std::string, Bytes> files_;
};

Bytes ReadFile(const std::string& path);
Bytes Gunzip(const Bytes& in);
Bytes InflateRaw(const uint8_t* data, size_t n, size_t out_size);

}  // namespace veles_rt
