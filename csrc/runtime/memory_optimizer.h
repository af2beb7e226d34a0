// memory_optimizer.h - plans one arena for all unit outputs.
// Behaviour of libVeles/src/memory_optimizer.cc:38-110: nodes
// [time_start, time_finish) x size, placed biggest first at the lowest
// offset that overlaps no time-overlapping node; returns the arena height.
#pragma once
#include <cstddef>
#include <ostream>
#include <vector>

namespace veles_rt {

struct MemoryNode {
  int time_start = 0;
  int time_finish = 0;   // exclusive
  size_t value = 0;      // size
  size_t position = 0;   // planned offset
};

class MemoryOptimizer {
 public:
  size_t Optimize(std::vector<MemoryNode>* nodes) const;
  void Print(const std::vector<MemoryNode>& nodes, std::ostream* out) const;
};

}  // namespace veles_rt
