#include "memory_optimizer.h"

#include <algorithm>
#include <numeric>
#include <utility>

namespace veles_rt {

size_t MemoryOptimizer::Optimize(std::vector<MemoryNode>* nodes) const {
  std::vector<size_t> order(nodes->size());
  std::iota(order.begin(), order.end(), 0);
  std::stable_sort(order.begin(), order.end(), [&](size_t a, size_t b) {
    return (*nodes)[a].value > (*nodes)[b].value;
  });
  std::vector<size_t> placed;
  size_t height = 0;
  for (size_t idx : order) {
    MemoryNode& n = (*nodes)[idx];
    // intervals occupied during n's lifetime
    std::vector<std::pair<size_t, size_t>> busy;
    for (size_t j : placed) {
      const MemoryNode& o = (*nodes)[j];
      if (o.time_start < n.time_finish && n.time_start < o.time_finish)
        busy.emplace_back(o.position, o.position + o.value);
    }
    std::sort(busy.begin(), busy.end());
    size_t pos = 0;
    for (auto& b : busy) {
      if (b.first >= pos + n.value) break;  // fits in the gap below b
      if (b.second > pos) pos = b.second;
    }
    n.position = pos;
    height = std::max(height, pos + n.value);
    placed.push_back(idx);
  }
  return height;
}

void MemoryOptimizer::Print(const std::vector<MemoryNode>& nodes,
                            std::ostream* out) const {
  for (auto& n : nodes)
    (*out) << n.position << '\t' << n.value << '\t' << n.time_start << '\t'
           << n.time_finish << '\n';
}

}  // namespace veles_rt
