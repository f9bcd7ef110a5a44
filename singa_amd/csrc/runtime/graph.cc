// Layer DAG: DFS topological sort + node-link JSON (reference C19,
// src/utils/graph.cc:8-101).  Sort order is deterministic: sources are
// visited in insertion order and each node is emitted after all of its
// predecessors.
#include <algorithm>
#include <functional>
#include <sstream>
#include <stdexcept>

#include "runtime.h"

namespace sgrt {

int Graph::AddNode(const std::string& name) {
  auto it = index.find(name);
  if (it != index.end()) return it->second;
  int id = (int)names.size();
  names.push_back(name);
  dst.emplace_back();
  index[name] = id;
  return id;
}

void Graph::AddEdge(const std::string& s, const std::string& d) {
  int a = AddNode(s), b = AddNode(d);
  if (std::find(dst[a].begin(), dst[a].end(), b) == dst[a].end()) dst[a].push_back(b);
}

std::vector<std::string> Graph::Sort() const {
  const int n = (int)names.size();
  std::vector<int> state(n, 0);  // 0 new, 1 on stack, 2 done
  std::vector<int> post;
  std::function<void(int)> dfs = [&](int u) {
    state[u] = 1;
    for (int v : dst[u]) {
      if (state[v] == 1) throw std::runtime_error("cycle in layer graph at " + names[v]);
      if (state[v] == 0) dfs(v);
    }
    state[u] = 2;
    post.push_back(u);
  };
  // visit in reverse insertion order so the reversed post-order keeps the
  // user's layer order whenever the DAG allows it
  for (int u = n - 1; u >= 0; --u)
    if (state[u] == 0) dfs(u);
  std::reverse(post.begin(), post.end());
  std::vector<std::string> out;
  out.reserve(n);
  for (int u : post) out.push_back(names[u]);
  return out;
}

std::string Graph::ToJson(const std::vector<int>& color) const {
  static const char* palette[] = {"red", "blue", "green", "orange", "purple", "cyan", "magenta", "black"};
  std::ostringstream os;
  os << "{\"directed\":1,\"nodes\":[";
  for (size_t i = 0; i < names.size(); ++i) {
    int c = i < color.size() ? color[i] : 0;
    os << (i ? "," : "") << "{\"id\":\"" << names[i] << "\",\"color\":\"" << palette[(c % 8 + 8) % 8]
       << "\",\"shape\":\"box\"}";
  }
  os << "],\"links\":[";
  bool first = true;
  for (size_t i = 0; i < names.size(); ++i)
    for (int j : dst[i]) {
      os << (first ? "" : ",") << "{\"source\":\"" << names[i] << "\",\"target\":\"" << names[j]
         << "\",\"color\":\"black\"}";
      first = false;
    }
  os << "]}";
  return os.str();
}

}  // namespace sgrt
