// Dev tool: the supernodal tree the symbolic analysis builds for a block pattern, level by level, and the quantities
// the GPU factor time follows (panel steps per level, flops per level, fronts). Reads a pattern file ("nb nnz" then
// "i j" pairs, i != j, either triangle) as tools/dump_pattern.py writes it.
//   g++ -O2 -std=c++17 -fopenmp -I g2o_amd/csrc tools/symexplore.cpp g2o_amd/csrc/symbolic.cpp -o /tmp/symexplore
//   /tmp/symexplore PATTERN [order]      order: nd (default: the cost-model choice), natural, nd-plain
#include <algorithm>
#include <cstdio>
#include <cstring>
#include <numeric>
#include <vector>

#include "symbolic.hpp"

using namespace g2ohip;

static void report(const char* name, const Symbolic& S) {
  printf("== %s: n %d, %zu supernodes, %d levels, GFLOP %.3f, nnzL %.2fM, max front %d, band leaf %d, model %.3f ms\n",
         name, S.n, S.sn.size(), S.num_levels, S.flops * 1e-9, S.nnzL * 1e-6, S.max_front, S.band_leaf,
         gpu_cost(S) * 1e3);
  int steps = 0;
  for (size_t l = 0; l < S.levels.size(); ++l) {
    const auto& lv = S.levels[l];
    int mx = 0, mm = 0;
    double fl = 0;
    for (int s : lv) {
      const Supernode& q = S.sn[s];
      mx = std::max(mx, q.ns);
      mm = std::max(mm, q.ns + q.nr);
      const double m = q.ns + q.nr;
      if (q.env_off >= 0) {  // band supernode: envelope count
        std::vector<int> hist(q.ns + 1, 0);
        for (int r = 0; r < q.ns + q.nr; ++r) hist[std::min(S.fnz[q.env_off + r], q.ns)]++;
        int le = 0;
        for (int c = 0; c < q.ns; ++c) { le += hist[c]; fl += (double)(le - c) * (le - c); }
      } else {
        for (int c = 0; c < q.ns; ++c) fl += (m - c) * (m - c);
      }
    }
    steps += (mx + 31) / 32;
    printf("  level %2zu: %4zu fronts, max ns %5d (%3d steps), max m %5d, GFLOP %7.3f\n", l, lv.size(), mx, (mx + 31) / 32,
           mm, fl * 1e-9);
  }
  printf("  panel steps (level-synchronous): %d\n", steps);
}

int main(int argc, char** argv) {
  if (argc < 2) return 1;
  FILE* f = fopen(argv[1], "r");
  if (!f) return 1;
  int nb, nnz;
  if (fscanf(f, "%d %d", &nb, &nnz) != 2) return 1;
  std::vector<std::vector<int>> adj(nb);
  for (int k = 0; k < nnz; ++k) {
    int a, b;
    if (fscanf(f, "%d %d", &a, &b) != 2) return 1;
    adj[a].push_back(b);
    adj[b].push_back(a);
  }
  fclose(f);
  BlockPattern P;
  P.nb = nb;
  P.dim.assign(nb, 6);
  P.offset.resize(nb + 1);
  for (int k = 0; k <= nb; ++k) P.offset[k] = 6 * k;
  P.adjp.assign(nb + 1, 0);
  for (int k = 0; k < nb; ++k) {
    std::sort(adj[k].begin(), adj[k].end());
    adj[k].erase(std::unique(adj[k].begin(), adj[k].end()), adj[k].end());
    P.adjp[k + 1] = P.adjp[k] + (int)adj[k].size();
    P.adji.insert(P.adji.end(), adj[k].begin(), adj[k].end());
  }
  const char* which = argc > 2 ? argv[2] : "nd";
  if (!strcmp(which, "natural")) {
    std::vector<int> ord(nb);
    std::iota(ord.begin(), ord.end(), 0);
    report("natural", analyze(P, ord));
  } else if (!strcmp(which, "nd-plain")) {
    report("nd-plain", analyze(P, nested_dissection(P, 48, false)));
  } else {
    report("nd (cost-model choice)", analyze(P));
  }
  return 0;
}
