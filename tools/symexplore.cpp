// Dev tool: explore the symbolic-analysis parameters (ND leaf size, relaxed amalgamation) on a
// block pattern file ("nb nnz" then "i j" upper pairs) and report the quantities the GPU factor
// time follows: level-synchronous panel steps, critical path, flops, fronts.
// g++ -O2 -std=c++17 -I g2o_amd/csrc tools/symexplore.cpp g2o_amd/csrc/symbolic.cpp -o /tmp/symexplore
#include <algorithm>
#include <cstdio>
#include <vector>

#include "symbolic.hpp"

using namespace g2ohip;

int main(int argc, char** argv) {
  if (argc < 2) return 1;
  FILE* f = fopen(argv[1], "r");
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
  printf("%6s %6s %5s | %8s %8s %5s %4s %6s %6s %6s %8s\n", "leaf", "relax", "rmax", "GFLOP", "nnzL(M)", "nsn", "lev",
         "lsteps", "crit", "maxm", "model_ms");
  for (int leaf : {8, 16, 24, 32, 48, 64, 96, 128, 192, 256, 400, 1000})
    for (double relax : {0.25})
      for (int rmax : {16, 64, 1000}) {
        std::vector<int> ord = nested_dissection(P, leaf);
        Symbolic S = analyze(P, ord, relax, rmax);
        // level-synchronous panel steps and critical path in panel steps
        int lsteps = 0;
        for (auto& lv : S.levels) {
          int mx = 0;
          for (int s : lv) mx = std::max(mx, (S.sn[s].ns + 31) / 32);
          lsteps += mx;
        }
        std::vector<int> crit(S.sn.size(), 0);
        int cmax = 0;
        for (size_t s = 0; s < S.sn.size(); ++s) {  // children first (postorder)
          int c = 0;
          for (int k = S.children_ptr[s]; k < S.children_ptr[s + 1]; ++k) c = std::max(c, crit[S.children[k]]);
          crit[s] = c + (S.sn[s].ns + 31) / 32;
          cmax = std::max(cmax, crit[s]);
        }
        // crude GPU model: 15 us per panel step, 80 us per level, 20 TF/s on the flops
        const double model = lsteps * 15e-3 + S.num_levels * 80e-3 + S.flops / 20e12 * 1e3;
        printf("%6d %6.2f %5d | %8.3f %8.2f %5zu %4d %6d %6d %6d %8.3f\n", leaf, relax, rmax, S.flops * 1e-9,
               S.nnzL * 1e-6, S.sn.size(), S.num_levels, lsteps, cmax, S.max_front, model);
      }
  return 0;
}
