// Host-side symbolic analysis (see symbolic.hpp).
#include "symbolic.hpp"

#include <algorithm>
#include <cassert>
#include <cstdio>
#include <cstdlib>
#include <numeric>
#include <stdexcept>

namespace g2ohip {
namespace {

struct NDState {
  const BlockPattern& P;
  std::vector<int> part;   // subgraph id per vertex
  std::vector<int> order;  // output order (new -> old)
  std::vector<int> dist, mark;
  int next_id = 1;
  int leaf;
  bool do_refine, do_windows, part_degree;
  std::vector<int> rank;  // scratch: position of a vertex in its part's BFS visitation order
  const bool no_small_windows = getenv("G2OHIP_ND_NO_SMALLWIN") != nullptr;  // dev A/B
  int band_leaf = 0;                  // parts of at most this many blocks become band leaves (0: off)
  std::vector<int>* groups = nullptr;  // band-leaf group per block
  int next_group = 0;
  explicit NDState(const BlockPattern& p, int leaf_, bool refine_, bool windows_, bool part_degree_)
      : P(p), part(p.nb, 0), dist(p.nb, -1), mark(p.nb, 0), leaf(leaf_), do_refine(refine_), do_windows(windows_),
        part_degree(part_degree_), rank(p.nb, -1) {}

  // BFS visitation order of a part's level structure, each level's vertices with fewer neighbours in the next level
  // first (ties: discovery order): on a band the prefix of this order grows one position at a time
  std::vector<int> level_order(const std::vector<std::vector<int>>& lv, int id) {
    const int h = (int)lv.size();
    std::vector<int> ord;
    for (int k = 0; k < h; ++k) {
      for (int v : lv[k]) rank[v] = k;  // level index, temporarily
      ord.insert(ord.end(), lv[k].begin(), lv[k].end());
    }
    for (int k = 0, base = 0; k < h; base += (int)lv[k].size(), ++k) {
      std::vector<std::pair<int, int>> key(lv[k].size());
      for (size_t q = 0; q < lv[k].size(); ++q) {
        const int v = lv[k][q];
        int nn = 0;
        for (int p = P.adjp[v]; p < P.adjp[v + 1]; ++p) nn += part[P.adji[p]] == id && rank[P.adji[p]] == k + 1;
        key[q] = {nn, (int)q};
      }
      std::sort(key.begin(), key.end());
      for (size_t q = 0; q < key.size(); ++q) ord[base + q] = lv[k][key[q].second];
    }
    for (int v : ord) rank[v] = -1;
    return ord;
  }

  // Exact minimum-degree elimination on a small vertex set.
  void min_degree(const std::vector<int>& vs) {
    const int n = (int)vs.size();
    if (n == 0) return;
    std::vector<int> local(P.nb, -1);
    for (int k = 0; k < n; ++k) local[vs[k]] = k;
    std::vector<std::vector<char>> adj(n, std::vector<char>(n, 0));
    for (int k = 0; k < n; ++k) {
      int v = vs[k];
      for (int p = P.adjp[v]; p < P.adjp[v + 1]; ++p) {
        int u = P.adji[p];
        if (part[u] == part[v] && local[u] >= 0) adj[k][local[u]] = 1;
      }
    }
    std::vector<char> alive(n, 1);
    for (int step = 0; step < n; ++step) {
      int best = -1, bd = 1 << 30;
      for (int k = 0; k < n; ++k)
        if (alive[k]) {
          int d = 0;
          for (int u = 0; u < n; ++u) d += alive[u] && adj[k][u];
          if (d < bd) { bd = d; best = k; }
        }
      alive[best] = 0;
      order.push_back(vs[best]);
      std::vector<int> nb;
      for (int u = 0; u < n; ++u)
        if (alive[u] && adj[best][u]) nb.push_back(u);
      for (int a : nb)
        for (int b : nb)
          if (a != b) adj[a][b] = 1;
    }
  }

  // BFS restricted to the subgraph `id`; returns level lists.
  std::vector<std::vector<int>> bfs_levels(int root, int id) {
    std::vector<std::vector<int>> levels;
    std::vector<int> cur{root}, touched{root};
    dist[root] = 0;
    while (!cur.empty()) {
      levels.push_back(cur);
      std::vector<int> nxt;
      for (int v : cur)
        for (int p = P.adjp[v]; p < P.adjp[v + 1]; ++p) {
          int u = P.adji[p];
          if (part[u] == id && dist[u] < 0) {
            dist[u] = dist[v] + 1;
            nxt.push_back(u);
            touched.push_back(u);
          }
        }
      cur.swap(nxt);
    }
    for (int v : touched) dist[v] = -1;
    return levels;
  }

  // Greedy vertex-separator refinement (Fiduccia-Mattheyses style, unit weights, positive or
  // balance-improving zero gains only): a separator vertex moves to side X when that pulls fewer than
  // one (gain > 0) or exactly one (gain 0, X the smaller side) of its neighbours on the other side
  // into the separator. Level-structure separators are ragged; this straightens them.
  void refine(std::vector<int>& S, int idA, int idB, int idS, int N, long long cntA, long long cntB) {
    auto count_side = [&](int v, int id) {
      int c = 0;
      for (int p = P.adjp[v]; p < P.adjp[v + 1]; ++p) c += part[P.adji[p]] == id;
      return c;
    };
    for (int pass = 0; pass < 8; ++pass) {
      bool changed = false;
      std::vector<int> next;
      next.reserve(S.size());
      for (size_t k = 0; k < S.size(); ++k) {
        const int v = S[k];
        if (part[v] != idS) continue;
        const int inA = count_side(v, idA), inB = count_side(v, idB);
        const int gA = 1 - inB, gB = 1 - inA;  // separator shrinkage when v moves to A / to B
        int to = -1;
        if (gA > 0 || gB > 0) to = gA >= gB ? idA : idB;
        else if (gA == 0 && gB == 0) to = cntA <= cntB ? idA : idB;
        else if (gA == 0 && cntA < cntB) to = idA;
        else if (gB == 0 && cntB < cntA) to = idB;
        if (to < 0) { next.push_back(v); continue; }
        const int other = to == idA ? idB : idA;
        if ((to == idA ? cntA : cntB) + 1 > (long long)(0.6 * N)) { next.push_back(v); continue; }
        part[v] = to;
        (to == idA ? cntA : cntB) += 1;
        for (int p = P.adjp[v]; p < P.adjp[v + 1]; ++p) {
          const int u = P.adji[p];
          if (part[u] == other) {
            part[u] = idS;
            (other == idA ? cntA : cntB) -= 1;
            next.push_back(u);
          }
        }
        changed = true;
      }
      S.swap(next);
      if (!changed) break;
    }
    std::sort(S.begin(), S.end());
    S.erase(std::unique(S.begin(), S.end()), S.end());
    S.erase(std::remove_if(S.begin(), S.end(), [&](int v) { return part[v] != idS; }), S.end());
  }

  void run(std::vector<int> vs, int id) {
    if ((int)vs.size() <= leaf) {
      min_degree(vs);
      return;
    }
    // connected components inside the subgraph
    {
      auto lv = bfs_levels(vs[0], id);
      size_t cnt = 0;
      for (auto& l : lv) cnt += l.size();
      if (cnt < vs.size()) {
        int cid = next_id++;
        for (auto& l : lv)
          for (int v : l) part[v] = cid;
        std::vector<int> a, rest;
        for (int v : vs) (part[v] == cid ? a : rest).push_back(v);
        int rid = next_id++;
        for (int v : rest) part[v] = rid;
        run(a, cid);
        run(rest, rid);
        return;
      }
    }
    // pseudo-peripheral root: repeat BFS from the last level's min-degree vertex
    int root = vs[0];
    int depth = 0;
    for (int it = 0; it < 4; ++it) {
      auto lv = bfs_levels(root, id);
      if ((int)lv.size() <= depth) break;
      depth = (int)lv.size();
      int best = lv.back()[0], bd = 1 << 30;
      for (int v : lv.back()) {
        int d = 0;  // degree inside the part (global degrees do not tell a part's ends from its middle)
        if (part_degree)
          for (int p = P.adjp[v]; p < P.adjp[v + 1]; ++p) d += part[P.adji[p]] == id;
        else
          d = P.adjp[v + 1] - P.adjp[v];
        if (d < bd) { bd = d; best = v; }
      }
      root = best;
    }
    auto lv = bfs_levels(root, id);
    const int h = (int)lv.size();
    if (h < 3) {  // nearly complete graph: no useful separator
      min_degree(vs);
      return;
    }
    const int N = (int)vs.size();
    if (band_leaf > 0 && N <= band_leaf && groups) {
      // band leaf: the sequential (band) order from one end; the analysis makes it one band supernode
      const int gid = next_group++;
      for (int v : level_order(lv, id)) {
        order.push_back(v);
        (*groups)[v] = gid;
      }
      return;
    }
    std::vector<int> before(h + 1, 0);
    for (int k = 0; k < h; ++k) before[k + 1] = before[k] + (int)lv[k].size();
    int kbest = -1;
    double best = 1e300;
    for (int k = 1; k < h - 1; ++k) {
      const int a = before[k], b = N - before[k + 1];
      if (a < 0.2 * N || b < 0.2 * N) continue;
      const double cost = (double)lv[k].size() * (1.0 + std::abs(a - b) / (double)N);
      if (cost < best) { best = cost; kbest = k; }
    }
    const int kbest_balanced = kbest;
    if (kbest < 0) {  // fall back to the median level
      for (int k = 1; k < h - 1; ++k)
        if (before[k + 1] >= N / 2) { kbest = k; break; }
      if (kbest < 0) kbest = h / 2;
    }
    // window separators (position-aware): in the BFS visitation order, the vertices [x, reach(x)] —
    // everything ranked after x that a vertex ranked before x touches — separate [0, x) from the rest, at any
    // offset x, not only at BFS-level starts. On band-like graphs (C4's cameras: a path of one-bandwidth
    // BFS levels) a level separator can only cut at multiples of the bandwidth, so the halves come out up to
    // one bandwidth apart and the tree one level deeper than an exact split; the window at the vertex-count
    // middle has the same size and balances exactly.
    if (do_windows) {
      // within a level, vertices with fewer neighbours in the next level first (ties: discovery order), so the
      // reach of a prefix grows gradually instead of jumping to the end of the next level
      const std::vector<int> ord = level_order(lv, id);
      for (int k = 0; k < N; ++k) rank[ord[k]] = k;
      // balanced windows as the level candidates (both sides >= 20 %); failing that, on a part too small to
      // split in balance (a leaf-sized band segment a bit wider than the bandwidth), the window that shortens
      // the chain through the part (separator + larger side < whole part), so leaves come out small instead of
      // one bandwidth plus a sliver
      int reach = -1, xbest = -1, wend = -1, xs = -1, ws = -1;
      double wcost = best, chain = 0.97 * N;
      for (int x = 1; x < N - 1; ++x) {
        const int v = ord[x - 1];
        for (int p = P.adjp[v]; p < P.adjp[v + 1]; ++p) {
          const int u = P.adji[p];
          if (part[u] == id) reach = std::max(reach, rank[u]);
        }
        if (reach < x || reach >= N - 1) continue;  // disconnected prefix / nothing left on the far side
        const int a = x, b = N - 1 - reach, w = reach - x + 1;
        if (a >= 0.2 * N && b >= 0.2 * N) {
          const double cost = (double)w * (1.0 + std::abs(a - b) / (double)N);
          if (cost < wcost * (1.0 - 1e-9)) { wcost = cost; xbest = x; wend = reach; }
        }
        if (w + std::max(a, b) < chain) { chain = w + std::max(a, b); xs = x; ws = reach; }
      }
      if (xbest < 0 && kbest_balanced < 0 && xs >= 0 && !no_small_windows) { xbest = xs; wend = ws; }
      for (int v : ord) rank[v] = -1;
      if (xbest >= 0) {
        int idA = next_id++, idB = next_id++, idS = next_id++;
        std::vector<int> A(ord.begin(), ord.begin() + xbest), S(ord.begin() + xbest, ord.begin() + wend + 1),
            B(ord.begin() + wend + 1, ord.end());
        for (int v : A) part[v] = idA;
        for (int v : B) part[v] = idB;
        for (int v : S) part[v] = idS;
        run(A, idA);
        run(B, idB);
        std::sort(S.begin(), S.end());
        for (int v : S) order.push_back(v);
        return;
      }
    }
    // refine: separator = vertices of level k with a neighbour in level k+1
    int idA = next_id++, idB = next_id++, idS = next_id++;
    for (int k = 0; k < h; ++k)
      for (int v : lv[k]) part[v] = k < kbest ? idA : (k == kbest ? idS : idB);
    std::vector<int> A, B, S;
    for (int v : lv[kbest]) {
      bool touchesB = false;
      for (int p = P.adjp[v]; p < P.adjp[v + 1] && !touchesB; ++p) touchesB = part[P.adji[p]] == idB;
      if (touchesB) S.push_back(v);
      else { part[v] = idA; }
    }
    {
      long long na = 0, nbb = 0;
      for (int k = 0; k < h; ++k)
        for (int v : lv[k]) { na += part[v] == idA; nbb += part[v] == idB; }
      if (do_refine) refine(S, idA, idB, idS, N, na, nbb);
    }
    for (int k = 0; k < h; ++k)
      for (int v : lv[k]) {
        if (part[v] == idA) A.push_back(v);
        else if (part[v] == idB) B.push_back(v);
      }
    run(A, idA);
    run(B, idB);
    std::sort(S.begin(), S.end());
    for (int v : S) order.push_back(v);
  }
};

}  // namespace

BlockPattern block_pattern(int nblocks, int bdim, const std::vector<int>& bi, const std::vector<int>& bj) {
  BlockPattern P;
  P.nb = nblocks;
  P.dim.assign(nblocks, bdim);
  P.offset.resize(nblocks + 1);
  for (int k = 0; k <= nblocks; ++k) P.offset[k] = k * bdim;
  std::vector<int> deg(nblocks, 0);
  for (size_t t = 0; t < bi.size(); ++t)
    if (bi[t] != bj[t]) { deg[bi[t]]++; deg[bj[t]]++; }
  P.adjp.assign(nblocks + 1, 0);
  for (int k = 0; k < nblocks; ++k) P.adjp[k + 1] = P.adjp[k] + deg[k];
  P.adji.assign(P.adjp[nblocks], 0);
  std::vector<int> fill(P.adjp.begin(), P.adjp.end() - 1);
  for (size_t t = 0; t < bi.size(); ++t)
    if (bi[t] != bj[t]) { P.adji[fill[bi[t]]++] = bj[t]; P.adji[fill[bj[t]]++] = bi[t]; }
  return P;
}

std::vector<int> nested_dissection(const BlockPattern& P, int leaf_size, bool refine, bool windows, bool part_degree,
                                   int band_leaf, std::vector<int>* groups) {
  NDState st(P, std::max(leaf_size, 1), refine, windows, part_degree || windows);
  if (groups) groups->assign(P.nb, -1);
  st.band_leaf = band_leaf;
  st.groups = groups;
  std::vector<int> all(P.nb);
  std::iota(all.begin(), all.end(), 0);
  st.run(all, 0);
  if ((int)st.order.size() != P.nb) throw std::runtime_error("nested_dissection: incomplete order");
  return st.order;
}

double gpu_cost(const Symbolic& S) {
  int lsteps = 0;
  for (auto& lv : S.levels) {
    int mx = 0;
    for (int s : lv) mx = std::max(mx, (S.sn[s].ns + 31) / 32);
    lsteps += mx;
  }
  return S.flops / 30e12 + lsteps * 12e-6;
}

Symbolic analyze(const BlockPattern& P, std::vector<int> bperm, double relax, int relax_max_blocks,
                 const std::vector<int>* groups) {
  const int nb = P.nb;
  if (bperm.empty() && nb > 0) {
    if (const char* rm = getenv("G2OHIP_ND_RMAX")) relax_max_blocks = atoi(rm);  // dev A/B
    // nested dissection variants; the ordering with the lowest modelled GPU factor time (flops at the MFMA
    // rate + the level-synchronous panel-step chain) wins, the plain one unless another is clearly (5 %) better:
    // with / without separator refinement, pseudo-peripheral roots by global or by in-part degree, and
    // position-aware window separators (see NDState::run)
    Symbolic best = analyze(P, nested_dissection(P, 48, false), relax, relax_max_blocks);
    if (getenv("G2OHIP_ND_PLAIN")) return best;  // dev A/B: round-1 ordering
    const double base = gpu_cost(best);
    double bc = base;
    const bool var[4][3] = {{true, false, false}, {false, false, true}, {true, false, true}, {false, true, true}};
    int bv = -1;  // the variant kept (-1: plain)
    for (int k = 0; k < 4; ++k) {
      const auto& v = var[k];
      Symbolic c = analyze(P, nested_dissection(P, 48, v[0], v[1], v[2]), relax, relax_max_blocks);
      const double cc = gpu_cost(c);
      if (cc < 0.95 * base && cc < bc) { bc = cc; best = std::move(c); bv = k; }
    }
    // band leaves (hybrid ordering): the kept variant's dissection down to parts of at most `bl` blocks, each such
    // part that is a long band ordered sequentially and factored as one band supernode — the reference's own
    // sequential order inside the leaves (fewer flops) for a chain no longer than the dissection levels it replaces
    // Off unless G2OHIP_BAND_LEAF is set (N: force leaves of N blocks, -1: let the cost model choose): measured at C5
    // (r04b, profiles/r04b_c5_bandleaf_factor_levels.txt) the 256-block band leaves cut the flops 18.9 -> 14.2 GFLOP
    // but their level took 1.21 ms against ~0.7 for the three dissection levels they replace (every panel of a band
    // leaf updates its whole border rows, 41 rank-32 passes instead of 12): factor 1.84 -> 1.93 ms
    const char* eb = getenv("G2OHIP_BAND_LEAF");
    const int force_bl = eb ? atoi(eb) : 0;
    if (force_bl != 0) {
      const bool* v = bv >= 0 ? var[bv] : nullptr;
      for (int bl : {96, 128, 192, 256, 384}) {
        if (force_bl > 0 && bl != 96) break;
        const int leafb = force_bl > 0 ? force_bl : bl;
        if (leafb >= nb) break;
        std::vector<int> grp;
        std::vector<int> ord = nested_dissection(P, 48, v ? v[0] : false, v ? v[1] : false, v ? v[2] : false, leafb, &grp);
        Symbolic c = analyze(P, ord, relax, relax_max_blocks, &grp);
        c.band_leaf = leafb;
        const double cc = gpu_cost(c);
        if (force_bl > 0 || cc < 0.95 * bc) { bc = cc; best = std::move(c); }
      }
    }
    return best;
  }
  Symbolic S;
  S.nb = nb;
  S.n = nb ? P.offset[nb] : 0;
  if (nb == 0) return S;
  std::vector<int> bpinv(nb);
  for (int k = 0; k < nb; ++k) bpinv[bperm[k]] = k;

  auto compute_etree = [&](const std::vector<int>& perm, const std::vector<int>& pinv) {
    std::vector<int> parent(nb, -1), anc(nb, -1);
    for (int k = 0; k < nb; ++k) {
      const int old = perm[k];
      for (int p = P.adjp[old]; p < P.adjp[old + 1]; ++p) {
        int i = pinv[P.adji[p]];
        if (i >= k) continue;
        while (i != -1 && i < k) {  // Liu's algorithm with path compression (cf. cs_etree.c)
          int nxt = anc[i];
          anc[i] = k;
          if (nxt == -1) parent[i] = k;
          i = nxt;
        }
      }
    }
    return parent;
  };
  // postorder the etree so supernodes are contiguous
  {
    std::vector<int> parent = compute_etree(bperm, bpinv);
    std::vector<int> head(nb, -1), next(nb, -1), post;
    post.reserve(nb);
    for (int j = nb - 1; j >= 0; --j)
      if (parent[j] != -1) { next[j] = head[parent[j]]; head[parent[j]] = j; }
    std::vector<int> stack;
    for (int j = 0; j < nb; ++j) {
      if (parent[j] != -1) continue;
      stack.push_back(j);
      while (!stack.empty()) {
        int p = stack.back();
        int i = head[p];
        if (i == -1) { stack.pop_back(); post.push_back(p); }
        else { head[p] = next[i]; stack.push_back(i); }
      }
    }
    std::vector<int> nperm(nb);
    for (int k = 0; k < nb; ++k) nperm[k] = bperm[post[k]];
    bperm.swap(nperm);
    for (int k = 0; k < nb; ++k) bpinv[bperm[k]] = k;
  }
  std::vector<int> parent = compute_etree(bperm, bpinv);
  S.bperm = bperm;
  S.bpinv = bpinv;
  S.bdim_new.resize(nb);
  S.boffset_new.assign(nb + 1, 0);
  for (int k = 0; k < nb; ++k) {
    S.bdim_new[k] = P.dim[bperm[k]];
    S.boffset_new[k + 1] = S.boffset_new[k] + S.bdim_new[k];
  }
  S.perm.resize(S.n);
  S.pinv.resize(S.n);
  for (int k = 0; k < nb; ++k)
    for (int d = 0; d < S.bdim_new[k]; ++d) {
      S.perm[S.boffset_new[k] + d] = P.offset[bperm[k]] + d;
      S.pinv[P.offset[bperm[k]] + d] = S.boffset_new[k] + d;
    }

  // block structure of L (rows > j), by merging children
  std::vector<std::vector<int>> st(nb);
  std::vector<int> nchild(nb, 0), mark(nb, -1);
  std::vector<std::vector<int>> kids(nb);
  for (int j = 0; j < nb; ++j)
    if (parent[j] != -1) { nchild[parent[j]]++; kids[parent[j]].push_back(j); }
  for (int j = 0; j < nb; ++j) {
    std::vector<int>& s = st[j];
    mark[j] = j;
    const int old = bperm[j];
    for (int p = P.adjp[old]; p < P.adjp[old + 1]; ++p) {
      int i = bpinv[P.adji[p]];
      if (i > j && mark[i] != j) { mark[i] = j; s.push_back(i); }
    }
    for (int c : kids[j]) {
      for (int i : st[c])
        if (i != j && mark[i] != j) { mark[i] = j; s.push_back(i); }
    }
    std::sort(s.begin(), s.end());
  }
  // fundamental supernodes
  std::vector<int> sn_start;
  for (int j = 0; j < nb; ++j) {
    bool merge = j > 0 && parent[j - 1] == j && nchild[j] == 1 && st[j - 1].size() == st[j].size() + 1;
    if (!merge) sn_start.push_back(j);
  }
  sn_start.push_back(nb);
  struct Tmp { int b0, b1; std::vector<int> rows; };  // rows: block rows >= b1
  std::vector<Tmp> sns;
  for (size_t s = 0; s + 1 < sn_start.size(); ++s) {
    Tmp t;
    t.b0 = sn_start[s];
    t.b1 = sn_start[s + 1];
    for (int i : st[t.b1 - 1]) t.rows.push_back(i);  // struct of the last column = rows below
    sns.push_back(std::move(t));
  }
  // relaxed amalgamation: merge a supernode into the next one when it is that one's
  // (postorder-last) child and the added explicit zeros stay small; blocks of one band-leaf group are merged whole
  auto grp_of = [&](int newb) { return groups ? (*groups)[bperm[newb]] : -1; };
  // small leaf absorption: a childless supernode at most 1/8 the width of its parent is merged into it even when it is
  // not the parent's postorder-last child. A dissection's last split of a part barely wider than its separator leaves
  // two slivers (C4: 3-block leaves beside a 63-block window separator) whose contribution blocks are as large as the
  // separator's front: one level of extend-add, panel step and contribution launches plus that traffic, for a few
  // columns. C4: 31 -> 15 supernodes, 5 -> 4 levels, factor 0.752 -> 0.733 ms; C5: 7 -> 6 levels, 84 -> 73 panel
  // steps, factor 1.84 -> 1.71 ms; C2 / C3 unchanged (profiles/r04_ab_absorb.log). G2OHIP_ND_ABSORB=k sets the ratio,
  // 0 turns it off (dev A/B).
  const char* absorb_env = getenv("G2OHIP_ND_ABSORB");
  const int absorb = absorb_env ? atoi(absorb_env) : 8;
  auto childless = [&](const Tmp& c) {
    for (int b = c.b0; b < c.b1; ++b)
      for (int k : kids[b])
        if (k < c.b0) return false;
    return true;
  };
  {
    std::vector<Tmp> out;
    for (auto& t : sns) {
      while (absorb > 0 && !out.empty()) {
        const Tmp& c = out.back();
        const int last = c.b1 - 1;
        if (c.b1 != t.b0 || parent[last] < t.b0 || parent[last] >= t.b1) break;
        if ((c.b1 - c.b0) * absorb > t.b1 - t.b0 || !childless(c)) break;
        if (grp_of(c.b0) >= 0 || grp_of(t.b0) >= 0) break;
        std::vector<int> rows;  // the merged front's rows: t's, plus any of c's beyond t (none in an exact etree)
        for (int i : c.rows)
          if (i >= t.b1) rows.push_back(i);
        rows.insert(rows.end(), t.rows.begin(), t.rows.end());
        std::sort(rows.begin(), rows.end());
        rows.erase(std::unique(rows.begin(), rows.end()), rows.end());
        t.b0 = c.b0;
        t.rows.swap(rows);
        out.pop_back();
      }
      if (!out.empty()) {
        Tmp& c = out.back();
        const int last = c.b1 - 1;
        if (parent[last] == t.b0) {
          const double wc = c.b1 - c.b0, wp = t.b1 - t.b0, w = wc + wp;
          const double rp = (double)t.rows.size(), rc = (double)c.rows.size();
          const double zeros = wc * (wp + rp - rc);
          const double total = w * (w + 1) / 2 + w * rp;
          const bool band = grp_of(c.b0) >= 0 && grp_of(c.b0) == grp_of(t.b0);
          if (band || (w <= relax_max_blocks && zeros <= relax * total)) {
            c.b1 = t.b1;
            c.rows = t.rows;
            continue;
          }
        }
      }
      out.push_back(std::move(t));
    }
    sns.swap(out);
  }
  const int ns_count = (int)sns.size();
  // envelopes of the band supernodes (a group merged into a supernode of more than one block): per front row the first
  // own column with a structural nonzero (see Supernode::env_off)
  std::vector<std::vector<int>> env(ns_count);
  for (int s = 0; s < ns_count; ++s) {
    const Tmp& t = sns[s];
    if (t.b1 - t.b0 < 2 || grp_of(t.b0) < 0 || grp_of(t.b0) != grp_of(t.b1 - 1)) continue;
    const int c0 = S.boffset_new[t.b0], ns = S.boffset_new[t.b1] - c0;
    std::vector<int> roff(t.rows.size() + 1, 0);
    for (size_t q = 0; q < t.rows.size(); ++q) roff[q + 1] = roff[q] + S.bdim_new[t.rows[q]];
    std::vector<int>& f = env[s];
    f.assign(ns + roff.back(), 1 << 30);
    auto setb = [&](int bi, int cb) {  // block row bi of the front gets column cb
      int r0, d = S.bdim_new[bi];
      if (bi < t.b1) r0 = S.boffset_new[bi] - c0;
      else r0 = ns + roff[std::lower_bound(t.rows.begin(), t.rows.end(), bi) - t.rows.begin()];
      for (int r = r0; r < r0 + d; ++r) f[r] = std::min(f[r], cb);
    };
    for (int b = t.b0; b < t.b1; ++b) {
      const int cb = S.boffset_new[b] - c0;
      setb(b, cb);
      for (int i : st[b]) setb(i, cb);
    }
  }
  std::vector<std::vector<int>>().swap(st);
  S.block_sn.assign(nb, -1);
  for (int s = 0; s < ns_count; ++s)
    for (int j = sns[s].b0; j < sns[s].b1; ++j) S.block_sn[j] = s;
  S.sn.resize(ns_count);
  int64_t roff = 0, foff = 0, voff = 0;
  for (int s = 0; s < ns_count; ++s) {
    Supernode& q = S.sn[s];
    q.b0 = sns[s].b0;
    q.b1 = sns[s].b1;
    q.c0 = S.boffset_new[q.b0];
    q.ns = S.boffset_new[q.b1] - q.c0;
    q.nr = 0;
    for (int bi : sns[s].rows) q.nr += S.bdim_new[bi];
    const int last = q.b1 - 1;
    q.parent = parent[last] == -1 ? -1 : S.block_sn[parent[last]];
    q.rows_off = roff;
    for (int bi : sns[s].rows)
      for (int d = 0; d < S.bdim_new[bi]; ++d) S.rows.push_back(S.boffset_new[bi] + d);
    roff += q.nr;
    const int64_t m = q.ns + q.nr;
    q.front_off = foff;
    foff += m * m;
    q.vec_off = voff;
    voff += m;
    S.max_front = std::max<int>(S.max_front, (int)m);
    if (!env[s].empty()) {
      // band supernode: column k's entries below the diagonal are the rows whose envelope starts at or before k
      q.env_off = (int64_t)S.fnz.size();
      S.fnz.insert(S.fnz.end(), env[s].begin(), env[s].end());
      std::vector<int> hist(q.ns + 1, 0);
      for (int f : env[s]) hist[std::min(f, q.ns)]++;
      int le = 0;
      for (int k = 0; k < q.ns; ++k) {
        le += hist[k];
        const double r = (double)(le - (k + 1));
        S.flops += 1 + r + r * (r + 1);
        S.nnzL += 1 + r;
      }
    } else {
      for (int k = 0; k < q.ns; ++k) {
        const double r = (double)(m - k - 1);
        S.flops += 1 + r + r * (r + 1);  // sqrt, column scale, rank-1 update of the lower trailing part
      }
      S.nnzL += (double)q.ns * (q.ns + 1) / 2 + (double)q.ns * q.nr;
    }
  }
  S.front_pool = foff;
  S.vec_pool = voff;
  // relmap: child's rows -> positions in parent's front
  S.relmap.assign(roff, -1);
  for (int s = 0; s < ns_count; ++s) {
    Supernode& q = S.sn[s];
    q.rel_off = q.rows_off;
    if (q.parent < 0) continue;
    const Supernode& p = S.sn[q.parent];
    const int* prow = S.rows.data() + p.rows_off;
    for (int r = 0; r < q.nr; ++r) {
      const int row = S.rows[q.rows_off + r];
      int pos;
      if (row >= p.c0 && row < p.c0 + p.ns) pos = row - p.c0;
      else {
        const int* it = std::lower_bound(prow, prow + p.nr, row);
        if (it == prow + p.nr || *it != row) throw std::runtime_error("symbolic: child row missing in parent");
        pos = p.ns + (int)(it - prow);
      }
      S.relmap[q.rows_off + r] = pos;
    }
  }
  // children lists and levels
  S.children_ptr.assign(ns_count + 1, 0);
  for (int s = 0; s < ns_count; ++s)
    if (S.sn[s].parent >= 0) S.children_ptr[S.sn[s].parent + 1]++;
  for (int s = 0; s < ns_count; ++s) S.children_ptr[s + 1] += S.children_ptr[s];
  S.children.assign(S.children_ptr[ns_count], 0);
  {
    std::vector<int> fill(S.children_ptr.begin(), S.children_ptr.end() - 1);
    for (int s = 0; s < ns_count; ++s)
      if (S.sn[s].parent >= 0) S.children[fill[S.sn[s].parent]++] = s;
  }
  int maxlev = 0;
  for (int s = 0; s < ns_count; ++s) {  // children precede parents (postorder)
    int lv = 0;
    for (int k = S.children_ptr[s]; k < S.children_ptr[s + 1]; ++k) lv = std::max(lv, S.sn[S.children[k]].level + 1);
    S.sn[s].level = lv;
    maxlev = std::max(maxlev, lv);
  }
  S.num_levels = maxlev + 1;
  S.levels.assign(S.num_levels, {});
  for (int s = 0; s < ns_count; ++s) S.levels[S.sn[s].level].push_back(s);
  return S;
}

DistPlan plan_distribution(const Symbolic& sym, const std::vector<int>& bi, const std::vector<int>& bj, int bdim,
                           int nblocks, int nranks, int rank, bool reduce_scatter, bool force, bool aligned,
                           const std::vector<double>* pose_work) {
  DistPlan P;
  if (nranks <= 1) return P;
  const int nsn = (int)sym.sn.size(), N = nranks;
  std::vector<double> fl(nsn), chain(nsn), st(nsn);
  for (int k = 0; k < nsn; ++k) {
    const double m = sym.sn[k].ns + sym.sn[k].nr;
    double f = 0;
    for (int c = 0; c < sym.sn[k].ns; ++c) f += (m - c) * (m - c);
    fl[k] = f;
    chain[k] = ((sym.sn[k].ns + 31) / 32) * dist_cost::STEP_S;
    st[k] = std::max(chain[k], f / dist_cost::TILE_FLOPS);
  }
  for (int k = 0; k < nsn; ++k)  // children precede parents (postorder): subtree serial work
    if (sym.sn[k].parent >= 0) st[sym.sn[k].parent] += st[k];
  // a set of fronts run level by level: per level the longer of its longest panel chain and its flops at the tile rate
  auto levels_time = [&](const std::vector<int>& owner, int who) {
    double t = 0;
    for (const auto& lv : sym.levels) {
      double ch = 0, f = 0;
      bool any = false;
      for (int sn : lv)
        if (owner[sn] == who) { any = true; ch = std::max(ch, chain[sn]); f += fl[sn]; }
      if (any) t += std::max(ch, f / dist_cost::TILE_FLOPS) + dist_cost::LEVEL_S;
    }
    return t;
  };
  auto allreduce_time = [&](double doubles) {
    return dist_cost::ALLREDUCE_LAT_S + 2.0 * (N - 1) / N * 8.0 * doubles / dist_cost::ALLREDUCE_BW;
  };
  auto segments_time = [&](double seg) {  // all-gather / reduce-scatter of N segments of `seg` doubles
    return dist_cost::ALLREDUCE_LAT_S + (N - 1) * 8.0 * seg / dist_cost::ALLREDUCE_BW;
  };
  // the reduced system's own communication: one all-reduce of every block + rhs when replicated; with reduce_scatter a
  // reduce-scatter of the blocks each rank's subtrees read (segments padded to the largest) + an all-reduce of the
  // shared blocks and the rhs. Blocks per supernode: a block lands in the front of its smaller permuted column.
  const double bb = (double)bdim * bdim;
  std::vector<double> sn_blocks(nsn, 0.0);
  for (size_t t = 0; t < bi.size(); ++t) sn_blocks[sym.block_sn[std::min(sym.bpinv[bi[t]], sym.bpinv[bj[t]])]] += 1.0;
  const double ar_full = allreduce_time(bi.size() * bb + (double)nblocks * bdim);
  auto input_cost = [&](const std::vector<int>& owner, long long& seg, long long& tail) {
    if (!reduce_scatter) { seg = 0; tail = (long long)(bi.size() * bb) + (long long)nblocks * bdim; return ar_full; }
    std::vector<double> ob(N + 1, 0.0);
    for (int k = 0; k < nsn; ++k) ob[owner[k] >= 0 ? owner[k] : N] += sn_blocks[k];
    tail = (long long)(ob[N] * bb) + (long long)nblocks * bdim;
    if (aligned) {  // subtree blocks complete where they are read (blocks written by pose-pose edges aside)
      seg = 0;
      return allreduce_time((double)tail);
    }
    seg = (long long)(*std::max_element(ob.begin(), ob.begin() + N) * bb);
    return segments_time((double)seg) + allreduce_time((double)tail);
  };
  // sharded work per supernode (its pose blocks' observations) and in total
  std::vector<double> sn_work(nsn, 0.0);
  double work_all = 0;
  if (pose_work)
    for (int b = 0; b < nblocks && b < (int)pose_work->size(); ++b) {
      sn_work[sym.block_sn[sym.bpinv[b]]] += (*pose_work)[b];
      work_all += (*pose_work)[b];
    }
  auto shard_cost = [&](const std::vector<int>& owner) {
    if (!aligned) return work_all / N;  // uniform split of the landmark order
    std::vector<double> w(N, 0.0);
    double sh = 0;
    for (int k = 0; k < nsn; ++k) (owner[k] >= 0 ? w[owner[k]] : sh) += sn_work[k];
    return *std::max_element(w.begin(), w.end()) + sh / N;
  };
  std::vector<int> none(nsn, -2);  // the replicated model: every front in one set
  P.shard_repl_s = work_all / N;
  P.repl_s = levels_time(none, -2) + ar_full + P.shard_repl_s;
  P.input_repl_s = ar_full;
  std::vector<int> cand;
  for (int k = 0; k < nsn; ++k)
    if (sym.sn[k].parent < 0) cand.push_back(k);
  std::vector<char> shared(nsn, 0);
  std::vector<int> owner(nsn);
  double best = 1e30;
  for (;;) {
    int arg = -1;
    for (size_t i = 0; i < cand.size(); ++i)
      if (sym.children_ptr[cand[i] + 1] > sym.children_ptr[cand[i]] && (arg < 0 || st[cand[i]] > st[cand[arg]])) arg = (int)i;
    if (arg < 0 || (int)cand.size() >= 4 * N) break;
    const int c = cand[arg];
    shared[c] = 1;
    cand.erase(cand.begin() + arg);
    for (int ci = sym.children_ptr[c]; ci < sym.children_ptr[c + 1]; ++ci) cand.push_back(sym.children[ci]);
    if (cand.size() < 2) continue;
    std::vector<int> srt(cand);
    std::sort(srt.begin(), srt.end(), [&](int a, int b) { return st[a] > st[b] || (st[a] == st[b] && a < b); });
    std::vector<double> load(N, 0.0), xr(N, 0.0);
    std::vector<int> sub_owner(nsn, -1);
    for (int s : srt) {
      const int r = (int)(std::min_element(load.begin(), load.end()) - load.begin());
      load[r] += st[s];
      sub_owner[s] = r;
      const double nr = sym.sn[s].nr;
      xr[r] += nr * (nr + 1) / 2 + nr;  // the root's contribution block (lower triangle) and update vector
    }
    for (int k = nsn - 1; k >= 0; --k)  // parents after children: walk down from the subtree roots
      owner[k] = shared[k] ? -1 : sub_owner[k] >= 0 ? sub_owner[k] : owner[sym.sn[k].parent];
    double tr = 0;
    for (int r = 0; r < N; ++r) tr = std::max(tr, levels_time(owner, r));
    const long long xseg = (long long)*std::max_element(xr.begin(), xr.end());
    const double ts = levels_time(owner, -1), tx = segments_time((double)xseg) + allreduce_time(sym.n + 1.0);
    long long seg = 0, tail = 0;
    const double ti = input_cost(owner, seg, tail), tw = shard_cost(owner);
    if (tr + ts + tx + ti + tw < best) {
      best = tr + ts + tx + ti + tw;
      P.shard_s = tw;
      P.owner = owner;
      P.rank_s = levels_time(owner, rank);
      P.max_rank_s = tr;
      P.shared_s = ts;
      P.xch_s = tx;
      P.input_s = ti;
      P.xch_seg = xseg;
      P.rs_seg = seg;
      P.tail = tail;
    }
  }
  P.on = !P.owner.empty() && (force || best < P.repl_s);
  return P;
}

std::vector<int> align_landmarks(const Symbolic& sym, const std::vector<int>& sn_owner, int nranks,
                                 const std::vector<int>& lm_ptr, const std::vector<int>& lm_cams) {
  const int nl = (int)lm_ptr.size() - 1;
  std::vector<int> own(std::max(nl, 0), -1);
  std::vector<long long> load(nranks, 0);
  std::vector<int> later;
  for (int l = 0; l < nl; ++l) {
    int first = -1;
    for (int a = lm_ptr[l]; a < lm_ptr[l + 1]; ++a) {
      const int p = sym.bpinv[lm_cams[a]];
      if (first < 0 || p < first) first = p;
    }
    const int o = first >= 0 ? sn_owner[sym.block_sn[first]] : -1;
    if (o >= 0) {
      own[l] = o;
      load[o] += lm_ptr[l + 1] - lm_ptr[l];
    } else {
      later.push_back(l);
    }
  }
  for (int l : later) {
    const int r = (int)(std::min_element(load.begin(), load.end()) - load.begin());
    own[l] = r;
    load[r] += std::max(lm_ptr[l + 1] - lm_ptr[l], 1);
  }
  return own;
}

}  // namespace g2ohip
