// Host-side symbolic analysis for the GPU supernodal multifrontal Cholesky.
//
// Replaces LinearSolverCSparse::computeSymbolicDecomposition
// (solvers/csparse/linear_solver_csparse.h:246-308): block ordering on the
// block pattern (the reference uses cs_amd; we use nested dissection because
// the GPU needs a wide, balanced elimination tree), block elimination tree,
// block structure of L, relaxed supernodes and the frontal index maps the
// numeric kernels consume.  Runs once per structure, like the reference.
#pragma once
#include <cstdint>
#include <vector>

namespace g2ohip {

struct BlockPattern {
  int nb = 0;                    // number of block columns
  std::vector<int> dim;          // block dims [nb]
  std::vector<int> offset;       // scalar offset of each block [nb+1]
  std::vector<int> adjp, adji;   // symmetric adjacency (no diagonal), CSR [nb+1]
};

struct Supernode {
  int b0, b1;        // block columns [b0, b1) in the final (permuted) order
  int c0, ns;        // first scalar column and number of scalar columns
  int nr;            // number of scalar rows below the diagonal block
  int parent;        // parent supernode (-1 root)
  int level;         // height: leaves 0
  int64_t front_off; // offset of the front (m x m col-major, m = ns+nr) in the front pool
  int64_t rows_off;  // offset into row index list (length nr): scalar rows (permuted numbering)
  int64_t rel_off;   // offset into relmap (length nr): position of each row in the parent front
  int64_t vec_off;   // offset into the front-vector pool (length m)
  // band supernode (a band leaf of the ordering, amalgamated whole): env_off >= 0 indexes Symbolic::fnz, the first own
  // column (front-relative) of each of the m front rows with a structural nonzero in L — the row's envelope. Entries of
  // L outside every row's envelope are zero, so the factor skips the tiles that lie entirely outside it.
  int64_t env_off = -1;
};

struct Symbolic {
  int n = 0;                       // scalar dimension
  int nb = 0;                      // number of blocks
  std::vector<int> bperm;          // new block k -> old block bperm[k]
  std::vector<int> bpinv;          // old block -> new block
  std::vector<int> perm;           // new scalar k -> old scalar perm[k]
  std::vector<int> pinv;           // old scalar -> new scalar
  std::vector<int> boffset_new;    // scalar offset of new block k
  std::vector<int> bdim_new;
  std::vector<int> block_sn;       // new block -> supernode
  std::vector<Supernode> sn;
  std::vector<int> rows;           // concatenated off-diagonal scalar rows of each supernode
  std::vector<int> relmap;         // concatenated: row r of child -> position in parent's front
  std::vector<std::vector<int>> levels;  // supernodes per level
  std::vector<int> children_ptr, children;  // CSR children lists (ordered)
  int64_t front_pool = 0;          // doubles
  int64_t vec_pool = 0;            // doubles
  double flops = 0;                // factorization flops (algorithmic)
  double nnzL = 0;                 // scalar nnz of L including the dense supernode fill
  int max_front = 0;
  int num_levels = 0;
  std::vector<int> fnz;            // envelopes of the band supernodes (see Supernode::env_off)
  int band_leaf = 0;               // ordering parameter that produced this analysis (0: plain nested dissection)
};

// Nested-dissection ordering of the block graph. leaf_size: subgraphs at most this
// large are ordered by minimum degree; refine: greedy separator refinement after each bisection.
// band_leaf > 0: parts of at most band_leaf blocks whose BFS level structure is a long band (at least 3 levels deep)
// become band leaves — ordered by BFS level from a pseudo-peripheral end (the reference's cs_amd order on a band is
// this sequential order too), their group ids (per block, -1 elsewhere) written to *groups; the analysis amalgamates
// each group into one band supernode whose structural zeros the factor skips.
std::vector<int> nested_dissection(const BlockPattern& P, int leaf_size = 48, bool refine = false, bool windows = false,
                                   bool part_degree = false, int band_leaf = 0, std::vector<int>* groups = nullptr);

// Modelled GPU factor time of a symbolic analysis (seconds): flops at the MFMA rate plus the
// level-synchronous panel-step chain.
double gpu_cost(const Symbolic& S);

// Full symbolic analysis with a given block ordering (bperm: new->old). If bperm is
// empty, nested dissection is used (with or without separator refinement, whichever models faster).
// groups (per original block, optional): blocks of one group >= 0 that are consecutive in the order and chained in the
// elimination tree are amalgamated into one band supernode regardless of the relaxation limits.
Symbolic analyze(const BlockPattern& P, std::vector<int> bperm = {}, double relax = 0.25, int relax_max_blocks = 64,
                 const std::vector<int>* groups = nullptr);

}  // namespace g2ohip
