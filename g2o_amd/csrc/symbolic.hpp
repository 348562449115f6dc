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

// Block pattern of a symmetric matrix given by its upper blocks (bi <= bj) of a uniform block size, adjacency in the
// order the blocks are listed (the order DeviceCholesky::setup analyses).
BlockPattern block_pattern(int nblocks, int bdim, const std::vector<int>& bi, const std::vector<int>& bj);

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

// ---- distribution of the factorization over ranks (landmark-sharded BA)
// Cost model of the cut, calibrated on C4 / C5 (rank schedules timed alone on one GPU, tools/dist_factor_time.py): a
// 32-column panel step on the chain, the panel steps' tile rate, a level's fixed launches, and collectives over xGMI
// (latency + bus bandwidth; ring traffic 2 (N-1)/N of the buffer for an all-reduce, (N-1) segments for an all-gather
// or reduce-scatter).
namespace dist_cost {
constexpr double STEP_S = 10e-6, TILE_FLOPS = 12e12, LEVEL_S = 20e-6, ALLREDUCE_LAT_S = 30e-6, ALLREDUCE_BW = 120e9;
// landmark-sharded work per observation (BA: linearize, camera pass, Schur rows, back-substitution, chi2): C4 0.35 ms
// for 1 M observations, C5 2.7 ms for 10 M (r04 stage times)
constexpr double OBS_S = 0.3e-9;
}

struct DistPlan {
  std::vector<int> owner;  // per supernode: owning rank, -1 shared (every rank); empty: no candidate cut
  bool on = false;         // the best cut beats the replicated factorization's model (or force)
  // modelled seconds: the given rank's subtrees, the shared top, the replicated factorization, the cut's exchanges
  // (root all-gather + x all-reduce), the input (reduce-scatter + tail all-reduce, or the whole all-reduce), the
  // replicated input (whole all-reduce), the slowest rank's subtrees
  double rank_s = 0, shared_s = 0, repl_s = 0, xch_s = 0, input_s = 0, input_repl_s = 0, max_rank_s = 0;
  // modelled seconds of the landmark-sharded assembly / Schur / back-substitution on the busiest rank: with aligned
  // shards each rank's share follows its subtrees (the shared poses' spread evenly), replicated the uniform split
  double shard_s = 0, shard_repl_s = 0;
  long long xch_seg = 0;   // doubles per rank of the root all-gather (the largest rank's roots)
  long long rs_seg = 0;    // doubles per rank of the input reduce-scatter (the largest rank's blocks), 0 without
  long long tail = 0;      // doubles of the input's tail all-reduce (shared blocks + rhs)
};

// Chooses the cut of the elimination tree of the block pattern (bi, bj: upper blocks of `nblocks` blocks of size bdim,
// analysed into sym) for `nranks` ranks: candidate cuts split the candidate subtree with the largest serial work (its
// root joins the shared top), up to 4 candidates per rank, subtrees to ranks largest first; the cheapest cut by the
// model above is kept. reduce_scatter: the input is reduce-scattered by subtree ownership (else one all-reduce);
// aligned: the landmark shards follow the cut (align_landmarks), so a rank's subtree blocks are complete on that rank
// and only the shared blocks and the rhs are reduced (one all-reduce).
// pose_work (optional, per pose block of the pattern, seconds): the landmark-sharded work that follows the pose (its
// observations), added to every candidate as the busiest rank's share.
DistPlan plan_distribution(const Symbolic& sym, const std::vector<int>& bi, const std::vector<int>& bj, int bdim,
                           int nblocks, int nranks, int rank, bool reduce_scatter, bool force, bool aligned = false,
                           const std::vector<double>* pose_work = nullptr);

// Landmark shards aligned with a cut: landmark l, observing the pose blocks lm_cams[lm_ptr[l] ..
// lm_ptr[l+1]) of the pattern, goes to the rank owning the supernode of its first-eliminated pose. Its poses form a
// clique of the pattern, so every other one is eliminated in an ancestor of that supernode: all of l's Schur blocks
// land in that rank's subtrees or in the shared top, and no other rank writes a block of that rank's subtrees. A
// landmark whose poses are all shared goes to the rank with the fewest observations so far (landmark order).
// Landmarks without free poses go to the least-loaded rank as well. Returns the rank per landmark.
std::vector<int> align_landmarks(const Symbolic& sym, const std::vector<int>& sn_owner, int nranks,
                                 const std::vector<int>& lm_ptr, const std::vector<int>& lm_cams);

}  // namespace g2ohip
