// Host-side launchers for the kernels in kernels.hip and cholesky.hip.
#pragma once
#include <hip/hip_runtime.h>

#include <cstddef>
#include <cstdint>

namespace g2ohip {

enum Family { FAM_NONE = 0, FAM_BA = 1, FAM_SE3 = 2, FAM_SE2 = 3, FAM_HOSTJ = 4, FAM_SE2XY = 5 };

struct EdgeArgs {
  const int* v0;
  const int* v1;
  const double* meas;  // host-J family: per edge [e | Ji | Jj]
  const double* info;
  const double* params;
  const double* s0;
  const double* s1;
  int rk = 0;          // robust kernel (G2OHIP_RK_*), uniform over the edge group
  double rk_delta = 1.0;
  int D = 0, DA = 0, DB = 0;  // host-J family dimensions
  int ue = 0;                 // uniform records (EdgeData::ue): bit 0 information, bit 1 intrinsics
};

namespace launch {
void error(int family, const EdgeArgs& a, int ne, double* chi, hipStream_t s);
// off_dst: destination of each edge's off-diagonal block, an offset into off_base (the Hessian) or, with bit 62
// set, into off_slot (per-edge slots of blocks several edges share)
void linearize(int family, const EdgeArgs& a, int ne, const int* h0, const int* h1, double* slot0, double* slot1,
               const long long* off_dst, const unsigned char* off_tr, double* off_base, double* off_slot, hipStream_t s);
// code[p] = slot index in `slots` (stride dim(dim+1)/2 + dim)
void vertex_reduce(int dim, int nv, int lanes, const int* ptr, const int* code, const double* slots, double* H,
                   double* b, const int* boff, hipStream_t s);
void offblock_reduce(int nb, int bsz, const int* ptr, const long long* soff, const double* slots, double* out,
                     const long long* dst, hipStream_t s);
// fused BA assembly (assembly.hip): chunks = (first edge, edges, partial slot or -1, 0) of whole landmarks per wave
// With a SchurSplit (sp != nullptr, lambda known at assembly, no shared off-diagonal blocks) the landmark side of the
// Schur complement is formed during assembly: the linearize waves factor each landmark's Hll + lambda I = U U^T and
// store G = Hpl U^-T in place of Hpl (in G's buffer, Hpl's block order), the camera pass adds S(i,i) and bschur_i
// beside Hpp(i,i) and b_i. No Hpl is stored then.
struct SchurSplit {
  double lam;            // lambda of every landmark block
  double lam_rank;       // lambda on S's diagonal (rank 0 only when sharded)
  const double* lamp;    // non-null: lam, lam_rank read from the device ([0], [1]) — the next iteration's assembly
                         // enqueued before the host knows the LM decision (lm_decide writes them)
  const unsigned char* lam_own;  // non-null (aligned shards): per camera, this rank adds lambda (lam) to S(i,i)
                                 // instead of lam_rank
  double* Ufac;          // per local landmark U record (6 doubles)
  double* cl;            // c = U^-1 b_l, global landmark index
  double* G;             // Hpl's block order: G (PD x LD) per observation, or with kx its 10-double Kt | x/z y/z 1/z record
  int kx;                // BA: store the Kt record instead of G (assembly.hip KXB; k_schur_rows rebuilds G from it)
  const int* cm_hpl;     // kx: per camera-major observation its record (Hpl block, or an extra one: fixed landmark)
  const int* kx_extra;   // kx: per (landmark-major) edge of a fixed landmark and a free camera its extra record, else -1
  long long hpl_base;    // offset of the first Hpl block in off_base (the Hessian)
  const int* lm_ptr;     // local landmark -> its Hpl/G block range (split landmarks' fixup)
  const int* hl;         // landmark vertex (local id) -> hessian index (-1 fixed), for the camera pass
  const int* sdiag;      // camera row -> S index of its diagonal block
  double* S;             // [S blocks | bschur]
  double* bschur;
  int* fail;             // landmark block not positive definite (informational, as k_schur_prep)
};
void linearize_fused(const EdgeArgs& a, const int4* chunks, int nchunks, const int* h0, const int* h1,
                     const long long* off_dst, const unsigned char* off_tr, double* off_base, double* off_slot,
                     double* Hll, double* b, int num_poses, int size_poses, int lm_begin, double* lpart,
                     const SchurSplit* sp, hipStream_t s);
void lm_fixup(int nfix, const int4* fix, const double* lpart, double* Hll, double* b, int num_poses, int size_poses,
              int lm_begin, const SchurSplit* sp, hipStream_t s);
void cam_assemble(const EdgeArgs& a, const int* cm_ptr, int npose, double* Hpp, double* b, int num_poses, int lm_begin,
                  const SchurSplit* sp, hipStream_t s, const int* cams = nullptr);
// back-substitution of the Schur split recomputing each observation's Jacobians (no G blocks read): per local landmark
// its edge range erng (landmark-major group order), hcam = camera vertex -> hessian index (-1 fixed)
void backsub_j(const EdgeArgs& a, int nl, const int2* erng, const int* hcam, const double* Ufac, const double* cl_all,
               int size_poses, int lm0, double* x, hipStream_t s);
// Schur kernels for (pd, ld) = (6, 3) (BlockSolver_6_3) and (3, 2) (BlockSolver_3_2)
void schur_prep(int ld, int nl, int lm0, const double* Hll, const double* bl_all, const double* lam, double* Dinv,
                double* Ufac, double* cl_all, int* fail, hipStream_t s);
int schur_ufac_stride(int ld);  // doubles of the per-landmark U factor record
// diagonal blocks + bschur (and G per observation): one workgroup per camera row over its observations (CSR rptr/robs)
void schur_diag(int pd, int ld, int nrows, const int* rptr, const int* robs, const int* obs_lm, int lm0,
                const double* Hpl, const double* Ufac, const double* cl_all, const int* sdiag, const int* s_hpp,
                const double* Hpp, const double* b, const double* lam, const unsigned char* lam_own,
                const double* lam_full, double* S, double* bschur, double* G, hipStream_t s);
// row-stationary off-diagonal Schur pass (k_schur_rows): task = (camera row, <= SCHUR_SL off-diagonal
// slots), batch = <= SCHUR_SB staged observation blocks of the row's landmarks
constexpr int SCHUR_SB = 128, SCHUR_SL = 64;  // 128: 4 workgroups per CU (LDS), 150 vs 172 us at C4
// batches of the BA split's 80-byte Kt records (assembly.hip KXB): 192 blocks are 30 KB of staging, still 4 workgroups
// per CU, and a third fewer batches per row task than 128
#ifndef G2OHIP_SCHUR_SB_KX
#define G2OHIP_SCHUR_SB_KX 192
#endif
constexpr int SCHUR_SB_KX = G2OHIP_SCHUR_SB_KX;
struct SchurTask {
  int row, noff;  // camera row, number of off-diagonal slots of this task
  int b0, b1;     // batches
  int soff;       // S index of the first off-diagonal slot
  int pad;        // 0: S = Hpp - sum; k > 0: one part of a split row chunk, its partial sums to part blocks k - 1 ...
};
// a row chunk split into parts: S(soff + s) = Hpp - sum over the np parts of part block (xo + p noff + s), parts in order
struct SchurPartGroup {
  int soff, noff, xo, np;
};
struct SchurBatch {
  int st0, nst;  // staged blocks (st_obs)
  int pr0, npr;  // pairs (posA | posB << 16), slot CSR in pp[batch * (SCHUR_SL + 1) ...]
};
// nzero > 0: nzero more workgroups (after the row tasks) zero the (offset, length) ranges zr of `fronts` — the
// factorization's pre-scattered fronts, cleared beside the Schur pass instead of by a launch of the factor's own
void schur_rows(int pd, int ld, int ntasks, const SchurTask* tasks, const SchurBatch* batches, const int* st_obs,
                const int* pairs, const int* pp, const double* G, const int* s_hpp, const double* Hpp, double* S,
                int nzero, const long long* zr, double* fronts, hipStream_t s, bool kx = false,
                int sb = SCHUR_SB, double* part = nullptr, const int* gmap = nullptr);
// the split row chunks' partial sums into S (fixed part order: bitwise reproducible)
void schur_part_sum(int pd, int ngroups, const SchurPartGroup* groups, const double* part, const int* s_hpp,
                    const double* Hpp, double* S, hipStream_t s);
void backsub(int pd, int ld, int nl, const int* lm_ptr, const int* blk_pose, const double* Hpl, const double* Dinv,
             const double* b, int size_poses, int lm0, double* x, hipStream_t s);
// back-substitution from the G blocks of an assembly-time Schur split: x_l = U^-T (c_l - G^T x_p)
void backsub_g(int pd, int ld, int nl, const int* lm_ptr, const int* blk_pose, const double* G, const double* Ufac,
               const double* cl_all, int size_poses, int lm0, double* x, hipStream_t s);
// vertex oplus of every type in one launch: per type (vertex type id 1..5, count, x offsets, states)
struct OplusList {
  int cnt = 0;
  int vt[5], n[5], blk0[5];
  const int* xoff[5];
  double* st[5];
  int* nopl = nullptr;
};
void oplus_multi(const OplusList& L, const double* x, hipStream_t s);
size_t sum_partials(long long n);
void sum(const double* v, long long n, double* partial, double* out, hipStream_t s);
void scale_terms(long long n, const double* x, const double* b, const double* lam, double* out, hipStream_t s);
// computeActiveErrors + activeRobustChi2 of one edge group fused with the first pass of the deterministic sum:
// writes the group's partials at partial[0..np) and returns np; sum_final adds all groups' partials in order
int error_partials(int family, const EdgeArgs& a, int ne, double* partial, hipStream_t s);
void sum_final(const double* partial, int np, double* out, hipStream_t s);
// error_partials (one edge group) + scale_sum in one launch and both finals in a second: chi2 -> out_chi, the
// computeScale sum -> out_scale (the same sums bit for bit). dec (one rank, out_chi = p + 1, out_scale = p + 2): the
// finals and lm_decide in one launch
struct LmDecide {
  double current_chi, ni;
  bool rank0;
  double* host_out;  // mapped, coherent host memory: the 16 scalars after the decision (replaces the readback copy)
};
void error_scale(int family, const EdgeArgs& a, int ne, long long n, long long npose, const double* x, const double* b,
                 const double* lam, double* partial, double* out_chi, double* out_scale, hipStream_t s,
                 const LmDecide* dec = nullptr);
// computeScale + sum (same chunking/tree as sum(): deterministic)
void scale_sum(long long n, long long npose, const double* x, const double* b, const double* lam, double* partial,
               double* out, hipStream_t s);
void set_scalars(double* p, double lam, double lam_rank, hipStream_t s, bool reset_fail = false);
// OptimizationAlgorithmLevenberg's trial decision (optimization_algorithm_levenberg.cpp:127-141) from the device chi2
// and scale of the trial: p[12] the next lambda, p[13] the same for S's diagonal (rank 0 only), p[14] 1 accepted,
// p[15] rho (the layout of dscal: engine.cpp)
void lm_decide(double* p, double current_chi, double ni, bool rank0, hipStream_t s);
// y = (A + lam I) x, A symmetric as upper blocks (block CSR with transposed entries); lam may be null; with b also
// per-row (y - b)^2 -> r2 and b^2 -> b2 (y may be null)
void block_symv(int pd, int n, const int* rptr, const int2* ent, const int* diag, const double* vals, const double* lam,
                const double* x, double* y, const double* b, double* r2, double* b2, hipStream_t s);
struct CopyList {  // up to 4 device-to-device copies of doubles in one launch (vertex push/pop)
  const double* src[4];
  double* dst[4];
  long long len[4];
  int n;
  // optional: set_scalars in the same launch (the LM trial's push + setLambda): sp[0] = lam, sp[4] = lam_rank,
  // sp[5] = 0, the not-PD flags cleared
  double* sp = nullptr;
  double lam = 0.0, lam_rank = 0.0;
};
void copy_multi(const CopyList& cl, hipStream_t s);
void diag_absmax(const double* H1, int nb1, int d1, const double* H2, int nb2, int d2, double* partial, double* out,
                 hipStream_t s);

// ---- supernodal multifrontal Cholesky (cholesky.hip) ----
struct FrontDesc {  // device view of one supernode (see symbolic.hpp)
  long long front_off;
  long long vec_off;
  long long l_off;  // factor columns [L11; L21] (m x ns, ld m) in lbuf
  long long rows_off;
  long long x_off;  // the front's explicit X = L11^-1 (ns x ns column-major) in xinv
  int c0, ns, nr, parent;
  int child_begin, child_end;  // into the children array
  int jt_off;  // into jtab: [rows into the parent's first diagonal block | first row of every parent slab]
  int cm_off;  // into cmptr: per column of this front, the range of (child, child column) pairs mapping to it
};
struct Task {  // one workgroup's work item (meaning per kernel, see cholesky.hip)
  int s, a, b, c;
};
struct StepTask {  // k_step work item, self-contained so a workgroup needs one dependent load
  long long f_off, l_off, v_off, x_off;
  int m, ns, c0;
  int k0kb;   // k0 | kb << 16
  int tile;   // ti | tj << 16 (inverse task: block column j | block row p << 16)
  int flags;  // 1 update the tile, 4 next-diagonal task, 8 reaches into the contribution block, 16 inverse,
              // 32 no next-diagonal task this step (blocked front, big-panel boundary): writers update every row
  int clim;   // tile updates stop at this front column (ns, m when fused, the big-panel end when blocked)
};
// the launch's first CHOL_HEAD tasks (the next-diagonal tasks among them) by value in the kernel arguments: those workgroups
// read their task with the kernel arguments instead of one more dependent global load
constexpr int CHOL_HEAD = 8;
struct StepHead {
  StepTask t[CHOL_HEAD];  // the launch's first min(CHOL_HEAD, ntask) tasks
  // deferred input scatter (DeviceCholesky::factor): workgroups past the launch's ntask tasks scatter the input entries
  // [sc0, sc1) of a later level's pre-scattered fronts (as k_chol_scatter: fronts[dst[k]] = vals[src[k] & 0x7fffffff],
  // + lambda when src[k] < 0), 256 entries each
  int ntask;
  long long sc0, sc1;
  const double* sc_vals;
  const long long* sc_dst;
  const int* sc_src;
  const double* sc_lam;
};
// k_extend_add's block-0 tasks (the launch's first nb0 workgroups, one per front: its first diagonal block assembled
// and factored) read their front and children from these self-contained records, built at setup, instead of the chain
// task -> FrontDesc -> children[] -> child FrontDesc -> jtab (four dependent round trips before the first data load)
struct B0Front {
  long long front_off, vec_off;
  int m, kb0, c0;
  int cb, ce;  // the front's children: B0Child records [cb, ce) (= FrontDesc::child_begin / child_end)
};
struct B0Child {      // one child, in the order of the children array (also read by the pre-scattered slab tasks)
  long long u_off;    // its update matrix U = fronts + u_off (leading dimension mc)
  long long vv_off;   // its update vector vecs + vv_off
  int mc, nrc, rel_off;
  int n0;             // its rows mapping into the parent's first diagonal block (jtab[jt_off])
  int jt_off;         // FrontDesc::jt_off
};
constexpr int EA_HEAD = 16;
// extend-add launch arguments: the first EA_HEAD block-0 fronts by value (no global load at all on the level's
// chain), and the deferred input scatter riding in the launch (DeviceCholesky::factor): workgroups past its ntask
// tasks scatter entries [sc0, sc1) as k_chol_scatter does, 256 each
struct ScatterJob {
  int ntask;
  int nb0;  // block-0 tasks (the first nb0 workgroups)
  long long sc0, sc1;
  const long long* dst;
  const int* src;
  B0Front b0[EA_HEAD];
};
// zero ranges (offset, length pairs) of the front pool, then scatter input entries: fronts[dst[k]] =
// vals[src[k] & 0x7fffffff] (+ lambda when src[k] < 0), and the front vectors v_s = [rhs(perm[c0 ..]) (own
// columns); 0] (in the scatter's launch when there are entries)
void chol_prescatter(int nzero, const long long* zr, long long nent, const double* vals, const long long* dst,
                     const int* src, const double* lam, double* fronts, int nfronts, const FrontDesc* fd,
                     const int* perm, const double* rhs, double* vecs, hipStream_t s);
// assembly + extend-add of a level (slab tasks, t.c == 0: columns [a, b)) with every front's first
// diagonal block assembled, factored and forward-solved beside it (t.c == 1). Input entries of scalar
// column c (permuted): ent_row/ent_src[colptr[c] .. colptr[c+1]) = row in the front | diag << 30, index in vals
void chol_extend_add(int ntasks, int nb0, const Task* tasks, const B0Front* b0f, const B0Child* b0c, const FrontDesc* fd,
                     const int* children, const int* relmap,
                     const int* jtab, const int* cmptr, const longlong2* cment, const int* colptr, const int* ent_row, const int* ent_src, const double* vals, const double* lam,
                     double* fronts, double* vecs, double* lbuf, double* ysol, double* linv, double* xinv,
                     int* fail, int assemble, hipStream_t s,  // assemble: 0 pre-scattered level, 1 in place,
                     const ScatterJob* sj = nullptr);          // 2 in place (m <= 512); sj: + scatter workgroups
void chol_step(int ntasks, const StepTask* tasks, const StepHead& head, double* fronts, double* lbuf, double* vecs, double* ysol,
               double* linv, double* xinv, int* fail, bool pairs, hipStream_t s);  // pairs: lagged-pair tasks present;
                                                                                    // + head's scatter workgroups
// C -= L(:, ka:kb) L(:, ka:kb)^T over rows/columns >= kb of a front (task: s, a = ka, b = tile, c = kb; c = 0 is
// the contribution block, K = [0, ns)); columns stop at ns unless kb = ns (then m)
void chol_syrk(int variant, int ntasks, const Task* tasks, const FrontDesc* fd, double* fronts, const double* lbuf,
               const double* ysol, double* vecs, hipStream_t s);
int syrk_variant();    // the k_syrk tile (G2OHIP_SYRK_DMA)
int syrk_tile_rows(int variant);  // rows per k_syrk tile of a variant (64 or 128): the task lists' row-tile unit
void chol_l21(int ntasks, const Task* tasks, const FrontDesc* fd, const double* fronts, const double* xinv, double* lbuf,
              hipStream_t s);
void chol_permute(int n, const int* perm, const double* in, double* out, hipStream_t s);   // out[k] = in[perm[k]]
void chol_ipermute(int n, const int* perm, const double* in, double* out, hipStream_t s);  // out[perm[k]] = in[k]
void chol_bwd_gemv(int ntasks, const Task* tasks, const FrontDesc* fd, const int* rows, const double* lbuf,
                   const double* ysol, const double* xsol, double* tsol, hipStream_t s);
void chol_bwd_inner(int ntasks, const Task* tasks, const FrontDesc* fd, const double* lbuf, const double* xsol, double* tsol,
                    hipStream_t s);
// x = X^T t per front column; each x also lands at xout[perm[k]] (the caller's order)
void chol_xdiag(int ntasks, const Task* tasks, const FrontDesc* fd, const double* linv, double* xinv, hipStream_t s);
void chol_bwd_x(int ntasks, const Task* tasks, const FrontDesc* fd, const double* xinv, const double* linv,
                const double* tsol, double* xsol, const int* perm, double* xout, hipStream_t s);
int debug_phases(unsigned long long* out, int maxrec);  // -DG2OHIP_PHASES builds only
constexpr int CHOL_NB = 32, CHOL_TT = 64, CHOL_EA = 16, CHOL_BW = 4;
// distributed factorization glue: contiguous range copies (src, dst, len) in doubles; the distributed
// solve's not-PD flag into / x and flag out of its all-reduce buffer; x[idx[k]] = 0
void chol_copy_ranges(int n, const long long* rng, const double* src, double* dst, hipStream_t s);
// dst[boff[t] + i] = src[t bb + i], i < bb, for nblk blocks of bb doubles (the reduce-scatter pack)
void chol_pack_blocks(long long nblk, int bb, const long long* boff, const double* src, double* dst, hipStream_t s);
void chol_dist_fail_in(const int* fail, double* xr, int n, hipStream_t s);
void chol_dist_x_out(const double* xr, int n, double* x, int* fail, hipStream_t s);
void chol_zero_idx(const int* idx, int n, double* x, hipStream_t s);
// measured roofline peaks (peaks.hip): out[0] HBM copy GB/s, out[1] FP64 MFMA TFLOP/s, out[2] FP64 VALU TFLOP/s, out[3] CUs
void measure_peaks(int device, double* out);
// computeMarginals multi-right-hand-side solves (marginals.hip): one launch per tree level, one workgroup per front
void marg_forward(int nf, const int* lfronts, const FrontDesc* fd, const int* children, const int* relmap,
                  const double* lbuf, const double* linv, const long long* woff, double* W, double* Y, double* T, int n,
                  int K, hipStream_t s);
void marg_backward(int nf, const int* lfronts, const FrontDesc* fd, const int* rows, const double* lbuf,
                   const double* linv, double* Y, double* T, int n, int K, hipStream_t s);
void marg_unit(int K, const int* prow, double* Y, int n, hipStream_t s);
void marg_gather(long long cnt, const long long* idx, const double* Y, double* out, hipStream_t s);
}  // namespace launch
}  // namespace g2ohip
