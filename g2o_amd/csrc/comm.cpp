// Comm implementations (see comm.hpp).
#include "comm.hpp"

#include <rccl/rccl.h>

#include <algorithm>
#include <condition_variable>
#include <cstdlib>
#include <cstring>
#include <map>
#include <memory>
#include <mutex>
#include <vector>

#include "common.hpp"

namespace g2ohip {

namespace {

enum : int { OP_SUM = 1, OP_MAX = 2, OP_RS = 3, OP_AG = 4 };
constexpr long long kCheckFirst = 8;  // RcclComm: collectives verified after each structure build by default

std::string call_desc(long long seq, size_t n, int op) {
  return "call #" + std::to_string(seq) + " (" +
         (op == OP_MAX ? "max" : op == OP_RS ? "reduce-scatter" : op == OP_AG ? "all-gather" : "sum") +
         ", n=" + std::to_string(n) + ")";
}

struct RcclComm : Comm {
  ncclComm_t c = nullptr;
  int rank = 0;
  long long check_all = 0;   // G2OHIP_COMM_CHECK: 1 every call, 0 none, unset: the first kCheckFirst calls per structure
  long long check_left = 0;  // calls still to verify (-1: all)
  double* dchk = nullptr;  // 6 doubles: [seq, n, op, -seq, -n, -op] max-reduced
  ~RcclComm() override {
    if (dchk) (void)hipFree(dchk);
    if (c) ncclCommDestroy(c);
  }
  // every rank must enter the same (call number, length, operation). max over ranks of (v, -v) gives (max, -min); any
  // difference between them is a rank-dependent collective sequence. The check synchronises the stream, so by default
  // it covers only the first kCheckFirst calls after each structure build (the structure decides the sequence);
  // G2OHIP_COMM_CHECK=1 checks every call, =0 none.
  void rearm() override { check_left = check_all; }
  void verify(size_t n, int op, hipStream_t s) {
    if (check_left == 0) return;
    if (check_left > 0) --check_left;
    if (!dchk) HIP_CHECK(hipMalloc(&dchk, 6 * sizeof(double)));
    const double v[6] = {(double)seq, (double)n, (double)op, -(double)seq, -(double)n, -(double)op};
    double r[6];
    HIP_CHECK(hipMemcpyAsync(dchk, v, sizeof v, hipMemcpyHostToDevice, s));
    const ncclResult_t e = ncclAllReduce(dchk, dchk, 6, ncclDouble, ncclMax, c, s);
    if (e != ncclSuccess) throw DeviceError(std::string("ncclAllReduce(check): ") + ncclGetErrorString(e));
    HIP_CHECK(hipMemcpyAsync(r, dchk, sizeof r, hipMemcpyDeviceToHost, s));
    HIP_CHECK(hipStreamSynchronize(s));
    if (r[0] != -r[3] || r[1] != -r[4] || r[2] != -r[5])
      throw DeviceError("collective mismatch across ranks at rank " + std::to_string(rank) + " " + call_desc(seq, n, op) +
                        ": another rank entered call #" + std::to_string((long long)(r[0] == seq ? -r[3] : r[0])) +
                        " with n in [" + std::to_string((long long)-r[4]) + ", " + std::to_string((long long)r[1]) + "]");
  }
  void allreduce_sum(double* p, size_t n, hipStream_t s) override {
    verify(n, OP_SUM, s);
    ++seq;
    const ncclResult_t r = ncclAllReduce(p, p, n, ncclDouble, ncclSum, c, s);
    if (r != ncclSuccess) throw DeviceError(std::string("ncclAllReduce(sum): ") + ncclGetErrorString(r));
  }
  void allreduce_max(double* p, size_t n, hipStream_t s) override {
    verify(n, OP_MAX, s);
    ++seq;
    const ncclResult_t r = ncclAllReduce(p, p, n, ncclDouble, ncclMax, c, s);
    if (r != ncclSuccess) throw DeviceError(std::string("ncclAllReduce(max): ") + ncclGetErrorString(r));
  }
  void reduce_scatter_sum(double* p, size_t count, hipStream_t s) override {
    verify(count, OP_RS, s);
    ++seq;
    // in place (recvbuff = sendbuff + rank * recvcount)
    const ncclResult_t r = ncclReduceScatter(p, p + (size_t)rank * count, count, ncclDouble, ncclSum, c, s);
    if (r != ncclSuccess) throw DeviceError(std::string("ncclReduceScatter(sum): ") + ncclGetErrorString(r));
  }
  void allgather(double* p, size_t count, hipStream_t s) override {
    verify(count, OP_AG, s);
    ++seq;
    // in place (sendbuff = recvbuff + rank * sendcount)
    const ncclResult_t r = ncclAllGather(p + (size_t)rank * count, p, count, ncclDouble, c, s);
    if (r != ncclSuccess) throw DeviceError(std::string("ncclAllGather: ") + ncclGetErrorString(r));
  }
};

// ---- in-process group for LocalComm ----
struct Group {
  int nranks;
  std::mutex mu;
  std::condition_variable cv;
  int arrived = 0;
  long long generation = 0;
  std::vector<std::vector<double>> bufs;
  struct Meta { long long seq = -1; size_t n = 0; int op = 0; };
  std::vector<Meta> meta;
  explicit Group(int n) : nranks(n), bufs(n), meta(n) {}
  void barrier() {
    std::unique_lock<std::mutex> lk(mu);
    const long long gen = generation;
    if (++arrived == nranks) {
      arrived = 0;
      ++generation;
      cv.notify_all();
    } else {
      cv.wait(lk, [&] { return generation != gen; });
    }
  }
  // Rank-ordered host reduction of every rank's buffer into `out`. Each rank first publishes its call (number,
  // length, operation); after the first barrier every rank compares all of them and, on any difference, throws
  // on every rank alike (no rank is left waiting in the second barrier, no buffer is read past its length).
  void reduce(int rank, long long seq, const double* in, double* out, size_t n, int op) {
    bufs[rank].assign(in, in + n);
    meta[rank] = Meta{seq, n, op};
    barrier();
    for (int r = 0; r < nranks; ++r)
      if (meta[r].seq != meta[0].seq || meta[r].n != meta[0].n || meta[r].op != meta[0].op)
        throw DeviceError("collective mismatch across ranks: rank 0 entered " +
                          call_desc(meta[0].seq, meta[0].n, meta[0].op) + ", rank " + std::to_string(r) + " " +
                          call_desc(meta[r].seq, meta[r].n, meta[r].op) + " (seen by rank " + std::to_string(rank) + ")");
    if (op == OP_AG) {  // n = nranks segments: segment r from rank r
      const size_t cnt = n / nranks;
      std::vector<double> all(n);
      for (int r = 0; r < nranks; ++r)
        std::copy(bufs[r].begin() + (size_t)r * cnt, bufs[r].begin() + (size_t)(r + 1) * cnt, all.begin() + (size_t)r * cnt);
      barrier();  // everyone has read every buffer
      std::copy(all.begin(), all.end(), out);
      return;
    }
    std::vector<double> acc(bufs[0]);
    for (int r = 1; r < nranks; ++r)
      for (size_t k = 0; k < n; ++k) acc[k] = op == OP_MAX ? std::max(acc[k], bufs[r][k]) : acc[k] + bufs[r][k];
    if (op == OP_RS) {  // n = nranks segments: only this rank's segment is summed into out (RCCL leaves the rest)
      const size_t cnt = n / nranks;
      barrier();
      std::copy(acc.begin() + (size_t)rank * cnt, acc.begin() + (size_t)(rank + 1) * cnt, out + (size_t)rank * cnt);
      return;
    }
    barrier();  // everyone has read every buffer
    std::copy(acc.begin(), acc.end(), out);
  }
};
std::mutex g_groups_mu;
std::map<std::string, std::shared_ptr<Group>> g_groups;

std::shared_ptr<Group> group_for(const std::string& key, int nranks) {
  std::lock_guard<std::mutex> lk(g_groups_mu);
  auto& slot = g_groups[key + "#" + std::to_string(nranks)];
  if (!slot) slot = std::make_shared<Group>(nranks);
  return slot;
}

struct LocalComm : Comm {
  std::shared_ptr<Group> g;
  int rank;
  std::vector<double> host;
  void reduce(double* p, size_t n, hipStream_t s, int op) {
    host.resize(n);
    HIP_CHECK(hipMemcpyAsync(host.data(), p, n * sizeof(double), hipMemcpyDeviceToHost, s));
    HIP_CHECK(hipStreamSynchronize(s));
    g->reduce(rank, seq++, host.data(), host.data(), n, op);
    HIP_CHECK(hipMemcpyAsync(p, host.data(), n * sizeof(double), hipMemcpyHostToDevice, s));
    HIP_CHECK(hipStreamSynchronize(s));
  }
  void allreduce_sum(double* p, size_t n, hipStream_t s) override { reduce(p, n, s, OP_SUM); }
  void allreduce_max(double* p, size_t n, hipStream_t s) override { reduce(p, n, s, OP_MAX); }
  void reduce_scatter_sum(double* p, size_t count, hipStream_t s) override { reduce(p, count * g->nranks, s, OP_RS); }
  void allgather(double* p, size_t count, hipStream_t s) override { reduce(p, count * g->nranks, s, OP_AG); }
};

// Timing-only transport (tools/dist_rank_times.py): one engine plays rank r of N alone, every collective a no-op. The
// engine then runs exactly the kernels rank r would (its landmark shard, the global Schur pattern, its subtrees and the
// shared top of the distributed factorization) on one GPU; its sums are partial, so its results are not meaningful.
struct SoloComm : Comm {
  void allreduce_sum(double*, size_t, hipStream_t) override { ++seq; }
  void allreduce_max(double*, size_t, hipStream_t) override { ++seq; }
  void reduce_scatter_sum(double*, size_t, hipStream_t) override { ++seq; }
  void allgather(double*, size_t, hipStream_t) override { ++seq; }
};

}  // namespace

Comm* make_rccl_comm(const unsigned char* uid128, int rank, int nranks, std::string& err) {
  ncclUniqueId id;
  static_assert(sizeof(ncclUniqueId) == 128, "ncclUniqueId size");
  std::memcpy(&id, uid128, sizeof id);
  auto* c = new RcclComm();
  const ncclResult_t r = ncclCommInitRank(&c->c, nranks, id, rank);
  if (r != ncclSuccess) {
    err = std::string("ncclCommInitRank: ") + ncclGetErrorString(r);
    c->c = nullptr;
    delete c;
    return nullptr;
  }
  c->rank = rank;
  const char* chk = std::getenv("G2OHIP_COMM_CHECK");
  c->check_all = !(chk && *chk) ? kCheckFirst : (std::strcmp(chk, "0") != 0 ? -1 : 0);
  c->check_left = c->check_all;
  return c;
}

Comm* make_local_comm(const std::string& key, int rank, int nranks) {
  if (key.rfind("solo:", 0) == 0) return new SoloComm();  // timing only: no other rank exists
  auto* c = new LocalComm();
  c->g = group_for(key, nranks);
  c->rank = rank;
  return c;
}

void local_comm_reduce_host(const std::string& key, int rank, int nranks, double* buf, size_t n, bool is_max) {
  // one call counter per (group, rank) for the host-only entry point
  static std::mutex mu;
  static std::map<std::string, long long> seqs;
  long long seq;
  {
    std::lock_guard<std::mutex> lk(mu);
    seq = seqs[key + "#" + std::to_string(nranks) + "@" + std::to_string(rank)]++;
  }
  group_for(key, nranks)->reduce(rank, seq, buf, buf, n, is_max ? OP_MAX : OP_SUM);
}

}  // namespace g2ohip
