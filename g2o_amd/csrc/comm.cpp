// Comm implementations (see comm.hpp).
#include "comm.hpp"

#include <rccl/rccl.h>

#include <algorithm>
#include <condition_variable>
#include <cstring>
#include <map>
#include <memory>
#include <mutex>
#include <vector>

#include "common.hpp"

namespace g2ohip {

namespace {

struct RcclComm : Comm {
  ncclComm_t c = nullptr;
  ~RcclComm() override {
    if (c) ncclCommDestroy(c);
  }
  void allreduce_sum(double* p, size_t n, hipStream_t s) override {
    const ncclResult_t r = ncclAllReduce(p, p, n, ncclDouble, ncclSum, c, s);
    if (r != ncclSuccess) throw DeviceError(std::string("ncclAllReduce(sum): ") + ncclGetErrorString(r));
  }
  void allreduce_max(double* p, size_t n, hipStream_t s) override {
    const ncclResult_t r = ncclAllReduce(p, p, n, ncclDouble, ncclMax, c, s);
    if (r != ncclSuccess) throw DeviceError(std::string("ncclAllReduce(max): ") + ncclGetErrorString(r));
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
  explicit Group(int n) : nranks(n), bufs(n) {}
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
};
std::mutex g_groups_mu;
std::map<std::string, std::shared_ptr<Group>> g_groups;

struct LocalComm : Comm {
  std::shared_ptr<Group> g;
  int rank;
  void reduce(double* p, size_t n, hipStream_t s, bool is_max) {
    std::vector<double>& mine = g->bufs[rank];
    mine.resize(n);
    HIP_CHECK(hipMemcpyAsync(mine.data(), p, n * sizeof(double), hipMemcpyDeviceToHost, s));
    HIP_CHECK(hipStreamSynchronize(s));
    g->barrier();
    std::vector<double> out(g->bufs[0]);
    for (int r = 1; r < g->nranks; ++r)
      for (size_t k = 0; k < n; ++k) out[k] = is_max ? std::max(out[k], g->bufs[r][k]) : out[k] + g->bufs[r][k];
    g->barrier();  // everyone has read every buffer
    HIP_CHECK(hipMemcpyAsync(p, out.data(), n * sizeof(double), hipMemcpyHostToDevice, s));
    HIP_CHECK(hipStreamSynchronize(s));
  }
  void allreduce_sum(double* p, size_t n, hipStream_t s) override { reduce(p, n, s, false); }
  void allreduce_max(double* p, size_t n, hipStream_t s) override { reduce(p, n, s, true); }
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
  return c;
}

Comm* make_local_comm(const std::string& key, int rank, int nranks) {
  std::lock_guard<std::mutex> lk(g_groups_mu);
  auto& slot = g_groups[key + "#" + std::to_string(nranks)];
  if (!slot) slot = std::make_shared<Group>(nranks);
  auto* c = new LocalComm();
  c->g = slot;
  c->rank = rank;
  return c;
}

}  // namespace g2ohip
