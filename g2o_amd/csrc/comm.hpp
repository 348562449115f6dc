// Collectives of the landmark-sharded BA path: the reduced camera system [Hschur upper blocks | bschur]
// per LM trial (one sum all-reduce, or with the distributed factorization a reduce-scatter of the blocks each rank's
// subtrees read plus an all-reduce of the shared ones) plus scalar reductions.
//
//   RcclComm   production transport: ncclAllReduce / ncclReduceScatter / ncclAllGather on the solver's stream (RCCL
//              over xGMI).
//   LocalComm  test transport: N engines driven by N host threads of ONE process on one GPU;
//              host-staged, summed in rank order. Lets the sharding logic run under pytest on
//              a single-GPU box; never selected by the product path.
//   SoloComm   timing transport (key "solo:..."): one engine plays rank r of N alone, every collective a no-op
//              (tools/dist_rank_times.py); its results are not meaningful.
//
// Every collective carries a per-communicator call number. LocalComm always checks that all ranks
// entered the same call (number, length, operation) and throws DeviceError on every rank otherwise (a
// rank-dependent call sequence was a heap over-read here and a silent hang under RCCL); RcclComm runs
// the same check as one extra 6-double max all-reduce (and a stream synchronisation) per call: for the first 8 calls
// after each structure build by default (rearm), for every call with G2OHIP_COMM_CHECK=1, never with =0.
#pragma once
#include <hip/hip_runtime.h>

#include <cstddef>
#include <string>

namespace g2ohip {

struct Comm {
  virtual ~Comm() = default;
  virtual void allreduce_sum(double* dptr, size_t n, hipStream_t s) = 0;
  virtual void allreduce_max(double* dptr, size_t n, hipStream_t s) = 0;
  // in place: dptr holds nranks segments of `count` doubles; afterwards segment `rank` holds the sum over ranks of that
  // segment (the other segments are left as they were: this rank's own partial values)
  virtual void reduce_scatter_sum(double* dptr, size_t count, hipStream_t s) = 0;
  // in place: dptr holds nranks segments of `count` doubles; afterwards every segment r holds rank r's segment r
  virtual void allgather(double* dptr, size_t count, hipStream_t s) = 0;
  // a new structure (a new collective sequence) starts: RcclComm re-arms its call-sequence check
  virtual void rearm() {}
  long long seq = 0;  // collectives issued so far on this communicator
};

Comm* make_rccl_comm(const unsigned char* uid128, int rank, int nranks, std::string& err);
Comm* make_local_comm(const std::string& key, int rank, int nranks);
// LocalComm's host-side reduction alone (no device copies): the collective-consistency check is testable on a
// host without a GPU. Throws DeviceError on a mismatched call.
void local_comm_reduce_host(const std::string& key, int rank, int nranks, double* buf, size_t n, bool is_max);

}  // namespace g2ohip
