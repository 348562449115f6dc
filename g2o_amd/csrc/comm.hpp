// Collectives of the landmark-sharded BA path: one sum all-reduce of the
// reduced camera system [Hschur upper blocks | bschur] per LM trial plus scalar reductions.
//
//   RcclComm   production transport: ncclAllReduce on the solver's stream (RCCL over xGMI).
//   LocalComm  test transport: N engines driven by N host threads of ONE process on one GPU;
//              host-staged, summed in rank order. Lets the sharding logic run under pytest on
//              a single-GPU box; never selected by the product path.
#pragma once
#include <hip/hip_runtime.h>

#include <cstddef>
#include <string>

namespace g2ohip {

struct Comm {
  virtual ~Comm() = default;
  virtual void allreduce_sum(double* dptr, size_t n, hipStream_t s) = 0;
  virtual void allreduce_max(double* dptr, size_t n, hipStream_t s) = 0;
};

Comm* make_rccl_comm(const unsigned char* uid128, int rank, int nranks, std::string& err);
Comm* make_local_comm(const std::string& key, int rank, int nranks);

}  // namespace g2ohip
