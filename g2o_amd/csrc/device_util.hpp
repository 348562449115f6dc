// Small device helpers shared by the HIP translation units.
#pragma once
#include <hip/hip_runtime.h>

namespace g2ohip {

// Load that never branches: the address is selected and the value masked. A guarded load
// (`ok ? p[i] : 0`) compiles to a branch with its own s_waitcnt, which serialises every load of an
// unrolled batch; this form keeps the whole batch in flight. p[0] must be a valid address.
template <class T>
__device__ __forceinline__ T ld0(const T* p, int idx, bool ok) {
  const T v = p[ok ? idx : 0];
  return ok ? v : T(0);
}

// XCD-aware workgroup order: the dispatcher deals workgroups to the 8 XCDs round-robin; this
// bijection gives XCD x a contiguous range of work items [x*n/8, (x+1)*n/8), so neighbouring items
// (camera rows that share landmarks) run side by side behind the same L2.
__device__ __forceinline__ int xcd_item(int bid, int n) {
  const int xcd = bid & 7, q = n >> 3, r = n & 7;
  return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (bid >> 3);
}

}  // namespace g2ohip
