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

}  // namespace g2ohip
