// expm.hip — batched matrix exponential for the model build (expm.py:9-167).
// Placeholder until the MFMA implementation lands: reports "not supported".
#include <hip/hip_runtime.h>

#include "sweeps.h"

namespace itr {
size_t expm_workspace_bytes(int, int64_t) { return 0; }
hipError_t launch_expm_batched(int, int64_t, const double*, double*, double*, hipStream_t) {
  return hipErrorNotSupported;
}
}  // namespace itr
