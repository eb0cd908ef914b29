// hg_err.hpp — where an HG_ERR_HIP came from.  Every site that turns a HIP
// runtime failure into HG_ERR_HIP writes HG_HIP_FAIL instead, which records
// the source location and the runtime's own error (hipPeekAtLastError) in a
// process-wide slot read back through hg_last_hip_error() (worker threads of
// the multi-context driver fail on threads the caller never sees).
#pragma once

namespace hgerr {
void note(const char* file, int line);
}  // namespace hgerr

#define HG_HIP_FAIL (::hgerr::note(__FILE__, __LINE__), HG_ERR_HIP)

namespace hgerr {
int launch_status(const char* file, int line);
}  // namespace hgerr

// After kernel launches: HG_OK, or HG_ERR_HIP with the launch error recorded
// (hipGetLastError also clears it, so it is read exactly once, here).
#define HG_LAUNCH_STATUS() (::hgerr::launch_status(__FILE__, __LINE__))
