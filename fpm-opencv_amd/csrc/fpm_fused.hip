// fpm_fused.hip -- placeholder until the fused per-patch kernel lands.
#include <hip/hip_runtime.h>
#include "fpm_state.hpp"
namespace fpm {
bool fused_supported(int, int, int) { return false; }
size_t fused_meas_bytes(int, int, int) { return 16; }
hipError_t fused_prepare(const DevState &, uint16_t *, hipStream_t) { return hipErrorNotSupported; }
hipError_t launch_fused_iteration(const DevState &, const uint16_t *, const int *, const int *, const int *, int,
                                  hipStream_t) {
    return hipErrorNotSupported;
}
}  // namespace fpm
