// Helpers shared by the DeviceSolver translation units (device_solver.cpp,
// item_layout.cpp, placement.cpp, checkpoint.cpp).  Internal: not installed,
// not part of the pe/ API.
#pragma once

#include <chrono>
#include <cstddef>

#include <rocprofiler-sdk-roctx/roctx.h>

namespace pe {
namespace detail {
// Host-side phase ranges for rocprofv3 --marker-trace (no-ops without a tool).
struct Range {
  explicit Range(const char* n) { roctxRangePushA(n); }
  ~Range() { roctxRangePop(); }
};
using clk = std::chrono::steady_clock;
inline double secs(clk::time_point a, clk::time_point b) { return std::chrono::duration<double>(b - a).count(); }

// Field allocation (placement.cpp): hipMalloc; field_try_alloc returns
// nullptr when the device is out of memory, field_alloc throws.
void* field_try_alloc(size_t bytes);
void* field_alloc(size_t bytes);
void field_free(void* p);
}  // namespace detail
}  // namespace pe
