// HIP runtime helpers: fail-loud error handling (reference checkCuda just
// exit()s one rank and can hang its peers — quirk A18; here the message
// names the rank/device and the process aborts, which tears down RCCL peers
// through the launcher), device selection (the reference never calls
// cudaSetDevice — quirk A5).
#include <hip/hip_runtime_api.h>

#include <cstdio>
#include <cstdlib>

#include "pe/device.hpp"

namespace pe {

void hip_fail(hipError_t e, const char* expr, const char* file, int line) {
  const char* rank = std::getenv("RANK");
  std::fprintf(stderr, "[pe] HIP error %d (%s) at %s:%d in `%s` (rank %s)\n", int(e), hipGetErrorString(e),
               file, line, expr, rank ? rank : "0");
  std::fflush(stderr);
  std::abort();
}

int device_count() {
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess) return 0;
  return n;
}

void set_device(int dev) { PE_HIP_CHECK(hipSetDevice(dev)); }

int current_device() {
  int d = -1;
  PE_HIP_CHECK(hipGetDevice(&d));
  return d;
}

// "dddd:bb:dd.f" of a device: which physical GPU a rank drives (bench.py
// reports it per rank, so "N ranks on N distinct GPUs" is checkable).
std::string device_pci_bus_id(int dev) {
  char buf[64] = {0};
  PE_HIP_CHECK(hipDeviceGetPCIBusId(buf, int(sizeof buf), dev));
  return std::string(buf);
}

std::string device_name(int dev) {
  hipDeviceProp_t p;
  PE_HIP_CHECK(hipGetDeviceProperties(&p, dev));
  return std::string(p.name) + " (" + p.gcnArchName + ", " + std::to_string(p.multiProcessorCount) + " CUs, " +
         std::to_string(p.totalGlobalMem >> 30) + " GiB)";
}

}  // namespace pe
