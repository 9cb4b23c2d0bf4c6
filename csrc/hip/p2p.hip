// One-shot peer-to-peer allreduce of a few doubles over xGMI.
//
// The reference's per-iteration global sums are 8-byte MPI_Allreduce calls
// preceded by a device sync (poisson_mpi_cuda2.cu:842, :871, :892, :925;
// SURVEY C26).  The solver here needs one 7-double sum per iteration; RCCL's
// allreduce for that is a latency-bound ring.  This kernel instead writes
// the local vector straight into a slot of every peer's receive buffer
// (fine-grained memory, IPC-mapped over xGMI), publishes it with a
// system-scope release of a sequence number, then waits for all P slots of
// its own buffer and sums them in rank order — every rank adds the same
// numbers in the same order, so the result is bitwise identical on all ranks
// (and run to run).  Two slot sets alternate by sequence parity: a rank can
// only reuse a set after every peer has published the next sequence, i.e.
// after that peer finished reading the set.
#include <hip/hip_runtime.h>

#include "kernels.hpp"

namespace pe {
namespace dev {
namespace {

// value of the 100 MHz constant clock (s_memrealtime)
__device__ __forceinline__ unsigned long long rtc() { return __builtin_amdgcn_s_memrealtime(); }

__global__ void kP2PSum(double* d, int n, double* const* peers, int me, int P, unsigned long long seq,
                        double timeout_s) {
  const int t = threadIdx.x;
  const int set = int(seq & 1);
  __shared__ int ok;
  if (t == 0) ok = 1;
  __syncthreads();
  if (t < P) {  // push my vector into slot [set][me] of peer t
    double* dst = peers[t] + (size_t(set) * P + me) * kP2PSlot;
    for (int i = 0; i < n; ++i) dst[i] = d[i];
    __hip_atomic_store(reinterpret_cast<unsigned long long*>(dst + kP2PSlot - 1), seq, __ATOMIC_RELEASE,
                       __HIP_MEMORY_SCOPE_SYSTEM);
  }
  if (t < P) {  // wait for slot [set][t] of my own buffer
    const unsigned long long* flag =
        reinterpret_cast<const unsigned long long*>(peers[me] + (size_t(set) * P + t) * kP2PSlot + kP2PSlot - 1);
    const unsigned long long t0 = rtc(), lim = (unsigned long long)(timeout_s * 1e8);
    while (__hip_atomic_load(flag, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_SYSTEM) != seq) {
      __builtin_amdgcn_s_sleep(1);
      if (rtc() - t0 > lim) {  // a peer never arrived: poison instead of hanging (the solver stops, status 4)
        ok = 0;
        break;
      }
    }
  }
  __syncthreads();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
  if (t < n) {
    double s = 0.0;
    for (int r = 0; r < P; ++r)
      s += __hip_atomic_load(peers[me] + (size_t(set) * P + r) * kP2PSlot + t, __ATOMIC_RELAXED,
                             __HIP_MEMORY_SCOPE_SYSTEM);
    d[t] = ok ? s : __builtin_nan("");
  }
}

}  // namespace

void launch_p2p_sum(double* d, int n, double* const* peers, int me, int P, unsigned long long seq, double timeout_s,
                    hipStream_t s) {
  hipLaunchKernelGGL(kP2PSum, dim3(1), dim3(64), 0, s, d, n, peers, me, P, seq, timeout_s);
}

}  // namespace dev
}  // namespace pe
