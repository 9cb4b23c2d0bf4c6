// Cross-rank sum of a few doubles over xGMI, as a block-cooperative device
// function: the standalone one-shot allreduce kernel (p2p.hip) and the
// sweep's final reduction (fused.hip — the per-iteration sums then need no
// separate allreduce launch) share it.
//
// Every rank owns a fine-grained receive buffer of 2 × P slots (kP2PSlot
// doubles: values, then a sequence flag), IPC-mapped into every peer
// (PeerSum::peers[r] = rank r's buffer; peers[me] = our own).  Reduction q
// (q = 1, 2, … from a per-rank device counter — ranks run the same sequence
// of reductions) writes the local values into slot [q & 1][me] of every
// peer's buffer and publishes them with a system-scope release of flag = q,
// waits for the P flags of slot set q & 1 of its own buffer, and sums the P
// slots in rank order: every rank adds the same numbers in the same order,
// so the result is bitwise identical on all ranks.  A slot set is reused two
// reductions later, which a rank only reaches after every peer has
// published reduction q + 1 — i.e. after that peer finished reading set q & 1.
// A peer that never arrives within the timeout poisons the result (NaN) so
// the solver stops with a non-finite status instead of hanging.
#pragma once

#include <hip/hip_runtime.h>

#include "kernels.hpp"

namespace pe {
namespace dev {

// The wait (from this rank's flag release to the last peer's flag) is
// accumulated into ps.wait_acc when set: the cross-rank part of T_MPI.
__device__ __forceinline__ void peer_sum_block(const PeerSum& ps, double* v, int n, unsigned long long* sseq,
                                               int* sok) {
  unsigned long long tw = 0;
  if (threadIdx.x == 0) {
    const unsigned long long q = *ps.seq + 1;
    *ps.seq = q;
    *sseq = q;
    *sok = 1;
    tw = __builtin_amdgcn_s_memrealtime();
  }
  __syncthreads();
  const unsigned long long seq = *sseq;
  const size_t set = size_t(seq & 1);
  const int t = int(threadIdx.x);
  if (t < ps.P) {
    double* dst = ps.peers[t] + (set * size_t(ps.P) + size_t(ps.me)) * kP2PSlot;
    for (int i = 0; i < n; ++i) dst[i] = v[i];
    __hip_atomic_store(reinterpret_cast<unsigned long long*>(dst + kP2PSlot - 1), seq, __ATOMIC_RELEASE,
                       __HIP_MEMORY_SCOPE_SYSTEM);
    const unsigned long long* flag = reinterpret_cast<const unsigned long long*>(
        ps.peers[ps.me] + (set * size_t(ps.P) + size_t(t)) * kP2PSlot + kP2PSlot - 1);
    const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
    // relaxed spin, one acquire after it (an acquire load per spin would
    // invalidate the caches on every poll)
    while (__hip_atomic_load(flag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) != seq) {
      __builtin_amdgcn_s_sleep(1);
      if ((long long)(__builtin_amdgcn_s_memrealtime() - t0) > ps.timeout_ticks) {
        *sok = 0;  // a peer never arrived: poison instead of hanging
        break;
      }
    }
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
  }
  __syncthreads();
  if (threadIdx.x == 0 && ps.wait_acc) {
    ps.wait_acc[0] += __builtin_amdgcn_s_memrealtime() - tw;
    ps.wait_acc[1] += 1;
  }
  if (t < n) {
    double s = 0.0;
    for (int r = 0; r < ps.P; ++r)
      s += __hip_atomic_load(ps.peers[ps.me] + (set * size_t(ps.P) + size_t(r)) * kP2PSlot + t, __ATOMIC_RELAXED,
                             __HIP_MEMORY_SCOPE_SYSTEM);
    v[t] = *sok ? s : __builtin_nan("");
  }
  __syncthreads();
}


}  // namespace dev
}  // namespace pe
