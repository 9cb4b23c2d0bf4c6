// Device helpers shared by the gfx950 kernel files (kernels.hip, fused.hip):
// constant-address-space table reads, fictitious-domain coefficients from the
// chord tables + row classes, the 5-point operator in both arithmetic
// variants, wave64 DPP / readlane helpers, and the deterministic
// last-workgroup reduction protocol.
#pragma once

#include <hip/hip_runtime.h>

#include "kernels.hpp"
#include "pe/decomp.hpp"
#include "pe/problem.hpp"

namespace pe {
namespace dev {
namespace {

constexpr int TJ = kTJ;
constexpr int SW = kSW;

// Read-only table access through the constant address space: uniform
// addresses lower to s_load (lgkmcnt), so a table read inside the marching
// loop never waits on the vector-memory prefetch queue (vmcnt).
template <class T>
__device__ __forceinline__ T cload(const T* p) {
  return *(const __attribute__((address_space(4))) T*)((uintptr_t)p);
}

__device__ __forceinline__ double fcoef(double l, double h, double eps, double inv_eps) {
  if (fabs(l - h) < 1e-9) return 1.0;
  if (l < 1e-9) return inv_eps;
  return (l / h) + (1.0 - l / h) / eps;
}

// Per-column chord-table values of one node column lj: the vertical-face
// y-range (sA, eA) and the horizontal-face half-widths of columns lj, lj+1.
// Kept in registers by the marching kernels (no table loads in the loop).
struct TV {
  double sA, eA, hB, hB1;
};
__device__ __forceinline__ TV tv_at(const KParams& k, int64_t lj) {
  const double* t = k.rowT + (lj + 1) * 4;
  return TV{t[0], t[1], t[2], t[6]};
}

// a_{q, lj}: vertical face left of node q.  colT is indexed by the
// wave-uniform row q → scalar loads, which do not drain vector-memory prefetch.
__device__ __forceinline__ double coefA(const KParams& k, int64_t q, const TV& t) {
  const double half = cload(k.colT + (q + 1) * 4 + 0);
  return fcoef(chord_len(half, t.sA, t.eA), k.h2, k.eps, k.inv_eps);
}
// b_{q, ·}: horizontal face below the node, chord half-width `half`.
__device__ __forceinline__ double coefB(const KParams& k, int64_t q, double half) {
  const double sB = cload(k.colT + (q + 1) * 4 + 1);
  const double eB = cload(k.colT + (q + 1) * 4 + 2);
  return fcoef(chord_len(half, sB, eB), k.h1, k.eps, k.inv_eps);
}

// Coefficients of node (q, lj): a(q), a(q+1), b(q, lj), b(q, lj+1), and the
// Jacobi diagonal (EXACT: D, used as r / D; fast: 1/D, used as r * dinv).
struct CS {
  double a0, a1, b0, b1, d;
};

template <bool EXACT>
__device__ __forceinline__ CS cset(const KParams& k, const int* rc, int64_t q, int64_t lj, const TV& t) {
  CS c;
  const int in_lo = cload(rc), in_hi = cload(rc + 1), out_lo = cload(rc + 2), out_hi = cload(rc + 3);
  if (lj >= in_lo && lj <= in_hi) {  // interior: every face fully inside D
    c.a0 = c.a1 = c.b0 = c.b1 = 1.0;
    c.d = EXACT ? k.D_in : k.dinv_in;
  } else if (lj < out_lo || lj > out_hi) {  // exterior: every face fully outside D
    c.a0 = c.a1 = c.b0 = c.b1 = k.inv_eps;
    c.d = EXACT ? k.D_out : k.dinv_out;
  } else {  // boundary band: evaluate the face lengths
    c.a0 = coefA(k, q, t);
    c.a1 = coefA(k, q + 1, t);
    c.b0 = coefB(k, q, t.hB);
    c.b1 = coefB(k, q, t.hB1);
    // D = (a_{i+1} + a_i)/h1² + (b_{j+1} + b_j)/h2²  (reference mat_D, same order)
    if constexpr (EXACT) c.d = (c.a1 + c.a0) / k.h1sq + (c.b1 + c.b0) / k.h2sq;
    else c.d = 1.0 / ((c.a1 + c.a0) * k.ih1sq + (c.b1 + c.b0) * k.ih2sq);
  }
  return c;
}
template <bool EXACT>
__device__ __forceinline__ CS cset_mem(const KParams& k, int64_t q, int64_t lj) {
  return cset<EXACT>(k, k.rowcls + (q + 1) * 4, q, lj, tv_at(k, lj));
}

template <bool EXACT>
__device__ __forceinline__ double zval(const CS& c, double r) {
  if constexpr (EXACT) return (c.d != 0.0) ? r / c.d : 0.0;
  else return r * c.d;
}

template <bool EXACT>
__device__ __forceinline__ double stencil(const KParams& k, const CS& c, double pm, double p0, double pn, double pl,
                                          double pr) {
  if constexpr (EXACT) {
    // Reference apply_A (poisson_mpi_cuda2.cu:526-535), same expression tree.
    const double Ax = k.nih1 * (c.a1 * (pn - p0) / k.h1 - c.a0 * (p0 - pm) / k.h1);
    const double Ay = k.nih2 * (c.b1 * (pr - p0) / k.h2 - c.b0 * (p0 - pl) / k.h2);
    return Ax + Ay;
  } else {
    return (c.a0 * (p0 - pm) - c.a1 * (pn - p0)) * k.ih1sq + (c.b0 * (p0 - pl) - c.b1 * (pr - p0)) * k.ih2sq;
  }
}

__device__ __forceinline__ bool row_valid(const KParams& k, int64_t q) {
  return (q >= 1 && q <= k.nx) || (q == 0 && k.has[LEFT]) || (q == k.nx + 1 && k.has[RIGHT]);
}
// Is local node (q, lj) a value this rank computes (owned, or a halo node
// whose neighbour exists)?  Global-boundary halos and halo corners are not.
__device__ __forceinline__ bool valid_node(const KParams& k, int64_t q, int64_t lj) {
  const bool rin = q >= 1 && q <= k.nx;
  const bool cin = lj >= 1 && lj <= k.ny;
  const bool ch = (lj == 0 && k.has[DOWN]) || (lj == k.ny + 1 && k.has[UP]);
  return (rin && (cin || ch)) || (row_valid(k, q) && !rin && cin);
}

__device__ __forceinline__ double load_r(const KParams& k, int64_t q, int64_t lj) {
  if (lj == 0) return k.recv_dn[q - 1];
  if (lj == k.ny + 1) return k.recv_up[q - 1];
  return k.r[q * k.pitch + lj];
}

// ---- wave-level helpers -------------------------------------------------
__device__ __forceinline__ double dpp_shr1(double v) {  // lane l ← lane l-1 (lane 0 ← 0)
  const long long x = __builtin_bit_cast(long long, v);
  const int lo = __builtin_amdgcn_update_dpp(0, int(x), 0x138, 0xF, 0xF, true);
  const int hi = __builtin_amdgcn_update_dpp(0, int(x >> 32), 0x138, 0xF, 0xF, true);
  return __builtin_bit_cast(double, (static_cast<long long>(hi) << 32) | static_cast<unsigned>(lo));
}
__device__ __forceinline__ double dpp_shl1(double v) {  // lane l ← lane l+1 (lane 63 ← 0)
  const long long x = __builtin_bit_cast(long long, v);
  const int lo = __builtin_amdgcn_update_dpp(0, int(x), 0x130, 0xF, 0xF, true);
  const int hi = __builtin_amdgcn_update_dpp(0, int(x >> 32), 0x130, 0xF, 0xF, true);
  return __builtin_bit_cast(double, (static_cast<long long>(hi) << 32) | static_cast<unsigned>(lo));
}
__device__ __forceinline__ double readlane(double v, int l) {
  const long long x = __builtin_bit_cast(long long, v);
  const int lo = __builtin_amdgcn_readlane(int(x), l);
  const int hi = __builtin_amdgcn_readlane(int(x >> 32), l);
  return __builtin_bit_cast(double, (static_cast<long long>(hi) << 32) | static_cast<unsigned>(lo));
}

// Deterministic block reduction of N sums (or maxima) → thread 0.
template <int N, bool MAX>
__device__ __forceinline__ void block_reduce(double (&v)[N], double* sm) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1)
#pragma unroll
    for (int n = 0; n < N; ++n) {
      const double t = __shfl_xor(v[n], o, 64);
      v[n] = MAX ? fmax(v[n], t) : v[n] + t;
    }
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  if (lane == 0)
#pragma unroll
    for (int n = 0; n < N; ++n) sm[n * 4 + wid] = v[n];
  __syncthreads();
  if (threadIdx.x == 0)
#pragma unroll
    for (int n = 0; n < N; ++n)
      v[n] = MAX ? fmax(fmax(sm[n * 4], sm[n * 4 + 1]), fmax(sm[n * 4 + 2], sm[n * 4 + 3]))
                 : ((sm[n * 4] + sm[n * 4 + 1]) + sm[n * 4 + 2]) + sm[n * 4 + 3];
}

// Publish this block's partials and take a ticket; true in the block that
// arrives last (all partials visible to it).  Protocol: producer store →
// vmcnt(0) → agent release → vmcnt(0) → relaxed agent fetch_add; the last
// arriver does an agent acquire before reading (cdna_hip_programming §6 G16).
__device__ __forceinline__ bool arrive_last(unsigned* ticket, unsigned nblocks, int* sflag) {
  if (threadIdx.x == 0) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    const unsigned t = __hip_atomic_fetch_add(ticket, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const int last = (t == nblocks - 1);
    if (last) {
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    *sflag = last;
  }
  __syncthreads();
  return *sflag != 0;
}

// Wave-level form of arrive_last for paths that waves of one workgroup reach
// at different program points (no workgroup barrier): every wave of the grid
// drains and releases its stores, then lane 0 takes a ticket counted against
// all `nwaves` waves; true (wave-uniform) in the wave that arrives last, after
// its acquire.
__device__ __forceinline__ bool arrive_last_wave(unsigned* ticket, unsigned nwaves) {
  int last = 0;
  if ((threadIdx.x & 63) == 0) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    const unsigned t = __hip_atomic_fetch_add(ticket, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    last = (t == nwaves - 1);
    if (last) {
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
  }
  return __builtin_amdgcn_readfirstlane(last) != 0;
}

// Write-through form of arrive_last for a block's N partial sums (thread 0
// holds them): stored `sc1` (relaxed agent-scope atomic stores), drained,
// then the ticket — no per-block L2 write-back (`buffer_wbl2`, ≈1.7-6.5 µs
// on a dirty L2, paid by every block of the grid); the last arriver does
// the agent acquire before reading (the image's CDNA4 guide,
// /opt/skills/guides/MI355X_MICROARCH.md — not part of this repo — visibility recipe R1).
template <int N>
__device__ __forceinline__ bool publish_last(double* dst, const double (&v)[N], unsigned* ticket, unsigned nblocks,
                                             int* sflag) {
  if (threadIdx.x == 0) {
#pragma unroll
    for (int n = 0; n < N; ++n) __hip_atomic_store(dst + n, v[n], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    const unsigned t = __hip_atomic_fetch_add(ticket, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const int last = (t == nblocks - 1);
    if (last) {
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    *sflag = last;
  }
  __syncthreads();
  return *sflag != 0;
}

// Sum N-tuples of partials [nblocks][N] in block order (deterministic).
// Two tuples per thread are loaded before either is added (the same sums in
// the same order): the grid's last block reads 512 tuples written by other
// XCDs, and one latency per pair instead of per tuple shortens the sweep's
// epilogue (last wave exit → state finalized: 9-10 µs, tools/stamp_probe.py).
template <int N>
__device__ __forceinline__ void reduce_partials(const double* partial, unsigned nblocks, double (&v)[N], double* sm) {
#pragma unroll
  for (int n = 0; n < N; ++n) v[n] = 0.0;
  unsigned m = threadIdx.x;
  for (; m + TJ < nblocks; m += 2 * TJ) {
    double a[N], b[N];
#pragma unroll
    for (int n = 0; n < N; ++n) {
      a[n] = partial[size_t(m) * N + n];
      b[n] = partial[size_t(m + TJ) * N + n];
    }
#pragma unroll
    for (int n = 0; n < N; ++n) v[n] = (v[n] + a[n]) + b[n];
  }
  if (m < nblocks)
#pragma unroll
    for (int n = 0; n < N; ++n) v[n] += partial[size_t(m) * N + n];
  block_reduce<N, false>(v, sm);
}

// ---- the s-step sweeps' grid reduction (kS3 / kSS) -------------------------
// Wave64 sum of one double by DPP (row_shr 1/2/4/8, then row_bcast 15/31):
// lane 63 ends with the total, in a fixed order (the same bits in every
// workgroup; no LDS round trips, unlike the __shfl_xor tree's ds_bpermute
// pairs).  Identity 0.0 for lanes a step does not feed.
template <int CTRL, int RM, int BM>
__device__ __forceinline__ double dpp_d(double v) {
  const long long x = __builtin_bit_cast(long long, v);
  const int lo = __builtin_amdgcn_update_dpp(0, int(x), CTRL, RM, BM, false);
  const int hi = __builtin_amdgcn_update_dpp(0, int(x >> 32), CTRL, RM, BM, false);
  return __builtin_bit_cast(double, (static_cast<long long>(hi) << 32) | static_cast<unsigned>(lo));
}
__device__ __forceinline__ double wave_sum63(double v) {
  v += dpp_d<0x111, 0xF, 0xF>(v);  // row_shr:1
  v += dpp_d<0x112, 0xF, 0xF>(v);  // row_shr:2
  v += dpp_d<0x114, 0xF, 0xE>(v);  // row_shr:4
  v += dpp_d<0x118, 0xF, 0xC>(v);  // row_shr:8
  v += dpp_d<0x142, 0xA, 0xF>(v);  // row_bcast:15
  v += dpp_d<0x143, 0xC, 0xF>(v);  // row_bcast:31
  return v;
}

// Block sums of N values → the grid's partials, laid out n-major
// (partial[n · nblocks + b]: the last block's loads are coalesced), one store
// instruction from lanes 0..N-1 of wave 0, then the ticket; true in the block
// that arrives last (after its acquire).  Replaces block_reduce + publish_last
// + reduce_partials for the sweeps' 19 sums: block-major tuples made the last
// block's reduction 9728 single-line lane requests, 4.6 µs of every sweep's
// epilogue (tools/stamp_probe.py "last block" line, profiles/r5_epilogue.txt).
template <int N>
__device__ __forceinline__ bool publish_last_nm(double* partial, const double (&v)[N], unsigned* ticket, int* sflag,
                                                double* sm) {
  static_assert(N <= 64, "one store instruction: lanes 0..N-1 of wave 0");
  const int lane = int(threadIdx.x & 63), wid = __builtin_amdgcn_readfirstlane(int(threadIdx.x >> 6));
  double w[N];
#pragma unroll
  for (int n = 0; n < N; ++n) w[n] = wave_sum63(v[n]);
  if (lane == 63)
#pragma unroll
    for (int n = 0; n < N; ++n) sm[n * kWPB + wid] = w[n];
  __syncthreads();
  if (wid == 0) {
    if (lane < N) {
      double s = sm[lane * kWPB];
#pragma unroll
      for (int q = 1; q < kWPB; ++q) s += sm[lane * kWPB + q];
      __hip_atomic_store(partial + size_t(lane) * gridDim.x + blockIdx.x, s, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    if (lane == 0) {
      const unsigned t = __hip_atomic_fetch_add(ticket, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      const int last = (t == gridDim.x - 1);
      if (last) {
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      }
      *sflag = last;
    }
  }
  __syncthreads();
  return *sflag != 0;
}

// The last block: the N grid sums from publish_last_nm's partials → thread 0.
// Wave q sums the values n ≡ q (mod kWPB); every lane loads its blocks
// lane, lane + 64, … (all loads of up to 512 blocks issued before the first
// add), then a DPP wave sum.  Deterministic: the order depends on nblocks only.
template <int N>
__device__ __forceinline__ void reduce_partials_nm(const double* partial, double (&t)[N], double* sm) {
  const int lane = int(threadIdx.x & 63), wid = __builtin_amdgcn_readfirstlane(int(threadIdx.x >> 6));
  const unsigned nb = gridDim.x;
  constexpr int PER = (N + kWPB - 1) / kWPB, U = 8;
  double s[PER];
#pragma unroll
  for (int j = 0; j < PER; ++j) s[j] = 0.0;
  for (unsigned m0 = 0; m0 < nb; m0 += U * 64) {
    double x[PER][U];
#pragma unroll
    for (int j = 0; j < PER; ++j)
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int n = wid + kWPB * j;
        const unsigned m = m0 + unsigned(64 * u + lane);
        x[j][u] = (n < N && m < nb) ? partial[size_t(n) * nb + m] : 0.0;
      }
#pragma unroll
    for (int j = 0; j < PER; ++j)
#pragma unroll
      for (int u = 0; u < U; ++u) s[j] += x[j][u];
  }
#pragma unroll
  for (int j = 0; j < PER; ++j) s[j] = wave_sum63(s[j]);
  __syncthreads();  // (sm: publish_last_nm's reads are done)
  if (lane == 63)
#pragma unroll
    for (int j = 0; j < PER; ++j)
      if (wid + kWPB * j < N) sm[wid + kWPB * j] = s[j];
  __syncthreads();
  if (threadIdx.x == 0)
#pragma unroll
    for (int n = 0; n < N; ++n) t[n] = sm[n];
}

// One p_k value at a single node (strip-edge columns, prologue only).
template <bool EXACT>
__device__ __forceinline__ double p_point(const KParams& k, int64_t q, int64_t lj, double beta, const double* pold) {
  return zval<EXACT>(cset_mem<EXACT>(k, q, lj), load_r(k, q, lj)) + beta * pold[q * k.pitch + lj];
}

// Unconditional 16-byte load (address already clamped in range): a
// predicated load would make hipcc branch around it and drain vmcnt(0),
// which serialises the row prefetch (measured in the .s).
__device__ __forceinline__ double2 ld2(const double* p) { return *reinterpret_cast<const double2*>(p); }

// Row class (interior interval / exterior hull) of one row, in SGPRs.
struct RowCls {
  int in_lo, in_hi, out_lo, out_hi;
};
__device__ __forceinline__ RowCls rcl_read(const int4& v, int l) {
  return RowCls{__builtin_amdgcn_readlane(v.x, l), __builtin_amdgcn_readlane(v.y, l),
                __builtin_amdgcn_readlane(v.z, l), __builtin_amdgcn_readlane(v.w, l)};
}
// Does columns [jlo, jhi] of this row contain a boundary-band node?  (scalar)
__device__ __forceinline__ bool has_gen(const RowCls& c, int64_t jlo, int64_t jhi) {
  const int64_t lo = max(jlo, int64_t(c.out_lo)), hi = min(jhi, int64_t(c.out_hi));
  if (lo > hi) return false;
  if (c.in_lo > c.in_hi) return true;
  return lo < c.in_lo || hi > c.in_hi;
}
// Coefficients of a node in a row without boundary-band nodes in this strip.
template <bool EXACT>
__device__ __forceinline__ CS cset_fast(const KParams& k, const RowCls& c, int64_t lj) {
  const bool in = lj >= c.in_lo && lj <= c.in_hi;
  const double f = in ? 1.0 : k.inv_eps;
  CS cs;
  cs.a0 = cs.a1 = cs.b0 = cs.b1 = f;
  cs.d = EXACT ? (in ? k.D_in : k.D_out) : (in ? k.dinv_in : k.dinv_out);
  return cs;
}

// Division-free face coefficient (single-sweep path): l·(1/h) and ·(1/eps)
// instead of the reference's l/h and /eps — one rounding apart, and it keeps
// boundary-band rows (4 coefficients × 3 uses per row) from costing 24 fp64
// divisions per lane and row.
__device__ __forceinline__ double fcoef_fast(double l, double h, double inv_h, double inv_eps) {
  if (fabs(l - h) < 1e-9) return 1.0;
  if (l < 1e-9) return inv_eps;
  const double t = l * inv_h;
  return t + (1.0 - t) * inv_eps;
}

// 1/x for the band diagonal (x = a sum of positive face terms ≥ 2/h², far
// from denormal / overflow): hardware reciprocal + two Newton steps, ≤ 1 ulp
// from the IEEE quotient — 5 instructions instead of the ≈10 of the scaled
// IEEE division sequence.
__device__ __forceinline__ double rcp_nr(double x) {
  double r = __builtin_amdgcn_rcp(x);
  double e = fma(-x, r, 1.0);
  r = fma(r, e, r);
  e = fma(-x, r, 1.0);
  return fma(r, e, r);
}

// Column-table values of one row q: chord half-width at the faces left of
// rows q and q+1 (vertical faces), and the y-range of the row's horizontal
// faces.  The single-sweep kernel reads them from lanes (one row per lane,
// loaded with the row classes), never through scalar loads in the loop.
struct CT {
  double half0, half1, sB, eB;
};

// 1/D from the four face coefficients (fast arithmetic; the one expression
// every single-sweep path uses, so a diagonal recomputed from stored faces
// has the bits of the one evaluated with them).
__device__ __forceinline__ double dinv_faces(const KParams& k, double a0, double a1, double b0, double b1) {
  return rcp_nr(fma(a1 + a0, k.ih1sq, (b1 + b0) * k.ih2sq));
}

// cset with the row class already in SGPRs (fast arithmetic).
__device__ __forceinline__ CS cset_rc(const KParams& k, const RowCls& c, const CT& ct, int64_t lj, const TV& t) {
  CS x;
  if (lj >= c.in_lo && lj <= c.in_hi) {
    x.a0 = x.a1 = x.b0 = x.b1 = 1.0;
    x.d = k.dinv_in;
  } else if (lj < c.out_lo || lj > c.out_hi) {
    x.a0 = x.a1 = x.b0 = x.b1 = k.inv_eps;
    x.d = k.dinv_out;
  } else {
    const double ih1 = -k.nih1, ih2 = -k.nih2;
    x.a0 = fcoef_fast(chord_len(ct.half0, t.sA, t.eA), k.h2, ih2, k.inv_eps);
    x.a1 = fcoef_fast(chord_len(ct.half1, t.sA, t.eA), k.h2, ih2, k.inv_eps);
    x.b0 = fcoef_fast(chord_len(t.hB, ct.sB, ct.eB), k.h1, ih1, k.inv_eps);
    x.b1 = fcoef_fast(chord_len(t.hB1, ct.sB, ct.eB), k.h1, ih1, k.inv_eps);
    x.d = dinv_faces(k, x.a0, x.a1, x.b0, x.b1);
  }
  return x;
}

}  // namespace
}  // namespace dev
}  // namespace pe
