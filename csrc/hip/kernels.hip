// gfx950 (MI355X) kernels of the device-resident Jacobi-PCG solver.
//
// What the reference does per iteration (poisson_mpi_cuda2.cu:846-942):
// 5 kernels (apply_A, dot, update_w_r, apply_Dinv, dot, update_p) on a
// 16x16 block whose threadIdx.x walks the STRIDED dimension, 3 × 256 KiB of
// dot partials copied to the host and summed there, 6 device syncs, and
// a/b/B arrays streamed from HBM every time — ≈21 array passes per point.
//
// What this file does instead (8 array passes per point, 0 host syncs):
//
//   kF  (p update ⊕ stencil ⊕ 2 dots)   reads r, p_{k-1}; writes p_k
//   kG  (stop test ⊕ w,r update ⊕ recomputed stencil ⊕ (z,r) dot)
//                                        reads p_k, r, w; writes r, w
//
// Execution shape (measured: the first LDS-row version spent 85 % of its
// wave cycles in s_waitcnt/s_barrier — latency-bound, not HBM- or
// ALU-bound).  Every wave64 is independent: it owns a strip of 128
// consecutive j (2 per lane, 16-byte loads/stores) and marches down ≤ 64
// rows of i with the NEXT TWO rows' loads already in flight.  The i±1
// stencil neighbours stay in registers, j±1 come from DPP wave shifts
// (v_mov_b32_dpp wave_shl/shr:1), and the two strip-edge columns are
// computed once per work item, one row per lane, and broadcast with
// v_readlane — no LDS and no barrier inside the loop.  Work items
// (strip × row chunk) are dealt to a persistent grid.
//
// Coefficients are never stored: a per-row class table (interior interval,
// exterior hull) gives a_ij = b_ij = 1 or 1/eps with two integer compares;
// only the boundary band evaluates the fictitious-domain face lengths from
// the 1-D chord tables.  Dot products end in a deterministic last-workgroup
// reduction (agent-scope release/acquire ticket; partials summed in block
// order), so results are bitwise reproducible run to run.
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

// Sum N-tuples of partials [nblocks][N] in block order (deterministic).
template <int N>
__device__ __forceinline__ void reduce_partials(const double* partial, unsigned nblocks, double (&v)[N], double* sm) {
#pragma unroll
  for (int n = 0; n < N; ++n) v[n] = 0.0;
  for (unsigned m = threadIdx.x; m < nblocks; m += TJ)
#pragma unroll
    for (int n = 0; n < N; ++n) v[n] += partial[size_t(m) * N + n];
  block_reduce<N, false>(v, sm);
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

constexpr int SEG = 60;  // rows per segment: rows seg-1 .. seg+SEG live one per lane

// Per-segment lane-resident data of a strip: row classes (lane t ↔ row
// s0-1+t), strip-edge p columns (lane t ↔ row s0+t) and, for F, r of an
// in-strip halo column ny+1 (lane t ↔ row s0+t).
struct SegData {
  int4 rcv;
  double hL, hR, rup;
};

// ---------------------------------------------------------------------------
// F: p_k = D⁻¹ r_k + β p_{k-1} on owned nodes and the halo ring, then
//    S_den = Σ (A p_k)·p_k and S_pp = Σ p_k·p_k over owned nodes.
// ---------------------------------------------------------------------------
template <bool EXACT>
__global__ __launch_bounds__(TJ) void kF(KParams k, int par) {
  DevState* st = k.st;
  if (st->done) return;
  __shared__ double sm[8];
  __shared__ int sflag;

  const double rz_new = (st->red_G[0] * k.h1) * k.h2;
  const double beta = rz_new / st->rz_cur;
  const double* __restrict__ pold = k.p[par ^ 1];
  double* __restrict__ pnew = k.p[par];
  const int64_t pitch = k.pitch;
  const int nx = int(k.nx), ny = int(k.ny);
  const int lane = threadIdx.x & 63;
  const int nw = gridDim.x * kWPB;
  double sden = 0.0, spp = 0.0;

  // Wave id made provably uniform so item geometry lives in SGPRs.
  const int wid = __builtin_amdgcn_readfirstlane(int(threadIdx.x >> 6));
  for (int item = blockIdx.x * kWPB + wid; item < k.nitems; item += nw) {
    // item → (strip, row range); strip-major so a wave's consecutive items
    // continue down the same strip.
    // order 0 (default): chunk-major — concurrently running waves cover a
    // compact window of rows (TLB/L2/MALL locality); order 1: strip-major.
    const int nchunks = (nx + k.ti - 1) / k.ti;
    const int s = k.order ? item / nchunks : item % k.nstrips;
    const int ch = k.order ? item % nchunks : item / k.nstrips;
    const int j0 = 1 + s * SW;
    const int ib = 1 + ch * k.ti, ie = min(ib + k.ti - 1, nx);
    const int c0 = j0 + 2 * lane, c1 = c0 + 1;
    const int jhi = min(j0 + SW - 1, ny + 1);
    const bool own0 = c0 <= ny, own1 = c1 <= ny;
    const bool live0 = own0 || (c0 == ny + 1 && k.has[UP]);
    const bool live1 = own1 || (c1 == ny + 1 && k.has[UP]);
    const int ca = (c0 <= ny + 1) ? c0 : 1;  // clamped column for loads

    auto seg_load = [&](int s0, int s1) {
      SegData d;
      const int t = lane;
      d.rcv = (t <= s1 - s0 + 2) ? *reinterpret_cast<const int4*>(k.rowcls + (s0 + t) * 4) : make_int4(1, 0, 0, -1);
      d.hL = d.hR = d.rup = 0.0;
      if (t <= s1 - s0) {
        const int q = s0 + t;
        const int jl = j0 - 1, jr = j0 + SW;
        if (valid_node(k, q, jl)) {
          d.hL = p_point<EXACT>(k, q, jl, beta, pold);
          if (jl == 0) pnew[q * pitch] = d.hL;  // rank-halo column: ours to write
        }
        if (jr <= ny + 1 && valid_node(k, q, jr)) {
          d.hR = p_point<EXACT>(k, q, jr, beta, pold);
          if (jr == ny + 1) pnew[q * pitch + jr] = d.hR;
        }
      }
      if (t <= s1 - s0 + 1 && s0 + t <= nx && k.has[UP]) d.rup = k.recv_up[s0 + t - 1];
      return d;
    };

    // p(q) for both elements from r(q), p_{k-1}(q); rh = r of the halo column.
    auto prow = [&](int q, const RowCls& rc, bool fast, double2 rr, double2 po, double rh, double& v0, double& v1) {
      const bool rin = q >= 1 && q <= nx;
      const bool rv = rin || (q == 0 && k.has[LEFT]) || (q == nx + 1 && k.has[RIGHT]);
      const double r0 = (c0 == ny + 1) ? rh : rr.x;
      const double r1 = (c1 == ny + 1) ? rh : rr.y;
      CS s0, s1;
      if (fast) {
        s0 = cset_fast<EXACT>(k, rc, c0);
        s1 = cset_fast<EXACT>(k, rc, c1);
      } else {
        const int* rcp = k.rowcls + (q + 1) * 4;
        s0 = cset<EXACT>(k, rcp, q, c0, tv_at(k, ca));
        s1 = cset<EXACT>(k, rcp, q, c1, tv_at(k, ca + 1));
      }
      const bool e0 = rv && (rin ? live0 : own0), e1 = rv && (rin ? live1 : own1);
      v0 = e0 ? zval<EXACT>(s0, r0) + beta * po.x : 0.0;
      v1 = e1 ? zval<EXACT>(s1, r1) + beta * po.y : 0.0;
    };
    auto store_row = [&](int q, double v0, double v1) {
      const bool rin = q >= 1 && q <= nx;
      const bool w0 = rin ? live0 : own0, w1 = rin ? live1 : own1;
      double* dst = pnew + q * pitch + c0;
      if (w0 && w1) *reinterpret_cast<double2*>(dst) = make_double2(v0, v1);
      else if (w0) dst[0] = v0;
    };

    const double* rptr = k.r + (ib - 1) * pitch + ca;  // row ib-1
    const double* pptr = pold + (ib - 1) * pitch + ca;
    const double2 rA = ld2(rptr), pA = ld2(pptr);
    const double2 rB = ld2(rptr + pitch), pB = ld2(pptr + pitch);
    double2 rN = ld2(rptr + 2 * pitch), pN = ld2(pptr + 2 * pitch);  // row ib+1
    rptr += 3 * pitch;                                                // → row ib+2
    pptr += 3 * pitch;
    SegData sd = seg_load(ib, min(ib + SEG - 1, ie));

    double pm0, pm1, p00, p01;
    RowCls ci = rcl_read(sd.rcv, 1);  // row ib
    bool gi = has_gen(ci, j0, jhi);
    {
      const RowCls cm = rcl_read(sd.rcv, 0);  // row ib-1
      const double rupA = (k.has[UP] && ib >= 2) ? k.recv_up[ib - 2] : 0.0;
      prow(ib - 1, cm, !has_gen(cm, j0, jhi), rA, pA, rupA, pm0, pm1);
      prow(ib, ci, !gi, rB, pB, readlane(sd.rup, 0), p00, p01);
    }
    if (ib == 1 && k.has[LEFT]) store_row(0, pm0, pm1);
    store_row(ib, p00, p01);

    for (int s0 = ib; s0 <= ie; s0 += SEG) {
      const int s1 = min(s0 + SEG - 1, ie);
      if (s0 != ib) sd = seg_load(s0, s1);
      // ---- march: only the prefetch stream touches vector memory ----
      for (int i = s0; i <= s1; ++i) {
        const int q = i + 1;
        const double2 rNN = ld2(rptr), pNN = ld2(pptr);  // row i+2 (≤ nx+3: padded)
        rptr += pitch;
        pptr += pitch;

        const int rl = i - s0;
        const RowCls cq = rcl_read(sd.rcv, rl + 2);
        const bool gq = has_gen(cq, j0, jhi);
        const double rh = readlane(sd.rup, rl + 1);
        double pn0, pn1;
        prow(q, cq, !gq, rN, pN, rh, pn0, pn1);
        if (q <= ie || (q == nx + 1 && k.has[RIGHT])) store_row(q, pn0, pn1);

        // j±1 neighbours of row i: DPP wave shifts, strip edges from hL/hR.
        const double eL = readlane(sd.hL, rl), eR = readlane(sd.hR, rl);
        double pl0 = dpp_shr1(p01);
        double pr1 = dpp_shl1(p00);
        if (lane == 0) pl0 = eL;
        if (lane == 63) pr1 = eR;
        CS x0, x1;
        if (!gi) {
          x0 = cset_fast<EXACT>(k, ci, c0);
          x1 = cset_fast<EXACT>(k, ci, c1);
        } else {
          const int* rcp = k.rowcls + (i + 1) * 4;
          x0 = cset<EXACT>(k, rcp, i, c0, tv_at(k, ca));
          x1 = cset<EXACT>(k, rcp, i, c1, tv_at(k, ca + 1));
        }
        const double Ap0 = stencil<EXACT>(k, x0, pm0, p00, pn0, pl0, p01);
        const double Ap1 = stencil<EXACT>(k, x1, pm1, p01, pn1, p00, pr1);
        if (own0) {
          sden += Ap0 * p00;
          spp += p00 * p00;
        }
        if (own1) {
          sden += Ap1 * p01;
          spp += p01 * p01;
        }
        pm0 = p00;
        pm1 = p01;
        p00 = pn0;
        p01 = pn1;
        rN = rNN;
        pN = pNN;
        ci = cq;
        gi = gq;
      }
    }
  }

  double v[2] = {sden, spp};
  block_reduce<2, false>(v, sm);
  if (threadIdx.x == 0) {
    k.partial[2 * size_t(blockIdx.x)] = v[0];
    k.partial[2 * size_t(blockIdx.x) + 1] = v[1];
  }
  if (arrive_last(&st->ticket[0], gridDim.x, &sflag)) {
    double t[2];
    reduce_partials<2>(k.partial, gridDim.x, t, sm);
    if (threadIdx.x == 0) {
      st->red_F[0] = t[0];
      st->red_F[1] = t[1];
      st->rz_cur = rz_new;
      st->beta = beta;
      __hip_atomic_store(&st->ticket[0], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
}

// ---------------------------------------------------------------------------
// G: α = rz/den, stop test, w += α p, r -= α A p, S_zr = Σ (D⁻¹r)·r.
// ---------------------------------------------------------------------------
template <bool EXACT>
__global__ __launch_bounds__(TJ) void kG(KParams k, int par) {
  DevState* st = k.st;
  if (st->done) return;
  __shared__ double sm[8];
  __shared__ int sflag;

  const double den = (st->red_F[0] * k.h1) * k.h2;
  const long long kiter = st->iter + 1;
  if (fabs(den) < 1e-15) {  // breakdown: stop before touching w (reference :413)
    if (blockIdx.x == 0 && threadIdx.x == 0) {
      st->status = 2;
      st->iter = kiter;
      st->done = 1;
    }
    return;
  }
  const double alpha = st->rz_cur / den;
  const double d2 = alpha * alpha * st->red_F[1];
  const double diff = k.weighted ? sqrt((d2 * k.h1) * k.h2) : sqrt(d2);

  const double* __restrict__ p = k.p[par];
  double* __restrict__ r = k.r;
  double* __restrict__ w = k.w;
  const int64_t pitch = k.pitch;
  const int nx = int(k.nx), ny = int(k.ny);
  const int lane = threadIdx.x & 63;
  const int nw = gridDim.x * kWPB;
  double szr = 0.0;

  const int wid = __builtin_amdgcn_readfirstlane(int(threadIdx.x >> 6));
  for (int item = blockIdx.x * kWPB + wid; item < k.nitems; item += nw) {
    // order 0 (default): chunk-major — concurrently running waves cover a
    // compact window of rows (TLB/L2/MALL locality); order 1: strip-major.
    const int nchunks = (nx + k.ti - 1) / k.ti;
    const int s = k.order ? item / nchunks : item % k.nstrips;
    const int ch = k.order ? item % nchunks : item / k.nstrips;
    const int j0 = 1 + s * SW;
    const int ib = 1 + ch * k.ti, ie = min(ib + k.ti - 1, nx);
    const int c0 = j0 + 2 * lane, c1 = c0 + 1;
    const int jhi = min(j0 + SW - 1, ny + 1);
    const bool own0 = c0 <= ny, own1 = c1 <= ny;
    const int ca = (c0 <= ny + 1) ? c0 : 1;

    auto seg_load = [&](int s0, int s1) {
      SegData d;
      const int t = lane;
      d.rcv = (t <= s1 - s0) ? *reinterpret_cast<const int4*>(k.rowcls + (s0 + 1 + t) * 4) : make_int4(1, 0, 0, -1);
      d.hL = d.hR = d.rup = 0.0;
      if (t <= s1 - s0) {
        const int q = s0 + t;
        d.hL = p[q * pitch + j0 - 1];
        if (j0 + SW <= ny + 1) d.hR = p[q * pitch + j0 + SW];
      }
      return d;
    };

    const double* pptr = p + (ib - 1) * pitch + ca;
    const double* rptr = r + ib * pitch + ca;
    const double* wptr = w + ib * pitch + ca;
    const double2 pA = ld2(pptr);
    double2 pB = ld2(pptr + pitch);
    double2 pN = ld2(pptr + 2 * pitch);
    double2 rC = ld2(rptr), wC = ld2(wptr);
    pptr += 3 * pitch;  // → row ib+2
    rptr += pitch;      // → row ib+1
    wptr += pitch;
    double pm0 = pA.x, pm1 = pA.y;
    SegData sd;

    for (int s0 = ib; s0 <= ie; s0 += SEG) {
      const int s1 = min(s0 + SEG - 1, ie);
      sd = seg_load(s0, s1);
      for (int i = s0; i <= s1; ++i) {
        const double2 pNN = ld2(pptr);  // row i+2 (padded)
        const double2 rNx = ld2(rptr);  // row i+1
        const double2 wNx = ld2(wptr);
        pptr += pitch;
        rptr += pitch;
        wptr += pitch;

        const int rl = i - s0;
        const RowCls ci = rcl_read(sd.rcv, rl);
        const double eL = readlane(sd.hL, rl), eR = readlane(sd.hR, rl);
        double pl0 = dpp_shr1(pB.y);
        double pr1 = dpp_shl1(pB.x);
        if (lane == 0) pl0 = eL;
        if (lane == 63) pr1 = eR;
        CS x0, x1;
        if (!has_gen(ci, j0, jhi)) {
          x0 = cset_fast<EXACT>(k, ci, c0);
          x1 = cset_fast<EXACT>(k, ci, c1);
        } else {
          const int* rcp = k.rowcls + (i + 1) * 4;
          x0 = cset<EXACT>(k, rcp, i, c0, tv_at(k, ca));
          x1 = cset<EXACT>(k, rcp, i, c1, tv_at(k, ca + 1));
        }
        const double Ap0 = stencil<EXACT>(k, x0, pm0, pB.x, pN.x, pl0, pB.y);
        const double Ap1 = stencil<EXACT>(k, x1, pm1, pB.y, pN.y, pB.x, pr1);
        const double wn0 = wC.x + alpha * pB.x, wn1 = wC.y + alpha * pB.y;
        const double rn0 = rC.x - alpha * Ap0, rn1 = rC.y - alpha * Ap1;
        if (own0) szr += zval<EXACT>(x0, rn0) * rn0;
        if (own1) szr += zval<EXACT>(x1, rn1) * rn1;
        double* rd = r + i * pitch + c0;
        double* wd = w + i * pitch + c0;
        if (own1) {
          *reinterpret_cast<double2*>(rd) = make_double2(rn0, rn1);
          *reinterpret_cast<double2*>(wd) = make_double2(wn0, wn1);
        } else if (own0) {
          rd[0] = rn0;
          wd[0] = wn0;
        }
        if (c0 == 1 && k.has[DOWN]) k.send_dn[i - 1] = rn0;
        if (k.has[UP]) {
          if (c0 == ny) k.send_up[i - 1] = rn0;
          if (c1 == ny) k.send_up[i - 1] = rn1;
        }
        pm0 = pB.x;
        pm1 = pB.y;
        pB = pN;
        pN = pNN;
        rC = rNx;
        wC = wNx;
      }
    }
  }

  double v[1] = {szr};
  block_reduce<1, false>(v, sm);
  if (threadIdx.x == 0) k.partial[blockIdx.x] = v[0];
  if (arrive_last(&st->ticket[1], gridDim.x, &sflag)) {
    double t[1];
    reduce_partials<1>(k.partial, gridDim.x, t, sm);
    if (threadIdx.x == 0) {
      st->red_G[0] = t[0];
      st->alpha = alpha;
      st->last_diff = diff;
      st->iter = kiter;
      if (k.check_tol && diff < k.tol) {
        st->status = 1;
        st->done = 1;
      } else if (kiter >= k.max_iter) {
        st->status = 3;
        st->done = 1;
      }
      __hip_atomic_store(&st->ticket[1], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
}

// ---------------------------------------------------------------------------
// Init: r⁰ = B - A w⁰ (w⁰ = 0 or a global-index hash), S_zr⁰ = Σ (D⁻¹r⁰)·r⁰.
// ---------------------------------------------------------------------------
template <bool EXACT>
__global__ __launch_bounds__(TJ) void kInit(KParams k, int init_random, unsigned long long seed, double amp) {
  __shared__ double sm[8];
  __shared__ int sflag;
  DevState* st = k.st;
  const int64_t n = k.nx * k.ny;
  double szr = 0.0;
  for (int64_t idx = int64_t(blockIdx.x) * TJ + threadIdx.x; idx < n; idx += int64_t(gridDim.x) * TJ) {
    const int64_t li = idx / k.ny + 1, lj = idx % k.ny + 1;
    const int64_t gi = k.gi0 + li, gj = k.gj0 + lj;
    const double x = k.A1 + gi * k.h1, y = k.A2 + gj * k.h2;
    const CS c = cset_mem<EXACT>(k, li, lj);
    double rr = in_ellipse(x, y, k.cx, k.cy) ? k.F : 0.0;
    const int64_t at = li * k.pitch + lj;
    if (init_random) {
      const double w0 = random_w0(gi, gj, k.M, k.N, seed, amp);
      const double Aw = stencil<EXACT>(k, c, random_w0(gi - 1, gj, k.M, k.N, seed, amp), w0,
                                       random_w0(gi + 1, gj, k.M, k.N, seed, amp),
                                       random_w0(gi, gj - 1, k.M, k.N, seed, amp),
                                       random_w0(gi, gj + 1, k.M, k.N, seed, amp));
      rr = rr - Aw;
      k.w[at] = w0;
    }
    k.r[at] = rr;
    if (lj == 1 && k.has[DOWN]) k.send_dn[li - 1] = rr;
    if (lj == k.ny && k.has[UP]) k.send_up[li - 1] = rr;
    szr += zval<EXACT>(c, rr) * rr;
  }
  double v[1] = {szr};
  block_reduce<1, false>(v, sm);
  if (threadIdx.x == 0) k.partial[blockIdx.x] = v[0];
  if (arrive_last(&st->ticket[2], gridDim.x, &sflag)) {
    double t[1];
    reduce_partials<1>(k.partial, gridDim.x, t, sm);
    if (threadIdx.x == 0) {
      st->red_G[0] = t[0];
      st->rz_cur = 1.0;
      st->iter = 0;
      st->done = 0;
      st->status = 0;
      __hip_atomic_store(&st->ticket[2], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
}

// Error against the analytic solution u = F(1 - cx x² - cy y²)/(2cx + 2cy).
__global__ __launch_bounds__(TJ) void kError(KParams k) {
  __shared__ double sm[8];
  __shared__ int sflag;
  DevState* st = k.st;
  const int64_t n = k.nx * k.ny;
  double e2 = 0.0, emax = 0.0, omax = 0.0;
  for (int64_t idx = int64_t(blockIdx.x) * TJ + threadIdx.x; idx < n; idx += int64_t(gridDim.x) * TJ) {
    const int64_t li = idx / k.ny + 1, lj = idx % k.ny + 1;
    const double x = k.A1 + (k.gi0 + li) * k.h1, y = k.A2 + (k.gj0 + lj) * k.h2;
    const double wv = k.w[li * k.pitch + lj];
    if (in_ellipse(x, y, k.cx, k.cy)) {
      const double e = wv - k.u_scale * (1.0 - k.cx * x * x - k.cy * y * y);
      e2 += e * e;
      emax = fmax(emax, fabs(e));
    } else {
      omax = fmax(omax, fabs(wv));
    }
  }
  double s[1] = {e2};
  double m[2] = {emax, omax};
  block_reduce<1, false>(s, sm);
  __syncthreads();
  block_reduce<2, true>(m, sm);
  if (threadIdx.x == 0) {
    k.partial[3 * size_t(blockIdx.x)] = s[0];
    k.partial[3 * size_t(blockIdx.x) + 1] = m[0];
    k.partial[3 * size_t(blockIdx.x) + 2] = m[1];
  }
  if (arrive_last(&st->ticket[3], gridDim.x, &sflag)) {
    double acc = 0.0, m0 = 0.0, m1 = 0.0;
    for (unsigned b = threadIdx.x; b < gridDim.x; b += TJ) {
      acc += k.partial[3 * size_t(b)];
      m0 = fmax(m0, k.partial[3 * size_t(b) + 1]);
      m1 = fmax(m1, k.partial[3 * size_t(b) + 2]);
    }
    double s2[1] = {acc};
    double mm[2] = {m0, m1};
    block_reduce<1, false>(s2, sm);
    __syncthreads();
    block_reduce<2, true>(mm, sm);
    if (threadIdx.x == 0) {
      st->err[0] = s2[0];
      st->err[1] = mm[0];
      st->err[2] = mm[1];
      __hip_atomic_store(&st->ticket[3], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
}

__global__ void kGroupReduce(double* const* bufs, int nranks, int n, int is_max) {
  const int i = threadIdx.x;
  if (i >= n) return;
  double acc = bufs[0][i];
  for (int r = 1; r < nranks; ++r) acc = is_max ? fmax(acc, bufs[r][i]) : acc + bufs[r][i];
  for (int r = 0; r < nranks; ++r) bufs[r][i] = acc;
}

// Test op: Ap = A p on owned nodes (p halo must be valid).
template <bool EXACT>
__global__ void kApplyA(KParams k, const double* p, double* Ap) {
  const int64_t n = k.nx * k.ny;
  for (int64_t idx = int64_t(blockIdx.x) * blockDim.x + threadIdx.x; idx < n;
       idx += int64_t(gridDim.x) * blockDim.x) {
    const int64_t li = idx / k.ny + 1, lj = idx % k.ny + 1;
    const int64_t c = li * k.pitch + lj;
    const CS cs = cset_mem<EXACT>(k, li, lj);
    Ap[c] = stencil<EXACT>(k, cs, p[c - k.pitch], p[c], p[c + k.pitch], p[c - 1], p[c + 1]);
  }
}

// Test op: a_ij, b_ij, D_ij through the class table (checks the classification).
__global__ void kCoef(KParams k, double* a, double* b, double* D) {
  const int64_t n = (k.nx + 2) * (k.ny + 2);
  for (int64_t idx = int64_t(blockIdx.x) * blockDim.x + threadIdx.x; idx < n;
       idx += int64_t(gridDim.x) * blockDim.x) {
    const int64_t li = idx / (k.ny + 2), lj = idx % (k.ny + 2);
    const CS cs = cset_mem<true>(k, li, lj);
    const int64_t c = li * k.pitch + lj;
    a[c] = cs.a0;
    b[c] = cs.b0;
    D[c] = cs.d;
  }
}

}  // namespace

int grid_blocks(const KParams& k) { return k.nblocks; }

static unsigned flat_blocks(const KParams& k) {
  const int64_t n = (k.nx + 2) * (k.ny + 2);
  int64_t b = (n + TJ - 1) / TJ;
  if (b > 4096) b = 4096;
  if (b < 1) b = 1;
  return unsigned(b);
}

void launch_init(const KParams& k, int init_random, unsigned long long seed, double amp, int variant,
                 hipStream_t s) {
  if (variant == 1) hipLaunchKernelGGL(kInit<true>, dim3(flat_blocks(k)), dim3(TJ), 0, s, k, init_random, seed, amp);
  else hipLaunchKernelGGL(kInit<false>, dim3(flat_blocks(k)), dim3(TJ), 0, s, k, init_random, seed, amp);
}

void launch_F(const KParams& k, int par, int variant, hipStream_t s) {
  if (variant == 1) hipLaunchKernelGGL(kF<true>, dim3(k.nblocks), dim3(TJ), 0, s, k, par);
  else hipLaunchKernelGGL(kF<false>, dim3(k.nblocks), dim3(TJ), 0, s, k, par);
}

void launch_G(const KParams& k, int par, int variant, hipStream_t s) {
  if (variant == 1) hipLaunchKernelGGL(kG<true>, dim3(k.nblocks), dim3(TJ), 0, s, k, par);
  else hipLaunchKernelGGL(kG<false>, dim3(k.nblocks), dim3(TJ), 0, s, k, par);
}

void launch_error(const KParams& k, hipStream_t s) {
  hipLaunchKernelGGL(kError, dim3(flat_blocks(k)), dim3(TJ), 0, s, k);
}

void launch_group_reduce(double* const* bufs, int nranks, int n, int is_max, hipStream_t s) {
  hipLaunchKernelGGL(kGroupReduce, dim3(1), dim3(64), 0, s, bufs, nranks, n, is_max);
}

void launch_apply_A(const KParams& k, const double* p, double* Ap, hipStream_t s) {
  hipLaunchKernelGGL(kApplyA<false>, dim3(flat_blocks(k)), dim3(TJ), 0, s, k, p, Ap);
}

void launch_coef(const KParams& k, double* a, double* b, double* D, hipStream_t s) {
  hipLaunchKernelGGL(kCoef, dim3(flat_blocks(k)), dim3(TJ), 0, s, k, a, b, D);
}

}  // namespace dev
}  // namespace pe
