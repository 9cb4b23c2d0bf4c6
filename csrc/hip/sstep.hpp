// Shared device pieces of the multi-iteration sweeps (fused2.hip: two
// iterations per pass, fused3.hip: three): the per-lane helpers of the row
// march, the boundary-band coefficient ring in LDS and the 5-point operator
// on a lane's two columns.  Both kernels march one wave64 strip down the rows
// of an item with a pipeline of stages; each stage applies the operator to a
// row of a vector the previous stage produced, j-neighbours through DPP lane
// shifts, i-neighbours from rotating register rings.
#pragma once

#include "kcommon.hpp"

// (the including sweeps are built with fast contraction; so are these helpers)
#pragma clang fp contract(fast)

namespace pe {
namespace dev {
namespace {

__device__ __forceinline__ double2 dd(double a, double b) { return make_double2(a, b); }
__device__ __forceinline__ int2 cload_i2(const int2* p) {
  const long long v = cload(reinterpret_cast<const long long*>(p));
  return make_int2(int(v), int(v >> 32));
}

// A wave-uniform double in scalar registers (the scalars of a sweep are a
// pure function of the state every lane read: pin them to SGPRs so the long
// marches keep their VGPRs for the row rings).
__device__ __forceinline__ double uni(double x) {
  const long long v = __double_as_longlong(x);
  const unsigned lo = unsigned(__builtin_amdgcn_readfirstlane(int(unsigned(v))));
  const unsigned hi = unsigned(__builtin_amdgcn_readfirstlane(int(v >> 32)));
  return __longlong_as_double((long long)((unsigned long long)hi << 32 | lo));
}

// A (uniform) value pinned to a VGPR from here on.
__device__ __forceinline__ double vreg(double x) {
  asm volatile("; vreg %0" : "+v"(x));
  return x;
}

__device__ __forceinline__ void hist_put(const KParams& k, long long kiter, double d) {
  if (k.hist && kiter <= k.hist_n) k.hist[kiter - 1] = d;
}

typedef double v2d __attribute__((ext_vector_type(2)));
__device__ __forceinline__ void st2nt(double* p, double2 v) {
  __builtin_nontemporal_store(v2d{v.x, v.y}, reinterpret_cast<v2d*>(p));
}
__device__ __forceinline__ double2 ldnt(const double* p) {
  const v2d t = __builtin_nontemporal_load(reinterpret_cast<const v2d*>(p));
  return make_double2(t.x, t.y);
}

// Per-wave LDS of a multi-iteration march: the tables a boundary-band row
// evaluates its coefficients from — the strip's row-table entries (per
// column) and the item's column-table entries and row classes (per row, rows
// segbase .. segbase+63) — and a ring of the face coefficients of the last
// RING rows (band items only).  A row is evaluated ONCE, when it enters the
// pipeline (its first stage): its vertical-face a0 and horizontal-face b0 per
// column go to a ring slot; the stages that apply the operator to a band row
// read a0 of the row and of the row below it (= its a1), b0 of the column and
// of the next one (= its b1, written by the neighbouring lane) and form 1/D
// from them (dinv_faces: the bits of the evaluation).  Plain rows keep the
// select path and no ring reads.  In LDS rather than lanes: the marches would
// spill.
template <int RING>
struct WaveTV {
  double sA[128], eA[128], hB[130];
  int4 rc[64];
  double half[65], sB[64], eB[64];
  double a0r[RING][128];
  double b0r[RING][130];  // (column 128: read by lane 63 for its b1, never written)
  static constexpr int kRing = RING;
};

struct RowCtx {
  int2 rcv;      // interior interval of row segbase + lane (lane l ↔ row segbase + l)
  unsigned long long genmask;
  unsigned long long allin;  // bit l: row segbase + l interior over the whole 128-column window
  int segbase;
};

// Stage rows below the item's first row (pipeline fill) are garbage rows
// whose results are never used: the lane index is wrapped, not trusted.
__device__ __forceinline__ void row_in(const RowCtx& rx, int q, int c0, bool& in0, bool& in1, bool& gen) {
  const int l = (q - rx.segbase) & 63;
  const int lo = __builtin_amdgcn_readlane(rx.rcv.x, l), hi = __builtin_amdgcn_readlane(rx.rcv.y, l);
  in0 = c0 >= lo && c0 <= hi;
  in1 = c0 + 1 >= lo && c0 + 1 <= hi;
  gen = (rx.genmask >> l) & 1ull;
}

__device__ __forceinline__ double lap(const KParams& k, double f, double pm, double p0, double pn, double pl,
                                      double pr) {
  return f * (((p0 - pm) - (pn - p0)) * k.ih1sq + ((p0 - pl) - (pr - p0)) * k.ih2sq);
}

// Row classes / column tables of rows base .. base+63 (one per lane) into the
// lane registers (strip window: WIN columns from J) (and, for band items with a boundary row in the window, the
// wave's LDS tables); rows past `last` get an empty interior interval.
// The row-class entry of window row `lane` (rows past `last`: an empty interior).
__device__ __forceinline__ int4 rowcls_entry(const KParams& k, int base, int last) {
  const int lane = threadIdx.x & 63;
  return lane < last + 1 - base ? *reinterpret_cast<const int4*>(k.rowcls + (base + 1 + lane) * 4) : make_int4(1, 0, 0, -1);
}

// (pre: the entry already loaded — fused3.hip loads the first item's at kernel entry)
template <bool BAND, class WT, int WIN = 128>
__device__ __forceinline__ void load_rows(const KParams& k, RowCtx& rx, WT& tvw, int base, int last, int J,
                                          const int4* pre = nullptr) {
  const int lane = threadIdx.x & 63;
  rx.segbase = base;
  const int nr = last + 1 - base;
  const int4 rc4 = pre ? *pre : rowcls_entry(k, base, last);
  rx.rcv = make_int2(rc4.x, rc4.y);
  rx.genmask = 0;
  rx.allin = __ballot(lane < nr && rc4.x <= J && rc4.y >= J + WIN - 1);
  if (BAND) {
    rx.genmask = __ballot(lane < nr && has_gen(RowCls{rc4.x, rc4.y, rc4.z, rc4.w}, J, J + WIN - 1));
    if (rx.genmask != 0) {
      const double* ctr = k.colT + (min(base + lane, last) + 1) * 4;
      tvw.rc[lane] = rc4;
      tvw.half[lane] = ctr[0];
      tvw.sB[lane] = ctr[1];
      tvw.eB[lane] = ctr[2];
      if (lane == 63) tvw.half[64] = ctr[4];
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    }
  }
}

// The strip's row-table entries (per column), once per band item.
template <class WT>
__device__ __forceinline__ void load_strip_tables(const KParams& k, WT& tvw, int c0) {
  const int lane = threadIdx.x & 63, jl = 2 * lane;
  const double* tb = k.rowT + (c0 + 1) * 4;
  const double4 a = *reinterpret_cast<const double4*>(tb);
  const double4 b = *reinterpret_cast<const double4*>(tb + 4);
  tvw.sA[jl] = a.x;
  tvw.eA[jl] = a.y;
  tvw.hB[jl] = a.z;
  tvw.sA[jl + 1] = b.x;
  tvw.eA[jl + 1] = b.y;
  tvw.hB[jl + 1] = b.z;
  if (lane == 63) {
    tvw.hB[128] = tb[10];
    tvw.hB[129] = tb[14];
  }
}

// First stage of a band item: row q's faces into ring slot `sl`; returns 1/D.
template <class WT>
__device__ __forceinline__ double2 enter_band(const KParams& k, const RowCtx& rx, WT& tv, int q, int c0, int jl,
                                              int sl) {
  bool in0, in1, gen;
  row_in(rx, q, c0, in0, in1, gen);
  double2 d, a0, b0;
  if (gen) {
    const int l = (q - rx.segbase) & 63;
    const int4 r4 = tv.rc[l];
    const RowCls rc{r4.x, r4.y, r4.z, r4.w};
    const CT ct{tv.half[l], tv.half[l + 1], tv.sB[l], tv.eB[l]};
    const CS x0 = cset_rc(k, rc, ct, c0, TV{tv.sA[jl], tv.eA[jl], tv.hB[jl], tv.hB[jl + 1]});
    const CS x1 = cset_rc(k, rc, ct, c0 + 1, TV{tv.sA[jl + 1], tv.eA[jl + 1], tv.hB[jl + 1], tv.hB[jl + 2]});
    d = dd(x0.d, x1.d);
    a0 = dd(x0.a0, x1.a0);
    b0 = dd(x0.b0, x1.b0);
  } else {
    const double f0 = in0 ? 1.0 : k.inv_eps, f1 = in1 ? 1.0 : k.inv_eps;
    d = dd(in0 ? k.dinv_in : k.dinv_out, in1 ? k.dinv_in : k.dinv_out);
    a0 = dd(f0, f1);
    b0 = a0;
  }
  *reinterpret_cast<double2*>(&tv.a0r[sl][jl]) = a0;
  *reinterpret_cast<double2*>(&tv.b0r[sl][jl]) = b0;
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  return d;
}

// The 5-point operator at row q (ring slot sl, the row above it in slot sln)
// for the lane's two columns; d = 1/D of the row.
template <bool BAND, class WT>
__device__ __forceinline__ double2 apply_row(const KParams& k, const RowCtx& rx, const WT& tv, int q, int c0, int jl,
                                             int sl, int sln, const double2& um, const double2& u0, const double2& un,
                                             double2& d) {
  const double ul = dpp_shr1(u0.y), ur = dpp_shl1(u0.x);
  bool in0, in1, gen;
  row_in(rx, q, c0, in0, in1, gen);
  if (BAND && gen) {
    const double2 a0 = *reinterpret_cast<const double2*>(&tv.a0r[sl][jl]);
    const double2 a1 = *reinterpret_cast<const double2*>(&tv.a0r[sln][jl]);
    const double2 b0 = *reinterpret_cast<const double2*>(&tv.b0r[sl][jl]);
    const double b2 = tv.b0r[sl][jl + 2];
    const CS x0{a0.x, a1.x, b0.x, b0.y, dinv_faces(k, a0.x, a1.x, b0.x, b0.y)};
    const CS x1{a0.y, a1.y, b0.y, b2, dinv_faces(k, a0.y, a1.y, b0.y, b2)};
    d = dd(x0.d, x1.d);
    return dd(stencil<false>(k, x0, um.x, u0.x, un.x, ul, u0.y), stencil<false>(k, x1, um.y, u0.y, un.y, u0.x, ur));
  }
  d = dd(in0 ? k.dinv_in : k.dinv_out, in1 ? k.dinv_in : k.dinv_out);
  return dd(lap(k, in0 ? 1.0 : k.inv_eps, um.x, u0.x, un.x, ul, u0.y),
            lap(k, in1 ? 1.0 : k.inv_eps, um.y, u0.y, un.y, u0.x, ur));
}

__device__ __forceinline__ double2 dinv_plain(const KParams& k, const RowCtx& rx, int q, int c0) {
  bool in0, in1, gen;
  row_in(rx, q, c0, in0, in1, gen);
  return dd(in0 ? k.dinv_in : k.dinv_out, in1 ? k.dinv_in : k.dinv_out);
}

__device__ __forceinline__ double dot2(const double2& a, const double2& b) { return a.x * b.x + a.y * b.y; }

// ---- one column per lane (fused3.hip: 64-column strips) ----------------
template <int RING>
struct WaveTV1 {
  double sA[64], eA[64], hB[66];
  int4 rc[64];
  double half[65], sB[64], eB[64];
  double a0r[RING][64];
  double b0r[RING][66];  // (column 64: read by lane 63 for its b1, never written)
  double d0r[RING][64];  // 1/D of the ring's rows, evaluated once at entry
};

// The strip's row-table entries (per column), once per band item.
template <class WT>
__device__ __forceinline__ void load_strip_tables1(const KParams& k, WT& tvw, int c0) {
  const int lane = threadIdx.x & 63;
  const double* tb = k.rowT + (c0 + 1) * 4;
  tvw.sA[lane] = tb[0];
  tvw.eA[lane] = tb[1];
  tvw.hB[lane] = tb[2];
  if (lane == 63) tvw.hB[64] = tb[6];
}

__device__ __forceinline__ void row_in1(const RowCtx& rx, int q, int c0, bool& in0, bool& gen) {
  const int l = (q - rx.segbase) & 63;
  const int lo = __builtin_amdgcn_readlane(rx.rcv.x, l), hi = __builtin_amdgcn_readlane(rx.rcv.y, l);
  in0 = c0 >= lo && c0 <= hi;
  gen = (rx.genmask >> l) & 1ull;
}

// First stage of a band item: row q's faces into ring slot `sl`; returns 1/D.
template <class WT>
__device__ __forceinline__ double enter_band1(const KParams& k, const RowCtx& rx, WT& tv, int q, int c0, int sl) {
  const int lane = threadIdx.x & 63;
  bool in0, gen;
  row_in1(rx, q, c0, in0, gen);
  double d, a0, b0;
  if (gen) {
    const int l = (q - rx.segbase) & 63;
    const int4 r4 = tv.rc[l];
    const RowCls rc{r4.x, r4.y, r4.z, r4.w};
    const CT ct{tv.half[l], tv.half[l + 1], tv.sB[l], tv.eB[l]};
    const CS x0 = cset_rc(k, rc, ct, c0, TV{tv.sA[lane], tv.eA[lane], tv.hB[lane], tv.hB[lane + 1]});
    d = x0.d;
    a0 = x0.a0;
    b0 = x0.b0;
  } else {
    d = in0 ? k.dinv_in : k.dinv_out;
    a0 = b0 = in0 ? 1.0 : k.inv_eps;
  }
  tv.a0r[sl][lane] = a0;
  tv.b0r[sl][lane] = b0;
  tv.d0r[sl][lane] = d;
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  return d;
}

// The 5-point operator at row q (ring slot sl, the row above it in slot sln)
// for the lane's column; d = 1/D of the node — read from the ring: the row's
// entry evaluated it once (cset_rc), where every stage used to form it again
// from the four faces (an fp64 reciprocal per operator application, eight
// per band row step).
template <bool BAND, class WT>
__device__ __forceinline__ double apply_row1(const KParams& k, const RowCtx& rx, const WT& tv, int q, int c0, int sl,
                                             int sln, double um, double u0, double un, double& d) {
  const int lane = threadIdx.x & 63;
  const double ul = dpp_shr1(u0), ur = dpp_shl1(u0);
  bool in0, gen;
  row_in1(rx, q, c0, in0, gen);
  if (BAND && gen) {
    const double a0 = tv.a0r[sl][lane], a1 = tv.a0r[sln][lane];
    const double b0 = tv.b0r[sl][lane], b1 = tv.b0r[sl][lane + 1];
    const CS x0{a0, a1, b0, b1, k.dring ? tv.d0r[sl][lane] : dinv_faces(k, a0, a1, b0, b1)};
    d = x0.d;
    return stencil<false>(k, x0, um, u0, un, ul, ur);
  }
  d = in0 ? k.dinv_in : k.dinv_out;
  return lap(k, in0 ? 1.0 : k.inv_eps, um, u0, un, ul, ur);
}

// Row scalars of a uniform row (fused3.hip uniform items):
// 1/h1², 1/h2² times the row's face coefficient, and 1/D (0 outside the
// global interior rows).
struct URow {
  double ih1, ih2, d;
};

// The 5-point operator of a uniform row on the lane's column.
__device__ __forceinline__ double lapu(const URow& r, double um, double u0, double un) {
  const double ul = dpp_shr1(u0), ur = dpp_shl1(u0);
  return ((u0 - um) - (un - u0)) * r.ih1 + ((u0 - ul) - (ur - u0)) * r.ih2;
}

__device__ __forceinline__ double dinv_plain1(const KParams& k, const RowCtx& rx, int q, int c0) {
  bool in0, gen;
  row_in1(rx, q, c0, in0, gen);
  return in0 ? k.dinv_in : k.dinv_out;
}

}  // namespace
}  // namespace dev
}  // namespace pe
