// Three-step single sweep: THREE Jacobi-PCG iterations per pass over memory.
//
// fused2.hip advances two iterations per pass from sums the previous pass
// formed around its outputs; this kernel takes the s-step recurrence one
// step further (s = 3).  With M = D⁻¹A (self-adjoint in the D inner
// product), every scalar of iterations K+1..K+3 is a quadratic form in the
// D-moments of z = D⁻¹r_K and p = p_K,
//
//   μ_n(x, y) = (x, D Mⁿ y),   n = 0..5,
//
// since r_{K+i-1} = D z_{K+i-1} and p_{K+i} are polynomials of degree ≤ 2 in
// M applied to z and p (tools/sstep_proto.py; the prototype and the device
// reproduce every golden iteration count up to 8192²:
// profiles/r3_sstep3_numerics.txt).  Each moment is ONE dot product of
// vectors the sweep forms anyway:
//
//   q = Az, u = D⁻¹q, v = D⁻¹s (s = Ap), Au, Av, ũ = D⁻¹Au, ṽ = D⁻¹Av, Aũ, Aṽ
//   zz: (r,z) (z,q) (q,u) (u,Au) (Au,ũ) (ũ,Aũ)      — sums 0..5
//   zp:       (z,s) (q,v) (u,Av) (Au,ṽ) (ũ,Aṽ)      — sums 6..10
//   pp:       (p,s) (s,v) (v,Av) (Av,ṽ) (ṽ,Aṽ)      — sums 11..15
//
// (μ_0 of zp / pp never enters: z_{K+i} has p-components of degree ≥ 1.)
// The stop test of iteration K+i, |α_i|‖p_i‖, uses ‖p_i‖² summed by the
// sweep that forms p_i (sums 16..18) — "late": the NEXT launch decides it
// (the sums are global only after the sweep's reduction), and when the sweep
// converged on its first or second iteration, w already holds the later
// α_j p_j: that launch subtracts them again (the same march over the same
// inputs with the saved scalars, w -= α_j p_j only) instead of sweeping on.
// Breakdown (|den| < 1e-15) and the iteration cap are known before the
// sweep: it applies only the iterations before them (an identity step is
// zc = 0, β = 1, α = 0).
// So the iteration count and every terminal case keep the reference's
// semantics (stage2-mpi/poisson_mpi_decomp.cpp:400-457); the moments are
// summed in a different order, which is the only numerical difference.
//
// Traffic: r_K, p_K, w in, r_{K+3}, p_{K+3}, w out: 48 B per node per THREE
// iterations (16 B / iteration, against 24 two-step and 40 single sweep) and
// one 19-sum reduction per three iterations.
//
// Machine mapping (gfx950): fused2.hip's march with a 6-deep pipeline, ONE
// column per lane: each wave64 strip loads 64 columns and outputs 48 (lanes
// 8..55; the dependence radius is 6, two more halo lanes per side make the
// strip's loads whole 128-B lines and its stores whole 64-B segments — 52
// outputs straddled segments: 5 lines touched per 4 lines loaded and partial
// writes from two strips).  Two columns per lane (116 of 128)
// needed ~380 VGPRs — one wave per SIMD, issue-bound at 53 % VALU and 3.3 TB/s
// (8192²: 0.94 ms per sweep); one column halves the rings, so two waves share
// a SIMD and hide each other's latencies.  Rows march with seven stages in
// flight
//   A  row t    p₁ = zc₁D⁻¹r + β₁p                          (loads of row t)
//   B  row t−1  s₁ = Ap₁, r₁, z₁, p₂                         ‖p₁‖²
//   C  row t−2  s₂ = Ap₂, r₂, z₂, p₃, w += Σ α_i p_i stored  ‖p₂‖²
//   D  row t−3  s = Ap₃, r₃, z = D⁻¹r₃ → r₃, p₃ stored       (r,z) (z,s) (p,s) ‖p₃‖²
//   E  row t−4  q = Az, u, v                                 (z,q) (q,u) (q,v) (s,v)
//   F  row t−5  Au, Av, ũ, ṽ                                 (u,Au) (u,Av) (v,Av) (Au,ũ) (Au,ṽ) (Av,ṽ)
//   G  row t−6  Aũ, Aṽ                                        (ũ,Aũ) (ũ,Aṽ) (ṽ,Aṽ)
// with register rings of period 2 / 3 (unroll 6) and, for band items, a
// 7-row LDS ring of face coefficients (runtime slot: row − t0 mod 7).
//
// Layout: fused.hip's (x[b] interleaves the r and p planes by row) with a
// 6-deep halo: local rows −5..nx+6 and columns −5..ny+6 hold data; buffer
// element 0 of a row is column −7 (KParams::xorg; rows and planes are whole
// 128-B lines, so strip s's first column 48s−7 starts a line).
#include <cstdlib>

#include "peer_sum.hpp"
#include "sstep.hpp"

#pragma clang fp contract(fast)

namespace pe {
namespace dev {

namespace {

constexpr int H3 = 6;  // dependence radius of a sweep (rows and columns)
constexpr int FSW3 = kFSW3;
constexpr int HL3 = kHL3, HR3 = 64 - kFSW3 - kHL3;  // a strip's left / right halo lanes
static_assert(HL3 >= H3 && HR3 >= H3, "three-step strip: 64 loaded columns (one per lane), >= H3 halo lanes per side");
#ifndef PE_S3_XD
#define PE_S3_XD 3  // rows of r / p loads in flight: a divisor of the 6-step unroll (the ring slot is JJ mod XD)
#endif
#ifndef PE_S3_WD
#define PE_S3_WD 3
#endif
#ifndef PE_S3_NTX
#define PE_S3_NTX 0  // 1: non-temporal loads of r and p (experiment)
#endif
constexpr int kS3XD = PE_S3_XD, kS3WD = PE_S3_WD;
static_assert(6 % kS3XD == 0 && 6 % kS3WD == 0, "register ring periods must divide the 6-step group");
constexpr int NS = kNS3;
constexpr int kRing3 = 7;  // band face ring: rows t-6 .. t
using WaveTV3 = WaveTV1<kRing3>;

// Scalars of a sweep (iterations K+1 .. K+m).  Iteration i applies
//   p_i = zc_i·z_{i-1} + β_i p_{i-1},  r_i = r_{i-1} − α_i A p_i
// and w += Σ cw_i p_i (cw = α; fix-up: −α_j of the iterations past the stop).
struct Coef3 {
  double zc[3], a[3], b[3], cw[3];
};

struct Scal3 {
  bool first;
  long long K;
  int m;    // iterations this sweep applies (0..3)
  int brk;  // 1..3: that iteration breaks down before its update (it follows the m applied ones); 0 none
  bool bad; // the breakdown is a non-finite scalar
  Coef3 c;
  double g[3];  // (r, z) before each applied iteration, h-weighted
};

// Quadratic form Σ_{a,b} x_a x_b μ_{a+b+sh} of the coefficient vector
// x = Σ_a xz_a M^a z + xp_a M^a p (sh = 0: D-form, sh = 1: A-form).
__device__ __forceinline__ double mform(const double (&xz)[3], const double (&xp)[3], const double (&mzz)[6],
                                        const double (&mzp)[6], const double (&mpp)[6], int sh) {
  double s = 0.0;
#pragma unroll
  for (int a = 0; a < 3; ++a)
#pragma unroll
    for (int b = 0; b < 3; ++b) {
      const int n = a + b + sh;
      s += xz[a] * (xz[b] * mzz[n] + 2.0 * xp[b] * mzp[n]) + xp[a] * xp[b] * mpp[n];
    }
  return s;
}

// The state a launch's prologue reads, loaded in one batch at kernel entry:
// plain loads in straight-line code, so every one is in flight before the
// first wait (the stop tests, the breakdown / cap checks and the scalar
// algebra each waited for their own loads — several serial round trips to
// memory in front of every wave's first item).
struct St3 {
  long long iter, brk3, k0;
  int done, late3, wpar, started, bad3;
  double gprev;
  double n2[2][3];  // fs2[0 / 1][16 + i]: the last sweep's ‖p_i‖² (either parity)
  double sc[12];    // sc3[0 .. 11]: that sweep's {zc, α, β, g}
  double R[16];     // fs2[par ^ 1][0 .. 15]: its moment sums
};
__device__ __forceinline__ St3 st3_load(const DevState* st, int par) {
  St3 S;
  S.done = st->done;
  S.iter = st->iter;
  S.late3 = st->late3;
  S.wpar = st->wpar;
  S.started = st->started;
  S.bad3 = st->bad3;
  S.brk3 = st->brk3;
  S.k0 = st->k0;
  S.gprev = st->gprev;
#pragma unroll
  for (int i = 0; i < 3; ++i) {
    S.n2[0][i] = st->fs2[0][16 + i];
    S.n2[1][i] = st->fs2[1][16 + i];
  }
#pragma unroll
  for (int i = 0; i < 12; ++i) S.sc[i] = st->sc3[i];
  const double* R = st->fs2[par ^ 1];
#pragma unroll
  for (int i = 0; i < 16; ++i) S.R[i] = R[i];
  return S;
}

// From the previous sweep's 19 unweighted sums (a pure function of the state:
// every wave evaluates it and gets the same bits).
__device__ __forceinline__ Scal3 sweep3_scalars(const KParams& k, const St3& st, int par) {
  Scal3 c;
  c.first = st.started == 0;
  c.K = st.iter;
  c.m = 0;
  c.brk = 0;
  c.bad = false;
#pragma unroll
  for (int i = 0; i < 3; ++i) {
    c.c.zc[i] = 0.0;
    c.c.a[i] = 0.0;
    c.c.b[i] = 1.0;
    c.c.cw[i] = 0.0;
    c.g[i] = 0.0;
  }
  if (c.first) return c;
  const double hh = k.h1 * k.h2;
  const double* R = st.R;
  const double mzz[6] = {R[0], R[1], R[2], R[3], R[4], R[5]};
  const double mzp[6] = {0.0, R[6], R[7], R[8], R[9], R[10]};
  const double mpp[6] = {0.0, R[11], R[12], R[13], R[14], R[15]};
  long long lim = k.max_iter - c.K;
  if (lim > 3) lim = 3;
  if (k.mlimit > 0 && lim > k.mlimit) lim = k.mlimit;
  double zz[3] = {1.0, 0.0, 0.0}, zp[3] = {0.0, 0.0, 0.0};  // z_{i-1}
  double pz[3] = {0.0, 0.0, 0.0}, pp[3] = {1.0, 0.0, 0.0};  // p_{i-1}
  double g = mform(zz, zp, mzz, mzp, mpp, 0) * hh;
  double gprev = st.gprev;
  bool live = true;  // (fully unrolled, no early exit: the arrays stay in registers)
#pragma unroll
  for (int i = 0; i < 3; ++i) {
    live = live && i < lim;
    const double beta = c.K + i == st.k0 ? 0.0 : g / gprev;  // (k0: 0, or a restart's iteration)
#pragma unroll
    for (int q = 0; q < 3; ++q) {
      pz[q] = zz[q] + beta * pz[q];
      pp[q] = zp[q] + beta * pp[q];
    }
    const double den = mform(pz, pp, mzz, mzp, mpp, 1) * hh;
    const bool tiny = fabs(den) < 1e-15;
    const bool bad = !isfinite(g) || !isfinite(den);
    if (live && (tiny || bad)) {
      c.brk = i + 1;
      c.bad = bad;
      live = false;
    }
    if (live) {
      const double alpha = g / den;
      c.c.zc[i] = 1.0;
      c.c.a[i] = alpha;
      c.c.b[i] = beta;
      c.c.cw[i] = alpha;
      c.g[i] = g;
      c.m = i + 1;
      gprev = g;
      // z_i = z_{i-1} − α M p_i
      zz[2] -= alpha * pz[1];
      zz[1] -= alpha * pz[0];
      zp[2] -= alpha * pp[1];
      zp[1] -= alpha * pp[0];
      g = mform(zz, zp, mzz, mzp, mpp, 0) * hh;
    }
  }
  return c;
}

// Stop tests are resolved one launch late.  The ‖p_i‖² of a sweep's
// iterations are among its own sums, which are global only after the
// sweep's reduction — inside the sweep (one rank, or the in-sweep P2P sum)
// or after it (the comm's allreduce of the sums) — so every launch first
// decides, from the state alone (every wave gets the same bits), the stop
// tests its predecessor left pending (DevState::late3 iterations ending at
// st->iter, coefficients in sc3 = {zc, α, β, g}), then the breakdown / cap
// that predecessor saw coming, and only then starts new iterations.  A
// launch with mlimit < 0 (DeviceSolver::enqueue_wflush, after the host loop)
// only resolves.
struct Late3 {
  int stop;    // 1..3: the pending iteration that stops the solve (0: none)
  int status;  // its status: 1 converged, 4 non-finite ‖Δw‖
};

__device__ __forceinline__ double late_diff(const KParams& k, const DevState* st, int i) {
  // (both parities' ‖p_i‖² loaded and selected: indexing by wpar made the
  // load wait for wpar's — one more round trip in every launch's prologue)
  const double s0 = st->fs2[0][16 + i], s1 = st->fs2[1][16 + i];
  const double n2 = fmax(st->wpar ? s1 : s0, 0.0), a = st->sc3[3 + i];
  const double hh = k.h1 * k.h2;
  return k.weighted ? fabs(a) * sqrt(n2 * hh) : fabs(a) * sqrt(n2);
}

__device__ __forceinline__ double late_diff(const KParams& k, const St3& st, int i) {
  const double n2 = fmax(st.wpar ? st.n2[1][i] : st.n2[0][i], 0.0), a = st.sc[3 + i];
  const double hh = k.h1 * k.h2;
  return k.weighted ? fabs(a) * sqrt(n2 * hh) : fabs(a) * sqrt(n2);
}

__device__ __forceinline__ Late3 late3_test(const KParams& k, const St3& st) {
  Late3 r{0, 0};
  const int m = st.late3;
#pragma unroll
  for (int i = 0; i < 3; ++i) {
    if (r.stop == 0 && i < m) {
      const double d = late_diff(k, st, i);
      if (!isfinite(d)) {
        r.stop = i + 1;
        r.status = 4;
      } else if (k.check_tol && d < k.tol) {
        r.stop = i + 1;
        r.status = 1;
      }
    }
  }
  return r;
}

// History and reported scalars of the first n pending iterations (one thread).
__device__ __forceinline__ void late3_record(const KParams& k, DevState* st, int n) {
  const long long K0 = st->iter - st->late3;
#pragma unroll
  for (int i = 0; i < 3; ++i) {
    if (i < n) {
      const double d = late_diff(k, st, i);
      hist_put(k, K0 + i + 1, d);
      st->last_diff = d;
      st->alpha = st->sc3[3 + i];
      st->beta = st->sc3[6 + i];
      st->rz_cur = st->sc3[9 + i];
    }
  }
}

// Terminal state (one thread, after every wave of the grid has read the
// state): the pending iterations' records up to `upto`, then iteration
// `iter` with `status`.
__device__ __forceinline__ void sweep3_stop(const KParams& k, DevState* st, int upto, long long iter, int status,
                                            int fixj = 0) {
  late3_record(k, st, upto);
  st->fixj = fixj;
  st->iter = iter;
  st->status = status;
  st->late3 = 0;
  st->brk3 = 0;
  st->done = 1;
  st->wpend = 0;
}

// The pending iterations' records as late3_record writes them, from values
// a wave of every workgroup read at kernel entry (struct Pend3, LDS): the
// finalize after the grid reduction then reloads nothing from the state (one
// L2-missing round trip, ≈1 µs of every sweep's epilogue).
struct Pend3 {
  double d[3], a[3], b[3], g[3];
  long long K0;
  int n;
};
__device__ __forceinline__ void pend3_load(const KParams& k, const St3& st, int m0, long long K0, Pend3& p) {
  p.K0 = K0;
  p.n = m0;
#pragma unroll
  for (int i = 0; i < 3; ++i)
    if (i < m0) {
      p.d[i] = late_diff(k, st, i);
      p.a[i] = st.sc[3 + i];
      p.b[i] = st.sc[6 + i];
      p.g[i] = st.sc[9 + i];
    }
}
__device__ __forceinline__ void pend3_record(const KParams& k, DevState* st, const Pend3& p) {
#pragma unroll
  for (int i = 0; i < 3; ++i)
    if (i < p.n) {
      hist_put(k, p.K0 + i + 1, p.d[i]);
      if (i + 1 == p.n) {
        st->last_diff = p.d[i];
        st->alpha = p.a[i];
        st->beta = p.b[i];
        st->rz_cur = p.g[i];
      }
    }
}

// State update after a full sweep (one thread; sums t[] global or, with the
// comm's allreduce after the sweep, this rank's): the previous sweep's
// pending records (its stop tests passed at this launch's entry), then this
// sweep's sums, coefficients and tentative iteration count; its own stop
// tests are pending until the next launch.
__device__ __forceinline__ void sweep3_finalize(const KParams& k, DevState* st, int par, const Scal3& c,
                                                const double (&t)[NS], const Pend3& pend) {
  if (!c.first) pend3_record(k, st, pend);
#pragma unroll
  for (int n = 0; n < NS; ++n) st->fs2[par][n] = t[n];
  // fault hooks (PE_FAULT_INJECT): the sums of the sweep completing iteration F
  if (!c.first && k.fault_iter > c.K && k.fault_iter <= c.K + c.m) st->fs2[par][1] = __builtin_nan("");
  if (!c.first && k.fault_zero > c.K && k.fault_zero <= c.K + c.m)
    st->fs2[par][1] = st->fs2[par][6] = st->fs2[par][11] = 0.0;
  st->wpend = 0;
  st->wpar = par;
  if (c.first) {
    st->started = 1;
    return;
  }
#pragma unroll
  for (int i = 0; i < 3; ++i) {
    st->sc3[i] = c.c.zc[i];
    st->sc3[3 + i] = c.c.a[i];
    st->sc3[6 + i] = c.c.b[i];
    st->sc3[9 + i] = c.g[i];
    if (i + 1 == c.m) {
      st->alpha = c.c.a[i];
      st->beta = c.c.b[i];
      st->rz_cur = c.g[i];
      st->gprev = c.g[i];
    }
  }
  st->iter = c.K + c.m;
  st->late3 = c.m;
  st->brk3 = c.brk ? c.K + c.brk : 0;
  st->bad3 = c.bad ? 1 : 0;
}

// Item kinds (list entry flags): band items (a boundary-band row in the
// window: coefficients from the chord tables, LDS face ring), uniform items
// (kUniBit: every row of the window lies wholly inside or wholly outside the
// interior in this strip — the row's coefficients are three scalars) and
// mixed plain items (per-lane interior tests).
enum { kMixed = 0, kBand = 1, kUniform = 2 };

// Lane / item constants of one march.
struct M3Ctx {
  const double* Xm;   // input rows, at column -5
  double* Ym;         // output rows
  double* Wm;         // w rows
  const double* hrd;  // PUSH: receive buffer of the parity this sweep reads
  int64_t pitch, poff, wp;
  int J, c0, ib, ie, t0, tmax, nx, par;
  unsigned off;
  bool lv0, o0, fix;
  bool scol;          // the lane's column is not past ny (2-D blocks: past ny are the UP neighbour's)
  double lf0;         // lv0 as 1.0 / 0.0 (uniform items of the edge strips)
  double oih1, oih2;  // inv_eps / h1², inv_eps / h2² (uniform exterior rows)
  double ih1, ih2, din, dout;  // 1/h1², 1/h2², 1/D interior / exterior (copies: a select between
                               // kernel-argument fields compiles to a scalar load per use)
  int rlo, rhi;       // local rows of the global interior: rlo ≤ q ≤ rhi
  double zc1, zc2, zc3, a1, a2, a3, b1, b2, b3, w1, w2, w3;
};

// The march's register state: prefetch rings and the stage row rings.
struct M3Rings {
  double RQ[kS3XD], PQ[kS3XD], WQ[kS3WD];
  double P1[3], RI[2], R1[2], P2[3], R2[2], P3[3], Z[3], S[2], U[3], V[3], UU[3], VV[3];
  bool pushed;
};

// A wave's first item as loaded at kernel entry: its list entry and the
// row-class entry of its first row window — the two dependent loads in front
// of its first row loads.  Neither depends on the sweep's scalars, so their
// latency overlaps the state reads and the scalar algebra instead of
// following them (kernel entry to the first item's first row step: 5.4-6.9
// µs, tools/stamp_probe.py, profiles/r5_stamps_concentrated.txt).  (Its first
// r / p / w rows too: live across the walk loop they spilled 5-11 VGPRs.)
struct Pre3 {
  int2 e;  // (rows field 0: no item)
  int4 rc4;
  bool staged;  // its first r / p / w rows were sent into the wave's LDS (stage_first3)
};

template <bool STEADY>
__device__ __forceinline__ URow urow(const M3Ctx& c, const RowCtx& rx, int q) {
  const int l = (q - rx.segbase) & 63;
  const bool in = (rx.allin >> l) & 1ull;
  URow r;
  r.ih1 = in ? c.ih1 : c.oih1;
  r.ih2 = in ? c.ih2 : c.oih2;
  r.d = in ? c.din : c.dout;
  if constexpr (!STEADY) {
    if (!(q >= c.rlo && q <= c.rhi)) r.d = 0.0;
  }
  return r;
}

template <bool PUSH>
__device__ __forceinline__ double ldx3(const KParams& k, const M3Ctx& c, int t, unsigned o) {
  if constexpr (PUSH) {
    if ((t < 1 && k.has[LEFT]) || (t > c.nx && k.has[RIGHT])) {
      const double* h = c.hrd + int64_t(t < 1 ? t + H3 - 1 : t - c.nx + H3 - 1) * c.pitch + o;
      return __hip_atomic_load(h, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    }
  }
#if PE_S3_NTX
  return __builtin_nontemporal_load(c.Xm + int64_t(t) * c.pitch + o);
#else
  return c.Xm[int64_t(t) * c.pitch + o];
#endif
}

__device__ __forceinline__ double ldnt1(const double* p) { return __builtin_nontemporal_load(p); }
__device__ __forceinline__ void stnt1(double* p, double v) { __builtin_nontemporal_store(v, p); }

// rows 1..6 → the LEFT neighbour's rows nx'+1..nx'+6; nx-5..nx → the RIGHT one's -5..0
__device__ __forceinline__ void push_row3(const KParams& k, const M3Ctx& c, M3Rings& x, int q, double r3, double p3) {
  auto put = [&](double* base, int slot) {
    double* d = base + int64_t(slot) * c.pitch + c.off;
    if (c.o0) {
      __hip_atomic_store(d, r3, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      __hip_atomic_store(d + c.poff, p3, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    }
    x.pushed = true;
  };
  if (q <= H3 && k.hpush_lo[c.par] != nullptr) put(k.hpush_lo[c.par], q - 1);
  if (q >= c.nx - H3 + 1 && k.hpush_hi[c.par] != nullptr) put(k.hpush_hi[c.par], q - (c.nx - H3 + 1));
}

// One row step of the march: stage A at row t = t0 + n, B..G at rows
// t-1..t-6.  JJ = n mod 6 fixes the register ring slots at compile time; bs
// is the band face-ring slot of row t.  STEADY (uniform items): every stage
// row lies inside the item — no row tests, no clamped loads.
template <int KIND, bool PUSH, bool EDGE, bool STEADY, int JJ>
__device__ __forceinline__ void step3(const KParams& k, const M3Ctx& c, M3Rings& x, const RowCtx& rx, WaveTV3& tvw,
                                      double (&sv)[NS], int n, int bs) {
  constexpr bool BAND = KIND == kBand, UNI = KIND == kUniform;
  constexpr int XD = kS3XD, WD = kS3WD;
  const double zc1 = c.zc1, zc2 = c.zc2, zc3 = c.zc3, w1 = c.w1, w2 = c.w2, w3 = c.w3;
  // register ring slots: row t-d ↦ (JJ - d) mod 3 / mod 2
  constexpr int m0 = JJ % 3, m1 = (JJ + 2) % 3, m2 = (JJ + 1) % 3;  // rows t, t-1, t-2 (t-3 ≡ t)
  constexpr int e0 = JJ & 1, e1 = (JJ + 1) & 1;                      // rows t, t-1 (t-2 ≡ t)
  constexpr int xs = JJ % XD, ws = JJ % WD;
  const int t = c.t0 + n;
  const int c0 = c.c0;
  // row inside the item (steady: always — tested as "not a fix-up launch",
  // which skips the sums there: the uniform branch keeps the compiler from
  // interleaving the stages' sums, which costs ~200 VGPRs)
  auto inr = [&](int q) { return STEADY ? !c.fix : (q >= c.ib && q <= c.ie); };
  auto own = [&](int q) { return STEADY || (q >= c.ib && q <= c.ie); };  // (stores)
  // sums of the item's rows; lane-tested kinds drop columns past ny (an UP
  // neighbour's, in the last strip of a 2-D block: never a uniform item) by a
  // select, not a branch — the stages' DPP neighbour reads need every lane
  // active (a disabled source lane reads as 0)
  auto put = [&](int n, double v) {
    if constexpr (UNI) sv[n] += v;
    else sv[n] += c.scol ? v : 0.0;
  };
  auto interior = [&](int q) { return q >= c.rlo && q <= c.rhi; };     // global interior row
  // pipeline fill: stage d (B = 1 … F = 5) first feeds a needed row at step
  // 2d (G's rows are tested by inr): skip it before — its rows are never used
  auto live = [&](int d) { return STEADY || n >= 2 * d; };
  // band ring slots (runtime, mod 7) of rows t .. t-6
  int bsl[7];
#pragma unroll
  for (int d = 0; d < 7; ++d) bsl[d] = bs >= d ? bs - d : bs - d + kRing3;
  // masked products z = D⁻¹·v (0 at global-boundary rows / columns)
  auto zmask = [&](int q, double v, double d) -> double {
    if constexpr (UNI) {  // d: the row scalar (interior rows folded in)
      return EDGE ? (v * d) * c.lf0 : v * d;
    } else {
      return (interior(q) && c.lv0) ? v * d : 0.0;
    }
  };
  // the operator at row q (band ring slots sl, sln) and 1/D of the node
  auto op = [&](int q, int sl, int sln, double um, double u0, double un, double& d) {
    if constexpr (UNI) {
      const URow r = urow<STEADY>(c, rx, q);
      d = r.d;
      return lapu(r, um, u0, un);
    } else {
      return apply_row1<BAND>(k, rx, tvw, q, c0, sl, sln, um, u0, un, d);
    }
  };
  // ---- A: row t ----
  const double rin = x.RQ[xs], pin = x.PQ[xs], wrow = x.WQ[ws];
  {
    const int tn = STEADY ? t + XD : min(t + XD, c.tmax);
    x.RQ[xs] = ldx3<PUSH>(k, c, tn, c.off);
    x.PQ[xs] = ldx3<PUSH>(k, c, tn, unsigned(c.poff) + c.off);
    const int wr = STEADY ? t - 2 + WD : min(max(t - 2 + WD, c.ib), c.ie);
    // (only the lanes that store w load it: the 12 halo lanes' columns are a
    // neighbouring strip's, and their lines would be fetched for nothing)
    x.WQ[ws] = c.o0 ? ldnt1(c.Wm + int64_t(wr) * c.wp + c.off) : 0.0;
  }
  {
    double d;
    if constexpr (UNI) d = urow<STEADY>(c, rx, t).d;
    else d = BAND ? enter_band1(k, rx, tvw, t, c0, bsl[0]) : dinv_plain1(k, rx, t, c0);
    const double z = zmask(t, rin, d);
    x.P1[m0] = zc1 * z + c.b1 * pin;
    x.RI[e0] = rin;
  }
  if (STEADY) __builtin_amdgcn_sched_barrier(0);  // (stage by stage, as the row tests of the generic steps)
  // ---- B: row t-1 ----
  if (live(1)) {
    const int q = t - 1;
    double d;
    const double s1 = op(q, bsl[1], bsl[0], x.P1[m2], x.P1[m1], x.P1[m0], d);
    const double r1 = x.RI[e1] - c.a1 * s1;
    const double z = zmask(q, r1, d);
    const double p1 = x.P1[m1];
    x.R1[e1] = r1;
    x.P2[m1] = zc2 * z + c.b2 * p1;
    if (inr(q)) put(16, p1 * p1);
  }
  if (STEADY) __builtin_amdgcn_sched_barrier(0);
  // ---- C: row t-2 (w) ----
  if (live(2)) {
    const int q = t - 2;
    double d;
    const double s2 = op(q, bsl[2], bsl[1], x.P2[m0], x.P2[m2], x.P2[m1], d);
    const double r2 = x.R1[e0] - c.a2 * s2;
    const double z = zmask(q, r2, d);
    const double p2 = x.P2[m2];
    x.R2[e0] = r2;
    const double p3 = zc3 * z + c.b3 * p2;
    x.P3[m2] = p3;
    if (own(q) && c.o0) stnt1(c.Wm + int64_t(q) * c.wp + c.off, wrow + w1 * x.P1[m2] + w2 * p2 + w3 * p3);
    if (inr(q)) put(17, p2 * p2);
  }
  if (STEADY) __builtin_amdgcn_sched_barrier(0);
  // ---- D: row t-3 (r, p outputs) ----
  if (live(3)) {
    const int q = t - 3;
    double d;
    const double s3 = op(q, bsl[3], bsl[2], x.P3[m1], x.P3[m0], x.P3[m2], d);
    const double r3 = x.R2[e1] - c.a3 * s3;
    const double z = zmask(q, r3, d);
    x.Z[m0] = z;
    x.S[e1] = s3;
    const double p3 = x.P3[m0];
    if (own(q) && !c.fix) {
      if (c.o0) {
        double* yr = c.Ym + int64_t(q) * c.pitch + c.off;
        stnt1(yr, r3);
        stnt1(yr + c.poff, p3);
      }
      if constexpr (PUSH) push_row3(k, c, x, q, r3, p3);
    }
    if (inr(q)) {
      put(0, r3 * z);    // (r,z)
      put(6, z * s3);    // (z,s)
      put(11, p3 * s3);  // (p,s)
      put(18, p3 * p3);  // ‖p₃‖²
    }
  }
  if (STEADY) __builtin_amdgcn_sched_barrier(0);
  // ---- E: row t-4 ----
  if (live(4)) {
    const int q = t - 4;
    double d;
    const double qv = op(q, bsl[4], bsl[3], x.Z[m2], x.Z[m1], x.Z[m0], d);
    const double sr = x.S[e0];
    const double u = zmask(q, qv, d);
    const double v = zmask(q, sr, d);
    x.U[m1] = u;
    x.V[m1] = v;
    if (inr(q)) {
      put(1, x.Z[m1] * qv);  // (z,q)
      put(2, qv * u);        // (q,u)
      put(7, qv * v);        // (q,v)
      put(12, sr * v);       // (s,v)
    }
  }
  if (STEADY) __builtin_amdgcn_sched_barrier(0);
  // ---- F: row t-5 ----
  if (live(5)) {
    const int q = t - 5;
    double d, d2;
    const double au = op(q, bsl[5], bsl[4], x.U[m0], x.U[m2], x.U[m1], d);
    const double av = op(q, bsl[5], bsl[4], x.V[m0], x.V[m2], x.V[m1], d2);
    const double uu = zmask(q, au, d);
    const double vv = zmask(q, av, d);
    x.UU[m2] = uu;
    x.VV[m2] = vv;
    if (inr(q)) {
      const double u = x.U[m2], v = x.V[m2];
      put(3, u * au);    // (u,Au)
      put(8, u * av);    // (u,Av)
      put(13, v * av);   // (v,Av)
      put(4, au * uu);   // (Au,ũ)
      put(9, au * vv);   // (Au,ṽ)
      put(14, av * vv);  // (Av,ṽ)
    }
  }
  if (STEADY) __builtin_amdgcn_sched_barrier(0);
  // ---- G: row t-6 ----
  {
    const int q = t - 6;
    if (inr(q)) {
      double d;
      const double auu = op(q, bsl[6], bsl[5], x.UU[m1], x.UU[m0], x.UU[m2], d);
      const double avv = op(q, bsl[6], bsl[5], x.VV[m1], x.VV[m0], x.VV[m2], d);
      const double uu = x.UU[m0], vv = x.VV[m0];
      put(5, uu * auu);   // (ũ,Aũ)
      put(10, uu * avv);  // (ũ,Aṽ)
      put(15, vv * avv);  // (ṽ,Aṽ)
    }
  }
}

// Six row steps (one period of the register rings).  Generic groups stop at
// the item's last step.  Steady groups are straight-line code: a scheduling
// barrier after each step keeps the scheduler from hoisting later steps'
// work into this one.
template <int KIND, bool PUSH, bool EDGE, bool STEADY>
__device__ __forceinline__ void group3(const KParams& k, const M3Ctx& c, M3Rings& x, const RowCtx& rx, WaveTV3& tvw,
                                       double (&sv)[NS], int n0, int nsteps, int& bs) {
  auto adv = [&]() { bs = bs == kRing3 - 1 ? 0 : bs + 1; };
#define PE_STEP3(JJ)                                                              \
  if (STEADY || n0 + JJ < nsteps) {                                               \
    step3<KIND, PUSH, EDGE, STEADY, JJ>(k, c, x, rx, tvw, sv, n0 + JJ, bs);       \
    adv();                                                                        \
    if (STEADY) __builtin_amdgcn_sched_barrier(0);                                \
  }
  PE_STEP3(0)
  PE_STEP3(1)
  PE_STEP3(2)
  PE_STEP3(3)
  PE_STEP3(4)
  PE_STEP3(5)
#undef PE_STEP3
}

// The item march (one strip × rows ib..ie), accumulating this wave's sums.
// FIX (fix-up launch): same march over the same inputs, w only.
// PUSH (row slabs over the P2P transport): output rows 1..6 / nx-5..nx are
// also stored into the x-neighbours' fine-grained receive buffers over xGMI
// (system-scope write-through stores, drained and released at the end of the
// item), and the halo rows -5..0 / nx+1..nx+6 are read from this rank's
// receive buffer (system-scope loads) — fused2.hip's halo push at depth 6.
// Sums are taken over the item's rows without per-term column masks: every
// sum has a factor among z, p, u, v, ũ, ṽ, which are exactly 0 at the
// global-boundary and padding columns, and the lanes that do not own their
// columns (0..7, 56..63) are dropped once, at the end of the sweep.
__device__ __forceinline__ unsigned long long rtc3() {
  unsigned long long t;  // one asm statement: never merged or moved by the compiler
  asm volatile("s_memrealtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t)::"memory");
  return t;
}

// PE_PRIO (KParams::prio > 0, experimental): the two waves on a SIMD — one of
// a CU's first workgroup, one of its second — take turns at issue priority
// every 2^prio ticks of the 100 MHz clock.  By default the older wave wins
// every tie and runs ≈12-23 % faster per row step, then the younger one
// marches alone at the end of the sweep (tools/stamp_probe.py "SIMD with one
// wave left", profiles/r5_wave_age.txt).
__device__ __forceinline__ void prio_turn(const KParams& k) {
  if (k.prio > 0) {
    const unsigned long long t = rtc3();
    const bool young = int(blockIdx.x) >= k.ncu;
    if ((((t >> k.prio) & 1ull) != 0) != young) __builtin_amdgcn_s_setprio(1);
    else __builtin_amdgcn_s_setprio(0);
  }
}

// (SST, the diagnostic build only: sst != nullptr stamps this item's
// prologue and every 6-step group into the wave's step stamps)
template <int KIND, bool PUSH, bool EDGE, bool SST = false>
__device__ __forceinline__ void march3(const KParams& k, const Coef3& cf, bool fix, int par, int s, int ib, int ie,
                                       WaveTV3& tvw, double (&sv)[NS], unsigned long long* sst, const Pre3& pre,
                                       bool use_pre) {
  const int lane = threadIdx.x & 63;
  const int ny = int(k.ny);
  M3Ctx c;
  c.pitch = k.pitch;
  c.poff = k.poff;
  c.wp = k.wpitch;
  c.Xm = k.x[par ^ 1] - (HL3 - 1);  // row pointers at column -(HL3-1) = element 0 (k.xorg)
  c.Ym = k.x[par] - (HL3 - 1);
  c.Wm = k.w - (HL3 - 1);
  c.J = -(HL3 - 1) + s * FSW3;
  c.c0 = c.J + lane;
  c.off = unsigned(c.c0 + HL3 - 1);
  const int64_t g0 = k.gj0 + c.c0;
  c.lv0 = c.c0 <= ny + H3 && g0 >= 1 && g0 <= k.N - 1;
  c.lf0 = c.lv0 ? 1.0 : 0.0;
  c.o0 = lane >= HL3 && lane < 64 - HR3 && c.c0 >= 1 && c.c0 <= ny;
  c.scol = c.c0 <= ny;
  c.fix = fix;
  c.ib = ib;
  c.ie = ie;
  c.t0 = ib - H3;
  c.tmax = ie + H3;
  c.nx = int(k.nx);
  c.par = par;
  c.hrd = PUSH ? k.hrecv + int64_t(par ^ 1) * 2 * H3 * k.pitch : nullptr;
  c.oih1 = uni(k.inv_eps * k.ih1sq);
  c.oih2 = uni(k.inv_eps * k.ih2sq);
  c.ih1 = k.ih1sq;
  c.ih2 = k.ih2sq;
  c.din = k.dinv_in;
  c.dout = k.dinv_out;
  c.rlo = int(max<int64_t>(1 - k.gi0, -(1 << 30)));
  c.rhi = int(min<int64_t>(k.M - 1 - k.gi0, 1 << 30));
  c.zc1 = cf.zc[0];
  c.zc2 = cf.zc[1];
  c.zc3 = cf.zc[2];
  c.a1 = cf.a[0];
  c.a2 = cf.a[1];
  c.a3 = cf.a[2];
  c.b1 = cf.b[0];
  c.b2 = cf.b[1];
  c.b3 = cf.b[2];
  c.w1 = cf.cw[0];
  c.w2 = cf.cw[1];
  c.w3 = cf.cw[2];

  // Row classes / column tables of a 64-row window, reloaded every ~58 rows
  // on tall items (stage rows t-6 .. t and the column-table row t+1 inside).
  RowCtx rx;
  auto load_seg = [&](int base) { load_rows<KIND == kBand, WaveTV3, 64>(k, rx, tvw, base, ie + H3 + 1, c.J); };
  if (KIND == kBand) load_strip_tables1(k, tvw, c.c0);
  if (use_pre) load_rows<KIND == kBand, WaveTV3, 64>(k, rx, tvw, c.t0, ie + H3 + 1, c.J, &pre.rc4);
  else load_seg(c.t0);

  M3Rings x;
  x.pushed = false;
  constexpr int XD = kS3XD, WD = kS3WD;
  static_assert(WD <= 6, "the first WD w rows are all row ib (t0 - 2 + q < ib)");
  if (use_pre && pre.staged && KIND != kBand) {  // (stage_first3: rows t0 .. t0+XD-1 ≤ tmax, w row ib)
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    const double* L = &tvw.a0r[0][0];
#pragma unroll
    for (int q = 0; q < XD; ++q) {
      x.RQ[q] = L[q * 128 + lane];
      x.PQ[q] = L[q * 128 + 64 + lane];
    }
    const double w0 = L[XD * 128 + lane];
#pragma unroll
    for (int q = 0; q < WD; ++q) x.WQ[q] = c.o0 ? w0 : 0.0;
  } else {
#pragma unroll
    for (int q = 0; q < XD; ++q) {
      const int t = min(c.t0 + q, c.tmax);
      x.RQ[q] = ldx3<PUSH>(k, c, t, c.off);
      x.PQ[q] = ldx3<PUSH>(k, c, t, unsigned(c.poff) + c.off);
    }
#pragma unroll
    for (int q = 0; q < WD; ++q)
      x.WQ[q] = c.o0 ? ldnt1(c.Wm + int64_t(min(max(c.t0 - 2 + q, ib), ie)) * c.wp + c.off) : 0.0;
  }
#pragma unroll
  for (int q = 0; q < 3; ++q) x.P1[q] = x.P2[q] = x.P3[q] = x.Z[q] = x.U[q] = x.V[q] = x.UU[q] = x.VV[q] = 0.0;
#pragma unroll
  for (int q = 0; q < 2; ++q) x.RI[q] = x.R1[q] = x.R2[q] = x.S[q] = 0.0;

  const int nsteps = ie + H3 - c.t0 + 1;
  const int rows = ie - ib + 1;
  int bs = 0;  // band ring slot of row t: (t - t0) mod 7
  int sg = 3;  // (SST: next step-stamp slot)
  if constexpr (SST) {
    if (sst && lane == 0) sst[2] = rtc3();
  }
  auto sstamp = [&]() {
    if constexpr (SST) {
      if (sst && lane == 0 && sg < 28) sst[sg] = rtc3();  // (slots 28/29: shader clock at entry / exit, 30: hardware id)
      ++sg;
    }
    prio_turn(k);
  };
  // steady groups (uniform items): stage rows t-6 .. t and the prefetched
  // rows inside the item for all six steps (n ≥ 12, n ≤ rows + 4); the fill
  // and drain groups around them test rows.  Three loops, not one with a
  // branch: the merged ring state would cost a copy of every ring.
  auto reload = [&](int n0) {
    if (c.t0 + n0 + 6 - rx.segbase > 63) load_seg(c.t0 + n0 - H3);  // tall items: next row window
  };
  int n0 = 0;
  const int nsteady_end = KIND == kUniform ? rows + 4 - 5 : -1;  // last steady group start
  for (; n0 < nsteps && !(n0 >= 12 && n0 <= nsteady_end); n0 += 6) {
    reload(n0);
    group3<KIND, PUSH, EDGE, false>(k, c, x, rx, tvw, sv, n0, nsteps, bs);
    sstamp();
  }
  if constexpr (KIND == kUniform) {
    for (; n0 <= nsteady_end; n0 += 6) {
      reload(n0);
      group3<KIND, PUSH, EDGE, true>(k, c, x, rx, tvw, sv, n0, nsteps, bs);
      sstamp();
    }
    for (; n0 < nsteps; n0 += 6) {
      reload(n0);
      group3<KIND, PUSH, EDGE, false>(k, c, x, rx, tvw, sv, n0, nsteps, bs);
      sstamp();
    }
  }
  if constexpr (PUSH) {
    // The pushed rows went out as system-scope atomic stores (sc0 sc1: write-
    // through to the neighbour's fine-grained buffer), so their completion is
    // their delivery: drained here, before this wave's ticket, and the last
    // block's flags (peer_sum_block's own release) follow them.  A system-
    // scope release fence here also wrote the XCD's whole L2 back
    // (buffer_wbl2) once per pushing item — 2 × 171 of them per sweep at the
    // 8-rank slab of 8192²: 70 → 65 µs per iteration with the push kernel
    // (PE_PUSH_LOOPBACK, profiles/r5_push_release.txt).
    if (x.pushed) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
}

// The first list position of wave gwave and that item's first loads (Pre3).
__device__ __forceinline__ void pre_load3(const KParams& k, int gwave, Pre3& pr) {
  pr.e = make_int2(0, 0);
  if (!(gwave < k.lwaves && gwave < k.nslots)) return;
  pr.e = cload_i2(k.ilist + gwave);
  const int rows = pr.e.y >> 20;
  if (rows == 0) return;
  const int ib = pr.e.x & kRowMask3;
  const int ie = min(ib + rows - 1, int(k.nx));
  pr.rc4 = rowcls_entry(k, ib - H3, ie + H3 + 1);
}

// The first item's first rows — r / p rows t0 .. t0+XD-1 and its w row ib —
// sent straight into the wave's LDS by LDS-DMA (global_load_lds: no VGPRs,
// so nothing is live across the walk loop) at kernel entry, where their DRAM
// latency overlaps the three iterations' scalar algebra instead of following
// it; march3 reads them from there (use_pre && staged).  The LDS is the band
// face ring's a0r (3.5 KB), free until the wave's first band item zeroes it:
// only items that are not band items are staged, and only rows of x itself
// (PUSH: not the receive buffer's halo rows).  PE_STAGE=0: off.
template <bool PUSH>
__device__ __forceinline__ void stage_first3(const KParams& k, int par, WaveTV3& tv, Pre3& pr) {
  pr.staged = false;
  const int rows = pr.e.y >> 20;
  if (rows == 0 || !k.stage || (pr.e.x & kBandBit)) return;
  const int sx = pr.e.y & 0xFFFFF, ib = pr.e.x & kRowMask3;
  const int t0 = ib - H3;
  if (PUSH && (t0 < 1 || t0 + kS3XD - 1 > int(k.nx))) return;
  typedef __attribute__((address_space(3))) void* lds_ptr;
  typedef __attribute__((address_space(1))) const void* g_ptr;
  const int lane = threadIdx.x & 63;
  const double* Xm = k.x[par ^ 1] - (HL3 - 1) + sx * FSW3;  // the strip's element 0 (march3: c.Xm + c.J + HL3 - 1)
  const double* Wm = k.w - (HL3 - 1) + sx * FSW3;
  static_assert((kS3XD * 128 + 64) * sizeof(double) <= sizeof(tv.a0r) + sizeof(tv.b0r), "staged rows fit the face ring");
  double* L = &tv.a0r[0][0];  // [q][r 64 | p 64] for q < XD, then [w 64] (a0r, then b0r right after it)
#pragma unroll
  for (int q = 0; q < kS3XD; ++q) {
    const char* rr = reinterpret_cast<const char*>(Xm + int64_t(t0 + q) * k.pitch);
    const char* pp = reinterpret_cast<const char*>(Xm + int64_t(t0 + q) * k.pitch + k.poff);
#pragma unroll
    for (int h = 0; h < 2; ++h) {  // 4 bytes per lane: two instructions per 512-B row
      __builtin_amdgcn_global_load_lds((g_ptr)(rr + 256 * h + 4 * lane), (lds_ptr)(L + q * 128 + 32 * h), 4, 0, 0);
      __builtin_amdgcn_global_load_lds((g_ptr)(pp + 256 * h + 4 * lane), (lds_ptr)(L + q * 128 + 64 + 32 * h), 4, 0, 0);
    }
  }
  const char* wr = reinterpret_cast<const char*>(Wm + int64_t(ib) * k.wpitch);
#pragma unroll
  for (int h = 0; h < 2; ++h)
    __builtin_amdgcn_global_load_lds((g_ptr)(wr + 256 * h + 4 * lane), (lds_ptr)(L + kS3XD * 128 + 32 * h), 4, 0, 0);
  pr.staged = true;
}

__device__ __forceinline__ Coef3 uni3(const Coef3& c) {
  Coef3 u;
#pragma unroll
  for (int i = 0; i < 3; ++i) {
    u.zc[i] = uni(c.zc[i]);
    u.a[i] = uni(c.a[i]);
    u.b[i] = uni(c.b[i]);
    u.cw[i] = uni(c.cw[i]);
  }
  return u;
}

// Walk this wave's positions of the static item list.
// Kernel variants (separate instantiations, so the production march is the
// plain one): kPlain; kStamp — diagnostic build (PE_STAMPS=1,
// tools/stamp_probe.py): lane 0 of every wave records s_memrealtime at its
// entry and exit and at the start and end of every item into k.stamps (the
// single sweep's layout: per position {start, end, wave | strip << 32, first
// row | rows << 32 | kind << 48}, kind 1 band, 2 uniform, 0 mixed; then per
// wave {entry, exit}); kReplay — the end-of-solve replay (kReplay3); kSignal
// — halo/interior overlap: the first k.lnb[0] positions of the static list
// are boundary items (outputs a neighbour needs), each of which bumps st->sig
// once its stores have left the wave (kWaitSig on the halo stream then
// writes the L2s back and the exchange starts while interior items run).
enum { kPlain = 0, kStamp = 1, kReplay = 2, kSignal = 3 };

template <bool PUSH, int MODE>
__device__ __forceinline__ void walk3(const KParams& k, const Coef3& cf, bool fix, int par, WaveTV3& tv, int wid,
                                      double (&acc)[NS], const Pre3& pre, bool have_pre) {
  constexpr bool STAMP = MODE == kStamp;
  const int W = k.lwaves;
  const int gwave = int(blockIdx.x) * kWPB + wid;
  const bool l0 = (threadIdx.x & 63) == 0;
  if constexpr (STAMP) {
    if (l0) k.stamps[4 * int64_t(k.nslots) + 2 * gwave] = rtc3();
  }
  // (waves past the layout's W — the overlap's reserved blocks when a launch
  // uses the whole grid: the construction's timing sweeps, S_0, the replay —
  // have no list positions; they used to march round r+1's first items twice)
  const int pend = gwave < W ? k.nslots : 0;
  unsigned long long* sst = STAMP ? k.stamps2 + 32 * int64_t(gwave) : nullptr;  // (the first item only)
  bool p1 = have_pre && !fix;  // (a fix-up marches other inputs than the ones loaded at entry)
  bool ring_zeroed = false;
  for (int pos = gwave; pos < pend; pos += W) {
    const int2 e = p1 ? pre.e : cload_i2(k.ilist + pos);
    const int rows = e.y >> 20;
    if (rows == 0) {  // empty position of the static layout
      p1 = false;
      continue;
    }
    const int s = e.y & 0xFFFFF, ib = e.x & kRowMask3;
    const int ie = min(ib + rows - 1, int(k.nx));
    const unsigned long long t_item = STAMP ? rtc3() : 0ull;
    if constexpr (STAMP) {
      if (sst && l0) sst[0] = t_item;
    }
    if (e.x & kBandBit) {
      // the face / 1/D ring: defined contents (the never-written column 64 of
      // b0 and the slots garbage pipeline-fill rows read stay finite) — before
      // each band item, not in every wave's launch prologue
      if (!ring_zeroed) {
        if (have_pre && pre.staged) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // (a0r: the staged rows' LDS)
        const int ln = threadIdx.x & 63;
        for (int i = ln; i < kRing3 * 64; i += 64) (&tv.a0r[0][0])[i] = 0.0;
        for (int i = ln; i < kRing3 * 66; i += 64) (&tv.b0r[0][0])[i] = 0.0;
        for (int i = ln; i < kRing3 * 64; i += 64) (&tv.d0r[0][0])[i] = 0.0;
        ring_zeroed = true;
      }
      march3<kBand, PUSH, true, STAMP>(k, cf, fix, par, s, ib, ie, tv, acc, sst, pre, p1);
    } else if (e.x & kUniBit) {
      // edge strips (a global-boundary or padding column in the window) mask z
      const int c0 = -(HL3 - 1) + s * FSW3 + int(threadIdx.x & 63);
      const int64_t g0 = k.gj0 + c0;
      const bool lv = c0 <= int(k.ny) + H3 && g0 >= 1 && g0 <= k.N - 1;
      if (__ballot(lv) == ~0ull) march3<kUniform, PUSH, false, STAMP>(k, cf, fix, par, s, ib, ie, tv, acc, sst, pre, p1);
      else march3<kUniform, PUSH, true, STAMP>(k, cf, fix, par, s, ib, ie, tv, acc, sst, pre, p1);
    } else {
      march3<kMixed, PUSH, true, STAMP>(k, cf, fix, par, s, ib, ie, tv, acc, sst, pre, p1);
    }
    p1 = false;
    if constexpr (STAMP) {
      if (sst && l0) sst[31] = rtc3();
      sst = nullptr;
    }
    if constexpr (MODE == kSignal) {
      if (pos < k.lnb[0]) {  // a boundary item: count it once its stores have left (no L2 writeback here)
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        if (l0) __hip_atomic_fetch_add(&k.st->sig, 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
    }
    if constexpr (STAMP) {
      if (l0) {
        const unsigned long long kind = (e.x & kBandBit) ? 1ull : (e.x & kUniBit) ? 2ull : 0ull;
        unsigned long long* d = k.stamps + 4 * int64_t(pos);
        d[0] = t_item;
        d[1] = rtc3();
        d[2] = (unsigned long long)gwave | ((unsigned long long)s << 32);
        d[3] = (unsigned long long)ib | ((unsigned long long)(ie - ib + 1) << 32) | (kind << 48);
      }
    }
  }
  if constexpr (STAMP) {
    if (l0) {
      k.stamps[4 * int64_t(k.nslots) + 2 * gwave + 1] = rtc3();
      k.stamps2[32 * int64_t(gwave) + 29] = __builtin_amdgcn_s_memtime();  // (shader clock: Δ / Δ realtime)
    }
  }
}

template <bool PUSH, int MODE = kPlain>
__global__ __launch_bounds__(TJ) __attribute__((amdgpu_waves_per_eu(2))) void kS3(KParams k, int par) {
  DevState* st = k.st;
  const St3 S = st3_load(st, par);  // (replay: only done is used from it)
  const int done = S.done;
  __shared__ double sm[4 * NS];
  __shared__ int sflag;
  __shared__ WaveTV3 tvs[kWPB];
  __shared__ Pend3 pend;
  __shared__ Scal3 scl;
  const int lane = int(threadIdx.x & 63);
  const int wid = __builtin_amdgcn_readfirstlane(int(threadIdx.x >> 6));
  constexpr bool replay = MODE == kReplay;
  if constexpr (MODE == kStamp) {  // wave entry; the previous launch's finalize time (grid stamp 2 → 0)
    const unsigned long long t_in = rtc3();
    if (lane == 0) {
      k.stamps2[32 * (int64_t(blockIdx.x) * kWPB + wid) + 1] = t_in;
      // where the wave runs: HW_ID (wave slot, SIMD, CU, SE) | XCC_ID << 32
      const unsigned hw = __builtin_amdgcn_s_getreg(4 | (31 << 11)), xcc = __builtin_amdgcn_s_getreg(20 | (31 << 11));
      k.stamps2[32 * (int64_t(blockIdx.x) * kWPB + wid) + 30] = hw | (static_cast<unsigned long long>(xcc) << 32);
      k.stamps2[32 * (int64_t(blockIdx.x) * kWPB + wid) + 28] = __builtin_amdgcn_s_memtime();
      if (blockIdx.x == 0 && wid == 0) k.stamps2[-8] = k.stamps2[-6];
    }
  }
  if (done && !replay) return;
  // the first item's loads, before the state reads (PE_PRE=0 at construction: off)
  Pre3 pre;
  const bool use_pre = !replay && k.pre_load;
  if (use_pre) {
    pre_load3(k, int(blockIdx.x) * kWPB + wid, pre);
    stage_first3<PUSH>(k, par, tvs[wid], pre);
  } else {
    pre.staged = false;
  }
  // terminal paths: every wave has read the state before the last one to
  // arrive writes it
  auto finish = [&](int upto, long long iter, int status, int fixj = 0) {
    if (arrive_last_wave(&st->ticket[4], gridDim.x * kWPB) && lane == 0) {
      sweep3_stop(k, st, upto, iter, status, fixj);
      __hip_atomic_store(&st->ticket[4], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  };
  double acc[NS];
#pragma unroll
  for (int n = 0; n < NS; ++n) acc[n] = 0.0;
  // 1. the previous sweep's pending stop tests
  const int m0 = S.late3;
  const long long K = S.iter, K0 = K - m0;
  // (kStamp: prologue points into the wave's step-stamp slots 24-27 — state
  // read and the stop tests decided / scalars formed / walk entered)
  auto pstamp = [&](int slot, double dep) {
    if constexpr (MODE == kStamp) {
      if (lane == 0) {
        // (dep: a value of the phase — the empty asm needs it in a register
        // before the clock read, which stays after it: both volatile)
        asm volatile("" ::"v"(dep));
        k.stamps2[32 * (int64_t(blockIdx.x) * kWPB + wid) + slot] = rtc3();
      }
    }
  };
  const Late3 lt = late3_test(k, S);
  pstamp(24, double(lt.stop) + double(m0) + double(K));
  if (!replay && threadIdx.x == 0) pend3_load(k, S, m0, K0, pend);
  Coef3 cf;
  Scal3 sc = {};
  bool fix = false;
  int rpar = par;
  if constexpr (replay) {
    // After a fix-up (the solve stopped at iteration j of its last sweep):
    // march the last sweep's inputs again with its first j iterations and
    // identity steps after them (zc = 0, β = 1, α = 0), w untouched, storing
    // (r_j, p_j) into x[wpar] — the recurrence's r of the returned w.  No
    // sums, no state update.
    const int j = st->fixj;
    if (j == 0) return;
#pragma unroll
    for (int i = 0; i < 3; ++i) {
      cf.zc[i] = i < j ? st->sc3[i] : 0.0;
      cf.a[i] = i < j ? st->sc3[3 + i] : 0.0;
      cf.b[i] = i < j ? st->sc3[6 + i] : 1.0;
      cf.cw[i] = 0.0;
    }
    rpar = st->wpar;
  } else if (lt.stop) {
    if (!(lt.stop < m0 && lt.status == 1)) {
      finish(lt.stop, K0 + lt.stop, lt.status);
      return;
    }
    // converged before that sweep's last iteration: w holds the later
    // iterations' α_j p_j — march the same inputs with the same coefficients
    // again and subtract them (w only; one walk call site below: a second
    // inlined copy of the marches costs the whole register budget)
#pragma unroll
    for (int i = 0; i < 3; ++i) {
      cf.zc[i] = S.sc[i];
      cf.a[i] = S.sc[3 + i];
      cf.b[i] = S.sc[6 + i];
      cf.cw[i] = (i >= lt.stop && i < m0) ? -S.sc[3 + i] : 0.0;
    }
    fix = true;
    rpar = S.wpar;
  } else {
    // 2. the breakdown / cap that sweep saw coming
    if (S.brk3) {
      finish(m0, S.brk3, S.bad3 ? 4 : 2);
      return;
    }
    if (m0 > 0 && K >= k.max_iter) {
      finish(m0, K, 3);
      return;
    }
    if (k.mlimit < 0) {  // a resolve-only launch: record the pending iterations
      if (m0 > 0 && arrive_last_wave(&st->ticket[4], gridDim.x * kWPB) && lane == 0) {
        late3_record(k, st, m0);
        st->late3 = 0;
        __hip_atomic_store(&st->ticket[4], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
      return;
    }
    // 3. this sweep's iterations
    sc = sweep3_scalars(k, S, par);
    pstamp(25, sc.c.a[2] + sc.c.b[2] + sc.g[2]);
    if (sc.m == 0 && !sc.first) {  // iteration K+1 breaks down before its update
      finish(m0, K + 1, sc.bad ? 4 : 2);
      return;
    }
    cf = sc.c;
    if (threadIdx.x == 0) scl = sc;  // (the finalize's copy: sc need not live across the walk)
  }
  walk3<PUSH, MODE>(k, uni3(cf), fix, rpar, tvs[wid], wid, acc, pre, use_pre);
  if (k.prio > 0) __builtin_amdgcn_s_setprio(0);
  if (replay) return;
  if (fix) {
    finish(lt.stop, K0 + lt.stop, lt.status, lt.stop);
    return;
  }
  if (lane < HL3 || lane >= 64 - HR3)  // strip halo lanes: recomputed copies of the neighbouring strips' columns
#pragma unroll
    for (int n = 0; n < NS; ++n) acc[n] = 0.0;
  const unsigned long long t_red = MODE == kStamp ? rtc3() : 0ull;
  if (publish_last_nm<NS>(k.partial, acc, &st->ticket[0], &sflag, sm)) {
    if constexpr (MODE == kStamp) {
      if (threadIdx.x == 0) {
        k.stamps2[-7] = rtc3();  // the last block starts the grid's reduction
        k.stamps2[-3] = t_red;   // … its block reduction began
        k.stamps2[-2] = t_red;
      }
    }
    double t[NS];
    reduce_partials_nm<NS>(k.partial, t, sm);
    if constexpr (MODE == kStamp) {
      if (threadIdx.x == 0) k.stamps2[-5] = rtc3();  // the 512 partials summed
    }
    __shared__ double xv[NS + 1];
    __shared__ unsigned long long sseq;
    __shared__ int sok;
    if (k.xr.peers) {  // cross-rank sum of the 19 sums inside the sweep (P2P transport)
      if (threadIdx.x == 0) {
#pragma unroll
        for (int n = 0; n < NS; ++n) xv[n] = t[n];
        if (k.slow_ticks > 0) {  // PE_FAULT_INJECT=slow@rank (test hook): idle before the cross-rank sum
          const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
          while ((long long)(__builtin_amdgcn_s_memrealtime() - t0) < k.slow_ticks) __builtin_amdgcn_s_sleep(2);
        }
      }
      peer_sum_block(k.xr, xv, NS, &sseq, &sok);
      if (threadIdx.x == 0)
#pragma unroll
        for (int n = 0; n < NS; ++n) t[n] = xv[n];
    }
    if (threadIdx.x == 0) {
      if constexpr (MODE == kStamp) k.stamps2[-4] = rtc3();  // (after the cross-rank sum, if any)
      sweep3_finalize(k, st, par, scl, t, pend);
      __hip_atomic_store(&st->ticket[0], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if constexpr (MODE == kStamp) k.stamps2[-6] = rtc3();  // finalized
    }
  }
}

}  // namespace

void launch_S3(const KParams& k, int par, hipStream_t s) {
  const dim3 g(unsigned(k.nblocks)), b(TJ);
  if (k.mlimit == kReplay3) {
    if (k.push) hipLaunchKernelGGL((kS3<true, kReplay>), g, b, 0, s, k, par);
    else hipLaunchKernelGGL((kS3<false, kReplay>), g, b, 0, s, k, par);
  } else if (k.stamps && !k.push) {
    hipLaunchKernelGGL((kS3<false, kStamp>), g, b, 0, s, k, par);
  } else if (k.lnb[0] > 0 && !k.push) {
    hipLaunchKernelGGL((kS3<false, kSignal>), g, b, 0, s, k, par);
  } else if (k.push) {
    hipLaunchKernelGGL((kS3<true, kPlain>), g, b, 0, s, k, par);
  } else {
    hipLaunchKernelGGL((kS3<false, kPlain>), g, b, 0, s, k, par);
  }
}

int resident_blocks_S3() {
  int n = 0;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, kS3<false>, TJ, 0) != hipSuccess) {
    (void)hipGetLastError();
    n = 0;
  }
  return n;
}

}  // namespace dev
}  // namespace pe
