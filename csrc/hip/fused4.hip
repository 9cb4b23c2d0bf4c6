// Four-step single sweep: FOUR Jacobi-PCG iterations per pass over memory.
//
// fused3.hip's moment form one step further (s = 4).  With M = D⁻¹A, every
// scalar of iterations K+1..K+4 is a quadratic form in the D-moments
//   μ_n(x, y) = (x, D Mⁿ y),  n = 0..7,  x, y ∈ {z = D⁻¹r_K, p = p_K}
// (tools/sstep_proto.py 4: every golden iteration count 40²..8192², scalars
// within 1.1e-11 of the directly computed α / β, recurrence gap 2.2e-10 at
// 8192² — profiles/r5_sstep4.txt).  The sweep forms them as single dot
// products of the vectors its pipeline makes anyway:
//   q = Az, u₁ = D⁻¹q, v₁ = D⁻¹s (s = Ap₄ of the last iteration), then
//   Au_j, Av_j, u_{j+1} = D⁻¹Au_j, v_{j+1} = D⁻¹Av_j (j = 1, 2), Au₃, Av₃:
//   zz: (r,z) (z,q) (q,u₁) (u₁,Au₁) (Au₁,u₂) (u₂,Au₂) (Au₂,u₃) (u₃,Au₃)  sums 0..7
//   zp:       (z,s) (q,v₁) (u₁,Av₁) (Au₁,v₂) (u₂,Av₂) (Au₂,v₃) (u₃,Av₃)  sums 8..14
//   pp:       (p,s) (s,v₁) (v₁,Av₁) (Av₁,v₂) (v₂,Av₂) (Av₂,v₃) (v₃,Av₃)  sums 15..21
//   ‖p_i‖², i = 1..4 (the late stop tests, as in fused3.hip)         sums 22..25
// Traffic: r, p, w in and out once per FOUR iterations — 12 B per node per
// iteration against 16 (three-step) — and one 26-sum reduction per sweep.
// The price: a nine-stage pipeline (10 operator applications per node per
// sweep, 2.5 per iteration against 2.67), an 8-deep halo (16 pipeline-fill
// rows per item), and registers (the rings below).
//
// Machine mapping: fused3.hip's (one column per lane, 64-column strips that
// output lanes 8..55 — the 8 halo lanes per side are exactly the dependence
// radius here — aligned to 128-B lines; register rings of period 2 / 3 with a
// 6-step unroll; band items evaluate a row's face coefficients and 1/D once,
// into a 9-row LDS ring).  The stages of row step t (S = 4):
//   A  row t    p₁ = zc₁D⁻¹r + β₁p
//   B  row t−1  s₁ = Ap₁, r₁, p₂, w-partial α₁p₁        ‖p₁‖²
//   C  row t−2  s₂ = Ap₂, r₂, p₃                         ‖p₂‖²
//   D  row t−3  s₃ = Ap₃, r₃, p₄, w += … α₄p₄ stored      ‖p₃‖²
//   E  row t−4  s = Ap₄, r₄, z → r₄, p₄ stored            (r,z) (z,s) (p,s) ‖p₄‖²
//   F  row t−5  q = Az, u₁, v₁                            μ1 zz, μ2 zz / zp / pp
//   G  row t−6  Au₁, Av₁, u₂, v₂                          μ3, μ4
//   H  row t−7  Au₂, Av₂, u₃, v₃                          μ5, μ6
//   I  row t−8  Au₃, Av₃                                  μ7
// Everything is written for a general S (template parameter, S ≤ 4: the
// w-partial above covers p₁ only); kS4 instantiates S = 4.
//
// Registers (profiles/r5_sstep4.txt): the march needs 304-312 registers — at
// two waves per SIMD (256) it spilled 187-300 to scratch — so kS4 runs ONE
// wave per SIMD (amdgpu_waves_per_eu(1): 256 VGPRs + ~50 AGPRs, no scratch)
// and keeps more rows of r / p loads in flight per wave instead (kXD4 = 6:
// the bytes in flight of two waves of three).  Opt-in (PE_STEPS=4 /
// --algo four-step) until measured against the three-step sweep.
#include <cstdlib>
#include <type_traits>

#include "peer_sum.hpp"
#include "sstep.hpp"

#pragma clang fp contract(fast)

namespace pe {
namespace dev {

namespace {

template <int B, int E, class F>
__device__ __forceinline__ void sfor(F&& f) {
  if constexpr (B < E) {
    f(std::integral_constant<int, B>{});
    sfor<B + 1, E>(f);
  }
}

constexpr int r3s(int jj, int d) { return ((jj - d) % 3 + 3) % 3; }  // period-3 ring slot of row t-d
constexpr int r2s(int jj, int d) { return ((jj - d) % 2 + 2) % 2; }  // period-2 ring slot of row t-d

template <int S>
struct SP {
  static constexpr int H = 2 * S;          // dependence radius (rows and columns)
  static constexpr int NS = 7 * S - 2;     // sums per sweep
  static constexpr int RING = 2 * S + 1;   // band face ring: rows t-2S .. t
  static constexpr int zz(int n) { return n; }               // n = 0 .. 2S-1
  static constexpr int zp(int n) { return 2 * S + n - 1; }   // n = 1 .. 2S-1
  static constexpr int pp(int n) { return 4 * S - 1 + n - 1; }
  static constexpr int pn(int i) { return 6 * S - 2 + i - 1; }  // ‖p_i‖², i = 1 .. S
};
static_assert(SP<3>::NS == kNS3 && SP<3>::pn(1) == 16 && SP<3>::pp(1) == 11, "S = 3 sum layout = fused3.hip's");

constexpr int FSW4 = kFSW3;
constexpr int HL4 = kHL3, HR4 = 64 - kFSW3 - kHL3;
static_assert(HL4 >= SP<4>::H && HR4 >= SP<4>::H, "four-step strip: >= 8 halo lanes per side");
#ifndef PE_S4_XD
#define PE_S4_XD 6
#endif
constexpr int kXD4 = PE_S4_XD, kWD4 = 3;  // rows of r / p (w) loads in flight: divisors of the 6-step unroll
static_assert(6 % kXD4 == 0, "the r / p prefetch ring's period divides the 6-step unroll");

// Scalars of a sweep (iterations K+1 .. K+m).
template <int S>
struct CoefS {
  double zc[S], a[S], b[S], cw[S];
};

template <int S>
struct ScalS {
  bool first;
  long long K;
  int m, brk;
  bool bad;
  CoefS<S> c;
  double g[S];
};

// Σ_{a,b} x_a x_b μ_{a+b+sh} of x = Σ_a xz_a Mᵃz + xp_a Mᵃp.
template <int S>
__device__ __forceinline__ double mformS(const double (&xz)[S], const double (&xp)[S], const double (&mzz)[2 * S],
                                         const double (&mzp)[2 * S], const double (&mpp)[2 * S], int sh) {
  double s = 0.0;
#pragma unroll
  for (int a = 0; a < S; ++a)
#pragma unroll
    for (int b = 0; b < S; ++b) {
      const int n = a + b + sh;
      if (n < 2 * S) s += xz[a] * (xz[b] * mzz[n] + 2.0 * xp[b] * mzp[n]) + xp[a] * xp[b] * mpp[n];
    }
  return s;
}

// From the previous sweep's unweighted sums (a pure function of the state:
// every wave evaluates it and gets the same bits) — fused3.hip's
// sweep3_scalars for S iterations.
template <int S>
__device__ __forceinline__ ScalS<S> sweep_scalars(const KParams& k, const DevState* st, int par) {
  using P = SP<S>;
  ScalS<S> c;
  c.first = st->started == 0;
  c.K = st->iter;
  c.m = 0;
  c.brk = 0;
  c.bad = false;
#pragma unroll
  for (int i = 0; i < S; ++i) {
    c.c.zc[i] = 0.0;
    c.c.a[i] = 0.0;
    c.c.b[i] = 1.0;
    c.c.cw[i] = 0.0;
    c.g[i] = 0.0;
  }
  if (c.first) return c;
  const double hh = k.h1 * k.h2;
  const double* R = st->fs2[par ^ 1];
  double mzz[2 * S], mzp[2 * S], mpp[2 * S];
#pragma unroll
  for (int n = 0; n < 2 * S; ++n) {
    mzz[n] = R[P::zz(n)];
    mzp[n] = n ? R[P::zp(n)] : 0.0;
    mpp[n] = n ? R[P::pp(n)] : 0.0;
  }
  long long lim = k.max_iter - c.K;
  if (lim > S) lim = S;
  if (k.mlimit > 0 && lim > k.mlimit) lim = k.mlimit;
  double zz[S], zp[S], pz[S], pq[S];
#pragma unroll
  for (int q = 0; q < S; ++q) zz[q] = zp[q] = pz[q] = pq[q] = 0.0;
  zz[0] = 1.0;
  pq[0] = 1.0;
  double g = mformS<S>(zz, zp, mzz, mzp, mpp, 0) * hh;
  double gprev = st->gprev;
  bool live = true;
#pragma unroll
  for (int i = 0; i < S; ++i) {
    live = live && i < lim;
    const double beta = c.K + i == st->k0 ? 0.0 : g / gprev;
#pragma unroll
    for (int q = 0; q < S; ++q) {
      pz[q] = zz[q] + beta * pz[q];
      pq[q] = zp[q] + beta * pq[q];
    }
    const double den = mformS<S>(pz, pq, mzz, mzp, mpp, 1) * hh;
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
#pragma unroll
      for (int q = S - 1; q >= 1; --q) {  // z_i = z_{i-1} − α M p_i
        zz[q] -= alpha * pz[q - 1];
        zp[q] -= alpha * pq[q - 1];
      }
      g = mformS<S>(zz, zp, mzz, mzp, mpp, 0) * hh;
    }
  }
  return c;
}

// Late stop tests (fused3.hip: Late3): the pending iterations' ‖Δw‖ from the
// previous sweep's ‖p_i‖² and its α_i (sc3 = {zc[S], α[S], β[S], g[S]}).
struct LateS {
  int stop, status;
};

template <int S>
__device__ __forceinline__ double late_diffS(const KParams& k, const DevState* st, int i) {
  const double n2 = fmax(st->fs2[st->wpar][SP<S>::pn(1) + i], 0.0), a = st->sc3[S + i];
  return k.weighted ? fabs(a) * sqrt(n2 * (k.h1 * k.h2)) : fabs(a) * sqrt(n2);
}

template <int S>
__device__ __forceinline__ LateS late_testS(const KParams& k, const DevState* st) {
  LateS r{0, 0};
  const int m = st->late3;
#pragma unroll
  for (int i = 0; i < S; ++i) {
    if (r.stop == 0 && i < m) {
      const double d = late_diffS<S>(k, st, i);
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

template <int S>
__device__ __forceinline__ void late_recordS(const KParams& k, DevState* st, int n) {
  const long long K0 = st->iter - st->late3;
#pragma unroll
  for (int i = 0; i < S; ++i) {
    if (i < n) {
      const double d = late_diffS<S>(k, st, i);
      hist_put(k, K0 + i + 1, d);
      st->last_diff = d;
      st->alpha = st->sc3[S + i];
      st->beta = st->sc3[2 * S + i];
      st->rz_cur = st->sc3[3 * S + i];
    }
  }
}

template <int S>
__device__ __forceinline__ void sweep_stopS(const KParams& k, DevState* st, int upto, long long iter, int status,
                                            int fixj = 0) {
  late_recordS<S>(k, st, upto);
  st->fixj = fixj;
  st->iter = iter;
  st->status = status;
  st->late3 = 0;
  st->brk3 = 0;
  st->done = 1;
  st->wpend = 0;
}

template <int S>
__device__ __forceinline__ void sweep_finalizeS(const KParams& k, DevState* st, int par, const ScalS<S>& c,
                                                const double (&t)[SP<S>::NS]) {
  using P = SP<S>;
  if (!c.first) late_recordS<S>(k, st, st->late3);
#pragma unroll
  for (int n = 0; n < P::NS; ++n) st->fs2[par][n] = t[n];
  if (!c.first && k.fault_iter > c.K && k.fault_iter <= c.K + c.m) st->fs2[par][P::zz(1)] = __builtin_nan("");
  if (!c.first && k.fault_zero > c.K && k.fault_zero <= c.K + c.m)
    st->fs2[par][P::zz(1)] = st->fs2[par][P::zp(1)] = st->fs2[par][P::pp(1)] = 0.0;
  st->wpend = 0;
  st->wpar = par;
  if (c.first) {
    st->started = 1;
    return;
  }
#pragma unroll
  for (int i = 0; i < S; ++i) {
    st->sc3[i] = c.c.zc[i];
    st->sc3[S + i] = c.c.a[i];
    st->sc3[2 * S + i] = c.c.b[i];
    st->sc3[3 * S + i] = c.g[i];
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

enum { kMixed4 = 0, kBand4 = 1, kUniform4 = 2 };

template <int S>
struct MCtx {
  const double* Xm;
  double* Ym;
  double* Wm;
  const double* hrd;
  int64_t pitch, poff, wp;
  int J, c0, ib, ie, t0, tmax, nx, par;
  unsigned off;
  bool lv0, o0, fix, scol;
  double lf0, oih1, oih2, ih1, ih2, din, dout;
  int rlo, rhi;
  double zc[S], a[S], b[S], w[S];
};

template <int S>
struct MRings {
  double RQ[kXD4], PQ[kXD4], WQ[kWD4];
  double P[S][3];      // P[i] = p_{i+1}, rows t-i+1 .. t-i-1
  double R[S][2];      // R[0] = the input r, R[i] = r_i
  double WP[3];        // (S ≥ 4) w partial α₁p₁ of rows t-1 .. t-3
  double Z[3], Sv[2];  // z, s = Ap_S
  double U[S - 1][3], V[S - 1][3];  // U[j] = u_{j+1}
  bool pushed;
};

template <bool STEADY, class C>
__device__ __forceinline__ URow urowS(const C& c, const RowCtx& rx, int q) {
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

template <int S, bool PUSH>
__device__ __forceinline__ double ldxS(const KParams& k, const MCtx<S>& c, int t, unsigned o) {
  constexpr int H = SP<S>::H;
  if constexpr (PUSH) {
    if ((t < 1 && k.has[LEFT]) || (t > c.nx && k.has[RIGHT])) {
      const double* h = c.hrd + int64_t(t < 1 ? t + H - 1 : t - c.nx + H - 1) * c.pitch + o;
      return __hip_atomic_load(h, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    }
  }
  return c.Xm[int64_t(t) * c.pitch + o];
}

__device__ __forceinline__ double ldnt4(const double* p) { return __builtin_nontemporal_load(p); }
__device__ __forceinline__ void stnt4(double* p, double v) { __builtin_nontemporal_store(v, p); }

// rows 1..H → the LEFT neighbour's rows nx'+1..nx'+H; nx-H+1..nx → the RIGHT one's -H+1..0
template <int S>
__device__ __forceinline__ void push_rowS(const KParams& k, const MCtx<S>& c, MRings<S>& x, int q, double r, double p) {
  constexpr int H = SP<S>::H;
  auto put = [&](double* base, int slot) {
    double* d = base + int64_t(slot) * c.pitch + c.off;
    if (c.o0) {
      __hip_atomic_store(d, r, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      __hip_atomic_store(d + c.poff, p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    }
    x.pushed = true;
  };
  if (q <= H && k.hpush_lo[c.par] != nullptr) put(k.hpush_lo[c.par], q - 1);
  if (q >= c.nx - H + 1 && k.hpush_hi[c.par] != nullptr) put(k.hpush_hi[c.par], q - (c.nx - H + 1));
}

template <int S>
using WaveTVS = WaveTV1<SP<S>::RING>;

// One row step: stage A at row t = t0 + n, stage d at row t - d (d = 1 .. 2S).
template <int S, int KIND, bool PUSH, bool EDGE, bool STEADY, int JJ>
__device__ __forceinline__ void stepS(const KParams& k, const MCtx<S>& c, MRings<S>& x, const RowCtx& rx,
                                      WaveTVS<S>& tvw, double (&sv)[SP<S>::NS], int n, int bs) {
  using P = SP<S>;
  constexpr int RING = P::RING;
  constexpr bool BAND = KIND == kBand4, UNI = KIND == kUniform4;
  constexpr int XD = kXD4, WD = kWD4;
  constexpr int xs = JJ % XD, ws = JJ % WD;
  const int t = c.t0 + n;
  const int c0 = c.c0;
  auto inr = [&](int q) { return STEADY ? !c.fix : (q >= c.ib && q <= c.ie); };
  auto own = [&](int q) { return STEADY || (q >= c.ib && q <= c.ie); };
  auto put = [&](int i, double v) {
    if constexpr (UNI) sv[i] += v;
    else sv[i] += c.scol ? v : 0.0;
  };
  auto interior = [&](int q) { return q >= c.rlo && q <= c.rhi; };
  auto live = [&](int d) { return STEADY || n >= 2 * d; };
  int bsl[RING];
#pragma unroll
  for (int d = 0; d < RING; ++d) bsl[d] = bs >= d ? bs - d : bs - d + RING;
  auto zmask = [&](int q, double v, double d) -> double {
    if constexpr (UNI) {
      return EDGE ? (v * d) * c.lf0 : v * d;
    } else {
      return (interior(q) && c.lv0) ? v * d : 0.0;
    }
  };
  auto op = [&](int q, int sl, int sln, double um, double u0, double un, double& d) {
    if constexpr (UNI) {
      const URow r = urowS<STEADY>(c, rx, q);
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
    x.RQ[xs] = ldxS<S, PUSH>(k, c, tn, c.off);
    x.PQ[xs] = ldxS<S, PUSH>(k, c, tn, unsigned(c.poff) + c.off);
    const int wr = STEADY ? t - (S - 1) + WD : min(max(t - (S - 1) + WD, c.ib), c.ie);
    x.WQ[ws] = c.o0 ? ldnt4(c.Wm + int64_t(wr) * c.wp + c.off) : 0.0;
  }
  {
    double d;
    if constexpr (UNI) d = urowS<STEADY>(c, rx, t).d;
    else d = BAND ? enter_band1(k, rx, tvw, t, c0, bsl[0]) : dinv_plain1(k, rx, t, c0);
    const double z = zmask(t, rin, d);
    x.P[0][r3s(JJ, 0)] = c.zc[0] * z + c.b[0] * pin;
    x.R[0][r2s(JJ, 0)] = rin;
  }
  if (STEADY) __builtin_amdgcn_sched_barrier(0);
  // ---- stages 1 .. S-1: row t-d: s_d = A p_d, r_d, p_{d+1} (and w at S-1) ----
  sfor<1, S>([&](auto dc) {
    constexpr int d = decltype(dc)::value;
    if (live(d)) {
      const int q = t - d;
      double dq;
      const double sd = op(q, bsl[d], bsl[d - 1], x.P[d - 1][r3s(JJ, d + 1)], x.P[d - 1][r3s(JJ, d)],
                           x.P[d - 1][r3s(JJ, d - 1)], dq);
      const double rd = x.R[d - 1][r2s(JJ, d)] - c.a[d - 1] * sd;
      const double z = zmask(q, rd, dq);
      const double pd = x.P[d - 1][r3s(JJ, d)];
      x.R[d][r2s(JJ, d)] = rd;
      const double pn = c.zc[d] * z + c.b[d] * pd;
      x.P[d][r3s(JJ, d)] = pn;
      if constexpr (S >= 4 && d == 1) x.WP[r3s(JJ, 1)] = c.w[0] * pd;
      if constexpr (d == S - 1) {
        if (own(q) && c.o0) {
          double wv;
          if constexpr (S >= 4) {
            wv = wrow + x.WP[r3s(JJ, d)];
#pragma unroll
            for (int i = 1; i < S - 1; ++i) wv += c.w[i] * x.P[i][r3s(JJ, d)];
          } else {
            wv = wrow;
#pragma unroll
            for (int i = 0; i < S - 1; ++i) wv += c.w[i] * x.P[i][r3s(JJ, d)];
          }
          stnt4(c.Wm + int64_t(q) * c.wp + c.off, wv + c.w[S - 1] * pn);
        }
      }
      if (inr(q)) put(P::pn(d), pd * pd);
    }
    if (STEADY) __builtin_amdgcn_sched_barrier(0);
  });
  // ---- stage S: row t-S: s = A p_S, r_S, z = D⁻¹r_S → r_S, p_S stored ----
  if (live(S)) {
    const int q = t - S;
    double dq;
    const double s3 = op(q, bsl[S], bsl[S - 1], x.P[S - 1][r3s(JJ, S + 1)], x.P[S - 1][r3s(JJ, S)],
                         x.P[S - 1][r3s(JJ, S - 1)], dq);
    const double r3 = x.R[S - 1][r2s(JJ, S)] - c.a[S - 1] * s3;
    const double z = zmask(q, r3, dq);
    x.Z[r3s(JJ, S)] = z;
    x.Sv[r2s(JJ, S)] = s3;
    const double p3 = x.P[S - 1][r3s(JJ, S)];
    if (own(q) && !c.fix) {
      if (c.o0) {
        double* yr = c.Ym + int64_t(q) * c.pitch + c.off;
        stnt4(yr, r3);
        stnt4(yr + c.poff, p3);
      }
      if constexpr (PUSH) push_rowS<S>(k, c, x, q, r3, p3);
    }
    if (inr(q)) {
      put(P::zz(0), r3 * z);
      put(P::zp(1), z * s3);
      put(P::pp(1), p3 * s3);
      put(P::pn(S), p3 * p3);
    }
  }
  if (STEADY) __builtin_amdgcn_sched_barrier(0);
  // ---- stage S+1: row t-S-1: q = Az, u₁, v₁ ----
  if (live(S + 1)) {
    constexpr int d = S + 1;
    const int q = t - d;
    double dq;
    const double qv = op(q, bsl[d], bsl[d - 1], x.Z[r3s(JJ, d + 1)], x.Z[r3s(JJ, d)], x.Z[r3s(JJ, d - 1)], dq);
    const double sr = x.Sv[r2s(JJ, d)];
    const double u = zmask(q, qv, dq);
    const double v = zmask(q, sr, dq);
    x.U[0][r3s(JJ, d)] = u;
    x.V[0][r3s(JJ, d)] = v;
    if (inr(q)) {
      put(P::zz(1), x.Z[r3s(JJ, d)] * qv);
      put(P::zz(2), qv * u);
      put(P::zp(2), qv * v);
      put(P::pp(2), sr * v);
    }
  }
  if (STEADY) __builtin_amdgcn_sched_barrier(0);
  // ---- stages S+1+j (j = 1 .. S-2): Au_j, Av_j, u_{j+1}, v_{j+1} ----
  sfor<1, S - 1>([&](auto jc) {
    constexpr int j = decltype(jc)::value;
    constexpr int d = S + 1 + j;
    if (live(d)) {
      const int q = t - d;
      double dq, dq2;
      const double au = op(q, bsl[d], bsl[d - 1], x.U[j - 1][r3s(JJ, d + 1)], x.U[j - 1][r3s(JJ, d)],
                           x.U[j - 1][r3s(JJ, d - 1)], dq);
      const double av = op(q, bsl[d], bsl[d - 1], x.V[j - 1][r3s(JJ, d + 1)], x.V[j - 1][r3s(JJ, d)],
                           x.V[j - 1][r3s(JJ, d - 1)], dq2);
      const double uu = zmask(q, au, dq);
      const double vv = zmask(q, av, dq);
      x.U[j][r3s(JJ, d)] = uu;
      x.V[j][r3s(JJ, d)] = vv;
      if (inr(q)) {
        const double u = x.U[j - 1][r3s(JJ, d)], v = x.V[j - 1][r3s(JJ, d)];
        put(P::zz(2 * j + 1), u * au);
        put(P::zp(2 * j + 1), u * av);
        put(P::pp(2 * j + 1), v * av);
        put(P::zz(2 * j + 2), au * uu);
        put(P::zp(2 * j + 2), au * vv);
        put(P::pp(2 * j + 2), av * vv);
      }
    }
    if (STEADY) __builtin_amdgcn_sched_barrier(0);
  });
  // ---- stage 2S: row t-2S: Au_{S-1}, Av_{S-1} ----
  {
    constexpr int d = 2 * S;
    const int q = t - d;
    if (inr(q)) {
      double dq;
      const double auu = op(q, bsl[d], bsl[d - 1], x.U[S - 2][r3s(JJ, d + 1)], x.U[S - 2][r3s(JJ, d)],
                            x.U[S - 2][r3s(JJ, d - 1)], dq);
      const double avv = op(q, bsl[d], bsl[d - 1], x.V[S - 2][r3s(JJ, d + 1)], x.V[S - 2][r3s(JJ, d)],
                            x.V[S - 2][r3s(JJ, d - 1)], dq);
      const double uu = x.U[S - 2][r3s(JJ, d)], vv = x.V[S - 2][r3s(JJ, d)];
      put(P::zz(2 * S - 1), uu * auu);
      put(P::zp(2 * S - 1), uu * avv);
      put(P::pp(2 * S - 1), vv * avv);
    }
  }
}

template <int S, int KIND, bool PUSH, bool EDGE, bool STEADY>
__device__ __forceinline__ void groupS(const KParams& k, const MCtx<S>& c, MRings<S>& x, const RowCtx& rx,
                                       WaveTVS<S>& tvw, double (&sv)[SP<S>::NS], int n0, int nsteps, int& bs) {
  constexpr int RING = SP<S>::RING;
  auto adv = [&]() { bs = bs == RING - 1 ? 0 : bs + 1; };
#define PE_STEPS4(JJ)                                                            \
  if (STEADY || n0 + JJ < nsteps) {                                              \
    stepS<S, KIND, PUSH, EDGE, STEADY, JJ>(k, c, x, rx, tvw, sv, n0 + JJ, bs);   \
    adv();                                                                       \
    if (STEADY) __builtin_amdgcn_sched_barrier(0);                               \
  }
  PE_STEPS4(0)
  PE_STEPS4(1)
  PE_STEPS4(2)
  PE_STEPS4(3)
  PE_STEPS4(4)
  PE_STEPS4(5)
#undef PE_STEPS4
}

__device__ __forceinline__ unsigned long long rtc4() {
  unsigned long long t;
  asm volatile("s_memrealtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t)::"memory");
  return t;
}

// The item march (one strip × rows ib..ie): fused3.hip's march3 for S steps.
template <int S, int KIND, bool PUSH, bool EDGE, bool SST = false>
__device__ __forceinline__ void marchS(const KParams& k, const CoefS<S>& cf, bool fix, int par, int s, int ib, int ie,
                                       WaveTVS<S>& tvw, double (&sv)[SP<S>::NS], unsigned long long* sst = nullptr) {
  using P = SP<S>;
  constexpr int H = P::H;
  const int lane = threadIdx.x & 63;
  const int ny = int(k.ny);
  MCtx<S> c;
  c.pitch = k.pitch;
  c.poff = k.poff;
  c.wp = k.wpitch;
  c.Xm = k.x[par ^ 1] - (HL4 - 1);
  c.Ym = k.x[par] - (HL4 - 1);
  c.Wm = k.w - (HL4 - 1);
  c.J = -(HL4 - 1) + s * FSW4;
  c.c0 = c.J + lane;
  c.off = unsigned(c.c0 + HL4 - 1);
  const int64_t g0 = k.gj0 + c.c0;
  c.lv0 = c.c0 <= ny + H && g0 >= 1 && g0 <= k.N - 1;
  c.lf0 = c.lv0 ? 1.0 : 0.0;
  c.o0 = lane >= HL4 && lane < 64 - HR4 && c.c0 >= 1 && c.c0 <= ny;
  c.scol = c.c0 <= ny;
  c.fix = fix;
  c.ib = ib;
  c.ie = ie;
  c.t0 = ib - H;
  c.tmax = ie + H;
  c.nx = int(k.nx);
  c.par = par;
  c.hrd = PUSH ? k.hrecv + int64_t(par ^ 1) * 2 * H * k.pitch : nullptr;
  c.oih1 = uni(k.inv_eps * k.ih1sq);
  c.oih2 = uni(k.inv_eps * k.ih2sq);
  c.ih1 = k.ih1sq;
  c.ih2 = k.ih2sq;
  c.din = k.dinv_in;
  c.dout = k.dinv_out;
  c.rlo = int(max<int64_t>(1 - k.gi0, -(1 << 30)));
  c.rhi = int(min<int64_t>(k.M - 1 - k.gi0, 1 << 30));
#pragma unroll
  for (int i = 0; i < S; ++i) {
    c.zc[i] = cf.zc[i];
    c.a[i] = cf.a[i];
    c.b[i] = cf.b[i];
    c.w[i] = cf.cw[i];
  }
  RowCtx rx;
  auto load_seg = [&](int base) { load_rows<KIND == kBand4, WaveTVS<S>, 64>(k, rx, tvw, base, ie + H + 1, c.J); };
  if (KIND == kBand4) load_strip_tables1(k, tvw, c.c0);
  load_seg(c.t0);

  MRings<S> x;
  x.pushed = false;
  constexpr int XD = kXD4, WD = kWD4;
#pragma unroll
  for (int q = 0; q < XD; ++q) {
    const int t = min(c.t0 + q, c.tmax);
    x.RQ[q] = ldxS<S, PUSH>(k, c, t, c.off);
    x.PQ[q] = ldxS<S, PUSH>(k, c, t, unsigned(c.poff) + c.off);
  }
#pragma unroll
  for (int q = 0; q < WD; ++q)
    x.WQ[q] = c.o0 ? ldnt4(c.Wm + int64_t(min(max(c.t0 - (S - 1) + q, ib), ie)) * c.wp + c.off) : 0.0;
#pragma unroll
  for (int q = 0; q < 3; ++q) {
    x.Z[q] = x.WP[q] = 0.0;
#pragma unroll
    for (int i = 0; i < S; ++i) x.P[i][q] = 0.0;
#pragma unroll
    for (int j = 0; j < S - 1; ++j) x.U[j][q] = x.V[j][q] = 0.0;
  }
#pragma unroll
  for (int q = 0; q < 2; ++q) {
    x.Sv[q] = 0.0;
#pragma unroll
    for (int i = 0; i < S; ++i) x.R[i][q] = 0.0;
  }

  const int nsteps = ie + H - c.t0 + 1;
  const int rows = ie - ib + 1;
  int bs = 0;
  int sg = 3;
  if constexpr (SST) {
    if (sst && lane == 0) sst[2] = rtc4();
  }
  auto sstamp = [&]() {
    if constexpr (SST) {
      if (sst && lane == 0 && sg < 31) sst[sg] = rtc4();
      ++sg;
    }
  };
  auto reload = [&](int n0) {
    if (c.t0 + n0 + 6 - rx.segbase > 63) load_seg(c.t0 + n0 - H);
  };
  // steady groups (uniform items, straight-line code): every stage row of
  // all six steps inside the item — n ≥ 2H = 4S — and below
  int n0 = 0;
  const int fill = 2 * H;
  // (every stage row t .. t-2S inside the item: n ≤ rows - 1 + 2S; the w row
  // prefetched, t - (S-1) + WD ≤ ie: n ≤ rows + 3S - 5 — fused3.hip: rows + 4)
  const int nsteady_end = KIND == kUniform4 ? min(rows - 1 + 2 * S, rows + 3 * S - 5) - 5 : -1;
  for (; n0 < nsteps && !(n0 >= fill && n0 <= nsteady_end); n0 += 6) {
    reload(n0);
    groupS<S, KIND, PUSH, EDGE, false>(k, c, x, rx, tvw, sv, n0, nsteps, bs);
    sstamp();
  }
  if constexpr (KIND == kUniform4) {
    for (; n0 <= nsteady_end; n0 += 6) {
      reload(n0);
      groupS<S, KIND, PUSH, EDGE, true>(k, c, x, rx, tvw, sv, n0, nsteps, bs);
      sstamp();
    }
    for (; n0 < nsteps; n0 += 6) {
      reload(n0);
      groupS<S, KIND, PUSH, EDGE, false>(k, c, x, rx, tvw, sv, n0, nsteps, bs);
      sstamp();
    }
  }
  if constexpr (PUSH) {
    if (x.pushed) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // (system-scope atomic stores: fused3.hip march3)
  }
}

template <int S>
__device__ __forceinline__ CoefS<S> uniS(const CoefS<S>& c) {
  CoefS<S> u;
#pragma unroll
  for (int i = 0; i < S; ++i) {
    u.zc[i] = uni(c.zc[i]);
    u.a[i] = uni(c.a[i]);
    u.b[i] = uni(c.b[i]);
    u.cw[i] = uni(c.cw[i]);
  }
  return u;
}

enum { kPlain4 = 0, kStamp4 = 1, kReplay4 = 2, kSignal4 = 3 };

template <int S, bool PUSH, int MODE>
__device__ __forceinline__ void walkS(const KParams& k, const CoefS<S>& cf, bool fix, int par, WaveTVS<S>& tv, int wid,
                                      double (&acc)[SP<S>::NS]) {
  constexpr int H = SP<S>::H;
  constexpr bool STAMP = MODE == kStamp4;
  const int W = k.lwaves;
  const int gwave = int(blockIdx.x) * kWPB + wid;
  const bool l0 = (threadIdx.x & 63) == 0;
  if constexpr (STAMP) {
    if (l0) k.stamps[4 * int64_t(k.nslots) + 2 * gwave] = rtc4();
  }
  const int pend = gwave < W ? k.nslots : 0;
  unsigned long long* sst = STAMP ? k.stamps2 + 32 * int64_t(gwave) : nullptr;
  for (int pos = gwave; pos < pend; pos += W) {
    const int2 e = cload_i2(k.ilist + pos);
    const int rows = e.y >> 20;
    if (rows == 0) continue;
    const int s = e.y & 0xFFFFF, ib = e.x & kRowMask3;
    const int ie = min(ib + rows - 1, int(k.nx));
    const unsigned long long t_item = STAMP ? rtc4() : 0ull;
    if constexpr (STAMP) {
      if (sst && l0) sst[0] = t_item;
    }
    if (e.x & kBandBit) {
      marchS<S, kBand4, PUSH, true, STAMP>(k, cf, fix, par, s, ib, ie, tv, acc, sst);
    } else if (e.x & kUniBit) {
      const int c0 = -(HL4 - 1) + s * FSW4 + int(threadIdx.x & 63);
      const int64_t g0 = k.gj0 + c0;
      const bool lv = c0 <= int(k.ny) + H && g0 >= 1 && g0 <= k.N - 1;
      if (__ballot(lv) == ~0ull) marchS<S, kUniform4, PUSH, false, STAMP>(k, cf, fix, par, s, ib, ie, tv, acc, sst);
      else marchS<S, kUniform4, PUSH, true, STAMP>(k, cf, fix, par, s, ib, ie, tv, acc, sst);
    } else {
      marchS<S, kMixed4, PUSH, true, STAMP>(k, cf, fix, par, s, ib, ie, tv, acc, sst);
    }
    if constexpr (STAMP) {
      if (sst && l0) sst[31] = rtc4();
      sst = nullptr;
    }
    if constexpr (MODE == kSignal4) {
      if (pos < k.lnb[0]) {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        if (l0) __hip_atomic_fetch_add(&k.st->sig, 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
    }
    if constexpr (STAMP) {
      if (l0) {
        const unsigned long long kind = (e.x & kBandBit) ? 1ull : (e.x & kUniBit) ? 2ull : 0ull;
        unsigned long long* d = k.stamps + 4 * int64_t(pos);
        d[0] = t_item;
        d[1] = rtc4();
        d[2] = (unsigned long long)gwave | ((unsigned long long)s << 32);
        d[3] = (unsigned long long)ib | ((unsigned long long)(ie - ib + 1) << 32) | (kind << 48);
      }
    }
  }
  if constexpr (STAMP) {
    if (l0) k.stamps[4 * int64_t(k.nslots) + 2 * gwave + 1] = rtc4();
  }
}

// fused3.hip's kS3 for S iterations per launch (same launch protocol: the
// previous launch's late stop tests, its fix-up, breakdown / cap, then this
// sweep; the replay launch; the overlap's boundary signal).
template <int S, bool PUSH, int MODE = kPlain4>
__global__ __launch_bounds__(TJ) __attribute__((amdgpu_waves_per_eu(1))) void kSS(KParams k, int par) {
  using P = SP<S>;
  constexpr int NS = P::NS;
  constexpr int RING = P::RING;
  DevState* st = k.st;
  const int lane = int(threadIdx.x & 63);
  const int wid = __builtin_amdgcn_readfirstlane(int(threadIdx.x >> 6));
  constexpr bool replay = MODE == kReplay4;
  if constexpr (MODE == kStamp4) {
    const unsigned long long t_in = rtc4();
    if (lane == 0) {
      k.stamps2[32 * (int64_t(blockIdx.x) * kWPB + wid) + 1] = t_in;
      if (blockIdx.x == 0 && wid == 0) k.stamps2[-8] = k.stamps2[-6];
    }
  }
  const int done = st->done;
  __shared__ double sm[4 * NS];
  __shared__ int sflag;
  __shared__ WaveTVS<S> tvs[kWPB];
  if (done && !replay) return;
  auto zero_ring = [&]() {
    WaveTVS<S>& tv = tvs[wid];
    for (int i = lane; i < RING * 64; i += 64) (&tv.a0r[0][0])[i] = 0.0;
    for (int i = lane; i < RING * 66; i += 64) (&tv.b0r[0][0])[i] = 0.0;
    for (int i = lane; i < RING * 64; i += 64) (&tv.d0r[0][0])[i] = 0.0;
  };
  auto finish = [&](int upto, long long iter, int status, int fixj = 0) {
    if (arrive_last_wave(&st->ticket[4], gridDim.x * kWPB) && lane == 0) {
      sweep_stopS<S>(k, st, upto, iter, status, fixj);
      __hip_atomic_store(&st->ticket[4], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  };
  double acc[NS];
#pragma unroll
  for (int n = 0; n < NS; ++n) acc[n] = 0.0;
  const int m0 = st->late3;
  const long long K = st->iter, K0 = K - m0;
  const LateS lt = late_testS<S>(k, st);
  CoefS<S> cf;
  ScalS<S> sc = {};
  bool fix = false;
  int rpar = par;
  if constexpr (replay) {
    const int j = st->fixj;
    if (j == 0) return;
#pragma unroll
    for (int i = 0; i < S; ++i) {
      cf.zc[i] = i < j ? st->sc3[i] : 0.0;
      cf.a[i] = i < j ? st->sc3[S + i] : 0.0;
      cf.b[i] = i < j ? st->sc3[2 * S + i] : 1.0;
      cf.cw[i] = 0.0;
    }
    rpar = st->wpar;
  } else if (lt.stop) {
    if (!(lt.stop < m0 && lt.status == 1)) {
      finish(lt.stop, K0 + lt.stop, lt.status);
      return;
    }
#pragma unroll
    for (int i = 0; i < S; ++i) {
      cf.zc[i] = st->sc3[i];
      cf.a[i] = st->sc3[S + i];
      cf.b[i] = st->sc3[2 * S + i];
      cf.cw[i] = (i >= lt.stop && i < m0) ? -st->sc3[S + i] : 0.0;
    }
    fix = true;
    rpar = st->wpar;
  } else {
    if (st->brk3) {
      finish(m0, st->brk3, st->bad3 ? 4 : 2);
      return;
    }
    if (m0 > 0 && K >= k.max_iter) {
      finish(m0, K, 3);
      return;
    }
    if (k.mlimit < 0) {
      if (m0 > 0 && arrive_last_wave(&st->ticket[4], gridDim.x * kWPB) && lane == 0) {
        late_recordS<S>(k, st, m0);
        st->late3 = 0;
        __hip_atomic_store(&st->ticket[4], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
      return;
    }
    sc = sweep_scalars<S>(k, st, par);
    if (sc.m == 0 && !sc.first) {
      finish(m0, K + 1, sc.bad ? 4 : 2);
      return;
    }
    cf = sc.c;
  }
  zero_ring();
  walkS<S, PUSH, MODE>(k, uniS<S>(cf), fix, rpar, tvs[wid], wid, acc);
  if (replay) return;
  if (fix) {
    finish(lt.stop, K0 + lt.stop, lt.status, lt.stop);
    return;
  }
  if (lane < HL4 || lane >= 64 - HR4)
#pragma unroll
    for (int n = 0; n < NS; ++n) acc[n] = 0.0;
  if (publish_last_nm<NS>(k.partial, acc, &st->ticket[0], &sflag, sm)) {  // (kcommon.hpp: n-major partials)
    if constexpr (MODE == kStamp4) {
      if (threadIdx.x == 0) k.stamps2[-7] = rtc4();
    }
    double t[NS];
    reduce_partials_nm<NS>(k.partial, t, sm);
    __shared__ double xv[NS + 1];
    __shared__ unsigned long long sseq;
    __shared__ int sok;
    if (k.xr.peers) {
      if (threadIdx.x == 0) {
#pragma unroll
        for (int n = 0; n < NS; ++n) xv[n] = t[n];
        if (k.slow_ticks > 0) {
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
      sweep_finalizeS<S>(k, st, par, sc, t);
      __hip_atomic_store(&st->ticket[0], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if constexpr (MODE == kStamp4) k.stamps2[-6] = rtc4();
    }
  }
}

}  // namespace

void launch_S4(const KParams& k, int par, hipStream_t s) {
  const dim3 g(unsigned(k.nblocks)), b(TJ);
  if (k.mlimit == kReplay3) {
    if (k.push) hipLaunchKernelGGL((kSS<4, true, kReplay4>), g, b, 0, s, k, par);
    else hipLaunchKernelGGL((kSS<4, false, kReplay4>), g, b, 0, s, k, par);
  } else if (k.stamps && !k.push) {
    hipLaunchKernelGGL((kSS<4, false, kStamp4>), g, b, 0, s, k, par);
  } else if (k.lnb[0] > 0 && !k.push) {
    hipLaunchKernelGGL((kSS<4, false, kSignal4>), g, b, 0, s, k, par);
  } else if (k.push) {
    hipLaunchKernelGGL((kSS<4, true, kPlain4>), g, b, 0, s, k, par);
  } else {
    hipLaunchKernelGGL((kSS<4, false, kPlain4>), g, b, 0, s, k, par);
  }
}

int resident_blocks_S4() {
  int n = 0;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, kSS<4, false>, TJ, 0) != hipSuccess) {
    (void)hipGetLastError();
    n = 0;
  }
  return n;
}

}  // namespace dev
}  // namespace pe
