// Single-sweep Jacobi-PCG for gfx950: ONE marching kernel and ONE global
// reduction per iteration.
//
// The reference iteration (poisson_mpi_cuda2.cu:846-942) needs two global
// reductions — (Ap,p) before α, (z,r) before β — so any implementation of it
// needs two passes over memory per iteration (the classic path here, kF+kG in
// kernels.hip, moves 8 fp64 arrays per point).  This file reorganises the
// same Krylov recurrence so that every dot product of iteration k+1 is a
// combination of dot products computable in ONE sweep over iteration k's data
// (a single-reduction CG in the spirit of Chronopoulos–Gear, but with the
// exact expansion instead of the s-recurrence, so no extra vector is kept):
//
//   p_k = z_{k-1} + β_k p_{k-1}             z = D⁻¹r
//   s_k = A p_k                              (recomputed, never stored)
//   (p_k, A p_k) = (z,Az) + 2β (z,s_{k-1}) + β² (p_{k-1},s_{k-1})
//   ‖p_k‖²        = (z,z)  + 2β (z,p_{k-1}) + β² (p_{k-1},p_{k-1})
//   α_k = (r,z)/(p_k,Ap_k),   ‖w_{k+1}-w_k‖ = |α_k| ‖p_k‖      (stop test)
//   w += α p_k,   r_k = r_{k-1} - α s_k,   z_k = D⁻¹ r_k,   q_k = A z_k
//   sums of sweep k: (r,z) (z,q) (z,s) (p,s) (z,z) (z,p) (p,p)
//
// so a sweep reads r_{k-1}, p_{k-1}, w and writes r_k, p_k, w: 6 array passes
// per point (48 B) instead of 8, and 1 reduction instead of 2 (half the
// latency-bound allreduces on multiple GPUs).  The price is a radius-2
// dependence (q needs z at ±1, z needs s at ±1, s needs p at ±1), handled by
// a 2-deep halo and by recomputation: each wave64 strip loads 128 columns but
// outputs the middle 124 (lanes 1..62), so every j-neighbour comes from a DPP
// lane shift and no strip-edge prologue is needed; rows march with the
// i-neighbours in registers and the next two rows' loads in flight.  The
// numpy prototype of this recurrence reproduces the reference's iteration
// counts exactly (tests/test_gpu.py checks the golden counts on the device).
//
// Layout: buffer x[b] interleaves the r- and p-planes by row (row stride
// `pitch` = 2 × plane width), so the two halo rows of both fields that an
// x-neighbour needs are ONE contiguous message.  Local rows -1..nx+2 and
// columns -1..ny+2 hold data (halo depth 2); everything a kernel reads past
// that is zero padding, and non-interior nodes are masked to z = 0.
#include <cstdlib>

#include "kcommon.hpp"
#include "peer_sum.hpp"

// The single-sweep formulation does not reproduce the reference rounding
// anyway: let the compiler contract a*b+c into v_fma_f64.
#pragma clang fp contract(fast)


namespace pe {
namespace dev {

namespace {

constexpr int FSW = kFSW;

__device__ __forceinline__ double2 dd(double a, double b) { return make_double2(a, b); }
// Item-list entry through the constant (scalar) path: one s_load_dwordx2.
__device__ __forceinline__ int2 cload_i2(const int2* p) {
  const long long v = cload(reinterpret_cast<const long long*>(p));
  return make_int2(int(v), int(v >> 32));
}

// Per-wave LDS copy of the strip's row-table entries (boundary-band rows
// only read them; LDS reads are counted by lgkmcnt, so they never drain
// the vector-memory prefetch queue).
struct WaveTV {
  double sA[128], eA[128], hB[130];
};

// Per-wave LDS ring of boundary-band coefficients.  A band row's face
// coefficients and 1/D (chord lengths, four face fits and a division per
// node) are evaluated ONCE, when the row enters the pipeline at the p_k
// stage, and re-read by the s = A p and q = A z stages of the next two row
// steps.  Evaluating them at each of the three stages made a band item cost
// ≈3.4× a plain one (800×1200: 31 vs 9 µs; the band items were the sweep's
// critical path, profiles/r2_small_before.txt).  Each lane reads back only
// its own two columns: no cross-lane synchronisation.
// [slot][field a0 a1 b0 b1 d][lane], one (column c0, c0+1) pair per entry.
struct BandRing {
  double2 v[3][5][64];
};
__device__ __forceinline__ void ring_put(BandRing& r, int slot, int lane, const CS& x0, const CS& x1) {
  r.v[slot][0][lane] = make_double2(x0.a0, x1.a0);
  r.v[slot][1][lane] = make_double2(x0.a1, x1.a1);
  r.v[slot][2][lane] = make_double2(x0.b0, x1.b0);
  r.v[slot][3][lane] = make_double2(x0.b1, x1.b1);
  r.v[slot][4][lane] = make_double2(x0.d, x1.d);
}
__device__ __forceinline__ void ring_get(const BandRing& r, int slot, int lane, CS& x0, CS& x1) {
  const double2 a0 = r.v[slot][0][lane], a1 = r.v[slot][1][lane], b0 = r.v[slot][2][lane], b1 = r.v[slot][3][lane],
                d = r.v[slot][4][lane];
  x0 = CS{a0.x, a1.x, b0.x, b1.x, d.x};
  x1 = CS{a0.y, a1.y, b0.y, b1.y, d.y};
}

// Row descriptor carried through the 3-row pipeline: lane-resident interior
// flags of the lane's two columns, and whether the strip has a boundary-band
// node in this row (uniform).
struct RowI {
  bool in0, in1, gen;
  int t;  // local row
};

// Select-only coefficients of a band-free row: f = 1 inside, 1/eps outside;
// d = 1/D accordingly.
__device__ __forceinline__ double fsel(const KParams& k, bool in) { return in ? 1.0 : k.inv_eps; }
__device__ __forceinline__ double dsel(const KParams& k, bool in) { return in ? k.dinv_in : k.dinv_out; }
__device__ __forceinline__ double lapf(const KParams& k, double f, double pm, double p0, double pn, double pl,
                                       double pr) {
  return f * (((p0 - pm) - (pn - p0)) * k.ih1sq + ((p0 - pl) - (pr - p0)) * k.ih2sq);
}
__device__ __forceinline__ CS cs_gen(const KParams& k, const RowCls& rc, const CT& ct, int lj, const WaveTV& tv, int jl) {
  const TV t{tv.sA[jl], tv.eA[jl], tv.hB[jl], tv.hB[jl + 1]};
  return cset_rc(k, rc, ct, lj, t);
}

typedef double v2d __attribute__((ext_vector_type(2)));
template <bool NT>
__device__ __forceinline__ void st2(double* p, double2 v) {
  if constexpr (NT) __builtin_nontemporal_store(v2d{v.x, v.y}, reinterpret_cast<v2d*>(p));
  else *reinterpret_cast<double2*>(p) = v;
}
template <bool NT>
__device__ __forceinline__ double2 ldw(const double* p) {
  if constexpr (NT) {
    const v2d t = __builtin_nontemporal_load(reinterpret_cast<const v2d*>(p));
    return make_double2(t.x, t.y);
  } else {
    return *reinterpret_cast<const double2*>(p);
  }
}

// Pointwise w += a1·p_{k-1} + a2·p_k over the owned nodes (rare paths:
// convergence / iteration cap in a deferring sweep, breakdown, host flush).
// p_k = zc·D⁻¹r_{k-1} + β p_{k-1} from the input buffer xin.
// (1/D from the march's own division-free coefficient path, cset_rc, so p_k
// has the bits the sweep would have produced.)
__device__ void w_pointwise(const KParams& k, const double* xin, double a1, double a2, double zc, double beta) {
  const int64_t n = k.nx * k.ny;
  for (int64_t idx = int64_t(blockIdx.x) * blockDim.x + threadIdx.x; idx < n; idx += int64_t(gridDim.x) * blockDim.x) {
    const int64_t li = idx / k.ny + 1, lj = idx % k.ny + 1;
    const double r = xin[li * k.pitch + lj], pold = xin[li * k.pitch + k.poff + lj];
    const int* rc = k.rowcls + (li + 1) * 4;
    const double* ctr = k.colT + (li + 1) * 4;
    const double* tv = k.rowT + (lj + 1) * 4;
    const double d = cset_rc(k, RowCls{rc[0], rc[1], rc[2], rc[3]}, CT{ctr[0], ctr[4], ctr[1], ctr[2]}, lj,
                             TV{tv[0], tv[1], tv[2], tv[6]}).d;
    const double pk = zc * (r * d) + beta * pold;
    double& w = k.w[li * k.wpitch + lj];
    w = w + a1 * pold + a2 * pk;
  }
}

// Scalars of sweep k from the previous sweep's global sums (pure function
// of the device state: the sweep kernel and the item-reduction kernel both
// evaluate it and get the same bits).
struct Scal {
  bool first;
  long long kiter;
  double g, alpha, beta, diff, zc, den;
};
__device__ __forceinline__ Scal sweep_scalars(const KParams& k, const DevState* st, int par) {
  Scal c;
  c.first = st->started == 0;
  c.kiter = st->iter + 1;
  c.g = c.alpha = c.beta = c.diff = c.zc = 0.0;
  c.den = 1.0;
  if (!c.first) {
    const double hh = k.h1 * k.h2;
    const double* R = st->fs[par ^ 1];
    c.g = R[0] * hh;
    c.beta = st->iter == 0 ? 0.0 : c.g / st->gprev;
    c.den = R[1] * hh + 2.0 * c.beta * (R[2] * hh) + c.beta * c.beta * (R[3] * hh);
    c.alpha = c.g / c.den;
    const double pn2 = fmax(R[4] + 2.0 * c.beta * R[5] + c.beta * c.beta * R[6], 0.0);
    c.diff = k.weighted ? fabs(c.alpha) * sqrt(pn2 * hh) : fabs(c.alpha) * sqrt(pn2);
    c.zc = 1.0;
  }
  return c;
}

// Does this sweep end the solve before its own work?  brk: breakdown /
// non-finite scalars (stop before this sweep's w term, reference :413);
// last: a deferring sweep (WM = 0) that converged or hit the cap — it only
// adds its own α_k p_k to w.  A pure function of the scalars, so every block
// of the sweep and of its reduction kernel decides the same.
struct Term {
  bool brk, bad, last, conv;
};
template <int WM>
__device__ __forceinline__ Term sweep_term(const KParams& k, const Scal& c) {
  Term t{false, false, false, false};
  if (c.first) return t;
  // breakdown first (reference :413 tests |den| before α exists); a
  // non-finite ‖Δw‖ only matters when α was formed
  const bool tiny = fabs(c.den) < 1e-15;
  t.bad = !isfinite(c.den) || !isfinite(c.g) || (!tiny && !isfinite(c.diff));
  t.brk = t.bad || tiny;
  t.conv = k.check_tol && c.diff < k.tol;
  t.last = !t.brk && WM == 0 && (t.conv || c.kiter >= k.max_iter);
  return t;
}

// Terminal state write (one thread, in the block that arrives last — never
// while another block of the grid may still be reading the state it read at
// entry: the ticket orders every block's reads before this write).
__device__ __forceinline__ void sweep_terminal(const KParams& k, DevState* st, const Scal& c, const Term& t) {
  if (t.brk) {
    st->status = t.bad ? 4 : 2;
    st->iter = c.kiter;
  } else {
    st->gprev = c.g;
    st->rz_cur = c.g;
    st->alpha = c.alpha;
    st->beta = c.beta;
    st->last_diff = c.diff;
    if (k.hist && c.kiter <= k.hist_n) k.hist[c.kiter - 1] = c.diff;
    st->iter = c.kiter;
    st->status = t.conv ? 1 : 3;
  }
  st->done = 1;
  st->wpend = 0;
}

// State update after a sweep's sums t[7] are known (one thread).
template <int WM>
__device__ __forceinline__ void sweep_finalize(const KParams& k, DevState* st, int par, const Scal& c,
                                               const double (&t)[7]) {
#pragma unroll
  for (int n = 0; n < 7; ++n) st->fs[par][n] = t[n];
  if (k.fault_iter > 0 && c.kiter == k.fault_iter) st->fs[par][1] = __builtin_nan("");  // PE_FAULT_INJECT=nan@iter:K
  if (k.fault_zero > 0 && c.kiter == k.fault_zero)  // PE_FAULT_INJECT=zero@iter:K: den of the next sweep = 0
    st->fs[par][1] = st->fs[par][2] = st->fs[par][3] = 0.0;
  st->wpend = WM == 0 ? 1 : 0;
  st->wpar = par;
  if (c.first) {
    st->started = 1;
  } else {
    st->gprev = c.g;
    st->rz_cur = c.g;
    st->alpha = c.alpha;
    st->beta = c.beta;
    st->last_diff = c.diff;
    if (k.hist && c.kiter <= k.hist_n) k.hist[c.kiter - 1] = c.diff;
    st->iter = c.kiter;
    if (k.check_tol && c.diff < k.tol) {
      st->status = 1;
      st->done = 1;
    } else if (c.kiter >= k.max_iter) {
      st->status = 3;
      st->done = 1;
    }
  }
#pragma unroll
  for (int x = 0; x < 8; ++x) __hip_atomic_store(&st->qhead[x][0], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// The final reduction block of a sweep (every thread calls it; the local
// sums t are valid in thread 0): with a P2P transport (k.xr) the 7 sums are
// summed over ranks right here (peer_sum.hpp) — the iteration then needs no
// allreduce launch — then thread 0 updates the state.
__device__ __forceinline__ void slow_inject(const KParams& k) {
  if (k.slow_ticks > 0) {  // PE_FAULT_INJECT=slow@rank (test hook): idle before the cross-rank sum
    const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
    while ((long long)(__builtin_amdgcn_s_memrealtime() - t0) < k.slow_ticks) __builtin_amdgcn_s_sleep(2);
  }
}

template <int WM>
__device__ __forceinline__ void finalize_block(const KParams& k, DevState* st, int par, const Scal& sc,
                                               double (&t)[7]) {
  __shared__ double v[8];
  __shared__ unsigned long long sseq;
  __shared__ int sok;
  if (k.xr.peers) {
    if (threadIdx.x == 0) slow_inject(k);
    if (threadIdx.x == 0)
#pragma unroll
      for (int n = 0; n < 7; ++n) v[n] = t[n];
    peer_sum_block(k.xr, v, 7, &sseq, &sok);
    if (threadIdx.x == 0)
#pragma unroll
      for (int n = 0; n < 7; ++n) t[n] = v[n];
  }
  if (threadIdx.x == 0) sweep_finalize<WM>(k, st, par, sc, t);
}

__device__ __forceinline__ void wave_sum7(double (&v)[7]) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1)
#pragma unroll
    for (int n = 0; n < 7; ++n) v[n] += __shfl_xor(v[n], o, 64);
}

// OCC > 0 caps registers for OCC waves per SIMD (amdgpu_waves_per_eu); PF =
// rows of loads in flight per wave; NT = non-temporal w and output streams
// (they are not re-read within the sweep, so they should not evict the halo
// rows neighbouring items re-read from L2).
//
// WM — deferred solution update.  w_{k+1} = w_k + α_k p_k needs a w read and
// write (16 of the 48 B/point) every sweep; but sweep k+1 still holds p_k
// (its input), so odd sweeps (WM = 0) leave α_k p_k pending and even sweeps
// (WM = 2) apply w += α_{k-1} p_{k-1} + α_k p_k: 40 B/point per iteration on
// average.  A deferring sweep that is the last one (converged / cap) applies
// its own term pointwise; a breakdown applies the pending one; the host
// flushes a pending term (launch_wflush) before w is read.
//
// STAMP — diagnostic build (PE_STAMPS=1, tools/stamp_probe.py): lane 0 of
// every wave records s_memrealtime at its entry and exit and at the start and
// end of every item into k.stamps.  Never the production kernel.
__device__ __forceinline__ unsigned long long rtc() {
  unsigned long long t;  // one asm statement: never merged or moved by the compiler
  asm volatile("s_memrealtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t)::"memory");
  return t;
}

// PUSH — in-sweep halo push (KParams::push): output rows 1, 2 / nx-1, nx are
// also stored into the x-neighbours' fine-grained receive buffers over xGMI
// (system-scope write-through stores, drained and released before the item
// ends, so they are delivered before this rank's cross-rank-sum flags).
template <int OCC, int PF, bool NT, int WM, bool STAMP = false, bool PUSH = false>
__global__ __launch_bounds__(TJ) __attribute__((amdgpu_waves_per_eu(OCC > 0 ? OCC : 1))) void kS(KParams k, int par) {
  DevState* st = k.st;
  const unsigned long long t_entry = STAMP ? rtc() : 0ull;
  // Every state word the sweep needs is loaded up front, together, and
  // nothing waits for them until the wave's first item has issued its
  // prologue row loads (`leave` below): the state round trip after the
  // kernel boundary (≈3 µs from wave entry to the first item when waited for
  // first, profiles/r2_small_before.txt) overlaps the row loads' own.
  const int done = st->done, wpend = st->wpend;
  const double alpha_st = st->alpha;
  // ---- scalars of this sweep from the previous sweep's global sums ----
  const Scal sc = sweep_scalars(k, st, par);
  __shared__ double sm[32];
  __shared__ int sflag;
  __shared__ WaveTV tvs[kWPB];
  __shared__ BandRing rings[kWPB];


  // Row pointers at column -1 (uniform, SGPR) + lane offset (unsigned VGPR).
  const double* __restrict__ Xm = k.x[par ^ 1] - 1;
  double* __restrict__ Ym = k.x[par] - 1;
  double* __restrict__ Wm = k.w - 1;
  const int64_t pitch = k.pitch, poff = k.poff, wp = k.wpitch;
  // halo push: the receive buffer of the parity this sweep reads ([side][2 rows])
  const double* hrd = PUSH ? k.hrecv + int64_t(par ^ 1) * 4 * pitch : nullptr;
  const int nx = int(k.nx), ny = int(k.ny);
  const int lane = threadIdx.x & 63;
  double sg = 0.0, sd = 0.0, se = 0.0, sps = 0.0, szz = 0.0, szp = 0.0, spp = 0.0;

  const int wid = __builtin_amdgcn_readfirstlane(int(threadIdx.x >> 6));
  WaveTV& tvw = tvs[wid];
  BandRing& rg = rings[wid];
  const int gwave = int(blockIdx.x) * kWPB + wid;
  if constexpr (STAMP) {
    if (lane == 0) k.stamps[4 * int64_t(k.nslots) + 2 * gwave] = t_entry;
  }
  // Item walk.  order 3 (default): dynamic — the chunks (row bands) are
  // split into 8 contiguous ranges, one per XCD shard (blocks are dealt
  // round-robin to the 8 XCDs), and the waves of shard x pull (strip, chunk)
  // items in chunk-major order from a device-scope counter of their own
  // (≤ 88 pulls/µs per counter; the next item is requested while the current
  // one runs).  Boundary-band strips cost more than interior ones, so pulling
  // beats any static deal; consecutive chunks stay on one XCD (halo rows
  // re-read from its L2).  order 2: the same ranges dealt statically; 0/1:
  // static global chunk-major / strip-major.
  const int nchunks = (nx + k.ti - 1) / k.ti;
  const bool listed = k.ilist != nullptr;
  const int nsh = listed ? k.lnsh : min(8, int(gridDim.x));  // shards (every shard must own blocks)
  const int xs = int(blockIdx.x) % nsh;
  int it0, istride, ilimit, chunk0;
  unsigned* head = &st->qhead[xs][0];
  if (k.order >= 2) {
    const int nbx = (int(gridDim.x) - xs + nsh - 1) / nsh;
    const int c_lo = (xs * nchunks) / nsh, c_hi = ((xs + 1) * nchunks) / nsh;
    it0 = (int(blockIdx.x) / nsh) * kWPB + wid;
    istride = nbx * kWPB;
    ilimit = (c_hi - c_lo) * k.nstrips;
    chunk0 = c_lo;
  } else {
    it0 = blockIdx.x * kWPB + wid;
    istride = gridDim.x * kWPB;
    ilimit = k.nitems;
    chunk0 = 0;
  }
  // Item list (halo/interior overlap): shard x walks its own list segment
  // (statically, or pulling from its queue under order 3), boundary items
  // first, so the items whose outputs feed the exchange finish in the first
  // round of pulls; the exchange waits for them on st->sig, not for the sweep.
  const int2* lst = nullptr;
  int lnb = 0;
  if (listed) {
    const int nbx = (int(gridDim.x) - xs + nsh - 1) / nsh;
    it0 = (int(blockIdx.x) / nsh) * kWPB + wid;
    istride = nbx * kWPB;
    lst = k.ilist + k.lbase[xs];
    ilimit = k.lbase[xs + 1] - k.lbase[xs];
    lnb = k.lnb[xs];
    chunk0 = 0;
    if (!(k.order == 3) && k.lwaves > 0) {  // static layout for exactly lwaves waves
      istride = k.lwaves;
      if (it0 >= k.lwaves) it0 = ilimit;
    }
  }
  const bool dyn = k.order == 3;
  const bool persum = dyn;
  auto pull = [&]() -> int {
    unsigned v = 0;
    if (lane == 0) v = __hip_atomic_fetch_add(head, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    return __builtin_amdgcn_readfirstlane(int(v));
  };
  // Dynamic listed walk: a wave whose shard queue is exhausted steals from
  // the next shards' queues (each item's sums go to its own slot, so the
  // reduction does not depend on who computed it): no XCD idles while
  // another still holds items.  The host orders every shard's list
  // boundary items (overlap), then heavy items, then the rest chunk-major,
  // and cuts the shards at equal estimated cost (setup_items).
  int sh = xs, visited = 1;
  auto next_shard = [&]() -> bool {
    if (!(dyn && listed) || visited >= nsh) return false;
    sh = sh + 1 == nsh ? 0 : sh + 1;
    ++visited;
    lst = k.ilist + k.lbase[sh];
    ilimit = k.lbase[sh + 1] - k.lbase[sh];
    lnb = k.lnb[sh];
    head = &st->qhead[sh][0];
    return true;
  };
  // Every wave's first item is static (its index within the shard); the
  // queue hands out the items after the first round, so a pull returns v and
  // the item is v + (waves of that shard).  The next item is requested when
  // an item starts and its list entry is fetched right after the item's
  // prologue (the atomic has returned by then), so an item boundary waits on
  // neither.
  auto shard_waves = [&](int x) { return ((int(gridDim.x) - x + nsh - 1) / nsh) * kWPB; };
  int item = it0;
  bool first_item = true;  // STAMP: the step timeline covers the wave's first item
  auto sstamp = [&](int n) {
    if constexpr (STAMP) {
      if (first_item && lane == 0) k.stamps2[int64_t(gwave) * 32 + n] = rtc();
    }
  };
  // prefetched list entry of `item` (have_next: valid); the first one is
  // requested before the scalar checks below wait for the state loads
  bool have_next = listed && it0 < ilimit;
  int2 enext = have_next ? cload_i2(lst + it0) : make_int2(0, 0);

  const double alpha = sc.alpha, beta = sc.beta, zc = sc.zc;
  // Once per wave, after its first prologue loads (or after the walk when it
  // gets no item): true → the wave leaves (solve done, or a terminal sweep).
  bool state_ok = false;
  auto leave = [&]() -> bool {
    state_ok = true;
    if (done) return true;
    const Term tm = sweep_term<WM>(k, sc);
    if (tm.brk || tm.last) {
      // breakdown: apply only the pending term; last sweep of the solve: only
      // w changes (w += α_k p_k, pointwise).  The state is written by the
      // last-arriving block here (static sweeps) or by the reduction kernel
      // that follows (dynamic sweeps) — never while blocks may still read it.
      if (tm.brk) {
        if (WM == 2 && wpend && !tm.bad) w_pointwise(k, k.x[par ^ 1], alpha_st, 0.0, 0.0, 0.0);
      } else {
        w_pointwise(k, k.x[par ^ 1], 0.0, alpha, zc, beta);
      }
      // A wave reaches this point after its first item's prologue or after
      // an empty walk — different program points within one workgroup — so
      // the hand-off counts waves (no workgroup barrier on this path).
      if (!persum && arrive_last_wave(&st->ticket[4], gridDim.x * kWPB) && lane == 0) {
        sweep_terminal(k, st, sc, tm);
        __hip_atomic_store(&st->ticket[4], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
      return true;
    }
    return false;
  };
  // α of the pending term left by the previous (deferring) sweep
  const double alpha_prev = (WM == 2 && wpend) ? alpha_st : 0.0;
  for (;;) {
    if (item >= ilimit) {
      if (!next_shard()) break;
      item = pull() + shard_waves(sh);
      have_next = false;
      continue;
    }
    unsigned nxt_v = 0;  // next item, requested now, read after the prologue
    if (dyn && lane == 0) nxt_v = __hip_atomic_fetch_add(head, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    // Item geometry: a list entry is {first row, strip | rows << 20} (items
    // of any height; its sums go to slot = list position), otherwise the
    // item index is (strip, ti-row chunk) and the slot is chunk-major.
    int s, ib, ie;
    int64_t slot;
    bool band = true;  // the item has boundary-band rows (general march); lists say which do not
    if (listed) {
      const int2 e = have_next ? enext : cload_i2(lst + item);
      s = e.y & 0xFFFFF;
      ib = e.x & kRowMask;
      band = (e.x & kBandBit) != 0;
      ie = min(ib + (e.y >> 20) - 1, nx);
      if (ie < ib) {  // empty position of a static layout
        item += istride;
        continue;
      }
      slot = int64_t(k.lbase[sh]) + item;
    } else {
      const int gitem = item;
      s = k.order == 1 ? gitem / nchunks : gitem % k.nstrips;
      const int ch = chunk0 + (k.order == 1 ? gitem % nchunks : gitem / k.nstrips);
      ib = 1 + ch * k.ti;
      ie = min(ib + k.ti - 1, nx);
      slot = int64_t(ch) * k.nstrips + s;
    }
    const unsigned long long t_item = STAMP ? rtc() : 0ull;
    sstamp(0);
    const int J = -1 + s * FSW;
    const int c0 = J + 2 * lane;               // odd → 16-byte aligned pair (c0, c0+1)
    const unsigned off = unsigned(c0 + 1);     // element offset from column -1
    const int64_t g0 = k.gj0 + c0;
    const bool lv0 = c0 <= ny + 2 && g0 >= 1 && g0 <= k.N - 1;
    const bool lv1 = c0 + 1 <= ny + 2 && g0 + 1 >= 1 && g0 + 1 <= k.N - 1;
    const bool inner = lane >= 1 && lane <= 62;
    const bool o0 = inner && c0 >= 1 && c0 <= ny;
    const bool o1 = inner && c0 + 1 <= ny;
    const int jl0 = 2 * lane;
    // y-direction halo strips (columns 1,2 and ny-1,ny) of output row i → send buffers
    auto send_strips = [&](int i, const double2& rkI, const double2& pa) {
      if (k.has[DOWN] && o0 && c0 == 1) {
        double* sb = k.send_dn + int64_t(i - 1) * 4;
        sb[0] = rkI.x;
        sb[1] = rkI.y;
        sb[2] = pa.x;
        sb[3] = pa.y;
      }
      if (k.has[UP]) {
        double* sb = k.send_up + int64_t(i - 1) * 4;
        if (o0 && c0 >= ny - 1) {
          sb[c0 - (ny - 1)] = rkI.x;
          sb[c0 - (ny - 1) + 2] = pa.x;
        }
        if (o1 && c0 + 1 >= ny - 1) {
          sb[c0 + 1 - (ny - 1)] = rkI.y;
          sb[c0 + 1 - (ny - 1) + 2] = pa.y;
        }
      }
    };
    // In-sweep halo push of output row i (PUSH): rows 1, 2 → the LEFT
    // neighbour's rows nx'+1, nx'+2, rows nx-1, nx → the RIGHT neighbour's
    // rows -1, 0 (row tests are uniform; owned columns only — the receive
    // buffers' halo columns stay zero, as the global boundary's are).
    bool pushed = false;
    auto push_row = [&](int i, const double2& rkI, const double2& pa) {
      auto put = [&](double* base, int slot) {
        double* d = base + int64_t(slot) * pitch + off;
        if (o0) {
          __hip_atomic_store(d, rkI.x, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
          __hip_atomic_store(d + poff, pa.x, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        }
        if (o1) {
          __hip_atomic_store(d + 1, rkI.y, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
          __hip_atomic_store(d + 1 + poff, pa.y, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        }
        pushed = true;
      };
      if (i <= 2 && k.hpush_lo[par] != nullptr) put(k.hpush_lo[par], i - 1);
      if (i >= nx - 1 && k.hpush_hi[par] != nullptr) put(k.hpush_hi[par], i - (nx - 1));
    };
    // Strip chord entries → LDS, read by boundary-band rows only: staged only
    // when the item has band rows in this strip (a few % of items).
    bool tv_ok = false;
    auto stage_tv = [&]() {
      const double* t0 = k.rowT + (c0 + 1) * 4;
      const double4 a = *reinterpret_cast<const double4*>(t0);
      const double4 b = *reinterpret_cast<const double4*>(t0 + 4);
      tvw.sA[jl0] = a.x;
      tvw.eA[jl0] = a.y;
      tvw.hB[jl0] = a.z;
      tvw.sA[jl0 + 1] = b.x;
      tvw.eA[jl0 + 1] = b.y;
      tvw.hB[jl0 + 1] = b.z;
      if (lane == 63) tvw.hB[128] = t0[10];
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
      tv_ok = true;
    };
    // Row classes of a 64-row segment, lane l ↔ row segbase+l; band rows as
    // a scalar bit mask.  Reloaded every 60 rows (items may be long).  The
    // load is issued before the prologue's row loads and waited for after
    // them (loads complete in order: waiting for it leaves the rows in flight).
    int segbase = 0;
    int4 rcv;
    double2 ctv;  // column table of row segbase+lane: {half-width, sB}
    double cte;   // ... eB
    unsigned long long genmask = 0;
    auto issue_seg = [&](int base) {
      segbase = base;
      const int nr = ie + 3 - base;
      rcv = lane < nr ? *reinterpret_cast<const int4*>(k.rowcls + (base + 1 + lane) * 4) : make_int4(1, 0, 0, -1);
      if (band) {
        const double* ctr = k.colT + (min(base + lane, ie + 3) + 1) * 4;  // rows base .. ie+3
        ctv = *reinterpret_cast<const double2*>(ctr);
        cte = ctr[2];
      }
    };
    auto finish_seg = [&]() {
      if (!band) return;  // plain items: the row classes are waited for at their first use
      const int nr = ie + 3 - segbase;
      genmask = __ballot(lane < nr && has_gen(RowCls{rcv.x, rcv.y, rcv.z, rcv.w}, J, J + 127));
      if (genmask != 0 && !tv_ok) stage_tv();
    };
    auto load_seg = [&](int base) {
      issue_seg(base);
      finish_seg();
    };
    issue_seg(ib - 2);
    auto rinfo = [&](int t) {
      RowI r;
      r.t = t;
      const int l = t - segbase;
      const int lo = __builtin_amdgcn_readlane(rcv.x, l), hi = __builtin_amdgcn_readlane(rcv.y, l);
      r.in0 = c0 >= lo && c0 <= hi;
      r.in1 = c0 + 1 >= lo && c0 + 1 <= hi;
      r.gen = (genmask >> l) & 1ull;
      return r;
    };
    // Row t enters the pipeline (its p_k stage): 1/D of both columns; a
    // band row evaluates its coefficients here, once, into ring slot `slot`.
    auto enter = [&](const RowI& R, int t, int slot, double& d0, double& d1) {
      if (!R.gen) {
        d0 = dsel(k, R.in0);
        d1 = dsel(k, R.in1);
      } else {
        const int l = R.t - segbase;
        const RowCls rc = rcl_read(rcv, l);
        const CT ct{readlane(ctv.x, l), readlane(ctv.x, l + 1), readlane(ctv.y, l), readlane(cte, l)};
        const CS x0 = cs_gen(k, rc, ct, c0, tvw, jl0), x1 = cs_gen(k, rc, ct, c0 + 1, tvw, jl0 + 1);
        ring_put(rg, slot, lane, x0, x1);
        d0 = x0.d;
        d1 = x1.d;
      }
    };
    // (A u)(row t) for both columns; d0/d1 = 1/D of row t.
    auto apply = [&](const RowI& R, int slot, const double2& um, const double2& u0, const double2& un, double ul,
                     double ur, double& a0, double& a1, double& d0, double& d1) {
      if (!R.gen) {
        const double f0 = fsel(k, R.in0), f1 = fsel(k, R.in1);
        a0 = lapf(k, f0, um.x, u0.x, un.x, ul, u0.y);
        a1 = lapf(k, f1, um.y, u0.y, un.y, u0.x, ur);
        d0 = dsel(k, R.in0);
        d1 = dsel(k, R.in1);
      } else {
        CS x0, x1;
        ring_get(rg, slot, lane, x0, x1);
        a0 = stencil<false>(k, x0, um.x, u0.x, un.x, ul, u0.y);
        a1 = stencil<false>(k, x1, um.y, u0.y, un.y, u0.x, ur);
        d0 = x0.d;
        d1 = x1.d;
      }
    };

    // x row t at element offset o.  Under the halo push the slab's halo rows
    // (-1, 0 from LEFT, nx+1, nx+2 from RIGHT) are read straight from the
    // receive buffer the neighbours pushed them into during the previous
    // sweep (system-scope loads: written over xGMI, never through this GPU's
    // caches; delivered before the cross-rank-sum flags that sweep waited
    // for) — no import kernel between the sweeps.  Row tests are uniform.
    auto ldx = [&](int t, unsigned o) -> double2 {
      if constexpr (PUSH) {
        if ((t < 1 && k.has[LEFT]) || (t > nx && k.has[RIGHT])) {
          const double* h = hrd + int64_t(t < 1 ? t + 1 : t - nx + 1) * pitch + o;
          return dd(__hip_atomic_load(h, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM),
                    __hip_atomic_load(h + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM));
        }
      }
      return ld2(Xm + int64_t(t) * pitch + o);
    };
    // prologue: p_k on rows ib-2, ib-1; x rows ib .. ib+PF-1 and w rows
    // ib-2 .. ib-3+PF queued
    const double2 rA = ldx(ib - 2, off), pA = ldx(ib - 2, poff + off);
    double2 rin1 = ldx(ib - 1, off);  // r_{k-1}(i+1) at step i
    const double2 pB = ldx(ib - 1, poff + off);
    double2 rq[PF], pq[PF], wq[PF];
#pragma unroll
    for (int q = 0; q < PF; ++q) {
      const int t = min(ib + q, ie + 2);
      rq[q] = ldx(t, off);
      pq[q] = ldx(t, poff + off);
      if constexpr (WM == 2) wq[q] = (ib - 2 + q >= ib) ? ldw<NT>(Wm + int64_t(ib - 2 + q) * wp + off) : dd(0.0, 0.0);
      else wq[q] = dd(0.0, 0.0);
    }
    if (!state_ok && leave()) return;
    sstamp(1);
    finish_seg();
    sstamp(2);
    // next item: the pull (older than the prologue loads) has returned
    int nxt_item = ilimit;
    have_next = false;
    if (dyn) {
      nxt_item = __builtin_amdgcn_readfirstlane(int(nxt_v)) + shard_waves(sh);
      if (listed && nxt_item < ilimit) {
        enext = cload_i2(lst + nxt_item);
        have_next = true;
      }
    }
    // ---- the row march ----
    // Row t's values live in slot (t - t0) & 3 of 4-entry register arrays and
    // the row loop is unrolled by 4 (= the prefetch depth), so every slot
    // index is a compile-time constant and nothing rotates (a rolled loop
    // spent ≈70 v_mov_b64 per row step moving its window; a row step is
    // instruction-issue-bound when a sweep gives each SIMD about one wave —
    // small blocks: 0.84 µs per step at 800×1200, profiles/r2_steps_before.txt).
    // The last group stops at row ie (a uniform early exit).
    // Boundary-band rows (items with the band flag only; a scalar test per
    // row) take the coefficient path: evaluated once when the row enters
    // (ring slot (t - t0) mod 3), re-read by its two stencil stages.
    static_assert(PF == 4, "row march: prefetch depth = unroll factor");
    const int t0 = ib - 2;
    double2 RQ[4], PQ[4], WQ[4], P[4], Z[4], Q[4], RIN[2], S[2], RK[2];
    RowI RW[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      RQ[(q + 2) & 3] = rq[q];  // x rows ib+q = t0+2+q
      PQ[(q + 2) & 3] = pq[q];
      WQ[q] = wq[q];  // w rows t0+q
      Z[q] = dd(0.0, 0.0);
      Q[q] = dd(0.0, 0.0);
      P[q] = dd(0.0, 0.0);
      RW[q] = RowI{false, false, false, 0};
    }
    RW[0] = rinfo(t0);
    RW[1] = rinfo(t0 + 1);
    {
      double d0, d1;
      enter(RW[0], t0, 0, d0, d1);
      P[0] = dd(zc * (rA.x * d0) + beta * pA.x, zc * (rA.y * d1) + beta * pA.y);
      enter(RW[1], t0 + 1, 1, d0, d1);
      P[1] = dd(zc * (rin1.x * d0) + beta * pB.x, zc * (rin1.y * d1) + beta * pB.y);
    }
    Q[0] = pA;
    Q[1] = pB;
    RIN[0] = rin1;
    RIN[1] = S[0] = S[1] = RK[0] = RK[1] = dd(0.0, 0.0);
    sstamp(3);
    const int nsteps = ie - t0 + 1;
    int sl = 0;  // ring slot of row i at step i ((i - t0) mod 3)
    for (int g = 0; 4 * g < nsteps; ++g) {
      if (g > 0 && g % 15 == 0) load_seg(t0 + 4 * g + 2);  // rows i+2 .. i+65 of this group's i
#pragma unroll
      for (int jj = 0; jj < 4; ++jj) {
        const int i = t0 + 4 * g + jj;
        if (i > ie) break;
        const int a = jj, b = (jj + 1) & 3, c = (jj + 2) & 3, m = (jj + 3) & 3;  // rows i, i+1, i+2, i-1
        const int sl1 = sl == 2 ? 0 : sl + 1, sl2 = sl == 0 ? 2 : sl - 1;  // ring slots of rows i+1, i+2
        const double2 rQ0 = RQ[c], pQ0 = PQ[c], wQ0 = WQ[a];
        {  // prefetch x row i+6 and w row i+4 into the slots just consumed
          const int t = min(i + 2 + PF, ie + 2);
          RQ[c] = ldx(t, off);
          PQ[c] = ldx(t, poff + off);
          if constexpr (WM == 2) WQ[a] = ldw<NT>(Wm + int64_t(min(i + PF, ie)) * wp + off);
        }
        // p_k(i+2) = z_{k-1} + β p_{k-1}
        RW[c] = rinfo(i + 2);
        {
          double d0, d1;
          enter(RW[c], i + 2, sl2, d0, d1);
          P[c] = dd(zc * (rQ0.x * d0) + beta * pQ0.x, zc * (rQ0.y * d1) + beta * pQ0.y);
        }
        if constexpr (WM == 2) Q[c] = pQ0;
        // s(i+1) = A p_k, r_k(i+1), z_k(i+1)
        double s0, s1, d10, d11;
        apply(RW[b], sl1, P[a], P[b], P[c], dpp_shr1(P[b].y), dpp_shl1(P[b].x), s0, s1, d10, d11);
        const double2 rin = RIN[jj & 1];
        const double rk0 = rin.x - alpha * s0, rk1 = rin.y - alpha * s1;
        const int64_t gr = k.gi0 + i + 1;
        const bool rl = gr >= 1 && gr <= k.M - 1;
        const double zn0 = (rl && lv0) ? rk0 * d10 : 0.0;
        const double zn1 = (rl && lv1) ? rk1 * d11 : 0.0;
        if (i >= ib) {
          // q(i) = A z_k, the 7 sums, the row-i outputs
          const double2 zI = Z[a], pa = P[a], sI = S[jj & 1], rkI = RK[jj & 1];
          double q0, q1, e0, e1;
          apply(RW[a], sl, Z[m], zI, dd(zn0, zn1), dpp_shr1(zI.y), dpp_shl1(zI.x), q0, q1, e0, e1);
          const double zo0 = o0 ? zI.x : 0.0, po0 = o0 ? pa.x : 0.0;
          const double zo1 = o1 ? zI.y : 0.0, po1 = o1 ? pa.y : 0.0;
          sg += rkI.x * zo0 + rkI.y * zo1;
          sd += zo0 * q0 + zo1 * q1;
          se += zo0 * sI.x + zo1 * sI.y;
          sps += po0 * sI.x + po1 * sI.y;
          szz += zo0 * zo0 + zo1 * zo1;
          szp += zo0 * po0 + zo1 * po1;
          spp += po0 * po0 + po1 * po1;
          double* yr = Ym + int64_t(i) * pitch + off;
          double* wd = Wm + int64_t(i) * wp + off;
          const double2 qa = Q[a];
          const double2 wv = dd(wQ0.x + alpha_prev * qa.x + alpha * pa.x, wQ0.y + alpha_prev * qa.y + alpha * pa.y);
          if (o1) {
            st2<NT>(yr, rkI);
            st2<NT>(yr + poff, pa);
            if constexpr (WM == 2) st2<NT>(wd, wv);
          } else if (o0) {
            yr[0] = rkI.x;
            yr[poff] = pa.x;
            if constexpr (WM == 2) wd[0] = wv.x;
          }
          send_strips(i, rkI, pa);
          if constexpr (PUSH) push_row(i, rkI, pa);
        }
        Z[b] = dd(zn0, zn1);
        S[(jj + 1) & 1] = dd(s0, s1);
        RK[(jj + 1) & 1] = dd(rk0, rk1);
        RIN[(jj + 1) & 1] = rQ0;
        sl = sl1;
        if (i - ib + 6 < 30) sstamp(i - ib + 6);  // after row step i: slots 4 ..
      }
    }
    if constexpr (PUSH) {
      if (pushed) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // (system-scope atomic stores: fused3.hip march3)
    }
    if (persum) {
      // per-item sums (wave-reduced) in a fixed slot: the reduction kernel
      // adds them in item order, so the result does not depend on which
      // wave pulled which item
      double v[7] = {sg, sd, se, sps, szz, szp, spp};
      wave_sum7(v);
      if (lane == 0) {
        double* dst = k.itemsum + 8 * slot;
#pragma unroll
        for (int n = 0; n < 7; ++n) dst[n] = v[n];
      }
      sg = sd = se = sps = szz = szp = spp = 0.0;
    }
    if (item < lnb) {
      // boundary item: once its stores (send strips included) have reached L2,
      // count it.  No agent-scope release here — that is an L2 writeback per
      // item (≈15 µs per 8-rank sweep); kWaitSig writes each XCD's L2 back once.
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      if (lane == 0) __hip_atomic_fetch_add(&st->sig, 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    if constexpr (STAMP) {
      if (lane == 0) {
        unsigned long long* d = k.stamps + 4 * slot;
        d[0] = t_item;
        d[1] = rtc();
        d[2] = (unsigned long long)gwave | ((unsigned long long)s << 32);
        d[3] = (unsigned long long)ib | ((unsigned long long)(ie - ib + 1) << 32) | ((unsigned long long)(band ? 1 : 0) << 48);
      }
    }
    sstamp(31);
    first_item = false;
    item = dyn ? nxt_item : item + istride;
  }
  if constexpr (STAMP) {
    if (lane == 0) k.stamps[4 * int64_t(k.nslots) + 2 * gwave + 1] = rtc();
  }
  if (!state_ok && leave()) return;
  if (persum) return;  // kRed reduces the item sums and finalizes

  double v[7] = {sg, sd, se, sps, szz, szp, spp};
  if (publish_last_nm<7>(k.partial, v, &st->ticket[0], &sflag, sm)) {  // (kcommon.hpp: n-major partials)
    double t[7];
    reduce_partials_nm<7>(k.partial, t, sm);
    finalize_block<WM>(k, st, par, sc, t);
    if (threadIdx.x == 0) __hip_atomic_store(&st->ticket[0], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
}

// Dynamic-queue sweeps: deterministic reduction of the per-item sums (item
// order, fixed per-block ranges) and the state update.
template <int WM>
__global__ __launch_bounds__(TJ) void kRed(KParams k, int par) {
  DevState* st = k.st;
  if (st->done) return;  // includes a breakdown / last sweep handled by kS
  __shared__ double sm[32];
  __shared__ int sflag;
  const Scal sc = sweep_scalars(k, st, par);
  {
    const Term tm = sweep_term<WM>(k, sc);
    if (tm.brk || tm.last) {  // the sweep stopped early (kS): only the terminal state is left to write
      if (arrive_last(&st->ticket[1], gridDim.x, &sflag) && threadIdx.x == 0) {
        sweep_terminal(k, st, sc, tm);
        __hip_atomic_store(&st->ticket[1], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
      return;
    }
  }
  const int64_t n = k.nslots, lo = n * blockIdx.x / gridDim.x, hi = n * (blockIdx.x + 1) / gridDim.x;
  double v[7] = {0, 0, 0, 0, 0, 0, 0};
  // RU items per thread in flight: all loads of a batch are issued before the
  // first add (clamped indices, no predicated loads), then added in item
  // order — the same order (and bits) as a plain loop, without one DRAM
  // round trip per item (≈8 per thread at 8192², ≈9 µs of the kernel).
  constexpr int RU = 8;
  for (int64_t i0 = lo + threadIdx.x; i0 < hi; i0 += RU * TJ) {
    double4 a[RU], b[RU];
#pragma unroll
    for (int u = 0; u < RU; ++u) {
      const int64_t i = min(i0 + int64_t(u) * TJ, hi - 1);
      const double4* src = reinterpret_cast<const double4*>(k.itemsum + 8 * i);
      a[u] = src[0];
      b[u] = src[1];
    }
    asm volatile("" ::: "memory");  // keep the batch's loads ahead of the adds
    // past-the-end slots add +0.0: v starts at +0.0 and is never -0.0, so
    // v + 0.0 == v bitwise and the order of the real terms is unchanged
#pragma unroll
    for (int u = 0; u < RU; ++u) {
      const bool in = i0 + int64_t(u) * TJ < hi;
      v[0] += in ? a[u].x : 0.0;
      v[1] += in ? a[u].y : 0.0;
      v[2] += in ? a[u].z : 0.0;
      v[3] += in ? a[u].w : 0.0;
      v[4] += in ? b[u].x : 0.0;
      v[5] += in ? b[u].y : 0.0;
      v[6] += in ? b[u].z : 0.0;
    }
  }
  if (publish_last_nm<7>(k.partial, v, &st->ticket[1], &sflag, sm)) {  // (kcommon.hpp: n-major partials)
    double t[7];
    reduce_partials_nm<7>(k.partial, t, sm);
    finalize_block<WM>(k, st, par, sc, t);
    if (threadIdx.x == 0) __hip_atomic_store(&st->ticket[1], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
}

// Single-workgroup variant for blocks of few items (multi-rank blocks): no
// partials, no release/acquire ticket — the multi-block form spends most of
// its ≈10 µs in that fan-in.  Thread t sums items t, t+1024, … (8 loads in
// flight), then a fixed wave → workgroup tree: deterministic.
constexpr int kRed1Threads = 1024;
template <int WM>
__global__ __launch_bounds__(kRed1Threads) void kRed1(KParams k, int par) {
  DevState* st = k.st;
  const int done = st->done;
  const Scal sc = sweep_scalars(k, st, par);
  if (done) return;
  {
    const Term tm = sweep_term<WM>(k, sc);
    if (tm.brk || tm.last) {  // the sweep stopped early (kS): only the terminal state is left to write
      if (threadIdx.x == 0) sweep_terminal(k, st, sc, tm);
      return;
    }
  }
  __shared__ double sm[7][kRed1Threads / 64];
  const int64_t n = k.nslots;
  double v[7] = {0, 0, 0, 0, 0, 0, 0};
  const double4* src = reinterpret_cast<const double4*>(k.itemsum);
  // one batch of RU items per thread in flight (clamped loads, +0.0 past the
  // end — see kRed): same order and bits as a plain strided loop
  constexpr int RU = 8;
  for (int64_t i0 = threadIdx.x; i0 < n; i0 += RU * kRed1Threads) {
    double4 a[RU], b[RU];
#pragma unroll
    for (int u = 0; u < RU; ++u) {
      const int64_t i = min(i0 + int64_t(u) * kRed1Threads, n - 1);
      a[u] = src[2 * i];
      b[u] = src[2 * i + 1];
    }
    asm volatile("" ::: "memory");
#pragma unroll
    for (int u = 0; u < RU; ++u) {
      const bool in = i0 + int64_t(u) * kRed1Threads < n;
      v[0] += in ? a[u].x : 0.0;
      v[1] += in ? a[u].y : 0.0;
      v[2] += in ? a[u].z : 0.0;
      v[3] += in ? a[u].w : 0.0;
      v[4] += in ? b[u].x : 0.0;
      v[5] += in ? b[u].y : 0.0;
      v[6] += in ? b[u].z : 0.0;
    }
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1)
#pragma unroll
    for (int q = 0; q < 7; ++q) v[q] += __shfl_xor(v[q], o, 64);
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  if (lane == 0)
#pragma unroll
    for (int q = 0; q < 7; ++q) sm[q][wid] = v[q];
  __syncthreads();
  double t[7];
  if (threadIdx.x == 0) {
#pragma unroll
    for (int q = 0; q < 7; ++q) {
      t[q] = 0.0;
      for (int w = 0; w < kRed1Threads / 64; ++w) t[q] += sm[q][w];
    }
  }
  finalize_block<WM>(k, st, par, sc, t);
}

// Apply a pending α_k p_k (p_k = p-plane of x[wpar]) before w is read.
__global__ void kWFlush(KParams k) {
  DevState* st = k.st;
  if (!st->wpend) return;
  const double a = st->alpha;
  const double* p = k.x[st->wpar] + k.poff;
  const int64_t n = k.nx * k.ny;
  for (int64_t idx = int64_t(blockIdx.x) * blockDim.x + threadIdx.x; idx < n; idx += int64_t(gridDim.x) * blockDim.x) {
    const int64_t li = idx / k.ny + 1, lj = idx % k.ny + 1;
    k.w[li * k.wpitch + lj] += a * p[li * k.pitch + lj];
  }
}
__global__ void kWFlushDone(KParams k) { k.st->wpend = 0; }

// Overlap: hold the halo stream until every boundary item of the running
// sweep is in L2 (kS counts them into sig), or the solve has ended (the sweep
// then stores nothing), then make those stores visible device-wide: L2s are
// per XCD and not coherent with each other, so each block — launched on 8
// consecutive workgroups, which the dispatcher deals to the 8 XCDs — writes
// its XCD's L2 back (agent-scope release).  Targets are cumulative per solve.
__global__ void kWaitSig(DevState* st, unsigned long long target) {
  if (threadIdx.x == 0) {
    // (polled every ≈1 µs: the boundary items take tens of µs, and a
    // tighter poll of the state's line competes with the sweep's traffic)
    const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
    while (__hip_atomic_load(&st->sig, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < target &&
           !__hip_atomic_load(&st->done, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) {
      __builtin_amdgcn_s_sleep(40);
      // a target the sweeps never reach (a host-side count error) ends the
      // solve as an internal error (status 5) after 30 s instead of hanging
      // the stream: every later kernel is then a no-op
      if (__builtin_amdgcn_s_memrealtime() - t0 > 3000000000ull) {
        __hip_atomic_store(&st->status, 5, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_store(&st->done, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        break;
      }
    }
    __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "agent");
  }
}

// y-direction halo strips of buffer b (one thread per owned row): the hdep
// owned columns next to each y neighbour, r then p — columns 1..h → DOWN
// (its ny'+1..ny'+h), ny-h+1..ny → UP (its 1-h..0).
__global__ void kPack(KParams k, int b) {
  const int64_t i = int64_t(blockIdx.x) * blockDim.x + threadIdx.x + 1;
  if (i > k.nx) return;
  const int h = k.hdep;
  const double* x = k.x[b] + i * k.pitch;
  if (k.has[DOWN]) {
    double* sb = k.send_dn + (i - 1) * 2 * h;
    for (int m = 0; m < h; ++m) {
      sb[m] = x[1 + m];
      sb[h + m] = x[k.poff + 1 + m];
    }
  }
  if (k.has[UP]) {
    double* sb = k.send_up + (i - 1) * 2 * h;
    for (int m = 0; m < h; ++m) {
      sb[m] = x[k.ny - h + 1 + m];
      sb[h + m] = x[k.poff + k.ny - h + 1 + m];
    }
  }
}

__global__ void kUnpack(KParams k, int b) {
  const int64_t i = int64_t(blockIdx.x) * blockDim.x + threadIdx.x + 1;
  if (i > k.nx) return;
  const int h = k.hdep;
  double* x = k.x[b] + i * k.pitch;
  if (k.has[DOWN]) {
    const double* rb = k.recv_dn + (i - 1) * 2 * h;
    for (int m = 0; m < h; ++m) {
      x[1 - h + m] = rb[m];
      x[k.poff + 1 - h + m] = rb[h + m];
    }
  }
  if (k.has[UP]) {
    const double* rb = k.recv_up + (i - 1) * 2 * h;
    for (int m = 0; m < h; ++m) {
      x[k.ny + 1 + m] = rb[m];
      x[k.poff + k.ny + 1 + m] = rb[h + m];
    }
  }
}

// In-sweep halo push, receiving side: rows -1, 0 (from LEFT) and nx+1, nx+2
// (from RIGHT) of x[b] ← the receive buffer of parity b.  The sweeps read the
// halo rows from the receive buffer themselves (kS, ldx); this copy only makes
// x[b] whole for a checkpoint or a field read-back.  The neighbours' stores
// reached the buffer before their cross-rank-sum flags, which this rank's
// last reduction waited for; the loads are system-scope (the buffer is
// written over xGMI, never through this GPU's caches).
__global__ __launch_bounds__(256) void kHaloImport(KParams k, int b) {
  const int h = k.hdep;
  const int64_t n = int64_t(h) * k.pitch;
  double* x = k.x[b] - k.xorg;  // row 0, column -xorg
  for (int side = 0; side < 2; ++side) {
    if (!k.has[side == 0 ? LEFT : RIGHT]) continue;
    const double* src = k.hrecv + (int64_t(b) * 2 + side) * n;
    double* dst = x + (side == 0 ? int64_t(1 - h) : k.nx + 1) * k.pitch;
    for (int64_t i = int64_t(blockIdx.x) * blockDim.x + threadIdx.x; i < n; i += int64_t(gridDim.x) * blockDim.x)
      dst[i] = __hip_atomic_load(src + i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  }
}

// The reverse copy: the receive buffer of parity b ← x[b]'s halo rows, after
// an exchange through the comm (the initial state) or a checkpoint load, so
// the next sweep's halo reads find them there.  System-scope stores, as the
// pushes': the sweep's loads bypass this GPU's caches.
__global__ __launch_bounds__(256) void kHaloSeed(KParams k, int b) {
  const int h = k.hdep;
  const int64_t n = int64_t(h) * k.pitch;
  const double* x = k.x[b] - k.xorg;  // row 0, column -xorg
  for (int side = 0; side < 2; ++side) {
    if (!k.has[side == 0 ? LEFT : RIGHT]) continue;
    double* dst = const_cast<double*>(k.hrecv) + (int64_t(b) * 2 + side) * n;  // this rank's own buffer
    const double* src = x + (side == 0 ? int64_t(1 - h) : k.nx + 1) * k.pitch;
    for (int64_t i = int64_t(blockIdx.x) * blockDim.x + threadIdx.x; i < n; i += int64_t(gridDim.x) * blockDim.x)
      __hip_atomic_store(dst + i, src[i], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  }
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
}

// Halo-push set-up self-test (DeviceSolver::setup_halo_push): every rank
// fills its neighbours' receive buffers through the push's own store form
// with values naming sender, side, parity and index; after a cross-rank
// barrier every rank checks what arrived (system-scope loads).
__device__ __forceinline__ double push_code(int rank, int side, int b, int64_t i) {
  return double((rank * 2 + side) * 2 + b) * 1e7 + double(i);
}
__global__ __launch_bounds__(256) void kPushTestWrite(KParams k, int me) {
  const int64_t n = int64_t(k.hdep) * k.pitch;
  for (int b = 0; b < 2; ++b)
    for (int64_t i = int64_t(blockIdx.x) * blockDim.x + threadIdx.x; i < n; i += int64_t(gridDim.x) * blockDim.x) {
      if (k.hpush_lo[b]) __hip_atomic_store(k.hpush_lo[b] + i, push_code(me, 1, b, i), __ATOMIC_RELAXED,
                                            __HIP_MEMORY_SCOPE_SYSTEM);
      if (k.hpush_hi[b]) __hip_atomic_store(k.hpush_hi[b] + i, push_code(me, 0, b, i), __ATOMIC_RELAXED,
                                            __HIP_MEMORY_SCOPE_SYSTEM);
    }
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
}
__global__ __launch_bounds__(256) void kPushTestCheck(KParams k, int left, int right, int* bad) {
  const int64_t n = int64_t(k.hdep) * k.pitch;
  int nbad = 0;
  for (int b = 0; b < 2; ++b)
    for (int side = 0; side < 2; ++side) {
      const int from = side == 0 ? left : right;
      if (from < 0) continue;
      const double* src = k.hrecv + (int64_t(b) * 2 + side) * n;
      for (int64_t i = int64_t(blockIdx.x) * blockDim.x + threadIdx.x; i < n; i += int64_t(gridDim.x) * blockDim.x)
        nbad += __hip_atomic_load(src + i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) != push_code(from, side, b, i);
    }
  if (nbad) atomicAdd(bad, nbad);
}

// Test op: the division-free coefficients the single-sweep kernels evaluate
// (cset_rc from the row classes and chord tables) for every node of the block
// plus its 1-wide ring, dense [(nx+2) × (ny+2)]: a(li, lj), b(li, lj), 1/D.
__global__ void kCoefFast(KParams k, double* a, double* b, double* dinv) {
  const int64_t W = k.ny + 2, n = (k.nx + 2) * W;
  for (int64_t idx = int64_t(blockIdx.x) * blockDim.x + threadIdx.x; idx < n; idx += int64_t(gridDim.x) * blockDim.x) {
    const int64_t li = idx / W, lj = idx % W;
    const int* rc = k.rowcls + (li + 1) * 4;
    const RowCls c{rc[0], rc[1], rc[2], rc[3]};
    const double* ctr = k.colT + (li + 1) * 4;
    const double* tv = k.rowT + (lj + 1) * 4;
    const CS x = cset_rc(k, c, CT{ctr[0], ctr[4], ctr[1], ctr[2]}, lj, TV{tv[0], tv[1], tv[2], tv[6]});
    a[idx] = x.a0;
    b[idx] = x.b0;
    dinv[idx] = x.d;
  }
}

}  // namespace

void launch_coef_fast(const KParams& k, double* a, double* b, double* dinv, hipStream_t s) {
  const int64_t n = (k.nx + 2) * (k.ny + 2);
  const unsigned g = unsigned(std::min<int64_t>(4096, std::max<int64_t>(1, (n + 255) / 256)));
  hipLaunchKernelGGL(kCoefFast, dim3(g), dim3(256), 0, s, k, a, b, dinv);
}

// Kernel configuration: 4 rows of loads in flight per wave + non-temporal
// w / output streams (8192² sweep: 1373 it/s vs 1119 for 2 rows / temporal
// streams at 3 waves per SIMD — the sweep is bound by HBM latency per wave,
// not by occupancy; round 1 also measured 2 / 3 / 5 rows in flight: 4 won,
// and the plain march's unroll is tied to it).
template <int WM, class F>
static auto with_kS(const KParams& k, F&& f) {
  if (k.stamps) return f(kS<2, 4, true, WM, true>);
  if (k.push) return f(kS<2, 4, true, WM, false, true>);
  return f(kS<2, 4, true, WM>);
}

void launch_S(const KParams& k, int par, hipStream_t s, bool with_red) {
  if (k.steps == 3) {  // three iterations per sweep (fused3.hip)
    launch_S3(k, par, s);
    return;
  }
  if (k.steps == 2) {  // two iterations per sweep (fused2.hip)
    launch_S2(k, par, s);
    return;
  }
  // each variant runs on its own resident grid (from the occupancy API; both
  // are 2 workgroups per CU since the band-coefficient LDS ring, 74 KB per
  // workgroup — the deferring sweep's 212 VGPRs alone would allow 2 as well)
  const int nb = par == 0 ? k.nblocks0 : k.nblocks;
  auto go = [&](auto kern) {
    hipLaunchKernelGGL(kern, dim3(nb), dim3(TJ), 0, s, k, par);
    return 0;
  };
  // odd iterations (par 0) defer their w term, even ones (par 1) apply both
  if (par == 0) with_kS<0>(k, go);
  else with_kS<2>(k, go);
  if (k.order == 3 && with_red) launch_red(k, par, s);
}

void launch_red(const KParams& k, int par, hipStream_t s) {
  // one workgroup streams ≈1.5 µs per 1000 slots (8192²'s 44 k slots: 71 µs
  // vs 10 µs for 64 blocks, tools/jobs/red_trace.sh): only tiny lists
  constexpr int red1_max = 4000;
  if (k.nslots <= red1_max) {
    if (par == 0) hipLaunchKernelGGL(kRed1<0>, dim3(1), dim3(kRed1Threads), 0, s, k, par);
    else hipLaunchKernelGGL(kRed1<2>, dim3(1), dim3(kRed1Threads), 0, s, k, par);
    return;
  }
  {
    // 8192² (44 k slots, 2.8 MB): 4 / 16 / 64 / 128 / 512 blocks = 26.7 / 13.5 /
    // 10.1 / 10.8 / 11.6 µs — load parallelism first, then the ticket fan-in
    const int rb = std::max(1, std::min(64, (k.nslots + 255) / 256));
    if (par == 0) hipLaunchKernelGGL(kRed<0>, dim3(unsigned(rb)), dim3(TJ), 0, s, k, par);
    else hipLaunchKernelGGL(kRed<2>, dim3(unsigned(rb)), dim3(TJ), 0, s, k, par);
  }
}

void launch_wait_sig(const KParams& k, unsigned long long target, hipStream_t s) {
  hipLaunchKernelGGL(kWaitSig, dim3(8), dim3(64), 0, s, k.st, target);
}

void launch_wflush(const KParams& k, hipStream_t s) {
  const int64_t n = k.nx * k.ny;
  const unsigned b = unsigned(std::min<int64_t>(4096, std::max<int64_t>(1, (n + 255) / 256)));
  hipLaunchKernelGGL(kWFlush, dim3(b), dim3(256), 0, s, k);
  hipLaunchKernelGGL(kWFlushDone, dim3(1), dim3(1), 0, s, k);
}

int resident_blocks_S(const KParams& k, int wm) {
  if (k.steps == 3) return resident_blocks_S3();
  if (k.steps == 2) return resident_blocks_S2();
  auto occ = [](auto kern) {
    int n = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, kern, TJ, 0) != hipSuccess) n = 0;
    return n;
  };
  return wm == 0 ? with_kS<0>(k, occ) : with_kS<2>(k, occ);
}

void launch_pack(const KParams& k, int b, hipStream_t s) {
  if (!k.has[DOWN] && !k.has[UP]) return;
  hipLaunchKernelGGL(kPack, dim3(unsigned((k.nx + 255) / 256)), dim3(256), 0, s, k, b);
}

void launch_push_test_write(const KParams& k, int me, hipStream_t s) {
  hipLaunchKernelGGL(kPushTestWrite, dim3(64), dim3(256), 0, s, k, me);
}
void launch_push_test_check(const KParams& k, int left, int right, int* bad, hipStream_t s) {
  hipLaunchKernelGGL(kPushTestCheck, dim3(64), dim3(256), 0, s, k, left, right, bad);
}

void launch_halo_import(const KParams& k, int b, hipStream_t s) {
  if (!k.push || (!k.has[LEFT] && !k.has[RIGHT])) return;
  const int64_t n = int64_t(k.hdep) * k.pitch;
  const unsigned g = unsigned(std::min<int64_t>(64, (n + 255) / 256));
  hipLaunchKernelGGL(kHaloImport, dim3(g), dim3(256), 0, s, k, b);
}

void launch_halo_seed(const KParams& k, int b, hipStream_t s) {
  if (!k.push || (!k.has[LEFT] && !k.has[RIGHT])) return;
  const int64_t n = int64_t(k.hdep) * k.pitch;
  const unsigned g = unsigned(std::min<int64_t>(64, (n + 255) / 256));
  hipLaunchKernelGGL(kHaloSeed, dim3(g), dim3(256), 0, s, k, b);
}

void launch_unpack(const KParams& k, int b, hipStream_t s) {
  if (!k.has[DOWN] && !k.has[UP]) return;
  hipLaunchKernelGGL(kUnpack, dim3(unsigned((k.nx + 255) / 256)), dim3(256), 0, s, k, b);
}

}  // namespace dev
}  // namespace pe
