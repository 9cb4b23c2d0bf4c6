// Device-resident Jacobi-PCG driver (host side).
//
// Reference: gradient_solver_mpi (poisson_mpi_cuda2.cu:687-982).  Where the
// reference assembles a/b/B on the CPU, copies them over, and then drives
// every iteration from the host (6 cudaDeviceSynchronize, 3 × 256 KiB D2H
// partial copies, 3 host MPI_Allreduce, host-staged halos), this driver:
//   * builds two 1-D chord tables (O(M+N) bytes) instead of 3 full arrays,
//   * keeps α, β, the stop test and the iteration count on the device,
//   * enqueues chunks of iterations (captured once into a hipGraph when the
//     transport allows it) and only looks at a pinned copy of the device
//     state once per chunk, with two chunks in flight so the GPU never idles
//     on the host,
//   * talks to peers through a stream-ordered DeviceComm (RCCL over xGMI).
#include <hip/hip_runtime_api.h>

#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstddef>
#include <cstring>
#include <deque>
#include <map>
#include <mutex>
#include <queue>
#include <limits>
#include <thread>

#include <unistd.h>

#include <rocprofiler-sdk-roctx/roctx.h>

#include "../hip/kernels.hpp"
#include "pe/device.hpp"
#include "solver_internal.hpp"

namespace pe {

using dev::DevState;
using dev::KParams;

using detail::clk;
using detail::field_alloc;
using detail::field_free;
using detail::field_try_alloc;
using detail::Range;
using detail::secs;


// Can the single-sweep kernel run this block?  It needs the fast arithmetic
// variant and neighbours at least two nodes deep in every split direction
// (its halo is two rows / columns deep).
static bool fused_possible(const Problem& P, const Block& b) {
  const int64_t min_rows = (P.M - 1) / b.Px, min_cols = (P.N - 1) / b.Py;
  return (b.Px == 1 || min_rows >= 2) && (b.Py == 1 || min_cols >= 2);
}

DeviceSolver::DeviceSolver(const Problem& prob, const Block& blk, DeviceComm* comm, const SolveOptions& opt)
    : prob_(prob), blk_(blk), comm_(comm), opt_(opt), kp_(std::make_unique<KParams>()) {
  const auto t_ctor = clk::now();
  // PE_CTOR_TRACE=1: wall time of each construction phase → stderr
  const bool ctor_trace = std::getenv("PE_CTOR_TRACE") && std::atoi(std::getenv("PE_CTOR_TRACE")) >= 1;
  auto t_mark = t_ctor;
  auto mark = [&](const char* phase) {
    if (!ctor_trace) return;
    PE_HIP_CHECK(hipDeviceSynchronize());
    const auto now = clk::now();
    std::fprintf(stderr, "[pe] ctor %-14s %8.3f ms\n", phase, 1e3 * secs(t_mark, now));
    t_mark = now;
  };
  if (!comm_) {
    self_ = std::make_unique<SelfDeviceComm>();
    comm_ = self_.get();
  }
  if (opt_.algo < 0 || opt_.algo > 4)
    throw std::invalid_argument("algo: 0 auto, 1 classic, 2 fused, 3 two-step, 4 three-step (got " +
                                std::to_string(opt_.algo) + ")");
  const bool can_fuse = opt_.variant == 0 && fused_possible(prob_, blk_);
  if (opt_.algo >= 2 && !can_fuse)
    throw std::invalid_argument("single-sweep algorithm needs variant 0 and >= 2 rows/columns per split block");
  fused_ = opt_.algo >= 2 || (opt_.algo == 0 && can_fuse);
  // Several iterations per sweep (fused2.hip: 2, fused3.hip: 3): single-rank
  // blocks of ≥ 8 × 8 nodes, or row slabs (Py = 1) over a multi-rank
  // transport of ≥ 4s rows per rank (the 2s-deep halo comes from one
  // neighbour and the pushed edge rows are distinct).  Every input is global: every rank
  // decides the same.  algo 3 / 4 force two / three steps; auto takes three
  // where it can (PE_STEPS=1/2/3 caps the iterations per sweep).
  {
    auto single = [&](int64_t m) { return comm_->size() == 1 && blk_.Px * blk_.Py == 1 && blk_.nx >= m && blk_.ny >= m; };
    auto slabs = [&](int64_t m) {
      return comm_->size() > 1 && blk_.Py == 1 && (prob_.M - 1) / blk_.Px >= m && prob_.N - 1 >= m;
    };
    // 2-D splits (three-step only): the 6-deep halo through the comm's
    // exchange — y strips packed after the sweep, then the x rows with their
    // halo columns (corners) — from blocks of >= 12 rows and columns each
    auto grid2d = [&](int64_t m) {
      return comm_->size() > 1 && blk_.Py > 1 && (prob_.M - 1) / blk_.Px >= m && (prob_.N - 1) / blk_.Py >= m;
    };
    // virtual ranks on one device (device_solve_group: no comm, a split block;
    // the group driver exchanges the halos and sums the sweeps' sums)
    auto vgroup = [&](int64_t m) {
      return comm_->size() == 1 && blk_.Px * blk_.Py > 1 && (prob_.M - 1) / blk_.Px >= m &&
             (prob_.N - 1) / blk_.Py >= m;
    };
    const bool two_ok = fused_ && (single(8) || slabs(8));
    const bool three_ok = fused_ && (single(8) || slabs(12) || grid2d(12) || vgroup(12));
    if (opt_.algo == 3 && !two_ok)
      throw std::invalid_argument("two-step sweep: single-rank blocks of >= 8 x 8 nodes or row slabs of >= 8 rows");
    if (opt_.algo == 4 && !three_ok)
      throw std::invalid_argument(
          "three-step sweep: single-rank blocks of >= 8 x 8 nodes, row slabs of >= 12 rows or 2-D blocks of >= 12 x 12");
    // auto: every single-rank block the LDS-resident kernel cannot hold
    // (1x MI355X, fresh processes, T_solver two-step vs single sweep:
    // 1600×2400 0.110 vs 0.127 s, 2048² 0.113 vs 0.133, 4096² 0.378 vs 0.584,
    // 8192² 2.60 vs 3.24, 16384² 13.7 vs 21.7; the resident kernel keeps
    // ≤ 800×1200: 0.044 vs 0.059 s — profiles/r3_grids_two.txt).  The
    // estimate mirrors setup_resident's geometry test.
    bool resident_likely = false;
    {
      const char* r = std::getenv("PE_RESIDENT");
      int ncu = 256, dv = 0;
      if (hipGetDevice(&dv) == hipSuccess) (void)hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dv);
      const int64_t ns = (blk_.ny + dev::kFSW - 1) / dev::kFSW;
      if (!(r && std::atoi(r) == 0) && opt_.variant == 0 && ns <= ncu) {
        const int64_t ntr = std::max<int64_t>(1, std::min<int64_t>(ncu / ns, blk_.nx / 8));
        resident_likely = blk_.nx >= 2 * ntr && (blk_.nx + ntr - 1) / ntr <= dev::kResMaxRows &&
                          ntr * ns <= dev::kResMaxTiles;
      }
    }
    bool auto_ms = slabs(8) || grid2d(12) || vgroup(12) || !resident_likely;
    int want = 3;
    if (const char* e = std::getenv("PE_STEPS")) want = std::max(1, std::min(3, std::atoi(e)));
    steps_ = 1;
    if (opt_.algo == 3) steps_ = 2;
    else if (opt_.algo == 4) steps_ = 3;
    else if (opt_.algo == 0 && auto_ms)
      steps_ = (want >= 3 && three_ok) ? 3 : (want >= 2 && two_ok) ? 2 : 1;
    sstep_ = steps_ > 1;
  }

  mark("start");
  stream_ = acquire_stream();  // (pooled: set_device created one — runtime.cpp)
  mark("stream");
  // Peer access of this rank's device toward every rank's (first cross-device
  // run diagnostics: the halo push and the in-sweep sums map peers' memory):
  // 1 / 0 hipDeviceCanAccessPeer, -1 the same physical device, -2 a device this
  // process cannot see (another node, or masked by HIP_VISIBLE_DEVICES).
  // Devices are compared by PCI location, not by process-local ordinals, and
  // gathered 64 ranks per collective (the comms' host scratch size); a failure
  // leaves the diagnostics empty and never aborts construction.
  if (comm_->size() > 1) {
    // key = (host hash << 32) | PCI domain / bus / device: exact in a double
    // (52 bits), so GPUs of different nodes never compare equal.  Every rank
    // runs every collective round whatever failed locally (a failure only
    // turns its own contribution into -1).
    const int P = comm_->size();
    auto host_hash = []() -> int64_t {
      char name[256] = {0};
      if (gethostname(name, sizeof(name) - 1) != 0) return 0;
      uint64_t h = 1469598103934665603ull;  // FNV-1a
      for (const char* c = name; *c; ++c) h = (h ^ uint64_t(uint8_t(*c))) * 1099511628211ull;
      return int64_t((h ^ (h >> 20) ^ (h >> 40)) & 0xFFFFF);
    };
    const int64_t hh = host_hash();
    auto pci_key = [hh](int dv) -> double {
      int dom = 0, bus = -1, dev = 0;
      if (hipDeviceGetAttribute(&dom, hipDeviceAttributePciDomainID, dv) != hipSuccess ||
          hipDeviceGetAttribute(&bus, hipDeviceAttributePciBusId, dv) != hipSuccess ||
          hipDeviceGetAttribute(&dev, hipDeviceAttributePciDeviceId, dv) != hipSuccess) {
        (void)hipGetLastError();
        return -1.0;
      }
      return double((hh << 32) | (int64_t(dom & 0xFFFF) << 16) | (int64_t(bus & 0xFF) << 8) | int64_t(dev & 0xFF));
    };
    int mydev = -1, ndev = 0;
    if (hipGetDevice(&mydev) != hipSuccess || hipGetDeviceCount(&ndev) != hipSuccess) {
      (void)hipGetLastError();
      mydev = -1;
      ndev = 0;
    }
    const double mykey = mydev >= 0 ? pci_key(mydev) : -1.0;
    std::vector<double> keys(size_t(P), -1.0);
    for (int c0 = 0; c0 < P; c0 += 64) {
      const int n = std::min(64, P - c0);
      double chunk[64];
      for (int i = 0; i < n; ++i) chunk[i] = c0 + i == comm_->rank() ? mykey : -1.0;
      comm_->host_max(chunk, n, stream_);
      for (int i = 0; i < n; ++i) keys[size_t(c0 + i)] = chunk[i];
    }
    for (int r = 0; r < P; ++r)
      if (r != comm_->rank() && mykey >= 0 && keys[size_t(r)] == mykey) shared_dev_ = true;
    std::vector<int> pa(size_t(P), -1);
    for (int r = 0; r < P && mykey >= 0; ++r) {
      const double key = keys[size_t(r)];
      if (key < 0 || key == mykey) continue;
      int d = -1;
      for (int i = 0; i < ndev && d < 0; ++i)
        if (pci_key(i) == key) d = i;
      if (d < 0) {
        pa[size_t(r)] = -2;
        continue;
      }
      int can = 0;
      if (hipDeviceCanAccessPeer(&can, mydev, d) != hipSuccess) {
        (void)hipGetLastError();
        can = 0;
      }
      pa[size_t(r)] = can;
    }
    peer_access_ = std::move(pa);
  }
  KParams& k = *kp_;
  std::memset(&k, 0, sizeof(KParams));
  const int64_t nx = blk_.nx, ny = blk_.ny;
  int ti = fused_ ? 16 : 8;  // 8192² sweeps: classic 8 rows, single-sweep 16 (4 halo rows per item)
  int ti_env = 0;
  if (const char* e = std::getenv("PE_TI")) ti_env = std::atoi(e);
  if (ti_env > 0) ti = ti_env;

  int64_t strips = 0, rows_hi = nx + 2, cols_hi = ny + 2;
  if (fused_) {
    // Planes: columns -1 .. 124·nstrips+2 (strip loads never leave the row),
    // rows -1 .. nx+4 (two prefetch rows past the halo).  x[b] interleaves the
    // r and p planes by row.  Two-step sweep: halo depth 4 — columns -3 ..
    // 120·nstrips+4, rows -3 .. nx+6.
    fsw_ = steps_ >= 3 ? dev::kFSW3 : steps_ == 2 ? dev::kFSW2 : dev::kFSW;
    hdep_ = 2 * steps_;
    xorg_ = steps_ >= 3 ? dev::kHL3 - 1 : hdep_ - 1;
    strips = (ny + fsw_ - 1) / fsw_;
    plane_ = ((fsw_ * strips + 2 * hdep_ + 7) / 8) * 8;
    // Three-step: strip s loads columns 48s-7 .. 48s+56 (one per lane) and
    // outputs 48s+1 .. 48s+48.  Element 0 of a row is column -7 and the
    // plane a whole number of 128-B lines, so every strip's loads are 4 whole
    // lines and its stores 6 whole 64-B segments of r, p and w (52 outputs of
    // 64 loaded straddled 64-B segments: partial writes from two strips, and
    // 5 lines touched for 4 lines of data).
    if (steps_ >= 3) plane_ = ((xorg_ + fsw_ * (strips - 1) + 64 - dev::kHL3 + 1 + 15) / 16) * 16;
    const int64_t rows = nx + 2 * hdep_ + 2;
    xsize_ = ((rows * 2 * plane_ + 64 + 31) / 32) * 32;
    wsize_ = ((rows * plane_ + 64 + 31) / 32) * 32;
    k.pitch = 2 * plane_;
    k.wpitch = plane_;
    k.poff = plane_;
    fields_ = static_cast<double*>(field_alloc(sizeof(double) * xsize_));
    xalt_ = static_cast<double*>(field_alloc(sizeof(double) * xsize_));
    walt_ = static_cast<double*>(field_alloc(sizeof(double) * wsize_));
    mark("field allocs");
    set_fused_fields(fields_, xalt_, walt_);
    hsize_ = std::max<int64_t>(1, nx) * 2 * hdep_;  // y strips: hdep columns of r and p per owned row
    // (multi-step: rows -hdep .. nx+hdep+2, columns -hdep .. fsw·strips+hdep+3)
    rows_hi = sstep_ ? nx + hdep_ + 2 : nx + 3;
    cols_hi = sstep_ ? fsw_ * strips + hdep_ + 3 : dev::kFSW * strips + 3;
    tab_lo_ = sstep_ ? -hdep_ : -1;
    if (steps_ >= 3) {  // the last strip's last lane + 3; the first strip's lane 0 is column -xorg
      cols_hi = fsw_ * (strips - 1) + 64 - dev::kHL3 + 3;
      tab_lo_ = -(xorg_ + 1);
    }
  } else {
    strips = (ny + dev::kSW - 1) / dev::kSW;
    const int64_t A = blk_.alloc;
    PE_HIP_CHECK(hipMalloc(&fields_, sizeof(double) * A * 4));
    k.pitch = blk_.pitch;
    k.wpitch = blk_.pitch;
    k.r = fields_ + blk_.base;
    k.w = fields_ + A + blk_.base;
    k.p[0] = fields_ + 2 * A + blk_.base;
    k.p[1] = fields_ + 3 * A + blk_.base;
    hsize_ = std::max<int64_t>(1, nx);
  }
  mark("fields");
  const int64_t nrow_tab = rows_hi - tab_lo_ + 1, ncol_tab = cols_hi - tab_lo_ + 1;
  const int64_t ntab = nrow_tab * 4 + ncol_tab * 4;
  PE_HIP_CHECK(hipMalloc(&tables_, sizeof(double) * ntab));
  PE_HIP_CHECK(hipMalloc(&rowcls_, sizeof(int) * nrow_tab * 4));
  PE_HIP_CHECK(hipMalloc(&halo_, sizeof(double) * hsize_ * 4));
  PE_HIP_CHECK(hipMalloc(&st_, sizeof(DevState)));
  PE_HIP_CHECK(hipHostMalloc(&hst_, sizeof(DevState) * 2, hipHostMallocDefault));
  std::memset(hst_, 0, sizeof(DevState) * 2);
  PE_HIP_CHECK(hipEventCreateWithFlags(&ev_[0], hipEventDisableTiming));
  PE_HIP_CHECK(hipEventCreateWithFlags(&ev_[1], hipEventDisableTiming));
  PE_HIP_CHECK(hipEventCreateWithFlags(&ev_sync_, hipEventDisableTiming));
  PE_HIP_CHECK(hipEventCreate(&t0_));
  PE_HIP_CHECK(hipEventCreate(&t1_));

  k.fused = fused_ ? 1 : 0;
  k.steps = steps_;
  k.hdep = hdep_;
  k.pre_load = 1;  // first item's list entry + row classes loaded at kernel entry (fused3.hip Pre3)
  k.dring = 1;     // band rows read 1/D from the LDS ring (+0.7 % at 8192², profiles/r5_ab_kernel.txt)
  // SIMD priority turns (fused3.hip prio_turn), opt-in: 1-GPU 2048² and
  // 1600×2400 T_iterate −0.8-1.5 % at PE_PRIO=10, but the 2-rank blocks of
  // 2048² / 1600×2400 +2-7 % (20.2 vs 18.9 µs per iteration), 8192² −4-6 %
  // it/s, the 8-rank slab and 4×2 blocks neutral — profiles/r5_prio.txt
  k.prio = std::getenv("PE_PRIO") ? std::max(0, std::min(20, std::atoi(std::getenv("PE_PRIO")))) : 0;
  k.stage = !(std::getenv("PE_STAGE") && std::atoi(std::getenv("PE_STAGE")) == 0);
  k.xorg = xorg_;
  k.nx = nx;
  k.ny = ny;
  k.M = prob_.M;
  k.N = prob_.N;
  k.gi0 = blk_.i0 - 1;
  k.gj0 = blk_.j0 - 1;
  k.A1 = prob_.A1;
  k.A2 = prob_.A2;
  k.h1 = prob_.h1();
  k.h2 = prob_.h2();
  k.eps = prob_.eps();
  k.inv_eps = 1.0 / k.eps;
  k.h1sq = k.h1 * k.h1;
  k.h2sq = k.h2 * k.h2;
  k.nih1 = -1.0 / k.h1;
  k.nih2 = -1.0 / k.h2;
  k.cx = prob_.cx;
  k.cy = prob_.cy;
  k.F = prob_.F;
  k.u_scale = prob_.u_scale();
  k.tol = prob_.tol;
  k.weighted = prob_.norm == Norm::Weighted ? 1 : 0;
  k.max_iter = prob_.iter_cap();
  for (int d = 0; d < 4; ++d) k.has[d] = blk_.has(d) ? 1 : 0;
  // tables start at local index tab_lo_; the kernels index them by (local + 1)
  k.colT = tables_ - (tab_lo_ + 1) * 4;
  k.rowcls = rowcls_ - (tab_lo_ + 1) * 4;
  k.rowT = tables_ + nrow_tab * 4 - (tab_lo_ + 1) * 4;
  k.send_dn = halo_;
  k.send_up = halo_ + hsize_;
  k.recv_dn = halo_ + 2 * hsize_;
  k.recv_up = halo_ + 3 * hsize_;
  k.st = st_;
  k.check_tol = opt_.check_tol ? 1 : 0;
  // Failure-detection hooks: PE_FAULT_INJECT=nan@iter:K poisons
  // the reduced sums after iteration K (the solver must stop with a
  // non-finite status), PE_FAULT_INJECT=stall (or stall@rank:R, one rank
  // only) makes the host believe the device never finishes (the watchdog
  // must fire); PE_WATCHDOG_S sets the
  // no-progress limit of the host loop.
  if (const char* e = std::getenv("PE_FAULT_INJECT")) {
    const std::string f = e;
    if (f.rfind("nan@iter:", 0) == 0) k.fault_iter = std::atoll(f.c_str() + 9);
    if (f.rfind("zero@iter:", 0) == 0) k.fault_zero = std::atoll(f.c_str() + 10);
    if (f == "stall") fault_stall_ = true;
    // stall@rank:R — only rank R hangs (its watchdog fires and aborts the
    // communicator; the peers then see the transport fail, not a hang)
    if (f.rfind("stall@rank:", 0) == 0 && std::atoi(f.c_str() + 11) == blk_.rank) fault_stall_ = true;
    // slow@rank:R,us:X — rank R's sweeps idle X µs before their cross-rank
    // sum (the peers' T_MPI must show it: iterations × X)
    if (f.rfind("slow@rank:", 0) == 0 && std::atoi(f.c_str() + 10) == blk_.rank) {
      const size_t u = f.find("us:");
      k.slow_ticks = u == std::string::npos ? 0 : (long long)(std::atof(f.c_str() + u + 3) * 100.0);
    }
    // drift@iter:K[,amp:X] — w(M/2, N/2) += X behind the recurrence's back
    // (the end-of-solve residual check must see the gap; three-step restarts)
    if (f.rfind("drift@iter:", 0) == 0) {
      fault_drift_ = std::atoll(f.c_str() + 11);
      const size_t u = f.find("amp:");
      if (u != std::string::npos) fault_drift_amp_ = std::atof(f.c_str() + u + 4);
    }
  }
  if (const char* e = std::getenv("PE_RESID_GAP")) gap_bound_ = std::atof(e);
  if (const char* e = std::getenv("PE_WATCHDOG_S")) watchdog_s_ = std::atof(e);
  if (opt_.keep_history) {  // per-iteration ‖Δw‖ on the device (capped at 2²⁴ iterations)
    k.hist_n = std::min<long long>(prob_.iter_cap(), 1LL << 24);
    PE_HIP_CHECK(hipMalloc(&hist_, sizeof(double) * size_t(std::max<long long>(1, k.hist_n))));
    k.hist = hist_;
  }
  // Work decomposition: wave strips (128 columns classic, 124 output
  // columns single-sweep) × `ti`-row chunks, dealt round-robin (chunk-major)
  // to a persistent grid of ~16 waves per CU, so the waves running at any
  // moment cover a compact window of rows (measured: long per-wave row
  // ranges spread over the whole array run 25 % slower than 8-16-row items
  // despite their halo-row re-reads, which then hit L2/MALL).
  // Persistent grid: exactly the resident waves (a second partial round of
  // blocks would run after the first finishes — a tail of up to one item
  // per wave).
  int cus = 256;
  {
    int dev = 0;
    PE_HIP_CHECK(hipGetDevice(&dev));
    PE_HIP_CHECK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
  }
  cus_ = cus;
  k.ncu = cus;
  // rows per item and item order first: they select the sweep kernel variant
  // whose occupancy sizes the grid
  const double npts = double(nx) * double(ny);
  const bool big = npts >= double(1 << 24), huge = npts > double(1 << 26);
  // Single-sweep item order and rows per item (profiles/r2_order.txt,
  // profiles/r2_bench_static.txt; one memory placement per comparison):
  //  * blocks > 2²⁶ nodes (16384²): the per-XCD dynamic queue, 18 rows —
  //    with ≈45 items per wave a static layout's per-wave durations drift
  //    apart (2150 vs 2195 µs per iteration static 24 rows);
  //  * 2²⁴ .. 2²⁶ (8192², the 2-rank 8192² block): the cost-aware static LPT
  //    layout, 24 rows, untuned — no item-sum reduction kernel, no queue
  //    atomics, and with 6-12 items per wave its load is even (8192²: 540-542
  //    vs 548 µs dynamic; 2-rank block 315-318 vs 333);
  //  * smaller blocks: static, rows per item tuned below (small blocks: the
  //    queue's pull latency and the reduction launch never pay — 4-rank block
  //    155-159 vs 188 µs, 2400×3200 80 vs 109).
  if (fused_ && ti_env == 0) ti = huge ? 18 : big ? 24 : 10;
  k.order = (fused_ && huge) ? 3 : 0;
  if (sstep_) {  // static LPT layout only; taller items (2·hdep pipeline-fill rows each)
    // (three-step beyond 2²⁶ nodes: 128 rows — 16384² 978 vs 999 µs/iteration
    // at 80, one placement, profiles/r3_ti_final.txt)
    if (ti_env == 0) ti = steps_ >= 3 ? (huge ? 448 : npts >= double(1 << 25) ? 112 : big ? 80 : 48) : (big ? 40 : 24);
    ti = std::max(4, std::min(ti, steps_ >= 3 ? dev::kTImax3 : dev::kTImax2));
    k.order = 0;
  }
  if (const char* e = std::getenv("PE_ORDER")) k.order = std::atoi(e);
  if (!fused_ && k.order > 1) k.order = 0;
  if (sstep_) k.order = 0;
  k.ti = (fused_ && ti_env < 0) ? 1 << 20 : ti;  // bands mode: long items → general kernel
  int per_cu = fused_ ? dev::resident_blocks_S(k, 2) : dev::resident_blocks_classic(opt_.variant);
  if (per_cu <= 0) per_cu = 4;
  int wave_cap = cus * per_cu * dev::kWPB;
  // PE_TI=-1 (single-sweep): "bands" — one item per resident wave, the rows
  // split into wave_cap/nstrips bands that the waves of a band march down
  // together (halo rows re-read once per band, perfect balance).
  if (fused_ && ti_env < 0) {
    const int64_t bands = std::max<int64_t>(1, wave_cap / std::max<int64_t>(1, strips));
    ti = int((nx + bands - 1) / bands);
  }
  k.nstrips = int(strips);
  int wave_cap0 = wave_cap;
  if (fused_) {
    const int per0 = dev::resident_blocks_S(k, 0);
    if (per0 > 0) wave_cap0 = cus * per0 * dev::kWPB;
  }
  wave_cap_ = std::min(wave_cap, wave_cap0);
  wave_caps_[0] = wave_cap;
  wave_caps_[1] = wave_cap0;
  // Rows per item: fixed (PE_TI, the classic path, blocks ≥ 2²⁴ nodes), or
  // tuned below among kTiCands for smaller static single sweeps (the best depends
  // on the block: 2400×3200 18 rows 76 µs vs 84 at 10; 1600×2400 and the
  // 8-rank 8192² block 10 rows — profiles/r2_mid_tune.txt).
  static constexpr int kTiCands[4] = {8, 10, 14, 18};
  tune_ti_ = fused_ && ti_env == 0 && k.order == 0 && npts >= double(1 << 20) && !big;
  // Two-step sweep: tuned among {16, 24, 32, 40, 48} below 2²⁵ nodes (the
  // best height moves with the block: 1600×2400 16 rows 39.9 µs/iter vs 47.7
  // at 40, 2048² 24 rows, 4096² 32 rows 102.3 vs 108.7; 8192² and 16384²
  // within ±2 % over 24-48 rows: fixed 40 — one placement per grid,
  // tools/ti_probe.py, profiles/r3_ti_probe.txt).  Three-step sweep (12
  // pipeline-fill rows per item): among {32 .. 96} (2400×3200 32 rows 45.7
  // µs/iter vs 57.1 at 64, 1600×2400 and 2048² 48, 4096² 64); fixed above,
  // with the aligned 48-column strips: 8192² 112 rows (240-247 µs/iter vs
  // 253-256 at 80, 266-271 at 104, 249 at 120, 255 at 128 — the same on two
  // boxes and with padded rows; a scan of 64-224 found only 132 as good),
  // 16384² 448 (867 vs 880 at 272, 891-899 at 256, 975 at 288, 934-940 at
  // 512; 256 was 939 vs 959 at 128 on another box) — tools/layout_probe.py,
  // tools/block_probe.py, profiles/r4_ti48.txt.
  static constexpr int kTiCands2[5] = {16, 24, 32, 40, 48};
  static constexpr int kTiCands3[5] = {32, 48, 64, 80, 96};
  const int* tic = steps_ >= 3 ? kTiCands3 : kTiCands2;
  // (from 2²⁰ nodes: a tuned layout depends on the timings, so two
  // constructions of a smaller block — a checkpointed solve and its resume —
  // could lay it out differently and the resume would not be bitwise; round 5
  // tuned from 2¹⁷ and test_three_step_checkpoint_resume_bitwise caught it)
  if (sstep_) tune_ti_ = ti_env == 0 && npts >= double(1 << 20) && npts < double(1 << 25);
  // Three-step static layout by block size, one placement per block
  // (tools/layout_probe.py, profiles/r4_layout2.txt, µs per iteration): the
  // LPT layout of whole items for ≥ 5·10⁷ nodes (8192²: 253 vs 260 filling,
  // 275 equal-cost), the filling layout from 2.5·10⁷ (the 2-rank 8192² block:
  // 137 vs 145-147), the equal-cost one below (4-rank block 83.4-84.2 vs
  // 87.4-87.9 LPT, 8-rank block 45.1 vs 47.6-49.6); tuned blocks also try the
  // other two at their best rows per item.
  if (steps_ >= 3) lay_name_ = npts >= 5e7 ? "lpt" : npts >= 2.5e7 ? "fill" : "equal";
  if (const char* e = std::getenv("PE_TI_TUNE")) tune_ti_ = tune_ti_ && std::atoi(e) != 0;
  // Tuning candidates: the fixed set plus, for q = 1..5 items per wave, the
  // smallest item height that gives every wave at most q items — a static
  // layout's sweep lasts as long as its most loaded wave, and 3.4 items per
  // wave means a quarter of the waves runs a 4th item while the rest idle
  // (8-rank 8192² block at 10 rows: busy fraction 0.74-0.78,
  // tools/stamp_probe.py).  (Round 5 measured one short item per wave — down
  // to 4 rows — on the 2-rank blocks of 1600×2400 and 2048²: 86.9-88.2 µs per
  // sweep against 58.9-64 at 32-96 rows; the 12 pipeline-fill rows of a short
  // item cost more than the waves it adds — profiles/r5_ab_layout.txt.)
  std::vector<int> ti_cands;
  if (tune_ti_) {
    ti_cands.assign(kTiCands, kTiCands + 4);
    if (sstep_) ti_cands.assign(tic, tic + 5);
    // taller items for the largest tuned blocks (4096²: 30 rows 158 µs vs 165
    // at 18, one placement, profiles/r2_ti_big.txt)
    if (npts >= 12e6 && !sstep_) ti_cands.insert(ti_cands.end(), {24, 30});
    const int64_t W = std::max(dev::kWPB, wave_cap_);
    const int tlo = sstep_ ? tic[0] : kTiCands[0], thi = steps_ >= 3 ? 128 : sstep_ ? dev::kTImax2 : 40;
    for (int q = 2; q <= 5; ++q)
      for (int t = tlo; t <= thi; ++t)
        if (int64_t(strips) * ((nx + t - 1) / t) <= int64_t(q) * W) {
          ti_cands.push_back(t);
          break;
        }
    std::sort(ti_cands.begin(), ti_cands.end());
    ti_cands.erase(std::unique(ti_cands.begin(), ti_cands.end()), ti_cands.end());
  }
  const int ti_min = tune_ti_ ? ti_cands.front() : ti;
  set_items(ti);
  // block partials: interior grid, then (overlap) the boundary grid after it
  const int64_t npart = 8 * std::max<int64_t>(2 * int64_t(std::max(wave_cap, wave_cap0) / dev::kWPB + 1), 4096);
  // item-sum slots: one per item, more when setup_items splits tail items
  // (static sweeps split heavy items into up to ti pieces: setup_items)
  const int64_t nitems_max = strips * ((nx + ti_min - 1) / ti_min);
  nslot_cap_ = fused_ ? int((k.order == 0 ? ti + 1 : 2) * nitems_max + 64) : 0;
  PE_HIP_CHECK(hipMalloc(&partial_, sizeof(double) * (npart + 8 * int64_t(nslot_cap_))));
  k.partial = partial_;
  k.itemsum = fused_ ? partial_ + npart : nullptr;
  k.ih1sq = 1.0 / k.h1sq;
  k.ih2sq = 1.0 / k.h2sq;
  k.D_in = (1.0 + 1.0) / k.h1sq + (1.0 + 1.0) / k.h2sq;
  k.D_out = (k.inv_eps + k.inv_eps) / k.h1sq + (k.inv_eps + k.inv_eps) / k.h2sq;
  k.dinv_in = 1.0 / ((1.0 + 1.0) * k.ih1sq + (1.0 + 1.0) * k.ih2sq);
  k.dinv_out = 1.0 / ((k.inv_eps + k.inv_eps) * k.ih1sq + (k.inv_eps + k.inv_eps) * k.ih2sq);
  mark("buffers");
  build_tables(rows_hi, cols_hi);
  mark("tables");
  if (const char* e = std::getenv("PE_P2P_TIMEOUT_S")) put_timeout_s_ = std::max(0.1, std::atof(e));
  setup_halo_push();
  setup_halo_put();
  // The placement search times the item layout the solve will run (after
  // setup_items): its best class then reaches the early-stop rate (8192²
  // static layout 0.536-0.545 ms vs 0.564-0.567 for the plain walk), so it
  // stops after 2-3 tries instead of 8 — construction 0.10-0.14 vs 0.15-0.25 s,
  // the same iteration speed (profiles/r2_bench_psearch.txt).
  if (comm_->size() > 1) measure_exchange();  // (diagnostic: the comm's exchange, bench JSON)
  setup_items();
  mark("items");
  if (fused_) choose_placement();
  mark("placement");
  setup_resident();
  mark("resident");
  if (tune_ti_ && !resident_) {
    // time S_0 + 1 + 4 local sweeps per candidate on real data (no
    // communication: the in-sweep cross-rank sum is not set up yet) and keep
    // the fastest; every rank tunes its own block
    Range range("pe.tune_rows_per_item");
    // candidates: the fixed set plus, for q = 2..5 items per wave, the
    // smallest item height that gives every wave at most q items — a static
    // layout's sweep lasts as long as its most loaded wave, and 3.4 items per
    // wave means a quarter of the waves runs a 4th item while the rest idle
    // (8-rank 8192² block at 10 rows: busy fraction 0.74-0.78, tools/stamp_probe.py)
    // (candidates: ti_cands above)
    std::vector<int> cands = ti_cands;
    float best_ms = 0.f;
    int best = ti;
    // one candidate: S_0 + 1 + kTimed local sweeps on real data, the last
    // kTimed timed (round 3: S_0 + 2 + 6 — construction is inside T_solver)
    constexpr int kTimed = 4;
    // Trials run pipelined: the host lays out trial i+1 while the GPU times
    // trial i (the list upload is stream-ordered after those sweeps), and
    // layouts already built come from the cache (the finalists, the final
    // one).  The host layouts were ≈ half of the tuning's time (4096²: 1-2.4
    // ms each against 1.7-2 ms of timing, PE_CTOR_TRACE=3,
    // profiles/r6_ctor_tuning.txt).
    struct Trial {
      int ti;
      std::string lay;
    };
    lay_cache_.clear();
    lay_cache_on_ = true;
    auto run_trials = [&](const std::vector<Trial>& trials) {
      std::vector<float> out;
      for (size_t i = 0; i <= trials.size(); ++i) {
        const auto tl = clk::now();
        if (i < trials.size()) {
          lay_name_ = trials[i].lay;
          set_items(trials[i].ti);
          setup_items();  // (its upload waits for trial i-1's sweeps)
        }
        const auto tg = clk::now();
        if (i > 0) {
          PE_HIP_CHECK(hipEventSynchronize(t1_));
          float ms = 0.f;
          PE_HIP_CHECK(hipEventElapsedTime(&ms, t0_, t1_));
          out.push_back(ms);
          if (ctor_trace)
            std::fprintf(stderr, "[pe] ctor   tune %3d rows %-5s %8.4f ms per sweep\n", trials[i - 1].ti,
                         trials[i - 1].lay.c_str(), ms / float(kTimed));
        }
        if (i == trials.size()) break;
        enqueue_init();
        dev::launch_S(*kp_, 1, stream_);
        dev::launch_S(*kp_, 0, stream_);
        PE_HIP_CHECK(hipEventRecord(t0_, stream_));
        for (int j = 0; j < kTimed; ++j) dev::launch_S(*kp_, (j + 1) & 1, stream_);
        PE_HIP_CHECK(hipEventRecord(t1_, stream_));
        if (ctor_trace)
          std::fprintf(stderr, "[pe] ctor   tune %3d rows %-5s layout %7.3f ms\n", trials[i].ti, trials[i].lay.c_str(),
                       1e3 * secs(tl, tg));
      }
      return out;
    };
    {
      std::vector<Trial> tr;
      for (int cand : cands) tr.push_back(Trial{cand, lay_name_});
      const std::vector<float> ms = run_trials(tr);
      for (size_t i = 0; i < tr.size(); ++i) {
        ti_ms_.push_back(ms[i] / float(kTimed));
        ti_rows_.push_back(tr[i].ti);
        if (best_ms == 0.f || ms[i] < best_ms) {
          best_ms = ms[i];
          best = tr[i].ti;
        }
      }
    }
    // three-step: the other static layouts at the best height
    std::string keep = lay_name_;
    struct Tried {
      int ti;
      std::string lay;
      float ms;
    };
    std::vector<Tried> tried;
    for (size_t i = 0; i < ti_rows_.size(); ++i) tried.push_back(Tried{ti_rows_[i], lay_name_, ti_ms_[i] * float(kTimed)});
    if (steps_ >= 3 && !std::getenv("PE_LAYOUT")) {
      const std::string base = lay_name_;
      std::vector<Trial> tr;
      for (const char* alt : {"equal", "fill", "lpt"})
        if (base != alt) tr.push_back(Trial{best, alt});
      const std::vector<float> ms = run_trials(tr);
      for (size_t i = 0; i < tr.size(); ++i) {
        ti_ms_.push_back(ms[i] / float(kTimed));
        ti_rows_.push_back(-best);  // (negative: a layout candidate at that height)
        tried.push_back(Tried{best, tr[i].lay, ms[i]});
        if (ms[i] < best_ms) {
          best_ms = ms[i];
          keep = tr[i].lay;
        }
      }
    }
    // Finalists: the two fastest candidates timed once more, each keeping its
    // faster timing — the GPU clock ramps up during construction, so the first
    // candidates were timed slow, and two within ≈2 % swapped places from one
    // process to the next (2400×3200: equal layout at 80 rows or filling at
    // 96, T_iterate 0.099 vs 0.095 s, profiles/r5_prio.txt).  Three-step only.
    if (steps_ >= 3 && tried.size() >= 2) {
      std::stable_sort(tried.begin(), tried.end(), [](const Tried& a, const Tried& b) { return a.ms < b.ms; });
      const std::vector<float> ms = run_trials({Trial{tried[0].ti, tried[0].lay}, Trial{tried[1].ti, tried[1].lay}});
      for (int f = 0; f < 2; ++f) {
        Tried& t = tried[size_t(f)];
        ti_ms_.push_back(ms[size_t(f)] / float(kTimed));
        ti_rows_.push_back(t.lay == keep && t.ti == best ? best : -t.ti);
        t.ms = std::min(t.ms, ms[size_t(f)]);
      }
      const Tried& w = tried[0].ms <= tried[1].ms ? tried[0] : tried[1];
      best = w.ti;
      keep = w.lay;
    }
    // the three best heights (any layout), for the overlap's own layout: its
    // boundary-first filling list ranks them differently (8-rank slab of
    // 8192²: 64, 80 and 96 rows tie within 1 % on the plain layout, 117-119 µs
    // per sweep, but the overlapped sweep runs 146, 157 and 128 µs —
    // profiles/r6_overlap_ti.txt)
    std::stable_sort(tried.begin(), tried.end(), [](const Tried& a, const Tried& b) { return a.ms < b.ms; });
    ti_alt_ = {best};
    for (const Tried& t : tried)
      if (ti_alt_.size() < 3 && std::find(ti_alt_.begin(), ti_alt_.end(), t.ti) == ti_alt_.end()) ti_alt_.push_back(t.ti);
    lay_name_ = keep;
    set_items(best);
    setup_items();
    lay_cache_on_ = false;
    lay_cache_.clear();
  }
  if (fused_ && std::getenv("PE_STAMPS") && std::atoi(std::getenv("PE_STAMPS")) == 1) {
    const size_t nw = size_t(dev::kWPB) * size_t(std::max(k.nblocks, k.nblocks0));
    nstamps_ = 4 * size_t(nslot_cap_) + 2 * nw + 32 * nw + 8;  // (+8 whole-grid stamps: three-step sweep)
    PE_HIP_CHECK(hipMalloc(&stamps_, sizeof(unsigned long long) * nstamps_));
    PE_HIP_CHECK(hipMemsetAsync(stamps_, 0, sizeof(unsigned long long) * nstamps_, stream_));
    k.stamps = stamps_;
    k.stamps2 = stamps_ + nstamps_ - 32 * nw;  // the last 32 × waves entries (the 8 grid stamps before them)
  }
  // In-sweep cross-rank reduction (after the placement search, whose sweeps
  // are local and differ in number between ranks).  PE_XR=0 keeps the
  // separate allreduce launch.
  xr_status_ = comm_->size() < 2 ? "none: one rank" : "allreduce launch (" + comm_->name() + ")";
  if (fused_ && comm_->size() > 1 && comm_->peer_sum()) {
    const char* e = std::getenv("PE_XR");
    if (!(e && std::atoi(e) == 0)) {
      k.xr = *comm_->peer_sum();
      k.xr.wait_acc = &st_->xr_wait;  // T_MPI of the in-sweep sum (DevState::xr_wait, xr_n)
      xr_status_ = "in-sweep P2P over xGMI";
    }
  }
  if (fused_ && comm_->size() > 1 && !comm_->peer_sum()) xr_status_ += "; P2P set-up " + p2p_setup_status();
  // The push's pointers (its kernel variant runs when choose_halo_path picks
  // it: the push is delivered by the in-sweep sum's flags, so the local
  // sweeps above ran without either).
  if (push_ok_) {
    const int64_t side = int64_t(hdep_) * k.pitch;
    double* lo = static_cast<double*>(hpeers_[size_t(blk_.nbr[LEFT] >= 0 ? blk_.nbr[LEFT] : blk_.rank)]);
    double* hi = static_cast<double*>(hpeers_[size_t(blk_.nbr[RIGHT] >= 0 ? blk_.nbr[RIGHT] : blk_.rank)]);
    for (int b = 0; b < 2; ++b) {
      // my rows 1, 2 → the LEFT neighbour's side 1 (its rows nx'+1, nx'+2);
      // my rows nx-1, nx → the RIGHT neighbour's side 0 (its rows -1, 0)
      k.hpush_lo[b] = blk_.has(LEFT) ? lo + (2 * b + 1) * side : nullptr;
      k.hpush_hi[b] = blk_.has(RIGHT) ? hi + (2 * b + 0) * side : nullptr;
    }
    k.hrecv = hrecv_;
  }
  k.push = 0;
  mark("ti tuning");
  choose_halo_path();
  mark("halo path");

  // Iterations per host check: aim for ~0.5 ms of device work per chunk.
  const double pts = double(nx) * double(ny);
  const double t_iter = pts * (sstep_ ? 48.0 / steps_ : fused_ ? 48.0 : 64.0) / 4.5e12 + 6e-6 + (comm_->size() > 1 ? 40e-6 : 0.0);
  int c = int(0.5e-3 / t_iter);
  c = std::max(8, std::min(128, c));
  c += c & 1;
  if (sstep_) c = (c + 2 * steps_ - 1) / (2 * steps_) * (2 * steps_);  // whole sweeps, an even number of them (graph parity)
  stream_chunk_ = opt_.chunk > 0 ? (opt_.chunk + (opt_.chunk & 1)) : c;
  if (resident_) c = 512;  // one launch per chunk (≈ 5 ms of iterations at 800×1200)
  chunk_ = opt_.chunk > 0 ? (opt_.chunk + (opt_.chunk & 1)) : c;
  if (sstep_) {
    chunk_ = (chunk_ + 2 * steps_ - 1) / (2 * steps_) * (2 * steps_);
    stream_chunk_ = chunk_;
  }
  mark("tuning+rest");
  // Graph-replayed solves (--graph): one small pageable copy at construction.
  // The runtime sets up its pageable-copy path lazily at the first such copy
  // of the process (≈19 ms, profiles/r2_init_probe.txt) — which a graph
  // instantiation triggers; this keeps that cost out of the iteration loop (4
  // µs per iteration at 1600×2400 otherwise).  The eager solve never takes
  // that path.
  if (opt_.use_graph) {
    double h = 0.0;
    PE_HIP_CHECK(hipMemcpy(partial_, &h, sizeof(double), hipMemcpyHostToDevice));
  }
  PE_HIP_CHECK(hipDeviceSynchronize());
  ctor_s_ = secs(t_ctor, clk::now());
}

void DeviceSolver::relayout(int ti, int order) {
  if (!fused_ || resident_) return;
  ti = std::max(2, std::min(ti, steps_ >= 3 ? dev::kTImax3 : 64));
  const int ord = (order == 0 || order == 3) ? order : kp_->order;  // static LPT list / dynamic per-XCD queue
  // the item-sum slots of the dynamic order were sized at
  // construction: a layout that needs more is refused before anything
  // changes (the static layout sums per block, not per item: any height)
  const int64_t nitems = int64_t(kp_->nstrips) * ((blk_.nx + ti - 1) / ti);
  const int64_t need = ord == 0 ? 0 : 2 * nitems + 64;
  if (need > nslot_cap_)
    throw std::invalid_argument("relayout: " + std::to_string(ti) + " rows per item (order " + std::to_string(ord) +
                                ") needs " + std::to_string(need) + " item-sum slots, " + std::to_string(nslot_cap_) +
                                " allocated");
  kp_->order = ord;
  PE_HIP_CHECK(hipStreamSynchronize(stream_));
  for (auto& g : graphs_) PE_HIP_CHECK(hipGraphExecDestroy(g.second));
  graphs_.clear();
  set_items(ti);
  setup_items();
}

void DeviceSolver::set_check_tol(bool on) {
  opt_.check_tol = on;
  kp_->check_tol = on ? 1 : 0;
  for (auto& g : graphs_) PE_HIP_CHECK(hipGraphExecDestroy(g.second));  // captured with the old parameters
  graphs_.clear();
}

void DeviceSolver::set_init(Init init, uint64_t seed, double amp) {
  opt_.init = init;
  opt_.seed = seed;
  opt_.init_amp = amp;
}

void DeviceSolver::set_fused_fields(double* x0, double* x1, double* w) {
  KParams& k = *kp_;
  fields_ = x0;
  xalt_ = x1;
  walt_ = w;
  // local (0, 0): row -(hdep-1), column -xorg at element 0
  const int64_t h = hdep_ - 1, hc = xorg_;
  k.x[0] = x0 + h * k.pitch + hc;
  k.x[1] = x1 + h * k.pitch + hc;
  k.w = w + h * plane_ + hc;
  k.r = k.x[0];
  k.p[0] = k.x[0] + plane_;
  k.p[1] = k.x[1] + plane_;
}

// Median time of this rank's halo exchange (every rank runs the same
// number of collective exchanges here), then the max over ranks.
void DeviceSolver::measure_exchange() {
  Range range("pe.measure_exchange");
  std::vector<float> t;
  for (int i = 0; i < 9; ++i) {
    PE_HIP_CHECK(hipEventRecord(t0_, stream_));
    if (fused_) enqueue_exchange(0);
    else comm_->exchange(halo_plan(), stream_);
    PE_HIP_CHECK(hipEventRecord(t1_, stream_));
    PE_HIP_CHECK(hipEventSynchronize(t1_));
    float ms = 0.f;
    PE_HIP_CHECK(hipEventElapsedTime(&ms, t0_, t1_));
    if (i >= 2) t.push_back(ms);  // two warm-up exchanges (connection set-up)
  }
  std::sort(t.begin(), t.end());
  double us[1] = {1e3 * double(t[t.size() / 2])};
  comm_->host_max(us, 1, stream_);
  exchange_us_ = us[0];
}


void DeviceSolver::create_halo_stream() {
  if (hs_) return;
  hs_ = acquire_halo_stream();  // (pooled: set_device created one next to the solver stream — runtime.cpp)
  PE_HIP_CHECK(hipEventCreateWithFlags(&ev_halo_, hipEventDisableTiming));
}


DeviceSolver::~DeviceSolver() {
  for (auto& g : graphs_) (void)hipGraphExecDestroy(g.second);
  (void)hipEventDestroy(ev_[0]);
  (void)hipEventDestroy(ev_[1]);
  (void)hipEventDestroy(ev_sync_);
  (void)hipEventDestroy(t0_);
  (void)hipEventDestroy(t1_);
  for (const PhaseRec& r : recs_) {
    (void)hipEventDestroy(r.a);
    (void)hipEventDestroy(r.b);
  }
  for (hipEvent_t e : evpool_) (void)hipEventDestroy(e);
  if (fused_) field_free(fields_);
  else (void)hipFree(fields_);
  field_free(xalt_);
  field_free(walt_);
  (void)hipFree(tables_);
  (void)hipFree(rowcls_);
  (void)hipFree(halo_);
  if (!hpeers_.empty() && !push_loop_) comm_->unmap_peer_buffers(hpeers_);
  if (hrecv_) (void)hipFree(hrecv_);
  if (!put_peers_.empty() && !put_loop_) comm_->unmap_peer_buffers(put_peers_);
  if (put_buf_) (void)hipFree(put_buf_);
  if (put_cnt_) (void)hipFree(put_cnt_);
  if (stage_) (void)hipHostFree(stage_);
  (void)hipFree(partial_);
  if (hist_) (void)hipFree(hist_);
  if (stamps_) (void)hipFree(stamps_);
  if (ilist_) (void)hipFree(ilist_);
  if (res_rowstart_) (void)hipFree(res_rowstart_);
  if (res_buf_) (void)hipFree(res_buf_);
  if (res_ctr_) (void)hipFree(res_ctr_);
  if (hs_) {
    (void)hipStreamSynchronize(hs_);
    release_halo_stream(hs_);
  }
  if (ev_halo_) (void)hipEventDestroy(ev_halo_);
  (void)hipFree(st_);
  (void)hipHostFree(hst_);
  (void)hipStreamSynchronize(stream_);
  release_stream(stream_);
}

KParams& DeviceSolver::params() { return *kp_; }

void DeviceSolver::clear_stamps() {
  if (nstamps_) PE_HIP_CHECK(hipMemsetAsync(stamps_, 0, sizeof(unsigned long long) * nstamps_, stream_));
}

std::vector<unsigned long long> DeviceSolver::stamps() {
  std::vector<unsigned long long> v(nstamps_);
  if (nstamps_) {
    PE_HIP_CHECK(hipStreamSynchronize(stream_));
    PE_HIP_CHECK(hipMemcpy(v.data(), stamps_, sizeof(unsigned long long) * nstamps_, hipMemcpyDeviceToHost));
  }
  return v;
}

// Host → device set-up data through a pinned staging buffer and a copy
// kernel (launch_copy_words: no hipMemcpy in T_solver); synchronous.
void DeviceSolver::upload(void* dst, const void* src, size_t bytes) {
  if (bytes == 0) return;
  if (bytes % 4) throw std::logic_error("upload: size must be a multiple of 4 bytes");
  if (bytes > stage_bytes_) {
    if (stage_) PE_HIP_CHECK(hipHostFree(stage_));
    stage_bytes_ = std::max(bytes, size_t(1) << 20);
    PE_HIP_CHECK(hipHostMalloc(&stage_, stage_bytes_, hipHostMallocDefault));
  }
  std::memcpy(stage_, src, bytes);
  dev::launch_copy_words(dst, stage_, bytes, false, stream_);
  PE_HIP_CHECK(hipGetLastError());
  PE_HIP_CHECK(hipStreamSynchronize(stream_));
}

void DeviceSolver::build_tables(int64_t rows_hi, int64_t cols_hi) {
  const std::vector<double> t = chord_tables(prob_, blk_, rows_hi, cols_hi, tab_lo_);
  const auto t0 = clk::now();
  upload(tables_, t.data(), sizeof(double) * t.size());
  copy_setup_s_ += secs(t0, clk::now());
  const double* col = t.data();
  const double* row = t.data() + (rows_hi - tab_lo_ + 1) * 4;
  rowcls_host_ = row_classes(col, row, rows_hi, cols_hi, tab_lo_);
  const std::vector<int>& rc = rowcls_host_;
  const auto t1 = clk::now();
  upload(rowcls_, rc.data(), sizeof(int) * rc.size());
  copy_setup_s_ += secs(t1, clk::now());
}

std::vector<Exchange> DeviceSolver::halo_plan() const {
  const KParams& k = *kp_;
  std::vector<Exchange> ex;
  if (blk_.has(LEFT))
    ex.push_back(Exchange{LEFT, blk_.nbr[LEFT], k.r + 1 * k.pitch + 1, k.r + 0 * k.pitch + 1, blk_.ny});
  if (blk_.has(RIGHT))
    ex.push_back(Exchange{RIGHT, blk_.nbr[RIGHT], k.r + blk_.nx * k.pitch + 1, k.r + (blk_.nx + 1) * k.pitch + 1,
                          blk_.ny});
  if (blk_.has(DOWN)) ex.push_back(Exchange{DOWN, blk_.nbr[DOWN], k.send_dn, const_cast<double*>(k.recv_dn), blk_.nx});
  if (blk_.has(UP)) ex.push_back(Exchange{UP, blk_.nbr[UP], k.send_up, const_cast<double*>(k.recv_up), blk_.nx});
  return ex;
}

std::vector<DeviceSolver::HaloPhase> DeviceSolver::halo_phases(int buf) const {
  if (!fused_) return {HaloPhase{halo_plan(), false}};
  const KParams& k = *kp_;
  std::vector<HaloPhase> ph(2);
  // Phase 0: y strips (2·hdep values per owned row: r and p of hdep columns;
  // the single sweep stores them from inside the sweep, the multi-step
  // sweeps' are packed after it — enqueue_exchange).
  const int64_t c = 2 * int64_t(hdep_) * blk_.nx;
  if (blk_.has(DOWN)) ph[0].ex.push_back(Exchange{DOWN, blk_.nbr[DOWN], k.send_dn, const_cast<double*>(k.recv_dn), c});
  if (blk_.has(UP)) ph[0].ex.push_back(Exchange{UP, blk_.nbr[UP], k.send_up, const_cast<double*>(k.recv_up), c});
  ph[0].unpack = blk_.has(DOWN) || blk_.has(UP);
  // Phase 1: hdep full interleaved (r, p) rows per side, halo columns
  // included (so the corners arrive from the diagonal rank through the x
  // neighbour): rows 1..h → the LEFT neighbour's rows nx'+1..nx'+h, rows
  // nx-h+1..nx → the RIGHT neighbour's rows 1-h..0.
  double* x = k.x[buf];
  const int64_t h = hdep_, n = h * k.pitch, hc = xorg_;  // (whole rows: from column -xorg)
  if (blk_.has(LEFT))
    ph[1].ex.push_back(Exchange{LEFT, blk_.nbr[LEFT], x + 1 * k.pitch - hc, x + (1 - h) * k.pitch - hc, n});
  if (blk_.has(RIGHT))
    ph[1].ex.push_back(Exchange{RIGHT, blk_.nbr[RIGHT], x + (blk_.nx - h + 1) * k.pitch - hc,
                                x + (blk_.nx + 1) * k.pitch - hc, n});
  return ph;
}

void DeviceSolver::enqueue_exchange(int buf, bool after_sweep) {
  // halo push: the sweep that wrote `buf` has pushed its edge rows into the
  // neighbours' receive buffers, from which the next sweep reads them
  if (push_ && after_sweep) return;
  if (sstep_ && after_sweep) dev::launch_pack(*kp_, buf, stream_);  // (no-op without a y neighbour)
  for (const HaloPhase& ph : halo_phases(buf)) {
    xfer(ph.ex, stream_);
    if (ph.unpack) dev::launch_unpack(*kp_, buf, stream_);
  }
  // initial state through the comm: its halo rows into the receive buffer
  if (push_) dev::launch_halo_seed(*kp_, buf, stream_);
}

// halo push: x's halo rows ← the receive buffers (checkpoint, read-back)
void DeviceSolver::import_halos() {
  if (!push_) return;
  for (int b = 0; b < 2; ++b) dev::launch_halo_import(*kp_, b, stream_);
  PE_HIP_CHECK(hipGetLastError());
}

double* DeviceSolver::red_F_dev() { return st_->red_F; }
double* DeviceSolver::red_G_dev() { return st_->red_G; }
double* DeviceSolver::fs_dev(int par) { return st_->fs[par]; }
double* DeviceSolver::fs2_dev(int par) { return st_->fs2[par]; }
double* DeviceSolver::err_dev() { return st_->err; }

void DeviceSolver::enqueue_init() {
  const int64_t n = fused_ ? 2 * xsize_ + wsize_ : 4 * blk_.alloc;
  if (fused_) {
    PE_HIP_CHECK(hipMemsetAsync(fields_, 0, sizeof(double) * xsize_, stream_));
    PE_HIP_CHECK(hipMemsetAsync(xalt_, 0, sizeof(double) * xsize_, stream_));
    PE_HIP_CHECK(hipMemsetAsync(walt_, 0, sizeof(double) * wsize_, stream_));
  } else {
    PE_HIP_CHECK(hipMemsetAsync(fields_, 0, sizeof(double) * n, stream_));
  }
  PE_HIP_CHECK(hipMemsetAsync(halo_, 0, sizeof(double) * hsize_ * 4, stream_));
  PE_HIP_CHECK(hipMemsetAsync(st_, 0, sizeof(DevState), stream_));
  ov_epoch_ = 0;
  dev::launch_init(*kp_, opt_.init == Init::Random ? 1 : 0, opt_.seed, opt_.init_amp, opt_.variant, stream_);
  PE_HIP_CHECK(hipGetLastError());
}

void DeviceSolver::enqueue_F(int par) { dev::launch_F(*kp_, par, opt_.variant, stream_); }
void DeviceSolver::enqueue_G(int par) { dev::launch_G(*kp_, par, opt_.variant, stream_); }
void DeviceSolver::enqueue_S(int par) { dev::launch_S(*kp_, par, stream_); }
void DeviceSolver::enqueue_pack(int buf) { dev::launch_pack(*kp_, buf, stream_); }
void DeviceSolver::enqueue_unpack(int buf) { dev::launch_unpack(*kp_, buf, stream_); }
void DeviceSolver::enqueue_error() { dev::launch_error(*kp_, stream_); }

// Cross-rank sum of sweep `par`'s 7 sums: nothing to enqueue when the sweep
// sums them over ranks itself (k.xr, P2P transport).
void DeviceSolver::enqueue_fs_reduce(int par) {
  if (kp_->xr.peers) return;
  if (sstep_) comm_->allreduce_sum(st_->fs2[par], dev::sweep_sums(steps_), stream_);
  else comm_->allreduce_sum(st_->fs[par], 7, stream_);
}

// Sampled phase timing: event pairs from a pool; a record's events are read
// (harvest) once the chunk that holds them has been waited for.
hipEvent_t DeviceSolver::pooled_event() {
  if (evpool_.empty()) {
    hipEvent_t e = nullptr;
    PE_HIP_CHECK(hipEventCreate(&e));
    return e;
  }
  hipEvent_t e = evpool_.back();
  evpool_.pop_back();
  return e;
}

void DeviceSolver::mark_begin(int ph, hipStream_t s) {
  if (!sampling_) return;
  PhaseRec r{ph, sample_iter_, steps_, pooled_event(), nullptr};  // (a multi-step sweep covers steps_ iterations)
  PE_HIP_CHECK(hipEventRecord(r.a, s));
  recs_.push_back(r);
}

void DeviceSolver::mark_end(hipStream_t s) {
  if (!sampling_) return;
  recs_.back().b = pooled_event();
  PE_HIP_CHECK(hipEventRecord(recs_.back().b, s));
}

void DeviceSolver::harvest(size_t n) {
  n = std::min(n, recs_.size());
  for (size_t i = 0; i < n; ++i) {
    float ms = 0.f;
    PE_HIP_CHECK(hipEventElapsedTime(&ms, recs_[i].a, recs_[i].b));
    samples_.push_back(PhaseSample{recs_[i].ph, recs_[i].iter, recs_[i].n, ms});
    evpool_.push_back(recs_[i].a);
    evpool_.push_back(recs_[i].b);
  }
  recs_.erase(recs_.begin(), recs_.begin() + std::ptrdiff_t(n));
}

void DeviceSolver::enqueue_iteration(int par, int mlimit) {
  const int ncomm = comm_->size();
  if (fused_ && overlap_) {
    KParams ko = *kp_;
    ko.ilist = ilist_;
    ko.lnsh = ov_lnsh_;
    for (int x = 0; x <= 8; ++x) ko.lbase[x] = ov_lbase_[x];
    for (int x = 0; x < 8; ++x) ko.lnb[x] = ov_lnb_[x];
    ko.nblocks = std::max(ov_lnsh_, kp_->nblocks - ov_reserve_);
    ko.nblocks0 = std::max(ov_lnsh_, kp_->nblocks0 - ov_reserve_);
    ko.mlimit = mlimit;
    ov_epoch_ += 1;
    const unsigned long long target = ov_epoch_ * (unsigned long long)(ov_nb_);
    mark_begin(kPhSweep, stream_);
    dev::launch_S(ko, par, stream_, false);  // boundary items first in every shard
    mark_end(stream_);
    if (ko.order == 3) {
      mark_begin(kPhDot, stream_);
      dev::launch_red(ko, par, stream_);
      mark_end(stream_);
    }
    if (ov_debug_ & 2) {
      dev::launch_wait_sig(ko, target, stream_);
      mark_begin(kPhHalo, stream_);
      enqueue_exchange(par);
      mark_end(stream_);
    } else {
      dev::launch_wait_sig(ko, target, hs_);  // the exchange starts once they are stored
      mark_begin(kPhHalo, hs_);
      if (sstep_) dev::launch_pack(*kp_, par, hs_);  // (multi-step: y strips packed after the boundary items)
      for (const HaloPhase& ph : halo_phases(par)) {
        xfer(ph.ex, hs_);
        if (ph.unpack) dev::launch_unpack(*kp_, par, hs_);
      }
      mark_end(hs_);
      PE_HIP_CHECK(hipEventRecord(ev_halo_, hs_));
      PE_HIP_CHECK(hipStreamWaitEvent(stream_, ev_halo_, 0));
    }
    if (!kp_->xr.peers) {
      mark_begin(kPhReduce, stream_);
      enqueue_fs_reduce(par);
      mark_end(stream_);
    }
  } else if (fused_) {
    mark_begin(kPhSweep, stream_);
    if (mlimit > 0) {  // a partial three-step sweep: the run's last mlimit < 3 iterations
      KParams kk = *kp_;
      kk.mlimit = mlimit;
      dev::launch_S(kk, par, stream_, false);
    } else {
      dev::launch_S(*kp_, par, stream_, false);
    }
    mark_end(stream_);
    if (kp_->order == 3) {
      mark_begin(kPhDot, stream_);
      dev::launch_red(*kp_, par, stream_);
      mark_end(stream_);
    }
    if (ncomm > 1) {
      mark_begin(kPhHalo, stream_);
      enqueue_exchange(par);
      mark_end(stream_);
      if (!kp_->xr.peers) {
        mark_begin(kPhReduce, stream_);
        enqueue_fs_reduce(par);
        mark_end(stream_);
      }
    }
  } else {
    mark_begin(kPhSweep, stream_);
    dev::launch_F(*kp_, par, opt_.variant, stream_);
    mark_end(stream_);
    if (ncomm > 1) {
      mark_begin(kPhReduce, stream_);
      comm_->allreduce_sum(st_->red_F, 2, stream_);
      mark_end(stream_);
    }
    mark_begin(kPhSweep, stream_);
    dev::launch_G(*kp_, par, opt_.variant, stream_);
    mark_end(stream_);
    if (ncomm > 1) {
      mark_begin(kPhHalo, stream_);
      comm_->exchange(halo_plan(), stream_);
      mark_end(stream_);
      mark_begin(kPhReduce, stream_);
      comm_->allreduce_sum(st_->red_G, 1, stream_);
      mark_end(stream_);
    }
  }
  if (sampling_) sample_iter_ += mlimit > 0 ? mlimit : steps_;
}

// Chunk graphs are cached per length (a run of n iterations uses the chunk
// length and its remainder), so alternating lengths never re-capture.
hipGraphExec_t DeviceSolver::graph_for(int iters) {
  for (const auto& g : graphs_)
    if (g.first == iters) return g.second;
  const int per = steps_;
  if (iters % (2 * per)) throw std::logic_error("graph chunks must hold an even number of sweeps");
  hipGraph_t g = nullptr;
  hipGraphExec_t ge = nullptr;
  PE_HIP_CHECK(hipStreamBeginCapture(stream_, hipStreamCaptureModeThreadLocal));
  for (int it = 0; it < iters / per; ++it) enqueue_iteration(it & 1);
  PE_HIP_CHECK(hipStreamEndCapture(stream_, &g));
  PE_HIP_CHECK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
  PE_HIP_CHECK(hipGraphDestroy(g));
  // stage the executable's launch resources now, so its first replay (in a
  // bench's timed window) costs what the later ones do; stream-ordered, and
  // an optimisation only: a runtime without it replays the same graph
  if (hipGraphUpload(ge, stream_) != hipSuccess) (void)hipGetLastError();
  graphs_.emplace_back(iters, ge);
  return ge;
}

// (overlap: a graph may serialise the two streams' branches in any order,
// and the halo branch waits on the sweep — always eager)
// (no comm call in the iteration: the sweep's push or the put kernel for the
// halo, the in-sweep P2P sums for the scalars)
bool DeviceSolver::graphs_usable() const {
  return (comm_->capturable() || push_ || (put_ && kp_->xr.peers)) && !overlap_ && !resident_;
}

void DeviceSolver::enqueue_chunk(int iters, int sample_iters) {
  // The captured graph starts at parity 0 and has an even length; iterations
  // that would break the p / x ping-pong parity run eagerly.  A sampled
  // chunk runs eagerly with event pairs around the phases of its first
  // `sample_iters` iterations.
  int it = 0;
  if (resident_ && iters > 0) {
    // one launch for the whole chunk (always timed: two events per chunk)
    dev::ResParams r = *rp_;
    r.niter = iters;
    r.par0 = par_;
    PE_HIP_CHECK(hipMemsetAsync(res_ctr_, 0, sizeof(unsigned) * 8 * 32, stream_));
    const bool was = sampling_;
    sampling_ = true;
    mark_begin(kPhSweep, stream_);
    recs_.back().n = iters;
    dev::launch_resident(*kp_, r, stream_);
    mark_end(stream_);
    sampling_ = was;
    sample_iter_ += iters;
    par_ ^= iters & 1;
    PE_HIP_CHECK(hipGetLastError());
    return;
  }
  // (multi-step sweep: one launch = steps_ iterations; chunks are multiples
  // of 2·steps_; a three-step run of n iterations ends with a partial sweep
  // when 3 ∤ n)
  const int per = steps_;
  if (sample_iters == 0 && opt_.use_graph && graphs_usable() && par_ == 0 && iters >= 2 * per) {
    const int n = iters - iters % (2 * per);
    PE_HIP_CHECK(hipGraphLaunch(graph_for(n), stream_));
    it = n;
  }
  for (; it < iters; it += per) {
    sampling_ = it < sample_iters;
    enqueue_iteration(par_, steps_ >= 3 && iters - it < per ? iters - it : 0);
    par_ ^= 1;
  }
  sampling_ = false;
  PE_HIP_CHECK(hipGetLastError());
}

void DeviceSolver::prepare_graphs(int64_t iters) {
  if (!graphs_usable()) return;
  // the chunk lengths run_iterations(iters) launches from parity 0
  const int64_t full = iters / chunk_, rest = iters % chunk_;
  const int64_t q = 2 * steps_;
  if (full > 0) graph_for(chunk_);
  if (rest >= q) graph_for(int(rest - rest % q));
  // the capture enqueued nothing: the stream state is unchanged
}


void DeviceSolver::wait_event(hipEvent_t ev) {
  const auto t0 = clk::now();
  for (;;) {
    const hipError_t q = fault_stall_ ? hipErrorNotReady : hipEventQuery(ev);
    if (q == hipSuccess) return;
    if (q != hipErrorNotReady) PE_HIP_CHECK(q);
    comm_->check_async();
    if (watchdog_s_ > 0 && secs(t0, clk::now()) > watchdog_s_) {
      comm_->abort();
      throw std::runtime_error("watchdog: device made no progress for " + std::to_string(watchdog_s_) +
                               " s (communicator aborted)");
    }
    // spin (yielding) for the first 250 ms, then poll every 20 µs: a sleeping
    // poll detects the end late by up to a scheduler tick, and a bench's
    // closing wait of a 5 ms window used to span the 2 ms the spin lasted
    if (secs(t0, clk::now()) > 0.25) std::this_thread::sleep_for(std::chrono::microseconds(20));
    else std::this_thread::yield();
  }
}

void DeviceSolver::enqueue_wflush() {
  if (!fused_) return;
  if (steps_ >= 3) {  // the last sweep's pending stop tests (and its w fix-up when it converged early)
    KParams kk = *kp_;
    kk.mlimit = -1;
    dev::launch_S(kk, par_, stream_);
    return;
  }
  dev::launch_wflush(*kp_, stream_);
}

void DeviceSolver::residual_pass(bool with_r, bool store) {
  const KParams& k = *kp_;
  dev::launch_w_to_p(k, 0, stream_);
  if (comm_->size() > 1) {  // w's halo: x[0]'s exchange (y strips packed first, as reset() does)
    dev::launch_pack(k, 0, stream_);
    enqueue_exchange(0, false);
  }
  dev::launch_resid(k, 0, with_r, store, stream_);
  if (comm_->size() > 1) comm_->allreduce_sum(st_->res, 4, stream_);
  PE_HIP_CHECK(hipGetLastError());
}

void DeviceSolver::read_state(DevState* out) {
  PE_HIP_CHECK(hipMemcpyAsync(out, st_, sizeof(DevState), hipMemcpyDeviceToHost, stream_));
  PE_HIP_CHECK(hipStreamSynchronize(stream_));
}

void DeviceSolver::synchronize() {
  if (watchdog_s_ <= 0 && !fault_stall_) {
    PE_HIP_CHECK(hipStreamSynchronize(stream_));
    return;
  }
  PE_HIP_CHECK(hipEventRecord(ev_sync_, stream_));
  wait_event(ev_sync_);
}

void DeviceSolver::reset() {
  par_ = 0;
  enqueue_init();
  if (fused_) {
    // r⁰ (and p = 0) in x[0] → halos → sweep S_0 (z₀, A z₀ and their sums,
    // no iteration counted) into x[1]; iteration 1 then reads x[1] (par 0).
    dev::launch_pack(*kp_, 0, stream_);
    enqueue_exchange(0, false);
    dev::launch_S(*kp_, 1, stream_);
    enqueue_exchange(1);
    enqueue_fs_reduce(1);
    return;
  }
  comm_->exchange(halo_plan(), stream_);
  comm_->allreduce_sum(st_->red_G, 1, stream_);
}

void DeviceSolver::run_iterations(int64_t iters, bool use_graph) {
  // (the three-step sweep ends an n-iteration run with a partial sweep when
  // 3 ∤ n; the two-step sweep has none — its one-iteration sweep ends the
  // solve — so an odd count would run one iteration too many)
  if (steps_ == 2 && iters % 2 != 0)
    throw std::invalid_argument("two-step sweep: run an even number of iterations (got " + std::to_string(iters) + ")");
  const bool saved = opt_.use_graph;
  opt_.use_graph = use_graph;
  int64_t done = 0;
  while (done < iters) {
    const int64_t n = std::min<int64_t>(chunk_, iters - done);
    enqueue_chunk(int(n));
    done += n;
  }
  opt_.use_graph = saved;
}

double DeviceSolver::time_iterations(int64_t iters, bool use_graph) {
  PE_HIP_CHECK(hipEventRecord(t0_, stream_));
  run_iterations(iters, use_graph);
  PE_HIP_CHECK(hipEventRecord(t1_, stream_));
  PE_HIP_CHECK(hipEventSynchronize(t1_));
  float ms = 0;
  PE_HIP_CHECK(hipEventElapsedTime(&ms, t0_, t1_));
  return ms * 1e-3;
}

SolveResult DeviceSolver::solve() {
  Range range("pe.solve");
  const auto t_start = clk::now();
  SolveResult res;
  res.backend = "hip";
  res.algo = resident_ ? "resident" : steps_ == 3 ? "three-step" : steps_ == 2 ? "two-step" : fused_ ? "fused" : "classic";
  res.Px = blk_.Px;
  res.Py = blk_.Py;
  // T_solver spans construction (allocation, tables, placement search) like
  // the reference's time_solver (poisson_mpi_cuda2.cu:1010-1016); a second
  // solve on the same solver reuses it and does not count it again.
  const double construct = ctor_counted_ ? 0.0 : ctor_s_;
  ctor_counted_ = true;
  double copy_s = construct > 0 ? copy_setup_s_ : 0.0;
  int64_t start_iter = 0;
  if (!opt_.resume_path.empty()) {
    const auto tc = clk::now();
    load_checkpoint(opt_.resume_path + ".r" + std::to_string(blk_.rank));
    copy_s += secs(tc, clk::now());
    DevState s0;
    read_state(&s0);
    start_iter = s0.iter;
  } else {
    reset();
  }
  PE_HIP_CHECK(hipStreamSynchronize(stream_));
  res.t.construct = construct;
  res.t.setup = construct + secs(t_start, clk::now());
  const int64_t ck_every = opt_.checkpoint_path.empty() ? 0 : opt_.checkpoint_every;

  // Phase sampling: every `sample_every`-th chunk, its first two iterations
  // (all of them with opt_.timing); no host sync beyond the per-chunk state
  // read the loop does anyway.
  int sample_every = 8, sample_iters = 2;
  if (const char* e = std::getenv("PE_TIMER_SAMPLE")) sample_every = std::max(0, std::atoi(e));
  if (opt_.timing) {
    sample_every = 1;
    sample_iters = chunk_;
  }
  samples_.clear();
  sample_iter_ = start_iter;

  const int64_t cap = prob_.iter_cap();
  const auto t_loop = clk::now();
  roctxRangePushA("pe.iterate");
  PE_HIP_CHECK(hipEventRecord(t0_, stream_));
  int64_t enq = start_iter;
  int64_t next_ck = ck_every > 0 ? (start_iter / ck_every + 1) * ck_every : std::numeric_limits<int64_t>::max();
  int64_t next_log = opt_.log_every > 0 ? opt_.log_every : 0;
  int slot = 0;
  struct Flight {
    int slot;
    size_t nrec;  // phase records enqueued up to and including this chunk
  };
  std::deque<Flight> inflight;
  int64_t nchunk = 0;
  bool stop = false;
  bool res_abort = false;  // a resident launch's grid barrier timed out (status 5)
  bool drift_done = fault_drift_ <= 0;
  int restarts = 0;
  DevState hs;
  double check_s = 0.0;
  for (;;) {  // (a three-step restart runs the loop again from the restart's iteration)
    for (;;) {
      while (!stop && enq < cap && inflight.size() < 2 && enq < next_ck) {
        const bool sample = sample_every > 0 && nchunk % sample_every == 0;
        sample_iter_ = enq;
        enqueue_chunk(chunk_, sample ? sample_iters : 0);
        enq += chunk_;
        if (!drift_done && enq >= fault_drift_) {  // PE_FAULT_INJECT=drift@iter:K
          drift_done = true;
          const int64_t li = prob_.M / 2 - kp_->gi0, lj = prob_.N / 2 - kp_->gj0;
          if (fused_ && li >= 1 && li <= blk_.nx && lj >= 1 && lj <= blk_.ny)
            dev::launch_poke_w(*kp_, li, lj, fault_drift_amp_, stream_);
        }
        sampling_ = sample;
        sample_iter_ = enq - 1;
        mark_begin(kPhCopy, stream_);
        // per-chunk state read: a copy kernel into mapped pinned memory (a
        // hipMemcpyAsync's first use initialises the runtime's copy path
        // inside T_solver)
        dev::launch_copy_words(&hst_[slot], st_, sizeof(DevState), true, stream_);
        mark_end(stream_);
        sampling_ = false;
        PE_HIP_CHECK(hipEventRecord(ev_[slot], stream_));
        inflight.push_back(Flight{slot, recs_.size()});
        slot ^= 1;
        ++nchunk;
      }
      if (inflight.empty()) {
        if (!stop && enq < cap && enq >= next_ck) {  // drained at a checkpoint boundary
          const auto tc = clk::now();
          save_checkpoint(opt_.checkpoint_path + ".r" + std::to_string(blk_.rank));
          copy_s += secs(tc, clk::now());
          while (next_ck <= enq) next_ck += ck_every;
          continue;
        }
        if (res_abort) {
          // Resident fallback: a workgroup of a resident launch timed out at a
          // grid barrier.  The aborted launch may still have written back part
          // of the grid (a late workgroup passes the barrier the others gave up
          // on), so its state is not resumed: the solve starts over from its
          // initial state (or its checkpoint) on the streaming sweep.
          res_abort = false;
          DevState s0;
          read_state(&s0);
          std::fprintf(stderr, "[pe] rank %d: resident kernel barrier timed out by iteration %lld; "
                               "restarting the solve with the streaming sweep\n", blk_.rank, (long long)s0.iter);
          resident_ = false;
          resident_fallback_ = true;
          chunk_ = stream_chunk_;
          harvest(recs_.size());
          samples_.clear();
          if (!opt_.resume_path.empty()) load_checkpoint(opt_.resume_path + ".r" + std::to_string(blk_.rank));
          else reset();
          enq = start_iter;
          sample_iter_ = start_iter;
          stop = false;
          continue;
        }
        break;
      }
      const Flight f = inflight.front();
      inflight.pop_front();
      wait_event(ev_[f.slot]);
      // this chunk's (and every earlier) phase events have completed
      const size_t done_recs = std::min(f.nrec, recs_.size());
      harvest(done_recs);
      for (Flight& g : inflight) g.nrec -= std::min(g.nrec, done_recs);
      if (hst_[f.slot].done) {
        stop = true;
        if ((hst_[f.slot].status == 5 || hst_[f.slot].res_abort) && resident_) res_abort = true;
      }
      if (opt_.log_every > 0 && blk_.rank == 0 && hst_[f.slot].iter >= next_log) {  // chunk-granular progress log
        std::fprintf(stderr, "[pe] iter %lld  |dw| = %.6e  (z,r) = %.6e\n", (long long)hst_[f.slot].iter,
                     hst_[f.slot].last_diff, hst_[f.slot].rz_cur);
        while (next_log <= hst_[f.slot].iter) next_log += opt_.log_every;
      }
    }
    // True-residual check of the returned w: ρ = B − A w.  Three-step: the
    // s-step moment recurrence (fused3.hip) is checked against it — after a
    // fix-up (the solve stopped inside the last sweep), the replay launch
    // first recomputes that iterate's r into x[wpar], so w and r belong to the
    // same iterate.
    const bool three = fused_ && steps_ >= 3;  // (three-step: the moment recurrence)
    enqueue_wflush();
    // (the check below is timed on its own: res.t.check, outside T_iterate, inside T_solver)
    PE_HIP_CHECK(hipStreamSynchronize(stream_));
    const auto t_chk = clk::now();
    if (three) {  // (after a fix-up: x[wpar] ← the r of the returned w)
      KParams kk = *kp_;
      kk.mlimit = dev::kReplay3;
      dev::launch_S(kk, par_, stream_);
    }
    if (fused_) residual_pass(three, three);
    read_state(&hs);
    check_s += secs(t_chk, clk::now());
    const double hh = prob_.h1() * prob_.h2();
    if (three) {
      res.res_rec = std::sqrt(hs.res[1] * hh);
      // relative to the recurrence's own ‖r‖: the fp64 gap of any CG recurrence
    // scales with the residuals it has summed, not with ‖B‖ (8192² random
    // init: 8e-3 absolute = 5e-7 of ‖r‖ = 1.5e4; zero init 2e-10 of ‖r‖ —
    // profiles/r4_resid.txt)
    res.res_gap = std::sqrt(hs.res[2] / std::max(hs.res[1], 1e-300));
    }
    if (fused_) {
      res.res_true = std::sqrt(hs.res[0] * hh);
      res.b_norm = std::sqrt(hs.res[3] * hh);
    }
    // Residual replacement: a converged three-step solve whose recurrence has
    // drifted from B − A w (gap above PE_RESID_GAP, default 1e-4 of ‖r‖) goes on
    // from the returned w with r = B − A w (stored by the pass above), p = 0 and
    // a fresh recurrence (β = 0 after the restart), at most twice.  Every rank
    // reads the same reduced sums: every rank decides the same.
    if (three && hs.status == 1 && res.res_gap > gap_bound_ && restarts < 2 && hs.iter < cap) {
      ++restarts;
      std::fprintf(stderr, "[pe] rank %d: residual gap %.3e > %.1e at iteration %lld; restarting the recurrence from w\n",
                   blk_.rank, res.res_gap, gap_bound_, (long long)hs.iter);
      dev::launch_zero_p(*kp_, 0, stream_);
      dev::launch_restart3(*kp_, stream_);
      ov_epoch_ = 0;
      dev::launch_pack(*kp_, 0, stream_);
      enqueue_exchange(0, false);
      dev::launch_S(*kp_, 1, stream_);
      enqueue_exchange(1);
      enqueue_fs_reduce(1);
      par_ = 0;
      enq = hs.iter;
      stop = false;
      continue;
    }
    break;
  }
  res.restarts = restarts;
  PE_HIP_CHECK(hipEventRecord(t1_, stream_));
  PE_HIP_CHECK(hipEventSynchronize(t1_));
  harvest(recs_.size());
  float ms = 0;
  PE_HIP_CHECK(hipEventElapsedTime(&ms, t0_, t1_));
  res.t.iterate = secs(t_loop, clk::now()) - check_s;
  res.t.check = check_s;
  roctxRangePop();

  if (opt_.compute_error) {
    dev::launch_error(*kp_, stream_);
    comm_->allreduce_sum(st_->err, 1, stream_);
    comm_->allreduce_max(st_->err + 1, 2, stream_);
  }
  read_state(&hs);
  res.iters = hs.iter;
  res.converged = hs.status == 1;
  res.breakdown = hs.status == 2;
  res.nonfinite = hs.status == 4;
  res.resident_fallback = resident_fallback_;
  if (resident_fallback_) res.algo = "fused (resident fallback)";
  if (hs.status == 5) throw std::runtime_error("single-sweep: internal error (status 5: a grid barrier or item sums never completed)");
  res.last_diff = hs.last_diff;
  if (hist_ && hs.iter > 0) {
    res.history.resize(size_t(std::min<long long>(hs.iter, kp_->hist_n)));
    PE_HIP_CHECK(hipMemcpyAsync(res.history.data(), hist_, sizeof(double) * res.history.size(), hipMemcpyDeviceToHost,
                                stream_));
    PE_HIP_CHECK(hipStreamSynchronize(stream_));
  }
  res.zr = hs.rz_cur;
  if (opt_.compute_error) {
    res.l2_err = std::sqrt(hs.err[0] * prob_.h1() * prob_.h2());
    res.max_err = hs.err[1];
    res.max_outside = hs.err[2];
  }
  // Per-phase totals: mean per sampled live iteration (samples taken after
  // the solve had stopped time no-op kernels and are dropped) × iterations
  // run; the state read per chunk likewise × chunks run.
  {
    const int64_t run = std::max<int64_t>(0, hs.iter - start_iter);
    double sum[kNPhase] = {};
    std::vector<char> seen(size_t(std::max<int64_t>(1, run)), 0);
    int64_t nit = 0, ncopy = 0;
    for (const PhaseSample& x : samples_) {
      if (x.iter >= hs.iter) continue;
      sum[x.ph] += x.ms * 1e-3;
      if (x.ph == kPhCopy) {
        ++ncopy;
      } else if (x.n > 1) {  // a resident launch: the iterations it ran before the solve stopped
        nit += std::min<int64_t>(x.n, hs.iter - x.iter);
      } else if (x.iter >= start_iter && !seen[size_t(x.iter - start_iter)]) {
        seen[size_t(x.iter - start_iter)] = 1;
        ++nit;
      }
    }
    const double scale = nit > 0 ? double(run) / double(nit) : 0.0;
    const int64_t chunks_run = (run + chunk_ - 1) / chunk_;
    res.t.gpu = (sum[kPhSweep] + sum[kPhDot]) * scale;
    res.t.dot = sum[kPhDot] * scale;
    res.t.halo = sum[kPhHalo] * scale;
    res.t.reduce = sum[kPhReduce] * scale;
    res.t.copy = copy_s + (ncopy > 0 ? sum[kPhCopy] * double(chunks_run) / double(ncopy) : 0.0);
    res.t.sampled = double(nit);
    // in-sweep cross-rank sum: the final blocks' wait for the peers' flags
    // (ticks of the 100 MHz s_memrealtime clock)
    res.t.wait = double(hs.xr_wait) * 1e-8;
    res.t.dot_fused = !(fused_ && kp_->order == 3);
    if (nit == 0) res.t.gpu = ms * 1e-3;  // sampling off: the loop's device span
  }
  // T_solver spans the whole solve, the end-of-solve residual check included
  // (it drives the residual-replacement restart: part of the solve, as the
  // reference's time_solver spans its whole gradient_solver_mpi call); t_check
  // reports it separately and T_iterate excludes it
  res.t.solver = construct + secs(t_start, clk::now());
  // Timers: max over ranks (reference MPI_Reduce(MAX), :962-966).
  double tv[11] = {res.t.gpu, res.t.copy, res.t.halo, res.t.reduce, res.t.setup, res.t.solver, res.t.iterate,
                   res.t.dot, res.t.construct, res.t.wait, res.t.check};
  comm_->host_max(tv, 11, stream_);
  res.t.check = tv[10];
  res.t.wait = tv[9];
  res.t.gpu = tv[0];
  res.t.copy = tv[1];
  res.t.halo = tv[2];
  res.t.reduce = tv[3];
  res.t.setup = tv[4];
  res.t.solver = tv[5];
  res.t.iterate = tv[6];
  res.t.dot = tv[7];
  res.t.construct = tv[8];
  return res;
}

void DeviceSolver::copy_w(double* host, bool owned_only) {
  const KParams& k = *kp_;
  enqueue_wflush();
  if (owned_only) {
    PE_HIP_CHECK(hipMemcpy2DAsync(host, sizeof(double) * blk_.ny, k.w + k.wpitch + 1, sizeof(double) * k.wpitch,
                                  sizeof(double) * blk_.ny, blk_.nx, hipMemcpyDeviceToHost, stream_));
  } else {
    PE_HIP_CHECK(hipMemcpyAsync(host, k.w, sizeof(double) * blk_.rows * k.wpitch, hipMemcpyDeviceToHost, stream_));
  }
  PE_HIP_CHECK(hipStreamSynchronize(stream_));
}

int64_t DeviceSolver::field_rows() const { return fused_ ? blk_.nx + 4 : blk_.rows; }
int64_t DeviceSolver::field_cols() const { return fused_ ? plane_ : blk_.pitch; }

void DeviceSolver::copy_field(int which, double* host) {
  const KParams& k = *kp_;
  if (fused_) {
    import_halos();
    // rows -1..nx+2 of one plane, columns -1.. (plane width)
    const double* base = which == 0 ? k.x[0] : which == 1 ? k.w : which == 2 ? k.x[0] + k.poff
                         : which == 3 ? k.x[1] + k.poff : k.x[1];
    const int64_t stride = which == 1 ? k.wpitch : k.pitch;
    PE_HIP_CHECK(hipMemcpy2DAsync(host, sizeof(double) * plane_, base - stride - 1, sizeof(double) * stride,
                                  sizeof(double) * plane_, blk_.nx + 4, hipMemcpyDeviceToHost, stream_));
  } else {
    const double* src = which == 0 ? k.r : which == 1 ? k.w : which == 2 ? k.p[0] : k.p[1];
    PE_HIP_CHECK(hipMemcpyAsync(host, src, sizeof(double) * blk_.rows * k.pitch, hipMemcpyDeviceToHost, stream_));
  }
  PE_HIP_CHECK(hipStreamSynchronize(stream_));
}

// ---------------------------------------------------------------------------
// Virtual ranks on one device.
// ---------------------------------------------------------------------------
SolveResult device_solve_group(const Problem& P, int ranks, DecompMode mode, const SolveOptions& opt,
                               std::vector<double>* w_out) {
  return device_solve_group(P, choose_process_grid(ranks, P.M, P.N, mode), opt, w_out);
}

SolveResult device_solve_group(const Problem& P, const ProcessGrid& pg, const SolveOptions& opt,
                               std::vector<double>* w_out) {
  const auto t_start = clk::now();
  const int ranks = pg.Px * pg.Py;
  std::vector<std::unique_ptr<DeviceSolver>> s;
  std::vector<Block> blks;
  for (int r = 0; r < ranks; ++r) {
    blks.push_back(decompose(P.M, P.N, pg, r));
    s.push_back(std::make_unique<DeviceSolver>(P, blks.back(), nullptr, opt));
  }
  const bool fused = s[0]->fused();
  // multi-step sweeps (three-step on blocks of >= 12 x 12): one launch per
  // `steps` iterations, the exchange after each, the kNS3 sums summed here
  const int steps = s[0]->sweep_steps();
  const bool ms = s[0]->two_step();
  const int nsum = dev::sweep_sums(steps);
  std::vector<hipEvent_t> ev(ranks);
  for (auto& e : ev) PE_HIP_CHECK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
  // Device pointer tables for the cross-rank reduction kernel:
  // [red_F | red_G | err | fs0 | fs1] × ranks (multi-step: fs2[0] / fs2[1]
  // in the fs slots).
  std::vector<double*> hp(5 * ranks);
  for (int r = 0; r < ranks; ++r) {
    hp[r] = s[r]->red_F_dev();
    hp[ranks + r] = s[r]->red_G_dev();
    hp[2 * ranks + r] = s[r]->err_dev();
    hp[3 * ranks + r] = ms ? s[r]->fs2_dev(0) : s[r]->fs_dev(0);
    hp[4 * ranks + r] = ms ? s[r]->fs2_dev(1) : s[r]->fs_dev(1);
  }
  double** dp = nullptr;
  PE_HIP_CHECK(hipMalloc(&dp, sizeof(double*) * 5 * ranks));
  PE_HIP_CHECK(hipMemcpy(dp, hp.data(), sizeof(double*) * 5 * ranks, hipMemcpyHostToDevice));
  hipStream_t s0 = s[0]->stream();

  auto join_all = [&]() {
    for (int r = 0; r < ranks; ++r) PE_HIP_CHECK(hipEventRecord(ev[r], s[r]->stream()));
    for (int r = 1; r < ranks; ++r) PE_HIP_CHECK(hipStreamWaitEvent(s0, ev[r], 0));
  };
  auto fork_all = [&]() {
    PE_HIP_CHECK(hipEventRecord(ev[0], s0));
    for (int r = 1; r < ranks; ++r) PE_HIP_CHECK(hipStreamWaitEvent(s[r]->stream(), ev[0], 0));
  };
  auto reduce = [&](double* const* table, int n, int is_max) {
    join_all();
    dev::launch_group_reduce(table, ranks, n, is_max, s0);
    fork_all();
  };
  // Same halo phases as under RCCL; the transport is a D2D copy from the
  // peer's send region once the peer's stream has produced it.
  auto exchange = [&](int buf, bool after_sweep) {
    // (multi-step sweeps do not store their y strips: packed here)
    if (ms && after_sweep)
      for (int r = 0; r < ranks; ++r) s[r]->enqueue_pack(buf);
    std::vector<std::vector<DeviceSolver::HaloPhase>> plan(ranks);
    for (int r = 0; r < ranks; ++r) plan[r] = s[r]->halo_phases(buf);
    for (size_t ph = 0; ph < plan[0].size(); ++ph) {
      for (int r = 0; r < ranks; ++r) PE_HIP_CHECK(hipEventRecord(ev[r], s[r]->stream()));
      for (int r = 0; r < ranks; ++r)
        for (const auto& e : plan[r][ph].ex) {
          const Exchange* src = nullptr;
          for (const auto& pe : plan[e.peer][ph].ex)
            if (pe.dir == opposite(e.dir)) src = &pe;
          if (!src || src->count != e.count) throw std::runtime_error("group halo plan mismatch");
          PE_HIP_CHECK(hipStreamWaitEvent(s[r]->stream(), ev[e.peer], 0));
          PE_HIP_CHECK(hipMemcpyAsync(e.recv, src->send, sizeof(double) * e.count, hipMemcpyDeviceToDevice,
                                      s[r]->stream()));
        }
      for (int r = 0; r < ranks; ++r)
        if (plan[r][ph].unpack) s[r]->enqueue_unpack(buf);
    }
  };

  for (int r = 0; r < ranks; ++r) s[r]->enqueue_init();
  if (fused) {
    for (int r = 0; r < ranks; ++r) s[r]->enqueue_pack(0);
    exchange(0, false);
    for (int r = 0; r < ranks; ++r) s[r]->enqueue_S(1);
    exchange(1, true);
    reduce(dp + 4 * ranks, nsum, 0);
  } else {
    exchange(0, false);
    reduce(dp + ranks, 1, 0);
  }
  PE_HIP_CHECK(hipStreamSynchronize(s0));
  SolveResult res;
  res.t.setup = secs(t_start, clk::now());
  const auto t_loop = clk::now();
  const int64_t cap = P.iter_cap();
  const int chunk = s[0]->chunk();
  DevState hs;
  int64_t k = 0;
  int64_t nsweep = 0;  // launches (parity)
  for (;;) {
    for (int it = 0; it < chunk; it += steps, k += steps, ++nsweep) {
      const int par = int(nsweep & 1);
      if (fused) {
        // (multi-step: the sweep applies min(steps, cap - K) iterations and
        // resolves its predecessor's stop tests itself)
        for (int r = 0; r < ranks; ++r) s[r]->enqueue_S(par);
        exchange(par, true);
        reduce(dp + (3 + par) * ranks, nsum, 0);
        continue;
      }
      for (int r = 0; r < ranks; ++r) s[r]->enqueue_F(par);
      reduce(dp, 2, 0);
      for (int r = 0; r < ranks; ++r) s[r]->enqueue_G(par);
      exchange(0, false);
      reduce(dp + ranks, 1, 0);
    }
    s[0]->read_state(&hs);
    if (hs.done || k >= cap + (ms ? steps : 0)) break;
  }
  for (int r = 0; r < ranks; ++r) s[r]->synchronize();
  res.t.iterate = secs(t_loop, clk::now());
  res.t.gpu = res.t.iterate;
  for (int r = 0; r < ranks; ++r) s[r]->enqueue_wflush();
  if (opt.compute_error) {
    for (int r = 0; r < ranks; ++r) s[r]->enqueue_error();
    reduce(dp + 2 * ranks, 1, 0);
    // max over the two max slots: table entries point at err[0]; offset by one.
    std::vector<double*> hm(ranks);
    for (int r = 0; r < ranks; ++r) hm[r] = s[r]->err_dev() + 1;
    double** dm = nullptr;
    PE_HIP_CHECK(hipMalloc(&dm, sizeof(double*) * ranks));
    PE_HIP_CHECK(hipMemcpy(dm, hm.data(), sizeof(double*) * ranks, hipMemcpyHostToDevice));
    reduce(dm, 2, 1);
    PE_HIP_CHECK(hipStreamSynchronize(s0));
    PE_HIP_CHECK(hipFree(dm));
  }
  for (int r = 0; r < ranks; ++r) s[r]->synchronize();
  s[0]->read_state(&hs);
  res.iters = hs.iter;
  res.converged = hs.status == 1;
  res.breakdown = hs.status == 2;
  res.nonfinite = hs.status == 4;
  if (hs.status == 5) throw std::runtime_error("single-sweep: boundary partials never arrived (internal error)");
  res.last_diff = hs.last_diff;
  res.zr = hs.rz_cur;
  if (opt.compute_error) {
    res.l2_err = std::sqrt(hs.err[0] * P.h1() * P.h2());
    res.max_err = hs.err[1];
    res.max_outside = hs.err[2];
  }
  if (w_out) {
    const int64_t ny = P.N - 1;
    w_out->assign(size_t((P.M - 1) * ny), 0.0);
    for (int r = 0; r < ranks; ++r) {
      const Block& b = blks[r];
      std::vector<double> tmp(size_t(b.nx * b.ny));
      s[r]->copy_w(tmp.data());
      for (int64_t li = 0; li < b.nx; ++li)
        std::copy(tmp.begin() + li * b.ny, tmp.begin() + (li + 1) * b.ny,
                  w_out->begin() + (b.i0 - 1 + li) * ny + (b.j0 - 1));
    }
  }
  PE_HIP_CHECK(hipFree(dp));
  for (auto& e : ev) PE_HIP_CHECK(hipEventDestroy(e));
  res.backend = "hip-group";
  res.algo = steps == 3 ? "three-step" : steps == 2 ? "two-step" : fused ? "fused" : "classic";
  res.Px = pg.Px;
  res.Py = pg.Py;
  res.t.solver = secs(t_start, clk::now());
  return res;
}

}  // namespace pe
