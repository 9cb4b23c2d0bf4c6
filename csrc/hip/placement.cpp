// Memory placement of the solver fields: the placement search that picks,
// among a few candidate allocations, the one the sweep streams fastest from
// (DeviceSolver::choose_placement).
#include <hip/hip_runtime_api.h>

#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <map>
#include <limits>
#include <mutex>
#include <queue>
#include <string>
#include <vector>

#include <rocprofiler-sdk-roctx/roctx.h>

#include "../hip/kernels.hpp"
#include "pe/device.hpp"
#include "solver_internal.hpp"

namespace pe {

namespace detail {
// Field allocation: plain hipMalloc.  (Physically contiguous memory and
// shuffled physical chunks mapped through the virtual memory API were
// measured as placement experiments in round 2 — contiguous slowest, chunks
// fast on one box and slow on the next, profiles/r2_placement.txt — and
// removed in round 6; the placement search below is what makes the speed
// robust.)  nullptr when the device is out of memory.
void* field_try_alloc(size_t bytes) {
  void* p = nullptr;
  if (hipMalloc(&p, bytes) != hipSuccess) {
    (void)hipGetLastError();
    return nullptr;
  }
  return p;
}

void* field_alloc(size_t bytes) {
  void* p = field_try_alloc(bytes);
  if (!p) PE_HIP_CHECK(hipErrorOutOfMemory);
  return p;
}

void field_free(void* p) {
  if (p) (void)hipFree(p);
}
}  // namespace detail

using detail::clk;
using detail::field_free;
using detail::field_try_alloc;
using detail::Range;
using detail::secs;
using dev::KParams;

// Memory-placement autotune (single-sweep, large blocks).  The same sweep
// runs at two distinct speeds depending on which physical memory its arrays
// land in (8192²: ≈1380 vs ≈1510 it/s; stable per allocation; consecutive
// allocations come in slow and fast runs of several GB; no dependence on
// row padding, virtual address or TLB misses — the slow placements show ~1.7×
// the DRAM credit stalls; docs/PERFORMANCE.md).  Try up to
// PE_PLACEMENT_TRIES (default 8) candidate allocations, each after a
// 8 GB spacer so it lands in another region;
// time a few local sweeps on real data (no communication) and keep the
// fastest (stop early once one is clearly in the fast class).  Everything else is freed; an allocation failure ends the search.
//
// Multi-rank jobs: the in-sweep sums couple the ranks every iteration, so the
// job runs at its slowest rank's placement.  After the local searches the
// ranks agree (max-allreduce) whether any of them missed the best class;
// if so, those ranks search once more (same 0.3 s cap, past the memory the
// first round tried) while the others wait at the next collective, and the
// job's max ms/sweep is recorded (bench.py reports it with every rank's
// candidates).  Every rank makes the same collective calls whatever its
// local search did (job-wide MAX semantics of the reference's timer
// reduction, poisson_mpi_cuda2.cu:962-966).
void DeviceSolver::choose_placement() {
  const double t_all = placement_s_;
  const auto t0 = clk::now();
  const bool fast = placement_search(false);
  if (comm_->size() > 1) {
    double v[1] = {(!placement_ms_.empty() && !fast) ? 1.0 : 0.0};
    comm_->host_max(v, 1, stream_);
    if (v[0] > 0.0 && !placement_ms_.empty() && !fast) placement_search(true);
    double m[1] = {placement_ms_.empty() ? 0.0 : double(placement_ms_[size_t(placement_best_)])};
    comm_->host_max(m, 1, stream_);
    placement_job_ms_ = m[0];
  } else if (!placement_ms_.empty()) {
    placement_job_ms_ = placement_ms_[size_t(placement_best_)];
  }
  placement_s_ = t_all + secs(t0, clk::now());
}

bool DeviceSolver::placement_search(bool retry) {
  Range range("pe.placement_search");
  double search_s = 0;
  struct Clock {
    double& out;
    clk::time_point t0 = clk::now();
    ~Clock() { out = secs(t0, clk::now()); }
  } clock{search_s};
  const double pts = double(blk_.nx) * double(blk_.ny);
  // Only large blocks: the two-speed placement was measured at 8192² (≈9 %);
  // at 2400×3200 / 4096² the candidates differ by ≤ 3-7 % while the spacer
  // allocations cost 0.02-6 s of construction (T_solver) depending on the
  // allocator state (profiles/r2_ctor_probe.txt).
  // 12 tries (the 40 % memory cap below allows 11 at 8192²): a box whose
  // first 8 held no best-class placement ran 1800 vs 1843 it/s
  // (profiles/r2_validate_s4b.txt), and the final validation's 2000-step
  // process found its best-class candidate at the 9th try (1838 it/s,
  // profiles/r2_validate_final.txt); a try costs ≈6 ms, and the search
  // stops at the first best-class candidate.
  // (Multi-GPU blocks of 4-24 M nodes have no search: their job runs at its
  // worst rank's placement — 8-rank slab block of 8192² 37.5-40.0 µs per
  // iteration over fresh solvers, 37.0-38.2 with a search — but the search
  // that found their fast placements took 0.5 s of construction in a fresh
  // process (8 tries past 12 GB spacers), and 4 tries past 8 GB stayed in one
  // slow run of allocations: profiles/r6_placement.txt, measured in round 6,
  // not adopted.)
  int tries = pts >= 24.0e6 ? 12 : 1;
  if (retry) tries = std::max(1, tries / 2 + 1);  // the kept candidate + half a round
  if (const char* e = std::getenv("PE_PLACEMENT_TRIES")) tries = std::max(1, std::atoi(e));
  const double skip_gb = 8.0;
  // best-class threshold: the single sweep's 40 B/node at ≥ 4.9 TB/s (8192²:
  // ≤ 0.548 ms); the two-step sweep's 48 B/node per sweep at ≥ 4.7 TB/s
  // (8192²: its classes are 0.676-0.69 and 0.83-0.85 ms per sweep); the
  // three-step sweep's 48 B/node per sweep at ≥ 4.4 TB/s (8192²: ≤ 0.732 ms;
  // with the aligned strips and 112-row items its classes are 0.709-0.722,
  // 0.74, 0.78-0.79 and 0.83-0.85 ms, the first fast one usually the 5th try —
  // profiles/r4_bench112.txt; 4.2 stopped at 0.743 ms candidates) — 4.45 TB/s
  // (≤ 0.724 ms) since round 6: 4.4 accepted a 0.7295 ms candidate and the
  // bench ran 3876 it/s against 4011-4136 with 0.701-0.722 ms picks
  // (profiles/r6_placement.txt)
  // Blocks of 24-50 M nodes (the 2-rank split of 8192²) stream slower per
  // byte: their best candidates are 0.396-0.400 ms per sweep at 33.5 M nodes =
  // 4.03-4.06 TB/s, so the three-step rate there is 4.0 TB/s — at 4.45 no
  // candidate ever qualified, every rank then ran the retry round, and its
  // spacer past the first round's memory took 1-4 s of construction
  // (profiles/r6_placement.txt)
  const bool mid_large = pts < 50.0e6;
  const double fast_tbs = steps_ >= 3 ? (mid_large ? 4.0 : 4.45) : sstep_ ? 4.7 : 4.9, max_s = 0.3;
  if (tries <= 1) return true;
  // spacers are transient; never let the search take more than 40 % of the
  // free memory (several solvers may share the device)
  {
    const double frac = 0.4;
    size_t free_b = 0, total_b = 0;
    if (hipMemGetInfo(&free_b, &total_b) == hipSuccess) {
      const double per_try = skip_gb * double(1ull << 30) + double(sizeof(double) * (2 * xsize_ + wsize_));
      tries = std::min<int>(tries, std::max(1, int(frac * double(free_b) / per_try)));
    }
  }
  if (tries <= 1) return true;
  struct Cand {
    double *x0, *x1, *w;
    float ms;
  };
  std::vector<Cand> c;
  std::vector<void*> spacers;
  c.push_back(Cand{fields_, xalt_, walt_, 0.f});
  // a retry first steps past the memory the first round tried (its spacers
  // and candidates were freed: the allocator would hand them out again)
  const size_t n_first = placement_ms_.size();
  if (retry && skip_gb > 0) {
    const double gb = double(n_first) * (skip_gb + double(sizeof(double) * (2 * xsize_ + wsize_)) / double(1ull << 30));
    void* sp = nullptr;
    if (hipMalloc(&sp, size_t(gb * double(1ull << 30))) == hipSuccess) spacers.push_back(sp);
    else (void)hipGetLastError();
  }
  bool fast = false;
  for (int t = 0; t < tries; ++t) {
    if (t > 0) {
      void* sp = nullptr;
      if (skip_gb > 0 && hipMalloc(&sp, size_t(skip_gb * double(1ull << 30))) != hipSuccess) break;
      if (sp) spacers.push_back(sp);
      void* a = field_try_alloc(sizeof(double) * xsize_);
      if (!a) break;
      void* b = field_try_alloc(sizeof(double) * xsize_);
      if (!b) {
        field_free(a);
        break;
      }
      void* w = field_try_alloc(sizeof(double) * wsize_);
      if (!w) {
        field_free(a);
        field_free(b);
        break;
      }
      c.push_back(Cand{static_cast<double*>(a), static_cast<double*>(b), static_cast<double*>(w), 0.f});
    }
    set_fused_fields(c[t].x0, c[t].x1, c[t].w);
    enqueue_init();
    dev::launch_S(*kp_, 1, stream_);  // S_0 on real data (local sums only)
    for (int i = 0; i < 2; ++i) dev::launch_S(*kp_, i & 1, stream_);
    PE_HIP_CHECK(hipEventRecord(t0_, stream_));
    for (int i = 0; i < 6; ++i) dev::launch_S(*kp_, i & 1, stream_);
    PE_HIP_CHECK(hipEventRecord(t1_, stream_));
    PE_HIP_CHECK(hipEventSynchronize(t1_));
    PE_HIP_CHECK(hipEventElapsedTime(&c[t].ms, t0_, t1_));
    // The placements fall into classes (8192²: 0.541-0.547, 0.556-0.562,
    // 0.59-0.61 and 0.62-0.65 ms per sweep; the bench follows them: 1792 vs
    // 1745 it/s for the first two, profiles/r2_bench_launch.txt).  A try costs
    // ≈6 ms (spacer, allocation, 9 sweeps), the best class saves ≈3 % of a
    // 3.3 s solve: keep the best of all tries, stopping early only at the
    // best class — the sweep's average 40 B/node streamed at >=
    // fast_tbs (4.9 TB/s = 0.548 ms at 8192²).  (Earlier stop
    // rules — 5 % / 7 % below the slowest seen, 4.6 / 4.75 TB/s — settled for
    // 0.56-0.60 ms placements when better ones were a try or two further.)
    const double bps = sstep_ ? 48.0 : 40.0;  // streamed bytes per node and sweep
    const double tbs = bps * pts / (double(c[t].ms) / 6.0 * 1e-3) / 1e12;
    if (tbs >= fast_tbs) {
      fast = true;
      break;
    }
    // spacer allocations are cheap on fresh memory but can take seconds
    // when the allocator must clear reused memory (profiles/r2_ctor_probe.txt):
    // the search is capped at 0.3 s of wall time
    if (secs(clock.t0, clk::now()) > max_s) break;
  }
  (void)hipGetLastError();  // clear a failed search allocation
  size_t best = 0;
  for (size_t i = 1; i < c.size(); ++i)
    if (c[i].ms < c[best].ms) best = i;
  for (size_t i = 0; i < c.size(); ++i)
    if (i != best) {
      field_free(c[i].x0);
      field_free(c[i].x1);
      field_free(c[i].w);
    }
  for (void* sp : spacers) PE_HIP_CHECK(hipFree(sp));
  set_fused_fields(c[best].x0, c[best].x1, c[best].w);
  if (!retry) placement_ms_.clear();
  // a retry appends its candidates (its first is the first round's pick, re-timed)
  placement_best_ = int(placement_ms_.size() + best);
  for (const Cand& x : c) placement_ms_.push_back(x.ms / 6.0f);
  // (below 50 M nodes no retry round: the best of this round stands)
  return fast || mid_large || (sstep_ ? 48.0 : 40.0) * pts / (double(c[best].ms) / 6.0 * 1e-3) / 1e12 >= fast_tbs;
}

}  // namespace pe
