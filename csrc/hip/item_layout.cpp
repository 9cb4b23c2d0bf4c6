// Work-item layout of the single-sweep kernel: rows per item, the item
// lists (cost-aware static LPT layout or per-XCD dynamic queues, boundary
// items first for the halo push / overlap) and the LDS-resident kernel's
// tiles (DeviceSolver::set_items / setup_items / setup_resident).
#include <hip/hip_runtime_api.h>

#include <algorithm>
#include <array>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <exception>
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

using detail::clk;
using detail::Range;
using detail::secs;
using dev::DevState;
using dev::KParams;

// Items of `ti` rows: counts and the persistent grids sized for them.
void DeviceSolver::set_items(int ti) {
  KParams& k = *kp_;
  k.ti = ti;
  k.nitems = int(int64_t(k.nstrips) * ((blk_.nx + ti - 1) / ti));
  // fewest waves that keep every wave's share of the n items equal
  auto grid_for = [&](int cap, int n) {
    const int per = (n + cap - 1) / cap;
    const int waves = (n + per - 1) / per;
    return std::max(1, (waves + dev::kWPB - 1) / dev::kWPB);
  };
  k.nblocks = grid_for(wave_caps_[0], k.nitems);
  k.nblocks0 = grid_for(wave_caps_[1], k.nitems);
  k.nslots = k.nitems;
  static_waves_ = 0;
}

// Halo/interior overlap (multi-rank single-sweep).  The sweep walks an item
// list in which, per XCD shard, the boundary items (outputs sent to a
// neighbour: first / last two owned rows and columns) come first; each bumps
// st->sig when stored.  A one-wave kernel on a high-priority halo stream waits
// for the count, then the exchange runs there while the interior items are
// still being computed.  The sweep keeps its full persistent grid minus
// 8 blocks left free for the wait / exchange /
// unpack kernels.  PE_OVERLAP=0 disables.
//
// Every dynamic (order 3) sweep walks such lists, overlap or not.  Item cost
// estimate (from stamps of the sweep, tools/stamp_probe.py): a row of a
// strip that contains boundary-band nodes (coefficients evaluated from the
// chord tables) costs ≈ kGenCost plain rows; an item's rows are its own plus
// the 4 halo rows it re-reads.  Shards are contiguous chunk ranges of equal
// estimated cost (consecutive chunks stay on one XCD), and each shard lists
// its boundary items (overlap) first, then its heavy items in decreasing
// cost, then the rest chunk-major: the sweep's tail is then made of light
// items, and waves steal from other shards once their own is empty.
void DeviceSolver::setup_items() {
  KParams& k = *kp_;
  const bool nb = blk_.has(LEFT) || blk_.has(RIGHT) || blk_.has(DOWN) || blk_.has(UP);
  // Halo/interior overlap: the construction's choice (choose_halo_path times
  // the exchange with and without it on the job's transport; PE_OVERLAP=1 / 0
  // restricts the choice).  Only where the sweep can signal its boundary items
  // (single sweep; the three-step sweep's kSignal variant, fused3.hip — not
  // the two-step sweep) and the halo is exchanged, not pushed.
  overlap_ = want_overlap_ && fused_ && (!sstep_ || steps_ >= 3) && comm_->size() > 1 && nb && !push_;
  // Lists: dynamic sweeps (order 3), static chunk-major sweeps (order 0:
  // heavy items split, below) and the overlap; orders 1 / 2 are plain
  // tuning walks.
  if (!fused_ || ((k.order == 1 || k.order == 2) && !overlap_)) return;
  if (lay_cache_on_) {
    auto it = lay_cache_.find({k.ti, overlap_, lay_name_});
    if (it != lay_cache_.end()) {
      if (!lay_dry_) restore_layout(it->second);
      return;
    }
  }
  struct Keep {  // (files the finished layout in the cache on every return below)
    DeviceSolver* s;
    ~Keep() {
      if (s->lay_cache_on_ && std::uncaught_exceptions() == 0)
        s->lay_cache_[{s->kp_->ti, s->overlap_, s->lay_name_}] = s->snap_layout();
    }
  } keep{this};
  const bool trace3 = std::getenv("PE_CTOR_TRACE") && std::atoi(std::getenv("PE_CTOR_TRACE")) >= 3;
  const auto tl0 = clk::now();
  auto lap = [&](const char* what) {
    if (trace3) std::fprintf(stderr, "[pe]   layout %-14s %7.3f ms\n", what, 1e3 * secs(tl0, clk::now()));
  };
  // (re-laid out by the rows-per-item tuning: the list buffer is reused while
  // it is large enough — a free per candidate synchronised the device)
  auto list_alloc = [&](size_t n) {
    if (n <= ilist_cap_) return;
    // (the rows-per-item tuning lays out while the previous candidate's
    // sweeps, which read the old list, may still run)
    PE_HIP_CHECK(hipStreamSynchronize(stream_));
    if (ilist_) PE_HIP_CHECK(hipFree(ilist_));
    ilist_cap_ = std::max(n, ilist_cap_ + ilist_cap_ / 2);
    PE_HIP_CHECK(hipMalloc(&ilist_, sizeof(int2) * ilist_cap_));
  };
  if (overlap_) {
    ov_reserve_ = 8;
    // timing experiments (PE_OV_DEBUG bits): 2 serial streams, 4 natural item
    // order (no boundary-first list)
    if (const char* d = std::getenv("PE_OV_DEBUG")) ov_debug_ = std::atoi(d);
  }
  const int gmin = std::max(1, std::min(k.nblocks, k.nblocks0) - (overlap_ ? ov_reserve_ : 0));
  const int nsh = k.order >= 2 ? std::min(8, gmin) : 1;
  const int nchunks = int((blk_.nx + k.ti - 1) / k.ti);
  // Cost of a boundary-band row in plain rows (item costs of the layouts).
  // Since the band coefficients are evaluated once per row (LDS ring) a band
  // row costs less than the round-1 weight of 3: blocks below 2²⁴ nodes lay
  // out better at 2 (8-rank 8192² block 84.2-85.1 vs 87.3-87.8 µs per
  // iteration, 4-rank 155 vs 160, 2400×3200 77.9-79.3 vs 79.5-80.3; 1 is
  // worse everywhere); larger blocks see no difference above the placement
  // noise and keep 3 (profiles/r2_gencost.txt).
  double gen_cost = double(blk_.nx) * double(blk_.ny) >= double(1 << 24) ? 3.0 : 2.0;
  // three-step LPT at 2²⁵-2²⁶ nodes (8192², 112-row items): 3.25-4 run ≈1 %
  // faster than 3 on three boxes, 5-8 ≈8 % slower (profiles/r4_ti48.txt)
  if (steps_ >= 3 && double(blk_.nx) * double(blk_.ny) >= double(1 << 25) &&
      double(blk_.nx) * double(blk_.ny) <= double(1 << 26))
    gen_cost = 3.5;
  const bool sort_heavy = true, split_heavy = true;  // heavy items first (dynamic) / split (static)
  // per-item cost: rows ib-2 .. ie+2, band rows weighted
  const int64_t rows_tab = int64_t(rowcls_host_.size() / 4);
  // Does local row q have a boundary-band node in strip s's loaded
  // columns?  (The kernel's has_gen on the same row-class table.)
  const int H = hdep_;  // halo rows an item re-reads per side (2 single sweep, 4 two-step, 6 three-step)
  const int HL = xorg_ + 1;  // a strip's left halo columns (three-step: 8, for aligned loads and stores)
  const int64_t Wc = steps_ >= 3 ? 64 : 128;  // columns a wave strip loads (three-step: one per lane)
  auto row_gen_x = [&](int64_t q, int s) {
    const int64_t J = -(HL - 1) + int64_t(s) * fsw_;
    const int64_t t = q - tab_lo_;  // table index of local row q
    if (t < 0 || t >= rows_tab) return false;
    const int* r = &rowcls_host_[size_t(t) * 4];
    const int64_t lo = std::max<int64_t>(J, r[2]), hi = std::min<int64_t>(J + Wc - 1, r[3]);
    return lo <= hi && (r[0] > r[1] || lo < r[0] || hi > r[1]);
  };
  // {first row | band flag, strip | rows << 20}; the band flag selects the
  // kernel's coefficient path (rows ib-H .. ie+H include a boundary-band row)
  // Three-step sweep: is every row of the item's window wholly interior or
  // wholly non-interior in the strip's 64 columns (kUniBit: the kernel's
  // uniform-row march)?  Rows with a band node are never uniform here: the
  // band flag wins.
  auto row_mixed_x = [&](int64_t q, int s) {
    const int64_t J = -(HL - 1) + int64_t(s) * fsw_;
    const int64_t t = q - tab_lo_;
    if (t < 0 || t >= rows_tab) return true;
    const int* r = &rowcls_host_[size_t(t) * 4];
    const int64_t lo = std::max<int64_t>(J, r[0]), hi = std::min<int64_t>(J + Wc - 1, r[1]);
    if (lo > hi) return false;                 // no interior column
    return !(r[0] <= J && r[1] >= J + Wc - 1);  // some interior, some not
  };
  // Per strip, prefix counts of the band / mixed rows q = 1-H .. nx+H (the
  // windows of every item; built once per solver: the rows-per-item tuning
  // re-lays out up to 11 times, and evaluating the rows one by one per item
  // took 4.5-5.7 ms per layout at 4096², inside T_solver).
  const int64_t q0 = 1 - H, R = blk_.nx + 2 * H;
  lap("start");
  if (pgen_.empty()) {
    pgen_.assign(size_t(k.nstrips) * size_t(R + 1), 0);
    pmix_.assign(size_t(k.nstrips) * size_t(R + 1), 0);
    for (int s = 0; s < k.nstrips; ++s) {
      int* g = &pgen_[size_t(s) * size_t(R + 1)];
      int* m = &pmix_[size_t(s) * size_t(R + 1)];
      for (int64_t i = 0; i < R; ++i) {
        g[i + 1] = g[i] + (row_gen_x(q0 + i, s) ? 1 : 0);
        m[i + 1] = m[i] + (row_mixed_x(q0 + i, s) ? 1 : 0);
      }
    }
  }
  // band / mixed rows among q = a .. b of strip s (inside 1-H .. nx+H)
  auto ngen = [&](int64_t a, int64_t b, int s) {
    const int* g = &pgen_[size_t(s) * size_t(R + 1)];
    return g[b - q0 + 1] - g[a - q0];
  };
  auto nmix = [&](int64_t a, int64_t b, int s) {
    const int* m = &pmix_[size_t(s) * size_t(R + 1)];
    return m[b - q0 + 1] - m[a - q0];
  };
  auto rows_cost = [&](int64_t ib, int64_t ie, int s) {
    const int64_t n = ie - ib + 1 + 2 * H, ng = ngen(ib - H, ie + H, s);
    return double(n - ng) + double(ng) * gen_cost;
  };
  auto rows_band = [&](int64_t ib, int64_t ie, int s) { return ngen(ib - H, ie + H, s) > 0; };
  auto rows_uniform = [&](int64_t ib, int64_t ie, int s) {
    return ngen(ib - H, ie + H, s) == 0 && nmix(ib - H, ie + H, s) == 0;
  };
  auto item_cost = [&](int ch, int s) {
    const int64_t ib = 1 + int64_t(ch) * k.ti, ie = std::min<int64_t>(ib + k.ti - 1, blk_.nx);
    return rows_cost(ib, ie, s);
  };
  auto entry = [&](int64_t ib, int64_t rows, int s) {
    int flag = rows_band(ib, ib + rows - 1, s) ? dev::kBandBit : 0;
    // (not the last strip of a block with an UP neighbour: its output lanes
    // past ny hold that neighbour's columns, which only the lane-tested
    // march keeps out of the sums)
    const bool cut = (blk_.has(UP) && int64_t(s + 1) * fsw_ > blk_.ny);
    if (flag == 0 && steps_ >= 3 && !cut && rows_uniform(ib, ib + rows - 1, s)) flag = dev::kUniBit;
    return int2{int(ib) | flag, s | int(rows << 20)};
  };
  // outputs a neighbour needs: first in the layout under the overlap (they
  // feed the exchange) and under the halo push (their xGMI stores then
  // overlap the rest of the sweep instead of ending it)
  // The halo push keeps the plain layout: cutting its boundary pieces off and
  // dealing them first (the pre-round-5 layout) cost the push kernel 10 % at
  // the 8-rank slab of 8192² (64.6-65.1 vs 58.2 µs per iteration) and 4 % at
  // 4 ranks, loopback probe, profiles/r5_push_release.txt
  const bool push_first = false;
  auto is_boundary = [&](int64_t ib, int64_t ie, int s) {
    const int64_t J = -(HL - 1) + int64_t(s) * fsw_;
    const int64_t jlo = std::max<int64_t>(1, J + HL), jhi = std::min<int64_t>(blk_.ny, J + fsw_ + HL - 1);
    // (the H owned rows / columns next to a neighbour: what the exchange sends)
    return ((overlap_ && !(ov_debug_ & 4)) || push_first) &&
           ((blk_.has(LEFT) && ib <= H) || (blk_.has(RIGHT) && ie >= blk_.nx - H + 1) || (blk_.has(DOWN) && jlo <= H) ||
            (blk_.has(UP) && jhi >= blk_.ny - H + 1));
  };

  if (k.order == 0) {
    // ---- Static sweeps: a longest-processing-time-first layout ----
    // Every wave walks list positions w, w + W, w + 2W, … (W = the grid's
    // waves), so the host decides who does what: items are cut where one
    // would exceed a wave's fair share (band items cost ≈2-3× a plain one;
    // on small blocks, where each wave gets about one item, the band items
    // alone were the sweep's tail — profiles/r2_small_before.txt), then
    // assigned heaviest first to the least-loaded wave, and a wave's k-th
    // item goes to position k·W + w (empty entries fill the gaps).  Equal
    // costs keep chunk-major order, so each round of positions still covers
    // a compact window of rows.  Overlap: boundary items take the first
    // positions (they run in the first round).
    struct Piece {
      int64_t ib, rows;
      int s;
      double cost;
      bool bnd;
    };
    const double overhead = 3.0;  // per-item prologue / epilogue, in row steps (stamps)
    int waves_avail = std::max(dev::kWPB, wave_cap_ - (overlap_ ? ov_reserve_ * dev::kWPB : 0));
    double total = 0.0;
    for (int id = 0; id < k.nitems; ++id) total += item_cost(id / k.nstrips, id % k.nstrips) + overhead;
    // cut only when there are fewer items than waves (small blocks): with
    // more items than waves the layout balances them, and every cut re-reads
    // 4 more halo rows (2048²: 96 vs 91 µs per iteration with cuts)
    const int W0 = std::max(1, std::min(waves_avail, k.nitems));
    const double share = k.nitems >= waves_avail ? 1e300 : std::max(total / W0, (double(k.ti + 2 * H) + overhead) * 1.15);
    std::vector<Piece> pcs;
    for (int ch = 0; ch < nchunks; ++ch)
      for (int s = 0; s < k.nstrips; ++s) {
        const int64_t ib = 1 + int64_t(ch) * k.ti, ie = std::min<int64_t>(ib + k.ti - 1, blk_.nx);
        const int64_t n = ie - ib + 1;
        const bool bnd = is_boundary(ib, ie, s);
        int parts = 1;
        if (split_heavy && !bnd) {
          for (; 2 * (parts + 1) <= n; ++parts) {  // pieces of >= 2 rows
            double worst = 0.0;
            for (int q = 0; q < parts; ++q)
              worst = std::max(worst, rows_cost(ib + n * q / parts, ib + n * (q + 1) / parts - 1, s) + overhead);
            if (worst <= share) break;
          }
        }
        for (int q = 0; q < parts; ++q) {
          const int64_t a0 = ib + n * q / parts, a1 = ib + n * (q + 1) / parts;
          pcs.push_back(Piece{a0, a1 - a0, s, rows_cost(a0, a1 - 1, s) + overhead, bnd});
        }
      }
    lap("pieces");
    // Three-step sweep: a filling layout instead.  The sweep's time per row
    // step depends on the item's kind — a boundary-band item ≈2.2×, a mixed
    // one ≈1.3× a uniform one (tools/stamp_probe.py, profiles/r4_stamps.txt)
    // — and the LPT layout below, with whole items, leaves some waves one item
    // more than the rest (8192²: 8 or 9 items of 92 row steps, wave busy
    // time max/mean 1.08) or a single band item longer than every other
    // wave's work (8-rank slab block: 1.33).  Here an item costs its steps ×
    // its kind's factor + the overhead, every wave is filled up to the fair
    // share T, and the item that would overflow the least-loaded wave is cut:
    // the rows that fit go there, the rest goes back into the queue (each cut
    // re-reads 2H fill rows, which T accounts for).  Largest first, ties in
    // chunk-major order, so each round of positions still covers a compact
    // window of rows.  PE_LAYOUT=lpt keeps the LPT layout.
    // three-step layouts: PE_LAYOUT forces one; else the construction's
    // choice (lay_name_: by block size, or by the rows-per-item tuning)
    std::string lay = std::getenv("PE_LAYOUT") ? std::getenv("PE_LAYOUT") : lay_name_;
    // (the overlap's short boundary pieces: the filling layout, below — on
    // blocks of about one item per wave, where whole boundary items end with
    // the sweep: 4×2 block of 8192² 59.3 µs per iteration at 15 / 8 µs delays
    // vs 57.5 without delays or overlap.  Larger blocks keep their layout with
    // whole boundary items first, which already runs them in the first of
    // several rounds; the filling layout cost the 2×2 block 18 % there —
    // 108 vs 90.9 µs at zero delay, profiles/r5_overlap.txt)
    if (overlap_ && !std::getenv("PE_LAYOUT") && double(blk_.nx) * double(blk_.ny) < 1.2e7) lay = "fill";
    const bool s3lay = steps_ >= 3;
    if (!s3lay) lay = "lpt";
    const bool equal = s3lay && lay == "equal";
    const bool fill = s3lay && lay == "fill";
    lay_used_ = equal ? "equal" : fill ? "fill" : "lpt";
    int W = std::max(dev::kWPB, (std::min<int>(waves_avail, int(pcs.size())) / dev::kWPB) * dev::kWPB);
    std::vector<std::vector<int>> per;
    std::vector<double> load;
    int nbnd = 0;
    // row-step cost of a band / mixed item, uniform = 1 (profiles/r4_stamps*.txt).
    // Band 2.8 since round 5 (the equal-cost / filling layouts of mid-size
    // blocks; one box, two constructions each, µs per iteration at 2.45 / 2.8
    // / 3.1 / 3.4: 8-rank slab of 8192² 43.0 / 40.4-40.8 / 40.4 / 40.0-40.6,
    // its 4×2 block 48.0 / 45.3-45.5 / 46.2-46.5 / 44.0-44.3, 4-rank ≈74
    // throughout, 2048² 28.1-28.7 / 28.4-28.5 / 29.3 / 30.5-30.7 —
    // profiles/r5_costband.txt; the slab's band row step runs ≈3.0× a uniform
    // one, 8192²'s 2.25×)
    double fband = 2.8, fmixed = 1.3;
    // (ties among equally loaded waves go in wave order; one wave per
    // workgroup in turn measured neutral to 1 % slower on the 8192² splits,
    // round 5 — removed in round 6)
    auto wfrom = [](int r, int) { return r; };
    auto wrank = [](int w, int) { return w; };
    // Wave capacity: workgroup b < cus_ is the first one dispatched to its CU,
    // b ≥ cus_ the second; the SIMDs' age-ordered issue runs the first
    // workgroup's waves ≈12 % faster per row step at the 8-rank slab of
    // 8192² and 2048² (0.86 vs 0.97 µs), ≈23 % at 8192² (0.77 vs 0.95) — and
    // the slow half follows the workgroup, not the rows it marches: with the
    // lists on the workgroups in reverse order the rows' speeds reverse and
    // the workgroups' stay (PE_WPERM, tools/stamp_probe.py,
    // profiles/r5_wave_age.txt).  The fill and LPT layouts can give the first
    // workgroups' waves rho times the load of the others (PE_YOUNG = rho).
    // Measured NEUTRAL on the mid-size blocks (8-rank slab 39.5-39.8 µs per
    // iteration at rho 1.0-1.3, 4×2 43.9-44.1, 4-rank 71.9-72.5) and slower
    // at 8192² from 1.2 (3975 / 3719 it/s vs 4009): a second-slot wave speeds
    // up once its SIMD partner is done, so the SIMD stays busy either way
    // (profiles/r5_epilogue.txt).  Default 1: equal loads.
    double rho = 1.0;
    if (const char* e = std::getenv("PE_YOUNG")) rho = std::max(0.5, std::atof(e));
    auto capw = [&](int w, int Wn) {
      return (Wn / dev::kWPB > cus_ && w / dev::kWPB < cus_) ? rho : 1.0;
    };
    if (equal) {
      // Three-step sweep: EQUAL-COST PIECES, EXACTLY k PER WAVE.  Whole items
      // cannot balance ~8 items per wave: the waves hold 8 or 9 uniform items,
      // or a band item of 2.3 uniform ones (8192²: wave busy time max/mean
      // 1.06-1.08; the 8-rank slab block's waves with one 41-row band item ran
      // 1.30× the mean — tools/stamp_probe.py, profiles/r4_stamps*.txt).  So
      // every strip is cut into runs of one march kind (a row is "band" when a
      // boundary-band row lies within H rows of it — the kernel marches an
      // item whose window holds one on the band path — else "mixed" likewise,
      // else uniform), every run into n_g pieces of equal rows, with the n_g
      // chosen so that a piece costs X ≈ (its rows + 2H fill rows) × its
      // kind's factor + overhead everywhere and there are exactly k·W pieces;
      // the pieces, sorted by cost (ties in row order), are dealt in rounds of
      // W, snaking, so each wave gets k pieces and each round a compact window
      // of rows.  k follows the rows-per-item knob: uniform pieces of ≈ ti rows.
      // PE_LAYOUT=fill / lpt select the earlier layouts.
      const int64_t nx = blk_.nx;
      const int ns = k.nstrips;
      struct Seg {
        int64_t a, rows;
        int s;
        double f;
        bool bnd;
        int n;
      };
      // (the runs do not depend on the rows per item: found once per solver
      // and overlap setting — the scan of every row of every strip was a
      // quarter of each of the tuning's layouts)
      std::vector<std::array<int64_t, 4>>& runs = eq_runs_[overlap_ ? 1 : 0];
      if (runs.empty()) {
        for (int sx = 0; sx < ns; ++sx) {
          auto kind = [&](int64_t q) {  // 2 band, 1 mixed, 0 uniform (window q-H .. q+H)
            return ngen(q - H, q + H, sx) > 0 ? 2 : nmix(q - H, q + H, sx) > 0 ? 1 : 0;
          };
          int64_t a = 1;
          int ka = kind(1);
          for (int64_t q = 2; q <= nx + 1; ++q) {
            const int kq = q <= nx ? kind(q) : -1;
            // (pieces: also split where a neighbour's halo rows begin, so the push /
            // overlap boundary pieces stay small)
            const bool cut_b = (push_first || overlap_) && ((blk_.has(LEFT) && q == H + 1) || (blk_.has(RIGHT) && q == nx - H + 1));
            if (kq != ka || cut_b) {
              runs.push_back({a, q - a, sx, ka});
              a = q;
              ka = kq;
            }
          }
        }
      }
      std::vector<Seg> segs;
      segs.reserve(runs.size());
      for (const auto& r : runs)
        segs.push_back(Seg{r[0], r[1], int(r[2]), r[3] == 2 ? fband : r[3] == 1 ? fmixed : 1.0,
                           is_boundary(r[0], r[0] + r[1] - 1, int(r[2])), 1});
      lap("equal: runs");
      const int64_t minr = 8, maxr = 128;  // (pieces of the tuned heights' range)
      auto Fk = [&](double f) { return double(2 * H) * f + overhead; };  // a piece's fill rows + overhead
      // pieces of a run for a piece cost X: rows·f / (X − F) rounded, within [rows/maxr, rows/minr]
      auto nfor = [&](const Seg& g, double X) {
        const double want = double(g.rows) * g.f / std::max(1e-9, X - Fk(g.f));
        const int64_t lo = std::max<int64_t>(1, (g.rows + maxr - 1) / maxr), hi = std::max<int64_t>(lo, g.rows / minr);
        return int(std::min<int64_t>(hi, std::max<int64_t>(lo, std::llround(want))));
      };
      auto count = [&](double X) {
        int64_t P = 0;
        for (const Seg& g : segs) P += nfor(g, X);
        return P;
      };
      int64_t Pmax = 0, Pmin = 0;
      for (const Seg& g : segs) {
        Pmax += std::max<int64_t>(1, g.rows / minr);
        Pmin += std::max<int64_t>(1, (g.rows + maxr - 1) / maxr);
      }
      W = std::max<int>(dev::kWPB, int(std::min<int64_t>(waves_avail, Pmax) / dev::kWPB) * dev::kWPB);
      const double X0 = double(k.ti + 2 * H) + overhead;  // a uniform piece of ti rows
      int kr = int(std::max<int64_t>(1, std::llround(double(count(X0)) / W)));
      while (int64_t(kr) * W < Pmin) ++kr;
      while (kr > 1 && int64_t(kr) * W > Pmax) --kr;
      const int64_t P = std::min<int64_t>(Pmax, int64_t(kr) * W);
      // the piece cost X that gives P pieces (count(X) falls as X grows)
      double lo = Fk(fband) + 1e-3, hi = 1e9;
      for (int it = 0; it < 200 && hi - lo > 1e-9 * hi; ++it) {
        const double mid = 0.5 * (lo + hi);
        (count(mid) > P ? lo : hi) = mid;
      }
      for (Seg& g : segs) g.n = nfor(g, hi);
      lap("equal: bisect");
      // exactly P: add pieces where they are largest, remove where the merge is cheapest
      int64_t have = count(hi);
      auto pc = [&](const Seg& g, int n) { return double(g.rows) * g.f / n + Fk(g.f); };
      while (have != P) {
        int best = -1;
        double bv = 0.0;
        for (int i = 0; i < int(segs.size()); ++i) {
          const Seg& g = segs[size_t(i)];
          if (have < P && g.rows / (g.n + 1) >= minr) {
            const double v = pc(g, g.n);
            if (best < 0 || v > bv) best = i, bv = v;
          } else if (have > P && g.n > 1 && (g.rows + g.n - 2) / (g.n - 1) <= maxr) {
            const double v = pc(g, g.n - 1);
            if (best < 0 || v < bv) best = i, bv = v;
          }
        }
        if (best < 0) break;
        segs[size_t(best)].n += have < P ? 1 : -1;
        have += have < P ? 1 : -1;
      }
      lap("equal: exact P");
      if (trace3) std::fprintf(stderr, "[pe]   layout equal: %zu runs, %lld pieces\n", segs.size(), (long long)P);
      pcs.clear();
      for (const Seg& g : segs)
        for (int j = 0; j < g.n; ++j) {
          const int64_t a0 = g.a + g.rows * j / g.n, a1 = g.a + g.rows * (j + 1) / g.n;
          pcs.push_back(Piece{a0, a1 - a0, g.s, double(a1 - a0) * g.f + Fk(g.f), is_boundary(a0, a1 - 1, g.s)});
        }
      // boundary pieces first (push / overlap), then in row order (chunk-major:
      // a round of W positions covers a compact window of rows, and the
      // neighbouring strips of the same rows run on one workgroup's waves —
      // sorting by cost first scattered the rounds: 8192² 287 vs 254 µs per
      // iteration, profiles/r4_layout2.txt)
      std::vector<int> ord(pcs.size());
      for (size_t i = 0; i < ord.size(); ++i) ord[i] = int(i);
      // (row bands of ~ti rows by the pieces' centres, then strips: the
      // neighbouring strips of the same rows run on one workgroup's waves —
      // sorting by first row alone interleaved strips whose pieces start a
      // row apart: 8192² 279 vs 254 µs, profiles/r4_layout2.txt)
      auto band_of = [&](const Piece& p) { return (2 * p.ib + p.rows - 1) / (2 * int64_t(k.ti)); };
      std::stable_sort(ord.begin(), ord.end(), [&](int x, int y) {
        const Piece &a = pcs[size_t(x)], &b = pcs[size_t(y)];
        if (a.bnd != b.bnd) return a.bnd;
        const int64_t ra = band_of(a), rb = band_of(b);
        if (ra != rb) return ra < rb;
        return a.s != b.s ? a.s < b.s : a.ib < b.ib;
      });
      // Dealt round by round, one piece per wave: a round's boundary pieces
      // take its first waves (the kernel's kSignal variant counts list
      // positions 0 .. nbnd-1 as the boundary items), its odd pieces (short
      // runs, rounding: up to ±50 % off the target cost) the least-loaded
      // waves so far, heaviest first, and the rest (within ±15 %) the
      // remaining waves in order, so neighbouring strips stay on
      // neighbouring waves.
      lap("equal: sorted");
      per.assign(size_t(W), {});
      std::vector<double> wl(size_t(W), 0.0);
      std::vector<char> taken(size_t(W), 0);
      std::vector<int> byload(static_cast<size_t>(W), 0);
      for (size_t r0 = 0; r0 < ord.size(); r0 += size_t(W)) {
        const size_t r1 = std::min(ord.size(), r0 + size_t(W));
        std::vector<int> odd, norm;
        std::fill(taken.begin(), taken.end(), 0);
        int wb = 0;
        for (size_t i = r0; i < r1; ++i) {
          const Piece& p = pcs[size_t(ord[i])];
          if (p.bnd) {  // (ord: boundary pieces first, so these are waves 0, 1, … of the round)
            per[size_t(wb)].push_back(ord[i]);
            wl[size_t(wb)] += p.cost;
            taken[size_t(wb++)] = 1;
            ++nbnd;
            continue;
          }
          (std::fabs(p.cost - hi) > 0.15 * hi ? odd : norm).push_back(ord[i]);
        }
        if (!odd.empty()) {
          std::stable_sort(odd.begin(), odd.end(), [&](int x, int y) { return pcs[size_t(x)].cost > pcs[size_t(y)].cost; });
          for (int r = 0; r < W; ++r) byload[size_t(r)] = wfrom(r, W);
          std::stable_sort(byload.begin(), byload.end(), [&](int x, int y) { return wl[size_t(x)] < wl[size_t(y)]; });
          size_t q = 0;
          for (size_t j = 0; j < odd.size(); ++j) {
            while (taken[size_t(byload[q])]) ++q;
            const int w = byload[q];
            per[size_t(w)].push_back(odd[j]);
            wl[size_t(w)] += pcs[size_t(odd[j])].cost;
            taken[size_t(w)] = 1;
          }
        }
        size_t w = 0;
        for (int id : norm) {
          while (taken[w]) ++w;
          per[w].push_back(id);
          wl[w] += pcs[size_t(id)].cost;
          taken[w] = 1;
        }
      }
      lay_cuts_ = int(pcs.size());
    } else if (fill) {
      auto pcost = [&](int64_t ib, int64_t rows, int sx) {
        const int2 e = entry(ib, rows, sx);
        const double f = (e.x & dev::kBandBit) ? fband : (e.x & dev::kUniBit) ? 1.0 : fmixed;
        return double(rows + 2 * H) * f + overhead;
      };
      std::vector<Piece> whole;
      double total = 0.0;
      // Overlap (2-D blocks): the outputs the exchange sends become short
      // pieces of their own — the H rows next to a LEFT / RIGHT neighbour per
      // strip, and a DOWN / UP boundary strip cut into kOvRows-row pieces — so
      // they all run in the first round and finish within ~(kOvRows + 2H) row
      // steps; the filling below then tops their waves up with interior rows
      // (later list positions).  With whole ti-row boundary items and about one
      // item per wave the boundary items ended with the sweep and a third of
      // the exchange stayed exposed (4×2 block: 56.8 vs 50.9 µs per
      // iteration at 15 / 8 µs delays, profiles/r4_overlap.txt).
      constexpr int64_t kOvRows = 8;
      const bool ov_split = overlap_ && !(ov_debug_ & 4);
      auto ystrip = [&](int sx) {
        const int64_t J = -(HL - 1) + int64_t(sx) * fsw_;
        const int64_t jlo = std::max<int64_t>(1, J + HL), jhi = std::min<int64_t>(blk_.ny, J + fsw_ + HL - 1);
        return (blk_.has(DOWN) && jlo <= H) || (blk_.has(UP) && jhi >= blk_.ny - H + 1);
      };
      auto add_whole = [&](int64_t a, int64_t rows, int sx, bool bnd) {
        whole.push_back(Piece{a, rows, sx, pcost(a, rows, sx), bnd});
        total += whole.back().cost;
      };
      for (int ch = 0; ch < nchunks; ++ch)
        for (int sx = 0; sx < k.nstrips; ++sx) {
          const int64_t ib = 1 + int64_t(ch) * k.ti, n = std::min<int64_t>(ib + k.ti - 1, blk_.nx) - ib + 1;
          const int64_t ie = ib + n - 1;
          if (!ov_split || !is_boundary(ib, ie, sx)) {
            add_whole(ib, n, sx, is_boundary(ib, ie, sx));
          } else if (ystrip(sx)) {
            for (int64_t a = ib; a <= ie; a += kOvRows) add_whole(a, std::min<int64_t>(kOvRows, ie - a + 1), sx, true);
          } else {
            const int64_t lo = blk_.has(LEFT) ? std::min<int64_t>(ie, H) : ib - 1;             // rows ib .. lo: LEFT's
            const int64_t hi = blk_.has(RIGHT) ? std::max<int64_t>(ib, blk_.nx - H + 1) : ie + 1;  // hi .. ie: RIGHT's
            if (lo >= ib) add_whole(ib, lo - ib + 1, sx, true);
            const int64_t m0 = std::max(ib, lo + 1), m1 = std::min(ie, hi - 1);
            if (m1 >= m0) add_whole(m0, m1 - m0 + 1, sx, false);
            const int64_t r0 = std::max(hi, std::max(ib, lo + 1));  // (never a row of the LEFT piece again)
            if (r0 <= ie) add_whole(r0, ie - r0 + 1, sx, true);
          }
        }
      lap("fill: pieces");
      const int64_t minr = 8;  // shortest cut piece (its 2H fill rows cost more than it)
      const double minc = double(minr + 2 * H) + overhead;
      W = std::max(dev::kWPB, (std::min<int>(waves_avail, int(total / minc)) / dev::kWPB) * dev::kWPB);
      const double cut_cost = double(2 * H) + overhead;  // a cut's extra (uniform) row steps
      int cuts = 0;
      // each piece's wave (pcs order; the per-wave lists are built once, after
      // the last pass)
      std::vector<int> own;
      // (on blocks of about one item per wave the passes alternate between
      // many cuts and few — 8-rank slab of 8192² at 96 rows: 1744 / 175 — and
      // the fourth pass's is kept; keeping the pass of the lowest estimated
      // makespan measured the same, whole pieces without cuts 1.5× slower:
      // profiles/r6_fill_passes.txt.  Once the cut count returns to an
      // earlier pass's input the rest of the passes repeat earlier ones, so
      // the loop stops there with the result the fourth pass would give.)
      struct PassRes {
        std::vector<Piece> pcs;
        std::vector<int> own;
        int nbnd = 0, ncut = 0;
      } prev;
      int in_prev = -1;
      for (int pass = 0; pass < 4; ++pass) {
        const double T = (total + cuts * cut_cost) / W;
        pcs.clear();
        own.clear();
        load.assign(size_t(W), 0.0);
        nbnd = 0;
        int ncut = 0;
        // (queued pieces by index into qp: a heap of 16-byte entries)
        struct QE {
          double cost;
          int seq, idx;
          bool operator<(const QE& o) const { return cost < o.cost || (cost == o.cost && seq > o.seq); }
        };
        std::vector<Piece> qp;
        qp.reserve(whole.size() + whole.size() / 2);
        std::vector<QE> qv;
        qv.reserve(whole.size());
        for (int i = 0; i < int(whole.size()); ++i) {
          const Piece& p = whole[size_t(i)];
          if (p.bnd) {  // boundary pieces: positions 0, 1, … in order (first round)
            own.push_back(nbnd % W);
            load[size_t(nbnd % W)] += p.cost;
            pcs.push_back(p);
            ++nbnd;
          } else {
            qv.push_back(QE{p.cost, i, int(qp.size())});
            qp.push_back(p);
          }
        }
        std::priority_queue<QE> q(std::less<QE>(), std::move(qv));
        using LW = std::pair<double, int>;
        std::priority_queue<LW, std::vector<LW>, std::greater<LW>> heap;
        double csum = 0.0;
        for (int w = 0; w < W; ++w) csum += capw(w, W);
        for (int w = 0; w < W; ++w) heap.push(LW{load[size_t(w)] / capw(w, W), wrank(w, W)});
        while (!q.empty()) {
          const QE e = q.top();
          q.pop();
          const Piece ep = qp[size_t(e.idx)];
          const LW t = heap.top();
          heap.pop();
          const int tw = wfrom(t.second, W);
          const double room = (rho == 1.0 ? T : T * W * capw(tw, W) / csum) - load[size_t(tw)];
          Piece give = ep;
          if (ep.cost > room && room >= minc && ep.rows >= 2 * minr) {
            // the most rows of ep that fit the room (binary search; cost grows with rows)
            int64_t lo = minr, hi = ep.rows - minr, best = 0;
            while (lo <= hi) {
              const int64_t mid = (lo + hi) / 2;
              if (pcost(ep.ib, mid, ep.s) <= room) {
                best = mid;
                lo = mid + 1;
              } else {
                hi = mid - 1;
              }
            }
            if (best > 0) {
              give = Piece{ep.ib, best, ep.s, pcost(ep.ib, best, ep.s), false};
              const Piece rest{ep.ib + best, ep.rows - best, ep.s, pcost(ep.ib + best, ep.rows - best, ep.s), false};
              q.push(QE{rest.cost, e.seq, int(qp.size())});
              qp.push_back(rest);
              ++ncut;
            }
          }
          own.push_back(tw);
          pcs.push_back(give);
          load[size_t(tw)] += give.cost;
          heap.push(LW{load[size_t(tw)] / capw(tw, W), t.second});
        }
        if (trace3) std::fprintf(stderr, "[pe]   layout fill pass %d: %zu pieces, %d cuts, W %d\n", pass, pcs.size(), ncut, W);
        lap("fill: pass");
        if (ncut == cuts) break;
        if (pass >= 1 && ncut == in_prev) {  // inputs now alternate: pass 3 repeats pass 1
          if (pass % 2 == 0) {
            pcs = std::move(prev.pcs);
            own = std::move(prev.own);
            nbnd = prev.nbnd;
            ncut = prev.ncut;
          }
          cuts = ncut;
          break;
        }
        if (pass < 3) prev = PassRes{pcs, own, nbnd, ncut};
        in_prev = cuts;
        cuts = ncut;
      }
      std::vector<int> cnt(size_t(W), 0);
      for (int w : own) ++cnt[size_t(w)];
      per.assign(size_t(W), {});
      for (int w = 0; w < W; ++w) per[size_t(w)].reserve(size_t(cnt[size_t(w)]));
      for (size_t i = 0; i < own.size(); ++i) per[size_t(own[i])].push_back(int(i));
      lay_cuts_ = cuts;
    } else {
    // Three-step LPT.  A band item runs EVERY row step on the band path
    // (≈2.25× a uniform one at 8192²: 221.8 vs 98.6 µs per 112-row item,
    // profiles/r4_stamps48.txt), but costed by its band rows alone it looks
    // barely heavier than a uniform one, so waves that take one still get as
    // many items as the rest: the sweep ended with band items of the last rows
    // (6945-7169) starting 607-631 µs into a 722 µs span (a 33-40 µs tail).
    // Both ways of costing items by kind measured slower, on one box against
    // the round-4 build (profiles/r5_ab_kernel.txt, profiles/r5_ab_layout.txt):
    // wave LOADS counted by kind (rows + 2H fill steps × the kind's factor):
    // 3632-3644 vs 3985-4005 it/s (the last rows' items then went to
    // whichever waves were least loaded, a 110-123 µs tail); items also
    // ORDERED by kind cost: every band item in the first round, all over
    // the grid, 3519-3606 (the first round lost its row window; band items ran
    // 4.1 µs per row step instead of 1.8).  The round-4 tail (late items of the
    // last rows) is made of UNIFORM items whose waves ran slow — the wave-time
    // spread the static costs do not predict (r4 stamps: correlation -0.1).
    // Band-row costs only (the kind-cost knob was removed in round 6).
    std::vector<double> kcost(pcs.size());
    for (size_t i = 0; i < pcs.size(); ++i) kcost[i] = pcs[i].cost;
    per.assign(size_t(W), {});
    load.assign(size_t(W), 0.0);
    std::vector<int> order;
    for (int i = 0; i < int(pcs.size()); ++i) {
      if (pcs[size_t(i)].bnd) {  // boundary pieces: positions 0, 1, … in order
        per[size_t(nbnd % W)].push_back(i);
        load[size_t(nbnd % W)] += kcost[size_t(i)];
        ++nbnd;
      } else {
        order.push_back(i);
      }
    }
    std::stable_sort(order.begin(), order.end(),
                     [&](int a, int b) { return pcs[size_t(a)].cost > pcs[size_t(b)].cost; });
    using LW = std::pair<double, int>;
    std::priority_queue<LW, std::vector<LW>, std::greater<LW>> heap;
    for (int w = 0; w < W; ++w) heap.push(LW{load[size_t(w)] / capw(w, W), wrank(w, W)});
    for (int i : order) {
      const LW t = heap.top();
      heap.pop();
      const int tw = wfrom(t.second, W);
      per[size_t(tw)].push_back(i);
      load[size_t(tw)] += kcost[size_t(i)];
      heap.push(LW{load[size_t(tw)] / capw(tw, W), t.second});
    }
    lay_cuts_ = 0;
    }
    lap(lay_used_.c_str());
    size_t rounds = 0;
    for (const auto& v : per) rounds = std::max(rounds, v.size());
    lay_max_ = 0.0;
    lay_mean_ = 0.0;
    for (int w = 0; w < W; ++w) {
      double l = 0.0;
      for (int i : per[size_t(w)]) l += pcs[size_t(i)].cost;
      lay_max_ = std::max(lay_max_, l);
      lay_mean_ += l / W;
    }
    lay_items_ = int(rounds);
    // List w runs on physical wave w (the persistent grid's workgroup b runs
    // on XCD b mod 8).  XCD-aware maps — each XCD marching a contiguous run of
    // strips so shared halo lines are fetched once into its L2 — read 3-7 %
    // fewer DRAM bytes but ran 0-12 % slower (profiles/r3_three_ti.txt,
    // profiles/r5_dram_layout.txt); removed in round 6.
    std::vector<int> phys(static_cast<size_t>(W));
    {
      const int nb = W / dev::kWPB;
      for (int w = 0; w < W; ++w) phys[size_t(w)] = w;
      // PE_WPERM (diagnostic: does a slow item stay slow on another wave?):
      // 1 lists on the workgroups in reverse order, 2 rotated by a quarter of
      // the grid (other co-resident workgroup pairs)
      if (const char* e = std::getenv("PE_WPERM")) {
        const int m = std::atoi(e);
        for (int w = 0; w < W; ++w) {
          const int b = w / dev::kWPB, l = w % dev::kWPB;
          const int pb = m == 1 ? nb - 1 - b : m == 2 ? (b + nb / 4) % nb : b;
          phys[size_t(w)] = pb * dev::kWPB + l;
        }
      }
    }
    std::vector<int2> all(rounds * size_t(W), int2{0, 0});  // {0, 0}: empty entry (0 rows)
    for (int w = 0; w < W; ++w)
      for (size_t r = 0; r < per[size_t(w)].size(); ++r) {
        const Piece& p = pcs[size_t(per[size_t(w)][r])];
        all[r * size_t(W) + size_t(phys[size_t(w)])] = entry(p.ib, p.rows, p.s);
      }
    static_waves_ = W;
    nslot_cap_ = std::max<int>(nslot_cap_, int(all.size()));
    ov_nb_ = nbnd;
    ov_lnsh_ = 1;
    ov_lbase_[0] = 0;
    for (int x = 1; x <= 8; ++x) ov_lbase_[x] = int(all.size());
    ov_lnb_[0] = nbnd;
    for (int x = 1; x < 8; ++x) ov_lnb_[x] = 0;
    const auto tc = clk::now();
    if (!lay_dry_) {  // (a dry layout only fills the cache: prepare_layout)
      list_alloc(all.size());
      upload(ilist_, all.data(), sizeof(int2) * all.size());
    }
    ilist_host_.assign(all.begin(), all.end());
    copy_setup_s_ += secs(tc, clk::now());
    k.ilist = ilist_;
    k.lnsh = 1;
    k.lwaves = W;
    k.nslots = int(all.size());
    for (int x = 0; x <= 8; ++x) k.lbase[x] = ov_lbase_[x];
    for (int x = 0; x < 8; ++x) k.lnb[x] = 0;
    // static list walk: the grid is the one the list was laid out for (plus
    // the blocks the overlap keeps free for the halo stream)
    k.nblocks = k.nblocks0 = static_waves_ / dev::kWPB + (overlap_ ? ov_reserve_ : 0);
    if (overlap_ && !lay_dry_) create_halo_stream();
    lap("list");
    return;
  }
  lay_max_ = lay_mean_ = 0.0;
  lay_items_ = 0;
  std::vector<double> cost(size_t(k.nitems));
  std::vector<double> ccost(size_t(nchunks) + 1, 0.0);  // prefix sums per chunk
  for (int ch = 0; ch < nchunks; ++ch) {
    double cc = 0.0;
    for (int s = 0; s < k.nstrips; ++s) cc += cost[size_t(ch) * k.nstrips + s] = item_cost(ch, s);
    ccost[size_t(ch) + 1] = ccost[size_t(ch)] + cc;
  }
  const double light = double(k.ti + 2 * H);
  std::vector<int> cut(size_t(nsh) + 1, 0);
  for (int x = 1; x < nsh; ++x) {
    const double target = ccost.back() * x / nsh;
    int c = cut[size_t(x) - 1];
    while (c < nchunks && ccost[size_t(c) + 1] <= target) ++c;
    cut[size_t(x)] = c;
  }
  cut[size_t(nsh)] = nchunks;
  // (no tail split of the last items: at one placement every extra item cost
  // more than the shorter drain saved — 8192², 18 rows: 545.5 µs per
  // iteration unsplit vs 550.6 / 552.1 / 556.1 with 5 / 10 / 30 % split; 2
  // ranks 297.8 vs 307.5, profiles/r2_layout.txt; the knob was removed in round 6)
  const double tail_frac = 0.0;
  const int tail_split = 2;
  std::vector<int2> all;
  ov_nb_ = 0;
  ov_lnsh_ = nsh;
  for (int x = 0; x < nsh; ++x) {
    std::vector<int> b, heavy, in;
    for (int ch = cut[size_t(x)]; ch < cut[size_t(x) + 1]; ++ch)
      for (int s = 0; s < k.nstrips; ++s) {
        const int id = ch * k.nstrips + s;
        const int64_t ib = 1 + int64_t(ch) * k.ti, ie = std::min<int64_t>(ib + k.ti - 1, blk_.nx);
        if (is_boundary(ib, ie, s)) b.push_back(id);
        else if (sort_heavy && cost[size_t(id)] > 1.25 * light) heavy.push_back(id);
        else in.push_back(id);
      }
    std::stable_sort(heavy.begin(), heavy.end(), [&](int a, int c) { return cost[size_t(a)] > cost[size_t(c)]; });
    ov_lbase_[x] = int(all.size());
    ov_lnb_[x] = int(b.size());
    ov_nb_ += int(b.size());
    const size_t nsplit = size_t(tail_frac * double(in.size()) + 0.5);
    auto push = [&](int id, int parts) {
      const int ch = id / k.nstrips, s = id % k.nstrips;
      const int64_t ib = 1 + int64_t(ch) * k.ti, ie = std::min<int64_t>(ib + k.ti - 1, blk_.nx);
      const int64_t n = ie - ib + 1;
      parts = int(std::min<int64_t>(parts, n));
      for (int q = 0; q < parts; ++q) {
        const int64_t a0 = ib + n * q / parts, a1 = ib + n * (q + 1) / parts;
        all.push_back(entry(a0, a1 - a0, s));
      }
    };
    for (int id : b) push(id, 1);
    for (int id : heavy) push(id, 1);
    for (size_t i = 0; i < in.size(); ++i) push(in[i], i + nsplit >= in.size() ? tail_split : 1);
  }
  ov_lbase_[nsh] = int(all.size());
  if (int(all.size()) < k.nitems || int(all.size()) > nslot_cap_) throw std::logic_error("item list does not fit");
  const auto tc = clk::now();
  if (!lay_dry_) {
    list_alloc(all.size());
    upload(ilist_, all.data(), sizeof(int2) * all.size());
  }
  ilist_host_.assign(all.begin(), all.end());
  copy_setup_s_ += secs(tc, clk::now());
  // Every dynamic sweep walks the list (the plain one counts no boundary
  // items: lnb = 0; the overlapped iteration's launch carries ov_lnb_).
  k.ilist = ilist_;
  k.lnsh = nsh;
  k.nslots = int(all.size());
  for (int x = 0; x <= 8; ++x) k.lbase[x] = x <= nsh ? ov_lbase_[x] : ov_lbase_[nsh];
  for (int x = 0; x < 8; ++x) k.lnb[x] = 0;
  if (overlap_ && !lay_dry_) create_halo_stream();
}

DeviceSolver::LayoutSnap DeviceSolver::snap_layout() const {
  const KParams& k = *kp_;
  LayoutSnap v;
  v.list = ilist_host_;
  v.static_waves = static_waves_;
  v.ov_nb = ov_nb_;
  v.ov_lnsh = ov_lnsh_;
  std::copy(ov_lbase_, ov_lbase_ + 9, v.ov_lbase);
  std::copy(ov_lnb_, ov_lnb_ + 8, v.ov_lnb);
  v.lay_items = lay_items_;
  v.lay_cuts = lay_cuts_;
  v.lay_max = lay_max_;
  v.lay_mean = lay_mean_;
  v.lay_used = lay_used_;
  v.lnsh = k.lnsh;
  v.lwaves = k.lwaves;
  v.nslots = k.nslots;
  std::copy(k.lbase, k.lbase + 9, v.lbase);
  std::copy(k.lnb, k.lnb + 8, v.lnb);
  v.nblocks = k.nblocks;
  v.nblocks0 = k.nblocks0;
  return v;
}

void DeviceSolver::restore_layout(const LayoutSnap& v) {
  KParams& k = *kp_;
  if (v.list.size() > ilist_cap_) {  // (laid out dry, ahead: prepare_layout)
    PE_HIP_CHECK(hipStreamSynchronize(stream_));
    if (ilist_) PE_HIP_CHECK(hipFree(ilist_));
    ilist_cap_ = v.list.size() + v.list.size() / 2;
    PE_HIP_CHECK(hipMalloc(&ilist_, sizeof(int2) * ilist_cap_));
  }
  nslot_cap_ = std::max<int>(nslot_cap_, int(v.list.size()));
  upload(ilist_, v.list.data(), sizeof(int2) * v.list.size());
  ilist_host_ = v.list;
  static_waves_ = v.static_waves;
  ov_nb_ = v.ov_nb;
  ov_lnsh_ = v.ov_lnsh;
  std::copy(v.ov_lbase, v.ov_lbase + 9, ov_lbase_);
  std::copy(v.ov_lnb, v.ov_lnb + 8, ov_lnb_);
  lay_items_ = v.lay_items;
  lay_cuts_ = v.lay_cuts;
  lay_max_ = v.lay_max;
  lay_mean_ = v.lay_mean;
  lay_used_ = v.lay_used;
  k.ilist = ilist_;
  k.lnsh = v.lnsh;
  k.lwaves = v.lwaves;
  k.nslots = v.nslots;
  std::copy(v.lbase, v.lbase + 9, k.lbase);
  std::copy(v.lnb, v.lnb + 8, k.lnb);
  k.nblocks = v.nblocks;
  k.nblocks0 = v.nblocks0;
  if (overlap_) create_halo_stream();
}

// Lays out (ti, overlap) into the layout cache without touching the live
// iteration — host work only, no list upload, every member it sets restored —
// so that the halo-path choice can build its next candidates' layouts while
// the GPU times the current one.
void DeviceSolver::prepare_layout(int ti, bool overlap) {
  if (!fused_ || !lay_cache_on_) return;
  const KParams keep_k = *kp_;
  const bool keep_want = want_overlap_, keep_ov = overlap_, keep_push = push_;
  const LayoutSnap keep = snap_layout();
  auto back = [&]() {
    lay_dry_ = false;
    *kp_ = keep_k;
    want_overlap_ = keep_want;
    overlap_ = keep_ov;
    push_ = keep_push;
    ilist_host_ = keep.list;
    static_waves_ = keep.static_waves;
    ov_nb_ = keep.ov_nb;
    ov_lnsh_ = keep.ov_lnsh;
    std::copy(keep.ov_lbase, keep.ov_lbase + 9, ov_lbase_);
    std::copy(keep.ov_lnb, keep.ov_lnb + 8, ov_lnb_);
    lay_items_ = keep.lay_items;
    lay_cuts_ = keep.lay_cuts;
    lay_max_ = keep.lay_max;
    lay_mean_ = keep.lay_mean;
    lay_used_ = keep.lay_used;
  };
  lay_dry_ = true;
  want_overlap_ = overlap;
  push_ = false;  // (the overlap's list: the push never overlaps)
  try {
    set_items(ti);
    setup_items();
  } catch (...) {
    back();
    throw;
  }
  back();
}

// LDS-resident geometry: tiles of one 124-column strip × R rows (the
// streaming sweep's strips), one workgroup each, at most one per CU, R ≥ 8
// where the block allows and ≤ kResMaxRows; the band-coefficient table is
// sized from the host row classes (the kernel's exact band test).
void DeviceSolver::setup_resident() {
  KParams& k = *kp_;
  resident_ = false;
  const char* e = std::getenv("PE_RESIDENT");
  if (e && std::atoi(e) == 0) return;
  if (!fused_ || sstep_ || comm_->size() != 1 || blk_.Px * blk_.Py != 1 || overlap_ || k.stamps || opt_.variant != 0)
    return;
  const int nx = int(blk_.nx);
  int cus = 256;
  {
    int dev = 0;
    PE_HIP_CHECK(hipGetDevice(&dev));
    PE_HIP_CHECK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
  }
  const int nstrips = k.nstrips;
  if (nstrips > cus) return;
  const int ntr = std::max(1, std::min(cus / nstrips, nx / 8));
  if (nx < 2 * ntr) return;
  std::vector<int> rs(size_t(ntr) + 1);
  for (int t = 0; t <= ntr; ++t) rs[size_t(t)] = 1 + int(int64_t(t) * nx / ntr);
  int rcap = 0;
  for (int t = 0; t < ntr; ++t) rcap = std::max(rcap, rs[size_t(t) + 1] - rs[size_t(t)]);
  if (rcap > dev::kResMaxRows) return;
  // band nodes per tile region (rows I0-2 .. I0+R+1, columns J0-2 .. J0+125)
  const int64_t rows_tab = int64_t(rowcls_host_.size() / 4);
  int nb_max = 0;
  for (int t = 0; t < ntr; ++t)
    for (int sx = 0; sx < nstrips; ++sx) {
      int nb = 0;
      const int J0 = 1 + dev::kFSW * sx;
      for (int q = rs[size_t(t)] - 2; q < rs[size_t(t) + 1] + 2; ++q) {
        if (q + 1 < 0 || q + 1 >= rows_tab) continue;
        const int* r = &rowcls_host_[size_t(q - tab_lo_) * 4];
        for (int c = J0 - 2; c < J0 + 126; ++c)
          if (c >= r[2] && c <= r[3] && !(c >= r[0] && c <= r[1])) ++nb;
      }
      nb_max = std::max(nb_max, nb);
    }
  const int nbcap = nb_max + 8;
  const size_t lds = dev::resident_lds_bytes(rcap, nbcap);
  if (lds > 163840) return;
  const int per_cu = dev::resident_max_blocks_per_cu(lds);
  const int nwg = ntr * nstrips;
  if (per_cu < 1 || nwg > per_cu * cus) return;
  if (nwg > dev::kResMaxTiles) return;  // the kernel's sum gather covers 256 tiles (parts with > 256 CUs)
  rp_ = std::make_unique<dev::ResParams>();
  dev::ResParams& r = *rp_;
  std::memset(&r, 0, sizeof(r));
  r.nstrips = nstrips;
  r.ntr = ntr;
  r.nwg = nwg;
  r.rcap = rcap;
  r.nbcap = nbcap;
  r.lds_bytes = unsigned(lds);
  r.timeout_ticks = 200000000LL;  // 2 s per barrier wait
  if (const char* t = std::getenv("PE_RES_TIMEOUT_S")) r.timeout_ticks = (long long)(std::atof(t) * 1e8);
  PE_HIP_CHECK(hipMalloc(&res_rowstart_, sizeof(int) * rs.size()));
  upload(res_rowstart_, rs.data(), sizeof(int) * rs.size());
  const size_t nedge = size_t(2) * size_t(nwg) * dev::kResEdge, npart = size_t(2) * size_t(nwg) * 8;
  PE_HIP_CHECK(hipMalloc(&res_buf_, sizeof(double) * (nedge + npart)));
  // stream-ordered: a null-stream operation would create that stream's
  // hardware queue (≈10 ms inside T_solver in a fresh process, profiles/r2_ctor_phases.txt)
  PE_HIP_CHECK(hipMemsetAsync(res_buf_, 0, sizeof(double) * (nedge + npart), stream_));
  PE_HIP_CHECK(hipMalloc(&res_ctr_, sizeof(unsigned) * 8 * 32));
  if (const char* t = std::getenv("PE_RES_STAMPS"); t && std::atoi(t) == 1) {
    nstamps_ = size_t(nwg) * dev::kResStampIters * 8;
    PE_HIP_CHECK(hipMalloc(&stamps_, sizeof(unsigned long long) * nstamps_));
    PE_HIP_CHECK(hipMemsetAsync(stamps_, 0, sizeof(unsigned long long) * nstamps_, stream_));
    r.stamps = stamps_;
  }
  r.rowstart = res_rowstart_;
  r.edges = res_buf_;
  r.partials = res_buf_ + nedge;
  r.ctr = res_ctr_;
  r.fault_wg = -1;
  r.fault_late = 0;
  if (const char* f = std::getenv("PE_FAULT_INJECT"); f && (std::string(f) == "resbarrier" || std::string(f) == "reslate")) {
    r.fault_wg = nwg - 1;
    r.fault_late = std::string(f) == "reslate" ? 1 : 0;
  }
  resident_ = true;
}

}  // namespace pe
