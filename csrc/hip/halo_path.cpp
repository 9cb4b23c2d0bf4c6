// The multi-rank halo paths (host side): the in-sweep push's and the peer
// put's set-up (collective: map, self-test, agree), one halo phase through the
// put kernel or the comm (xfer), switching paths on the live iteration, and
// the construction's choice of path by timing the candidates on the job's own
// transport (choose_halo_path).  Split out of device_solver.cpp in round 6.
//
// Reference: the fixed serial halo exchange then stencil of
// poisson_mpi_cuda2.cu:850-859 (host-staged MPI_Isend/Irecv, :331-500).
#include <hip/hip_runtime_api.h>

#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <functional>
#include <string>
#include <vector>

#include <rocprofiler-sdk-roctx/roctx.h>

#include "../hip/kernels.hpp"
#include "pe/device.hpp"
#include "solver_internal.hpp"

namespace pe {

using dev::DevState;
using dev::KParams;

using detail::clk;
using detail::Range;
using detail::secs;

// In-sweep halo push over xGMI (KParams::push).  Row-slab blocks (Py = 1:
// one contiguous 2-row message per x-neighbour) whose per-iteration sums run
// inside the sweep over the P2P transport: the sweep stores its edge rows
// straight into the neighbours' fine-grained receive buffers, the sum's flags
// tell the neighbours they have arrived, and the next sweep reads them from
// there (no import copy) — no exchange launch, no RCCL call, and the iteration
// becomes graph-capturable.  Every input of the decision is global (grid,
// process grid, environment, transport type), so every rank reaches
// map_peer_buffers (collective) or none does.  This only maps and self-tests
// the buffers (push_ok_): whether the job pushes is choose_halo_path's
// decision (PE_HALO=exchange / put: never).
void DeviceSolver::setup_halo_push() {
  push_ = push_ok_ = false;
  const char* hm = std::getenv("PE_HALO");
  const bool allowed = !hm || std::string(hm) == "push";
  // PE_PUSH_LOOPBACK=1 (diagnostic, tools/block_probe.py on one GPU): the
  // push kernel's work without peers — every push lands in this rank's own
  // receive buffer and the halo rows are read back from it (wrong values,
  // the real stores and loads), so a row slab's per-rank time includes what
  // the 8-GPU job's push kernel does
  if (const char* e = std::getenv("PE_PUSH_LOOPBACK"); allowed && e && std::atoi(e) == 1 && comm_->size() > 1 &&
                                                       fused_ && blk_.Py == 1 && (prob_.M - 1) / blk_.Px >= 2 * hdep_) {
    const size_t bytes = sizeof(double) * 4 * size_t(hdep_) * size_t(kp_->pitch);
    void* buf = nullptr;
    PE_HIP_CHECK(hipExtMallocWithFlags(&buf, bytes, hipDeviceMallocFinegrained));
    PE_HIP_CHECK(hipMemsetAsync(buf, 0, bytes, stream_));
    PE_HIP_CHECK(hipDeviceSynchronize());
    hrecv_ = static_cast<double*>(buf);
    hpeers_.assign(size_t(comm_->size()), buf);
    push_ok_ = push_loop_ = true;
    push_status_ = "loopback (diagnostic)";
    return;
  }
  push_status_ = comm_->size() < 2 ? "off: one rank" : !fused_ ? "off: classic path" : !comm_->peer_sum()
                 ? "off: no P2P transport (" + p2p_setup_status() + ")" : blk_.Py != 1 ? "off: 2-D blocks"
                 : "";
  if (!push_status_.empty()) return;
  push_status_ = "off: slabs thinner than 2 halo depths";
  if ((prob_.M - 1) / blk_.Px < 2 * hdep_) return;  // edge rows 1..h and nx-h+1..nx distinct
  push_status_ = "off: PE_XR=0";
  if (const char* e = std::getenv("PE_XR"); e && std::atoi(e) == 0) return;
  push_status_ = std::string("off: PE_HALO=") + (hm ? hm : "");
  if (!allowed) return;
  push_status_ = "fallback: the receive buffers could not be mapped on every rank";
  const size_t bytes = sizeof(double) * 4 * size_t(hdep_) * size_t(kp_->pitch);  // [parity][side][hdep rows]
  void* buf = nullptr;
  if (hipExtMallocWithFlags(&buf, bytes, hipDeviceMallocFinegrained) != hipSuccess) {
    buf = nullptr;
    (void)hipGetLastError();
  } else {
    PE_HIP_CHECK(hipMemsetAsync(buf, 0, bytes, stream_));
    PE_HIP_CHECK(hipDeviceSynchronize());
  }
  // a rank without a buffer still takes part (its map fails → every rank gets
  // an empty result and keeps the exchange)
  hpeers_ = comm_->map_peer_buffers(buf);
  if (hpeers_.empty()) {
    if (buf) PE_HIP_CHECK(hipFree(buf));
    return;
  }
  hrecv_ = static_cast<double*>(buf);
  push_ok_ = true;
  push_status_ = "available";
  // Collective self-test of the path, in its own store / load forms: every
  // rank fills its neighbours' receive buffers with rank-coded values, the
  // ranks synchronise, every rank checks what arrived; all ranks keep the
  // exchange if any check fails.  The buffers are then cleared (their halo
  // columns must stay zero) and the ranks synchronise again before any
  // sweep can push.
  {
    KParams t = *kp_;
    const int64_t side = int64_t(hdep_) * t.pitch;
    for (int b = 0; b < 2; ++b) {
      t.hpush_lo[b] = blk_.has(LEFT) ? static_cast<double*>(hpeers_[size_t(blk_.nbr[LEFT])]) + (2 * b + 1) * side
                                     : nullptr;
      t.hpush_hi[b] = blk_.has(RIGHT) ? static_cast<double*>(hpeers_[size_t(blk_.nbr[RIGHT])]) + (2 * b + 0) * side
                                      : nullptr;
    }
    t.hrecv = hrecv_;
    int* bad = nullptr;
    PE_HIP_CHECK(hipMalloc(&bad, sizeof(int)));
    PE_HIP_CHECK(hipMemsetAsync(bad, 0, sizeof(int), stream_));
    dev::launch_push_test_write(t, blk_.rank, stream_);
    PE_HIP_CHECK(hipGetLastError());
    PE_HIP_CHECK(hipStreamSynchronize(stream_));
    comm_->barrier(stream_);
    dev::launch_push_test_check(t, blk_.has(LEFT) ? blk_.nbr[LEFT] : -1, blk_.has(RIGHT) ? blk_.nbr[RIGHT] : -1, bad,
                                stream_);
    PE_HIP_CHECK(hipGetLastError());
    int hbad = 0;
    PE_HIP_CHECK(hipMemcpyAsync(&hbad, bad, sizeof(int), hipMemcpyDeviceToHost, stream_));
    PE_HIP_CHECK(hipStreamSynchronize(stream_));
    PE_HIP_CHECK(hipFree(bad));
    // PE_FAULT_INJECT=pushtest@rank:R — rank R's check fails (fallback test)
    if (const char* e = std::getenv("PE_FAULT_INJECT"); e && std::string(e).rfind("pushtest@rank:", 0) == 0 &&
                                                        std::atoi(e + 14) == blk_.rank)
      hbad = 1;
    double fail[1] = {hbad != 0 ? 1.0 : 0.0};
    if (hbad) std::fprintf(stderr, "[pe] rank %d: halo-push self-test: %d wrong values received\n", blk_.rank, hbad);
    comm_->host_max(fail, 1, stream_);
    PE_HIP_CHECK(hipMemsetAsync(buf, 0, bytes, stream_));
    PE_HIP_CHECK(hipStreamSynchronize(stream_));
    comm_->barrier(stream_);
    if (fail[0] != 0.0) {
      if (blk_.rank == 0) std::fprintf(stderr, "[pe] halo push unavailable on this job (self-test), using the exchange\n");
      push_status_ = hbad ? "fallback: self-test failed on this rank" : "fallback: self-test failed on a peer";
      comm_->unmap_peer_buffers(hpeers_);
      hpeers_.clear();
      PE_HIP_CHECK(hipFree(buf));
      hrecv_ = nullptr;
      push_ok_ = false;
    }
  }
}

// Halo exchange by peer put (p2p.hip kPut): every rank maps its neighbours'
// fine-grained inboxes and one kernel per halo phase stores this rank's
// message straight into them over xGMI, flags it, waits for the neighbours'
// messages in its own inbox and copies them into place — no RCCL launch, no
// proxy thread, and the same pack / unpack kernels and halo plan as the
// comm's exchange.  Set-up is collective and fail-safe like the push's: map
// (every rank or none), self-test with rank-coded messages, agree.
// PE_PUT_LOOPBACK=1 (one GPU: probes, tests): the rank is its own peer on
// every side — each message lands in its own receive buffer, as with the
// loopback delay transport — so the kernel's real stores, flags and copies run
// on one device.  PE_HALO=exchange / push: off.
void DeviceSolver::setup_halo_put() {
  put_ = put_ok_ = false;
  const char* hm = std::getenv("PE_HALO");
  const bool allowed = !hm || std::string(hm) == "put";
  const char* lb = std::getenv("PE_PUT_LOOPBACK");
  put_loop_ = lb && std::atoi(lb) == 1;
  put_status_ = comm_->size() < 2 ? "off: one rank" : !fused_ ? "off: classic path" : !allowed
                ? std::string("off: PE_HALO=") + hm : (!put_loop_ && !comm_->peer_sum())
                ? "off: no P2P transport (" + p2p_setup_status() + ")" : "";
  if (!put_status_.empty()) return;
  // inbox slot: the largest message of a phase — y strips (2·hdep values per
  // owned row) or hdep whole interleaved rows
  const std::vector<HaloPhase> ph = halo_phases(0);
  int64_t cmax = 1;
  for (const HaloPhase& p : ph)
    for (const Exchange& e : p.ex) cmax = std::max(cmax, e.count);
  // (every rank takes part in the collectives below, a rank without
  // neighbours too: its buffer simply stays unused)
  cmax = std::max<int64_t>({cmax, 2 * int64_t(hdep_) * blk_.nx, int64_t(hdep_) * kp_->pitch});
  put_stride_ = (cmax + dev::kPutBoxOff + 31) / 32 * 32;  // (+ the slot's 16-B phase offset)
  const size_t flag_bytes = sizeof(unsigned long long) * 4 * dev::kPutParts * dev::kPutFlagStride;
  const size_t bytes = flag_bytes + sizeof(double) * 4 * 2 * size_t(put_stride_);
  void* buf = nullptr;
  if (hipExtMallocWithFlags(&buf, bytes, hipDeviceMallocFinegrained) != hipSuccess) {
    buf = nullptr;
    (void)hipGetLastError();
  } else {
    PE_HIP_CHECK(hipMemsetAsync(buf, 0, bytes, stream_));
  }
  PE_HIP_CHECK(hipMalloc(&put_cnt_, sizeof(unsigned) * 8));
  PE_HIP_CHECK(hipMemsetAsync(put_cnt_, 0, sizeof(unsigned) * 8, stream_));
  PE_HIP_CHECK(hipStreamSynchronize(stream_));
  if (put_loop_) {
    if (!buf) PE_HIP_CHECK(hipErrorOutOfMemory);
    put_peers_.assign(size_t(comm_->size()), buf);
  } else {
    put_peers_ = comm_->map_peer_buffers(buf);
  }
  put_status_ = "fallback: the inboxes could not be mapped on every rank";
  if (put_peers_.empty()) {
    if (buf) PE_HIP_CHECK(hipFree(buf));
    return;
  }
  put_buf_ = buf;
  // Self-test: one exchange of every halo phase's messages (at most 4096
  // values each) with rank-coded data, checked on arrival; every rank keeps
  // the comm's exchange if any check failed anywhere.
  {
    const int64_t n = std::min<int64_t>(4096, put_stride_ - dev::kPutBoxOff);
    double *sbuf = nullptr, *rbuf = nullptr, *codes = nullptr;
    int* bad = nullptr;
    PE_HIP_CHECK(hipMalloc(&sbuf, sizeof(double) * 4 * n));
    PE_HIP_CHECK(hipMalloc(&rbuf, sizeof(double) * 4 * n));
    PE_HIP_CHECK(hipMalloc(&codes, sizeof(double) * 4));
    PE_HIP_CHECK(hipMalloc(&bad, sizeof(int)));
    std::vector<double> hs(size_t(4 * n));
    const double me = double(blk_.rank + 1);
    for (int64_t i = 0; i < 4 * n; ++i) hs[size_t(i)] = me + double((i % n) % 7);
    upload(sbuf, hs.data(), sizeof(double) * hs.size());
    PE_HIP_CHECK(hipMemsetAsync(bad, 0, sizeof(int), stream_));
    int hbad = 0;
    for (const HaloPhase& p : ph) {
      std::vector<Exchange> ex;
      double hc[4] = {0, 0, 0, 0};
      for (const Exchange& e : p.ex) {
        const int m = int(ex.size());
        ex.push_back(Exchange{e.dir, e.peer, sbuf + m * n, rbuf + m * n, n});
        hc[m] = put_loop_ ? me : double(e.peer + 1);
      }
      if (ex.empty()) continue;
      upload(codes, hc, sizeof(hc));
      const double keep = put_timeout_s_;
      put_timeout_s_ = std::min(keep, 5.0);
      put_ = true;
      xfer(ex, stream_);
      put_ = false;
      put_timeout_s_ = keep;
      dev::PutArgs a{};
      a.nmsg = int(ex.size());
      for (size_t m = 0; m < ex.size(); ++m) {
        a.m[m].dst = ex[m].recv;
        a.m[m].n = n;
      }
      dev::launch_put_check(a, codes, bad, stream_);
      PE_HIP_CHECK(hipGetLastError());
      PE_HIP_CHECK(hipStreamSynchronize(stream_));
    }
    PE_HIP_CHECK(hipMemcpyAsync(&hbad, bad, sizeof(int), hipMemcpyDeviceToHost, stream_));
    PE_HIP_CHECK(hipStreamSynchronize(stream_));
    PE_HIP_CHECK(hipFree(sbuf));
    PE_HIP_CHECK(hipFree(rbuf));
    PE_HIP_CHECK(hipFree(codes));
    PE_HIP_CHECK(hipFree(bad));
    // PE_FAULT_INJECT=puttest@rank:R — rank R's check fails (fallback test)
    if (const char* e = std::getenv("PE_FAULT_INJECT"); e && std::string(e).rfind("puttest@rank:", 0) == 0 &&
                                                        std::atoi(e + 13) == blk_.rank)
      hbad = 1;
    if (hbad) std::fprintf(stderr, "[pe] rank %d: halo-put self-test: %d wrong values received\n", blk_.rank, hbad);
    double fail[1] = {hbad != 0 ? 1.0 : 0.0};
    comm_->host_max(fail, 1, stream_);
    if (fail[0] != 0.0) {
      if (blk_.rank == 0) std::fprintf(stderr, "[pe] halo put unavailable on this job (self-test), using the exchange\n");
      put_status_ = hbad ? "fallback: self-test failed on this rank" : "fallback: self-test failed on a peer";
      if (!put_loop_) comm_->unmap_peer_buffers(put_peers_);
      put_peers_.clear();
      PE_HIP_CHECK(hipFree(put_buf_));
      put_buf_ = nullptr;
      return;
    }
  }
  put_ok_ = true;
  put_status_ = put_loop_ ? "loopback (diagnostic)" : "available";
}

void DeviceSolver::xfer(const std::vector<Exchange>& ex, hipStream_t s) {
  if (!put_) {
    comm_->exchange(ex, s);
    return;
  }
  if (ex.empty()) return;
  if (ex.size() > 4) throw std::logic_error("put: at most 4 messages per halo phase");
  const size_t flag_words = size_t(4) * dev::kPutParts * dev::kPutFlagStride;
  auto flags = [&](void* buf, int d) {
    return static_cast<unsigned long long*>(buf) + size_t(d) * dev::kPutParts * dev::kPutFlagStride;
  };
  auto box = [&](void* buf, int d) {
    return reinterpret_cast<double*>(static_cast<unsigned long long*>(buf) + flag_words) + size_t(d) * 2 * put_stride_;
  };
  dev::PutArgs a{};
  a.nmsg = int(ex.size());
  a.stride = put_stride_;
  a.cnt = put_cnt_;
  a.timeout_ticks = (long long)(put_timeout_s_ * 1e8);
  // 64 blocks per message alone on the GPU (8x1 block of 8192², one GPU,
  // loopback: 134 vs 141 µs per sweep at 16); 8 under the overlap, whose
  // halo stream gets the 8 blocks the sweep leaves free (64: 164 vs 140)
  a.parts = want_overlap_ ? 8 : dev::kPutParts;
  for (size_t m = 0; m < ex.size(); ++m) {
    const Exchange& e = ex[m];
    if (e.count + dev::kPutBoxOff > put_stride_) throw std::logic_error("put: message larger than the inbox");
    void* peer = put_peers_[size_t(put_loop_ ? blk_.rank : e.peer)];
    // the peer files this rank's message under the direction it sees us in;
    // a loopback rank under the message's own direction (send → own receive)
    const int rd = put_loop_ ? e.dir : opposite(e.dir);
    a.m[m] = dev::PutMsg{e.send, box(peer, rd), flags(peer, rd), box(put_buf_, e.dir), flags(put_buf_, e.dir),
                         e.recv, (long long)e.count, e.dir};
  }
  dev::launch_put(a, s);
  PE_HIP_CHECK(hipGetLastError());
}

void DeviceSolver::apply_halo_path(const std::string& path, bool overlap, bool live, int ti) {
  const bool was_push = push_, was_ov = overlap_;
  if (live) {  // (the state carries on: nothing of the old path may still be in flight)
    PE_HIP_CHECK(hipStreamSynchronize(stream_));
    if (hs_) PE_HIP_CHECK(hipStreamSynchronize(hs_));
  }
  push_ = path == "push" && push_ok_;
  put_ = path == "put" && put_ok_;
  kp_->push = push_ ? 1 : 0;
  bool relay = overlap != want_overlap_;
  want_overlap_ = overlap;
  for (auto& g : graphs_) PE_HIP_CHECK(hipGraphExecDestroy(g.second));  // captured on the old path
  graphs_.clear();
  if (ti > 0 && ti != kp_->ti) {  // (another height for the overlap's layout)
    set_items(ti);
    relay = true;
  }
  // the overlap's boundary-first list, or the plain one (the exchange, the put
  // and the push share the plain layout: no re-layout between them)
  const bool relaid = relay || overlap_ != (overlap && !push_);
  if (relaid) {
    const auto t0 = clk::now();
    const double up0 = copy_setup_s_;
    setup_items();
    if (live && std::getenv("PE_CTOR_TRACE") && std::atoi(std::getenv("PE_CTOR_TRACE")) >= 2)
      std::fprintf(stderr, "[pe] halo path re-layout %s at %d rows: %6.3f ms (list upload %6.3f ms)\n",
                   overlap_ ? "overlap" : "plain", kp_->ti, 1e3 * secs(t0, clk::now()), 1e3 * (copy_setup_s_ - up0));
  }
  if (!live) return;
  // The next sweep (parity par_) reads x[par_ ^ 1]'s halo: the push keeps it in
  // the receive buffer, the exchange and the put in x — move it across.
  if (was_push && !push_)
    for (int b = 0; b < 2; ++b) dev::launch_halo_import(*kp_, b, stream_);
  if (!was_push && push_) dev::launch_halo_seed(*kp_, par_ ^ 1, stream_);
  // a fresh boundary-item count for the overlap's targets (epoch × boundary
  // items of the list: another list — another height — has another count)
  if (overlap_ != was_ov || (relaid && overlap_)) {
    PE_HIP_CHECK(hipMemsetAsync(&st_->sig, 0, sizeof(st_->sig), stream_));
    ov_epoch_ = 0;
  }
  PE_HIP_CHECK(hipGetLastError());
}

// The multi-rank halo path, chosen on the job's own transport.  Candidates:
// the comm's exchange (RCCL grouped send / receive: pack, exchange, unpack
// after the sweep), the same through the peer-put kernel (setup_halo_put), each
// with and without the halo/interior overlap (the exchange on the halo stream
// under the interior items), and — row slabs with in-sweep P2P sums — the
// sweep's own halo push.  From one reset, the candidates take turns on the
// live iteration (cross-rank sums included, the stop test off; the halo is
// moved between x and the push's receive buffer at a switch): 1 + 3 sweeps
// each, the last 3 timed, then the two fastest once more (min of the two);
// every time is the max over ranks, so every rank keeps the same path.  (A
// reset per candidate and 2 + 4 sweeps cost 27-30 ms at the 8-rank slab of
// 8192², round 6.)  Until round 5 the choice was a
// fixed rule (exchange; overlap when a measured exchange exceeded 12 µs) set
// from one-GPU probes with simulated 15 / 8 µs delays; the first cross-device
// run must not rest on a simulation.  PE_HALO=exchange / put / push and
// PE_OVERLAP=0 / 1 restrict the candidates; PE_HALO_TUNE=0 takes the first one
// left (exchange, no overlap, when allowed) without timing.
void DeviceSolver::choose_halo_path() {
  halo_cands_.clear();
  if (comm_->size() < 2 || !fused_ || resident_) {
    halo_path_ = comm_->size() < 2 ? "none: one rank" : !fused_ ? "exchange (classic path)" : "none: resident";
    apply_halo_path("exchange", false);
    return;
  }
  const char* hm = std::getenv("PE_HALO");
  const char* ov = std::getenv("PE_OVERLAP");
  // (the two-step sweep has no boundary-item signal; every rank decides this
  // from global inputs — a rank without neighbours still takes part, its
  // overlap is simply off in setup_items)
  const bool ov_able = !sstep_ || steps_ >= 3;
  struct Cand {
    std::string path;
    bool ov;
    double ms;
    int ti;  // rows per item (0: the construction's)
  };
  std::vector<Cand> cands;
  // The overlapped candidates run at each of the rows-per-item tuning's three
  // best heights (its boundary-first layout ranks them differently); with the
  // exchange among the candidates the put's overlap runs only at the height
  // the exchange's overlap timed best (the halo path does not move that rank).
  const int ti0 = kp_->ti;
  std::vector<int> heights = ti_alt_.empty() ? std::vector<int>{ti0} : ti_alt_;
  {  // every rank times as many candidates (and calls host_max as often): each
     // rank tunes its own block's rows per item — or none, when its block is
     // past the tuning's size — so the number of heights can differ
    double v[1] = {-double(heights.size())};
    comm_->host_max(v, 1, stream_);
    heights.resize(size_t(std::max(1.0, -v[0])));
  }
  auto add = [&](const char* path, bool o) {
    if (o && !ov_able) return;
    if (ov && (std::atoi(ov) != 0) != o) return;
    if (!o) {
      cands.push_back(Cand{path, o, 0.0, 0});
      return;
    }
    for (int h : heights) cands.push_back(Cand{path, o, 0.0, h});
  };
  // (the plain-layout candidates first, then the overlapped ones, height by height)
  const bool ex_ok = !hm || std::string(hm) == "exchange";
  if (ex_ok) add("exchange", false);
  if (put_ok_) add("put", false);
  if (push_ok_ && !(ov && std::atoi(ov) != 0)) cands.push_back(Cand{"push", false, 0.0, 0});
  if (ex_ok) add("exchange", true);
  // (not when ranks share a GPU — test jobs: put blocks spinning on the halo
  // stream under another process's persistent sweep can starve it of CUs; a
  // 6-process 2×3 job on one GPU stalled past 3 minutes, round 6)
  const bool put_ov_forced = hm && std::string(hm) == "put" && ov && std::atoi(ov) != 0;
  const bool put_ov = put_ok_ && (!shared_dev_ || put_ov_forced) && ov_able && !(ov && std::atoi(ov) == 0);
  const bool put_ov_late = put_ov && ex_ok && !cands.empty() && cands.back().ov;  // (after the exchange's heights)
  if (put_ov && !put_ov_late) add("put", true);
  if (cands.empty()) {  // (the forced path is not available here: the exchange, at every height when overlapped)
    if (ov && std::atoi(ov) != 0 && ov_able) {
      for (int h : heights) cands.push_back(Cand{"exchange", true, 0.0, h});
    } else {
      cands.push_back(Cand{"exchange", false, 0.0, 0});
    }
  }
  auto name = [](const Cand& c) { return c.path + (c.ov ? "+overlap" : ""); };
  // (an overlap at another height than the tuned one is reported as "exchange+overlap @96")
  auto label = [&](const Cand& c) { return name(c) + (c.ov && c.ti != ti0 ? " @" + std::to_string(c.ti) : std::string()); };
  const bool tune = !(std::getenv("PE_HALO_TUNE") && std::atoi(std::getenv("PE_HALO_TUNE")) == 0);
  if ((cands.size() == 1 && !put_ov_late) || !tune) {
    apply_halo_path(cands[0].path, cands[0].ov, false, cands[0].ti);
    halo_path_ = name(cands[0]) + (cands.size() == 1 ? " (only candidate)" : " (PE_HALO_TUNE=0)");
    return;
  }
  Range range("pe.choose_halo_path");
  lay_cache_.clear();
  lay_cache_on_ = true;
  if (fused_) lay_cache_[{kp_->ti, overlap_, lay_name_}] = snap_layout();  // (the construction's)
  const int keep_tol = kp_->check_tol;
  kp_->check_tol = 0;
  // (PE_CTOR_TRACE=1: rank 0's candidate times; 2: every rank's, with the
  // host-side split of each candidate into switch and timing)
  const int trace_lvl = std::getenv("PE_CTOR_TRACE") ? std::atoi(std::getenv("PE_CTOR_TRACE")) : 0;
  const bool trace = trace_lvl >= 2 || (trace_lvl == 1 && blk_.rank == 0);
  const auto t_reset = clk::now();
  reset();
  if (trace_lvl >= 2) {
    PE_HIP_CHECK(hipStreamSynchronize(stream_));
    std::fprintf(stderr, "[pe] halo path reset %6.3f ms\n", 1e3 * secs(t_reset, clk::now()));
  }
  // the overlapped candidates' layouts are built ahead, on the host, while
  // the GPU times the candidates before them (1.3-2.6 ms of host work each
  // at the 8-rank slab of 8192², against 0.5-0.7 ms of timing)
  std::vector<int> ahead;
  for (const Cand& c : cands)
    if (c.ov && std::find(ahead.begin(), ahead.end(), c.ti) == ahead.end()) ahead.push_back(c.ti);
  struct IdleOff {  // (the hook captures this frame: off on every way out)
    std::function<void()>& f;
    ~IdleOff() { f = nullptr; }
  } idle_off{halo_idle_};
  halo_idle_ = [&]() {
    if (ahead.empty()) return;
    const int h = ahead.front();
    ahead.erase(ahead.begin());
    const auto t0 = clk::now();
    prepare_layout(h, true);
    if (trace_lvl >= 2)
      std::fprintf(stderr, "[pe] halo path layout ahead: overlap at %d rows %6.3f ms\n", h, 1e3 * secs(t0, clk::now()));
  };
  auto time_path = [&](const Cand& c) {
    const auto ta = clk::now();
    apply_halo_path(c.path, c.ov, true, c.ov ? c.ti : ti0);
    const auto tb = clk::now();
    const double ms = time_halo_path(3, 1, false);
    if (trace_lvl >= 2)
      std::fprintf(stderr, "[pe] halo path %-24s apply %6.3f ms, timing %6.3f ms\n", label(c).c_str(),
                   1e3 * secs(ta, tb), 1e3 * secs(tb, clk::now()));
    return ms;
  };
  for (Cand& c : cands) {
    c.ms = time_path(c);
    halo_cands_.emplace_back(label(c), 1e3 * c.ms);
  }
  if (put_ov_late) {  // the put's overlap at the exchange overlap's best height
    int h = ti0;
    double bms = 1e300;
    for (const Cand& c : cands)
      if (c.ov && c.ms < bms) bms = c.ms, h = c.ti;
    cands.push_back(Cand{"put", true, 0.0, h});
    cands.back().ms = time_path(cands.back());
    halo_cands_.emplace_back(label(cands.back()), 1e3 * cands.back().ms);
  }
  // finalists: the two fastest once more (the clock ramps during construction)
  std::vector<size_t> order(cands.size());
  for (size_t i = 0; i < order.size(); ++i) order[i] = i;
  std::stable_sort(order.begin(), order.end(), [&](size_t a, size_t b) { return cands[a].ms < cands[b].ms; });
  for (size_t f = 0; f < 2 && f < order.size(); ++f) {
    Cand& c = cands[order[f]];
    const double ms = time_path(c);
    halo_cands_.emplace_back(label(c) + " (again)", 1e3 * ms);
    c.ms = std::min(c.ms, ms);
  }
  size_t best = 0;
  for (size_t i = 1; i < cands.size(); ++i)
    if (cands[i].ms < cands[best].ms) best = i;
  apply_halo_path(cands[best].path, cands[best].ov, true, cands[best].ov ? cands[best].ti : ti0);
  PE_HIP_CHECK(hipStreamSynchronize(stream_));  // (the solve resets the state)
  halo_path_ = name(cands[best]);
  halo_idle_ = nullptr;
  lay_cache_on_ = false;
  lay_cache_.clear();
  kp_->check_tol = keep_tol;
  if (trace) {
    for (const auto& c : halo_cands_) std::fprintf(stderr, "[pe] halo path %-24s %8.2f us/sweep\n", c.first.c_str(), c.second);
    std::fprintf(stderr, "[pe] halo path chosen: %s\n", halo_path_.c_str());
  }
}

void DeviceSolver::set_halo_path(const std::string& path, bool overlap) {
  if ((path == "push" && !push_ok_) || (path == "put" && !put_ok_) ||
      (path != "push" && path != "put" && path != "exchange"))
    throw std::invalid_argument("set_halo_path: '" + path + "' is not available (push: " + push_status_ +
                                ", put: " + put_status_ + ")");
  apply_halo_path(path, overlap, true);
  halo_path_ = path + (overlap_ ? "+overlap" : "") + " (set)";
}

// `warm` + `sweeps` sweeps of the real iteration (the stop test off), from the
// initial state when `from_reset`, else from the current one; the last
// `sweeps` timed; ms per sweep, max over ranks.
double DeviceSolver::time_halo_path(int sweeps, int warm, bool from_reset) {
  const int keep_tol = kp_->check_tol;
  kp_->check_tol = 0;
  if (from_reset) reset();
  if (warm > 0) run_iterations(int64_t(warm) * steps_, false);
  PE_HIP_CHECK(hipEventRecord(t0_, stream_));
  run_iterations(int64_t(sweeps) * steps_, false);
  PE_HIP_CHECK(hipEventRecord(t1_, stream_));
  if (halo_idle_) halo_idle_();  // (host work under the timed sweeps: GPU-event timing)
  wait_event(t1_);
  kp_->check_tol = keep_tol;
  float ms = 0.f;
  PE_HIP_CHECK(hipEventElapsedTime(&ms, t0_, t1_));
  double v[1] = {double(ms) / sweeps};
  comm_->host_max(v, 1, stream_);
  return v[0];
}

}  // namespace pe
