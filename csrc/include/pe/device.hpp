// Device (MI355X) runtime: stream-ordered communication + the device-resident
// PCG solver.  Replaces the stage-4 driver gradient_solver_mpi
// (poisson_mpi_cuda2.cu:687-982) and its host-staged halo exchange
// exchange_halos_2d_gpu (:331-500).
#pragma once

#include <hip/hip_runtime_api.h>

#include <memory>
#include <stdexcept>
#include <array>
#include <functional>
#include <map>
#include <tuple>
#include <string>
#include <vector>

#include "pe/comm.hpp"
#include "pe/solver.hpp"

#define PE_HIP_CHECK(expr)                                                                     \
  do {                                                                                         \
    hipError_t _e = (expr);                                                                    \
    if (_e != hipSuccess) ::pe::hip_fail(_e, #expr, __FILE__, __LINE__);                       \
  } while (0)

namespace pe {

namespace dev {
struct PeerSum;
}  // namespace dev

[[noreturn]] void hip_fail(hipError_t e, const char* expr, const char* file, int line);
int device_count();
void set_device(int dev);  // hipSetDevice + one pooled solver stream and halo stream for that device
// Solver streams (non-blocking) from / back to the per-device idle pool.
hipStream_t acquire_stream();
void release_stream(hipStream_t s);
// High-priority halo streams (the overlap's), pooled the same way.
hipStream_t acquire_halo_stream();
void release_halo_stream(hipStream_t s);
std::string device_name(int dev);
int current_device();
std::string device_pci_bus_id(int dev);

// Stream-ordered transport over device buffers.
class DeviceComm {
 public:
  virtual ~DeviceComm() = default;
  virtual int rank() const = 0;
  virtual int size() const = 0;
  virtual void allreduce_sum(double* dbuf, int n, hipStream_t s) = 0;
  virtual void allreduce_max(double* dbuf, int n, hipStream_t s) = 0;
  virtual void exchange(const std::vector<Exchange>& ex, hipStream_t s) = 0;
  // Host-side max of a few doubles (timer reduction); may synchronize.
  virtual void host_max(double* hbuf, int n, hipStream_t s) = 0;
  virtual void barrier(hipStream_t s) = 0;
  virtual bool capturable() const { return false; }
  virtual std::string name() const = 0;
  // Failure detection: poll asynchronous transport errors (throws), and
  // abort the communicator so peers blocked in it fail instead of hanging.
  virtual void check_async() {}
  virtual void abort() {}
  // One-shot P2P sum tables (P2P transport only): the single-sweep solver
  // then sums its per-iteration scalars over ranks inside the sweep.
  virtual const dev::PeerSum* peer_sum() const { return nullptr; }
  // Collective (every rank calls it, in the same order): map every rank's
  // `mine` — a fine-grained device buffer of that process — into this one.
  // result[r] = rank r's buffer (result[rank()] = mine); empty on EVERY rank
  // when any rank cannot map (no peer-mapping transport, or a failure).
  virtual std::vector<void*> map_peer_buffers(void* mine) {
    (void)mine;
    return {};
  }
  // Release a mapping made by map_peer_buffers (this process's side only).
  virtual void unmap_peer_buffers(const std::vector<void*>& peers) { (void)peers; }
};

class SelfDeviceComm final : public DeviceComm {
 public:
  int rank() const override { return 0; }
  int size() const override { return 1; }
  void allreduce_sum(double*, int, hipStream_t) override {}
  void allreduce_max(double*, int, hipStream_t) override {}
  void exchange(const std::vector<Exchange>&, hipStream_t) override {}
  void host_max(double*, int, hipStream_t) override {}
  void barrier(hipStream_t) override {}
  bool capturable() const override { return true; }
  std::string name() const override { return "self"; }
};

// RCCL (NCCL API) over xGMI.  The 128-byte unique id is produced by rank 0
// (rccl_unique_id) and distributed by the caller (torch.distributed store,
// or the pe_launch bootstrap file).
std::string rccl_unique_id();
std::unique_ptr<DeviceComm> make_rccl_comm(const std::string& uid, int rank, int size);
// Wrap an existing ncclComm_t (e.g. one owned by another runtime); not owned.
std::unique_ptr<DeviceComm> make_rccl_comm_from_handle(void* nccl_comm);

// Host-staged transport over caller callbacks (e.g. torch.distributed gloo):
// device → host copy, host collective, host → device copy — the reference's
// stage-4 pattern (poisson_mpi_cuda2.cu:331-500).  A test/fallback transport
// for several ranks sharing one GPU (RCCL refuses duplicate devices); the
// production transport is RCCL.
// Timing-only test transport (stream-ordered busy waits; no data moves).
// loopback: the exchange also copies each send buffer into its own receive
// buffer, stream-ordered (an asynchronous transport that moves data).
std::unique_ptr<DeviceComm> make_delay_comm(int size, double exchange_us, double allreduce_us, bool loopback = false);
// One-shot P2P allreduce (IPC-mapped receive buffers, p2p.hip) for the
// per-iteration sums; everything else through `base` (PE_ALLREDUCE=p2p).
std::unique_ptr<DeviceComm> make_p2p_allreduce_comm(std::unique_ptr<DeviceComm> base);
// The last make_p2p_allreduce_comm of this process: "not attempted", "ok" or
// "fallback: <reason>" (its self-tests; bench / CLI diagnostics).
const std::string& p2p_setup_status();
std::unique_ptr<DeviceComm> make_callback_device_comm(int rank, int size, CallbackHostComm::ReduceFn reduce,
                                                      CallbackHostComm::ExchangeFn exch,
                                                      CallbackHostComm::BarrierFn barrier);

namespace dev {
struct DevState;
struct KParams;
struct ResParams;
}  // namespace dev

class DeviceSolver {
 public:
  DeviceSolver(const Problem& prob, const Block& blk, DeviceComm* comm, const SolveOptions& opt);
  ~DeviceSolver();
  DeviceSolver(const DeviceSolver&) = delete;
  DeviceSolver& operator=(const DeviceSolver&) = delete;

  // Full solve: init + iterations until convergence / cap + error.
  SolveResult solve();
  // Benchmark helpers: reset to the initial state, then run exactly `iters`
  // iterations (convergence test off when check_tol == false).
  void reset();
  void run_iterations(int64_t iters, bool use_graph);
  // Capture + instantiate every chunk graph run_iterations(iters, true)
  // will launch, so a timed run_iterations contains no capture.
  void prepare_graphs(int64_t iters);
  // Switch the convergence test on / off (drops cached graphs): the bench
  // times fixed-work steps, then solves to convergence on the same solver.
  void set_check_tol(bool on);
  // Initial guess of the next reset() / solve() (bench: the BASELINE
  // random-init solve on the same solver as the zero-init one).
  void set_init(Init init, uint64_t seed, double amp);
  // Tuning probe: re-lay out the work items for `ti` rows per item, re-reading
  // the PE_* layout knobs (same allocation, so configurations compare at one
  // memory placement).  Drops cached graphs.
  void relayout(int ti, int order = -1);  // probe: re-lay out the items (ti rows; order 0 / 3, -1 keeps)
  double time_iterations(int64_t iters, bool use_graph);  // device seconds (events)
  // Wait for the stream; with PE_WATCHDOG_S set (or a stall injected) the
  // wait is bounded: no progress for that long aborts the communicator and
  // throws (the bench's timed region and solve are both covered).
  void synchronize();

  // Phases (used by the virtual-rank group driver and tests).
  void enqueue_init();
  void enqueue_F(int par);
  void enqueue_G(int par);
  void enqueue_S(int par);      // single-sweep iteration kernel
  void enqueue_pack(int buf);   // single-sweep: y strips of buffer `buf` → send buffers
  void enqueue_unpack(int buf); // single-sweep: recv buffers → y halo columns of `buf`
  void enqueue_error();
  void enqueue_wflush();        // single-sweep: add a deferred α·p term to w (no-op if none)
  double* red_F_dev();
  double* red_G_dev();
  double* fs_dev(int par);
  double* fs2_dev(int par);  // multi-step sweeps' sums (kNS2 / kNS3 of them)
  double* err_dev();
  // Halo exchange as ordered phases; after a phase with `unpack` set the
  // received y strips are scattered into buffer `buf` (single-sweep layout:
  // y phase, unpack, then x phase whose rows carry the corners).  The
  // classic path has one phase (r: x rows + y strips).
  struct HaloPhase {
    std::vector<Exchange> ex;
    bool unpack = false;
  };
  std::vector<HaloPhase> halo_phases(int buf) const;
  std::vector<Exchange> halo_plan() const;  // classic: the single phase
  bool fused() const { return fused_; }
  // two iterations per sweep (fused2.hip)
  bool two_step() const { return sstep_; }     // a multi-iteration sweep (two- or three-step)
  int sweep_steps() const { return steps_; }   // iterations per sweep launch: 1, 2 or 3
  // LDS-resident single sweep (resident.hip): small single-rank blocks run
  // each chunk of iterations as one launch.  PE_RESIDENT=0 disables.
  bool resident() const { return resident_; }
  bool resident_fallback() const { return resident_fallback_; }
  bool overlap() const { return overlap_; }
  // Halo rows pushed by the sweep itself over xGMI (row slabs + in-sweep P2P
  // sums): no exchange call in the iteration, which is then graph-capturable.
  bool halo_push() const { return push_; }
  // Halo exchange by the solver's own peer-put kernel (p2p.hip kPut) instead
  // of the comm's exchange (RCCL grouped send / receive).
  bool halo_put() const { return put_; }
  // The iteration replays from captured hipGraphs (run_iterations(.., true)):
  // no comm call inside it and no two-stream overlap
  bool graphs_usable() const;
  // Multi-rank halo path chosen at construction by timing the candidates on
  // the job's own transport (max over ranks): "exchange", "put" or "push",
  // "+overlap" when the exchange runs on the halo stream under the interior
  // items; halo_candidates() = {path, µs per sweep} as timed ("forced: …" /
  // "none: …" when there was nothing to choose).
  const std::string& halo_path() const { return halo_path_; }
  const std::vector<std::pair<std::string, double>>& halo_candidates() const { return halo_cands_; }
  const std::string& put_status() const { return put_status_; }
  // Probes: switch to another halo path after construction (one of the
  // candidates the construction could pick; the item list is re-laid out for
  // the overlap), and time `sweeps` sweeps of the current path after `warm`
  // ones, from a reset or from the current state (ms per sweep, max over
  // ranks; collective).
  void set_halo_path(const std::string& path, bool overlap);
  double time_halo_path(int sweeps, int warm = 2, bool from_reset = true);
  uintptr_t fields_address() const { return reinterpret_cast<uintptr_t>(fields_); }
  const std::vector<float>& placement_ms() const { return placement_ms_; }
  int placement_choice() const { return placement_best_; }       // index into placement_ms()
  // multi-rank: the slowest rank's chosen ms/sweep (the job runs at its pace;
  // this rank's own choice when alone, 0 without a search)
  double placement_job_ms() const { return placement_job_ms_; }
  double placement_seconds() const { return placement_s_; }      // wall time of the search
  double construct_seconds() const { return ctor_s_; }           // wall time of the constructor
  double exchange_us() const { return exchange_us_; }            // measured halo exchange (multi-rank)
  const std::vector<float>& ti_tuning_ms() const { return ti_ms_; }  // per candidate (8, 10, 14, 18 rows)
  const std::vector<int>& ti_tuning_rows() const { return ti_rows_; }  // the candidates
  // static layout: {most loaded wave, mean wave load, max items on a wave}
  // in row-step cost units (0s for a dynamic layout)
  std::vector<double> layout_load() const { return {lay_max_, lay_mean_, double(lay_items_)}; }
  int layout_cuts() const { return lay_cuts_; }
  // the static layout in use: "lpt", "fill" or "equal" (three-step sweep)
  const std::string& layout_name() const { return lay_used_; }
  // the item list as laid out (host copy of KParams::ilist; empty for walks
  // without a list): {first row | flags, strip | rows << 20} per position
  const std::vector<int2>& layout_entries() const { return ilist_host_; }
  // overlap: list positions 0 .. n-1 hold the boundary items (0: no overlap)
  int layout_boundary() const { return overlap_ ? ov_lnb_[0] : 0; }
  // First cross-device run diagnostics: hipDeviceCanAccessPeer of this
  // rank's device toward each rank's (1 / 0; -1 the same device; empty on
  // one rank), why the halo push is on / off / fell back, and the transport
  // of the per-sweep sums.
  const std::vector<int>& peer_access() const { return peer_access_; }
  const std::string& push_status() const { return push_status_; }
  const std::string& xr_status() const { return xr_status_; }
  hipStream_t stream() const { return stream_; }

  // Checkpoint / resume of the full device state of this rank (raw fields,
  // halo buffers, scalar block, iteration parity).  Synchronizes the stream.
  void save_checkpoint(const std::string& path);
  void load_checkpoint(const std::string& path);

  // State / data access.
  void read_state(dev::DevState* out);
  void copy_w(double* host, bool owned_only = true);  // nx × ny row-major
  // 0 r, 1 w, 2 p0, 3 p1 (single-sweep: 0 r of x[0], 2 p of x[0], 3 p of
  // x[1], 4 r of x[1]) as field_rows() × field_cols(), local (-h, -h) first.
  void copy_field(int which, double* host);
  int64_t field_rows() const;
  int64_t field_cols() const;
  const Block& block() const { return blk_; }
  const Problem& problem() const { return prob_; }
  int chunk() const { return chunk_; }
  dev::KParams& params();
  // PE_STAMPS=1 diagnostic timeline of the last sweep (see KParams::stamps);
  // empty when off.
  std::vector<unsigned long long> stamps();
  void clear_stamps();  // stream-ordered: the next sweep's stamps only

 private:
  void build_tables(int64_t rows_hi, int64_t cols_hi);
  void upload(void* dst, const void* src, size_t bytes);  // set-up data via pinned staging + copy kernel
  void set_fused_fields(double* x0, double* x1, double* w);
  void setup_items();  // item lists: static LPT layout or dynamic per-XCD shards (+ halo/interior overlap)
  void create_halo_stream();
  void choose_placement();   // local search, then (multi-rank) the coordinated retry round
  bool placement_search(bool retry);  // local; true when the kept candidate is in the best class
  void measure_exchange();  // sets exchange_us_ (collective)
  void setup_resident();    // tile geometry, band-table size, buffers (single rank, small blocks)
  void set_items(int ti);   // item counts and persistent grids for `ti` rows per item
  void enqueue_iteration(int par, int mlimit = 0);  // mlimit > 0: a partial three-step sweep
  void enqueue_fs_reduce(int par);  // cross-rank sum of sweep sums (no-op when the sweep does it)
  // after_sweep: the halo of `buf` was produced by a sweep (with the halo
  // push: import it); false for the initial state (the comm's exchange).
  void enqueue_exchange(int buf, bool after_sweep = true);
  void setup_halo_push();  // collective: maps the push's receive buffers (push_ok_) identically on every rank
  void setup_halo_put();   // collective: maps the put's inboxes + self-test (put_ok_) identically on every rank
  // collective: time the available halo paths (exchange / put / push, with and
  // without the overlap) for a few sweeps each and keep the fastest (max over ranks)
  void choose_halo_path();
  // Item lists already laid out, while the rows per item are tuned and the
  // halo path is chosen (their candidates come back to layouts already built:
  // 0.3-2.6 ms of host work each)
  struct LayoutSnap {
    std::vector<int2> list;
    int static_waves, ov_nb, ov_lnsh, ov_lbase[9], ov_lnb[8], lay_items, lay_cuts;
    double lay_max, lay_mean;
    std::string lay_used;
    int lnsh, lwaves, nslots, lbase[9], lnb[8], nblocks, nblocks0;
  };
  // switch path + re-lay the items; live: the iteration state carries on (halo moved between x and the push buffer)
  // ti > 0: rows per item of the overlap's layout (another height than the tuning's)
  void apply_halo_path(const std::string& path, bool overlap, bool live = false, int ti = 0);
  LayoutSnap snap_layout() const;
  void restore_layout(const LayoutSnap& v);
  void prepare_layout(int ti, bool overlap);  // into the cache, host only (item_layout.cpp)
  // one halo phase through the put kernel (put_) or the comm
  void xfer(const std::vector<Exchange>& ex, hipStream_t s);
  void import_halos();     // halo push: x's halo rows <- the receive buffers (enqueued)
  // End-of-solve true residual (single-sweep layouts): w → the p-plane of
  // x[0], the sweep's halo exchange, then kResid into DevState::res
  // (with_r: against the recurrence's r; store: ρ → x[0]'s r-plane) and the
  // cross-rank sum of the four sums.
  void residual_pass(bool with_r, bool store);
  void wait_event(hipEvent_t ev);  // event wait with transport-error polling + watchdog
  void enqueue_chunk(int iters, int sample_iters = 0);
  // Sampled phase timing (Timers): hipEvent pairs around the phases of the
  // sampled iterations, read once their chunk has completed.
  enum Phase { kPhSweep, kPhDot, kPhHalo, kPhReduce, kPhCopy, kNPhase };
  struct PhaseRec {
    int ph;
    int64_t iter;  // first iteration covered (kPhCopy: the chunk's last), for dropping post-convergence samples
    int64_t n;     // iterations covered (a resident launch covers its whole chunk)
    hipEvent_t a, b;
  };
  struct PhaseSample {
    int ph;
    int64_t iter, n;
    float ms;
  };
  hipEvent_t pooled_event();
  void mark_begin(int ph, hipStream_t s);
  void mark_end(hipStream_t s);
  void harvest(size_t n);  // read the first n records (their events have completed)
  hipGraphExec_t graph_for(int iters);

  Problem prob_;
  Block blk_;
  DeviceComm* comm_;
  std::unique_ptr<DeviceComm> self_;
  SolveOptions opt_;
  hipStream_t stream_ = nullptr;
  bool fused_ = false;
  bool sstep_ = false;    // multi-iteration sweep (fused2.hip / fused3.hip): steps_ iterations per launch
  int steps_ = 1;         // iterations per sweep launch (1, 2, 3)
  int fsw_ = 124;         // output columns per strip (kFSW / kFSW2 / kFSW3)
  int hdep_ = 2;          // halo depth of the single-sweep layouts (2 / 4 / 6)
  int xorg_ = 1;          // columns stored left of column 0 (KParams::xorg)
  int64_t tab_lo_ = -1;   // first local index of the chord tables / row classes
  double* fields_ = nullptr;  // classic: r, w, p0, p1 (alloc each); single-sweep: x0, x1, w
  double* xalt_ = nullptr;    // single-sweep: x1 (separate allocation)
  double* walt_ = nullptr;    // single-sweep: w
  std::vector<float> placement_ms_;  // per-candidate sweep time of the placement search
  int64_t xsize_ = 0, wsize_ = 0, plane_ = 0;
  double* tables_ = nullptr;
  int* rowcls_ = nullptr;
  std::vector<int> rowcls_host_;  // host copy of the row classes (item cost estimates)
  double* halo_ = nullptr;    // send_dn, send_up, recv_dn, recv_up (nx each; ×4 single-sweep)
  int64_t hsize_ = 0;
  double* partial_ = nullptr;
  double* hist_ = nullptr;
  unsigned long long* stamps_ = nullptr;
  size_t nstamps_ = 0;
  // halo/interior overlap (multi-rank single-sweep)
  bool overlap_ = false;
  int2* ilist_ = nullptr;  // per shard: boundary items, heavy items, the rest (dev::KParams::ilist)
  size_t ilist_cap_ = 0;   // entries allocated at ilist_
  std::vector<int> pgen_, pmix_;  // item layout: per strip, prefix counts of band / mixed rows (item_layout.cpp)
  std::vector<std::array<int64_t, 4>> eq_runs_[2];  // equal-cost layout: runs {first row, rows, strip, kind} (no overlap / overlap)
  int nslot_cap_ = 0;      // item-sum slots allocated
  int ov_lnsh_ = 1, ov_nb_ = 0, ov_reserve_ = 8, ov_debug_ = 0;
  int wave_cap_ = 0;     // resident waves of the sweep grid (occupancy)
  int static_waves_ = 0; // static list walk: waves the list is laid out for (0: no static list)
  int ov_lbase_[9] = {}, ov_lnb_[8] = {};
  unsigned long long ov_epoch_ = 0;  // overlapped sweeps since the state was last cleared (sig targets)
  hipStream_t hs_ = nullptr;
  hipEvent_t ev_halo_ = nullptr;
  dev::DevState* st_ = nullptr;
  dev::DevState* hst_ = nullptr;  // pinned, 2 slots
  std::unique_ptr<dev::KParams> kp_;
  std::vector<std::pair<int, hipGraphExec_t>> graphs_;  // instantiated chunk graphs, by length
  int chunk_ = 16;
  int par_ = 0;  // parity of the next iteration (x / p ping-pong)
  double watchdog_s_ = 0;   // PE_WATCHDOG_S: abort if a chunk makes no progress this long (0 = off)
  bool fault_stall_ = false;  // PE_FAULT_INJECT=stall: pretend the device never finishes (watchdog test)
  // PE_FAULT_INJECT=drift@iter:K,amp:X — w(M/2, N/2) += X once the host has
  // enqueued iteration K (the residual check's test hook)
  long long fault_drift_ = 0;
  double fault_drift_amp_ = 1e-6;
  // three-step restart threshold on ‖B − A w − r‖_E / ‖r‖_E (PE_RESID_GAP)
  double gap_bound_ = 1e-4;
  hipEvent_t ev_[2] = {nullptr, nullptr};
  hipEvent_t ev_sync_ = nullptr;  // synchronize() under the watchdog
  hipEvent_t t0_ = nullptr, t1_ = nullptr;
  std::vector<hipEvent_t> evpool_;
  std::vector<PhaseRec> recs_;
  std::vector<PhaseSample> samples_;
  bool sampling_ = false;
  int64_t sample_iter_ = 0;  // iteration index of the next enqueued iteration (sampled chunks)
  double ctor_s_ = 0, copy_setup_s_ = 0, placement_s_ = 0;
  bool ctor_counted_ = false;
  int placement_best_ = 0;
  double placement_job_ms_ = 0;
  bool tune_ti_ = false;          // rows per item chosen by timing candidate sweeps
  std::vector<float> ti_ms_;      // their per-sweep times
  std::vector<int> ti_rows_;      // the candidates timed
  std::vector<int> ti_alt_;       // the tuning's best two heights (the overlap is timed at both)
  double lay_max_ = 0, lay_mean_ = 0;  // static layout: heaviest / mean wave load (row steps)
  int lay_items_ = 0;                  // static layout: most items on one wave
  int lay_cuts_ = 0;                   // three-step filling layout: items cut to fill the waves
  // three-step static layout: lay_name_ the construction's choice (by block
  // size / rows-per-item tuning; PE_LAYOUT overrides), lay_used_ the last laid out
  std::string lay_name_ = "lpt", lay_used_ = "lpt";
  std::vector<int> peer_access_;
  std::vector<int2> ilist_host_;
  std::map<std::tuple<int, bool, std::string>, LayoutSnap> lay_cache_;  // (rows per item, overlap, layout name)
  bool lay_cache_on_ = false;
  bool lay_dry_ = false;                   // setup_items lays out for the cache only (no upload)
  std::function<void()> halo_idle_;        // host work while time_halo_path's sweeps run (the choice's next layouts)
  std::string push_status_ = "off", xr_status_ = "none";
  int wave_caps_[2] = {0, 0};     // resident waves of the applying / deferring sweep
  int cus_ = 256;                  // compute units of the device (a static layout's first cus_ workgroups run first on their CU)
  bool resident_ = false;
  bool resident_fallback_ = false;  // a resident launch aborted (status 5): switched to the streaming sweep
  int stream_chunk_ = 16;           // chunk length of the streaming sweep (after a resident fallback)
  std::unique_ptr<dev::ResParams> rp_;
  int* res_rowstart_ = nullptr;
  double* res_buf_ = nullptr;  // edges then partials
  unsigned* res_ctr_ = nullptr;
  void* stage_ = nullptr;           // pinned staging buffer of upload()
  size_t stage_bytes_ = 0;
  bool push_ = false;               // in-sweep halo push (KParams::push)
  bool push_ok_ = false;            // push set up on every rank: a halo-path candidate
  bool push_loop_ = false;          // PE_PUSH_LOOPBACK diagnostic (own receive buffer)
  bool put_ = false;                // halo phases through kPut (peer put) instead of comm_->exchange
  bool put_ok_ = false;             // put set up and self-tested on every rank: a halo-path candidate
  bool put_loop_ = false;           // PE_PUT_LOOPBACK: this rank is its own peer (one-GPU probes / tests)
  bool want_overlap_ = false;       // the chosen path's overlap (setup_items)
  bool shared_dev_ = false;         // another rank of the job runs on this rank's GPU (test jobs)
  void* put_buf_ = nullptr;         // fine-grained: [4 dirs][kPutParts] flags, then [4 dirs][2][put_stride_] inbox
  std::vector<void*> put_peers_;    // every rank's put_buf_ mapped here
  unsigned* put_cnt_ = nullptr;     // PutArgs::cnt (device)
  int64_t put_stride_ = 0;          // doubles per inbox parity
  double put_timeout_s_ = 120.0;    // a peer that never arrives poisons the halo after this long (PE_P2P_TIMEOUT_S)
  std::string put_status_ = "off";
  std::string halo_path_ = "none: one rank";
  std::vector<std::pair<std::string, double>> halo_cands_;
  double* hrecv_ = nullptr;         // its fine-grained receive buffer [2][2][2 × pitch]
  std::vector<void*> hpeers_;       // every rank's receive buffer mapped here (comm_->map_peer_buffers)
  double exchange_us_ = 0;  // measured halo exchange (max over ranks), multi-rank only  // the first solve() carries the construction time
};

// Per-row coefficient classes from the chord tables (see row_classes.cpp):
// for each local row q ∈ [-1, rows_hi-1], {in_lo, in_hi, out_lo, out_hi} such
// that every face coefficient of node (q, lj) is exactly 1 for lj ∈ [in_lo,
// in_hi] and exactly 1/eps for lj ∉ [out_lo, out_hi], lj ∈ [-1, cols_hi].
// Conservative: anything else is evaluated exactly.  (rows_hi+2) × 4 ints.
// Tables and classes start at local index `lo` (-1; the two-step sweep's
// 4-deep halo: -4): entry of local q at (q - lo).
std::vector<int> row_classes(const double* colT, const double* rowT, int64_t rows_hi, int64_t cols_hi,
                             int64_t lo = -1);
// Chord tables of a block: (rows_hi+2)×4 column entries {halfA, sB, eB, x}
// for li ∈ [-1, rows_hi], then (cols_hi+2)×4 row entries {sA, eA, halfB, y}
// for lj ∈ [-1, cols_hi]; indexed by local index + 1.  The classic kernels
// use rows_hi = nx+2, cols_hi = ny+2; the single-sweep kernel reaches two
// halo nodes further and past ny into strip padding.
std::vector<double> chord_tables(const Problem& P, const Block& blk, int64_t rows_hi, int64_t cols_hi,
                                 int64_t lo = -1);
// Host mirror of the kernels' coefficient path for local (li, lj) ∈
// [0, nx+1] × [0, ny+1]: a(li, lj), b(li, lj) and the class (0 interior,
// 1 exterior, 2 boundary band).  Row-major (nx+2) × (ny+2).
void host_coefficients(const Problem& P, const Block& blk, std::vector<double>& a, std::vector<double>& b,
                       std::vector<int>& cls);

// P virtual ranks on ONE device (LocalComm).  Every rank runs the
// same kernels and the same halo plan as under RCCL; the transport is
// device-to-device copies + a cross-stream reduction kernel.
SolveResult device_solve_group(const Problem& prob, int ranks, DecompMode mode, const SolveOptions& opt,
                               std::vector<double>* w_out = nullptr);
SolveResult device_solve_group(const Problem& prob, const ProcessGrid& pg, const SolveOptions& opt,
                               std::vector<double>* w_out = nullptr);

}  // namespace pe
