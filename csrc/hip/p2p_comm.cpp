// P2P allreduce transport: a DeviceComm that keeps its base transport (RCCL,
// or host-staged for tests) for the halo exchange and everything else, but
// runs the sums of a few doubles as one kernel writing into IPC-mapped
// receive buffers of every peer (peer_sum.hpp).  It also hands its buffer
// table to the single-sweep solver (peer_sum()), whose final reduction block
// then does the cross-rank sum itself: an iteration needs no allreduce launch.
//
// Set-up is collective and fail-safe: every rank maps the peers' buffers,
// the ranks agree (through the base transport) that all of them succeeded,
// run one test sum with a short timeout against the exact expected value,
// and agree again; if anything failed anywhere, every rank falls back to the
// base transport (make_p2p_allreduce_comm returns it unwrapped).
#include <hip/hip_runtime_api.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <stdexcept>
#include <string>
#include <vector>

#include "../hip/kernels.hpp"
#include "pe/device.hpp"

namespace pe {
namespace {

// What the last P2P set-up of this process decided (bench / CLI diagnostics).
std::string g_p2p_status = "not attempted";

class P2PAllreduceComm final : public DeviceComm {
 public:
  explicit P2PAllreduceComm(std::unique_ptr<DeviceComm> base) : base_(std::move(base)) {
    const int P = base_->size(), me = base_->rank();
    if (P > 64) throw std::invalid_argument("p2p allreduce: at most 64 ranks");
    if (const char* e = std::getenv("PE_P2P_TIMEOUT_S")) timeout_s_ = std::atof(e);
    hipStream_t s = nullptr;
    PE_HIP_CHECK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    bool ok = setup(P, me, s);
    const bool mapped_here = ok;
    ok = agree(ok, s);
    if (!ok) why_ = mapped_here ? "a peer could not map the receive buffers" : "this rank could not map the receive buffers";
    if (ok) {
      // test sum with a short timeout: rank r contributes r+1 (and -(r+1)):
      // exact in fp64, the same bits on every rank
      ps_.timeout_ticks = 500000000LL;  // 5 s at 100 MHz
      double h[2] = {double(me + 1), -double(me + 1)};
      double* d = nullptr;
      PE_HIP_CHECK(hipMalloc(&d, sizeof(h)));
      PE_HIP_CHECK(hipMemcpyAsync(d, h, sizeof(h), hipMemcpyHostToDevice, s));
      dev::launch_p2p_sum(d, 2, ps_, s);
      PE_HIP_CHECK(hipGetLastError());
      PE_HIP_CHECK(hipMemcpyAsync(h, d, sizeof(h), hipMemcpyDeviceToHost, s));
      PE_HIP_CHECK(hipStreamSynchronize(s));
      PE_HIP_CHECK(hipFree(d));
      const double want = 0.5 * double(P) * double(P + 1);
      bool good = h[0] == want && h[1] == -want;
      // PE_FAULT_INJECT=p2ptest@rank:R — rank R's check fails (fallback test)
      if (const char* e = std::getenv("PE_FAULT_INJECT"); e && std::string(e).rfind("p2ptest@rank:", 0) == 0 &&
                                                          std::atoi(e + 13) == me)
        good = false;
      ok = agree(good, s);
      if (!ok) why_ = good ? "self-test sum wrong on a peer" : "self-test sum wrong on this rank";
    }
    ps_.timeout_ticks = (long long)(timeout_s_ * 1e8);
    PE_HIP_CHECK(hipStreamDestroy(s));
    ok_ = ok;
  }
  ~P2PAllreduceComm() override {
    for (void* p : opened_) (void)hipIpcCloseMemHandle(p);
    if (peers_dev_) (void)hipFree(peers_dev_);
    if (seq_dev_) (void)hipFree(seq_dev_);
    if (mine_) (void)hipFree(mine_);
  }
  bool ok() const { return ok_; }
  const std::string& why() const { return why_; }
  std::unique_ptr<DeviceComm> release_base() { return std::move(base_); }

  int rank() const override { return base_->rank(); }
  int size() const override { return base_->size(); }
  void allreduce_sum(double* d, int n, hipStream_t s) override {
    if (n > dev::kP2PSlot - 1) {
      base_->allreduce_sum(d, n, s);
      return;
    }
    dev::launch_p2p_sum(d, n, ps_, s);
    PE_HIP_CHECK(hipGetLastError());
  }
  void allreduce_max(double* d, int n, hipStream_t s) override { base_->allreduce_max(d, n, s); }
  void exchange(const std::vector<Exchange>& ex, hipStream_t s) override { base_->exchange(ex, s); }
  void host_max(double* h, int n, hipStream_t s) override { base_->host_max(h, n, s); }
  void barrier(hipStream_t s) override { base_->barrier(s); }
  // the sequence counter lives on the device: replayable from a graph when
  // the base transport is
  bool capturable() const override { return base_->capturable(); }
  std::string name() const override { return "p2p-allreduce+" + base_->name(); }
  void check_async() override { base_->check_async(); }
  void abort() override { base_->abort(); }
  const dev::PeerSum* peer_sum() const override { return &ps_; }

  std::vector<void*> map_peer_buffers(void* mine) override {
    const int P = size(), me = rank();
    hipStream_t s = nullptr;
    PE_HIP_CHECK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    std::vector<void*> peers;
    bool ok = open_peers(mine, P, me, s, peers);
    ok = agree(ok, s);
    PE_HIP_CHECK(hipStreamDestroy(s));
    if (!ok) {
      unmap_peer_buffers(peers);
      return {};
    }
    return peers;
  }
  void unmap_peer_buffers(const std::vector<void*>& peers) override {
    for (size_t r = 0; r < peers.size(); ++r)
      if (int(r) != rank() && peers[r]) (void)hipIpcCloseMemHandle(peers[r]);
  }

 private:
  // All-gather the IPC handles of every rank's `mine` through the base
  // transport (byte b of rank r's handle at table[r*HB + b]: a max-allreduce
  // of a zero table; every rank takes part even after a local failure) and
  // open the peers'.  peers[r] = rank r's buffer in this process (peers[me] =
  // mine; null where not opened).  False on any local failure.
  bool open_peers(void* mine, int P, int me, hipStream_t s, std::vector<void*>& peers) {
    hipIpcMemHandle_t h{};
    bool ok = mine != nullptr && hipIpcGetMemHandle(&h, mine) == hipSuccess;
    if (!ok) (void)hipGetLastError();
    constexpr int HB = int(sizeof(hipIpcMemHandle_t));
    std::vector<double> tbl(size_t(P) * HB, 0.0);
    const unsigned char* hb = reinterpret_cast<const unsigned char*>(&h);
    for (int b = 0; b < HB; ++b) tbl[size_t(me) * HB + b] = hb[b];
    double* dt = nullptr;
    PE_HIP_CHECK(hipMalloc(&dt, sizeof(double) * tbl.size()));
    PE_HIP_CHECK(hipMemcpy(dt, tbl.data(), sizeof(double) * tbl.size(), hipMemcpyHostToDevice));
    base_->allreduce_max(dt, int(tbl.size()), s);
    PE_HIP_CHECK(hipStreamSynchronize(s));
    PE_HIP_CHECK(hipMemcpy(tbl.data(), dt, sizeof(double) * tbl.size(), hipMemcpyDeviceToHost));
    PE_HIP_CHECK(hipFree(dt));
    peers.assign(size_t(P), nullptr);
    for (int r = 0; r < P && ok; ++r) {
      if (r == me) {
        peers[r] = mine;
        continue;
      }
      hipIpcMemHandle_t hr;
      unsigned char* pb = reinterpret_cast<unsigned char*>(&hr);
      for (int b = 0; b < HB; ++b) pb[b] = static_cast<unsigned char>(tbl[size_t(r) * HB + b]);
      void* p = nullptr;
      if (hipIpcOpenMemHandle(&p, hr, hipIpcMemLazyEnablePeerAccess) != hipSuccess) {
        (void)hipGetLastError();
        std::fprintf(stderr, "[pe] rank %d: cannot map the P2P buffer of rank %d\n", me, r);
        ok = false;
        break;
      }
      peers[r] = p;
    }
    return ok;
  }

  // Map every peer's receive buffer; false on any local failure (no abort:
  // the ranks must still reach the agreement collective).
  bool setup(int P, int me, hipStream_t s) {
    const size_t bytes = sizeof(double) * 2 * size_t(P) * dev::kP2PSlot;
    if (hipExtMallocWithFlags(reinterpret_cast<void**>(&mine_), bytes, hipDeviceMallocFinegrained) != hipSuccess) {
      mine_ = nullptr;
      (void)hipGetLastError();
    }
    bool ok = mine_ != nullptr;
    if (ok) ok = hipMemset(mine_, 0, bytes) == hipSuccess && hipDeviceSynchronize() == hipSuccess;
    std::vector<void*> opened;
    ok = open_peers(ok ? mine_ : nullptr, P, me, s, opened);
    std::vector<double*> peers(size_t(P), nullptr);
    for (int r = 0; r < P; ++r) {
      peers[r] = static_cast<double*>(opened.empty() ? nullptr : opened[r]);
      if (r != me && peers[r]) opened_.push_back(peers[r]);
    }
    PE_HIP_CHECK(hipMalloc(&peers_dev_, sizeof(double*) * P));
    PE_HIP_CHECK(hipMemcpy(peers_dev_, peers.data(), sizeof(double*) * P, hipMemcpyHostToDevice));
    PE_HIP_CHECK(hipMalloc(&seq_dev_, sizeof(unsigned long long)));
    PE_HIP_CHECK(hipMemset(seq_dev_, 0, sizeof(unsigned long long)));
    PE_HIP_CHECK(hipDeviceSynchronize());  // before any stream uses the counter (non-blocking streams)
    ps_.peers = peers_dev_;
    ps_.seq = seq_dev_;
    ps_.me = me;
    ps_.P = P;
    return ok;
  }
  // true on every rank iff `ok` on every rank (max-allreduce of the failures)
  bool agree(bool ok, hipStream_t s) {
    double* d = nullptr;
    double h = ok ? 0.0 : 1.0;
    PE_HIP_CHECK(hipMalloc(&d, sizeof(double)));
    PE_HIP_CHECK(hipMemcpy(d, &h, sizeof(double), hipMemcpyHostToDevice));
    base_->allreduce_max(d, 1, s);
    PE_HIP_CHECK(hipStreamSynchronize(s));
    PE_HIP_CHECK(hipMemcpy(&h, d, sizeof(double), hipMemcpyDeviceToHost));
    PE_HIP_CHECK(hipFree(d));
    return h == 0.0;
  }

  std::unique_ptr<DeviceComm> base_;
  double* mine_ = nullptr;
  double** peers_dev_ = nullptr;
  unsigned long long* seq_dev_ = nullptr;
  std::vector<void*> opened_;
  dev::PeerSum ps_{};
  double timeout_s_ = 120.0;
  bool ok_ = false;
  std::string why_;
};

}  // namespace

std::unique_ptr<DeviceComm> make_p2p_allreduce_comm(std::unique_ptr<DeviceComm> base) {
  if (!base || base->size() == 1) return base;
  auto c = std::make_unique<P2PAllreduceComm>(std::move(base));
  if (c->ok()) {
    g_p2p_status = "ok";
    return c;
  }
  g_p2p_status = "fallback: " + c->why();
  std::fprintf(stderr, "[pe] rank %d: P2P allreduce unavailable on this job (%s), using %s\n", c->rank(),
               c->why().c_str(), c->name().c_str());
  return c->release_base();
}

const std::string& p2p_setup_status() { return g_p2p_status; }

}  // namespace pe
