// P2P allreduce transport: a DeviceComm that keeps its base transport (RCCL,
// or host-staged for tests) for the halo exchange and everything else, but
// runs the per-iteration sum of a few doubles as one kernel writing into
// IPC-mapped receive buffers of every peer (p2p.hip).  Opt-in
// (PE_ALLREDUCE=p2p): the latency it removes is RCCL's small-message ring.
#include <hip/hip_runtime_api.h>

#include <cstdlib>
#include <cstring>
#include <stdexcept>
#include <string>
#include <vector>

#include "../hip/kernels.hpp"
#include "pe/device.hpp"

namespace pe {
namespace {

class P2PAllreduceComm final : public DeviceComm {
 public:
  explicit P2PAllreduceComm(std::unique_ptr<DeviceComm> base) : base_(std::move(base)) {
    const int P = base_->size(), me = base_->rank();
    if (P > 64) throw std::invalid_argument("p2p allreduce: at most 64 ranks");
    if (const char* e = std::getenv("PE_P2P_TIMEOUT_S")) timeout_s_ = std::atof(e);
    const size_t bytes = sizeof(double) * 2 * size_t(P) * dev::kP2PSlot;
    PE_HIP_CHECK(hipExtMallocWithFlags(reinterpret_cast<void**>(&mine_), bytes, hipDeviceMallocFinegrained));
    PE_HIP_CHECK(hipMemset(mine_, 0, bytes));
    PE_HIP_CHECK(hipDeviceSynchronize());
    hipIpcMemHandle_t h;
    PE_HIP_CHECK(hipIpcGetMemHandle(&h, mine_));
    // all-gather the handles through the base transport: byte b of rank r's
    // handle at table[r*HB + b] (a max-allreduce of a zero table)
    constexpr int HB = int(sizeof(hipIpcMemHandle_t));
    std::vector<double> tbl(size_t(P) * HB, 0.0);
    const unsigned char* hb = reinterpret_cast<const unsigned char*>(&h);
    for (int b = 0; b < HB; ++b) tbl[size_t(me) * HB + b] = hb[b];
    double* dt = nullptr;
    hipStream_t s = nullptr;
    PE_HIP_CHECK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    PE_HIP_CHECK(hipMalloc(&dt, sizeof(double) * tbl.size()));
    PE_HIP_CHECK(hipMemcpy(dt, tbl.data(), sizeof(double) * tbl.size(), hipMemcpyHostToDevice));
    base_->allreduce_max(dt, int(tbl.size()), s);
    PE_HIP_CHECK(hipStreamSynchronize(s));
    PE_HIP_CHECK(hipMemcpy(tbl.data(), dt, sizeof(double) * tbl.size(), hipMemcpyDeviceToHost));
    PE_HIP_CHECK(hipFree(dt));
    PE_HIP_CHECK(hipStreamDestroy(s));
    std::vector<double*> peers(size_t(P), nullptr);
    for (int r = 0; r < P; ++r) {
      if (r == me) {
        peers[r] = mine_;
        continue;
      }
      hipIpcMemHandle_t hr;
      unsigned char* pb = reinterpret_cast<unsigned char*>(&hr);
      for (int b = 0; b < HB; ++b) pb[b] = static_cast<unsigned char>(tbl[size_t(r) * HB + b]);
      void* p = nullptr;
      PE_HIP_CHECK(hipIpcOpenMemHandle(&p, hr, hipIpcMemLazyEnablePeerAccess));
      peers[r] = static_cast<double*>(p);
      opened_.push_back(p);
    }
    PE_HIP_CHECK(hipMalloc(&peers_dev_, sizeof(double*) * P));
    PE_HIP_CHECK(hipMemcpy(peers_dev_, peers.data(), sizeof(double*) * P, hipMemcpyHostToDevice));
  }
  ~P2PAllreduceComm() override {
    for (void* p : opened_) (void)hipIpcCloseMemHandle(p);
    if (peers_dev_) (void)hipFree(peers_dev_);
    if (mine_) (void)hipFree(mine_);
  }
  int rank() const override { return base_->rank(); }
  int size() const override { return base_->size(); }
  void allreduce_sum(double* d, int n, hipStream_t s) override {
    if (n > dev::kP2PSlot - 1) {
      base_->allreduce_sum(d, n, s);
      return;
    }
    dev::launch_p2p_sum(d, n, peers_dev_, base_->rank(), base_->size(), ++seq_, timeout_s_, s);
    PE_HIP_CHECK(hipGetLastError());
  }
  void allreduce_max(double* d, int n, hipStream_t s) override { base_->allreduce_max(d, n, s); }
  void exchange(const std::vector<Exchange>& ex, hipStream_t s) override { base_->exchange(ex, s); }
  void host_max(double* h, int n, hipStream_t s) override { base_->host_max(h, n, s); }
  void barrier(hipStream_t s) override { base_->barrier(s); }
  // the sequence number is a launch argument: not replayable from a graph
  bool capturable() const override { return false; }
  std::string name() const override { return "p2p-allreduce+" + base_->name(); }
  void check_async() override { base_->check_async(); }
  void abort() override { base_->abort(); }

 private:
  std::unique_ptr<DeviceComm> base_;
  double* mine_ = nullptr;
  double** peers_dev_ = nullptr;
  std::vector<void*> opened_;
  unsigned long long seq_ = 0;
  double timeout_s_ = 120.0;
};

}  // namespace

std::unique_ptr<DeviceComm> make_p2p_allreduce_comm(std::unique_ptr<DeviceComm> base) {
  if (!base || base->size() == 1) return base;
  return std::make_unique<P2PAllreduceComm>(std::move(base));
}

}  // namespace pe
