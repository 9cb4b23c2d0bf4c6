// RCCL transport over xGMI (one process per GPU).
//
// Replaces the reference's MPI layer for the GPU stage
// (poisson_mpi_cuda2.cu:331-500 halo: D2H → serial blocking MPI_Sendrecv
// chain → H2D; :842/:871/:892/:925 8-byte host MPI_Allreduce after a
// device sync).  Here:
//   * halo  = one ncclGroupStart/End with every neighbour's ncclSend/ncclRecv
//             posted together, straight from/to device memory (no host
//             staging, no serial chain),
//   * dots  = in-place ncclAllReduce on device scalars, stream-ordered, so
//             the solver never waits on the host inside the iteration loop.
// Small messages on xGMI are latency-bound: the solver fuses
// the reference's 3 scalar allreduces per iteration into 2.
#include <hip/hip_runtime_api.h>
#include <rccl/rccl.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <stdexcept>
#include <vector>

#include "../hip/kernels.hpp"
#include "pe/device.hpp"

#define PE_NCCL_CHECK(expr)                                                                             \
  do {                                                                                                  \
    ncclResult_t _r = (expr);                                                                           \
    if (_r != ncclSuccess) {                                                                            \
      std::fprintf(stderr, "[pe] RCCL error %d (%s) at %s:%d in `%s`\n", int(_r), ncclGetErrorString(_r), \
                   __FILE__, __LINE__, #expr);                                                          \
      std::fflush(stderr);                                                                              \
      std::abort();                                                                                     \
    }                                                                                                   \
  } while (0)

namespace pe {
namespace {

class RcclComm final : public DeviceComm {
 public:
  RcclComm(ncclComm_t c, bool owned) : comm_(c), owned_(owned) {
    PE_NCCL_CHECK(ncclCommUserRank(comm_, &rank_));
    PE_NCCL_CHECK(ncclCommCount(comm_, &size_));
    PE_HIP_CHECK(hipMalloc(&scratch_, 64 * sizeof(double)));
  }
  ~RcclComm() override {
    if (scratch_) (void)hipFree(scratch_);
    if (owned_ && comm_) ncclCommDestroy(comm_);
  }
  int rank() const override { return rank_; }
  int size() const override { return size_; }
  void allreduce_sum(double* d, int n, hipStream_t s) override {
    if (size_ == 1) return;
    PE_NCCL_CHECK(ncclAllReduce(d, d, size_t(n), ncclDouble, ncclSum, comm_, s));
  }
  void allreduce_max(double* d, int n, hipStream_t s) override {
    if (size_ == 1) return;
    PE_NCCL_CHECK(ncclAllReduce(d, d, size_t(n), ncclDouble, ncclMax, comm_, s));
  }
  void exchange(const std::vector<Exchange>& ex, hipStream_t s) override {
    if (ex.empty()) return;
    PE_NCCL_CHECK(ncclGroupStart());
    for (const auto& e : ex) {
      PE_NCCL_CHECK(ncclSend(e.send, size_t(e.count), ncclDouble, e.peer, comm_, s));
      PE_NCCL_CHECK(ncclRecv(e.recv, size_t(e.count), ncclDouble, e.peer, comm_, s));
    }
    PE_NCCL_CHECK(ncclGroupEnd());
  }
  void host_max(double* h, int n, hipStream_t s) override {
    if (size_ == 1) return;
    if (n > 64) throw std::invalid_argument("host_max: too many values");
    PE_HIP_CHECK(hipMemcpyAsync(scratch_, h, sizeof(double) * n, hipMemcpyHostToDevice, s));
    PE_NCCL_CHECK(ncclAllReduce(scratch_, scratch_, size_t(n), ncclDouble, ncclMax, comm_, s));
    PE_HIP_CHECK(hipMemcpyAsync(h, scratch_, sizeof(double) * n, hipMemcpyDeviceToHost, s));
    PE_HIP_CHECK(hipStreamSynchronize(s));
  }
  void barrier(hipStream_t s) override {
    if (size_ == 1) return;
    PE_NCCL_CHECK(ncclAllReduce(scratch_, scratch_, 1, ncclDouble, ncclSum, comm_, s));
    PE_HIP_CHECK(hipStreamSynchronize(s));
  }
  // RCCL calls are not captured into the iteration graphs (the put / push
  // paths with in-sweep sums replay from graphs without a comm call)
  bool capturable() const override { return false; }
  std::string name() const override { return "rccl"; }
  void check_async() override {
    if (!comm_) return;
    ncclResult_t r = ncclSuccess;
    if (ncclCommGetAsyncError(comm_, &r) != ncclSuccess || (r != ncclSuccess && r != ncclInProgress)) {
      const std::string msg = std::string("RCCL asynchronous error: ") + ncclGetErrorString(r);
      abort();
      throw std::runtime_error(msg);
    }
  }
  void abort() override {
    if (comm_) (void)ncclCommAbort(comm_);
    comm_ = nullptr;
  }

 private:
  ncclComm_t comm_;
  bool owned_;
  int rank_ = 0, size_ = 1;
  double* scratch_ = nullptr;
};

// Timing-only test transport: every exchange / allreduce is a stream-ordered
// busy wait of a fixed duration (no data moves).  Lets one GPU measure how
// much of a given communication latency the halo/interior overlap hides.
// loopback: the exchange also moves data, asynchronously — after the wait,
// each message's send buffer is copied into its own receive buffer by a
// stream-ordered device-to-device copy (a rank that is its own neighbour on
// every side).  Nothing synchronises the host, as with RCCL, so a run with the
// halo/interior overlap must end bitwise where the serial one does: any
// ordering hole (pack before the boundary items' stores, next sweep before
// the unpack) shows up as different data.
class DelayComm final : public DeviceComm {
 public:
  DelayComm(int size, double exchange_us, double allreduce_us, bool loopback)
      : size_(size), ex_us_(exchange_us), ar_us_(allreduce_us), loop_(loopback) {}
  int rank() const override { return 0; }
  int size() const override { return size_; }
  // (a zero delay launches nothing: one rank's block then runs its sweeps back
  // to back, as with the in-sweep push and P2P sums — the per-rank block
  // probes used to pay 2-3 µs of empty delay launches per sweep)
  void allreduce_sum(double*, int, hipStream_t s) override {
    if (ar_us_ > 0) dev::launch_delay(ar_us_, s);
  }
  void allreduce_max(double*, int, hipStream_t s) override {
    if (ar_us_ > 0) dev::launch_delay(ar_us_, s);
  }
  void exchange(const std::vector<Exchange>& ex, hipStream_t s) override {
    if (ex.empty()) return;
    if (ex_us_ > 0) dev::launch_delay(ex_us_, s);
    if (loop_)
      for (const Exchange& e : ex)
        if (e.count > 0 && e.send && e.recv && e.send != e.recv)
          PE_HIP_CHECK(hipMemcpyAsync(e.recv, e.send, sizeof(double) * size_t(e.count), hipMemcpyDeviceToDevice, s));
  }
  void host_max(double*, int, hipStream_t) override {}
  void barrier(hipStream_t) override {}
  bool capturable() const override { return true; }
  std::string name() const override { return "delay"; }

 private:
  int size_;
  double ex_us_, ar_us_;
  bool loop_;
};

class HostStagedComm final : public DeviceComm {
 public:
  HostStagedComm(int rank, int size, CallbackHostComm::ReduceFn r, CallbackHostComm::ExchangeFn e,
                 CallbackHostComm::BarrierFn b)
      : host_(rank, size, std::move(r), std::move(e), std::move(b)) {}
  int rank() const override { return host_.rank(); }
  int size() const override { return host_.size(); }
  void allreduce_sum(double* d, int n, hipStream_t s) override { reduce(d, n, s, false); }
  void allreduce_max(double* d, int n, hipStream_t s) override { reduce(d, n, s, true); }
  void exchange(const std::vector<Exchange>& ex, hipStream_t s) override {
    if (ex.empty()) return;
    PE_HIP_CHECK(hipStreamSynchronize(s));
    std::vector<std::vector<double>> snd(ex.size()), rcv(ex.size());
    std::vector<Exchange> hx;
    for (size_t k = 0; k < ex.size(); ++k) {
      snd[k].resize(size_t(ex[k].count));
      rcv[k].resize(size_t(ex[k].count));
      PE_HIP_CHECK(hipMemcpy(snd[k].data(), ex[k].send, sizeof(double) * ex[k].count, hipMemcpyDeviceToHost));
      hx.push_back(Exchange{ex[k].dir, ex[k].peer, snd[k].data(), rcv[k].data(), ex[k].count});
    }
    host_.exchange(hx);
    for (size_t k = 0; k < ex.size(); ++k)
      PE_HIP_CHECK(hipMemcpy(ex[k].recv, rcv[k].data(), sizeof(double) * ex[k].count, hipMemcpyHostToDevice));
  }
  void host_max(double* h, int n, hipStream_t s) override {
    PE_HIP_CHECK(hipStreamSynchronize(s));
    host_.allreduce_max(h, n);
  }
  void barrier(hipStream_t s) override {
    PE_HIP_CHECK(hipStreamSynchronize(s));
    host_.barrier();
  }
  std::string name() const override { return "host-staged"; }

 private:
  void reduce(double* d, int n, hipStream_t s, bool is_max) {
    std::vector<double> h(static_cast<size_t>(n));
    PE_HIP_CHECK(hipStreamSynchronize(s));
    PE_HIP_CHECK(hipMemcpy(h.data(), d, sizeof(double) * n, hipMemcpyDeviceToHost));
    if (is_max) host_.allreduce_max(h.data(), n);
    else host_.allreduce_sum(h.data(), n);
    PE_HIP_CHECK(hipMemcpy(d, h.data(), sizeof(double) * n, hipMemcpyHostToDevice));
  }
  CallbackHostComm host_;
};

}  // namespace

std::unique_ptr<DeviceComm> make_delay_comm(int size, double exchange_us, double allreduce_us, bool loopback) {
  return std::make_unique<DelayComm>(size, exchange_us, allreduce_us, loopback);
}

std::unique_ptr<DeviceComm> make_callback_device_comm(int rank, int size, CallbackHostComm::ReduceFn reduce,
                                                      CallbackHostComm::ExchangeFn exch,
                                                      CallbackHostComm::BarrierFn barrier) {
  return std::make_unique<HostStagedComm>(rank, size, std::move(reduce), std::move(exch), std::move(barrier));
}

std::string rccl_unique_id() {
  ncclUniqueId id;
  PE_NCCL_CHECK(ncclGetUniqueId(&id));
  return std::string(id.internal, sizeof(id.internal));
}

std::unique_ptr<DeviceComm> make_rccl_comm(const std::string& uid, int rank, int size) {
  if (uid.size() != sizeof(ncclUniqueId::internal))
    throw std::invalid_argument("rccl unique id must be " + std::to_string(sizeof(ncclUniqueId::internal)) + " bytes");
  ncclUniqueId id;
  std::memcpy(id.internal, uid.data(), uid.size());
  ncclComm_t c;
  PE_NCCL_CHECK(ncclCommInitRank(&c, size, id, rank));
  return std::make_unique<RcclComm>(c, true);
}

std::unique_ptr<DeviceComm> make_rccl_comm_from_handle(void* handle) {
  return std::make_unique<RcclComm>(reinterpret_cast<ncclComm_t>(handle), false);
}

}  // namespace pe
