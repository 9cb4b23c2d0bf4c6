// Communication interfaces.
//
// The reference uses MPI for (a) the 4-neighbour halo exchange of p
// (stage2-mpi/poisson_mpi_decomp.cpp:241-347, stage4 host-staged Sendrecv
// chain poisson_mpi_cuda2.cu:331-500) and (b) 8-byte MPI_Allreduce(SUM)
// global inner products (:396,:412,:435,:439).  Here the solver talks to an
// abstract transport; the halo *plan* (which strip goes to which neighbour)
// is shared by every transport, only the bytes-moving part differs:
//
//   HostComm   — host memory (CPU backends): SelfHostComm, ThreadHostComm
//                (ranks = threads of one process, MPI-free stage2/3 runs),
//                and a callback transport bound from Python
//                (torch.distributed gloo process groups).
//   DeviceComm — device memory, stream-ordered (GPU backend): RCCL over
//                xGMI (rccl_comm.cpp) and the self transport.
#pragma once

#include <cstdint>
#include <functional>
#include <memory>
#include <vector>

#include "pe/decomp.hpp"

namespace pe {

// One neighbour exchange: send `count` doubles from `send` to `peer`,
// receive `count` doubles from `peer` into `recv`.  Buffers are contiguous.
struct Exchange {
  int dir;    // Dir of the neighbour, as seen from this rank
  int peer;   // neighbour rank
  const double* send;
  double* recv;
  int64_t count;
};

class HostComm {
 public:
  virtual ~HostComm() = default;
  virtual int rank() const = 0;
  virtual int size() const = 0;
  // In-place global sum; every rank receives bitwise-identical values.
  virtual void allreduce_sum(double* buf, int n) = 0;
  virtual void allreduce_max(double* buf, int n) = 0;
  // All exchanges of one halo update, posted together (no serial chain,
  // unlike the reference's Sendrecv chain — quirk A8).
  virtual void exchange(const std::vector<Exchange>& ex) = 0;
  virtual void barrier() = 0;
};

class SelfHostComm final : public HostComm {
 public:
  int rank() const override { return 0; }
  int size() const override { return 1; }
  void allreduce_sum(double*, int) override {}
  void allreduce_max(double*, int) override {}
  void exchange(const std::vector<Exchange>&) override {}
  void barrier() override {}
};

// Transport implemented by callbacks (bound from Python: torch.distributed).
class CallbackHostComm final : public HostComm {
 public:
  using ReduceFn = std::function<void(double*, int, bool /*is_max*/)>;
  using ExchangeFn = std::function<void(const std::vector<Exchange>&)>;
  using BarrierFn = std::function<void()>;
  CallbackHostComm(int rank, int size, ReduceFn r, ExchangeFn e, BarrierFn b)
      : rank_(rank), size_(size), reduce_(std::move(r)), exch_(std::move(e)), bar_(std::move(b)) {}
  int rank() const override { return rank_; }
  int size() const override { return size_; }
  void allreduce_sum(double* buf, int n) override { reduce_(buf, n, false); }
  void allreduce_max(double* buf, int n) override { reduce_(buf, n, true); }
  void exchange(const std::vector<Exchange>& ex) override { exch_(ex); }
  void barrier() override { bar_(); }

 private:
  int rank_, size_;
  ReduceFn reduce_;
  ExchangeFn exch_;
  BarrierFn bar_;
};

// Shared state for P thread-ranks in one process (see thread_comm.cpp).
struct ThreadGroup;
std::shared_ptr<ThreadGroup> make_thread_group(int size);
std::unique_ptr<HostComm> make_thread_comm(std::shared_ptr<ThreadGroup> g, int rank);

}  // namespace pe
