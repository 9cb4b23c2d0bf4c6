// ThreadHostComm: P ranks as threads of one process, sharing mailboxes.
// This is the MPI-free replacement for the reference's stage2/stage3
// multi-process runs (there is no MPI on the build or GPU boxes): the same
// decomposition, halo plan and reduction order, with shared memory as the
// transport.  Reductions sum rank contributions in rank order, so every rank
// gets bitwise-identical scalars (deterministic, like a fixed-tree allreduce).
#include <algorithm>
#include <condition_variable>
#include <mutex>
#include <stdexcept>

#include "pe/comm.hpp"

namespace pe {

struct ThreadGroup {
  explicit ThreadGroup(int n) : size(n), slots(n), mail(n * 4) {}
  int size;
  std::mutex mu;
  std::condition_variable cv;
  int arrived = 0;
  uint64_t generation = 0;
  std::vector<std::vector<double>> slots;  // per-rank reduction contributions
  std::vector<std::vector<double>> mail;   // [rank*4 + dir] outgoing strip

  void barrier() {
    std::unique_lock<std::mutex> lk(mu);
    const uint64_t gen = generation;
    if (++arrived == size) {
      arrived = 0;
      ++generation;
      cv.notify_all();
    } else {
      cv.wait(lk, [&] { return generation != gen; });
    }
  }
};

std::shared_ptr<ThreadGroup> make_thread_group(int size) {
  if (size < 1) throw std::invalid_argument("thread group size must be >= 1");
  return std::make_shared<ThreadGroup>(size);
}

namespace {

class ThreadHostComm final : public HostComm {
 public:
  ThreadHostComm(std::shared_ptr<ThreadGroup> g, int rank) : g_(std::move(g)), rank_(rank) {}
  int rank() const override { return rank_; }
  int size() const override { return g_->size; }

  void allreduce_sum(double* buf, int n) override { reduce(buf, n, false); }
  void allreduce_max(double* buf, int n) override { reduce(buf, n, true); }

  void exchange(const std::vector<Exchange>& ex) override {
    for (const auto& e : ex) {
      auto& box = g_->mail[rank_ * 4 + e.dir];
      box.assign(e.send, e.send + e.count);
    }
    g_->barrier();
    for (const auto& e : ex) {
      const auto& box = g_->mail[e.peer * 4 + opposite(e.dir)];
      if (int64_t(box.size()) != e.count)
        throw std::runtime_error("ThreadHostComm: halo size mismatch");
      std::copy(box.begin(), box.end(), e.recv);
    }
    g_->barrier();
  }

  void barrier() override { g_->barrier(); }

 private:
  void reduce(double* buf, int n, bool is_max) {
    g_->slots[rank_].assign(buf, buf + n);
    g_->barrier();
    for (int k = 0; k < n; ++k) {
      double acc = g_->slots[0][k];
      for (int r = 1; r < g_->size; ++r)
        acc = is_max ? std::max(acc, g_->slots[r][k]) : acc + g_->slots[r][k];
      buf[k] = acc;
    }
    g_->barrier();
  }

  std::shared_ptr<ThreadGroup> g_;
  int rank_;
};

}  // namespace

std::unique_ptr<HostComm> make_thread_comm(std::shared_ptr<ThreadGroup> g, int rank) {
  if (rank < 0 || rank >= g->size) throw std::invalid_argument("thread comm rank out of range");
  return std::make_unique<ThreadHostComm>(std::move(g), rank);
}

}  // namespace pe
