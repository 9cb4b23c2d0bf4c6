// Checkpoint / resume of a device solve (DeviceSolver::save_checkpoint /
// load_checkpoint).
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

using detail::Range;
using dev::DevState;
using dev::KParams;

// ---------------------------------------------------------------------------
// Checkpoint / resume.  File = header + DevState + field buffers + halo
// buffers, raw bytes; the header pins everything the byte layout depends on.
// ---------------------------------------------------------------------------
namespace {
struct CkptHeader {
  char magic[8];
  int32_t version, M, N, rank, Px, Py, fused, variant, par;
  int64_t i0, j0, nx, ny, state_bytes, field_bytes, halo_bytes;
};
void ck_io(FILE* f, void* host, size_t n, bool write, const std::string& path) {
  const size_t got = write ? std::fwrite(host, 1, n, f) : std::fread(host, 1, n, f);
  if (got != n) throw std::runtime_error("checkpoint " + path + ": short " + (write ? "write" : "read"));
}
}  // namespace

void DeviceSolver::save_checkpoint(const std::string& path) {
  Range range("pe.checkpoint");
  import_halos();  // whole x planes (the halo push keeps halo rows in the receive buffers)
  PE_HIP_CHECK(hipStreamSynchronize(stream_));
  std::vector<std::pair<void*, size_t>> bufs;
  if (fused_) {
    bufs = {{fields_, sizeof(double) * xsize_}, {xalt_, sizeof(double) * xsize_}, {walt_, sizeof(double) * wsize_}};
  } else {
    bufs = {{fields_, sizeof(double) * 4 * blk_.alloc}};
  }
  size_t field_bytes = 0;
  for (auto& b : bufs) field_bytes += b.second;
  CkptHeader h{};
  std::memcpy(h.magic, "PECKPT1", 8);
  h.version = 1;
  h.M = prob_.M;
  h.N = prob_.N;
  h.rank = blk_.rank;
  h.Px = blk_.Px;
  h.Py = blk_.Py;
  h.fused = sstep_ ? steps_ : fused_ ? 1 : 0;  // 2 / 3: two- / three-step layout (4- / 6-deep halo)
  h.variant = opt_.variant;
  h.par = par_;
  h.i0 = blk_.i0;
  h.j0 = blk_.j0;
  h.nx = blk_.nx;
  h.ny = blk_.ny;
  h.state_bytes = sizeof(DevState);
  h.field_bytes = int64_t(field_bytes);
  h.halo_bytes = int64_t(sizeof(double) * hsize_ * 4);
  const std::string tmp = path + ".tmp";
  FILE* f = std::fopen(tmp.c_str(), "wb");
  if (!f) throw std::runtime_error("checkpoint: cannot open " + tmp);
  std::vector<char> host(size_t(64) << 20);
  auto dump = [&](const void* dev, size_t n) {
    for (size_t o = 0; o < n; o += host.size()) {
      const size_t m = std::min(host.size(), n - o);
      PE_HIP_CHECK(hipMemcpy(host.data(), static_cast<const char*>(dev) + o, m, hipMemcpyDeviceToHost));
      ck_io(f, host.data(), m, true, path);
    }
  };
  ck_io(f, &h, sizeof(h), true, path);
  dump(st_, sizeof(DevState));
  for (auto& b : bufs) dump(b.first, b.second);
  dump(halo_, size_t(h.halo_bytes));
  std::fclose(f);
  if (std::rename(tmp.c_str(), path.c_str()) != 0) throw std::runtime_error("checkpoint: cannot rename " + tmp);
}

void DeviceSolver::load_checkpoint(const std::string& path) {
  PE_HIP_CHECK(hipStreamSynchronize(stream_));
  FILE* f = std::fopen(path.c_str(), "rb");
  if (!f) throw std::runtime_error("resume: cannot open " + path);
  CkptHeader h{};
  ck_io(f, &h, sizeof(h), false, path);
  size_t field_bytes = fused_ ? sizeof(double) * (2 * xsize_ + wsize_) : sizeof(double) * 4 * blk_.alloc;
  const bool ok = std::memcmp(h.magic, "PECKPT1", 8) == 0 && h.version == 1 && h.M == prob_.M && h.N == prob_.N &&
                  h.rank == blk_.rank && h.Px == blk_.Px && h.Py == blk_.Py && h.fused == (sstep_ ? steps_ : fused_ ? 1 : 0) &&
                  h.variant == opt_.variant && h.i0 == blk_.i0 && h.j0 == blk_.j0 && h.nx == blk_.nx &&
                  h.ny == blk_.ny && h.state_bytes == int64_t(sizeof(DevState)) &&
                  h.field_bytes == int64_t(field_bytes) && h.halo_bytes == int64_t(sizeof(double) * hsize_ * 4);
  const int mine = sstep_ ? steps_ : fused_ ? 1 : 0;
  if (!ok && std::memcmp(h.magic, "PECKPT1", 8) == 0 && h.fused != mine) {
    // the usual mismatch: a checkpoint of another sweep layout (e.g. one
    // written before the default became the three-step sweep)
    static const char* algo[4] = {"classic", "fused", "two-step", "three-step"};
    auto name = [](int v) -> std::string { return v >= 0 && v < 4 ? algo[v] : "unknown (steps=" + std::to_string(v) + ")"; };
    const int hf = int(h.fused);
    std::fclose(f);
    throw std::runtime_error("resume: " + path + " has the " + name(hf) + " layout (steps=" + std::to_string(hf) +
                             "), this solver runs " + name(mine) + " (steps=" + std::to_string(mine) + "); pass --algo " +
                             name(hf));
  }
  if (!ok) {
    std::fclose(f);
    throw std::runtime_error("resume: " + path + " does not match this problem / block / algorithm");
  }
  std::vector<char> host(size_t(64) << 20);
  auto load = [&](void* dev, size_t n) {
    for (size_t o = 0; o < n; o += host.size()) {
      const size_t m = std::min(host.size(), n - o);
      ck_io(f, host.data(), m, false, path);
      PE_HIP_CHECK(hipMemcpy(static_cast<char*>(dev) + o, host.data(), m, hipMemcpyHostToDevice));
    }
  };
  load(st_, sizeof(DevState));
  if (fused_) {
    load(fields_, sizeof(double) * xsize_);
    load(xalt_, sizeof(double) * xsize_);
    load(walt_, sizeof(double) * wsize_);
  } else {
    load(fields_, sizeof(double) * 4 * blk_.alloc);
  }
  load(halo_, size_t(h.halo_bytes));
  std::fclose(f);
  par_ = h.par;
  PE_HIP_CHECK(hipMemsetAsync(&st_->sig, 0, sizeof(st_->sig), stream_));  // overlap targets restart
  // halo push: the next sweep (parity par_) reads x[par_ ^ 1]'s halo rows
  // from the receive buffer
  if (push_ && fused_) dev::launch_halo_seed(*kp_, par_ ^ 1, stream_);
  ov_epoch_ = 0;
}

}  // namespace pe
