// Host-visible interface of the gfx950 kernels (kernels.hip).  Plain C++ so
// the host runtime (compiled by g++) can launch them.
//
// Per-iteration device work (replaces the reference's 7 kernels K1-K7,
// poisson_mpi_cuda2.cu:507-676, and its host-side dot finalizers C16/C17):
//
//   F  (pcg_dir_stencil):  p_k = D⁻¹r_k + β_{k-1} p_{k-1}     (owned + halo ring)
//                          S_den += (A p_k)·p_k,  S_pp += p_k·p_k
//   G  (pcg_update):       α_k = (z,r)_{k-1} / den_k ; stop test on α²·S_pp
//                          w += α p_k ; r -= α A p_k (A p_k recomputed)
//                          S_zr += (D⁻¹r)·r ; strided halo strips → send buffers
//
// Both kernels march down i in column strips (wave64 lanes along contiguous
// j), keep the 3-row stencil window in registers + one LDS row, compute the
// fictitious-domain coefficients on the fly from two 1-D chord tables (no
// a/b/D arrays in HBM), and finish their dot products with a deterministic
// last-workgroup reduction into a device scalar.  Scalars (α, β, the
// convergence flag, the iteration count) never leave the device.
#pragma once

#include <hip/hip_runtime_api.h>

#include <cstdint>

namespace pe {
namespace dev {

// Device-resident solver state (one per rank).
struct DevState {
  double red_F[2];   // Σ(Ap·p), Σ(p·p) — local, then global after allreduce
  double red_G[2];   // Σ(z·r) — local, then global; [1] pad
  double err[4];     // Σ(w-u)² in D, max|w-u| in D, max|w| outside D, pad
  double rz_cur;     // (z, r) of the previous iteration, h-weighted
  double alpha, beta, last_diff;
  long long iter;    // completed iterations
  int done;          // 1 → every later kernel is a no-op
  int status;        // 0 running, 1 converged, 2 breakdown, 3 iteration cap, 4 non-finite scalars, 5 internal
  unsigned ticket[5];  // last-arriver tickets: [0] sweep / F, [1] reduction / G, [2] init, [3] error,
                       // [4] single-sweep terminal path (counts waves)
  unsigned pad[3];
  // Single-sweep (fused) PCG: the 7 local/global sums of sweep k live in
  // fs[k & 1] = {(r,z), (z,Az), (z,s), (p,s), (z,z), (z,p), (p,p)}, unweighted.
  double fs[2][8];
  double gprev;      // (r,z) consumed by the previous sweep (β denominator), h-weighted
  int started;       // 0 until sweep S_0 (z_0, A z_0 and their dots) has run
  int wpend;         // 1: α·p_k of the last (deferring) sweep not yet added to w
  int wpar;          // buffer x[wpar] holding that p_k
  int pad2;
  unsigned qhead[8][16];  // single-sweep work queue heads, one 64-B line per XCD shard
  unsigned long long sig;  // overlap: boundary items stored, cumulative over the solve's sweeps
  // In-sweep cross-rank sum (KParams::xr): s_memrealtime ticks (100 MHz) the
  // final block spent waiting for the peers' flags, summed over the solve's
  // sweeps, and the number of such waits — the T_MPI of the default
  // multi-rank path (the halo push's delivery is signalled by the same flags,
  // so its wait is inside this one).
  unsigned long long xr_wait;
  unsigned long long xr_n;
  // Multi-step sweeps: the unweighted sums of sweep k in fs2[k & 1] — 20
  // (two-step, layout: fused2.hip, sweep2_scalars) or 19 (three-step:
  // fused3.hip, sweep3_scalars).
  double fs2[2][32];
  // Three-step sweep (fused3.hip): the last sweep's coefficients {zc[3],
  // α[3], β[3], g[3]}; late3 of its iterations (ending at iter) still await
  // their stop tests (decided by the next launch from fs2[wpar]); brk3 > 0:
  // the iteration that breaks down after them (bad3: non-finite scalars).
  double sc3[16];
  long long brk3;
  int late3;
  int bad3;
  // End-of-solve true-residual check (kResid): unweighted sums over the
  // owned nodes {Σρ², Σr², Σ(ρ − r)², ΣB²} of ρ = B − A w (the returned w)
  // and r the recurrence's residual of the same iterate (three-step).
  double res[4];
  // Three-step restart (residual replacement): β of iteration k0 + 1 is 0.
  long long k0;
  // Three-step fix-up: the iterations of the last sweep it kept (0: the
  // solve ended on a sweep's last iteration — no fix-up).  The replay launch
  // (mlimit == kReplay3) then recomputes x[wpar] = (r, p) of that iterate,
  // so the end-of-solve residual check compares w with ITS r.
  int fixj;
  // Resident kernel: a workgroup's grid-barrier wait timed out (sticky: set
  // only by the aborting workgroups; the host falls back on it whatever the
  // other workgroups wrote after them)
  int res_abort;
};

// One-shot cross-rank sum over IPC-mapped receive buffers (peer_sum.hpp):
// peers[r] = rank r's buffer (2 × P slots of kP2PSlot doubles: n ≤ kP2PSlot-1
// values + a sequence flag) mapped into this process, seq = this rank's
// reduction counter (device), timeout in s_memrealtime ticks (100 MHz).
constexpr int kP2PSlot = 32;  // ≥ 19 sums of the three-step sweep + the flag
struct PeerSum {
  double* const* peers;
  unsigned long long* seq;
  int me, P;
  long long timeout_ticks;
  // non-null: the ticks spent waiting for the peers' flags are added here
  // (and one count at wait_acc[1]) — DevState::xr_wait of the solver
  unsigned long long* wait_acc;
};

// Halo exchange by peer put over xGMI (p2p.hip kPut; DeviceSolver's "put"
// halo path).  Every rank owns one fine-grained buffer, IPC-mapped into its
// neighbours: per direction d (as seen by the owner) kPutParts flags, then
// an inbox of 2 parities × `stride` doubles.  Message m (direction d) of one
// launch: block part b copies its 1/kPutParts of `src` into the peer's inbox
// slot for this rank (parity c & 1, c = the exchanges done towards d so far),
// releases it (system scope) with flag = c + 1, waits for this rank's own
// flag of that part (the peer's matching store), and copies the inbox part
// into `dst`.  One launch per halo phase, no host involvement, no RCCL call;
// a peer that never arrives poisons `dst` with NaN (the sweep then stops with
// a non-finite status) instead of hanging.
constexpr int kPutParts = 64;  // most blocks per message (PutArgs::parts); each waits only on its own part's flag
constexpr int kPutFlagStride = 16;  // u64 words per part flag (one 128-B line each)
constexpr int kPutBoxOff = 1;       // element i of a message at inbox slot[1 + i]: 16-B phase of the x rows (pitch even, column −7 first)
struct PutMsg {
  const double* src;                  // local send buffer
  double* rbox;                       // the peer's inbox slot for this message (parity 0)
  unsigned long long* rflag;          // the peer's flags of that slot (kPutParts × kPutFlagStride)
  const double* lbox;                 // this rank's inbox slot of direction dir (parity 0)
  const unsigned long long* lflag;    // this rank's flags of that slot
  double* dst;                        // local receive buffer
  long long n;                        // doubles
  int dir;
};
struct PutArgs {
  PutMsg m[4];
  int nmsg;
  long long stride;        // doubles between an inbox slot's two parities
  unsigned* cnt;           // [0..3] exchanges done per direction, [4..7] part tickets (device, local)
  int parts;               // blocks per message (≤ kPutParts; the same on every rank)
  long long timeout_ticks; // s_memrealtime ticks (100 MHz)
};
void launch_put(const PutArgs& a, hipStream_t s);
// Set-up self-test of the put path: rank-coded values through the same
// protocol (kPut with src = a device buffer of `code`), then *bad counts the
// received values differing from each peer's code (codes[m] = the peer of m).
void launch_put_check(const PutArgs& a, const double* codes, int* bad, hipStream_t s);

// Per-block launch description.  Local indexing: (li, lj), li ∈ [0, nx+1],
// lj ∈ [0, ny+1], element = base + li*pitch + lj.
struct KParams {
  int64_t nx, ny, pitch;
  int M, N;
  int64_t gi0, gj0;              // global index of local (0, 0)  (= i0-1, j0-1)
  double A1, A2, h1, h2, eps, inv_eps, h1sq, h2sq, nih1, nih2;
  double cx, cy, F, u_scale;
  double tol;
  int weighted;
  long long max_iter;
  int has[4];                    // neighbour present (LEFT, RIGHT, DOWN, UP)
  const double* colT;            // (nx+4) × 4: {halfA, sB, eB, x} at index li+1
  const double* rowT;            // (ny+4) × 4: {sA, eA, halfB, y} at index lj+1
  double* r;
  double* w;
  double* p[2];
  double* send_dn; double* send_up;        // y-direction (strided) send strips, nx each
  const double* recv_dn; const double* recv_up;
  const int* rowcls;             // (nx+4) × 4 ints at index q+1: {in_lo, in_hi, out_lo, out_hi}
  double* partial;               // ≥ 3 × blocks doubles
  DevState* st;
  int ti;                        // rows per work item (≤ 64)
  int nstrips;                   // 128-column wave strips across ny (+ halo column)
  int nitems;                    // nstrips × ceil(nx / ti)
  int nblocks;                   // persistent grid size of the marching kernels
  int nblocks0;                  // single-sweep: grid of the deferring (w-free) sweep
  int order;                     // item order: 0 chunk-major (compact active window), 1 strip-major,
                                 // 2 per-XCD chunk ranges, 3 per-XCD dynamic queue (single-sweep)
  int check_tol;                 // 0 → never stop on ‖Δw‖ (fixed-iteration runs)
  double D_in, D_out;            // exact-arithmetic diagonal in the interior / exterior class
  double dinv_in, dinv_out;      // fast-arithmetic 1/D in the interior / exterior class
  double ih1sq, ih2sq;           // 1/h1², 1/h2² (fast arithmetic)
  // Single-sweep layout (fused = 1): x[b] points at local (0,0) of the r-plane
  // of buffer b; its p-plane is at +poff; both planes share row stride
  // `pitch` (rows interleave r and p so the 2 halo rows of both fields are one
  // contiguous message).  w has its own row stride `wpitch`.
  int fused;
  int64_t wpitch;
  int64_t poff;
  double* x[2];
  double* itemsum;               // dynamic single-sweep: per-item sums [nslots][8]
  int nslots;                    // item-sum slots: list entries (listed walk) or nitems
  long long fault_iter;          // > 0: poison the reduced sums after this iteration (PE_FAULT_INJECT=nan@iter:K)
  long long fault_zero;          // > 0: zero the (p, A p) sums after this iteration → breakdown (zero@iter:K)
  double* hist;                  // keep_history: ‖Δw‖ of iteration k at hist[k-1] (k ≤ hist_n)
  long long hist_n;
  // Item lists (dynamic sweeps, setup_items): entries {first row, strip |
  // rows << 20}, split into lnsh shards; shard x owns ilist[lbase[x] ..
  // lbase[x+1]) and (halo/interior overlap) its first lnb[x] entries are
  // boundary items (outputs sent to a neighbour), each of which bumps st->sig
  // once its stores are visible.
  const int2* ilist;
  int lnsh;
  int lwaves;                    // static list layout: wave w walks positions w, w + lwaves, … (0: the grid's waves)
  int lbase[9];
  int lnb[8];
  // Diagnostic timeline (PE_STAMPS=1, single-sweep only; null otherwise;
  // a separate kernel build records it): per item {start, end, wave, block}
  // in s_memrealtime ticks (100 MHz), then per wave {entry, exit}.
  // Overwritten by every sweep.
  unsigned long long* stamps;
  unsigned long long* stamps2;   // per wave, 32 stamps along its FIRST item (start, prologue, row steps)
  // Cross-rank reduction inside the sweep (PE_XR, with a P2P comm): the final
  // reduction block sums the 7 sums over ranks itself (xr.peers == null: the
  // host enqueues the comm's allreduce instead).
  PeerSum xr;
  // In-sweep halo push over xGMI (row-slab blocks, P2P transport, k.xr set):
  // the sweep that writes buffer b also stores its owned rows 1, 2 into the
  // LEFT neighbour's receive buffer (hpush_lo[b]) and rows nx-1, nx into the
  // RIGHT neighbour's (hpush_hi[b]) with system-scope write-through stores;
  // the in-sweep cross-rank sum's flags then double as "halo delivered", and
  // the next sweep (PUSH) reads the halo rows of x[b] from this rank's receive
  // buffer hrecv itself (kHaloImport copies them into x only for checkpoints /
  // read-back; kHaloSeed fills hrecv from x after an exchange or a resume).
  // hrecv = [parity b][side: 0 rows -1,0 from
  // LEFT, 1 rows nx+1,nx+2 from RIGHT][2 × pitch], laid out like x rows from
  // column -1.  push = 0: the halo travels through the comm's exchange.
  double* hpush_lo[2];
  double* hpush_hi[2];
  const double* hrecv;
  int push;
  // PE_FAULT_INJECT=slow@rank:R,us:X — this rank's final reduction block
  // idles X µs (in ticks) before the cross-rank sum (T_MPI test hook)
  long long slow_ticks;
  // iterations per sweep: 1 single sweep (fused.hip kS), 2 two-step sweep
  // (fused2.hip kS2: 4-deep halo, 120-column strips, 20 sums), 3 three-step
  // sweep (fused3.hip kS3: 6-deep halo, 116-column strips, 19 sums)
  int steps;
  int hdep;  // halo depth of the single-sweep layouts: 2 (kS), 4 (kS2), 6 (kS3); rows per side of a push message
  int xorg;  // columns stored left of column 0: element 0 of an x / w row is column -xorg (hdep - 1; kS3: kHL3 - 1)
  // three-step sweep: > 0 → this launch applies at most mlimit iterations (a
  // run of n iterations ends with a partial sweep when 3 ∤ n)
  int mlimit;
  // three-step sweep: load each wave's first item at kernel entry (fused3.hip Pre3)
  int pre_load;
  // band items: 1/D from the LDS ring (1) or re-formed from the faces (0, PE_DRING=0)
  int dring;
  // three-step sweep, PE_PRIO (opt-in): > 0 → the two waves sharing a
  // SIMD take turns at issue priority (s_setprio), switching every
  // 2^prio × 10 ns; ncu: workgroups ≥ ncu are the second ones on their CU
  int prio;
  int ncu;
  // three-step sweep: stage each wave's first item's first rows into LDS at
  // kernel entry (fused3.hip stage_first3; PE_STAGE=0: off)
  int stage;
};
// KParams::mlimit of the three-step replay launch (DevState::fixj)
constexpr int kReplay3 = -2;

constexpr int kTJ = 256;         // threads per block (4 wave64s)
constexpr int kWPB = 4;          // waves per block
constexpr int kSW = 128;         // columns per wave strip (2 per lane, 16-B accesses)
constexpr int kTImax = 62;       // max rows per work item (rows ib-1..ie+1 live one per lane)
// Item-list entries {first row | band flag, strip | rows << 20}: kBandBit set
// when the item's rows ib-2 .. ie+2 contain a boundary-band row in its strip
// (general march); clear → the plain unrolled march.
constexpr int kBandBit = 1 << 30;
constexpr int kRowMask = kBandBit - 1;
// Three-step sweep only: kUniBit set when every row ib-6 .. ie+6 of the item
// lies wholly inside or wholly outside the interior in its strip's window
// (the kernel's uniform-row march: three scalars per row, no lane tests).
constexpr int kUniBit = 1 << 29;
constexpr int kRowMask3 = kUniBit - 1;
constexpr int kFSW = 124;        // fused sweep: output columns per wave strip (128 loaded, 2-column halo per side)
constexpr int kFSW2 = 120;       // two-step sweep: output columns per strip (4-column halo per side)
constexpr int kNS2 = 20;         // two-step sweep: sums per sweep
constexpr int kTImax2 = 48;      // two-step sweep: max rows per item (rows ib-4 .. ie+5 live one per lane)
constexpr int kFSW3 = 48;        // three-step sweep: output columns per 64-column strip (one per lane; 6-column halo needed per side)
constexpr int kHL3 = 8;          // three-step sweep: left halo lanes of a strip (right: 64 - kFSW3 - kHL3); with the
                                 // rows' element 0 at column -(kHL3 - 1), every strip's loads are whole 128-B lines
                                 // and its outputs whole 64-B segments
constexpr int kNS3 = 19;         // three-step sweep: sums per sweep
constexpr int kTImax3 = 512;     // three-step sweep: max rows per item (row windows reload every ~58 rows)

// LDS-resident single sweep (resident.hip): small single-rank blocks run many
// iterations in ONE launch.  The block is cut into tiles of one 124-column
// strip × R rows, one workgroup per tile (≤ one per CU, all co-resident);
// each keeps r, p (with a 2-deep ring) in LDS and w in registers, and per
// iteration exchanges only the second ring of r with its 8 neighbours and
// its 7 partial sums through global memory, behind one grid barrier.
constexpr int kResThreads = 512;   // 8 waves
constexpr int kResMaxRows = 64;    // R ≤ 64 rows per tile
constexpr int kResEdge = 376;      // edge record: rowT[124] rowB[124] colL[64] colR[64]
struct ResParams {
  int nstrips, ntr, nwg;             // tiles: nwg = ntr × nstrips, tile = (band tr, strip s), wg = tr·nstrips + s
  int rcap, nbcap;                   // LDS sizing: max tile rows, band-coefficient slots
  const int* rowstart;               // ntr+1: first local row of band tr (rowstart[ntr] = nx + 1)
  double* edges;                     // [2][nwg][kResEdge]
  double* partials;                  // [2][nwg][8]
  unsigned* ctr;                     // [8][32] barrier counters (zeroed before every launch);
                                     // ctr[16]: workgroups past their entry state reads
  int niter;                         // iterations of this launch
  int par0;                          // parity of its first iteration
  long long timeout_ticks;           // barrier wait limit (s_memrealtime ticks, 100 MHz)
  unsigned lds_bytes;
  // PE_RES_STAMPS=1 diagnostic: s_memrealtime of every workgroup at 8 points
  // of its first kResStampIters iterations, [nwg][kResStampIters][8] (null: off)
  unsigned long long* stamps;
  // PE_FAULT_INJECT=resbarrier: this workgroup never arrives at the first
  // grid barrier (-1: none) — the barrier times out, the launch aborts with
  // status 5 and the solver must fall back to the streaming sweep.
  // fault_late (PE_FAULT_INJECT=reslate): that workgroup arrives after the
  // others have timed out instead, passes the barrier and writes its tile back
  int fault_wg;
  int fault_late;
};
constexpr int kResStampIters = 64;
constexpr int kResMaxTiles = 256;  // the per-iteration sum gather reads ≤ 4 × 64 tile partials
size_t resident_lds_bytes(int rcap, int nbcap);
// Launch n iterations (the caller zeroes rp.ctr on the same stream first).
void launch_resident(const KParams& k, const ResParams& rp, hipStream_t s);
int resident_max_blocks_per_cu(size_t lds_bytes);

void launch_init(const KParams& k, int init_random, unsigned long long seed, double amp, int variant,
                 hipStream_t s);
void launch_F(const KParams& k, int par, int variant, hipStream_t s);
void launch_G(const KParams& k, int par, int variant, hipStream_t s);
void launch_error(const KParams& k, hipStream_t s);
// True residual ρ = B − A w (w from the p-plane of x[bw], halo exchanged; r
// from x[st->wpar] when with_r) → st->res; store: ρ → x[bw]'s r-plane.
void launch_resid(const KParams& k, int bw, bool with_r, bool store, hipStream_t s);
void launch_w_to_p(const KParams& k, int b, hipStream_t s);   // owned w → the p-plane of x[b]
void launch_zero_p(const KParams& k, int b, hipStream_t s);   // the p-plane of x[b] ← 0 (halos included)
void launch_restart3(const KParams& k, hipStream_t s);        // three-step restart state (kRestart3)
void launch_poke_w(const KParams& k, int64_t li, int64_t lj, double v, hipStream_t s);  // fault hook
// 4-byte-word copy by a kernel (bytes % 4 == 0); either side may be pinned
// host memory (to_host: system-scope fence after the stores).
void launch_copy_words(void* dst, const void* src, size_t bytes, bool to_host, hipStream_t s);
// Single-sweep PCG (fused.hip): one kernel + one 7-scalar reduction per iteration.
void launch_S(const KParams& k, int par, hipStream_t s, bool with_red = true);  // with_red: + launch_red (dynamic order)
// Deterministic reduction of per-item sums + state update (dynamic / listed sweeps).
void launch_red(const KParams& k, int par, hipStream_t s);
// y-direction halo strips of buffer b: pack columns {1,2} / {ny-1,ny} of r,p
// into send_dn / send_up ([nx][4]); unpack recv_dn / recv_up into columns
// {-1,0} / {ny+1,ny+2}.
void launch_pack(const KParams& k, int b, hipStream_t s);
// Add a pending deferred w term (no-op when none is pending).
void launch_wflush(const KParams& k, hipStream_t s);
void launch_unpack(const KParams& k, int b, hipStream_t s);
// In-sweep halo push: copy the receive buffer's rows of parity b (filled by
// the neighbours' sweeps, delivered once the sweep's cross-rank sum has
// completed) into x[b]'s halo rows -1, 0 / nx+1, nx+2.  The sweeps read them
// from the buffer directly; this makes x[b] whole for checkpoints / read-back.
void launch_halo_import(const KParams& k, int b, hipStream_t s);
void launch_halo_seed(const KParams& k, int b, hipStream_t s);  // receive buffer b <- x[b]'s halo rows
// Halo-push set-up self-test: write rank-coded values into the neighbours'
// receive buffers (k.hpush_*), then — after a cross-rank barrier — count in
// *bad the received values (k.hrecv) that differ from the neighbours' codes
// (left / right: neighbour ranks, -1 where none).
void launch_push_test_write(const KParams& k, int me, hipStream_t s);
void launch_push_test_check(const KParams& k, int left, int right, int* bad, hipStream_t s);
// Overlap: spin until st->sig reaches `target` (every boundary item of the
// running sweep is in L2) or the solve is done, then write every XCD's L2
// back.  Put on the halo stream ahead of the exchange.
void launch_wait_sig(const KParams& k, unsigned long long target, hipStream_t s);
// One-shot P2P allreduce kernel (p2p.hip) of n ≤ kP2PSlot-1 doubles, in place.  P ≤ 64.
void launch_p2p_sum(double* d, int n, const PeerSum& ps, hipStream_t s);
// Group-comm helper: out[i] = Σ_r in_r[i] (or max), written to every rank's buffer.
void launch_group_reduce(double* const* bufs, int nranks, int n, int is_max, hipStream_t s);
// Debug/test ops (single-shot, no convergence logic).
void launch_apply_A(const KParams& k, const double* p, double* Ap, hipStream_t s);
void launch_coef(const KParams& k, double* a, double* b, double* D, hipStream_t s);
// Single-sweep (division-free) coefficients of every node incl. the ring, dense (nx+2) × (ny+2).
void launch_coef_fast(const KParams& k, double* a, double* b, double* dinv, hipStream_t s);
int grid_blocks(const KParams& k);
void launch_delay(double us, hipStream_t s);  // test transport: stream-ordered busy wait
// Resident 256-thread blocks per CU of the marching kernels (occupancy API;
// 0 when unavailable).  Sizes the persistent grids.
int resident_blocks_S(const KParams& k, int wm);  // wm 0: deferring sweep, 2: applying sweep
// Two-step sweep (fused2.hip): one launch = iterations K+1 and K+2 (static
// item list only; launch_S dispatches here when k.steps == 2).
void launch_S2(const KParams& k, int par, hipStream_t s);
int resident_blocks_S2();
// Three-step sweep (fused3.hip): one launch = the previous launch's pending
// stop tests (and, when it converged early, its w fix-up), then iterations
// K+1..K+3 (or fewer: k.mlimit > 0, breakdown, cap; none: k.mlimit < 0);
// launch_S dispatches here when k.steps == 3.
void launch_S3(const KParams& k, int par, hipStream_t s);
int resident_blocks_S3();
constexpr int sweep_sums(int steps) { return steps >= 3 ? kNS3 : steps == 2 ? kNS2 : 7; }
// (k.ti / k.order select the kernel variant: set them first)
int resident_blocks_classic(int variant);

}  // namespace dev
}  // namespace pe
