// dse_runtime.hip -- host runtime behind the C ABI of include/dse.h.
//
// Replaces qt.sesolve (dipolar_ensemble_with_rare.py:653-666) for many independent evolutions
// per device.  Per output interval [t_m, t_{m+1}] every problem runs
//     k = 1 (MODE_FIRST), k = 2..K_p (MODE_GEN), observables of the new state
// on one of several HIP streams ("lanes").  Problems are independent, so lanes never
// synchronise with each other until observable partials are copied back; the GPU overlaps
// the tail of one lane's launch with the next launches of the others.  Within a lane,
// items (problem, tile) are sorted by Chebyshev degree so the items still active at term k are
// a prefix of the lane's item list.
//
// HBM layout per problem: three 2^n double2 state buffers B0, B1, B2.  In interval m (parity q):
//   psi = B[q ? 2 : 0], acc = B[q ? 0 : 2], scratch = B1;  w_j lives in (j odd ? scratch : psi)
// and MODE_GEN overwrites w_{k-2} in place with w_k.  At the end of the interval acc holds
// psi(t_{m+1}) and becomes psi of the next interval.
#include <algorithm>
#include <chrono>
#include <cmath>
#include <complex>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <numeric>
#include <string>
#include <atomic>
#include <condition_variable>
#include <functional>
#include <memory>
#include <mutex>
#include <thread>
#include <deque>
#include <vector>

#include <unistd.h>

#include <rccl/rccl.h>
#include <rocblas/rocblas.h>
#include <rocsolver/rocsolver.h>

#include "../../include/dse.h"
#include "dse_internal.h"
#include "dse_dense.h"
#include "dse_small.h"
#include "dse_wht.h"

using namespace dse;

namespace {

struct HostProblem {
  int n = 0;
  std::vector<double> field, zz, pair, flip;
  double shift = 0.0;
  uint64_t psi0 = 0, sea_mask = 0;
  int rare_bit = -1;
  double rare_z = 0.0;
  double e_min = 0.0, e_max = 0.0;
  // device state
  int L = 0;
  int64_t n_tiles = 0;
  double2* buf[3] = {nullptr, nullptr, nullptr};
  void* tables = nullptr;
  double2* coef = nullptr;   // into dse_ctx::d_coef (compact rows, coef_row)
  int degree = 1;
  double flops_per_amp = 0.0;  // algorithmic flops of one H application per amplitude
  int2* d_items = nullptr;  // this problem's tiles (apply_h / observables hooks)
  // partitioned register (dse_add_problem_sharded): shard `shard_rank` of 2^shard_bits
  int shard_bits = 0, shard_rank = 0;
  int n_local = 0;           // qubits held by this shard (n - shard_bits)
  int group_first = -1;      // loopback group: index of shard 0 (all shards in this context)
  bool dist = false;         // shard of a register partitioned over processes (RCCL exchange)
  uint32_t xmasks = 0;       // bit m set: terms or observables read shard rank ^ m
  double2* rbuf_own[kMaxShards] = {};  // dist: receive buffers of the exchange, per mask
  bool imag = false;         // every drive coefficient purely imaginary (drive phase pi/2)
  // Walsh-Hadamard engine (dse_wht.hip): X- and Y-branch vectors and the pair matrix
  double2* wvec[4] = {nullptr, nullptr, nullptr, nullptr};  // A, B (+ index-swapped A, B)
  double* d_cquad = nullptr;
  double* d_wtab = nullptr;  // ztab | xytab
  int wht_groups = 0;        // passes' tile-bit groups; 0: this problem uses the step kernels
  // small-register engine (dse_small.hip): n <= 9 qubits, whole evolution one wave per problem
  bool sm = false;           // this evolve runs the problem on that engine
  // dense eigen-propagator engine (dse_dense.hip): this evolve diagonalises the register instead
  bool dn = false;
  // propagator-matrix mode (matrix_run): the context's single register, U = exp(-iH dt) built
  // column by column, the outputs by repeated products
  bool mx = false;
  bool side() const { return sm || dn || mx; }  // not on the per-interval Chebyshev launches
  double2* sm_coef = nullptr;  // into dse_ctx::d_sm_coef
  int* sm_deg = nullptr;
  int final_bsel = 0;        // buffer holding the final state after dse_evolve
  // spanning register (dse_span.hip): this evolve runs the register over 2^span_s workgroups of
  // 2^(n - span_s) amplitudes (0: not spanned)
  int span_s = 0;
  // real-component mode (dse_real.hip): this evolve runs the register as two real recurrences
  bool rl = false;
};

// One stream's share of the problems, grouped by tile size.
struct LaneGroup {
  int L = 0;
  int tiles = 1;            // tiles per problem (persistent mode: 1 or 2)
  int wht_groups = 0;       // > 0: every problem of the group runs on the Walsh-Hadamard engine
  std::vector<std::pair<int, int>> wht_regs;  // partitioned registers: (first shard, degree)
  int64_t off = 0;          // first position in the global item array
  int64_t count = 0;        // items of this group
  std::vector<int> active;     // active[k] = items with degree >= k (prefix of the group)
  std::vector<double> bytes;   // bytes[k] = algorithmic HBM bytes of the term-k launch
  std::vector<double> flops;   // flops[k] = algorithmic flops of the term-k launch
  // spanning registers (tiles < 0): k_span<span_L, span_rb> over span_count launch items from
  // span_off in dse_ctx::d_span_items (tiles of one register 8 apart, padding items x = -1)
  int span_L = 0, span_rb = 0;
  int64_t span_off = 0, span_count = 0;
  // launch boundaries inside those items (relative to span_off, last = span_count): whole blocks of
  // 8 registers, each launch at most what the chip holds at once (every register's tiles resident
  // together: its hand-offs wait on each other)
  std::vector<int64_t> span_cuts;
  std::vector<double> span_am, span_fl;  // per launch: amplitudes x terms, algorithmic flops
  // real-component registers: k_real over real_count items (problem, component) from real_off in
  // dse_ctx::d_real_items, then k_real_combine over real_np items (problem, 0) from real_poff
  bool real = false;
  int64_t real_off = 0, real_count = 0, real_poff = 0, real_np = 0;
};
struct Lane {
  hipStream_t stream = nullptr;
  // persistent mode, option obs_overlap: the observables of interval group g run on obs_stream
  // behind ev_iv[g & 1] (its interval launches), and interval group g + 2, which rewrites the
  // buffers they read, waits for ev_obs[g & 1]
  hipStream_t obs_stream = nullptr;
  hipEvent_t ev_iv[2] = {nullptr, nullptr}, ev_obs[2] = {nullptr, nullptr};
  bool obs_pending[2] = {false, false};
  std::vector<LaneGroup> groups;
  std::vector<hipEvent_t> ev[2];
  size_t ev_used[2] = {0, 0};
  int max_deg = 0;
};

}  // namespace

// internal return code of evolve_impl: a persistent hand-off timed out (dse_evolve falls back)
constexpr int kRcHandoffTimeout = 1000;

struct dse_ctx {
  int device = 0;
  std::string err;
  std::vector<HostProblem> probs;
  DevProb* d_probs = nullptr;
  std::vector<DevProb> h_desc;
  std::vector<Lane> lanes;
  int2* d_items = nullptr;          // all items, lane-major, degree-sorted inside each group
  int2* d_items_iv = nullptr;       // the same, 2-tile groups reordered for the interval kernel
  std::vector<int64_t> item_pos;    // first item position of every problem (evolve layout)
  int64_t total_items = 0;
  double* d_partial = nullptr;
  size_t partial_slots = 0;
  std::map<std::vector<double>, double*> zzlo_tables;  // identical in-tile ZZ tables are shared
  bool prepared = false;
  bool evolved = false;
  int last_q = 0;
  int tile_bits = 13;
  int n_streams = 4;
  int persistent = 1;               // use k_interval when every problem fits <= 2 tiles
  int wht = 1;                      // Walsh-Hadamard engine for registers of more tiles
  int wht_group_bits = 0;           // high bits per pass of that engine (0: tile bits - 2)
  int wht_tile_bits = 0;            // its tile: 12, 13 (0 = 13)
  int wht_persist = 0;              // bit 1: MID as a persistent launch (k_wht_mid_p), option wht_persist
  int wht_contiguous = 0;           // option wht_contiguous: hipDeviceMallocContiguous X/Y vectors
  int wht_fuse = 1;                 // option wht_fuse: FINAL of term k runs term k + 1's FIRST
  int wht_mid_inpage = 0;           // option wht_mid_inpage: in-page high bits of the MID group
  int wht_half = 7;                 // option wht_half: half-LDS passes (k_wht_h), bit 0 FIRST, 1 FWD/INV, 2 MID
  WhtProb* d_wht = nullptr;         // per problem (zero entries: not on that engine)
  bool wht_ready = false;
  int xcd_pairs = 1;                // diagnostics: 0 keeps the two tiles of a problem adjacent
  int mixed_launch = 1;             // persistent: 1- and 2-tile problems of one tile size in one launch
  int span_partial = 1;             // option span_partial: the auto span policy's partial form
  int span_chunks = 2;              // option span_chunks: resident launches the auto policy allows (0-2)
  int span_partial_tile = 11;       // option span_partial_tile: the partial form's tile (10, 11)
  int obs_overlap = 0;              // persistent: observables off the interval launches' stream
  int n_cu = 256;                   // compute units of the device
  int coresident = 0;               // diagnostics: workgroups per 2-tile interval chunk (0: occupancy)
  int handoff_fallbacks = 0;        // this evolve call re-ran on the streaming kernels after a hand-off timeout (0/1)
  bool rerun = false;               // that re-run: the dense engine's results of the first pass are kept
  int* d_err_cur = nullptr;         // the hand-off error word of the running persistent evolve (else null)
  double* d_allreduce = nullptr;    // RCCL all-reduce staging buffer of the observable sums (grow-only)
  size_t allreduce_cap = 0;         // in doubles
  int* d_flags = nullptr;           // hand-off flags (2 tiles x kIvWaves per problem) + error word
  size_t flags_cap = 0;
  double2* d_xslots = nullptr;      // hand-off slots of the interval kernel
  size_t xslot_cap = 0;             // in amplitudes
  double2* d_xacc = nullptr;        // intermediate outputs of multi-output launches
  size_t xacc_cap = 0;              // in amplitudes
  // per-evolve uploads, one device arena each (one copy per evolve, not one per problem)
  unsigned char* d_coef = nullptr;  // Chebyshev coefficient rows of every problem
  size_t coef_cap = 0;
  unsigned char* d_sm_coef = nullptr;  // small-engine coefficients and degrees
  size_t sm_coef_cap = 0;
  BasisInit* d_init = nullptr;      // psi(t0) list
  size_t init_cap = 0;
  int outputs_per_launch = 2;       // M of the interval kernel (dse_evolve picks 1 on coarse grids)
  int span_outputs = 4;             // M when every register spans (k_span, staggered sums)
  int64_t probe_items = 0;          // 0: all items
  int time_every = 1;               // 0: no kernel timing; N: time intervals with m % N == 0
  double max_degree = 2e6;
  // partitioned registers over processes: one RCCL communicator, one rank per GPU
  ncclComm_t comm = nullptr;
  int dist_rank = 0, dist_world = 1;
  // or a host transport (dse_dist_init_exchange): device data staged through host buffers
  dse_exchange_fn xfn = nullptr;
  void* xuser = nullptr;
  std::vector<unsigned char> xsend, xrecv;
  double xbytes = 0.0;              // bytes this rank sent to other ranks (current evolve)
  // exchange timing (current evolve): HIP event pairs around RCCL calls (summed at the end of
  // dse_evolve) plus host wall time of host-transport exchanges
  std::vector<hipEvent_t> xev;
  size_t xev_used = 0;
  double xms = 0.0;
  // small-register engine
  int dbg = 0;                      // diagnostics switches (option "dbg")
  int small = 1;                    // registers of <= 9 qubits run on dse_small.hip
  int small_chunk = 64;             // output intervals per launch of that engine
  hipStream_t small_stream = nullptr;
  // partitioned registers on the Walsh-Hadamard engine: the index swaps run on swap_stream, one
  // vector's swap under the other vector's pass (option "swap_overlap"); swap_ev orders the two
  int swap_overlap = 1;
  hipStream_t swap_stream = nullptr;
  hipEvent_t swap_ev[8] = {};
  SmallProb* d_small = nullptr;
  size_t small_cap = 0;             // descriptors allocated
  double* d_small_out = nullptr;    // [problem][n_t][8] raw observable sums
  size_t small_out_cap = 0;
  int* d_small_aux = nullptr;       // problem selections per register size, interval -> set map
  size_t small_aux_cap = 0;
  // dense eigen-propagator engine (dse_dense.h): option "dense" 0 off, 1 when cheaper than the
  // Chebyshev propagator by the cost model of dense_cheaper (default), 2 for every eligible register
  int dense = 1;
  // propagator-matrix mode for a context holding one register on a uniform grid: 0 off, 1 when
  // the model of matrix_cheaper says so (default), 2 whenever eligible
  int matrix = 1;
  // matrix mode's device buffers (U, the states, the products' partial sums, tables), kept across
  // evolves of the same register size (simulate_rare calls one register at a time; a 2^12 register
  // holds 256 MiB of U) and released by dse_destroy or when a larger register needs more
  unsigned char* d_mx = nullptr;
  size_t mx_cap = 0;
  // option "symv_fused": each product's reduction inside the product's launch (agent-scope counters
  // with a release per workgroup): measured 22.9 vs 10.4 ms for config 2, so off by default
  int symv_fused = 0;
  double mx_build_ms = 0.0, mx_products_ms = 0.0, mx_products = 0.0, mx_bytes_per_product = 0.0;  // last matrix_run

  // spanning registers (dse_span.hip): option "span" 0 off; s = 1..4: every register that fits
  // runs over 2^s workgroups (one per CU) of 2^(n - s) amplitudes; "span_rb": amplitudes per
  // thread 2^span_rb (0: 512 threads per workgroup)
  int span = 0;
  int span_tile = -1;               // option "span_tile": L > 0 every register of n > L qubits spans 2^(n-L)
                                    // tiles; -1 (default) auto: L = 11 when all tiles fit the chip at once
  // real-component mode (dse_real.hip, option "real", default 0): registers of 13 or 14 qubits with
  // imaginary drives run as two real recurrences, one workgroup per component, no hand-off
  int real_mode = 0;
  unsigned char* d_real = nullptr;  // [a | b] inputs and propagator sums of the real-mode registers
  size_t real_cap = 0;
  unsigned char* d_real_tab = nullptr;
  size_t real_tab_cap = 0;
  int2* d_real_items = nullptr;
  size_t real_items_cap = 0;
  int span_rb = 0;
  SpanDesc* d_span = nullptr;       // per problem
  size_t span_cap = 0;
  unsigned char* d_span_tab = nullptr;
  size_t span_tab_cap = 0;
  double2* d_span_slots = nullptr;  // hand-off slots of the spanned registers
  size_t span_slot_cap = 0;         // in amplitudes
  int* d_span_flags = nullptr;
  size_t span_flag_cap = 0;
  int2* d_span_items = nullptr;
  size_t span_items_cap = 0;

  hipStream_t dense_stream = nullptr;
  rocblas_handle blas = nullptr;
  // dense engine: registers of >= 2^10 amplitudes are diagonalised up to eig_streams at a time (one
  // host thread, stream and rocBLAS handle each; option "eig_streams", default 3: one N = 14 point
  // of the 30 s grid (two 2^14 registers through the two-stage solver, one 2^13) 4.54 / 4.00 / 3.75 /
  // 3.87 s with 1 / 2 / 3 / 4 streams, profiles/r04/eig_streams_point_2stage.jsonl)
  int eig_streams = 3;
  // dense engine eigensolver: 0 rocSOLVER dsyevd at every size; 1 eig_sym_lower (dse_sytrd.hip: the
  // half-matrix tridiagonalisation from 2^13, rocSOLVER dstedc, the blocked back-transformation)
  // from kEigHalfMinDim amplitudes, dsyevd below; 2 eig_sym_lower from 2^10 (tests)
  int eig_impl = 1;
  // the two-stage eigensolver's cross-workgroup polls give up after this many rounds (option
  // eig_spin_limit; < 0: at once, tests); a give-up re-solves that register with dsyevd
  int eig_spin = kEig2DefaultSpin;
  HandoffKnobs hk;  // options spin_limit, handoff_fences: every persistent launch of this context
  std::atomic<int> eig_fallbacks{0};  // registers re-solved that way in the last evolve
  // dense engine: eigenvalues refined by double-double Rayleigh quotients and output phases reduced
  // in double-double (option "dense_refine", default 1; 0: the eigensolver's eigenvalues and fp64
  // phases, whose error grows like eps |lambda| t: ~1e-8 at the reference grid's 30 s)
  int dense_refine = 1;
  // dense engine: output times of registers of >= kNufftMinDim amplitudes by a type-1 non-uniform
  // FFT on uniform grids (option "dense_nufft": 1 default, from kNufftMinOutputs outputs; 2 every
  // register from two outputs (tests); 0 the [cos | -sin] GEMM for every output), dse_nufft.hip;
  // its rocFFT plans
  int dense_nufft = 1;
  NufftCache* nufft = nullptr;
  int nufft_problems = 0;     // last evolve: registers whose outputs came from the transform
  double dense_out_ms = 0.0;  // last evolve: host wall time of the dense engine's output stage
  std::vector<hipStream_t> eig_st;
  std::vector<rocblas_handle> eig_h;
};

namespace {

thread_local std::string g_create_err;

int fail(dse_ctx* c, int code, const std::string& msg) {
  if (c) c->err = msg;
  return code;
}

#define HIPC(expr)                                                                      \
  do {                                                                                  \
    hipError_t _e = (expr);                                                             \
    if (_e != hipSuccess)                                                               \
      return fail(ctx, DSE_ERR_HIP, std::string(#expr) + ": " + hipGetErrorString(_e)); \
  } while (0)

size_t align_up(size_t v, size_t a) { return (v + a - 1) / a * a; }

// Host worker threads kept for the process (created on first use, never joined: they only wait
// on a condition variable between jobs), so a dse_evolve does not pay ~16 thread creations per
// parallel section.  One job at a time; a caller that finds the pool busy (another context on
// another host thread) runs its job on threads of its own instead.
class HostPool {
 public:
  static HostPool& get() {
    static HostPool* p = new HostPool();  // intentionally never destroyed (detached workers)
    return *p;
  }
  size_t size() const { return workers_; }
  // body(w) for w < nb, on the pool and the calling thread; false if the pool was busy
  bool run(size_t nb, const std::function<void(size_t)>& body) {
    if (getpid() != pid_) return false;  // a forked child has none of the workers
    std::unique_lock<std::mutex> busy(busy_, std::try_to_lock);
    if (!busy.owns_lock()) return false;
    {
      std::lock_guard<std::mutex> lk(m_);
      job_ = &body;
      nb_ = nb;
      next_.store(0);
      active_ = workers_;
      ++gen_;
    }
    cv_.notify_all();
    drain();
    std::unique_lock<std::mutex> lk(m_);
    done_.wait(lk, [&] { return active_ == 0; });
    job_ = nullptr;
    return true;
  }

 private:
  HostPool() : workers_(std::min<size_t>(15, std::max(1u, std::thread::hardware_concurrency()) - 1)), pid_(getpid()) {
    for (size_t w = 0; w < workers_; ++w) std::thread([this] { loop(); }).detach();
  }
  void drain() {
    for (size_t b = next_++; b < nb_; b = next_++) (*job_)(b);
  }
  void loop() {
    uint64_t seen = 0;
    for (;;) {
      {
        std::unique_lock<std::mutex> lk(m_);
        cv_.wait(lk, [&] { return gen_ != seen; });
        seen = gen_;
      }
      drain();
      std::lock_guard<std::mutex> lk(m_);
      if (--active_ == 0) done_.notify_all();
    }
  }
  const size_t workers_;
  const pid_t pid_;
  std::mutex busy_, m_;
  std::condition_variable cv_, done_;
  const std::function<void(size_t)>* job_ = nullptr;
  size_t nb_ = 0, active_ = 0;
  uint64_t gen_ = 0;
  std::atomic<size_t> next_{0};
};

// f(i) for i < n on up to 16 host threads (contiguous blocks; f must touch only item i's data).
template <class F>
void parallel_for(size_t n, F&& f) {
  const size_t nth = std::min<size_t>({(size_t)std::max(1u, std::thread::hardware_concurrency()), 16, (n + 7) / 8});
  if (nth <= 1) {
    for (size_t i = 0; i < n; ++i) f(i);
    return;
  }
  const std::function<void(size_t)> block = [&](size_t w) {
    for (size_t i = n * w / nth; i < n * (w + 1) / nth; ++i) f(i);
  };
  if (HostPool::get().run(nth, block)) return;
  std::vector<std::thread> th;
  th.reserve(nth);
  for (size_t w = 0; w < nth; ++w) th.emplace_back(block, w);
  for (auto& x : th) x.join();
}

// Host bytes gathered for one upload: pieces 64-B aligned, offsets into the device arena.
struct Arena {
  std::vector<unsigned char> host;
  size_t add(const void* src, size_t bytes) {
    const size_t off = place(bytes);
    if (bytes) std::memcpy(host.data() + off, src, bytes);
    return off;
  }
  size_t place(size_t bytes) {  // room for a piece filled later
    const size_t off = align_up(host.size(), 64);
    host.resize(off + bytes);
    return off;
  }
};

// The arena's device copy: grows *dev to fit, then one copy on stream st (stream-ordered before
// every later launch on st; the caller synchronises st before other streams use it).
int upload_arena(dse_ctx* ctx, const Arena& a, unsigned char** dev, size_t* cap, hipStream_t st) {
  if (a.host.empty()) return DSE_OK;
  if (a.host.size() > *cap) {
    if (*dev) (void)hipFree(*dev), *dev = nullptr;
    *cap = 0;
    if (hipMalloc(dev, a.host.size()) != hipSuccess)
      return fail(ctx, DSE_ERR_OOM, "coefficient allocation failed (" + std::to_string(a.host.size()) + " bytes)");
    *cap = a.host.size();
  }
  HIPC(hipMemcpyAsync(*dev, a.host.data(), a.host.size(), hipMemcpyHostToDevice, st));
  HIPC(hipStreamSynchronize(st));  // the host bytes may be released after return
  return DSE_OK;
}

void free_wht(HostProblem& p) {
  for (auto& b : p.wvec)
    if (b) (void)hipFree(b), b = nullptr;
  if (p.d_cquad) (void)hipFree(p.d_cquad), p.d_cquad = nullptr;
  if (p.d_wtab) (void)hipFree(p.d_wtab), p.d_wtab = nullptr;
  p.wht_groups = 0;
}

void free_device(dse_ctx* ctx) {
  for (auto& p : ctx->probs) {
    for (auto& b : p.buf)
      if (b) (void)hipFree(b), b = nullptr;
    if (p.tables) (void)hipFree(p.tables), p.tables = nullptr;
    p.coef = nullptr;
    if (p.d_items) (void)hipFree(p.d_items), p.d_items = nullptr;
    for (auto& b : p.rbuf_own)
      if (b) (void)hipFree(b), b = nullptr;
    p.sm_coef = nullptr;
    p.sm_deg = nullptr;
    free_wht(p);
  }
  if (ctx->d_wht) (void)hipFree(ctx->d_wht), ctx->d_wht = nullptr;
  ctx->wht_ready = false;
  if (ctx->d_probs) (void)hipFree(ctx->d_probs), ctx->d_probs = nullptr;
  if (ctx->d_items) (void)hipFree(ctx->d_items), ctx->d_items = nullptr;
  if (ctx->d_items_iv) (void)hipFree(ctx->d_items_iv), ctx->d_items_iv = nullptr;
  if (ctx->d_partial) (void)hipFree(ctx->d_partial), ctx->d_partial = nullptr;
  for (auto& kv : ctx->zzlo_tables) (void)hipFree(kv.second);
  if (ctx->d_flags) (void)hipFree(ctx->d_flags), ctx->d_flags = nullptr;
  ctx->flags_cap = 0;
  if (ctx->d_xslots) (void)hipFree(ctx->d_xslots), ctx->d_xslots = nullptr;
  ctx->xslot_cap = 0;
  if (ctx->d_xacc) (void)hipFree(ctx->d_xacc), ctx->d_xacc = nullptr;
  ctx->xacc_cap = 0;
  if (ctx->d_span) (void)hipFree(ctx->d_span), ctx->d_span = nullptr;
  if (ctx->d_real) (void)hipFree(ctx->d_real), ctx->d_real = nullptr;
  if (ctx->d_real_tab) (void)hipFree(ctx->d_real_tab), ctx->d_real_tab = nullptr;
  if (ctx->d_real_items) (void)hipFree(ctx->d_real_items), ctx->d_real_items = nullptr;
  ctx->real_cap = ctx->real_tab_cap = ctx->real_items_cap = 0;
  if (ctx->d_span_tab) (void)hipFree(ctx->d_span_tab), ctx->d_span_tab = nullptr;
  if (ctx->d_span_slots) (void)hipFree(ctx->d_span_slots), ctx->d_span_slots = nullptr;
  if (ctx->d_span_flags) (void)hipFree(ctx->d_span_flags), ctx->d_span_flags = nullptr;
  if (ctx->d_span_items) (void)hipFree(ctx->d_span_items), ctx->d_span_items = nullptr;
  ctx->span_cap = ctx->span_tab_cap = ctx->span_slot_cap = ctx->span_flag_cap = ctx->span_items_cap = 0;
  if (ctx->d_coef) (void)hipFree(ctx->d_coef), ctx->d_coef = nullptr;
  if (ctx->d_sm_coef) (void)hipFree(ctx->d_sm_coef), ctx->d_sm_coef = nullptr;
  if (ctx->d_init) (void)hipFree(ctx->d_init), ctx->d_init = nullptr;
  ctx->coef_cap = ctx->sm_coef_cap = ctx->init_cap = 0;
  if (ctx->d_small) (void)hipFree(ctx->d_small), ctx->d_small = nullptr;
  if (ctx->d_small_out) (void)hipFree(ctx->d_small_out), ctx->d_small_out = nullptr;
  if (ctx->d_small_aux) (void)hipFree(ctx->d_small_aux), ctx->d_small_aux = nullptr;
  ctx->small_cap = ctx->small_out_cap = ctx->small_aux_cap = 0;
  if (ctx->d_allreduce) (void)hipFree(ctx->d_allreduce), ctx->d_allreduce = nullptr;
  ctx->allreduce_cap = 0;
  ctx->zzlo_tables.clear();
  ctx->partial_slots = 0;
  ctx->total_items = 0;
  ctx->prepared = false;
  ctx->evolved = false;
}

void destroy_lanes(dse_ctx* ctx) {
  if (ctx->swap_stream) {
    (void)hipStreamSynchronize(ctx->swap_stream);
    for (auto& e : ctx->swap_ev)
      if (e) (void)hipEventDestroy(e), e = nullptr;
    (void)hipStreamDestroy(ctx->swap_stream);
    ctx->swap_stream = nullptr;
  }
  if (ctx->small_stream) {
    (void)hipStreamSynchronize(ctx->small_stream);
    (void)hipStreamDestroy(ctx->small_stream);
    ctx->small_stream = nullptr;
  }
  if (ctx->blas) (void)rocblas_destroy_handle(ctx->blas), ctx->blas = nullptr;
  for (auto& h : ctx->eig_h) (void)rocblas_destroy_handle(h);
  ctx->eig_h.clear();
  for (auto& e : ctx->eig_st) (void)hipStreamSynchronize(e), (void)hipStreamDestroy(e);
  ctx->eig_st.clear();
  for (auto e : ctx->xev) (void)hipEventDestroy(e);
  ctx->xev.clear();
  ctx->xev_used = 0;
  if (ctx->dense_stream) {
    (void)hipStreamSynchronize(ctx->dense_stream);
    (void)hipStreamDestroy(ctx->dense_stream);
    ctx->dense_stream = nullptr;
  }
  nufft_release(ctx->nufft);
  ctx->nufft = nullptr;
  for (auto& ln : ctx->lanes) {
    if (ln.stream) (void)hipStreamSynchronize(ln.stream);
    if (ln.obs_stream) (void)hipStreamSynchronize(ln.obs_stream);
    for (auto& pool : ln.ev)
      for (auto e : pool) (void)hipEventDestroy(e);
    for (int i = 0; i < 2; ++i) {
      if (ln.ev_iv[i]) (void)hipEventDestroy(ln.ev_iv[i]);
      if (ln.ev_obs[i]) (void)hipEventDestroy(ln.ev_obs[i]);
    }
    if (ln.obs_stream) (void)hipStreamDestroy(ln.obs_stream);
    if (ln.stream) (void)hipStreamDestroy(ln.stream);
  }
  ctx->lanes.clear();
}

int ensure_lanes(dse_ctx* ctx) {
  if ((int)ctx->lanes.size() == ctx->n_streams) return DSE_OK;
  destroy_lanes(ctx);
  ctx->lanes.resize(ctx->n_streams);
  for (auto& ln : ctx->lanes) {
    HIPC(hipStreamCreateWithFlags(&ln.stream, hipStreamNonBlocking));
    // lowest priority: the observables take the CUs the next interval launch leaves, not the
    // other way round
    int least = 0, greatest = 0;
    HIPC(hipDeviceGetStreamPriorityRange(&least, &greatest));
    HIPC(hipStreamCreateWithPriority(&ln.obs_stream, hipStreamNonBlocking, least));
    for (int i = 0; i < 2; ++i) {
      HIPC(hipEventCreateWithFlags(&ln.ev_iv[i], hipEventDisableTiming));
      HIPC(hipEventCreateWithFlags(&ln.ev_obs[i], hipEventDisableTiming));
    }
  }
  return DSE_OK;
}

// the interval / step / observable streams (not the small-register engine's, which small_gather
// waits for): what flush_partials needs before it reads the observable partials
int sync_lanes(dse_ctx* ctx) {
  if (ctx->swap_stream) HIPC(hipStreamSynchronize(ctx->swap_stream));
  for (auto& ln : ctx->lanes) {
    HIPC(hipStreamSynchronize(ln.stream));
    if (ln.obs_stream) HIPC(hipStreamSynchronize(ln.obs_stream));
  }
  return DSE_OK;
}

int sync_all(dse_ctx* ctx) {
  if (ctx->swap_stream) HIPC(hipStreamSynchronize(ctx->swap_stream));
  for (auto& ln : ctx->lanes) {
    HIPC(hipStreamSynchronize(ln.stream));
    if (ln.obs_stream) HIPC(hipStreamSynchronize(ln.obs_stream));
  }
  if (ctx->small_stream) HIPC(hipStreamSynchronize(ctx->small_stream));
  return DSE_OK;
}

// ---- per-problem device tables ------------------------------------------------------------
int build_tables(dse_ctx* ctx, HostProblem& p, DevProb& d) {
  const int n = p.n;
  const int nl = p.n_local;   // qubits held in this context (n unless partitioned)
  int L = std::max(std::min(nl, ctx->tile_bits), std::max(kMinTile, nl - 32));
  // registers for the Walsh-Hadamard engine (whole, more than two 2^13 tiles) take its tile size
  if (ctx->wht && ctx->tile_bits == kMaxTile && nl > kMaxTile + 1)
    L = ctx->wht_tile_bits ? ctx->wht_tile_bits : 13;
  if (L > kMaxTile) return fail(ctx, DSE_ERR_ARG, "problem too large for the tile range");
  p.L = L;
  p.n_tiles = int64_t(1) << (nl - L);
  const size_t T = size_t(1) << L;
  const uint64_t lo_mask = (uint64_t(1) << L) - 1;
  const bool rb = L >= kRegBlockMinTile;
  const int TB = L - kRegBits;

  std::vector<double> zzlo(T, 0.0);
  for (size_t x = 0; x < T; ++x) {
    double acc = 0.0;
    for (int i = 0; i < L; ++i) {
      const double si = 0.5 - (double)((x >> i) & 1);
      for (int j = i + 1; j < L; ++j) acc += p.zz[i * n + j] * (si * (0.5 - (double)((x >> j) & 1)));
    }
    zzlo[x] = acc;
  }
  std::memset(&d, 0, sizeof(d));
  std::vector<DPair> plo, phi, ptt;
  std::vector<DFlip> flo, fhi;
  std::vector<DSweep> sweeps(rb ? TB : 0);
  for (auto& s : sweeps) std::memset(&s, 0, sizeof(s));
  for (int i = 0; i < n; ++i)
    for (int j = i + 1; j < n; ++j) {
      const double g = p.pair[i * n + j];
      if (g == 0.0) continue;
      const uint64_t m = (uint64_t(1) << i) | (uint64_t(1) << j);
      DPair q;
      q.mask_lo = (uint32_t)(m & lo_mask);
      q.tile_xor = (uint32_t)(m >> L);
      q.g = g;
      if (q.tile_xor) {
        phi.push_back(q);
      } else if (!rb) {
        plo.push_back(q);
      } else if (j < TB) {
        ptt.push_back(q);  // both thread bits
      } else if (i >= TB) {
        d.rr_g[rr_index(i - TB, j - TB)] = g;  // both register bits
      } else {
        sweeps[i].g[j - TB] = g;  // thread bit i, register bit j - TB
        sweeps[i].has_pair = 1;
      }
    }
  p.imag = true;
  for (int b = 0; b < n; ++b) {
    // A real part below 1e-15 of the coefficient's modulus is the rounding residue of cos(pi/2)
    // (the reference's drive phase, dipolar_ensemble_with_rare.py:516-530): it is dropped, so
    // drives at phase pi/2 take the imaginary-coefficient kernels (2 FMAs per amplitude, not 4).
    // The dropped entry is 1e-16 of its row's drive term, below the rounding of H itself.
    double f[4];
    for (int c = 0; c < 4; c += 2) {
      f[c] = p.flip[4 * b + c];
      f[c + 1] = p.flip[4 * b + c + 1];
      if (std::fabs(f[c]) <= 1e-15 * std::hypot(f[c], f[c + 1])) f[c] = 0.0;
    }
    if (f[0] == 0.0 && f[1] == 0.0 && f[2] == 0.0 && f[3] == 0.0) continue;
    if (f[0] != 0.0 || f[2] != 0.0) p.imag = false;
    const uint64_t m = uint64_t(1) << b;
    DFlip q;
    q.mask_lo = (uint32_t)(m & lo_mask);
    q.tile_xor = (uint32_t)(m >> L);
    q.re0 = f[0];
    q.im0 = f[1];
    q.re1 = f[2];
    q.im1 = f[3];
    q.pad = 0.0;
    if (q.tile_xor) {
      fhi.push_back(q);
    } else if (!rb) {
      flo.push_back(q);
    } else if (b < TB) {
      DSweep& s = sweeps[b];
      s.re0 = f[0];
      s.im0 = f[1];
      s.re1 = f[2];
      s.im1 = f[3];
      s.has_flip = 1;
    } else {
      const int i = b - TB;
      for (int c = 0; c < 4; ++c) d.rflip[i][c] = f[c];
      d.rflip_mask |= 1 << i;
    }
  }
  const size_t o_field = 0;
  const size_t o_zz = align_up(o_field + n * sizeof(double), 256);
  const size_t o_plo = align_up(o_zz + size_t(n) * n * sizeof(double), 256);
  const size_t o_phi = align_up(o_plo + plo.size() * sizeof(DPair), 256);
  const size_t o_ptt = align_up(o_phi + phi.size() * sizeof(DPair), 256);
  const size_t o_flo = align_up(o_ptt + ptt.size() * sizeof(DPair), 256);
  const size_t o_fhi = align_up(o_flo + flo.size() * sizeof(DFlip), 256);
  const size_t o_sw = align_up(o_fhi + fhi.size() * sizeof(DFlip), 256);
  const size_t total = align_up(o_sw + sweeps.size() * sizeof(DSweep) + 16, 256);
  std::vector<char> blob(total, 0);
  auto put = [&](size_t off, const void* src, size_t bytes) {
    if (bytes) std::memcpy(blob.data() + off, src, bytes);
  };
  put(o_field, p.field.data(), n * sizeof(double));
  put(o_zz, p.zz.data(), size_t(n) * n * sizeof(double));
  put(o_plo, plo.data(), plo.size() * sizeof(DPair));
  put(o_phi, phi.data(), phi.size() * sizeof(DPair));
  put(o_ptt, ptt.data(), ptt.size() * sizeof(DPair));
  put(o_flo, flo.data(), flo.size() * sizeof(DFlip));
  put(o_fhi, fhi.data(), fhi.size() * sizeof(DFlip));
  put(o_sw, sweeps.data(), sweeps.size() * sizeof(DSweep));
  if (hipMalloc(&p.tables, total) != hipSuccess)
    return fail(ctx, DSE_ERR_OOM, "device allocation of coefficient tables failed");
  HIPC(hipMemcpy(p.tables, blob.data(), total, hipMemcpyHostToDevice));
  const size_t vbytes = (size_t(1) << nl) * sizeof(double2);
  for (auto& b : p.buf) {
    if (hipMalloc(&b, vbytes) != hipSuccess)
      return fail(ctx, DSE_ERR_OOM, "device allocation of state buffers failed (" +
                                        std::to_string(3 * vbytes) + " bytes per problem)");
    HIPC(hipMemset(b, 0, vbytes));
  }
  char* tb = static_cast<char*>(p.tables);
  for (int i = 0; i < 3; ++i) d.buf[i] = p.buf[i];
  auto zt = ctx->zzlo_tables.find(zzlo);
  if (zt == ctx->zzlo_tables.end()) {
    double* dz = nullptr;
    if (hipMalloc(&dz, T * sizeof(double)) != hipSuccess)
      return fail(ctx, DSE_ERR_OOM, "device allocation of the ZZ table failed");
    HIPC(hipMemcpy(dz, zzlo.data(), T * sizeof(double), hipMemcpyHostToDevice));
    zt = ctx->zzlo_tables.emplace(zzlo, dz).first;
  }
  d.zzlo = zt->second;
  d.field = reinterpret_cast<const double*>(tb + o_field);
  d.zz = reinterpret_cast<const double*>(tb + o_zz);
  d.pairs_lo = reinterpret_cast<const DPair*>(tb + o_plo);
  d.pairs_hi = reinterpret_cast<const DPair*>(tb + o_phi);
  d.pairs_tt = reinterpret_cast<const DPair*>(tb + o_ptt);
  d.flips_lo = reinterpret_cast<const DFlip*>(tb + o_flo);
  d.flips_hi = reinterpret_cast<const DFlip*>(tb + o_fhi);
  d.sweeps = reinterpret_cast<const DSweep*>(tb + o_sw);
  d.coef = nullptr;
  d.sea_mask = p.sea_mask;
  d.shift = p.shift;
  d.beta = 0.0;
  d.s1 = 1.0;
  d.n = n;
  d.L = L;
  d.n_pairs_lo = (int)plo.size();
  d.n_pairs_hi = (int)phi.size();
  d.n_pairs_tt = (int)ptt.size();
  d.n_flips_lo = (int)flo.size();
  d.n_flips_hi = (int)fhi.size();
  d.kcap1 = 0;
  d.rare_bit = p.rare_bit;
  d.n_sea = __builtin_popcountll(p.sea_mask);
  // partitioned register: global tile index = rank << tbl | local tile; partner masks
  d.tbl = nl - L;
  d.h_base = (uint32_t)p.shard_rank << d.tbl;
  p.xmasks = 0;
  if (p.shard_bits > 0) {
    for (const auto& q : phi)
      if (q.tile_xor >> d.tbl) p.xmasks |= 1u << (q.tile_xor >> d.tbl);
    for (const auto& q : fhi)
      if (q.tile_xor >> d.tbl) p.xmasks |= 1u << (q.tile_xor >> d.tbl);
    for (int b = nl; b < n; ++b)  // <Ix>, <Iy> of a global qubit pair amplitudes across shards
      if (((p.sea_mask >> b) & 1ull) || b == p.rare_bit) p.xmasks |= 1u << (1u << (b - nl));
  }
  return DSE_OK;
}

int prepare(dse_ctx* ctx) {
  if (ctx->prepared) return DSE_OK;
  if (ctx->probs.empty()) return fail(ctx, DSE_ERR_STATE, "no problems added");
  int rc = ensure_lanes(ctx);
  if (rc) return rc;
  std::vector<DevProb> dp(ctx->probs.size());
  int64_t total = 0;
  for (size_t pi = 0; pi < ctx->probs.size(); ++pi) {
    if ((rc = build_tables(ctx, ctx->probs[pi], dp[pi]))) {
      free_device(ctx);
      return rc;
    }
    HostProblem& p = ctx->probs[pi];
    std::vector<int2> its(p.n_tiles);
    for (int64_t t = 0; t < p.n_tiles; ++t) its[t] = make_int2((int)pi, (int)t);
    if (hipMalloc(&p.d_items, its.size() * sizeof(int2)) != hipSuccess) {
      free_device(ctx);
      return fail(ctx, DSE_ERR_OOM, "device allocation of item lists failed");
    }
    HIPC(hipMemcpy(p.d_items, its.data(), its.size() * sizeof(int2), hipMemcpyHostToDevice));
    total += p.n_tiles;
  }
  // partitioned registers: partner shards' buffers (same context) or exchange receive buffers
  for (size_t pi = 0; pi < ctx->probs.size(); ++pi) {
    HostProblem& p = ctx->probs[pi];
    if (p.shard_bits == 0) continue;
    for (int m = 1; m < (1 << p.shard_bits); ++m) {
      if (!((p.xmasks >> m) & 1u)) continue;
      if (p.dist) {
        const size_t vbytes = (size_t(1) << p.n_local) * sizeof(double2);
        if (hipMalloc(&p.rbuf_own[m], vbytes) != hipSuccess) {
          free_device(ctx);
          return fail(ctx, DSE_ERR_OOM, "device allocation of exchange buffers failed");
        }
        for (int r = 0; r < 3; ++r) dp[pi].rbuf[m][r] = p.rbuf_own[m];
      } else {
        const HostProblem& q = ctx->probs[p.group_first + (p.shard_rank ^ m)];
        for (int r = 0; r < 3; ++r) dp[pi].rbuf[m][r] = q.buf[r];
      }
    }
  }
  if (hipMalloc(&ctx->d_probs, dp.size() * sizeof(DevProb)) != hipSuccess ||
      hipMalloc(&ctx->d_items, total * sizeof(int2)) != hipSuccess ||
      hipMalloc(&ctx->d_items_iv, total * sizeof(int2)) != hipSuccess) {
    free_device(ctx);
    return fail(ctx, DSE_ERR_OOM, "device allocation of descriptors failed");
  }
  HIPC(hipMemcpy(ctx->d_probs, dp.data(), dp.size() * sizeof(DevProb), hipMemcpyHostToDevice));
  ctx->h_desc = dp;
  ctx->total_items = total;
  HIPC(hipDeviceSynchronize());
  ctx->prepared = true;
  return DSE_OK;
}

// ---- Walsh-Hadamard engine ------------------------------------------------------------------

// WhtGroup of the given high bits: completed to wl tile bits by the lowest carried bits; every
// other local bit is an outer bit.
WhtGroup make_group(const std::vector<int>& bits, int wl, int n_local) {
  WhtGroup g;
  std::memset(&g, 0, sizeof(g));
  const int s = (int)bits.size();
  g.c = wl - s;
  std::vector<int> in(n_local, 0);
  for (int q = 0; q < g.c; ++q) g.pos[q] = q, in[q] = 1;
  for (int i = 0; i < s; ++i) g.pos[g.c + i] = bits[i], in[bits[i]] = 1;
  int o = 0;
  for (int b = 0; b < n_local; ++b)
    if (!in[b]) g.opos[o++] = b;
  g.n_outer = o;
  return g;
}

// balanced split of bits into ceil(|bits| / max_bits) contiguous groups
std::vector<std::vector<int>> split_bits(const std::vector<int>& bits, int max_bits) {
  std::vector<std::vector<int>> out;
  const int h = (int)bits.size();
  if (h == 0) return out;
  const int ng = (h + max_bits - 1) / max_bits;
  int first = 0;
  for (int gi = 0; gi < ng; ++gi) {
    const int s = h / ng + (gi < h % ng ? 1 : 0);
    out.emplace_back(bits.begin() + first, bits.begin() + first + s);
    first += s;
  }
  return out;
}

// Tile-bit groups of a register of n_local local qubits (w.grp, returns G; 0: not possible).
// Group 0 = local bits 0..wl-1.  Unpartitioned: the high bits in balanced groups of <= max_bits,
// the last one is MID's.  Partitioned (S shard bits): the pre-swap groups must transform the top
// S local bits T (they leave with the index swap); MID transforms the shard bits that arrive in
// T's positions together with up to max_bits - S other local high bits.
//
// mid_inpage m > 0 (option wht_mid_inpage, unpartitioned registers): the MID group takes the top m
// high bits below the 2-MiB page (local bits < kWhtPageBit) in place of its lowest above-page
// bits, the other groups the rest.  A pass's tile touches 2^(its group's above-page bits) pages;
// with the contiguous split MID's group lies wholly above the page (N = 30: 256 pages per tile,
// a TLB miss on 61% of its requests) while FWD's keeps every in-page bit (32 pages).
constexpr int kWhtPageBit = 17;  // 2^17 amplitudes of 16 B = 2 MiB
int wht_layout(int n_local, int S, int wl, int max_bits, WhtProb& w, int mid_inpage = 0) {
  const int h = n_local - wl;
  if (h < 1 || h > kWhtMaxOuter || h < S || max_bits <= S) return 0;
  std::vector<int> high;
  for (int b = wl; b < n_local; ++b) high.push_back(b);
  std::vector<std::vector<int>> groups;
  if (S == 0) {
    groups = split_bits(high, max_bits);
    if (mid_inpage > 0 && groups.size() >= 2) {
      std::vector<int> inpage, above;
      for (int b : high) (b < kWhtPageBit ? inpage : above).push_back(b);
      const int smid = (int)groups.back().size();
      const int m = std::min({mid_inpage, (int)inpage.size(), smid});
      if (m > 0 && (int)above.size() >= smid - m) {
        std::vector<int> mid(inpage.end() - m, inpage.end());
        mid.insert(mid.end(), above.end() - (smid - m), above.end());
        std::vector<int> rest;
        for (int b : high)
          if (std::find(mid.begin(), mid.end(), b) == mid.end()) rest.push_back(b);
        groups = split_bits(rest, max_bits);
        groups.push_back(mid);
      }
    }
  } else {
    const std::vector<int> rest(high.begin(), high.end() - S), T(high.end() - S, high.end());
    const int m = std::min(max_bits - S, (int)rest.size());
    std::vector<int> mid(rest.begin(), rest.begin() + m), pre(rest.begin() + m, rest.end());
    pre.insert(pre.end(), T.begin(), T.end());
    groups = split_bits(pre, max_bits);
    mid.insert(mid.end(), T.begin(), T.end());
    groups.push_back(mid);
  }
  if ((int)groups.size() + 1 > kWhtMaxGroups) return 0;
  w.grp[0] = make_group({}, wl, n_local);  // pos = 0..wl-1, outer = the high bits
  w.grp[0].c = 0;                           // group 0 transforms all its tile bits
  for (size_t gi = 0; gi < groups.size(); ++gi) w.grp[gi + 1] = make_group(groups[gi], wl, n_local);
  return (int)groups.size() + 1;
}

// Builds the engine's tables and vectors for the problems it can take: registers of more than one
// tile, whole or partitioned (loopback shards or one shard per process).  Idempotent until
// free_device.
int ensure_wht(dse_ctx* ctx) {
  if (ctx->wht_ready) return DSE_OK;
  std::vector<WhtProb> hw(ctx->probs.size());
  std::memset(hw.data(), 0, hw.size() * sizeof(WhtProb));
  for (size_t pi = 0; pi < ctx->probs.size(); ++pi) {
    HostProblem& p = ctx->probs[pi];
    p.wht_groups = 0;
    if (!ctx->wht || p.L < kWhtMinTile || p.L > kWhtMaxTile || p.n_tiles < 2) continue;
    const int n = p.n, nl = p.n_local, S = p.shard_bits;
    WhtProb& w = hw[pi];
    const int gb = ctx->wht_group_bits ? std::min(ctx->wht_group_bits, p.L - 2) : p.L - 2;
    const int G = wht_layout(nl, S, p.L, gb, w, ctx->wht_mid_inpage);
    if (G < 2) continue;
    const double sc = std::ldexp(1.0, -n);
    std::vector<double> cq(size_t(n) * n, 0.0);
    for (int i = 0; i < n; ++i)
      for (int j = i + 1; j < n; ++j) cq[size_t(i) * n + j] = cq[size_t(j) * n + i] = 0.5 * p.pair[i * n + j] * sc;
    for (int b = 0; b < n; ++b) {
      double re = p.flip[4 * b + 2], im = p.flip[4 * b + 3];
      if (std::fabs(re) <= 1e-15 * std::hypot(re, im)) re = 0.0;  // as build_tables
      w.lin_x[b] = re * sc;
      w.lin_y[b] = im * sc;
    }
    const size_t vbytes = (size_t(1) << nl) * sizeof(double2);
    const int nvec = S > 0 ? 4 : 2;
    bool ok = hipMalloc(&p.d_cquad, cq.size() * sizeof(double)) == hipSuccess &&
              hipMalloc(&p.d_wtab, ((size_t)p.n_tiles * 48 + 2 * (5 * 512 + 16)) * sizeof(double)) == hipSuccess;
    // option wht_contiguous: the X/Y-branch vectors physically contiguous (large translation
    // fragments for the strided passes), else (or when that fails) a plain allocation
    for (int v = 0; v < nvec && ok; ++v) {
      if (ctx->wht_contiguous &&
          hipExtMallocWithFlags((void**)&p.wvec[v], vbytes, hipDeviceMallocContiguous) == hipSuccess)
        continue;
      (void)hipGetLastError();
      ok = hipMalloc(&p.wvec[v], vbytes) == hipSuccess;
    }
    if (!ok) {  // HBM too small for the engine's two extra vectors: this problem keeps the step kernels
      (void)hipGetLastError();
      free_wht(p);
      std::memset(&w, 0, sizeof(w));
      continue;
    }
    HIPC(hipMemcpy(p.d_cquad, cq.data(), cq.size() * sizeof(double), hipMemcpyHostToDevice));
    w.vec_a = p.wvec[0];
    w.vec_b = p.wvec[1];
    w.vec_at = S > 0 ? p.wvec[2] : p.wvec[0];
    w.vec_bt = S > 0 ? p.wvec[3] : p.wvec[1];
    for (int b = 0; b < n; ++b) w.gmap[b] = b;
    if (S > 0) {  // MID state: local bits nl-S+i hold global nl+i, the rank holds global nl-S+i
      for (int i = 0; i < S; ++i) w.gmap[nl - S + i] = nl + i;
      w.fix_mask = ((uint64_t(1) << S) - 1) << (nl - S);
      w.fix_val = (uint64_t)p.shard_rank << (nl - S);
      w.phase0 = __builtin_popcount((unsigned)p.shard_rank);
    }
    w.cquad = p.d_cquad;
    w.ztab = p.d_wtab;
    w.xytab = p.d_wtab + (size_t)p.n_tiles * 16;
    w.qtab = p.d_wtab + (size_t)p.n_tiles * 48;
    w.n = n;
    w.n_local = nl;
    w.wl = p.L;
    w.n_groups = G;
    p.wht_groups = G;
  }
  // the shards of a loopback register run the same launches: all on the engine or none
  for (size_t pi = 0; pi < ctx->probs.size(); ++pi) {
    const HostProblem& P = ctx->probs[pi];
    if (P.shard_bits == 0 || P.dist || P.shard_rank != 0) continue;
    bool all = true;
    for (int r = 0; r < (1 << P.shard_bits); ++r) all = all && ctx->probs[pi + r].wht_groups > 0;
    if (all) continue;
    for (int r = 0; r < (1 << P.shard_bits); ++r) {
      free_wht(ctx->probs[pi + r]);
      std::memset(&hw[pi + r], 0, sizeof(WhtProb));
    }
  }
  if (!ctx->d_wht && hipMalloc(&ctx->d_wht, hw.size() * sizeof(WhtProb)) != hipSuccess)
    return fail(ctx, DSE_ERR_OOM, "device allocation of descriptors failed");
  HIPC(hipMemcpy(ctx->d_wht, hw.data(), hw.size() * sizeof(WhtProb), hipMemcpyHostToDevice));
  for (size_t pi = 0; pi < ctx->probs.size(); ++pi)
    if (ctx->probs[pi].wht_groups)
      HIPC(launch_wht_tables(ctx->probs[pi].L, ctx->d_wht + pi, ctx->d_probs + pi, ctx->probs[pi].n_tiles, ctx->lanes[0].stream));
  HIPC(hipStreamSynchronize(ctx->lanes[0].stream));
  ctx->wht_ready = true;
  return DSE_OK;
}

// ---- exchanges of a register partitioned over processes: RCCL, or the host transport ----
// all-to-all of equal chunks (chunk p -> rank p), device buffers
// Exchange timing: xt_begin/xt_end bracket one exchange on stream st with a HIP event pair
// (RCCL path; pairs beyond the pool are not timed); xt_sum adds the finished pairs to ctx->xms.
int xt_begin(dse_ctx* ctx, hipStream_t st, size_t* slot) {
  *slot = SIZE_MAX;
  if (ctx->xev_used >= 4096) return DSE_OK;
  while (ctx->xev.size() < 2 * (ctx->xev_used + 1)) {
    hipEvent_t e;
    HIPC(hipEventCreate(&e));
    ctx->xev.push_back(e);
  }
  *slot = ctx->xev_used++;
  HIPC(hipEventRecord(ctx->xev[2 * *slot], st));
  return DSE_OK;
}

int xt_end(dse_ctx* ctx, hipStream_t st, size_t slot) {
  if (slot != SIZE_MAX) HIPC(hipEventRecord(ctx->xev[2 * slot + 1], st));
  return DSE_OK;
}

int xt_sum(dse_ctx* ctx) {
  for (size_t i = 0; i < ctx->xev_used; ++i) {
    HIPC(hipEventSynchronize(ctx->xev[2 * i + 1]));
    float ms = 0.f;
    HIPC(hipEventElapsedTime(&ms, ctx->xev[2 * i], ctx->xev[2 * i + 1]));
    ctx->xms += ms;
  }
  ctx->xev_used = 0;
  return DSE_OK;
}

double host_ms_since(std::chrono::steady_clock::time_point t0) {
  return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
}

int xchg_alltoall(dse_ctx* ctx, const void* src, void* dst, size_t cbytes, hipStream_t st) {
  ctx->xbytes += (double)cbytes * (ctx->dist_world - 1);
  if (!ctx->xfn) {
    size_t slot;
    int rc = xt_begin(ctx, st, &slot);
    if (rc) return rc;
    const ncclResult_t r = ncclAllToAll(src, dst, cbytes, ncclUint8, ctx->comm, st);
    if (r != ncclSuccess) return fail(ctx, DSE_ERR_HIP, std::string("ncclAllToAll: ") + ncclGetErrorString(r));
    return xt_end(ctx, st, slot);
  }
  const auto h0 = std::chrono::steady_clock::now();
  struct AddMs {
    dse_ctx* c;
    std::chrono::steady_clock::time_point t0;
    ~AddMs() { c->xms += host_ms_since(t0); }
  } add_ms{ctx, h0};
  const size_t total = cbytes * ctx->dist_world;
  ctx->xsend.resize(total);
  ctx->xrecv.resize(total);
  HIPC(hipMemcpyAsync(ctx->xsend.data(), src, total, hipMemcpyDeviceToHost, st));
  HIPC(hipStreamSynchronize(st));
  if (ctx->xfn(ctx->xuser, DSE_XCHG_ALLTOALL, ctx->xsend.data(), ctx->xrecv.data(), cbytes, -1) != 0)
    return fail(ctx, DSE_ERR_HIP, "exchange callback (all-to-all) failed");
  HIPC(hipMemcpyAsync(dst, ctx->xrecv.data(), total, hipMemcpyHostToDevice, st));
  HIPC(hipStreamSynchronize(st));
  return DSE_OK;
}

// in-place sum over ranks of host doubles
int xchg_allreduce_host(dse_ctx* ctx, double* v, size_t count, hipStream_t st) {
  if (ctx->xfn) {
    if (ctx->xfn(ctx->xuser, DSE_XCHG_ALLREDUCE_F64, v, v, count * sizeof(double), -1) != 0)
      return fail(ctx, DSE_ERR_HIP, "exchange callback (all-reduce) failed");
    return DSE_OK;
  }
  if (ctx->allreduce_cap < count) {  // one staging buffer per context, grown on demand
    if (ctx->d_allreduce) (void)hipFree(ctx->d_allreduce), ctx->d_allreduce = nullptr;
    ctx->allreduce_cap = 0;
    if (hipMalloc(&ctx->d_allreduce, count * sizeof(double)) != hipSuccess)
      return fail(ctx, DSE_ERR_OOM, "all-reduce staging allocation failed");
    ctx->allreduce_cap = count;
  }
  double* d = ctx->d_allreduce;
  hipError_t e = hipMemcpyAsync(d, v, count * sizeof(double), hipMemcpyHostToDevice, st);
  const ncclResult_t r = ncclAllReduce(d, d, count, ncclFloat64, ncclSum, ctx->comm, st);
  if (e == hipSuccess) e = hipMemcpyAsync(v, d, count * sizeof(double), hipMemcpyDeviceToHost, st);
  if (e == hipSuccess) e = hipStreamSynchronize(st);
  if (r != ncclSuccess) return fail(ctx, DSE_ERR_HIP, std::string("ncclAllReduce: ") + ncclGetErrorString(r));
  HIPC(e);
  return DSE_OK;
}

// Index swap of the X/Y vectors of partitioned registers (local top S bits <-> shard bits):
// chunk p of shard r -> chunk r of shard p; an involution, so back = the same exchange from the
// swapped copies.  Loopback registers: device copies; one shard per process: RCCL all-to-all.
int wht_swap(dse_ctx* ctx, const std::vector<int>& regs, bool back, hipStream_t st, int vsel = 3) {
  for (int first : regs) {
    const HostProblem& P0 = ctx->probs[first];
    const int S = P0.shard_bits;
    const size_t chunk = size_t(1) << (P0.n_local - S);
    const size_t cbytes = chunk * sizeof(double2);
    for (int v = 0; v < 2; ++v) {
      if (!((vsel >> v) & 1)) continue;
      if (P0.dist) {
        const double2* src = P0.wvec[back ? 2 + v : v];
        double2* dst = P0.wvec[back ? v : 2 + v];
        const int rc = xchg_alltoall(ctx, src, dst, cbytes, st);
        if (rc) return rc;
        continue;
      }
      for (int r = 0; r < (1 << S); ++r)
        for (int p = 0; p < (1 << S); ++p) {
          const HostProblem& Pr = ctx->probs[first + r];
          const HostProblem& Pp = ctx->probs[first + p];
          const double2* src = (back ? Pr.wvec[2 + v] : Pr.wvec[v]) + p * chunk;
          double2* dst = (back ? Pp.wvec[v] : Pp.wvec[2 + v]) + r * chunk;
          HIPC(hipMemcpyAsync(dst, src, cbytes, hipMemcpyDeviceToDevice, st));
        }
    }
  }
  return DSE_OK;
}

// One WHT application (mode / term k) over items of problems with wht_groups == G, tile wl;
// regs: first problem of every partitioned register among them (index swaps around MID).
// segs: (items, count) launches of the same wl / G.
int wht_run(dse_ctx* ctx, int wl, int G, const std::vector<std::pair<const int2*, int>>& segs,
            const std::vector<int>& regs, int mode, int k, int q, int set, hipStream_t st) {
  int rc;
  auto part = [&](int pt, int vsel) -> int {
    for (const auto& sg : segs)
      HIPC(launch_wht_part(pt, wl, mode, G, ctx->d_wht, ctx->d_probs, sg.first, sg.second, k, q, set, vsel, st,
                           ctx->n_cu * (wl == 13 ? 1 : 2),
                           ctx->wht_persist | ctx->wht_half << 8 | (ctx->wht_fuse && regs.empty()) << 16));
    return DSE_OK;
  };
  if (regs.empty() || !ctx->swap_overlap) {
    for (int pt = WHT_PART_PRE; pt <= WHT_PART_POST; ++pt) {
      if (pt == WHT_PART_MID && !regs.empty() && (rc = wht_swap(ctx, regs, false, st))) return rc;
      if (pt == WHT_PART_POST && !regs.empty() && (rc = wht_swap(ctx, regs, true, st))) return rc;
      if ((rc = part(pt, 3))) return rc;
    }
    return DSE_OK;
  }
  // Partitioned registers: the X-branch vector A and the Y-branch vector B are transformed in
  // separate launches, and each index swap (all-to-all over the shards) runs on swap_stream while
  // the compute stream works on the other vector:
  //   st    FIRST+FWD(A) | FWD(B) |        MID(A) |        MID(B) |        INV(A) |  INV(B)+FINAL
  //   swap               | swap A | swap B        | back A        | back B
  // ev[v]: vector v ready on st for its swap, ev[2+v]: swapped, ev[4+v]: MID done, ev[6+v]: back.
  if (!ctx->swap_stream) {
    HIPC(hipStreamCreateWithFlags(&ctx->swap_stream, hipStreamNonBlocking));
    for (auto& e : ctx->swap_ev) HIPC(hipEventCreateWithFlags(&e, hipEventDisableTiming));
  }
  hipStream_t sw = ctx->swap_stream;
  hipEvent_t* ev = ctx->swap_ev;
  // the swap stream takes over vector v once event i is reached on the compute stream, swaps it
  // (there, or back), and marks event j when done
  auto swap_after = [&](int i, int v, bool back, int j) -> int {
    HIPC(hipEventRecord(ev[i], st));
    HIPC(hipStreamWaitEvent(sw, ev[i], 0));
    const int r = wht_swap(ctx, regs, back, sw, 1 << v);
    if (r) return r;
    HIPC(hipEventRecord(ev[j], sw));
    return DSE_OK;
  };
  auto wait_swap = [&](int j) -> int {
    HIPC(hipStreamWaitEvent(st, ev[j], 0));
    return DSE_OK;
  };
  for (int v = 0; v < 2; ++v)  // PRE of A (with FIRST), then of B; each vector's swap behind it
    if ((rc = part(WHT_PART_PRE, 1 << v)) || (rc = swap_after(v, v, false, 2 + v))) return rc;
  for (int v = 0; v < 2; ++v)  // MID of a vector once it is swapped; its swap back behind it
    if ((rc = wait_swap(2 + v)) || (rc = part(WHT_PART_MID, 1 << v)) || (rc = swap_after(4 + v, v, true, 6 + v)))
      return rc;
  for (int v = 0; v < 2; ++v)  // POST: INV(A), then INV(B) + FINAL
    if ((rc = wait_swap(6 + v)) || (rc = part(WHT_PART_POST, 1 << v))) return rc;
  return DSE_OK;
}

int ensure_partial(dse_ctx* ctx, size_t slots) {
  if (ctx->partial_slots >= slots) return DSE_OK;
  if (ctx->d_partial) (void)hipFree(ctx->d_partial), ctx->d_partial = nullptr;
  if (hipMalloc(&ctx->d_partial, slots * ctx->total_items * 8 * sizeof(double)) != hipSuccess)
    return fail(ctx, DSE_ERR_OOM, "device allocation of observable partials failed");
  ctx->partial_slots = slots;
  return DSE_OK;
}

void finish_obs(const HostProblem& P, const double* v, double* o, size_t stride) {
  const double n2 = v[6];
  const double inv = n2 > 0.0 ? 1.0 / n2 : 0.0;
  o[0 * stride] = v[0] * inv;
  o[1 * stride] = v[1] * inv;
  o[2 * stride] = v[2] * inv;
  o[3 * stride] = P.rare_bit >= 0 ? v[3] * inv : P.rare_z;
  o[4 * stride] = P.rare_bit >= 0 ? v[4] * inv : 0.0;
  o[5 * stride] = P.rare_bit >= 0 ? v[5] * inv : 0.0;
  o[6 * stride] = std::sqrt(n2);
}

// Observable sums of output slots [t0, t0 + nslots).  A loopback shard group sums the tiles of all
// its shards and writes the result to every shard's row; a dist shard keeps its raw local sums in
// dist_raw for the all-reduce at the end of dse_evolve.
int flush_partials(dse_ctx* ctx, size_t nslots, size_t t0, int n_t, double* obs_out,
                   std::vector<double>* dist_raw) {
  if ((int)sync_lanes(ctx)) return DSE_ERR_HIP;
  if (ctx->d_err_cur) {  // a persistent hand-off timed out: abandon this run (dse_evolve falls back)
    int herr = 0;
    HIPC(hipMemcpy(&herr, ctx->d_err_cur, sizeof(int), hipMemcpyDeviceToHost));
    if (herr) return kRcHandoffTimeout;
  }
  std::vector<double> h(nslots * ctx->total_items * 8);
  HIPC(hipMemcpy(h.data(), ctx->d_partial, h.size() * sizeof(double), hipMemcpyDeviceToHost));
  for (size_t pi = 0; pi < ctx->probs.size(); ++pi) {
    const HostProblem& P = ctx->probs[pi];
    if (P.side()) continue;  // the small-register engine writes its own sums
    const bool grouped = P.shard_bits > 0 && !P.dist;
    const size_t first_member = grouped ? (size_t)P.group_first : pi;
    const size_t n_members = grouped ? (size_t(1) << P.shard_bits) : 1;
    for (size_t s = 0; s < nslots; ++s) {
      double v[7] = {0, 0, 0, 0, 0, 0, 0};
      for (size_t mi = first_member; mi < first_member + n_members; ++mi) {
        const double* row = h.data() + (s * ctx->total_items + ctx->item_pos[mi]) * 8;
        for (int64_t t = 0; t < ctx->probs[mi].n_tiles; ++t)
          for (int j = 0; j < 7; ++j) v[j] += row[t * 8 + j];
      }
      if (P.dist) {
        double* raw = dist_raw->data() + (pi * (size_t)n_t + t0 + s) * 7;
        for (int j = 0; j < 7; ++j) raw[j] = v[j];
      } else {
        finish_obs(P, v, obs_out + pi * DSE_N_OBS * (size_t)n_t + (t0 + s), (size_t)n_t);
      }
    }
  }
  return DSE_OK;
}

// RCCL exchange for dist shards: every shard sends its role-`role` vector to each partner rank ^ m
// it shares terms with and receives the partner's into rbuf_own[m] (min_degree: only problems
// whose Chebyshev degree reaches the current term).
int dist_exchange(dse_ctx* ctx, int role, int min_degree, hipStream_t st) {
  for (auto& P : ctx->probs) {
    if (!P.dist || P.degree < min_degree || !P.xmasks) continue;
    const size_t bytes = (size_t(1) << P.n_local) * sizeof(double2);
    if (ctx->xfn) {  // host transport: one blocking send/recv per partner, masks in ascending order
      struct AddMs {
        dse_ctx* c;
        std::chrono::steady_clock::time_point t0;
        ~AddMs() { c->xms += host_ms_since(t0); }
      } add_ms{ctx, std::chrono::steady_clock::now()};
      ctx->xsend.resize(bytes);
      ctx->xrecv.resize(bytes);
      HIPC(hipMemcpyAsync(ctx->xsend.data(), P.buf[role], bytes, hipMemcpyDeviceToHost, st));
      HIPC(hipStreamSynchronize(st));
      for (int m = 1; m < (1 << P.shard_bits); ++m) {
        if (!((P.xmasks >> m) & 1u)) continue;
        ctx->xbytes += (double)bytes;
        if (ctx->xfn(ctx->xuser, DSE_XCHG_SENDRECV, ctx->xsend.data(), ctx->xrecv.data(), bytes,
                     ctx->dist_rank ^ m) != 0)
          return fail(ctx, DSE_ERR_HIP, "exchange callback (send/recv) failed");
        HIPC(hipMemcpyAsync(P.rbuf_own[m], ctx->xrecv.data(), bytes, hipMemcpyHostToDevice, st));
        HIPC(hipStreamSynchronize(st));
      }
      continue;
    }
    size_t slot;
    int rc = xt_begin(ctx, st, &slot);
    if (rc) return rc;
    if (ncclGroupStart() != ncclSuccess) return fail(ctx, DSE_ERR_HIP, "ncclGroupStart failed");
    for (int m = 1; m < (1 << P.shard_bits); ++m) {
      if (!((P.xmasks >> m) & 1u)) continue;
      const int peer = ctx->dist_rank ^ m;
      ctx->xbytes += (double)bytes;
      ncclResult_t r1 = ncclSend(P.buf[role], bytes, ncclUint8, peer, ctx->comm, st);
      ncclResult_t r2 = ncclRecv(P.rbuf_own[m], bytes, ncclUint8, peer, ctx->comm, st);
      if (r1 != ncclSuccess || r2 != ncclSuccess) {
        (void)ncclGroupEnd();
        return fail(ctx, DSE_ERR_HIP, std::string("RCCL send/recv: ") + ncclGetErrorString(r1 != ncclSuccess ? r1 : r2));
      }
    }
    const ncclResult_t r = ncclGroupEnd();
    if (r != ncclSuccess) return fail(ctx, DSE_ERR_HIP, std::string("ncclGroupEnd: ") + ncclGetErrorString(r));
    if ((rc = xt_end(ctx, st, slot))) return rc;
  }
  return DSE_OK;
}

int ensure_events(dse_ctx* ctx, Lane& ln, size_t per_pool) {
  for (int p = 0; p < 2; ++p)
    while (ln.ev[p].size() < 2 * per_pool) {
      hipEvent_t e;
      HIPC(hipEventCreate(&e));
      ln.ev[p].push_back(e);
    }
  return DSE_OK;
}

}  // namespace

// ------------------------------------------------------------------------------------------
// C ABI
// ------------------------------------------------------------------------------------------
extern "C" {

int dse_device_count(void) {
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess) return 0;
  return n;
}

const char* dse_create_error(void) { return g_create_err.c_str(); }

int dse_device_memory(int device, double* free_total) {
  if (!free_total) return DSE_ERR_ARG;
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess || device < 0 || device >= n) return DSE_ERR_NODEVICE;
  int prev = 0;
  (void)hipGetDevice(&prev);
  size_t fr = 0, tot = 0;
  const bool ok = hipSetDevice(device) == hipSuccess && hipMemGetInfo(&fr, &tot) == hipSuccess;
  (void)hipSetDevice(prev);
  if (!ok) return DSE_ERR_HIP;
  free_total[0] = (double)fr;
  free_total[1] = (double)tot;
  return DSE_OK;
}

dse_ctx* dse_create(int device) {
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess || n <= 0) {
    g_create_err = "no HIP device available";
    return nullptr;
  }
  if (device < 0 || device >= n) {
    g_create_err = "device index out of range";
    return nullptr;
  }
  if (hipSetDevice(device) != hipSuccess) {
    g_create_err = "hipSetDevice failed";
    return nullptr;
  }
  dse_ctx* ctx = new (std::nothrow) dse_ctx();
  if (!ctx) {
    g_create_err = "out of host memory";
    return nullptr;
  }
  ctx->device = device;
  {
    int ncu = 0;
    if (hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, device) == hipSuccess && ncu > 0)
      ctx->n_cu = ncu;
  }
  if (ensure_lanes(ctx) != DSE_OK) {
    g_create_err = "stream creation failed: " + ctx->err;
    delete ctx;
    return nullptr;
  }
  return ctx;
}

void dse_destroy(dse_ctx* ctx) {
  if (!ctx) return;
  (void)hipSetDevice(ctx->device);
  (void)sync_all(ctx);
  free_device(ctx);
  if (ctx->d_mx) (void)hipFree(ctx->d_mx), ctx->d_mx = nullptr;
  destroy_lanes(ctx);
  if (ctx->comm) (void)ncclCommDestroy(ctx->comm);
  delete ctx;
}

const char* dse_last_error(const dse_ctx* ctx) { return ctx ? ctx->err.c_str() : "null context"; }

int dse_set_option(dse_ctx* ctx, const char* key, double value) {
  if (!ctx || !key) return DSE_ERR_ARG;
  const std::string k(key);
  (void)hipSetDevice(ctx->device);
  if (k == "tile_bits") {
    if (!(value >= 1 && value <= kMaxTile)) return fail(ctx, DSE_ERR_ARG, "tile_bits must be in 1..13");
    if ((int)value != ctx->tile_bits) {
      (void)sync_all(ctx);
      free_device(ctx);
      ctx->tile_bits = (int)value;
    }
  } else if (k == "streams") {
    if (!(value >= 1 && value <= 16)) return fail(ctx, DSE_ERR_ARG, "streams must be in 1..16");
    (void)sync_all(ctx);
    ctx->n_streams = (int)value;
    ctx->evolved = false;
    return ensure_lanes(ctx);
  } else if (k == "persistent") {
    ctx->persistent = value != 0.0;
  } else if (k == "swap_overlap") {
    ctx->swap_overlap = value != 0.0;
  } else if (k == "wht") {
    if ((value != 0.0) != (ctx->wht != 0)) {
      (void)sync_all(ctx);
      free_device(ctx);
      ctx->wht = value != 0.0;
    }
  } else if (k == "wht_contiguous") {  // Walsh-Hadamard engine's vectors physically contiguous
    if (!(value == 0.0 || value == 1.0)) return fail(ctx, DSE_ERR_ARG, "wht_contiguous must be 0 or 1");
    if ((int)value != ctx->wht_contiguous) {
      (void)sync_all(ctx);
      free_device(ctx);
      ctx->wht_contiguous = (int)value;
    }
  } else if (k == "wht_fuse") {  // Walsh-Hadamard engine: FINAL of term k + FIRST of term k + 1
    if (!(value == 0.0 || value == 1.0)) return fail(ctx, DSE_ERR_ARG, "wht_fuse must be 0 or 1");
    ctx->wht_fuse = (int)value;
  } else if (k == "wht_mid_inpage") {  // Walsh-Hadamard plan: MID group's high bits below the page
    if (!(value >= 0.0 && value <= 8.0 && value == (int)value)) return fail(ctx, DSE_ERR_ARG, "wht_mid_inpage must be 0..8");
    if ((int)value != ctx->wht_mid_inpage) {
      (void)sync_all(ctx);
      free_device(ctx);
      ctx->wht_mid_inpage = (int)value;
    }
  } else if (k == "wht_half") {  // Walsh-Hadamard passes through half the LDS, two workgroups per CU
    if (!(value >= 0.0 && value <= 7.0 && value == (int)value)) return fail(ctx, DSE_ERR_ARG, "wht_half must be 0..7");
    ctx->wht_half = (int)value;
  } else if (k == "wht_persist") {  // Walsh-Hadamard passes as persistent launches: bit 1 MID
    ctx->wht_persist = (int)value;
  } else if (k == "wht_tile_bits") {
    if (!(value == 0 || value == 12 || value == 13)) return fail(ctx, DSE_ERR_ARG, "wht_tile_bits must be 0, 12 or 13");
    if ((int)value != ctx->wht_tile_bits) {
      (void)sync_all(ctx);
      free_device(ctx);
      ctx->wht_tile_bits = (int)value;
    }
  } else if (k == "wht_group_bits") {
    if (!(value == 0 || (value >= 2 && value <= 11)))
      return fail(ctx, DSE_ERR_ARG, "wht_group_bits must be 0 or in 2..11");
    if ((int)value != ctx->wht_group_bits) {
      (void)sync_all(ctx);
      free_device(ctx);
      ctx->wht_group_bits = (int)value;
    }
  } else if (k == "outputs_per_launch") {
    if (!(value >= 1 && value <= kMaxOut))
      return fail(ctx, DSE_ERR_ARG, "outputs_per_launch must be in 1.." + std::to_string(kMaxOut));
    ctx->outputs_per_launch = (int)value;
  } else if (k == "span_outputs") {  // M of an evolve whose registers all span (k_span)
    if (!(value >= 1 && value <= kSpanMaxOut))
      return fail(ctx, DSE_ERR_ARG, "span_outputs must be in 1.." + std::to_string(kSpanMaxOut));
    ctx->span_outputs = (int)value;
  } else if (k == "coresident") {  // diagnostics: workgroups per chunk of a 2-tile interval launch
    if (!(value == 0 || (value >= 2 && value <= 4096)))
      return fail(ctx, DSE_ERR_ARG, "coresident must be 0 or in 2..4096");
    ctx->coresident = (int)value;
  } else if (k == "dbg") {  // diagnostics bit mask: 1 one observable launch per output, 2 psi0 by
                            // memset/copy, 4 coefficient tables on one host thread
    ctx->dbg = (int)value;
  } else if (k == "small") {  // registers of <= 9 qubits on the one-wave engine (dse_small.hip)
    ctx->small = value != 0.0;
  } else if (k == "matrix") {  // propagator-matrix mode: 0 off, 1 auto, 2 always (when eligible)
    if (!(value == 0 || value == 1 || value == 2)) return fail(ctx, DSE_ERR_ARG, "matrix must be 0, 1 or 2");
    ctx->matrix = (int)value;
  } else if (k == "eig_streams") {  // dense engine: large eigendecompositions at a time (1..8)
    if (!(value >= 1 && value <= 8)) return fail(ctx, DSE_ERR_ARG, "eig_streams must be in 1..8");
    ctx->eig_streams = (int)value;
  } else if (k == "eig_impl") {  // dense engine eigensolver: 0 dsyevd, 1 auto, 2 half-matrix from 2^10,
                                 // 3 two-stage from 2^10
    if (!(value >= 0 && value <= 3)) return fail(ctx, DSE_ERR_ARG, "eig_impl must be 0, 1, 2 or 3");
    ctx->eig_impl = (int)value;
  } else if (k == "eig_spin_limit") {  // two-stage eigensolver: poll rounds before a give-up (< 0: at once)
    if (!(value >= -1 && value <= 1 << 30)) return fail(ctx, DSE_ERR_ARG, "eig_spin_limit must be in -1..2^30");
    ctx->eig_spin = (int)value;
  } else if (k == "dense_refine") {  // dense engine: refined eigenvalues + double-double phases
    ctx->dense_refine = value != 0.0;
  } else if (k == "dense_nufft") {  // dense engine: output times by the non-uniform FFT (0, 1, 2)
    if (!(value == 0.0 || value == 1.0 || value == 2.0)) return fail(ctx, DSE_ERR_ARG, "dense_nufft must be 0, 1 or 2");
    ctx->dense_nufft = (int)value;
  } else if (k == "symv_fused") {  // matrix mode: each product's reduction in the product's launch
    ctx->symv_fused = value != 0.0;
  } else if (k == "dense") {  // dense eigen-propagator engine: 0 off, 1 auto (cost model), 2 always
    if (!(value == 0 || value == 1 || value == 2)) return fail(ctx, DSE_ERR_ARG, "dense must be 0, 1 or 2");
    ctx->dense = (int)value;
  } else if (k == "small_chunk") {
    if (!(value >= 1 && value <= 1e6)) return fail(ctx, DSE_ERR_ARG, "small_chunk must be in 1..1e6");
    ctx->small_chunk = (int)value;
  } else if (k == "handoff_fences") {  // interval kernel: agent release/acquire around each hand-off
    ctx->hk.fences = value != 0.0;
  } else if (k == "spin_limit") {  // diagnostics: partner-flag polls per hand-off (< 0: always fail)
    if (!(value >= -1 && value <= 1 << 30)) return fail(ctx, DSE_ERR_ARG, "spin_limit must be in -1..2^30");
    ctx->hk.spin_limit = (int)value;
  } else if (k == "xcd_pairs") {
    ctx->xcd_pairs = value != 0.0;
  } else if (k == "span") {  // spanning registers: 0 off, 1..4 top bits (workgroups 2^s per register)
    if (!(value >= 0 && value <= kSpanMaxTop)) return fail(ctx, DSE_ERR_ARG, "span must be in 0..4");
    ctx->span = (int)value;
  } else if (k == "real") {  // real-component mode for registers of 13 / 14 qubits (imaginary drives)
    if (!(value == 0 || value == 1 || value == 2)) return fail(ctx, DSE_ERR_ARG, "real must be 0, 1 or 2");
    ctx->real_mode = (int)value;
  } else if (k == "span_tile") {  // spanning registers: tile bits L (0 off, -1 auto); n > L qubits span 2^(n-L) tiles
    if (!(value == 0 || value == -1 || (value >= 10 && value <= 13)))
      return fail(ctx, DSE_ERR_ARG, "span_tile must be -1, 0 or in 10..13");
    ctx->span_tile = (int)value;
  } else if (k == "span_rb") {  // amplitudes per thread of k_span: 2^span_rb (0: 512 threads)
    if (!(value >= 0 && value <= 3)) return fail(ctx, DSE_ERR_ARG, "span_rb must be in 0..3");
    ctx->span_rb = (int)value;
  } else if (k == "span_partial") {  // auto span policy: span the stiffest registers beside k_interval
    ctx->span_partial = value != 0.0;
  } else if (k == "span_chunks") {  // auto span policy: resident launches per interval for all-span
    if (!(value == 0.0 || value == 1.0 || value == 2.0)) return fail(ctx, DSE_ERR_ARG, "span_chunks must be 0, 1 or 2");
    ctx->span_chunks = (int)value;
  } else if (k == "span_partial_tile") {  // auto span policy, partial form: log2 tile (10, 11)
    if (!(value == 10.0 || value == 11.0)) return fail(ctx, DSE_ERR_ARG, "span_partial_tile must be 10 or 11");
    ctx->span_partial_tile = (int)value;
  } else if (k == "mixed_launch") {
    ctx->mixed_launch = value != 0.0;
  } else if (k == "obs_overlap") {
    ctx->obs_overlap = value != 0.0;
  } else if (k == "time_kernels") {
    if (!(value >= 0)) return fail(ctx, DSE_ERR_ARG, "time_kernels must be >= 0");
    ctx->time_every = (int)value;
  } else if (k == "ablate" || k == "real_ablate" || k == "span_ablate") {
    // diagnostics builds only (-DDSE_DIAG): skip kernel sections (results become wrong); process-wide
    const int m = (int)value;
    const hipError_t e = k == "ablate" ? (set_ablate(m) == hipSuccess ? set_ablate_interval(m) : hipErrorNotSupported)
                         : k == "real_ablate" ? set_real_ablate(m) : set_span_ablate(m);
    if (e == hipErrorNotSupported)
      return fail(ctx, DSE_ERR_ARG, "option " + k + " needs a diagnostics build of libdse (-DDSE_DIAG)");
    if (e != hipSuccess) return fail(ctx, DSE_ERR_ARG, "bad " + k + " mask");
  } else if (k == "probe_items") {  // diagnostics only: dse_time_step_kernel launches this many items
    ctx->probe_items = (int64_t)value;
  } else if (k == "max_degree") {
    if (!(value >= 1)) return fail(ctx, DSE_ERR_ARG, "max_degree must be >= 1");
    ctx->max_degree = value;
  } else {
    return fail(ctx, DSE_ERR_ARG, "unknown option " + k);
  }
  return DSE_OK;
}

}  // extern "C"

namespace {

// Validated host copy of one problem's tables (dse_add_problem / dse_add_problem_sharded).
int make_problem(dse_ctx* ctx, HostProblem& p, int n, const double* field, const double* zz,
                 const double* pair, const double* flip, double shift, uint64_t psi0_index,
                 uint64_t sea_mask, int rare_bit, double rare_z_const) {
  if (n < 1 || n > DSE_MAX_QUBITS) return fail(ctx, DSE_ERR_ARG, "n_qubits out of range 1..34");
  if (!field || !zz || !pair || !flip) return fail(ctx, DSE_ERR_ARG, "null coefficient table");
  const uint64_t dim = uint64_t(1) << n;
  if (psi0_index >= dim) return fail(ctx, DSE_ERR_ARG, "psi0_index >= 2^n");
  if ((sea_mask >> n) != 0) return fail(ctx, DSE_ERR_ARG, "sea_mask has bits >= n");
  if (rare_bit >= n || rare_bit < -1) return fail(ctx, DSE_ERR_ARG, "rare_bit out of range");
  p.n = n;
  p.field.assign(field, field + n);
  p.zz.assign(zz, zz + size_t(n) * n);
  p.pair.assign(pair, pair + size_t(n) * n);
  p.flip.assign(flip, flip + 4 * size_t(n));
  for (double v : p.field)
    if (!std::isfinite(v)) return fail(ctx, DSE_ERR_ARG, "non-finite field");
  for (double v : p.zz)
    if (!std::isfinite(v)) return fail(ctx, DSE_ERR_ARG, "non-finite zz");
  for (double v : p.pair)
    if (!std::isfinite(v)) return fail(ctx, DSE_ERR_ARG, "non-finite pair");
  for (int b = 0; b < n; ++b) {
    const double* f = &p.flip[4 * b];
    if (!(std::isfinite(f[0]) && std::isfinite(f[1]) && std::isfinite(f[2]) && std::isfinite(f[3])))
      return fail(ctx, DSE_ERR_ARG, "non-finite flip");
    const double scale = std::fabs(f[0]) + std::fabs(f[1]) + std::fabs(f[2]) + std::fabs(f[3]);
    if (std::fabs(f[0] - f[2]) > 1e-12 * scale || std::fabs(f[1] + f[3]) > 1e-12 * scale)
      return fail(ctx, DSE_ERR_ARG, "flip coefficients are not Hermitian (need c1 = conj(c0))");
  }
  if (!std::isfinite(shift)) return fail(ctx, DSE_ERR_ARG, "non-finite shift");
  p.shift = shift;
  p.psi0 = psi0_index;
  p.sea_mask = sea_mask;
  p.rare_bit = rare_bit;
  p.rare_z = rare_z_const;
  p.n_local = n;
  dse_spectral_bounds(n, p.field.data(), p.zz.data(), p.pair.data(), p.flip.data(), shift, &p.e_min, &p.e_max);
  {  // diagonal 4, drive flip 8 (complex coefficient), pair 4 on the half of the rows where it acts
    double f = 4.0;
    for (int b = 0; b < n; ++b)
      if (p.flip[4 * b] != 0.0 || p.flip[4 * b + 1] != 0.0) f += 8.0;
    for (int i = 0; i < n; ++i)
      for (int j = i + 1; j < n; ++j)
        if (p.pair[i * n + j] != 0.0) f += 2.0;
    p.flops_per_amp = f;
  }
  return DSE_OK;
}

}  // namespace

extern "C" {

int dse_add_problem(dse_ctx* ctx, int n, const double* field, const double* zz, const double* pair,
                    const double* flip, double shift, uint64_t psi0_index, uint64_t sea_mask,
                    int rare_bit, double rare_z_const) {
  if (!ctx) return DSE_ERR_ARG;
  HostProblem p;
  int rc = make_problem(ctx, p, n, field, zz, pair, flip, shift, psi0_index, sea_mask, rare_bit,
                        rare_z_const);
  if (rc) return rc;
  (void)hipSetDevice(ctx->device);
  (void)sync_all(ctx);
  free_device(ctx);  // device layout is rebuilt lazily
  ctx->probs.push_back(std::move(p));
  return (int)ctx->probs.size() - 1;
}

int dse_add_problem_sharded(dse_ctx* ctx, int n, const double* field, const double* zz,
                            const double* pair, const double* flip, double shift,
                            uint64_t psi0_index, uint64_t sea_mask, int rare_bit,
                            double rare_z_const, int shard_bits, int shard_rank) {
  if (!ctx) return DSE_ERR_ARG;
  if (shard_bits < 1 || shard_bits > kMaxShardBits)
    return fail(ctx, DSE_ERR_ARG, "shard_bits must be in 1..3");
  if (shard_rank < -1 || shard_rank >= (1 << shard_bits))
    return fail(ctx, DSE_ERR_ARG, "shard_rank out of range");
  HostProblem p;
  int rc = make_problem(ctx, p, n, field, zz, pair, flip, shift, psi0_index, sea_mask, rare_bit,
                        rare_z_const);
  if (rc) return rc;
  if (n - shard_bits < kMinTile + 1)
    return fail(ctx, DSE_ERR_ARG, "register too small to partition");
  if (shard_rank >= 0 && ((!ctx->comm && !ctx->xfn) || ctx->dist_world != (1 << shard_bits) ||
                          ctx->dist_rank != shard_rank))
    return fail(ctx, DSE_ERR_STATE, "dist shard needs dse_dist_init with world = 2^shard_bits "
                                    "and rank = shard_rank");
  p.shard_bits = shard_bits;
  p.n_local = n - shard_bits;
  (void)hipSetDevice(ctx->device);
  (void)sync_all(ctx);
  free_device(ctx);
  const int first = (int)ctx->probs.size();
  if (shard_rank >= 0) {
    p.shard_rank = shard_rank;
    p.dist = true;
    ctx->probs.push_back(std::move(p));
    return first;
  }
  for (int r = 0; r < (1 << shard_bits); ++r) {
    HostProblem q = p;
    q.shard_rank = r;
    q.group_first = first;
    ctx->probs.push_back(std::move(q));
  }
  return first;
}

int dse_dist_unique_id(unsigned char* id_out) {
  if (!id_out) return DSE_ERR_ARG;
  static_assert(sizeof(ncclUniqueId) == DSE_DIST_ID_BYTES, "ncclUniqueId size");
  ncclUniqueId id;
  if (ncclGetUniqueId(&id) != ncclSuccess) return DSE_ERR_HIP;
  std::memcpy(id_out, &id, sizeof(id));
  return DSE_OK;
}

int dse_dist_init(dse_ctx* ctx, int rank, int world, const unsigned char* id) {
  if (!ctx || !id) return DSE_ERR_ARG;
  if (world < 2 || world > kMaxShards || (world & (world - 1)) || rank < 0 || rank >= world)
    return fail(ctx, DSE_ERR_ARG, "world must be 2, 4 or 8 and 0 <= rank < world");
  if (ctx->comm || ctx->xfn) return fail(ctx, DSE_ERR_STATE, "dse_dist_init called twice");
  HIPC(hipSetDevice(ctx->device));
  ncclUniqueId uid;
  std::memcpy(&uid, id, sizeof(uid));
  const ncclResult_t r = ncclCommInitRank(&ctx->comm, world, uid, rank);
  if (r != ncclSuccess) {
    ctx->comm = nullptr;
    return fail(ctx, DSE_ERR_HIP, std::string("ncclCommInitRank: ") + ncclGetErrorString(r));
  }
  ctx->dist_rank = rank;
  ctx->dist_world = world;
  return DSE_OK;
}

int dse_dist_init_exchange(dse_ctx* ctx, int rank, int world, dse_exchange_fn fn, void* user) {
  if (!ctx || !fn) return DSE_ERR_ARG;
  if (world < 2 || world > kMaxShards || (world & (world - 1)) || rank < 0 || rank >= world)
    return fail(ctx, DSE_ERR_ARG, "world must be 2, 4 or 8 and 0 <= rank < world");
  if (ctx->comm || ctx->xfn) return fail(ctx, DSE_ERR_STATE, "dse_dist_init called twice");
  ctx->xfn = fn;
  ctx->xuser = user;
  ctx->dist_rank = rank;
  ctx->dist_world = world;
  return DSE_OK;
}

int dse_wht_plan(int n_local, int shard_bits, int tile_bits, int max_bits, int32_t* groups_out) {
  if (!groups_out || (tile_bits != 12 && tile_bits != 13) || n_local < 1 || n_local > kWhtMaxQubits ||
      shard_bits < 0 || shard_bits > kMaxShardBits)
    return DSE_ERR_ARG;
  WhtProb w;
  std::memset(&w, 0, sizeof(w));
  const int mb = max_bits & 0xff;  // bits 8-15: the MID group's in-page bits (option wht_mid_inpage)
  const int gb = mb ? std::min(mb, tile_bits - 2) : tile_bits - 2;
  const int G = wht_layout(n_local, shard_bits, tile_bits, gb, w, (max_bits >> 8) & 0xff);
  for (int g = 0; g < G; ++g) {
    groups_out[g * 14] = w.grp[g].c;
    for (int q = 0; q < tile_bits; ++q) groups_out[g * 14 + 1 + q] = w.grp[g].pos[q];
  }
  return G;
}

int64_t dse_problem_dim(const dse_ctx* ctx, int problem) {
  if (!ctx || problem < 0 || problem >= (int)ctx->probs.size()) return DSE_ERR_ARG;
  const HostProblem& P = ctx->probs[problem];
  return int64_t(1) << (P.dist ? P.n_local : P.n);
}

int dse_num_problems(const dse_ctx* ctx) { return ctx ? (int)ctx->probs.size() : DSE_ERR_ARG; }

int dse_clear(dse_ctx* ctx) {
  if (!ctx) return DSE_ERR_ARG;
  (void)hipSetDevice(ctx->device);
  (void)sync_all(ctx);
  free_device(ctx);
  ctx->probs.clear();
  return DSE_OK;
}

}  // extern "C"

namespace {

// The problems a hook call on `problem` acts on: the whole loopback group for its shard 0, else
// the problem itself.  Host vectors are the whole register (group) or the local shard.
int hook_members(dse_ctx* ctx, int problem, int* first, int* count) {
  if (problem < 0 || problem >= (int)ctx->probs.size()) return fail(ctx, DSE_ERR_ARG, "bad problem id");
  const HostProblem& P = ctx->probs[problem];
  *first = problem;
  *count = 1;
  if (P.shard_bits > 0 && !P.dist) {
    if (P.shard_rank != 0) return fail(ctx, DSE_ERR_ARG, "use shard 0 of a partitioned register");
    *count = 1 << P.shard_bits;
  }
  return DSE_OK;
}

// buf[1] = H buf[0] for the members [first, first + count) of one register (the engine that
// evolves it: Walsh-Hadamard passes or the step kernels; dist shards exchange first).
int apply_members(dse_ctx* ctx, int first, int count, hipStream_t st) {
  int rc;
  if ((rc = ensure_wht(ctx))) return rc;
  if (ctx->probs[first].wht_groups) {  // all members alike
    const HostProblem& P0 = ctx->probs[first];
    std::vector<std::pair<const int2*, int>> segs;
    for (int i = 0; i < count; ++i) segs.push_back({ctx->probs[first + i].d_items, (int)ctx->probs[first + i].n_tiles});
    std::vector<int> regs;
    if (P0.shard_bits > 0) regs.push_back(first);
    return wht_run(ctx, P0.L, P0.wht_groups, segs, regs, MODE_APPLY, 0, 0, 0, st);
  }
  if (ctx->probs[first].dist && (rc = dist_exchange(ctx, 0, 0, st))) return rc;
  for (int i = 0; i < count; ++i) {
    HostProblem& P = ctx->probs[first + i];
    HIPC(launch_step(P.L, MODE_APPLY, ctx->d_probs, P.d_items, (int)P.n_tiles, 0, 0, 0, st));
  }
  return DSE_OK;
}

// ---- small-register engine (dse_small.hip) ------------------------------------------------
// Problems with P.sm: Chebyshev coefficients per distinct interval length (one output per series),
// descriptors, then every launch of the whole evolve is enqueued on the engine's own stream
// (ceil((n_t - 1) / small_chunk) per register size); small_gather waits for them and fills obs_out.
int small_launch(dse_ctx* ctx, const double* t, int n_t, double tol, double* h_applications,
                 double* launches) {
  std::vector<int> sm;
  for (size_t pi = 0; pi < ctx->probs.size(); ++pi)
    if (ctx->probs[pi].sm) sm.push_back((int)pi);
  *h_applications = 0.0;
  *launches = 0.0;
  if (sm.empty()) return DSE_OK;
  if (!ctx->small_stream) HIPC(hipStreamCreateWithFlags(&ctx->small_stream, hipStreamNonBlocking));
  // distinct interval lengths -> sets
  std::vector<double> taus;
  std::vector<int> iv_set(std::max(n_t - 1, 1), 0);
  std::map<double, int> tau_id;
  for (int m = 0; m + 1 < n_t; ++m) {
    const double tau = t[m + 1] - t[m];
    auto it = tau_id.find(tau);
    if (it == tau_id.end()) {
      if (taus.size() >= 4096) return fail(ctx, DSE_ERR_ARG, "more than 4096 distinct output intervals");
      it = tau_id.emplace(tau, (int)taus.size()).first;
      taus.push_back(tau);
    }
    iv_set[m] = it->second;
  }
  if (taus.empty()) taus.push_back(0.0);
  const int n_sets = (int)taus.size();
  std::vector<SmallProb> desc(ctx->probs.size());
  std::memset(desc.data(), 0, desc.size() * sizeof(SmallProb));
  Arena arena;  // every problem's coefficients and degrees, one upload
  std::vector<std::pair<size_t, size_t>> aoff(ctx->probs.size());
  for (int pi : sm) {
    HostProblem& P = ctx->probs[pi];
    const double alpha = std::max(0.5 * (P.e_max - P.e_min), 1e-300);
    const double beta = 0.5 * (P.e_max + P.e_min);
    std::vector<std::vector<double>> J(n_sets);
    std::vector<int> deg(n_sets, 1);
    int kcap = 1;
    for (int sidx = 0; sidx < n_sets; ++sidx) {
      const double z = alpha * taus[sidx];
      const int kmax = (int)std::ceil(z + 12.0 * std::cbrt(z + 1.0) + 60.0);
      if (kmax > ctx->max_degree)
        return fail(ctx, DSE_ERR_CONVERGENCE, "Chebyshev degree " + std::to_string(kmax) +
                                                  " exceeds max_degree; use a finer output grid");
      J[sidx].resize(kmax + 1);
      if (dse_bessel_j(z, kmax, J[sidx].data(), tol, &deg[sidx]) != DSE_OK) return fail(ctx, DSE_ERR_ARG, "bessel failed");
      kcap = std::max(kcap, deg[sidx]);
    }
    for (int m = 0; m + 1 < n_t; ++m) *h_applications += deg[iv_set[m]];
    const int kcap1 = kcap + 1;
    std::vector<double2> a((size_t)n_sets * kcap1, make_double2(0.0, 0.0));
    for (int sidx = 0; sidx < n_sets; ++sidx) {
      const double ph = -beta * taus[sidx];
      const std::complex<double> e(std::cos(ph), std::sin(ph));
      std::complex<double> mi(1.0, 0.0);
      for (int k = 0; k <= deg[sidx]; ++k) {
        const std::complex<double> v = e * mi * ((k == 0 ? 1.0 : 2.0) * J[sidx][k]);
        a[(size_t)sidx * kcap1 + k] = make_double2(v.real(), v.imag());
        mi *= std::complex<double>(0.0, -1.0);
      }
    }
    aoff[pi].first = arena.add(a.data(), a.size() * sizeof(double2));
    aoff[pi].second = arena.add(deg.data(), deg.size() * sizeof(int));
    P.degree = kcap;
    const DevProb& d = ctx->h_desc[pi];
    SmallProb& q = desc[pi];
    q.state = P.buf[0];
    q.field = d.field;
    q.zz = d.zz;
    q.pair = nullptr;
    q.flip = nullptr;
    q.sea_mask = P.sea_mask;
    q.shift = P.shift;
    q.beta = beta;
    q.s1 = 1.0 / alpha;
    q.n = P.n;
    q.rare_bit = P.rare_bit;
    q.kcap1 = kcap1;
    q.n_t = n_t;
    P.final_bsel = 0;
  }
  {
    int rc = upload_arena(ctx, arena, &ctx->d_sm_coef, &ctx->sm_coef_cap, ctx->small_stream);
    if (rc) return rc;
  }
  for (int pi : sm) {
    HostProblem& P = ctx->probs[pi];
    P.sm_coef = reinterpret_cast<double2*>(ctx->d_sm_coef + aoff[pi].first);
    P.sm_deg = reinterpret_cast<int*>(ctx->d_sm_coef + aoff[pi].second);
    desc[pi].coef = P.sm_coef;
    desc[pi].deg = P.sm_deg;
  }
  // pair / flip tables: the problem's full n x n and 4n arrays (the device tables hold field, zz)
  size_t extra = 0;
  for (int pi : sm) extra += (size_t)ctx->probs[pi].n * ctx->probs[pi].n + 4 * (size_t)ctx->probs[pi].n;
  // aux ints: per register size the selection of problems, then the interval -> set map
  const size_t aux = ctx->probs.size() + (size_t)std::max(n_t - 1, 1) + 2 * extra + 64;
  if (aux > ctx->small_aux_cap) {
    if (ctx->d_small_aux) (void)hipFree(ctx->d_small_aux), ctx->d_small_aux = nullptr;
    if (hipMalloc(&ctx->d_small_aux, aux * sizeof(int)) != hipSuccess) return fail(ctx, DSE_ERR_OOM, "small-engine allocation failed");
    ctx->small_aux_cap = aux;
  }
  // tables after the ints (8-byte aligned)
  double* tab = reinterpret_cast<double*>(ctx->d_small_aux + ((ctx->probs.size() + std::max(n_t - 1, 1) + 1) & ~size_t(1)));
  {
    std::vector<double> ht;
    ht.reserve(extra);
    std::vector<size_t> off(ctx->probs.size(), 0);
    for (int pi : sm) {
      const HostProblem& P = ctx->probs[pi];
      off[pi] = ht.size();
      ht.insert(ht.end(), P.pair.begin(), P.pair.end());
      // drives as the engine's kernels see them (cos(pi/2) residue dropped, build_tables)
      for (int b = 0; b < P.n; ++b)
        for (int c = 0; c < 4; c += 2) {
          double re = P.flip[4 * b + c], im = P.flip[4 * b + c + 1];
          if (std::fabs(re) <= 1e-15 * std::hypot(re, im)) re = 0.0;
          ht.push_back(re);
          ht.push_back(im);
        }
    }
    if (!ht.empty()) HIPC(hipMemcpy(tab, ht.data(), ht.size() * sizeof(double), hipMemcpyHostToDevice));
    for (int pi : sm) {
      desc[pi].pair = tab + off[pi];
      desc[pi].flip = tab + off[pi] + (size_t)ctx->probs[pi].n * ctx->probs[pi].n;
    }
  }
  if (desc.size() > ctx->small_cap) {
    if (ctx->d_small) (void)hipFree(ctx->d_small), ctx->d_small = nullptr;
    if (hipMalloc(&ctx->d_small, desc.size() * sizeof(SmallProb)) != hipSuccess) return fail(ctx, DSE_ERR_OOM, "small-engine allocation failed");
    ctx->small_cap = desc.size();
  }
  HIPC(hipMemcpy(ctx->d_small, desc.data(), desc.size() * sizeof(SmallProb), hipMemcpyHostToDevice));
  const size_t outn = ctx->probs.size() * (size_t)n_t * 8;
  if (outn > ctx->small_out_cap) {
    if (ctx->d_small_out) (void)hipFree(ctx->d_small_out), ctx->d_small_out = nullptr;
    if (hipMalloc(&ctx->d_small_out, outn * sizeof(double)) != hipSuccess) return fail(ctx, DSE_ERR_OOM, "small-engine output allocation failed");
    ctx->small_out_cap = outn;
  }
  // selections per register size, then the interval -> set map
  std::vector<int> ints;
  std::vector<std::pair<int, std::pair<int, int>>> groups;  // n -> (offset, count)
  for (int n = 1; n <= kSmallMaxQubits; ++n) {
    const int o = (int)ints.size();
    for (int pi : sm)
      if (ctx->probs[pi].n == n) ints.push_back(pi);
    if ((int)ints.size() > o) groups.push_back({n, {o, (int)ints.size() - o}});
  }
  const int iv_off = (int)ints.size();
  ints.insert(ints.end(), iv_set.begin(), iv_set.end());
  HIPC(hipMemcpy(ctx->d_small_aux, ints.data(), ints.size() * sizeof(int), hipMemcpyHostToDevice));
  hipStream_t st = ctx->small_stream;
  for (const auto& g : groups)
    HIPC(launch_small_obs0(g.first, ctx->d_small, ctx->d_small_aux + g.second.first, g.second.second,
                           ctx->d_small_out, st));
  const int chunk = std::max(1, ctx->small_chunk);
  for (int m0 = 0; m0 + 1 < n_t; m0 += chunk) {
    const int cnt = std::min(chunk, n_t - 1 - m0);
    for (const auto& g : groups) {
      HIPC(launch_small(g.first, ctx->d_small, ctx->d_small_aux + g.second.first, g.second.second, m0,
                        cnt, ctx->d_small_aux + iv_off, ctx->d_small_out, st));
      *launches += 1.0;
    }
  }
  return DSE_OK;
}

int small_gather(dse_ctx* ctx, int n_t, double* obs_out) {
  bool any = false;
  for (auto& P : ctx->probs) any = any || P.sm;
  if (!any) return DSE_OK;
  HIPC(hipStreamSynchronize(ctx->small_stream));
  std::vector<double> h(ctx->probs.size() * (size_t)n_t * 8);
  HIPC(hipMemcpy(h.data(), ctx->d_small_out, h.size() * sizeof(double), hipMemcpyDeviceToHost));
  for (size_t pi = 0; pi < ctx->probs.size(); ++pi) {
    const HostProblem& P = ctx->probs[pi];
    if (!P.sm) continue;
    for (int ti = 0; ti < n_t; ++ti)
      finish_obs(P, h.data() + (pi * (size_t)n_t + ti) * 8, obs_out + pi * DSE_N_OBS * (size_t)n_t + ti,
                 (size_t)n_t);
  }
  return DSE_OK;
}

// ---- dense eigen-propagator engine (dse_dense.h) ------------------------------------------
// A register qualifies when it is whole (not partitioned), holds at most kDenseMaxQubits qubits
// and its drive coefficients are all purely imaginary (H' = D H D^dagger is real) or all real.
bool dense_eligible(const HostProblem& P) {
  if (P.shard_bits != 0 || P.n_local > kDenseMaxQubits) return false;
  if (P.imag) return true;
  for (int b = 0; b < P.n; ++b)
    if (P.flip[4 * b + 1] != 0.0 || P.flip[4 * b + 3] != 0.0) return false;
  return true;
}

// eig_impl 1 from 2^11 amplitudes: eig_sym_lower (rocSOLVER's tridiagonalisation below 2^13, the
// half-matrix one above; dstedc; the 256-reflector back-transformation) against dsyevd measured
// 0.46 vs 0.68 s at 2^13, 2.35 vs 4.12 s at 2^14 (profiles/r03/sytrd_probe.jsonl,
// profiles/r03/ab/sytrd_column_kernels_ab.jsonl)
constexpr size_t kEigHalfMinDim = 2048;
// eig_impl 1 from 2^13: eig_sym_2stage (dse_eig2.hip: band reduction, bulge chase, dstedc, Q2, Q1)
// measured 1.43 s against eig_sym_lower's 2.25 s at 2^14, 0.428 against 0.430 s at 2^13
// (profiles/r04/eig_one_vs_two_stage.jsonl); an N = 14 point of the 30 s grid (two 2^14 registers,
// one 2^13, three solver streams) 3.46-3.75 s with the 2^13 one two-stage against 3.62-3.72 s
// one-stage (profiles/r04/eig_impl_point_ab.jsonl).  Per-register output GEMMs (a register's outputs
// as soon as it is solved, instead of a job's) measured 3.66-3.77 s against 3.45-3.62 s and were
// dropped (profiles/r04/eig_point_outputs_per_register.jsonl).
constexpr size_t kEig2MinDim = 8192;

// Seconds of device time, by the measured rates: the Chebyshev propagator at ~15 TF/s of its
// algorithmic FP64 work (the N = 14 bench runs at 16.5 chip-level) with ~25 extra terms per
// output interval, against one eigendecomposition plus the Psi' GEMM at ~40 TF/s and the
// observable pass.  The eigendecomposition: dsyevd (profiles/r03/probe.jsonl: 0.15 / 0.68 / 4.1 s
// at dim 4096 / 8192 / 16384, 3 ms for 39 registers of dim 128 together: 6.4e-13 dim^3 + 4.9e-9
// dim^2, + 20 ms from dim 1024 up), or with eig_impl from 2^11 eig_sym_lower (0.13 / 0.46 / 2.35
// s: 2.96e-13 dim^3 + 3.73e-9 dim^2 + 0.047).  The long reference grid (30 s, 20 000 outputs)
// goes dense at every register size; the 1 ms head-to-head grid at N = 14 and config 2 (N = 12,
// 2 ms) stay on Chebyshev.
bool dense_cheaper(const HostProblem& P, const double* t, int n_t, int eig_impl) {
  if (n_t < 2) return false;
  const double dim = std::ldexp(1.0, P.n_local);
  const double alpha = 0.5 * (P.e_max - P.e_min);
  const double terms = alpha * (t[n_t - 1] - t[0]) + 25.0 * (n_t - 1);
  const double cheb = terms * dim * (P.flops_per_amp > 0 ? P.flops_per_amp : 300.0) / 15e12;
  // the solver eig_impl takes for this size (dense_run's half_min / two_min)
  const size_t d = (size_t)dim;
  const size_t half_min = eig_impl == 1 ? kEigHalfMinDim : (eig_impl == 2 || eig_impl == 3) ? 1024 : SIZE_MAX;
  const size_t two_min = eig_impl == 1 ? kEig2MinDim : eig_impl == 3 ? 1024 : SIZE_MAX;
  double eig = d >= half_min ? 0.047 + 2.96e-13 * dim * dim * dim + 3.73e-9 * dim * dim
                             : 1e-4 + 6.4e-13 * dim * dim * dim + 4.9e-9 * dim * dim + (dim >= 1024 ? 2e-2 : 0.0);
  if (d >= two_min && dim >= 16384.0) eig *= 0.61;  // two-stage: 1.43 vs 2.35 s at 2^14 (level at 2^13)
  const double dense = eig + 4.0 * dim * dim * n_t / 40e12 + (double)n_t * dim * P.n_local * 32.0 / 2e12;
  return dense < cheb;
}

struct DevArena {  // device allocations of one dense_run, freed on every exit path
  std::vector<void*> ptrs;
  ~DevArena() { free_all(); }
  void free_all() {
    for (void* p : ptrs) (void)hipFree(p);
    ptrs.clear();
  }
  template <typename T>
  T* get(size_t count) {
    void* p = nullptr;
    if (hipMalloc(&p, std::max<size_t>(count, 1) * sizeof(T)) != hipSuccess) return nullptr;
    ptrs.push_back(p);
    return static_cast<T*>(p);
  }
};

// Every problem with P.dn: H' built on the device, diagonalised (rocSOLVER dsyevd, batched for
// registers of equal size below 2^10 amplitudes, one call per register above), outputs in blocks of
// TB times as Psi' = V [cos | -sin] (rocBLAS dgemm_strided_batched), observables and the final
// state from Psi'.  Work proceeds in rounds that fit 60% of the free device memory: every job
// (registers of one size) of a round is built, then all its eigendecompositions run on up to
// eig_streams solver streams at once (largest first, across sizes), then the output GEMMs.
// Blocking; writes obs_out.

struct DenseJob {
  int n = 0, cnt = 0, TB = 1;
  size_t dim = 0, pstride = 0;
  std::vector<int> list;  // problem indices
  DevArena ba;
  double *V = nullptr, *lam = nullptr, *lam_lo = nullptr, *E = nullptr, *Pm = nullptr, *Psi = nullptr, *obs = nullptr;
  double* diag_dd = nullptr;
  rocblas_int* info = nullptr;
  DenseProb* d_desc = nullptr;
};

int dense_run(dse_ctx* ctx, const double* t, int n_t, double* obs_out, double* ms_all, double* ms_eig) {
  std::vector<int> order;  // dense problems, by register size
  {
    std::map<int, std::vector<int>> by_n;
    for (size_t pi = 0; pi < ctx->probs.size(); ++pi)
      if (ctx->probs[pi].dn) by_n[ctx->probs[pi].n_local].push_back((int)pi);
    for (auto& kv : by_n) order.insert(order.end(), kv.second.begin(), kv.second.end());
  }
  if (order.empty()) return DSE_OK;
  const auto c0 = std::chrono::steady_clock::now();
  double eig_ms = 0.0;
  if (!ctx->dense_stream) HIPC(hipStreamCreateWithFlags(&ctx->dense_stream, hipStreamNonBlocking));
  if (!ctx->blas && rocblas_create_handle(&ctx->blas) != rocblas_status_success)
    return fail(ctx, DSE_ERR_HIP, "rocblas_create_handle failed");
  hipStream_t st = ctx->dense_stream;
  if (rocblas_set_stream(ctx->blas, st) != rocblas_status_success)
    return fail(ctx, DSE_ERR_HIP, "rocblas_set_stream failed");
  DevArena arena;
  std::vector<double> tau(n_t);
  for (int i = 0; i < n_t; ++i) tau[i] = t[i] - t[0];
  double* d_tau = arena.get<double>(n_t);
  if (!d_tau) return fail(ctx, DSE_ERR_OOM, "dense engine: allocation failed");
  HIPC(hipMemcpyAsync(d_tau, tau.data(), n_t * sizeof(double), hipMemcpyHostToDevice, st));
  // the non-uniform FFT's grid and device buffers (sized for the largest eligible register), or none
  ctx->nufft_problems = 0;
  NufftGrid ngrid;
  NufftScratch nscr;
  DevArena nufft_arena;
  bool use_nufft = false;
  if (ctx->dense_nufft && (ctx->dense_nufft == 2 || n_t >= kNufftMinOutputs)) {
    size_t nmax = 0;
    double lam_max = 0.0;
    for (int pi : order) {
      const HostProblem& P = ctx->probs[pi];
      if ((size_t(1) << P.n_local) < (size_t)kNufftMinDim && ctx->dense_nufft != 2) continue;
      nmax = std::max(nmax, size_t(1) << P.n_local);
      lam_max = std::max({lam_max, std::fabs(P.e_min - P.shift), std::fabs(P.e_max - P.shift)});
    }
    if (nmax && nufft_grid(tau.data(), n_t, lam_max, ngrid)) {
      nscr.U = nufft_arena.get<double2>((size_t)ngrid.M * nmax);
      nscr.U2 = nufft_arena.get<double2>((size_t)ngrid.M * nmax);
      nscr.c = nufft_arena.get<double>(nmax);
      nscr.off = nufft_arena.get<int>((size_t)ngrid.M + 1);
      nscr.nnz_cap = nmax * (size_t)(kNufftW + 2);
      nscr.src = nufft_arena.get<int>(nscr.nnz_cap);
      nscr.wt = nufft_arena.get<double>(4 * nscr.nnz_cap);
      nscr.scale = nufft_arena.get<double>(n_t);
      nscr.delta = nufft_arena.get<double>(n_t);
      use_nufft = nscr.U && nscr.U2 && nscr.c && nscr.off && nscr.src && nscr.wt && nscr.scale && nscr.delta;
      if (use_nufft) {
        HIPC(hipMemcpyAsync(nscr.scale, ngrid.scale.data(), n_t * sizeof(double), hipMemcpyHostToDevice, st));
        HIPC(hipMemcpyAsync(nscr.delta, ngrid.delta.data(), n_t * sizeof(double), hipMemcpyHostToDevice, st));
        HIPC(hipStreamSynchronize(st));
      } else {  // no room: the GEMM outputs
        (void)hipGetLastError();
        nufft_arena.free_all();
      }
    }
  }
  double out_ms = 0.0;
  struct EigScratch {
    double *A = nullptr, *tau = nullptr, *work = nullptr;
  };
  std::unique_ptr<DevArena> scr_arena;
  std::vector<EigScratch> scr;
  size_t scr_dim = 0, scr_work = 0;
  size_t idx = 0;
  while (idx < order.size()) {
    // ---- round: jobs while 60% of the free memory lasts (at least one register) ----
    size_t free_b = 0, total_b = 0;
    HIPC(hipMemGetInfo(&free_b, &total_b));
    const double budget = 0.6 * (double)free_b;
    double used = 0.0;
    std::vector<std::unique_ptr<DenseJob>> jobs;
    while (idx < order.size()) {
      const int n = ctx->probs[order[idx]].n_local;
      const size_t dim = size_t(1) << n;
      // outputs per block: P and Psi' of a problem take 2 x dim x 2 TB doubles (<= 256 MiB each)
      const int TB = (int)std::max<size_t>(1, std::min<size_t>((size_t)n_t, (size_t(256) << 20) / (16 * dim)));
      const size_t pstride = dim * 2 * (size_t)TB;
      const double per = (double)((dim * dim + 2 * pstride + 5 * dim + (size_t)n_t * 8 + 2 * n * n + 4 * n) * sizeof(double));
      size_t same = 0;
      while (idx + same < order.size() && ctx->probs[order[idx + same]].n_local == n) ++same;
      size_t cnt = (size_t)std::max(0.0, (budget - used) / per);
      if (cnt == 0 && !jobs.empty()) break;
      cnt = std::max<size_t>(1, std::min(cnt, same));
      auto J = std::make_unique<DenseJob>();
      J->n = n, J->dim = dim, J->TB = TB, J->pstride = pstride, J->cnt = (int)cnt;
      J->list.assign(order.begin() + idx, order.begin() + idx + cnt);
      DevArena& ba = J->ba;
      J->V = ba.get<double>(dim * dim * cnt);
      J->lam = ba.get<double>(dim * cnt);
      J->lam_lo = ba.get<double>(dim * cnt);
      J->diag_dd = ba.get<double>(2 * dim * cnt);
      J->E = ba.get<double>(dim * cnt);
      J->info = ba.get<rocblas_int>(cnt);
      J->Pm = ba.get<double>(pstride * cnt);
      J->Psi = ba.get<double>(pstride * cnt);
      J->obs = ba.get<double>((size_t)n_t * 8 * cnt);
      const size_t tsz = (size_t)(2 * n * n + 5 * n);
      double* tabs = ba.get<double>(tsz * cnt);
      J->d_desc = ba.get<DenseProb>(cnt);
      if (!J->V || !J->lam || !J->lam_lo || !J->diag_dd || !J->E || !J->info || !J->Pm || !J->Psi || !J->obs || !tabs || !J->d_desc) {
        if (!jobs.empty()) break;  // this round is full: the register waits for the next one
        return fail(ctx, DSE_ERR_OOM, "dense engine: allocation failed (dim " + std::to_string(dim) + ")");
      }
      std::vector<double> htabs(tsz * cnt, 0.0);
      std::vector<DenseProb> desc(cnt);
      for (size_t i = 0; i < cnt; ++i) {
        const HostProblem& P = ctx->probs[J->list[i]];
        double* h = htabs.data() + tsz * i;
        std::copy(P.field.begin(), P.field.begin() + n, h);
        std::copy(P.zz.begin(), P.zz.begin() + n * n, h + n);
        std::copy(P.pair.begin(), P.pair.begin() + n * n, h + n + n * n);
        std::copy(P.flip.begin(), P.flip.begin() + 4 * n, h + n + 2 * n * n);
        double* d = tabs + tsz * i;
        DenseProb& D = desc[i];
        D.n = n;
        D.rot = P.imag ? 1 : 0;
        D.sea_mask = P.sea_mask;
        D.rare_bit = P.rare_bit;
        D.n_sea = __builtin_popcountll(P.sea_mask);
        D.x0 = P.psi0;
        D.shift = P.shift;
        D.field = d;
        D.zz = d + n;
        D.pair = d + n + n * n;
        D.flip = d + n + 2 * n * n;
        D.V = J->V + dim * dim * i;
        D.lam = J->lam + dim * i;
        D.lam_lo = J->lam_lo + dim * i;
        D.diag_dd = J->diag_dd + 2 * dim * i;
        D.refine = ctx->dense_refine;
        D.obs = J->obs + (size_t)n_t * 8 * i;
        D.final_state = P.buf[0];
      }
      HIPC(hipMemcpyAsync(tabs, htabs.data(), htabs.size() * sizeof(double), hipMemcpyHostToDevice, st));
      HIPC(hipMemcpyAsync(J->d_desc, desc.data(), desc.size() * sizeof(DenseProb), hipMemcpyHostToDevice, st));
      HIPC(hipMemsetAsync(J->V, 0, dim * dim * cnt * sizeof(double), st));
      HIPC(launch_dense_h(J->d_desc, (int)cnt, (int)dim, st));
      HIPC(hipStreamSynchronize(st));  // the host tables may go
      used += per * (double)cnt;
      idx += cnt;
      jobs.push_back(std::move(J));
    }
    // ---- the round's eigendecompositions: one task per large register, one batched task per job of
    // small ones, largest first, over up to eig_streams solver streams ----
    const auto e0 = std::chrono::steady_clock::now();
    struct Task {
      DenseJob* j;
      int i;  // register within the job; -1: the whole job, batched
    };
    std::vector<Task> tasks;
    for (auto& J : jobs) {
      if (J->dim >= 1024)
        for (int i = 0; i < J->cnt; ++i) tasks.push_back({J.get(), i});
      else
        tasks.push_back({J.get(), -1});
    }
    std::stable_sort(tasks.begin(), tasks.end(), [](const Task& x, const Task& y) { return x.j->dim > y.j->dim; });
    const int K = std::max(1, std::min(ctx->eig_streams, (int)tasks.size()));
    while ((int)ctx->eig_h.size() < K) {
      hipStream_t es = nullptr;
      rocblas_handle eh = nullptr;
      HIPC(hipStreamCreateWithFlags(&es, hipStreamNonBlocking));
      if (rocblas_create_handle(&eh) != rocblas_status_success || rocblas_set_stream(eh, es) != rocblas_status_success) {
        if (eh) (void)rocblas_destroy_handle(eh);
        (void)hipStreamDestroy(es);
        return fail(ctx, DSE_ERR_HIP, "rocblas handle for the eigensolver streams failed");
      }
      ctx->eig_st.push_back(es);
      ctx->eig_h.push_back(eh);
    }
    // half-matrix eigensolver scratch per solver stream: a copy of H' (the solver's A; V receives
    // the eigenvectors), tau and the tridiagonalisation workspace, sized for the round's largest
    // such register; kept across rounds
    size_t half_min = ctx->eig_impl == 2 ? 1024 : ctx->eig_impl == 1 ? kEigHalfMinDim : ctx->eig_impl == 3 ? 1024 : SIZE_MAX;
    const size_t two_min = ctx->eig_impl == 3 ? 1024 : ctx->eig_impl == 1 ? kEig2MinDim : SIZE_MAX;
    size_t half_dim = 0, two_dim = 0;
    for (const Task& T : tasks)
      if (T.i >= 0 && T.j->dim >= half_min) {
        half_dim = std::max(half_dim, T.j->dim);
        if (T.j->dim >= two_min) two_dim = std::max(two_dim, T.j->dim);
      }
    const size_t work_b = std::max(sytrd_workspace((int)half_dim), two_dim ? eig2_workspace((int)two_dim) : (size_t)0);
    if (half_dim > scr_dim || work_b > scr_work) {
      scr.clear();
      scr_arena.reset(new DevArena);
      scr_dim = 0, scr_work = 0;
      for (int w = 0; w < K; ++w) {
        EigScratch S;
        S.A = scr_arena->get<double>(half_dim * half_dim);
        S.tau = scr_arena->get<double>(half_dim);
        S.work = scr_arena->get<double>(work_b / sizeof(double) + 1);
        if (!S.A || !S.tau || !S.work) break;
        scr.push_back(S);
      }
      if ((int)scr.size() == K) {
        scr_dim = half_dim, scr_work = work_b;
      } else {  // no room beside the round's jobs: dsyevd in place
        (void)hipGetLastError();
        scr.clear();
        scr_arena.reset();
        half_min = SIZE_MAX;
      }
    }
    // the workers take tasks largest first; a job whose last register is solved goes to the output
    // queue, and this thread runs its output GEMMs (dense_stream) while the other solves go on
    // (outputs per register as each solve ends measured the same: 3.51-3.56 s per N = 14 point
    // either way over 16 points, profiles/r05/fullsweep_outputs_ab.jsonl)
    std::atomic<size_t> next{0};
    std::atomic<bool> abort_all{false};
    std::vector<rocblas_status> wst(K, rocblas_status_success);
    std::vector<int> wrc(K, 0);
    std::vector<hipError_t> werr(K, hipSuccess);
    std::mutex qm;
    std::condition_variable qcv;
    std::deque<DenseJob*> ready;        // jobs whose registers are all solved: their outputs next
    std::map<DenseJob*, int> pending;  // per job: its registers not yet solved
    for (const Task& T : tasks) pending[T.j] += 1;
    int workers_left = K;
    auto e1 = e0;
    auto worker = [&](int w) {
      for (size_t ti = next++; ti < tasks.size() && !abort_all; ti = next++) {
        const Task& T = tasks[ti];
        DenseJob& J = *T.j;
        const rocblas_int dim = (rocblas_int)J.dim;
        if (T.i >= 0 && J.dim >= half_min) {
          const size_t i = (size_t)T.i;
          double* Vi = J.V + J.dim * J.dim * i;
          werr[w] = hipMemcpyAsync(scr[w].A, Vi, J.dim * J.dim * sizeof(double), hipMemcpyDeviceToDevice,
                                   ctx->eig_st[w]);
          if (werr[w] == hipSuccess && J.dim >= two_min) {
            wrc[w] = eig_sym_2stage(ctx->eig_h[w], ctx->eig_st[w], dim, scr[w].A, dim, J.lam + J.dim * i, Vi, dim,
                                    J.E + J.dim * i, scr[w].work, J.info + i, ctx->n_cu, ctx->eig_spin);
            if (wrc[w] == kEig2PollTimeout) {  // a poll gave up (workgroups not co-resident): H' again, dsyevd
              ctx->eig_fallbacks++;
              wrc[w] = 0;
              werr[w] = hipMemsetAsync(Vi, 0, J.dim * J.dim * sizeof(double), ctx->eig_st[w]);
              if (werr[w] == hipSuccess) werr[w] = launch_dense_h(J.d_desc + i, 1, (int)J.dim, ctx->eig_st[w]);
              if (werr[w] == hipSuccess)
                wst[w] = rocsolver_dsyevd(ctx->eig_h[w], rocblas_evect_original, rocblas_fill_upper, dim, Vi, dim,
                                          J.lam + J.dim * i, J.E + J.dim * i, J.info + i);
            }
          }
          else if (werr[w] == hipSuccess)
            wrc[w] = eig_sym_lower(ctx->eig_h[w], ctx->eig_st[w], dim, scr[w].A, dim, J.lam + J.dim * i, Vi, dim,
                                   J.E + J.dim * i, scr[w].tau, scr[w].work, J.info + i);
        } else if (T.i >= 0) {
          const size_t i = (size_t)T.i;
          wst[w] = rocsolver_dsyevd(ctx->eig_h[w], rocblas_evect_original, rocblas_fill_upper, dim,
                                    J.V + J.dim * J.dim * i, dim, J.lam + J.dim * i, J.E + J.dim * i, J.info + i);
        } else {
          wst[w] = rocsolver_dsyevd_strided_batched(ctx->eig_h[w], rocblas_evect_original, rocblas_fill_upper, dim,
                                                    J.V, dim, (rocblas_stride)(J.dim * J.dim), J.lam,
                                                    (rocblas_stride)J.dim, J.E, (rocblas_stride)J.dim, J.info, J.cnt);
        }
        const hipError_t se = hipStreamSynchronize(ctx->eig_st[w]);
        if (werr[w] == hipSuccess) werr[w] = se;
        if (werr[w] != hipSuccess || wst[w] != rocblas_status_success || wrc[w] != 0) {
          abort_all = true;
          break;
        }
        std::lock_guard<std::mutex> lk(qm);
        if (--pending[&J] == 0) {
          ready.push_back(&J);
          qcv.notify_one();
        }
      }
      std::lock_guard<std::mutex> lk(qm);
      if (--workers_left == 0) e1 = std::chrono::steady_clock::now();
      qcv.notify_one();
    };
    auto outputs = [&](DenseJob& J) -> int {  // every register of job J
      const int i0 = 0, cnt = J.cnt, TB = J.TB;
      const size_t dim = J.dim, pstride = J.pstride;
      const DenseProb* desc = J.d_desc + i0;
      double* const V = J.V + dim * dim * i0;
      double* const Pm = J.Pm + pstride * i0;
      double* const Psi = J.Psi + pstride * i0;
      std::vector<rocblas_int> hinfo(cnt);
      HIPC(hipMemcpyAsync(hinfo.data(), J.info + i0, cnt * sizeof(rocblas_int), hipMemcpyDeviceToHost, st));
      HIPC(hipStreamSynchronize(st));
      for (int i = 0; i < cnt; ++i)
        if (hinfo[i] != 0)
          return fail(ctx, DSE_ERR_CONVERGENCE, "dense engine: eigensolver did not converge (info " +
                                                    std::to_string(hinfo[i]) + ")");
      const double one = 1.0, zero = 0.0;
      const auto o0 = std::chrono::steady_clock::now();
      if (ctx->dense_refine) HIPC(launch_dense_rq(desc, cnt, (int)dim, st));
      if (use_nufft && (dim >= (size_t)kNufftMinDim || ctx->dense_nufft == 2)) {  // per register, Psi' interleaved
        for (int i = 0; i < cnt; ++i) {
          const DenseProb* di = desc + i;
          auto per_block = [&](int tb0, int tb) -> int {
            if (launch_dense_obs_c(di, (int)dim, Psi, tb, tb0, st) != hipSuccess) return -1;
            if (tb0 + tb == n_t && launch_dense_final_c(di, (int)dim, Psi, tb, tau[n_t - 1], st) != hipSuccess)
              return -1;
            return 0;
          };
          const int rc = nufft_outputs(ctx->nufft, st, ngrid, nscr, V + dim * dim * i, J.lam + dim * (i0 + i),
                                       J.lam_lo + dim * (i0 + i), ctx->probs[J.list[i0 + i]].psi0, (int)dim, Psi, TB,
                                       per_block);
          if (rc) return fail(ctx, DSE_ERR_HIP, "dense engine: non-uniform FFT outputs failed (" + std::to_string(rc) + ")");
          ctx->nufft_problems++;
        }
      } else
      for (int tb0 = 0; tb0 < n_t; tb0 += TB) {
        const int tb = std::min(TB, n_t - tb0);
        HIPC(launch_dense_phase(desc, cnt, (int)dim, d_tau + tb0, tb, Pm, pstride, st));
        const rocblas_status rs = rocblas_dgemm_strided_batched(
            ctx->blas, rocblas_operation_none, rocblas_operation_none, (rocblas_int)dim, 2 * tb, (rocblas_int)dim, &one,
            V, (rocblas_int)dim, (rocblas_stride)(dim * dim), Pm, (rocblas_int)dim, (rocblas_stride)pstride, &zero,
            Psi, (rocblas_int)dim, (rocblas_stride)pstride, cnt);
        if (rs != rocblas_status_success)
          return fail(ctx, DSE_ERR_HIP, "rocblas dgemm failed (status " + std::to_string((int)rs) + ")");
        HIPC(launch_dense_obs(desc, cnt, (int)dim, Psi, pstride, tb, tb0, st));
        if (tb0 + tb == n_t) HIPC(launch_dense_final(desc, cnt, (int)dim, Psi, pstride, tb, tau[n_t - 1], st));
      }
      std::vector<double> h((size_t)n_t * 8 * cnt);
      HIPC(hipMemcpyAsync(h.data(), J.obs + (size_t)n_t * 8 * i0, h.size() * sizeof(double), hipMemcpyDeviceToHost, st));
      HIPC(hipStreamSynchronize(st));
      out_ms += std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - o0).count();
      for (int i = 0; i < cnt; ++i) {
        const int pi = J.list[i0 + i];
        for (int ti = 0; ti < n_t; ++ti)
          finish_obs(ctx->probs[pi], h.data() + ((size_t)i * n_t + ti) * 8,
                     obs_out + (size_t)pi * DSE_N_OBS * n_t + ti, (size_t)n_t);
      }
      return DSE_OK;
    };
    std::vector<std::thread> th;
    for (int w = 0; w < K; ++w) th.emplace_back(worker, w);
    int orc = DSE_OK;
    size_t done = 0;
    const size_t n_out_tasks = jobs.size();
    while (done < n_out_tasks) {
      DenseJob* J = nullptr;
      {
        std::unique_lock<std::mutex> lk(qm);
        qcv.wait(lk, [&] { return !ready.empty() || workers_left == 0; });
        if (ready.empty()) break;  // the workers stopped early: an error below
        J = ready.front();
        ready.pop_front();
      }
      orc = outputs(*J);
      if (orc != DSE_OK) {
        abort_all = true;
        break;
      }
      ++done;
    }
    for (auto& x : th) x.join();
    if (orc != DSE_OK) return orc;
    for (int w = 0; w < K; ++w) {
      if (werr[w] != hipSuccess)
        return fail(ctx, DSE_ERR_HIP, std::string("eigensolver stream: ") + hipGetErrorString(werr[w]));
      if (wst[w] != rocblas_status_success)
        return fail(ctx, DSE_ERR_HIP, "rocsolver dsyevd failed (status " + std::to_string((int)wst[w]) + ")");
      if (wrc[w] != 0)
        return fail(ctx, DSE_ERR_HIP, "half-matrix eigensolver failed (step " + std::to_string(-wrc[w]) + ")");
    }
    if (done < n_out_tasks) return fail(ctx, DSE_ERR_HIP, "dense engine: eigensolver workers stopped early");
    eig_ms += std::chrono::duration<double, std::milli>(e1 - e0).count();
  }
  if (ms_all) *ms_all = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - c0).count();
  if (ms_eig) *ms_eig = eig_ms;
  ctx->dense_out_ms = out_ms;
  return DSE_OK;
}

// ---- propagator-matrix mode ----------------------------------------------------------------
// One evolution alone in a context runs its Chebyshev terms on one workgroup per tile: a chain of
// ~alpha t_final + 30 (n_t - 1) terms at ~11 us each on one CU (config 2, N = 12: ~9e3 terms,
// ~0.1 s) while the other 255 CUs idle.  On a uniform grid the whole evolution is psi_j =
// U^j psi_0 with U = exp(-iH dt): U's 2^n columns are independent Chebyshev evolutions over one
// interval (k_interval in column mode: 2^n workgroups, the whole chip), then the outputs are
// n_t - 1 dependent products psi_{j+1} = U psi_j (rocBLAS zgemv, HBM-bound) and one observable
// launch over all states.
bool matrix_eligible(const HostProblem& P, const double* t, int n_t, double* dt_out) {
  if (P.shard_bits != 0 || P.n_tiles != 1 || !interval_supported(P.L) || n_t < 17) return false;
  if (P.n_local > 13) return false;
  const double dt = (t[n_t - 1] - t[0]) / (n_t - 1);
  for (int i = 1; i < n_t; ++i)
    if (std::fabs((t[i] - t[i - 1]) - dt) > 1e-9 * dt) return false;
  *dt_out = dt;
  return true;
}

// seconds: the chain on one workgroup (~11.4 us per term at 2^12 amplitudes, linear in the tile)
// against the column build spread over the chip plus n_t - 1 matrix-vector products.  Real build
// (k_ucols, imaginary or real drives): ~10 us per term and workgroup at 2^12 amplitudes with two
// workgroups per CU (one at 2^13, LDS), products over the half matrix at ~5 TB/s plus ~5 us for the
// reduction launch; complex build (k_interval column mode): as the chain's terms, two workgroups
// per CU below 2^13, products over the whole matrix (zgemv) at ~3 TB/s.
// device bytes of matrix_run for register P on n_t outputs (U's stored tiles or columns, the
// states, the products' partials; the small tables are within the rounding)
double matrix_bytes(const HostProblem& P, int n_t) {
  const double dim = std::ldexp(1.0, P.n_local);
  const double nb = dim / kSymvBlock;
  const bool real = dense_eligible(P) && ucols_supported(P.L) && P.n_local == P.L;
  const double u = real ? nb * (nb + 1) / 2 * kSymvBlock * kSymvBlock : dim * dim;
  return 16.0 * (u + dim * n_t + (real ? nb * dim : 0.0)) + (1 << 20);
}

bool matrix_cheaper(const HostProblem& P, double dt, int n_t, int n_cu) {
  const double dim = std::ldexp(1.0, P.n_local);
  const double alpha = 0.5 * (P.e_max - P.e_min);
  const double z = alpha * dt;
  const double deg1 = z + 12.0 * std::cbrt(z + 1.0) + 20.0;
  const double t_term = 11.4e-6 * std::max(dim / 4096.0, 0.25);
  const double chain = (n_t - 1) * deg1 * t_term;
  const bool real = dense_eligible(P) && ucols_supported(P.L) && P.n_local == P.L;
  const double slots = (double)n_cu * (P.L < 13 ? 2.0 : 1.0);
  const double t_col = real ? 10e-6 * std::max(dim / 4096.0, 0.25) : t_term;
  const double build = std::ceil(dim / slots) * deg1 * t_col;
  const double chain_u = (n_t - 1) * (real ? dim * dim * 8.0 / 5e12 + 5e-6 : dim * dim * 16.0 / 3e12);
  return build + chain_u < chain;
}

int matrix_run(dse_ctx* ctx, int pi, const double* t, int n_t, double dt, double tol, double* obs_out,
               double* h_apps) {
  HostProblem& P = ctx->probs[pi];
  const int n = P.n_local;
  const size_t dim = size_t(1) << n;
  hipStream_t st = ctx->lanes[0].stream;
  // Chebyshev coefficients of one interval dt (one set, one output)
  const double alpha = std::max(0.5 * (P.e_max - P.e_min), 1e-300);
  const double beta = 0.5 * (P.e_max + P.e_min);
  const double z = alpha * dt;
  const int kmax = (int)std::ceil(z + 12.0 * std::cbrt(z + 1.0) + 60.0);
  if (kmax > ctx->max_degree) return fail(ctx, DSE_ERR_CONVERGENCE, "Chebyshev degree exceeds max_degree");
  std::vector<double> J(kmax + 1);
  int deg = 1;
  if (dse_bessel_j(z, kmax, J.data(), tol, &deg) != DSE_OK) return fail(ctx, DSE_ERR_ARG, "bessel failed");
  // U's rotated form is symmetric when the drives are all imaginary (parity twist s_r s_c) or all
  // real: the column build runs in real arithmetic (k_ucols) and the products read the tiles on and
  // above the diagonal (k_symv); otherwise the complex column build and rocBLAS zgemv on the whole
  // column-major matrix
  const bool real_build = dense_eligible(P) && ucols_supported(P.L) && P.n_local == P.L;
  std::vector<double2> row(deg + 2, make_double2(0.0, 0.0));  // complex build: a_k
  std::vector<double> cf(deg + 1);                               // real build: (-1)^{k/2} c_k
  row[0] = make_double2((double)deg, 0.0);
  {
    const std::complex<double> e(std::cos(-beta * dt), std::sin(-beta * dt));
    std::complex<double> mi(1.0, 0.0);
    for (int k = 0; k <= deg; ++k) {
      const double ck = (k == 0 ? 1.0 : 2.0) * J[k];
      const std::complex<double> a = e * mi * ck;
      row[1 + k] = make_double2(a.real(), a.imag());
      cf[k] = ((k >> 1) & 1) ? -ck : ck;
      mi *= std::complex<double>(0.0, -1.0);
    }
  }
  // device buffers: kept in the context between calls (ctx->d_mx)
  const size_t nb = dim / kSymvBlock;
  size_t off = 0;
  auto take = [&](size_t bytes) {
    const size_t o = off;
    off = align_up(off + std::max<size_t>(bytes, 1), 256);
    return o;
  };
  const size_t u_elems = real_build ? nb * (nb + 1) / 2 * kSymvBlock * kSymvBlock : dim * dim;
  const size_t oU = take(u_elems * sizeof(double2)), oS = take(dim * (size_t)n_t * sizeof(double2)),
               oPart = take(real_build ? nb * dim * sizeof(double2) : 0), oObs = take((size_t)n_t * 8 * sizeof(double)),
               oDesc = take(sizeof(DenseProb)), oProb = take(sizeof(DevProb)),
               oCoef = take(std::max(row.size() * sizeof(double2), cf.size() * sizeof(double))), oErr = take(sizeof(int)),
               oCnt = take(nb * sizeof(int));
  if (off > ctx->mx_cap) {
    if (ctx->d_mx) (void)hipFree(ctx->d_mx), ctx->d_mx = nullptr;
    ctx->mx_cap = 0;
    if (hipMalloc(&ctx->d_mx, off) != hipSuccess) return fail(ctx, DSE_ERR_OOM, "propagator-matrix mode: allocation failed");
    ctx->mx_cap = off;
  }
  unsigned char* base = ctx->d_mx;
  double2* U = reinterpret_cast<double2*>(base + oU);     // tiles (real build) or columns: U e_c
  double2* S = reinterpret_cast<double2*>(base + oS);     // psi(t_j), consecutive
  double2* part = real_build ? reinterpret_cast<double2*>(base + oPart) : nullptr;
  double* d_obs = reinterpret_cast<double*>(base + oObs);
  DenseProb* d_desc = reinterpret_cast<DenseProb*>(base + oDesc);
  DevProb* d_p = reinterpret_cast<DevProb*>(base + oProb);
  int* d_err = reinterpret_cast<int*>(base + oErr);
  int* d_cnt = reinterpret_cast<int*>(base + oCnt);
  DevProb d = ctx->h_desc[pi];
  d.beta = beta;
  d.s1 = 1.0 / alpha;
  d.degree = deg;
  HIPC(hipMemsetAsync(d_err, 0, sizeof(int), st));
  HIPC(hipMemsetAsync(d_cnt, 0, nb * sizeof(int), st));
  DevArena ar;  // complex build only: the basis columns
  // HIP events: build | products | (observables), read back for dse_stats (matrix_*)
  hipEvent_t mev[3] = {nullptr, nullptr, nullptr};
  struct EvGuard {
    hipEvent_t* e;
    ~EvGuard() {
      for (int i = 0; i < 3; ++i)
        if (e[i]) (void)hipEventDestroy(e[i]);
    }
  } mev_guard{mev};
  for (auto& e : mev) HIPC(hipEventCreate(&e));
  HIPC(hipEventRecord(mev[0], st));
  if (real_build) {
    double* d_cf = reinterpret_cast<double*>(base + oCoef);
    HIPC(hipMemcpyAsync(d_cf, cf.data(), cf.size() * sizeof(double), hipMemcpyHostToDevice, st));
    HIPC(hipMemcpyAsync(d_p, &d, sizeof(DevProb), hipMemcpyHostToDevice, st));
    HIPC(launch_ucols(P.L, d_p, d_cf, deg, P.imag ? 1 : 0, std::cos(-beta * dt), std::sin(-beta * dt), U, (int)dim,
                      0, (int)P.psi0, S + dim, st));
  } else {
    if (!ctx->blas && rocblas_create_handle(&ctx->blas) != rocblas_status_success)
      return fail(ctx, DSE_ERR_HIP, "rocblas_create_handle failed");
    if (rocblas_set_stream(ctx->blas, st) != rocblas_status_success)
      return fail(ctx, DSE_ERR_HIP, "rocblas_set_stream failed");
    double2* B0 = ar.get<double2>(dim * dim);  // columns: e_c, then scratch
    int2* d_items = ar.get<int2>(dim);
    BasisInit* d_init = ar.get<BasisInit>(dim);
    if (!B0 || !d_items || !d_init) return fail(ctx, DSE_ERR_OOM, "propagator-matrix mode: allocation failed");
    double2* d_row = reinterpret_cast<double2*>(base + oCoef);
    d.buf[0] = B0;
    d.buf[1] = B0;
    d.buf[2] = U;
    d.coef = d_row;
    d.kcap1 = deg + 1;
    d.n_acc = 1;
    d.xacc_q = 0;
    std::vector<int2> items(dim);
    std::vector<BasisInit> init(dim);
    for (size_t c = 0; c < dim; ++c) {
      items[c] = make_int2(0, (int)c);
      init[c].ptr = B0 + c * dim;
      init[c].n = dim;
      init[c].one_at = (int64_t)c;
    }
    HIPC(hipMemcpyAsync(d_row, row.data(), row.size() * sizeof(double2), hipMemcpyHostToDevice, st));
    HIPC(hipMemcpyAsync(d_p, &d, sizeof(DevProb), hipMemcpyHostToDevice, st));
    HIPC(hipMemcpyAsync(d_items, items.data(), dim * sizeof(int2), hipMemcpyHostToDevice, st));
    HIPC(hipMemcpyAsync(d_init, init.data(), dim * sizeof(BasisInit), hipMemcpyHostToDevice, st));
    HIPC(launch_basis_init(d_init, (int)dim, dim, st));
    HIPC(launch_interval(P.L, P.imag, d_p, d_items, (int)dim, 0, 0, 1, d_err, d_err, ctx->hk, st, (long)dim));
  }
  HIPC(hipEventRecord(mev[1], st));
  // psi_0 = e_x0, psi_1 = U e_x0 (column x0), psi_{j+1} = U psi_j
  HIPC(hipMemsetAsync(S, 0, dim * sizeof(double2), st));
  static const double2 one_c = {1.0, 0.0};
  HIPC(hipMemcpyAsync(S + P.psi0, &one_c, sizeof(double2), hipMemcpyHostToDevice, st));
  if (!real_build)  // (the real build wrote column x0 itself)
    HIPC(hipMemcpyAsync(S + dim, U + P.psi0 * dim, dim * sizeof(double2), hipMemcpyDeviceToDevice, st));
  const rocblas_double_complex one(1.0, 0.0), zero(0.0, 0.0);
  for (int j = 1; j + 1 < n_t && real_build; ++j) {
    if (ctx->symv_fused) {
      HIPC(launch_symv(U, (int)dim, S + dim * j, part, P.imag ? 1 : 0, st, d_cnt, S + dim * (j + 1)));
    } else {
      HIPC(launch_symv(U, (int)dim, S + dim * j, part, P.imag ? 1 : 0, st));
      HIPC(launch_symv_reduce(part, (int)dim, S + dim * (j + 1), st));
    }
  }
  for (int j = 1; j + 1 < n_t && !real_build; ++j) {
    const rocblas_status rs = rocblas_zgemv(ctx->blas, rocblas_operation_none, (rocblas_int)dim, (rocblas_int)dim,
                                            &one, reinterpret_cast<const rocblas_double_complex*>(U),
                                            (rocblas_int)dim,
                                            reinterpret_cast<const rocblas_double_complex*>(S + dim * j), 1,
                                            &zero, reinterpret_cast<rocblas_double_complex*>(S + dim * (j + 1)), 1);
    if (rs != rocblas_status_success)
      return fail(ctx, DSE_ERR_HIP, "rocblas zgemv failed (status " + std::to_string((int)rs) + ")");
  }
  HIPC(hipEventRecord(mev[2], st));
  DenseProb D = {};
  D.n = n;
  D.rot = 0;
  D.sea_mask = P.sea_mask;
  D.rare_bit = P.rare_bit;
  D.n_sea = __builtin_popcountll(P.sea_mask);
  D.x0 = P.psi0;
  D.obs = d_obs;
  HIPC(hipMemcpyAsync(d_desc, &D, sizeof(DenseProb), hipMemcpyHostToDevice, st));
  HIPC(launch_state_obs(d_desc, (int)dim, S, n_t, 0, st));
  HIPC(hipMemcpyAsync(P.buf[0], S + dim * (size_t)(n_t - 1), dim * sizeof(double2), hipMemcpyDeviceToDevice, st));
  std::vector<double> h((size_t)n_t * 8);
  int herr = 0;
  HIPC(hipMemcpyAsync(h.data(), d_obs, h.size() * sizeof(double), hipMemcpyDeviceToHost, st));
  HIPC(hipMemcpyAsync(&herr, d_err, sizeof(int), hipMemcpyDeviceToHost, st));
  HIPC(hipStreamSynchronize(st));
  if (herr) return fail(ctx, DSE_ERR_HIP, "propagator-matrix mode: column build failed");
  for (int ti = 0; ti < n_t; ++ti)
    finish_obs(P, h.data() + (size_t)ti * 8, obs_out + (size_t)pi * DSE_N_OBS * n_t + ti, (size_t)n_t);
  P.degree = deg;
  *h_apps = (double)deg * (double)dim;
  float b_ms = 0.f, p_ms = 0.f;
  HIPC(hipEventElapsedTime(&b_ms, mev[0], mev[1]));
  HIPC(hipEventElapsedTime(&p_ms, mev[1], mev[2]));
  ctx->mx_build_ms = b_ms;
  ctx->mx_products_ms = p_ms;
  ctx->mx_products = (double)std::max(0, n_t - 2);
  ctx->mx_bytes_per_product = (double)(u_elems * sizeof(double2) + dim * sizeof(double2));
  return DSE_OK;
}

}  // namespace

extern "C" {

int dse_apply_h(dse_ctx* ctx, int problem, const double* psi_in, double* psi_out) {
  if (!ctx) return DSE_ERR_ARG;
  if (!psi_in || !psi_out) return fail(ctx, DSE_ERR_ARG, "null state");
  int first = 0, count = 1;
  int rc = hook_members(ctx, problem, &first, &count);
  if (rc) return rc;
  HIPC(hipSetDevice(ctx->device));
  if ((rc = prepare(ctx))) return rc;
  hipStream_t st = ctx->lanes[0].stream;
  const double2* in = reinterpret_cast<const double2*>(psi_in);
  double2* out = reinterpret_cast<double2*>(psi_out);
  for (int i = 0; i < count; ++i) {
    HostProblem& P = ctx->probs[first + i];
    const size_t amps = size_t(1) << P.n_local;
    HIPC(hipMemcpyAsync(P.buf[0], in + i * amps, amps * sizeof(double2), hipMemcpyHostToDevice, st));
  }
  if ((rc = apply_members(ctx, first, count, st))) return rc;
  for (int i = 0; i < count; ++i) {
    HostProblem& P = ctx->probs[first + i];
    const size_t amps = size_t(1) << P.n_local;
    HIPC(hipMemcpyAsync(out + i * amps, P.buf[1], amps * sizeof(double2), hipMemcpyDeviceToHost, st));
  }
  HIPC(hipStreamSynchronize(st));
  ctx->evolved = false;
  return DSE_OK;
}

int dse_observables(dse_ctx* ctx, int problem, const double* psi, double* obs7) {
  if (!ctx) return DSE_ERR_ARG;
  if (!psi || !obs7) return fail(ctx, DSE_ERR_ARG, "null pointer");
  int first = 0, count = 1;
  int rc = hook_members(ctx, problem, &first, &count);
  if (rc) return rc;
  HIPC(hipSetDevice(ctx->device));
  if ((rc = prepare(ctx))) return rc;
  int64_t tiles = 0;
  for (int i = 0; i < count; ++i) tiles += ctx->probs[first + i].n_tiles;
  if ((rc = ensure_partial(ctx, 1))) return rc;
  hipStream_t st = ctx->lanes[0].stream;
  const double2* in = reinterpret_cast<const double2*>(psi);
  for (int i = 0; i < count; ++i) {
    HostProblem& P = ctx->probs[first + i];
    const size_t amps = size_t(1) << P.n_local;
    HIPC(hipMemcpyAsync(P.buf[0], in + i * amps, amps * sizeof(double2), hipMemcpyHostToDevice, st));
  }
  if (ctx->probs[first].dist && (rc = dist_exchange(ctx, 0, 0, st))) return rc;
  int64_t off = 0;
  for (int i = 0; i < count; ++i) {
    HostProblem& P = ctx->probs[first + i];
    HIPC(launch_obs(P.L, ctx->d_probs, P.d_items, (int)P.n_tiles, 0, ctx->d_partial + off * 8, st));
    off += P.n_tiles;
  }
  std::vector<double> h(tiles * 8);
  HIPC(hipMemcpyAsync(h.data(), ctx->d_partial, h.size() * sizeof(double), hipMemcpyDeviceToHost, st));
  HIPC(hipStreamSynchronize(st));
  double v[7] = {0, 0, 0, 0, 0, 0, 0};
  for (int64_t t = 0; t < tiles; ++t)
    for (int j = 0; j < 7; ++j) v[j] += h[t * 8 + j];
  if (ctx->probs[first].dist && (rc = xchg_allreduce_host(ctx, v, 7, st))) return rc;  // all shards
  finish_obs(ctx->probs[first], v, obs7, 1);
  ctx->evolved = false;
  return DSE_OK;
}

// ---- spanning registers (dse_span.hip) ------------------------------------------------------

// option span_tile = -1: the automatic choice takes the first of these (tile bits, resident
// launches) whose workgroups fit: 2^10 tiles one per CU, all at once (a lone N = 14 register over
// 16 CUs: 78 vs 85 ms at 150 kHz); 2^11 at the kernel's occupancy, all at once (one GPU's share of
// an 8-GPU strong split); 2^11 in two resident launches per interval (span_cuts; the registers in
// degree order, so the stiff ones share the first): one GPU's share of a 4-GPU split, 169 against
// 225 ms on k_interval, while three launches (a 2-GPU share) lose, 246 against 234 ms
// (profiles/r06/span_chunks_shard{4,2}.jsonl)
constexpr int kSpanAutoTiles[3][2] = {{10, 1}, {11, 1}, {11, 2}};

// amplitudes per thread of k_span for an L-bit tile: 2^rb (option span_rb, else 512 threads)
int span_rb_for(const dse_ctx* ctx, int L) { return ctx->span_rb > 0 ? ctx->span_rb : L - 9; }

// whether register P can span its top s bits (2^s tiles of n - s bits)
bool span_eligible(const dse_ctx* ctx, const HostProblem& P, int s) {
  if (P.side() || P.shard_bits != 0 || s < 1 || s > kSpanMaxTop) return false;
  const int L = P.n_local - s;
  return L >= 1 && span_supported(L, span_rb_for(ctx, L));
}

// The tables k_span reads for register P cut into 2^s tiles of L bits, RB of them register bits
// (dse_internal.h SpanTab).  Same coefficients as build_tables, sorted by k_span's layout.
int build_span_table(const HostProblem& P, int L, int RB, int s, SpanTab& T) {
  const int n = P.n;
  const int TB = L - RB;
  const int npi = (TB * (TB - 1) / 2 + TB - 1) / TB;
  const int iw = 4 + npi;
  if (TB * iw > kSpanMaxIt || L > 16 || RB > 4 || s > kSpanMaxTop || n != L + s) return DSE_ERR_ARG;
  std::memset(&T, 0, sizeof(T));
  T.n_it = TB * iw;
  auto it = [&](int j, int e) -> double2& { return T.it[j * iw + e]; };
  std::vector<std::pair<uint32_t, double>> tpairs;
  for (int i = 0; i < n; ++i)
    for (int j = i + 1; j < n; ++j) {
      const double g = P.pair[i * n + j];
      if (g == 0.0) continue;
      if (j < TB) {
        tpairs.push_back({(1u << i) | (1u << j), g});
      } else if (j < L && i < TB) {
        const int r = j - TB;
        (r & 1 ? it(i, 2 + r / 2).y : it(i, 2 + r / 2).x) = g;
      } else if (j < L) {
        T.rr_g[rr_index(i - TB, j - TB)] = g;
      } else if (i < L) {
        T.ug[j - L][i] = g;
        T.u_mask |= 1 << (j - L);
      } else {
        SpanOp& o = T.ops[T.n_ops++];
        o.kind = 2;
        o.b = i - L;
        o.b2 = j - L;
        o.pmask = (1u << o.b) | (1u << o.b2);
        o.c[0] = g;
        T.need_raw = 1;
      }
    }
  if ((int)tpairs.size() > TB * npi) return DSE_ERR_ARG;
  for (size_t p = 0; p < tpairs.size(); ++p) {
    double2& e = it((int)(p / npi), 4 + (int)(p % npi));
    e.x = __builtin_bit_cast(double, (uint64_t)tpairs[p].first);
    e.y = tpairs[p].second;
  }
  for (int b = 0; b < n; ++b) {
    double f[4];
    for (int c = 0; c < 4; c += 2) {  // as build_tables: cos(pi/2) residues dropped
      f[c] = P.flip[4 * b + c];
      f[c + 1] = P.flip[4 * b + c + 1];
      if (std::fabs(f[c]) <= 1e-15 * std::hypot(f[c], f[c + 1])) f[c] = 0.0;
    }
    if (f[0] == 0.0 && f[1] == 0.0 && f[2] == 0.0 && f[3] == 0.0) continue;
    if (b < TB) {
      it(b, 0) = make_double2(f[0], f[1]);
      it(b, 1) = make_double2(f[2], f[3]);
    } else if (b < L) {
      for (int c = 0; c < 4; ++c) T.rflip[b - TB][c] = f[c];
      T.rflip_mask |= 1 << (b - TB);
    } else {
      for (int c = 0; c < 4; ++c) T.uflip[b - L][c] = f[c];
    }
  }
  // operands: u of every top bit with crossing pairs; the raw partner under the drive of every
  // top bit without them (and with a drive)
  for (int b = 0; b < s; ++b) {
    const bool has_flip = T.uflip[b][0] != 0.0 || T.uflip[b][1] != 0.0 || T.uflip[b][2] != 0.0 || T.uflip[b][3] != 0.0;
    if (!((T.u_mask >> b) & 1) && !has_flip) continue;
    SpanOp& o = T.ops[T.n_ops++];
    o.kind = ((T.u_mask >> b) & 1) ? 0 : 1;
    o.b = o.b2 = b;
    o.pmask = 1u << b;
    if (o.kind == 1) {
      for (int c = 0; c < 4; ++c) o.c[c] = T.uflip[b][c];
      T.need_raw = 1;
    }
  }
  return DSE_OK;
}

// ---- real-component registers (dse_real.hip) ---------------------------------------------------

bool real_eligible(const HostProblem& P) {
  return !P.side() && P.span_s == 0 && P.shard_bits == 0 && P.imag && (P.n_local == 13 || P.n_local == 14);
}

// RealTab of register P (n = 13 or 14: 9 thread bits, n - 9 register bits): the coefficients of
// H' = D H D^dagger, D|x> = i^|x| |x>: pairs -g (i^{+-2}), drives by the output bit value v of the
// flipped bit: v = 0 -> +Im c0, v = 1 -> -Im c1 (i^{-+1} times the imaginary coefficient, k_dense_h)
int build_real_table(const HostProblem& P, RealTab& T) {
  const int n = P.n, TB = 9, RB = n - TB;
  if (RB < 4 || RB > kRealRB) return DSE_ERR_ARG;
  std::memset(&T, 0, sizeof(T));
  auto row = [&](int j, int e) -> double& {
    double2& d = T.it[j * 6 + e / 2];
    return (e & 1) ? d.y : d.x;
  };
  for (int i = 0; i < n; ++i)
    for (int j = i + 1; j < n; ++j) {
      const double g = -P.pair[i * n + j];
      if (g == 0.0) continue;
      if (j < TB) {  // canonical slot of (i, j): lexicographic over a < b < 9, 4 per iteration
        const int p = i * TB - i * (i + 1) / 2 + (j - i - 1);
        row(p / 4, 8 + p % 4) = g;
      } else if (i < TB) {
        row(i, 2 + (j - TB)) = g;
      } else {
        T.rr_g[real_rr_index(i - TB, j - TB)] = g;
      }
    }
  for (int b = 0; b < n; ++b) {
    double f[4];
    for (int c = 0; c < 4; c += 2) {  // as build_tables: cos(pi/2) residues dropped
      f[c] = P.flip[4 * b + c];
      f[c + 1] = P.flip[4 * b + c + 1];
      if (std::fabs(f[c]) <= 1e-15 * std::hypot(f[c], f[c + 1])) f[c] = 0.0;
    }
    if (f[0] != 0.0 || f[2] != 0.0) return DSE_ERR_ARG;  // not an imaginary drive
    if (f[1] == 0.0 && f[3] == 0.0) continue;
    if (b < TB) {
      row(b, 0) = f[1];
      row(b, 1) = -f[3];
    } else {
      T.rflip[b - TB][0] = f[1];
      T.rflip[b - TB][1] = -f[3];
      T.rflip_mask |= 1 << (b - TB);
    }
  }
  T.x0 = P.psi0;
  T.x0pop = __builtin_popcountll(P.psi0);
  return DSE_OK;
}

static int evolve_impl(dse_ctx* ctx, const double* t, int n_t, double tol, double* obs_out, dse_stats* stats) {
  const auto wall0 = std::chrono::steady_clock::now();
  // DSE_HOST_TIMING=1: host time of each phase of this call on stderr (diagnostics)
  static const bool host_timing = std::getenv("DSE_HOST_TIMING") != nullptr;
  auto tmark = wall0;
  auto phase = [&](const char* name) {
    if (!host_timing) return;
    const auto now = std::chrono::steady_clock::now();
    std::fprintf(stderr, "[dse_evolve] %-12s %9.3f ms\n", name,
                 std::chrono::duration<double, std::milli>(now - tmark).count());
    tmark = now;
  };
  if (!t || !obs_out) return fail(ctx, DSE_ERR_ARG, "null pointer");
  if (n_t < 1) return fail(ctx, DSE_ERR_ARG, "n_t must be >= 1");
  if (!(tol > 0.0 && tol < 1e-2)) return fail(ctx, DSE_ERR_ARG, "tol must be in (0, 1e-2)");
  for (int i = 0; i < n_t; ++i)
    if (!std::isfinite(t[i])) return fail(ctx, DSE_ERR_ARG, "non-finite time");
  for (int i = 1; i < n_t; ++i)
    if (!(t[i] > t[i - 1])) return fail(ctx, DSE_ERR_ARG, "times must be strictly increasing");
  HIPC(hipSetDevice(ctx->device));
  // timing-event records of an earlier call that ended early (an error, or the hand-off timeout
  // dse_evolve re-runs) are dropped: their per-launch counters lived in that call
  for (auto& ln : ctx->lanes) ln.ev_used[0] = ln.ev_used[1] = 0;
  int rc = prepare(ctx);
  if (rc) return rc;
  ctx->xbytes = 0.0;
  ctx->xms = 0.0;
  ctx->xev_used = 0;

  phase("prepare");
  // ---- execution mode ----
  // small registers (n <= 9): the one-wave engine (dse_small.hip) on its own stream, whatever the
  // other problems run on.  Of the rest -- persistent: every problem fits one or two
  // register-block tiles -> one k_interval launch per group of output intervals and lane;
  // streaming: per-term kernels, one output per group.
  // dense engine first (option "dense"): a register it takes is off every Chebyshev path
  bool any_small = false, any_big = false, any_dense = false;
  for (auto& P : ctx->probs) {
    P.dn = ctx->dense && dense_eligible(P) && (ctx->dense == 2 || dense_cheaper(P, t, n_t, ctx->eig_impl));
    any_dense = any_dense || P.dn;
  }
  for (auto& P : ctx->probs) {
    P.mx = false;
    P.sm = !P.dn && ctx->small && P.shard_bits == 0 && P.n_local <= kSmallMaxQubits;
    any_small = any_small || P.sm;
  }
  // a context whose Chebyshev work is one register: propagator-matrix mode (matrix_run) when the
  // persistent kernel is allowed and the model prefers it
  int matrix_pi = -1;
  double matrix_dt = 0.0;
  {
    int n_cheb = 0, last = -1;
    for (size_t pi = 0; pi < ctx->probs.size(); ++pi)
      if (!ctx->probs[pi].side()) ++n_cheb, last = (int)pi;
    if (n_cheb == 1 && ctx->matrix && ctx->persistent) {
      HostProblem& P = ctx->probs[last];
      // the matrix-mode buffers must fit 80% of the free memory (plus what the context already
      // holds for them); otherwise the register stays on the per-interval kernels
      size_t free_b = 0, total_b = 0;
      HIPC(hipMemGetInfo(&free_b, &total_b));
      const bool fits = matrix_bytes(P, n_t) <= 0.8 * (double)free_b + (double)ctx->mx_cap;
      if (fits && matrix_eligible(P, t, n_t, &matrix_dt) &&
          (ctx->matrix == 2 || matrix_cheaper(P, matrix_dt, n_t, ctx->n_cu))) {
        P.mx = true;
        matrix_pi = last;
      }
    }
  }
  for (auto& P : ctx->probs) any_big = any_big || !P.side();
  bool persistent = ctx->persistent != 0;
  bool any_dist = false;
  // spanning registers (options span / span_tile): every register that fits runs on k_span over
  // 2^s tiles.  span_tile = -1 (default, auto): when the context's registers are few enough that
  // all their 2^11-amplitude tiles fit the chip in at most two resident launches (one GPU's share
  // of a 4- or 8-GPU strong split, a lone simulate_rare register), a shorter chain per register;
  // otherwise none spans (kSpanAutoTiles)
  {
    int tile = ctx->span_tile;
    // the all-span candidates kSpanAutoTiles[ti0, ti1): the smallest tile whose workgroups fit
    auto all_span_tile = [&](int ti0, int ti1) {
      int tl = 0;
      for (int ti = ti0; ti < ti1 && tl == 0; ++ti) {
        const int L = kSpanAutoTiles[ti][0], chunks = kSpanAutoTiles[ti][1];
        int64_t wg = 0;
        bool all = persistent && ctx->span == 0;
        for (auto& P : ctx->probs) {
          if (P.side()) continue;
          const int s = P.n_local - L;
          if (!span_eligible(ctx, P, s)) all = false;
          wg += int64_t(1) << std::max(0, s);
        }
        int per_cu = 1;
        if (ti > 0 && span_occupancy(L, span_rb_for(ctx, L), true, &per_cu) != hipSuccess) per_cu = 0;
        if (all && wg > 0 && chunks <= ctx->span_chunks && wg <= (int64_t)chunks * per_cu * ctx->n_cu) tl = L;
      }
      return tl;
    };
    auto assign = [&]() {
      for (auto& P : ctx->probs) {
        const int s = tile > 0 ? P.n_local - tile : ctx->span;
        P.span_s = (persistent && span_eligible(ctx, P, s)) ? s : 0;
      }
    };
    // order: every register spanned in one resident launch; else the partial span below; else
    // every register spanned in two resident launches (the partial form measured faster on the
    // 4-GPU share, 151 against 167 ms, profiles/r06/span_partial_shards.jsonl)
    if (tile < 0) tile = all_span_tile(0, 2);
    assign();
    // Partial span (option span_partial, round 6): when the registers do not all fit spanned (one
    // GPU's share of a 2-GPU split: 96 registers), the ones with the longest predicted chains span
    // over 2^11-amplitude tiles on a lane of their own while the rest stay on k_interval, as long
    // as every workgroup of both launches fits the chip at once (each takes a CU: residency of
    // every hand-off partner is guaranteed, whatever order the two streams' workgroups land in).
    // Predicted chain of a register: its spectral half-width (degree per interval ~ alpha dt) times
    // the measured term time of its kernel under load (kTermUs); applied when the longest chain
    // shrinks by at least 10%.
    bool partial = false;
    if (ctx->span_tile < 0 && tile == 0 && ctx->span == 0 && persistent && ctx->span_partial &&
        std::min<int>(ctx->n_streams, (int)ctx->probs.size()) >= 2) {
      const int Lp = ctx->span_partial_tile;
      // term time under load: k_interval 1-tile, 2-tile; k_span over 2^Lp-amplitude tiles
      const double kTermUs[3] = {19.5, 24.0, Lp == 11 ? 14.0 : 11.0};
      struct C {
        double chain;
        int pi, kind;  // kind 0 / 1: k_interval of 1 / 2 tiles, 2: spanned
      };
      std::vector<C> cs;
      int64_t wg = 0;
      bool ok = true;
      for (size_t pi = 0; pi < ctx->probs.size(); ++pi) {
        const HostProblem& P = ctx->probs[pi];
        if (P.side()) continue;
        if (P.shard_bits != 0 || !(P.n_tiles == 1 || P.n_tiles == 2) || !interval_supported(P.L)) {
          ok = false;  // (and kTermUs has entries for 1- and 2-tile registers only)
          break;
        }
        wg += P.n_tiles;
        const double alpha = 0.5 * (P.e_max - P.e_min);
        cs.push_back({alpha * kTermUs[P.n_tiles - 1], (int)pi, (int)P.n_tiles - 1});
      }
      auto worst = [&]() { return std::max_element(cs.begin(), cs.end(), [](const C& a, const C& b) { return a.chain < b.chain; }); };
      if (ok && !cs.empty() && wg <= ctx->n_cu) {
        const double before = worst()->chain;
        std::vector<int> spanned;
        for (;;) {
          auto w = worst();
          if (w->kind == 2) break;
          const HostProblem& P = ctx->probs[w->pi];
          const int sp = P.n_local - Lp;
          if (!span_eligible(ctx, P, sp)) break;
          const int64_t extra = (int64_t(1) << sp) - P.n_tiles;
          if (wg + extra > ctx->n_cu) break;
          wg += extra;
          w->chain = w->chain / kTermUs[w->kind] * kTermUs[2];
          w->kind = 2;
          spanned.push_back(w->pi);
        }
        if (!spanned.empty() && worst()->chain <= 0.9 * before) {
          for (int pi : spanned) ctx->probs[pi].span_s = ctx->probs[pi].n_local - Lp;
          partial = true;
        }
      }
    }
    if (ctx->span_tile < 0 && tile == 0 && !partial && (tile = all_span_tile(2, 3)) > 0) assign();
  }
  for (auto& P : ctx->probs) {
    if (P.side()) continue;
    if (P.span_s == 0 && (!(interval_supported(P.L) && P.n_tiles <= 2) || P.shard_bits > 0)) persistent = false;
    any_dist = any_dist || P.dist;
  }
  if (!persistent)
    for (auto& P : ctx->probs) P.span_s = 0;
  // real-component mode: option real = 1 when every Chebyshev register qualifies (one launch kind
  // per interval); real = 2 the 2-tile (14-qubit) registers only, on their own stream beside the
  // 1-tile registers' k_interval launches (neither kernel waits on another workgroup, so the two
  // persistent launches share the chip without a residency condition)
  {
    bool real_mode = persistent && ctx->real_mode && !ctx->obs_overlap;
    int n_cheb = 0;
    for (auto& P : ctx->probs) {
      if (P.side()) continue;
      ++n_cheb;
      if (ctx->real_mode == 1) real_mode = real_mode && real_eligible(P);
    }
    for (auto& P : ctx->probs)
      P.rl = real_mode && n_cheb > 0 && !P.side() && (ctx->real_mode == 1 || (real_eligible(P) && P.n_tiles == 2));
  }
  // streaming: registers of more than one 2^13 tile take the Walsh-Hadamard engine (option wht)
  bool used_wht = false;
  bool any_dist_step = any_dist;  // dist shards on the step kernels: per-term shard exchange
  if (!persistent) {
    if ((rc = ensure_wht(ctx))) return rc;
    any_dist_step = false;
    for (auto& P : ctx->probs) {
      used_wht = used_wht || P.wht_groups > 0;
      any_dist_step = any_dist_step || (P.dist && P.wht_groups == 0);
    }
  }
  // Outputs per launch M: the Chebyshev series of e^{-iH tau} converges after ~ alpha tau +
  // O((alpha tau)^{1/3}) terms, so M outputs from one series (one propagator sum per output, same
  // vectors T_k(H~) psi) need fewer H applications than M series of one interval each when alpha
  // dt is small (the N = 14 sweep on its 1 ms grid: -23% for the stiffest problem at M = 4).  On
  // coarse grids (alpha dt >= 400) the saving is nil and the coefficient tables grow, so M = 1.
  double max_z = 0.0;
  for (int m = 0; m + 1 < n_t; ++m)
    for (auto& P : ctx->probs)
      if (!P.side()) max_z = std::max(max_z, 0.5 * (P.e_max - P.e_min) * (t[m + 1] - t[m]));
  // k_span staggers its outputs' sums over the terms (coef_nterm phases), so an evolve whose
  // registers all span takes up to kSpanMaxOut outputs per series (option span_outputs);
  // k_interval and k_real update every output's sum in one term, from registers: at most two
  bool all_span = true;
  for (auto& P : ctx->probs)
    if (!P.side()) all_span = all_span && P.span_s > 0 && !P.rl;
  int M = 1;
  if (persistent && max_z < 400.0)
    M = std::max(1, std::min(all_span ? ctx->span_outputs : ctx->outputs_per_launch, n_t - 1));

  // ---- groups of M consecutive output intervals -> coefficient sets (distinct offset lists) ----
  struct Group {
    int m0, n_out, set;
  };
  std::vector<Group> groups;
  std::vector<std::vector<double>> set_tau;  // offsets t[m0 + j + 1] - t[m0], j < n_out
  for (int m0 = 0; m0 + 1 < n_t; m0 += M) {
    Group g;
    g.m0 = m0;
    g.n_out = std::min(M, n_t - 1 - m0);
    std::vector<double> tau(g.n_out);
    for (int j = 0; j < g.n_out; ++j) tau[j] = t[m0 + j + 1] - t[m0];
    g.set = -1;
    for (size_t q = 0; q < set_tau.size(); ++q)
      if (set_tau[q] == tau) {
        g.set = (int)q;
        break;
      }
    if (g.set < 0) {
      if (set_tau.size() >= 4096) return fail(ctx, DSE_ERR_ARG, "more than 4096 distinct output intervals");
      g.set = (int)set_tau.size();
      set_tau.push_back(tau);
    }
    groups.push_back(g);
  }
  if (set_tau.empty()) set_tau.push_back(std::vector<double>(1, 0.0));
  const int n_sets = (int)set_tau.size();
  const int n_groups = (int)groups.size();

  phase("groups");
  // ---- Chebyshev coefficients per problem: rows [set][output j][term k], all problems' rows
  // gathered into one arena and uploaded with one copy ----
  // Problems are independent: computed on up to 16 host threads (Bessel series of every distinct
  // offset set, ~3 us each), then gathered in problem order.
  std::vector<std::vector<double2>> coef_rows(ctx->probs.size());
  std::vector<int> coef_rc(ctx->probs.size(), DSE_OK);
  std::vector<std::string> coef_msg(ctx->probs.size());
  auto coef_one = [&](size_t pi) {
    HostProblem& P = ctx->probs[pi];
    if (P.side()) return;
    const double alpha = std::max(0.5 * (P.e_max - P.e_min), 1e-300);
    const double beta = 0.5 * (P.e_max + P.e_min);
    int deg = 1;
    std::vector<std::vector<double>> J((size_t)n_sets * M);
    std::vector<int> deg_sj((size_t)n_sets * M, 0);
    for (int s = 0; s < n_sets; ++s)
      for (size_t j = 0; j < set_tau[s].size(); ++j) {
        const double z = alpha * set_tau[s][j];
        const int kmax = (int)std::ceil(z + 12.0 * std::cbrt(z + 1.0) + 60.0);
        if (kmax > ctx->max_degree) {
          coef_rc[pi] = DSE_ERR_CONVERGENCE;
          coef_msg[pi] = "Chebyshev degree " + std::to_string(kmax) + " exceeds max_degree; use a finer output grid";
          return;
        }
        std::vector<double>& Jv = J[(size_t)s * M + j];
        Jv.resize(kmax + 1);
        int d = 1;
        if (dse_bessel_j(z, kmax, Jv.data(), tol, &d) != DSE_OK) {
          coef_rc[pi] = DSE_ERR_ARG;
          coef_msg[pi] = "bessel failed";
          return;
        }
        deg_sj[(size_t)s * M + j] = d;
        deg = std::max(deg, d);
      }
    P.degree = deg;
    const int kcap1 = deg + 1;
    // compact rows (coef_row): [set][j] x (kcap1 + 1) entries, [0].x = degree, [1 + k] = a_k
    std::vector<double2>& coef = coef_rows[pi];
    coef.assign((size_t)n_sets * M * (kcap1 + 1), make_double2(0.0, 0.0));
    for (int s = 0; s < n_sets; ++s)
      for (size_t j = 0; j < set_tau[s].size(); ++j) {
        const std::vector<double>& Jv = J[(size_t)s * M + j];
        const int dj = deg_sj[(size_t)s * M + j];
        const double ph = -beta * set_tau[s][j];
        const std::complex<double> e(std::cos(ph), std::sin(ph));
        std::complex<double> mi(1.0, 0.0);  // (-i)^k
        double2* row = coef.data() + ((size_t)s * M + j) * (kcap1 + 1);
        row[0] = make_double2((double)dj, 0.0);
        for (int k = 0; k <= dj; ++k) {
          const std::complex<double> a = e * mi * ((k == 0 ? 1.0 : 2.0) * Jv[k]);
          row[1 + k] = make_double2(a.real(), a.imag());
          mi *= std::complex<double>(0.0, -1.0);
        }
      }
    DevProb& d = ctx->h_desc[pi];
    d.kcap1 = kcap1;
    d.degree = deg;
    d.beta = beta;
    d.s1 = 1.0 / alpha;
    d.n_acc = M;
    d.xacc_q = (persistent && ctx->obs_overlap) ? M - 1 : 0;
  };
  if (ctx->dbg & 4)
    for (size_t pi = 0; pi < ctx->probs.size(); ++pi) coef_one(pi);
  else
    parallel_for(ctx->probs.size(), coef_one);
  Arena coef_arena;
  std::vector<size_t> coef_off(ctx->probs.size(), 0);
  size_t coef_total = 0;
  for (size_t pi = 0; pi < ctx->probs.size(); ++pi) {
    if (coef_rc[pi] != DSE_OK) return fail(ctx, coef_rc[pi], coef_msg[pi]);
    coef_total += align_up(coef_rows[pi].size() * sizeof(double2), 64);
  }
  coef_arena.host.reserve(coef_total);
  for (size_t pi = 0; pi < ctx->probs.size(); ++pi)
    if (!ctx->probs[pi].side()) coef_off[pi] = coef_arena.place(coef_rows[pi].size() * sizeof(double2));
  parallel_for(ctx->probs.size(), [&](size_t pi) {
    if (!coef_rows[pi].empty())
      std::memcpy(coef_arena.host.data() + coef_off[pi], coef_rows[pi].data(), coef_rows[pi].size() * sizeof(double2));
  });

  phase("coefficients");
  if ((rc = upload_arena(ctx, coef_arena, &ctx->d_coef, &ctx->coef_cap, ctx->lanes[0].stream))) return rc;
  for (size_t pi = 0; pi < ctx->probs.size(); ++pi) {
    HostProblem& P = ctx->probs[pi];
    if (P.side()) continue;
    P.coef = reinterpret_cast<double2*>(ctx->d_coef + coef_off[pi]);
    ctx->h_desc[pi].coef = P.coef;
  }

  phase("coef upload");
  // intermediate outputs of multi-output launches: (M - 1) state vectors per problem, two sets
  // (one per launch parity) when the observables are overlapped
  const bool obs_ovl = persistent && ctx->obs_overlap;
  {
    const size_t xsets = obs_ovl ? 2 : 1;
    size_t need = 0;
    if (M > 1)
      for (auto& P : ctx->probs)
        if (!P.side()) need += xsets * ((size_t)(M - 1) << P.n_local);
    if (need > ctx->xacc_cap) {
      if (ctx->d_xacc) (void)hipFree(ctx->d_xacc), ctx->d_xacc = nullptr;
      ctx->xacc_cap = 0;
      if (hipMalloc(&ctx->d_xacc, need * sizeof(double2)) != hipSuccess)
        return fail(ctx, DSE_ERR_OOM, "output accumulator allocation failed (" +
                                          std::to_string(need * sizeof(double2)) + " bytes)");
      ctx->xacc_cap = need;
    }
    size_t off = 0;
    for (size_t pi = 0; pi < ctx->probs.size(); ++pi) {
      const bool use = M > 1 && !ctx->probs[pi].side();
      ctx->h_desc[pi].xacc = use ? ctx->d_xacc + off : nullptr;
      if (use) off += xsets * ((size_t)(M - 1) << ctx->probs[pi].n_local);
    }
  }
  // real-component registers: tables, [a | b] inputs and per-output, per-component sums
  {
    Arena tabs;
    std::vector<size_t> tab_off(ctx->probs.size(), 0);
    size_t need = 0;  // in double2 units
    for (size_t pi = 0; pi < ctx->probs.size(); ++pi) {
      const HostProblem& P = ctx->probs[pi];
      ctx->h_desc[pi].rtab = nullptr;
      ctx->h_desc[pi].rin = nullptr;
      ctx->h_desc[pi].racc = nullptr;
      if (!P.rl) continue;
      RealTab T;
      if ((rc = build_real_table(P, T)) != DSE_OK) return fail(ctx, rc, "real-mode tables: drives not imaginary");
      tab_off[pi] = tabs.add(&T, sizeof(T));
      need += ((size_t)1 + 2 * (size_t)M) << P.n_local;
    }
    if (need > 0) {
      if ((rc = upload_arena(ctx, tabs, &ctx->d_real_tab, &ctx->real_tab_cap, ctx->lanes[0].stream))) return rc;
      HIPC(hipStreamSynchronize(ctx->lanes[0].stream));
      if (need * sizeof(double2) > ctx->real_cap) {
        if (ctx->d_real) (void)hipFree(ctx->d_real), ctx->d_real = nullptr;
        ctx->real_cap = 0;
        if (hipMalloc(&ctx->d_real, need * sizeof(double2)) != hipSuccess)
          return fail(ctx, DSE_ERR_OOM, "real-mode buffer allocation failed (" +
                                            std::to_string(need * sizeof(double2)) + " bytes)");
        ctx->real_cap = need * sizeof(double2);
      }
      double2* base = reinterpret_cast<double2*>(ctx->d_real);
      size_t off = 0;
      for (size_t pi = 0; pi < ctx->probs.size(); ++pi) {
        const HostProblem& P = ctx->probs[pi];
        if (!P.rl) continue;
        DevProb& d = ctx->h_desc[pi];
        d.rtab = reinterpret_cast<const RealTab*>(ctx->d_real_tab + tab_off[pi]);
        d.rin = reinterpret_cast<double*>(base + off);  // [a | b]: 2 x 2^n doubles
        d.racc = base + off + ((size_t)1 << P.n_local);
        off += ((size_t)1 + 2 * (size_t)M) << P.n_local;
      }
    }
  }

  // ---- lanes ----
  // persistent: 2-tile problems on lane 0 (their workgroup pairs must be co-resident), 1-tile
  // problems on lane 1.  streaming: problems by degree dealt round-robin over the lanes.
  if (persistent) {
    // hand-off slots of the 2-tile problems: [2 tiles][kXSlots][2^L] amplitudes each
    // (dse_interval.hip)
    size_t need = 0;
    for (auto& P : ctx->probs)
      if (P.n_tiles == 2) need += (size_t)2 * kXSlots << P.L;
    if (need > ctx->xslot_cap) {
      if (ctx->d_xslots) (void)hipFree(ctx->d_xslots), ctx->d_xslots = nullptr;
      ctx->xslot_cap = 0;
      if (hipMalloc(&ctx->d_xslots, need * sizeof(double2)) != hipSuccess)
        return fail(ctx, DSE_ERR_OOM, "hand-off slot allocation failed (" +
                                          std::to_string(need * sizeof(double2)) + " bytes)");
      ctx->xslot_cap = need;
    }
    size_t off = 0;
    for (size_t pi = 0; pi < ctx->probs.size(); ++pi) {
      const HostProblem& P = ctx->probs[pi];
      ctx->h_desc[pi].xslots = P.n_tiles == 2 ? ctx->d_xslots + off : nullptr;
      if (P.n_tiles == 2) off += (size_t)2 * kXSlots << P.L;
    }
    // spanning registers: tables (one arena), descriptors, hand-off slots and flags
    size_t slot_need = 0, flag_need = 0;
    Arena tabs;
    std::vector<size_t> tab_off(ctx->probs.size(), 0);
    for (size_t pi = 0; pi < ctx->probs.size(); ++pi) {
      const HostProblem& P = ctx->probs[pi];
      if (!P.span_s) continue;
      const int Ls = P.n_local - P.span_s;
      SpanTab T;
      if (build_span_table(P, Ls, span_rb_for(ctx, Ls), P.span_s, T) != DSE_OK)
        return fail(ctx, DSE_ERR_ARG, "spanning-register tables do not fit (n = " + std::to_string(P.n) + ")");
      tab_off[pi] = tabs.add(&T, sizeof(T));
      slot_need += (size_t)(P.span_s + 1) * kXSlots << P.n_local;
      flag_need += (size_t)kSpanWaves << P.span_s;
    }
    if (flag_need > 0) {
      if ((rc = upload_arena(ctx, tabs, &ctx->d_span_tab, &ctx->span_tab_cap, ctx->lanes[0].stream))) return rc;
      HIPC(hipStreamSynchronize(ctx->lanes[0].stream));
      auto grow = [&](auto** ptr, size_t* cap, size_t need_bytes, const char* what) -> int {
        if (need_bytes <= *cap) return DSE_OK;
        if (*ptr) (void)hipFree(*ptr), *ptr = nullptr;
        *cap = 0;
        if (hipMalloc(ptr, need_bytes) != hipSuccess)
          return fail(ctx, DSE_ERR_OOM, std::string(what) + " allocation failed (" + std::to_string(need_bytes) + " bytes)");
        *cap = need_bytes;
        return DSE_OK;
      };
      if ((rc = grow(&ctx->d_span_slots, &ctx->span_slot_cap, slot_need * sizeof(double2), "span slot"))) return rc;
      if ((rc = grow(&ctx->d_span_flags, &ctx->span_flag_cap, flag_need * sizeof(int), "span flag"))) return rc;
      if ((rc = grow(&ctx->d_span, &ctx->span_cap, ctx->probs.size() * sizeof(SpanDesc), "span descriptor"))) return rc;
      std::vector<SpanDesc> sd(ctx->probs.size());
      size_t so = 0, fo = 0;
      for (size_t pi = 0; pi < ctx->probs.size(); ++pi) {
        const HostProblem& P = ctx->probs[pi];
        std::memset(&sd[pi], 0, sizeof(SpanDesc));
        if (!P.span_s) continue;
        sd[pi].tab = reinterpret_cast<const SpanTab*>(ctx->d_span_tab + tab_off[pi]);
        sd[pi].slots = ctx->d_span_slots + so;
        sd[pi].flags = ctx->d_span_flags + fo;
        sd[pi].s = P.span_s;
        sd[pi].L = P.n_local - P.span_s;
        so += (size_t)(P.span_s + 1) * kXSlots << P.n_local;
        fo += (size_t)kSpanWaves << P.span_s;
      }
      HIPC(hipMemcpy(ctx->d_span, sd.data(), sd.size() * sizeof(SpanDesc), hipMemcpyHostToDevice));
    }
  }
  HIPC(hipMemcpy(ctx->d_probs, ctx->h_desc.data(), ctx->h_desc.size() * sizeof(DevProb), hipMemcpyHostToDevice));
  // dist shards: one lane, so the RCCL exchanges are stream-ordered with every launch
  int n_big = 0;
  for (auto& P : ctx->probs) n_big += P.side() ? 0 : 1;
  const int n_lanes = any_dist ? 1 : std::max(1, std::min<int>(ctx->n_streams, n_big));
  bool imag_all = true;
  for (auto& P : ctx->probs) imag_all = imag_all && (P.side() || P.imag);
  // 2-tile interval launches go out in chunks whose workgroups can all be resident at once (the
  // pairs hand off every term): the occupancy query x compute units, even.
  int64_t pair_cap = 2;
  if (persistent) {
    int per_cu = 1;
    if (ctx->coresident > 0) {
      pair_cap = ctx->coresident;
    } else {
      HIPC(interval_occupancy(13, imag_all, &per_cu));
      pair_cap = (int64_t)std::max(1, per_cu) * ctx->n_cu;
    }
    pair_cap = std::max<int64_t>(2, pair_cap / 2 * 2);
  }
  const int64_t cap = pair_cap;
  // Mixed launches (option mixed_launch): the 1- and 2-tile problems of one tile size share one
  // launch per interval instead of one stream each, so the 1-tile problems run in the CUs the
  // light 2-tile problems leave, inside the launch, and never hold a CU the next launch's stiff
  // pairs need.  Only when every 2-tile workgroup fits at once (2P <= cap): the 1-tile problems
  // and the lightest pairs beyond the first cap workgroups are dispatched as CUs free up, and a
  // pair whose partner is still queued waits only for a workgroup that needs no partner.
  std::map<int, std::pair<int64_t, int64_t>> tiles_per_L;  // L -> (1-tile problems, 2-tile problems)
  for (auto& P : ctx->probs)
    if (!P.side() && !P.span_s && !P.rl && P.shard_bits == 0 && (P.n_tiles == 1 || P.n_tiles == 2))
      (P.n_tiles == 1 ? tiles_per_L[P.L].first : tiles_per_L[P.L].second) += 1;
  auto mixed_L = [&](const HostProblem& P) {
    if (!persistent || !ctx->mixed_launch || P.side() || P.span_s || P.rl || P.shard_bits != 0 || P.n_tiles > 2)
      return false;
    const auto it = tiles_per_L.find(P.L);
    return it != tiles_per_L.end() && it->second.first > 0 && it->second.second > 0 &&
           2 * it->second.second <= cap;
  };
  std::vector<int> order;
  for (size_t pi = 0; pi < ctx->probs.size(); ++pi)
    if (!ctx->probs[pi].side()) order.push_back((int)pi);
  std::stable_sort(order.begin(), order.end(), [&](int a, int b) {
    return ctx->probs[a].degree > ctx->probs[b].degree;
  });
  // lane -> (L, tiles per problem) -> problems
  std::vector<std::map<std::pair<int, int64_t>, std::vector<int>>> lane_probs(n_lanes);
  for (size_t i = 0; i < order.size(); ++i) {
    const HostProblem& P = ctx->probs[order[i]];
    const bool mixed = mixed_L(P);
    // tiles 0: a mixed group; < 0: spanning registers, -(16 L_span + rb)
    const int Ls = P.n_local - P.span_s;
    const std::pair<int, int64_t> key(P.L, P.rl ? -1000 : P.span_s ? -(16 * Ls + span_rb_for(ctx, Ls))
                                                                : (mixed ? 0 : P.n_tiles));
    int lane = (int)(i % n_lanes);
    if (persistent) lane = (P.n_tiles == 2 || n_lanes == 1 || mixed || P.span_s || P.rl) ? 0 : 1;
    // partial span: the spanned registers on a lane of their own, concurrent with k_interval's
    if (persistent && P.span_s && !all_span && n_lanes >= 2) lane = n_lanes >= 3 ? 2 : 1;
    // shards of one register read each other's vectors: same lane, hence the same launches
    if (P.shard_bits > 0 && !P.dist) lane = P.group_first % n_lanes;
    lane_probs[lane][key].push_back(order[i]);
  }
  std::vector<int2> items;
  items.reserve(ctx->total_items);
  ctx->item_pos.assign(ctx->probs.size(), 0);
  int max_deg = 1;
  for (int li = 0; li < (int)ctx->lanes.size(); ++li) {
    Lane& ln = ctx->lanes[li];
    ln.groups.clear();
    ln.max_deg = 0;
    if (li >= n_lanes) continue;
    for (auto& kv : lane_probs[li]) {
      LaneGroup g;
      g.L = kv.first.first;
      g.tiles = (int)kv.first.second;
      g.real = g.tiles == -1000;
      if (g.real) g.tiles = 1;  // no hand-off flags, no pair placement
      if (g.tiles < 0) g.span_L = (-g.tiles) / 16, g.span_rb = (-g.tiles) % 16;
      g.off = (int64_t)items.size();
      for (int pi : kv.second) {  // already in degree order
        ctx->item_pos[pi] = (int64_t)items.size();
        for (int64_t tt = 0; tt < ctx->probs[pi].n_tiles; ++tt) items.push_back(make_int2(pi, (int)tt));
        ln.max_deg = std::max(ln.max_deg, ctx->probs[pi].degree);
      }
      g.count = (int64_t)items.size() - g.off;
      g.wht_groups = persistent ? 0 : ctx->probs[kv.second.front()].wht_groups;
      for (int pi : kv.second)
        if (ctx->probs[pi].wht_groups != g.wht_groups) g.wht_groups = 0;
      g.wht_regs.clear();
      if (g.wht_groups)
        for (int pi : kv.second) {
          const HostProblem& P = ctx->probs[pi];
          if (P.shard_bits == 0) continue;
          const int first = P.dist ? pi : P.group_first;
          if (P.dist || P.shard_rank == 0) g.wht_regs.push_back({first, P.degree});
        }
      const int gdeg = ctx->probs[kv.second.front()].degree;
      g.active.assign(gdeg + 2, 0);
      g.bytes.assign(gdeg + 2, 0.0);
      g.flops.assign(gdeg + 2, 0.0);
      const double T = (double)(int64_t(1) << g.L);
      for (int k = 0; k <= gdeg + 1; ++k) {
        int64_t c = 0;
        double by = 0.0, fl = 0.0;
        for (int pi : kv.second) {
          const int K = ctx->probs[pi].degree;
          if (K < k) continue;
          c += ctx->probs[pi].n_tiles;
          fl += (double)ctx->probs[pi].n_tiles * T * ctx->probs[pi].flops_per_amp;
          // read w_{k-1}, read+write w_{k-2}/w_k (48 B/amp), plus acc read+write on update terms
          const bool upd = (k >= 2) && (((k - 1) % 3 == 0) || k == K);
          by += (double)ctx->probs[pi].n_tiles * T * (upd ? 80.0 : 48.0);
        }
        g.active[k] = (int)c;
        g.bytes[k] = by;
        g.flops[k] = fl;
      }
      ln.groups.push_back(std::move(g));
    }
    max_deg = std::max(max_deg, ln.max_deg);
  }
  HIPC(hipMemcpy(ctx->d_items, items.data(), items.size() * sizeof(int2), hipMemcpyHostToDevice));
  if (persistent) {
    // Interval-kernel order of 2-tile groups: the two tiles of a problem exchange data every
    // term, so place them 8 blocks apart -- blocks b and b + 8 land on one XCD under the
    // observed round-robin dispatch and then hand off through that XCD's L2 (speed only; the
    // hand-off protocol does not depend on placement).  Chunks of one launch are multiples of 16.
    std::vector<int2> iv = items;
    for (auto& ln : ctx->lanes)
      for (auto& g : ln.groups) {
        if (g.tiles == 0) {
          // mixed group: the stiffest pairs first (as many as fit beside the 1-tile problems), then
          // the 1-tile problems, then the remaining pairs, each segment in degree order; pairs in
          // blocks of 16 with their tiles 8 apart, as below
          std::vector<int2> pr, sg;
          for (int64_t i = 0; i < g.count; ++i) {
            const int2 e = items[g.off + i];
            (ctx->probs[e.x].n_tiles == 2 ? pr : sg).push_back(e);
          }
          const int64_t np = (int64_t)pr.size() / 2, ns = (int64_t)sg.size();
          const int64_t h = std::min<int64_t>(np, std::max<int64_t>(0, (cap - ns) / 2));
          int64_t o = g.off;
          auto put_pairs = [&](int64_t p0, int64_t p1) {
            for (int64_t b0 = p0; b0 < p1; b0 += 8) {
              const int64_t m = std::min<int64_t>(8, p1 - b0);
              if (ctx->xcd_pairs) {
                for (int64_t i = 0; i < m; ++i) {
                  iv[o + i] = pr[2 * (b0 + i)];
                  iv[o + m + i] = pr[2 * (b0 + i) + 1];
                }
              } else {
                for (int64_t i = 0; i < 2 * m; ++i) iv[o + i] = pr[2 * b0 + i];
              }
              o += 2 * m;
            }
          };
          put_pairs(0, h);
          for (const int2& e : sg) iv[o++] = e;
          put_pairs(h, np);
          continue;
        }
        if (g.tiles != 2 || !ctx->xcd_pairs) continue;
        for (int64_t off = 0; off < g.count; off += cap) {
          const int64_t cnt = std::min<int64_t>(cap, g.count - off);
          for (int64_t b0 = 0; b0 < cnt; b0 += 16) {
            const int64_t m = std::min<int64_t>(16, cnt - b0) / 2;  // problems in this block
            for (int64_t i = 0; i < m; ++i) {
              iv[g.off + off + b0 + i] = items[g.off + off + b0 + 2 * i];
              iv[g.off + off + b0 + m + i] = items[g.off + off + b0 + 2 * i + 1];
            }
          }
        }
      }
    HIPC(hipMemcpy(ctx->d_items_iv, iv.data(), iv.size() * sizeof(int2), hipMemcpyHostToDevice));
    // spanning groups: launch items (problem, tile); the tiles of one register 8 items apart, so
    // under the round-robin dispatch of workgroups to the 8 XCDs they share one XCD's L2 (speed
    // only), in blocks of 8 registers padded with items x = -1 (return at once)
    std::vector<int2> sitems;
    for (auto& ln : ctx->lanes)
      for (auto& g : ln.groups) {
        if (g.tiles >= 0) continue;
        std::vector<int> pis;
        for (int64_t i = 0; i < g.count; ++i) {
          const int2 e = items[g.off + i];
          if (pis.empty() || pis.back() != e.x) pis.push_back(e.x);
        }
        g.span_off = (int64_t)sitems.size();
        int per_cu = 1;
        HIPC(span_occupancy(g.span_L, g.span_rb, imag_all, &per_cu));
        const int64_t resident = (int64_t)std::max(1, per_cu) * ctx->n_cu;
        g.span_cuts.assign(1, 0);
        g.span_am.assign(1, 0.0);
        g.span_fl.assign(1, 0.0);
        for (size_t b0 = 0; b0 < pis.size(); b0 += 8) {
          int s = 0;  // the block's widest register sets its size (span_tile mixes 13 and 14 qubits)
          for (size_t i = b0; i < std::min(pis.size(), b0 + 8); ++i) s = std::max(s, ctx->probs[pis[i]].span_s);
          const size_t base = sitems.size();
          if ((int64_t)(base + ((size_t)8 << s)) - g.span_off - g.span_cuts.back() > resident &&
              (int64_t)base - g.span_off > g.span_cuts.back()) {
            g.span_cuts.push_back((int64_t)base - g.span_off);  // this block starts the next launch
            g.span_am.push_back(0.0);
            g.span_fl.push_back(0.0);
          }
          for (size_t i = b0; i < std::min(pis.size(), b0 + 8); ++i) {
            const HostProblem& P = ctx->probs[pis[i]];
            g.span_am.back() += std::ldexp(1.0, P.n_local) * P.degree;
            g.span_fl.back() += std::ldexp(1.0, P.n_local) * P.degree * P.flops_per_amp;
          }
          sitems.resize(base + ((size_t)8 << s), make_int2(-1, 0));
          for (size_t i = b0; i < std::min(pis.size(), b0 + 8); ++i)
            for (int h = 0; h < (1 << ctx->probs[pis[i]].span_s); ++h)
              sitems[base + (size_t)h * 8 + (i - b0)] = make_int2(pis[i], h);
        }
        g.span_count = (int64_t)sitems.size() - g.span_off;
        g.span_cuts.push_back(g.span_count);
      }
    // real-component groups: items (problem, component) in degree order, then (problem, 0) per
    // problem for the combine launch
    std::vector<int2> ritems;
    for (auto& ln : ctx->lanes)
      for (auto& g : ln.groups) {
        if (!g.real) continue;
        std::vector<int> pis;
        for (int64_t i = 0; i < g.count; ++i) {
          const int2 e = items[g.off + i];
          if (pis.empty() || pis.back() != e.x) pis.push_back(e.x);
        }
        g.real_off = (int64_t)ritems.size();
        for (int pi : pis) ritems.push_back(make_int2(pi, 0)), ritems.push_back(make_int2(pi, 1));
        g.real_count = (int64_t)ritems.size() - g.real_off;
        g.real_poff = (int64_t)ritems.size();
        for (int pi : pis) ritems.push_back(make_int2(pi, 0));
        g.real_np = (int64_t)pis.size();
      }
    if (!ritems.empty()) {
      if (ritems.size() > ctx->real_items_cap) {
        if (ctx->d_real_items) (void)hipFree(ctx->d_real_items), ctx->d_real_items = nullptr;
        ctx->real_items_cap = 0;
        if (hipMalloc(&ctx->d_real_items, ritems.size() * sizeof(int2)) != hipSuccess)
          return fail(ctx, DSE_ERR_OOM, "real item allocation failed");
        ctx->real_items_cap = ritems.size();
      }
      HIPC(hipMemcpy(ctx->d_real_items, ritems.data(), ritems.size() * sizeof(int2), hipMemcpyHostToDevice));
    }
    if (!sitems.empty()) {
      if (sitems.size() > ctx->span_items_cap) {
        if (ctx->d_span_items) (void)hipFree(ctx->d_span_items), ctx->d_span_items = nullptr;
        ctx->span_items_cap = 0;
        if (hipMalloc(&ctx->d_span_items, sitems.size() * sizeof(int2)) != hipSuccess)
          return fail(ctx, DSE_ERR_OOM, "span item allocation failed");
        ctx->span_items_cap = sitems.size();
      }
      HIPC(hipMemcpy(ctx->d_span_items, sitems.data(), sitems.size() * sizeof(int2), hipMemcpyHostToDevice));
    }
  }
  if (persistent) {
    const size_t need = 2 * kIvWaves * ctx->probs.size() + 1;  // flags, error word
    if (ctx->flags_cap < need) {
      if (ctx->d_flags) (void)hipFree(ctx->d_flags), ctx->d_flags = nullptr;
      if (hipMalloc(&ctx->d_flags, need * sizeof(int)) != hipSuccess)
        return fail(ctx, DSE_ERR_OOM, "flag allocation failed");
      ctx->flags_cap = need;
    }
    HIPC(hipMemset(ctx->d_flags, 0, need * sizeof(int)));
  }
  int* d_err = persistent ? ctx->d_flags + 2 * kIvWaves * ctx->probs.size() : nullptr;
  ctx->d_err_cur = d_err;  // checked by every flush_partials (reset by dse_evolve on return)

  phase("lanes/items");
  // ---- psi(t0) = |psi0> ----
  hipStream_t st0 = ctx->lanes[0].stream;
  {
    std::vector<BasisInit> init;
    uint64_t max_amps = 0;
    for (auto& P : ctx->probs) {
      // the re-run after a hand-off timeout keeps the dense registers' first-pass results, whose
      // final state k_dense_final wrote into buf[0]
      if (ctx->rerun && P.dn) continue;
      BasisInit e;
      e.ptr = P.buf[0];
      e.n = uint64_t(1) << P.n_local;
      // the shard holding psi0 (every unsharded register)
      e.one_at = ((P.psi0 >> P.n_local) == (uint64_t)P.shard_rank)
                     ? (int64_t)(P.psi0 & ((uint64_t(1) << P.n_local) - 1)) : -1;
      init.push_back(e);
      max_amps = std::max(max_amps, e.n);
    }
    if (init.size() > ctx->init_cap) {
      if (ctx->d_init) (void)hipFree(ctx->d_init), ctx->d_init = nullptr;
      ctx->init_cap = 0;
      if (hipMalloc(&ctx->d_init, init.size() * sizeof(BasisInit)) != hipSuccess)
        return fail(ctx, DSE_ERR_OOM, "initial-state list allocation failed");
      ctx->init_cap = init.size();
    }
    if (ctx->dbg & 2) {
      for (auto& e : init) {
        HIPC(hipMemsetAsync(e.ptr, 0, e.n * sizeof(double2), st0));
        static const double2 one = {1.0, 0.0};
        if (e.one_at >= 0) HIPC(hipMemcpyAsync(e.ptr + e.one_at, &one, sizeof(double2), hipMemcpyHostToDevice, st0));
      }
    } else {
      HIPC(hipMemcpyAsync(ctx->d_init, init.data(), init.size() * sizeof(BasisInit), hipMemcpyHostToDevice, st0));
      for (size_t i0 = 0; i0 < init.size(); i0 += 65535)
        HIPC(launch_basis_init(ctx->d_init + i0, (int)std::min<size_t>(65535, init.size() - i0), max_amps, st0));
    }
    for (auto& ln : ctx->lanes)  // real-component registers: [a | b] = [e_x0 | 0]
      for (auto& g : ln.groups)
        if (g.real) HIPC(launch_real_init(ctx->d_probs, ctx->d_real_items + g.real_poff, (int)g.real_np, st0));
    HIPC(hipStreamSynchronize(st0));
  }
  double small_happl = 0.0, small_launches = 0.0;
  if (any_small && (rc = small_launch(ctx, t, n_t, tol, &small_happl, &small_launches))) return rc;

  double dense_ms = 0.0, dense_eig_ms = 0.0;
  // (the re-run after a hand-off timeout keeps the first pass's dense results: dense_run completed
  // and wrote them before any interval launch, and its register choice depends only on t)
  if (any_dense && !ctx->rerun && (rc = dense_run(ctx, t, n_t, obs_out, &dense_ms, &dense_eig_ms))) return rc;
  double matrix_happl = 0.0;
  if (matrix_pi >= 0 && (rc = matrix_run(ctx, matrix_pi, t, n_t, matrix_dt, tol, obs_out, &matrix_happl))) return rc;
  phase("psi0/small");
  const size_t chunk = (size_t)std::max<int64_t>(M, std::min<int64_t>(
      n_t, std::max<int64_t>(1, (int64_t)(256ll << 20) / (ctx->total_items * 64))));
  if ((rc = ensure_partial(ctx, chunk))) return rc;
  if (ctx->time_every > 0)
    for (auto& ln : ctx->lanes) {
      // timed launches per interval and pool: one per term and group (streaming), one per
      // co-resident chunk and group (persistent); records beyond the pool are skipped, not timed
      size_t need = 1;
      for (const auto& g : ln.groups)
        need += persistent ? (g.tiles < 0 ? g.span_cuts.size() - 1 : (size_t)((g.count + cap - 1) / cap))
                           : (size_t)(ln.max_deg + 1);
      if ((rc = ensure_events(ctx, ln, need))) return rc;
    }

  double step_ms = 0.0, launches_timed = 0.0, bytes_timed = 0.0, amps_timed = 0.0;
  double lane0_ms = 0.0, lane0_launches = 0.0, lane0_amps = 0.0;  // lane 0 alone (stats)
  double launches = 0.0, amp_updates = 0.0, all_bytes = 0.0, all_flops = 0.0, flops_timed = 0.0;
  // per timed launch: algorithmic flops (pool_bytes), HBM bytes (pool_bytes2, streaming only) and
  // amplitude-terms (pool_amps: amplitudes x Chebyshev terms the launch computes)
  std::vector<std::vector<double>> pool_bytes(ctx->lanes.size() * 2), pool_bytes2(ctx->lanes.size() * 2),
      pool_amps(ctx->lanes.size() * 2);
  auto drain = [&](Lane& ln, size_t li, int pool) -> int {
    if (ln.ev_used[pool] == 0) return DSE_OK;
    HIPC(hipEventSynchronize(ln.ev[pool][2 * ln.ev_used[pool] - 1]));
    for (size_t i = 0; i < ln.ev_used[pool]; ++i) {
      float ms = 0.f;
      HIPC(hipEventElapsedTime(&ms, ln.ev[pool][2 * i], ln.ev[pool][2 * i + 1]));
      step_ms += ms;
      flops_timed += pool_bytes[li * 2 + pool][i];
      amps_timed += pool_amps[li * 2 + pool][i];
      if (li == 0) lane0_ms += ms, lane0_amps += pool_amps[li * 2 + pool][i], lane0_launches += 1.0;
      if (i < pool_bytes2[li * 2 + pool].size()) bytes_timed += pool_bytes2[li * 2 + pool][i];
    }
    launches_timed += (double)ln.ev_used[pool];
    ln.ev_used[pool] = 0;
    pool_bytes[li * 2 + pool].clear();
    pool_bytes2[li * 2 + pool].clear();
    pool_amps[li * 2 + pool].clear();
    return DSE_OK;
  };
  // observables of n_out consecutive output slots (one launch per lane group): outputs
  // j < n_out - 1 from the intermediate accumulators, the last from state role bsel_q
  // obs_ovl: on each lane's obs_stream behind the lane's interval launches of parity xq (event
  // ev_iv[xq]), then ev_obs[xq] for the launches two groups later, which rewrite these buffers
  auto obs_all = [&](int bsel_q, size_t slot, int n_out, int xq) -> int {
    for (auto& ln : ctx->lanes) {
      if (ln.groups.empty()) continue;
      hipStream_t os = obs_ovl ? ln.obs_stream : ln.stream;
      if (obs_ovl) {
        HIPC(hipEventRecord(ln.ev_iv[xq], ln.stream));
        HIPC(hipStreamWaitEvent(os, ln.ev_iv[xq], 0));
      }
      for (auto& g : ln.groups)
        HIPC(launch_obs(g.L, ctx->d_probs, ctx->d_items + g.off, (int)g.count, bsel_q,
                        ctx->d_partial + (slot * ctx->total_items + g.off) * 8, os, n_out,
                        (size_t)ctx->total_items * 8, xq));
      if (obs_ovl) {
        HIPC(hipEventRecord(ln.ev_obs[xq], os));
        ln.obs_pending[xq] = true;
      }
    }
    return DSE_OK;
  };
  for (auto& ln : ctx->lanes) ln.obs_pending[0] = ln.obs_pending[1] = false;

  std::vector<double> dist_raw(any_dist ? ctx->probs.size() * (size_t)n_t * 7 : 0, 0.0);
  size_t slot = 0, t_flushed = 0;
  if (any_dist && (rc = dist_exchange(ctx, 0, 0, ctx->lanes[0].stream))) return rc;
  if ((rc = obs_all(0, slot++, 1, 1))) return rc;
  for (int gi = 0; gi < n_groups; ++gi) {
    const Group& G = groups[gi];
    const int q = gi & 1;
    const int set = G.set;
    const bool timed = ctx->time_every > 0 && (gi % ctx->time_every) == 0;
    const int pool = gi & 1;
    for (size_t li = 0; li < ctx->lanes.size(); ++li) {
      Lane& ln = ctx->lanes[li];
      if (ln.groups.empty()) continue;
      if ((rc = drain(ln, li, pool))) return rc;
      if (obs_ovl && ln.obs_pending[q]) {  // the observables that read what this group rewrites
        HIPC(hipStreamWaitEvent(ln.stream, ln.ev_obs[q], 0));
        ln.obs_pending[q] = false;
      }
      for (auto& g : ln.groups) {
        const int T = 1 << g.L;
        if (persistent) {
          // all K terms of the interval in one launch; 2-tile groups in co-resident chunks;
          // spanning registers: one k_span launch per chunk of span_cuts (each chunk's registers'
          // tiles all resident at once: the cuts are sized to the chip's resident capacity), flags
          // zeroed first
          if (g.tiles < 0) HIPC(hipMemsetAsync(ctx->d_span_flags, 0, ctx->span_flag_cap, ln.stream));
          else if (g.tiles != 1) HIPC(zero_flags(ctx->d_items + g.off, (int)g.count, ctx->d_flags, ln.stream));
          auto launch_g = [&](int64_t off, int cnt) -> hipError_t {
            if (g.real)
              return launch_real(ctx->d_probs, ctx->d_real_items + g.real_off, (int)g.real_count, set, G.n_out,
                                 ln.stream);
            if (g.tiles < 0)  // chunk [off, off + cnt) of the group's span launches
              return launch_span(g.span_L, g.span_rb, imag_all, ctx->d_probs, ctx->d_span,
                                 ctx->d_span_items + g.span_off + g.span_cuts[off],
                                 (int)(g.span_cuts[off + cnt] - g.span_cuts[off]), q, set, G.n_out, d_err, ctx->hk,
                                 ln.stream);
            return launch_interval(g.L, imag_all, ctx->d_probs, ctx->d_items_iv + g.off + off, cnt, q, set, G.n_out,
                                   ctx->d_flags, d_err, ctx->hk, ln.stream);
          };
          // mixed (0): one launch; 2-tile: co-resident chunks of cap items; span (< 0): one launch
          // per chunk of span_cuts (off / cnt then count chunks, not items)
          const int64_t gcap = g.tiles == 2 ? cap : g.tiles < 0 ? 1 : g.count;
          const int64_t gn = g.tiles < 0 ? (int64_t)g.span_cuts.size() - 1 : g.count;
          for (int64_t off = 0; off < gn; off += gcap) {
            const int cnt = (int)std::min<int64_t>(gcap, gn - off);
            double fl = 0.0, am = 0.0;
            if (g.tiles < 0) {  // the chunk's registers
              am = g.span_am[off];
              fl = g.span_fl[off];
            } else {
              for (int64_t i = off; i < off + cnt; ++i) {
                const HostProblem& P = ctx->probs[items[g.off + i].x];
                am += (double)T * P.degree;
                fl += (double)T * P.degree * P.flops_per_amp;
              }
            }
            if (timed && 2 * ln.ev_used[pool] + 2 <= ln.ev[pool].size()) {
              const size_t i = ln.ev_used[pool]++;
              HIPC(hipEventRecord(ln.ev[pool][2 * i], ln.stream));
              HIPC(launch_g(off, cnt));
              HIPC(hipEventRecord(ln.ev[pool][2 * i + 1], ln.stream));
              pool_bytes[li * 2 + pool].push_back(fl);
              pool_amps[li * 2 + pool].push_back(am);
            } else {
              HIPC(launch_g(off, cnt));
            }
            launches += 1.0;
            amp_updates += am;
            all_flops += fl;
          }
          // real-component registers: psi of every output (computational frame) and the next [a | b]
          if (g.real)
            HIPC(launch_real_combine(ctx->d_probs, ctx->d_real_items + g.real_poff, (int)g.real_np, q, G.n_out,
                                     ln.stream));
          continue;
        }
        if (any_dist_step && (rc = dist_exchange(ctx, q ? 2 : 0, 1, ln.stream))) return rc;
        auto step = [&](int mode, int na, int k) -> int {
          if (g.wht_groups) {
            std::vector<int> regs;
            for (const auto& rg : g.wht_regs)
              if (rg.second >= k) regs.push_back(rg.first);
            return wht_run(ctx, g.L, g.wht_groups, {{ctx->d_items + g.off, na}}, regs, mode, k, q, set, ln.stream);
          }
          HIPC(launch_step(g.L, mode, ctx->d_probs, ctx->d_items + g.off, na, k, q, set, ln.stream));
          return DSE_OK;
        };
        if ((rc = step(MODE_FIRST, g.active[1], 1))) return rc;
        for (int k = 2; k < (int)g.active.size(); ++k) {
          const int na = g.active[k];
          if (na <= 0) break;
          if (any_dist_step && (rc = dist_exchange(ctx, ((k - 1) & 1) ? 1 : (q ? 2 : 0), k, ln.stream)))
            return rc;
          if (timed && 2 * ln.ev_used[pool] + 2 <= ln.ev[pool].size()) {
            const size_t i = ln.ev_used[pool]++;
            HIPC(hipEventRecord(ln.ev[pool][2 * i], ln.stream));
            if ((rc = step(MODE_GEN, na, k))) return rc;
            HIPC(hipEventRecord(ln.ev[pool][2 * i + 1], ln.stream));
            pool_bytes[li * 2 + pool].push_back(g.flops[k]);
            pool_bytes2[li * 2 + pool].push_back(g.bytes[k]);
            pool_amps[li * 2 + pool].push_back((double)na * T);
          } else {
            if ((rc = step(MODE_GEN, na, k))) return rc;
          }
          launches += 1.0;
          amp_updates += (double)na * T;
          all_bytes += g.bytes[k];
          all_flops += g.flops[k];
        }
      }
    }
    // new psi of every problem sits in acc(q) = buf[q ? 0 : 2]; outputs j < n_out - 1 of a
    // multi-output launch in the intermediate accumulators
    if (any_dist && (rc = dist_exchange(ctx, q ? 0 : 2, 0, ctx->lanes[0].stream))) return rc;
    if (slot + G.n_out > chunk) {  // the group's outputs share one launch: one chunk
      if ((rc = flush_partials(ctx, slot, t_flushed, n_t, obs_out, &dist_raw))) return rc;
      t_flushed += slot;
      slot = 0;
    }
    if (ctx->dbg & 1) {
      for (int j = 0; j < G.n_out; ++j) {
        for (auto& ln : ctx->lanes)
          for (auto& g : ln.groups)
            HIPC(launch_obs(g.L, ctx->d_probs, ctx->d_items + g.off, (int)g.count,
                            j == G.n_out - 1 ? (q ? 0 : 2) : 3 + j,
                            ctx->d_partial + ((slot + j) * ctx->total_items + g.off) * 8, ln.stream,
                            1, 0, q));
      }
    } else if ((rc = obs_all(q ? 0 : 2, slot, G.n_out, q))) {
      return rc;
    }
    slot += G.n_out;
    if (slot == chunk) {
      if ((rc = flush_partials(ctx, slot, t_flushed, n_t, obs_out, &dist_raw))) return rc;
      t_flushed += slot;
      slot = 0;
    }
  }
  phase("launch loop");
  if (slot > 0) {
    if ((rc = flush_partials(ctx, slot, t_flushed, n_t, obs_out, &dist_raw))) return rc;
    t_flushed += slot;
  }
  for (size_t li = 0; li < ctx->lanes.size(); ++li)
    for (int pool = 0; pool < 2; ++pool)
      if ((rc = drain(ctx->lanes[li], li, pool))) return rc;
  if ((rc = sync_all(ctx))) return rc;
  if ((rc = small_gather(ctx, n_t, obs_out))) return rc;
  phase("flush/drain");
  if (persistent && any_big) {
    int herr = 0;
    HIPC(hipMemcpy(&herr, d_err, sizeof(int), hipMemcpyDeviceToHost));
    if (herr) return kRcHandoffTimeout;
  }
  if (any_dist) {  // sums over all shards of the register, then normalisation (finish_obs)
    if ((rc = xchg_allreduce_host(ctx, dist_raw.data(), dist_raw.size(), ctx->lanes[0].stream))) return rc;
    for (size_t pi = 0; pi < ctx->probs.size(); ++pi) {
      if (!ctx->probs[pi].dist) continue;
      for (int ti = 0; ti < n_t; ++ti)
        finish_obs(ctx->probs[pi], dist_raw.data() + (pi * (size_t)n_t + ti) * 7,
                   obs_out + pi * DSE_N_OBS * (size_t)n_t + ti, (size_t)n_t);
    }
  }
  phase("tail");
  ctx->last_q = n_groups & 1;
  for (auto& P : ctx->probs) P.final_bsel = P.side() ? 0 : (ctx->last_q ? 2 : 0);
  ctx->evolved = true;

  if (stats) {
    double happl = small_happl + matrix_happl;
    for (auto& P : ctx->probs)
      if (!P.side()) happl += (double)P.degree * n_groups;
    std::memset(stats, 0, sizeof(*stats));
    stats->h_applications = happl;
    stats->amplitude_updates = amp_updates;
    stats->step_bytes = all_bytes;
    stats->h_flops = all_flops;
    stats->timed_flops = flops_timed;
    stats->timed_amp_terms = amps_timed;
    stats->mode = matrix_pi >= 0 ? 5 : (!any_big ? (any_dense ? 4 : 3) : (persistent ? 1 : (used_wht ? 2 : 0)));
    int n_dense = 0;
    for (auto& P : ctx->probs) n_dense += P.dn ? 1 : 0;
    stats->dense_problems = n_dense;
    int n_span = 0;
    for (auto& P : ctx->probs) n_span += P.span_s ? 1 : 0;
    stats->span_problems = n_span;
    int n_real = 0;
    for (auto& P : ctx->probs) n_real += P.rl ? 1 : 0;
    stats->real_problems = n_real;
    stats->eig_fallbacks = ctx->eig_fallbacks.load();
    stats->dense_ms = dense_ms;
    stats->dense_eig_ms = dense_eig_ms;
    stats->dense_nufft_problems = any_dense ? ctx->nufft_problems : 0;
    stats->dense_output_ms = any_dense ? ctx->dense_out_ms : 0.0;
    stats->step_kernel_ms = launches_timed > 0 ? step_ms : -1.0;
    stats->step_launches = launches + small_launches;
    stats->timed_launches = launches_timed;
    stats->timed_bytes = bytes_timed;
    stats->wall_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - wall0).count();
    for (auto& P : ctx->probs)
      if (P.sm || P.mx) max_deg = std::max(max_deg, P.degree);
    stats->max_degree = max_deg;
    stats->n_intervals = n_t - 1;
    stats->tile_bits = ctx->probs.empty() ? 0 : ctx->probs.front().L;
    stats->streams = n_lanes;
    stats->outputs_per_launch = M;
    stats->handoff_fallbacks = ctx->handoff_fallbacks;
    stats->exchange_bytes = ctx->xbytes;
    if ((rc = xt_sum(ctx))) return rc;
    stats->exchange_ms = ctx->xms;
    stats->lane0_kernel_ms = lane0_ms;
    stats->lane0_launches = lane0_launches;
    stats->lane0_amp_terms = lane0_amps;
    if (matrix_pi >= 0) {
      stats->matrix_build_ms = ctx->mx_build_ms;
      stats->matrix_products_ms = ctx->mx_products_ms;
      stats->matrix_products = ctx->mx_products;
      stats->matrix_bytes_per_product = ctx->mx_bytes_per_product;
    }
  }
  return DSE_OK;
}

int dse_evolve(dse_ctx* ctx, const double* t, int n_t, double tol, double* obs_out, dse_stats* stats) {
  if (!ctx) return DSE_ERR_ARG;
  ctx->handoff_fallbacks = 0;
  ctx->eig_fallbacks = 0;
  int rc = evolve_impl(ctx, t, n_t, tol, obs_out, stats);
  int* const d_err = ctx->d_err_cur;
  ctx->d_err_cur = nullptr;
  if (rc != kRcHandoffTimeout) return rc;
  // A workgroup pair of a 2-tile problem was not resident together within the spin limit (the
  // device shared with long-running work of another stream or process).  The first flush after
  // the timeout saw it (launches queued behind it return at once: k_interval checks the error
  // word on entry), so the call runs again on the per-term streaming kernels, which have no
  // inter-workgroup dependency.
  (void)sync_all(ctx);
  const int zero = 0;
  HIPC(hipMemcpy(d_err, &zero, sizeof(int), hipMemcpyHostToDevice));
  const int saved = ctx->persistent;
  ctx->persistent = 0;
  ctx->rerun = true;
  rc = evolve_impl(ctx, t, n_t, tol, obs_out, stats);
  ctx->rerun = false;
  ctx->persistent = saved;
  ctx->d_err_cur = nullptr;
  ctx->handoff_fallbacks = 1;
  if (stats) stats->handoff_fallbacks = 1;
  return rc;
}

int dse_get_state(dse_ctx* ctx, int problem, double* psi_out) {
  if (!ctx) return DSE_ERR_ARG;
  if (problem < 0 || problem >= (int)ctx->probs.size()) return fail(ctx, DSE_ERR_ARG, "bad problem id");
  if (!psi_out) return fail(ctx, DSE_ERR_ARG, "null state");
  if (!ctx->evolved) return fail(ctx, DSE_ERR_STATE, "no evolved state (call dse_evolve first)");
  HIPC(hipSetDevice(ctx->device));
  int first = 0, count = 1;
  int rc = hook_members(ctx, problem, &first, &count);
  if (rc) return rc;
  double2* out = reinterpret_cast<double2*>(psi_out);
  for (int i = 0; i < count; ++i) {
    HostProblem& P = ctx->probs[first + i];
    const size_t amps = size_t(1) << P.n_local;
    HIPC(hipMemcpy(out + i * amps, P.buf[P.final_bsel], amps * sizeof(double2), hipMemcpyDeviceToHost));
  }
  return DSE_OK;
}

int dse_energy(dse_ctx* ctx, int problem, double* e_out) {
  if (!ctx) return DSE_ERR_ARG;
  if (!e_out) return fail(ctx, DSE_ERR_ARG, "null pointer");
  if (!ctx->evolved) return fail(ctx, DSE_ERR_STATE, "no evolved state (call dse_evolve first)");
  int first = 0, count = 1;
  int rc = hook_members(ctx, problem, &first, &count);
  if (rc) return rc;
  if (ctx->probs[first].dist) return fail(ctx, DSE_ERR_ARG, "dse_energy: not available for a dist shard");
  HIPC(hipSetDevice(ctx->device));
  hipStream_t st = ctx->lanes[0].stream;
  for (int i = 0; i < count; ++i) {  // H reads buf[0]: copy the state there (it stays in its buffer)
    HostProblem& P = ctx->probs[first + i];
    if (P.final_bsel != 0)
      HIPC(hipMemcpyAsync(P.buf[0], P.buf[P.final_bsel], (size_t(1) << P.n_local) * sizeof(double2),
                          hipMemcpyDeviceToDevice, st));
  }
  if ((rc = apply_members(ctx, first, count, st))) return rc;
  constexpr int kBlocks = 1024;
  double* d = nullptr;
  HIPC(hipMalloc(&d, (size_t)count * kBlocks * 2 * sizeof(double)));
  hipError_t e = hipSuccess;
  for (int i = 0; i < count && e == hipSuccess; ++i) {
    const HostProblem& P = ctx->probs[first + i];
    e = launch_dot(P.buf[0], P.buf[1], size_t(1) << P.n_local, d + (size_t)i * kBlocks * 2, kBlocks, st);
  }
  std::vector<double> h((size_t)count * kBlocks * 2);
  if (e == hipSuccess) e = hipMemcpyAsync(h.data(), d, h.size() * sizeof(double), hipMemcpyDeviceToHost, st);
  if (e == hipSuccess) e = hipStreamSynchronize(st);
  (void)hipFree(d);
  HIPC(e);
  double en = 0.0, n2 = 0.0;
  for (size_t b = 0; b < h.size(); b += 2) {
    en += h[b];
    n2 += h[b + 1];
  }
  e_out[0] = n2 > 0.0 ? en / n2 : 0.0;
  e_out[1] = n2;
  return DSE_OK;
}

int dse_time_step_kernel(dse_ctx* ctx, int reps, double* ms_per_launch, double* bytes_per_launch) {
  if (!ctx) return DSE_ERR_ARG;
  if (reps < 1 || !ms_per_launch || !bytes_per_launch) return fail(ctx, DSE_ERR_ARG, "bad arguments");
  if (!ctx->evolved) return fail(ctx, DSE_ERR_STATE, "call dse_evolve first (coefficients needed)");
  HIPC(hipSetDevice(ctx->device));
  Lane& ln = ctx->lanes[0];
  int rc = ensure_events(ctx, ln, (size_t)reps);
  if (rc) return rc;
  // one launch over every item of every lane: the whole batch at term k = 2
  std::vector<int2> items(ctx->total_items);
  HIPC(hipMemcpy(items.data(), ctx->d_items, items.size() * sizeof(int2), hipMemcpyDeviceToHost));
  std::map<int, std::vector<int2>> by_L;
  if (ctx->probe_items > 0 && (int64_t)items.size() > ctx->probe_items) items.resize(ctx->probe_items);
  for (auto& it : items) by_L[ctx->probs[it.x].L].push_back(it);
  int2* d_tmp = nullptr;
  HIPC(hipMalloc(&d_tmp, items.size() * sizeof(int2)));
  double bytes = 0.0, tot = 0.0;
  int64_t off = 0;
  std::vector<std::pair<int, int64_t>> segs;
  for (auto& kv : by_L) {
    HIPC(hipMemcpy(d_tmp + off, kv.second.data(), kv.second.size() * sizeof(int2), hipMemcpyHostToDevice));
    segs.push_back({kv.first, off});
    off += (int64_t)kv.second.size();
    bytes += 48.0 * (double)kv.second.size() * (double)(1 << kv.first);
  }
  for (int r = 0; r < reps; ++r) {
    HIPC(hipEventRecord(ln.ev[0][2 * r], ln.stream));
    for (size_t s = 0; s < segs.size(); ++s) {
      const int64_t cnt = (s + 1 < segs.size() ? segs[s + 1].second : off) - segs[s].second;
      HIPC(launch_step(segs[s].first, MODE_GEN, ctx->d_probs, d_tmp + segs[s].second, (int)cnt, 2, 0, 0, ln.stream));
    }
    HIPC(hipEventRecord(ln.ev[0][2 * r + 1], ln.stream));
  }
  HIPC(hipStreamSynchronize(ln.stream));
  for (int r = 0; r < reps; ++r) {
    float ms = 0.f;
    HIPC(hipEventElapsedTime(&ms, ln.ev[0][2 * r], ln.ev[0][2 * r + 1]));
    tot += ms;
  }
  (void)hipFree(d_tmp);
  *ms_per_launch = tot / reps;
  *bytes_per_launch = bytes;
  ctx->evolved = false;  // buffers now hold timing garbage
  return DSE_OK;
}

}  // extern "C"
