/*
 * dse.h -- C ABI of the MI355X dipolar spin-ensemble state-vector engine (libdse.so).
 *
 * The reference has no native boundary: its only solver entry is the Python call
 *   simulate_rare(params) -> (t, obs)          dipolar_ensemble_with_rare.py:611-680
 * which builds H with QuTiP (:453-588), prepares psi0 (:591-606) and hands both to
 *   qt.sesolve(H, psi0, t, e_ops=[6 ops], options)   dipolar_ensemble_with_rare.py:653-666
 * The functions below replace that sesolve call (and the operator algebra feeding it)
 * for any number of independent evolutions per device.  The Python host
 * (quantumsimulations_amd/dipolar_ensemble_with_rare.py) reduces a DipolarRareParams to the
 * coefficient tables taken by dse_add_problem and calls dse_evolve; INTEGRATION.md shows the
 * ctypes binding a maintainer of the reference would add.
 *
 * Conventions
 *   - A problem is an n-qubit register, state = 2^n complex doubles, interleaved (re, im).
 *   - s_b(x) = 1/2 - bit_b(x); bit value 0 = spin up (QuTiP basis(2, 0)).
 *   - H x-th row:  D(x) psi[x]
 *                + sum_b flip(b, bit_b(x)) psi[x ^ e_b]
 *                + sum_{i<j, bit_i(x)==bit_j(x)} pair[i][j] psi[x ^ e_i ^ e_j]
 *     D(x) = shift + sum_b field[b] s_b(x) + sum_{i<j} zz[i][j] s_i(x) s_j(x).
 *     flip is given as 4 doubles per bit: (re0, im0, re1, im1) where index v = bit_b(x) is the
 *     bit value of the OUTPUT row; H must be Hermitian: (re1, im1) = conj(re0, im0).
 *   - Observables (dse_obs order = the key order of simulate_rare's dict, :671-679):
 *       Ix_sea, Iy_sea, Iz_sea: sums over the bits of sea_mask;  Iz_R, Ix_R, Iy_R on rare_bit
 *       (rare_bit < 0: the rare spin is not in the register; Iz_R = rare_z_const, Ix_R = Iy_R = 0);
 *       state_norm = ||psi||.  Expectations are of the normalised state (QuTiP 5 normalize_output).
 *   - Status: 0 = ok, negative = error; dse_last_error(ctx) has the message.  No C++ exception
 *     crosses this boundary.
 *   - Threading: a context is bound to one device and is not thread-safe; distinct contexts are.
 *     Calls block until results are in host memory.
 */
#ifndef DSE_H
#define DSE_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define DSE_ABI_VERSION 13
#define DSE_MAX_QUBITS 34
#define DSE_N_OBS 7

enum dse_status {
  DSE_OK = 0,
  DSE_ERR_ARG = -1,         /* invalid argument (reference: ValueError, :620-621)           */
  DSE_ERR_OOM = -2,         /* device or host allocation failed                             */
  DSE_ERR_HIP = -3,         /* HIP runtime error                                             */
  DSE_ERR_CONVERGENCE = -4, /* Chebyshev degree cap exceeded (reference: sesolve failure)    */
  DSE_ERR_STATE = -5,       /* call order (e.g. dse_get_state before dse_evolve)             */
  DSE_ERR_NODEVICE = -6     /* no HIP device / bad device index                             */
};

enum dse_obs {
  DSE_OBS_IX_SEA = 0,
  DSE_OBS_IY_SEA = 1,
  DSE_OBS_IZ_SEA = 2,
  DSE_OBS_IZ_R = 3,
  DSE_OBS_IX_R = 4,
  DSE_OBS_IY_R = 5,
  DSE_OBS_NORM = 6
};

typedef struct dse_ctx dse_ctx;

/* Per-call counters filled by dse_evolve (all sums over every problem of the context). */
typedef struct dse_stats {
  double h_applications;      /* Chebyshev terms = applications of H, summed over problems     */
  double amplitude_updates;   /* sum over step launches of the amplitudes they updated          */
  double step_bytes;          /* algorithmic HBM bytes of all step launches (80 B / amplitude)  */
  double step_kernel_ms;      /* summed HIP-event time of the timed launches of the dominant    */
                              /* kernel (streaming: k_step_rb, k >= 2; persistent: k_interval)  */
  double step_launches;       /* launches of the dominant kernel                                */
  double timed_launches;      /* dominant-kernel launches bracketed by HIP events               */
  double timed_bytes;         /* algorithmic bytes of the timed launches                        */
  double wall_ms;             /* host wall time of the call                                     */
  double h_flops;             /* algorithmic flops of all H applications (4 + 8/drive + 2/pair  */
                              /* per amplitude)                                                 */
  double timed_flops;         /* algorithmic flops of the timed launches                        */
  double timed_amp_terms;     /* amplitudes x Chebyshev terms of the timed launches (SURVEY.md  */
                              /* §8(d) prices a fused Chebyshev term at 80 B per amplitude)     */
  double exchange_bytes;      /* partitioned registers over processes: bytes this rank sent to  */
                              /* other ranks (index swaps / shard exchanges)                     */
  int32_t max_degree;         /* largest Chebyshev degree of any problem / interval             */
  int32_t n_intervals;        /* output intervals propagated                                    */
  int32_t tile_bits;          /* LDS tile of the first problem (log2 amplitudes per workgroup)  */
  int32_t streams;            /* HIP streams ("lanes") the problems were spread over            */
  int32_t mode;               /* 0: per-term streaming kernels, 1: persistent interval kernel, 
                                 2: streaming with the Walsh-Hadamard engine, 3: every problem on
                                 the small-register engine, 4: every problem on the dense
                                 engine (or small and dense), 5: the context's register in
                                 propagator-matrix mode (U = exp(-iH dt) built column-parallel,
                                 outputs by repeated products; option "matrix")                 */
  int32_t outputs_per_launch; /* persistent mode: output times per launch (shared series)   */
  int32_t handoff_fallbacks;  /* 1: this call re-ran on the streaming kernels after a          */
                              /* cross-tile hand-off timed out (device shared with other work)  */
  int32_t dense_problems;     /* problems this call ran on the dense eigen-propagator engine    */
                              /* (option "dense")                           */
  int32_t span_problems;      /* registers this call ran spread over 2^s workgroups (k_span,  */
                              /* option "span"; ABI 9)                                          */
  double dense_ms;            /* host wall time of the dense engine (all of its device work)    */
  double dense_eig_ms;        /* of which the eigendecompositions (rocSOLVER dsyevd)            */
  double exchange_ms;         /* partitioned registers over processes: time of the exchanges    */
                              /* (HIP events around each RCCL call on its stream; host wall     */
                              /* time of each host-transport exchange)                           */
  double lane0_kernel_ms;     /* the timed launches of stream ("lane") 0 alone: summed HIP-event */
  double lane0_launches;      /* time, their count and their amplitudes x terms -- in persistent */
  double lane0_amp_terms;     /* mode lane 0 holds the 2-tile registers (the critical stream)    */
  double matrix_build_ms;     /* propagator-matrix mode (mode 5): HIP-event time of the column   */
  double matrix_products_ms;  /* build of U (k_ucols) and of all products psi_{j+1} = U psi_j    */
  double matrix_products;     /* (k_symv + k_symv_reduce, or zgemv), their count, and the        */
  double matrix_bytes_per_product; /* bytes one product reads (U's stored tiles + x; ABI 10)     */
  int32_t real_problems;      /* registers run as two real recurrences in the rotated frame      */
                              /* (k_real, option "real"; ABI 11)                                 */
  int32_t eig_fallbacks;      /* dense registers whose two-stage eigensolve gave up a bounded     */
                              /* cross-workgroup poll and were re-solved by rocSOLVER dsyevd     */
                              /* (option "eig_spin_limit"; ABI 12)                                */
  int32_t dense_nufft_problems; /* dense registers whose output times came from the non-uniform  */
                              /* FFT instead of the GEMM (option "dense_nufft"; ABI 13)           */
  int32_t reserved13;
  double dense_output_ms;     /* host wall time of the dense engine's output stage (refinement,   */
                              /* transform or GEMM, observables)                                   */
} dse_stats;

/* ---- library / device ------------------------------------------------------------------- */
int dse_abi_version(void);
int dse_device_count(void);                 /* number of HIP devices, 0 if none              */
/* free_total[0] = free, free_total[1] = total device memory in bytes (hipMemGetInfo), so a caller
 * can batch evolutions to fit HBM. */
int dse_device_memory(int device, double* free_total /* [2] */);

/* ---- host-only helpers (no device needed; also used by the tests) ------------------------- */
/* Rigorous spectral bounds of the H defined by the tables (Weyl's inequality over the 1- and
 * 2-qubit pieces; exact for the non-interacting part).  Arrays as in dse_add_problem. */
int dse_spectral_bounds(int n_qubits, const double* field, const double* zz, const double* pair,
                        const double* flip, double shift, double* e_min, double* e_max);
/* Bessel J_k(z), k = 0..kmax (Miller's backward recurrence, normalised by
 * J_0 + 2 sum J_2k = 1).  *degree = the Chebyshev truncation degree for tolerance tol
 * (largest k with |J_k(z)| > tol, at least 1). */
int dse_bessel_j(double z, int kmax, double* out, double tol, int* degree);

/* ---- context ------------------------------------------------------------------------------ */
dse_ctx* dse_create(int device);            /* NULL on failure, see dse_create_error()       */
const char* dse_create_error(void);
void dse_destroy(dse_ctx* ctx);
const char* dse_last_error(const dse_ctx* ctx);
/* Options: "tile_bits"    LDS tile, log2 amplitudes per workgroup, 1..13 (default 13)
 *          "streams"      HIP streams the problems are spread over, 1..16 (default 4)
 *          "persistent"   1 (default): one persistent launch per group of output intervals
 *                         when every problem fits one or two LDS tiles (n <= tile_bits + 1);
 *                         0: per-term streaming launches
 *          "outputs_per_launch"  persistent mode: up to this many (1..2) consecutive output
 *                         times from one Chebyshev series (default 2; 1 on coarse grids,
 *                         alpha dt >= 400)
 *          "wht"          1 (default): streaming registers of more than one tile apply H as
 *                         D_Z + W D_X W + V D_Y V^+ (Walsh-Hadamard passes, two extra state-sized
 *                         vectors per problem, four per shard of a partitioned register; a problem
 *                         whose vectors do not fit in HBM keeps the step kernels); 0: step kernels
 *          "wht_tile_bits"   tile of that engine: 12 (two workgroups per CU), 13, or 0 (default:
 *                         13)
 *          "wht_group_bits"  high qubits transformed per pass of that engine, 2..11, or 0
 *                         (default: tile bits - 2)
 *          "swap_overlap" partitioned registers on that engine: 1 (default) the X- and Y-branch
 *                         vectors take separate passes and each one's index swap runs on a
 *                         second stream under the other's pass; 0: both swapped between passes
 *          "time_kernels" 0 = off, N = bracket the step launches of every N-th interval with
 *                         HIP events (default 1)
 *          "max_degree"   Chebyshev degree cap per interval (default 2e6)
 *          "obs_overlap"  persistent mode: 1 runs each interval group's observables on a second
 *                         stream per lane (lowest priority) while the next group's launches run,
 *                         with two sets of intermediate-output accumulators; 0 (default) in line
 *          "mixed_launch" persistent mode: 1 (default) puts the 1- and 2-tile problems of one tile
 *                         size in one interval launch (stiffest pairs, 1-tile problems, remaining
 *                         pairs) when all 2-tile workgroups fit at once; 0 one stream each
 *          "handoff_fences"  persistent mode, 2-tile registers: 0 (default) the sc1 hand-off
 *                         (write-through payload, per-wave vmcnt(0) + barrier, sc1 flag and
 *                         poll); 1 adds an agent-scope release before every flag store and an
 *                         acquire after every poll
 *          "wht_persist"  Walsh-Hadamard engine: bit 1 runs MID as a persistent launch (one
 *                         workgroup per CU looping over tiles, next tile's loads under the other
 *                         vector's transposes); 0 (default)
 *          "wht_fuse"     Walsh-Hadamard engine, unpartitioned registers: 1 (default) the FINAL pass
 *                         of term k also runs term k + 1's FIRST on the new vector while it is in
 *                         registers (one read of it and one launch less per term; the group-0
 *                         butterflies in another order: results agree to rounding); 0 separate
 *          "wht_mid_inpage"  Walsh-Hadamard plan: the MID group's high bits below the 2-MiB page
 *                         (0 default; measured slower, kept for experiments)
 *          "wht_half"     Walsh-Hadamard engine, 13-bit tiles: passes with one vector in registers
 *                         and the LDS transposes in halves (real, then imaginary parts), two
 *                         workgroups per CU: bit 0 FIRST, bit 1 FWD / INV, bit 2 MID (default 7;
 *                         0 the one-workgroup-per-CU passes); results bitwise identical
 *          "dense"        dense eigen-propagator: 0 off, 1 by cost model (default), 2 always
 *          "eig_streams"  dense engine: eigendecompositions of registers of >= 2^10 amplitudes
 *                         run this many at a time, one stream and rocBLAS handle each, 1..8
 *                         (default 3)
 *          "eig_impl"     dense engine eigensolver: 0 rocSOLVER dsyevd; 1 (default) for
 *                         registers of >= 2^11 amplitudes a tridiagonalisation (the half-matrix
 *                         one of dse_sytrd.hip from 2^13, rocSOLVER's below), rocSOLVER dstedc
 *                         and a blocked back-transformation, dsyevd below 2^11, and from 2^13
 *                         the two-stage solver of dse_eig2.hip (dense -> band 32 -> tridiagonal
 *                         by bulge chasing, dstedc, both back-transformations); 2 the half-matrix
 *                         path from 2^10; 3 the two-stage solver from 2^10.  Costs one extra
 *                         dim x dim matrix per solver stream (two-stage: two, plus ~n^2 / 2 for
 *                         the chase's reflectors)
 *          "matrix"       propagator-matrix mode for a lone register: 0 off, 1 by model
 *                         (default), 2 whenever eligible
 *          "symv_fused"   propagator-matrix mode: 1 sums each product's partials inside the
 *                         product's launch (agent-scope counters); 0 (default) a second launch
 *          "real"         1: registers of 13 / 14 qubits whose drives are all imaginary
 *                         (the sweep's phase pi/2) run in the rotated frame, where H is real: two
 *                         real Chebyshev recurrences, one workgroup each holding the whole
 *                         register in LDS (k_real, dse_real.hip); 2: only the 2-tile (14-qubit)
 *                         registers real, beside the 13-qubit ones on the 1-tile k_interval;
 *                         0 (default): the complex kernels (k_real measured at the 2-tile
 *                         k_interval's CU cost: slower on the bench's mix, 1 and 2 alike)
 *          "spin_limit"   persistent kernels: polls of a partner workgroup's flag before a
 *                         cross-tile hand-off is declared failed (default 2^22 poll rounds, each an s_sleep 1 and
 *                         one flag load, so its wall time is set by that load's latency; the call
 *                         then re-runs on the streaming kernels, stats handoff_fallbacks);
 *                         -1: every hand-off fails at once (tests)
 *          "ablate", "span_ablate", "real_ablate"  diagnostics builds only (-DDSE_DIAG): skip
 *                         kernel sections for timing (results become wrong); DSE_ERR_ARG here
 *          "span_tile"    L > 0 (10 or 11): every register of n > L qubits runs over 2^(n - L)
 *                         cooperating workgroups, one per CU, with per-term cross-tile hand-offs
 *                         (k_span, dse_span.hip): a shorter chain per register for few registers
 *                         (one simulate_rare call, one GPU's share of a strong split); -1
 *                         (default): when every Chebyshev register of the evolve is 12..15 qubits,
 *                         L = 10 if all their tiles fit one per CU, else L = 11 if they fit the
 *                         chip at once; else the partial form (option span_partial); else L = 11
 *                         in two resident launches per interval; else none; 0 never
 *          "span_partial" 1 (default): the auto policy's partial form -- when not every register
 *                         fits spanned in one launch, the registers with the longest predicted
 *                         chains (spectral half-width x measured term time) span over
 *                         2^span_partial_tile-amplitude tiles on a stream of their own beside
 *                         k_interval, as long as every workgroup of both launches fits the chip
 *                         and the longest chain shrinks by 10% (one GPU's share of a 2- or 4-GPU
 *                         strong split); 0 off
 *          "span_chunks"  resident launches per interval the auto policy allows for every
 *                         register spanned (0, 1, 2; default 2)
 *          "span_partial_tile"  log2 tile of the partial form (10 or 11, default 11)
 *          "span"         the same with a fixed number s = 1..4 of top bits per register
 *          "span_rb"      k_span's rows per thread 2^span_rb (0: 512 threads per workgroup)
 *          "span_outputs" outputs per launch (1..4, default 4) of an evolve whose registers all
 *                         span: k_span staggers the outputs' sums over the terms, so more
 *                         outputs per Chebyshev series cost no extra registers
 *          "eig_spin_limit"  two-stage eigensolver: rounds a poll of another workgroup's result
 *                         waits before it gives up (default 2^22 poll rounds, each one buffer load of the
 *                         polled value; counted in rounds, not time, as spin_limit); a give-up voids that
 *                         solve and the register is re-solved by rocSOLVER dsyevd (stats
 *                         eig_fallbacks); -1: every solve gives up at once (tests)
 *          "dense_nufft"  dense engine: output times of registers of >= 2^10 amplitudes on a
 *                         uniform grid (np.linspace: tau_j = j s + delta_j, |delta_j| an ulp) by a
 *                         type-1 non-uniform FFT of the eigenvalue phases (spreading, rocFFT,
 *                         deconvolution; ~1e11 flops per 2^14 register) instead of the
 *                         [cos | -sin] GEMM (4 dim^2 T flops): 1 (default) from 2048 outputs, 2
 *                         every register from two outputs (tests), 0 never (stats
 *                         dense_nufft_problems; ABI 13)
 *          "dense_refine" dense engine: 1 (default) eigenvalues refined by double-double
 *                         Rayleigh quotients (exact diagonal) and output phases reduced modulo
 *                         2 pi in double-double; 0 the eigensolver's values and fp64 phases */
int dse_set_option(dse_ctx* ctx, const char* key, double value);

/* ---- problems ----------------------------------------------------------------------------- */
/* Adds an evolution to the context.  field[n], zz[n*n] and pair[n*n] (row-major, upper
 * triangle i<j read), flip[4n].  Returns the problem id (>= 0) or a negative status. */
int dse_add_problem(dse_ctx* ctx, int n_qubits, const double* field, const double* zz,
                    const double* pair, const double* flip, double shift, uint64_t psi0_index,
                    uint64_t sea_mask, int rare_bit, double rare_z_const);
int dse_num_problems(const dse_ctx* ctx);
int dse_clear(dse_ctx* ctx);

/* ---- partitioned registers (SURVEY.md §8(e), configs with N >= 28) ----------------------------
 * A register whose top shard_bits (1..3) qubits are "global": shard r holds the 2^(n-shard_bits)
 * amplitudes whose global bits equal r.  Same tables as dse_add_problem.
 *   shard_rank = -1  all 2^shard_bits shards in this context (one device); terms that cross
 *                    shards read the partner shard's buffers directly.  Returns the id of shard 0;
 *                    the other shards take the next ids.  Every shard's row of obs_out holds the
 *                    observables of the whole register; dse_apply_h / dse_observables /
 *                    dse_get_state on shard 0 take and return the whole 2^n state.
 *   shard_rank >= 0  this context holds shard shard_rank of a register partitioned over
 *                    processes (one per GPU, rank = shard_rank, world = 2^shard_bits) joined by
 *                    dse_dist_init; before every Chebyshev term the shards that terms couple
 *                    exchange their current vector with RCCL send/recv, and the observable sums
 *                    are all-reduced.  dse_get_state returns the local shard (2^(n-shard_bits)).
 * No reference counterpart: replaces QuTiP's single-process CSR product at sizes it cannot hold. */
int dse_add_problem_sharded(dse_ctx* ctx, int n_qubits, const double* field, const double* zz,
                            const double* pair, const double* flip, double shift,
                            uint64_t psi0_index, uint64_t sea_mask, int rare_bit,
                            double rare_z_const, int shard_bits, int shard_rank);
/* RCCL bootstrap: rank 0 creates the id (DSE_DIST_ID_BYTES bytes), every rank passes it to
 * dse_dist_init with its rank and the world size (out-of-band broadcast, e.g. torch.distributed). */
#define DSE_DIST_ID_BYTES 128
int dse_dist_unique_id(unsigned char* id_out);
int dse_dist_init(dse_ctx* ctx, int rank, int world, const unsigned char* id);
/* The same with a host transport instead of RCCL (tests, or a deployment without RCCL between
 * the devices): every exchange is handed to fn on the calling host thread with HOST buffers (the
 * library stages device data through them; fn must not call back into libdse):
 *   DSE_XCHG_ALLTOALL      send/recv hold world chunks of `bytes` each, chunk p goes to rank p
 *   DSE_XCHG_SENDRECV      send `bytes` to rank `peer` and receive `bytes` from it into recv
 *   DSE_XCHG_ALLREDUCE_F64 sum bytes / 8 doubles in place over all ranks (send == recv)
 * Every rank issues the same sequence of calls.  fn returns 0 on success. */
enum dse_exchange_op { DSE_XCHG_ALLTOALL = 1, DSE_XCHG_SENDRECV = 2, DSE_XCHG_ALLREDUCE_F64 = 3 };
typedef int (*dse_exchange_fn)(void* user, int op, void* send, void* recv, uint64_t bytes, int peer);
int dse_dist_init_exchange(dse_ctx* ctx, int rank, int world, dse_exchange_fn fn, void* user);
/* Local state size (amplitudes) of a problem: 2^n, or 2^(n - shard_bits) for a dist shard. */
int64_t dse_problem_dim(const dse_ctx* ctx, int problem);

/* Diagnostics (host only, no device): the Walsh-Hadamard engine's pass plan for a register of
 * n_local local qubits (shard_bits of them global), tile_bits 12 or 13, max_bits high qubits per
 * pass (0: tile_bits - 2).  Writes groups_out[g][0] = carried low bits c, [g][1 + q] = the local
 * qubit of tile bit q (q < tile_bits), for g < G; returns G (group 0 = FIRST/FINAL, 1..G-2 =
 * FWD/INV, G-1 = MID), or 0 when the engine cannot take the register. */
int dse_wht_plan(int n_local, int shard_bits, int tile_bits, int max_bits, int32_t* groups_out /* [4][14] */);

/* ---- hot path ----------------------------------------------------------------------------- */
/* psi_out = H psi_in for one problem (interleaved complex, 2^n each).  Test/diagnostic hook:
 * runs the same matrix-free tile kernel as the propagator. */
int dse_apply_h(dse_ctx* ctx, int problem, const double* psi_in, double* psi_out);
/* The 7 observables of an arbitrary state of one problem (same kernel as dse_evolve). */
int dse_observables(dse_ctx* ctx, int problem, const double* psi, double* obs7);
/* Evolves every problem from its basis state psi0 at t[0] through the output times t[0..n_t)
 * (strictly increasing) with an exact Chebyshev propagator (truncation tolerance tol, e.g.
 * 1e-14) and writes obs_out[problem][DSE_N_OBS][n_t].  stats may be NULL. */
int dse_evolve(dse_ctx* ctx, const double* t, int n_t, double tol, double* obs_out,
               dse_stats* stats);
/* Final state of one problem after dse_evolve (2^n interleaved complex). */
int dse_get_state(dse_ctx* ctx, int problem, double* psi_out);
/* Energy of the final state after dse_evolve, on the device: e_out[0] = <psi|H|psi> / <psi|psi>,
 * e_out[1] = <psi|psi> (a partitioned loopback register: shard 0's id, whole register).  Unitary
 * evolution conserves both exactly, so they check a run whose state is too large to compare
 * (the reference has no counterpart; its only diagnostic is state_norm, :669).  Not available
 * for a dist shard (DSE_ERR_ARG). */
int dse_energy(dse_ctx* ctx, int problem, double* e_out /* [2] */);
/* Times the Chebyshev step kernel alone: reps launches over all problems, HIP events around
 * each launch.  Returns the mean launch duration and the algorithmic bytes per launch. */
int dse_time_step_kernel(dse_ctx* ctx, int reps, double* ms_per_launch, double* bytes_per_launch);

#ifdef __cplusplus
}
#endif
#endif /* DSE_H */
