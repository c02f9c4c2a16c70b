/*
 * gymnast_acrobot.h -- C-ABI of the MI355X (gfx950) batched acrobot Newton/Armijo engine.
 *
 * Drop-in boundary for the reference's hot path (francescoolivieri/Gymnast_OptimalControl):
 * the Python module surface of dynamics.py / trajectory_generation.py is re-implemented by
 * gymnast_optimalcontrol_amd/{dynamics,trajectory_generation}.py on top of these entry points
 * (ctypes).  Every entry point cites the reference function it replaces.
 *
 * Conventions
 *   - All pointers are DEVICE pointers (hipMalloc / torch CUDA tensors) unless marked [host].
 *   - `stream` is a hipStream_t passed as void* (0 = null stream).  Work is stream-ordered;
 *     no entry point synchronises the device (gym_timing_collect only reads events the
 *     caller has already synchronised).
 *   - Return value: 0 on success, otherwise a hipError_t code (launch / argument errors:
 *     GYM_EINVAL).  Per-lane numerical outcomes are reported in status arrays, never as errors.
 *   - Callers own every buffer; kernels never allocate.
 *   - fp64 (IEEE binary64) throughout.
 *
 * Layouts
 *   lane-major  : the reference's own arrays stacked over lanes: x (B,N,4), u (B,T,2),
 *                 K (B,T,2,4), sigma (B,T,2), row-major.
 *   SoA         : time-major, lane innermost (lane stride Bp >= B, a multiple of 64):
 *     pairs  (W = 2): two fp64 components per 16-byte element, one 1 KiB load per wavefront and row,
 *                   WAVE-BLOCKED: a P-row stream is (L, Bp/64, P, 64) double2, i.e. the P rows of one
 *                   64-lane group at one stage are one contiguous P KiB block (ABI 4; element of
 *                   (t, row p, lane l) = t*P*Bp + (l & ~63)*P + 64 p + (l & 63))
 *                   states   x  : (N, Bp/64, 2, 64) double2   (th1, th2), (w1, w2)
 *                   gains    K1 : (T, Bp/64, 2, 64) double2   row 1 of K_t (row 0 is identically 0)
 *                   gains    Kf : (T, Bp/64, 4, 64) double2   full K_t: (K00,K01)(K02,K03)(K10,K11)(K12,K13)
 *     planes (W = 1): one component per element, (L, P, Bp)
 *                   controls u  : (T, 2, Bp) double    planes tau1, tau2
 *                   sigma    s  : (T, 2, Bp) double
 *                   offsets  cs : (T, 2, Bp) double    planes cg = (u1 - K1 x) + gamma0 sigma1 (written by every
 *                                                      solver sweep) and sigma1 (written only by the sigma1
 *                                                      re-runs: backtracking lanes, gym_newton_sigma, gamma sweeps)
 */
#ifndef GYMNAST_ACROBOT_H
#define GYMNAST_ACROBOT_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define GYM_ABI_VERSION 17
#define GYM_MAX_BP (1LL << 26) /* lane stride limit: stream offsets are 32-bit inside one stage      */

/* gym_batch.flags */
#define GYM_FLAG_U0_ZERO 1  /* u_ref[:,0] == 0: the unactuated tau1 channel stays exactly zero (u0 starts
                             * at 0 and sigma0 = -(u0 - ur0) = -0, dynamics.py:205 ignores it), so the
                             * solver neither reads nor writes its planes; both u buffers are zeroed by
                             * gym_newton_init. Results are bit-identical to the general path.          */
#define GYM_FLAG_X_CKPT 2   /* state checkpointing: the Armijo trials store x only at the checkpoint knots
                             * t % GYM_CKPT_INTERVAL == 0 and t == N-1; the backward sweep re-integrates the
                             * knots between two checkpoints (RK4 from the checkpoint with the stored controls,
                             * the trial's own arithmetic, so bit-identical) instead of reading them: 48 B per
                             * stage less HBM traffic, for 0.75 extra RK4 steps per sweep stage (opt-in: on
                             * MI355X the solver kernels are VALU- as much as HBM-bound and it measured 13%
                             * slower).  The other knots of x[] are stale until gym_newton_fill_states
                             * rebuilds them (gym_newton_finalize does so itself).                          */
#define GYM_FLAG_RUN_SINGLE 4 /* gym_newton_run: the single-wavefront persistent kernel instead of the default
                               * two-wavefront one (helper wavefront per 64 lanes; same bits) */
#define GYM_FLAG_REF_LANE 8  /* per-lane references: gym_batch.x_ref is (Bp, N, 4) and u_ref (Bp, T, 2), lane-major
                              * (lane l follows rows l; padding lanes any valid rows).  Every schedule
                              * (gym_newton_init / _iteration / _phase / _run / _sigma / _finalize) and
                              * gym_newton_gamma_sweep; X_CKPT with it: GYM_EINVAL.  Same per-lane
                              * arithmetic as a shared reference (vector instead of scalar loads: the same bits). */
#define GYM_FLAG_SIGMA_STREAM 16 /* gym_newton_iteration: the backward sweep also stores sigma1 (the cs plane 1),
                                  * so the lanes that reject Armijo trial 1 skip the sigma1 re-run; the same values.
                                  * gym_newton_run (four-wavefront kernel): one iteration per launch (k1 = k0 + 1,
                                  * else GYM_EINVAL), its sweep storing sigma1, the lanes that reject trial 1 put on
                                  * the retry list and finished by the serial schedule's parallel candidates and
                                  * accepted re-run in the same call.  The solver sets it in its low-occupancy
                                  * regime; ignored by the pipelined phases. */
#define GYM_CKPT_INTERVAL 4
#define GYM_EINVAL 1  /* == hipErrorInvalidValue */

/* Lane status codes (per-lane outcome of newton_Algorithm, trajectory_generation.py:329-396). */
enum {
    GYM_ACTIVE = 0,     /* still iterating                                              */
    GYM_CONVERGED = 1,  /* max|sigma| < tol after an accepted step            (:394-396) */
    GYM_LS_FAILED = 2,  /* Armijo exhausted max_ls trials, no update          (:367-369) */
    GYM_MAX_ITERS = 3,  /* loop ran out of iterations                          (:329)    */
    GYM_PAD = 4         /* padding lane (lane >= B)                                     */
};

/* Acrobot model, reduced to the coefficients the dynamics use (dynamics.py:63-90):
 *   M11 = a + 2 b cos(th2), M12 = d + b cos(th2), M22 = d,
 *   C   = b sin(th2) [[-w2, -(w1+w2)], [w1, 0]],   G = [g1 sin th1 + g2 sin(th1+th2), g2 sin(th1+th2)],
 *   F   = diag(f1, f2);  tau = [0, u1] (dynamics.py:153, :205);  dt = RK4 / Euler step. */
typedef struct gym_model {
    double a, b, d, g1, g2, f1, f2, dt;
} gym_model;

/* Diagonal cost weights (trajectory_generation.py:16-18): stage Q, R; terminal Q_T. */
typedef struct gym_weights {
    double Q[4], R[2], QT[4];
} gym_weights;

/* Armijo / stopping parameters (newton_Algorithm kwargs, trajectory_generation.py:298, :345). */
typedef struct gym_armijo {
    double tol, beta, c, gamma0;
    int32_t max_ls;     /* 20 in the reference (:345) */
    int32_t record_history;
} gym_armijo;

/* Optional per-kernel timing of gym_newton_iteration / gym_newton_phase with HIP events on the solver's
 * stream.  Kernel kinds: 0 backward sweep, 1 Armijo trial 1, 2 candidate trials, 3 accepted-candidate
 * rollout, 4 statistics, 5 / 6 fused pipeline phase (odd / even p), 7 sigma1 re-run of the lanes that
 * backtrack, 8 persistent run (gym_newton_run), 9 straggler tail (gym_newton_tail).  Every launch of kinds
 * 0, 1, 5, 6, 8, 9 is timed while the pool has room (gym_timing_collect empties it; the solvers collect at every
 * host synchronisation); beyond that, and always for kinds 2, 3, 4, 7 (the short post-trial launches), a launch
 * is timed only if the previous sampled pair of its kind was collected. */
#define GYM_NK 10
#define GYM_TIMING_POOL 512  /* event pairs for EVERY launch between two collects (then one sampled pair per kind) */
typedef struct gym_timing {
    void* ev[2 * GYM_NK];    /* hipEvent_t start/stop pairs (gym_timing_create)          */
    double ms[GYM_NK];       /* accumulated device time per kernel kind                   */
    int64_t launches[GYM_NK];/* collected launches per kernel kind                        */
    int32_t pending;         /* bitmask: pairs recorded but not yet collected            */
    int32_t pool_used;       /* pool pairs recorded since the last collect               */
    void* pool_ev[2 * GYM_TIMING_POOL];  /* hipEvent_t pairs: every timed launch while the pool has room */
    int32_t pool_kind[GYM_TIMING_POOL];  /* the kernel kind of each pool pair                          */
} gym_timing;

/* Device state of a batched solve (all device pointers, sizes in lanes / knots). */
typedef struct gym_batch {
    int64_t B, Bp;      /* lanes, lane stride (multiple of 64)                     */
    int32_t N, hist_len;/* knots (T = N-1); rows of the optional history buffers   */
    int32_t flags, pad; /* GYM_FLAG_*                                               */
    double* x[2];       /* (N, Bp/64, 2, 64) double2 state trajectories, wave-blocked pairs, double-buffered */
    double* u[2];       /* (T, 2, Bp) control planes tau1, tau2, double-buffered  */
    double* K1;         /* (T, Bp/64, 2, 64) double2 feedback gains, row 1, wave-blocked pairs */
    double* cs;         /* (T, 2, Bp) planes: cg = (u1 - K1 x) + gamma0 sigma1, sigma1 (re-runs only) */
    const double* x_ref;/* (N,4) shared reference states; (Bp,N,4) with GYM_FLAG_REF_LANE */
    const double* u_ref;/* (T,2) shared reference controls (already trimmed); (Bp,T,2) per lane */
    double* cost;       /* (Bp) current J_k                                       */
    double* dJ;         /* (Bp) expected reduction sum g^T sigma                  */
    double* smax;       /* (Bp) max|sigma| of the last backward sweep             */
    double* gamma;      /* (Bp) last accepted step size                           */
    int32_t* status;    /* (Bp) GYM_* codes                                       */
    int32_t* n_iter;    /* (Bp) outer iterations executed (incl. a final failed)  */
    int32_t* res_buf;   /* (Bp) which x/u buffer holds a finished lane's result   */
    int32_t* n_roll;    /* (Bp) closed-loop rollouts evaluated                     */
    int32_t* retry_list;/* (Bp) lanes that need Armijo trials 2..max_ls           */
    int32_t* counters;  /* (4)  retry counts: [0] serial schedule / half H0, [1] half H1 */
    uint8_t* cand_ok;   /* (max_ls, Bp) Armijo acceptance of candidate j           */
    double* partials;   /* (256*8) per-block statistics                           */
    double* stats;      /* (24) [0,8) totals (see gym_newton_iteration), [8,16) H0, [16,24) H1 */
    double* hist_cost;  /* optional (hist_len, Bp): J after iteration k            */
    double* hist_smax;  /* optional (hist_len, Bp): max|sigma| of iteration k      */
    const int64_t* lane_map; /* optional (B): lane i's results go to row lane_map[i] of the lane-major outputs
                         * of gym_newton_finalize / gym_newton_sigma (a permutation; NULL: identity)  */
    gym_timing* timing; /* [host] optional kernel timing (NULL: none)               */
    /* optional (ABI 13) candidate scratch of the post-trial Armijo search.  Used by every post-trial launch when
     * cand_slots > 0 and neither GYM_FLAG_X_CKPT nor GYM_FLAG_RUN_SINGLE is set: gym_newton_iteration and
     * gym_newton_phase always, gym_newton_run when GYM_FLAG_SIGMA_STREAM sends its retries to the post-trial search
     * (a caller must not hand over a buffer it expects untouched on those paths).  Candidate i = r (max_ls - 1) + j - 1 (retry-list entry r, step gamma0 beta^j) stores
     * its trajectory, controls and cost in slot i while i < cand_slots, and the accepted one is then copied into
     * the lane's next iterate instead of re-running its rollout (a chain of T RK4 steps); candidates without a
     * slot are re-run as before.  cand_scratch: gym_newton_cand_scratch(N, cand_slots) doubles, laid out as
     * x (N, V/64, 2, 64) double2 | u (T, 2, V) planes | J (V), V = cand_slots (a multiple of 64).
     * cand_slots = 0 (or NULL): every accepted candidate is re-run.  With GYM_FLAG_X_CKPT or GYM_FLAG_RUN_SINGLE
     * the candidates keep the single-lane re-run path and the buffer is not touched.  Bits are the same either way;
     * the caller may install it between launches (the Python solver does so on demand). */
    double* cand_scratch;
    int64_t cand_slots;
} gym_batch;

int gym_abi_version(void);
/* Build id: 16 hex digits of the sha256 over the kernel sources and this header the library was compiled from
 * (gymnast_optimalcontrol_amd/_build.py source_hash).  The Python binding refuses a library whose id differs
 * from its tree's sources (a stale binary), and the build rebuilds on a mismatch instead of trusting mtimes. */
const char* gym_build_id(void);

/* [host] Reduce a reference parameter set {m1,m2,l1,lc1,l2,lc2,I1,I2,g,f1,f2} (dynamics.py:15-61). */
int gym_model_from_params(const double params[11], double dt, gym_model* out);

/* ---------------- per-point primitives (lane-major x (n,4), u (n,2)) ---------------- */
/* dynamics.py:197-213 continuous_dynamics -> xdot (n,4) */
int gym_continuous_dynamics(const gym_model* m, const double* x, const double* u, double* xdot, int64_t n, void* stream);
/* dynamics.py:177-195 dynamics (RK4 step) -> xnext (n,4) */
int gym_rk4_step(const gym_model* m, const double* x, const double* u, double* xnext, int64_t n, void* stream);
/* dynamics.py:217-226 Calculate_A_B_matrixes -> A_c (n,4,4), B_c (n,4,2) */
int gym_jacobians(const gym_model* m, const double* x, const double* u, double* A_c, double* B_c, int64_t n, void* stream);
/* trajectory_generation.py:89-114 derivatives_Cost (general Q (4,4), R (2,2) or Q_T) [host matrices]:
 * terminal == 0: l (n), gx (n,4), gu (n,2);  terminal != 0: l (n), gx (n,4) with Q_T, gu unused. */
int gym_stage_cost_derivs(const double* x, const double* xr, const double* u, const double* ur, const double Q[16],
                          const double R[4], int32_t terminal, double* l, double* gx, double* gu, int64_t n, void* stream);

/* ---------------- layout transposes ---------------- */
/* lane-major (B,L,C) -> SoA (L, C/W, Bp, W), W = 2 (pairs, wave-blocked) or 1 (planes).  Padding lanes are
 * zero-filled.  Here and below "(L,P,Bp) pairs" names the wave-blocked pair layout of the Layouts note. */
int gym_pack_lanes(const double* src, double* dst, int64_t B, int64_t Bp, int32_t L, int32_t C, int32_t W,
                   void* stream);
/* SoA -> lane-major; if sel != NULL lane b reads from (sel[b] ? src1 : src0).  Tiled through LDS (64 lanes x a few
 * knots per workgroup: coalesced reads and writes); C <= 63 components per knot (GYM_EINVAL otherwise). */
int gym_unpack_lanes(const double* src0, const double* src1, const int32_t* sel, double* dst, int64_t B, int64_t Bp,
                     int32_t L, int32_t C, int32_t W, void* stream);
/* compact gains K1 (T,2,Bp) -> full lane-major K (B,T,2,4) with row 0 = 0 */
int gym_unpack_gains(const double* K1, double* K, int64_t B, int64_t Bp, int32_t T, void* stream);

/* ---------------- trajectory kernels (SoA) ---------------- */
/* trajectory_generation.py:74-87 simulate_open_loop: x0 (B,4) lane-major, u (T,2,Bp) planes -> x (N,2,Bp);
 * if cost != NULL also total_cost (:231-252) of (x,u) with diagonal weights. */
int gym_rollout_open_loop(const gym_model* m, const gym_weights* w, const double* x0, const double* u,
                          const double* x_ref, const double* u_ref, double* x, double* cost, int64_t B, int64_t Bp,
                          int32_t N, void* stream);
/* trajectory_generation.py:218-229 forward_closed_loop_update with FULL gains Kf (T,4,Bp) and per-lane gamma (Bp);
 * u, sigma, u_new planes (T,2,Bp); writes x_new (N,2,Bp), u_new; cost (Bp) of the new trajectory if non-NULL. */
int gym_closed_loop(const gym_model* m, const gym_weights* w, const double* x, const double* u, const double* Kf,
                    const double* sigma, const double* gamma, const double* x_ref, const double* u_ref,
                    double* x_new, double* u_new, double* cost, int64_t B, int64_t Bp, int32_t N, void* stream);
/* trajectory_generation.py:231-252 total_cost with general Q, R, Q_T [host matrices]. */
int gym_total_cost(const double* x, const double* u, const double* x_ref, const double* u_ref, const double Q[16],
                   const double R[4], const double QT[16], double* cost, int64_t B, int64_t Bp, int32_t N, void* stream);
/* Fused backward sweep = compute_costate_trajectory (:138-159) + build_stage_lists (:166-181) +
 * calculate_K_and_sigma (:183-216) for the Gauss-Newton blocks (2Q, 2R, S = 0, terminal 2Q_T):
 * K1 (T,2,Bp), sigma planes (T,2,Bp), dJ (Bp), smax = max|sigma| (Bp); lambda (N,2,Bp) costates if non-NULL. */
int gym_backward_sweep(const gym_model* m, const gym_weights* w, const double* x, const double* u,
                       const double* x_ref, const double* u_ref, double* K1, double* sigma, double* dJ, double* smax,
                       double* lambda, int64_t B, int64_t Bp, int32_t N, void* stream);
/* build_stage_lists (:166-181): A_d (T,16,Bp), B_d (T,8,Bp), q (T,4,Bp), r (T,2,Bp), qT (4,Bp); plain doubles. */
int gym_linearize(const gym_model* m, const gym_weights* w, const double* x, const double* u, const double* x_ref,
                  const double* u_ref, double* A_d, double* B_d, double* q, double* r, double* qT, int64_t B,
                  int64_t Bp, int32_t N, void* stream);
/* calculate_K_and_sigma (:183-216) on general dense stage data, plain-double SoA:
 * A (T,16,Bp) B (T,8,Bp) Q (T,16,Bp) R (T,4,Bp) S (T,8,Bp) q (T,4,Bp) r (T,2,Bp) QT (16,Bp) qT (4,Bp)
 * -> K (T,8,Bp), sigma (T,2,Bp), dJ (Bp).  2x2 solves by LU with partial pivoting (LAPACK dgesv order). */
int gym_riccati_general(const double* A, const double* Bm, const double* Q, const double* R, const double* S,
                        const double* q, const double* r, const double* QT, const double* qT, double* K, double* sigma,
                        double* dJ, int64_t B, int64_t Bp, int32_t T, void* stream);

/* ---------------- batched Newton / Armijo solver (newton_Algorithm, :298-398) ---------------- */
/* Open-loop init (u = 0, :311-312), J_0 (:319), status/counters reset.  x0 (B,4) lane-major. */
int gym_newton_init(const gym_model* m, const gym_weights* w, const double* x0, const gym_batch* bt, void* stream);
/* One outer iteration k for every ACTIVE lane: backward sweep (K1, cs), Armijo trial 1 (gamma0) fused with its cost,
 * parallel candidate rollouts gamma0*beta^j (j = 1..max_ls-1) for lanes that rejected trial 1, accepted-
 * candidate rollout, lane status update, then device statistics into bt->stats:
 *   [0] lanes still active  [1] sum J over lanes  [2] sum max|sigma|^2 over lanes that ran
 *   [3] lanes that ran (lane-iterations)  [4] lanes that needed trials >= 2  [5] converged  [6] failed
 *   [7] rollouts evaluated in total.
 * Buffer roles: x/u[k&1] = current, x/u[(k+1)&1] = candidate.  Stream-ordered, no host sync. */
int gym_newton_iteration(const gym_model* m, const gym_weights* w, const gym_armijo* a, const gym_batch* bt,
                         int32_t k, void* stream);
/* Pipelined schedule: lanes split into halves H0 = [0, Bh), H1 = [Bh, B) (gym_newton_pipeline_split) whose
 * iterations are offset by one phase.  Phase p runs ONE fused launch: the backward sweep of H0 (p even,
 * iteration p/2) or H1 (p odd, iteration (p-1)/2) -- skipped if do_backward == 0, i.e. past max_iters --
 * beside the Armijo trial of the other half (H0 for odd p, iteration (p-1)/2; H1 for even p >= 2,
 * iteration (p-2)/2); then that half's candidate trials, retries and statistics.  After phase 2k+2 both
 * halves have completed iteration k and stats[0,8) holds the totals.  Call p = 0 once after init; every
 * lane follows exactly the serial schedule's arithmetic. */
int gym_newton_pipeline_split(const gym_batch* bt, int64_t* Bh);
int gym_newton_phase(const gym_model* m, const gym_weights* w, const gym_armijo* a, const gym_batch* bt, int32_t p,
                     int32_t do_backward, void* stream);
/* Which build of the phase kernel gym_newton_phase launches for this batch's full phases on the current device:
 * *low_out = 1 for the two-wavefront build (more than 7/8 and at most two wavefronts per SIMD, no X_CKPT: compiled
 * for two wavefronts, its stage loops prefetching two stages ahead), 0 for the four-wavefront build.  Both give the
 * same bits; this reports the choice (tests, the bench line).  ABI 17. */
int gym_newton_phase_kind(const gym_batch* bt, int32_t* low_out);
/* Persistent schedule: ONE launch in which every lane still ACTIVE runs its own outer iterations k0 .. k1-1 back to
 * back (newton_Algorithm :329-396 per lane: sweep, Armijo trial 1, and for a lane that rejects it the sigma1 re-run
 * and trials 2..max_ls in sequence), stopping at convergence or LS failure; then the statistics of iteration k1-1
 * into stats[0,8) ([4] = 0: no retry list is kept).  Lanes need no grid-wide step between iterations, so there is
 * none.  Same per-lane arithmetic as gym_newton_iteration / gym_newton_phase (bit-identical results).  k0 = the
 * iterations every active lane has done (0 after gym_newton_init).  Not with GYM_FLAG_X_CKPT (GYM_EINVAL). */
int gym_newton_run(const gym_model* m, const gym_weights* w, const gym_armijo* a, const gym_batch* bt, int32_t k0,
                   int32_t k1, void* stream);
/* Straggler tail: the n_lanes lanes of lanes[] (device, each ACTIVE with k0 iterations done) run their own outer
 * iterations k0 .. k1-1 back to back, ONE workgroup per lane: the sweep stores K row 1, cg and sigma1 in one pass
 * (the 64 threads linearise 64 stages at a time), then Armijo trials 1..max_ls are evaluated AT ONCE (thread c:
 * gamma_0 beta^c, into scratch slot c) and the first accepted one becomes the next iterate -- the sequential
 * search's decision and the serial schedule's bits (newton_Algorithm :329-396 per lane).  Then the statistics of
 * iteration k1-1 into stats[0,8) over the whole batch.  scratch: device doubles, at least
 * gym_newton_tail_scratch(N, n_lanes, max_ls); max_ls <= 64; not with GYM_FLAG_X_CKPT (GYM_EINVAL).
 * Replaces, for the last few lanes of a solve, the per-iteration launches of newton_Algorithm's loop (:329). */
int gym_newton_tail(const gym_model* m, const gym_weights* w, const gym_armijo* a, const gym_batch* bt,
                    const int32_t* lanes, int32_t n_lanes, double* scratch, int64_t scratch_doubles, int32_t k0,
                    int32_t k1, void* stream);
/* [host] Scratch doubles gym_newton_tail needs for n_lanes lanes (candidate trajectories of every trial). */
int gym_newton_tail_scratch(int32_t N, int32_t n_lanes, int32_t max_ls, int64_t* doubles_out);
/* [host] Doubles of gym_batch.cand_scratch for `slots` candidate slots (a multiple of 64, >= 0) at horizon N. */
int gym_newton_cand_scratch(int32_t N, int64_t slots, int64_t* doubles_out);
/* LDS per workgroup the tail kernel needs at horizon N (*bytes_out; ~72 KiB at N = 501), and, if limit_out is not
 * NULL, the current device's opt-in limit (hipDeviceAttributeSharedMemPerBlockOptin; a HIP error code if the
 * device cannot be queried).  A caller turns the tail off up front when bytes > limit (solver.py tail_ok). */
int gym_newton_tail_lds(int32_t N, int64_t* bytes_out, int64_t* limit_out);
/* After k_done iterations: ACTIVE lanes -> GYM_MAX_ITERS; gather each lane's result buffer into lane-major
 * x_out (B,N,4), u_out (B,T,2), K_out (B,T,2,4) and sigma_out (B,T,2) of the lane's last iteration
 * (sigma0 recomputed from that iteration's u0).  Any output may be NULL.  With GYM_FLAG_X_CKPT the result
 * buffers' states are first rebuilt from their checkpoints (gym_newton_fill_states, buf = -1). */
int gym_newton_finalize(const gym_model* m, const gym_weights* w, const gym_batch* bt, int32_t k_done, double* x_out,
                        double* u_out, double* K_out, double* sigma_out, void* stream);
/* GYM_FLAG_X_CKPT: rebuild every knot of the state buffer x[buf] (buf = 0 / 1; -1 = each lane's result buffer
 * res_buf) from its checkpoints and the controls u[buf]: x_{t+1} = RK4(x_t, u_t) from each checkpoint, the
 * trial's arithmetic bit for bit.  Lanes [0, B); a no-op without the flag. */
int gym_newton_fill_states(const gym_model* m, const gym_batch* bt, int32_t buf, void* stream);
/* Placement probe: the pipelined phase kernel's stream traffic (gym_newton_phase's bytes per launch: the sweep's
 * pattern on lanes [0, Bp/2), the trial's on [Bp/2, Bp), buffers cb / cb ^ 1) with no arithmetic, for timing where
 * the driver placed the six stream buffers (the phase kernel's speed depends on it).  Overwrites x, u, K1
 * and cs with garbage: call before gym_newton_init.  Bp a multiple of 128. */
int gym_placement_probe(const gym_batch* bt, int32_t cb, void* stream);
/* sigma (B,T,2) of each lane's last completed iteration (n_iter - 1): sigma1 by re-running that iteration's
 * sweep (the solver does not stream sigma1; the re-run reproduces it bit for bit), sigma0 recomputed. */
int gym_newton_sigma(const gym_model* m, const gym_weights* w, const gym_batch* bt, double* sigma_out, void* stream);

/* ---------------- Armijo gamma sweeps (plot_armijo_line_search, trajectory_generation.py:254-296) ---------------- */
/* J(gamma_g) = total_cost (:231-252) of forward_closed_loop_update(x, u, K, sigma, gamma_g) (:218-229) for G step
 * sizes per lane -- the reference's 200-point line-search curve (:258-264) -- cost only, one thread per
 * (lane, step).  x (N,2,Bp) pairs, u and sigma (T,2,Bp) planes, Kf (T,4,Bp) full gains, gammas (G); cost_out
 * (G,Bp), NaN for padding lanes. */
int gym_gamma_sweep(const gym_model* m, const gym_weights* w, const double* x, const double* u, const double* Kf,
                    const double* sigma, const double* gammas, int32_t G, const double* x_ref, const double* u_ref,
                    double* cost_out, int64_t B, int64_t Bp, int32_t N, void* stream);
/* The same curve for every lane of a batched solve at the iterate iteration k starts from (k = iterations done;
 * either schedule): runs iteration k's backward sweep (K1, cg, dJ, smax -- exactly what iteration k computes, so
 * the solve is unaffected) and then the Armijo trial's own rollout for each gamma_g: at the trial's step sizes
 * gamma0 beta^i the costs equal the trial costs bit for bit.  cost_out (G,Bp); NaN for lanes not ACTIVE. */
int gym_newton_gamma_sweep(const gym_model* m, const gym_weights* w, const gym_armijo* a, const gym_batch* bt,
                           int32_t k, const double* gammas, int32_t G, double* cost_out, void* stream);

/* ---------------- LQR / receding-horizon MPC trackers (trajectory_tracking.py) ---------------- */
/* Time-varying LQR gains over windows of a stage array.  Stages: A (S,4,4), B (S,4,2) [device], continuous
 * Jacobians if discretize != 0 (A_d = I + dt A, B_d = dt B, trajectory_generation.py:161-164), stage index >= S
 * reads the pad stage A_pad (4,4), B_pad (4,2) [device].  Window w runs the reference's recursion
 * (trajectory_tracking.py:195-200)  aux1 = R + B'PB, aux2 = B'PA, K = -inv(aux1) aux2, P <- Q + A'PA + (A'PB) K
 * over stages w+L-2 .. w from P = QT.  all_gains != 0 (nwin == 1): K_out (L-1,2,4) = every gain
 * (solve_LQR_tracking :170-203 with L = S+1);  else K_out (nwin,2,4) = each window's first gain, the exact
 * solution u0 = K x0 of solver_mpc's equality-constrained QP (:73-140, T_pred = L) at control step w
 * (solve_mpc_tracking :8-69).  Q, R [host]; QT (4,4) [device] (e.g. gym_dare_fixed_point's P, no host round trip). */
int gym_tv_lqr_gains(const double* A, const double* B, int32_t S, const double* A_pad, const double* B_pad,
                     const double Q[16], const double R[4], const double QT[16], int32_t L, int32_t nwin,
                     int32_t all_gains, int32_t discretize, double dt, double* K_out, void* stream);
/* compute_P_inf (trajectory_tracking.py:144-165): P (4,4) and the iteration count [device outputs]; A, B discrete
 * [device], Q, R [host].  iters_out = the iteration at which max|P_next - P| < tol held, or max_iter + 1 if it never
 * did (the reference then prints "P_inf did not converge!!!" and returns the last P, :164-165). */
int gym_dare_fixed_point(const double* A, const double* B, const double Q[16], const double R[4], int32_t max_iter,
                         double tol, double* P_out, int32_t* iters_out, void* stream);
/* Fused MPC gains (solve_mpc_tracking :14-38 and every control step's QP, :43-49 / :73-140) in one launch:
 * the discretised linearisation (Calculate_A_B_matrixes + discretize_linearization) of the reference's stages
 * (x_ref (N,4), u_ref (N-1,2) [device], S = N-1 stages) and of the pad (A_f, B_f) at x_f (4), u_f (2) [device];
 * Q_T = compute_P_inf(A_f, B_f, Q, R) (max_iter, tol as :144-165); the first gain of windows 0..nwin-1 of length
 * L = T_pred (stage index >= S -> pad).  Replaces gym_dare_fixed_point + gym_tv_lqr_gains(discretize, !all_gains)
 * on host-side Jacobians.  Q_T is the reference's stop iterate: doubling steps (the structure-preserving doubling
 * algorithm, whose k-th iterate is the fixed point's iterate 2^k - 1) jump ahead while one map still moves the
 * iterate by >= tol, then the reference's loop and test (max|P_next - P| < tol, at most max_iter maps) run from the
 * last such iterate (cfg 5 pad: 9 doublings + ~180 maps instead of 434 dependent maps).  Outputs [device]: K_out
 * (nwin,2,4), QT_out (4,4), iters_out (1) = the reference's iteration count as gym_dare_fixed_point reports it
 * (max_iter + 1: never converged; ABI 15 -- ABI 14 reported doublings).  Q, R [host].  2 <= L <= 254. */
int gym_mpc_gains(const gym_model* m, const double* x_ref, const double* u_ref, int32_t S, const double* x_f,
                  const double* u_f, const double Q[16], const double R[4], int32_t L, int32_t nwin, int32_t max_iter,
                  double tol, double* K_out, double* QT_out, int32_t* iters_out, void* stream);
/* solver_mpc's X_opt (L,4), U_opt (L-1,2): forward pass x_{s+1} = A_s x_s + B_s u_s, u_s = K_s x_s of one window
 * (gains from gym_tv_lqr_gains with all_gains), x0 (4) [device]. */
int gym_lq_forward(const double* A, const double* B, int32_t S, const double* A_pad, const double* B_pad,
                   int32_t discretize, double dt, const double* K, const double* x0, int32_t L, double* X, double* U,
                   void* stream);
/* Batched closed-loop tracking (simulate_tracking :206-216; the MPC loop :43-60):
 *   u_t = u_ff[t] + K[t] (x_t - x_ff[t]),  x_{t+1} = RK4(x_t, u_t)
 * x0 (B,4); shared x_ff (N,4), u_ff (T,2), K (T,2,4); lane-major x_out (B,N,4), u_out (B,T,2). */
int gym_track_rollout(const gym_model* m, const double* x0, const double* x_ff, const double* u_ff, const double* K,
                      int64_t B, int32_t N, double* x_out, double* u_out, void* stream);
/* gym_track_rollout with kernel selection: flags 0 = each trajectory on a lane pair (the default above: the
 * joint-angle trigonometry of every RK4 step split between two lanes, DPP exchange; bit-identical results),
 * GYM_TRACK_SINGLE = one lane per trajectory.  B <= 2^30. */
#define GYM_TRACK_SINGLE 1
int gym_track_rollout_ex(const gym_model* m, const double* x0, const double* x_ff, const double* u_ff,
                         const double* K, int64_t B, int32_t N, int32_t flags, double* x_out, double* u_out,
                         void* stream);

/* [host] create / destroy the events of a gym_timing; collect = add the elapsed time of every pending
 * pair (call only after the stream that recorded them has been synchronised). */
int gym_timing_create(gym_timing* t);
int gym_timing_destroy(gym_timing* t);
int gym_timing_collect(gym_timing* t);

#ifdef __cplusplus
}
#endif
#endif /* GYMNAST_ACROBOT_H */
