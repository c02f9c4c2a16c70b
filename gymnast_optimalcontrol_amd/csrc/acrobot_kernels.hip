// MI355X (gfx950) kernels + C-ABI of the batched acrobot Newton/Armijo engine.
//
// One trajectory ("lane") per GPU thread, 64-thread workgroups (one wavefront), time-major SoA
// streams with the lane innermost.  States and gains are stored as 16-byte pairs (one 1 KiB
// transaction per wavefront load), controls and sigma as 8-byte planes.  The shared references
// x_ref (N,4), u_ref (T,2) are read with wave-uniform addresses (scalar loads).  The whole
// per-lane recursion (Jacobians, Riccati state P/p, RK4 state, running cost) is register-resident;
// no LDS is needed because lanes never exchange data.
//
// The solver's two HBM streams per Newton iteration:
//   backward sweep : read x (2 pairs) + u (2 planes), write K row 1 (2 pairs) + cg (1 plane)
//   Armijo trial   : read K row 1 + cg + u0, write x_new (2 pairs) + u_new (2 planes)
// where cg = (u1 - K1 x) + gamma0 sigma1 folds the reference's u1 + K1 (x_new - x) + gamma0 sigma1 into
// cg + K1 x_new, so the first trial never re-reads the old trajectory x nor sigma1; sigma0 = -r0 / (2R0) is
// recomputed from u0 bit-identically.  sigma1 itself is not streamed: the rare consumers (trials 2..20 of
// lanes that backtrack, the final sigma output, gamma sweeps) re-run the lane's sweep, which reproduces it
// bit for bit, into the sigma1 plane.  Streamed once per pass, these use non-temporal loads/stores.
//
// Reference: /root/reference/trajectory_generation.py (newton_Algorithm :298-398 and the
// primitives it calls) and dynamics.py.  See include/gymnast_acrobot.h for the ABI.
#include <hip/hip_runtime.h>

#include <cstddef>
#include <cstdint>

#include "acrobot_device.hpp"
#include "gymnast_acrobot.h"

using gym::Dyn;

namespace {

constexpr int BLK = 64;           // one wavefront per workgroup for the per-lane recursions
constexpr int STAT_BLOCKS = 256;  // first stage of the deterministic statistics reduction
constexpr int STAT_THREADS = 256;
constexpr int NSTAT = 8;
constexpr int CKI = GYM_CKPT_INTERVAL;   // state checkpoint interval (GYM_FLAG_X_CKPT)

// Cost weights as the kernels take them: the reference's diagonal Q, R, Q_T plus the Gauss-Newton
// blocks' constants (Q_t = 2Q, R_t = 2R, G00 = 2 R0 and its inverse), formed once on the host so that
// they are kernel arguments (SGPRs) rather than per-lane VGPRs.  2x is exact and 1/G00 correctly rounded
// on both sides, so the values are those the device would compute.
struct KW {
    double Q[4], R[2], QT[4];
    double twoQ[4], G00, twoR1, iG00;
};
static_assert(sizeof(Dyn) == 12 * sizeof(double) && sizeof(KW) == 17 * sizeof(double), "kernarg layout");

// The solver kernels take (Dyn m, KW w, ...) as their FIRST two parameters, i.e. at byte offsets 0 and 96 of
// the kernel argument segment.  Inside the stage loops the sweep re-reads them from there every stage with
// scalar loads (the pointer is made opaque per call so the loads are not hoisted): they are then short-
// lived SGPRs instead of 36 loop-invariant dwords that overflow the SGPR file, whose spills to VGPR lanes
// cost one v_readlane (a VALU slot) per dword per stage.
typedef const __attribute__((address_space(4))) double* kptr_t;
struct KArgs {
    Dyn m;
    KW w;
};
__device__ __forceinline__ KArgs kernarg_consts() {
    kptr_t p = (kptr_t)__builtin_amdgcn_kernarg_segment_ptr();
    asm volatile("" : "+s"(p));
    KArgs a;
    a.m.b = p[0]; a.m.d = p[1]; a.m.a2b = p[2]; a.m.bb = p[3]; a.m.dad = p[4]; a.m.g1 = p[5]; a.m.g2 = p[6];
    a.m.f1 = p[7]; a.m.f2 = p[8]; a.m.h = p[9]; a.m.h2 = p[10]; a.m.h6 = p[11];
    for (int i = 0; i < 4; ++i) { a.w.Q[i] = p[12 + i]; a.w.QT[i] = p[18 + i]; a.w.twoQ[i] = p[22 + i]; }
    a.w.R[0] = p[16]; a.w.R[1] = p[17];
    a.w.G00 = p[26]; a.w.twoR1 = p[27]; a.w.iG00 = p[28];
    return a;
}

inline KW kw(const gym_weights& w) {
    KW k;
    for (int i = 0; i < 4; ++i) { k.Q[i] = w.Q[i]; k.QT[i] = w.QT[i]; k.twoQ[i] = 2.0 * w.Q[i]; }
    k.R[0] = w.R[0]; k.R[1] = w.R[1];
    k.G00 = 2.0 * w.R[0]; k.twoR1 = 2.0 * w.R[1]; k.iG00 = 1.0 / k.G00;
    return k;
}

typedef double d2v __attribute__((ext_vector_type(2)));

inline int grid_for(int64_t n, int block, int64_t cap = (int64_t)1 << 30) {
    int64_t g = (n + block - 1) / block;
    if (g < 1) g = 1;
    if (g > cap) g = cap;
    return (int)g;
}

// streamed (read-once / write-once per pass) accesses: non-temporal
__device__ __forceinline__ double2 ld_nt(const double2* p) {
    const d2v v = __builtin_nontemporal_load(reinterpret_cast<const d2v*>(p));
    return make_double2(v.x, v.y);
}
__device__ __forceinline__ double ld_nt(const double* p) { return __builtin_nontemporal_load(p); }
__device__ __forceinline__ void st_nt(double2* p, double a, double b) {
    d2v v = {a, b};
    __builtin_nontemporal_store(v, reinterpret_cast<d2v*>(p));
}
__device__ __forceinline__ void st_nt(double* p, double a) { __builtin_nontemporal_store(a, p); }

// Completes the prefetch loads of the first stage before a software-pipelined stage loop is entered
// (an empty asm that reads the registers forces the wait here, in the preheader).  Without it the loop
// header merges the preheader's pending loads with the back edge's pending stores, and the compiler
// then waits for every store of the previous stage at the top of each iteration, i.e. one full HBM
// write round trip per stage.
// Solver streams through buffer instructions: the stage row's base address lives in a wave-uniform
// buffer resource (SGPRs, rebased per stage by scalar adds), the lane's byte offset in one 32-bit VGPR
// and the row-within-stage offset in an SGPR.  Compared with 64-bit per-lane pointers this frees ~14
// VGPRs and the per-stage 64-bit address arithmetic.  Offsets stay below 2^31 (Bp <= GYM_MAX_BP).
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
typedef unsigned int u32x2 __attribute__((ext_vector_type(2)));
constexpr int kNT = 2;  // gfx950 cache-policy bits: nt (streamed once; other policies measured, profiles/r05/policy)
__device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc(const char* base) {
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<char*>(base), (short)0, 0x7fffffff, 0x00020000);
}
template <int CP = kNT>   // CP: cache policy (kNT for the read-once solver streams, 0 for re-read ones)
__device__ __forceinline__ double2 bld2(__amdgpu_buffer_rsrc_t r, uint32_t vo, uint32_t so) {
    return __builtin_bit_cast(double2, __builtin_amdgcn_raw_buffer_load_b128(r, vo, so, CP));
}
template <int CP = kNT>
__device__ __forceinline__ double bld1(__amdgpu_buffer_rsrc_t r, uint32_t vo, uint32_t so) {
    return __builtin_bit_cast(double, __builtin_amdgcn_raw_buffer_load_b64(r, vo, so, CP));
}
template <int CP = kNT>
__device__ __forceinline__ void bst2(__amdgpu_buffer_rsrc_t r, uint32_t vo, uint32_t so, double a, double b) {
    __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, make_double2(a, b)), r, vo, so, CP);
}
template <int CP = kNT>
__device__ __forceinline__ void bst1(__amdgpu_buffer_rsrc_t r, uint32_t vo, uint32_t so, double a) {
    __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(u32x2, a), r, vo, so, CP);
}

__device__ __forceinline__ void pin(double v) { asm volatile("" : : "v"(v)); }

// Progress-banded wave priority: every solver stream loop starts at priority 3 and steps down one level
// per quarter of its stages.  Without it the SIMD's oldest-first issue arbitration runs the oldest of its
// (at most 4) resident waves far ahead of the youngest (measured: the ranks finish at 0.88 / 1.39 / 1.95
// / 2.49 ms of a 2.5 ms launch), so the launch ends with one wave per SIMD and few loads in flight.  With
// the bands the lagging waves win arbitration, all finish together, and the launch is 6% shorter.
// The stage index is wave-uniform: these are scalar compares and s_setprio, no VALU.
// KIND: 0 = sweep, 1 = trial, 2 = no banding (the caller sets the priority).  (Measured alternatives: sweep
// banded above the trial, 1.3% slower; trial above the sweep, 9.6% slower.)
constexpr int PRIO_NONE = 2;
template <int KIND>
__device__ __forceinline__ void prio_start() {
    if (KIND != PRIO_NONE) __builtin_amdgcn_s_setprio(3);
}
template <int KIND>
__device__ __forceinline__ void prio_band(int done, int T) {
    if (KIND == PRIO_NONE) return;
    asm volatile("" : "+s"(T));   // thresholds recomputed per stage (3 SALU) rather than held: no spills
    if (done >= ((3 * T) >> 2)) __builtin_amdgcn_s_setprio(0);
    else if (done >= (T >> 1)) __builtin_amdgcn_s_setprio(1);
    else if (done >= (T >> 2)) __builtin_amdgcn_s_setprio(2);
}
__device__ __forceinline__ void pin(double2 v) { asm volatile("" : : "v"(v.x), "v"(v.y)); }

// element index of (t, row p of P, lane) in a time-major plane stream (W = 1 doubles): (L, P, Bp)
__device__ __forceinline__ int64_t pix(int t, int p, int P, int64_t l, int64_t Bp) { return ((int64_t)t * P + p) * Bp + l; }
// Per-lane references (GYM_FLAG_REF_LANE, every schedule): x_ref (Bp, N, 4), u_ref (Bp, T, 2), lane-major.
// RL kernels offset the reference pointers by the lane once; everything downstream reads stage t at +4t / +2t as
// with the shared reference (then by vector instead of scalar loads: the same values, the same bits).
template <bool RL>
__device__ __forceinline__ const double* lane_ref(const double* r, int64_t l, int64_t per_lane) {
    return RL ? r + l * per_lane : r;
}
// element index of (t, row p of P, lane) in a wave-blocked pair stream (W = 2, double2): (L, Bp/64, P, 64), i.e.
// the P rows of one wavefront's 64 lanes at one stage form one contiguous P KiB block (one DRAM burst sequence
// instead of P 1-KiB pieces Bp*16 bytes apart).  The stage stride is P*Bp elements, as for planes.
__device__ __forceinline__ int64_t wix(int64_t t, int p, int P, int64_t l, int64_t Bp) {
    return t * P * Bp + (l & ~(int64_t)(BLK - 1)) * P + p * BLK + (l & (BLK - 1));
}
// the same as a byte offset within one stage (buffer-resource addressing), and the row-to-row step
__device__ __forceinline__ uint32_t wbo(int64_t l, int P) {
    return (uint32_t)(((l & ~(int64_t)(BLK - 1)) * P + (l & (BLK - 1))) * 16);
}
constexpr uint32_t WROW = BLK * 16;

// stage cost exactly as total_cost accumulates it (:244-245): J += dx^T Q dx ; J += du^T R du
__device__ __forceinline__ double xcost(const double* w, double n0, double n1, double n2, double n3,
                                        const double* xr) {
#pragma clang fp contract(on)   // context-independent bits (the cost of k_nt_run2's helper wavefront)
    const double e0 = n0 - xr[0], e1 = n1 - xr[1], e2 = n2 - xr[2], e3 = n3 - xr[3];
    return ((e0 * (w[0] * e0) + e1 * (w[1] * e1)) + e2 * (w[2] * e2)) + e3 * (w[3] * e3);
}
// one stage of total_cost (:244-245) added to the running J, with FMA contraction inside each expression only:
// the same bits in every kernel that accumulates a trial's cost.  U0Z: f0 = +0, so f0 (R0 f0) + f1 (R1 f1) is
// f1 (R1 f1) exactly (both contractions of the general expression round to it)
template <bool U0Z = false>
__device__ __forceinline__ double stage_cost(double J, const double* Q, const double* R, double n0, double n1,
                                            double n2, double n3, const double* xrt, double f0, double f1) {
#pragma clang fp contract(on)
    J += xcost(Q, n0, n1, n2, n3, xrt);
    if (U0Z) {
        const double c1 = f1 * (R[1] * f1);
        J += c1;
    } else {
        J += f0 * (R[0] * f0) + f1 * (R[1] * f1);
    }
    return J;
}

// ------------------------------------------------------------------------------------------
// Reference-form rollouts (forward_closed_loop_update :218-229 + total_cost :231-252;
// simulate_open_loop :74-87) for the API entry points:
//   u_new_t = u_t + K_t (x_new_t - x_t) + gamma sigma_t ;  x_new_{t+1} = RK4(x_new_t, u_new_t)
// FULLK = false: open loop, u_new_t = u_t.  x pairs (N,2,Bp); u, sigma planes (T,2,Bp); K pairs (T,4,Bp).
// ------------------------------------------------------------------------------------------
template <bool FULLK, bool WRITE = true>
__device__ __forceinline__ double rollout_ref(const Dyn& m, const KW& w, const double2* __restrict__ x,
                                              const double* __restrict__ u, const double2* __restrict__ K,
                                              const double* __restrict__ s, const double* __restrict__ xr,
                                              const double* __restrict__ ur, double2* __restrict__ xn,
                                              double* __restrict__ un, double gamma, int64_t l, int64_t Bp, int N,
                                              double n0, double n1, double n2, double n3) {
    const int T = N - 1;
    double J = 0.0;
    if (WRITE) {
        xn[wix(0, 0, 2, l, Bp)] = make_double2(n0, n1);
        xn[wix(0, 1, 2, l, Bp)] = make_double2(n2, n3);
    }
    for (int t = 0; t < T; ++t) {
        double v0 = u[pix(t, 0, 2, l, Bp)], v1 = u[pix(t, 1, 2, l, Bp)];
        if (FULLK) {
            const double2 a = x[wix(t, 0, 2, l, Bp)], b = x[wix(t, 1, 2, l, Bp)];
            const double2 k0 = K[wix(t, 0, 4, l, Bp)], k1 = K[wix(t, 1, 4, l, Bp)];
            const double2 k2 = K[wix(t, 2, 4, l, Bp)], k3 = K[wix(t, 3, 4, l, Bp)];
            const double d0 = n0 - a.x, d1 = n1 - a.y, d2 = n2 - b.x, d3 = n3 - b.y;
            const double kd0 = ((k0.x * d0 + k0.y * d1) + k1.x * d2) + k1.y * d3;
            const double kd1 = ((k2.x * d0 + k2.y * d1) + k3.x * d2) + k3.y * d3;
            v0 = (v0 + kd0) + gamma * s[pix(t, 0, 2, l, Bp)];
            v1 = (v1 + kd1) + gamma * s[pix(t, 1, 2, l, Bp)];
            if (WRITE) {
                un[pix(t, 0, 2, l, Bp)] = v0;
                un[pix(t, 1, 2, l, Bp)] = v1;
            }
        }
        const double* urt = ur + 2 * t;
        const double f0 = v0 - urt[0], f1 = v1 - urt[1];
        J = stage_cost(J, w.Q, w.R, n0, n1, n2, n3, xr + 4 * t, f0, f1);
        gym::rk4(m, n0, n1, n2, n3, v1);
        if (WRITE) {
            xn[wix(t + 1, 0, 2, l, Bp)] = make_double2(n0, n1);
            xn[wix(t + 1, 1, 2, l, Bp)] = make_double2(n2, n3);
        }
    }
    return J + xcost(w.QT, n0, n1, n2, n3, xr + 4 * T);
}

// ------------------------------------------------------------------------------------------
// Solver rollout (Armijo trial / candidate / accepted-candidate re-run), offset form:
//   u_new0 = u0 + gamma sigma0,  sigma0 = -(2R0 (u0 - ur0)) / (2R0)     (bit-identical to the sweep)
//   u_new1 = cg + K1 x_new,  cg = (u1 - K1 x) + gamma0 sigma1  (the sweep's offset)          first trial
//   u_new1 = fma(gamma - gamma0, sigma1, cg + K1 x_new)                          SIG: any other step size
// (at gamma = gamma0 the SIG form returns the first trial's value exactly).
// Streams per stage: K1 (2 pairs) + cg (plane) [+ sigma1 (plane) if SIG] + u0 (plane) in; x_new, u_new out.
// cs: (T, 2, Bp) planes, plane 0 = cg, plane 1 = sigma1.
// ------------------------------------------------------------------------------------------
// Streams of one stage of the offset-form rollout, prefetched into registers one stage ahead.
struct TrialStage {
    double2 k0, k1;      // K row 1 (two pairs)
    double cg, s1;       // offset cg, sigma1 (SIG only)
    double u0;           // tau1 control (0 when U0Z)
};

// The trial's controls of one stage, each with FMA contraction inside its expression only (the same bits in
// every kernel, including k_nt_run2 where the helper wavefront forms u0 and the cost):
//   u0_new = u0 + gamma sigma0,  sigma0 = -(2R0 (u0 - ur0)) / (2R0)  == the sweep's sigma0, bit for bit
//   (U0Z: u0 = ur0 = 0  =>  u0_new = +0 exactly)
__device__ __forceinline__ double trial_u0(double u0, double ur0, double gamma, double G00, double iG00) {
#pragma clang fp contract(on)
    const double s0 = -(G00 * (u0 - ur0)) * iG00;
    return u0 + gamma * s0;
}
//   u1_new = cg + K1 x_new  (the first trial, gamma = gamma0)
__device__ __forceinline__ double trial_u1(double2 k0, double2 k1, double cg, double n0, double n1, double n2,
                                          double n3) {
#pragma clang fp contract(on)
    const double kx = ((k0.x * n0 + k0.y * n1) + k1.x * n2) + k1.y * n3;
    return cg + kx;
}
//   u1_new = fma(gamma - gamma0, sigma1, cg + K1 x_new)  (any other step size)
__device__ __forceinline__ double trial_u1_sig(double2 k0, double2 k1, double cg, double s1, double dg, double n0,
                                              double n1, double n2, double n3) {
#pragma clang fp contract(on)
    const double kx = ((k0.x * n0 + k0.y * n1) + k1.x * n2) + k1.y * n3;
    return __builtin_fma(dg, s1, cg + kx);
}

template <bool WRITE, bool U0Z, bool SIG, bool CK = false, int CP = kNT, bool BAND = true, int PD = 1>
__device__ __forceinline__ double rollout_cform(const Dyn& m, const KW& w, const double* __restrict__ u,
                                                const double2* __restrict__ K1, const double* __restrict__ cs,
                                                const double* __restrict__ xr, const double* __restrict__ ur,
                                                double2* __restrict__ xn, double* __restrict__ un, double gamma,
                                                double gamma0, int64_t l, int64_t Bp, int N, double n0, double n1,
                                                double n2, double n3) {
    const int T = N - 1;
    const double G00 = w.G00, iG00 = w.iG00;
    // lane byte offsets: 2-row wave-blocked pairs (K1, x), planes (cs, u)
    const uint32_t o2 = wbo(l, 2), o1 = (uint32_t)l * 8u;
    const uint32_t row = (uint32_t)Bp * 16u, plane = (uint32_t)Bp * 8u;
    const double dg = gamma - gamma0;                     // SIG: step size relative to the first trial's
    const char* Kb = reinterpret_cast<const char*>(K1);   // stage stride 2 rows
    const char* Cb = reinterpret_cast<const char*>(cs);   // stage stride 2 planes = 1 row
    const char* Ub = reinterpret_cast<const char*>(u);    // stage stride 2 planes = 1 row
    const char* Xb = reinterpret_cast<const char*>(xn);   // stage stride 2 rows
    const char* Ob = reinterpret_cast<const char*>(un);   // stage stride 1 row
    double J = 0.0;
    if (WRITE) {
        const auto rX = rsrc(Xb);
        bst2(rX, o2, 0, n0, n1);
        bst2(rX, o2, WROW, n2, n3);
    }
    auto fetch = [&](TrialStage& q, int t) {   // stage t's streams into register set q
        const auto rK = rsrc(Kb + (int64_t)t * (2 * (int64_t)row));
        q.k0 = bld2<CP>(rK, o2, 0);
        q.k1 = bld2<CP>(rK, o2, WROW);
        const auto rC = rsrc(Cb + (int64_t)t * row);
        q.cg = bld1<CP>(rC, o1, 0);
        q.s1 = SIG ? bld1<CP>(rC, o1, plane) : 0.0;
        q.u0 = U0Z ? 0.0 : bld1<CP>(rsrc(Ub + (int64_t)t * row), o1, 0);
    };
    const gym::PolyRegs pk = gym::poly_vgprs();   // loop-invariant coefficients held in VGPRs
    // stage t with its streams in q (prefetched earlier)
    auto body = [&](const TrialStage& q, int t) {
        prio_band<BAND ? 1 : PRIO_NONE>(t, T);
        const double* urt = ur + 2 * t;
        const double v0 = U0Z ? 0.0 : trial_u0(q.u0, urt[0], gamma, G00, iG00);   // U0Z: +0 exactly
        const double v1 = SIG ? trial_u1_sig(q.k0, q.k1, q.cg, q.s1, dg, n0, n1, n2, n3)
                              : trial_u1(q.k0, q.k1, q.cg, n0, n1, n2, n3);
        const double f0 = U0Z ? 0.0 : v0 - urt[0], f1 = v1 - urt[1];
        const KArgs ka = kernarg_consts();   // cost weights re-read per stage (no SGPR spills)
        J = stage_cost<U0Z>(J, ka.w.Q, ka.w.R, n0, n1, n2, n3, xr + 4 * t, f0, f1);
        if (WRITE) {
            const auto rO = rsrc(Ob + (int64_t)t * row);
            if (!U0Z) bst1(rO, o1, 0, v0);             // U0Z: the u0 planes stay zero
            bst1(rO, o1, plane, v1);
        }
        gym::rk4_fast(m, n0, n1, n2, n3, v1, pk);      // near path without sub-step branches
        if (WRITE && (!CK || (t + 1) % CKI == 0 || t + 1 == T)) {   // CK: checkpoint knots only
            const auto rX = rsrc(Xb + (int64_t)(t + 1) * (2 * (int64_t)row));
            bst2(rX, o2, 0, n0, n1);
            bst2(rX, o2, WROW, n2, n3);
        }
    };
    if constexpr (PD == 1) {
        TrialStage pre;   // software prefetch of stage t+1's streams while stage t computes
        fetch(pre, 0);
        pin(pre.k0); pin(pre.k1); pin(pre.cg); pin(pre.s1); pin(pre.u0);
        prio_start<BAND ? 1 : PRIO_NONE>();
        for (int t = 0; t < T; ++t) {
            const TrialStage q = pre;
            fetch(pre, t + 1 < T ? t + 1 : t);   // unconditional (the last stage's copy unused): no phi, no copies
            body(q, t);
        }
    } else {
        // prefetch distance 2 (few wavefronts per SIMD: two stages of loads in flight behind each stage's compute):
        // three register sets in rotation, unrolled by 3 so that no set is copied (a copy waits for its load)
        static_assert(PD == 2, "prefetch distance 1 or 2");
        auto clampT = [&](int v) { return __builtin_amdgcn_readfirstlane(v < T ? v : T - 1); };
        TrialStage s0, s1, s2;
        fetch(s0, 0);
        fetch(s1, clampT(1));
        prio_start<BAND ? 1 : PRIO_NONE>();
        int t = 0;
        for (; t + 3 <= T; t += 3) {
            fetch(s2, clampT(t + 2));
            body(s0, t);
            fetch(s0, clampT(t + 3));
            body(s1, t + 1);
            fetch(s1, clampT(t + 4));
            body(s2, t + 2);
        }
        if (t < T) body(s0, t);
        if (t + 1 < T) body(s1, t + 1);
    }
    return J + xcost(w.QT, n0, n1, n2, n3, xr + 4 * T);
}

// ------------------------------------------------------------------------------------------
// Fused backward sweep of one lane (compute_costate_trajectory :138-159, build_stage_lists
// :166-181, calculate_K_and_sigma :183-216) exploiting the model structure:
//   A_d = I + dt A_c with A_c rows 0,1 = e3^T, e4^T ; B_d = dt B_c with only column 1 non-zero
//   Q_t = 2Q, R_t = 2R (diagonal), S_t = 0  =>  G = diag(2R0, 2R1 + b^T P b), K_t row 0 = 0.
// P is kept symmetric (10 registers), p and (optionally) the costate lambda in registers.
// ------------------------------------------------------------------------------------------
// Stage t's linearisation (build_stage_lists :166-181 with discretize_linearization :161-164): rows 2, 3 of
// A_d = I + dt A_c (rows 0, 1 are [1 0 dt 0], [0 1 0 dt]), column 1 of B_d = dt B_c, q_t = 2Q dx_t, r_t = 2R du_t.
// A function of x_t, u_t only (not of P), so it can be evaluated apart from the Riccati chain.
// U0Z (GYM_FLAG_U0_ZERO: u0 = ur0 = 0): r0 = 2R0 (u0 - ur0) is +0 (the bits the general expression gives), and the
// Riccati step drops the terms it zeroes (sigma0 = -0, its dJ and max|sigma| contributions): the same bits.
struct Lin {
    double A20, A21, A22, A23, A30, A31, A32, A33, bd2, bd3, q0, q1, q2, q3, r0, r1, dt;
};
template <bool U0Z = false>
__device__ __forceinline__ Lin stage_lin(const Dyn& m, const KW& w, const gym::Jac& J, double2 xa, double2 xb,
                                         double ut0, double ut1, const double* xrt, const double* urt) {
#pragma clang fp contract(on)
    const double dt = m.h;
    Lin L;
    L.A20 = dt * J.a2[0]; L.A21 = dt * J.a2[1]; L.A22 = 1.0 + dt * J.a2[2]; L.A23 = dt * J.a2[3];
    L.A30 = dt * J.a3[0]; L.A31 = dt * J.a3[1]; L.A32 = dt * J.a3[2]; L.A33 = 1.0 + dt * J.a3[3];
    L.bd2 = dt * J.bc2; L.bd3 = dt * J.bc3;
    L.q0 = w.twoQ[0] * (xa.x - xrt[0]); L.q1 = w.twoQ[1] * (xa.y - xrt[1]);
    L.q2 = w.twoQ[2] * (xb.x - xrt[2]); L.q3 = w.twoQ[3] * (xb.y - xrt[3]);
    L.r0 = U0Z ? 0.0 : w.G00 * (ut0 - urt[0]);
    L.r1 = w.twoR1 * (ut1 - urt[1]);
    L.dt = dt;
    return L;
}

template <bool LAMBDA>
struct Sweep {
    double P00, P01, P02, P03, P11, P12, P13, P22, P23, P33, p0, p1, p2, p3;
    double l0 = 0, l1 = 0, l2 = 0, l3 = 0;
    double dJ = 0.0, smax = 0.0;

    // terminal conditions from x_N (P = 2 Q_T, p = 2 Q_T dx_N; lambda_N = p)
    __device__ __forceinline__ Sweep(const KW& w, double2 xa, double2 xb, const double* xrT) {
        P00 = 2.0 * w.QT[0]; P11 = 2.0 * w.QT[1]; P22 = 2.0 * w.QT[2]; P33 = 2.0 * w.QT[3];
        P01 = P02 = P03 = P12 = P13 = P23 = 0.0;
        p0 = P00 * (xa.x - xrT[0]); p1 = P11 * (xa.y - xrT[1]);
        p2 = P22 * (xb.x - xrT[2]); p3 = P33 * (xb.y - xrT[3]);
        if (LAMBDA) { l0 = p0; l1 = p1; l2 = p2; l3 = p3; }
    }

    // stage t (x_t = (xa, xb), u_t = (ut0, ut1)): gain row 1 k[0..3], sigma (s0, s1); updates P, p, dJ, smax
    template <bool U0Z = false>
    __device__ __forceinline__ void step(const Dyn& m, const KW& w, double2 xa, double2 xb, double ut0, double ut1,
                                         const double* xrt, const double* urt, double& k0, double& k1,
                                         double& k2, double& k3, double& s0, double& s1,
                                         const gym::PolyRegs& pk = gym::poly_lits()) {
        step_j<U0Z>(m, w, gym::jacobian(m, xa.x, xa.y, xb.x, xb.y, ut1, pk), xa, xb, ut0, ut1, xrt, urt, k0, k1, k2,
                    k3, s0, s1);
    }
    // the same with the stage's Jacobian already evaluated (it depends on x_t, u_t only, not on P)
    template <bool U0Z = false>
    __device__ __forceinline__ void step_j(const Dyn& m, const KW& w, const gym::Jac& J, double2 xa, double2 xb,
                                           double ut0, double ut1, const double* xrt, const double* urt, double& k0,
                                           double& k1, double& k2, double& k3, double& s0, double& s1) {
        step_lin<U0Z>(w, stage_lin<U0Z>(m, w, J, xa, xb, ut0, ut1, xrt, urt), k0, k1, k2, k3, s0, s1);
    }
    // the Riccati update of stage t from its linearisation (stage_lin: a function of x_t, u_t only): the matrix half
    // (gain row 1, P) and then the vector half (sigma, dJ, p, ||sigma||_inf)
    template <bool U0Z = false>
    __device__ __forceinline__ void step_lin(const KW& w, const Lin& L, double& k0, double& k1, double& k2,
                                             double& k3, double& s0, double& s1) {
        double G11, iG;
        step_P(w, L, k0, k1, k2, k3, G11, iG);
        step_p<U0Z>(w, L, k0, k1, k2, k3, G11, iG, s0, s1);
    }
    // The matrix half of step_lin: gain row 1 k = -(P b)^T A_d / G11, G11 = 2R1 + b^T P b and its reciprocal, and
    // P <- 2Q + A_d^T P A_d - G11 k k^T.  A function of P and the stage's A_d, b only (not of p), so k_nt_run2
    // runs it alone on its main wavefront and hands k, G11, 1/G11 to another wavefront for the vector half.
    // FMA contraction within each expression only, never across statements: the bits then do not depend on the
    // context the stage is compiled into (the interleaved sweep of backward_solver_lane_ilp, the sigma1 re-runs,
    // the split sweep of k_nt_run2) -- with cross-statement fusion they did
    __device__ __forceinline__ void step_P(const KW& w, const Lin& L, double& k0, double& k1, double& k2, double& k3,
                                           double& G11, double& iG) {
#pragma clang fp contract(on)
        const double dt = L.dt;
        const double A20 = L.A20, A21 = L.A21, A22 = L.A22, A23 = L.A23;
        const double A30 = L.A30, A31 = L.A31, A32 = L.A32, A33 = L.A33;
        const double bd2 = L.bd2, bd3 = L.bd3;
        // Pb = P B_d[:,1]
        const double Pb0 = P02 * bd2 + P03 * bd3, Pb1 = P12 * bd2 + P13 * bd3;
        const double Pb2 = P22 * bd2 + P23 * bd3, Pb3 = P23 * bd2 + P33 * bd3;
        G11 = w.twoR1 + (bd2 * Pb2 + bd3 * Pb3);
        // F row 1 = (P b)^T A_d
        const double F0 = Pb0 + A20 * Pb2 + A30 * Pb3;
        const double F1 = Pb1 + A21 * Pb2 + A31 * Pb3;
        const double F2 = dt * Pb0 + A22 * Pb2 + A32 * Pb3;
        const double F3 = dt * Pb1 + A23 * Pb2 + A33 * Pb3;
        iG = gym::recip(G11);   // G11 = 2 R1 + b^T P b >= 2 R1 > 0: rcp + two Newton steps
        k0 = -F0 * iG; k1 = -F1 * iG; k2 = -F2 * iG; k3 = -F3 * iG;
        // W = P A_d
        const double W00 = P00 + P02 * A20 + P03 * A30, W01 = P01 + P02 * A21 + P03 * A31;
        const double W02 = dt * P00 + P02 * A22 + P03 * A32, W03 = dt * P01 + P02 * A23 + P03 * A33;
        const double W10 = P01 + P12 * A20 + P13 * A30, W11 = P11 + P12 * A21 + P13 * A31;
        const double W12 = dt * P01 + P12 * A22 + P13 * A32, W13 = dt * P11 + P12 * A23 + P13 * A33;
        const double W20 = P02 + P22 * A20 + P23 * A30, W21 = P12 + P22 * A21 + P23 * A31;
        const double W22 = dt * P02 + P22 * A22 + P23 * A32, W23 = dt * P12 + P22 * A23 + P23 * A33;
        const double W30 = P03 + P23 * A20 + P33 * A30, W31 = P13 + P23 * A21 + P33 * A31;
        const double W32 = dt * P03 + P23 * A22 + P33 * A32, W33 = dt * P13 + P23 * A23 + P33 * A33;
        // P <- 2Q + A_d^T W - K^T G K   (K^T G K = G11 k k^T)
        const double gk0 = G11 * k0, gk1 = G11 * k1, gk2 = G11 * k2, gk3 = G11 * k3;
        const double nP00 = w.twoQ[0] + (W00 + A20 * W20 + A30 * W30) - gk0 * k0;
        const double nP01 = (W01 + A20 * W21 + A30 * W31) - gk0 * k1;
        const double nP02 = (W02 + A20 * W22 + A30 * W32) - gk0 * k2;
        const double nP03 = (W03 + A20 * W23 + A30 * W33) - gk0 * k3;
        const double nP11 = w.twoQ[1] + (W11 + A21 * W21 + A31 * W31) - gk1 * k1;
        const double nP12 = (W12 + A21 * W22 + A31 * W32) - gk1 * k2;
        const double nP13 = (W13 + A21 * W23 + A31 * W33) - gk1 * k3;
        const double nP22 = w.twoQ[2] + (dt * W02 + A22 * W22 + A32 * W32) - gk2 * k2;
        const double nP23 = (dt * W03 + A22 * W23 + A32 * W33) - gk2 * k3;
        const double nP33 = w.twoQ[3] + (dt * W13 + A23 * W23 + A33 * W33) - gk3 * k3;
        P00 = nP00; P01 = nP01; P02 = nP02; P03 = nP03; P11 = nP11; P12 = nP12; P13 = nP13;
        P22 = nP22; P23 = nP23; P33 = nP33;
    }
    // The vector half of step_lin from the stage's gain row, G11 and 1/G11 (step_P): the costate (LAMBDA), sigma,
    // dJ, p <- q + A_d^T p - K^T G sigma and the running ||sigma||_inf.  Not a function of P.
    template <bool U0Z = false>
    __device__ __forceinline__ void step_p(const KW& w, const Lin& L, double k0, double k1, double k2, double k3,
                                           double G11, double iG, double& s0, double& s1) {
#pragma clang fp contract(on)
        const double dt = L.dt;
        const double A20 = L.A20, A21 = L.A21, A22 = L.A22, A23 = L.A23;
        const double A30 = L.A30, A31 = L.A31, A32 = L.A32, A33 = L.A33;
        const double bd2 = L.bd2, bd3 = L.bd3;
        const double q0 = L.q0, q1 = L.q1, q2 = L.q2, q3 = L.q3, r0 = L.r0, r1 = L.r1;
        if (LAMBDA) {  // lambda_t = 2Q dx_t + A_d^T lambda_{t+1}
            const double n0 = q0 + (l0 + A20 * l2 + A30 * l3);
            const double n1 = q1 + (l1 + A21 * l2 + A31 * l3);
            const double n2 = q2 + (dt * l0 + A22 * l2 + A32 * l3);
            const double n3 = q3 + (dt * l1 + A23 * l2 + A33 * l3);
            l0 = n0; l1 = n1; l2 = n2; l3 = n3;
        }
        const double g1 = r1 + (bd2 * p2 + bd3 * p3);
        s1 = -g1 * iG;
        if (U0Z) {   // r0 = +0: sigma0 = -0, and r0 sigma0 + g1 sigma1 = g1 sigma1 exactly
            s0 = -0.0;
            const double d1 = g1 * s1;
            dJ += d1;
        } else {
            s0 = -r0 * w.iG00;
            dJ += r0 * s0 + g1 * s1;
        }
        // p <- q + A_d^T p - K^T G sigma
        const double gs = G11 * s1;
        const double np0 = q0 + (p0 + A20 * p2 + A30 * p3) - k0 * gs;
        const double np1 = q1 + (p1 + A21 * p2 + A31 * p3) - k1 * gs;
        const double np2 = q2 + (dt * p0 + A22 * p2 + A32 * p3) - k2 * gs;
        const double np3 = q3 + (dt * p1 + A23 * p2 + A33 * p3) - k3 * gs;
        p0 = np0; p1 = np1; p2 = np2; p3 = np3;
        // U0Z: |sigma0| = 0 never raises smax (>= 0 or NaN)
        smax = U0Z ? gym::nanmax_abs(smax, s1) : gym::nanmax_abs(gym::nanmax_abs(smax, s0), s1);
    }
};

// API form: writes K row 1 (pairs), sigma planes and optionally lambda; register prefetch of stage t-1.
template <bool LAMBDA>
__device__ __forceinline__ void backward_lane(const Dyn& m, const KW& w, const double2* __restrict__ x,
                                              const double* __restrict__ u, const double* __restrict__ xr,
                                              const double* __restrict__ ur, double2* __restrict__ K1,
                                              double* __restrict__ sig, double2* __restrict__ lam, int64_t l,
                                              int64_t Bp, int N, double& dJ_out, double& smax_out) {
    const int T = N - 1;
    Sweep<LAMBDA> S(w, x[wix(T, 0, 2, l, Bp)], x[wix(T, 1, 2, l, Bp)], xr + 4 * T);
    if (LAMBDA) {
        lam[wix(T, 0, 2, l, Bp)] = make_double2(S.l0, S.l1);
        lam[wix(T, 1, 2, l, Bp)] = make_double2(S.l2, S.l3);
    }
    double2 pa = x[wix(T - 1, 0, 2, l, Bp)], pb = x[wix(T - 1, 1, 2, l, Bp)];
    double pu0 = u[pix(T - 1, 0, 2, l, Bp)], pu1 = u[pix(T - 1, 1, 2, l, Bp)];
    for (int t = T - 1; t >= 0; --t) {
        const double2 xa = pa, xb = pb;
        const double ut0 = pu0, ut1 = pu1;
        if (t > 0) {
            pa = x[wix(t - 1, 0, 2, l, Bp)];
            pb = x[wix(t - 1, 1, 2, l, Bp)];
            pu0 = u[pix(t - 1, 0, 2, l, Bp)];
            pu1 = u[pix(t - 1, 1, 2, l, Bp)];
        }
        double k0, k1, k2, k3, s0, s1;
        S.step(m, w, xa, xb, ut0, ut1, xr + 4 * t, ur + 2 * t, k0, k1, k2, k3, s0, s1);
        if (LAMBDA) {
            lam[wix(t, 0, 2, l, Bp)] = make_double2(S.l0, S.l1);
            lam[wix(t, 1, 2, l, Bp)] = make_double2(S.l2, S.l3);
        }
        K1[wix(t, 0, 2, l, Bp)] = make_double2(k0, k1);
        K1[wix(t, 1, 2, l, Bp)] = make_double2(k2, k3);
        sig[pix(t, 0, 2, l, Bp)] = s0;
        sig[pix(t, 1, 2, l, Bp)] = s1;
    }
    dJ_out = S.dJ;
    smax_out = S.smax;
}

// Streams of one sweep stage (x_t pairs, u_t planes), prefetched into registers ahead of the stage.
struct SweepStage {
    double2 xa, xb;
    double u0, u1;
};

// What a solver sweep stores: K row 1 + cg (every iteration), sigma1 only (re-run for the trials 2..20 and
// the final sigma), or all three (gamma sweeps).
enum SweepOut { OUT_SOLVER = 0, OUT_SIGMA = 1, OUT_ALL = 2 };

// stage t's sweep outputs: K row 1 (wave-blocked pairs), cg (plane 0 of cs), sigma1 (plane 1)
// the stage's offset cg = (u1 - K1 x) + gamma0 sigma1 (FMA contraction inside the expression only)
__device__ __forceinline__ double stage_cg(double2 xa, double2 xb, double ut1, double g0, double k0, double k1,
                                           double k2, double k3, double s1) {
#pragma clang fp contract(on)
    const double c1 = ut1 - (((k0 * xa.x + k1 * xa.y) + k2 * xb.x) + k3 * xb.y);
    return __builtin_fma(g0, s1, c1);
}
template <int OUT>
__device__ __forceinline__ void store_stage(const char* Kb, const char* Cb, int t, uint32_t row, uint32_t plane,
                                            uint32_t o2, uint32_t o1, double2 xa, double2 xb, double ut1, double g0,
                                            double k0, double k1, double k2, double k3, double s1) {
    const auto rC = rsrc(Cb + (int64_t)t * row);
    if (OUT != OUT_SIGMA) {
        const auto rK = rsrc(Kb + (int64_t)t * (2 * (int64_t)row));
        bst2(rK, o2, 0, k0, k1);
        bst2(rK, o2, WROW, k2, k3);
        bst1(rC, o1, 0, stage_cg(xa, xb, ut1, g0, k0, k1, k2, k3, s1));
    }
    if (OUT != OUT_SOLVER) bst1(rC, o1, plane, s1);
}

// Solver sweep of one lane: writes K row 1 and cg = (u1 - K1 x) + gamma0 sigma1 (and / or sigma1, OUT),
// prefetching stage t-1's streams while stage t computes.  U0Z: the tau1 channel is identically zero
// (u0 = ur0 = 0, GYM_FLAG_U0_ZERO) and its plane is not read.
template <bool U0Z, int OUT, bool BAND = true, int PD = 1>
__device__ __forceinline__ void backward_solver_lane(const Dyn& m, const KW& w,
                                                     const double2* __restrict__ x, const double* __restrict__ u,
                                                     const double* __restrict__ xr, const double* __restrict__ ur,
                                                     double2* __restrict__ K1, double* __restrict__ cs, double g0,
                                                     int64_t l, int64_t Bp, int N, double& dJ_out, double& smax_out) {
    const int T = N - 1;
    // lane byte offsets: 2-row wave-blocked pairs (x, K1), planes (cs, u)
    const uint32_t o2 = wbo(l, 2), o1 = (uint32_t)l * 8u;
    const uint32_t row = (uint32_t)Bp * 16u, plane = (uint32_t)Bp * 8u;
    const char* Xb = reinterpret_cast<const char*>(x);    // stage stride 2 rows
    const char* Ub = reinterpret_cast<const char*>(u);    // stage stride 1 row
    const char* Kb = reinterpret_cast<const char*>(K1);
    const char* Cb = reinterpret_cast<const char*>(cs);
    Sweep<false> S(w, x[wix(T, 0, 2, l, Bp)], x[wix(T, 1, 2, l, Bp)], xr + 4 * T);
    const gym::PolyRegs pk = gym::poly_vgprs();
    if constexpr (PD == 2) {
        // prefetch distance 2: three stream sets in rotation, unrolled by 3 (see rollout_cform)
        auto fetch = [&](SweepStage& q, int t) {
            const int tp = __builtin_amdgcn_readfirstlane(t > 0 ? t : 0);
            const auto rX = rsrc(Xb + (int64_t)tp * (2 * (int64_t)row));
            const auto rU = rsrc(Ub + (int64_t)tp * row);
            q.xa = bld2(rX, o2, 0);
            q.xb = bld2(rX, o2, WROW);
            q.u0 = U0Z ? 0.0 : bld1(rU, o1, 0);
            q.u1 = bld1(rU, o1, plane);
        };
        auto body = [&](const SweepStage& q, int t) {
            prio_band<BAND ? 0 : PRIO_NONE>(T - 1 - t, T);
            double k0, k1, k2, k3, s0, s1;
            const KArgs ka = kernarg_consts();
            S.template step<U0Z>(ka.m, ka.w, q.xa, q.xb, q.u0, q.u1, xr + 4 * t, ur + 2 * t, k0, k1, k2, k3, s0, s1,
                                 pk);
            store_stage<OUT>(Kb, Cb, t, row, plane, o2, o1, q.xa, q.xb, q.u1, g0, k0, k1, k2, k3, s1);
        };
        SweepStage s0, s1, s2;
        fetch(s0, T - 1);
        fetch(s1, T - 2);
        prio_start<BAND ? 0 : PRIO_NONE>();
        int t = T - 1;
        for (; t >= 2; t -= 3) {
            fetch(s2, t - 2);
            body(s0, t);
            fetch(s0, t - 3);
            body(s1, t - 1);
            fetch(s1, t - 4);
            body(s2, t - 2);
        }
        if (t >= 0) body(s0, t);
        if (t >= 1) body(s1, t - 1);
        dJ_out = S.dJ;
        smax_out = S.smax;
        return;
    }
    double2 pa, pb;
    double pu0 = 0.0, pu1;
    {
        const auto rX = rsrc(Xb + (int64_t)(T - 1) * (2 * (int64_t)row)), rU = rsrc(Ub + (int64_t)(T - 1) * row);
        pa = bld2(rX, o2, 0); pb = bld2(rX, o2, WROW); pu1 = bld1(rU, o1, plane);
        if (!U0Z) pu0 = bld1(rU, o1, 0);
    }
    pin(pa); pin(pb); pin(pu0); pin(pu1);
    prio_start<BAND ? 0 : PRIO_NONE>();
    for (int t = T - 1; t >= 0; --t) {
        prio_band<BAND ? 0 : PRIO_NONE>(T - 1 - t, T);
        const double2 xa = pa, xb = pb;
        const double ut0 = pu0, ut1 = pu1;
        {   // unconditional (at t = 0 stage 0 again, unused): no phi, no copies of the prefetch registers
            const int tp = __builtin_amdgcn_readfirstlane(t > 0 ? t - 1 : 0);   // wave-uniform
            const auto rX = rsrc(Xb + (int64_t)tp * (2 * (int64_t)row));
            const auto rU = rsrc(Ub + (int64_t)tp * row);
            pa = bld2(rX, o2, 0);
            pb = bld2(rX, o2, WROW);
            if (!U0Z) pu0 = bld1(rU, o1, 0);
            pu1 = bld1(rU, o1, plane);
        }
        double k0, k1, k2, k3, s0, s1;
        const KArgs ka = kernarg_consts();   // the kernel's (Dyn, KW) arguments, re-read: no SGPR spills
        S.step<U0Z>(ka.m, ka.w, xa, xb, ut0, ut1, xr + 4 * t, ur + 2 * t, k0, k1, k2, k3, s0, s1, pk);
        store_stage<OUT>(Kb, Cb, t, row, plane, o2, o1, xa, xb, ut1, g0, k0, k1, k2, k3, s1);
    }
    dJ_out = S.dJ;
    smax_out = S.smax;
}

// The solver sweep for ONE wavefront per SIMD (the persistent kernel at its batch sizes), where a stage's time is
// its dependency chain, not the SIMD's issue rate: stage t-1's Jacobian (a function of x_{t-1}, u_{t-1} only) is
// evaluated beside stage t's Riccati update, so the two chains interleave.  That needs stage t-1's streams in
// registers one stage early: prefetch distance 2, three stream sets and two Jacobians in rotation (unrolled by
// 6, so that no set is copied -- a copy of a loading register waits for its load).  Same per-stage arithmetic
// as backward_solver_lane (step = jacobian + step_j): the same bits.
template <bool U0Z, int OUT>
__device__ __forceinline__ void backward_solver_lane_ilp(const Dyn& m, const KW& w,
                                                         const double2* __restrict__ x, const double* __restrict__ u,
                                                         const double* __restrict__ xr, const double* __restrict__ ur,
                                                         double2* __restrict__ K1, double* __restrict__ cs, double g0,
                                                         int64_t l, int64_t Bp, int N, double& dJ_out,
                                                         double& smax_out) {
    const int T = N - 1;
    const uint32_t o2 = wbo(l, 2), o1 = (uint32_t)l * 8u;
    const uint32_t row = (uint32_t)Bp * 16u, plane = (uint32_t)Bp * 8u;
    const char* Xb = reinterpret_cast<const char*>(x);
    const char* Ub = reinterpret_cast<const char*>(u);
    const char* Kb = reinterpret_cast<const char*>(K1);
    const char* Cb = reinterpret_cast<const char*>(cs);
    Sweep<false> S(w, x[wix(T, 0, 2, l, Bp)], x[wix(T, 1, 2, l, Bp)], xr + 4 * T);
    const gym::PolyRegs pk = gym::poly_vgprs();
    auto fetch = [&](SweepStage& q, int t) {
        const auto rX = rsrc(Xb + (int64_t)t * (2 * (int64_t)row)), rU = rsrc(Ub + (int64_t)t * row);
        q.xa = bld2(rX, o2, 0);
        q.xb = bld2(rX, o2, WROW);
        q.u0 = U0Z ? 0.0 : bld1(rU, o1, 0);
        q.u1 = bld1(rU, o1, plane);
    };
    auto jac = [&](const SweepStage& q) {
        const KArgs ka = kernarg_consts();
        return gym::jacobian(ka.m, q.xa.x, q.xa.y, q.xb.x, q.xb.y, q.u1, pk);
    };
    // stage t: c = its streams, Jc = its Jacobian; n = stage t-1's streams (landed), f <- stage t-2's
    auto stage = [&](const SweepStage& c, const SweepStage& n, SweepStage& f, const gym::Jac& Jc, gym::Jac& Jn,
                     int t) {
        if (t < 0) return;
        if (t >= 2) fetch(f, t - 2);
        if (t >= 1) Jn = jac(n);
        double k0, k1, k2, k3, s0, s1;
        const KArgs ka = kernarg_consts();
        S.step_j<U0Z>(ka.m, ka.w, Jc, c.xa, c.xb, c.u0, c.u1, xr + 4 * t, ur + 2 * t, k0, k1, k2, k3, s0, s1);
        store_stage<OUT>(Kb, Cb, t, row, plane, o2, o1, c.xa, c.xb, c.u1, g0, k0, k1, k2, k3, s1);
    };
    SweepStage A, B, C;
    gym::Jac J0, J1;
    fetch(A, T - 1);
    if (T >= 2) fetch(B, T - 2);
    J0 = jac(A);
    for (int t = T - 1; t >= 0; t -= 6) {
        stage(A, B, C, J0, J1, t);
        stage(B, C, A, J1, J0, t - 1);
        stage(C, A, B, J0, J1, t - 2);
        stage(A, B, C, J1, J0, t - 3);
        stage(B, C, A, J0, J1, t - 4);
        stage(C, A, B, J1, J0, t - 5);
    }
    dJ_out = S.dJ;
    smax_out = S.smax;
}

// Checkpointed solver sweep (GYM_FLAG_X_CKPT): the trial stored x only at the knots c0 = 0, CKI, 2 CKI, ...
// and T.  Going backward one block [c0, c0 + len) at a time, the sweep takes the block's checkpoint x_c0
// and controls, re-integrates x_{c0+1} .. x_{c0+len-1} with the trial's RK4 (same inputs, same code: the
// same bits) into a lane-private LDS slot, then runs the block's stages t = c0+len-1 .. c0 from it.  The
// earlier block's streams are requested after the re-integration, so they land while the block's
// Riccati stages compute and the prefetch registers are not live across the RK4 (128-VGPR budget).
// lds: this wavefront's CKI x 2 rows of 64 double2 (knot c0 + j in rows 2j, 2j+1), then CKI rows of 64
// tau2 controls and (unless U0Z) CKI rows of tau1 controls.
struct CkBlock {
    double2 a, b;          // checkpoint x_c0
    double u0[CKI], u1[CKI];
};

template <bool U0Z, int OUT>
__device__ __forceinline__ void backward_solver_lane_ck(const Dyn& m, const KW& w,
                                                        const double2* __restrict__ x, const double* __restrict__ u,
                                                        const double* __restrict__ xr, const double* __restrict__ ur,
                                                        double2* __restrict__ K1, double* __restrict__ cs, double g0,
                                                        double2* __restrict__ lds, int64_t l, int64_t Bp, int N,
                                                        double& dJ_out, double& smax_out) {
    const int T = N - 1;
    const uint32_t o2 = wbo(l, 2), o1 = (uint32_t)l * 8u;
    const uint32_t row = (uint32_t)Bp * 16u, plane = (uint32_t)Bp * 8u;
    const char* Xb = reinterpret_cast<const char*>(x);
    const char* Ub = reinterpret_cast<const char*>(u);
    const char* Kb = reinterpret_cast<const char*>(K1);
    const char* Cb = reinterpret_cast<const char*>(cs);
    const int ln = threadIdx.x;
    double* lu1 = reinterpret_cast<double*>(lds + 2 * CKI * BLK);   // (CKI, 64) tau2 controls
    double* lu0 = lu1 + CKI * BLK;                                   // (CKI, 64) tau1 controls (!U0Z)
    Sweep<false> S(w, x[wix(T, 0, 2, l, Bp)], x[wix(T, 1, 2, l, Bp)], xr + 4 * T);
    auto fetch = [&](CkBlock& q, int c0, int len) {
        const auto rX = rsrc(Xb + (int64_t)c0 * (2 * (int64_t)row));
        q.a = bld2(rX, o2, 0);
        q.b = bld2(rX, o2, WROW);
#pragma unroll
        for (int j = 0; j < CKI; ++j) {
            q.u0[j] = 0.0;
            q.u1[j] = 0.0;
            if (j < len) {
                const auto rU = rsrc(Ub + (int64_t)(c0 + j) * row);
                if (!U0Z) q.u0[j] = bld1(rU, o1, 0);
                q.u1[j] = bld1(rU, o1, plane);
            }
        }
    };
    const int nblk = (T + CKI - 1) / CKI;
    CkBlock q;
    {
        const int c0 = (nblk - 1) * CKI;
        fetch(q, c0, T - c0);
    }
    prio_start<0>();
    for (int bk = nblk - 1; bk >= 0; --bk) {
        const int c0 = bk * CKI;
        const int len = (T - c0 < CKI) ? T - c0 : CKI;
        prio_band<0>(T - c0 - len, T);
        // knots c0 .. c0+len-1 into LDS: the checkpoint, then the trial's x_{t+1} = RK4(x_t, u1_t); the
        // block's controls too, so that no register holds them across the stages
        {
            double n0 = q.a.x, n1 = q.a.y, n2 = q.b.x, n3 = q.b.y;
            lds[ln] = q.a;
            lds[BLK + ln] = q.b;
#pragma unroll
            for (int j = 0; j < CKI; ++j) {
                lu1[j * BLK + ln] = q.u1[j];
                if (!U0Z) lu0[j * BLK + ln] = q.u0[j];
            }
#pragma unroll
            for (int j = 0; j < CKI - 1; ++j) {
                if (j < len - 1) {
                    gym::rk4(m, n0, n1, n2, n3, q.u1[j]);
                    lds[(2 * j + 2) * BLK + ln] = make_double2(n0, n1);
                    lds[(2 * j + 3) * BLK + ln] = make_double2(n2, n3);
                }
                __builtin_amdgcn_sched_barrier(0);   // keep the unrolled steps apart (register pressure)
            }
        }
        if (bk > 0) fetch(q, c0 - CKI, CKI);   // the earlier block (always full) lands during the stages below
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int j = CKI - 1; j >= 0; --j) {
            if (j < len) {
                const int t = c0 + j;
                const double2 xa = lds[(2 * j) * BLK + ln], xb = lds[(2 * j + 1) * BLK + ln];
                const double ut1 = lu1[j * BLK + ln], ut0 = U0Z ? 0.0 : lu0[j * BLK + ln];
                double k0, k1, k2, k3, s0, s1;
                const KArgs ka = kernarg_consts();
                S.step<U0Z>(ka.m, ka.w, xa, xb, ut0, ut1, xr + 4 * t, ur + 2 * t, k0, k1, k2, k3, s0, s1);
                store_stage<OUT>(Kb, Cb, t, row, plane, o2, o1, xa, xb, ut1, g0, k0, k1, k2, k3, s1);
            }
            __builtin_amdgcn_sched_barrier(0);
        }
    }
    dJ_out = S.dJ;
    smax_out = S.smax;
}

// ------------------------------------------------------------------------------------------
// kernels: API primitives
// ------------------------------------------------------------------------------------------
__global__ __launch_bounds__(BLK) void k_backward_api(Dyn m, KW w, const double2* __restrict__ x,
                                                      const double* __restrict__ u, const double* __restrict__ xr,
                                                      const double* __restrict__ ur, double2* __restrict__ K1,
                                                      double* __restrict__ sig, double* __restrict__ dJ,
                                                      double* __restrict__ smax, double2* __restrict__ lam, int64_t B,
                                                      int64_t Bp, int N) {
    const int64_t l = (int64_t)blockIdx.x * BLK + threadIdx.x;
    if (l >= B) return;
    double d, s;
    if (lam)
        backward_lane<true>(m, w, x, u, xr, ur, K1, sig, lam, l, Bp, N, d, s);
    else
        backward_lane<false>(m, w, x, u, xr, ur, K1, sig, nullptr, l, Bp, N, d, s);
    if (dJ) dJ[l] = d;
    if (smax) smax[l] = s;
}

__global__ __launch_bounds__(BLK) void k_open_loop(Dyn m, KW w, const double* __restrict__ x0,
                                                   const double* __restrict__ u, const double* __restrict__ xr,
                                                   const double* __restrict__ ur, double2* __restrict__ xn,
                                                   double* __restrict__ cost, int64_t B, int64_t Bp, int N) {
    const int64_t l = (int64_t)blockIdx.x * BLK + threadIdx.x;
    if (l >= B) return;
    const double J = rollout_ref<false>(m, w, nullptr, u, nullptr, nullptr, xr, ur, xn, nullptr, 0.0, l, Bp, N,
                                        x0[4 * l + 0], x0[4 * l + 1], x0[4 * l + 2], x0[4 * l + 3]);
    if (cost) cost[l] = J;
}

__global__ __launch_bounds__(BLK) void k_closed_loop(Dyn m, KW w, const double2* __restrict__ x,
                                                     const double* __restrict__ u, const double2* __restrict__ Kf,
                                                     const double* __restrict__ s, const double* __restrict__ gamma,
                                                     const double* __restrict__ xr, const double* __restrict__ ur,
                                                     double2* __restrict__ xn, double* __restrict__ un,
                                                     double* __restrict__ cost, int64_t B, int64_t Bp, int N) {
    const int64_t l = (int64_t)blockIdx.x * BLK + threadIdx.x;
    if (l >= B) return;
    const double2 a = x[wix(0, 0, 2, l, Bp)], b = x[wix(0, 1, 2, l, Bp)];
    const double J = rollout_ref<true>(m, w, x, u, Kf, s, xr, ur, xn, un, gamma[l], l, Bp, N, a.x, a.y, b.x, b.y);
    if (cost) cost[l] = J;
}

__global__ void k_point(Dyn m, const double* __restrict__ x, const double* __restrict__ u,
                        double* __restrict__ out, double* __restrict__ out2, int64_t n, int what) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    double x0 = x[4 * i], x1 = x[4 * i + 1], x2 = x[4 * i + 2], x3 = x[4 * i + 3];
    const double tau2 = u[2 * i + 1];  // tau1 is not an acrobot input (dynamics.py:205, :153)
    if (what == 0) {                   // continuous_dynamics
        double q1, q2;
        gym::accel(m, x0, x1, x2, x3, tau2, q1, q2);
        out[4 * i] = x2; out[4 * i + 1] = x3; out[4 * i + 2] = q1; out[4 * i + 3] = q2;
    } else if (what == 1) {            // dynamics (RK4)
        gym::rk4(m, x0, x1, x2, x3, tau2);
        out[4 * i] = x0; out[4 * i + 1] = x1; out[4 * i + 2] = x2; out[4 * i + 3] = x3;
    } else {                           // Calculate_A_B_matrixes
        const gym::Jac J = gym::jacobian(m, x0, x1, x2, x3, tau2);
        double* A = out + 16 * i;
        double* Bc = out2 + 8 * i;
#pragma unroll
        for (int j = 0; j < 4; ++j) { A[j] = 0.0; A[4 + j] = 0.0; A[8 + j] = J.a2[j]; A[12 + j] = J.a3[j]; }
        A[2] = 1.0; A[7] = 1.0;
#pragma unroll
        for (int j = 0; j < 8; ++j) Bc[j] = 0.0;
        Bc[5] = J.bc2; Bc[7] = J.bc3;
    }
}

struct Mat4 { double v[16]; };
struct Mat2 { double v[4]; };

__device__ __forceinline__ double quad4(const double* M, const double e[4]) {
    double l = 0.0;  // (e^T M) e
#pragma unroll
    for (int c = 0; c < 4; ++c) {
        double s = 0.0;
#pragma unroll
        for (int k = 0; k < 4; ++k) s += e[k] * M[4 * k + c];
        l += s * e[c];
    }
    return l;
}

__device__ __forceinline__ double quad2(const double* M, double f0, double f1) {
    return (f0 * M[0] + f1 * M[2]) * f0 + (f0 * M[1] + f1 * M[3]) * f1;
}

__global__ void k_stage_cost_derivs(const double* __restrict__ x, const double* __restrict__ xr,
                                    const double* __restrict__ u, const double* __restrict__ ur, Mat4 Q, Mat2 R,
                                    int terminal, double* __restrict__ lo, double* __restrict__ gx,
                                    double* __restrict__ gu, int64_t n) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    double e[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) e[k] = x[4 * i + k] - xr[4 * i + k];
    double l = quad4(Q.v, e);
#pragma unroll
    for (int r = 0; r < 4; ++r) {
        double s = 0.0;
#pragma unroll
        for (int k = 0; k < 4; ++k) s += Q.v[4 * r + k] * e[k];
        gx[4 * i + r] = 2.0 * s;
    }
    if (!terminal) {
        const double f0 = u[2 * i] - ur[2 * i], f1 = u[2 * i + 1] - ur[2 * i + 1];
        l += quad2(R.v, f0, f1);
        gu[2 * i] = 2.0 * (R.v[0] * f0 + R.v[1] * f1);
        gu[2 * i + 1] = 2.0 * (R.v[2] * f0 + R.v[3] * f1);
    }
    lo[i] = l;
}

__global__ __launch_bounds__(BLK) void k_total_cost(const double2* __restrict__ x, const double* __restrict__ u,
                                                    const double* __restrict__ xr, const double* __restrict__ ur,
                                                    Mat4 Q, Mat2 R, Mat4 QT, double* __restrict__ cost, int64_t B,
                                                    int64_t Bp, int N) {
    const int64_t l = (int64_t)blockIdx.x * BLK + threadIdx.x;
    if (l >= B) return;
    double J = 0.0;
    for (int t = 0; t < N - 1; ++t) {
        const double2 a = x[wix(t, 0, 2, l, Bp)], b = x[wix(t, 1, 2, l, Bp)];
        const double e[4] = {a.x - xr[4 * t], a.y - xr[4 * t + 1], b.x - xr[4 * t + 2], b.y - xr[4 * t + 3]};
        J += quad4(Q.v, e);
        J += quad2(R.v, u[pix(t, 0, 2, l, Bp)] - ur[2 * t], u[pix(t, 1, 2, l, Bp)] - ur[2 * t + 1]);
    }
    const int T = N - 1;
    const double2 a = x[wix(T, 0, 2, l, Bp)], b = x[wix(T, 1, 2, l, Bp)];
    const double e[4] = {a.x - xr[4 * T], a.y - xr[4 * T + 1], b.x - xr[4 * T + 2], b.y - xr[4 * T + 3]};
    cost[l] = J + quad4(QT.v, e);
}

// build_stage_lists (:166-181) as plain-double SoA for the generic Riccati path
__global__ __launch_bounds__(BLK) void k_linearize(Dyn m, KW w, const double2* __restrict__ x,
                                                   const double* __restrict__ u, const double* __restrict__ xr,
                                                   const double* __restrict__ ur, double* __restrict__ Ad,
                                                   double* __restrict__ Bd, double* __restrict__ q,
                                                   double* __restrict__ r, double* __restrict__ qT, int64_t B,
                                                   int64_t Bp, int N) {
    const int64_t l = (int64_t)blockIdx.x * BLK + threadIdx.x;
    if (l >= B) return;
    const double dt = m.h;
    const int T = N - 1;
    for (int t = 0; t < T; ++t) {
        const double2 a = x[wix(t, 0, 2, l, Bp)], b = x[wix(t, 1, 2, l, Bp)];
        const double v0 = u[pix(t, 0, 2, l, Bp)], v1 = u[pix(t, 1, 2, l, Bp)];
        const gym::Jac J = gym::jacobian(m, a.x, a.y, b.x, b.y, v1);
        double A[16] = {1.0, 0.0, dt, 0.0, 0.0, 1.0, 0.0, dt};
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            A[8 + j] = (j == 2 ? 1.0 : 0.0) + dt * J.a2[j];
            A[12 + j] = (j == 3 ? 1.0 : 0.0) + dt * J.a3[j];
        }
        double Bv[8] = {0, 0, 0, 0, 0, dt * J.bc2, 0, dt * J.bc3};
#pragma unroll
        for (int c = 0; c < 16; ++c) Ad[((int64_t)t * 16 + c) * Bp + l] = A[c];
#pragma unroll
        for (int c = 0; c < 8; ++c) Bd[((int64_t)t * 8 + c) * Bp + l] = Bv[c];
        const double xe[4] = {a.x - xr[4 * t], a.y - xr[4 * t + 1], b.x - xr[4 * t + 2], b.y - xr[4 * t + 3]};
#pragma unroll
        for (int c = 0; c < 4; ++c) q[((int64_t)t * 4 + c) * Bp + l] = (2.0 * w.Q[c]) * xe[c];
        r[((int64_t)t * 2) * Bp + l] = (2.0 * w.R[0]) * (v0 - ur[2 * t]);
        r[((int64_t)t * 2 + 1) * Bp + l] = (2.0 * w.R[1]) * (v1 - ur[2 * t + 1]);
    }
    const double2 a = x[wix(T, 0, 2, l, Bp)], b = x[wix(T, 1, 2, l, Bp)];
    const double xe[4] = {a.x - xr[4 * T], a.y - xr[4 * T + 1], b.x - xr[4 * T + 2], b.y - xr[4 * T + 3]};
#pragma unroll
    for (int c = 0; c < 4; ++c) qT[(int64_t)c * Bp + l] = (2.0 * w.QT[c]) * xe[c];
}

// 2x2 solve G X = Y (X, Y 2 x ncol) by LU with partial pivoting, as LAPACK dgesv orders it.
template <int NC>
__device__ __forceinline__ void solve2(double g00, double g01, double g10, double g11, double (&y)[2][NC]) {
    if (fabs(g10) > fabs(g00)) {
        double t;
        t = g00; g00 = g10; g10 = t;
        t = g01; g01 = g11; g11 = t;
#pragma unroll
        for (int c = 0; c < NC; ++c) { t = y[0][c]; y[0][c] = y[1][c]; y[1][c] = t; }
    }
    const double l10 = g10 / g00;
    const double u11 = g11 - l10 * g01;
#pragma unroll
    for (int c = 0; c < NC; ++c) {
        const double z1 = y[1][c] - l10 * y[0][c];
        const double x1 = z1 / u11;
        y[1][c] = x1;
        y[0][c] = (y[0][c] - g01 * x1) / g00;
    }
}

// calculate_K_and_sigma (:183-216) on general dense stage data (plain-double SoA).
__global__ __launch_bounds__(BLK) void k_riccati_general(
    const double* __restrict__ A, const double* __restrict__ Bm, const double* __restrict__ Q,
    const double* __restrict__ R, const double* __restrict__ S, const double* __restrict__ q,
    const double* __restrict__ r, const double* __restrict__ QT, const double* __restrict__ qT,
    double* __restrict__ K, double* __restrict__ sigma, double* __restrict__ dJo, int64_t B, int64_t Bp, int T) {
    const int64_t l = (int64_t)blockIdx.x * BLK + threadIdx.x;
    if (l >= B) return;
    double P[16], p[4];
#pragma unroll
    for (int c = 0; c < 16; ++c) P[c] = QT[(int64_t)c * Bp + l];
#pragma unroll
    for (int c = 0; c < 4; ++c) p[c] = qT[(int64_t)c * Bp + l];
    double dJ = 0.0;
    for (int t = T - 1; t >= 0; --t) {
        double a[16], b[8];
#pragma unroll
        for (int c = 0; c < 16; ++c) a[c] = A[((int64_t)t * 16 + c) * Bp + l];
#pragma unroll
        for (int c = 0; c < 8; ++c) b[c] = Bm[((int64_t)t * 8 + c) * Bp + l];
        double PB[8], PA[16];
#pragma unroll
        for (int i = 0; i < 4; ++i) {
#pragma unroll
            for (int j = 0; j < 2; ++j) {
                double s = 0.0;
#pragma unroll
                for (int k = 0; k < 4; ++k) s += P[4 * i + k] * b[2 * k + j];
                PB[2 * i + j] = s;
            }
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                double s = 0.0;
#pragma unroll
                for (int k = 0; k < 4; ++k) s += P[4 * i + k] * a[4 * k + j];
                PA[4 * i + j] = s;
            }
        }
        double G[4], Y[2][5];
#pragma unroll
        for (int i = 0; i < 2; ++i) {
#pragma unroll
            for (int j = 0; j < 2; ++j) {
                double s = 0.0;
#pragma unroll
                for (int k = 0; k < 4; ++k) s += b[2 * k + i] * PB[2 * k + j];
                G[2 * i + j] = R[((int64_t)t * 4 + 2 * i + j) * Bp + l] + s;
            }
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                double s = 0.0;
#pragma unroll
                for (int k = 0; k < 4; ++k) s += b[2 * k + i] * PA[4 * k + j];
                Y[i][j] = S[((int64_t)t * 8 + 4 * i + j) * Bp + l] + s;   // F
            }
            double s = 0.0;
#pragma unroll
            for (int k = 0; k < 4; ++k) s += b[2 * k + i] * p[k];
            Y[i][4] = r[((int64_t)t * 2 + i) * Bp + l] + s;                // g
        }
        const double g0 = Y[0][4], g1 = Y[1][4];
        solve2<5>(G[0], G[1], G[2], G[3], Y);
        double Kt[8], st[2];
#pragma unroll
        for (int i = 0; i < 2; ++i) {
#pragma unroll
            for (int j = 0; j < 4; ++j) Kt[4 * i + j] = -Y[i][j];
            st[i] = -Y[i][4];
        }
        dJ += g0 * st[0] + g1 * st[1];
        double GK[8], Gs[2];
#pragma unroll
        for (int i = 0; i < 2; ++i) {
#pragma unroll
            for (int j = 0; j < 4; ++j) GK[4 * i + j] = G[2 * i] * Kt[j] + G[2 * i + 1] * Kt[4 + j];
            Gs[i] = G[2 * i] * st[0] + G[2 * i + 1] * st[1];
        }
        double Pn[16], pn[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) {
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                double s = 0.0;
#pragma unroll
                for (int k = 0; k < 4; ++k) s += a[4 * k + i] * PA[4 * k + j];
                Pn[4 * i + j] = Q[((int64_t)t * 16 + 4 * i + j) * Bp + l] + s - (Kt[i] * GK[j] + Kt[4 + i] * GK[4 + j]);
            }
            double s = 0.0;
#pragma unroll
            for (int k = 0; k < 4; ++k) s += a[4 * k + i] * p[k];
            pn[i] = q[((int64_t)t * 4 + i) * Bp + l] + s - (Kt[i] * Gs[0] + Kt[4 + i] * Gs[1]);
        }
#pragma unroll
        for (int c = 0; c < 16; ++c) P[c] = Pn[c];
#pragma unroll
        for (int c = 0; c < 4; ++c) p[c] = pn[c];
#pragma unroll
        for (int c = 0; c < 8; ++c) K[((int64_t)t * 8 + c) * Bp + l] = Kt[c];
        sigma[((int64_t)t * 2) * Bp + l] = st[0];
        sigma[((int64_t)t * 2 + 1) * Bp + l] = st[1];
    }
    dJo[l] = dJ;
}

// ------------------------------------------------------------------------------------------
// kernels: layout.  Lane-major (B, L, C) <-> SoA (L, C/W, Bp, W), W = 1 (planes) or 2 (pairs).
// ------------------------------------------------------------------------------------------
__global__ void k_pack(const double* __restrict__ src, double* __restrict__ dst, int64_t B, int64_t Bp, int L,
                       int C, int W) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;  // element (of W doubles) index
    const int P = C / W;
    if (i >= (int64_t)L * P * Bp) return;
    const int64_t lane = i % Bp;
    const int64_t rest = i / Bp;
    const int p = (int)(rest % P);
    const int64_t t = rest / P;
    const double* s = src + (lane * L + t) * C + W * p;
    const int64_t d = W == 2 ? wix(t, p, P, lane, Bp) : i;   // pairs: wave-blocked
    for (int k = 0; k < W; ++k) dst[W * d + k] = (lane < B) ? s[k] : 0.0;
}

// SoA -> lane-major transposes through LDS.  One workgroup (256 threads) moves the tile of one 64-lane group x
// TS knots: the SoA rows are read coalesced (a 64-lane row is 512 B or 1 KiB contiguous), the tile is staged in
// LDS as [knot][component][lane] with a 65-double row pitch (a lane's column is read conflict-free), and each
// lane's TS x C output doubles -- contiguous in the lane-major array -- are written by consecutive threads.
// Src supplies component c of knot t of a lane (which may be derived, e.g. sigma0, or a constant 0).
constexpr int TILE_PITCH = BLK + 1;
constexpr int TILE_THREADS = 256;
constexpr int TILE_DOUBLES = 4096;   // 32 KiB of LDS per workgroup (5 per CU): TS * C * TILE_PITCH <= TILE_DOUBLES
inline int tile_knots(int C) {
    int ts = TILE_DOUBLES / (C * TILE_PITCH);
    return ts < 1 ? 1 : (ts > 32 ? 32 : ts);
}

struct SrcPairs {   // wave-blocked pairs (L, P, Bp) double2, per-lane buffer select
    const double2 *s0, *s1;
    const int32_t* sel;
    int P;
    __device__ __forceinline__ double operator()(int64_t t, int c, int64_t lane, int64_t Bp) const {
        const double2* b = (sel && sel[lane]) ? s1 : s0;
        const double2 v = b[wix(t, c >> 1, P, lane, Bp)];
        return (c & 1) ? v.y : v.x;
    }
};
struct SrcPlanes {  // planes (L, C, Bp) double, per-lane buffer select
    const double *s0, *s1;
    const int32_t* sel;
    int C;
    __device__ __forceinline__ double operator()(int64_t t, int c, int64_t lane, int64_t Bp) const {
        const double* b = (sel && sel[lane]) ? s1 : s0;
        return b[(t * C + c) * Bp + lane];
    }
};
struct SrcGains {   // full K_t (2,4) from its row 1 (K1 pairs); row 0 is identically 0
    const double2* K1;
    __device__ __forceinline__ double operator()(int64_t t, int c, int64_t lane, int64_t Bp) const {
        if (c < 4) return 0.0;
        const double2 v = K1[wix(t, (c - 4) >> 1, 2, lane, Bp)];
        return (c & 1) ? v.y : v.x;
    }
};
struct SrcSigma {   // sigma of each lane's last iteration: sigma0 recomputed from that iteration's u0, sigma1 plane
    KW w;
    const double *cs, *u0b, *u1b, *ur;
    const int32_t* n_iter;
    int64_t ur_lane;   // per-lane references: doubles per lane of u_ref (0: shared)
    __device__ __forceinline__ double operator()(int64_t t, int c, int64_t lane, int64_t Bp) const {
        const int it = n_iter[lane];
        if (it <= 0) return 0.0;
        if (c == 1) return cs[pix((int)t, 1, 2, lane, Bp)];
        const double* u = ((it - 1) & 1) ? u1b : u0b;
        return -(w.G00 * (u[pix((int)t, 0, 2, lane, Bp)] - ur[lane * ur_lane + 2 * t])) * w.iG00;
    }
};

// dst (B, L, C) lane-major; grid (Bp / 64) x ceil(L / TS); dynamic LDS TS * C * TILE_PITCH doubles.
// CT: C at compile time (the solver's outputs: 2, 4, 8 -- the divisions by C become shifts and the stores 16 B
// wide), 0 = C at run time (gym_unpack_lanes' general form).
template <class Src, int CT>
__global__ __launch_bounds__(TILE_THREADS) void k_unpack_tiled(Src src, double* __restrict__ dst,
                                                               const int64_t* __restrict__ map, int64_t B,
                                                               int64_t Bp, int L, int C_rt, int TS) {
    extern __shared__ double tile[];
    __shared__ int64_t rows_of[BLK];                        // output row of each lane of the group
    const int C = CT ? CT : C_rt;
    const int64_t g0 = (int64_t)blockIdx.x * BLK;          // first lane of the group
    const int t0 = (int)blockIdx.y * TS;
    const int ts = (L - t0 < TS) ? L - t0 : TS;
    const int rows = ts * C;
    if (threadIdx.x < BLK) {
        const int64_t l = g0 + threadIdx.x;
        rows_of[threadIdx.x] = map ? (l < B ? map[l] : 0) : l;
    }
    for (int i = threadIdx.x; i < rows * BLK; i += TILE_THREADS) {
        const int ln = i & (BLK - 1), r = i >> 6;          // r = knot * C + component
        tile[r * TILE_PITCH + ln] = src(t0 + r / C, r % C, g0 + ln, Bp);
    }
    __syncthreads();
    const int64_t nl = (B - g0 < BLK) ? B - g0 : BLK;      // real lanes of the group
    if (CT > 0 && CT % 2 == 0) {   // component pairs: 16-byte stores
        const int half = rows / 2;
        double2* d2 = reinterpret_cast<double2*>(dst);
        for (int i = threadIdx.x; i < nl * half; i += TILE_THREADS) {
            const int ln = i / half, r2 = i - ln * half;
            d2[((rows_of[ln] * L + t0) * C) / 2 + r2] =
                make_double2(tile[(2 * r2) * TILE_PITCH + ln], tile[(2 * r2 + 1) * TILE_PITCH + ln]);
        }
    } else {
        for (int i = threadIdx.x; i < nl * rows; i += TILE_THREADS) {
            const int ln = i / rows, r = i - ln * rows;
            dst[(rows_of[ln] * L + t0) * C + r] = tile[r * TILE_PITCH + ln];
        }
    }
}

// ------------------------------------------------------------------------------------------
// kernels: batched Newton / Armijo solver (newton_Algorithm :298-398)
// ------------------------------------------------------------------------------------------
template <bool RL = false>
__global__ __launch_bounds__(BLK) void k_init(Dyn m, KW w, const double* __restrict__ x0,
                                              const double* __restrict__ u, const double* __restrict__ xr,
                                              const double* __restrict__ ur, double2* __restrict__ xn,
                                              double* __restrict__ cost, int32_t* __restrict__ status,
                                              int32_t* __restrict__ n_iter, int32_t* __restrict__ res_buf,
                                              int32_t* __restrict__ n_roll, double* __restrict__ gamma,
                                              double* __restrict__ smax, double* __restrict__ dJ, int64_t B,
                                              int64_t Bp, int N) {
    const int64_t l = (int64_t)blockIdx.x * BLK + threadIdx.x;
    if (l >= Bp) return;
    n_iter[l] = 0; res_buf[l] = 0; n_roll[l] = 0; gamma[l] = 0.0; smax[l] = 0.0; dJ[l] = 0.0;
    if (l >= B) {
        status[l] = GYM_PAD;
        cost[l] = 0.0;
        return;
    }
    status[l] = GYM_ACTIVE;
    cost[l] = rollout_ref<false>(m, w, nullptr, u, nullptr, nullptr, lane_ref<RL>(xr, l, 4 * (int64_t)N),
                                 lane_ref<RL>(ur, l, 2 * (int64_t)(N - 1)), xn, nullptr, 0.0, l, Bp, N,
                                 x0[4 * l + 0], x0[4 * l + 1], x0[4 * l + 2], x0[4 * l + 3]);
}

// Diagnostic build only (-DGYM_WAVE_TRACE, tools/wave_trace.py): per-wavefront start/end time and
// hardware placement of the serial schedule's sweep (kind 0) and trial (kind 1) launches.
#ifdef GYM_WAVE_TRACE
__device__ unsigned long long g_wave_trace[2][8192][4];
struct WaveTrace {
    int kind;
    unsigned long long t0;
    __device__ explicit WaveTrace(int k) : kind(k), t0(__builtin_amdgcn_s_memrealtime()) {}
    __device__ ~WaveTrace() {
        if (threadIdx.x == 0 && blockIdx.x < 8192) {
            unsigned long long* r = g_wave_trace[kind][blockIdx.x];
            r[0] = t0;
            r[1] = __builtin_amdgcn_s_memrealtime();
            r[2] = (unsigned)__builtin_amdgcn_s_getreg((31 << 11) | 4);    // HW_REG_HW_ID
            r[3] = (unsigned)__builtin_amdgcn_s_getreg((31 << 11) | 20);   // HW_REG_XCC_ID
        }
    }
};
#define GYM_TRACE_WAVE(k) WaveTrace wave_trace_(k)
#else
#define GYM_TRACE_WAVE(k)
#endif

// lane-private LDS of the checkpointed sweep: CKI knots x 2 pairs + CKI controls (tau2; and tau1 unless
// U0Z) x 64 lanes: 10 KiB per wave with U0Z, so 16 waves fill one CU's 160 KiB exactly.
constexpr int ck_lds_doubles(bool ck, bool u0z) { return ck ? (4 + (u0z ? 1 : 2)) * CKI * BLK : 2; }
#define GYM_CK_LDS(CK, U0Z) __shared__ double2 ck_lds[ck_lds_doubles(CK, U0Z) / 2]

// Lane ranges: the serial schedule runs every lane [0, B); the pipelined schedule splits the batch
// into two halves H0 = [0, Bh), H1 = [Bh, B) whose iterations are offset by one phase.
struct Range {
    int64_t lo, hi;
};

template <bool U0Z, bool CK, int OUT = OUT_SOLVER>
__device__ __forceinline__ void backward_solver(const Dyn& m, const KW& w, const double2* __restrict__ x,
                                                const double* __restrict__ u, const double* __restrict__ xr,
                                                const double* __restrict__ ur, double2* __restrict__ K1,
                                                double* __restrict__ cs, double g0, double* __restrict__ dJ,
                                                double* __restrict__ smax, double* __restrict__ hist_smax, int64_t l,
                                                int64_t Bp, int N, int k, int hist_len, double2* __restrict__ lds) {
    double d, s;
    if (CK)
        backward_solver_lane_ck<U0Z, OUT>(m, w, x, u, xr, ur, K1, cs, g0, lds, l, Bp, N, d, s);
    else
        backward_solver_lane<U0Z, OUT>(m, w, x, u, xr, ur, K1, cs, g0, l, Bp, N, d, s);
    if (OUT == OUT_SIGMA) return;   // a re-run: the lane's dJ / smax are those of the original sweep
    dJ[l] = d;
    smax[l] = s;
    if (hist_smax && k < hist_len) hist_smax[(int64_t)k * Bp + l] = s;
}

#define GYM_NT_BACKWARD_PARAMS                                                                                  \
    Dyn m, KW w, const double2 *__restrict__ x, const double *__restrict__ u, const double *__restrict__ xr,   \
        const double *__restrict__ ur, double2 *__restrict__ K1, double *__restrict__ cs, double g0,           \
        double *__restrict__ dJ, double *__restrict__ smax, const int32_t *__restrict__ status,               \
        double *__restrict__ hist_smax, Range rg, int64_t Bp, int N, int k, int hist_len
#define GYM_NT_BACKWARD_BODY(OUT)                                                                               \
    GYM_TRACE_WAVE(0);                                                                                          \
    const int64_t l = rg.lo + (int64_t)blockIdx.x * BLK + threadIdx.x;                                          \
    GYM_CK_LDS(CK, U0Z);                                                                                        \
    if (l >= rg.hi || status[l] != GYM_ACTIVE) return;                                                          \
    backward_solver<U0Z, CK, OUT>(m, w, x, u, lane_ref<RL>(xr, l, 4 * (int64_t)N),                               \
                                  lane_ref<RL>(ur, l, 2 * (int64_t)(N - 1)), K1, cs, g0, dJ, smax, hist_smax, l, Bp, \
                                  N, k, hist_len, ck_lds);

// the solver's serial-schedule sweep (K1, cg) ...
template <bool U0Z, bool CK, bool RL = false>
__global__ __launch_bounds__(BLK, 4) void k_nt_backward(GYM_NT_BACKWARD_PARAMS) { GYM_NT_BACKWARD_BODY(OUT_SOLVER) }
// ... and the same sweep also storing sigma1, for the gamma sweeps of gym_newton_gamma_sweep
template <bool U0Z, bool CK, bool RL = false>
__global__ __launch_bounds__(BLK, 4) void k_nt_backward_all(GYM_NT_BACKWARD_PARAMS) { GYM_NT_BACKWARD_BODY(OUT_ALL) }

struct SolverCtl {
    double tol, beta, c, gamma0;
    int max_ls, k, hist_len, pad;
};

__device__ __forceinline__ void accept_lane(const SolverCtl& a, int64_t l, double Jn, double g, double smax,
                                            double* cost, double* gamma, int32_t* status, int32_t* res_buf,
                                            double* hist_cost, int64_t Bp) {
    cost[l] = Jn;
    gamma[l] = g;
    if (smax < a.tol) {  // convergence is tested after the update (:383-396)
        status[l] = GYM_CONVERGED;
        res_buf[l] = (a.k + 1) & 1;
    }
    if (hist_cost && a.k < a.hist_len) hist_cost[(int64_t)a.k * Bp + l] = Jn;
}

__device__ __forceinline__ void fail_lane(const SolverCtl& a, int64_t l, int32_t* status, int32_t* res_buf) {
    status[l] = GYM_LS_FAILED;  // no update (:367-369): the result is the current trajectory
    res_buf[l] = a.k & 1;
}

// The per-lane state and streams one Armijo trial touches.
struct TrialIO {
    const double2* x;   // current trajectory (only x_0 is read)
    const double* u;    // current control planes (u0 is read)
    double2* xn;        // candidate trajectory (written)
    double* un;         // candidate controls (written)
};

// Armijo trial 1 (gamma0) fused with the candidate rollout and its cost (:352-365, first pass).
template <bool U0Z, bool CK>
__device__ __forceinline__ void trial_solver(const Dyn& m, const KW& w, const SolverCtl& a, const TrialIO& io,
                                             const double2* __restrict__ K1, const double* __restrict__ cs,
                                             const double* __restrict__ xr, const double* __restrict__ ur,
                                             double* __restrict__ cost, const double* __restrict__ dJ,
                                             const double* __restrict__ smax, double* __restrict__ gamma,
                                             int32_t* __restrict__ status, int32_t* __restrict__ n_iter,
                                             int32_t* __restrict__ res_buf, int32_t* __restrict__ n_roll,
                                             int32_t* __restrict__ retry_list, int32_t* __restrict__ counter,
                                             double* __restrict__ hist_cost, int64_t l, int64_t Bp, int N) {
    const double2 xa = io.x[wix(0, 0, 2, l, Bp)], xb = io.x[wix(0, 1, 2, l, Bp)];
    const double g = a.gamma0;
    const double Jn = rollout_cform<true, U0Z, false, CK>(m, w, io.u, K1, cs, xr, ur, io.xn, io.un, g, g, l, Bp, N,
                                                          xa.x, xa.y, xb.x, xb.y);
    n_roll[l] += 1;
    if (Jn < cost[l] + a.c * g * dJ[l]) {  // strict Armijo test (:361)
        n_iter[l] += 1;
        accept_lane(a, l, Jn, g, smax[l], cost, gamma, status, res_buf, hist_cost, Bp);
    } else if (a.max_ls > 1) {
        retry_list[atomicAdd(counter, 1)] = (int32_t)l;
    } else {
        n_iter[l] += 1;
        fail_lane(a, l, status, res_buf);
    }
}

template <bool U0Z, bool CK, bool RL = false>
__global__ __launch_bounds__(BLK, 4) void k_nt_trial(Dyn m, KW w, SolverCtl a, TrialIO io,
                                                     const double2* __restrict__ K1, const double* __restrict__ cs,
                                                     const double* __restrict__ xr, const double* __restrict__ ur,
                                                     double* __restrict__ cost, const double* __restrict__ dJ,
                                                     const double* __restrict__ smax, double* __restrict__ gamma,
                                                     int32_t* __restrict__ status, int32_t* __restrict__ n_iter,
                                                     int32_t* __restrict__ res_buf, int32_t* __restrict__ n_roll,
                                                     int32_t* __restrict__ retry_list, int32_t* __restrict__ counter,
                                                     double* __restrict__ hist_cost, Range rg, int64_t Bp, int N) {
    const int64_t l = rg.lo + (int64_t)blockIdx.x * BLK + threadIdx.x;
    if (l >= rg.hi || status[l] != GYM_ACTIVE) return;
    GYM_TRACE_WAVE(1);
    trial_solver<U0Z, CK>(m, w, a, io, K1, cs, lane_ref<RL>(xr, l, 4 * (int64_t)N), lane_ref<RL>(ur, l, 2 * (int64_t)(N - 1)),
                          cost, dJ, smax, gamma, status, n_iter, res_buf, n_roll,
                      retry_list + rg.lo, counter, hist_cost, l, Bp, N);
}

// One pipeline phase: the first nb_b workgroups run the backward sweep of one half, the rest run the
// Armijo trial of the other half.  The sweep is HBM-bound and the trial fp64-VALU-bound, so co-resident
// waves of the two kinds overlap memory and arithmetic on every CU.  The two halves' lanes are disjoint.
// Every operand is in one by-value argument struct, re-read from the kernel-argument segment at each use
// (phase_args(), as the persistent kernel's run_args()): no pointer or control value is held in SGPRs across
// the stage loops, where their spills cost v_readlane VALU slots (13 per trial stage before; 1 now;
// same-box A/B +0.3%).
struct PhaseArgs {
    Dyn m;
    KW w;
    SolverCtl a;
    TrialIO io;
    const double2* xb_in;
    const double* ub_in;
    double2* K1;
    double* cs;
    const double* xr;
    const double* ur;
    double *cost, *dJ, *smax, *gamma;
    int32_t *status, *n_iter, *res_buf, *n_roll, *retry_list, *counter;
    double *hist_cost, *hist_smax;
    Range rb, rt;
    int64_t Bp;
    int32_t N, kb, nb_b, pad;
};
static_assert(offsetof(PhaseArgs, w) == 96, "kernarg layout: KW at byte 96 (kernarg_consts)");
typedef const PhaseArgs* pargs_t;
__device__ __forceinline__ pargs_t phase_args() {
    const __attribute__((address_space(4))) PhaseArgs* p =
        (const __attribute__((address_space(4))) PhaseArgs*)__builtin_amdgcn_kernarg_segment_ptr();
    asm volatile("" : "+s"(p));
    return (pargs_t)p;
}

// LO: the phase for at most two wavefronts per SIMD (gym_newton_phase's choice by the launch's size), compiled for
// two (up to 256 VGPRs) with both stage loops prefetching two stages ahead (three stream sets in rotation): with
// half the headline's waves a stage's loads must be issued further ahead to keep as many bytes in flight.  The same
// arithmetic in the same order (the same bits; tests/test_gpu_workloads.py).  Not with CK.
template <bool U0Z, bool CK, bool RL = false, bool LO = false>
__global__ __launch_bounds__(BLK, LO ? 2 : 4) void k_nt_phase(PhaseArgs args) {
    constexpr int PD = LO && !CK ? 2 : 1;
    GYM_CK_LDS(CK, U0Z);
    if ((int)blockIdx.x < args.nb_b) {
        const int64_t l = args.rb.lo + (int64_t)blockIdx.x * BLK + threadIdx.x;
        if (l >= args.rb.hi || args.status[l] != GYM_ACTIVE) return;
        double d, s;
        {
            const pargs_t R = phase_args();
            const double* xr = lane_ref<RL>(R->xr, l, 4 * (int64_t)R->N);
            const double* ur = lane_ref<RL>(R->ur, l, 2 * (int64_t)(R->N - 1));
            if (CK)
                backward_solver_lane_ck<U0Z, OUT_SOLVER>(R->m, R->w, R->xb_in, R->ub_in, xr, ur, R->K1, R->cs,
                                                         R->a.gamma0, ck_lds, l, R->Bp, R->N, d, s);
            else
                backward_solver_lane<U0Z, OUT_SOLVER, true, PD>(R->m, R->w, R->xb_in, R->ub_in, xr, ur, R->K1,
                                                                R->cs, R->a.gamma0, l, R->Bp, R->N, d, s);
        }
        const pargs_t Q = phase_args();
        Q->dJ[l] = d;
        Q->smax[l] = s;
        if (Q->hist_smax && Q->kb < Q->a.hist_len) Q->hist_smax[(int64_t)Q->kb * Q->Bp + l] = s;
    } else {
        const int64_t l = args.rt.lo + (int64_t)(blockIdx.x - args.nb_b) * BLK + threadIdx.x;
        if (l >= args.rt.hi || args.status[l] != GYM_ACTIVE) return;
        double Jn;
        {   // Armijo trial 1 (gamma0) fused with the candidate rollout and its cost (:352-365, first pass)
            const pargs_t R = phase_args();
            const double2 xa = R->io.x[wix(0, 0, 2, l, R->Bp)], xb = R->io.x[wix(0, 1, 2, l, R->Bp)];
            Jn = rollout_cform<true, U0Z, false, CK, kNT, true, PD>(
                R->m, R->w, R->io.u, R->K1, R->cs, lane_ref<RL>(R->xr, l, 4 * (int64_t)R->N),
                lane_ref<RL>(R->ur, l, 2 * (int64_t)(R->N - 1)), R->io.xn, R->io.un, R->a.gamma0, R->a.gamma0, l,
                R->Bp, R->N, xa.x, xa.y, xb.x, xb.y);
        }
        const pargs_t R = phase_args();
        const SolverCtl a = R->a;
        const double g = a.gamma0;
        R->n_roll[l] += 1;
        if (Jn < R->cost[l] + a.c * g * R->dJ[l]) {  // strict Armijo test (:361)
            R->n_iter[l] += 1;
            accept_lane(a, l, Jn, g, R->smax[l], R->cost, R->gamma, R->status, R->res_buf, R->hist_cost, R->Bp);
        } else if (a.max_ls > 1) {
            R->retry_list[R->rt.lo + atomicAdd(R->counter, 1)] = (int32_t)l;
        } else {
            R->n_iter[l] += 1;
            fail_lane(a, l, R->status, R->res_buf);
        }
    }
}

// Armijo trials 2..max_ls evaluated in parallel: one thread per (lane, j), cost only.
template <bool U0Z, bool RL = false>
__global__ __launch_bounds__(BLK) void k_nt_candidates(Dyn m, KW w, SolverCtl a, TrialIO io,
                                                       const double2* __restrict__ K1, const double* __restrict__ cs,
                                                       const double* __restrict__ xr, const double* __restrict__ ur,
                                                       const double* __restrict__ cost, const double* __restrict__ dJ,
                                                       const int32_t* __restrict__ retry_list,
                                                       const int32_t* __restrict__ counter,
                                                       uint8_t* __restrict__ cand_ok, int64_t Bp, int N) {
    const int nj = a.max_ls - 1;
    const int64_t total = (int64_t)(*counter) * nj;
    for (int64_t i = (int64_t)blockIdx.x * BLK + threadIdx.x; i < total; i += (int64_t)gridDim.x * BLK) {
        const int64_t r = i / nj;
        const int j = 1 + (int)(i % nj);
        const int64_t l = retry_list[r];
        double g = a.gamma0;
        for (int q = 0; q < j; ++q) g *= a.beta;  // gamma_i *= beta, sequentially (:365)
        const double2 xa = io.x[wix(0, 0, 2, l, Bp)], xb = io.x[wix(0, 1, 2, l, Bp)];
        const double Jn = rollout_cform<false, U0Z, true>(m, w, io.u, K1, cs, lane_ref<RL>(xr, l, 4 * (int64_t)N),
                                                          lane_ref<RL>(ur, l, 2 * (int64_t)(N - 1)), nullptr, nullptr,
                                                          g, a.gamma0, l, Bp, N, xa.x, xa.y, xb.x, xb.y);
        cand_ok[(int64_t)j * Bp + l] = (Jn < cost[l] + a.c * g * dJ[l]) ? 1 : 0;
    }
}

// Candidate scratch (gym_batch.cand_scratch, ABI 13): slot v holds candidate v's trajectory x (N, V/64, 2, 64) double2,
// controls u (T, 2, V) planes and cost J (V); V = 0: no scratch (every accepted candidate is re-run).
struct CandScratch {
    double2* sx;
    double* su;
    double* sJ;
    int64_t V;
};

// Armijo trials 2..max_ls on lane PAIRS: candidate i = r (max_ls - 1) + j - 1 (retry-list entry r, step gamma0 beta^j)
// on lanes (2q, 2q + 1) of a wavefront, the offset-form feedback and gym::rk4_pair_fast -- the chain of
// k_nt_candidates' single-lane rollout_cform<false, U0Z, true> with the joint-angle trigonometry split over the pair
// (the same operations, the same bits).  Candidate i's trajectory, controls and cost also go to scratch slot i while
// i < V, so that k_nt_retry copies the accepted one instead of re-running its chain.  The candidates of a launch
// are few lanes' (most iterations of a hard solve have 0-30 lanes backtracking), so each launch is one chain long:
// this halves the post-trial chains (candidates, then a copy instead of a second chain).  Stress workload, same
// process (tools/cand_ab.py, profiles/r04/cand/): +6.3% against re-running the accepted candidate; the candidates
// launch 42.5 ms per 193 sampled launches on pairs with the stores, 47.5 on single lanes with the stores, 39.1 for the
// former single-lane cost-only chain.
template <bool U0Z, bool RL = false>
__global__ __launch_bounds__(BLK) void k_nt_cand_pair(Dyn m, KW w, SolverCtl a, TrialIO io,
                                                      const double2* __restrict__ K1, const double* __restrict__ cs,
                                                      const double* __restrict__ xr, const double* __restrict__ ur,
                                                      const double* __restrict__ cost, const double* __restrict__ dJ,
                                                      const int32_t* __restrict__ retry_list,
                                                      const int32_t* __restrict__ counter,
                                                      uint8_t* __restrict__ cand_ok, CandScratch sc, int64_t Bp, int N) {
    const int nj = a.max_ls - 1;
    const int64_t total = (int64_t)(*counter) * nj;
    const int T = N - 1;
    const bool odd = threadIdx.x & 1;
    const uint32_t srow = (uint32_t)sc.V * 16u, splane = (uint32_t)sc.V * 8u;
    const uint32_t row = (uint32_t)Bp * 16u, plane = (uint32_t)Bp * 8u;
    const char* Kb = reinterpret_cast<const char*>(K1);
    const char* Cb = reinterpret_cast<const char*>(cs);
    const char* Ub = reinterpret_cast<const char*>(io.u);
    const char* Xs = reinterpret_cast<const char*>(sc.sx);
    const char* Us = reinterpret_cast<const char*>(sc.su);
    const gym::PolyRegs pk = gym::poly_vgprs_all();
    Dyn dm = m;
    gym::in_vgpr(dm.b); gym::in_vgpr(dm.d); gym::in_vgpr(dm.a2b); gym::in_vgpr(dm.bb); gym::in_vgpr(dm.dad);
    gym::in_vgpr(dm.g1); gym::in_vgpr(dm.g2); gym::in_vgpr(dm.f1); gym::in_vgpr(dm.f2); gym::in_vgpr(dm.h);
    gym::in_vgpr(dm.h2); gym::in_vgpr(dm.h6);
    // wave-uniform trip count: every lane of the wavefront runs the pair step (DPP partners, its ballot)
    for (int64_t base = (int64_t)blockIdx.x * (BLK / 2); base < total; base += (int64_t)gridDim.x * (BLK / 2)) {
        const int64_t i0 = base + (threadIdx.x >> 1);
        const bool act = i0 < total;
        const int64_t i = act ? i0 : total - 1;          // a padding pair repeats the last candidate, unrecorded
        const int64_t r = i / nj;
        const int j = 1 + (int)(i % nj);
        const int64_t l = retry_list[r];
        double g = a.gamma0;
        for (int q = 0; q < j; ++q) g *= a.beta;         // gamma_i *= beta, sequentially (:365)
        const double dg = g - a.gamma0;
        // this candidate's trajectory into slot i: the even lane stores (th1, th2) and the controls, the odd lane
        // (w1, w2).  A store that must not land gets an offset past the buffer resource's range, which the
        // hardware drops -- no branch around the stores, so the loop's wait counts stay exact (a store under a
        // divergent branch would make the compiler wait for every store before the next stage's operands).
        const bool keep = act && i < sc.V;
        constexpr uint32_t OOB = 0x80000000u;            // > the resources' num_records (0x7fffffff)
        const uint32_t o2 = wbo(l, 2), o1 = (uint32_t)l * 8u;
        const uint32_t v2 = keep ? wbo(i, 2) + (odd ? WROW : 0u) : OOB;
        const uint32_t v1o = keep && !odd ? (uint32_t)i * 8u : OOB;
        const double* xrl = lane_ref<RL>(xr, l, 4 * (int64_t)N);
        const double* url = lane_ref<RL>(ur, l, 2 * (int64_t)T);
        const double2 xa = io.x[wix(0, 0, 2, l, Bp)], xb = io.x[wix(0, 1, 2, l, Bp)];
        double n0 = xa.x, n1 = xa.y, n2 = xb.x, n3 = xb.y;
        bst2(rsrc(Xs), v2, 0, odd ? n2 : n0, odd ? n3 : n1);
        auto fetch = [&](TrialStage& q, int t) {
            const auto rK = rsrc(Kb + (int64_t)t * (2 * (int64_t)row));
            q.k0 = bld2(rK, o2, 0);
            q.k1 = bld2(rK, o2, WROW);
            const auto rC = rsrc(Cb + (int64_t)t * row);
            q.cg = bld1(rC, o1, 0);
            q.s1 = bld1(rC, o1, plane);
            q.u0 = U0Z ? 0.0 : bld1(rsrc(Ub + (int64_t)t * row), o1, 0);
        };
        const double G00 = w.G00, iG00 = w.iG00;
        double J = 0.0;
        TrialStage pre;
        fetch(pre, 0);
        for (int t = 0; t < T; ++t) {
            const TrialStage q = pre;
            if (t + 1 < T) fetch(pre, t + 1);
            const double* urt = url + 2 * t;
            const double v0 = U0Z ? 0.0 : trial_u0(q.u0, urt[0], g, G00, iG00);   // U0Z: +0 exactly
            const double v1 = trial_u1_sig(q.k0, q.k1, q.cg, q.s1, dg, n0, n1, n2, n3);
            const double f0 = U0Z ? 0.0 : v0 - urt[0], f1 = v1 - urt[1];
            J = stage_cost<U0Z>(J, w.Q, w.R, n0, n1, n2, n3, xrl + 4 * t, f0, f1);
            {
                const auto rO = rsrc(Us + (int64_t)t * srow);
                if (!U0Z) bst1(rO, v1o, 0, v0);
                bst1(rO, v1o, splane, v1);
            }
            gym::rk4_pair_fast<true>(dm, odd, n0, n1, n2, n3, v1, pk);
            bst2(rsrc(Xs + (int64_t)(t + 1) * (2 * (int64_t)srow)), v2, 0, odd ? n2 : n0, odd ? n3 : n1);
        }
        const double Jn = J + xcost(w.QT, n0, n1, n2, n3, xrl + 4 * T);
        if (act && !odd) {
            cand_ok[(int64_t)j * Bp + l] = (Jn < cost[l] + a.c * g * dJ[l]) ? 1 : 0;
            if (keep) sc.sJ[i] = Jn;
        }
    }
}

// First accepted candidate per retry lane: its trajectory into the lane's next iterate (io.xn / io.un), the lane
// updated.  Work items: first one head item per retry-list entry r (its bookkeeping; without a scratch slot for its
// accepted candidate -- V = 0, or a slot index past V -- the re-run of that candidate writing the trajectory, its
// rollout_cform: the same bits as the copy), then, with scratch, one copy item per entry and knot chunk (CPK knots).
// Head items on consecutive threads: the re-runs of a launch with more backtracking lanes than slots run side by
// side, one chain each (with the copy items interleaved, a thread could draw several: stress trace, launches of
// up to 2.2 ms).
constexpr int CPK = 8;   // knots per copy item
template <bool U0Z, bool CK, bool RL = false>
__global__ __launch_bounds__(BLK) void k_nt_retry(Dyn m, KW w, SolverCtl a, TrialIO io,
                                                  const double2* __restrict__ K1, const double* __restrict__ cs,
                                                  const double* __restrict__ xr, const double* __restrict__ ur,
                                                  double* __restrict__ cost, const double* __restrict__ smax,
                                                  double* __restrict__ gamma, int32_t* __restrict__ status,
                                                  int32_t* __restrict__ n_iter, int32_t* __restrict__ res_buf,
                                                  int32_t* __restrict__ n_roll, const int32_t* __restrict__ retry_list,
                                                  const int32_t* __restrict__ counter,
                                                  const uint8_t* __restrict__ cand_ok, double* __restrict__ hist_cost,
                                                  CandScratch sc, int64_t Bp, int N) {
    const int nr = *counter;
    const int nj = a.max_ls - 1;
    const int T = N - 1;
    const int nc = sc.V > 0 ? (N + CPK - 1) / CPK : 0;   // copy items per retry lane
    const int64_t total = (int64_t)nr * (1 + nc);
    for (int64_t it = (int64_t)blockIdx.x * BLK + threadIdx.x; it < total; it += (int64_t)gridDim.x * BLK) {
        const bool head = it < nr;
        const int64_t ri = head ? it : (it - nr) / nc;
        const int c = head ? 0 : (int)((it - nr) % nc);
        const int64_t l = retry_list[ri];
        int jacc = 0;                                    // the first accepted candidate (0: none)
        for (int j0 = 1; j0 <= nj && jacc == 0; j0 += 8) {   // eight independent byte loads per round
            uint8_t ok[8];
#pragma unroll
            for (int q = 0; q < 8; ++q) ok[q] = j0 + q <= nj ? cand_ok[(int64_t)(j0 + q) * Bp + l] : 0;
#pragma unroll
            for (int q = 7; q >= 0; --q)
                if (ok[q]) jacc = j0 + q;
        }
        const int64_t v = ri * nj + jacc - 1;
        const bool copy = jacc > 0 && v < sc.V;
        if (!head) {
            if (copy) {
#pragma unroll
                for (int q = 0; q < CPK; ++q) {
                    const int t = c * CPK + q;
                    if (t < N) {
                        io.xn[wix(t, 0, 2, l, Bp)] = sc.sx[wix(t, 0, 2, v, sc.V)];
                        io.xn[wix(t, 1, 2, l, Bp)] = sc.sx[wix(t, 1, 2, v, sc.V)];
                    }
                    if (t < T) {
                        if (!U0Z) io.un[pix(t, 0, 2, l, Bp)] = sc.su[pix(t, 0, 2, v, sc.V)];
                        io.un[pix(t, 1, 2, l, Bp)] = sc.su[pix(t, 1, 2, v, sc.V)];
                    }
                }
            }
            continue;
        }
        n_iter[l] += 1;
        if (jacc == 0) {
            n_roll[l] += nj;
            fail_lane(a, l, status, res_buf);
            continue;
        }
        n_roll[l] += jacc;
        double g = a.gamma0;
        for (int q = 0; q < jacc; ++q) g *= a.beta;
        double Jn;
        if (copy) {
            Jn = sc.sJ[v];
        } else {
            const double2 xa = io.x[wix(0, 0, 2, l, Bp)], xb = io.x[wix(0, 1, 2, l, Bp)];
            Jn = rollout_cform<true, U0Z, true, CK>(m, w, io.u, K1, cs, lane_ref<RL>(xr, l, 4 * (int64_t)N),
                                                    lane_ref<RL>(ur, l, 2 * (int64_t)(N - 1)), io.xn, io.un, g,
                                                    a.gamma0, l, Bp, N, xa.x, xa.y, xb.x, xb.y);
        }
        accept_lane(a, l, Jn, g, smax[l], cost, gamma, status, res_buf, hist_cost, Bp);
    }
}

// ------------------------------------------------------------------------------------------
// Persistent schedule (gym_newton_run): every lane runs its own outer iterations k0 .. k1-1 of
// newton_Algorithm (:329-396) back to back inside ONE launch -- sweep, Armijo trial 1, and only for a lane
// that rejects it the sigma1 re-run and trials 2..max_ls one after another (:352-365), exactly the
// sequential search of the reference.  Lanes are independent problems, so nothing orders one lane's
// iteration against another's: the only dependences are the lane's own stores -> loads through K1 / cs
// (sweep -> trial) and x / u (trial -> next sweep), ordered by a fence per pass.  The waves of a SIMD drift
// apart and mix sweep (HBM-heavy) and trial (fp64-heavy) passes by themselves, with no launch boundary, tail
// or host round trip per iteration.  Per lane the arithmetic is the other schedules' (same device functions):
// bit-identical results.  No wave priority bands (measured: the phase kernels' per-pass bands 4-8% slower here,
// each pass restarting at priority 3 undoes them; cyclic bands of the iteration count no faster than none).
// The kernel serves batches of at most 128 lanes per CU (the solver's default: 64), i.e. at most one wavefront per
// SIMD, so it is compiled for one (__launch_bounds__(BLK, 1)), and its sweep interleaves stage t-1's Jacobian with
// stage t's Riccati update (backward_solver_lane_ilp).
// ------------------------------------------------------------------------------------------
// Everything the kernel needs beyond the stage loops' own operands is one by-value struct whose fields are
// re-read from the kernel-argument segment at each use (run_args(): scalar loads behind an opaque pointer),
// so that none of its ~20 pointers is held in SGPRs across the stage loops (spilled, they cost v_readlane
// VALU slots in every stage).  Dyn and KW come first: kernarg_consts() reads them at offsets 0 and 96.
struct RunArgs {
    Dyn m;
    KW w;
    SolverCtl a;
    double2* x[2];
    double* u[2];
    double2* K1;
    double* cs;
    const double* xr;
    const double* ur;
    double *cost, *dJ, *smax, *gamma;
    int32_t *status, *n_iter, *res_buf, *n_roll;
    double *hist_cost, *hist_smax;
    int32_t *retry_list, *counter;   // ext: the lanes that reject trial 1 (GYM_FLAG_SIGMA_STREAM)
    int64_t B, Bp;
    int32_t N, k0, k1, ext;
};
static_assert(offsetof(RunArgs, w) == 96, "kernarg layout: KW at byte 96 (kernarg_consts)");
typedef const RunArgs* rargs_t;   // generic pointer into the kernarg segment (inferred back to scalar loads)
__device__ __forceinline__ rargs_t run_args() {
    const __attribute__((address_space(4))) RunArgs* p =
        (const __attribute__((address_space(4))) RunArgs*)__builtin_amdgcn_kernarg_segment_ptr();
    asm volatile("" : "+s"(p));
    return (rargs_t)p;
}

// the lane's reference rows in the persistent kernels (per-lane references: GYM_FLAG_REF_LANE)
template <bool RL>
__device__ __forceinline__ const double* run_xr(rargs_t R, int64_t l) {
    return lane_ref<RL>(R->xr, l, 4 * (int64_t)R->N);
}
template <bool RL>
__device__ __forceinline__ const double* run_ur(rargs_t R, int64_t l) {
    return lane_ref<RL>(R->ur, l, 2 * (int64_t)(R->N - 1));
}

__device__ __forceinline__ void lane_fence() {   // this lane's stores visible to its own later loads
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "agent");
}

#ifdef GYM_RUN2_TRACE
// Diagnostic build only (tools/run2_trace.py): per workgroup and wavefront role, cycles (s_memtime) spent in the
// sweep, the trial and the post-trial part, accumulated in registers and written once at the kernel's end.
__device__ unsigned long long g_run2_trace[8192][2][6];
#endif
#if defined(GYM_RUN2_TRACE) || defined(GYM_TAIL_TRACE)
#define R2T_NOW() __builtin_amdgcn_s_memtime()
#else
#define R2T_NOW() 0ull
#endif
template <bool U0Z, bool RL>
__global__ __launch_bounds__(BLK, 1) void k_nt_run(RunArgs args) {
    constexpr bool BAND = false;
    const int64_t l = (int64_t)blockIdx.x * BLK + threadIdx.x;
    if (l >= args.B) return;
    // Nothing but the lane index, the iteration counter and the lane's status stays live across a pass: J, dJ,
    // max|sigma| and x_0 are re-read from memory where needed (once per iteration).
    int st = run_args()->status[l];
    unsigned long long acc[4] = {0, 0, 0, 0};   // GYM_RUN2_TRACE only: sweep / trial / post cycles, iterations
    for (int k = run_args()->k0; st == GYM_ACTIVE && k < run_args()->k1; ++k) {
        unsigned long long tt = R2T_NOW();
        ++acc[3];
        const int cb = k & 1;
        {
            const rargs_t R = run_args();
            double d, s;
            backward_solver_lane_ilp<U0Z, OUT_SOLVER>(R->m, R->w, R->x[cb], R->u[cb], run_xr<RL>(R, l),
                                                      run_ur<RL>(R, l), R->K1,
                                                      R->cs, R->a.gamma0, l, R->Bp, R->N, d, s);
            const rargs_t Q = run_args();
            Q->dJ[l] = d;
            Q->smax[l] = s;
            if (Q->hist_smax && k < Q->a.hist_len) Q->hist_smax[(int64_t)k * Q->Bp + l] = s;
        }
        lane_fence();
        acc[0] += R2T_NOW() - tt;
        tt = R2T_NOW();
        double Jn;
        {
            const rargs_t R = run_args();
            const double2 xa = R->x[cb][wix(0, 0, 2, l, R->Bp)], xb = R->x[cb][wix(0, 1, 2, l, R->Bp)];
            Jn = rollout_cform<true, U0Z, false, false, kNT, BAND>(R->m, R->w, R->u[cb], R->K1, R->cs,
                                                                   run_xr<RL>(R, l), run_ur<RL>(R, l),
                                                                   R->x[cb ^ 1], R->u[cb ^ 1], R->a.gamma0,
                                                                   R->a.gamma0, l, R->Bp, R->N, xa.x, xa.y, xb.x, xb.y);
        }
        acc[1] += R2T_NOW() - tt;
        const rargs_t R = run_args();
        double g = R->a.gamma0;
        int nr = 1;
        bool ok = Jn < R->cost[l] + R->a.c * g * R->dJ[l];   // strict Armijo test (:361)
        if (!ok && R->a.max_ls > 1) {
            // sigma1 of this sweep (not streamed): the sweep re-run, same code and inputs -> the same bits
            {
                const rargs_t P = run_args();
                double d2, s2;
                backward_solver_lane<U0Z, OUT_SIGMA, BAND>(P->m, P->w, P->x[cb], P->u[cb], run_xr<RL>(P, l),
                                                           run_ur<RL>(P, l), P->K1,
                                                           P->cs, 0.0, l, P->Bp, P->N, d2, s2);
            }
            lane_fence();
            for (int j = 1; !ok && j < run_args()->a.max_ls; ++j) {
                const rargs_t P = run_args();
                g *= P->a.beta;   // gamma_i *= beta, sequentially (:365)
                const double2 xa = P->x[cb][wix(0, 0, 2, l, P->Bp)], xb = P->x[cb][wix(0, 1, 2, l, P->Bp)];
                Jn = rollout_cform<true, U0Z, true, false, kNT, BAND>(P->m, P->w, P->u[cb], P->K1, P->cs,
                                                                      run_xr<RL>(P, l), run_ur<RL>(P, l), P->x[cb ^ 1], P->u[cb ^ 1], g,
                                                                      P->a.gamma0, l, P->Bp, P->N, xa.x, xa.y, xb.x,
                                                                      xb.y);
                ++nr;
                const rargs_t Q = run_args();
                ok = Jn < Q->cost[l] + Q->a.c * g * Q->dJ[l];
            }
        }
        const rargs_t F = run_args();
        F->n_roll[l] += nr;
        F->n_iter[l] += 1;
        SolverCtl c = F->a;
        c.k = k;
        if (ok) {
            const double s = F->smax[l];
            accept_lane(c, l, Jn, g, s, F->cost, F->gamma, F->status, F->res_buf, F->hist_cost, F->Bp);
            if (s < c.tol) st = GYM_CONVERGED;
        } else {
            fail_lane(c, l, F->status, F->res_buf);
            st = GYM_LS_FAILED;
        }
        lane_fence();   // the candidate buffer is the next sweep's input
    }
#ifdef GYM_RUN2_TRACE
    if (threadIdx.x == 0 && blockIdx.x < 8192)
        for (int i = 0; i < 4; ++i) g_run2_trace[blockIdx.x][0][i] = acc[i];
#endif
}

// ------------------------------------------------------------------------------------------
// Persistent schedule on TWO wavefronts per 64 lanes (k_nt_run2, the default persistent kernel).
// In the latency-bound regime (BASELINE cfg 2: 4,096 lanes = 64 wavefronts on 1,024 SIMDs) every wavefront is
// alone on its SIMD and issues about one fp64 instruction per 4.4-5 cycles (profiles/r02_probe/README.md), so a
// stage costs its instruction count.  A second wavefront per 64 lanes, on another SIMD, takes every instruction
// that is not on the lane's dependency chain:
//   sweep : the helper evaluates stage t's Jacobian and linearisation (stage_lin: a function of x_t, u_t only)
//           and hands them, with x_t and u_t, to the main wavefront through an LDS ring; the main wavefront runs
//           only the Riccati recursion (step_lin) and stores K row 1 / cg;
//   trial : the main wavefront runs the feedback + RK4 chain and hands (x_{t+1}, u1_t) to the helper, which
//           forms u0, accumulates the cost and stores the candidate trajectory.
// The two advance in chunks of R2C stages, the producer one chunk ahead (two chunks of ring slots), separated by
// workgroup barriers; a chunk's ring slots hold R2W pairs per lane ([slot][pair][lane]: one 1 KiB row per wave
// instruction).  Per lane the arithmetic is the single-wavefront kernel's -- the same functions (jacobian,
// stage_lin, step_lin, trial_u0 / trial_u1, stage_cost, rk4), each contracting FMAs inside its expressions only
// -- so the results are the same bits.  The rare Armijo retries (sigma1 re-run, trials 2..20) run on the main
// wavefront alone, with the single-wavefront code, while the helper waits at the end-of-iteration barrier.
// Lanes that are not active (finished, padding) run along without storing anything: every barrier is reached by
// every thread, and the iteration loop ends when no lane of the workgroup is active.
// ------------------------------------------------------------------------------------------
constexpr int R2C = 2;            // stages per chunk (even)
constexpr int R2S = 3 * R2C;      // ring slots (the trial uses two chunks of them, the split sweep three)
constexpr int R2W = 11;           // pairs per lane and slot: sweep x_t (2), u_t, Lin (8); trial x_{t+1} (2), u1_t
// The sweep's Riccati update is split over two wavefronts: the main one runs only the matrix half (Sweep::step_P:
// gain row, P) and hands k, G11, 1/G11 to the pair wavefront, which runs the vector half (step_p: sigma, dJ, p,
// ||sigma||) and the K1 / cg stores one chunk behind.  Nothing flows back, so the main wavefront's chain loses the
// vector half, the stores and 6 of its 11 ring reads per stage.  The helpers' ring is three chunks deep (the pair
// wavefront reads chunk c - 1 while the main one reads c and the helpers write c + 1).
constexpr int R2RD = 3;           // helper ring depth in chunks (sweep)
// Prefetch distance of the producers' stream loads, in stages (= register sets in rotation).  A stage of either
// wavefront is ~2x shorter than the single-wavefront kernel's, and the loads of data the previous pass wrote
// take ~1 us: with one stage of prefetch both passes ran at the load latency (~2,400 cycles per stage measured,
// whatever the instruction count, tools/run2_trace.py).
constexpr int R2PD = 4;
static_assert(R2PD % R2C == 0, "the prefetch distance is a whole number of chunks");
// chunks per pass, rounded up to whole register-set rotations: producer and consumer both run this many chunk
// phases (the consumer skips the stages past T), so their barrier counts match
// a stage index the compiler may compute on the VALU (e.g. a clamp as v_sub_u32 ... clamp) made wave-uniform
// again: a buffer resource built from a VGPR value becomes a waterfall loop of v_readfirstlane
__device__ __forceinline__ int uni(int v) { return __builtin_amdgcn_readfirstlane(v); }
// x_ref / u_ref rows through the constant address space: the compiler then reads a stage's row with scalar loads
// (it cannot prove that no store of the kernel clobbers a plain global pointer, and falls back to vector loads
// that count in vmcnt -- and the stage then waits for them behind its prefetches)
typedef const __attribute__((address_space(4))) double* cptr_t;
template <int NV>
struct Row {
    double v[NV];
};
template <int NV>
__device__ __forceinline__ Row<NV> const_row(const double* base, int t) {
    const cptr_t p = (cptr_t)base + (int64_t)NV * t;
    Row<NV> r;
#pragma unroll
    for (int i = 0; i < NV; ++i) r.v[i] = p[i];
    return r;
}
// ... or, for per-lane references, the lane's own row (vector loads)
template <int NV, bool RL>
__device__ __forceinline__ Row<NV> ref_row(const double* base, int t) {
    if (!RL) return const_row<NV>(base, t);
    Row<NV> r;
#pragma unroll
    for (int i = 0; i < NV; ++i) r.v[i] = base[(int64_t)NV * t + i];
    return r;
}
__device__ __forceinline__ void in_vgpr2(double2& v) { asm volatile("" : "+v"(v.x), "+v"(v.y)); }
__device__ __forceinline__ int run2_chunks(int T) {
    constexpr int per = R2PD / R2C;
    return ((T + R2C - 1) / R2C + per - 1) / per * per;
}
typedef double2 (*ring_t)[R2W][BLK];

// The chunk hand-off: this wavefront's LDS writes complete, then the workgroup barrier.  Not __syncthreads(): its
// workgroup-scope release also drains every outstanding global load and store (s_waitcnt vmcnt(0)), i.e. the
// next stages' prefetches and the last stores' round trip at every chunk.  Only LDS crosses between the two
// wavefronts inside a pass; global memory is handed over at the iteration's end (lane_fence + __syncthreads).
// The "memory" clobber keeps the compiler from moving LDS accesses across it.
__device__ __forceinline__ void lds_barrier(unsigned long long& wait) {
    const unsigned long long t0 = R2T_NOW();
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
    wait += R2T_NOW() - t0;   // GYM_RUN2_TRACE only (otherwise 0 + 0: removed)
}

// helper wavefront HID of NH, sweep: the stages i = HID, HID + NH, ... of the reverse pass (t = T-1-i) into slot
// (chunk & 1) * R2C + (i % R2C)
template <bool U0Z, int HID, int NH, bool RL>
__device__ __forceinline__ void run2_sweep_helper(ring_t ring, int lane, int64_t l, int cb, const double* __restrict__ xr,
                                                  const double* __restrict__ ur, unsigned long long& bw) {
    const rargs_t R = run_args();
    const int T = R->N - 1;
    const uint32_t o2 = wbo(l, 2), o1 = (uint32_t)l * 8u;
    const uint32_t row = (uint32_t)R->Bp * 16u, plane = (uint32_t)R->Bp * 8u;
    const char* Xb = reinterpret_cast<const char*>(R->x[cb]);
    const char* Ub = reinterpret_cast<const char*>(R->u[cb]);
    // x_ref / u_ref rows: wave-uniform scalar loads (restrict parameters: no store can alias them); per-lane
    // references (RL): the lane's own rows
    // the model, the weights stage_lin reads and every Horner coefficient held in VGPRs across the stage loop: no
    // per-stage kernel-argument loads (and their lgkmcnt(0) waits) and no per-use copies of scalar operands
    const gym::PolyRegs pk = gym::poly_vgprs_all();
    Dyn dm = R->m;
    KW wv = R->w;
    gym::in_vgpr(dm.b); gym::in_vgpr(dm.d); gym::in_vgpr(dm.a2b); gym::in_vgpr(dm.bb); gym::in_vgpr(dm.dad);
    gym::in_vgpr(dm.g1); gym::in_vgpr(dm.g2); gym::in_vgpr(dm.f1); gym::in_vgpr(dm.f2); gym::in_vgpr(dm.h);
    gym::in_vgpr(dm.h2); gym::in_vgpr(dm.h6);
    gym::in_vgpr(wv.twoQ[0]); gym::in_vgpr(wv.twoQ[1]); gym::in_vgpr(wv.twoQ[2]); gym::in_vgpr(wv.twoQ[3]);
    gym::in_vgpr(wv.G00); gym::in_vgpr(wv.twoR1);
    auto fetch = [&](SweepStage& q, int t) {
        const auto rX = rsrc(Xb + (int64_t)t * (2 * (int64_t)row)), rU = rsrc(Ub + (int64_t)t * row);
        q.xa = bld2(rX, o2, 0);
        q.xb = bld2(rX, o2, WROW);
        q.u0 = U0Z ? 0.0 : bld1(rU, o1, 0);
        q.u1 = bld1(rU, o1, plane);
    };
    auto produce = [&](const SweepStage& q, int t, int slot) {
        const gym::Jac J = gym::jacobian(dm, q.xa.x, q.xa.y, q.xb.x, q.xb.y, q.u1, pk);
        const Row<4> xrt = ref_row<4, RL>(xr, t);
        const Row<2> urt = ref_row<2, RL>(ur, t);
        const Lin L = stage_lin<U0Z>(dm, wv, J, q.xa, q.xb, q.u0, q.u1, xrt.v, urt.v);
        double2(*s)[BLK] = ring[slot];
        s[0][lane] = q.xa;                          s[1][lane] = q.xb;
        s[2][lane] = make_double2(q.u0, q.u1);      s[3][lane] = make_double2(L.A20, L.A21);
        s[4][lane] = make_double2(L.A22, L.A23);    s[5][lane] = make_double2(L.A30, L.A31);
        s[6][lane] = make_double2(L.A32, L.A33);    s[7][lane] = make_double2(L.bd2, L.bd3);
        s[8][lane] = make_double2(L.q0, L.q1);      s[9][lane] = make_double2(L.q2, L.q3);
        s[10][lane] = make_double2(L.r0, L.r1);
    };
    // Branch-free stream loads: every producer stage loads (a clamped stage index past the end), so the
    // compiler's wait-count tracking stays exact and a stage waits only for its own loads, R2PD stages old
    // (with loads on conditional paths it fell back to vmcnt(0) at every stage: the prefetch was void).
    static_assert(R2C % NH == 0, "every helper takes the same number of stages per chunk");
    const int nch = run2_chunks(T);
    SweepStage P[R2PD / NH];               // stage i's streams in set (i % R2PD) / NH, loaded R2PD stages ahead
#pragma unroll
    for (int j = HID; j < R2PD; j += NH) fetch(P[j / NH], uni(max(T - 1 - j, 0)));
    for (int c0 = 0; c0 < nch; c0 += R2PD / R2C) {
#pragma unroll
        for (int cc = 0; cc < R2PD / R2C; ++cc) {
            const int c = c0 + cc;
#pragma unroll
            for (int j = HID; j < R2C; j += NH) {
                const int i = c * R2C + j, set = (cc * R2C + j) / NH;
                // the stage's streams moved out of the loading registers first (the only wait: for this set, R2PD
                // stages old), so that the set is re-armed at once and every later use reads the copy
                SweepStage w = P[set];
                in_vgpr2(w.xa); in_vgpr2(w.xb); gym::in_vgpr(w.u0); gym::in_vgpr(w.u1);
                fetch(P[set], uni(max(T - 1 - (i + R2PD), 0)));
                produce(w, uni(max(T - 1 - i, 0)), (c % R2RD) * R2C + j);   // past the end: not consumed
            }
            lds_barrier(bw);
        }
    }
    lds_barrier(bw);
    lds_barrier(bw);                       // the vector half's last chunk
}

// main wavefront, sweep: the matrix half of the Riccati recursion (Sweep::step_P) from the ring's
// A_d rows and b; stage i's gain row, G11 and 1/G11 into the gain ring (slot (c & 1) * R2C + j) for the pair
// wavefront.  Chunk c between barriers c and c + 1, as run2_sweep_main.
typedef double2 (*gring_t)[3][BLK];
template <bool U0Z, bool RL>
__device__ __forceinline__ void run2_sweep_gain(ring_t ring, gring_t gring, int lane, int64_t l, int cb,
                                                unsigned long long& bw) {
    const rargs_t R = run_args();
    const int T = R->N - 1;
    const double2* x = R->x[cb];
    Sweep<false> S(R->w, x[wix(T, 0, 2, l, R->Bp)], x[wix(T, 1, 2, l, R->Bp)], run_xr<RL>(R, l) + 4 * T);
    const int nch = run2_chunks(T);
    KW wv = R->w;                          // step_P's weights and dt in VGPRs: no per-stage kernel-argument loads
    double dtv = R->m.h;
    gym::in_vgpr(wv.twoQ[0]); gym::in_vgpr(wv.twoQ[1]); gym::in_vgpr(wv.twoQ[2]); gym::in_vgpr(wv.twoQ[3]);
    gym::in_vgpr(wv.twoR1); gym::in_vgpr(dtv);
    lds_barrier(bw);                       // the helpers' chunk 0
    for (int c = 0; c < nch; ++c) {
#pragma unroll
        for (int j = 0; j < R2C; ++j) {
            const int i = c * R2C + j;
            if (i < T) {
                const double2(*s)[BLK] = ring[(c % R2RD) * R2C + j];
                const double2 a0 = s[3][lane], a1 = s[4][lane], a2 = s[5][lane], a3 = s[6][lane];
                const double2 bd = s[7][lane];
                const Lin L{a0.x, a0.y, a1.x, a1.y, a2.x, a2.y, a3.x, a3.y, bd.x, bd.y,
                            0.0, 0.0, 0.0, 0.0, 0.0, 0.0, dtv};      // q, r: the vector half's
                double k0, k1, k2, k3, G11, iG;
                S.step_P(wv, L, k0, k1, k2, k3, G11, iG);
                double2(*g)[BLK] = gring[(c & 1) * R2C + j];
                g[0][lane] = make_double2(k0, k1);
                g[1][lane] = make_double2(k2, k3);
                g[2][lane] = make_double2(G11, iG);
            }
        }
        lds_barrier(bw);
    }
    lds_barrier(bw);                       // the vector half's last chunk
}

// pair wavefront, sweep: the vector half (Sweep::step_p) of stage i from the helpers' ring (chunk
// c, still in its slot: three chunks deep) and the main wavefront's gain ring; K row 1 / cg stored for active lanes.
// Chunk c between barriers c + 1 and c + 2.
template <bool U0Z, bool RL>
__device__ __forceinline__ void run2_sweep_vec(ring_t ring, gring_t gring, int lane, int64_t l, int cb, bool act,
                                               double& dJ_out, double& smax_out, unsigned long long& bw) {
    const rargs_t R = run_args();
    const bool ext = R->ext != 0;
    const int T = R->N - 1;
    const int64_t Bp = R->Bp;
    const uint32_t o2 = wbo(l, 2), o1 = (uint32_t)l * 8u;
    const uint32_t so2 = act ? o2 : 0x80000000u, so1 = act ? o1 : 0x80000000u;   // inactive: dropped (OOB)
    const uint32_t row = (uint32_t)Bp * 16u, plane = (uint32_t)Bp * 8u;
    const char* Kb = reinterpret_cast<const char*>(R->K1);
    const char* Cb = reinterpret_cast<const char*>(R->cs);
    const double g0 = R->a.gamma0;
    const double2* x = R->x[cb];
    Sweep<false> S(R->w, x[wix(T, 0, 2, l, Bp)], x[wix(T, 1, 2, l, Bp)], run_xr<RL>(R, l) + 4 * T);
    const int nch = run2_chunks(T);
    KW wv = R->w;                          // step_p's weights and dt in VGPRs: no per-stage kernel-argument loads
    double dtv = R->m.h;
    gym::in_vgpr(wv.iG00); gym::in_vgpr(dtv);
    lds_barrier(bw);                       // the helpers' chunk 0
    lds_barrier(bw);                       // the main wavefront's chunk 0
    for (int c = 0; c < nch; ++c) {
#pragma unroll
        for (int j = 0; j < R2C; ++j) {
            const int i = c * R2C + j;
            if (i < T) {
                const double2(*s)[BLK] = ring[(c % R2RD) * R2C + j];
                const double2 xa = s[0][lane], xb = s[1][lane], uu = s[2][lane];
                const double2 a0 = s[3][lane], a1 = s[4][lane], a2 = s[5][lane], a3 = s[6][lane];
                const double2 bd = s[7][lane], qa = s[8][lane], qb = s[9][lane], rr = s[10][lane];
                const double2(*g)[BLK] = gring[(c & 1) * R2C + j];
                const double2 ka01 = g[0][lane], ka23 = g[1][lane], gi = g[2][lane];
                const Lin L{a0.x, a0.y, a1.x, a1.y, a2.x, a2.y, a3.x, a3.y, bd.x, bd.y,
                            qa.x, qa.y, qb.x, qb.y, rr.x, rr.y, dtv};
                double s0, s1;
                S.step_p<U0Z>(wv, L, ka01.x, ka01.y, ka23.x, ka23.y, gi.x, gi.y, s0, s1);
                // an inactive lane's stores take an offset past the resources' range (dropped): no exec-mask branch
                if (ext)   // external retries: sigma1 stored too (the candidates read it; no re-run)
                    store_stage<OUT_ALL>(Kb, Cb, T - 1 - i, row, plane, so2, so1, xa, xb, uu.y, g0, ka01.x,
                                         ka01.y, ka23.x, ka23.y, s1);
                else
                    store_stage<OUT_SOLVER>(Kb, Cb, T - 1 - i, row, plane, so2, so1, xa, xb, uu.y, g0, ka01.x,
                                            ka01.y, ka23.x, ka23.y, s1);
            }
        }
        lds_barrier(bw);
    }
    dJ_out = S.dJ;
    smax_out = S.smax;
}

// The first Armijo trial's chain runs on lane pairs: two wavefronts share the 64 lanes' RK4 chains, trajectory
// tl (< 64) of the workgroup on lanes (2q, 2q+1) of wavefront tl / 32 with q = tl % 32; the even lane reduces /
// rotates th1, the odd lane th2 (gym::rk4_pair_fast, bit-identical to rk4).  The second sweep helper, idle in the
// trial, is the chains' loader.  It reads K row 1 and cg of the stages two chunks ahead from global memory and writes them into
// an LDS ring three chunks deep ([slot][k0, k1, cg][trajectory]); the two RK4-chain wavefronts read each stage's row
// from LDS one stage ahead and issue no global loads at all.  With the global loads on the chains the compiler's
// wait-count placement (loop rotation around the branchy RK4 step) waited for the most recent prefetches once per
// unrolled body: a load round trip on the chain.  The loader waits for its own loads, off every chain.
typedef double2 (*kring_t)[3][BLK];

// loader wavefront: chunks 0, 1 before the pass's leading barrier, chunk c + 2 during phase c
template <bool U0Z>
__device__ __forceinline__ void run2_trial_kload(kring_t kr, int lane, int64_t l, unsigned long long& bw) {
    const rargs_t R = run_args();
    const int T = R->N - 1;
    const int64_t Bp = R->Bp;
    const uint32_t o2 = wbo(l, 2), o1 = (uint32_t)l * 8u;
    const uint32_t row = (uint32_t)Bp * 16u;
    const char* Kb = reinterpret_cast<const char*>(R->K1);
    const char* Cb = reinterpret_cast<const char*>(R->cs);
    auto fetch = [&](TrialStage& q, int t) {
        const auto rK = rsrc(Kb + (int64_t)t * (2 * (int64_t)row));
        q.k0 = bld2(rK, o2, 0);
        q.k1 = bld2(rK, o2, WROW);
        q.cg = bld1(rsrc(Cb + (int64_t)t * row), o1, 0);
    };
    auto put = [&](const TrialStage& q, int slot) {
        kr[slot][0][lane] = q.k0;
        kr[slot][1][lane] = q.k1;
        kr[slot][2][lane] = make_double2(q.cg, 0.0);
    };
    const int nch = run2_chunks(T);
    {
        TrialStage P0[2 * R2C];
#pragma unroll
        for (int j = 0; j < 2 * R2C; ++j) fetch(P0[j], uni(min(j, T - 1)));
#pragma unroll
        for (int j = 0; j < 2 * R2C; ++j) put(P0[j], j);
    }
    TrialStage P[R2C];                     // chunk c + 2's rows, loaded during phase c - 1
#pragma unroll
    for (int j = 0; j < R2C; ++j) fetch(P[j], uni(min(2 * R2C + j, T - 1)));
    lds_barrier(bw);                       // the pass's leading barrier: chunks 0, 1 in the ring
    int s2 = 2;                            // (c + 2) % 3
    for (int c = 0; c < nch; ++c) {
#pragma unroll
        for (int j = 0; j < R2C; ++j) {
            put(P[j], s2 * R2C + j);
            fetch(P[j], uni(min((c + 3) * R2C + j, T - 1)));
        }
        s2 = s2 == 2 ? 0 : s2 + 1;
        lds_barrier(bw);
    }
    lds_barrier(bw);
}

// the pair trial's chain fed from the loader's LDS ring: stage t's row is read during stage
// t - 1 (chunk c + 1's first row during chunk c's last stage: written in phase c - 1)
template <bool U0Z>
__device__ __forceinline__ void run2_trial_pair_lds(ring_t ring, kring_t kr, int tl, int64_t l, bool odd, int cb,
                                                    unsigned long long& bw) {
    const rargs_t R = run_args();
    const int T = R->N - 1;
    const int64_t Bp = R->Bp;
    const double2 xa = R->x[cb][wix(0, 0, 2, l, Bp)], xb = R->x[cb][wix(0, 1, 2, l, Bp)];
    double n0 = xa.x, n1 = xa.y, n2 = xb.x, n3 = xb.y;
    auto get = [&](TrialStage& q, int slot) {
        q.k0 = kr[slot][0][tl];
        q.k1 = kr[slot][1][tl];
        q.cg = kr[slot][2][tl].x;
    };
    // every Horner coefficient of the minimax kernels and the model held in VGPRs across the stage loop: no scalar
    // loads in it (the LDS reads' lgkmcnt waits are not merged with kernarg loads) and no per-stage copies of second
    // scalar operands
    const gym::PolyRegs pk = gym::poly_vgprs_all();
    Dyn dm = R->m;
    gym::in_vgpr(dm.b); gym::in_vgpr(dm.d); gym::in_vgpr(dm.a2b); gym::in_vgpr(dm.bb); gym::in_vgpr(dm.dad);
    gym::in_vgpr(dm.g1); gym::in_vgpr(dm.g2); gym::in_vgpr(dm.f1); gym::in_vgpr(dm.f2); gym::in_vgpr(dm.h);
    gym::in_vgpr(dm.h2); gym::in_vgpr(dm.h6);
    auto step = [&](const TrialStage& q, int slot) {
        const double v1 = trial_u1(q.k0, q.k1, q.cg, n0, n1, n2, n3);
        // branch-free near-path step (a wave-uniform fallback to the full reduction inside); three-address Horner
        gym::rk4_pair_fast<true>(dm, odd, n0, n1, n2, n3, v1, pk);
        double2(*s)[BLK] = ring[slot];
        s[0][tl] = make_double2(n0, n1);    // both lanes of the pair: the same values, no per-lane select
        s[1][tl] = make_double2(n2, n3);
        s[2][tl] = make_double2(v1, 0.0);   // both lanes of the pair: the same value
    };
    const int nch = run2_chunks(T);
    lds_barrier(bw);                       // the loader's chunks 0, 1
    TrialStage cur;
    get(cur, 0);
    int s0 = 0, s1 = 1;                    // c % 3, (c + 1) % 3
    for (int c = 0; c < nch; ++c) {
#pragma unroll
        for (int j = 0; j < R2C; ++j) {
            TrialStage nxt;
            get(nxt, j + 1 < R2C ? s0 * R2C + j + 1 : s1 * R2C);
            step(cur, (c & 1) * R2C + j);   // past the end: harmless, not consumed
            cur = nxt;
        }
        s0 = s1;
        s1 = s1 == 2 ? 0 : s1 + 1;
        lds_barrier(bw);
    }
    lds_barrier(bw);
}

// helper wavefront, first Armijo trial: u0, the running cost and the candidate's stores; returns J
template <bool U0Z, bool RL>
__device__ __forceinline__ double run2_trial_helper(ring_t ring, int lane, int64_t l, int cb, bool act,
                                                  const double* __restrict__ xr, const double* __restrict__ ur,
                                                  unsigned long long& bw) {
    const rargs_t R = run_args();
    const int T = R->N - 1;
    const int64_t Bp = R->Bp;
    const uint32_t o2 = wbo(l, 2), o1 = (uint32_t)l * 8u;
    const uint32_t so2 = act ? o2 : 0x80000000u, so1 = act ? o1 : 0x80000000u;   // inactive: dropped (OOB)
    const uint32_t row = (uint32_t)Bp * 16u, plane = (uint32_t)Bp * 8u;
    const char* Ub = reinterpret_cast<const char*>(R->u[cb]);
    const char* Xb = reinterpret_cast<const char*>(R->x[cb ^ 1]);
    const char* Ob = reinterpret_cast<const char*>(R->u[cb ^ 1]);
    // x_ref / u_ref rows: wave-uniform scalar loads (restrict parameters: no store can alias them); per-lane
    // references (RL): the lane's own rows
    const double gamma = R->a.gamma0;
    const double2 xa = R->x[cb][wix(0, 0, 2, l, Bp)], xb = R->x[cb][wix(0, 1, 2, l, Bp)];
    double n0 = xa.x, n1 = xa.y, n2 = xb.x, n3 = xb.y;
    if (act) {
        const auto rX = rsrc(Xb);
        bst2(rX, o2, 0, n0, n1);
        bst2(rX, o2, WROW, n2, n3);
    }
    double J = 0.0;
    const int nch = run2_chunks(T);
    lds_barrier(bw);                       // the loader's leading barrier
    lds_barrier(bw);                       // the main wavefront's chunk 0
    for (int c = 0; c < nch; ++c) {
#pragma unroll
        for (int j = 0; j < R2C; ++j) {
            const int t = c * R2C + j;
            if (t < T) {
                const double2(*s)[BLK] = ring[(c & 1) * R2C + j];
                const double2 na = s[0][lane], nb = s[1][lane], vv = s[2][lane];
                const Row<2> urt = ref_row<2, RL>(ur, t);
                const Row<4> xrt = ref_row<4, RL>(xr, t);
                const KArgs ka = kernarg_consts();
                const double u0 = U0Z ? 0.0 : bld1(rsrc(Ub + (int64_t)t * row), o1, 0);
                const double v0 = U0Z ? 0.0 : trial_u0(u0, urt.v[0], gamma, ka.w.G00, ka.w.iG00);
                const double v1 = vv.x;
                const double f0 = U0Z ? 0.0 : v0 - urt.v[0], f1 = v1 - urt.v[1];
                J = stage_cost<U0Z>(J, ka.w.Q, ka.w.R, n0, n1, n2, n3, xrt.v, f0, f1);
                {   // an inactive lane's stores fall outside the resources' range (dropped): no exec-mask branch
                    const auto rO = rsrc(Ob + (int64_t)t * row);
                    if (!U0Z) bst1(rO, so1, 0, v0);
                    bst1(rO, so1, plane, v1);
                    const auto rX = rsrc(Xb + (int64_t)(t + 1) * (2 * (int64_t)row));
                    bst2(rX, so2, 0, na.x, na.y);
                    bst2(rX, so2, WROW, nb.x, nb.y);
                }
                n0 = na.x; n1 = na.y; n2 = nb.x; n3 = nb.y;
            }
        }
        lds_barrier(bw);
    }
    const Row<4> xrT = ref_row<4, RL>(xr, T);
    return J + xcost(R->w.QT, n0, n1, n2, n3, xrT.v);
}

// Four wavefronts per 64 lanes.  Sweep: 0 the matrix half of the Riccati update, 1 and 2 the stage linearisations
// (dealt round-robin), 3 the vector half and the stores.  Trial: 0 and 3 the RK4 chains on lane pairs, 1 the cost
// and the candidate's stores, 2 the chains' loader.
constexpr int R2H = 2;            // sweep helper wavefronts
constexpr int R2WAVES = 4;

template <bool U0Z, bool RL>
__global__ __launch_bounds__(R2WAVES * BLK, 1) void k_nt_run2(RunArgs args) {
    __shared__ double2 ring[R2S][R2W][BLK];
    __shared__ double2 gring[2 * R2C][3][BLK];   // the split sweep's gain rows, G11, 1/G11
    __shared__ double2 kring[3 * R2C][3][BLK];   // the trial's K row 1 / cg (loader wavefront)
    __shared__ double shJ[BLK];
    __shared__ int shst[BLK];
    const int lane = threadIdx.x & (BLK - 1);
    const int wave = threadIdx.x / BLK;          // 0: main; 1 .. R2H: helpers
    const bool helper = wave > 0;
    const int64_t l = (int64_t)blockIdx.x * BLK + lane;   // < Bp: padding lanes hold GYM_PAD
    int st = run_args()->status[l];
    // GYM_RUN2_TRACE only: sweep / trial / post cycles, iterations, barrier waits in the sweep / the trial
    unsigned long long acc[6] = {0, 0, 0, 0, 0, 0};
    for (int k = run_args()->k0; k < run_args()->k1; ++k) {
        if (!__syncthreads_or(st == GYM_ACTIVE)) break;    // workgroup-uniform
        const bool act = st == GYM_ACTIVE;
        const int cb = k & 1;
        unsigned long long tt = R2T_NOW();
        ++acc[3];
        if (wave == 1) {
            run2_sweep_helper<U0Z, 0, R2H, RL>(ring, lane, l, cb, run_xr<RL>(run_args(), l), run_ur<RL>(run_args(), l),
                                               acc[4]);
        } else if (wave == 2) {
            run2_sweep_helper<U0Z, 1, R2H, RL>(ring, lane, l, cb, run_xr<RL>(run_args(), l),
                                               run_ur<RL>(run_args(), l), acc[4]);
        } else if (wave == 0) {
            run2_sweep_gain<U0Z, RL>(ring, gring, lane, l, cb, acc[4]);
        } else {   // the pair wavefront: the vector half, the stores
            double d, s;
            run2_sweep_vec<U0Z, RL>(ring, gring, lane, l, cb, act, d, s, acc[4]);
            const rargs_t Q = run_args();
            if (act) {
                Q->dJ[l] = d;
                Q->smax[l] = s;
                if (Q->hist_smax && k < Q->a.hist_len) Q->hist_smax[(int64_t)k * Q->Bp + l] = s;
            }
            lane_fence();                                  // K1 / cg visible to this wavefront's trial loads
        }
        __syncthreads();                                   // K1 / cg stored by the pair wavefront, read by the loader
        acc[0] += R2T_NOW() - tt;
        tt = R2T_NOW();
        if (wave == 1) {
            shJ[lane] = run2_trial_helper<U0Z, RL>(ring, lane, l, cb, act, run_xr<RL>(run_args(), l),
                                                   run_ur<RL>(run_args(), l), acc[5]);
        } else if (wave == 2) {
            run2_trial_kload<U0Z>(kring, lane, l, acc[5]);
        } else {                                           // waves 0 and 3: lane pairs, rows from LDS
            const int tl = (wave == 0 ? 0 : BLK / 2) + (lane >> 1);
            run2_trial_pair_lds<U0Z>(ring, kring, tl, (int64_t)blockIdx.x * BLK + tl, lane & 1, cb, acc[5]);
        }
        __syncthreads();                                   // shJ written; the helper's stores are complete
        acc[1] += R2T_NOW() - tt;
        tt = R2T_NOW();
        if (!helper && act) {
            const rargs_t R = run_args();
            double Jn = shJ[lane];
            double g = R->a.gamma0;
            int nr = 1;
            bool ok = Jn < R->cost[l] + R->a.c * g * R->dJ[l];   // strict Armijo test (:361)
            const bool deferred = !ok && R->a.max_ls > 1 && R->ext;
            if (deferred) {
                // external retries (one iteration per launch): the lane joins the retry list, as after the serial
                // schedule's trial (k_nt_trial); the candidates / accepted re-run kernels finish its iteration
                R->n_roll[l] += 1;
                R->retry_list[atomicAdd(R->counter, 1)] = (int32_t)l;
            } else if (!ok && R->a.max_ls > 1) {
                lane_fence();                              // the helper's candidate stores, before they are rewritten
                {
                    const rargs_t P = run_args();
                    double d2, s2;
                    backward_solver_lane<U0Z, OUT_SIGMA, false>(P->m, P->w, P->x[cb], P->u[cb], run_xr<RL>(P, l),
                                                                run_ur<RL>(P, l), P->K1,
                                                                P->cs, 0.0, l, P->Bp, P->N, d2, s2);
                }
                lane_fence();
                for (int j = 1; !ok && j < run_args()->a.max_ls; ++j) {
                    const rargs_t P = run_args();
                    g *= P->a.beta;                        // gamma_i *= beta, sequentially (:365)
                    const double2 xa = P->x[cb][wix(0, 0, 2, l, P->Bp)], xb = P->x[cb][wix(0, 1, 2, l, P->Bp)];
                    Jn = rollout_cform<true, U0Z, true, false, kNT, false>(P->m, P->w, P->u[cb], P->K1, P->cs,
                                                                          run_xr<RL>(P, l), run_ur<RL>(P, l),
                                                                          P->x[cb ^ 1], P->u[cb ^ 1], g,
                                                                          P->a.gamma0, l, P->Bp, P->N, xa.x, xa.y,
                                                                          xb.x, xb.y);
                    ++nr;
                    const rargs_t Q = run_args();
                    ok = Jn < Q->cost[l] + Q->a.c * g * Q->dJ[l];
                }
            }
            if (!deferred) {
                const rargs_t F = run_args();
                F->n_roll[l] += nr;
                F->n_iter[l] += 1;
                SolverCtl c = F->a;
                c.k = k;
                if (ok) {
                    const double sm = F->smax[l];
                    accept_lane(c, l, Jn, g, sm, F->cost, F->gamma, F->status, F->res_buf, F->hist_cost, F->Bp);
                    if (sm < c.tol) st = GYM_CONVERGED;
                } else {
                    fail_lane(c, l, F->status, F->res_buf);
                    st = GYM_LS_FAILED;
                }
            }
        }
        if (!helper) shst[lane] = st;
        lane_fence();                                      // every store of this iteration visible to both wavefronts
        __syncthreads();
        if (helper) st = shst[lane];
        acc[2] += R2T_NOW() - tt;
    }
#ifdef GYM_RUN2_TRACE
    if (lane == 0 && blockIdx.x < 8192 && wave <= 1)
        for (int i = 0; i < 6; ++i) g_run2_trace[blockIdx.x][wave][i] = acc[i];
#endif
}

// ------------------------------------------------------------------------------------------
// Straggler tail (gym_newton_tail).  Late in a hard solve a handful of lanes keep iterating for thousands of
// outer iterations, many of them backtracking (SURVEY 8(d)'s stress variant: one lane to 5,000 iterations, the
// last ~4,000 serving a few lanes).  The lock-step schedules then pay, per iteration and lane, one sweep chain
// and one trial chain on one thread each, plus for a backtracking lane the sigma1 re-run, the candidate pass and
// the accepted candidate's re-run.  Here one workgroup (one wavefront) owns one listed lane and runs its own
// iterations k0 .. k1-1 back to back (lanes are independent problems; the persistent schedule's argument):
//   sweep  : the 64 threads evaluate the Jacobians / linearisations of 64 stages at once (stage_lin, a function
//            of x_t, u_t only) into LDS, then run the Riccati recursion (step_lin) over those stages, reading
//            them back; K row 1, cg and sigma1 are stored in the same pass (no sigma1 re-run);
//   trials : thread c evaluates Armijo trial c (gamma_0 beta^c, formed sequentially as the reference does) --
//            all max_ls of them at once, each writing its candidate into a scratch slot -- and the first
//            accepted one (ballot) is copied into the lane's next state buffer.
// Every value is the one the serial schedule computes (the same device functions: jacobian, stage_lin, step_lin,
// store_stage, trial_u0 / trial_u1, stage_cost, rk4): trial 1 is the offset form cg + K1 x_new, trial c > 0
// fma(gamma_c - gamma_0, sigma1, cg + K1 x_new), so decisions, rollout counts and trajectories are the same bits.
// ------------------------------------------------------------------------------------------
constexpr int TL_STAGES = BLK;   // stages per linearisation pass (one per thread)
constexpr int TL_PITCH = 22;     // doubles per stage in LDS: Lin (16), x_t (4), u1_t; padded to an even count
struct TailArgs {
    Dyn m;
    KW w;
    SolverCtl a;
    double2* x[2];
    double* u[2];
    double2* K1;
    double* cs;
    const double* xr;
    const double* ur;
    double *cost, *dJ, *smax, *gamma;
    int32_t *status, *n_iter, *res_buf, *n_roll;
    double *hist_cost, *hist_smax;
    const int32_t* list;   // the lanes, one workgroup each
    double2* sx;           // candidate scratch: x (N, Vp/64, 2, 64) double2 over virtual lanes (slot * max_ls + c)
    double* su;            // ... and u planes (T, 2, Vp)
    int64_t Bp, Vp;
    int32_t N, k0, k1, pad;
};
static_assert(offsetof(TailArgs, w) == 96, "kernarg layout: KW at byte 96 (kernarg_consts)");
typedef const TailArgs* targs_t;
__device__ __forceinline__ targs_t tail_args() {
    const __attribute__((address_space(4))) TailArgs* p =
        (const __attribute__((address_space(4))) TailArgs*)__builtin_amdgcn_kernarg_segment_ptr();
    asm volatile("" : "+s"(p));
    return (targs_t)p;
}

// The trials' per-stage inputs are staged in LDS by the sweep (K row 1, cg, sigma1 and u0: 8 doubles per stage), so
// the trial loop issues no global loads: its scratch stores are never waited on (the GFX9 vmcnt counts both)
constexpr int TL_TST = 8;
constexpr int TL_MAX_T = 640;    // T * 64 B of trial staging (40 KiB) + the linearisation / gain / exchange areas: tail_lds_bytes(T),
                                 // ~72 KiB at T = 500, ~87 KiB at T = 640: above the 64 KiB default, so every launch raises
                                 // the kernel's dynamic-LDS limit (gfx950: 160 KiB); gym_newton_tail_lds reports both
// Two wavefronts per tail lane: the sweep's Riccati update split as in k_nt_run2 (Sweep::step_P on wavefront 0,
// Sweep::step_p, the stores and the next pass's linearisations on wavefront 1, one 64-stage pass behind;
// linearisations triple-buffered, the gain rows double-buffered)
constexpr int TL_THREADS = 2 * BLK;
constexpr int TL_GK = 6;         // doubles per stage in the gain ring: k row 1 (4), G11, 1/G11
// Trials on lane pairs: wavefront 0 runs the candidates' RK4 chains and hands each stage's (x_{t+1}, u1_t) to
// wavefront 1 through a ring of 2 chunks x TL_RC stages x 32 trials x 3 pairs; wavefront 1 (lane c: trial c)
// accumulates the cost and stores the candidate.  (Single-thread trials, GYM_FLAG_RUN_SINGLE or more than 32
// trials: wavefront 0 alone, tail_candidate.)
constexpr int TL_RC = 2;
constexpr int TL_RING = 2 * TL_RC * (BLK / 2) * 3 * 2;   // doubles
constexpr size_t tail_lds_bytes(int T) {
    return sizeof(double) * ((size_t)3 * TL_STAGES * TL_PITCH + (size_t)2 * TL_STAGES * TL_GK + 4 +
                             (size_t)TL_RING + (size_t)T * TL_TST);
}
// The sweep of lane l at iterate cb on two wavefronts: K row 1, cg and sigma1 of every stage (global, and staged in
// tst).  Pass j covers stages T-1-64j down to T-64-64j.  Between
// workgroup barriers j and j+1, wavefront 0 runs the matrix half over pass j (linearisations lin3[j % 3], gain rows
// into gk2[j & 1]) while wavefront 1 runs the vector half over pass j - 1 (its linearisations and gain rows, K row
// 1 / cg / sigma1 stored and staged in tst) and then evaluates pass j + 1's linearisations.  Every thread of a
// wavefront runs the same recursion (the same bits); its lane 0 writes.  dJ and max|sigma| land in shd[0..1].
template <bool U0Z, bool RL>
__device__ __forceinline__ void tail_sweep_split(double* lin3, double* gk2, double* shd, double* tst, int wave,
                                                 int lane, int64_t l, int cb) {
    const targs_t R = tail_args();
    const int T = R->N - 1;
    const int64_t Bp = R->Bp;
    const double2* x = R->x[cb];
    const double* u = R->u[cb];
    const double* xr = lane_ref<RL>(R->xr, l, 4 * (int64_t)R->N);
    const double* ur = lane_ref<RL>(R->ur, l, 2 * (int64_t)T);
    const uint32_t o2 = wbo(l, 2), o1 = (uint32_t)l * 8u;
    const uint32_t so2 = lane == 0 ? o2 : 0x80000000u, so1 = lane == 0 ? o1 : 0x80000000u;   // OOB: dropped
    const uint32_t row = (uint32_t)Bp * 16u, plane = (uint32_t)Bp * 8u;
    const char* Kb = reinterpret_cast<const char*>(R->K1);
    const char* Cb = reinterpret_cast<const char*>(R->cs);
    const double g0 = R->a.gamma0;
    const double dt = R->m.h;
    Sweep<false> S(R->w, x[wix(T, 0, 2, l, Bp)], x[wix(T, 1, 2, l, Bp)], xr + 4 * T);
    const int np = (T + TL_STAGES - 1) / TL_STAGES;
    auto linearise = [&](int j) {   // wavefront 1: pass j's linearisations, thread i stage T-1-64j-i
        const int t = T - 1 - j * TL_STAGES - lane;
        if (t >= 0) {
            const double2 xa = x[wix(t, 0, 2, l, Bp)], xb = x[wix(t, 1, 2, l, Bp)];
            const double u0 = U0Z ? 0.0 : u[pix(t, 0, 2, l, Bp)], u1 = u[pix(t, 1, 2, l, Bp)];
            const KArgs ka = kernarg_consts();
            const gym::Jac J = gym::jacobian(ka.m, xa.x, xa.y, xb.x, xb.y, u1);
            const Lin L = stage_lin<U0Z>(ka.m, ka.w, J, xa, xb, u0, u1, xr + 4 * t, ur + 2 * t);
            double* s = lin3 + ((j % 3) * TL_STAGES + lane) * TL_PITCH;
            s[0] = L.A20; s[1] = L.A21; s[2] = L.A22; s[3] = L.A23;
            s[4] = L.A30; s[5] = L.A31; s[6] = L.A32; s[7] = L.A33;
            s[8] = L.bd2; s[9] = L.bd3; s[10] = L.q0; s[11] = L.q1;
            s[12] = L.q2; s[13] = L.q3; s[14] = L.r0; s[15] = L.r1;
            s[16] = xa.x; s[17] = xa.y; s[18] = xb.x; s[19] = xb.y; s[20] = u1;
            tst[t * TL_TST + 6] = u0;
        }
    };
    KW wv = R->w;                          // the Riccati halves' weights in VGPRs: no per-stage kernel-argument loads
    gym::in_vgpr(wv.twoQ[0]); gym::in_vgpr(wv.twoQ[1]); gym::in_vgpr(wv.twoQ[2]); gym::in_vgpr(wv.twoQ[3]);
    gym::in_vgpr(wv.twoR1); gym::in_vgpr(wv.iG00);
    if (wave == 1) linearise(0);
    __syncthreads();
    for (int j = 0; j <= np; ++j) {
        if (wave == 0) {
            if (j < np) {
                const int tb = T - 1 - j * TL_STAGES;
                const int n = tb + 1 < TL_STAGES ? tb + 1 : TL_STAGES;
                const double* L3 = lin3 + (j % 3) * TL_STAGES * TL_PITCH;
                double* G = gk2 + (j & 1) * TL_STAGES * TL_GK;
                for (int i = 0; i < n; ++i) {
                    const double* s = L3 + i * TL_PITCH;
                    const KW& kw = wv;
                    const Lin L{s[0], s[1], s[2], s[3], s[4], s[5], s[6], s[7], s[8], s[9],
                                0.0, 0.0, 0.0, 0.0, 0.0, 0.0, dt};   // q, r: the vector half's
                    double k0, k1, k2, k3, G11, iG;
                    S.step_P(kw, L, k0, k1, k2, k3, G11, iG);
                    double* g = G + i * TL_GK;     // every thread: the same values at the same addresses
                    g[0] = k0; g[1] = k1; g[2] = k2; g[3] = k3; g[4] = G11; g[5] = iG;
                }
            }
        } else {
            if (j >= 1) {
                const int jj = j - 1;
                const int tb = T - 1 - jj * TL_STAGES;
                const int n = tb + 1 < TL_STAGES ? tb + 1 : TL_STAGES;
                const double* L3 = lin3 + (jj % 3) * TL_STAGES * TL_PITCH;
                const double* G = gk2 + (jj & 1) * TL_STAGES * TL_GK;
                for (int i = 0; i < n; ++i) {
                    const double* s = L3 + i * TL_PITCH;
                    const double* g = G + i * TL_GK;
                    const double k0 = g[0], k1 = g[1], k2 = g[2], k3 = g[3];
                    const KW& kw = wv;
                    const Lin L{s[0], s[1], s[2], s[3], s[4], s[5], s[6], s[7], s[8], s[9],
                                s[10], s[11], s[12], s[13], s[14], s[15], dt};
                    double s0, s1;
                    S.step_p<U0Z>(kw, L, k0, k1, k2, k3, g[4], g[5], s0, s1);
                    {   // every thread: the same values; lane 0's global stores land, the others' fall outside the
                        // resources' range (dropped by the hardware) -- no exec-mask branch on the pass
                        const int ts = tb - i;
                        const double2 xa = make_double2(s[16], s[17]), xb = make_double2(s[18], s[19]);
                        const double cg = stage_cg(xa, xb, s[20], g0, k0, k1, k2, k3, s1);
                        double* q = tst + ts * TL_TST;
                        q[0] = k0; q[1] = k1; q[2] = k2; q[3] = k3; q[4] = cg; q[5] = s1;
                        const auto rC = rsrc(Cb + (int64_t)ts * row);
                        const auto rK = rsrc(Kb + (int64_t)ts * (2 * (int64_t)row));
                        bst2(rK, so2, 0, k0, k1);
                        bst2(rK, so2, WROW, k2, k3);
                        bst1(rC, so1, 0, cg);
                        bst1(rC, so1, plane, s1);
                    }
                }
            }
            if (j + 1 < np) linearise(j + 1);
            if (j == np && lane == 0) { shd[0] = S.dJ; shd[1] = S.smax; }
        }
        __syncthreads();
    }
}

// Armijo trial c of lane l (step size g; c = 0: the first trial's offset form) on one thread into virtual lane v of
// the scratch, its streams from the staging tst; returns the candidate's cost
template <bool U0Z, bool RL>
__device__ __forceinline__ double tail_candidate(const double* tst, int64_t l, int cb, int c, double g, int64_t v) {
    const targs_t R = tail_args();
    const int T = R->N - 1;
    const int64_t Bp = R->Bp;
    const double* xr = lane_ref<RL>(R->xr, l, 4 * (int64_t)R->N);
    const double* ur = lane_ref<RL>(R->ur, l, 2 * (int64_t)T);
    const uint32_t v2 = wbo(v, 2), v1o = (uint32_t)v * 8u;
    const uint32_t srow = (uint32_t)R->Vp * 16u, splane = (uint32_t)R->Vp * 8u;
    const char* Xs = reinterpret_cast<const char*>(R->sx);
    const char* Us = reinterpret_cast<const char*>(R->su);
    const double gamma0 = R->a.gamma0, dg = g - gamma0;
    const double2 xa = R->x[cb][wix(0, 0, 2, l, Bp)], xb = R->x[cb][wix(0, 1, 2, l, Bp)];
    double n0 = xa.x, n1 = xa.y, n2 = xb.x, n3 = xb.y;
    {
        const auto rX = rsrc(Xs);
        bst2(rX, v2, 0, n0, n1);
        bst2(rX, v2, WROW, n2, n3);
    }
    double J = 0.0;
    const gym::PolyRegs pk = gym::poly_vgprs();
    const KArgs ka = kernarg_consts();
    const Dyn m = ka.m;
    const double G00 = ka.w.G00, iG00 = ka.w.iG00;
    for (int t = 0; t < T; ++t) {
        const double* q = tst + t * TL_TST;
        const double2 k0 = make_double2(q[0], q[1]), k1 = make_double2(q[2], q[3]);
        const double cg = q[4], s1 = q[5];
        const Row<2> urt = ref_row<2, RL>(ur, t);
        const Row<4> xrt = ref_row<4, RL>(xr, t);
        const double v0 = U0Z ? 0.0 : trial_u0(q[6], urt.v[0], g, G00, iG00);
        const double y = trial_u1(k0, k1, cg, n0, n1, n2, n3);   // cg + K1 x_new: trial 1's value
        const double ysig = __builtin_fma(dg, s1, y);            // trial_u1_sig's value
        const double u1 = c == 0 ? y : ysig;
        const double f0 = U0Z ? 0.0 : v0 - urt.v[0], f1 = u1 - urt.v[1];
        const KArgs kc = kernarg_consts();
        J = stage_cost<U0Z>(J, kc.w.Q, kc.w.R, n0, n1, n2, n3, xrt.v, f0, f1);
        {
            const auto rO = rsrc(Us + (int64_t)t * srow);
            if (!U0Z) bst1(rO, v1o, 0, v0);
            bst1(rO, v1o, splane, u1);
        }
        gym::rk4(m, n0, n1, n2, n3, u1, pk);
        const auto rX = rsrc(Xs + (int64_t)(t + 1) * (2 * (int64_t)srow));
        bst2(rX, v2, 0, n0, n1);
        bst2(rX, v2, WROW, n2, n3);
    }
    const Row<4> xrT = ref_row<4, RL>(xr, T);
    return J + xcost(ka.w.QT, n0, n1, n2, n3, xrT.v);
}

// Wavefront 0: the RK4 chain of Armijo trial c on the lane pair (2c, 2c + 1) -- the offset-form feedback
// and gym::rk4_pair, exactly tail_candidate's chain -- handing each stage's state and control to wavefront 1 (ring
// [chunk & 1][stage in chunk][trial][(th1, th2) | (w1, w2) | (u1, -)]).  Chunk cc between barriers cc and cc + 1.
typedef double2 (*tring_t)[TL_RC][BLK / 2][3];
template <bool U0Z, bool RL>
__device__ __forceinline__ void tail_trial_chain(const double* tst, tring_t ring, int64_t l, int cb, int c, double g,
                                                 bool odd) {
    const targs_t R = tail_args();
    const int T = R->N - 1;
    const int64_t Bp = R->Bp;
    const double dg = g - R->a.gamma0;
    const double2 xa = R->x[cb][wix(0, 0, 2, l, Bp)], xb = R->x[cb][wix(0, 1, 2, l, Bp)];
    double n0 = xa.x, n1 = xa.y, n2 = xb.x, n3 = xb.y;
    // every Horner coefficient and the model in VGPRs across the chain's loop (as k_nt_run2's trial chain)
    const gym::PolyRegs pk = gym::poly_vgprs_all();
    Dyn m = kernarg_consts().m;
    gym::in_vgpr(m.b); gym::in_vgpr(m.d); gym::in_vgpr(m.a2b); gym::in_vgpr(m.bb); gym::in_vgpr(m.dad);
    gym::in_vgpr(m.g1); gym::in_vgpr(m.g2); gym::in_vgpr(m.f1); gym::in_vgpr(m.f2); gym::in_vgpr(m.h);
    gym::in_vgpr(m.h2); gym::in_vgpr(m.h6);
    const int nch = (T + TL_RC - 1) / TL_RC;
    const int tc = c < BLK / 2 ? c : 0;
    for (int cc = 0; cc < nch; ++cc) {
#pragma unroll
        for (int j = 0; j < TL_RC; ++j) {
            const int t = cc * TL_RC + j;
            if (t < T) {
                const double* q = tst + t * TL_TST;
                const double2 k0 = make_double2(q[0], q[1]), k1 = make_double2(q[2], q[3]);
                const double y = trial_u1(k0, k1, q[4], n0, n1, n2, n3);   // cg + K1 x_new: trial 1's value
                const double ysig = __builtin_fma(dg, q[5], y);             // trial_u1_sig's value
                const double u1 = c == 0 ? y : ysig;
                gym::rk4_pair_fast<true>(m, odd, n0, n1, n2, n3, u1, pk);   // branch-free near path, as k_nt_run2
                double2* r = ring[cc & 1][j][tc];   // both lanes of the pair: the same values, no per-lane select
                r[0] = make_double2(n0, n1);
                r[1] = make_double2(n2, n3);
                r[2] = make_double2(u1, 0.0);
            }
        }
        __syncthreads();
    }
    __syncthreads();                       // the helper's last chunk
}

// Wavefront 1, lane c (< max_ls): trial c's cost (stage costs in stage order, as tail_candidate) and its
// candidate trajectory into virtual lane v of the scratch; returns J.  Chunk cc between barriers cc + 1 and cc + 2.
template <bool U0Z, bool RL>
__device__ __forceinline__ double tail_trial_helper(const double* tst, tring_t ring, int64_t l, int cb, int c, double g,
                                                    int64_t v, bool act) {
    const targs_t R = tail_args();
    const int T = R->N - 1;
    const int64_t Bp = R->Bp;
    const double* xr = lane_ref<RL>(R->xr, l, 4 * (int64_t)R->N);
    const double* ur = lane_ref<RL>(R->ur, l, 2 * (int64_t)T);
    const uint32_t v2 = wbo(v, 2), v1o = (uint32_t)v * 8u;
    const uint32_t srow = (uint32_t)R->Vp * 16u, splane = (uint32_t)R->Vp * 8u;
    const char* Xs = reinterpret_cast<const char*>(R->sx);
    const char* Us = reinterpret_cast<const char*>(R->su);
    const double2 xa = R->x[cb][wix(0, 0, 2, l, Bp)], xb = R->x[cb][wix(0, 1, 2, l, Bp)];
    double n0 = xa.x, n1 = xa.y, n2 = xb.x, n3 = xb.y;
    if (act) {
        const auto rX = rsrc(Xs);
        bst2(rX, v2, 0, n0, n1);
        bst2(rX, v2, WROW, n2, n3);
    }
    double J = 0.0;
    const KArgs ka = kernarg_consts();
    const double G00 = ka.w.G00, iG00 = ka.w.iG00;
    const int nch = (T + TL_RC - 1) / TL_RC;
    const int tc = c < BLK / 2 ? c : 0;
    __syncthreads();                       // the chain's chunk 0
    for (int cc = 0; cc < nch; ++cc) {
#pragma unroll
        for (int j = 0; j < TL_RC; ++j) {
            const int t = cc * TL_RC + j;
            if (t < T) {
                const double2* r = ring[cc & 1][j][tc];
                const double2 na = r[0], nb = r[1], uu = r[2];
                const Row<2> urt = ref_row<2, RL>(ur, t);
                const Row<4> xrt = ref_row<4, RL>(xr, t);
                const double v0 = U0Z ? 0.0 : trial_u0(tst[t * TL_TST + 6], urt.v[0], g, G00, iG00);
                const double u1 = uu.x;
                const double f0 = U0Z ? 0.0 : v0 - urt.v[0], f1 = u1 - urt.v[1];
                const KArgs kc = kernarg_consts();
                J = stage_cost<U0Z>(J, kc.w.Q, kc.w.R, n0, n1, n2, n3, xrt.v, f0, f1);
                if (act) {
                    const auto rO = rsrc(Us + (int64_t)t * srow);
                    if (!U0Z) bst1(rO, v1o, 0, v0);
                    bst1(rO, v1o, splane, u1);
                    const auto rX = rsrc(Xs + (int64_t)(t + 1) * (2 * (int64_t)srow));
                    bst2(rX, v2, 0, na.x, na.y);
                    bst2(rX, v2, WROW, nb.x, nb.y);
                }
                n0 = na.x; n1 = na.y; n2 = nb.x; n3 = nb.y;
            }
        }
        __syncthreads();
    }
    const Row<4> xrT = ref_row<4, RL>(xr, T);
    return J + xcost(ka.w.QT, n0, n1, n2, n3, xrT.v);
}

#ifdef GYM_TAIL_TRACE
// Diagnostic build only (tools/tail_trace.py): per workgroup, cycles (s_memtime) in the sweep, the trials, the rest
// of the iteration, and the iterations run
__device__ unsigned long long g_tail_trace[4096][4];
#endif
template <bool U0Z, bool RL, bool PAIR>
__global__ __launch_bounds__(TL_THREADS, 1) void k_nt_tail(TailArgs args) {
    extern __shared__ double tail_lds[];          // tail_lds_bytes(T)
    // lin3 (3 passes) | gk2 (2 passes of gain rows) | shd (dJ, max|sigma|, the decision) | ring | tst
    double* lin = tail_lds;
    double* gk2 = lin + 3 * TL_STAGES * TL_PITCH;
    double* shd = gk2 + 2 * TL_STAGES * TL_GK;
    const tring_t ring = reinterpret_cast<tring_t>(shd + 4);   // PAIR: the trials' hand-off
    double* tst = shd + 4 + TL_RING;
    const int lane = threadIdx.x & (BLK - 1);
    const int wave = threadIdx.x / BLK;           // 0 the matrix half and the trials, 1 the vector half
    const int64_t l = tail_args()->list[blockIdx.x];
    int st = tail_args()->status[l];
    unsigned long long acc[4] = {0, 0, 0, 0};   // GYM_TAIL_TRACE only
    for (int k = tail_args()->k0; st == GYM_ACTIVE && k < tail_args()->k1; ++k) {
        const int cb = k & 1;
        double dJ, sm;
        unsigned long long tt = R2T_NOW();
        ++acc[3];
        tail_sweep_split<U0Z, RL>(lin, gk2, shd, tst, wave, lane, l, cb);   // ends at a workgroup barrier
        dJ = shd[0];
        sm = shd[1];
        acc[0] += R2T_NOW() - tt;
        tt = R2T_NOW();
        {
            const targs_t Q = tail_args();
            if (lane == 0 && wave == 0) {
                Q->dJ[l] = dJ;
                Q->smax[l] = sm;
                if (Q->hist_smax && k < Q->a.hist_len) Q->hist_smax[(int64_t)k * Q->Bp + l] = sm;
            }
        }
        __syncthreads();   // the staged trial inputs (LDS) complete
        const int max_ls = tail_args()->a.max_ls;
        // PAIR: wavefront 0 runs the trials' chains (trial c on lanes 2c, 2c + 1), wavefront 1 (lane c: trial c) their
        // costs, stores and Armijo tests; otherwise wavefront 0 does all of it, one trial per thread
        const int dec = PAIR ? 1 : 0;               // the wavefront holding the decisions
        const bool helper_wave = PAIR && wave == 1;  // lane c: trial c's cost
        const int cand = (PAIR && !helper_wave) ? lane >> 1 : lane;   // this thread's trial
        const int64_t v = (int64_t)blockIdx.x * max_ls + cand;
        double g = tail_args()->a.gamma0;
        for (int q = 0; q < cand && q < max_ls; ++q) g *= tail_args()->a.beta;   // gamma_i *= beta (:365)
        bool ok = false;
        double Jn = 0.0;
        if (PAIR) {
            if (wave == 0) {
                tail_trial_chain<U0Z, RL>(tst, ring, l, cb, cand, g, lane & 1);
            } else {
                Jn = tail_trial_helper<U0Z, RL>(tst, ring, l, cb, cand, g, v, cand < max_ls);
                const targs_t R = tail_args();
                ok = cand < max_ls && Jn < R->cost[l] + R->a.c * g * dJ;   // strict Armijo test (:361)
            }
        } else if (cand < max_ls && wave == 0) {
            Jn = tail_candidate<U0Z, RL>(tst, l, cb, cand, g, v);
            const targs_t R = tail_args();
            ok = Jn < R->cost[l] + R->a.c * g * dJ;   // strict Armijo test (:361)
        }
        const unsigned long long okm = __ballot(ok);
        acc[1] += R2T_NOW() - tt;
        tt = R2T_NOW();
        // the first accepted trial, in order, handed from the deciding wavefront to the other so that both leave the
        // iteration loop together
        int first = okm ? __ffsll((long long)okm) - 1 : -1;
        lane_fence();   // the candidates' scratch stores, before the copy reads them
        if (wave == dec && lane == 0) shd[2] = (double)first;
        __syncthreads();
        first = (int)shd[2];
        const int nr = first >= 0 ? first + 1 : max_ls;
        if (first >= 0 && wave == 0) {   // the accepted candidate becomes the lane's next iterate (buffer cb ^ 1)
            const targs_t R = tail_args();
            const int T = R->N - 1;
            const int64_t vf = (int64_t)blockIdx.x * max_ls + first;
            for (int t0 = 0; t0 <= T; t0 += 4 * BLK) {   // four knots per thread in flight
                double2 a[4], b[4];
                double c0[4], c1[4];
#pragma unroll
                for (int j = 0; j < 4; ++j) {
                    const int t = t0 + j * BLK + lane;
                    if (t <= T) {
                        a[j] = R->sx[wix(t, 0, 2, vf, R->Vp)];
                        b[j] = R->sx[wix(t, 1, 2, vf, R->Vp)];
                    }
                    if (t < T) {
                        c0[j] = U0Z ? 0.0 : R->su[pix(t, 0, 2, vf, R->Vp)];
                        c1[j] = R->su[pix(t, 1, 2, vf, R->Vp)];
                    }
                }
#pragma unroll
                for (int j = 0; j < 4; ++j) {
                    const int t = t0 + j * BLK + lane;
                    if (t <= T) {
                        R->x[cb ^ 1][wix(t, 0, 2, l, R->Bp)] = a[j];
                        R->x[cb ^ 1][wix(t, 1, 2, l, R->Bp)] = b[j];
                    }
                    if (t < T) {
                        if (!U0Z) R->u[cb ^ 1][pix(t, 0, 2, l, R->Bp)] = c0[j];
                        R->u[cb ^ 1][pix(t, 1, 2, l, R->Bp)] = c1[j];
                    }
                }
            }
        }
        const int src = first >= 0 ? first : 0;
        const double Jf = __shfl(Jn, src);
        const double gf = __shfl(g, src);
        if (lane == 0 && wave == dec) {
            const targs_t F = tail_args();
            F->n_roll[l] += nr;
            F->n_iter[l] += 1;
            SolverCtl c = F->a;
            c.k = k;
            if (first >= 0)
                accept_lane(c, l, Jf, gf, sm, F->cost, F->gamma, F->status, F->res_buf, F->hist_cost, F->Bp);
            else
                fail_lane(c, l, F->status, F->res_buf);
        }
        st = first < 0 ? GYM_LS_FAILED : (sm < tail_args()->a.tol ? GYM_CONVERGED : GYM_ACTIVE);
        lane_fence();   // the next iterate and the lane's state visible to the next iteration
        __syncthreads();
        acc[2] += R2T_NOW() - tt;
    }
#ifdef GYM_TAIL_TRACE
    if (threadIdx.x == 0 && blockIdx.x < 4096)
        for (int i = 0; i < 4; ++i) g_tail_trace[blockIdx.x][i] += acc[i];
#endif
}

// ------------------------------------------------------------------------------------------
// Armijo gamma sweeps (plot_armijo_line_search :254-265): J(gamma_g) of the candidate rollout for G step
// sizes per lane, cost only, one thread per (lane, g).  The G blocks of one lane group re-read the same
// streams, so a group's blocks are mapped onto one XCD (blocks are dealt round-robin over the 8 XCDs) and
// run back to back there: the re-reads hit that XCD's L2.  gridDim.x is a multiple of 8.
// ------------------------------------------------------------------------------------------
__device__ __forceinline__ bool sweep_block(int G, int64_t groups, int64_t& grp, int& g) {
    const int64_t per = gridDim.x / 8;
    const int64_t i = (int64_t)(blockIdx.x % 8) * per + blockIdx.x / 8;
    grp = i / G;
    g = (int)(i % G);
    return grp < groups;
}

// reference form: full gains Kf (T,4,Bp), sigma planes, u_new = u + K (x_new - x) + gamma sigma
__global__ __launch_bounds__(BLK) void k_gamma_sweep(Dyn m, KW w, const double2* __restrict__ x,
                                                     const double* __restrict__ u, const double2* __restrict__ Kf,
                                                     const double* __restrict__ sig, const double* __restrict__ gammas,
                                                     int G, const double* __restrict__ xr,
                                                     const double* __restrict__ ur, double* __restrict__ cost_out,
                                                     int64_t B, int64_t Bp, int N) {
    int64_t grp;
    int g;
    if (!sweep_block(G, Bp / BLK, grp, g)) return;
    const int64_t l = grp * BLK + threadIdx.x;
    if (l >= B) {
        cost_out[(int64_t)g * Bp + l] = __builtin_nan("");
        return;
    }
    const double2 a = x[wix(0, 0, 2, l, Bp)], b = x[wix(0, 1, 2, l, Bp)];
    cost_out[(int64_t)g * Bp + l] = rollout_ref<true, false>(m, w, x, u, Kf, sig, xr, ur, nullptr, nullptr, gammas[g],
                                                             l, Bp, N, a.x, a.y, b.x, b.y);
}

// solver form: the Armijo trial's own rollout (offset form) on a batch's iteration-k streams; at the
// trial's step sizes the costs are bit-identical to the trial's.  Non-active lanes get NaN.
template <bool U0Z, bool RL>
__global__ __launch_bounds__(BLK) void k_nt_gamma_sweep(Dyn m, KW w, const double2* __restrict__ x,
                                                        const double* __restrict__ u, const double2* __restrict__ K1,
                                                        const double* __restrict__ cs, double g0,
                                                        const double* __restrict__ gammas, int G,
                                                        const double* __restrict__ xr, const double* __restrict__ ur,
                                                        const int32_t* __restrict__ status,
                                                        double* __restrict__ cost_out, int64_t B, int64_t Bp, int N) {
    int64_t grp;
    int g;
    if (!sweep_block(G, Bp / BLK, grp, g)) return;
    const int64_t l = grp * BLK + threadIdx.x;
    if (l >= B || status[l] != GYM_ACTIVE) {
        cost_out[(int64_t)g * Bp + l] = __builtin_nan("");
        return;
    }
    const double2 a = x[wix(0, 0, 2, l, Bp)], b = x[wix(0, 1, 2, l, Bp)];
    cost_out[(int64_t)g * Bp + l] = rollout_cform<false, U0Z, true, false, 0>(
        m, w, u, K1, cs, lane_ref<RL>(xr, l, 4 * (int64_t)N), lane_ref<RL>(ur, l, 2 * (int64_t)(N - 1)), nullptr,
        nullptr, gammas[g], g0, l, Bp, N, a.x, a.y, b.x, b.y);
}

// Deterministic two-stage statistics reduction (fixed lane->thread map, fixed trees).
__device__ __forceinline__ double wave_sum(double v) {
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) v += __shfl_down(v, off, 64);
    return v;
}

__global__ __launch_bounds__(STAT_THREADS) void k_stats_partial(const int32_t* __restrict__ status,
                                                                const double* __restrict__ cost,
                                                                const double* __restrict__ smax,
                                                                const int32_t* __restrict__ n_iter,
                                                                const int32_t* __restrict__ n_roll,
                                                                double* __restrict__ partials, Range rg, int k) {
    __shared__ double red[STAT_THREADS / 64][NSTAT];
    double acc[NSTAT] = {0, 0, 0, 0, 0, 0, 0, 0};
    const int64_t n = rg.hi - rg.lo;
    const int64_t chunk = (n + gridDim.x - 1) / gridDim.x;
    const int64_t lo = rg.lo + (int64_t)blockIdx.x * chunk;
    const int64_t hi = (lo + chunk < rg.hi) ? lo + chunk : rg.hi;
    for (int64_t l = lo + threadIdx.x; l < hi; l += STAT_THREADS) {
        const int st = status[l];
        const bool ran = n_iter[l] == k + 1;
        acc[0] += (st == GYM_ACTIVE) ? 1.0 : 0.0;
        acc[1] += cost[l];
        acc[2] += ran ? smax[l] * smax[l] : 0.0;
        acc[3] += ran ? 1.0 : 0.0;
        acc[5] += (st == GYM_CONVERGED) ? 1.0 : 0.0;
        acc[6] += (st == GYM_LS_FAILED) ? 1.0 : 0.0;
        acc[7] += (double)n_roll[l];
    }
    const int wv = threadIdx.x / 64, ln = threadIdx.x % 64;
#pragma unroll
    for (int s = 0; s < NSTAT; ++s) {
        const double v = wave_sum(acc[s]);
        if (ln == 0) red[wv][s] = v;
    }
    __syncthreads();
    if (threadIdx.x < NSTAT) {
        double v = 0.0;
        for (int q = 0; q < STAT_THREADS / 64; ++q) v += red[q][threadIdx.x];
        partials[(int64_t)blockIdx.x * NSTAT + threadIdx.x] = v;
    }
}

// stats_out[0..7] = this range's statistics; if other != NULL, total[s] = other[s] + stats_out[s].
// One wavefront per statistic: lane i adds partials i, i+64, ... in order, then a fixed shuffle tree.
__global__ __launch_bounds__(64 * NSTAT) void k_stats_final(const double* __restrict__ partials,
                                                            int32_t* __restrict__ counter,
                                                            double* __restrict__ stats_out,
                                                            const double* __restrict__ other,
                                                            double* __restrict__ total, int nblocks) {
    const int s = threadIdx.x / 64, ln = threadIdx.x % 64;
    double v = 0.0;
    for (int b = ln; b < nblocks; b += 64) v += partials[(int64_t)b * NSTAT + s];
    v = wave_sum(v);
    if (ln == 0) {
        if (s == 4) v = (double)(*counter);
        stats_out[s] = v;
        if (other) total[s] = other[s] + v;
    }
    __syncthreads();
    if (threadIdx.x == 0) *counter = 0;  // the retry list is rebuilt every iteration
}

// sigma1 re-run: the sweep of an earlier pass, recomputed (same inputs, same code: the same bits) into the
// sigma1 plane.  retry mode (list != nullptr): the lanes list[0 .. *count) at the iterate (x, u); final mode:
// the lanes whose last iteration started from this buffer, (n_iter - 1) & 1 == parity (one launch per
// buffer, so the streams' base addresses stay wave-uniform).
template <bool U0Z, bool CK, bool RL = false>
__global__ __launch_bounds__(BLK, 4) void k_nt_sigma(Dyn m, KW w, const double2* __restrict__ x,
                                                     const double* __restrict__ u, const double* __restrict__ xr,
                                                     const double* __restrict__ ur, double* __restrict__ cs,
                                                     const int32_t* __restrict__ list, const int32_t* __restrict__ count,
                                                     const int32_t* __restrict__ n_iter, int parity, int64_t B,
                                                     int64_t Bp, int N) {
    GYM_CK_LDS(CK, U0Z);
    const int64_t n = list ? (int64_t)*count : B;
    for (int64_t i = (int64_t)blockIdx.x * BLK + threadIdx.x; i < n; i += (int64_t)gridDim.x * BLK) {
        const int64_t l = list ? (int64_t)list[i] : i;
        if (!list) {
            const int it = n_iter[l];
            if (it <= 0 || ((it - 1) & 1) != parity) continue;
        }
        backward_solver<U0Z, CK, OUT_SIGMA>(m, w, x, u, lane_ref<RL>(xr, l, 4 * (int64_t)N),
                                            lane_ref<RL>(ur, l, 2 * (int64_t)(N - 1)), nullptr, cs, 0.0, nullptr,
                                            nullptr, nullptr, l, Bp, N, 0, 0, ck_lds);
    }
}

__global__ void k_finalize_status(int32_t* __restrict__ status, int32_t* __restrict__ res_buf, int64_t B, int k_done) {
    const int64_t l = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (l >= B) return;
    if (status[l] == GYM_ACTIVE) {
        status[l] = GYM_MAX_ITERS;
        res_buf[l] = k_done & 1;
    }
}


// GYM_FLAG_X_CKPT: rebuild every knot of a state buffer from x_0 and the tau2 controls, x_{t+1} =
// RK4(x_t, u1_t) -- the same recursion (and code) the trial ran, so the rebuilt knots equal the bits it
// would have stored and the checkpoints are rewritten unchanged.  sel_buf < 0: lane l's res_buf.
__global__ __launch_bounds__(BLK) void k_fill_states(Dyn m, double2* __restrict__ x0b, double2* __restrict__ x1b,
                                                     const double* __restrict__ u0b, const double* __restrict__ u1b,
                                                     const int32_t* __restrict__ res_buf, int sel_buf, int64_t B,
                                                     int64_t Bp, int N) {
    const int64_t l = (int64_t)blockIdx.x * BLK + threadIdx.x;
    if (l >= B) return;
    const int sel = sel_buf >= 0 ? sel_buf : res_buf[l];
    double2* xs = sel ? x1b : x0b;
    const double* us = sel ? u1b : u0b;
    const double2 a = xs[wix(0, 0, 2, l, Bp)], b = xs[wix(0, 1, 2, l, Bp)];
    double n0 = a.x, n1 = a.y, n2 = b.x, n3 = b.y;
    for (int t = 0; t < N - 1; ++t) {
        gym::rk4(m, n0, n1, n2, n3, us[pix(t, 1, 2, l, Bp)]);
        st_nt(xs + wix(t + 1, 0, 2, l, Bp), n0, n1);
        st_nt(xs + wix(t + 1, 1, 2, l, Bp), n2, n3);
    }
}

// The kinds timed at every launch (pool pairs): the solver's main kernels (sweep, trial, phase, run, tail), whose
// average duration is the roofline's denominator.  The short post-trial kernels (candidates, retry, statistics,
// sigma1 re-run: five per phase) keep one sampled pair per kind and collect: an event pair around each of them
// lengthened the phase-to-phase gap from ~28 to ~73 us in the rocprofv3 trace (+1-2% per solve).
constexpr int TIMING_POOL_KINDS = (1 << 0) | (1 << 1) | (1 << 5) | (1 << 6) | (1 << 8) | (1 << 9);
struct TimedLaunch {  // records a start/stop event pair around one launch: a pool pair, else the kind's free slot
    gym_timing* t;
    int kind;
    hipStream_t s;
    int slot;            // pool index, -1: the kind's sampled pair, -2: not timed
    TimedLaunch(gym_timing* t_, int kind_, hipStream_t s_) : t(t_), kind(kind_), s(s_), slot(-2) {
        if (!t) return;
        if (((TIMING_POOL_KINDS >> kind) & 1) && t->pool_used < GYM_TIMING_POOL && t->pool_ev[0]) {
            slot = t->pool_used++;
            t->pool_kind[slot] = kind;
            (void)hipEventRecord((hipEvent_t)t->pool_ev[2 * slot], s);
        } else if (!(t->pending & (1 << kind))) {
            slot = -1;
            (void)hipEventRecord((hipEvent_t)t->ev[2 * kind], s);
        }
    }
    ~TimedLaunch() {
        if (slot >= 0) {
            (void)hipEventRecord((hipEvent_t)t->pool_ev[2 * slot + 1], s);
        } else if (slot == -1) {
            (void)hipEventRecord((hipEvent_t)t->ev[2 * kind + 1], s);
            t->pending |= 1 << kind;
        }
    }
};

// kernel instantiation for the batch's tau1 mode (GYM_FLAG_U0_ZERO)
#define U0Z_SEL(b, kern) (((b)->flags & GYM_FLAG_U0_ZERO) ? kern<true> : kern<false>)
// ... and its state-checkpointing mode (GYM_FLAG_X_CKPT)
#define SOLVER_SEL(b, kern)                                                                               \
    (((b)->flags & GYM_FLAG_U0_ZERO) ? (((b)->flags & GYM_FLAG_X_CKPT) ? kern<true, true> : kern<true, false>) \
                                     : (((b)->flags & GYM_FLAG_X_CKPT) ? kern<false, true> : kern<false, false>))

// ... and per-lane references (GYM_FLAG_REF_LANE; never with X_CKPT), for the serial / pipelined kernels
#define SERIAL_SEL(b, kern)                                                                                      \
    (((b)->flags & GYM_FLAG_REF_LANE) ? (((b)->flags & GYM_FLAG_U0_ZERO) ? kern<true, false, true>              \
                                                                          : kern<false, false, true>)           \
                                      : SOLVER_SEL(b, kern))
#define RUN_SEL(b, kern) CAND_SEL(b, kern)   // the persistent kernels: <U0Z, RL>
// the two-wavefront phase kernel (k_nt_phase<..., LO = true>; never with X_CKPT)
#define PHASE_LO_SEL(b)                                                                                          \
    (((b)->flags & GYM_FLAG_REF_LANE) ? (((b)->flags & GYM_FLAG_U0_ZERO) ? k_nt_phase<true, false, true, true>  \
                                                                          : k_nt_phase<false, false, true, true>) \
                                      : (((b)->flags & GYM_FLAG_U0_ZERO) ? k_nt_phase<true, false, false, true> \
                                                                          : k_nt_phase<false, false, false, true>))
#define CAND_SEL(b, kern)                                                                                        \
    (((b)->flags & GYM_FLAG_REF_LANE) ? (((b)->flags & GYM_FLAG_U0_ZERO) ? kern<true, true> : kern<false, true>) \
                                      : (((b)->flags & GYM_FLAG_U0_ZERO) ? kern<true, false> : kern<false, false>))

inline bool bad_dims(int64_t B, int64_t Bp, int N) {
    return B <= 0 || Bp < B || (Bp % 64) != 0 || Bp > GYM_MAX_BP || N < 2;
}

inline int launch_status() { return (int)hipGetLastError(); }

template <class Src>
int launch_unpack_tiled(const Src& src, double* dst, int64_t B, int64_t Bp, int L, int C, hipStream_t st,
                        const int64_t* map = nullptr) {
    const int ts = tile_knots(C);
    if (C * TILE_PITCH > TILE_DOUBLES) return GYM_EINVAL;
    const dim3 grid((unsigned)(Bp / BLK), (unsigned)((L + ts - 1) / ts));
    const size_t lds = sizeof(double) * ts * C * TILE_PITCH;
    if (C == 2)
        hipLaunchKernelGGL((k_unpack_tiled<Src, 2>), grid, dim3(TILE_THREADS), lds, st, src, dst, map, B, Bp, L, C, ts);
    else if (C == 4)
        hipLaunchKernelGGL((k_unpack_tiled<Src, 4>), grid, dim3(TILE_THREADS), lds, st, src, dst, map, B, Bp, L, C, ts);
    else if (C == 8)
        hipLaunchKernelGGL((k_unpack_tiled<Src, 8>), grid, dim3(TILE_THREADS), lds, st, src, dst, map, B, Bp, L, C, ts);
    else
        hipLaunchKernelGGL((k_unpack_tiled<Src, 0>), grid, dim3(TILE_THREADS), lds, st, src, dst, map, B, Bp, L, C, ts);
    return launch_status();
}

inline Mat4 mat4(const double* p) { Mat4 m; for (int i = 0; i < 16; ++i) m.v[i] = p[i]; return m; }
inline Mat2 mat2(const double* p) { Mat2 m; for (int i = 0; i < 4; ++i) m.v[i] = p[i]; return m; }

}  // namespace

// ==========================================================================================
// C-ABI
// ==========================================================================================
extern "C" {

int gym_abi_version(void) { return GYM_ABI_VERSION; }

// _build.source_hash() of the sources this library was compiled from (-DGYM_BUILD_ID); the tag lets the build
// script read it from the file without loading the library
#ifndef GYM_BUILD_ID
#define GYM_BUILD_ID "unversioned"
#endif
static const char gym_build_id_tagged[] = "gym-build-id:" GYM_BUILD_ID;
const char* gym_build_id(void) { return gym_build_id_tagged + sizeof("gym-build-id:") - 1; }

int gym_model_from_params(const double p[11], double dt, gym_model* out) {
    if (!p || !out) return GYM_EINVAL;
    const double m1 = p[0], m2 = p[1], l1 = p[2], lc1 = p[3], lc2 = p[5], I1 = p[6], I2 = p[7], g = p[8];
    out->a = I1 + I2 + lc1 * lc1 * m1 + m2 * (l1 * l1 + lc2 * lc2);
    out->b = m2 * l1 * lc2;
    out->d = I2 + lc2 * lc2 * m2;
    out->g1 = g * (lc1 * m1 + m2 * l1);
    out->g2 = g * m2 * lc2;
    out->f1 = p[9];
    out->f2 = p[10];
    out->dt = dt;
    return 0;
}

static int point_op(const gym_model* m, const double* x, const double* u, double* o1, double* o2, int64_t n, void* s,
                    int what) {
    if (!m || !x || !u || !o1 || n < 0 || (what == 2 && !o2)) return GYM_EINVAL;
    if (n == 0) return 0;
    hipLaunchKernelGGL(k_point, dim3(grid_for(n, 256)), dim3(256), 0, (hipStream_t)s, Dyn(*m), x, u, o1, o2, n, what);
    return launch_status();
}

int gym_continuous_dynamics(const gym_model* m, const double* x, const double* u, double* xdot, int64_t n, void* s) {
    return point_op(m, x, u, xdot, nullptr, n, s, 0);
}
int gym_rk4_step(const gym_model* m, const double* x, const double* u, double* xnext, int64_t n, void* s) {
    return point_op(m, x, u, xnext, nullptr, n, s, 1);
}
int gym_jacobians(const gym_model* m, const double* x, const double* u, double* A, double* Bc, int64_t n, void* s) {
    return point_op(m, x, u, A, Bc, n, s, 2);
}

int gym_stage_cost_derivs(const double* x, const double* xr, const double* u, const double* ur, const double Q[16],
                          const double R[4], int32_t terminal, double* l, double* gx, double* gu, int64_t n,
                          void* s) {
    if (!x || !xr || !Q || !l || !gx || n < 0) return GYM_EINVAL;
    if (!terminal && (!u || !ur || !R || !gu)) return GYM_EINVAL;
    if (n == 0) return 0;
    const double zero4[4] = {0, 0, 0, 0};
    hipLaunchKernelGGL(k_stage_cost_derivs, dim3(grid_for(n, 256)), dim3(256), 0, (hipStream_t)s, x, xr, u, ur,
                       mat4(Q), mat2(R ? R : zero4), (int)terminal, l, gx, gu, n);
    return launch_status();
}

int gym_pack_lanes(const double* src, double* dst, int64_t B, int64_t Bp, int32_t L, int32_t C, int32_t W, void* s) {
    if (!src || !dst || bad_dims(B, Bp, 2) || L <= 0 || C <= 0 || (W != 1 && W != 2) || (C % W)) return GYM_EINVAL;
    const int64_t n = (int64_t)L * (C / W) * Bp;
    hipLaunchKernelGGL(k_pack, dim3(grid_for(n, 256)), dim3(256), 0, (hipStream_t)s, src, dst, B, Bp, L, C, W);
    return launch_status();
}

int gym_unpack_lanes(const double* s0, const double* s1, const int32_t* sel, double* dst, int64_t B, int64_t Bp,
                     int32_t L, int32_t C, int32_t W, void* s) {
    if (!s0 || !dst || bad_dims(B, Bp, 2) || L <= 0 || C <= 0 || (W != 1 && W != 2) || (C % W) || (sel && !s1))
        return GYM_EINVAL;
    if (W == 2)
        return launch_unpack_tiled(SrcPairs{(const double2*)s0, (const double2*)(s1 ? s1 : s0), sel, C / 2}, dst, B,
                                   Bp, L, C, (hipStream_t)s);
    return launch_unpack_tiled(SrcPlanes{s0, s1 ? s1 : s0, sel, C}, dst, B, Bp, L, C, (hipStream_t)s);
}

int gym_unpack_gains(const double* K1, double* K, int64_t B, int64_t Bp, int32_t T, void* s) {
    if (!K1 || !K || bad_dims(B, Bp, 2) || T <= 0) return GYM_EINVAL;
    return launch_unpack_tiled(SrcGains{(const double2*)K1}, K, B, Bp, T, 8, (hipStream_t)s);
}

int gym_rollout_open_loop(const gym_model* m, const gym_weights* w, const double* x0, const double* u,
                          const double* xr, const double* ur, double* x, double* cost, int64_t B, int64_t Bp,
                          int32_t N, void* s) {
    if (!m || !w || !x0 || !u || !xr || !ur || !x || bad_dims(B, Bp, N)) return GYM_EINVAL;
    hipLaunchKernelGGL(k_open_loop, dim3(grid_for(B, BLK)), dim3(BLK), 0, (hipStream_t)s, Dyn(*m), kw(*w), x0, u, xr, ur,
                       (double2*)x, cost, B, Bp, N);
    return launch_status();
}

int gym_closed_loop(const gym_model* m, const gym_weights* w, const double* x, const double* u, const double* Kf,
                    const double* sigma, const double* gamma, const double* xr, const double* ur, double* xn,
                    double* un, double* cost, int64_t B, int64_t Bp, int32_t N, void* s) {
    if (!m || !w || !x || !u || !Kf || !sigma || !gamma || !xr || !ur || !xn || !un || bad_dims(B, Bp, N))
        return GYM_EINVAL;
    hipLaunchKernelGGL(k_closed_loop, dim3(grid_for(B, BLK)), dim3(BLK), 0, (hipStream_t)s, Dyn(*m), kw(*w),
                       (const double2*)x, u, (const double2*)Kf, sigma, gamma, xr, ur, (double2*)xn, un, cost, B, Bp,
                       N);
    return launch_status();
}

int gym_total_cost(const double* x, const double* u, const double* xr, const double* ur, const double Q[16],
                   const double R[4], const double QT[16], double* cost, int64_t B, int64_t Bp, int32_t N, void* s) {
    if (!x || !u || !xr || !ur || !Q || !R || !QT || !cost || bad_dims(B, Bp, N)) return GYM_EINVAL;
    hipLaunchKernelGGL(k_total_cost, dim3(grid_for(B, BLK)), dim3(BLK), 0, (hipStream_t)s, (const double2*)x, u, xr,
                       ur, mat4(Q), mat2(R), mat4(QT), cost, B, Bp, N);
    return launch_status();
}

int gym_backward_sweep(const gym_model* m, const gym_weights* w, const double* x, const double* u, const double* xr,
                       const double* ur, double* K1, double* sigma, double* dJ, double* smax, double* lambda, int64_t B,
                       int64_t Bp, int32_t N, void* s) {
    if (!m || !w || !x || !u || !xr || !ur || !K1 || !sigma || bad_dims(B, Bp, N)) return GYM_EINVAL;
    hipLaunchKernelGGL(k_backward_api, dim3(grid_for(B, BLK)), dim3(BLK), 0, (hipStream_t)s, Dyn(*m), kw(*w),
                       (const double2*)x, u, xr, ur, (double2*)K1, sigma, dJ, smax, (double2*)lambda, B, Bp, N);
    return launch_status();
}

int gym_linearize(const gym_model* m, const gym_weights* w, const double* x, const double* u, const double* xr,
                  const double* ur, double* Ad, double* Bd, double* q, double* r, double* qT, int64_t B, int64_t Bp,
                  int32_t N, void* s) {
    if (!m || !w || !x || !u || !xr || !ur || !Ad || !Bd || !q || !r || !qT || bad_dims(B, Bp, N)) return GYM_EINVAL;
    hipLaunchKernelGGL(k_linearize, dim3(grid_for(B, BLK)), dim3(BLK), 0, (hipStream_t)s, Dyn(*m), kw(*w), (const double2*)x, u,
                       xr, ur, Ad, Bd, q, r, qT, B, Bp, N);
    return launch_status();
}

int gym_riccati_general(const double* A, const double* Bm, const double* Q, const double* R, const double* S,
                        const double* q, const double* r, const double* QT, const double* qT, double* K, double* sigma,
                        double* dJ, int64_t B, int64_t Bp, int32_t T, void* s) {
    if (!A || !Bm || !Q || !R || !S || !q || !r || !QT || !qT || !K || !sigma || !dJ || bad_dims(B, Bp, T + 1))
        return GYM_EINVAL;
    hipLaunchKernelGGL(k_riccati_general, dim3(grid_for(B, BLK)), dim3(BLK), 0, (hipStream_t)s, A, Bm, Q, R, S, q, r,
                       QT, qT, K, sigma, dJ, B, Bp, T);
    return launch_status();
}

// every batch entry point: the buffers, the sizes and the flag combination (per-lane references are never
// combined with state checkpointing: no kernel instantiates both)
static bool bad_batch(const gym_batch* b) {
    return !b || bad_dims(b->B, b->Bp, b->N) || (b->cand_scratch && (b->cand_slots < 0 || b->cand_slots % BLK != 0 ||
                                                                    b->cand_slots > GYM_MAX_BP)) || !b->x[0] || !b->x[1] || !b->u[0] || !b->u[1] || !b->K1 || !b->cs ||
           !b->x_ref || !b->u_ref || !b->cost || !b->dJ || !b->smax || !b->gamma || !b->status || !b->n_iter ||
           !b->res_buf || !b->n_roll || !b->retry_list || !b->counters || !b->partials || !b->stats ||
           ((b->flags & GYM_FLAG_REF_LANE) && (b->flags & GYM_FLAG_X_CKPT));
}

int gym_newton_init(const gym_model* m, const gym_weights* w, const double* x0, const gym_batch* b, void* s) {
    if (!m || !w || !x0 || bad_batch(b)) return GYM_EINVAL;
    hipStream_t st = (hipStream_t)s;
    const int T = b->N - 1;
    hipError_t e = hipMemsetAsync(b->u[0], 0, sizeof(double) * 2 * (size_t)T * b->Bp, st);
    if (e != hipSuccess) return (int)e;
    if (b->flags & GYM_FLAG_U0_ZERO) {  // the trials never write the u0 planes: keep both buffers' zero
        e = hipMemsetAsync(b->u[1], 0, sizeof(double) * 2 * (size_t)T * b->Bp, st);
        if (e != hipSuccess) return (int)e;
    }
    e = hipMemsetAsync(b->counters, 0, sizeof(int32_t) * 4, st);
    if (e != hipSuccess) return (int)e;
    e = hipMemsetAsync(b->stats, 0, sizeof(double) * 24, st);
    if (e != hipSuccess) return (int)e;
    hipLaunchKernelGGL(((b->flags & GYM_FLAG_REF_LANE) ? k_init<true> : k_init<false>), dim3(grid_for(b->Bp, BLK)),
                       dim3(BLK), 0, st, Dyn(*m), kw(*w), x0, b->u[0], b->x_ref, b->u_ref,
                       (double2*)b->x[0], b->cost, b->status, b->n_iter, b->res_buf, b->n_roll, b->gamma, b->smax,
                       b->dJ, b->B, b->Bp, b->N);
    return launch_status();
}

// Grid caps of the post-trial kernels (grid-stride over the retry list; any cap is correct).  They launch every
// phase, also when no lane rejected trial 1 (the device-side count is not known to the host).  Lower caps (256 /
// 64) measured the same at 262,144 lanes and 2% slower on the stress start: the gap between phases is
// launch latency, not workgroup dispatch.
constexpr int64_t POST_CAP = 2048;
constexpr int64_t CAND_CAP = 4096;
// the candidate scratch of the batch (gym_batch.cand_scratch): none without lane-pair candidates or with state
// checkpointing (whose accepted re-run stores the checkpoint knots only)
static CandScratch cand_scratch(const gym_batch* b, bool pair) {
    CandScratch c{nullptr, nullptr, nullptr, 0};
    if (!pair || !b->cand_scratch || b->cand_slots <= 0 || (b->flags & GYM_FLAG_X_CKPT)) return c;
    const int64_t V = b->cand_slots, N = b->N;
    c.sx = (double2*)b->cand_scratch;
    c.su = b->cand_scratch + 4 * N * V;
    c.sJ = c.su + 2 * (N - 1) * V;
    c.V = V;
    return c;
}
static void launch_post_trial(const gym_model* m, const gym_weights* w, const gym_armijo* a, const gym_batch* b,
                              const SolverCtl& c, const TrialIO& io, Range rg, int32_t* counter, double* stats_out,
                              const double* other, double* total, hipStream_t st, bool sigma_streamed = false) {
    const int64_t n = rg.hi - rg.lo;
    const double2* K1 = (const double2*)b->K1;
    const double* cs = b->cs;
    double* hc = a->record_history ? b->hist_cost : nullptr;
    if (a->max_ls > 1 && n > 0) {
        if (!sigma_streamed) {   // the lanes that reject trial 1 need sigma1: re-run their sweep into its plane
            TimedLaunch tl(b->timing, 7, st);
            hipLaunchKernelGGL(SERIAL_SEL(b, k_nt_sigma), dim3(grid_for(n, BLK, POST_CAP)), dim3(BLK), 0, st, Dyn(*m),
                               kw(*w), io.x, io.u, b->x_ref, b->u_ref, b->cs, b->retry_list + rg.lo, counter,
                               (const int32_t*)nullptr, -1, b->B, b->Bp, b->N);
        }
        // candidates on lane pairs (recorded in the scratch slots, if any) unless single-lane chains were asked for
        const bool pair = !(b->flags & GYM_FLAG_RUN_SINGLE);
        const CandScratch sc = cand_scratch(b, pair);
        const int64_t ncand = n * (int64_t)(a->max_ls - 1);
        {
            TimedLaunch tl(b->timing, 2, st);
            if (pair)
                hipLaunchKernelGGL(CAND_SEL(b, k_nt_cand_pair), dim3(grid_for(2 * ncand, BLK, CAND_CAP)), dim3(BLK), 0,
                                   st, Dyn(*m), kw(*w), c, io, K1, cs, b->x_ref, b->u_ref, b->cost, b->dJ,
                                   b->retry_list + rg.lo, counter, b->cand_ok, sc, b->Bp, b->N);
            else
                hipLaunchKernelGGL(CAND_SEL(b, k_nt_candidates), dim3(grid_for(ncand, BLK, CAND_CAP)), dim3(BLK), 0,
                                   st, Dyn(*m), kw(*w), c, io, K1, cs, b->x_ref, b->u_ref, b->cost, b->dJ,
                                   b->retry_list + rg.lo, counter, b->cand_ok, b->Bp, b->N);
        }
        const int64_t items = sc.V > 0 ? n * (1 + (b->N + CPK - 1) / CPK) : n;
        TimedLaunch tl(b->timing, 3, st);
        hipLaunchKernelGGL(SERIAL_SEL(b, k_nt_retry), dim3(grid_for(items, BLK, POST_CAP)), dim3(BLK), 0, st, Dyn(*m),
                           kw(*w), c, io, K1, cs, b->x_ref, b->u_ref, b->cost, b->smax, b->gamma, b->status, b->n_iter,
                           b->res_buf, b->n_roll, b->retry_list + rg.lo, counter, b->cand_ok, hc, sc, b->Bp, b->N);
    }
    TimedLaunch tl(b->timing, 4, st);
    hipLaunchKernelGGL(k_stats_partial, dim3(STAT_BLOCKS), dim3(STAT_THREADS), 0, st, b->status, b->cost, b->smax,
                       b->n_iter, b->n_roll, b->partials, rg, c.k);
    hipLaunchKernelGGL(k_stats_final, dim3(1), dim3(64 * NSTAT), 0, st, b->partials, counter, stats_out, other, total,
                       STAT_BLOCKS);
}

static TrialIO trial_io(const gym_batch* b, int k) {
    return TrialIO{(const double2*)b->x[k & 1], b->u[k & 1], (double2*)b->x[(k + 1) & 1], b->u[(k + 1) & 1]};
}

static bool bad_iter_args(const gym_model* m, const gym_weights* w, const gym_armijo* a, const gym_batch* b) {
    return !m || !w || !a || bad_batch(b) || a->max_ls < 1 || (a->max_ls > 1 && !b->cand_ok);
}

int gym_newton_iteration(const gym_model* m, const gym_weights* w, const gym_armijo* a, const gym_batch* b, int32_t k,
                         void* s) {
    if (bad_iter_args(m, w, a, b) || k < 0) return GYM_EINVAL;
    hipStream_t st = (hipStream_t)s;
    const Range all{0, b->B};
    const TrialIO io = trial_io(b, k);
    const int grid = grid_for(b->B, BLK);
    const bool hist = a->record_history != 0;
    // GYM_FLAG_SIGMA_STREAM: the sweep also stores sigma1 (8 B per stage), so the lanes that reject trial 1 need no
    // re-run of it (a chain as long as the sweep's, for however few lanes)
    const bool sig = (b->flags & GYM_FLAG_SIGMA_STREAM) != 0;
    {
        TimedLaunch tl(b->timing, 0, st);
        hipLaunchKernelGGL(sig ? SERIAL_SEL(b, k_nt_backward_all) : SERIAL_SEL(b, k_nt_backward), dim3(grid),
                           dim3(BLK), 0, st, Dyn(*m), kw(*w), io.x, io.u, b->x_ref, b->u_ref,
                           (double2*)b->K1, b->cs, a->gamma0, b->dJ, b->smax, b->status,
                           hist ? b->hist_smax : nullptr, all, b->Bp, b->N, k, b->hist_len);
    }
    const SolverCtl c{a->tol, a->beta, a->c, a->gamma0, a->max_ls, k, b->hist_len, 0};
    {
        TimedLaunch tl(b->timing, 1, st);
        hipLaunchKernelGGL(SERIAL_SEL(b, k_nt_trial), dim3(grid), dim3(BLK), 0, st, Dyn(*m), kw(*w), c, io, (const double2*)b->K1,
                           (const double*)b->cs, b->x_ref, b->u_ref, b->cost, b->dJ, b->smax, b->gamma, b->status,
                           b->n_iter, b->res_buf, b->n_roll, b->retry_list, b->counters, hist ? b->hist_cost : nullptr,
                           all, b->Bp, b->N);
    }
    launch_post_trial(m, w, a, b, c, io, all, b->counters, b->stats, nullptr, nullptr, st, sig);
    return launch_status();
}

// compute units of the current device (cached per device index; 0 if the query fails)
static int device_cus() {
    static int cache[64] = {0};
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return 0;
    if (!cache[dev]) {
        int n = 0;
        if (hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) == hipSuccess) cache[dev] = n;
    }
    return cache[dev];
}

// The phase kernel for a launch of `waves` wavefronts: the two-wavefront build (k_nt_phase<..., LO>) when the
// launch fills the SIMDs with between LO_MIN_EIGHTHS/8 and two wavefronts each (profiles/r06/README.md "pd2":
// same-buffer A/B over batch sizes), the four-wavefront build otherwise.
constexpr int LO_MIN_EIGHTHS = 14;
static bool phase_low_occupancy(const gym_batch* b, int64_t waves) {
    if (b->flags & GYM_FLAG_X_CKPT) return false;
    const int64_t simds = 4 * (int64_t)device_cus();
    return simds > 0 && 8 * waves > LO_MIN_EIGHTHS * simds && waves <= 2 * simds;
}

int gym_newton_phase_kind(const gym_batch* b, int32_t* low_out) {
    if (bad_batch(b) || !low_out) return GYM_EINVAL;
    int64_t Bh;
    gym_newton_pipeline_split(b, &Bh);
    const int64_t waves = (Bh + BLK - 1) / BLK + (b->B - Bh + BLK - 1) / BLK;
    *low_out = phase_low_occupancy(b, waves) ? 1 : 0;
    return 0;
}

int gym_newton_pipeline_split(const gym_batch* b, int64_t* Bh) {
    if (!b || !Bh || b->B <= 0) return GYM_EINVAL;
    int64_t h = ((b->B + 1) / 2 + 63) / 64 * 64;
    *Bh = h < b->B ? h : b->B;
    return 0;
}

int gym_newton_phase(const gym_model* m, const gym_weights* w, const gym_armijo* a, const gym_batch* b, int32_t p,
                     int32_t do_backward, void* s) {
    if (bad_iter_args(m, w, a, b) || p < 0) return GYM_EINVAL;
    hipStream_t st = (hipStream_t)s;
    int64_t Bh;
    gym_newton_pipeline_split(b, &Bh);
    const Range half[2] = {{0, Bh}, {Bh, b->B}};
    const bool hist = a->record_history != 0;
    // backward half: H0 on even phases (iteration p/2), H1 on odd phases (iteration (p-1)/2)
    const int hb = p & 1, kb = p >> 1;
    const Range rb = do_backward ? half[hb] : Range{0, 0};
    // trial half: H0 on odd phases (iteration (p-1)/2), H1 on even phases >= 2 (iteration (p-2)/2)
    const int ht = (p & 1) ? 0 : 1;
    const int kt = (p & 1) ? (p - 1) >> 1 : (p - 2) >> 1;
    const Range rt = (p >= 1) ? half[ht] : Range{0, 0};
    const int nb_b = (int)((rb.hi - rb.lo + BLK - 1) / BLK), nb_t = (int)((rt.hi - rt.lo + BLK - 1) / BLK);
    const SolverCtl c{a->tol, a->beta, a->c, a->gamma0, a->max_ls, kt < 0 ? 0 : kt, b->hist_len, 0};
    const TrialIO io = trial_io(b, kt < 0 ? 0 : kt);
    if (nb_b + nb_t > 0) {
        TimedLaunch tl(b->timing, (p & 1) ? 5 : 6, st);
        PhaseArgs pa;
        pa.m = Dyn(*m);
        pa.w = kw(*w);
        pa.a = c;
        pa.io = io;
        pa.xb_in = (const double2*)b->x[kb & 1]; pa.ub_in = b->u[kb & 1];
        pa.K1 = (double2*)b->K1; pa.cs = b->cs; pa.xr = b->x_ref; pa.ur = b->u_ref;
        pa.cost = b->cost; pa.dJ = b->dJ; pa.smax = b->smax; pa.gamma = b->gamma;
        pa.status = b->status; pa.n_iter = b->n_iter; pa.res_buf = b->res_buf; pa.n_roll = b->n_roll;
        pa.retry_list = b->retry_list; pa.counter = b->counters + ht;
        pa.hist_cost = hist ? b->hist_cost : nullptr; pa.hist_smax = hist ? b->hist_smax : nullptr;
        pa.rb = rb; pa.rt = rt; pa.Bp = b->Bp; pa.N = b->N; pa.kb = kb; pa.nb_b = nb_b; pa.pad = 0;
        hipLaunchKernelGGL(phase_low_occupancy(b, nb_b + nb_t) ? PHASE_LO_SEL(b) : SERIAL_SEL(b, k_nt_phase),
                           dim3(nb_b + nb_t), dim3(BLK), 0, st, pa);
    }
    if (p >= 1)  // the trial half's retries and statistics; H1 closes the iteration: total = H0 + H1
        launch_post_trial(m, w, a, b, c, io, rt, b->counters + ht, b->stats + 8 + 8 * ht,
                          ht ? b->stats + 8 : nullptr, ht ? b->stats : nullptr, st);
    return launch_status();
}

int gym_newton_run(const gym_model* m, const gym_weights* w, const gym_armijo* a, const gym_batch* b, int32_t k0,
                   int32_t k1, void* s) {
    // GYM_FLAG_SIGMA_STREAM with the four-wavefront kernel: one iteration per launch, its sweep storing sigma1, the
    // lanes that reject trial 1 finished by the serial schedule's parallel candidates and accepted re-run
    const bool ext = (b->flags & GYM_FLAG_SIGMA_STREAM) && !(b->flags & GYM_FLAG_RUN_SINGLE);
    if (bad_iter_args(m, w, a, b) || k0 < 0 || k1 < k0 || (b->flags & GYM_FLAG_X_CKPT) || (ext && k1 > k0 + 1))
        return GYM_EINVAL;
    hipStream_t st = (hipStream_t)s;
    const bool hist = a->record_history != 0;
    const SolverCtl c{a->tol, a->beta, a->c, a->gamma0, a->max_ls, k0, b->hist_len, 0};
    if (ext) {
        if (k1 > k0) {
            TimedLaunch tl(b->timing, 8, st);
            RunArgs ra;
            ra.m = Dyn(*m);
            ra.w = kw(*w);
            ra.a = c;
            for (int i = 0; i < 2; ++i) { ra.x[i] = (double2*)b->x[i]; ra.u[i] = b->u[i]; }
            ra.K1 = (double2*)b->K1; ra.cs = b->cs; ra.xr = b->x_ref; ra.ur = b->u_ref;
            ra.cost = b->cost; ra.dJ = b->dJ; ra.smax = b->smax; ra.gamma = b->gamma;
            ra.status = b->status; ra.n_iter = b->n_iter; ra.res_buf = b->res_buf; ra.n_roll = b->n_roll;
            ra.hist_cost = hist ? b->hist_cost : nullptr; ra.hist_smax = hist ? b->hist_smax : nullptr;
            ra.retry_list = b->retry_list; ra.counter = b->counters;
            ra.B = b->B; ra.Bp = b->Bp; ra.N = b->N; ra.k0 = k0; ra.k1 = k1; ra.ext = 1;
            hipLaunchKernelGGL(RUN_SEL(b, k_nt_run2), dim3((unsigned)(b->Bp / BLK)), dim3(R2WAVES * BLK), 0, st, ra);
            launch_post_trial(m, w, a, b, c, trial_io(b, k0), Range{0, b->B}, b->counters, b->stats, nullptr,
                              nullptr, st, true);
            return launch_status();
        }
    }
    if (k1 > k0) {
        TimedLaunch tl(b->timing, 8, st);
        RunArgs ra;
        ra.m = Dyn(*m);
        ra.w = kw(*w);
        ra.a = c;
        for (int i = 0; i < 2; ++i) { ra.x[i] = (double2*)b->x[i]; ra.u[i] = b->u[i]; }
        ra.K1 = (double2*)b->K1; ra.cs = b->cs; ra.xr = b->x_ref; ra.ur = b->u_ref;
        ra.cost = b->cost; ra.dJ = b->dJ; ra.smax = b->smax; ra.gamma = b->gamma;
        ra.status = b->status; ra.n_iter = b->n_iter; ra.res_buf = b->res_buf; ra.n_roll = b->n_roll;
        ra.hist_cost = hist ? b->hist_cost : nullptr; ra.hist_smax = hist ? b->hist_smax : nullptr;
        ra.retry_list = b->retry_list; ra.counter = b->counters;
        ra.B = b->B; ra.Bp = b->Bp; ra.N = b->N; ra.k0 = k0; ra.k1 = k1; ra.ext = ext ? 1 : 0;
        if (b->flags & GYM_FLAG_RUN_SINGLE)
            hipLaunchKernelGGL(RUN_SEL(b, k_nt_run), dim3(grid_for(b->B, BLK)), dim3(BLK), 0, st, ra);
        else   // two wavefronts per 64 lanes; every lane of the padded batch takes part (padding: GYM_PAD)
            hipLaunchKernelGGL(RUN_SEL(b, k_nt_run2), dim3((unsigned)(b->Bp / BLK)), dim3(R2WAVES * BLK), 0, st, ra);
    }
    // the statistics after iteration k1 - 1 ("lanes that ran" = the lanes that executed it; [4] = 0: this
    // schedule keeps no retry list)
    hipLaunchKernelGGL(k_stats_partial, dim3(STAT_BLOCKS), dim3(STAT_THREADS), 0, st, b->status, b->cost, b->smax,
                       b->n_iter, b->n_roll, b->partials, Range{0, b->B}, (int)k1 - 1);
    hipLaunchKernelGGL(k_stats_final, dim3(1), dim3(64 * NSTAT), 0, st, b->partials, b->counters, b->stats,
                       (const double*)nullptr, (double*)nullptr, STAT_BLOCKS);
    return launch_status();
}

int gym_newton_tail_scratch(int32_t N, int32_t n_lanes, int32_t max_ls, int64_t* doubles_out) {
    if (!doubles_out || N < 2 || N - 1 > TL_MAX_T || n_lanes < 0 || max_ls < 1 || max_ls > BLK) return GYM_EINVAL;
    const int64_t v = (int64_t)n_lanes * max_ls;
    const int64_t Vp = v > 0 ? (v + BLK - 1) / BLK * BLK : BLK;
    *doubles_out = Vp * (4 * (int64_t)N + 2 * (int64_t)(N - 1));
    return 0;
}

int gym_newton_cand_scratch(int32_t N, int64_t slots, int64_t* doubles_out) {
    if (!doubles_out || N < 2 || slots < 0 || slots % BLK != 0 || slots > GYM_MAX_BP) return GYM_EINVAL;
    *doubles_out = slots * (4 * (int64_t)N + 2 * (int64_t)(N - 1) + 1);
    return 0;
}

int gym_newton_tail_lds(int32_t N, int64_t* bytes_out, int64_t* limit_out) {
    if (!bytes_out || N < 2 || N - 1 > TL_MAX_T) return GYM_EINVAL;
    *bytes_out = (int64_t)tail_lds_bytes(N - 1);
    if (limit_out) {   // the current device's opt-in LDS per workgroup
        int dev = 0, lim = 0;
        hipError_t e = hipGetDevice(&dev);
        if (e == hipSuccess) e = hipDeviceGetAttribute(&lim, hipDeviceAttributeSharedMemPerBlockOptin, dev);
        if (e != hipSuccess) return (int)e;
        *limit_out = lim;
    }
    return 0;
}

int gym_newton_tail(const gym_model* m, const gym_weights* w, const gym_armijo* a, const gym_batch* b,
                    const int32_t* lanes, int32_t n_lanes, double* scratch, int64_t scratch_doubles, int32_t k0,
                    int32_t k1, void* s) {
    int64_t need = 0;
    if (bad_iter_args(m, w, a, b) || k0 < 0 || k1 < k0 || n_lanes < 0 || (n_lanes > 0 && (!lanes || !scratch)) ||
        (b->flags & GYM_FLAG_X_CKPT) || gym_newton_tail_scratch(b->N, n_lanes, a->max_ls, &need) ||
        scratch_doubles < need || (int64_t)n_lanes > b->B)
        return GYM_EINVAL;
    hipStream_t st = (hipStream_t)s;
    const bool hist = a->record_history != 0;
    if (k1 > k0 && n_lanes > 0) {
        TimedLaunch tl(b->timing, 9, st);
        TailArgs ta;
        ta.m = Dyn(*m);
        ta.w = kw(*w);
        ta.a = SolverCtl{a->tol, a->beta, a->c, a->gamma0, a->max_ls, k0, b->hist_len, 0};
        for (int i = 0; i < 2; ++i) { ta.x[i] = (double2*)b->x[i]; ta.u[i] = b->u[i]; }
        ta.K1 = (double2*)b->K1; ta.cs = b->cs; ta.xr = b->x_ref; ta.ur = b->u_ref;
        ta.cost = b->cost; ta.dJ = b->dJ; ta.smax = b->smax; ta.gamma = b->gamma;
        ta.status = b->status; ta.n_iter = b->n_iter; ta.res_buf = b->res_buf; ta.n_roll = b->n_roll;
        ta.hist_cost = hist ? b->hist_cost : nullptr; ta.hist_smax = hist ? b->hist_smax : nullptr;
        ta.list = lanes;
        const int64_t v = (int64_t)n_lanes * a->max_ls;
        ta.Vp = (v + BLK - 1) / BLK * BLK;
        ta.sx = (double2*)scratch;
        ta.su = scratch + 4 * (int64_t)b->N * ta.Vp;
        ta.Bp = b->Bp; ta.N = b->N; ta.k0 = k0; ta.k1 = k1; ta.pad = 0;
        // trials on lane pairs while they fit one wavefront (gym::rk4_pair: the same bits, a shorter chain)
        const bool pair = a->max_ls <= BLK / 2 && !(b->flags & GYM_FLAG_RUN_SINGLE);
        const bool u0z = b->flags & GYM_FLAG_U0_ZERO, rl = b->flags & GYM_FLAG_REF_LANE;
        const auto kern = pair ? (rl ? (u0z ? k_nt_tail<true, true, true> : k_nt_tail<false, true, true>)
                                     : (u0z ? k_nt_tail<true, false, true> : k_nt_tail<false, false, true>))
                               : (rl ? (u0z ? k_nt_tail<true, true, false> : k_nt_tail<false, true, false>)
                                     : (u0z ? k_nt_tail<true, false, false> : k_nt_tail<false, false, false>));
        const size_t lds = tail_lds_bytes(b->N - 1);
        if (lds > 65536) {   // above the default dynamic-LDS limit (gfx950: 160 KiB per workgroup)
            const hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(kern),
                                                     hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
            if (e != hipSuccess) return (int)e;
        }
        hipLaunchKernelGGL(kern, dim3((unsigned)n_lanes), dim3(TL_THREADS), lds, st, ta);
    }
    // the statistics after iteration k1 - 1, over the whole batch (as gym_newton_run)
    hipLaunchKernelGGL(k_stats_partial, dim3(STAT_BLOCKS), dim3(STAT_THREADS), 0, st, b->status, b->cost, b->smax,
                       b->n_iter, b->n_roll, b->partials, Range{0, b->B}, (int)k1 - 1);
    hipLaunchKernelGGL(k_stats_final, dim3(1), dim3(64 * NSTAT), 0, st, b->partials, b->counters, b->stats,
                       (const double*)nullptr, (double*)nullptr, STAT_BLOCKS);
    return launch_status();
}

int gym_newton_fill_states(const gym_model* m, const gym_batch* b, int32_t buf, void* s) {
    if (!m || bad_batch(b) || buf < -1 || buf > 1) return GYM_EINVAL;
    if (!(b->flags & GYM_FLAG_X_CKPT)) return 0;
    hipLaunchKernelGGL(k_fill_states, dim3(grid_for(b->B, BLK)), dim3(BLK), 0, (hipStream_t)s, Dyn(*m), (double2*)b->x[0],
                       (double2*)b->x[1], b->u[0], b->u[1], b->res_buf, (int)buf, b->B, b->Bp, b->N);
    return launch_status();
}

int gym_newton_finalize(const gym_model* m, const gym_weights* w, const gym_batch* b, int32_t k_done, double* x_out,
                        double* u_out, double* K_out, double* sig_out, void* s) {
    if (!m || !w || bad_batch(b) || k_done < 0) return GYM_EINVAL;
    hipStream_t st = (hipStream_t)s;
    hipLaunchKernelGGL(k_finalize_status, dim3(grid_for(b->B, 256)), dim3(256), 0, st, b->status, b->res_buf, b->B,
                       (int)k_done);
    int e = launch_status();
    if (e) return e;
    const int T = b->N - 1;
    if (x_out && (e = gym_newton_fill_states(m, b, -1, s))) return e;
    const int64_t* map = b->lane_map;   // results straight into the caller's lane order
    if (x_out && (e = launch_unpack_tiled(SrcPairs{(const double2*)b->x[0], (const double2*)b->x[1], b->res_buf, 2},
                                          x_out, b->B, b->Bp, b->N, 4, st, map)))
        return e;
    if (u_out && (e = launch_unpack_tiled(SrcPlanes{b->u[0], b->u[1], b->res_buf, 2}, u_out, b->B, b->Bp, T, 2, st,
                                          map)))
        return e;
    if (K_out && (e = launch_unpack_tiled(SrcGains{(const double2*)b->K1}, K_out, b->B, b->Bp, T, 8, st, map)))
        return e;
    if (sig_out && (e = gym_newton_sigma(m, w, b, sig_out, s))) return e;
    return 0;
}

// Placement probe (gym_placement_probe): the pipelined phase kernel's stream traffic with no arithmetic.  The first
// half of the workgroups runs the sweep's pattern on lanes [0, Bp/2) (stage T-1 .. 0: read the 2 KiB x_cb block and
// the 512 B tau2 row of u_cb, write the K1 block and the cg row), the rest the trial's on [Bp/2, Bp) (stage 0 .. T-1:
// read K1 and cg, write x_cb' at t + 1 and u_cb'), one stage prefetched, non-temporal, four wavefronts per SIMD -- the
// phase kernel's bytes per launch.  How fast this moves depends on where the driver placed the six streams the same
// way the phase kernel's speed does (profiles/r06/README.md: 1.84-2.13 ms on eight sets of one process, Pearson
// 0.87-0.93 against the kernel's own phase times), so a solver ranks candidate stream sets with it in a few ms each.
// It overwrites the streams (garbage; no NaN traps on the GPU): only before gym_newton_init.
__global__ __launch_bounds__(BLK, 4) void k_placement_probe(double2* __restrict__ xc, double2* __restrict__ xn,
                                                            double* __restrict__ uc, double* __restrict__ un,
                                                            double2* __restrict__ K1, double* __restrict__ cs,
                                                            int64_t Bp, int T) {
    const int64_t w = blockIdx.x, j = threadIdx.x;
    const bool sweep = w < (Bp / BLK) / 2;
    const int64_t px = w * 2 * BLK + j, pl = w * BLK + j;
    const int64_t row = 2 * Bp;                  // double2 per knot row of a pair stream; doubles per stage of planes
    if (sweep) {
        double2 a = ld_nt(xc + (int64_t)(T - 1) * row + px), b = ld_nt(xc + (int64_t)(T - 1) * row + px + BLK);
        double c = ld_nt(uc + (int64_t)(T - 1) * row + Bp + pl);
        for (int t = T - 1; t >= 0; --t) {
            double2 na = a, nb = b;
            double nc = c;
            if (t > 0) {
                na = ld_nt(xc + (int64_t)(t - 1) * row + px); nb = ld_nt(xc + (int64_t)(t - 1) * row + px + BLK);
                nc = ld_nt(uc + (int64_t)(t - 1) * row + Bp + pl);
            }
            st_nt(K1 + (int64_t)t * row + px, a.x + c, a.y); st_nt(K1 + (int64_t)t * row + px + BLK, b.x, b.y);
            st_nt(cs + (int64_t)t * row + pl, c);
            a = na; b = nb; c = nc;
        }
    } else {
        double2 a = ld_nt(K1 + px), b = ld_nt(K1 + px + BLK);
        double c = ld_nt(cs + pl);
        for (int t = 0; t < T; ++t) {
            double2 na = a, nb = b;
            double nc = c;
            if (t + 1 < T) {
                na = ld_nt(K1 + (int64_t)(t + 1) * row + px); nb = ld_nt(K1 + (int64_t)(t + 1) * row + px + BLK);
                nc = ld_nt(cs + (int64_t)(t + 1) * row + pl);
            }
            st_nt(xn + (int64_t)(t + 1) * row + px, a.x + c, a.y); st_nt(xn + (int64_t)(t + 1) * row + px + BLK, b.x, b.y);
            st_nt(un + (int64_t)t * row + Bp + pl, c);
            a = na; b = nb; c = nc;
        }
    }
}

int gym_placement_probe(const gym_batch* b, int32_t cb, void* s) {
    if (bad_batch(b) || cb < 0 || cb > 1 || b->Bp % (2 * BLK) != 0) return GYM_EINVAL;
    hipLaunchKernelGGL(k_placement_probe, dim3((unsigned)(b->Bp / BLK)), dim3(BLK), 0, (hipStream_t)s,
                       (double2*)b->x[cb], (double2*)b->x[cb ^ 1], b->u[cb], b->u[cb ^ 1], (double2*)b->K1, b->cs,
                       b->Bp, b->N - 1);
    return launch_status();
}

int gym_newton_sigma(const gym_model* m, const gym_weights* w, const gym_batch* b, double* sig_out, void* s) {
    if (!m || !w || bad_batch(b) || !sig_out) return GYM_EINVAL;
    hipStream_t st = (hipStream_t)s;
    const int T = b->N - 1;
    for (int parity = 0; parity < 2; ++parity) {   // sigma1 of each lane's last sweep, one launch per buffer
        hipLaunchKernelGGL(SERIAL_SEL(b, k_nt_sigma), dim3(grid_for(b->B, BLK)), dim3(BLK), 0, st, Dyn(*m), kw(*w),
                           (const double2*)b->x[parity], b->u[parity], b->x_ref, b->u_ref, b->cs,
                           (const int32_t*)nullptr, (const int32_t*)nullptr, b->n_iter, parity, b->B, b->Bp, b->N);
        const int e = launch_status();
        if (e) return e;
    }
    return launch_unpack_tiled(SrcSigma{kw(*w), b->cs, b->u[0], b->u[1], b->u_ref, b->n_iter,
                                        (b->flags & GYM_FLAG_REF_LANE) ? 2 * (int64_t)(b->N - 1) : 0}, sig_out, b->B, b->Bp,
                               T, 2, st, b->lane_map);
}

static int sweep_grid(int64_t Bp, int G) {
    const int64_t nb = (Bp / BLK) * (int64_t)G;
    return (int)((nb + 7) / 8 * 8);
}

int gym_gamma_sweep(const gym_model* m, const gym_weights* w, const double* x, const double* u, const double* Kf,
                    const double* sigma, const double* gammas, int32_t G, const double* xr, const double* ur,
                    double* cost_out, int64_t B, int64_t Bp, int32_t N, void* s) {
    if (!m || !w || !x || !u || !Kf || !sigma || !gammas || !xr || !ur || !cost_out || G < 1 || bad_dims(B, Bp, N) ||
        (Bp / BLK) * (int64_t)G > ((int64_t)1 << 31) - 8)
        return GYM_EINVAL;
    hipLaunchKernelGGL(k_gamma_sweep, dim3(sweep_grid(Bp, G)), dim3(BLK), 0, (hipStream_t)s, Dyn(*m), kw(*w),
                       (const double2*)x, u, (const double2*)Kf, sigma, gammas, (int)G, xr, ur, cost_out, B, Bp, N);
    return launch_status();
}

int gym_newton_gamma_sweep(const gym_model* m, const gym_weights* w, const gym_armijo* a, const gym_batch* b,
                           int32_t k, const double* gammas, int32_t G, double* cost_out, void* s) {
    if (!m || !w || !a || bad_batch(b) || k < 0 || !gammas || !cost_out || G < 1 ||
        (b->Bp / BLK) * (int64_t)G > ((int64_t)1 << 31) - 8)
        return GYM_EINVAL;
    hipStream_t st = (hipStream_t)s;
    const TrialIO io = trial_io(b, k);
    // iteration k's backward sweep (K1, cg, dJ, smax: the values iteration k itself computes) plus sigma1
    hipLaunchKernelGGL(SERIAL_SEL(b, k_nt_backward_all), dim3(grid_for(b->B, BLK)), dim3(BLK), 0, st, Dyn(*m), kw(*w),
                       io.x, io.u, b->x_ref, b->u_ref, (double2*)b->K1, b->cs, a->gamma0, b->dJ, b->smax, b->status,
                       (double*)nullptr, Range{0, b->B}, b->Bp, b->N, (int)k, 0);
    int e = launch_status();
    if (e) return e;
    hipLaunchKernelGGL(CAND_SEL(b, k_nt_gamma_sweep), dim3(sweep_grid(b->Bp, G)), dim3(BLK), 0, st, Dyn(*m), kw(*w),
                       io.x, io.u, (const double2*)b->K1, (const double*)b->cs, a->gamma0, gammas, (int)G, b->x_ref, b->u_ref,
                       b->status, cost_out, b->B, b->Bp, b->N);
    return launch_status();
}

#ifdef GYM_TAIL_TRACE
int gym_debug_tail_trace(void* host_out, int reset) {   // diagnostic build only: 4096 x 4 uint64
    if (reset) {
        static unsigned long long zero[4096][4];
        return (int)hipMemcpyToSymbol(HIP_SYMBOL(g_tail_trace), zero, sizeof(zero));
    }
    return (int)hipMemcpyFromSymbol(host_out, HIP_SYMBOL(g_tail_trace), sizeof(g_tail_trace));
}
#endif
#ifdef GYM_RUN2_TRACE
int gym_debug_run2_trace(void* host_out, int reset) {   // diagnostic build only: 8192 x 2 x 6 uint64
    if (reset) {
        static unsigned long long zero[8192][2][6];
        return (int)hipMemcpyToSymbol(HIP_SYMBOL(g_run2_trace), zero, sizeof(zero));
    }
    return (int)hipMemcpyFromSymbol(host_out, HIP_SYMBOL(g_run2_trace), sizeof(g_run2_trace));
}
#endif
#ifdef GYM_WAVE_TRACE
int gym_debug_wave_trace(void* host_out) {   // diagnostic build only: 2 x 8192 x 4 uint64
    return (int)hipMemcpyFromSymbol(host_out, HIP_SYMBOL(g_wave_trace), sizeof(g_wave_trace));
}
#endif

int gym_timing_create(gym_timing* t) {
    if (!t) return GYM_EINVAL;
    for (int i = 0; i < 2 * GYM_NK; ++i) {
        hipEvent_t e;
        hipError_t r = hipEventCreate(&e);
        if (r != hipSuccess) return (int)r;
        t->ev[i] = (void*)e;
    }
    for (int i = 0; i < 2 * GYM_TIMING_POOL; ++i) {
        hipEvent_t e;
        hipError_t r = hipEventCreate(&e);
        if (r != hipSuccess) return (int)r;
        t->pool_ev[i] = (void*)e;
    }
    for (int i = 0; i < GYM_NK; ++i) { t->ms[i] = 0.0; t->launches[i] = 0; }
    t->pending = 0;
    t->pool_used = 0;
    return 0;
}

int gym_timing_destroy(gym_timing* t) {
    if (!t) return GYM_EINVAL;
    for (int i = 0; i < 2 * GYM_NK; ++i)
        if (t->ev[i]) { (void)hipEventDestroy((hipEvent_t)t->ev[i]); t->ev[i] = nullptr; }
    for (int i = 0; i < 2 * GYM_TIMING_POOL; ++i)
        if (t->pool_ev[i]) { (void)hipEventDestroy((hipEvent_t)t->pool_ev[i]); t->pool_ev[i] = nullptr; }
    t->pool_used = 0;
    return 0;
}

int gym_timing_collect(gym_timing* t) {
    if (!t) return GYM_EINVAL;
    // every recorded pair is read first and committed only when all of them succeeded: on an error (e.g.
    // hipErrorNotReady, the stream not synchronised) the record is unchanged and a later collect counts each pair once
    double ms_add[GYM_NK] = {};
    int n_add[GYM_NK] = {};
    for (int i = 0; i < GYM_NK; ++i) {
        if (!(t->pending & (1 << i))) continue;
        float ms = 0.f;
        hipError_t r = hipEventElapsedTime(&ms, (hipEvent_t)t->ev[2 * i], (hipEvent_t)t->ev[2 * i + 1]);
        if (r != hipSuccess) return (int)r;
        ms_add[i] += ms;
        n_add[i] += 1;
    }
    for (int j = 0; j < t->pool_used; ++j) {
        float ms = 0.f;
        hipError_t r = hipEventElapsedTime(&ms, (hipEvent_t)t->pool_ev[2 * j], (hipEvent_t)t->pool_ev[2 * j + 1]);
        if (r != hipSuccess) return (int)r;
        ms_add[t->pool_kind[j]] += ms;
        n_add[t->pool_kind[j]] += 1;
    }
    for (int i = 0; i < GYM_NK; ++i) {
        t->ms[i] += ms_add[i];
        t->launches[i] += n_add[i];
    }
    t->pending = 0;
    t->pool_used = 0;
    return 0;
}

}  // extern "C"
