// MI355X (gfx950) kernels of the LQR / receding-horizon MPC trackers (trajectory_tracking.py), C-ABI part 2.
//
// Both trackers follow ONE reference trajectory that every lane shares (main.py task_3 / task_4), so their
// feedback gains are lane-independent:
//   * LQR (solve_LQR_tracking :170-203): one backward recursion along the reference;
//   * MPC (solve_mpc_tracking :8-69 with solver_mpc :73-140): at control step t the QP over the window
//     [t, t + T_pred - 1] of the shifted reference (padded with (A_f, B_f)) has only equality constraints
//     (test_constraints = False, :87), so its exact solution is u_0 = K_0(t) x_0 with K_0(t) the first gain of
//     the window's finite-horizon LQ recursion.  All T windows are solved in parallel, one thread each.
// The batched part is the closed-loop RK4 simulation of B perturbed initial states under the shared
// feed-forward / feedback sequence (simulate_tracking :206-216 and the MPC loop :43-60), one lane per thread
// with the gains, reference and feed-forward read through wave-uniform (scalar) loads.
#include <hip/hip_runtime.h>

#include <cstdint>

#ifndef GYM_HORNER_VOP3
#define GYM_HORNER_VOP3 1   // three-address Horner steps (acrobot_device.hpp): no per-step constant copies
#endif
#include "acrobot_device.hpp"
#include "gymnast_acrobot.h"

using gym::Dyn;

namespace {

struct M44 { double v[16]; };
struct M22 { double v[4]; };

// one step of the reference's recursion (trajectory_tracking.py:158-160 / :195-200):
//   aux1 = R + B'PB, aux2 = B'PA, K = -inv(aux1) aux2, P <- Q + A'PA + (A'PB) K
__device__ __forceinline__ void lqr_step(const double* A, const double* Bm, double* P, const M44& Q, const M22& R,
                                         double* K) {
    double PA[16], PB[8];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
#pragma unroll
        for (int j = 0; j < 4; ++j)
            PA[4 * i + j] = ((P[4 * i] * A[j] + P[4 * i + 1] * A[4 + j]) + P[4 * i + 2] * A[8 + j]) + P[4 * i + 3] * A[12 + j];
#pragma unroll
        for (int j = 0; j < 2; ++j)
            PB[2 * i + j] = ((P[4 * i] * Bm[j] + P[4 * i + 1] * Bm[2 + j]) + P[4 * i + 2] * Bm[4 + j]) + P[4 * i + 3] * Bm[6 + j];
    }
    double a1[4], a2[8];
#pragma unroll
    for (int i = 0; i < 2; ++i) {
#pragma unroll
        for (int j = 0; j < 2; ++j)
            a1[2 * i + j] = R.v[2 * i + j] + (((Bm[i] * PB[j] + Bm[2 + i] * PB[2 + j]) + Bm[4 + i] * PB[4 + j]) + Bm[6 + i] * PB[6 + j]);
#pragma unroll
        for (int j = 0; j < 4; ++j)
            a2[4 * i + j] = ((Bm[i] * PA[j] + Bm[2 + i] * PA[4 + j]) + Bm[4 + i] * PA[8 + j]) + Bm[6 + i] * PA[12 + j];
    }
    const double idet = 1.0 / (a1[0] * a1[3] - a1[1] * a1[2]);
    const double i00 = a1[3] * idet, i01 = -a1[1] * idet, i10 = -a1[2] * idet, i11 = a1[0] * idet;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        K[j] = -(i00 * a2[j] + i01 * a2[4 + j]);
        K[4 + j] = -(i10 * a2[j] + i11 * a2[4 + j]);
    }
    double nP[16];
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const double apa = ((A[i] * PA[j] + A[4 + i] * PA[4 + j]) + A[8 + i] * PA[8 + j]) + A[12 + i] * PA[12 + j];
            const double apb0 = ((A[i] * PB[0] + A[4 + i] * PB[2]) + A[8 + i] * PB[4]) + A[12 + i] * PB[6];
            const double apb1 = ((A[i] * PB[1] + A[4 + i] * PB[3]) + A[8 + i] * PB[5]) + A[12 + i] * PB[7];
            nP[4 * i + j] = (Q.v[4 * i + j] + apa) + (apb0 * K[j] + apb1 * K[4 + j]);
        }
#pragma unroll
    for (int k = 0; k < 16; ++k) P[k] = nP[k];
}

// stage s of a stage array (continuous Jacobians if disc: A_d = I + dt A_c, B_d = dt B_c, :161-164)
__device__ __forceinline__ void load_stage(const double* A, const double* Bm, int s, int S, const double* Ap,
                                           const double* Bp, int disc, double dt, double* Ad, double* Bd) {
    const double* a = s < S ? A + 16 * (int64_t)s : Ap;
    const double* b = s < S ? Bm + 8 * (int64_t)s : Bp;
#pragma unroll
    for (int k = 0; k < 16; ++k) Ad[k] = disc ? ((k % 5 == 0 ? 1.0 : 0.0) + dt * a[k]) : a[k];
#pragma unroll
    for (int k = 0; k < 8; ++k) Bd[k] = disc ? dt * b[k] : b[k];
}

// window w: recursion over stages w + L-2 .. w (stage index >= S -> pad), terminal P = QT.
// all_gains: K_out (L-1, 2, 4) of window 0;  else K_out (nwin, 2, 4) = the first gain of every window.
__global__ __launch_bounds__(64) void k_tv_lqr_gains(const double* __restrict__ A, const double* __restrict__ Bm,
                                                     int S, const double* __restrict__ Ap,
                                                     const double* __restrict__ Bp, M44 Q, M22 R,
                                                     const double* __restrict__ QT, int L,
                                                     int nwin, int all_gains, int disc, double dt,
                                                     double* __restrict__ K_out) {
    const int w = blockIdx.x * blockDim.x + threadIdx.x;
    if (w >= nwin) return;
    double P[16], K[8], Ad[16], Bd[8];
#pragma unroll
    for (int k = 0; k < 16; ++k) P[k] = QT[k];
    for (int s = L - 2; s >= 0; --s) {
        load_stage(A, Bm, w + s, S, Ap, Bp, disc, dt, Ad, Bd);
        lqr_step(Ad, Bd, P, Q, R, K);
        if (all_gains) {
#pragma unroll
            for (int k = 0; k < 8; ++k) K_out[8 * (int64_t)s + k] = K[k];
        }
    }
    if (!all_gains) {
#pragma unroll
        for (int k = 0; k < 8; ++k) K_out[8 * (int64_t)w + k] = K[k];
    }
}

// compute_P_inf (:144-165): P <- Riccati map of (A, B, Q, R) from P = Q until max|dP| < tol.  One wavefront;
// lane 4i+j (< 16) owns P[i][j] and evaluates that entry of every product of the map (the same sums, in
// the same order, as one lane would), exchanging rows/columns through LDS: each iteration is a few
// dependent steps instead of ~400 dependent flops of a single lane.  max|dP| is a wave reduction.
__global__ __launch_bounds__(64) void k_dare_fixed_point(const double* __restrict__ A, const double* __restrict__ Bm,
                                                         M44 Q, M22 R, int max_iter, double tol,
                                                         double* __restrict__ P_out, int32_t* __restrict__ iters) {
    __shared__ double sP[16], sPA[16], sPB[8];
    const int ln = threadIdx.x, i = (ln >> 2) & 3, j = ln & 3;
    const bool own = ln < 16;
    double a[16], b[8];
#pragma unroll
    for (int k = 0; k < 16; ++k) a[k] = A[k];
#pragma unroll
    for (int k = 0; k < 8; ++k) b[k] = Bm[k];
    double P = Q.v[4 * i + j];
    int it = max_iter + 1;                 // max_iter + 1: the tolerance was never met
    for (int n = 0; n < max_iter; ++n) {
        if (own) sP[ln] = P;
        __syncthreads();
        const double* Pi = sP + 4 * i;   // row i of P
        const double PA = ((Pi[0] * a[j] + Pi[1] * a[4 + j]) + Pi[2] * a[8 + j]) + Pi[3] * a[12 + j];
        const double PB0 = ((Pi[0] * b[0] + Pi[1] * b[2]) + Pi[2] * b[4]) + Pi[3] * b[6];
        const double PB1 = ((Pi[0] * b[1] + Pi[1] * b[3]) + Pi[2] * b[5]) + Pi[3] * b[7];
        if (own) {
            sPA[ln] = PA;
            if (j == 0) { sPB[2 * i] = PB0; sPB[2 * i + 1] = PB1; }
        }
        __syncthreads();
        double a1[4];
#pragma unroll
        for (int r = 0; r < 2; ++r)
#pragma unroll
            for (int c = 0; c < 2; ++c)
                a1[2 * r + c] = R.v[2 * r + c] + (((b[r] * sPB[c] + b[2 + r] * sPB[2 + c]) + b[4 + r] * sPB[4 + c]) +
                                                  b[6 + r] * sPB[6 + c]);
        const double a20 = ((b[0] * sPA[j] + b[2] * sPA[4 + j]) + b[4] * sPA[8 + j]) + b[6] * sPA[12 + j];
        const double a21 = ((b[1] * sPA[j] + b[3] * sPA[4 + j]) + b[5] * sPA[8 + j]) + b[7] * sPA[12 + j];
        const double idet = 1.0 / (a1[0] * a1[3] - a1[1] * a1[2]);
        const double i00 = a1[3] * idet, i01 = -a1[1] * idet, i10 = -a1[2] * idet, i11 = a1[0] * idet;
        const double K0 = -(i00 * a20 + i01 * a21), K1 = -(i10 * a20 + i11 * a21);
        const double apa = ((a[i] * sPA[j] + a[4 + i] * sPA[4 + j]) + a[8 + i] * sPA[8 + j]) + a[12 + i] * sPA[12 + j];
        const double apb0 = ((a[i] * sPB[0] + a[4 + i] * sPB[2]) + a[8 + i] * sPB[4]) + a[12 + i] * sPB[6];
        const double apb1 = ((a[i] * sPB[1] + a[4 + i] * sPB[3]) + a[8 + i] * sPB[5]) + a[12 + i] * sPB[7];
        const double nP = (Q.v[4 * i + j] + apa) + (apb0 * K0 + apb1 * K1);
        // np.max(np.abs(P_next - P)) < tol (:160-163) as a wave vote: every entry below tol (a NaN entry is not,
        // as np.max would return NaN); no cross-lane data movement on the iteration's critical path
        const bool conv = __all(!own || fabs(nP - P) < tol);
        P = nP;
        __syncthreads();   // every lane has read sP / sPA / sPB before the next iteration rewrites them
        if (conv) { it = n + 1; break; }
    }
    if (own) P_out[ln] = P;
    if (ln == 0) *iters = it;
}

// ------------------------------------------------------------------------------------------
// Fused MPC gains (solve_mpc_tracking :14-38 + the exact solution of every control step's QP): one launch.
//
// Every stage matrix the MPC uses is the acrobot's discretised linearisation (:18-23, the pad (A_f, B_f) :31-33),
// so it has a fixed structure: A_d rows 0,1 = [1,0,h,0], [0,1,0,h] (I + dt A_c with A_c rows e3', e4'),
// B_d = [0, b] with b = (0, 0, b2, b3)' (tau1 unactuated, dynamics.py:205).  The Riccati map
//   aux1 = R + B'PB, aux2 = B'PA, K = -inv(aux1) aux2, P <- Q + A'PA + (A'PB) K            (:158-160)
// then needs, per entry, only the terms those zeros leave (the skipped products are exact zeros / ones in the
// dense form; rounding of the rest is the reference's up to sum order, checked against the oracle at 1e-9).
//
// Lane-parallel map: a 16-lane group evaluates one map; lane 4i+j owns P[i][j] and the (i, j) entry of every
// product.  Row i of P comes from the lane's own quad (DPP quad broadcasts); rows 2, 3 and i&1 of PA and PB
// come from the group's other quads: the PB rows (uniform in a quad, on the gain's critical path) through
// row broadcasts (one v_mov_b64_dpp each), the PA rows through ds_swizzle (no LDS storage, no barrier).  A map is then ~35 fp64
// instructions per lane and a handful of exchanges on the critical path, instead of ~400 dependent flops of one
// lane (k_tv_lqr_gains) or three LDS round trips with barriers (k_dare_fixed_point).
// ------------------------------------------------------------------------------------------
struct StageLin {
    double a2[4], a3[4], b2, b3;   // rows 2, 3 of A_d; B_d[2][1], B_d[3][1]
};

// Calculate_A_B_matrixes + discretize_linearization (dynamics.py:217-226, trajectory_generation.py:161-164):
// A_d = I + dt A_c, B_d = dt B_c, with the same operations as load_stage() on k_point's Jacobians
__device__ __forceinline__ void disc_stage(const Dyn& m, double x0, double x1, double x2, double x3, double tau2,
                                           StageLin& s) {
    const gym::Jac J = gym::jacobian(m, x0, x1, x2, x3, tau2);
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        s.a2[j] = (j == 2 ? 1.0 : 0.0) + m.h * J.a2[j];
        s.a3[j] = (j == 3 ? 1.0 : 0.0) + m.h * J.a3[j];
    }
    s.b2 = m.h * J.bc2;
    s.b3 = m.h * J.bc3;
}

using gym::dpp_d;
template <int N>   // v_mov_b64_dpp row_newbcast:N -- lane N of each 16-lane row to the whole row (gfx90a+ DPP64)
__device__ __forceinline__ double bcast_d(double v) {
    return __longlong_as_double(
        __builtin_amdgcn_update_dpp(0ll, __double_as_longlong(v), 0x150 + N, 0xF, 0xF, false));
}
template <int AND, int OR>   // ds_swizzle bit mode inside 32-lane halves: lane' = (lane & AND) | OR
__device__ __forceinline__ double swz_d(double v) {
    constexpr int pat = (AND & 31) | ((OR & 31) << 5);
    const long long b = __double_as_longlong(v);
    const int lo = __builtin_amdgcn_ds_swizzle((int)b, pat);
    const int hi = __builtin_amdgcn_ds_swizzle((int)(b >> 32), pat);
    return __longlong_as_double(((long long)hi << 32) | (unsigned)lo);
}

// per-lane constants of the map: lane 4i+j of its group
struct MapLane {
    bool hi;           // i & 1
    double c0j, c1j;   // A_d[0][j], A_d[1][j]
    double ci;         // A_d[0][i] + A_d[1][i] (exactly one of the two is nonzero): 1, 1, h, h
    double Qij, R00, R01, R10, R11;
};
__device__ __forceinline__ MapLane map_lane(int i, int j, double h, const M44& Q, const M22& R) {
    MapLane c;
    c.hi = i & 1;
    c.c0j = j == 0 ? 1.0 : (j == 2 ? h : 0.0);
    c.c1j = j == 1 ? 1.0 : (j == 3 ? h : 0.0);
    c.ci = i < 2 ? 1.0 : h;
    c.Qij = Q.v[4 * i + j];
    c.R00 = R.v[0]; c.R01 = R.v[1]; c.R10 = R.v[2]; c.R11 = R.v[3];
    return c;
}

// One Riccati map on the structured stage (a2j = A_d[2][j], a3j = A_d[3][j], a2i = A_d[2][i], a3i = A_d[3][i]);
// returns P_next[i][j] and this lane's column j of the gain K (K0j, K1j).
__device__ __forceinline__ double riccati_map_lane(double P, const MapLane& c, double a2j, double a3j, double a2i,
                                                   double a3i, double b2, double b3, double& K0j, double& K1j) {
#pragma clang fp contract(on)
    // the gain's critical path is P -> PB -> aux1 -> 1/det -> K: PB and its exchanges are issued first
    const double P2 = dpp_d<0xAA>(P), P3 = dpp_d<0xFF>(P);                    // P[i][2], P[i][3]
    const double PB = P2 * b2 + P3 * b3;                                      // (PB)[i][1]; (PB)[i][0] = 0
    const double PB2 = bcast_d<8>(PB), PB3 = bcast_d<12>(PB);                 // (PB)[2][1], (PB)[3][1]
    const double P0 = dpp_d<0x00>(P), P1 = dpp_d<0x55>(P);
    const double PA = ((P0 * c.c0j + P1 * c.c1j) + P2 * a2j) + P3 * a3j;     // (PA)[i][j]
    const double a1 = c.R11 + (b2 * PB2 + b3 * PB3);                           // aux1[1][1]; aux1[0][*] = R[0][*]
    const double idet = gym::recip(c.R00 * a1 - c.R01 * c.R10);              // rcp + 2 Newton steps
    const double PA2 = swz_d<0x13, 0x08>(PA), PA3 = swz_d<0x13, 0x0C>(PA), PAh = swz_d<0x17, 0x00>(PA);
    const double B0 = bcast_d<0>(PB), B4 = bcast_d<4>(PB);
    const double PBh = c.hi ? B4 : B0;                                        // (PB)[i&1][1]
    const double a2 = b2 * PA2 + b3 * PA3;                                    // aux2[1][j]; aux2[0][j] = 0
    K0j = -((-c.R01 * idet) * a2);                                            // -(inv(aux1) aux2)[0][j]
    K1j = -((c.R00 * idet) * a2);                                             // -(inv(aux1) aux2)[1][j]
    const double APA = (c.ci * PAh + a2i * PA2) + a3i * PA3;                  // (A'PA)[i][j]
    const double APB = (c.ci * PBh + a2i * PB2) + a3i * PB3;                  // (A'PB)[i][1]; [i][0] = 0
    return (c.Qij + APA) + APB * K1j;
}

constexpr int kMpcMaxStages = 256;   // LDS stage table of one workgroup: its 4 windows' stages (L + 2 <= 256)

// ------------------------------------------------------------------------------------------
// compute_P_inf (:144-165) with doubling jumps.  The reference iterates the Riccati map F from P_0 = Q and stops at
// the first n with max|P_{n+1} - P_n| < tol, returning P_{n+1}.  The structure-preserving doubling algorithm
//   A_0 = A, G_0 = B R^-1 B', H_0 = Q;  W = (I + G_k H_k)^-1,
//   A_{k+1} = A_k W A_k,   G_{k+1} = G_k + A_k W G_k A_k',   H_{k+1} = H_k + A_k' H_k W A_k
// gives H_k = F^(2^k)(0) = P_{2^k - 1}, the reference's own iterate (up to rounding), in k steps.  k_mpc_gains jumps
// with it while the map still moves H_k by >= tol (the reference has not stopped there yet) and then runs the
// reference's loop, with its own test, from the last such H_k: the same stop iterate as the reference, ~2^(k-1)
// maps instead of ~2^k (the cfg 5 pad: 434 maps -> 9 doublings + 179 maps).  Doubling all the way to the limit
// (round 5) overshoots the reference's stop by ~tol rho^2 / (1 - rho^2) absolute, which is invisible at the cfg 5
// pad's scale (P ~ 2e7) but not for smaller Q / R.
// On a 16-lane group as the Riccati map below: lane 4i+j owns entry (i, j) of every 4x4 matrix; each product is one
// round through a per-group LDS scratch (one wavefront: its LDS accesses are in order, so no barrier), W by
// Gauss-Jordan elimination with partial pivoting (every lane finds the same pivot row).  Every group of every
// workgroup computes the same bits.
// ------------------------------------------------------------------------------------------
constexpr int kSdaMaxSteps = 30;   // 2^30 - 1 maps: beyond any max_iter an int holds

__device__ __forceinline__ void wave_lds_order() {   // LDS writes of this wavefront visible to its later reads
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}
// (X Y)[i][j], (X Y')[i][j], (X' Y)[i][j] from 16-double LDS matrices (row-major)
__device__ __forceinline__ double dot_xy(const double* X, const double* Y, int i, int j) {
    return ((X[4 * i] * Y[j] + X[4 * i + 1] * Y[4 + j]) + X[4 * i + 2] * Y[8 + j]) + X[4 * i + 3] * Y[12 + j];
}
__device__ __forceinline__ double dot_xyt(const double* X, const double* Y, int i, int j) {
    return ((X[4 * i] * Y[4 * j] + X[4 * i + 1] * Y[4 * j + 1]) + X[4 * i + 2] * Y[4 * j + 2]) + X[4 * i + 3] * Y[4 * j + 3];
}
__device__ __forceinline__ double dot_xty(const double* X, const double* Y, int i, int j) {
    return ((X[i] * Y[j] + X[4 + i] * Y[4 + j]) + X[8 + i] * Y[8 + j]) + X[12 + i] * Y[12 + j];
}

// The doubling's initial triple on the pad (lane 4i+j: entry (i, j) of A_0, G_0, H_0)
__device__ __forceinline__ void sda16_init(double h, const StageLin& pad, const M44& Q, const M22& R, int i, int j,
                                           double& a, double& g, double& hh) {
    // A_f: rows 0, 1 = [1 0 h 0], [0 1 0 h]; rows 2, 3 the StageLin's.  G_0 = (R^-1)[1][1] b b', b = (0, 0, b2, b3)'
    a = i == 0 ? (j == 0 ? 1.0 : (j == 2 ? h : 0.0)) : i == 1 ? (j == 1 ? 1.0 : (j == 3 ? h : 0.0))
                                                   : (i == 2 ? pad.a2[j] : pad.a3[j]);
    const double r11 = R.v[0] / (R.v[0] * R.v[3] - R.v[1] * R.v[2]);
    const double bi = i == 2 ? pad.b2 : (i == 3 ? pad.b3 : 0.0), bj = j == 2 ? pad.b2 : (j == 3 ? pad.b3 : 0.0);
    g = r11 * bi * bj;
    hh = Q.v[4 * i + j];
}

// One doubling step of (a, g, hh) in place; sm = this group's 8 x 16 doubles of LDS.  Returns false (for every lane of
// the wavefront) on a zero / non-finite pivot or a non-finite H.  Every lane of the wavefront must call it.
__device__ bool sda16_step(int i, int j, double* sm, double& a, double& g, double& hh) {
    double* sA = sm;        double* sG = sm + 16;  double* sH = sm + 32;  double* sM = sm + 48;
    double* sV = sm + 64;   double* sW = sm + 80;  double* sT = sm + 96;  double* sU = sm + 112;
    const int l = 4 * i + j;
    wave_lds_order();                                               // reads of the previous step before these writes
    sA[l] = a; sG[l] = g; sH[l] = hh;
    wave_lds_order();
    double m = dot_xy(sG, sH, i, j) + (i == j ? 1.0 : 0.0);        // I + G H
    double v = i == j ? 1.0 : 0.0;                                  // its inverse, built alongside
    bool ok = true;
#pragma unroll
    for (int c = 0; c < 4; ++c) {
        wave_lds_order();                                           // earlier reads of sM / sV are done
        sM[l] = m; sV[l] = v;
        wave_lds_order();
        int p = c;                                                  // the largest |M[r][c]|, r >= c
        double best = fabs(sM[4 * c + c]);
#pragma unroll
        for (int r = c + 1; r < 4; ++r) {
            const double t = fabs(sM[4 * r + c]);
            p = t > best ? r : p;
            best = t > best ? t : best;
        }
        const int row = i == c ? p : (i == p ? c : i);            // this lane's row after swapping rows c, p
        const double piv = sM[4 * p + c];
        ok &= (piv != 0.0) & (fabs(piv) <= 1.7976931348623157e308);
        const double ip = 1.0 / piv;
        const double mm = sM[4 * row + j], vv = sV[4 * row + j];
        const double f = sM[4 * row + c];
        const double mc = sM[4 * p + j] * ip, vc = sV[4 * p + j] * ip;
        m = i == c ? mc : fma(-f, mc, mm);
        v = i == c ? vc : fma(-f, vc, vv);
    }
    wave_lds_order();
    sW[l] = v;
    wave_lds_order();
    const double wa = dot_xy(sW, sA, i, j), wg = dot_xy(sW, sG, i, j);
    sM[l] = wa; sV[l] = wg;                                         // W A, W G
    wave_lds_order();
    const double awg = dot_xy(sA, sV, i, j), hwa = dot_xy(sH, sM, i, j), awa = dot_xy(sA, sM, i, j);
    sT[l] = awg; sU[l] = hwa;
    wave_lds_order();
    const double gn = g + dot_xyt(sT, sA, i, j);                   // G + A W G A'
    const double hn = hh + dot_xty(sA, sU, i, j);                  // H + A' H W A
    const bool bad = !ok || !(fabs(hn) <= 1.7976931348623157e308);
    a = awa; g = gn; hh = hn;
    return !__any(bad);
}

// Workgroup = 4 windows (16 lanes each).  1) every stage the 4 windows use, discretised, into LDS (one lane per
// stage), and the pad (A_f, B_f) at x_f, u_f;  2) compute_P_inf (:144-165) on the pad (doubling jumps, then the
// reference's loop to its stop iterate), in every workgroup (the same bits everywhere: no grid-wide dependency);  3) each window's recursion from P = P_inf over stages
// w+L-2 .. w;  its first gain is the QP's solution u0 = K x0 at control step w.
__global__ __launch_bounds__(64) void k_mpc_gains(Dyn m, const double* __restrict__ x_ref,
                                                  const double* __restrict__ u_ref, int S,
                                                  const double* __restrict__ xf, const double* __restrict__ uf,
                                                  M44 Q, M22 R, int L, int nwin, int max_iter, double tol,
                                                  double* __restrict__ K_out, double* __restrict__ QT_out,
                                                  int32_t* __restrict__ iters_out) {
    __shared__ StageLin st[kMpcMaxStages];
    __shared__ StageLin pad;
    const int ln = threadIdx.x, g = ln >> 4, i = (ln >> 2) & 3, j = ln & 3;
    const int w0 = blockIdx.x * 4;
    const int nst = min(3 + L - 1, kMpcMaxStages);      // local stages 0 .. 3 + L - 2
    if (ln == 0) disc_stage(m, xf[0], xf[1], xf[2], xf[3], uf[1], pad);
    for (int s = ln; s < nst; s += 64) {
        const int gs = w0 + s;
        if (gs < S) {
            disc_stage(m, x_ref[4 * (int64_t)gs], x_ref[4 * (int64_t)gs + 1], x_ref[4 * (int64_t)gs + 2],
                       x_ref[4 * (int64_t)gs + 3], u_ref[2 * (int64_t)gs + 1], st[s]);
        }
    }
    __syncthreads();
    // compute_P_inf (:144-165) on the pad stage, the same bits in every group: doubling jumps while the map still
    // moves the iterate by >= tol, then the reference's loop and test from the last such iterate (see sda16_step)
    __shared__ double sm[4][128];
    const MapLane c = map_lane(i, j, m.h, Q, R);
    const double fa2j = pad.a2[j], fa3j = pad.a3[j], fa2i = pad.a2[i], fa3i = pad.a3[i], fb2 = pad.b2, fb3 = pad.b3;
    double P, K0j, K1j;
    double Pst = c.Qij;                                   // P_{n0}: the loop below resumes from it
    int n0 = 0;
    {
        double da, dg, dh;
        sda16_init(m.h, pad, Q, R, i, j, da, dg, dh);
        for (int s = 1; s <= kSdaMaxSteps; ++s) {
            if (!sda16_step(i, j, sm[g], da, dg, dh)) break;      // (not a stabilisable pad: the loop from P_{n0})
            const int idx = (1 << s) - 1;                          // dh = P_idx
            if (idx >= max_iter) break;                            // the reference never gets past max_iter maps
            const double nP = riccati_map_lane(dh, c, fa2j, fa3j, fa2i, fa3i, fb2, fb3, K0j, K1j);
            if (__all(fabs(nP - dh) < tol)) break;                 // the reference stops at or before map idx + 1
            Pst = dh;
            n0 = idx;
        }
    }
    P = Pst;
    int it = max_iter + 1;                                // the reference's count; max_iter + 1: never converged
    for (int n = n0; n < max_iter; ++n) {
        const double nP = riccati_map_lane(P, c, fa2j, fa3j, fa2i, fa3i, fb2, fb3, K0j, K1j);
        const bool conv = __all(fabs(nP - P) < tol);      // np.abs(P - P_prev).max() < tol (a NaN entry fails)
        P = nP;
        if (conv) { it = n + 1; break; }
    }
    if (blockIdx.x == 0 && ln < 16) {
        QT_out[ln] = P;
        if (ln == 0) *iters_out = it;
    }
    // window w0 + g: stages w + L - 2 .. w (local g + L - 2 .. g), pad past S
    const int w = w0 + g;
    for (int s = L - 2; s >= 0; --s) {
        const StageLin* q = (w + s < S) ? &st[g + s] : &pad;
        P = riccati_map_lane(P, c, q->a2[j], q->a3[j], q->a2[i], q->a3[i], q->b2, q->b3, K0j, K1j);
    }
    if (w < nwin && i == 0) {
        K_out[8 * (int64_t)w + j] = K0j;
        K_out[8 * (int64_t)w + 4 + j] = K1j;
    }
}

// LQ forward pass of one window (solver_mpc's X_opt, U_opt): x_{s+1} = A_s x_s + B_s u_s, u_s = K_s x_s
__global__ void k_lq_forward(const double* __restrict__ A, const double* __restrict__ Bm, int S,
                             const double* __restrict__ Ap, const double* __restrict__ Bp, int disc, double dt,
                             const double* __restrict__ K, const double* __restrict__ x0, int L,
                             double* __restrict__ X, double* __restrict__ U) {
    if (blockIdx.x != 0 || threadIdx.x != 0) return;
    double x[4] = {x0[0], x0[1], x0[2], x0[3]}, Ad[16], Bd[8];
    for (int s = 0; s < L - 1; ++s) {
        const double* k = K + 8 * s;
        const double u0 = ((k[0] * x[0] + k[1] * x[1]) + k[2] * x[2]) + k[3] * x[3];
        const double u1 = ((k[4] * x[0] + k[5] * x[1]) + k[6] * x[2]) + k[7] * x[3];
        X[4 * s] = x[0]; X[4 * s + 1] = x[1]; X[4 * s + 2] = x[2]; X[4 * s + 3] = x[3];
        U[2 * s] = u0; U[2 * s + 1] = u1;
        load_stage(A, Bm, s, S, Ap, Bp, disc, dt, Ad, Bd);
        double n[4];
#pragma unroll
        for (int i = 0; i < 4; ++i)
            n[i] = (((Ad[4 * i] * x[0] + Ad[4 * i + 1] * x[1]) + Ad[4 * i + 2] * x[2]) + Ad[4 * i + 3] * x[3]) +
                   (Bd[2 * i] * u0 + Bd[2 * i + 1] * u1);
        x[0] = n[0]; x[1] = n[1]; x[2] = n[2]; x[3] = n[3];
    }
    X[4 * (L - 1)] = x[0]; X[4 * (L - 1) + 1] = x[1]; X[4 * (L - 1) + 2] = x[2]; X[4 * (L - 1) + 3] = x[3];
}

// The tracking feedback u = u_ff + K (x - x_ff) (simulate_tracking :210, the MPC loop's u = K x0 + u_ref :50) with
// FMA contraction inside the expression only: the frontend then fuses the same product of every sum in every kernel
// and code context.  Under the file's default -ffp-contract=fast the backend chose per context: a pair rollout
// unrolled by two with double-buffered rows (round 3) fused k1 d1 instead of k0 d0 in its second step and lost
// bitwise equality with the single-lane kernel (tools/mpc_rowbuf_probe.py, profiles/r04/mpc_rowbuf/).
__device__ __forceinline__ void track_feedback(const double* k, const double* f, double d0, double d1, double d2,
                                               double d3, double& v0, double& v1) {
#pragma clang fp contract(on)
    v0 = f[0] + (((k[0] * d0 + k[1] * d1) + k[2] * d2) + k[3] * d3);
    v1 = f[1] + (((k[4] * d0 + k[5] * d1) + k[6] * d2) + k[7] * d3);
}

// Batched closed-loop tracking simulation (simulate_tracking :206-216; MPC loop :43-60):
//   u_t = u_ff[t] + K[t] (x_t - x_ff[t]),  x_{t+1} = RK4(x_t, u_t)
// x0 (B,4); shared x_ff (N,4), u_ff (T,2), K (T,2,4); outputs lane-major x (B,N,4), u (B,T,2).  Each lane is a
// chain of T dependent RK4 steps (B/64 wavefronts: latency-bound), so the step's shared operands are loaded
// one step ahead (wave-uniform, scalar) and the lane writes its own rows directly: consecutive steps fill
// its 128-B lines in L2, no transpose pass afterwards.
__global__ __launch_bounds__(64) void k_track_rollout(Dyn m, const double* __restrict__ x0,
                                                      const double* __restrict__ x_ff, const double* __restrict__ u_ff,
                                                      const double* __restrict__ K, int64_t B, int N,
                                                      double* __restrict__ xo, double* __restrict__ uo) {
    const int64_t l = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (l >= B) return;
    const int T = N - 1;
    double2* xl = reinterpret_cast<double2*>(xo + 4 * (int64_t)N * l);
    double2* ul = reinterpret_cast<double2*>(uo + 2 * (int64_t)T * l);
    double n0 = x0[4 * l], n1 = x0[4 * l + 1], n2 = x0[4 * l + 2], n3 = x0[4 * l + 3];
    xl[0] = make_double2(n0, n1);
    xl[1] = make_double2(n2, n3);
    double k[8], r[4], f[2];
#pragma unroll
    for (int q = 0; q < 8; ++q) k[q] = K[q];
#pragma unroll
    for (int q = 0; q < 4; ++q) r[q] = x_ff[q];
    f[0] = u_ff[0]; f[1] = u_ff[1];
    const gym::PolyRegs pk = gym::poly_vgprs();   // minimax coefficients held in VGPRs (acrobot_device.hpp)
    for (int t = 0; t < T; ++t) {
        const double d0 = n0 - r[0], d1 = n1 - r[1], d2 = n2 - r[2], d3 = n3 - r[3];
        double v0, v1;
        track_feedback(k, f, d0, d1, d2, d3, v0, v1);
        if (t + 1 < T) {   // next step's shared operands, in flight during this step's RK4
            const double* kn = K + 8 * (t + 1);
#pragma unroll
            for (int q = 0; q < 8; ++q) k[q] = kn[q];
#pragma unroll
            for (int q = 0; q < 4; ++q) r[q] = x_ff[4 * (t + 1) + q];
            f[0] = u_ff[2 * (t + 1)]; f[1] = u_ff[2 * (t + 1) + 1];
        }
        ul[t] = make_double2(v0, v1);
        gym::rk4(m, n0, n1, n2, n3, v1, pk);
        xl[2 * (t + 1)] = make_double2(n0, n1);
        xl[2 * (t + 1) + 1] = make_double2(n2, n3);
    }
}

// 16-B non-temporal store: the trajectories are written once and not read back by this kernel.  The per-step
// stores land in rows 16 KB apart (the reference's lane-major arrays); streamed past the caches they cost the
// latency-bound rollout less (cfg 5: 426 -> 412 us, tools/rollout_probe.py; staging the steps in LDS to write
// whole-trajectory runs was slower, 458 us: LDS traffic shares lgkmcnt with the per-step scalar loads)
__device__ __forceinline__ void st_nt2(double2* p, double a, double b) {
    typedef double d2v __attribute__((ext_vector_type(2)));
    __builtin_nontemporal_store(d2v{a, b}, reinterpret_cast<d2v*>(p));
}

// k_track_rollout with each trajectory on a lane pair (gym::rk4_pair): 2B threads, 128 B... of one lane's rows
// split between the pair (even lane: (th1, th2) and u; odd lane: (w1, w2)).  The chain of 500 dependent RK4 steps
// is the whole cost of this latency-bound kernel (B/32 wavefronts, one per SIMD), and the split shortens each
// step's instruction stream by ~1/3.  Bit-identical to k_track_rollout (tested).
__global__ __launch_bounds__(64) void k_track_rollout_pair(Dyn m, const double* __restrict__ x0,
                                                           const double* __restrict__ x_ff,
                                                           const double* __restrict__ u_ff,
                                                           const double* __restrict__ K, int64_t B, int N,
                                                           double* __restrict__ xo, double* __restrict__ uo) {
    const int64_t th = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const int64_t l = th >> 1;
    const bool odd = th & 1;
    if (l >= B) return;                    // both lanes of a pair, so the pair's DPP partners are always active
    const int T = N - 1;
    double2* xl = reinterpret_cast<double2*>(xo + 4 * (int64_t)N * l) + (odd ? 1 : 0);
    double2* ul = reinterpret_cast<double2*>(uo + 2 * (int64_t)T * l);
    double n0 = x0[4 * l], n1 = x0[4 * l + 1], n2 = x0[4 * l + 2], n3 = x0[4 * l + 3];
    xl[0] = odd ? make_double2(n2, n3) : make_double2(n0, n1);
    double k[8], r[4], f[2];
#pragma unroll
    for (int q = 0; q < 8; ++q) k[q] = K[q];
#pragma unroll
    for (int q = 0; q < 4; ++q) r[q] = x_ff[q];
    f[0] = u_ff[0]; f[1] = u_ff[1];
    const gym::PolyRegs pk = gym::poly_vgprs_all();   // every Horner coefficient in VGPRs
    Dyn dm = m;                            // the model in VGPRs across the step loop
    gym::in_vgpr(dm.b); gym::in_vgpr(dm.d); gym::in_vgpr(dm.a2b); gym::in_vgpr(dm.bb); gym::in_vgpr(dm.dad);
    gym::in_vgpr(dm.g1); gym::in_vgpr(dm.g2); gym::in_vgpr(dm.f1); gym::in_vgpr(dm.f2); gym::in_vgpr(dm.h);
    gym::in_vgpr(dm.h2); gym::in_vgpr(dm.h6);
    for (int t = 0; t < T; ++t) {
        const double d0 = n0 - r[0], d1 = n1 - r[1], d2 = n2 - r[2], d3 = n3 - r[3];
        double v0, v1;
        track_feedback(k, f, d0, d1, d2, d3, v0, v1);
        if (t + 1 < T) {
            const double* kn = K + 8 * (t + 1);
#pragma unroll
            for (int q = 0; q < 8; ++q) k[q] = kn[q];
#pragma unroll
            for (int q = 0; q < 4; ++q) r[q] = x_ff[4 * (t + 1) + q];
            f[0] = u_ff[2 * (t + 1)]; f[1] = u_ff[2 * (t + 1) + 1];
        }
        if (!odd) st_nt2(ul + t, v0, v1);
        gym::rk4_pair_fast(dm, odd, n0, n1, n2, n3, v1, pk);   // branch-free near path (gym::rk4_pair_fast)
        if (odd) st_nt2(xl + 2 * (t + 1), n2, n3);
        else st_nt2(xl + 2 * (t + 1), n0, n1);
    }
}

inline M44 m44(const double* p) { M44 m; for (int i = 0; i < 16; ++i) m.v[i] = p[i]; return m; }
inline M22 m22(const double* p) { M22 m; for (int i = 0; i < 4; ++i) m.v[i] = p[i]; return m; }
inline int launch_status() { return (int)hipGetLastError(); }

}  // namespace

extern "C" {

int gym_tv_lqr_gains(const double* A, const double* Bm, int32_t S, const double* A_pad, const double* B_pad,
                     const double Q[16], const double R[4], const double QT[16], int32_t L, int32_t nwin,
                     int32_t all_gains, int32_t discretize, double dt, double* K_out, void* s) {
    if (!A || !Bm || !Q || !R || !QT || !K_out || S <= 0 || L < 2 || nwin <= 0 || (all_gains && nwin != 1))
        return GYM_EINVAL;
    if ((nwin - 1) + (L - 2) >= S && (!A_pad || !B_pad)) return GYM_EINVAL;   // a window runs past the stages
    hipLaunchKernelGGL(k_tv_lqr_gains, dim3((nwin + 63) / 64), dim3(64), 0, (hipStream_t)s, A, Bm, S, A_pad, B_pad,
                       m44(Q), m22(R), QT, L, nwin, all_gains, discretize, dt, K_out);
    return launch_status();
}

int gym_dare_fixed_point(const double* A, const double* Bm, const double Q[16], const double R[4], int32_t max_iter,
                         double tol, double* P_out, int32_t* iters_out, void* s) {
    if (!A || !Bm || !Q || !R || !P_out || !iters_out || max_iter <= 0) return GYM_EINVAL;
    hipLaunchKernelGGL(k_dare_fixed_point, dim3(1), dim3(64), 0, (hipStream_t)s, A, Bm, m44(Q), m22(R), max_iter, tol,
                       P_out, iters_out);
    return launch_status();
}

int gym_mpc_gains(const gym_model* m, const double* x_ref, const double* u_ref, int32_t S, const double* x_f,
                  const double* u_f, const double Q[16], const double R[4], int32_t L, int32_t nwin, int32_t max_iter,
                  double tol, double* K_out, double* QT_out, int32_t* iters_out, void* s) {
    if (!m || !x_ref || !u_ref || !x_f || !u_f || !Q || !R || !K_out || !QT_out || !iters_out || S <= 0 || L < 2 ||
        L + 2 > kMpcMaxStages || nwin <= 0 || max_iter <= 0)
        return GYM_EINVAL;
    hipLaunchKernelGGL(k_mpc_gains, dim3((unsigned)((nwin + 3) / 4)), dim3(64), 0, (hipStream_t)s, Dyn(*m), x_ref,
                       u_ref, S, x_f, u_f, m44(Q), m22(R), L, nwin, max_iter, tol, K_out, QT_out, iters_out);
    return launch_status();
}

int gym_lq_forward(const double* A, const double* Bm, int32_t S, const double* A_pad, const double* B_pad,
                   int32_t discretize, double dt, const double* K, const double* x0, int32_t L, double* X, double* U,
                   void* s) {
    if (!A || !Bm || !K || !x0 || !X || !U || S <= 0 || L < 2) return GYM_EINVAL;
    if (L - 2 >= S && (!A_pad || !B_pad)) return GYM_EINVAL;
    hipLaunchKernelGGL(k_lq_forward, dim3(1), dim3(64), 0, (hipStream_t)s, A, Bm, S, A_pad, B_pad, discretize, dt, K,
                       x0, L, X, U);
    return launch_status();
}

int gym_track_rollout_ex(const gym_model* m, const double* x0, const double* x_ff, const double* u_ff,
                         const double* K, int64_t B, int32_t N, int32_t flags, double* x_out, double* u_out, void* s) {
    if (!m || !x0 || !x_ff || !u_ff || !K || !x_out || !u_out || B <= 0 || B > ((int64_t)1 << 30) || N < 2 ||
        (flags & ~GYM_TRACK_SINGLE))
        return GYM_EINVAL;
    if (flags & GYM_TRACK_SINGLE)
        hipLaunchKernelGGL(k_track_rollout, dim3((unsigned)((B + 63) / 64)), dim3(64), 0, (hipStream_t)s, Dyn(*m), x0,
                           x_ff, u_ff, K, B, N, x_out, u_out);
    else
        hipLaunchKernelGGL(k_track_rollout_pair, dim3((unsigned)((2 * B + 63) / 64)), dim3(64), 0, (hipStream_t)s,
                           Dyn(*m), x0, x_ff, u_ff, K, B, N, x_out, u_out);
    return launch_status();
}

int gym_track_rollout(const gym_model* m, const double* x0, const double* x_ff, const double* u_ff, const double* K,
                      int64_t B, int32_t N, double* x_out, double* u_out, void* s) {
    return gym_track_rollout_ex(m, x0, x_ff, u_ff, K, B, N, 0, x_out, u_out, s);
}

}  // extern "C"
