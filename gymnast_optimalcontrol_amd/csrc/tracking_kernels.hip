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
        const double v0 = f[0] + (((k[0] * d0 + k[1] * d1) + k[2] * d2) + k[3] * d3);
        const double v1 = f[1] + (((k[4] * d0 + k[5] * d1) + k[6] * d2) + k[7] * d3);
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

int gym_lq_forward(const double* A, const double* Bm, int32_t S, const double* A_pad, const double* B_pad,
                   int32_t discretize, double dt, const double* K, const double* x0, int32_t L, double* X, double* U,
                   void* s) {
    if (!A || !Bm || !K || !x0 || !X || !U || S <= 0 || L < 2) return GYM_EINVAL;
    if (L - 2 >= S && (!A_pad || !B_pad)) return GYM_EINVAL;
    hipLaunchKernelGGL(k_lq_forward, dim3(1), dim3(64), 0, (hipStream_t)s, A, Bm, S, A_pad, B_pad, discretize, dt, K,
                       x0, L, X, U);
    return launch_status();
}

int gym_track_rollout(const gym_model* m, const double* x0, const double* x_ff, const double* u_ff, const double* K,
                      int64_t B, int32_t N, double* x_out, double* u_out, void* s) {
    if (!m || !x0 || !x_ff || !u_ff || !K || !x_out || !u_out || B <= 0 || B > ((int64_t)1 << 31) || N < 2)
        return GYM_EINVAL;
    hipLaunchKernelGGL(k_track_rollout, dim3((unsigned)((B + 63) / 64)), dim3(64), 0, (hipStream_t)s, Dyn(*m), x0, x_ff,
                       u_ff, K, B, N, x_out, u_out);
    return launch_status();
}

}  // extern "C"
