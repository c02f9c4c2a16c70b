/*
 * CPU ORACLE (test infrastructure only) -- plain-C restatement of the reference hot path.
 *
 * Checker and CPU baseline, never the product: only tests/, __graft_entry__.smoke() and
 * bench.py's cpu_baseline leg load this library (oracle/build/libacrobot_oracle.so).
 *
 * Scalar fp64, one lane per OpenMP iteration. It restates the per-lane algorithm of
 * /root/reference/trajectory_generation.py:298-398 (newton_Algorithm) with its primitives:
 *   rk4 ............... dynamics.py:177-195 (classic RK4, u held, dt = 2e-2)
 *   accel ............. dynamics.py:197-213 (M(q) qdd = tau - (C+F) qdot - G, tau = [0, u1])
 *   jac ............... dynamics.py:217-226 (A_c = df/dx, B_c = df/du, closed form)
 *   backward sweep .... trajectory_generation.py:166-216 (Euler A_d = I + dt A_c, B_d = dt B_c,
 *                       Gauss-Newton blocks 2Q, 2R, S = 0, Riccati K, sigma, dJ)
 *   closed loop ....... trajectory_generation.py:218-229
 *   total cost ........ trajectory_generation.py:231-252
 * Dense algebra is replaced by the closed forms that follow from the model's structure
 * (B_c[:,0] == 0, G diagonal => K row 0 == 0); the NumPy oracle (acrobot_np.py) keeps the
 * dense form and both are pinned to the reference's golden vectors in tests/.
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

typedef struct {
    double a, b, d, g1, g2, f1, f2, dt;  /* M11 = a + 2 b c2, M12 = d + b c2, M22 = d */
} orc_model;

typedef struct {
    double Q[4], R[2], QT[4];            /* diagonal weights (trajectory_generation.py:16-18) */
} orc_cost;

enum { ORC_ACTIVE = 0, ORC_CONVERGED = 1, ORC_LS_FAILED = 2, ORC_MAX_ITERS = 3 };

void orc_model_from_params(const double p[11], double dt, orc_model* m) {
    /* p = m1 m2 l1 lc1 l2 lc2 I1 I2 g f1 f2 (dynamics.py:15-61) */
    double m1 = p[0], m2 = p[1], l1 = p[2], lc1 = p[3], lc2 = p[5], I1 = p[6], I2 = p[7], g = p[8];
    m->a = I1 + I2 + lc1 * lc1 * m1 + m2 * (l1 * l1 + lc2 * lc2);
    m->b = m2 * l1 * lc2;
    m->d = I2 + lc2 * lc2 * m2;
    m->g1 = g * (lc1 * m1 + m2 * l1);
    m->g2 = g * m2 * lc2;
    m->f1 = p[9];
    m->f2 = p[10];
    m->dt = dt;
}

static inline void accel(const orc_model* m, const double x[4], double tau2, double qdd[2]) {
    double s1 = sin(x[0]), c1 = cos(x[0]), s2 = sin(x[1]), c2 = cos(x[1]);
    double s12 = s1 * c2 + c1 * s2;
    double w1 = x[2], w2 = x[3];
    double bs2 = m->b * s2;
    double M11 = m->a + 2.0 * m->b * c2, M12 = m->d + m->b * c2, M22 = m->d;
    double r1 = bs2 * w2 * (2.0 * w1 + w2) - m->f1 * w1 - (m->g1 * s1 + m->g2 * s12);
    double r2 = tau2 - bs2 * w1 * w1 - m->f2 * w2 - m->g2 * s12;
    double inv = 1.0 / (M11 * M22 - M12 * M12);
    qdd[0] = (M22 * r1 - M12 * r2) * inv;
    qdd[1] = (M11 * r2 - M12 * r1) * inv;
}

void orc_xdot(const orc_model* m, const double x[4], const double u[2], double xd[4]) {
    double q[2];
    accel(m, x, u[1], q);
    xd[0] = x[2]; xd[1] = x[3]; xd[2] = q[0]; xd[3] = q[1];
}

void orc_rk4(const orc_model* m, const double x[4], const double u[2], double xn[4]) {
    double k1[4], k2[4], k3[4], k4[4], y[4];
    const double h = m->dt, h2 = m->dt / 2;
    orc_xdot(m, x, u, k1);
    for (int i = 0; i < 4; i++) y[i] = x[i] + h2 * k1[i];
    orc_xdot(m, y, u, k2);
    for (int i = 0; i < 4; i++) y[i] = x[i] + h2 * k2[i];
    orc_xdot(m, y, u, k3);
    for (int i = 0; i < 4; i++) y[i] = x[i] + h * k3[i];
    orc_xdot(m, y, u, k4);
    for (int i = 0; i < 4; i++) xn[i] = x[i] + h * (k1[i] + 2 * k2[i] + 2 * k3[i] + k4[i]) / 6.0;
}

/* A_c rows 2,3 (rows 0,1 are e3^T, e4^T) and B_c[2:,1] (B_c[:,0] == 0). */
void orc_jac(const orc_model* m, const double x[4], const double u[2], double a2[4], double a3[4], double bc[2]) {
    double s1 = sin(x[0]), c1 = cos(x[0]), s2 = sin(x[1]), c2 = cos(x[1]);
    double s12 = s1 * c2 + c1 * s2, c12 = c1 * c2 - s1 * s2;
    double w1 = x[2], w2 = x[3];
    double b = m->b, bs2 = b * s2, bc2 = b * c2;
    double M11 = m->a + 2.0 * bc2, M12 = m->d + bc2, M22 = m->d;
    double r1 = bs2 * w2 * (2.0 * w1 + w2) - m->f1 * w1 - (m->g1 * s1 + m->g2 * s12);
    double r2 = u[1] - bs2 * w1 * w1 - m->f2 * w2 - m->g2 * s12;
    double inv = 1.0 / (M11 * M22 - M12 * M12);
    double q1 = (M22 * r1 - M12 * r2) * inv, q2 = (M11 * r2 - M12 * r1) * inv;
    /* column vectors v_j = d r/d x_j - (dM/dx_j) qdd */
    double v1[4], v2[4];
    v1[0] = -(m->g1 * c1 + m->g2 * c12);              v2[0] = -m->g2 * c12;
    v1[1] = bc2 * w2 * (2.0 * w1 + w2) - m->g2 * c12 + bs2 * (2.0 * q1 + q2);
    v2[1] = -bc2 * w1 * w1 - m->g2 * c12 + bs2 * q1;
    v1[2] = 2.0 * bs2 * w2 - m->f1;                   v2[2] = -2.0 * bs2 * w1;
    v1[3] = 2.0 * bs2 * (w1 + w2);                    v2[3] = -m->f2;
    for (int j = 0; j < 4; j++) {
        a2[j] = (M22 * v1[j] - M12 * v2[j]) * inv;
        a3[j] = (M11 * v2[j] - M12 * v1[j]) * inv;
    }
    bc[0] = -M12 * inv;
    bc[1] = M11 * inv;
}

static double stage_cost(const orc_cost* c, const double* x, const double* xr, const double* u, const double* ur) {
    double j = 0.0, ju = 0.0;
    for (int i = 0; i < 4; i++) { double e = x[i] - xr[i]; j += e * (c->Q[i] * e); }
    for (int i = 0; i < 2; i++) { double e = u[i] - ur[i]; ju += e * (c->R[i] * e); }
    return j + ju;
}

static double term_cost(const orc_cost* c, const double* x, const double* xr) {
    double j = 0.0;
    for (int i = 0; i < 4; i++) { double e = x[i] - xr[i]; j += e * (c->QT[i] * e); }
    return j;
}

double orc_total_cost(const orc_cost* c, const double* x, const double* u, const double* xr, const double* ur, int N) {
    double J = 0.0;
    for (int t = 0; t < N - 1; t++) J += stage_cost(c, x + 4 * t, xr + 4 * t, u + 2 * t, ur + 2 * t);
    return J + term_cost(c, x + 4 * (N - 1), xr + 4 * (N - 1));
}

/* Backward sweep: K1 (T,4) = row 1 of K_t (row 0 == 0), sig (T,2); returns dJ, *smax = max|sigma| */
double orc_backward(const orc_model* m, const orc_cost* c, const double* x, const double* u,
                    const double* xr, const double* ur, int N, double* K1, double* sig, double* smax) {
    const double dt = m->dt;
    double P[4][4] = {{0}}, p[4];
    for (int i = 0; i < 4; i++) { P[i][i] = 2.0 * c->QT[i]; p[i] = 2.0 * c->QT[i] * (x[4 * (N - 1) + i] - xr[4 * (N - 1) + i]); }
    double dJ = 0.0, sm = 0.0;
    for (int t = N - 2; t >= 0; t--) {
        const double* xt = x + 4 * t;
        const double* ut = u + 2 * t;
        double a2[4], a3[4], bc[2];
        orc_jac(m, xt, ut, a2, a3, bc);
        double A[4][4] = {{1, 0, dt, 0}, {0, 1, 0, dt}, {dt * a2[0], dt * a2[1], 1 + dt * a2[2], dt * a2[3]},
                          {dt * a3[0], dt * a3[1], dt * a3[2], 1 + dt * a3[3]}};
        double bd2 = dt * bc[0], bd3 = dt * bc[1];
        double q[4], r0, r1;
        for (int i = 0; i < 4; i++) q[i] = 2.0 * c->Q[i] * (xt[i] - xr[4 * t + i]);
        r0 = 2.0 * c->R[0] * (ut[0] - ur[2 * t]);
        r1 = 2.0 * c->R[1] * (ut[1] - ur[2 * t + 1]);
        double Pb[4];
        for (int i = 0; i < 4; i++) Pb[i] = P[i][2] * bd2 + P[i][3] * bd3;
        double G11 = 2.0 * c->R[1] + (bd2 * Pb[2] + bd3 * Pb[3]);
        double G00 = 2.0 * c->R[0];
        double F1[4];
        for (int j = 0; j < 4; j++) { F1[j] = 0; for (int k = 0; k < 4; k++) F1[j] += A[k][j] * Pb[k]; }
        double g0 = r0, g1 = r1 + (bd2 * p[2] + bd3 * p[3]);
        double k1[4];
        for (int j = 0; j < 4; j++) k1[j] = -F1[j] / G11;
        double s0 = -g0 / G00, s1 = -g1 / G11;
        dJ += g0 * s0 + g1 * s1;
        /* P <- 2Q + A^T P A - K^T G K ;  p <- q + A^T p - K^T G sigma */
        double PA[4][4], Pn[4][4], pn[4];
        for (int i = 0; i < 4; i++)
            for (int j = 0; j < 4; j++) { double s = 0; for (int k = 0; k < 4; k++) s += P[i][k] * A[k][j]; PA[i][j] = s; }
        for (int i = 0; i < 4; i++)
            for (int j = 0; j < 4; j++) {
                double s = 0; for (int k = 0; k < 4; k++) s += A[k][i] * PA[k][j];
                Pn[i][j] = (i == j ? 2.0 * c->Q[i] : 0.0) + s - k1[i] * G11 * k1[j];
            }
        for (int i = 0; i < 4; i++) {
            double s = 0; for (int k = 0; k < 4; k++) s += A[k][i] * p[k];
            pn[i] = q[i] + s - k1[i] * G11 * s1;
        }
        memcpy(P, Pn, sizeof P); memcpy(p, pn, sizeof p);
        for (int j = 0; j < 4; j++) K1[4 * t + j] = k1[j];
        sig[2 * t] = s0; sig[2 * t + 1] = s1;
        double a0 = fabs(s0), a1 = fabs(s1);
        if (a0 > sm || a0 != a0) sm = a0;
        if (a1 > sm || a1 != a1) sm = a1;
        if (sm != sm) sm = NAN;
    }
    *smax = sm;
    return dJ;
}

/* Closed-loop rollout with compact gains; returns total cost. */
double orc_forward(const orc_model* m, const orc_cost* c, const double* x, const double* u, const double* K1,
                   const double* sig, double gamma, const double* xr, const double* ur, int N, double* xn, double* un) {
    double J = 0.0;
    memcpy(xn, x, 4 * sizeof(double));
    for (int t = 0; t < N - 1; t++) {
        const double* xt = x + 4 * t;
        double* xnt = xn + 4 * t;
        double kd = 0.0;
        for (int j = 0; j < 4; j++) kd += K1[4 * t + j] * (xnt[j] - xt[j]);
        un[2 * t] = u[2 * t] + gamma * sig[2 * t];
        un[2 * t + 1] = (u[2 * t + 1] + kd) + gamma * sig[2 * t + 1];
        J += stage_cost(c, xnt, xr + 4 * t, un + 2 * t, ur + 2 * t);
        orc_rk4(m, xnt, un + 2 * t, xnt + 4);
    }
    return J + term_cost(c, xn + 4 * (N - 1), xr + 4 * (N - 1));
}

/* Optional per-iteration record of one lane (NULL pointers: not recorded).  Row k holds iteration k:
 * cost after the iteration (the reference's history['cost'][k+1]; NaN for a failed one, which appends none),
 * max|sigma| of its sweep (history['sigma_norm'][k]), the Armijo trials it evaluated, and the tightest
 * Armijo test of the iteration: min over its trials of |J_new - (J + c gamma dJ)| / max(|J|, tiny) --
 * how far the closest accept / reject call was from a tie (a rounding-level value flags a decision that
 * another restatement may take the other way). */
typedef struct {
    int hist_len;
    double* cost;
    double* smax;
    int32_t* trials;
    double* margin;
} orc_hist;

/* Newton / Armijo for one lane (trajectory_generation.py:298-398). Work buffers owned here. */
static void solve_lane(const orc_model* m, const orc_cost* c, const double* x0, const double* xr, const double* ur,
                       int N, int max_iters, double tol, double beta, double cc, double gamma0, int max_ls,
                       double* x, double* u, double* K1, double* sig, int32_t* n_iter, int32_t* status,
                       double* cost, int32_t* n_roll, const orc_hist* h, int64_t lane) {
    const int T = N - 1;
    double* xn = (double*)malloc(sizeof(double) * 4 * N);
    double* un = (double*)malloc(sizeof(double) * 2 * T);
    memset(u, 0, sizeof(double) * 2 * T);
    memcpy(x, x0, 4 * sizeof(double));
    for (int t = 0; t < T; t++) orc_rk4(m, x + 4 * t, u + 2 * t, x + 4 * (t + 1));
    double J = orc_total_cost(c, x, u, xr, ur, N);
    int st = ORC_ACTIVE, it = 0, nr = 0;
    for (int k = 0; k < max_iters && st == ORC_ACTIVE; k++) {
        double smax;
        double dJ = orc_backward(m, c, x, u, xr, ur, N, K1, sig, &smax);
        double g = gamma0, Jn = 0.0, tight = INFINITY;
        int ok = 0, i;
        for (i = 0; i < max_ls; i++) {
            Jn = orc_forward(m, c, x, u, K1, sig, g, xr, ur, N, xn, un);
            nr++;
            double rhs = J + cc * g * dJ;
            double mg = fabs(Jn - rhs) / fmax(fabs(J), 1e-300);
            if (mg < tight || mg != mg) tight = mg;
            if (Jn < rhs) { ok = 1; break; }
            g *= beta;
        }
        if (h && k < h->hist_len) {
            int64_t o = lane * h->hist_len + k;
            if (h->cost) h->cost[o] = ok ? Jn : NAN;
            if (h->smax) h->smax[o] = smax;
            if (h->trials) h->trials[o] = ok ? i + 1 : max_ls;
            if (h->margin) h->margin[o] = tight;
        }
        it++;
        if (!ok) { st = ORC_LS_FAILED; break; }
        memcpy(x, xn, sizeof(double) * 4 * N);
        memcpy(u, un, sizeof(double) * 2 * T);
        J = Jn;
        if (smax < tol) st = ORC_CONVERGED;
    }
    if (st == ORC_ACTIVE) st = ORC_MAX_ITERS;
    *n_iter = it; *status = st; *cost = J; *n_roll = nr;
    free(xn); free(un);
}

static void solve_batch(const orc_model* m, const orc_cost* c, const double* x0, const double* xr, const double* ur,
                        int64_t B, int N, int max_iters, double tol, double beta, double cc, double gamma0, int max_ls,
                        double* x, double* u, double* K1, double* sig, int32_t* n_iter, int32_t* status, double* cost,
                        int32_t* n_roll, const orc_hist* h) {
    const int64_t T = N - 1;
#pragma omp parallel for schedule(dynamic, 1)
    for (int64_t l = 0; l < B; l++)
        solve_lane(m, c, x0 + 4 * l, xr, ur, N, max_iters, tol, beta, cc, gamma0, max_ls, x + 4 * N * l,
                   u + 2 * T * l, K1 + 4 * T * l, sig + 2 * T * l, n_iter + l, status + l, cost + l, n_roll + l, h, l);
}

/* Batched entry: lanes are independent; x0 (B,4) -> x (B,N,4), u (B,T,2), K1 (B,T,4), sig (B,T,2). */
void orc_newton_solve(const orc_model* m, const orc_cost* c, const double* x0, const double* xr, const double* ur,
                      int64_t B, int N, int max_iters, double tol, double beta, double cc, double gamma0, int max_ls,
                      double* x, double* u, double* K1, double* sig, int32_t* n_iter, int32_t* status, double* cost,
                      int32_t* n_roll) {
    solve_batch(m, c, x0, xr, ur, B, N, max_iters, tol, beta, cc, gamma0, max_ls, x, u, K1, sig, n_iter, status, cost,
                n_roll, NULL);
}

/* The same, with the per-iteration record of every lane: hist_* (B, hist_len), row-major per lane. */
void orc_newton_solve_hist(const orc_model* m, const orc_cost* c, const double* x0, const double* xr,
                           const double* ur, int64_t B, int N, int max_iters, double tol, double beta, double cc,
                           double gamma0, int max_ls, double* x, double* u, double* K1, double* sig, int32_t* n_iter,
                           int32_t* status, double* cost, int32_t* n_roll, int hist_len, double* hist_cost,
                           double* hist_smax, int32_t* hist_trials, double* hist_margin) {
    orc_hist h = {hist_len, hist_cost, hist_smax, hist_trials, hist_margin};
    solve_batch(m, c, x0, xr, ur, B, N, max_iters, tol, beta, cc, gamma0, max_ls, x, u, K1, sig, n_iter, status, cost,
                n_roll, &h);
}

/* Fixed number of Newton iterations per lane (no convergence stop) -- a bounded CPU sample for bench.py. */
void orc_newton_iters(const orc_model* m, const orc_cost* c, const double* x0, const double* xr, const double* ur,
                      int64_t B, int N, int iters, double beta, double cc, double gamma0, int max_ls,
                      double* x, double* u, double* K1, double* sig, int32_t* n_iter, int32_t* status, double* cost,
                      int32_t* n_roll) {
    orc_newton_solve(m, c, x0, xr, ur, B, N, iters, -1.0, beta, cc, gamma0, max_ls, x, u, K1, sig, n_iter, status,
                     cost, n_roll);
}
