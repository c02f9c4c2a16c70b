// Device-side building blocks of the acrobot engine (gfx950, fp64, one trajectory per lane).
//
// Model and algorithm: /root/reference/dynamics.py and trajectory_generation.py (see the
// citations on each function).  Everything here is register-resident per lane; the HBM
// traffic of a kernel is exactly the SoA streams it loads/stores per stage.
#pragma once
#include <hip/hip_runtime.h>

#include "gymnast_acrobot.h"

namespace gym {

constexpr int kWave = 64;

// Coefficients hoisted out of the time loop (uniform per launch).
struct Dyn {
    double b, d, a2b, bb, dad, g1, g2, f1, f2, h, h2, h6;
    __device__ __forceinline__ explicit Dyn(const gym_model& m)
        : b(m.b), d(m.d), a2b(m.a), bb(m.b * m.b), dad(m.d * (m.a - m.d)), g1(m.g1), g2(m.g2), f1(m.f1),
          f2(m.f2), h(m.dt), h2(m.dt * 0.5), h6(1.0 / 6.0) {}
};

// Joint accelerations qdd = M(th2)^-1 (tau - (C+F) w - G), tau = [0, tau2]   (dynamics.py:197-213,
// M/C/G/F of dynamics.py:63-90).  det M = d (a - d) - b^2 cos^2(th2) > 0 is formed without cancellation.
__device__ __forceinline__ void accel(const Dyn& m, double th1, double th2, double w1, double w2, double tau2,
                                      double& q1, double& q2) {
    double s1, c1, s2, c2;
    sincos(th1, &s1, &c1);
    sincos(th2, &s2, &c2);
    const double s12 = s1 * c2 + c1 * s2;            // sin(th1 + th2)
    const double bs2 = m.b * s2;
    const double M11 = m.a2b + 2.0 * m.b * c2;
    const double M12 = m.d + m.b * c2;
    const double r1 = bs2 * w2 * (2.0 * w1 + w2) - m.f1 * w1 - (m.g1 * s1 + m.g2 * s12);
    const double r2 = tau2 - bs2 * w1 * w1 - m.f2 * w2 - m.g2 * s12;
    const double inv = 1.0 / (m.dad - m.bb * (c2 * c2));
    q1 = (m.d * r1 - M12 * r2) * inv;
    q2 = (M11 * r2 - M12 * r1) * inv;
}

// Classic RK4 with the control held over the step (dynamics.py:177-195), in place.
__device__ __forceinline__ void rk4(const Dyn& m, double& x0, double& x1, double& x2, double& x3, double tau2) {
    double a1, b1, a2, b2, a3, b3, a4, b4;
    accel(m, x0, x1, x2, x3, tau2, a1, b1);                       // k1 = (x2, x3, a1, b1)
    const double y0 = x0 + m.h2 * x2, y1 = x1 + m.h2 * x3, y2 = x2 + m.h2 * a1, y3 = x3 + m.h2 * b1;
    accel(m, y0, y1, y2, y3, tau2, a2, b2);                       // k2 = (y2, y3, a2, b2)
    const double z0 = x0 + m.h2 * y2, z1 = x1 + m.h2 * y3, z2 = x2 + m.h2 * a2, z3 = x3 + m.h2 * b2;
    accel(m, z0, z1, z2, z3, tau2, a3, b3);                       // k3 = (z2, z3, a3, b3)
    const double v0 = x0 + m.h * z2, v1 = x1 + m.h * z3, v2 = x2 + m.h * a3, v3 = x3 + m.h * b3;
    accel(m, v0, v1, v2, v3, tau2, a4, b4);                       // k4 = (v2, v3, a4, b4)
    const double n0 = x0 + (m.h * (((x2 + 2.0 * y2) + 2.0 * z2) + v2)) * m.h6;
    const double n1 = x1 + (m.h * (((x3 + 2.0 * y3) + 2.0 * z3) + v3)) * m.h6;
    const double n2 = x2 + (m.h * (((a1 + 2.0 * a2) + 2.0 * a3) + a4)) * m.h6;
    const double n3 = x3 + (m.h * (((b1 + 2.0 * b2) + 2.0 * b3) + b4)) * m.h6;
    x0 = n0; x1 = n1; x2 = n2; x3 = n3;
}

// Continuous Jacobians (dynamics.py:157-170, 217-226): rows 0,1 of A_c are e3^T, e4^T; B_c[:,0] == 0.
// Returns rows 2,3 of A_c (a2, a3) and B_c[2:,1] (bc2, bc3).
struct Jac {
    double a2[4], a3[4], bc2, bc3;
};

__device__ __forceinline__ Jac jacobian(const Dyn& m, double th1, double th2, double w1, double w2, double tau2) {
    double s1, c1, s2, c2;
    sincos(th1, &s1, &c1);
    sincos(th2, &s2, &c2);
    const double s12 = s1 * c2 + c1 * s2, c12 = c1 * c2 - s1 * s2;
    const double bs2 = m.b * s2, bc2 = m.b * c2;
    const double M11 = m.a2b + 2.0 * bc2, M12 = m.d + bc2;
    const double r1 = bs2 * w2 * (2.0 * w1 + w2) - m.f1 * w1 - (m.g1 * s1 + m.g2 * s12);
    const double r2 = tau2 - bs2 * w1 * w1 - m.f2 * w2 - m.g2 * s12;
    const double inv = 1.0 / (m.dad - m.bb * (c2 * c2));
    const double q1 = (m.d * r1 - M12 * r2) * inv, q2 = (M11 * r2 - M12 * r1) * inv;
    // d qdd / d x_j = M^-1 (d r/d x_j - (d M/d x_j) qdd);  only dM/dth2 != 0.
    const double gc = m.g2 * c12;
    double v1[4], v2[4];
    v1[0] = -(m.g1 * c1 + gc);                               v2[0] = -gc;
    v1[1] = bc2 * w2 * (2.0 * w1 + w2) - gc + bs2 * (2.0 * q1 + q2);
    v2[1] = -bc2 * w1 * w1 - gc + bs2 * q1;
    v1[2] = 2.0 * bs2 * w2 - m.f1;                           v2[2] = -2.0 * bs2 * w1;
    v1[3] = 2.0 * bs2 * (w1 + w2);                           v2[3] = -m.f2;
    Jac J;
    const double Md = m.d * inv, M12i = M12 * inv, M11i = M11 * inv;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        J.a2[j] = Md * v1[j] - M12i * v2[j];
        J.a3[j] = M11i * v2[j] - M12i * v1[j];
    }
    J.bc2 = -M12i;
    J.bc3 = M11i;
    return J;
}

// NaN-propagating running max of |v| (np.max(np.abs(sigma)) returns NaN if any entry is NaN).
__device__ __forceinline__ double nanmax_abs(double acc, double v) {
    const double a = fabs(v);
    return (acc != acc || a <= acc) ? acc : a;
}

}  // namespace gym
