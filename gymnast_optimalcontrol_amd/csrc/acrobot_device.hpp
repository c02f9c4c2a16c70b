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

// Coefficients hoisted out of the time loop (uniform per launch).  Built on the host and passed to the
// kernels by value, so they sit in SGPRs (kernel arguments) instead of occupying per-lane VGPRs; the
// derived products are IEEE-rounded identically on host and device.
struct Dyn {
    double b, d, a2b, bb, dad, g1, g2, f1, f2, h, h2, h6;
    Dyn() = default;
    __host__ __device__ __forceinline__ explicit Dyn(const gym_model& m)
        : b(m.b), d(m.d), a2b(m.a), bb(m.b * m.b), dad(m.d * (m.a - m.d)), g1(m.g1), g2(m.g2), f1(m.f1),
          f2(m.f2), h(m.dt), h2(m.dt * 0.5), h6(1.0 / 6.0) {}
};

// ------------------------------------------------------------------------------------------
// fp64 sin/cos for the arguments this model produces.  ocml's sincos carries the reduced
// argument as a double-double and a Payne-Hanek path (~60-75 VALU per call); the angles of an
// acrobot trajectory are moderate, so a 2-term Cody-Waite reduction with FMA (exact first step
// for |k| < 2^20) and the fdlibm minimax kernels on [-pi/4, pi/4] give the same absolute accuracy
// (~1.5 ulp absolute, checked against long-double sin/cos) in ~30 instructions.
// Domain: |x| < 2^20 * pi/2 ~ 1.6e6 rad.  Beyond it (or for inf/NaN) both results are NaN: a lane
// whose joint angle has reached 2.5e5 revolutions has diverged (RK4 at dt = 0.02 is unstable long
// before), and NaN makes its cost NaN so the Armijo test fails exactly as the reference's does for
// a non-finite trajectory.  Keeping ocml's full-range path out of the kernels saves ~25 VGPRs.
// ------------------------------------------------------------------------------------------
// fdlibm minimax kernels: sin(r), cos(r) for |r| <= pi/4.
// The innermost Horner step fma(z, C6, C5) has two constant operands; a VALU instruction reads at most
// one SGPR/literal, so the compiler re-materialises one of them with a v_mov_b64 at every use (16 per
// RK4 step).  PolyRegs carries those four coefficients; a stage loop takes a VGPR-resident copy
// (poly_vgprs) once, outside the loop.  Same constants, same operations: the same bits.
// The other coefficients (s4..s1, c4..c1) are literals in poly_lits() / poly_vgprs(); poly_vgprs_all() holds them
// in VGPRs too, for a latency-bound loop whose three-address Horner steps (GYM_HORNER_VOP3) need every addend in a
// VGPR and whose register budget lets them stay there (otherwise each is re-copied from an SGPR at every use).
struct PolyRegs {
    double s6, s5, c6, c5;
    double s4, s3, s2, s1, c4, c3, c2, c1;
};
__device__ __forceinline__ PolyRegs poly_lits() {
    return PolyRegs{1.58969099521155010221e-10, -2.50507602534068634195e-08, -1.13596475577881948265e-11,
                    2.08757232129817482790e-09,
                    2.75573137070700676789e-06, -1.98412698298579493134e-04, 8.33333333332248946124e-03,
                    -1.66666666666666324348e-01,
                    -2.75573143513906633035e-07, 2.48015872894767294178e-05, -1.38888888888741095749e-03,
                    4.16666666666666019037e-02};
}
__device__ __forceinline__ void in_vgpr(double& v) { asm volatile("" : "+v"(v)); }
__device__ __forceinline__ PolyRegs poly_vgprs() {
    PolyRegs k = poly_lits();
    in_vgpr(k.s6); in_vgpr(k.s5); in_vgpr(k.c6); in_vgpr(k.c5);
    return k;
}
__device__ __forceinline__ PolyRegs poly_vgprs_all() {
    PolyRegs k = poly_vgprs();
    in_vgpr(k.s4); in_vgpr(k.s3); in_vgpr(k.s2); in_vgpr(k.s1);
    in_vgpr(k.c4); in_vgpr(k.c3); in_vgpr(k.c2); in_vgpr(k.c1);
    return k;
}

// Horner step fma(z, p, c) with a constant addend c.  GYM_HORNER_VOP3 (set by a translation unit before this
// header) emits it as a three-address v_fma_f64 with c held in a VGPR: the compiler otherwise forms the
// two-address v_fmac_f64 (accumulator = addend) and, c being live across the loop, copies it first with a
// v_mov_b64 at every step (8 per rotation).  Same operation, same bits.  Every operand is a plain VGPR and the
// result is consumed by ordinary VALU code (never directly by DPP), so no hazard is hidden in the asm.
#ifndef GYM_HORNER_VOP3
#define GYM_HORNER_VOP3 0
#endif
template <bool V3 = GYM_HORNER_VOP3>
__device__ __forceinline__ double hfma(double z, double p, double c) {
    if constexpr (V3) {
        double r;
        asm("v_fma_f64 %0, %1, %2, %3" : "=v"(r) : "v"(z), "v"(p), "v"(c));
        return r;
    } else {
        return fma(z, p, c);
    }
}

template <bool V3 = GYM_HORNER_VOP3>
__device__ __forceinline__ double ksin(double r, double z, const PolyRegs& k) {
#pragma clang fp contract(on)   // context-independent bits: FMA contraction inside an expression only
    return fma(r * z, hfma<V3>(z, hfma<V3>(z, hfma<V3>(z, hfma<V3>(z, fma(z, k.s6, k.s5), k.s4), k.s3), k.s2),
        k.s1), r);
}
template <bool V3 = GYM_HORNER_VOP3>
__device__ __forceinline__ double kcos(double z, const PolyRegs& k) {
#pragma clang fp contract(on)   // context-independent bits: FMA contraction inside an expression only
    return fma(z * z, hfma<V3>(z, hfma<V3>(z, hfma<V3>(z, hfma<V3>(z, fma(z, k.c6, k.c5), k.c4), k.c3), k.c2),
        k.c1), fma(-0.5, z, 1.0));
}

template <bool V3 = GYM_HORNER_VOP3>
__device__ __forceinline__ void fast_sincos(double x, double* s, double* c, const PolyRegs& k = poly_lits()) {
#pragma clang fp contract(on)   // context-independent bits: FMA contraction inside an expression only
    constexpr double kTwoOverPi = 6.36619772367581382433e-01;
    constexpr double kPio2Hi = 1.57079632679489655800e+00;   // 0x3FF921FB54442D18
    constexpr double kPio2Lo = 6.12323399573676603587e-17;   // 0x3C91A62633145C07
    const double kq = __builtin_rint(x * kTwoOverPi);
    // outside the domain: NaN, by replacing the high word only (kq's bits otherwise: one select, not two)
    const uint64_t kb = __builtin_bit_cast(uint64_t, kq);
    const uint32_t qh = (fabs(kq) < 1048576.0) ? (uint32_t)(kb >> 32) : 0x7FF80000u;
    const double qn = __builtin_bit_cast(double, ((uint64_t)qh << 32) | (kb & 0xFFFFFFFFull));
    const double r = fma(-qn, kPio2Lo, fma(-qn, kPio2Hi, x));
    const double z = r * r;
    const double sr = ksin<V3>(r, z, k);
    const double cr = kcos<V3>(z, k);
    const uint32_t q = (uint32_t)(int)qn;  // v_cvt_i32_f64 maps NaN to 0
    const double ss = (q & 1) ? cr : sr;   // quadrant rotation
    const double cc = (q & 1) ? sr : cr;
    // signs: quadrant bit 1 of q (of q + 1 for the cosine) moved to the sign bit and xor'ed in, which is negation
    // bit for bit (NaN included), without a compare and a select
    const uint64_t ns = (uint64_t)((q << 30) & 0x80000000u) << 32;
    const uint64_t nc = (uint64_t)(((q + 1u) << 30) & 0x80000000u) << 32;
    *s = __builtin_bit_cast(double, __builtin_bit_cast(uint64_t, ss) ^ ns);
    *c = __builtin_bit_cast(double, __builtin_bit_cast(uint64_t, cc) ^ nc);
}

// 1/v for v in the well-conditioned range of det M: hardware reciprocal + two Newton steps.
__device__ __forceinline__ double recip(double v) {
#pragma clang fp contract(on)   // context-independent bits: FMA contraction inside an expression only
    double r = __builtin_amdgcn_rcp(v);
    double e = fma(-v, r, 1.0);
    r = fma(r, e, r);
    e = fma(-v, r, 1.0);
    return fma(r, e, r);
}

// Joint accelerations qdd = M(th2)^-1 (tau - (C+F) w - G), tau = [0, tau2]   (dynamics.py:197-213,
// M/C/G/F of dynamics.py:63-90).  det M = d (a - d) - b^2 cos^2(th2) > 0 is formed without cancellation.
__device__ __forceinline__ void accel(const Dyn& m, double th1, double th2, double w1, double w2, double tau2,
                                      double& q1, double& q2) {
#pragma clang fp contract(on)   // context-independent bits: FMA contraction inside an expression only
    double s1, c1, s2, c2;
    fast_sincos(th1, &s1, &c1);
    fast_sincos(th2, &s2, &c2);
    const double s12 = s1 * c2 + c1 * s2;            // sin(th1 + th2)
    const double bs2 = m.b * s2;
    const double M11 = m.a2b + 2.0 * m.b * c2;
    const double M12 = m.d + m.b * c2;
    const double r1 = bs2 * w2 * (2.0 * w1 + w2) - m.f1 * w1 - (m.g1 * s1 + m.g2 * s12);
    const double r2 = tau2 - bs2 * w1 * w1 - m.f2 * w2 - m.g2 * s12;
    const double inv = recip(m.dad - m.bb * (c2 * c2));
    q1 = (m.d * r1 - M12 * r2) * inv;
    q2 = (M11 * r2 - M12 * r1) * inv;
}

// accel() from precomputed sin/cos of both joint angles.
__device__ __forceinline__ void accel_sc(const Dyn& m, double s1, double c1, double s2, double c2, double w1,
                                         double w2, double tau2, double& q1, double& q2) {
#pragma clang fp contract(on)   // context-independent bits: FMA contraction inside an expression only
    const double s12 = s1 * c2 + c1 * s2;            // sin(th1 + th2)
    const double bs2 = m.b * s2;
    const double M11 = m.a2b + 2.0 * m.b * c2;
    const double M12 = m.d + m.b * c2;
    const double r1 = bs2 * w2 * (2.0 * w1 + w2) - m.f1 * w1 - (m.g1 * s1 + m.g2 * s12);
    const double r2 = tau2 - bs2 * w1 * w1 - m.f2 * w2 - m.g2 * s12;
    const double inv = recip(m.dad - m.bb * (c2 * c2));
    q1 = (m.d * r1 - M12 * r2) * inv;
    q2 = (M11 * r2 - M12 * r1) * inv;
}

// sin/cos of the RK4 sub-step angles (th1 + d1, th2 + d2) from those of the step's base angles by angle
// addition: cos/sin(d) from the minimax kernels (no argument reduction, no quadrant logic) plus a
// rotation, ~20 VALU instead of ~40 for a reduction from scratch.  d = (h/2) w or h w is small; a lane
// with |d| > pi/4 (|w| > 39 rad/s) reduces both arguments from scratch instead.  The choice is per lane,
// so a lane's arithmetic never depends on which other lanes share its wavefront.
template <bool V3 = GYM_HORNER_VOP3>
__device__ __forceinline__ void rotate(double s, double c, double d, double& so, double& co, const PolyRegs& k) {
#pragma clang fp contract(on)   // context-independent bits: FMA contraction inside an expression only
    const double z = d * d;
    const double sd = ksin<V3>(d, z, k), cd = kcos<V3>(z, k);
    so = fma(s, cd, c * sd);
    co = fma(c, cd, -(s * sd));
}

__device__ __forceinline__ void substep_sincos(double th1, double th2, double d1, double d2, double s1, double c1,
                                               double s2, double c2, double& t1, double& u1, double& t2,
                                               double& u2, const PolyRegs& k) {
    constexpr double kPio4 = 0.78539816339744830962;
    if (__builtin_expect(fabs(d1) <= kPio4 && fabs(d2) <= kPio4, 1)) {
        rotate(s1, c1, d1, t1, u1, k);
        rotate(s2, c2, d2, t2, u2, k);
    } else {   // also taken by NaN lanes
        fast_sincos(th1 + d1, &t1, &u1, k);
        fast_sincos(th2 + d2, &t2, &u2, k);
    }
}

// Classic RK4 with the control held over the step (dynamics.py:177-195), in place.  Only the step's
// base angles are reduced from scratch; the three sub-step states' angles x + d, d = (h/2) k1, (h/2) k2,
// h k3, get their sin/cos by angle addition (substep_sincos).
__device__ __forceinline__ void rk4(const Dyn& m, double& x0, double& x1, double& x2, double& x3, double tau2,
                                    const PolyRegs& k = poly_lits()) {
#pragma clang fp contract(on)   // context-independent bits: FMA contraction inside an expression only
    double a1, b1, a2, b2, a3, b3, a4, b4;
    double s1, c1, s2, c2, t1, u1, t2, u2;
    fast_sincos(x0, &s1, &c1, k);
    fast_sincos(x1, &s2, &c2, k);
    accel_sc(m, s1, c1, s2, c2, x2, x3, tau2, a1, b1);            // k1 = (x2, x3, a1, b1)
    const double y2 = x2 + m.h2 * a1, y3 = x3 + m.h2 * b1;
    substep_sincos(x0, x1, m.h2 * x2, m.h2 * x3, s1, c1, s2, c2, t1, u1, t2, u2, k);
    accel_sc(m, t1, u1, t2, u2, y2, y3, tau2, a2, b2);            // k2 = (y2, y3, a2, b2)
    const double z2 = x2 + m.h2 * a2, z3 = x3 + m.h2 * b2;
    substep_sincos(x0, x1, m.h2 * y2, m.h2 * y3, s1, c1, s2, c2, t1, u1, t2, u2, k);
    accel_sc(m, t1, u1, t2, u2, z2, z3, tau2, a3, b3);            // k3 = (z2, z3, a3, b3)
    const double v2 = x2 + m.h * a3, v3 = x3 + m.h * b3;
    substep_sincos(x0, x1, m.h * z2, m.h * z3, s1, c1, s2, c2, t1, u1, t2, u2, k);
    accel_sc(m, t1, u1, t2, u2, v2, v3, tau2, a4, b4);            // k4 = (v2, v3, a4, b4)
    const double n0 = x0 + (m.h * (((x2 + 2.0 * y2) + 2.0 * z2) + v2)) * m.h6;
    const double n1 = x1 + (m.h * (((x3 + 2.0 * y3) + 2.0 * z3) + v3)) * m.h6;
    const double n2 = x2 + (m.h * (((a1 + 2.0 * a2) + 2.0 * a3) + a4)) * m.h6;
    const double n3 = x3 + (m.h * (((b1 + 2.0 * b2) + 2.0 * b3) + b4)) * m.h6;
    x0 = n0; x1 = n1; x2 = n2; x3 = n3;
}

// rk4 with every sub-step on the near path and no per-sub-step branch (as rk4_pair_near below): false for a lane
// whose sub-step increments leave |d| <= pi/4 (or are NaN); where true, rk4's values bit for bit.
__device__ __forceinline__ bool rk4_near(const Dyn& m, double& x0, double& x1, double& x2, double& x3, double tau2,
                                         const PolyRegs& k = poly_lits()) {
#pragma clang fp contract(on)   // context-independent bits: FMA contraction inside an expression only
    constexpr double kPio4 = 0.78539816339744830962;
    double a1, b1, a2, b2, a3, b3, a4, b4;
    double s1, c1, s2, c2, t1, u1, t2, u2;
    bool ok = true;
    auto sub = [&](double d1, double d2) {
        ok &= (fabs(d1) <= kPio4) & (fabs(d2) <= kPio4);
        rotate(s1, c1, d1, t1, u1, k);
        rotate(s2, c2, d2, t2, u2, k);
    };
    fast_sincos(x0, &s1, &c1, k);
    fast_sincos(x1, &s2, &c2, k);
    accel_sc(m, s1, c1, s2, c2, x2, x3, tau2, a1, b1);            // k1 = (x2, x3, a1, b1)
    const double y2 = x2 + m.h2 * a1, y3 = x3 + m.h2 * b1;
    sub(m.h2 * x2, m.h2 * x3);
    accel_sc(m, t1, u1, t2, u2, y2, y3, tau2, a2, b2);            // k2 = (y2, y3, a2, b2)
    const double z2 = x2 + m.h2 * a2, z3 = x3 + m.h2 * b2;
    sub(m.h2 * y2, m.h2 * y3);
    accel_sc(m, t1, u1, t2, u2, z2, z3, tau2, a3, b3);            // k3 = (z2, z3, a3, b3)
    const double v2 = x2 + m.h * a3, v3 = x3 + m.h * b3;
    sub(m.h * z2, m.h * z3);
    accel_sc(m, t1, u1, t2, u2, v2, v3, tau2, a4, b4);            // k4 = (v2, v3, a4, b4)
    const double n0 = x0 + (m.h * (((x2 + 2.0 * y2) + 2.0 * z2) + v2)) * m.h6;
    const double n1 = x1 + (m.h * (((x3 + 2.0 * y3) + 2.0 * z3) + v3)) * m.h6;
    const double n2 = x2 + (m.h * (((a1 + 2.0 * a2) + 2.0 * a3) + a4)) * m.h6;
    const double n3 = x3 + (m.h * (((b1 + 2.0 * b2) + 2.0 * b3) + b4)) * m.h6;
    x0 = n0; x1 = n1; x2 = n2; x3 = n3;
    return ok;
}
// rk4 through rk4_near, re-run by rk4 only for the lanes that need a far-path sub-step (per lane: no DPP here, so
// the re-run branch may be divergent).  Bit-identical to rk4.
__device__ __forceinline__ void rk4_fast(const Dyn& m, double& x0, double& x1, double& x2, double& x3, double tau2,
                                         const PolyRegs& k = poly_lits()) {
    const double s0 = x0, s1 = x1, s2 = x2, s3 = x3;
    if (__builtin_expect(!rk4_near(m, x0, x1, x2, x3, tau2, k), 0)) {
        x0 = s0; x1 = s1; x2 = s2; x3 = s3;
        rk4(m, x0, x1, x2, x3, tau2, k);
    }
}

// ------------------------------------------------------------------------------------------
// One trajectory on a lane pair (lanes 2p, 2p+1 of a wavefront): RK4 with the joint-angle trigonometry split.
// For a latency-bound rollout (one wavefront per SIMD, each step a dependent chain) the wave's instruction
// count per step is its time.  Both lanes hold the whole state; the even lane reduces / rotates the joint-1
// angle, the odd lane the joint-2 angle, and four DPP broadcasts inside the quad give both lanes all four
// sin/cos values; the accelerations and the update are evaluated by both (the same inputs, the same code:
// the same bits).  Every value is the one gym::rk4 computes with the same operations, so the result is
// bit-identical to rk4() (tested); ~200 instead of ~290 fp64 instructions per lane and step.
// ------------------------------------------------------------------------------------------
template <int CTRL>   // DPP move of a double (two 32-bit halves) within quads
__device__ __forceinline__ double dpp_d(double v) {
    const long long b = __double_as_longlong(v);
    const int lo = __builtin_amdgcn_mov_dpp((int)b, CTRL, 0xF, 0xF, false);
    const int hi = __builtin_amdgcn_mov_dpp((int)(b >> 32), CTRL, 0xF, 0xF, false);
    return __longlong_as_double(((long long)hi << 32) | (unsigned)lo);
}
__device__ __forceinline__ double pair_even(double v) { return dpp_d<0xA0>(v); }   // quad_perm [0,0,2,2]
__device__ __forceinline__ double pair_odd(double v) { return dpp_d<0xF5>(v); }    // quad_perm [1,1,3,3]

// substep_sincos() on a lane pair: this lane's angle tho (th1 on the even lane, th2 on the odd one), its
// base sin/cos (so, co) and the angle increments d1, d2 of both joints (both lanes: the same branch)
template <bool V3 = GYM_HORNER_VOP3>
__device__ __forceinline__ void substep_sincos_pair(bool odd, double tho, double d1, double d2, double so, double co,
                                                    double& t1, double& u1, double& t2, double& u2,
                                                    const PolyRegs& k) {
    constexpr double kPio4 = 0.78539816339744830962;
    const double d = odd ? d2 : d1;
    double to, uo;
    if (__builtin_expect(fabs(d1) <= kPio4 && fabs(d2) <= kPio4, 1)) {
        rotate<V3>(so, co, d, to, uo, k);
    } else {   // also taken by NaN lanes
        fast_sincos<V3>(tho + d, &to, &uo, k);
    }
    t1 = pair_even(to); u1 = pair_even(uo);
    t2 = pair_odd(to);  u2 = pair_odd(uo);
}

template <bool V3 = GYM_HORNER_VOP3>
__device__ __forceinline__ void rk4_pair(const Dyn& m, bool odd, double& x0, double& x1, double& x2, double& x3,
                                         double tau2, const PolyRegs& k = poly_lits()) {
#pragma clang fp contract(on)   // context-independent bits: FMA contraction inside an expression only
    double a1, b1, a2, b2, a3, b3, a4, b4;
    double t1, u1, t2, u2;
    const double tho = odd ? x1 : x0;
    double so, co;
    fast_sincos<V3>(tho, &so, &co, k);
    const double s1 = pair_even(so), c1 = pair_even(co), s2 = pair_odd(so), c2 = pair_odd(co);
    accel_sc(m, s1, c1, s2, c2, x2, x3, tau2, a1, b1);            // k1 = (x2, x3, a1, b1)
    const double y2 = x2 + m.h2 * a1, y3 = x3 + m.h2 * b1;
    substep_sincos_pair<V3>(odd, tho, m.h2 * x2, m.h2 * x3, so, co, t1, u1, t2, u2, k);
    accel_sc(m, t1, u1, t2, u2, y2, y3, tau2, a2, b2);            // k2 = (y2, y3, a2, b2)
    const double z2 = x2 + m.h2 * a2, z3 = x3 + m.h2 * b2;
    substep_sincos_pair<V3>(odd, tho, m.h2 * y2, m.h2 * y3, so, co, t1, u1, t2, u2, k);
    accel_sc(m, t1, u1, t2, u2, z2, z3, tau2, a3, b3);            // k3 = (z2, z3, a3, b3)
    const double v2 = x2 + m.h * a3, v3 = x3 + m.h * b3;
    substep_sincos_pair<V3>(odd, tho, m.h * z2, m.h * z3, so, co, t1, u1, t2, u2, k);
    accel_sc(m, t1, u1, t2, u2, v2, v3, tau2, a4, b4);            // k4 = (v2, v3, a4, b4)
    const double n0 = x0 + (m.h * (((x2 + 2.0 * y2) + 2.0 * z2) + v2)) * m.h6;
    const double n1 = x1 + (m.h * (((x3 + 2.0 * y3) + 2.0 * z3) + v3)) * m.h6;
    const double n2 = x2 + (m.h * (((a1 + 2.0 * a2) + 2.0 * a3) + a4)) * m.h6;
    const double n3 = x3 + (m.h * (((b1 + 2.0 * b2) + 2.0 * b3) + b4)) * m.h6;
    x0 = n0; x1 = n1; x2 = n2; x3 = n3;
}

// rk4_pair with every sub-step on the near path (angle addition), no per-sub-step branch: returns false for a
// lane where a sub-step's increment is outside |d| <= pi/4 (or NaN), whose result must then be discarded and the
// step re-run by rk4_pair.  Where it returns true the values are rk4_pair's bit for bit (the same near-path code).
// A lone wavefront issues about one instruction per 4-5 cycles whatever its kind, and each per-sub-step branch
// costs ~10 of them (compares, exec-mask saves / restores, two conditional jumps); here the three tests fold into
// two compares and a mask AND per sub-step, and the caller takes one wave-uniform branch per step.
template <bool V3 = GYM_HORNER_VOP3>
__device__ __forceinline__ bool rk4_pair_near(const Dyn& m, bool odd, double& x0, double& x1, double& x2, double& x3,
                                              double tau2, const PolyRegs& k = poly_lits()) {
#pragma clang fp contract(on)   // context-independent bits: FMA contraction inside an expression only
    constexpr double kPio4 = 0.78539816339744830962;
    double a1, b1, a2, b2, a3, b3, a4, b4;
    double t1, u1, t2, u2;
    const double tho = odd ? x1 : x0;
    double so, co;
    fast_sincos<V3>(tho, &so, &co, k);
    // each lane tests its own joint's increment only: the partner lane tests the other, and one failing lane
    // sends the whole wavefront (the caller's ballot) through rk4_pair, whose test is per pair
    bool ok = true;
    auto sub = [&](double w, double w1, double w2) {   // d = w * (this lane's joint velocity)
        const double d = w * (odd ? w2 : w1);
        ok &= fabs(d) <= kPio4;
        double to, uo;
        rotate<V3>(so, co, d, to, uo, k);
        t1 = pair_even(to); u1 = pair_even(uo);
        t2 = pair_odd(to);  u2 = pair_odd(uo);
    };
    const double s1 = pair_even(so), c1 = pair_even(co), s2 = pair_odd(so), c2 = pair_odd(co);
    accel_sc(m, s1, c1, s2, c2, x2, x3, tau2, a1, b1);            // k1 = (x2, x3, a1, b1)
    const double y2 = x2 + m.h2 * a1, y3 = x3 + m.h2 * b1;
    sub(m.h2, x2, x3);
    accel_sc(m, t1, u1, t2, u2, y2, y3, tau2, a2, b2);            // k2 = (y2, y3, a2, b2)
    const double z2 = x2 + m.h2 * a2, z3 = x3 + m.h2 * b2;
    sub(m.h2, y2, y3);
    accel_sc(m, t1, u1, t2, u2, z2, z3, tau2, a3, b3);            // k3 = (z2, z3, a3, b3)
    const double v2 = x2 + m.h * a3, v3 = x3 + m.h * b3;
    sub(m.h, z2, z3);
    accel_sc(m, t1, u1, t2, u2, v2, v3, tau2, a4, b4);            // k4 = (v2, v3, a4, b4)
    const double n0 = x0 + (m.h * (((x2 + 2.0 * y2) + 2.0 * z2) + v2)) * m.h6;
    const double n1 = x1 + (m.h * (((x3 + 2.0 * y3) + 2.0 * z3) + v3)) * m.h6;
    const double n2 = x2 + (m.h * (((a1 + 2.0 * a2) + 2.0 * a3) + a4)) * m.h6;
    const double n3 = x3 + (m.h * (((b1 + 2.0 * b2) + 2.0 * b3) + b4)) * m.h6;
    x0 = n0; x1 = n1; x2 = n2; x3 = n3;
    return ok;
}

// rk4_pair through rk4_pair_near: the branch-free step, re-run with rk4_pair (per-lane sub-step branches) only when
// a lane of the wavefront needs a far-path sub-step.  Bit-identical to rk4_pair.  Every lane of the wavefront must
// run it (wave-uniform branch; the pairs' DPP partners are always active).
template <bool V3 = GYM_HORNER_VOP3>
__device__ __forceinline__ void rk4_pair_fast(const Dyn& m, bool odd, double& x0, double& x1, double& x2, double& x3,
                                              double tau2, const PolyRegs& k = poly_lits()) {
    const double s0 = x0, s1 = x1, s2 = x2, s3 = x3;
    const bool ok = rk4_pair_near<V3>(m, odd, x0, x1, x2, x3, tau2, k);
    if (__builtin_expect(__builtin_amdgcn_ballot_w64(!ok) != 0, 0)) {
        x0 = s0; x1 = s1; x2 = s2; x3 = s3;
        rk4_pair<V3>(m, odd, x0, x1, x2, x3, tau2, k);
    }
}

// Continuous Jacobians (dynamics.py:157-170, 217-226): rows 0,1 of A_c are e3^T, e4^T; B_c[:,0] == 0.
// Returns rows 2,3 of A_c (a2, a3) and B_c[2:,1] (bc2, bc3).
struct Jac {
    double a2[4], a3[4], bc2, bc3;
};

__device__ __forceinline__ Jac jacobian(const Dyn& m, double th1, double th2, double w1, double w2, double tau2,
                                        const PolyRegs& k = poly_lits()) {
#pragma clang fp contract(on)   // context-independent bits (see Sweep::step_j)
    double s1, c1, s2, c2;
    fast_sincos(th1, &s1, &c1, k);
    fast_sincos(th2, &s2, &c2, k);
    const double s12 = s1 * c2 + c1 * s2, c12 = c1 * c2 - s1 * s2;
    const double bs2 = m.b * s2, bc2 = m.b * c2;
    const double M11 = m.a2b + 2.0 * bc2, M12 = m.d + bc2;
    const double r1 = bs2 * w2 * (2.0 * w1 + w2) - m.f1 * w1 - (m.g1 * s1 + m.g2 * s12);
    const double r2 = tau2 - bs2 * w1 * w1 - m.f2 * w2 - m.g2 * s12;
    const double inv = recip(m.dad - m.bb * (c2 * c2));
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
