// Bandwidth probe for the solver's HBM access pattern (measurement tool, not part of the product).
//
// Times, with hipEvents on one stream, kernels that move exactly the bytes of the solver's
// trial rollout / backward sweep but do (almost) no arithmetic, for the SoA "pairs" layout used
// today and for an AoSoA layout where each 64-lane wavefront owns a contiguous stream:
//   copy       : double2 copy (1:1 read/write), the practical HBM ceiling for a mixed stream
//   trial_soa  : per stage read x(2) u K(2) s, write xn(2) un   -- SoA (t, pair, lane)
//   trial_aos  : same streams, AoSoA (wave, t, pair, lane%64)
//   bwd_soa    : per stage (reverse t) read x(2) u, write K(2) s
//   bwd_aos    : AoSoA
// Build: hipcc --offload-arch=gfx950 -O3 tools/stream_probe.hip -o tools/stream_probe
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                                  \
    do {                                                                                       \
        hipError_t e_ = (x);                                                                   \
        if (e_ != hipSuccess) {                                                                \
            fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_));          \
            exit(1);                                                                           \
        }                                                                                      \
    } while (0)

template <bool AOS>
__device__ __forceinline__ long long ix(int t, int p, int P, long long l, long long B, int T) {
    if (AOS) {
        const long long w = l >> 6, q = l & 63;
        return ((w * T + t) * P + p) * 64 + q;
    }
    return ((long long)t * P + p) * B + l;
}

__global__ void k_copy(const double2* __restrict__ a, double2* __restrict__ b, long long n) {
    for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (long long)gridDim.x * blockDim.x)
        b[i] = a[i];
}

template <bool AOS>
__global__ __launch_bounds__(64) void k_trial(const double2* __restrict__ x, const double2* __restrict__ u,
                                              const double2* __restrict__ K, const double2* __restrict__ s,
                                              double2* __restrict__ xn, double2* __restrict__ un, long long B, int N,
                                              double* sink) {
    const long long l = (long long)blockIdx.x * 64 + threadIdx.x;
    const int T = N - 1;
    double acc = 0.0, a0 = 0.1, a1 = 0.2, a2 = 0.3, a3 = 0.4;
    for (int t = 0; t < T; ++t) {
        const double2 xa = x[ix<AOS>(t, 0, 2, l, B, N)], xb = x[ix<AOS>(t, 1, 2, l, B, N)];
        const double2 uu = u[ix<AOS>(t, 0, 1, l, B, T)];
        const double2 k0 = K[ix<AOS>(t, 0, 2, l, B, T)], k1 = K[ix<AOS>(t, 1, 2, l, B, T)];
        const double2 ss = s[ix<AOS>(t, 0, 1, l, B, T)];
        const double d = (a0 - xa.x) * k0.x + (a1 - xa.y) * k0.y + (a2 - xb.x) * k1.x + (a3 - xb.y) * k1.y;
        const double v = uu.y + d + ss.y;
        acc += v;
        a0 += 1e-3 * v; a1 -= 1e-3 * v; a2 += 1e-4 * uu.x; a3 += 1e-4 * ss.x;
        un[ix<AOS>(t, 0, 1, l, B, T)] = make_double2(uu.x, v);
        xn[ix<AOS>(t + 1, 0, 2, l, B, N)] = make_double2(a0, a1);
        xn[ix<AOS>(t + 1, 1, 2, l, B, N)] = make_double2(a2, a3);
    }
    if (acc == 12345.678) sink[0] = acc;
}

template <bool AOS>
__global__ __launch_bounds__(64) void k_bwd(const double2* __restrict__ x, const double2* __restrict__ u,
                                            double2* __restrict__ K, double2* __restrict__ s, long long B, int N) {
    const long long l = (long long)blockIdx.x * 64 + threadIdx.x;
    const int T = N - 1;
    double p0 = 1.0, p1 = 2.0;
    for (int t = T - 1; t >= 0; --t) {
        const double2 xa = x[ix<AOS>(t, 0, 2, l, B, N)], xb = x[ix<AOS>(t, 1, 2, l, B, N)];
        const double2 uu = u[ix<AOS>(t, 0, 1, l, B, T)];
        p0 = 0.5 * p0 + xa.x * xb.y + uu.x;
        p1 = 0.5 * p1 + xa.y * xb.x + uu.y;
        K[ix<AOS>(t, 0, 2, l, B, T)] = make_double2(p0, p1);
        K[ix<AOS>(t, 1, 2, l, B, T)] = make_double2(p1, p0);
        s[ix<AOS>(t, 0, 1, l, B, T)] = make_double2(p0 * p1, p0 - p1);
    }
}

// ---- v2 streams (feedback offset c = u1 - K x precomputed by the backward sweep) ----
template <bool AOS, bool NT>
__device__ __forceinline__ double2 ld2(const double2* p) {
    if (NT) return make_double2(__builtin_nontemporal_load(&p->x), __builtin_nontemporal_load(&p->y));
    return *p;
}
template <bool NT>
__device__ __forceinline__ void st2(double2* p, double2 v) {
    if (NT) { __builtin_nontemporal_store(v.x, &p->x); __builtin_nontemporal_store(v.y, &p->y); }
    else *p = v;
}
// trial v2: read K(2) cs(1) u0 ; write xn(2) u (pair or split)
template <bool AOS, bool SPLIT, bool NT>
__global__ __launch_bounds__(64) void k_trial2(const double2* __restrict__ K, const double2* __restrict__ cs,
                                               const double* __restrict__ u0p, const double2* __restrict__ up,
                                               double2* __restrict__ xn, double* __restrict__ un0,
                                               double* __restrict__ un1, double2* __restrict__ unp, long long B,
                                               int N, double* sink) {
    const long long l = (long long)blockIdx.x * 64 + threadIdx.x;
    const int T = N - 1;
    double acc = 0.0, a0 = 0.1, a1 = 0.2, a2 = 0.3, a3 = 0.4;
    for (int t = 0; t < T; ++t) {
        const double2 k0 = ld2<AOS, NT>(&K[ix<AOS>(t, 0, 2, l, B, T)]), k1 = ld2<AOS, NT>(&K[ix<AOS>(t, 1, 2, l, B, T)]);
        const double2 c = ld2<AOS, NT>(&cs[ix<AOS>(t, 0, 1, l, B, T)]);
        double u0;
        if (SPLIT) u0 = NT ? __builtin_nontemporal_load(&u0p[ix<AOS>(t, 0, 1, l, B, T)]) : u0p[ix<AOS>(t, 0, 1, l, B, T)];
        else u0 = ld2<AOS, NT>(&up[ix<AOS>(t, 0, 1, l, B, T)]).x;
        const double v = c.x + a0 * k0.x + a1 * k0.y + a2 * k1.x + a3 * k1.y + c.y;
        acc += v;
        a0 += 1e-3 * v; a1 -= 1e-3 * v; a2 += 1e-4 * u0; a3 += 1e-4 * c.y;
        if (SPLIT) {
            if (NT) { __builtin_nontemporal_store(u0 + 1.0, &un0[ix<AOS>(t, 0, 1, l, B, T)]); __builtin_nontemporal_store(v, &un1[ix<AOS>(t, 0, 1, l, B, T)]); }
            else { un0[ix<AOS>(t, 0, 1, l, B, T)] = u0 + 1.0; un1[ix<AOS>(t, 0, 1, l, B, T)] = v; }
        } else {
            st2<NT>(&unp[ix<AOS>(t, 0, 1, l, B, T)], make_double2(u0 + 1.0, v));
        }
        st2<NT>(&xn[ix<AOS>(t + 1, 0, 2, l, B, N)], make_double2(a0, a1));
        st2<NT>(&xn[ix<AOS>(t + 1, 1, 2, l, B, N)], make_double2(a2, a3));
    }
    if (acc == 12345.678) sink[0] = acc;
}
// direction probes: the same backward streams walked with ascending t, and the trial writing x at reversed t
__global__ __launch_bounds__(64) void k_bwd2_asc(const double2* __restrict__ x, const double2* __restrict__ up,
                                                 double2* __restrict__ K, double2* __restrict__ cs, long long B, int N) {
    const long long l = (long long)blockIdx.x * 64 + threadIdx.x;
    const int T = N - 1;
    double p0 = 1.0, p1 = 2.0;
    for (int t = 0; t < T; ++t) {
        const double2 xa = x[(2LL * t) * B + l], xb = x[(2LL * t + 1) * B + l];
        const double2 uu = up[(long long)t * B + l];
        p0 = 0.5 * p0 + xa.x * xb.y + uu.x;
        p1 = 0.5 * p1 + xa.y * xb.x + uu.y;
        K[(2LL * t) * B + l] = make_double2(p0, p1);
        K[(2LL * t + 1) * B + l] = make_double2(p1, p0);
        cs[(long long)t * B + l] = make_double2(p0 * p1, p0 - p1);
    }
}
__global__ __launch_bounds__(64) void k_trial2_rev(const double2* __restrict__ K, const double2* __restrict__ cs,
                                                   const double* __restrict__ u0p, double2* __restrict__ xn,
                                                   double* __restrict__ un0, double* __restrict__ un1, long long B,
                                                   int N, double* sink) {
    const long long l = (long long)blockIdx.x * 64 + threadIdx.x;
    const int T = N - 1;
    double acc = 0.0, a0 = 0.1, a1 = 0.2, a2 = 0.3, a3 = 0.4;
    for (int t = 0; t < T; ++t) {
        const double2 k0 = ld2<false, true>(&K[(2LL * t) * B + l]), k1 = ld2<false, true>(&K[(2LL * t + 1) * B + l]);
        const double2 c = ld2<false, true>(&cs[(long long)t * B + l]);
        const double u0 = __builtin_nontemporal_load(&u0p[(long long)t * B + l]);
        const double v = c.x + a0 * k0.x + a1 * k0.y + a2 * k1.x + a3 * k1.y + c.y;
        acc += v;
        a0 += 1e-3 * v; a1 -= 1e-3 * v; a2 += 1e-4 * u0; a3 += 1e-4 * c.y;
        const long long tr = T - 1 - t;
        __builtin_nontemporal_store(u0 + 1.0, &un0[tr * B + l]);
        __builtin_nontemporal_store(v, &un1[tr * B + l]);
        st2<true>(&xn[(2LL * (T - t - 1)) * B + l], make_double2(a0, a1));
        st2<true>(&xn[(2LL * (T - t - 1) + 1) * B + l], make_double2(a2, a3));
    }
    if (acc == 12345.678) sink[0] = acc;
}
// backward v2: read x(2) u (pair or split) ; write K(2) cs
template <bool AOS, bool SPLIT, bool NT>
__global__ __launch_bounds__(64) void k_bwd2(const double2* __restrict__ x, const double* __restrict__ u0p,
                                             const double* __restrict__ u1p, const double2* __restrict__ up,
                                             double2* __restrict__ K, double2* __restrict__ cs, long long B, int N) {
    const long long l = (long long)blockIdx.x * 64 + threadIdx.x;
    const int T = N - 1;
    double p0 = 1.0, p1 = 2.0;
    for (int t = T - 1; t >= 0; --t) {
        const double2 xa = ld2<AOS, NT>(&x[ix<AOS>(t, 0, 2, l, B, N)]), xb = ld2<AOS, NT>(&x[ix<AOS>(t, 1, 2, l, B, N)]);
        double u0, u1;
        if (SPLIT) { u0 = u0p[ix<AOS>(t, 0, 1, l, B, T)]; u1 = u1p[ix<AOS>(t, 0, 1, l, B, T)]; }
        else { const double2 uu = ld2<AOS, NT>(&up[ix<AOS>(t, 0, 1, l, B, T)]); u0 = uu.x; u1 = uu.y; }
        p0 = 0.5 * p0 + xa.x * xb.y + u0;
        p1 = 0.5 * p1 + xa.y * xb.x + u1;
        st2<NT>(&K[ix<AOS>(t, 0, 2, l, B, T)], make_double2(p0, p1));
        st2<NT>(&K[ix<AOS>(t, 1, 2, l, B, T)], make_double2(p1, p0));
        st2<NT>(&cs[ix<AOS>(t, 0, 1, l, B, T)], make_double2(p0 * p1, p0 - p1));
    }
}

int main(int argc, char** argv) {
    const long long Bl = argc > 1 ? atoll(argv[1]) : 262144;          // lanes
    const long long B = argc > 2 ? atoll(argv[2]) : Bl;               // SoA lane stride (padding)
    const int N = 501, T = N - 1, reps = 5;
    const size_t xs = (size_t)N * 2 * B, us = (size_t)T * B, ks = (size_t)T * 2 * B;
    double2 *x, *u, *K, *s, *xn, *un;
    double* sink;
    CK(hipMalloc(&x, xs * 16)); CK(hipMalloc(&xn, xs * 16));
    CK(hipMalloc(&u, us * 16)); CK(hipMalloc(&un, us * 16));
    CK(hipMalloc(&K, ks * 16)); CK(hipMalloc(&s, us * 16));
    CK(hipMalloc(&sink, 64));
    CK(hipMemset(x, 0, xs * 16)); CK(hipMemset(u, 0, us * 16)); CK(hipMemset(K, 0, ks * 16));
    CK(hipMemset(s, 0, us * 16)); CK(hipMemset(xn, 0, xs * 16)); CK(hipMemset(un, 0, us * 16));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
    auto timeit = [&](const char* name, double bytes, auto&& launch) {
        launch();
        CK(hipDeviceSynchronize());
        float best = 1e30f;
        for (int r = 0; r < reps; ++r) {
            CK(hipEventRecord(e0, 0));
            launch();
            CK(hipEventRecord(e1, 0));
            CK(hipEventSynchronize(e1));
            float ms;
            CK(hipEventElapsedTime(&ms, e0, e1));
            if (ms < best) best = ms;
        }
        printf("{\"probe\": \"%s\", \"ms\": %.4f, \"GBs\": %.1f, \"bytes\": %.0f}\n", name, best, bytes / best / 1e6, bytes);
        fflush(stdout);
    };
    const int grid = (int)(Bl / 64);
    printf("{\"lanes\": %lld, \"stride\": %lld}\n", Bl, B);
    const double trial_bytes = 16.0 * Bl * (2.0 * N + T + 2.0 * T + T) + 16.0 * Bl * (2.0 * T + T);
    const double bwd_bytes = 16.0 * Bl * (2.0 * T + T) + 16.0 * Bl * (2.0 * T + T);
    timeit("copy_x", 2.0 * 16.0 * xs, [&] { hipLaunchKernelGGL(k_copy, dim3(4096), dim3(256), 0, 0, x, xn, (long long)xs); });
    timeit("trial_soa", trial_bytes, [&] { hipLaunchKernelGGL(k_trial<false>, dim3(grid), dim3(64), 0, 0, x, u, K, s, xn, un, B, N, sink); });
    timeit("trial_aos", trial_bytes, [&] { hipLaunchKernelGGL(k_trial<true>, dim3(grid), dim3(64), 0, 0, x, u, K, s, xn, un, B, N, sink); });
    timeit("bwd_soa", bwd_bytes, [&] { hipLaunchKernelGGL(k_bwd<false>, dim3(grid), dim3(64), 0, 0, x, u, K, s, B, N); });
    timeit("bwd_aos", bwd_bytes, [&] { hipLaunchKernelGGL(k_bwd<true>, dim3(grid), dim3(64), 0, 0, x, u, K, s, B, N); });
    // v2 streams: K (2 pairs), cs (1 pair), u (pair or 2 planes)
    double2* cs; double *u0p, *u1p, *un0, *un1;
    CK(hipMalloc(&cs, us * 16)); CK(hipMemset(cs, 0, us * 16));
    CK(hipMalloc(&u0p, us * 8)); CK(hipMalloc(&u1p, us * 8)); CK(hipMalloc(&un0, us * 8)); CK(hipMalloc(&un1, us * 8));
    CK(hipMemset(u0p, 0, us * 8)); CK(hipMemset(u1p, 0, us * 8));
    const double t2_split = 16.0 * Bl * (2.0 * T + T) + 8.0 * Bl * T + 16.0 * Bl * 2.0 * T + 16.0 * Bl * T;
    const double t2_pair = 16.0 * Bl * (2.0 * T + T) + 16.0 * Bl * T + 16.0 * Bl * 2.0 * T + 16.0 * Bl * T;
    const double b2 = 16.0 * Bl * 2.0 * T + 16.0 * Bl * T + 16.0 * Bl * 3.0 * T;
#define T2(AOS, SPLIT, NT, name) timeit(name, SPLIT ? t2_split : t2_pair, [&] { hipLaunchKernelGGL((k_trial2<AOS, SPLIT, NT>), dim3(grid), dim3(64), 0, 0, K, cs, u0p, u, xn, un0, un1, un, B, N, sink); })
#define B2(AOS, SPLIT, NT, name) timeit(name, b2, [&] { hipLaunchKernelGGL((k_bwd2<AOS, SPLIT, NT>), dim3(grid), dim3(64), 0, 0, x, u0p, u1p, u, K, cs, B, N); })
    T2(false, true, false, "trial2_soa_split"); T2(false, false, false, "trial2_soa_pair");
    T2(true, true, false, "trial2_aos_split"); T2(true, false, false, "trial2_aos_pair");
    T2(false, true, true, "trial2_soa_split_nt"); T2(true, false, true, "trial2_aos_pair_nt");
    B2(false, true, false, "bwd2_soa_split"); B2(false, false, false, "bwd2_soa_pair");
    B2(true, true, false, "bwd2_aos_split"); B2(true, false, false, "bwd2_aos_pair");
    B2(false, false, true, "bwd2_soa_pair_nt");
    timeit("bwd2_asc", b2, [&] { hipLaunchKernelGGL(k_bwd2_asc, dim3(grid), dim3(64), 0, 0, x, u, K, cs, B, N); });
    timeit("trial2_revwrite_nt", t2_split, [&] { hipLaunchKernelGGL(k_trial2_rev, dim3(grid), dim3(64), 0, 0, K, cs, u0p, xn, un0, un1, B, N, sink); });
    T2(false, true, true, "trial2_soa_split_nt_again"); B2(true, false, true, "bwd2_aos_pair_nt");
    CK(hipFree(x)); CK(hipFree(xn)); CK(hipFree(u)); CK(hipFree(un)); CK(hipFree(K)); CK(hipFree(s));
    return 0;
}
