// Layout probe for the solver's per-stage streams (measurement tool, not part of the product).
//
// Moves exactly the bytes of the tau1-zero solver streams with (almost) no arithmetic:
//   sweep : per stage (reverse t) read x (2 pair rows) + u1 (plane); write K1 (2 pair rows) + cs (1 pair row)
//   trial : per stage read K1 (2) + cs (1); write x (2) + u1 (plane)
//   phase : half the blocks sweep lanes [0, B/2), half trial lanes [B/2, B) (the pipelined launch)
// in three layouts of the multi-row streams:
//   soa   : today's (t, row, lane) -- a wave's rows of one stage are Bp*16 bytes apart
//   wb    : wave-blocked (t, wave, row, lane%64) -- a wave's rows of one stage are one contiguous block
//   wbm   : wb with K1 and cs merged into one 3-row stream (one 3 KiB block per wave-stage)
//   aos   : AoSoA (wave, t, row, lane%64) -- a wave's stages of a stream are one contiguous region (planes too)
// Build: hipcc --offload-arch=gfx950 -O3 tools/layout_probe.hip -o tools/layout_probe
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#define CK(x)                                                                                  \
    do {                                                                                       \
        hipError_t e_ = (x);                                                                   \
        if (e_ != hipSuccess) {                                                                \
            fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_));          \
            exit(1);                                                                           \
        }                                                                                      \
    } while (0)

typedef double d2v __attribute__((ext_vector_type(2)));
__device__ __forceinline__ double2 ld2(const double2* p) {
    const d2v v = __builtin_nontemporal_load(reinterpret_cast<const d2v*>(p));
    return make_double2(v.x, v.y);
}
__device__ __forceinline__ void st2(double2* p, double a, double b) {
    d2v v = {a, b};
    __builtin_nontemporal_store(v, reinterpret_cast<d2v*>(p));
}

enum { SOA = 0, WB = 1, WBM = 2, AOS = 3 };
constexpr int kTn = 501;   // AOS: stages per wave region (N for every stream; the probe pads the T-stage ones)

// element index (double2 units) of row p of a P-row stream at stage t for lane l
template <int L>
__device__ __forceinline__ long long ix(int t, int p, int P, long long l, long long B) {
    if (L == SOA) return ((long long)t * P + p) * B + l;
    if (L == AOS) return (((l >> 6) * kTn + t) * P + p) * 64 + (l & 63);
    const long long w = l >> 6, q = l & 63, nW = B >> 6;
    return (((long long)t * nW + w) * P + p) * 64 + q;
}

template <int L>   // plane element (double units) of stage t, lane l
__device__ __forceinline__ long long px(int t, long long l, long long B) {
    if (L == AOS) return ((l >> 6) * kTn + t) * 64 + (l & 63);
    return (long long)t * B + l;
}

template <int L>
__device__ __forceinline__ void sweep_lane(const double2* __restrict__ x, const double* __restrict__ u1,
                                           double2* __restrict__ K, double2* __restrict__ cs, long long l, long long B,
                                           int T) {
    double p0 = 1.0, p1 = 2.0;
    for (int t = T - 1; t >= 0; --t) {
        const double2 xa = ld2(&x[ix<L>(t, 0, 2, l, B)]), xb = ld2(&x[ix<L>(t, 1, 2, l, B)]);
        const double uu = __builtin_nontemporal_load(&u1[px<L>(t, l, B)]);
        p0 = 0.5 * p0 + xa.x * xb.y + uu;
        p1 = 0.5 * p1 + xa.y * xb.x;
        if (L == WBM) {
            st2(&K[ix<L>(t, 0, 3, l, B)], p0, p1);
            st2(&K[ix<L>(t, 1, 3, l, B)], p1, p0);
            st2(&K[ix<L>(t, 2, 3, l, B)], p0 * p1, p0 - p1);
        } else {
            st2(&K[ix<L>(t, 0, 2, l, B)], p0, p1);
            st2(&K[ix<L>(t, 1, 2, l, B)], p1, p0);
            st2(&cs[ix<L>(t, 0, 1, l, B)], p0 * p1, p0 - p1);
        }
    }
}

template <int L>
__device__ __forceinline__ void trial_lane(const double2* __restrict__ K, const double2* __restrict__ cs,
                                           double2* __restrict__ xn, double* __restrict__ u1, long long l, long long B,
                                           int T, double* sink) {
    double acc = 0.0, a0 = 0.1, a1 = 0.2, a2 = 0.3, a3 = 0.4;
    for (int t = 0; t < T; ++t) {
        double2 k0, k1, c;
        if (L == WBM) {
            k0 = ld2(&K[ix<L>(t, 0, 3, l, B)]); k1 = ld2(&K[ix<L>(t, 1, 3, l, B)]); c = ld2(&K[ix<L>(t, 2, 3, l, B)]);
        } else {
            k0 = ld2(&K[ix<L>(t, 0, 2, l, B)]); k1 = ld2(&K[ix<L>(t, 1, 2, l, B)]); c = ld2(&cs[ix<L>(t, 0, 1, l, B)]);
        }
        const double v = c.x + a0 * k0.x + a1 * k0.y + a2 * k1.x + a3 * k1.y + c.y;
        acc += v;
        a0 += 1e-3 * v; a1 -= 1e-3 * v; a2 += 1e-4 * c.x; a3 += 1e-4 * c.y;
        __builtin_nontemporal_store(v, &u1[px<L>(t, l, B)]);
        st2(&xn[ix<L>(t + 1, 0, 2, l, B)], a0, a1);
        st2(&xn[ix<L>(t + 1, 1, 2, l, B)], a2, a3);
    }
    if (acc == 12345.678) sink[0] = acc;
}

template <int L>
__global__ __launch_bounds__(64, 4) void k_sweep(const double2* x, const double* u1, double2* K, double2* cs,
                                                 long long B, int T) {
    sweep_lane<L>(x, u1, K, cs, (long long)blockIdx.x * 64 + threadIdx.x, B, T);
}
template <int L>
__global__ __launch_bounds__(64, 4) void k_trial(const double2* K, const double2* cs, double2* xn, double* u1,
                                                 long long B, int T, double* sink) {
    trial_lane<L>(K, cs, xn, u1, (long long)blockIdx.x * 64 + threadIdx.x, B, T, sink);
}
// phase: even blocks sweep half 0 (x0 -> K), odd blocks trial half 1 (K -> x1); disjoint lanes
template <int L>
__global__ __launch_bounds__(64, 4) void k_phase(const double2* x0, const double* u0, double2* K, double2* cs,
                                                 double2* x1, double* u1, long long B, int T, double* sink) {
    const long long wv = blockIdx.x >> 1;
    if (blockIdx.x & 1) trial_lane<L>(K, cs, x1, u1, (B >> 1) + wv * 64 + threadIdx.x, B, T, sink);
    else sweep_lane<L>(x0, u0, K, cs, wv * 64 + threadIdx.x, B, T);
}

int main(int argc, char** argv) {
    const long long B = argc > 1 ? atoll(argv[1]) : 262144;
    const int N = 501, T = N - 1, reps = 5;
    const size_t xs = (size_t)N * 2 * B, ks = (size_t)N * 3 * B, us = (size_t)N * B;
    double2 *x, *xn, *K, *cs;
    double *u, *un, *sink;
    CK(hipMalloc(&x, xs * 16)); CK(hipMalloc(&xn, xs * 16)); CK(hipMalloc(&K, ks * 16)); CK(hipMalloc(&cs, us * 16));
    CK(hipMalloc(&u, us * 8)); CK(hipMalloc(&un, us * 8)); CK(hipMalloc(&sink, 64));
    CK(hipMemset(x, 0, xs * 16)); CK(hipMemset(xn, 0, xs * 16)); CK(hipMemset(K, 0, ks * 16));
    CK(hipMemset(cs, 0, us * 16)); CK(hipMemset(u, 0, us * 8)); CK(hipMemset(un, 0, us * 8));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
    const double stage_bytes = 32.0 + 8.0 + 32.0 + 16.0;   // per lane-stage, sweep and trial alike
    const double bytes = stage_bytes * T * B;
    auto timeit = [&](const char* name, auto&& launch) {
        launch();
        CK(hipDeviceSynchronize());
        float best = 1e30f, sum = 0.f;
        for (int r = 0; r < reps; ++r) {
            CK(hipEventRecord(e0));
            launch();
            CK(hipEventRecord(e1));
            CK(hipEventSynchronize(e1));
            float ms;
            CK(hipEventElapsedTime(&ms, e0, e1));
            best = ms < best ? ms : best;
            sum += ms;
        }
        printf("%-12s best %.3f ms  avg %.3f ms  %.0f GB/s (best)\n", name, best, sum / reps, bytes / (best * 1e-3) / 1e9);
        fflush(stdout);
    };
    const int g = (int)(B / 64);
#define RUN3(L, NAME)                                                                                                  \
    timeit("sweep_" NAME, [&] { hipLaunchKernelGGL(k_sweep<L>, dim3(g), dim3(64), 0, 0, x, u, K, cs, B, T); });       \
    timeit("trial_" NAME, [&] { hipLaunchKernelGGL(k_trial<L>, dim3(g), dim3(64), 0, 0, K, cs, xn, un, B, T, sink); }); \
    timeit("phase_" NAME, [&] { hipLaunchKernelGGL(k_phase<L>, dim3(g), dim3(64), 0, 0, x, u, K, cs, xn, un, B, T, sink); });
    const bool all = argc > 2 && atoi(argv[2]);
    for (int pass = 0; pass < 3; ++pass) {
        if (all) { RUN3(SOA, "soa") }
        RUN3(WB, "wb")
        RUN3(AOS, "aos")
        if (all) { RUN3(WBM, "wbm") }
    }
    CK(hipGetLastError());
    return 0;
}
