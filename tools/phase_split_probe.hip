// Phase-asymmetry probe (measurement tool, not part of the product).
//
// The pipelined schedule alternates two launch patterns over the double-buffered state x / u (lanes split into
// halves H0 = [0, B/2), H1 = [B/2, B)):
//   odd  phase: the sweep of H1 READS x[cb]; the trial of H0 WRITES x[cb^1]      (read and write in different buffers)
//   even phase: the sweep of H0 READS x[cb^1]; the trial of H1 WRITES x[cb^1]    (the same buffer, other half)
// and the r02 launch trace showed odd phases 1.1-1.4% longer than even ones in every solve.  This probe moves the
// solver's tau1-zero stream bytes with no arithmetic (layout_probe.hip's wave-blocked streams) in both patterns,
// with each buffer one allocation ("same") or each half of each buffer its own allocation ("split"), and times
// the two patterns alternately.  If the gap came from the two halves sharing an allocation, "split" closes it.
// Build: hipcc --offload-arch=gfx950 -O3 tools/phase_split_probe.hip -o tools/phase_split_probe
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
// wave-blocked pair stream element (t, row p of P, lane l) with lane stride S (multiple of 64)
__device__ __forceinline__ long long ix(int t, int p, int P, long long l, long long S) {
    return (((long long)t * (S >> 6) + (l >> 6)) * P + p) * 64 + (l & 63);
}
struct View {          // a half's state: x pairs (N, S/64, 2, 64), u1 plane (T, S); lanes l -> l - off
    double2* x;
    double* u;
    long long off, S;
};

__global__ __launch_bounds__(64, 4) void k_phase(View sv, View tv, double2* K, double2* cs, long long sweep_lo,
                                                  long long trial_lo, long long B, int T, double* sink) {
    const long long wv = blockIdx.x >> 1;
    if (blockIdx.x & 1) {   // trial: K, cs (global lanes, stride B) -> x, u of the view
        const long long l = trial_lo + wv * 64 + threadIdx.x, lv = l - tv.off;
        double acc = 0.0, a0 = 0.1, a1 = 0.2, a2 = 0.3, a3 = 0.4;
        for (int t = 0; t < T; ++t) {
            const double2 k0 = ld2(&K[ix(t, 0, 2, l, B)]), k1 = ld2(&K[ix(t, 1, 2, l, B)]);
            const double2 c = ld2(&cs[ix(t, 0, 1, l, B)]);
            const double v = c.x + a0 * k0.x + a1 * k0.y + a2 * k1.x + a3 * k1.y + c.y;
            acc += v;
            a0 += 1e-3 * v; a1 -= 1e-3 * v; a2 += 1e-4 * c.x; a3 += 1e-4 * c.y;
            __builtin_nontemporal_store(v, &tv.u[(long long)t * tv.S + lv]);
            st2(&tv.x[ix(t + 1, 0, 2, lv, tv.S)], a0, a1);
            st2(&tv.x[ix(t + 1, 1, 2, lv, tv.S)], a2, a3);
        }
        if (acc == 12345.678) sink[0] = acc;
    } else {                // sweep: x, u of the view -> K, cs (global lanes)
        const long long l = sweep_lo + wv * 64 + threadIdx.x, lv = l - sv.off;
        double p0 = 1.0, p1 = 2.0;
        for (int t = T - 1; t >= 0; --t) {
            const double2 xa = ld2(&sv.x[ix(t, 0, 2, lv, sv.S)]), xb = ld2(&sv.x[ix(t, 1, 2, lv, sv.S)]);
            const double uu = __builtin_nontemporal_load(&sv.u[(long long)t * sv.S + lv]);
            p0 = 0.5 * p0 + xa.x * xb.y + uu;
            p1 = 0.5 * p1 + xa.y * xb.x;
            st2(&K[ix(t, 0, 2, l, B)], p0, p1);
            st2(&K[ix(t, 1, 2, l, B)], p1, p0);
            st2(&cs[ix(t, 0, 1, l, B)], p0 * p1, p0 - p1);
        }
    }
}

int main(int argc, char** argv) {
    const long long B = argc > 1 ? atoll(argv[1]) : 262144, H = B / 2;
    const int pairs = argc > 2 ? atoi(argv[2]) : 40;
    const int N = 501, T = N - 1;
    auto alloc = [&](long long lanes, double2** x, double** u) {
        CK(hipMalloc(x, (size_t)N * 2 * lanes * 16)); CK(hipMemset(*x, 0, (size_t)N * 2 * lanes * 16));
        CK(hipMalloc(u, (size_t)N * lanes * 8)); CK(hipMemset(*u, 0, (size_t)N * lanes * 8));
    };
    double2 *X[2], *Xh[2][2], *K, *cs;
    double *U[2], *Uh[2][2], *sink;
    for (int b = 0; b < 2; ++b) {
        alloc(B, &X[b], &U[b]);
        for (int h = 0; h < 2; ++h) alloc(H, &Xh[b][h], &Uh[b][h]);
    }
    CK(hipMalloc(&K, (size_t)N * 2 * B * 16)); CK(hipMalloc(&cs, (size_t)N * B * 16)); CK(hipMalloc(&sink, 64));
    CK(hipMemset(K, 0, (size_t)N * 2 * B * 16)); CK(hipMemset(cs, 0, (size_t)N * B * 16));
    hipEvent_t ev[4];
    for (auto& e : ev) CK(hipEventCreate(&e));
    const double bytes = (32.0 + 8.0 + 32.0 + 16.0) * T * B;   // per lane-stage, both kinds
    const int g = (int)(B / 64);
    for (int split = 0; split < 2; ++split) {
        // odd: sweep H1 reads buffer 0, trial H0 writes buffer 1;  even: sweep H0 reads buffer 1, trial H1 writes it
        const View odd_s = split ? View{Xh[0][1], Uh[0][1], H, H} : View{X[0], U[0], 0, B};
        const View odd_t = split ? View{Xh[1][0], Uh[1][0], 0, H} : View{X[1], U[1], 0, B};
        const View even_s = split ? View{Xh[1][0], Uh[1][0], 0, H} : View{X[1], U[1], 0, B};
        const View even_t = split ? View{Xh[1][1], Uh[1][1], H, H} : View{X[1], U[1], 0, B};
        double sum[2] = {0, 0};
        for (int r = -2; r < pairs; ++r) {   // 2 warm-up pairs
            CK(hipEventRecord(ev[0]));
            hipLaunchKernelGGL(k_phase, dim3(g), dim3(64), 0, 0, odd_s, odd_t, K, cs, H, 0, B, T, sink);
            CK(hipEventRecord(ev[1]));
            hipLaunchKernelGGL(k_phase, dim3(g), dim3(64), 0, 0, even_s, even_t, K, cs, 0, H, B, T, sink);
            CK(hipEventRecord(ev[2]));
            CK(hipEventSynchronize(ev[2]));
            float a, b;
            CK(hipEventElapsedTime(&a, ev[0], ev[1]));
            CK(hipEventElapsedTime(&b, ev[1], ev[2]));
            if (r >= 0) { sum[0] += a; sum[1] += b; }
        }
        const double o = sum[0] / pairs, e = sum[1] / pairs;
        printf("%-5s odd %.4f ms (%.0f GB/s)  even %.4f ms (%.0f GB/s)  odd/even %.4f\n", split ? "split" : "same",
               o, bytes / (o * 1e-3) / 1e9, e, bytes / (e * 1e-3) / 1e9, o / e);
        fflush(stdout);
    }
    CK(hipGetLastError());
    return 0;
}
