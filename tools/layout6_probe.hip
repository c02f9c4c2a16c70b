// Would an interleaved record layout move the phase kernel's streams better than six separate streams?
// (measurement tool, not the product; profiles/r06/README.md "layout6")
//
// The phase kernel runs, per launch, the backward sweep of one lane half beside the Armijo trial of the other:
//   sweep (stage t = T-1 .. 0): reads x_cb[t] (a 2 KiB pair block per wavefront) and u_cb[t] (512 B of the tau2 plane),
//                               writes K1[t] (2 KiB) and cg[t] (512 B);
//   trial (stage t = 0 .. T-1): reads K1[t], cg[t], writes x_cb'[t+1] and u_cb'[t].
// Its speed depends on where the six streams land (1.89-2.08 ms for the same kernel, the slow placements
// with ~2x the L2's fabric-side stalls).  This probe moves the same bytes with no arithmetic in two layouts:
//   k_sep : six separate allocations in the solver's layout (x pairs (N, W, 2, 64) d2v; u (T, 2, Bp) planes, plane 1;
//           K1 (T, W, 2, 64) d2v; cs (T, 2, Bp) planes, plane 0);
//   k_rec : one allocation of records, one per (knot t, wavefront w): [x_b0 2 KiB | x_b1 2 KiB | u_b0 512 B |
//           u_b1 512 B | K1 2 KiB | cg 512 B] (7.5 KiB), so every stream a wavefront touches at a stage lies in one
//           contiguous 7.5 KiB record and the streams' relative placement is fixed.
// 262,144 lanes, 64-thread workgroups, four per SIMD (the phase kernel's occupancy): the first half of the
// workgroups run the sweep pattern on lanes [0, B/2), the rest the trial pattern on [B/2, B); non-temporal.
// Build: hipcc --offload-arch=gfx950 -O3 -fPIC -shared tools/layout6_probe.hip -o tools/liblayout6_probe.so
#include <hip/hip_runtime.h>

#include <cstdint>

namespace {

typedef double d2v __attribute__((ext_vector_type(2)));

__device__ __forceinline__ d2v ld2(const d2v* p) { return __builtin_nontemporal_load(p); }
__device__ __forceinline__ void st2(d2v* p, d2v v) { __builtin_nontemporal_store(v, p); }
__device__ __forceinline__ double ld1(const double* p) { return __builtin_nontemporal_load(p); }
__device__ __forceinline__ void st1(double* p, double v) { __builtin_nontemporal_store(v, p); }

struct Sep {
    d2v* x[2];
    double* u[2];
    d2v* K;
    double* cs;
};

// separate streams; W = B / 64 wavefronts; cb = the current buffer
__global__ __launch_bounds__(64, 4) void k_sep(Sep s, int64_t B, int T, int cb) {
    const int64_t W = B / 64, half = W / 2;
    const int64_t wb = blockIdx.x, j = threadIdx.x;
    const bool sweep = wb < half;
    const int64_t w = sweep ? wb : wb;                   // lanes [0, B/2) sweep, [B/2, B) trial
    const int64_t px = w * 128 + j;                      // pair block of wavefront w inside a knot row
    const int64_t pl = w * 64 + j;                       // lane inside a plane row
    if (sweep) {
        const d2v* x = s.x[cb];
        const double* u = s.u[cb];
        d2v a = ld2(x + (int64_t)(T - 1) * 2 * B + px), b = ld2(x + (int64_t)(T - 1) * 2 * B + px + 64);
        double c = ld1(u + (int64_t)(T - 1) * 2 * B + B + pl);
        for (int t = T - 1; t >= 0; --t) {
            d2v na = a, nb = b;
            double nc = c;
            if (t > 0) {
                na = ld2(x + (int64_t)(t - 1) * 2 * B + px); nb = ld2(x + (int64_t)(t - 1) * 2 * B + px + 64);
                nc = ld1(u + (int64_t)(t - 1) * 2 * B + B + pl);
            }
            a.x += c;
            st2(s.K + (int64_t)t * 2 * B + px, a); st2(s.K + (int64_t)t * 2 * B + px + 64, b);
            st1(s.cs + (int64_t)t * 2 * B + pl, c);
            a = na; b = nb; c = nc;
        }
    } else {
        d2v* x = s.x[cb ^ 1];
        double* u = s.u[cb ^ 1];
        d2v a = ld2(s.K + px), b = ld2(s.K + px + 64);
        double c = ld1(s.cs + pl);
        for (int t = 0; t < T; ++t) {
            d2v na = a, nb = b;
            double nc = c;
            if (t + 1 < T) {
                na = ld2(s.K + (int64_t)(t + 1) * 2 * B + px); nb = ld2(s.K + (int64_t)(t + 1) * 2 * B + px + 64);
                nc = ld1(s.cs + (int64_t)(t + 1) * 2 * B + pl);
            }
            a.x += c;
            st2(x + (int64_t)(t + 1) * 2 * B + px, a); st2(x + (int64_t)(t + 1) * 2 * B + px + 64, b);
            st1(u + (int64_t)t * 2 * B + B + pl, c);
            a = na; b = nb; c = nc;
        }
    }
}

// record layout: record (t, w) of REC doubles at ((t * W) + w) * REC
constexpr int REC = 256 + 256 + 64 + 64 + 256 + 64;   // doubles: x_b0, x_b1 (2 KiB each), u_b0, u_b1, K1, cg
constexpr int OX0 = 0, OX1 = 256, OU0 = 512, OU1 = 576, OK = 640, OC = 896;

__global__ __launch_bounds__(64, 4) void k_rec(double* __restrict__ r, int64_t B, int T, int cb) {
    const int64_t W = B / 64, half = W / 2;
    const int64_t w = blockIdx.x, j = threadIdx.x;
    const bool sweep = w < half;
    const int ox = cb ? OX1 : OX0, ou = cb ? OU1 : OU0, oxn = cb ? OX0 : OX1, oun = cb ? OU0 : OU1;
    auto rec = [&](int t) { return r + ((int64_t)t * W + w) * REC; };
    if (sweep) {
        const double* p = rec(T - 1);
        d2v a = ld2((const d2v*)(p + ox) + j), b = ld2((const d2v*)(p + ox) + 64 + j);
        double c = ld1(p + ou + j);
        for (int t = T - 1; t >= 0; --t) {
            d2v na = a, nb = b;
            double nc = c;
            if (t > 0) {
                const double* q = rec(t - 1);
                na = ld2((const d2v*)(q + ox) + j); nb = ld2((const d2v*)(q + ox) + 64 + j); nc = ld1(q + ou + j);
            }
            double* o = rec(t);
            a.x += c;
            st2((d2v*)(o + OK) + j, a); st2((d2v*)(o + OK) + 64 + j, b); st1(o + OC + j, c);
            a = na; b = nb; c = nc;
        }
    } else {
        const double* p = rec(0);
        d2v a = ld2((const d2v*)(p + OK) + j), b = ld2((const d2v*)(p + OK) + 64 + j);
        double c = ld1(p + OC + j);
        for (int t = 0; t < T; ++t) {
            d2v na = a, nb = b;
            double nc = c;
            if (t + 1 < T) {
                const double* q = rec(t + 1);
                na = ld2((const d2v*)(q + OK) + j); nb = ld2((const d2v*)(q + OK) + 64 + j); nc = ld1(q + OC + j);
            }
            a.x += c;
            double* o1 = rec(t + 1);
            st2((d2v*)(o1 + oxn) + j, a); st2((d2v*)(o1 + oxn) + 64 + j, b);
            st1(rec(t) + oun + j, c);
            a = na; b = nb; c = nc;
        }
    }
}

}  // namespace

extern "C" {
int l6_rec_doubles(void) { return REC; }
// variant 0: separate streams (ptrs = x0, x1, u0, u1, K1, cs); 1: records (ptrs[0] = the record array, N * W records)
int l6_run(int variant, void* const* ptrs, int64_t B, int T, int cb, void* stream) {
    if (B % 128 != 0 || T < 2) return 1;
    const dim3 grid((unsigned)(B / 64)), block(64);
    if (variant == 0) {
        Sep s;
        s.x[0] = (d2v*)ptrs[0]; s.x[1] = (d2v*)ptrs[1]; s.u[0] = (double*)ptrs[2]; s.u[1] = (double*)ptrs[3];
        s.K = (d2v*)ptrs[4]; s.cs = (double*)ptrs[5];
        hipLaunchKernelGGL(k_sep, grid, block, 0, (hipStream_t)stream, s, B, T, cb);
    } else {
        hipLaunchKernelGGL(k_rec, grid, block, 0, (hipStream_t)stream, (double*)ptrs[0], B, T, cb);
    }
    return (int)hipGetLastError();
}
}
