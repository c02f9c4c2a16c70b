// Does a longer contiguous burst per wavefront cost less energy per byte? (measurement tool, not the product)
//
// The phase kernel moves, per lane and stage, 40 B in and 40 B out over wave-blocked streams: one wavefront reads a
// contiguous 2 KiB pair block and a 512 B plane row per stage, the next stage's block Bp*32 B away.  At the package
// power cap its throughput is set by energy per lane-iteration, half of it the bytes.  DRAM row
// activations are a large part of the energy per byte, so this probe moves the same bytes in two layouts:
//   k_sb1 : the solver's: per stage a 2 KiB pair block + a 512 B plane row per wavefront, stage by stage;
//   k_sb2 : two stages per block: per stage pair a 4 KiB pair block + a 1 KiB plane block per wavefront, both
//           stages' loads issued together (what a two-stage layout with a two-stage prefetch would do).
// 262,144 lanes in 64-thread workgroups (four waves per SIMD, as the phase kernel), T stages, non-temporal.
// Build: hipcc --offload-arch=gfx950 -O3 -fPIC -shared tools/burst_probe.hip -o tools/libburst_probe.so
#include <hip/hip_runtime.h>

#include <cstdint>

namespace {

typedef double d2v __attribute__((ext_vector_type(2)));

__device__ __forceinline__ d2v ld2(const d2v* p) { return __builtin_nontemporal_load(p); }
__device__ __forceinline__ void st2(d2v* p, d2v v) { __builtin_nontemporal_store(v, p); }
__device__ __forceinline__ double ld1(const double* p) { return __builtin_nontemporal_load(p); }
__device__ __forceinline__ void st1(double* p, double v) { __builtin_nontemporal_store(v, p); }

// pairs: (T, B/64, 2, 64) d2v; planes: (T, B) double
__global__ __launch_bounds__(64, 4) void k_sb1(const d2v* __restrict__ in2, const double* __restrict__ in1,
                                               d2v* __restrict__ out2, double* __restrict__ out1, int64_t B, int T) {
    const int64_t w = blockIdx.x, j = threadIdx.x;
    const int64_t o2 = w * 128 + j, o1 = w * 64 + j;
    d2v a = ld2(in2 + o2), b = ld2(in2 + o2 + 64);
    double c = ld1(in1 + o1);
    for (int t = 0; t < T; ++t) {
        d2v na = a, nb = b;
        double nc = c;
        if (t + 1 < T) {   // one-stage register prefetch, as the solver
            const int64_t r2 = (int64_t)(t + 1) * 2 * B, r1 = (int64_t)(t + 1) * B;
            na = ld2(in2 + r2 + o2); nb = ld2(in2 + r2 + o2 + 64); nc = ld1(in1 + r1 + o1);
        }
        const int64_t r2 = (int64_t)t * 2 * B, r1 = (int64_t)t * B;
        a.x += c;
        st2(out2 + r2 + o2, a); st2(out2 + r2 + o2 + 64, b); st1(out1 + r1 + o1, c);
        a = na; b = nb; c = nc;
    }
}

// pairs: (T/2, B/64, 2 stages, 2, 64) d2v; planes: (T/2, B/64, 2 stages, 64) double
__global__ __launch_bounds__(64, 4) void k_sb2(const d2v* __restrict__ in2, const double* __restrict__ in1,
                                               d2v* __restrict__ out2, double* __restrict__ out1, int64_t B, int T) {
    const int64_t w = blockIdx.x, j = threadIdx.x;
    const int64_t o2 = w * 256 + j, o1 = w * 128 + j;
    d2v a0 = ld2(in2 + o2), b0 = ld2(in2 + o2 + 64), a1 = ld2(in2 + o2 + 128), b1 = ld2(in2 + o2 + 192);
    double c0 = ld1(in1 + o1), c1 = ld1(in1 + o1 + 64);
    for (int t = 0; t < T; t += 2) {
        d2v na0 = a0, nb0 = b0, na1 = a1, nb1 = b1;
        double nc0 = c0, nc1 = c1;
        if (t + 2 < T) {   // the next stage pair's block, all at once
            const int64_t r2 = (int64_t)(t + 2) * 2 * B, r1 = (int64_t)(t + 2) * B;
            na0 = ld2(in2 + r2 + o2); nb0 = ld2(in2 + r2 + o2 + 64);
            na1 = ld2(in2 + r2 + o2 + 128); nb1 = ld2(in2 + r2 + o2 + 192);
            nc0 = ld1(in1 + r1 + o1); nc1 = ld1(in1 + r1 + o1 + 64);
        }
        const int64_t r2 = (int64_t)t * 2 * B, r1 = (int64_t)t * B;
        a0.x += c0; a1.x += c1;
        st2(out2 + r2 + o2, a0); st2(out2 + r2 + o2 + 64, b0);
        st2(out2 + r2 + o2 + 128, a1); st2(out2 + r2 + o2 + 192, b1);
        st1(out1 + r1 + o1, c0); st1(out1 + r1 + o1 + 64, c1);
        a0 = na0; b0 = nb0; a1 = na1; b1 = nb1; c0 = nc0; c1 = nc1;
    }
}

}  // namespace

extern "C" {
// B a multiple of 64, T even; in2 / out2 hold T*2*B d2v, in1 / out1 T*B doubles
int bp_run(int variant, const void* in2, const void* in1, void* out2, void* out1, int64_t B, int T, void* stream) {
    if (B % 64 != 0 || T % 2 != 0 || T < 2) return 1;
    const dim3 grid((unsigned)(B / 64)), block(64);
    if (variant == 1)
        hipLaunchKernelGGL(k_sb1, grid, block, 0, (hipStream_t)stream, (const d2v*)in2, (const double*)in1,
                           (d2v*)out2, (double*)out1, B, T);
    else
        hipLaunchKernelGGL(k_sb2, grid, block, 0, (hipStream_t)stream, (const d2v*)in2, (const double*)in1,
                           (d2v*)out2, (double*)out1, B, T);
    return (int)hipGetLastError();
}
}
