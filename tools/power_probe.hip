// Energy probes for the power-capped phase kernel (measurement tool, not part of the product).
//
// Two kernels that each load the chip like one side of the solver's phase kernel, with the same launch shape
// (262,144 lanes in 64-thread workgroups: four waves per SIMD):
//   k_stream : the phase kernel's HBM streams with no arithmetic: per stage 40 B read + 40 B written per lane
//              (16-B and 8-B accesses, SoA rows of the lane batch, non-temporal), T = 500 stages per launch;
//   k_valu   : fp64 FMAs only (8 independent chains per lane, no memory traffic but the final store).
// tools/power_probe.py launches each back to back for a few seconds while sampling power / clocks (box_state) and
// reports the achieved rate (bytes/s or fp64 wave-instructions/s) and the energy per unit at the power it drew.
// Build: hipcc --offload-arch=gfx950 -O3 -fPIC -shared tools/power_probe.hip -o tools/libpower_probe.so
#include <hip/hip_runtime.h>

#include <cstdint>

namespace {

__device__ __forceinline__ double2 ld_nt2(const double2* p) {
    typedef double d2v __attribute__((ext_vector_type(2)));
    const d2v v = __builtin_nontemporal_load(reinterpret_cast<const d2v*>(p));
    return make_double2(v.x, v.y);
}
__device__ __forceinline__ void st_nt2(double2* p, double2 v) {
    typedef double d2v __attribute__((ext_vector_type(2)));
    __builtin_nontemporal_store(d2v{v.x, v.y}, reinterpret_cast<d2v*>(p));
}

// in: (T, 2, B) double2 pairs + (T, B) doubles; out likewise.  Per stage and lane: 2 x 16 B + 8 B read, the same
// written (stage t reads row t, writes row t of the other buffer).
__global__ __launch_bounds__(64, 4) void k_stream(const double2* __restrict__ in2, const double* __restrict__ in1,
                                                  double2* __restrict__ out2, double* __restrict__ out1, int64_t B,
                                                  int T) {
    const int64_t l = (int64_t)blockIdx.x * 64 + threadIdx.x;
    if (l >= B) return;
    for (int t = 0; t < T; ++t) {
        const int64_t r2 = (int64_t)t * 2 * B, r1 = (int64_t)t * B;
        const double2 a = ld_nt2(in2 + r2 + l), b = ld_nt2(in2 + r2 + B + l);
        const double c = __builtin_nontemporal_load(in1 + r1 + l);
        st_nt2(out2 + r2 + l, make_double2(a.x + c, a.y));
        st_nt2(out2 + r2 + B + l, b);
        __builtin_nontemporal_store(c, out1 + r1 + l);
    }
}

// n_iter x 8 chains x 4 FMAs per lane: 32 fp64 FMAs per iteration
__global__ __launch_bounds__(64, 4) void k_valu(double* __restrict__ out, int64_t B, int n_iter, double s) {
    const int64_t l = (int64_t)blockIdx.x * 64 + threadIdx.x;
    if (l >= B) return;
    double a[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) a[k] = 1.0 + 1e-3 * (double)(k + (l & 7));
    for (int i = 0; i < n_iter; ++i) {
#pragma unroll
        for (int r = 0; r < 4; ++r)
#pragma unroll
            for (int k = 0; k < 8; ++k) a[k] = fma(a[k], s, -0.5 * s);
    }
    double acc = 0.0;
#pragma unroll
    for (int k = 0; k < 8; ++k) acc += a[k];
    out[l] = acc;
}

}  // namespace

extern "C" {
int pp_stream(const void* in2, const void* in1, void* out2, void* out1, int64_t B, int T, void* stream) {
    hipLaunchKernelGGL(k_stream, dim3((unsigned)((B + 63) / 64)), dim3(64), 0, (hipStream_t)stream,
                       (const double2*)in2, (const double*)in1, (double2*)out2, (double*)out1, B, T);
    return (int)hipGetLastError();
}
int pp_valu(void* out, int64_t B, int n_iter, double s, void* stream) {
    hipLaunchKernelGGL(k_valu, dim3((unsigned)((B + 63) / 64)), dim3(64), 0, (hipStream_t)stream, (double*)out, B,
                       n_iter, s);
    return (int)hipGetLastError();
}
}
