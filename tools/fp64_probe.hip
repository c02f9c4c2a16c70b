// fp64 VALU issue / latency probe for one wavefront alone on its SIMD (the latency-bound regime of BASELINE
// cfg 2 and cfg 5: 64-128 wavefronts on 1024 SIMDs).  Each wave runs CHAINS independent chains of dependent
// v_fma_f64 for ITERS steps and records the elapsed s_memtime cycles; cycles per instruction =
// elapsed / (ITERS * CHAINS).  Also: a DPP quad_perm exchange of a double between lane pairs inside a chain
// (what splitting one trajectory over several lanes costs per exchanged value).
//   hipcc --offload-arch=gfx950 -O3 tools/fp64_probe.hip -o tools/fp64_probe && tools/fp64_probe
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

constexpr int ITERS = 4096;

template <int CHAINS>
__global__ void k_fma_chains(const double* in, double* out, long long* cyc) {
    double x[CHAINS];
    const double a = in[0], b = in[1];
#pragma unroll
    for (int c = 0; c < CHAINS; ++c) x[c] = in[2 + c] + threadIdx.x;
    __syncthreads();
    const long long t0 = __builtin_amdgcn_s_memtime();
    for (int i = 0; i < ITERS; ++i) {
#pragma unroll
        for (int c = 0; c < CHAINS; ++c) x[c] = __builtin_fma(x[c], a, b);
    }
    double s = 0;
#pragma unroll
    for (int c = 0; c < CHAINS; ++c) s += x[c];
    const long long t1 = __builtin_amdgcn_s_memtime();
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
    if (threadIdx.x % 64 == 0) cyc[(blockIdx.x * blockDim.x + threadIdx.x) / 64] = t1 - t0;
}

// the same chains with only the wave's first ACTIVE lanes executing the loop (exec mask): does a partly masked
// fp64 instruction issue faster than a full one (fewer 16-lane passes)?
template <int CHAINS, int ACTIVE>
__global__ void k_fma_masked(const double* in, double* out, long long* cyc) {
    double x[CHAINS];
    const double a = in[0], b = in[1];
#pragma unroll
    for (int c = 0; c < CHAINS; ++c) x[c] = in[2 + c] + threadIdx.x;
    __syncthreads();
    const long long t0 = __builtin_amdgcn_s_memtime();
    if ((threadIdx.x & 63) < ACTIVE) {
        for (int i = 0; i < ITERS; ++i) {
#pragma unroll
            for (int c = 0; c < CHAINS; ++c) x[c] = __builtin_fma(x[c], a, b);
        }
    }
    double s = 0;
#pragma unroll
    for (int c = 0; c < CHAINS; ++c) s += x[c];
    const long long t1 = __builtin_amdgcn_s_memtime();
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
    if (threadIdx.x % 64 == 0) cyc[(blockIdx.x * blockDim.x + threadIdx.x) / 64] = t1 - t0;
}

__device__ __forceinline__ double swap_pair(double v) {   // exchange with the neighbouring lane (quad_perm 1,0,3,2)
    int lo = __double2loint(v), hi = __double2hiint(v);
    lo = __builtin_amdgcn_mov_dpp(lo, 0xB1, 0xF, 0xF, false);
    hi = __builtin_amdgcn_mov_dpp(hi, 0xB1, 0xF, 0xF, false);
    return __hiloint2double(hi, lo);
}

// one dependent fma, then the value crosses to the partner lane and back into the chain
__global__ void k_dpp_chain(const double* in, double* out, long long* cyc) {
    double x = in[2] + threadIdx.x;
    const double a = in[0], b = in[1];
    __syncthreads();
    const long long t0 = __builtin_amdgcn_s_memtime();
    for (int i = 0; i < ITERS; ++i) {
        x = __builtin_fma(x, a, b);
        x = swap_pair(x);
    }
    const long long t1 = __builtin_amdgcn_s_memtime();
    out[blockIdx.x * blockDim.x + threadIdx.x] = x;
    if (threadIdx.x % 64 == 0) cyc[(blockIdx.x * blockDim.x + threadIdx.x) / 64] = t1 - t0;
}

// a chain of dependent fp64 divisions-by-reciprocal (v_rcp_f64 + 2 Newton steps), the recip() of the kernels
__global__ void k_rcp_chain(const double* in, double* out, long long* cyc) {
    double x = in[2] + threadIdx.x + 2.0;
    __syncthreads();
    const long long t0 = __builtin_amdgcn_s_memtime();
    for (int i = 0; i < ITERS; ++i) {
        double r = __builtin_amdgcn_rcp(x);
        double e = __builtin_fma(-x, r, 1.0);
        r = __builtin_fma(r, e, r);
        e = __builtin_fma(-x, r, 1.0);
        x = __builtin_fma(r, e, r) + 2.0;
    }
    const long long t1 = __builtin_amdgcn_s_memtime();
    out[blockIdx.x * blockDim.x + threadIdx.x] = x;
    if (threadIdx.x % 64 == 0) cyc[(blockIdx.x * blockDim.x + threadIdx.x) / 64] = t1 - t0;
}

template <class K>
static void run(const char* name, K kern, int blocks, int threads, double per_iter_instr, double* din, double* dout,
                long long* dcyc) {
    hipLaunchKernelGGL(kern, dim3(blocks), dim3(threads), 0, 0, din, dout, dcyc);
    hipLaunchKernelGGL(kern, dim3(blocks), dim3(threads), 0, 0, din, dout, dcyc);
    hipDeviceSynchronize();
    const int waves = blocks * threads / 64;
    long long h[4096];
    hipMemcpy(h, dcyc, sizeof(long long) * waves, hipMemcpyDeviceToHost);
    double avg = 0;
    for (int i = 0; i < waves; ++i) avg += (double)h[i];
    avg /= waves;
    printf("%-34s blocks %5d x %4d thr: %8.1f cyc/iter  %6.2f cyc/instr\n", name, blocks, threads, avg / ITERS,
           avg / ITERS / per_iter_instr);
}

int main() {
    double hin[16] = {0.999999, 1e-7, 1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11, 12, 13, 14};
    double *din, *dout;
    long long* dcyc;
    hipMalloc(&din, sizeof(hin));
    hipMalloc(&dout, sizeof(double) * 1024 * 1024);
    hipMalloc(&dcyc, sizeof(long long) * 4096);
    hipMemcpy(din, hin, sizeof(hin), hipMemcpyHostToDevice);
    // 1 block of 64: one wave alone on a SIMD; 1024 blocks of 256: 4 waves per CU = one per SIMD on every CU;
    // 1024 blocks of 512: two waves per SIMD
    // 1 block of 128: are the two wavefronts of a workgroup on different SIMDs? (4.4 cyc/instr if so, ~6.5 if not)
    if (getenv("PROBE_MASK")) {
        run("masked: 64 lanes, chains=4", k_fma_masked<4, 64>, 1, 64, 4, din, dout, dcyc);
        run("masked: 32 lanes, chains=4", k_fma_masked<4, 32>, 1, 64, 4, din, dout, dcyc);
        run("masked: 16 lanes, chains=4", k_fma_masked<4, 16>, 1, 64, 4, din, dout, dcyc);
        run("masked: 8 lanes, chains=4", k_fma_masked<4, 8>, 1, 64, 4, din, dout, dcyc);
        run("masked: 64 lanes, chains=1", k_fma_masked<1, 64>, 1, 64, 1, din, dout, dcyc);
        run("masked: 32 lanes, chains=1", k_fma_masked<1, 32>, 1, 64, 1, din, dout, dcyc);
        run("masked: 16 lanes, chains=1", k_fma_masked<1, 16>, 1, 64, 1, din, dout, dcyc);
        run("masked: 32 lanes, chains=4, 1024x256", k_fma_masked<4, 32>, 1024, 256, 4, din, dout, dcyc);
        run("masked: 64 lanes, chains=4, 1024x256", k_fma_masked<4, 64>, 1024, 256, 4, din, dout, dcyc);
        return 0;
    }
    run("fma chains=4, 1 block x 128", k_fma_chains<4>, 1, 128, 4, din, dout, dcyc);
    run("fma chains=4, 256 blocks x 128", k_fma_chains<4>, 256, 128, 4, din, dout, dcyc);
    for (int thr : {64, 256, 512}) {
        const int blocks = thr == 64 ? 1 : 256;
        run("fma chains=1", k_fma_chains<1>, blocks, thr, 1, din, dout, dcyc);
        run("fma chains=2", k_fma_chains<2>, blocks, thr, 2, din, dout, dcyc);
        run("fma chains=4", k_fma_chains<4>, blocks, thr, 4, din, dout, dcyc);
        run("fma chains=8", k_fma_chains<8>, blocks, thr, 8, din, dout, dcyc);
        run("fma + dpp swap (2 x v_mov_b32_dpp)", k_dpp_chain, blocks, thr, 1, din, dout, dcyc);
        run("rcp + 2 newton (5 dep)", k_rcp_chain, blocks, thr, 5, din, dout, dcyc);
    }
    return 0;
}
