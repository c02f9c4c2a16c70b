// Calibration of rocprofv3 FETCH_SIZE / WRITE_SIZE on gfx950 for the solver's access widths (measurement tool).
//
// MI355X_MICROARCH.md calibrates FETCH_SIZE only for 16-B-per-lane streaming reads (it reports exactly half of
// the bytes) and WRITE_SIZE for 16-B-per-lane streaming stores (exact).  The solver's phase kernel also moves
// 8-B-per-lane planes (the cg offset, the tau2 controls).  Each kernel below moves a KNOWN byte count, once,
// through buffers far larger than the 256 MiB Infinity Cache, with the solver's access shape (one wavefront per
// 64 lanes, one row per stage, non-temporal as the solver's streams):
//   k_cal_rd16 : 16 B per lane per row (double2)        k_cal_wr16 : 16 B per lane per row stores
//   k_cal_rd8  :  8 B per lane per row (double)         k_cal_wr8  :  8 B per lane per row stores
// Run:  rocprofv3 --pmc FETCH_SIZE --kernel-include-regex k_cal -- tools/fetch_calib   (and WRITE_SIZE)
// and divide the counter by the printed byte count.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

typedef double d2v __attribute__((ext_vector_type(2)));
constexpr long long LANES = 262144;    // the bench's lanes per GPU
constexpr int ROWS = 1000;             // rows of LANES elements: 2.1 GB (16 B) / 1.05 GB (8 B) per pass

__global__ __launch_bounds__(64) void k_cal_rd16(const d2v* __restrict__ a, double* __restrict__ sink) {
    const long long l = (long long)blockIdx.x * 64 + threadIdx.x;
    double s = 0.0;
    for (int r = 0; r < ROWS; ++r) {
        const d2v v = __builtin_nontemporal_load(a + (long long)r * LANES + l);
        s += v.x + v.y;
    }
    if (s == 1.2345) sink[l] = s;   // never true for the zero-filled input: keeps the loads, stores nothing
}

__global__ __launch_bounds__(64) void k_cal_rd8(const double* __restrict__ a, double* __restrict__ sink) {
    const long long l = (long long)blockIdx.x * 64 + threadIdx.x;
    double s = 0.0;
    for (int r = 0; r < ROWS; ++r) s += __builtin_nontemporal_load(a + (long long)r * LANES + l);
    if (s == 1.2345) sink[l] = s;
}

__global__ __launch_bounds__(64) void k_cal_wr16(d2v* __restrict__ a, double v) {
    const long long l = (long long)blockIdx.x * 64 + threadIdx.x;
    for (int r = 0; r < ROWS; ++r) {
        const d2v w = {v + r, v - r};
        __builtin_nontemporal_store(w, a + (long long)r * LANES + l);
    }
}

__global__ __launch_bounds__(64) void k_cal_wr8(double* __restrict__ a, double v) {
    const long long l = (long long)blockIdx.x * 64 + threadIdx.x;
    for (int r = 0; r < ROWS; ++r) __builtin_nontemporal_store(v + r, a + (long long)r * LANES + l);
}

#define CK(x)                                                                                  \
    do {                                                                                       \
        hipError_t e_ = (x);                                                                   \
        if (e_ != hipSuccess) {                                                                \
            fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_));          \
            return 1;                                                                          \
        }                                                                                      \
    } while (0)

int main() {
    const size_t b16 = sizeof(d2v) * LANES * ROWS, b8 = sizeof(double) * LANES * ROWS;
    d2v *a16, *w16;
    double *a8, *w8, *sink;
    CK(hipMalloc(&a16, b16)); CK(hipMalloc(&w16, b16));
    CK(hipMalloc(&a8, b8)); CK(hipMalloc(&w8, b8));
    CK(hipMalloc(&sink, sizeof(double) * LANES));
    CK(hipMemset(a16, 0, b16)); CK(hipMemset(a8, 0, b8));
    CK(hipDeviceSynchronize());
    const dim3 grid(LANES / 64), blk(64);
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
    struct { const char* name; size_t bytes; } rows[4] = {{"k_cal_rd16", b16}, {"k_cal_rd8", b8},
                                                          {"k_cal_wr16", b16}, {"k_cal_wr8", b8}};
    for (int k = 0; k < 4; ++k) {
        for (int rep = 0; rep < 2; ++rep) {
            CK(hipEventRecord(e0));
            if (k == 0) hipLaunchKernelGGL(k_cal_rd16, grid, blk, 0, 0, a16, sink);
            if (k == 1) hipLaunchKernelGGL(k_cal_rd8, grid, blk, 0, 0, a8, sink);
            if (k == 2) hipLaunchKernelGGL(k_cal_wr16, grid, blk, 0, 0, w16, 1.0);
            if (k == 3) hipLaunchKernelGGL(k_cal_wr8, grid, blk, 0, 0, w8, 1.0);
            CK(hipEventRecord(e1));
            CK(hipEventSynchronize(e1));
            float ms = 0;
            CK(hipEventElapsedTime(&ms, e0, e1));
            printf("%-11s bytes %12zu  %8.3f ms  %7.1f GB/s\n", rows[k].name, rows[k].bytes, ms,
                   rows[k].bytes / (ms * 1e-3) / 1e9);
        }
    }
    return 0;
}
