// Device allocations with explicit HIP flags, for placement experiments (measurement tool, not part of the product):
// hipExtMallocWithFlags(hipDeviceMallocContiguous) asks the driver for physically contiguous VRAM.
// Build: hipcc --offload-arch=gfx950 -O3 -fPIC -shared tools/contig_alloc.hip -o tools/libcontig_alloc.so
#include <hip/hip_runtime.h>
#include <cstdint>

extern "C" {
int ca_malloc(int64_t bytes, unsigned flags, void** out) {
    *out = nullptr;
    return (int)hipExtMallocWithFlags(out, (size_t)bytes, flags);
}
int ca_free(void* p) { return (int)hipFree(p); }
}
