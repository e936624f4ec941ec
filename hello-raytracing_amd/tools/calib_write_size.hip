// calib_write_size — calibrates rocprofv3's WRITE_SIZE for the sample buffer's store form (MI355X_MICROARCH.md § HBM: widths
// other than 16 B per lane are uncalibrated). Each sample is 3 floats (12 B) at a contiguous place, as k_trace_split's
// ring_store writes the sample buffer (global_store_dwordx3). Two launches over the same byte count:
//   coalesced : every lane of a wave stores its sample in one instruction (a tile-frame's 768 B at once: whole lines);
//   staggered : lane l of a wave stores in round l, s_sleep between rounds (the tile-frame's lines written over 64
//               rounds, as samples finish at different times in the tracing kernel).
// usage: calib_write_size [MiB]   then divide the launches' WRITE_SIZE by the printed bytes (rocprofv3 --pmc WRITE_SIZE).
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

__global__ __launch_bounds__(256) void k_coalesced(float* o, unsigned n) {
    const unsigned i = blockIdx.x * 256u + threadIdx.x;
    if (i < n) {
        float* p = o + 3ull * i;
        p[0] = (float)i;
        p[1] = (float)(i + 1u);
        p[2] = (float)(i + 2u);
    }
}

__global__ __launch_bounds__(256) void k_staggered(float* o, unsigned n) {
    const unsigned i = blockIdx.x * 256u + threadIdx.x, lane = threadIdx.x & 63u;
    for (unsigned r = 0; r < 64u; r++) {
        if (r == lane && i < n) {
            float* p = o + 3ull * i;
            p[0] = (float)i;
            p[1] = (float)(i + 1u);
            p[2] = (float)(i + 2u);
        }
        __builtin_amdgcn_s_sleep(8);
    }
}

int main(int argc, char** argv) {
    const size_t mib = argc > 1 ? (size_t)atoi(argv[1]) : 768;
    const unsigned n = (unsigned)((mib << 20) / 12u / 64u * 64u);
    float* o = nullptr;
    if (hipMalloc(&o, 12ull * n) != hipSuccess) return 2;
    const unsigned blocks = (n + 255u) / 256u;
    hipLaunchKernelGGL(k_coalesced, dim3(blocks), dim3(256), 0, 0, o, n);
    hipLaunchKernelGGL(k_staggered, dim3(blocks), dim3(256), 0, 0, o, n);
    if (hipDeviceSynchronize() != hipSuccess) return 3;
    printf("{\"samples\": %u, \"bytes_per_launch\": %llu}\n", n, 12ull * n);
    (void)hipFree(o);
    return 0;
}
