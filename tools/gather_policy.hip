// gather_policy.hip -- design probe (not product code): does the cache
// policy of a random 4-byte gather change the rate at which MI355X serves
// it from a 64 MB table (the pipeline kernel's route-root and pool lookups,
// capped at ~55 G gathers/s)?  Two gathers per item into two
// tables, 4 items per lane per step, 125M items, through buffer loads whose
// aux operand sets the gfx950 cache-policy bits (sc0 = 1, nt = 2, sc1 = 16):
// one kernel per combination, each timed over 5 launches after a warmup.
//
//   hipcc -O3 --offload-arch=gfx950 tools/gather_policy.hip -o tools/gather_policy
//   tools/gather_policy [table_MB ...]     -> CSV on stdout
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <string>

#define CK(x)                                                                    \
    do {                                                                         \
        hipError_t e_ = (x);                                                     \
        if (e_ != hipSuccess) {                                                  \
            printf("%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_));     \
            exit(1);                                                             \
        }                                                                        \
    } while (0)

__host__ __device__ inline uint32_t mixh(uint32_t x) {
    x ^= x >> 16;
    x *= 0x7feb352du;
    x ^= x >> 15;
    x *= 0x846ca68bu;
    x ^= x >> 16;
    return x;
}

__global__ void fill_keys(uint32_t* k, int64_t n, uint32_t seed) {
    for (int64_t i = blockIdx.x * int64_t(blockDim.x) + threadIdx.x; i < n;
         i += int64_t(gridDim.x) * blockDim.x)
        k[i] = mixh(uint32_t(i) * 2654435761u + seed);
}

__global__ void fill_table(uint32_t* t, int64_t n) {
    for (int64_t i = blockIdx.x * int64_t(blockDim.x) + threadIdx.x; i < n;
         i += int64_t(gridDim.x) * blockDim.x)
        t[i] = uint32_t(i) * 7u;
}

template <int AUX>
__device__ __forceinline__ uint32_t ld(__amdgpu_buffer_rsrc_t r, uint32_t idx) {
    return __builtin_amdgcn_raw_buffer_load_b32(r, int(idx * 4u), 0, AUX);
}

template <int AUX>
__global__ __launch_bounds__(512) void gather2(const uint32_t* __restrict__ keys, int64_t n,
                                               const uint32_t* t0, const uint32_t* t1,
                                               uint32_t mask, uint32_t* __restrict__ out) {
    const __amdgpu_buffer_rsrc_t r0 =
        __builtin_amdgcn_make_buffer_rsrc(const_cast<uint32_t*>(t0), 0, int((mask + 1) * 4), 0x00020000);
    const __amdgpu_buffer_rsrc_t r1 =
        __builtin_amdgcn_make_buffer_rsrc(const_cast<uint32_t*>(t1), 0, int((mask + 1) * 4), 0x00020000);
    const int64_t steps = n / 4;
    for (int64_t g = blockIdx.x * int64_t(blockDim.x) + threadIdx.x; g < steps;
         g += int64_t(gridDim.x) * blockDim.x) {
        const uint4 k = reinterpret_cast<const uint4*>(keys)[g];
        const uint32_t kk[4] = {k.x, k.y, k.z, k.w};
        uint32_t r[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) r[j] = ld<AUX>(r0, kk[j] & mask);
#pragma unroll
        for (int j = 0; j < 4; ++j) r[j] += ld<AUX>(r1, mixh(kk[j]) & mask);
        reinterpret_cast<uint4*>(out)[g] = make_uint4(r[0], r[1], r[2], r[3]);
    }
}

template <int AUX>
static void run(const char* name, const uint32_t* keys, int64_t n, const uint32_t* t0,
                const uint32_t* t1, uint32_t mask, uint32_t* out, int grid, int mb) {
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    hipLaunchKernelGGL(gather2<AUX>, dim3(grid), dim3(512), 0, 0, keys, n, t0, t1, mask, out);
    CK(hipDeviceSynchronize());
    CK(hipEventRecord(a, 0));
    const int reps = 5;
    for (int i = 0; i < reps; ++i)
        hipLaunchKernelGGL(gather2<AUX>, dim3(grid), dim3(512), 0, 0, keys, n, t0, t1, mask, out);
    CK(hipEventRecord(b, 0));
    CK(hipEventSynchronize(b));
    float ms = 0;
    CK(hipEventElapsedTime(&ms, a, b));
    ms /= reps;
    printf("%s,%d,%d,%.4f,%.2f\n", name, AUX, mb, ms, 2.0 * n / (ms * 1e-3) / 1e9);
    fflush(stdout);
}

int main(int argc, char** argv) {
    const int64_t n = 125000000;
    int cus = 0;
    CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
    const int grid = cus * 4;
    uint32_t *keys, *out, *t0, *t1;
    CK(hipMalloc(&keys, n * 4));
    CK(hipMalloc(&out, n * 4));
    fill_keys<<<4096, 256>>>(keys, n, 12345u);
    printf("policy,aux,table_MB,ms,G_gathers_per_s\n");
    for (int a = 1; a < argc || a == 1; ++a) {
        const int mb = argc > 1 ? atoi(argv[a]) : 64;
        const int64_t entries = int64_t(mb) << 18;          // 4-byte entries
        CK(hipMalloc(&t0, entries * 4));
        CK(hipMalloc(&t1, entries * 4));
        fill_table<<<4096, 256>>>(t0, entries);
        fill_table<<<4096, 256>>>(t1, entries);
        CK(hipDeviceSynchronize());
        const uint32_t mask = uint32_t(entries - 1);
        run<0>("default", keys, n, t0, t1, mask, out, grid, mb);
        run<1>("sc0", keys, n, t0, t1, mask, out, grid, mb);
        run<2>("nt", keys, n, t0, t1, mask, out, grid, mb);
        run<3>("sc0_nt", keys, n, t0, t1, mask, out, grid, mb);
        run<16>("sc1", keys, n, t0, t1, mask, out, grid, mb);
        run<17>("sc0_sc1", keys, n, t0, t1, mask, out, grid, mb);
        run<18>("sc1_nt", keys, n, t0, t1, mask, out, grid, mb);
        run<19>("sc0_sc1_nt", keys, n, t0, t1, mask, out, grid, mb);
        run<0>("default_again", keys, n, t0, t1, mask, out, grid, mb);
        CK(hipFree(t0));
        CK(hipFree(t1));
        if (argc <= 1) break;
    }
    CK(hipFree(keys));
    CK(hipFree(out));
    return 0;
}
