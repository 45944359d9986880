// gather_paths.hip -- design probe (not product code): WHERE the random
// 4-byte gather rate of MI355X is capped, and whether another load path
// adds capacity.  The pipeline kernel makes two uniformly random 4-byte
// gathers per packet into 64 MB tables and runs at ~92 % of the rate
// gather_probe.hip measures; this probe asks what that rate is made of.
//
//   cus:    G gathers/item, 4 items/lane, one 512-thread workgroup on K CUs,
//           K = 8..256, spread over the 8 XCDs (workgroup i -> XCD i % 8) or
//           packed onto XCD 0 only (the grid is 8K, blocks with i % 8 != 0
//           exit at once).  Rate proportional to K at equal placement means
//           a per-CU cap; packed < spread at equal K means a per-XCD one.
//
// Result (profiles/r03_gather_paths.csv): ~700 M gathers/s per CU with few
// CUs, one XCD tops out near 10.4 G/s, and the chip at ~56 G/s from 128 CUs
// on (53 G/s at 256): the cap is past the CUs, in the miss path from the
// L2s, so no other load path of a CU (the scalar cache) can add to it.
//
//   hipcc -O3 --offload-arch=gfx950 tools/gather_paths.hip -o tools/gather_paths
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
        t[i] = uint32_t(i);
}

// Workgroups whose index is not a multiple of `stride` exit at once; the
// others split the items evenly (vid = blockIdx / stride of nwork).
template <int G>
__global__ __launch_bounds__(512) void gather_cus(const uint32_t* __restrict__ keys, int64_t n,
                                                  const uint32_t* __restrict__ t0,
                                                  const uint32_t* __restrict__ t1, uint32_t mask,
                                                  uint32_t* __restrict__ out, int stride,
                                                  int nwork) {
    if (blockIdx.x % stride) return;
    const int64_t vid = blockIdx.x / stride;
    const int64_t steps = n / 4;
    for (int64_t g = vid * 512 + threadIdx.x; g < steps; g += int64_t(nwork) * 512) {
        const uint4 k = reinterpret_cast<const uint4*>(keys)[g];
        const uint32_t kk[4] = {k.x, k.y, k.z, k.w};
        uint32_t r[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) r[j] = t0[kk[j] & mask];
        if (G == 2) {
#pragma unroll
            for (int j = 0; j < 4; ++j) r[j] += t1[mixh(kk[j]) & mask];
        }
        reinterpret_cast<uint4*>(out)[g] = make_uint4(r[0], r[1], r[2], r[3]);
    }
}

static hipEvent_t ea, eb;

template <class F>
float best_of(F launch) {
    float best = 1e30f;
    for (int rep = 0; rep < 4; ++rep) {
        CK(hipEventRecord(ea, 0));
        launch();
        CK(hipEventRecord(eb, 0));
        CK(hipEventSynchronize(eb));
        float ms;
        CK(hipEventElapsedTime(&ms, ea, eb));
        if (rep > 0 && ms < best) best = ms;
    }
    return best;
}

int main(int argc, char** argv) {
    const int64_t n = 125000000 / 8 * 8;
    const std::string mode = argc > 1 ? argv[1] : "all";
    hipDeviceProp_t p;
    CK(hipGetDeviceProperties(&p, 0));
    const int cus = p.multiProcessorCount;
    uint32_t *keys, *out, *t0, *t1;
    const int64_t words = int64_t(64) << 18;            // 64 MiB tables
    CK(hipMalloc(&keys, n * 4));
    CK(hipMalloc(&out, n * 4));
    CK(hipMalloc(&t0, words * 4));
    CK(hipMalloc(&t1, words * 4));
    hipLaunchKernelGGL(fill_keys, dim3(4096), dim3(256), 0, 0, keys, n, 1u);
    hipLaunchKernelGGL(fill_table, dim3(4096), dim3(256), 0, 0, t0, words);
    hipLaunchKernelGGL(fill_table, dim3(4096), dim3(256), 0, 0, t1, words);
    CK(hipDeviceSynchronize());
    CK(hipEventCreate(&ea));
    CK(hipEventCreate(&eb));
    const uint32_t mask = uint32_t(words - 1);
    if (mode == "all" || mode == "cus") {
        printf("probe,placement,cus_used,gathers_per_item,ms,G_gathers_per_s,M_gathers_per_s_per_cu\n");
        for (int G = 1; G <= 2; ++G)
            for (int k : {8, 16, 32, 64, 128, 256}) {
                for (int packed = 0; packed < 2; ++packed) {
                    if (packed && k > cus / 8) continue;
                    // spread: grid k, stride 1 -> workgroup i on XCD i % 8;
                    // packed: grid 8k, stride 8 -> every live workgroup on XCD 0
                    const int stride = packed ? 8 : 1, grid = k * stride;
                    const float ms = best_of([&] {
                        if (G == 1)
                            hipLaunchKernelGGL(gather_cus<1>, dim3(grid), dim3(512), 0, 0, keys, n,
                                               t0, t1, mask, out, stride, k);
                        else
                            hipLaunchKernelGGL(gather_cus<2>, dim3(grid), dim3(512), 0, 0, keys, n,
                                               t0, t1, mask, out, stride, k);
                    });
                    const double gps = G * n / (ms * 1e-3);
                    printf("cus,%s,%d,%d,%.3f,%.2f,%.1f\n", packed ? "xcd0" : "spread", k, G, ms,
                           gps / 1e9, gps / k / 1e6);
                    fflush(stdout);
                }
            }
    }
    return 0;
}
