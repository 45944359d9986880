// gather_probe.hip -- design probe (not product code): the rate of random
// 4-byte gathers on MI355X, the access pattern of the pipeline kernel's
// route-root and hostname-pool lookups, by table size, gathers per item,
// items in flight per lane and workgroups per CU.  Each item streams a
// 4-byte key in and a 4-byte result out.
//
//   hipcc -O3 --offload-arch=gfx950 tools/gather_probe.hip -o tools/gather_probe
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

// G gathers per item, U (1, 4 or 8) items per lane per step: all U*G
// gathers of a step are independent and issued before any is used.
template <int G, int U>
__global__ __launch_bounds__(512) void gather(const uint32_t* __restrict__ keys, int64_t n,
                                              const uint32_t* __restrict__ t0,
                                              const uint32_t* __restrict__ t1, uint32_t mask,
                                              uint32_t* __restrict__ out) {
    const int64_t steps = n / U;
    for (int64_t g = blockIdx.x * int64_t(blockDim.x) + threadIdx.x; g < steps;
         g += int64_t(gridDim.x) * blockDim.x) {
        uint32_t kk[U], r[U];
        if (U == 1) {
            kk[0] = keys[g];
        } else {
#pragma unroll
            for (int q = 0; q < U; q += 4) {
                const uint4 k = reinterpret_cast<const uint4*>(keys)[g * (U / 4) + q / 4];
                kk[q] = k.x;
                kk[q + 1] = k.y;
                kk[q + 2] = k.z;
                kk[q + 3] = k.w;
            }
        }
#pragma unroll
        for (int j = 0; j < U; ++j) r[j] = t0[kk[j] & mask];
        if (G == 2) {
#pragma unroll
            for (int j = 0; j < U; ++j) r[j] += t1[mixh(kk[j]) & mask];
        }
        if (U == 1) {
            out[g] = r[0];
        } else {
#pragma unroll
            for (int q = 0; q < U; q += 4)
                reinterpret_cast<uint4*>(out)[g * (U / 4) + q / 4] =
                    make_uint4(r[q], r[q + 1], r[q + 2], r[q + 3]);
        }
    }
}

// Two tables of different sizes: per item one gather into t0 (mask0, the
// candidate route root) and one into t1 (mask1, the 64 MB pool results);
// kNt: the t1 gather is a nontemporal load, so its lines should not push
// t0's out of L2.
template <bool kNt>
__global__ __launch_bounds__(512) void gather_mix(const uint32_t* __restrict__ keys, int64_t n,
                                                  const uint32_t* __restrict__ t0, uint32_t mask0,
                                                  const uint32_t* __restrict__ t1, uint32_t mask1,
                                                  uint32_t* __restrict__ out) {
    const int64_t steps = n / 4;
    for (int64_t g = blockIdx.x * int64_t(blockDim.x) + threadIdx.x; g < steps;
         g += int64_t(gridDim.x) * blockDim.x) {
        const uint4 k = reinterpret_cast<const uint4*>(keys)[g];
        const uint32_t kk[4] = {k.x, k.y, k.z, k.w};
        uint32_t r[4], q[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) r[j] = t0[kk[j] & mask0];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const uint32_t* a = t1 + (mixh(kk[j]) & mask1);
            q[j] = kNt ? __builtin_nontemporal_load(a) : *a;
        }
        reinterpret_cast<uint4*>(out)[g] =
            make_uint4(r[0] + q[0], r[1] + q[1], r[2] + q[2], r[3] + q[3]);
    }
}

template <int G, int U>
float run(int grid, const uint32_t* keys, int64_t n, const uint32_t* t0, const uint32_t* t1,
          uint32_t mask, uint32_t* out, hipEvent_t a, hipEvent_t b) {
    float best = 1e30f;
    for (int rep = 0; rep < 4; ++rep) {
        CK(hipEventRecord(a, 0));
        hipLaunchKernelGGL((gather<G, U>), dim3(grid), dim3(512), 0, 0, keys, n, t0, t1, mask,
                           out);
        CK(hipEventRecord(b, 0));
        CK(hipEventSynchronize(b));
        float ms;
        CK(hipEventElapsedTime(&ms, a, b));
        if (rep > 0 && ms < best) best = ms;
    }
    return best;
}

int main(int argc, char** argv) {
    const int64_t n = 125000000 / 8 * 8;               // one C5 batch
    const bool cal = argc > 1 && std::string(argv[1]) == "cal";
    hipDeviceProp_t p;
    CK(hipGetDeviceProperties(&p, 0));
    const int cus = p.multiProcessorCount;
    uint32_t *keys, *out, *t0, *t1;
    const int64_t max_words = int64_t(1) << 28;        // 1 GiB tables
    CK(hipMalloc(&keys, n * 4));
    CK(hipMalloc(&out, n * 4));
    CK(hipMalloc(&t0, max_words * 4));
    CK(hipMalloc(&t1, max_words * 4));
    hipLaunchKernelGGL(fill_keys, dim3(4096), dim3(256), 0, 0, keys, n, 1u);
    hipLaunchKernelGGL(fill_table, dim3(4096), dim3(256), 0, 0, t0, max_words);
    hipLaunchKernelGGL(fill_table, dim3(4096), dim3(256), 0, 0, t1, max_words);
    CK(hipDeviceSynchronize());
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    if (argc > 1 && std::string(argv[1]) == "mix") {
        // route-root candidates (t0: 1-64 MB) beside the 64 MB pool table (t1)
        printf("root_MB,pool_MB,pool_nt,blocks_per_cu,ms,G_items_per_s,G_gathers_per_s\n");
        const uint32_t mask1 = uint32_t((int64_t(64) << 20) / 4 - 1);
        for (int mb : {1, 2, 4, 8, 16, 64})
            for (int nt = 0; nt < 2; ++nt)
                for (int bpc : {2, 4}) {
                    const uint32_t mask0 = uint32_t((int64_t(mb) << 20) / 4 - 1);
                    float best = 1e30f;
                    for (int rep = 0; rep < 4; ++rep) {
                        CK(hipEventRecord(a, 0));
                        if (nt)
                            hipLaunchKernelGGL(gather_mix<true>, dim3(cus * bpc), dim3(512), 0, 0,
                                               keys, n, t0, mask0, t1, mask1, out);
                        else
                            hipLaunchKernelGGL(gather_mix<false>, dim3(cus * bpc), dim3(512), 0, 0,
                                               keys, n, t0, mask0, t1, mask1, out);
                        CK(hipEventRecord(b, 0));
                        CK(hipEventSynchronize(b));
                        float ms;
                        CK(hipEventElapsedTime(&ms, a, b));
                        if (rep > 0 && ms < best) best = ms;
                    }
                    printf("%d,64,%d,%d,%.3f,%.2f,%.2f\n", mb, nt, bpc, best, n / (best * 1e-3) / 1e9,
                           2 * n / (best * 1e-3) / 1e9);
                    fflush(stdout);
                }
        return 0;
    }
    if (cal) {
        // PMC calibration (run under rocprofv3 --pmc): one launch per line, in
        // this order, 4 items per lane, 4 workgroups per CU.  The 4 KiB table
        // stays in L2, so its launch counts only the key stream (n x 4 B,
        // 16-B loads) and the result stream (n x 4 B, 16-B stores); the others
        // add n x G uniformly random 4-byte gathers into the table.
        // Launch 5 (round 4) streams the keys with 4-byte loads (one item per
        // lane, consecutive lanes consecutive words), the width the string
        // kernels stage names and read offsets with.
        printf("launch,table_KB,gathers_per_item,items,ms\n");
        const int64_t kb[] = {4, 64 << 10, 64 << 10, 1 << 20, 1 << 20, 4};
        const int gs[] = {1, 1, 2, 1, 2, 1};
        for (int l = 0; l < 6; ++l) {
            const uint32_t mask = uint32_t(kb[l] * 1024 / 4 - 1);
            CK(hipEventRecord(a, 0));
            if (l == 5)
                hipLaunchKernelGGL((gather<1, 1>), dim3(cus * 4), dim3(512), 0, 0, keys, n, t0, t1,
                                   mask, out);
            else if (gs[l] == 1)
                hipLaunchKernelGGL((gather<1, 4>), dim3(cus * 4), dim3(512), 0, 0, keys, n, t0, t1,
                                   mask, out);
            else
                hipLaunchKernelGGL((gather<2, 4>), dim3(cus * 4), dim3(512), 0, 0, keys, n, t0, t1,
                                   mask, out);
            CK(hipEventRecord(b, 0));
            CK(hipEventSynchronize(b));
            float ms;
            CK(hipEventElapsedTime(&ms, a, b));
            printf("%d,%lld,%d,%lld,%.3f\n", l, (long long)kb[l], gs[l], (long long)n, ms);
        }
        return 0;
    }
    printf("table_MB,gathers_per_item,items_per_lane,blocks_per_cu,ms,G_items_per_s,G_gathers_per_s\n");
    const int sizes_mb[] = {4, 16, 64, 256, 1024};
    for (int mb : sizes_mb) {
        const uint32_t mask = uint32_t((int64_t(mb) << 20) / 4 - 1);
        for (int G = 1; G <= 2; ++G)
            for (int U : {1, 4, 8})
                for (int bpc : {2, 4, 8}) {
                    const int grid = cus * bpc;
                    float ms;
                    if (G == 1)
                        ms = U == 1 ? run<1, 1>(grid, keys, n, t0, t1, mask, out, a, b)
                           : U == 4 ? run<1, 4>(grid, keys, n, t0, t1, mask, out, a, b)
                                    : run<1, 8>(grid, keys, n, t0, t1, mask, out, a, b);
                    else
                        ms = U == 1 ? run<2, 1>(grid, keys, n, t0, t1, mask, out, a, b)
                           : U == 4 ? run<2, 4>(grid, keys, n, t0, t1, mask, out, a, b)
                                    : run<2, 8>(grid, keys, n, t0, t1, mask, out, a, b);
                    printf("%d,%d,%d,%d,%.3f,%.2f,%.2f\n", mb, G, U, bpc, ms,
                           n / (ms * 1e-3) / 1e9, G * n / (ms * 1e-3) / 1e9);
                    fflush(stdout);
                }
    }
    return 0;
}
