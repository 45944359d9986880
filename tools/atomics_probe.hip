// atomics_probe.hip -- design probe (not product code): what do per-rule hit
// counters cost on MI355X?  Scattered device atomics vs LDS-chunked
// histograms over the classifier's output arrays.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s\n", hipGetErrorString(e)); exit(1); } } while (0)

__global__ void atom64(const int* idx, long n, unsigned long long* c) {
    for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x)
        atomicAdd(c + idx[i], 1ull);
}
__global__ void atom32(const int* idx, long n, unsigned* c) {
    for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x)
        atomicAdd(c + idx[i], 1u);
}
// LDS-chunked histogram: grid.y = chunk; each block counts its slice of items
// falling into [chunk*CH, (chunk+1)*CH) in LDS, then flushes coalesced.
template <int CH>
__global__ __launch_bounds__(1024) void lds_hist(const int* idx, long n, unsigned long long* c, int m) {
    __shared__ unsigned h[CH];
    const int base = blockIdx.y * CH;
    for (int k = threadIdx.x; k < CH; k += blockDim.x) h[k] = 0;
    __syncthreads();
    const long per = (n + gridDim.x - 1) / gridDim.x;
    const long lo = blockIdx.x * per, hi = lo + per < n ? lo + per : n;
    for (long i = lo + threadIdx.x * 4; i < hi; i += blockDim.x * 4) {
        int4 v = i + 3 < hi ? *reinterpret_cast<const int4*>(idx + i) : make_int4(-1, -1, -1, -1);
        if (i + 3 >= hi) { int* p = &v.x; for (int t = 0; t < 4 && i + t < hi; ++t) p[t] = idx[i + t]; }
        int vv[4] = {v.x, v.y, v.z, v.w};
        for (int t = 0; t < 4; ++t) {
            unsigned d = unsigned(vv[t] - base);
            if (d < CH) atomicAdd(&h[d], 1u);
        }
    }
    __syncthreads();
    for (int k = threadIdx.x; k < CH && base + k < m; k += blockDim.x)
        if (h[k]) atomicAdd(c + base + k, (unsigned long long)h[k]);
}

int main() {
    const long n = 125000000;
    const int M = 1200000;
    std::vector<int> host(n);
    srand(1);
    for (long i = 0; i < n; ++i) host[i] = (int)(((unsigned)rand() * 2654435761u) % M);
    std::vector<int> hot(host);
    for (long i = 0; i < n; i += 5) hot[i] = 7;   // 20% to one bin
    int *d, *dh;
    unsigned long long* c;
    unsigned* c32;
    CK(hipMalloc(&d, n * 4)); CK(hipMalloc(&dh, n * 4));
    CK(hipMalloc(&c, M * 8)); CK(hipMalloc(&c32, M * 4));
    CK(hipMemcpy(d, host.data(), n * 4, hipMemcpyHostToDevice));
    CK(hipMemcpy(dh, hot.data(), n * 4, hipMemcpyHostToDevice));
    hipEvent_t a, b;
    hipEventCreate(&a); hipEventCreate(&b);
    auto time = [&](const char* name, auto fn) {
        fn(); CK(hipDeviceSynchronize());
        hipEventRecord(a); for (int r = 0; r < 3; ++r) fn(); hipEventRecord(b);
        CK(hipEventSynchronize(b)); float ms; hipEventElapsedTime(&ms, a, b);
        printf("%-40s %8.3f ms  (%.2f G ops/s)\n", name, ms / 3, n / (ms / 3 * 1e6));
    };
    time("u64 atomics uniform 1.2M bins", [&] { atom64<<<2048, 256>>>(d, n, c); });
    time("u32 atomics uniform 1.2M bins", [&] { atom32<<<2048, 256>>>(d, n, c32); });
    time("u64 atomics 20% one bin", [&] { atom64<<<2048, 256>>>(dh, n, c); });
    time("u32 atomics 20% one bin", [&] { atom32<<<2048, 256>>>(dh, n, c32); });
    const int chunks = (M + 32767) / 32768;
    time("lds hist 32K-bin chunks (38 passes)", [&] { lds_hist<32768><<<dim3(512, chunks), 1024>>>(d, n, c, M); });
    time("lds hist 32K chunks, hot input", [&] { lds_hist<32768><<<dim3(512, chunks), 1024>>>(dh, n, c, M); });
    return 0;
}
