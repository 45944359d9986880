// partition_probe.hip -- design probe (not product code): can the C5
// pipeline's two random table lookups per packet (route root and hostname
// pool, 64 MB each) run faster as a radix-partitioned lookup than as direct
// gathers?  Direct gathers are bound by the L2-to-fabric request rate (one
// 64-byte request per 4-byte gather, profiles/r01_gather_probe.csv).  The
// partitioned form streams instead:
//   pass 0  per-wave histogram of each key's bucket (its top bits)
//   scan    bucket-major exclusive scan of the per-wave counts
//   pass 1  each wave writes its keys to its segment of each bucket, in order
//   pass 2  the chip sweeps the bucket-sorted keys front to back, so the
//           table slice it gathers from at any moment (64 MB / NB) stays in
//           the XCDs' L2; results are written in the sorted order
//   pass 3  each wave recomputes its keys' sorted positions (same order as
//           pass 1) and reads its results back into packet order
// Streamed bytes per key: 4 + (4 + 4) + (4 + 4) + (4 + 4 + 4) = 32.
//
//   hipcc -O3 --offload-arch=gfx950 tools/partition_probe.hip -o tools/partition_probe
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>

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

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
__device__ __forceinline__ uint4 ntl(const uint4* p) {
    const u32x4 v = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(p));
    return make_uint4(v.x, v.y, v.z, v.w);
}
__device__ __forceinline__ void nts(uint4* p, uint4 v) {
    u32x4 w = {v.x, v.y, v.z, v.w};
    __builtin_nontemporal_store(w, reinterpret_cast<u32x4*>(p));
}

__global__ void fill(uint32_t* d, uint32_t* h, uint32_t* tr, uint32_t* tg, int64_t n, int64_t tn) {
    for (int64_t i = blockIdx.x * int64_t(blockDim.x) + threadIdx.x; i < n;
         i += int64_t(gridDim.x) * blockDim.x) {
        d[i] = mixh(uint32_t(i) * 2654435761u + 17u);
        h[i] = mixh(uint32_t(i) * 2246822519u + 91u) & 0xFFFFFFu;
        if (i < tn) {
            tr[i] = mixh(uint32_t(i) + 5u);
            tg[i] = mixh(uint32_t(i) + 7u);
        }
    }
}

// Direct: the pipeline kernel's lookups (4 packets per lane, both gathers in flight).
__global__ __launch_bounds__(1024) void direct(const uint32_t* __restrict__ d,
                                               const uint32_t* __restrict__ h,
                                               const uint32_t* __restrict__ tr,
                                               const uint32_t* __restrict__ tg, int64_t n4,
                                               uint32_t* __restrict__ orr, uint32_t* __restrict__ og) {
    for (int64_t g = blockIdx.x * int64_t(blockDim.x) + threadIdx.x; g < n4;
         g += int64_t(gridDim.x) * blockDim.x) {
        const uint4 a = ntl(reinterpret_cast<const uint4*>(d) + g);
        const uint4 b = ntl(reinterpret_cast<const uint4*>(h) + g);
        const uint4 r = make_uint4(tr[a.x >> 8], tr[a.y >> 8], tr[a.z >> 8], tr[a.w >> 8]);
        const uint4 q = make_uint4(tg[b.x], tg[b.y], tg[b.z], tg[b.w]);
        nts(reinterpret_cast<uint4*>(orr) + g, r);
        nts(reinterpret_cast<uint4*>(og) + g, q);
    }
}

constexpr int kWaves = 4;          // waves per workgroup of passes 0, 1, 3
constexpr int kBlock = 64 * kWaves;

template <int NB>
__device__ __forceinline__ uint32_t bucket_of(uint32_t key, int kbits) {
    return key >> (kbits - __builtin_ctz(NB));
}

// lanes with the same bucket: their mask, via log2(NB) ballots
template <int NB>
__device__ __forceinline__ uint64_t same_bucket(uint32_t b) {
    uint64_t m = ~0ull;
#pragma unroll
    for (int bit = 0; bit < __builtin_ctz(NB); ++bit) {
        const bool s = (b >> bit) & 1u;
        const uint64_t v = __ballot(s);
        m &= s ? v : ~v;
    }
    return m;
}

__device__ __forceinline__ uint32_t lanes_below(uint64_t m) {
    return __builtin_amdgcn_mbcnt_hi(uint32_t(m >> 32), __builtin_amdgcn_mbcnt_lo(uint32_t(m), 0u));
}

// wave w's tile: [w*S, min(n, (w+1)*S)), S a multiple of 256; n % 4 == 0 here
template <int NB>
__global__ __launch_bounds__(kBlock) void hist(const uint32_t* __restrict__ key, int kbits,
                                               int64_t n, int64_t S, int W,
                                               uint32_t* __restrict__ cnt) {
    __shared__ uint32_t h[kWaves][NB];
    const int wl = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int w = blockIdx.x * kWaves + wl;
    for (int b = lane; b < NB; b += 64) h[wl][b] = 0;
    __builtin_amdgcn_wave_barrier();
    const int64_t lo = int64_t(w) * S, hi = lo + S < n ? lo + S : n;
    for (int64_t i = lo + 4 * lane; i < hi; i += 256) {
        const uint4 k = ntl(reinterpret_cast<const uint4*>(key + i));
        atomicAdd(&h[wl][bucket_of<NB>(k.x, kbits)], 1u);
        atomicAdd(&h[wl][bucket_of<NB>(k.y, kbits)], 1u);
        atomicAdd(&h[wl][bucket_of<NB>(k.z, kbits)], 1u);
        atomicAdd(&h[wl][bucket_of<NB>(k.w, kbits)], 1u);
    }
    __builtin_amdgcn_wave_barrier();
    for (int b = lane; b < NB; b += 64) cnt[int64_t(b) * W + w] = h[wl][b];
}

// exclusive scan of m words in place, one workgroup
__global__ __launch_bounds__(1024) void scan(uint32_t* v, int m) {
    __shared__ uint32_t part[1024];
    const int per = (m + 1023) / 1024;
    const int lo = threadIdx.x * per, hi = lo + per < m ? lo + per : m;
    uint32_t s = 0;
    for (int i = lo; i < hi; ++i) s += v[i];
    part[threadIdx.x] = s;
    __syncthreads();
    for (int o = 1; o < 1024; o <<= 1) {
        const uint32_t x = threadIdx.x >= o ? part[threadIdx.x - o] : 0;
        __syncthreads();
        part[threadIdx.x] += x;
        __syncthreads();
    }
    uint32_t run = part[threadIdx.x] - s;
    for (int i = lo; i < hi; ++i) {
        const uint32_t x = v[i];
        v[i] = run;
        run += x;
    }
}

// Pass 1 (kScatter) and pass 3 (!kScatter) walk a wave's tile in the same
// order: (step, k, lane).  Pass 1 writes key to sorted[pos]; pass 3 reads
// res[pos] into out[i].
template <int NB, bool kScatter>
__global__ __launch_bounds__(kBlock) void place(const uint32_t* __restrict__ key, int kbits,
                                                int64_t n, int64_t S, int W,
                                                const uint32_t* __restrict__ off,
                                                uint32_t* __restrict__ sorted,
                                                const uint32_t* __restrict__ res,
                                                uint32_t* __restrict__ out) {
    __shared__ uint32_t base[kWaves][NB];
    const int wl = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int w = blockIdx.x * kWaves + wl;
    for (int b = lane; b < NB; b += 64) base[wl][b] = off[int64_t(b) * W + w];
    __builtin_amdgcn_wave_barrier();
    const int64_t lo = int64_t(w) * S, hi = lo + S < n ? lo + S : n;
    for (int64_t i = lo + 4 * lane; i < hi; i += 256) {
        const uint4 k4 = ntl(reinterpret_cast<const uint4*>(key + i));
        const uint32_t kk[4] = {k4.x, k4.y, k4.z, k4.w};
        uint32_t pos[4];
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const uint32_t b = bucket_of<NB>(kk[q], kbits);
            const uint64_t m = same_bucket<NB>(b);
            const uint32_t r = lanes_below(m);
            pos[q] = base[wl][b] + r;
            __builtin_amdgcn_wave_barrier();
            if (r == 0) base[wl][b] += uint32_t(__builtin_popcountll(m));
            __builtin_amdgcn_wave_barrier();
        }
        if (kScatter) {
#pragma unroll
            for (int q = 0; q < 4; ++q) sorted[pos[q]] = kk[q];
        } else {
            const uint4 v = make_uint4(res[pos[0]], res[pos[1]], res[pos[2]], res[pos[3]]);
            nts(reinterpret_cast<uint4*>(out + i), v);
        }
    }
}

// Pass 2: the chip sweeps the sorted keys in 4096-key chunks, chunk c on
// workgroup c % G, so the workgroups stay within a bucket or two.
__global__ __launch_bounds__(1024) void lookup(const uint32_t* __restrict__ sorted, int64_t n4,
                                               int shift, const uint32_t* __restrict__ t,
                                               uint32_t* __restrict__ res) {
    for (int64_t g = blockIdx.x * int64_t(blockDim.x) + threadIdx.x; g < n4;
         g += int64_t(gridDim.x) * blockDim.x) {
        const uint4 k = ntl(reinterpret_cast<const uint4*>(sorted) + g);
        const uint4 r = make_uint4(t[k.x >> shift], t[k.y >> shift], t[k.z >> shift], t[k.w >> shift]);
        nts(reinterpret_cast<uint4*>(res) + g, r);
    }
}

struct Timer {
    hipEvent_t a, b;
    Timer() { CK(hipEventCreate(&a)); CK(hipEventCreate(&b)); }
    void start() { CK(hipEventRecord(a)); }
    float stop() {
        CK(hipEventRecord(b));
        CK(hipEventSynchronize(b));
        float ms;
        CK(hipEventElapsedTime(&ms, a, b));
        return ms;
    }
};

template <int NB>
void run_partitioned(const char* tag, uint32_t* d, uint32_t* h, uint32_t* tr, uint32_t* tg,
                     int64_t n, int G, uint32_t* orr, uint32_t* og, const uint32_t* ref_r,
                     const uint32_t* ref_g, int reps, int lookup_grid) {
    const int W = G * kWaves;
    const int64_t S = ((n + W - 1) / W + 255) / 256 * 256;
    uint32_t *cr, *cg, *sr, *sg, *rr, *rg;
    CK(hipMalloc(&cr, size_t(NB) * W * 4));
    CK(hipMalloc(&cg, size_t(NB) * W * 4));
    CK(hipMalloc(&sr, n * 4));
    CK(hipMalloc(&sg, n * 4));
    CK(hipMalloc(&rr, n * 4));
    CK(hipMalloc(&rg, n * 4));
    Timer T;
    float best[6] = {1e9, 1e9, 1e9, 1e9, 1e9, 1e9};
    for (int rep = 0; rep < reps; ++rep) {
        float t[6];
        T.start();
        hist<NB><<<G, kBlock>>>(d, 32, n, S, W, cr);
        hist<NB><<<G, kBlock>>>(h, 24, n, S, W, cg);
        t[0] = T.stop();
        T.start();
        scan<<<1, 1024>>>(cr, NB * W);
        scan<<<1, 1024>>>(cg, NB * W);
        t[1] = T.stop();
        T.start();
        place<NB, true><<<G, kBlock>>>(d, 32, n, S, W, cr, sr, nullptr, nullptr);
        place<NB, true><<<G, kBlock>>>(h, 24, n, S, W, cg, sg, nullptr, nullptr);
        t[2] = T.stop();
        T.start();
        lookup<<<lookup_grid, 1024>>>(sr, n / 4, 8, tr, rr);
        lookup<<<lookup_grid, 1024>>>(sg, n / 4, 0, tg, rg);
        t[3] = T.stop();
        T.start();
        place<NB, false><<<G, kBlock>>>(d, 32, n, S, W, cr, nullptr, rr, orr);
        place<NB, false><<<G, kBlock>>>(h, 24, n, S, W, cg, nullptr, rg, og);
        t[4] = T.stop();
        t[5] = t[0] + t[1] + t[2] + t[3] + t[4];
        for (int j = 0; j < 6; ++j) best[j] = t[j] < best[j] ? t[j] : best[j];
    }
    CK(hipDeviceSynchronize());
    std::vector<uint32_t> a(n), b(n);
    CK(hipMemcpy(a.data(), orr, n * 4, hipMemcpyDeviceToHost));
    CK(hipMemcpy(b.data(), ref_r, n * 4, hipMemcpyDeviceToHost));
    int64_t bad = 0;
    for (int64_t i = 0; i < n; ++i) bad += a[i] != b[i];
    CK(hipMemcpy(a.data(), og, n * 4, hipMemcpyDeviceToHost));
    CK(hipMemcpy(b.data(), ref_g, n * 4, hipMemcpyDeviceToHost));
    for (int64_t i = 0; i < n; ++i) bad += a[i] != b[i];
    printf("{\"form\": \"%s\", \"NB\": %d, \"G\": %d, \"lookup_grid\": %d, \"hist_ms\": %.4f, "
           "\"scan_ms\": %.4f, \"scatter_ms\": %.4f, \"lookup_ms\": %.4f, \"gather_back_ms\": %.4f, "
           "\"total_ms\": %.4f, \"mismatches\": %lld}\n",
           tag, NB, G, lookup_grid, best[0], best[1], best[2], best[3], best[4], best[5],
           (long long)bad);
    fflush(stdout);
    CK(hipFree(cr)); CK(hipFree(cg)); CK(hipFree(sr)); CK(hipFree(sg));
    CK(hipFree(rr)); CK(hipFree(rg));
}

int main(int argc, char** argv) {
    const int64_t n = 124999936;        // 125M rounded down to 256
    const int64_t tn = int64_t(1) << 24;
    const int reps = argc > 1 ? atoi(argv[1]) : 5;
    uint32_t *d, *h, *tr, *tg, *r0, *g0, *r1, *g1;
    CK(hipMalloc(&d, n * 4)); CK(hipMalloc(&h, n * 4));
    CK(hipMalloc(&tr, tn * 4)); CK(hipMalloc(&tg, tn * 4));
    CK(hipMalloc(&r0, n * 4)); CK(hipMalloc(&g0, n * 4));
    CK(hipMalloc(&r1, n * 4)); CK(hipMalloc(&g1, n * 4));
    fill<<<4096, 256>>>(d, h, tr, tg, n, tn);
    CK(hipDeviceSynchronize());
    Timer T;
    float best = 1e9;
    for (int rep = 0; rep < reps; ++rep) {
        T.start();
        direct<<<1024, 1024>>>(d, h, tr, tg, n / 4, r0, g0);
        const float ms = T.stop();
        best = ms < best ? ms : best;
    }
    printf("{\"form\": \"direct\", \"total_ms\": %.4f}\n", best);
    fflush(stdout);
    // (NB, workgroups of passes 0/1/3, workgroups of the lookup sweep)
    run_partitioned<32>("partitioned", d, h, tr, tg, n, 512, r1, g1, r0, g0, reps, 1024);
    run_partitioned<32>("partitioned", d, h, tr, tg, n, 1024, r1, g1, r0, g0, reps, 256);
    run_partitioned<32>("partitioned", d, h, tr, tg, n, 1024, r1, g1, r0, g0, reps, 128);
    run_partitioned<64>("partitioned", d, h, tr, tg, n, 512, r1, g1, r0, g0, reps, 1024);
    run_partitioned<64>("partitioned", d, h, tr, tg, n, 1024, r1, g1, r0, g0, reps, 256);
    run_partitioned<64>("partitioned", d, h, tr, tg, n, 256, r1, g1, r0, g0, reps, 256);
    run_partitioned<128>("partitioned", d, h, tr, tg, n, 512, r1, g1, r0, g0, reps, 1024);
    run_partitioned<128>("partitioned", d, h, tr, tg, n, 1024, r1, g1, r0, g0, reps, 256);
    return 0;
}
