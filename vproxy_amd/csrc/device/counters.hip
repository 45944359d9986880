// counters.hip -- per-rule hit counters from a classify launch's outputs.
//
// Counting with one device atomic per item is memory-side and serialises on
// hot bins: a wildcard group or default route taking 20 % of a batch ran at
// 0.4 G adds/s on MI355X (tools/atomics_probe.hip), 60x slower than the
// classify kernel itself.  Instead each workgroup histograms a slice of the
// output array in LDS (hot bins cost LDS atomics only), one 32K-bin chunk of
// the counter space per grid row, then flushes its non-zero bins with
// consecutive-lane (coalesced) device atomics into the uint64 counters.
#include "dev_common.h"
#include "launch.h"

namespace vcd {

constexpr int kHistBins = 32768;   // 128 KiB of LDS per workgroup
constexpr int kHistBlock = 1024;

// bin of item i in the chunked value space [0, nval); -1 = the null bin
__device__ __forceinline__ int64_t hist_value(int mode, const int32_t* idx, const uint8_t* aux,
                                              int64_t i, int32_t nt, bool* tcp_null) {
    const int32_t v = idx[i];
    *tcp_null = false;
    if (mode == VC_HIST_ACL) {
        const bool tcp = aux[i] == VC_PROTO_TCP;
        if (v < 0) {
            *tcp_null = tcp;
            return -1;
        }
        return tcp ? int64_t(v) : int64_t(nt) + v;
    }
    if (mode == VC_HIST_DNS && aux[i] != VC_DNS_GROUP) return -1;
    return v;
}

__global__ __launch_bounds__(kHistBlock) void hist_kernel(
    int mode, const int32_t* __restrict__ idx, const uint8_t* __restrict__ aux, int64_t n,
    int64_t nval, int64_t base, int64_t null_bin, int32_t nt, unsigned long long* __restrict__ cnt) {
    __shared__ uint32_t h[kHistBins];
    __shared__ uint32_t nulls[2];
    const int64_t lo_bin = int64_t(blockIdx.y) * kHistBins;
    for (int k = threadIdx.x; k < kHistBins; k += blockDim.x) h[k] = 0;
    if (threadIdx.x < 2) nulls[threadIdx.x] = 0;
    __syncthreads();
    const int64_t per = (n + gridDim.x - 1) / gridDim.x;
    const int64_t lo = int64_t(blockIdx.x) * per;
    const int64_t hi = lo + per < n ? lo + per : n;
    const bool count_nulls = blockIdx.y == 0;
    uint32_t my_null[2] = {0, 0};
    for (int64_t i = lo + threadIdx.x; i < hi; i += blockDim.x) {
        bool tcp_null;
        const int64_t v = hist_value(mode, idx, aux, i, nt, &tcp_null);
        if (v < 0) {
            my_null[tcp_null ? 0 : 1] += count_nulls;
        } else {
            const uint64_t d = uint64_t(v - lo_bin);
            if (d < uint64_t(kHistBins)) atomicAdd(&h[d], 1u);
        }
    }
    if (count_nulls) {
        if (my_null[0]) atomicAdd(&nulls[0], my_null[0]);
        if (my_null[1]) atomicAdd(&nulls[1], my_null[1]);
    }
    __syncthreads();
    for (int k = threadIdx.x; k < kHistBins && lo_bin + k < nval; k += blockDim.x)
        if (h[k]) atomicAdd(cnt + base + lo_bin + k, (unsigned long long)h[k]);
    if (count_nulls && threadIdx.x == 0) {
        // ACL: [tcp default, udp default] at null_bin, null_bin + 1
        if (mode == VC_HIST_ACL) {
            if (nulls[0]) atomicAdd(cnt + null_bin, (unsigned long long)nulls[0]);
            if (nulls[1]) atomicAdd(cnt + null_bin + 1, (unsigned long long)nulls[1]);
        } else if (nulls[1]) {
            atomicAdd(cnt + null_bin, (unsigned long long)nulls[1]);
        }
    }
}

// ---- bucketed path for large counter spaces (route tables) ----------------
// Items are first partitioned by 32K-bin chunk ("bucket") with a per-block
// count / scan / scatter, so each chunk's histogram then reads only its own
// items: ~4 passes over the outputs instead of one pass per chunk.
constexpr int kMaxBuckets = 4096;

__global__ __launch_bounds__(kHistBlock) void bucket_count_kernel(
    int mode, const int32_t* __restrict__ idx, const uint8_t* __restrict__ aux, int64_t n,
    int32_t nt, int nbk, uint32_t* __restrict__ counts, unsigned long long* __restrict__ cnt,
    int64_t null_bin) {
    __shared__ uint32_t c[kMaxBuckets];
    __shared__ uint32_t nulls[2];
    for (int k = threadIdx.x; k < nbk; k += blockDim.x) c[k] = 0;
    if (threadIdx.x < 2) nulls[threadIdx.x] = 0;
    __syncthreads();
    const int64_t per = (n + gridDim.x - 1) / gridDim.x;
    const int64_t lo = int64_t(blockIdx.x) * per;
    const int64_t hi = lo + per < n ? lo + per : n;
    uint32_t my_null[2] = {0, 0};
    for (int64_t i = lo + threadIdx.x; i < hi; i += blockDim.x) {
        bool tcp_null;
        const int64_t v = hist_value(mode, idx, aux, i, nt, &tcp_null);
        if (v < 0) my_null[tcp_null ? 0 : 1]++;
        else atomicAdd(&c[v / kHistBins], 1u);
    }
    if (my_null[0]) atomicAdd(&nulls[0], my_null[0]);
    if (my_null[1]) atomicAdd(&nulls[1], my_null[1]);
    __syncthreads();
    for (int k = threadIdx.x; k < nbk; k += blockDim.x) counts[int64_t(k) * gridDim.x + blockIdx.x] = c[k];
    if (threadIdx.x == 0) {
        if (mode == VC_HIST_ACL) {
            if (nulls[0]) atomicAdd(cnt + null_bin, (unsigned long long)nulls[0]);
            if (nulls[1]) atomicAdd(cnt + null_bin + 1, (unsigned long long)nulls[1]);
        } else if (nulls[1]) {
            atomicAdd(cnt + null_bin, (unsigned long long)nulls[1]);
        }
    }
}

// exclusive scan of counts (bucket-major, m entries) -> offsets; one block
__global__ __launch_bounds__(kHistBlock) void bucket_scan_kernel(const uint32_t* __restrict__ counts,
                                                                 uint32_t* __restrict__ offsets,
                                                                 int64_t m) {
    __shared__ uint32_t part[kHistBlock];
    __shared__ uint32_t carry;
    if (threadIdx.x == 0) carry = 0;
    __syncthreads();
    for (int64_t base = 0; base < m; base += kHistBlock) {
        const int64_t i = base + threadIdx.x;
        const uint32_t v = i < m ? counts[i] : 0;
        part[threadIdx.x] = v;
        __syncthreads();
        for (int off = 1; off < kHistBlock; off <<= 1) {      // Hillis-Steele inclusive scan
            const uint32_t t = int(threadIdx.x) >= off ? part[threadIdx.x - off] : 0;
            __syncthreads();
            part[threadIdx.x] += t;
            __syncthreads();
        }
        if (i < m) offsets[i] = carry + part[threadIdx.x] - v;
        __syncthreads();
        if (threadIdx.x == kHistBlock - 1) carry += part[kHistBlock - 1];
        __syncthreads();
    }
    if (threadIdx.x == 0) offsets[m] = carry;     // grand total: end of the last bucket
}

__global__ __launch_bounds__(kHistBlock) void bucket_scatter_kernel(
    int mode, const int32_t* __restrict__ idx, const uint8_t* __restrict__ aux, int64_t n,
    int32_t nt, int nbk, const uint32_t* __restrict__ offsets, int32_t* __restrict__ tmp) {
    __shared__ uint32_t cur[kMaxBuckets];
    for (int k = threadIdx.x; k < nbk; k += blockDim.x)
        cur[k] = offsets[int64_t(k) * gridDim.x + blockIdx.x];
    __syncthreads();
    const int64_t per = (n + gridDim.x - 1) / gridDim.x;
    const int64_t lo = int64_t(blockIdx.x) * per;
    const int64_t hi = lo + per < n ? lo + per : n;
    for (int64_t i = lo + threadIdx.x; i < hi; i += blockDim.x) {
        bool tcp_null;
        const int64_t v = hist_value(mode, idx, aux, i, nt, &tcp_null);
        if (v >= 0) tmp[atomicAdd(&cur[v / kHistBins], 1u)] = int32_t(v);
    }
}

// grid (slices, buckets): histogram bucket b's items in LDS, flush
__global__ __launch_bounds__(kHistBlock) void bucket_hist_kernel(
    const int32_t* __restrict__ tmp, const uint32_t* __restrict__ offsets, int nblk, int nbk,
    int64_t nval, int64_t base, unsigned long long* __restrict__ cnt) {
    __shared__ uint32_t h[kHistBins];
    const int b = blockIdx.y;
    const uint32_t s0 = offsets[int64_t(b) * nblk];
    const uint32_t s1 = offsets[int64_t(b + 1) * nblk];   // offsets[nbk * nblk] = total
    for (int k = threadIdx.x; k < kHistBins; k += blockDim.x) h[k] = 0;
    __syncthreads();
    const uint32_t len = s1 - s0;
    const uint32_t per = (len + gridDim.x - 1) / gridDim.x;
    const uint32_t lo = s0 + blockIdx.x * per;
    const uint32_t hi = lo + per < s1 ? lo + per : s1;
    const int64_t lo_bin = int64_t(b) * kHistBins;
    for (uint32_t i = lo + threadIdx.x; i < hi; i += blockDim.x)
        atomicAdd(&h[tmp[i] - lo_bin], 1u);
    __syncthreads();
    for (int k = threadIdx.x; k < kHistBins && lo_bin + k < nval; k += blockDim.x)
        if (h[k]) atomicAdd(cnt + base + lo_bin + k, (unsigned long long)h[k]);
}

}  // namespace vcd

namespace vc {

hipError_t launch_hist(const LaunchCfg& c, int mode, const int32_t* idx, const uint8_t* aux,
                       int64_t n, int64_t nval, int64_t base, int64_t null_bin, int32_t nt,
                       unsigned long long* counters) {
    if (n <= 0 || !counters) return hipSuccess;
    const int64_t chunks = nval > 0 ? (nval + vcd::kHistBins - 1) / vcd::kHistBins : 1;
    if (chunks <= 2 || chunks > vcd::kMaxBuckets || n >= (int64_t(1) << 32)) {
        // small counter space: one pass per chunk over the outputs
        int64_t slices = (int64_t(c.num_cus) * 2 + chunks - 1) / chunks;
        const int64_t max_slices = (n + 65535) / 65536;     // >= 64K items per workgroup
        if (slices > max_slices) slices = max_slices;
        if (slices < 1) slices = 1;
        hipLaunchKernelGGL(vcd::hist_kernel, dim3(unsigned(slices), unsigned(chunks)),
                           dim3(vcd::kHistBlock), 0, c.stream, mode, idx, aux, n, nval, base,
                           null_bin, nt, counters);
        return hipGetLastError();
    }
    // large counter space: partition by chunk first (count, scan, scatter)
    const int nbk = int(chunks);
    int nblk = c.num_cus * 2;
    const int64_t max_blk = (n + 16383) / 16384;
    if (nblk > max_blk) nblk = int(max_blk < 1 ? 1 : max_blk);
    const int64_t m = int64_t(nbk) * nblk;
    uint32_t *counts = nullptr, *offsets = nullptr;
    int32_t* tmp = nullptr;
    hipError_t e = hipMallocAsync(reinterpret_cast<void**>(&counts), size_t(m) * 4, c.stream);
    if (e == hipSuccess)
        e = hipMallocAsync(reinterpret_cast<void**>(&offsets), size_t(m + 1) * 4, c.stream);
    if (e == hipSuccess) e = hipMallocAsync(reinterpret_cast<void**>(&tmp), size_t(n) * 4, c.stream);
    if (e == hipSuccess) {
        hipLaunchKernelGGL(vcd::bucket_count_kernel, dim3(nblk), dim3(vcd::kHistBlock), 0,
                           c.stream, mode, idx, aux, n, nt, nbk, counts, counters, null_bin);
        hipLaunchKernelGGL(vcd::bucket_scan_kernel, dim3(1), dim3(vcd::kHistBlock), 0, c.stream,
                           counts, offsets, m);
        hipLaunchKernelGGL(vcd::bucket_scatter_kernel, dim3(nblk), dim3(vcd::kHistBlock), 0,
                           c.stream, mode, idx, aux, n, nt, nbk, offsets, tmp);
        int64_t per_bucket = (n / nbk + 65535) / 65536;
        int slices = int(per_bucket < 1 ? 1 : (per_bucket > 64 ? 64 : per_bucket));
        if (slices * nbk < c.num_cus) slices = (c.num_cus + nbk - 1) / nbk;
        hipLaunchKernelGGL(vcd::bucket_hist_kernel, dim3(slices, nbk), dim3(vcd::kHistBlock), 0,
                           c.stream, tmp, offsets, nblk, nbk, nval, base, counters);
        e = hipGetLastError();
    }
    if (counts) (void)hipFreeAsync(counts, c.stream);
    if (offsets) (void)hipFreeAsync(offsets, c.stream);
    if (tmp) (void)hipFreeAsync(tmp, c.stream);
    return e;
}

}  // namespace vc
