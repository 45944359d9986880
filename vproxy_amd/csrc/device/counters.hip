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

}  // namespace vcd

namespace vc {

hipError_t launch_hist(const LaunchCfg& c, int mode, const int32_t* idx, const uint8_t* aux,
                       int64_t n, int64_t nval, int64_t base, int64_t null_bin, int32_t nt,
                       unsigned long long* counters) {
    if (n <= 0 || !counters) return hipSuccess;
    const int64_t chunks = nval > 0 ? (nval + vcd::kHistBins - 1) / vcd::kHistBins : 1;
    int64_t slices = (int64_t(c.num_cus) * 2 + chunks - 1) / chunks;
    const int64_t max_slices = (n + 65535) / 65536;     // >= 64K items per workgroup
    if (slices > max_slices) slices = max_slices;
    if (slices < 1) slices = 1;
    hipLaunchKernelGGL(vcd::hist_kernel, dim3(unsigned(slices), unsigned(chunks)),
                       dim3(vcd::kHistBlock), 0, c.stream, mode, idx, aux, n, nval, base,
                       null_bin, nt, counters);
    return hipGetLastError();
}

}  // namespace vc
