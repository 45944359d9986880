// counters.hip -- per-rule hit counters from a classify launch's outputs.
//
// Counting with one device atomic per item is memory-side and serialises on
// hot bins: a wildcard group or default route taking 20 % of a batch ran at
// 0.4 G adds/s on MI355X (tools/atomics_probe.hip), 60x slower than the
// classify kernel itself.  So counts are built in LDS and flushed once per
// workgroup with consecutive-lane (coalesced) device atomics:
//
// * small counter spaces (<= 64K bins: ACL rules): every workgroup
//   histograms a contiguous slice of the outputs into a 32K-bin LDS
//   histogram per grid row, 4 items per lane per 16-byte load;
// * large spaces (routes: ~1.2M bins; groups: 100K) are first partitioned
//   into 8K-bin buckets -- count, scan, then a scatter that sorts each
//   8K-item tile by bucket in LDS so the bucket runs leave as contiguous
//   stores of 16-bit in-bucket bins -- and each bucket is then histogrammed in LDS by segments of at
//   most kSeg items (a hot bucket is split over many workgroups).
//
// Null results (no rule / default) are counted in registers and added once
// per workgroup; a thread collapses runs of equal values before touching
// LDS, which keeps hot bins off a single LDS address.
#include <vector>

#include "dev_common.h"
#include "launch.h"

namespace vcd {

constexpr int kHistBlock = 1024;
constexpr int kHistBins = 32768;      // small path: 128 KiB of LDS per workgroup
constexpr int kBW = 8192;             // large path: bins per bucket (32 KiB of LDS)
constexpr int kMaxBuckets = 4096;
constexpr int kTile = 32768;          // scatter tile: items sorted by bucket in LDS (128 KiB)
constexpr uint32_t kSeg = 256 * 1024; // max items per histogram segment

// Item i -> bin in [0, nval), or -1 for a null result (*udp_or_plain_null
// tells the ACL's two default bins apart).
struct Item {
    int64_t v;
    bool tcp_null;
};

__device__ __forceinline__ Item item_of(int mode, int32_t v, uint8_t a, int32_t nt) {
    if (mode == VC_HIST_ACL) {
        const bool tcp = a == VC_PROTO_TCP;
        if (v < 0) return Item{-1, tcp};
        return Item{tcp ? int64_t(v) : int64_t(nt) + v, false};
    }
    if (mode == VC_HIST_ROUTE) {                 // aux = family; v6 rules follow the nt v4 rules
        const bool v4 = a != 6;
        if (v < 0) return Item{-1, v4};
        return Item{v4 ? int64_t(v) : int64_t(nt) + v, false};
    }
    if (mode == VC_HIST_DNS && a != VC_DNS_GROUP) return Item{-2, false};   // not counted
    return Item{v < 0 ? -1 : int64_t(v), false};
}

// 4 consecutive items starting at i (i % 4 == 0, i + 3 < n) with one 16-byte
// load of the outputs (and one 4-byte load of aux).
__device__ __forceinline__ void load4(int mode, const int32_t* idx, const uint8_t* aux, int64_t i,
                                      int32_t nt, Item it[4]) {
    const int4 v = *reinterpret_cast<const int4*>(idx + i);
    const uint32_t a = aux ? *reinterpret_cast<const uint32_t*>(aux + i) : 0u;
    it[0] = item_of(mode, v.x, a & 255u, nt);
    it[1] = item_of(mode, v.y, (a >> 8) & 255u, nt);
    it[2] = item_of(mode, v.z, (a >> 16) & 255u, nt);
    it[3] = item_of(mode, v.w, a >> 24, nt);
}

__device__ __forceinline__ Item load1(int mode, const int32_t* idx, const uint8_t* aux, int64_t i,
                                      int32_t nt) {
    return item_of(mode, idx[i], aux ? aux[i] : 0, nt);
}

// Adds n (>0) to LDS bin b.
__device__ __forceinline__ void lds_add(uint32_t* h, int64_t b, uint32_t c) {
    if (c) atomicAdd(&h[b], c);
}

// Per-thread run-length collapse in front of LDS atomics.
struct Run {
    int64_t v = -1;
    uint32_t c = 0;
    __device__ __forceinline__ void add(int64_t x, uint32_t* h, int64_t lo, int64_t width) {
        if (x == v) {
            ++c;
            return;
        }
        if (c && uint64_t(v - lo) < uint64_t(width)) atomicAdd(&h[v - lo], c);
        v = x;
        c = 1;
    }
    __device__ __forceinline__ void flush(uint32_t* h, int64_t lo, int64_t width) {
        if (c && uint64_t(v - lo) < uint64_t(width)) atomicAdd(&h[v - lo], c);
        c = 0;
    }
};

__device__ __forceinline__ void flush_nulls(int mode, uint32_t n_tcp, uint32_t n_other,
                                            int64_t null_bin, unsigned long long* cnt) {
    // ACL: [tcp default, udp default] at null_bin, null_bin + 1; ROUTE:
    // [v4 null, v6 null] there (n_tcp counts the first bin's nulls)
    __shared__ uint32_t nulls[2];
    if (threadIdx.x < 2) nulls[threadIdx.x] = 0;
    __syncthreads();
    if (n_tcp) atomicAdd(&nulls[0], n_tcp);
    if (n_other) atomicAdd(&nulls[1], n_other);
    __syncthreads();
    if (threadIdx.x == 0) {
        if (mode == VC_HIST_ACL || mode == VC_HIST_ROUTE) {
            if (nulls[0]) atomicAdd(cnt + null_bin, (unsigned long long)nulls[0]);
            if (nulls[1]) atomicAdd(cnt + null_bin + 1, (unsigned long long)nulls[1]);
        } else if (nulls[1]) {
            atomicAdd(cnt + null_bin, (unsigned long long)nulls[1]);
        }
    }
}

__device__ __forceinline__ void count_null(const Item& it, uint32_t* nt, uint32_t* no) {
    if (it.v == -1) {
        if (it.tcp_null) ++*nt;
        else ++*no;
    }
}

// Contiguous slice [lo, hi) of n items owned by this workgroup, split on
// 4-item boundaries.
__device__ __forceinline__ void slice_of(int64_t n, int64_t* lo, int64_t* hi) {
    const int64_t groups = (n + 3) >> 2;
    const int64_t per = (groups + gridDim.x - 1) / gridDim.x;
    *lo = int64_t(blockIdx.x) * per * 4;
    const int64_t h = *lo + per * 4;
    *hi = h < n ? h : n;
    if (*lo > n) *lo = n;
}

// ---- small counter spaces --------------------------------------------------
template <bool kVec>
__global__ __launch_bounds__(kHistBlock) void hist_kernel(
    int mode, const int32_t* __restrict__ idx, const uint8_t* __restrict__ aux, int64_t n,
    int64_t nval, int64_t base, int64_t null_bin, int32_t nt, unsigned long long* __restrict__ cnt) {
    extern __shared__ uint32_t h[];            // `width` words: one chunk of the counter space
    const int width = nval < kHistBins ? int(nval < 1 ? 1 : nval) : kHistBins;
    const int64_t lo_bin = int64_t(blockIdx.y) * kHistBins;
    for (int k = threadIdx.x; k < width; k += blockDim.x) h[k] = 0;
    __syncthreads();
    int64_t lo, hi;
    slice_of(n, &lo, &hi);
    uint32_t ntc = 0, noth = 0;
    Run run;
    if (kVec) {
        for (int64_t i = lo + 4 * threadIdx.x; i < hi; i += 4 * blockDim.x) {
            Item it[4];
            if (i + 3 < n) {
                load4(mode, idx, aux, i, nt, it);
            } else {
                for (int k = 0; k < 4; ++k) it[k] = i + k < n ? load1(mode, idx, aux, i + k, nt)
                                                               : Item{-2, false};
            }
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                count_null(it[k], &ntc, &noth);
                if (it[k].v >= 0) run.add(it[k].v, h, lo_bin, width);
            }
        }
    } else {
        for (int64_t i = lo + threadIdx.x; i < hi; i += blockDim.x) {
            const Item it = load1(mode, idx, aux, i, nt);
            count_null(it, &ntc, &noth);
            if (it.v >= 0) run.add(it.v, h, lo_bin, width);
        }
    }
    run.flush(h, lo_bin, width);
    if (blockIdx.y != 0) ntc = noth = 0;      // nulls counted by grid row 0 only
    flush_nulls(mode, ntc, noth, null_bin, cnt);
    for (int k = threadIdx.x; k < width && lo_bin + k < nval; k += blockDim.x)
        if (h[k]) atomicAdd(cnt + base + lo_bin + k, (unsigned long long)h[k]);
}

// ---- large counter spaces --------------------------------------------------
// (1) per-workgroup bucket counts: counts[b * nblk + blk]
template <bool kVec>
__global__ __launch_bounds__(kHistBlock) void bucket_count_kernel(
    int mode, const int32_t* __restrict__ idx, const uint8_t* __restrict__ aux, int64_t n,
    int32_t nt, int nbk, int64_t nval, uint32_t* __restrict__ counts,
    unsigned long long* __restrict__ cnt, int64_t null_bin) {
    extern __shared__ uint32_t c[];            // nbk words
    for (int k = threadIdx.x; k < nbk; k += blockDim.x) c[k] = 0;
    __syncthreads();
    int64_t lo, hi;
    slice_of(n, &lo, &hi);
    uint32_t ntc = 0, noth = 0;
    Run run;
    const int64_t step = (kVec ? 4 : 1) * int64_t(blockDim.x);
    for (int64_t i = lo + (kVec ? 4 : 1) * threadIdx.x; i < hi; i += step) {
        Item it[4];
        int m = 1;
        if (kVec && i + 3 < n) {
            load4(mode, idx, aux, i, nt, it);
            m = 4;
        } else if (kVec) {
            for (int k = 0; k < 4; ++k) it[k] = i + k < n ? load1(mode, idx, aux, i + k, nt)
                                                           : Item{-2, false};
            m = 4;
        } else {
            it[0] = load1(mode, idx, aux, i, nt);
        }
        for (int k = 0; k < m; ++k) {
            count_null(it[k], &ntc, &noth);
            if (it[k].v >= 0 && it[k].v < nval) run.add(it[k].v / kBW, c, 0, nbk);
        }
    }
    run.flush(c, 0, nbk);
    flush_nulls(mode, ntc, noth, null_bin, cnt);
    for (int k = threadIdx.x; k < nbk; k += blockDim.x)
        counts[int64_t(k) * gridDim.x + blockIdx.x] = c[k];
}

// Exclusive prefix sum over one wave's 64 lanes (no LDS, no barrier).
__device__ __forceinline__ uint32_t wave_scan_excl(uint32_t v, uint32_t* total) {
    const int lane = int(threadIdx.x & 63);
    uint32_t x = v;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        const uint32_t y = __shfl_up(x, d, 64);
        if (lane >= d) x += y;
    }
    *total = __shfl(x, 63, 64);
    return x - v;
}

// (2) one workgroup: exclusive scan of counts (bucket-major, m entries) ->
// offsets[0..m]; then the segment table seg_off[0..nbk] (segments of at
// most kSeg items per bucket, prefix-summed).
__device__ __forceinline__ uint32_t block_scan_excl(uint32_t v, uint32_t* part, uint32_t* total) {
    part[threadIdx.x] = v;
    __syncthreads();
    for (int off = 1; off < kHistBlock; off <<= 1) {      // Hillis-Steele inclusive scan
        const uint32_t t = int(threadIdx.x) >= off ? part[threadIdx.x - off] : 0;
        __syncthreads();
        part[threadIdx.x] += t;
        __syncthreads();
    }
    const uint32_t incl = part[threadIdx.x];
    *total = part[kHistBlock - 1];
    __syncthreads();
    return incl - v;
}

__global__ __launch_bounds__(kHistBlock) void bucket_scan_kernel(
    const uint32_t* __restrict__ counts, uint32_t* __restrict__ offsets, int64_t m, int nbk,
    int nblk, uint32_t* __restrict__ seg_off) {
    __shared__ uint32_t part[kHistBlock];
    // each thread scans a contiguous run of the m entries
    const int64_t per = (m + kHistBlock - 1) / kHistBlock;
    const int64_t a = int64_t(threadIdx.x) * per;
    const int64_t b = a + per < m ? a + per : m;
    uint32_t sum = 0;
    for (int64_t i = a; i < b; ++i) sum += counts[i];
    uint32_t total;
    uint32_t run = block_scan_excl(sum, part, &total);
    for (int64_t i = a; i < b; ++i) {
        const uint32_t v = counts[i];
        offsets[i] = run;
        run += v;
    }
    if (threadIdx.x == 0) offsets[m] = total;
    __syncthreads();
    __threadfence_block();
    // segment table over buckets (nbk <= kMaxBuckets = 4 * kHistBlock)
    uint32_t segs[4];
    uint32_t mine = 0;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        const int bk = threadIdx.x * 4 + k;
        uint32_t s = 0;
        if (bk < nbk) {
            const uint32_t len = offsets[int64_t(bk + 1) * nblk] - offsets[int64_t(bk) * nblk];
            s = (len + kSeg - 1) / kSeg;
        }
        segs[k] = s;
        mine += s;
    }
    uint32_t st = block_scan_excl(mine, part, &total);
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        const int bk = threadIdx.x * 4 + k;
        if (bk < nbk) seg_off[bk] = st;
        st += segs[k];
    }
    if (threadIdx.x == 0) seg_off[nbk] = total;
}

// (3) scatter each workgroup's slice into bucket-contiguous order, a tile of
// kTile items at a time sorted by bucket in LDS, so bucket runs are written
// with consecutive lanes.  The 32K-item tile (128 KiB of LDS) runs as fast
// alone as 8K ones, but in the C5 schedule, where the next hostname-pool
// pass runs beside this finish, a scatter workgroup then never shares its
// CU with pool-pass workgroups: the pool pass takes 1.12 instead of 1.40 ms
// and the step 6.29 instead of 6.42 ms (profiles/r02_ab_scatter_tile.txt).
template <bool kVec>
__global__ __launch_bounds__(kHistBlock) void bucket_scatter_kernel(
    int mode, const int32_t* __restrict__ idx, const uint8_t* __restrict__ aux, int64_t n,
    int32_t nt, int nbk, int64_t nval, const uint32_t* __restrict__ offsets,
    uint16_t* __restrict__ tmp) {
    // LDS sized by the bucket count, so the kernel can share a CU with the
    // classify kernels of the next batch
    extern __shared__ uint32_t dyn[];
    uint32_t* cur = dyn;                      // next global write position per bucket
    uint32_t* tcnt = dyn + nbk;               // this tile's count per bucket
    uint32_t* tst = dyn + 2 * nbk;            // this tile's exclusive start per bucket
    __shared__ int32_t sorted[kTile];
    __shared__ uint32_t part[kHistBlock];
    for (int k = threadIdx.x; k < nbk; k += blockDim.x) {
        cur[k] = offsets[int64_t(k) * gridDim.x + blockIdx.x];
        tcnt[k] = 0;
    }
    __syncthreads();
    int64_t lo, hi;
    slice_of(n, &lo, &hi);
    constexpr int kPer = kTile / kHistBlock;  // items per thread per tile
    for (int64_t t0 = lo; t0 < hi; t0 += kTile) {
        int32_t v[kPer];
        uint32_t r[kPer];
#pragma unroll
        for (int q = 0; q < kPer; q += 4) {
            const int64_t i = t0 + int64_t(q) * kHistBlock + 4 * threadIdx.x;
            Item it[4];
            if (kVec && i + 3 < hi) {
                load4(mode, idx, aux, i, nt, it);
            } else {
                for (int k = 0; k < 4; ++k) it[k] = i + k < hi ? load1(mode, idx, aux, i + k, nt)
                                                                : Item{-2, false};
            }
            // values at or past the counter space (a caller-supplied output
            // classified against another snapshot) are not counted -- the
            // bucket counts (bucket_count_kernel, or the pipeline kernel's
            // pipe_count) drop exactly the same values, so every bucket's run
            // has the length its offsets reserve
#pragma unroll
            for (int k = 0; k < 4; ++k)
                v[q + k] = it[k].v >= 0 && it[k].v < nval ? int32_t(it[k].v) : -1;
        }
#pragma unroll
        for (int q = 0; q < kPer; ++q)
            r[q] = v[q] >= 0 ? atomicAdd(&tcnt[v[q] / kBW], 1u) : 0u;
        __syncthreads();
        // exclusive scan of tcnt over the buckets, 4 per lane: one wave
        // when there are at most 256 buckets (every counter space of the
        // benchmark), else the whole workgroup
        uint32_t total;
        if (nbk <= 256) {
            if (threadIdx.x < 64) {
                uint32_t c4[4], s4 = 0;
#pragma unroll
                for (int k = 0; k < 4; ++k) {
                    const int bk = threadIdx.x * 4 + k;
                    c4[k] = bk < nbk ? tcnt[bk] : 0u;
                    s4 += c4[k];
                }
                uint32_t st = wave_scan_excl(s4, &total);
#pragma unroll
                for (int k = 0; k < 4; ++k) {
                    const int bk = threadIdx.x * 4 + k;
                    if (bk < nbk) tst[bk] = st;
                    st += c4[k];
                }
                if (threadIdx.x == 0) part[0] = total;
            }
            __syncthreads();
            total = part[0];
        } else {
            uint32_t c4[4], s4 = 0;
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                const int bk = threadIdx.x * 4 + k;
                c4[k] = bk < nbk ? tcnt[bk] : 0u;
                s4 += c4[k];
            }
            uint32_t st = block_scan_excl(s4, part, &total);
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                const int bk = threadIdx.x * 4 + k;
                if (bk < nbk) tst[bk] = st;
                st += c4[k];
            }
            __syncthreads();
        }
#pragma unroll
        for (int q = 0; q < kPer; ++q)
            if (v[q] >= 0) sorted[tst[v[q] / kBW] + r[q]] = v[q];
        __syncthreads();
        for (uint32_t j = threadIdx.x; j < total; j += blockDim.x) {
            const int32_t x = sorted[j];
            const int bk = x / kBW;
            tmp[cur[bk] + (j - tst[bk])] = uint16_t(x & (kBW - 1));   // bin within its bucket
        }
        __syncthreads();
        for (int k = threadIdx.x; k < nbk; k += blockDim.x) {
            cur[k] += tcnt[k];
            tcnt[k] = 0;
        }
        __syncthreads();
    }
}

// (4) one workgroup per segment of a bucket: LDS histogram, coalesced flush
__global__ __launch_bounds__(kHistBlock) void bucket_hist_kernel(
    const uint16_t* __restrict__ tmp, const uint32_t* __restrict__ offsets,
    const uint32_t* __restrict__ seg_off, int nblk, int nbk, int64_t nval, int64_t base,
    unsigned long long* __restrict__ cnt) {
    __shared__ uint32_t h[kBW];
    __shared__ int s_bucket;
    const uint32_t seg = blockIdx.x;
    if (seg >= seg_off[nbk]) return;                       // uniform per workgroup
    if (threadIdx.x == 0) {                                // last bucket with seg_off <= seg
        int a = 0, len = nbk + 1;
        while (len > 1) {
            const int half = len >> 1;
            a = seg_off[a + half] <= seg ? a + half : a;
            len -= half;
        }
        s_bucket = a;
    }
    for (int k = threadIdx.x; k < kBW; k += blockDim.x) h[k] = 0;
    __syncthreads();
    const int b = s_bucket;
    const uint32_t b0 = offsets[int64_t(b) * nblk], b1 = offsets[int64_t(b + 1) * nblk];
    const uint32_t s0 = b0 + (seg - seg_off[b]) * kSeg;
    const uint32_t s1 = s0 + kSeg < b1 ? s0 + kSeg : b1;
    const int64_t lo_bin = int64_t(b) * kBW;
    Run run;
    // 8 bins per lane per 16-byte load over the segment's aligned middle
    const uint32_t a0 = (s0 + 7) & ~7u, a1 = s1 & ~7u;
    if (a0 < a1) {
        for (uint32_t i = s0 + threadIdx.x; i < a0; i += blockDim.x)
            run.add(lo_bin + tmp[i], h, lo_bin, kBW);
        for (uint32_t i = a1 + threadIdx.x; i < s1; i += blockDim.x)
            run.add(lo_bin + tmp[i], h, lo_bin, kBW);
        const uint4* t8 = reinterpret_cast<const uint4*>(tmp);
        for (uint32_t c = (a0 >> 3) + threadIdx.x; c < (a1 >> 3); c += blockDim.x) {
            const uint4 w = t8[c];
            const uint32_t p[4] = {w.x, w.y, w.z, w.w};
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                run.add(lo_bin + (p[k] & 0xFFFFu), h, lo_bin, kBW);
                run.add(lo_bin + (p[k] >> 16), h, lo_bin, kBW);
            }
        }
    } else {
        for (uint32_t i = s0 + threadIdx.x; i < s1; i += blockDim.x)
            run.add(lo_bin + tmp[i], h, lo_bin, kBW);
    }
    run.flush(h, lo_bin, kBW);
    __syncthreads();
    for (int k = threadIdx.x; k < kBW && lo_bin + k < nval; k += blockDim.x)
        if (h[k]) atomicAdd(cnt + base + lo_bin + k, (unsigned long long)h[k]);
}

}  // namespace vcd

namespace vc {

namespace {
// Dynamic LDS beyond 64 KiB must be opted into per kernel (once).
void allow_big_lds() {
    static const bool once = [] {
        (void)hipFuncSetAttribute(reinterpret_cast<const void*>(vcd::hist_kernel<true>),
                                  hipFuncAttributeMaxDynamicSharedMemorySize, vcd::kHistBins * 4);
        (void)hipFuncSetAttribute(reinterpret_cast<const void*>(vcd::hist_kernel<false>),
                                  hipFuncAttributeMaxDynamicSharedMemorySize, vcd::kHistBins * 4);
        return true;
    }();
    (void)once;
}
}  // namespace

hipError_t launch_hist(const LaunchCfg& c, int mode, const int32_t* idx, const uint8_t* aux,
                       int64_t n, int64_t nval, int64_t base, int64_t null_bin, int32_t nt,
                       unsigned long long* counters) {
    if (n <= 0 || !counters) return hipSuccess;
    const bool vec = (reinterpret_cast<uintptr_t>(idx) & 15) == 0 &&
                     (!aux || (reinterpret_cast<uintptr_t>(aux) & 3) == 0);
    const int64_t chunks = nval > 0 ? (nval + vcd::kHistBins - 1) / vcd::kHistBins : 1;
    const int64_t nbk64 = nval > 0 ? (nval + vcd::kBW - 1) / vcd::kBW : 1;
    if (chunks <= 2 || nbk64 > vcd::kMaxBuckets || n >= (int64_t(1) << 32)) {
        // small counter space: one pass per 32K-bin chunk over the outputs
        int64_t slices = (int64_t(c.num_cus) * 2 + chunks - 1) / chunks;
        const int64_t max_slices = (n + 65535) / 65536;     // >= 64K items per workgroup
        if (slices > max_slices) slices = max_slices;
        if (slices < 1) slices = 1;
        const size_t shmem = size_t(nval < vcd::kHistBins ? (nval < 1 ? 1 : nval) : vcd::kHistBins) * 4;
        if (shmem > 64 * 1024) allow_big_lds();
        if (vec)
            hipLaunchKernelGGL(vcd::hist_kernel<true>, dim3(unsigned(slices), unsigned(chunks)),
                               dim3(vcd::kHistBlock), shmem, c.stream, mode, idx, aux, n, nval,
                               base, null_bin, nt, counters);
        else
            hipLaunchKernelGGL(vcd::hist_kernel<false>, dim3(unsigned(slices), unsigned(chunks)),
                               dim3(vcd::kHistBlock), shmem, c.stream, mode, idx, aux, n, nval,
                               base, null_bin, nt, counters);
        return hipGetLastError();
    }
    // large counter space: bucket partition (count, scan, sorted scatter),
    // then per-segment LDS histograms
    int nblk = c.num_cus * 2;
    const int64_t max_blk = (n + 65535) / 65536;
    if (nblk > max_blk) nblk = int(max_blk < 1 ? 1 : max_blk);
    BigHist h;
    int slot = -1;
    uint8_t* scratch = nullptr;
    hipError_t e = c.scratch ? c.scratch->acquire(big_hist_bytes(n, nval, nblk), c.stream, &slot,
                                                  &scratch)
                             : hipErrorInvalidValue;
    if (e == hipSuccess) {
        big_hist_begin(scratch, n, nval, nblk, &h);
        if (vec)
            hipLaunchKernelGGL(vcd::bucket_count_kernel<true>, dim3(nblk), dim3(vcd::kHistBlock),
                               size_t(h.nbk) * 4, c.stream, mode, idx, aux, n, nt, h.nbk, nval,
                               h.counts, counters, null_bin);
        else
            hipLaunchKernelGGL(vcd::bucket_count_kernel<false>, dim3(nblk), dim3(vcd::kHistBlock),
                               size_t(h.nbk) * 4, c.stream, mode, idx, aux, n, nt, h.nbk, nval,
                               h.counts, counters, null_bin);
        e = hipGetLastError();
    }
    const hipError_t e2 = big_hist_finish(c, &h, mode, idx, aux, n, nt, nval, base, counters,
                                          e == hipSuccess);
    const hipError_t e3 = slot >= 0 ? c.scratch->release(slot, c.stream) : hipSuccess;
    return e != hipSuccess ? e : e2 != hipSuccess ? e2 : e3;
}

bool big_hist_applies(int64_t n, int64_t nval) {
    const int64_t chunks = nval > 0 ? (nval + vcd::kHistBins - 1) / vcd::kHistBins : 1;
    const int64_t nbk = nval > 0 ? (nval + vcd::kBW - 1) / vcd::kBW : 1;
    return !(chunks <= 2 || nbk > vcd::kMaxBuckets || n >= (int64_t(1) << 32));
}

int big_hist_bucket_shift() { return 13; }   // log2(kBW)

namespace {
size_t up256(size_t x) { return (x + 255) & ~size_t(255); }
}  // namespace

size_t big_hist_bytes(int64_t n, int64_t nval, int nblk) {
    const int64_t nbk = (nval + vcd::kBW - 1) / vcd::kBW;
    const int64_t m = nbk * nblk;
    return up256(size_t(m) * 4) + up256(size_t(m + 1) * 4) + up256(size_t(nbk + 1) * 4) +
           up256(size_t(n > 0 ? n : 1) * 2);
}

void big_hist_begin(uint8_t* scratch, int64_t n, int64_t nval, int nblk, BigHist* h) {
    static_assert(vcd::kBW == 8192, "big_hist_bucket_shift");
    *h = BigHist{};
    h->nbk = int((nval + vcd::kBW - 1) / vcd::kBW);
    h->nblk = nblk;
    const int64_t m = int64_t(h->nbk) * nblk;
    uint8_t* p = scratch;
    h->counts = reinterpret_cast<uint32_t*>(p);
    p += up256(size_t(m) * 4);
    h->offsets = reinterpret_cast<uint32_t*>(p);
    p += up256(size_t(m + 1) * 4);
    h->seg_off = reinterpret_cast<uint32_t*>(p);
    p += up256(size_t(h->nbk + 1) * 4);
    h->tmp = reinterpret_cast<uint16_t*>(p);
}

hipError_t ScratchRing::init(bool grow_all) {
    grow_all_ = grow_all;
    for (Slot& s : slots_) {
        hipError_t e = hipEventCreateWithFlags(&s.ev, hipEventDisableTiming);
        if (e != hipSuccess) return e;
    }
    return hipSuccess;
}

void ScratchRing::destroy() {
    for (Slot& s : slots_) {
        if (s.p) (void)hipFree(s.p);
        if (s.ev) (void)hipEventDestroy(s.ev);
        s = Slot{};
    }
}

hipError_t ScratchRing::acquire(size_t bytes, hipStream_t st, int* slot, uint8_t** base) {
    int k = -1;
    {
        std::unique_lock<std::mutex> lk(mu_);
        for (;;) {
            for (int i = 0; i < kSlots && k < 0; ++i) {
                const int j = (next_ + i) % kSlots;
                if (!slots_[j].busy) k = j;
            }
            if (k >= 0 && !grow_all_) {
                // an idle arena that fits, else the largest idle one
                int fit = -1, big = k;
                for (int j = 0; j < kSlots; ++j) {
                    if (slots_[j].busy) continue;
                    if (slots_[j].cap >= bytes && (fit < 0 || slots_[j].cap < slots_[fit].cap))
                        fit = j;
                    if (slots_[j].cap > slots_[big].cap) big = j;
                }
                k = fit >= 0 ? fit : big;
            }
            if (k >= 0) break;
            cv_.wait(lk);                      // more concurrent calls than arenas
        }
        slots_[k].busy = true;
        next_ = (k + 1) % kSlots;
    }
    Slot& s = slots_[k];
    hipError_t e = hipSuccess;
    if (s.cap < bytes) {
        // Grow every idle arena to the new size at once (a batch larger
        // than any before): one host stall here instead of one per arena
        // on the next few calls, which would land in the caller's stream of
        // batches as bubbles.
        const size_t cap = up256(bytes + bytes / 4);
        std::vector<int> grow{k};
        if (grow_all_) {
            std::lock_guard<std::mutex> lk(mu_);
            for (int j = 0; j < kSlots; ++j)
                if (j != k && !slots_[j].busy && slots_[j].cap < cap) {
                    slots_[j].busy = true;
                    grow.push_back(j);
                }
        }
        for (int j : grow) {
            Slot& g = slots_[j];
            hipError_t eg = g.used ? hipEventSynchronize(g.ev) : hipSuccess;
            if (eg == hipSuccess && g.p) eg = hipFree(g.p);
            g.p = nullptr;
            g.cap = 0;
            if (eg == hipSuccess) eg = hipMalloc(reinterpret_cast<void**>(&g.p), cap);
            if (eg == hipSuccess) g.cap = cap;
            else g.p = nullptr;
            g.used = false;
            if (j == k) e = eg;
        }
        {
            std::lock_guard<std::mutex> lk(mu_);
            for (int j : grow)
                if (j != k) slots_[j].busy = false;
        }
        cv_.notify_all();
    } else if (s.used) {
        e = hipStreamWaitEvent(st, s.ev, 0);
    }
    if (e != hipSuccess) {
        std::lock_guard<std::mutex> lk(mu_);
        s.busy = false;
        cv_.notify_one();
        return e;
    }
    *slot = k;
    *base = s.p;
    return hipSuccess;
}

hipError_t ScratchRing::release(int slot, hipStream_t st) {
    Slot& s = slots_[slot];
    const hipError_t e = hipEventRecord(s.ev, st);
    std::lock_guard<std::mutex> lk(mu_);
    s.used = s.used || e == hipSuccess;
    s.busy = false;
    cv_.notify_one();
    return e;
}

hipError_t big_hist_finish(const LaunchCfg& c, BigHist* h, int mode, const int32_t* idx,
                           const uint8_t* aux, int64_t n, int32_t nt, int64_t nval, int64_t base,
                           unsigned long long* counters, bool run) {
    hipError_t e = hipSuccess;
    if (run) {
        const bool vec = (reinterpret_cast<uintptr_t>(idx) & 15) == 0 &&
                         (!aux || (reinterpret_cast<uintptr_t>(aux) & 3) == 0);
        const int nbk = h->nbk, nblk = h->nblk;
        const int64_t m = int64_t(nbk) * nblk;
        const int64_t max_segs = (n + vcd::kSeg - 1) / vcd::kSeg + nbk;
        hipLaunchKernelGGL(vcd::bucket_scan_kernel, dim3(1), dim3(vcd::kHistBlock), 0, c.stream,
                           h->counts, h->offsets, m, nbk, nblk, h->seg_off);
        if (vec)
            hipLaunchKernelGGL(vcd::bucket_scatter_kernel<true>, dim3(nblk), dim3(vcd::kHistBlock),
                               size_t(nbk) * 12, c.stream, mode, idx, aux, n, nt, nbk, nval,
                               h->offsets, h->tmp);
        else
            hipLaunchKernelGGL(vcd::bucket_scatter_kernel<false>, dim3(nblk),
                               dim3(vcd::kHistBlock), size_t(nbk) * 12, c.stream, mode, idx, aux,
                               n, nt, nbk, nval, h->offsets, h->tmp);
        hipLaunchKernelGGL(vcd::bucket_hist_kernel, dim3(unsigned(max_segs)), dim3(vcd::kHistBlock),
                           0, c.stream, h->tmp, h->offsets, h->seg_off, nblk, nbk, nval, base,
                           counters);
        e = hipGetLastError();
    }
    *h = BigHist{};
    return e;
}

}  // namespace vc

VC_DEVCHECK_READER(counters)
