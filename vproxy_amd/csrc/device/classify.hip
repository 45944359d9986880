// classify.hip -- ACL, route and combined-pipeline kernels for gfx950.
//
// One lane per header.  Inputs are SoA arrays streamed from HBM with 4
// items per lane per step (16-byte address loads, 4-byte proto loads, 8-byte
// port loads, 16-byte index stores); the ACL interval boundaries are staged
// in LDS once per workgroup of a grid-stride (persistent-style) launch.
#include <algorithm>
#include <cstdlib>
#include <map>
#include <mutex>

#include "acl_dev.h"
#include "launch.h"
#include "route_dev.h"

#ifndef VC_PIPE_NT
#define VC_PIPE_NT 1
#endif

namespace vcd {

constexpr int kBlock = 512;
// The pipeline is bound by the rate of random table gathers, which 16 waves
// per CU already saturate (tools/gather_probe.hip): one 1024-thread
// workgroup per CU, so the LDS it does not use stays free for kernels
// running beside it on other streams (hit counters, the next hostname pool).
constexpr int kPipeBlock = 1024;

// ---------------------------------------------------------------------------
// ACL (SecurityGroup.allow) on IPv4 sources.  The boundaries of both lists
// are staged in LDS; when they exceed the LDS budget, every (1 << shift)-th
// boundary is staged as a fence and the search finishes in one block of
// 1 << shift boundaries in global memory (the same two levels as IPv6).
// ---------------------------------------------------------------------------
struct AclV4Ctx {
    const uint32_t* f[2];          // LDS: every boundary (shift 0) or the fences
    const uint32_t* b[2];          // global boundaries
    const uint32_t* rec[2];
    const uint32_t* pieces[2];
    int nf[2], nb[2];
    int shift;                     // uniform per launch
};

__device__ __forceinline__ int fence_count(int nb, int shift) {
    return (nb + (1 << shift) - 1) >> shift;
}

// The protocol's member of a per-list pair, chosen by value.  Indexing the
// pair with a runtime list number (a.f[tcp ? 0 : 1]) keeps the whole context
// struct in scratch memory and reads every member through it: the two-quad
// ACL kernel carried a 96-byte private segment that way and its speed
// depended on the build (profiles/r03_ab_acl_quads.txt).
// tests/test_codegen_cpu.py checks the hot kernels use no scratch.
template <class T>
__device__ __forceinline__ T per_list(bool tcp, T x0, T x1) { return tcp ? x0 : x1; }

// kL: a.f is staged in LDS (else it is the global boundary list, shift 0)
template <bool kL>
__device__ __forceinline__ uint32_t acl_v4_one(const AclV4Ctx& a, bool tcp, uint32_t key,
                                               uint32_t port) {
    int j = bsearch_u32<kL>(per_list(tcp, a.f[0], a.f[1]), per_list(tcp, a.nf[0], a.nf[1]), key);
    if (kL && a.shift) {
        const int base = j << a.shift;
        const int rest = per_list(tcp, a.nb[0], a.nb[1]) - base;
        j = base + bsearch_u32(per_list(tcp, a.b[0], a.b[1]) + base,
                               rest < (1 << a.shift) ? rest : (1 << a.shift), key);
    }
    return acl_value(per_list(tcp, a.rec[0], a.rec[1]), per_list(tcp, a.pieces[0], a.pieces[1]),
                     j, port);
}

// Four lookups in lockstep (VC_ACL_LOCKSTEP, boundaries fully staged in
// LDS): acl_v4_one runs each interval search as its own loop, so the four
// searches of a lane wait on their ds_reads one after another (~14 waits
// each).  Here one loop steps all four: its trip count is that of the longer
// list, and a search whose range is down to one interval keeps reading the
// same boundary (half = 0 leaves lo as it is), so no step needs a bound
// check; the four record loads then go out together.
#ifndef VC_ACL_LOCKSTEP
#define VC_ACL_LOCKSTEP 1
#endif
#ifndef VC_ACL_QUADS
#define VC_ACL_QUADS 2
#endif
#ifndef VC_ACL_PREFETCH
#define VC_ACL_PREFETCH 0
#endif
template <bool kL, int kN = 4>
__device__ __forceinline__ void acl_v4_four(const AclV4Ctx& a, const bool tcp[kN],
                                            const uint32_t key[kN], const uint32_t port[kN],
                                            uint32_t v[kN]) {
    if (!VC_ACL_LOCKSTEP || !kL || a.shift) {
#pragma unroll
        for (int k = 0; k < kN; ++k) v[k] = acl_v4_one<kL>(a, tcp[k], key[k], port[k]);
        return;
    }
    const int nmax = a.nf[0] > a.nf[1] ? a.nf[0] : a.nf[1];
    const int steps = nmax > 1 ? 32 - __builtin_clz(uint32_t(nmax - 1)) : 0;
    // 32-bit LDS pointers, cast once (a generic-to-LDS cast per access
    // costs a null check and 64-bit address arithmetic)
    const VC_AS_LDS uint32_t* f0 = (const VC_AS_LDS uint32_t*)a.f[0];
    const VC_AS_LDS uint32_t* f1 = (const VC_AS_LDS uint32_t*)a.f[1];
    const VC_AS_LDS uint32_t* f[kN];
    int lo[kN], len[kN];
#pragma unroll
    for (int k = 0; k < kN; ++k) {
        f[k] = tcp[k] ? f0 : f1;
        len[k] = tcp[k] ? a.nf[0] : a.nf[1];
        lo[k] = 0;
    }
#if defined(VC_ABL_NOSEARCH)        // timing ablation only: no interval search
#pragma unroll
    for (int k = 0; k < kN; ++k) lo[k] = int(key[k] % uint32_t(len[k]));
    if (steps > 0) goto records;
#endif
    for (int s = 0; s < steps; ++s) {
        uint32_t x[kN];
        int half[kN];
#pragma unroll
        for (int k = 0; k < kN; ++k) {
            half[k] = len[k] >> 1;
            x[k] = f[k][lo[k] + half[k]];
        }
#pragma unroll
        for (int k = 0; k < kN; ++k) {
            lo[k] = x[k] <= key[k] ? lo[k] + half[k] : lo[k];
            len[k] -= half[k];
        }
    }
#if defined(VC_ABL_NOSEARCH)
records:
#endif
    uint4 r[kN];
#pragma unroll
    for (int k = 0; k < kN; ++k)
        r[k] = glb_ld(reinterpret_cast<const uint4*>(tcp[k] ? a.rec[0] : a.rec[1]) + lo[k]);
#pragma unroll
    for (int k = 0; k < kN; ++k)
        v[k] = acl_rec_value(r[k], tcp[k] ? a.pieces[0] : a.pieces[1], port[k]);
}

// The IPv4 pipeline's ACL: four separate searches (VC_PIPE_LOCKSTEP 0).  The
// lockstep form that takes C2 from 0.82 to 0.70 ms made the gather-bound
// pipeline kernel 0.5-0.7 % slower (profiles/r03_ab_acl_lockstep.txt).
#ifndef VC_PIPE_LOCKSTEP
#define VC_PIPE_LOCKSTEP 0
#endif
#if VC_PIPE_LOCKSTEP
#define VC_PIPE_ACL4(a, tcp, key, po, v) acl_v4_four<kLds>(a, tcp, key, po, v)
#else
#define VC_PIPE_ACL4(a, tcp, key, po, v)                                              \
    do {                                                                             \
        for (int k_ = 0; k_ < 4; ++k_) v[k_] = acl_v4_one<kLds>(a, tcp[k_], key[k_], po[k_]); \
    } while (0)
#endif

__device__ __forceinline__ void acl_emit(const AclImage& img, bool tcp, uint32_t v,
                                         uint8_t* allow_out, int32_t* idx_out) {
    *idx_out = out_index(v);
    if (allow_out) {
        *allow_out = v == VC_NONE ? uint8_t(img.default_allow)
                                  : glb_ld(img.allow + (tcp ? 0 : img.n_tcp) + v);
    }
}

// lds: the staged boundaries or fences (stage_bounds), or null: one-level
// search of the global boundaries
__device__ __forceinline__ AclV4Ctx acl_v4_ctx(const AclImage& img, const uint32_t* lds,
                                               int shift) {
    AclV4Ctx a;
    a.shift = lds ? shift : 0;
    int off = 0;
    for (int l = 0; l < 2; ++l) {
        const AclFamilyImage& f = img.fam[l][0];
        a.nb[l] = f.nb;
        a.nf[l] = fence_count(f.nb, a.shift);
        a.b[l] = f.bounds4;
        a.f[l] = lds ? lds + off : f.bounds4;
        a.rec[l] = f.rec;
        a.pieces[l] = f.pieces;
        off += a.nf[l];
    }
    return a;
}

// LDS words stage_bounds fills
__device__ __forceinline__ int staged_words(const AclImage& img, int shift) {
    return fence_count(img.fam[0][0].nb, shift) + fence_count(img.fam[1][0].nb, shift);
}

__device__ __forceinline__ void stage_bounds(const AclImage& img, uint32_t* lds, int shift) {
    const int nf0 = fence_count(img.fam[0][0].nb, shift);
    const int nf1 = fence_count(img.fam[1][0].nb, shift);
    const uint32_t* b0 = img.fam[0][0].bounds4;
    const uint32_t* b1 = img.fam[1][0].bounds4;
    for (int k = threadIdx.x; k < nf0; k += blockDim.x) lds[k] = b0[int64_t(k) << shift];
    for (int k = threadIdx.x; k < nf1; k += blockDim.x) lds[nf0 + k] = b1[int64_t(k) << shift];
    __syncthreads();
}

template <bool kLds, int kQ>
__global__ __launch_bounds__(kBlock) void acl_v4_kernel(
    AclImage img, int shift, const uint8_t* __restrict__ proto, const uint32_t* __restrict__ src,
    const uint16_t* __restrict__ port, int64_t n, int32_t* __restrict__ out,
    uint8_t* __restrict__ allow) {
    extern __shared__ __attribute__((aligned(16))) uint32_t lds[];
    if (kLds) stage_bounds(img, lds, shift);
    const AclV4Ctx a = acl_v4_ctx(img, kLds ? lds : nullptr, shift);
    const int64_t stride = int64_t(gridDim.x) * blockDim.x;
    const int64_t n4 = n >> 2;
    // kQ quads of 4 tuples per lane per pass (g, g + stride, ...): the kQ * 4
    // interval searches step in lockstep, so a pass waits on its LDS reads
    // (and its loads and record reads) once for all of them
    // the next pass's tuples are loaded before this pass's searches
    // (VC_ACL_PREFETCH), so their HBM latency hides behind the LDS steps
    uint4 s_n[kQ];
    uint32_t pr_n[kQ];
    uint2 pt_n[kQ];
    auto load_pass = [&](int64_t g0) {
#pragma unroll
        for (int q = 0; q < kQ; ++q) {
            // a quad past the end reads the last quad (searched, not stored)
            const int64_t g = g0 + q * stride < n4 ? g0 + q * stride : n4 - 1;
            s_n[q] = reinterpret_cast<const uint4*>(src)[g];
            pr_n[q] = reinterpret_cast<const uint32_t*>(proto)[g];
            pt_n[q] = reinterpret_cast<const uint2*>(port)[g];
        }
    };
    const int64_t gfirst = int64_t(blockIdx.x) * blockDim.x + threadIdx.x;
    if (VC_ACL_PREFETCH && gfirst < n4) load_pass(gfirst);
    for (int64_t g0 = gfirst; g0 < n4; g0 += kQ * stride) {
        uint32_t key[4 * kQ], po[4 * kQ], v[4 * kQ];
        bool tcp[4 * kQ];
        if (!VC_ACL_PREFETCH) load_pass(g0);
        uint4 s_c[kQ];
        uint32_t pr_c[kQ];
        uint2 pt_c[kQ];
#pragma unroll
        for (int q = 0; q < kQ; ++q) {
            s_c[q] = s_n[q];
            pr_c[q] = pr_n[q];
            pt_c[q] = pt_n[q];
        }
        if (VC_ACL_PREFETCH && g0 + kQ * stride < n4) load_pass(g0 + kQ * stride);
#pragma unroll
        for (int q = 0; q < kQ; ++q) {
            const uint4 s = s_c[q];
            const uint32_t pr = pr_c[q];
            const uint2 pt = pt_c[q];
            key[4 * q + 0] = s.x;
            key[4 * q + 1] = s.y;
            key[4 * q + 2] = s.z;
            key[4 * q + 3] = s.w;
            po[4 * q + 0] = pt.x & 0xFFFFu;
            po[4 * q + 1] = pt.x >> 16;
            po[4 * q + 2] = pt.y & 0xFFFFu;
            po[4 * q + 3] = pt.y >> 16;
#pragma unroll
            for (int k = 0; k < 4; ++k) tcp[4 * q + k] = ((pr >> (8 * k)) & 0xFFu) == VC_PROTO_TCP;
        }
        acl_v4_four<kLds, 4 * kQ>(a, tcp, key, po, v);
#pragma unroll
        for (int q = 0; q < kQ; ++q) {
            const int64_t g = g0 + q * stride;
            if (q > 0 && g >= n4) break;
            int4 o;
            uint32_t al = 0;
            int32_t* op = reinterpret_cast<int32_t*>(&o);
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                uint8_t b = 0;
                acl_emit(img, tcp[4 * q + k], v[4 * q + k], allow ? &b : nullptr, op + k);
                al |= uint32_t(b) << (8 * k);
            }
            reinterpret_cast<int4*>(out)[g] = o;
            if (allow) reinterpret_cast<uint32_t*>(allow)[g] = al;
        }
    }
    // tail (n % 4 items), handled by the first threads of block 0
    if (blockIdx.x == 0 && threadIdx.x < (n & 3)) {
        const int64_t i = (n4 << 2) + threadIdx.x;
        const bool t = proto[i] == VC_PROTO_TCP;
        const uint32_t v = acl_v4_one<kLds>(a, t, src[i], port[i]);
        acl_emit(img, t, v, allow ? allow + i : nullptr, out + i);
    }
}

// Unaligned-pointer variant: one item per lane.
template <bool kLds>
__global__ __launch_bounds__(kBlock) void acl_v4_kernel_scalar(
    AclImage img, int shift, const uint8_t* __restrict__ proto, const uint32_t* __restrict__ src,
    const uint16_t* __restrict__ port, int64_t n, int32_t* __restrict__ out,
    uint8_t* __restrict__ allow) {
    extern __shared__ __attribute__((aligned(16))) uint32_t lds[];
    if (kLds) stage_bounds(img, lds, shift);
    const AclV4Ctx a = acl_v4_ctx(img, kLds ? lds : nullptr, shift);
    const int64_t stride = int64_t(gridDim.x) * blockDim.x;
    for (int64_t i = int64_t(blockIdx.x) * blockDim.x + threadIdx.x; i < n; i += stride) {
        const bool t = proto[i] == VC_PROTO_TCP;
        const uint32_t v = acl_v4_one<kLds>(a, t, src[i], port[i]);
        acl_emit(img, t, v, allow ? allow + i : nullptr, out + i);
    }
}

// ---------------------------------------------------------------------------
// ACL on IPv6 sources: 128-bit interval search, two levels.  Every
// (1 << shift)-th boundary of both protocol lists is staged in LDS as a
// fence; the search runs over the fences in LDS, then over one block of
// 1 << shift boundaries in global memory (L2-resident): shift dependent
// global loads instead of log2(nb) (~15 at 10k rules).
// ---------------------------------------------------------------------------
struct AclV6Ctx {
    const uint64_t* f[2];          // LDS fences, (hi, lo) pairs
    const uint64_t* b[2];          // global boundaries
    const uint32_t* rec[2];
    const uint32_t* pieces[2];
    int nf[2], nb[2];
    int v4only[2];                 // AclFamilyImage.v4_only of the list's v6 image
    int shift;
};

// Stages the fences of both lists at lds (16-byte aligned); the caller syncs.
__device__ __forceinline__ AclV6Ctx stage_fences(const AclImage& img, uint64_t* lds, int shift) {
    AclV6Ctx a;
    a.shift = shift;
    int off = 0;
    for (int l = 0; l < 2; ++l) {
        const AclFamilyImage& f = img.fam[l][1];
        a.nb[l] = f.nb;
        a.nf[l] = fence_count(f.nb, shift);
        a.v4only[l] = f.v4_only;
        a.b[l] = f.bounds6;
        a.rec[l] = f.rec;
        a.pieces[l] = f.pieces;
        a.f[l] = lds + 2 * off;
        for (int k = threadIdx.x; k < a.nf[l]; k += blockDim.x)
            reinterpret_cast<ulonglong2*>(lds)[off + k] =
                reinterpret_cast<const ulonglong2*>(f.bounds6)[int64_t(k) << shift];
        off += a.nf[l];
    }
    return a;
}

__device__ __forceinline__ uint32_t acl_v6_fenced(const AclV6Ctx& a, bool tcp, uint4 w,
                                                  uint32_t port) {
    uint64_t hi, lo;
    v6_key(w, &hi, &lo);
    const int k = bsearch_u128<true>(per_list(tcp, a.f[0], a.f[1]), per_list(tcp, a.nf[0], a.nf[1]),
                                     hi, lo);
    const int base = k << a.shift;
    const int rest = per_list(tcp, a.nb[0], a.nb[1]) - base;
    const int len = rest < (1 << a.shift) ? rest : (1 << a.shift);
    const int j = base + bsearch_u128(per_list(tcp, a.b[0], a.b[1]) + 2 * int64_t(base), len, hi, lo);
    return acl_value(per_list(tcp, a.rec[0], a.rec[1]), per_list(tcp, a.pieces[0], a.pieces[1]),
                     j, port);
}

// An IPv6 source on a list of plain IPv4 rules classifies like its low 32
// bits on the v4 image when it has an IPv4 form, else as no rule
// (acl_dev.h v6_v4_form / acl6_global); other lists take the fenced search.
// The mixed pipeline has the v4 boundaries in LDS (kLds): the IPv6 packets
// of a C5-style batch then cost a v4 search instead of the fence search and
// its dependent block loads.
template <bool kLds>
__device__ __forceinline__ uint32_t acl_v6_any(const AclV4Ctx& a, const AclV6Ctx& a6, bool tcp,
                                               uint4 w, uint32_t port) {
    if (per_list(tcp, a6.v4only[0], a6.v4only[1])) {
        uint64_t hi, lo;
        v6_key(w, &hi, &lo);
        return v6_v4_form(hi, lo) ? acl_v4_one<kLds>(a, tcp, uint32_t(lo), port) : VC_NONE;
    }
    return acl_v6_fenced(a6, tcp, w, port);
}

__global__ __launch_bounds__(kBlock) void acl_v6_kernel(
    AclImage img, int shift, const uint8_t* __restrict__ proto,
    const uint8_t* __restrict__ src6, const uint16_t* __restrict__ port, int64_t n,
    int32_t* __restrict__ out, uint8_t* __restrict__ allow) {
    extern __shared__ __attribute__((aligned(16))) uint64_t fences[];
    const AclV6Ctx a = stage_fences(img, fences, shift);
    __syncthreads();
    const int64_t stride = int64_t(gridDim.x) * blockDim.x;
    for (int64_t i = int64_t(blockIdx.x) * blockDim.x + threadIdx.x; i < n; i += stride) {
        const bool t = proto[i] == VC_PROTO_TCP;
        const uint4 w = reinterpret_cast<const uint4*>(src6)[i];
        uint32_t v;
        if (per_list(t, a.v4only[0], a.v4only[1])) {
            uint64_t hi, lo;
            v6_key(w, &hi, &lo);
            v = t ? acl6_global(img.fam[0][1], img.fam[0][0], hi, lo, port[i])
                  : acl6_global(img.fam[1][1], img.fam[1][0], hi, lo, port[i]);
        } else {
            v = acl_v6_fenced(a, t, w, port[i]);
        }
        acl_emit(img, t, v, allow ? allow + i : nullptr, out + i);
    }
}

// ---------------------------------------------------------------------------
// RouteTable.lookup
// ---------------------------------------------------------------------------
__device__ __forceinline__ void route_emit(uint32_t e, int32_t* o) { *o = out_index(e); }

__global__ __launch_bounds__(kBlock) void route_v4_kernel(
    const uint32_t* __restrict__ nodes, int rb, const uint32_t* __restrict__ dst, int64_t n,
    int32_t* __restrict__ out) {
    const int64_t stride = int64_t(gridDim.x) * blockDim.x;
    const int64_t n4 = n >> 2;
    for (int64_t g = int64_t(blockIdx.x) * blockDim.x + threadIdx.x; g < n4; g += stride) {
        const uint4 d = reinterpret_cast<const uint4*>(dst)[g];
        const uint32_t key[4] = {d.x, d.y, d.z, d.w};
        uint32_t e[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) e[k] = nodes[key[k] >> (32 - rb)];   // 4 probes in flight
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            int bits = rb;
            while (e[k] & VC_PTR) {
                const int s = trie_stride(bits);
                e[k] = trie_next(nodes, 1u << rb, e[k], v4_sub(key[k], bits, s),
                                 uint64_t(key[k]) << 32);
                bits += s;
            }
        }
        int4 o;
        int32_t* op = reinterpret_cast<int32_t*>(&o);
#pragma unroll
        for (int k = 0; k < 4; ++k) route_emit(e[k], op + k);
        reinterpret_cast<int4*>(out)[g] = o;
    }
    if (blockIdx.x == 0 && threadIdx.x < (n & 3)) {
        const int64_t i = (n4 << 2) + threadIdx.x;
        route_emit(trie_v4(nodes, rb, dst[i]), out + i);
    }
}

__global__ __launch_bounds__(kBlock) void route_v4_kernel_scalar(
    const uint32_t* __restrict__ nodes, int rb, const uint32_t* __restrict__ dst, int64_t n,
    int32_t* __restrict__ out) {
    const int64_t stride = int64_t(gridDim.x) * blockDim.x;
    for (int64_t i = int64_t(blockIdx.x) * blockDim.x + threadIdx.x; i < n; i += stride)
        route_emit(trie_v4(nodes, rb, dst[i]), out + i);
}

// The IPv6 wide root (images.h TrieImage.wide) from the root and its
// one-prefix records, one slot per thread, at compile time.
__global__ __launch_bounds__(kBlock) void wide_root_kernel(const uint32_t* __restrict__ nodes,
                                                           uint32_t slots,
                                                           uint4* __restrict__ wide) {
    const uint32_t stride = gridDim.x * blockDim.x;
    for (uint32_t s = blockIdx.x * blockDim.x + threadIdx.x; s < slots; s += stride) {
        uint32_t w[4];
        wide_entry(nodes, s, w);
        wide[s] = make_uint4(w[0], w[1], w[2], w[3]);
    }
}

// 4 IPv6 lookups per lane: the trie walk is a chain of dependent gathers
// (root, then one 8-bit stride per level down to /48 or /64), so four
// independent walks advance level by level together to keep four gathers in
// flight per lane.
__global__ __launch_bounds__(kBlock) void route_v6_kernel_x4(
    const uint32_t* __restrict__ nodes, const uint32_t* __restrict__ wide, int rb,
    const uint8_t* __restrict__ dst6, int64_t n, int32_t* __restrict__ out) {
    const int64_t stride = int64_t(gridDim.x) * blockDim.x;
    const int64_t n4 = n >> 2;
    const uint32_t root = 1u << rb;
    for (int64_t g = int64_t(blockIdx.x) * blockDim.x + threadIdx.x; g < n4; g += stride) {
        uint64_t hi[4], lo[4];
        uint32_t e[4];
        int bits[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            v6_key(reinterpret_cast<const uint4*>(dst6)[4 * g + k], &hi[k], &lo[k]);
            bits[k] = rb;
        }
        if (wide) {                               // one load answers a one-prefix slot
#pragma unroll
            for (int k = 0; k < 4; ++k)
                e[k] = wide_first(reinterpret_cast<const uint4*>(wide)[hi[k] >> (64 - rb)], hi[k]);
        } else {
#pragma unroll
            for (int k = 0; k < 4; ++k) e[k] = nodes[hi[k] >> (64 - rb)];
        }
        for (;;) {
            bool any = false;
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                if (e[k] & VC_PTR) {
                    const int s = trie_stride(bits[k]);
                    e[k] = trie_next(nodes, root, e[k], v6_sub(hi[k], lo[k], bits[k], s), hi[k]);
                    bits[k] += s;
                    any = true;
                }
            }
            if (!any) break;
        }
        int4 o;
        int32_t* op = reinterpret_cast<int32_t*>(&o);
#pragma unroll
        for (int k = 0; k < 4; ++k) route_emit(e[k], op + k);
        reinterpret_cast<int4*>(out)[g] = o;
    }
    if (blockIdx.x == 0 && threadIdx.x < (n & 3)) {
        const int64_t i = (n4 << 2) + threadIdx.x;
        uint64_t hi, lo;
        v6_key(reinterpret_cast<const uint4*>(dst6)[i], &hi, &lo);
        route_emit(trie_v6w(nodes, wide, rb, hi, lo), out + i);
    }
}

__global__ __launch_bounds__(kBlock) void route_v6_kernel(
    const uint32_t* __restrict__ nodes, const uint32_t* __restrict__ wide, int rb,
    const uint8_t* __restrict__ dst6, int64_t n, int32_t* __restrict__ out) {
    const int64_t stride = int64_t(gridDim.x) * blockDim.x;
    for (int64_t i = int64_t(blockIdx.x) * blockDim.x + threadIdx.x; i < n; i += stride) {
        uint64_t hi, lo;
        v6_key(reinterpret_cast<const uint4*>(dst6)[i], &hi, &lo);
        route_emit(trie_v6w(nodes, wide, rb, hi, lo), out + i);
    }
}

// ---------------------------------------------------------------------------
// Combined pipeline (C5): ACL(src, dport) -> route(dst) -> pool group gather
// ---------------------------------------------------------------------------
// The packet SoA streams are read and the outputs written once; with
// VC_PIPE_NT they carry the nontemporal hint so they do not displace the
// gathered tables (route root, pool results) from the caches.
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));

__device__ __forceinline__ uint4 stream_ld(const uint4* p) {
#if VC_PIPE_NT
    const u32x4 v = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(p));
    return make_uint4(v.x, v.y, v.z, v.w);
#else
    return *p;
#endif
}
__device__ __forceinline__ uint2 stream_ld(const uint2* p) {
#if VC_PIPE_NT
    const u32x2 v = __builtin_nontemporal_load(reinterpret_cast<const u32x2*>(p));
    return make_uint2(v.x, v.y);
#else
    return *p;
#endif
}
__device__ __forceinline__ uint32_t stream_ld(const uint32_t* p) {
#if VC_PIPE_NT
    return __builtin_nontemporal_load(p);
#else
    return *p;
#endif
}
__device__ __forceinline__ void stream_st(int4* p, int4 v) {
#if VC_PIPE_NT
    u32x4 w = {uint32_t(v.x), uint32_t(v.y), uint32_t(v.z), uint32_t(v.w)};
    __builtin_nontemporal_store(w, reinterpret_cast<u32x4*>(p));
#else
    *p = v;
#endif
}
__device__ __forceinline__ void stream_st(uint32_t* p, uint32_t v) {
#if VC_PIPE_NT
    __builtin_nontemporal_store(v, p);
#else
    *p = v;
#endif
}
// Random table gathers (route roots, pool results) of the mixed-family
// kernels; with VC_GATHER_NT they carry the nontemporal hint, so the lines
// they pull through L2 do not evict the small tables the IPv6 packets read
// next (one-prefix records, ACL records).
#ifndef VC_GATHER_NT
#define VC_GATHER_NT 0
#endif
template <class T>
__device__ __forceinline__ T gather_ld(const T* p) {
#if VC_GATHER_NT
    return __builtin_nontemporal_load(p);
#else
    return *p;
#endif
}
// The compact-row kernel's SoA streams through stream_ld / stream_st too
// (VC_C6_NT = 0: plain loads and stores, the round-4 form).
#ifndef VC_C6_NT
#define VC_C6_NT 1
#endif
template <class T>
__device__ __forceinline__ T c6_ld(const T* p) {
#if VC_C6_NT
    return stream_ld(p);
#else
    return *p;
#endif
}
__device__ __forceinline__ void c6_st(int4* p, int4 v) {
#if VC_C6_NT
    stream_st(p, v);
#else
    *p = v;
#endif
}
__device__ __forceinline__ void c6_st(uint32_t* p, uint32_t v) {
#if VC_C6_NT
    stream_st(p, v);
#else
    *p = v;
#endif
}

__device__ __forceinline__ uint32_t route_chase(const uint32_t* nodes, int rb, uint32_t e,
                                                uint32_t d) {
    int bits = rb;
    while (e & VC_PTR) {
        const int s = trie_stride(bits);
        e = trie_next(nodes, 1u << rb, e, v4_sub(d, bits, s), uint64_t(d) << 32);
        bits += s;
    }
    return e;
}

__device__ __forceinline__ uint32_t route6_chase(const uint32_t* nodes, int rb, uint32_t e,
                                                 uint64_t hi, uint64_t lo) {
    int bits = rb;
    const uint32_t root = 1u << rb;
    while (e & VC_PTR) {
        const int s = trie_stride(bits);
        e = trie_next(nodes, root, e, v6_sub(hi, lo, bits, s), hi);
        bits += s;
    }
    return e;
}

// In-kernel hit counting of the pipeline (launch_pipeline): the ACL
// histogram in LDS next to the staged boundaries, and per-workgroup bucket
// counts of the route and group outputs -- the first pass of the large
// counter-space histogram (counters.hip), which then only scans, scatters
// and histograms.  The kernel is bound by its table gathers, so the LDS
// atomics ride along for free and two passes over the outputs disappear.
// Route values are counted in the combined space [v4 rules][v6 rules].
struct PipeCount {
    unsigned long long* acl;       // ACL counters, or null: not counted here
    int32_t acl_bins;              // n_tcp + n_udp (LDS words)
    int32_t n_tcp;
    uint32_t* rcounts;             // route bucket counts [bucket * grid + block], or null
    int32_t r_nbk;
    int32_t n4;                    // v6 route index r counts as n4 + r
    unsigned long long* route;     // route counters (v4 null at route_none_at, v6 null next)
    int64_t route_none_at;
    uint32_t* gcounts;             // group bucket counts, or null
    int32_t g_nbk;
    unsigned long long* group;     // group counters (null bin at n_groups)
    int32_t n_groups;
    int32_t bw_shift;              // log2(bucket width)
};

struct PipeTally {                 // per-thread null counts
    uint32_t acl_tcp = 0, acl_udp = 0, route = 0, route6 = 0, group = 0;
};

__device__ __forceinline__ void pipe_count(const PipeCount& pc, uint32_t* ah, uint32_t* rc,
                                           uint32_t* gc, bool tcp, uint32_t v, bool v6,
                                           int32_t r, int32_t g, PipeTally* t) {
    if (pc.acl) {
        if (v != VC_NONE) atomicAdd(&ah[tcp ? v : uint32_t(pc.n_tcp) + v], 1u);
        else if (tcp) ++t->acl_tcp;
        else ++t->acl_udp;
    }
    if (pc.rcounts) {
        if (r >= 0) atomicAdd(&rc[(v6 ? r + pc.n4 : r) >> pc.bw_shift], 1u);
        else if (v6) ++t->route6;
        else ++t->route;
    }
    if (pc.gcounts) {
        // pool results at or past n_groups (a pool classified against an
        // older Upstream snapshot) are not counted, as in counters.hip
        if (g >= 0) {
            if (g < pc.n_groups) atomicAdd(&gc[g >> pc.bw_shift], 1u);
        } else {
            ++t->group;
        }
    }
}

// Flush of the in-kernel counts (every thread of the workgroup calls it).
__device__ __forceinline__ void pipe_count_flush(const PipeCount& pc, uint32_t* ah, uint32_t* rc,
                                                 uint32_t* gc, uint32_t* tally,
                                                 const PipeTally& t) {
    if (t.acl_tcp) atomicAdd(&tally[0], t.acl_tcp);
    if (t.acl_udp) atomicAdd(&tally[1], t.acl_udp);
    if (t.route) atomicAdd(&tally[2], t.route);
    if (t.group) atomicAdd(&tally[3], t.group);
    if (t.route6) atomicAdd(&tally[4], t.route6);
    __syncthreads();
    if (pc.acl) {
        for (int k = threadIdx.x; k < pc.acl_bins; k += blockDim.x)
            if (ah[k]) atomicAdd(pc.acl + k, (unsigned long long)ah[k]);
        if (threadIdx.x == 0) {                   // [tcp default][udp default]
            if (tally[0]) atomicAdd(pc.acl + pc.acl_bins, (unsigned long long)tally[0]);
            if (tally[1]) atomicAdd(pc.acl + pc.acl_bins + 1, (unsigned long long)tally[1]);
        }
    }
    if (pc.rcounts) {
        for (int k = threadIdx.x; k < pc.r_nbk; k += blockDim.x)
            pc.rcounts[int64_t(k) * gridDim.x + blockIdx.x] = rc[k];
        if (threadIdx.x == 0 && tally[2])
            atomicAdd(pc.route + pc.route_none_at, (unsigned long long)tally[2]);
        if (threadIdx.x == 0 && tally[4])
            atomicAdd(pc.route + pc.route_none_at + 1, (unsigned long long)tally[4]);
    }
    if (pc.gcounts) {
        for (int k = threadIdx.x; k < pc.g_nbk; k += blockDim.x)
            pc.gcounts[int64_t(k) * gridDim.x + blockIdx.x] = gc[k];
        if (threadIdx.x == 0 && tally[3])
            atomicAdd(pc.group + pc.n_groups, (unsigned long long)tally[3]);
    }
}

// LDS layout of a pipeline workgroup: staged v4 ACL boundaries, then the
// ACL histogram, route bucket counts and group bucket counts.
struct PipeLds {
    uint32_t* ah;
    uint32_t* rc;
    uint32_t* gc;
};

template <bool kLds, bool kCount>
__device__ __forceinline__ PipeLds pipe_lds_setup(const AclImage& img, const PipeCount& pc,
                                                  uint32_t* lds, uint32_t* tally, int shift) {
    const int words = kLds ? staged_words(img, shift) : 0;
    PipeLds L;
    L.ah = lds + words;
    L.rc = L.ah + (pc.acl ? pc.acl_bins : 0);
    L.gc = L.rc + (pc.rcounts ? pc.r_nbk : 0);
    if (kCount) {
        const int cw = (pc.acl ? pc.acl_bins : 0) + (pc.rcounts ? pc.r_nbk : 0) +
                       (pc.gcounts ? pc.g_nbk : 0);
        for (int k = threadIdx.x; k < cw; k += blockDim.x) L.ah[k] = 0;
        if (threadIdx.x < 5) tally[threadIdx.x] = 0;
    }
    if (kLds) stage_bounds(img, lds, shift);
    else if (kCount) __syncthreads();
    return L;
}

// One IPv4 packet through ACL -> route -> pool group (scalar form, also the tail).
template <bool kLds, bool kCount>
__device__ __forceinline__ void pipeline_one(
    const AclImage& img, const AclV4Ctx& a, const uint32_t* nodes, int rb, const uint8_t* proto,
    const uint32_t* src, const uint32_t* dst, const uint16_t* dport, const uint32_t* host_id,
    const int32_t* pool_group, int64_t n_pool, int64_t i, int32_t* out_acl, int32_t* out_route,
    int32_t* out_group, uint8_t* out_allow, const PipeCount& pc, const PipeLds& L,
    PipeTally* t) {
    const uint32_t d = dst[i];
    const uint32_t e = nodes[d >> (32 - rb)];
    const uint32_t h = host_id[i];
    const int32_t grp = int64_t(h) < n_pool ? pool_group[h] : -1;
    const bool tcp = proto[i] == VC_PROTO_TCP;
    const uint32_t v = acl_v4_one<kLds>(a, tcp, src[i], dport[i]);
    acl_emit(img, tcp, v, out_allow ? out_allow + i : nullptr, out_acl + i);
    const int32_t r = out_index(route_chase(nodes, rb, e, d));
    out_route[i] = r;
    out_group[i] = grp;
    if (kCount) pipe_count(pc, L.ah, L.rc, L.gc, tcp, v, false, r, grp, t);
}

// Contiguous slice [lo, hi) of n items owned by this workgroup, on 4-item
// boundaries (the same split as counters.hip, which reads the bucket counts
// per workgroup).
__device__ __forceinline__ void pipe_slice(int64_t n, int64_t* lo, int64_t* hi) {
    const int64_t groups = (n + 3) >> 2;
    const int64_t per = (groups + gridDim.x - 1) / gridDim.x;
    *lo = int64_t(blockIdx.x) * per * 4;
    const int64_t h = *lo + per * 4;
    *hi = h < n ? h : n;
    if (*lo > n) *lo = n;
}

// kVec: 4 packets per lane per step -- 16-byte SoA loads/stores and four
// independent route-root and pool gathers in flight before the ACL search.
template <bool kLds, bool kVec, bool kCount>
__global__ __launch_bounds__(kPipeBlock) void pipeline_v4_kernel(
    AclImage img, const uint32_t* __restrict__ nodes, int rb, const uint8_t* __restrict__ proto,
    const uint32_t* __restrict__ src, const uint32_t* __restrict__ dst,
    const uint16_t* __restrict__ dport, const uint32_t* __restrict__ host_id,
    const int32_t* __restrict__ pool_group, int64_t n_pool, int64_t n,
    int32_t* __restrict__ out_acl, int32_t* __restrict__ out_route,
    int32_t* __restrict__ out_group, uint8_t* __restrict__ out_allow, PipeCount pc, int shift) {
    extern __shared__ __attribute__((aligned(16))) uint32_t lds[];
    __shared__ uint32_t tally[5];
    const PipeLds L = pipe_lds_setup<kLds, kCount>(img, pc, lds, tally, shift);
    const AclV4Ctx a = acl_v4_ctx(img, kLds ? lds : nullptr, shift);
    int64_t lo, hi;
    pipe_slice(n, &lo, &hi);
    PipeTally t;
    if (!kVec) {
        for (int64_t i = lo + threadIdx.x; i < hi; i += blockDim.x)
            pipeline_one<kLds, kCount>(img, a, nodes, rb, proto, src, dst, dport, host_id, pool_group,
                                 n_pool, i, out_acl, out_route, out_group, out_allow, pc, L, &t);
    } else {
        for (int64_t i = lo + 4 * threadIdx.x; i + 3 < hi; i += 4 * blockDim.x) {
            const int64_t g = i >> 2;
            const uint4 d4 = stream_ld(reinterpret_cast<const uint4*>(dst) + g);
            const uint4 h4 = stream_ld(reinterpret_cast<const uint4*>(host_id) + g);
            const uint4 s4 = stream_ld(reinterpret_cast<const uint4*>(src) + g);
            const uint32_t pr = stream_ld(reinterpret_cast<const uint32_t*>(proto) + g);
            const uint2 pt = stream_ld(reinterpret_cast<const uint2*>(dport) + g);
            const uint32_t d[4] = {d4.x, d4.y, d4.z, d4.w};
            const uint32_t h[4] = {h4.x, h4.y, h4.z, h4.w};
            const uint32_t sk[4] = {s4.x, s4.y, s4.z, s4.w};
            const uint32_t po[4] = {pt.x & 0xFFFFu, pt.x >> 16, pt.y & 0xFFFFu, pt.y >> 16};
            uint32_t e[4];
            int32_t grp[4];
#pragma unroll
            for (int k = 0; k < 4; ++k) e[k] = nodes[d[k] >> (32 - rb)];
#pragma unroll
            for (int k = 0; k < 4; ++k) grp[k] = int64_t(h[k]) < n_pool ? pool_group[h[k]] : -1;
            uint32_t v[4];
            bool tcp[4];
#pragma unroll
            for (int k = 0; k < 4; ++k) tcp[k] = ((pr >> (8 * k)) & 0xFFu) == VC_PROTO_TCP;
            VC_PIPE_ACL4(a, tcp, sk, po, v);
            int4 oa, orr;
            uint32_t al = 0;
            int32_t* pa = reinterpret_cast<int32_t*>(&oa);
            int32_t* pr_ = reinterpret_cast<int32_t*>(&orr);
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                uint8_t b = 0;
                acl_emit(img, tcp[k], v[k], out_allow ? &b : nullptr, pa + k);
                al |= uint32_t(b) << (8 * k);
                pr_[k] = out_index(route_chase(nodes, rb, e[k], d[k]));
            }
            stream_st(reinterpret_cast<int4*>(out_acl) + g, oa);
            stream_st(reinterpret_cast<int4*>(out_route) + g, orr);
            stream_st(reinterpret_cast<int4*>(out_group) + g, make_int4(grp[0], grp[1], grp[2], grp[3]));
            if (out_allow) stream_st(reinterpret_cast<uint32_t*>(out_allow) + g, al);
            if (kCount) {
#pragma unroll
                for (int k = 0; k < 4; ++k)
                    pipe_count(pc, L.ah, L.rc, L.gc, tcp[k], v[k], false, pr_[k], grp[k], &t);
            }
        }
        // last partial group of 4 (only the final slice, when n % 4 != 0)
        const int64_t tail = hi & ~int64_t(3);
        if (hi == n && tail >= lo && int(threadIdx.x) < int(hi - tail))
            pipeline_one<kLds, kCount>(img, a, nodes, rb, proto, src, dst, dport, host_id, pool_group,
                                 n_pool, tail + threadIdx.x, out_acl, out_route, out_group,
                                 out_allow, pc, L, &t);
    }
    if (kCount) pipe_count_flush(pc, L.ah, L.rc, L.gc, tally, t);
}

// ---------------------------------------------------------------------------
// Mixed-family pipeline: per packet, `family` (4 or 6) is the `instanceof
// IPv4` dispatch of RouteTable.lookup (RouteTable.java:44-58) and of the
// caller's IP object: an IPv4 packet runs the v4 ACL projection and rulesV4,
// an IPv6 packet (IPv4-mapped ones included) the v6 ACL projection and
// rulesV6.  host_id may be absent (no hostname stage: group -1).
// ---------------------------------------------------------------------------
struct PipeIn {
    const uint8_t* family;         // null: every packet IPv4
    const uint8_t* proto;
    const uint32_t* src4;
    const uint32_t* dst4;
    const uint8_t* src6;           // 16 bytes per packet (or per IPv6 packet), 16-byte aligned
    const uint8_t* dst6;
    const uint16_t* dport;
    const uint32_t* host_id;       // null: no hostnames
    const int32_t* pool_group;
    int64_t n_pool;
    // compact IPv6 rows (kC6): base6[wave] = IPv6 packets before the wave's
    // sub-slice (pipe_wave_groups), n6c = rows in src6 / dst6
    const uint32_t* base6;
    int64_t n6c;
};

struct PipeOut {
    int32_t* acl;
    int32_t* route;
    int32_t* group;
    uint8_t* allow;
};

struct PipeTries {
    const uint32_t* n4;
    const uint32_t* n6;
    int32_t rb4, rb6;
    const uint32_t* w6;            // IPv6 wide root, or null
};

// First entry of an IPv6 packet's route walk: the wide root's answer for a
// one-prefix slot (one gather), else the root entry.
__device__ __forceinline__ uint32_t route6_first(const PipeTries& tr, uint64_t hh) {
    if (tr.w6) return wide_first(gather_ld(reinterpret_cast<const uint4*>(tr.w6) +
                                           (hh >> (64 - tr.rb6))), hh);
    return gather_ld(tr.n6 + (hh >> (64 - tr.rb6)));
}

template <bool kLds, bool kCount>
__device__ __forceinline__ void pipe_mix_one(const AclImage& img, const AclV4Ctx& a,
                                             const AclV6Ctx& a6, const PipeTries& tr,
                                             const PipeIn& in, int64_t i, const PipeOut& out,
                                             const PipeCount& pc, const PipeLds& L,
                                             PipeTally* t) {
    const bool v6 = in.family && in.family[i] == 6;
    const bool tcp = in.proto[i] == VC_PROTO_TCP;
    const uint32_t port = in.dport[i];
    int32_t grp = -1;
    if (in.host_id) {
        const uint32_t h = in.host_id[i];
        grp = int64_t(h) < in.n_pool ? in.pool_group[h] : -1;
    }
    uint32_t v, e;
    if (v6) {
        uint64_t hi, lo;
        v6_key(reinterpret_cast<const uint4*>(in.dst6)[i], &hi, &lo);
        e = route6_chase(tr.n6, tr.rb6, route6_first(tr, hi), hi, lo);
        v = acl_v6_any<kLds>(a, a6, tcp, reinterpret_cast<const uint4*>(in.src6)[i], port);
    } else {
        const uint32_t d = in.dst4[i];
        e = route_chase(tr.n4, tr.rb4, tr.n4[d >> (32 - tr.rb4)], d);
        v = acl_v4_one<kLds>(a, tcp, in.src4[i], port);
    }
    acl_emit(img, tcp, v, out.allow ? out.allow + i : nullptr, out.acl + i);
    const int32_t r = out_index(e);
    out.route[i] = r;
    out.group[i] = grp;
    if (kCount) pipe_count(pc, L.ah, L.rc, L.gc, tcp, v, v6, r, grp, t);
}

constexpr int kPipeWaves = kPipeBlock / 64;

// Cross-lane LDS exchange inside one wave (no workgroup barrier needed).
__device__ __forceinline__ void wave_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// Compact IPv6 rows (vc_pipeline_c6_dev): src6 / dst6 hold the addresses of
// the batch's IPv6 packets only, in packet order, so the k-th IPv6 packet's
// addresses are row k.  With a row per packet, an IPv6 packet's 32 address
// bytes sit in cache lines no IPv4 packet reads: at 15 % IPv6 the mixed
// kernel took ~2.6 more L2 misses per IPv6 packet than the IPv4 one and ran
// 15 % longer (profiles/r04_mix_v6frac.jsonl, pmc_traffic.json `mix`).
// Compact rows are read by consecutive lanes.  Each wave of the compact
// kernel takes a contiguous share of its workgroup's slice (not the 4096-
// packet interleave of the sparse form), so the rows it needs start at
// base6[wave], counted by pipe6_count_kernel + pipe6_scan_kernel first.
__device__ __forceinline__ void pipe_wave_groups(int64_t lo, int64_t hi, int w, int64_t* g0,
                                                 int64_t* g1) {
    const int64_t ng = (hi - lo + 3) >> 2;                 // groups of 4 packets
    const int64_t per = (ng + kPipeWaves - 1) / kPipeWaves;
    const int64_t a = int64_t(w) * per, b = a + per;
    *g0 = a < ng ? a : ng;
    *g1 = b < ng ? b : ng;
}

// IPv6 packets in each wave's share (launched with the pipeline's grid).
__global__ __launch_bounds__(kPipeBlock) void pipe6_count_kernel(const uint8_t* __restrict__ family,
                                                                 int64_t n, uint32_t* __restrict__ cnt) {
    int64_t lo, hi, g0, g1;
    pipe_slice(n, &lo, &hi);
    const int w = int(threadIdx.x >> 6), lane = int(threadIdx.x & 63);
    pipe_wave_groups(lo, hi, w, &g0, &g1);
    uint32_t c = 0;
    for (int64_t g = g0 + lane; g < g1; g += 64) {
        const int64_t i = lo + 4 * g;
        if (i + 3 < hi) {
            const uint32_t f = reinterpret_cast<const uint32_t*>(family)[i >> 2];
#pragma unroll
            for (int k = 0; k < 4; ++k) c += ((f >> (8 * k)) & 0xFFu) == 6;
        } else {
            for (int64_t j = i; j < hi; ++j) c += family[j] == 6;
        }
    }
#pragma unroll
    for (int d = 32; d > 0; d >>= 1) c += __shfl_xor(c, d, 64);
    if (lane == 0) cnt[int64_t(blockIdx.x) * kPipeWaves + w] = c;
}

// Exclusive scan of the m wave counts in place (one workgroup, m <= 4 * 1024).
__global__ __launch_bounds__(1024) void pipe6_scan_kernel(uint32_t* __restrict__ v, int m) {
    __shared__ uint32_t part[1024];
    uint32_t x[4], s = 0;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        const int j = int(threadIdx.x) * 4 + k;
        x[k] = j < m ? v[j] : 0u;
        s += x[k];
    }
    part[threadIdx.x] = s;
    __syncthreads();
    for (int off = 1; off < 1024; off <<= 1) {
        const uint32_t t = int(threadIdx.x) >= off ? part[threadIdx.x - off] : 0u;
        __syncthreads();
        part[threadIdx.x] += t;
        __syncthreads();
    }
    uint32_t run = part[threadIdx.x] - s;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        const int j = int(threadIdx.x) * 4 + k;
        if (j < m) v[j] = run;
        run += x[k];
    }
}

// One wave's share of the compact form: 256 packets (4 per lane) per step,
// the IPv6 ones queued in packet order so round r's lane l reads compact row
// base + (packets so far) + r * 64 + l -- consecutive rows, consecutive lanes.
template <bool kLds, bool kCount>
__device__ __forceinline__ void pipe_mix_c6(const AclImage& img, const AclV4Ctx& a,
                                            const AclV6Ctx& a6, const PipeTries& tr,
                                            const PipeIn& in, int64_t lo, int64_t hi,
                                            const PipeOut& out, const PipeCount& pc,
                                            const PipeLds& L, PipeTally* t, uint8_t* q6,
                                            uint32_t (*r6)[2]) {
    const int lane = int(threadIdx.x & 63), w = int(threadIdx.x >> 6);
    const uint64_t below_me = (uint64_t(1) << lane) - 1;
    int64_t g0, g1;
    pipe_wave_groups(lo, hi, w, &g0, &g1);
    int64_t row = in.base6[int64_t(blockIdx.x) * kPipeWaves + w];
    const int64_t last = in.n6c - 1;
    for (int64_t gb = g0; gb < g1; gb += 64) {            // uniform per wave
        const int64_t g = gb + lane;
        const int64_t i = lo + 4 * g;
        const bool full = g < g1 && i + 3 < hi;
        bool ok[4];
        uint32_t fm = 0, pr = 0, hh4[4] = {0, 0, 0, 0};
        uint32_t d[4] = {0, 0, 0, 0}, sk[4] = {0, 0, 0, 0}, po[4] = {0, 0, 0, 0};
        if (full) {
            const int64_t q = i >> 2;
            fm = c6_ld(reinterpret_cast<const uint32_t*>(in.family) + q);
            pr = c6_ld(reinterpret_cast<const uint32_t*>(in.proto) + q);
            const uint2 pt = c6_ld(reinterpret_cast<const uint2*>(in.dport) + q);
            const uint4 d4 = c6_ld(reinterpret_cast<const uint4*>(in.dst4) + q);
            const uint4 s4 = c6_ld(reinterpret_cast<const uint4*>(in.src4) + q);
            d[0] = d4.x; d[1] = d4.y; d[2] = d4.z; d[3] = d4.w;
            sk[0] = s4.x; sk[1] = s4.y; sk[2] = s4.z; sk[3] = s4.w;
            po[0] = pt.x & 0xFFFFu; po[1] = pt.x >> 16; po[2] = pt.y & 0xFFFFu; po[3] = pt.y >> 16;
            if (in.host_id) {
                const uint4 h4 = c6_ld(reinterpret_cast<const uint4*>(in.host_id) + q);
                hh4[0] = h4.x; hh4[1] = h4.y; hh4[2] = h4.z; hh4[3] = h4.w;
            }
#pragma unroll
            for (int k = 0; k < 4; ++k) ok[k] = true;
        } else {
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                ok[k] = g < g1 && i + k < hi;
                if (ok[k]) {
                    fm |= uint32_t(in.family[i + k]) << (8 * k);
                    pr |= uint32_t(in.proto[i + k]) << (8 * k);
                    d[k] = in.dst4[i + k];
                    sk[k] = in.src4[i + k];
                    po[k] = in.dport[i + k];
                    if (in.host_id) hh4[k] = in.host_id[i + k];
                }
            }
        }
        bool v6[4], tcp[4];
        uint32_t e[4], v[4];
        int32_t grp[4] = {-1, -1, -1, -1};
        int c = 0;
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            v6[k] = ok[k] && ((fm >> (8 * k)) & 0xFFu) == 6;
            tcp[k] = ((pr >> (8 * k)) & 0xFFu) == VC_PROTO_TCP;
            v[k] = VC_NONE;
            c += v6[k] ? 1 : 0;
        }
        // rank of each IPv6 packet among the step's IPv6 packets, packet order
        // (lane-major): the lanes below hold sum(c) of them (c <= 4: three
        // bit-plane ballots), then this lane's earlier slots
        const uint64_t b0 = __ballot(c & 1), b1 = __ballot(c & 2), b2 = __ballot(c & 4);
        const int before = __popcll(b0 & below_me) + 2 * __popcll(b1 & below_me) +
                           4 * __popcll(b2 & below_me);
        const int total = __popcll(b0) + 2 * __popcll(b1) + 4 * __popcll(b2);
        // the first round's rows are consecutive whatever packets they belong
        // to: issue them before the IPv4 gathers, so their latency hides
        // behind those.  Rows past n6c (a caller whose n6 is short) read the
        // last row, or the zero address when there is none: never memory
        // outside the rows.
        const uint4 z = make_uint4(0, 0, 0, 0);
        uint4 dw0 = z, sw0 = z;
        if (lane < total && last >= 0) {
            const int64_t k6 = row + lane;
            const int64_t rw = k6 < last ? k6 : last;
            dw0 = c6_ld(reinterpret_cast<const uint4*>(in.dst6) + rw);
            sw0 = c6_ld(reinterpret_cast<const uint4*>(in.src6) + rw);
        }
#pragma unroll
        for (int k = 0; k < 4; ++k)
            e[k] = ok[k] && !v6[k] ? gather_ld(tr.n4 + (d[k] >> (32 - tr.rb4))) : 0u;   // root gathers
        if (in.host_id) {
#pragma unroll
            for (int k = 0; k < 4; ++k)
                if (ok[k]) grp[k] = int64_t(hh4[k]) < in.n_pool ? gather_ld(in.pool_group + hh4[k]) : -1;
        }
        int pos[4];
        int r = before;
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            pos[k] = r;
            if (v6[k]) {
                q6[r] = uint8_t(lane * 4 + k);
                ++r;
            }
        }
        if (total) {                                      // wave-uniform
            wave_sync();
            const uint32_t pa = po[0] | po[1] << 16, pb = po[2] | po[3] << 16;
            for (int r0 = 0; r0 < total; r0 += 64) {
                // the queued packet's protocol and port come from the lane
                // that loaded them (three cross-lane reads), not from memory
                const int qe = r0 + lane < total ? int(q6[r0 + lane]) : 0;
                const int sl = qe >> 2, ks = qe & 3;
                const uint32_t prs = __shfl(pr, sl, 64);
                // every lane takes part in both reads (a lane outside a
                // divergent read's mask supplies no data to it)
                const uint32_t wa = __shfl(pa, sl, 64), wb = __shfl(pb, sl, 64);
                const uint32_t pw = ks < 2 ? wa : wb;
                if (r0 + lane < total) {
                    uint4 dw = dw0, sw = sw0;
                    if (r0 > 0 && last >= 0) {
                        const int64_t k6 = row + r0 + lane;
                        const int64_t rw = k6 < last ? k6 : last;
                        dw = c6_ld(reinterpret_cast<const uint4*>(in.dst6) + rw);
                        sw = c6_ld(reinterpret_cast<const uint4*>(in.src6) + rw);
                    }
                    const bool t6 = ((prs >> (8 * ks)) & 0xFFu) == VC_PROTO_TCP;
                    const uint32_t port6 = (ks & 1) ? pw >> 16 : pw & 0xFFFFu;
                    uint64_t hh, ll;
                    v6_key(dw, &hh, &ll);
                    const uint32_t root = route6_first(tr, hh);
                    const uint32_t vv = acl_v6_any<kLds>(a, a6, t6, sw, port6);
                    r6[lane][1] = route6_chase(tr.n6, tr.rb6, root, hh, ll);
                    r6[lane][0] = vv;
                }
                wave_sync();
#pragma unroll
                for (int k = 0; k < 4; ++k)
                    if (v6[k] && pos[k] >= r0 && pos[k] < r0 + 64) {
                        v[k] = r6[pos[k] - r0][0];
                        e[k] = r6[pos[k] - r0][1];
                    }
                wave_sync();
            }
            row += total;
        }
#pragma unroll
        for (int k = 0; k < 4; ++k)
            if (ok[k] && !v6[k]) v[k] = acl_v4_one<kLds>(a, tcp[k], sk[k], po[k]);
        int32_t oa[4], orr[4];
        uint8_t al[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            al[k] = 0;
            acl_emit(img, tcp[k], v[k], out.allow ? &al[k] : nullptr, &oa[k]);
            orr[k] = out_index(v6[k] || !ok[k] ? e[k] : route_chase(tr.n4, tr.rb4, e[k], d[k]));
        }
        if (full) {
            const int64_t q = i >> 2;
            c6_st(reinterpret_cast<int4*>(out.acl) + q, make_int4(oa[0], oa[1], oa[2], oa[3]));
            c6_st(reinterpret_cast<int4*>(out.route) + q, make_int4(orr[0], orr[1], orr[2], orr[3]));
            c6_st(reinterpret_cast<int4*>(out.group) + q, make_int4(grp[0], grp[1], grp[2], grp[3]));
            if (out.allow)
                c6_st(reinterpret_cast<uint32_t*>(out.allow) + q,
                      uint32_t(al[0]) | uint32_t(al[1]) << 8 | uint32_t(al[2]) << 16 |
                          uint32_t(al[3]) << 24);
        } else {
#pragma unroll
            for (int k = 0; k < 4; ++k)
                if (ok[k]) {
                    out.acl[i + k] = oa[k];
                    out.route[i + k] = orr[k];
                    out.group[i + k] = grp[k];
                    if (out.allow) out.allow[i + k] = al[k];
                }
        }
        if (kCount) {
#pragma unroll
            for (int k = 0; k < 4; ++k)
                if (ok[k]) pipe_count(pc, L.ah, L.rc, L.gc, tcp[k], v[k], v6[k], orr[k], grp[k], t);
        }
    }
}

// The vector path keeps IPv4 and IPv6 packets from diverging: a wave's 256
// packets (4 per lane) are classified by family with a ballot, the IPv6
// ones are queued in LDS and spread over all 64 lanes (one round per 64
// IPv6 packets), their results handed back through LDS, and only then does
// every lane finish its IPv4 packets.  Without it every wave ran the IPv6
// path (ACL search + trie walk) once per packet slot whenever any of its
// lanes had an IPv6 packet there -- i.e. always, at a 15 % IPv6 mix.
template <bool kLds, bool kVec, bool kCount, bool kC6 = false>
__global__ __launch_bounds__(kPipeBlock) void pipeline_mix_kernel(AclImage img, PipeTries tr,
                                                                   PipeIn in, int64_t n,
                                                                   PipeOut out, PipeCount pc,
                                                                   int fshift, int fence_words,
                                                                   int shift) {
    extern __shared__ __attribute__((aligned(16))) uint32_t lds[];
    __shared__ uint32_t tally[5];
    __shared__ uint8_t q6[kPipeWaves][256];        // queued IPv6 packets: lane * 4 + slot
    __shared__ uint32_t r6[kPipeWaves][64][2];     // per round: ACL value, route entry
    const AclV6Ctx a6 = stage_fences(img, reinterpret_cast<uint64_t*>(lds + fence_words), fshift);
    const PipeLds L = pipe_lds_setup<kLds, kCount>(img, pc, lds, tally, shift);
    __syncthreads();
    const AclV4Ctx a = acl_v4_ctx(img, kLds ? lds : nullptr, shift);
    int64_t lo, hi;
    pipe_slice(n, &lo, &hi);
    PipeTally t;
    if (kC6) {
        pipe_mix_c6<kLds, kCount>(img, a, a6, tr, in, lo, hi, out, pc, L, &t, q6[threadIdx.x >> 6],
                                  r6[threadIdx.x >> 6]);
    } else if (!kVec) {
        for (int64_t i = lo + threadIdx.x; i < hi; i += blockDim.x)
            pipe_mix_one<kLds, kCount>(img, a, a6, tr, in, i, out, pc, L, &t);
    } else {
        const int lane = int(threadIdx.x & 63), w = int(threadIdx.x >> 6);
        const uint64_t below_me = (uint64_t(1) << lane) - 1;
        const int64_t per_iter = 4 * int64_t(blockDim.x);
        const int64_t iters = (hi - lo + per_iter - 1) / per_iter;    // uniform
        for (int64_t it = 0; it < iters; ++it) {
            const int64_t i = lo + it * per_iter + 4 * int64_t(threadIdx.x);
            const bool act = i + 3 < hi;
            const int64_t g = i >> 2;
            uint32_t fm = 0x04040404u, pr = 0;
            uint2 pt = make_uint2(0, 0);
            uint4 d4 = make_uint4(0, 0, 0, 0), s4 = d4;
            if (act) {
                if (in.family) fm = reinterpret_cast<const uint32_t*>(in.family)[g];
                pr = reinterpret_cast<const uint32_t*>(in.proto)[g];
                pt = reinterpret_cast<const uint2*>(in.dport)[g];
                d4 = reinterpret_cast<const uint4*>(in.dst4)[g];
                s4 = reinterpret_cast<const uint4*>(in.src4)[g];
            }
            const uint32_t d[4] = {d4.x, d4.y, d4.z, d4.w};
            const uint32_t sk[4] = {s4.x, s4.y, s4.z, s4.w};
            const uint32_t po[4] = {pt.x & 0xFFFFu, pt.x >> 16, pt.y & 0xFFFFu, pt.y >> 16};
            bool v6[4], tcp[4];
            uint32_t e[4], v[4];
            int32_t grp[4] = {-1, -1, -1, -1};
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                v6[k] = act && ((fm >> (8 * k)) & 0xFFu) == 6;
                tcp[k] = ((pr >> (8 * k)) & 0xFFu) == VC_PROTO_TCP;
                e[k] = act && !v6[k] ? gather_ld(tr.n4 + (d[k] >> (32 - tr.rb4))) : 0u;   // root gathers
                v[k] = VC_NONE;
            }
            if (act && in.host_id) {
                const uint4 h4 = reinterpret_cast<const uint4*>(in.host_id)[g];
                const uint32_t h[4] = {h4.x, h4.y, h4.z, h4.w};
#pragma unroll
                for (int k = 0; k < 4; ++k)
                    grp[k] = int64_t(h[k]) < in.n_pool ? gather_ld(in.pool_group + h[k]) : -1;
            }
            // queue this wave's IPv6 packets (slot-major, then lane order)
            int pos[4];
            int total = 0;
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                const uint64_t m = __ballot(v6[k]);
                pos[k] = total + __popcll(m & below_me);
                total += __popcll(m);
                if (v6[k]) q6[w][pos[k]] = uint8_t(lane * 4 + k);
            }
            if (total) {                                  // wave-uniform
                wave_sync();
                const int64_t wbase = lo + it * per_iter + 256 * int64_t(w);
                for (int r0 = 0; r0 < total; r0 += 64) {
                    // protocol and port from the lane that loaded them
                    const int qe = r0 + lane < total ? int(q6[w][r0 + lane]) : 0;
                    const int sl = qe >> 2, ks = qe & 3;
                    const uint32_t prs = __shfl(pr, sl, 64);
                    const uint32_t wa = __shfl(pt.x, sl, 64), wb = __shfl(pt.y, sl, 64);
                    const uint32_t pw = ks < 2 ? wa : wb;
                    if (r0 + lane < total) {
                        const int64_t gi = wbase + qe;
                        const bool t6 = ((prs >> (8 * ks)) & 0xFFu) == VC_PROTO_TCP;
                        const uint32_t port6 = (ks & 1) ? pw >> 16 : pw & 0xFFFFu;
                        uint64_t hh, ll;
                        v6_key(reinterpret_cast<const uint4*>(in.dst6)[gi], &hh, &ll);
                        const uint32_t root = route6_first(tr, hh);
                        const uint32_t vv = acl_v6_any<kLds>(a, a6, t6,
                                                             reinterpret_cast<const uint4*>(in.src6)[gi],
                                                             port6);
                        r6[w][lane][1] = route6_chase(tr.n6, tr.rb6, root, hh, ll);
                        r6[w][lane][0] = vv;
                    }
                    wave_sync();
#pragma unroll
                    for (int k = 0; k < 4; ++k)
                        if (v6[k] && pos[k] >= r0 && pos[k] < r0 + 64) {
                            v[k] = r6[w][pos[k] - r0][0];
                            e[k] = r6[w][pos[k] - r0][1];
                        }
                    wave_sync();
                }
            }
            if (act) {
#pragma unroll
                for (int k = 0; k < 4; ++k)
                    if (!v6[k]) v[k] = acl_v4_one<kLds>(a, tcp[k], sk[k], po[k]);
                int4 oa, orr;
                uint32_t al = 0;
                int32_t* pa = reinterpret_cast<int32_t*>(&oa);
                int32_t* pr_ = reinterpret_cast<int32_t*>(&orr);
#pragma unroll
                for (int k = 0; k < 4; ++k) {
                    uint8_t b = 0;
                    acl_emit(img, tcp[k], v[k], out.allow ? &b : nullptr, pa + k);
                    al |= uint32_t(b) << (8 * k);
                    pr_[k] = out_index(v6[k] ? e[k] : route_chase(tr.n4, tr.rb4, e[k], d[k]));
                }
                reinterpret_cast<int4*>(out.acl)[g] = oa;
                reinterpret_cast<int4*>(out.route)[g] = orr;
                reinterpret_cast<int4*>(out.group)[g] = make_int4(grp[0], grp[1], grp[2], grp[3]);
                if (out.allow) reinterpret_cast<uint32_t*>(out.allow)[g] = al;
                if (kCount) {
#pragma unroll
                    for (int k = 0; k < 4; ++k)
                        pipe_count(pc, L.ah, L.rc, L.gc, tcp[k], v[k], v6[k], pr_[k], grp[k], &t);
                }
            }
        }
        const int64_t tail = hi & ~int64_t(3);
        if (hi == n && tail >= lo && int(threadIdx.x) < int(hi - tail))
            pipe_mix_one<kLds, kCount>(img, a, a6, tr, in, tail + threadIdx.x, out, pc, L, &t);
    }
    if (kCount) pipe_count_flush(pc, L.ah, L.rc, L.gc, tally, t);
}

}  // namespace vcd

namespace vc {

namespace {

// LDS budget for the staged v4 ACL boundaries (words); above it every
// (1 << shift)-th boundary is staged as a fence (acl_v4_one).
#ifndef VC_ACL_LDS_WORDS
#define VC_ACL_LDS_WORDS (30 * 1024)
#endif
constexpr int kLdsWords = VC_ACL_LDS_WORDS;

int vcd_fences(int nb, int shift) { return (nb + (1 << shift) - 1) >> shift; }

// Smallest fence shift whose staged v4 words fit `words`.
int v4_fence_shift(const AclImage& img, size_t words) {
    int shift = 0;
    while (size_t(vcd_fences(img.fam[0][0].nb, shift) + vcd_fences(img.fam[1][0].nb, shift)) >
               words && shift < 30)
        ++shift;
    return shift;
}

int v4_staged_words(const AclImage& img, int shift) {
    return vcd_fences(img.fam[0][0].nb, shift) + vcd_fences(img.fam[1][0].nb, shift);
}


}  // namespace

#ifndef VC_LDS_GRANULE
#define VC_LDS_GRANULE 1024
#endif

#if defined(VC_DEVCHECK)
hipError_t devcheck_take_classify(uint32_t out[4]);
hipError_t devcheck_take_hint(uint32_t out[4]);
hipError_t devcheck_take_packet(uint32_t out[4]);
hipError_t devcheck_take_mirror(uint32_t out[4]);
hipError_t devcheck_take_select(uint32_t out[4]);
hipError_t devcheck_take_counters(uint32_t out[4]);
#endif

hipError_t devcheck_take(uint32_t out[4]) {
    out[0] = out[1] = out[2] = out[3] = 0;
#if defined(VC_DEVCHECK)
    hipError_t (*const take[])(uint32_t*) = {devcheck_take_classify, devcheck_take_hint,
                                              devcheck_take_packet,   devcheck_take_mirror,
                                              devcheck_take_select,   devcheck_take_counters};
    for (auto f : take) {
        uint32_t w[4];
        const hipError_t e = f(w);
        if (e != hipSuccess) return e;
        if (w[0] && !out[0]) {
            out[0] = w[0];
            out[2] = w[2];
            out[3] = w[3];
        }
        out[1] += w[1];
    }
#endif
    return hipSuccess;
}

int resident_per_cu(const void* kernel, int block, size_t shmem) {
    static std::mutex mu;
    static std::map<std::pair<const void*, size_t>, int> cache;
    std::lock_guard<std::mutex> lk(mu);
    auto it = cache.find({kernel, shmem});
    if (it != cache.end()) return it->second;
    int per_cu = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, kernel, block, shmem) != hipSuccess ||
        per_cu < 1) {
        (void)hipGetLastError();
        per_cu = 1;
    }
    // LDS is handed out per workgroup in VC_LDS_GRANULE-byte units; the
    // occupancy query counts exact bytes, and a grid sized from it can hold a
    // second, partial round of workgroups that runs after the first
    hipFuncAttributes fa;
    int dev = 0, lds_cu = 0;
    if (hipFuncGetAttributes(&fa, kernel) == hipSuccess && hipGetDevice(&dev) == hipSuccess &&
        hipDeviceGetAttribute(&lds_cu, hipDeviceAttributeMaxSharedMemoryPerMultiprocessor, dev) ==
            hipSuccess) {
        const size_t g = VC_LDS_GRANULE;
        const size_t wg = (fa.sharedSizeBytes + shmem + g - 1) / g * g;
        if (wg > 0 && lds_cu > 0) per_cu = std::max(1, std::min(per_cu, int(size_t(lds_cu) / wg)));
    } else {
        (void)hipGetLastError();
    }
    cache[{kernel, shmem}] = per_cu;
    return per_cu;
}

namespace {

int grid_for(const LaunchCfg& c, int64_t work_items, int blocks_per_cu) {
    int64_t want = (work_items + vcd::kBlock - 1) / vcd::kBlock;
    int64_t cap = int64_t(c.num_cus) * blocks_per_cu;
    if (want < 1) want = 1;
    return int(want < cap ? want : cap);
}

bool aligned(const void* p, uintptr_t a) { return (reinterpret_cast<uintptr_t>(p) & (a - 1)) == 0; }

// LDS budget of the IPv6 ACL fences: blocks of at least 16 boundaries
constexpr size_t kFenceBytes = 40 * 1024;

int v6_fence_shift(const AclImage& img) {
    int shift = 4;
    auto bytes = [&](int s) {
        return size_t(vcd_fences(img.fam[0][1].nb, s) + vcd_fences(img.fam[1][1].nb, s)) * 16;
    };
    while (bytes(shift) > kFenceBytes && shift < 30) ++shift;
    return shift;
}

size_t v6_fence_bytes(const AclImage& img, int shift) {
    return std::max<size_t>(16, size_t(vcd_fences(img.fam[0][1].nb, shift) +
                                       vcd_fences(img.fam[1][1].nb, shift)) * 16);
}

// Dynamic LDS beyond 64 KiB must be opted into per kernel.  Keyed by the
// kernel's address: template instances share a function-pointer type.
template <class K>
hipError_t allow_lds(K kernel, size_t bytes = kLdsWords * 4) {
    return hipFuncSetAttribute(reinterpret_cast<const void*>(kernel),
                               hipFuncAttributeMaxDynamicSharedMemorySize, int(bytes));
}

}  // namespace

hipError_t launch_acl_v4(const LaunchCfg& c, const AclImage& img, const uint8_t* proto,
                         const uint32_t* src4, const uint16_t* port, int64_t n, int32_t* out,
                         uint8_t* allow, unsigned long long* counters) {
    if (n <= 0) return hipSuccess;
    const int shift = v4_fence_shift(img, kLdsWords);
    const int words = v4_staged_words(img, shift);
    const size_t shmem = size_t(words) * 4;
    const bool vec = aligned(proto, 4) && aligned(src4, 16) && aligned(port, 8) &&
                     aligned(out, 16) && (!allow || aligned(allow, 4));
    const int per_cu = words <= 16 * 1024 ? 4 : 2;
    if (vec) {
        // VC_ACL_QUADS quads per lane per pass once the batch fills every
        // lane that many times; a smaller batch takes one quad per lane
        // (a second quad past the end would be searched for nothing)
        const int64_t quads = n / 4;
        const int grid = grid_for(c, (n + 3) / 4, per_cu);
        const bool multi = quads >= int64_t(grid) * vcd::kBlock * VC_ACL_QUADS;
        const auto kern = multi ? vcd::acl_v4_kernel<true, VC_ACL_QUADS> : vcd::acl_v4_kernel<true, 1>;
        if (hipError_t e = allow_lds(kern)) return e;
        hipLaunchKernelGGL(kern, dim3(grid), dim3(vcd::kBlock), shmem, c.stream, img, shift, proto,
                           src4, port, n, out, allow);
    } else {
        const int grid = grid_for(c, n, per_cu);
        if (hipError_t e = allow_lds(vcd::acl_v4_kernel_scalar<true>)) return e;
        hipLaunchKernelGGL(vcd::acl_v4_kernel_scalar<true>, dim3(grid), dim3(vcd::kBlock),
                           shmem, c.stream, img, shift, proto, src4, port, n, out, allow);
    }
    hipError_t e = hipGetLastError();
    if (e != hipSuccess || !counters) return e;
    return launch_hist(c, VC_HIST_ACL, out, proto, n, int64_t(img.n_tcp) + img.n_udp, 0,
                       int64_t(img.n_tcp) + img.n_udp, img.n_tcp, counters);
}

hipError_t launch_acl_v6(const LaunchCfg& c, const AclImage& img, const uint8_t* proto,
                         const uint8_t* src6, const uint16_t* port, int64_t n, int32_t* out,
                         uint8_t* allow, unsigned long long* counters) {
    if (n <= 0) return hipSuccess;
    if (!aligned(src6, 16)) return hipErrorInvalidValue;
    const int shift = v6_fence_shift(img);
    const size_t shmem = v6_fence_bytes(img, shift);
    if (shmem > 64 * 1024)
        if (hipError_t e = allow_lds(vcd::acl_v6_kernel, shmem)) return e;
    hipLaunchKernelGGL(vcd::acl_v6_kernel, dim3(grid_for(c, n, 4)), dim3(vcd::kBlock), shmem,
                       c.stream, img, shift, proto, src6, port, n, out, allow);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess || !counters) return e;
    return launch_hist(c, VC_HIST_ACL, out, proto, n, int64_t(img.n_tcp) + img.n_udp, 0,
                       int64_t(img.n_tcp) + img.n_udp, img.n_tcp, counters);
}

hipError_t launch_route_v4(const LaunchCfg& c, const TrieImage& t, const uint32_t* dst4, int64_t n,
                           int32_t* out, unsigned long long* counters, int64_t rule_base,
                           int64_t none_at) {
    if (n <= 0) return hipSuccess;
    if (aligned(dst4, 16) && aligned(out, 16))
        hipLaunchKernelGGL(vcd::route_v4_kernel, dim3(grid_for(c, (n + 3) / 4, 8)),
                           dim3(vcd::kBlock), 0, c.stream, t.nodes, t.root_bits, dst4, n, out);
    else
        hipLaunchKernelGGL(vcd::route_v4_kernel_scalar, dim3(grid_for(c, n, 8)), dim3(vcd::kBlock),
                           0, c.stream, t.nodes, t.root_bits, dst4, n, out);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess || !counters) return e;
    return launch_hist(c, VC_HIST_PLAIN, out, nullptr, n, t.n_rules, rule_base, none_at, 0,
                       counters);
}

hipError_t launch_route_v6(const LaunchCfg& c, const TrieImage& t, const uint8_t* dst6, int64_t n,
                           int32_t* out, unsigned long long* counters, int64_t rule_base,
                           int64_t none_at) {
    if (n <= 0) return hipSuccess;
    if (!aligned(dst6, 16)) return hipErrorInvalidValue;
    if (aligned(out, 16))
        hipLaunchKernelGGL(vcd::route_v6_kernel_x4, dim3(grid_for(c, (n + 3) / 4, 8)),
                           dim3(vcd::kBlock), 0, c.stream, t.nodes, t.wide, t.root_bits, dst6, n,
                           out);
    else
        hipLaunchKernelGGL(vcd::route_v6_kernel, dim3(grid_for(c, n, 8)), dim3(vcd::kBlock), 0,
                           c.stream, t.nodes, t.wide, t.root_bits, dst6, n, out);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess || !counters) return e;
    return launch_hist(c, VC_HIST_PLAIN, out, nullptr, n, t.n_rules, rule_base, none_at, 0,
                       counters);
}

hipError_t build_wide_root(const uint32_t* nodes, int root_bits, uint32_t* wide,
                           hipStream_t stream) {
    const uint32_t slots = 1u << root_bits;
    const uint32_t blocks = std::min<uint32_t>((slots + vcd::kBlock - 1) / vcd::kBlock, 4096u);
    hipLaunchKernelGGL(vcd::wide_root_kernel, dim3(blocks), dim3(vcd::kBlock), 0, stream, nodes,
                       slots, reinterpret_cast<uint4*>(wide));
    return hipGetLastError();
}

hipError_t launch_pipeline(const LaunchCfg& c, const AclImage& acl, const RouteImage& route,
                           int32_t n4, int32_t n6, const PipeArgs& p, const PipeCounters& cnt,
                           hipEvent_t kernel_done, hipStream_t count_stream) {
    const int64_t n = p.n;
    if (n <= 0) return kernel_done ? hipEventRecord(kernel_done, c.stream) : hipSuccess;
    // the tuned C5 kernel: IPv4 packets with hostnames; everything else
    // (per-packet family, no hostname stage) runs the mixed kernel
    const bool mix = p.family != nullptr || p.host_id == nullptr;
    // LDS: the mixed kernel always stages the IPv6 ACL fences (and holds its
    // per-wave IPv6 queues statically); the v4 boundaries and the in-kernel
    // counts take what is left
    constexpr size_t kLdsMax = 160 * 1024 - 256;
    constexpr size_t kMixStatic = 13 * 1024;
    const int fshift = mix ? v6_fence_shift(acl) : 0;
    const size_t fbytes = mix ? v6_fence_bytes(acl, fshift) : 0;
    const size_t lds_max = mix ? kLdsMax - kMixStatic - fbytes : kLdsMax;
    // v4 boundaries (or their fences) always staged; the counts fit after
    const int shift = v4_fence_shift(acl, std::min<size_t>(kLdsWords, lds_max / 4));
    const int words = v4_staged_words(acl, shift);
    bool vec = aligned(p.proto, 4) && aligned(p.src4, 16) && aligned(p.dst4, 16) &&
               aligned(p.dport, 8) && aligned(p.host_id, 16) && aligned(p.out_acl, 16) &&
               aligned(p.out_route, 16) && aligned(p.out_group, 16) &&
               (!p.out_allow || aligned(p.out_allow, 4));
    if (mix) vec = vec && aligned(p.family, 4);
    // compact IPv6 rows: the wave shares of pipe_mix_c6 (vector loads for
    // whole groups of four)
    const bool c6 = mix && p.n6c >= 0;
    if (c6 && (!p.family || !vec)) return hipErrorInvalidValue;
    int64_t want = ((vec ? (n + 3) / 4 : n) + vcd::kPipeBlock - 1) / vcd::kPipeBlock;
    // Workgroups (one per CU): on an unmasked stream the IPv4 kernel takes 7/8
    // of the CUs (28 of each XCD's 32); a CU-masked stream's share is all its own.  Its rate is set by the chip's random-gather cap, which 224
    // CUs reach as well as 256 (4.78 vs 4.83 ms alone), and the CUs left over
    // run the counter finish of the previous batch beside it instead of
    // squeezing in between its workgroups: C5 6.12-6.14 ms/step against
    // 6.19-6.24 with all 256 (profiles/r03_ab_pipe_grid.jsonl).  VC_PIPE_GRID
    // overrides the count (A/B runs).
    static const int grid_cap = [] {
        const char* g = std::getenv("VC_PIPE_GRID");
        return g ? std::atoi(g) : 0;
    }();
    const int cus = grid_cap > 0 ? std::min(grid_cap, c.num_cus)
                  : (!mix && !c.cu_masked && c.num_cus >= 64 ? (c.num_cus * 7 / 8) & ~7
                                                                : c.num_cus);
    int grid = int(want < cus ? (want < 1 ? 1 : want) : cus);
    if (c6 && grid > 256) grid = 256;           // pipe6_scan_kernel: <= 4096 wave shares
    // In-kernel counting where it fits the workgroup's LDS; the rest is
    // counted by separate passes over the outputs afterwards.
    size_t shmem = size_t(words) * 4;
    vcd::PipeCount pc{};
    pc.bw_shift = big_hist_bucket_shift();
    pc.n4 = n4;
    const int64_t route_nval = int64_t(n4) + n6;     // combined [v4 rules][v6 rules]
    BigHist rh, gh;
    hipError_t e = hipSuccess;
    const int32_t acl_bins = acl.n_tcp + acl.n_udp;
    // one scratch lease for both large counter spaces, released on the
    // stream the finish passes run on
    const bool r_big = cnt.route && big_hist_applies(n, route_nval);
    const bool g_big = cnt.group && big_hist_applies(n, cnt.n_groups);
    const size_t rbytes = r_big ? big_hist_bytes(n, route_nval, grid) : 0;
    const size_t gbytes = g_big ? big_hist_bytes(n, cnt.n_groups, grid) : 0;
    const size_t bbytes = c6 ? (size_t(grid) * vcd::kPipeWaves * 4 + 255) & ~size_t(255) : 0;
    int slot = -1;
    uint8_t* scratch = nullptr;
    if (rbytes + gbytes + bbytes)
        e = c.scratch ? c.scratch->acquire(rbytes + gbytes + bbytes, c.stream, &slot, &scratch)
                      : hipErrorInvalidValue;
    uint32_t* base6 = c6 && e == hipSuccess
                          ? reinterpret_cast<uint32_t*>(scratch + rbytes + gbytes) : nullptr;
    if (c6 && e == hipSuccess) {
        hipLaunchKernelGGL(vcd::pipe6_count_kernel, dim3(grid), dim3(vcd::kPipeBlock), 0, c.stream,
                           p.family, n, base6);
        hipLaunchKernelGGL(vcd::pipe6_scan_kernel, dim3(1), dim3(1024), 0, c.stream, base6,
                           grid * vcd::kPipeWaves);
        e = hipGetLastError();
    }
    if (cnt.acl && shmem + size_t(acl_bins) * 4 <= lds_max) {
        pc.acl = cnt.acl;
        pc.acl_bins = acl_bins;
        pc.n_tcp = acl.n_tcp;
        shmem += size_t(acl_bins) * 4;
    }
    if (r_big && e == hipSuccess) {
        big_hist_begin(scratch, n, route_nval, grid, &rh);
        if (shmem + size_t(rh.nbk) * 4 <= lds_max) {
            pc.rcounts = rh.counts;
            pc.r_nbk = rh.nbk;
            pc.route = cnt.route;
            pc.route_none_at = route_nval;
            shmem += size_t(rh.nbk) * 4;
        }
    }
    if (g_big && e == hipSuccess) {
        big_hist_begin(scratch + rbytes, n, cnt.n_groups, grid, &gh);
        if (shmem + size_t(gh.nbk) * 4 <= lds_max) {
            pc.gcounts = gh.counts;
            pc.g_nbk = gh.nbk;
            pc.group = cnt.group;
            pc.n_groups = cnt.n_groups;
            shmem += size_t(gh.nbk) * 4;
        }
    }
    const bool count = pc.acl || pc.rcounts || pc.gcounts;
    const int fence_words = int((shmem / 4 + 3) & ~size_t(3));
    if (mix) shmem = size_t(fence_words) * 4 + fbytes;
    if (e == hipSuccess) {
        const TrieImage& r4 = route.fam[0];
#define VC_PIPE(L, V, K)                                                                           \
    do {                                                                                           \
        if (shmem > 64 * 1024) e = allow_lds(vcd::pipeline_v4_kernel<L, V, K>, kLdsMax);           \
        if (e != hipSuccess) break;                                                                \
        hipLaunchKernelGGL((vcd::pipeline_v4_kernel<L, V, K>), dim3(grid),                         \
                           dim3(vcd::kPipeBlock), shmem, c.stream, acl, r4.nodes, r4.root_bits,   \
                           p.proto, p.src4, p.dst4, p.dport, p.host_id, p.pool_group, p.n_pool,    \
                           n, p.out_acl, p.out_route, p.out_group, p.out_allow, pc, shift);        \
    } while (0)
#define VC_MIX(L, V, K, C6)                                                                        \
    do {                                                                                           \
        if (shmem > 64 * 1024)                                                                     \
            e = allow_lds(vcd::pipeline_mix_kernel<L, V, K, C6>, kLdsMax - kMixStatic);            \
        if (e != hipSuccess) break;                                                                \
        hipLaunchKernelGGL((vcd::pipeline_mix_kernel<L, V, K, C6>), dim3(grid),                    \
                           dim3(vcd::kPipeBlock), shmem, c.stream, acl, tr, in, n, out, pc,        \
                           fshift, fence_words, shift);                                            \
    } while (0)
        if (!mix) {
            if (count) {
                if (vec) VC_PIPE(true, true, true);
                else VC_PIPE(true, false, true);
            } else {
                if (vec) VC_PIPE(true, true, false);
                else VC_PIPE(true, false, false);
            }
        } else {
            const vcd::PipeTries tr{route.fam[0].nodes, route.fam[1].nodes, route.fam[0].root_bits,
                                    route.fam[1].root_bits, route.fam[1].wide};
            const vcd::PipeIn in{p.family, p.proto, p.src4, p.dst4, p.src6, p.dst6,
                                 p.dport, p.host_id, p.pool_group, p.n_pool, base6, p.n6c};
            const vcd::PipeOut out{p.out_acl, p.out_route, p.out_group, p.out_allow};
            if (c6) {
                if (count) VC_MIX(true, true, true, true);
                else VC_MIX(true, true, false, true);
            } else if (count) {
                if (vec) VC_MIX(true, true, true, false);
                else VC_MIX(true, false, true, false);
            } else {
                if (vec) VC_MIX(true, true, false, false);
                else VC_MIX(true, false, false, false);
            }
        }
#undef VC_PIPE
#undef VC_MIX
        if (e == hipSuccess) e = hipGetLastError();
        if (e == hipSuccess && kernel_done) e = hipEventRecord(kernel_done, c.stream);
    }
    // The second halves of the in-kernel counts, and whatever was not
    // counted inside, run on the counting stream when one is given (after
    // the kernel), so they overlap the caller's next batch.
    LaunchCfg cf = c;
    if (count_stream && count_stream != c.stream && (rh.counts || gh.counts || cnt.acl ||
                                                     cnt.route || cnt.group)) {
        const hipError_t e2 = c.handoff.ev ? c.handoff(c.stream, count_stream)
                                           : hipErrorInvalidValue;
        if (e2 == hipSuccess) cf.stream = count_stream;
        else if (e == hipSuccess) e = e2;
    }
    if (rh.counts) {
        const hipError_t e2 = big_hist_finish(cf, &rh, VC_HIST_ROUTE, p.out_route, p.family, n, n4,
                                              route_nval, 0, cnt.route,
                                              e == hipSuccess && pc.rcounts != nullptr);
        if (e == hipSuccess) e = e2;
    }
    if (gh.counts) {
        const hipError_t e2 = big_hist_finish(cf, &gh, VC_HIST_PLAIN, p.out_group, nullptr, n, 0,
                                              cnt.n_groups, 0, cnt.group,
                                              e == hipSuccess && pc.gcounts != nullptr);
        if (e == hipSuccess) e = e2;
    }
    if (slot >= 0) {
        const hipError_t e2 = c.scratch->release(slot, cf.stream);
        if (e == hipSuccess) e = e2;
    }
    if (e == hipSuccess && cnt.acl && !pc.acl)
        e = launch_hist(cf, VC_HIST_ACL, p.out_acl, p.proto, n, acl_bins, 0, acl_bins, acl.n_tcp,
                        cnt.acl);
    if (e == hipSuccess && cnt.route && !pc.rcounts)
        e = launch_hist(cf, VC_HIST_ROUTE, p.out_route, p.family, n, route_nval, 0, route_nval,
                        n4, cnt.route);
    if (e == hipSuccess && cnt.group && !pc.gcounts)
        e = launch_hist(cf, VC_HIST_PLAIN, p.out_group, nullptr, n, cnt.n_groups, 0,
                        cnt.n_groups, 0, cnt.group);
    return e;
}

}  // namespace vc

VC_DEVCHECK_READER(classify)
