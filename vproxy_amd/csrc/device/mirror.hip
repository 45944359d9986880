// mirror.hip -- traffic-mirror filter kernels (see mirror_dev.h).
//
// One lane per item.  An origin with 1..64 filters is matched through its
// bit-set image (images.h MirrorSwImage): one interval
// search per address (and per port) gives every filter's network (port)
// match at once, the MAC and protocol lists are uniform loops through the
// scalar cache.  Other origins take the per-filter loop: the list is read by
// every lane of a wave at the same address, through the scalar cache into
// SGPRs (mirror_dev.h load_filter), so its branches are scalar.
#include "launch.h"
#include "mirror_dev.h"
#include "chunks.h"
#include "stage.h"

namespace vcd {

constexpr int kMirrorBlock = 256;
// kSw: the origin's bit-set image (mirror_match_sw), else every filter in
// turn (mirror_eval).  kL: its three interval tables (at most kMatchL
// intervals each) copied into LDS first.
constexpr int kMatchL = 128;
template <bool kSw, bool kL>
__global__ __launch_bounds__(kMirrorBlock) void mirror_match_kernel(
    MirrorImage img, MirrorSwImage sw, int32_t origin, vc_mirror_items in, int64_t n,
    uint64_t* __restrict__ out) {
    __shared__ uint32_t l4b[kL ? kMatchL : 1], lpb[kL ? kMatchL : 1];
    __shared__ ulonglong2 l4p[kL ? kMatchL : 1], l6b[kL ? kMatchL : 1], l6p[kL ? kMatchL : 1],
        lpp[kL ? kMatchL : 1], lmp[kL ? kMatchL : 1];
    __shared__ uint64_t lmb[kL ? kMatchL : 1];
    const MirrorImage& fi = img;
    SwTables tb = sw_tables(sw);
    if (kL) {
        const int t = int(threadIdx.x);
        typedef const ulonglong2* P2;
        if (t < sw.nb4) {
            l4b[t] = glb_ld(sw.b4 + t);
            l4p[t] = glb_ld(reinterpret_cast<P2>(sw.p4) + t);
        }
        if (t < sw.nb6) {
            l6b[t] = glb_ld(reinterpret_cast<P2>(sw.b6) + t);
            l6p[t] = glb_ld(reinterpret_cast<P2>(sw.p6) + t);
        }
        if (t < sw.nbp) {
            lpb[t] = glb_ld(sw.bp + t);
            lpp[t] = glb_ld(reinterpret_cast<P2>(sw.pp) + t);
        }
        if (t < sw.nbm) {
            lmb[t] = glb_ld(sw.bm + t);
            lmp[t] = glb_ld(reinterpret_cast<P2>(sw.pm) + t);
        }
        __syncthreads();
        typedef const uint64_t* P1;
        tb = SwTables{l4b, reinterpret_cast<P1>(l4p), reinterpret_cast<P1>(l6b),
                      reinterpret_cast<P1>(l6p), lpb, reinterpret_cast<P1>(lpp), lmb,
                      reinterpret_cast<P1>(lmp)};
    }
    const int64_t stride = int64_t(gridDim.x) * blockDim.x;
    for (int64_t i = int64_t(blockIdx.x) * blockDim.x + threadIdx.x; i < n; i += stride) {
        const MirrorItem it = mirror_item(in, i);
        out[i] = kSw ? mirror_match_sw<kL>(sw, tb, it, mirror_level(it))
                     : mirror_eval(fi, origin, it, mirror_level(it));
    }
}
static_assert(kMatchL <= kMirrorBlock, "one copy pass per workgroup");

// Frames staged per wave in LDS as in packet.hip (kStage), parsed from there.
constexpr int kMirrorWaves = kMirrorBlock / 64;
constexpr uint32_t kMirrorStage = 7168;      // as packet.hip kPktStage: 5 blocks per CU
constexpr uint32_t kMirrorStageWords = (kMirrorStage + 2 * kApron) / 4;

// kSw: the origin's filters as bit sets (MirrorSwImage, mirror_switch_sw);
// otherwise every filter of the list in turn (mirror_switch_one).  kL: the
// interval tables (at most kMirrorL intervals per family) copied into LDS
// first -- with 48 + 48 the kernel keeps its 5 workgroups per CU.
constexpr int kMirrorL = 48;
static_assert(kMirrorL <= kMirrorBlock, "one copy pass per workgroup");
template <bool kStage, bool kSw, bool kL>
__global__ __launch_bounds__(kMirrorBlock) void mirror_switch_kernel(
    MirrorImage img, MirrorSwImage sw, int32_t origin, const uint8_t* __restrict__ blob,
    const uint32_t* __restrict__ off, int64_t n, int layer, uint64_t* __restrict__ out,
    uint32_t* __restrict__ ticket) {
    __shared__ uint32_t stage[kStage ? kMirrorWaves : 1][kStage ? kMirrorStageWords : 1];
    __shared__ uint32_t l4b[kL ? kMirrorL : 1];
    __shared__ ulonglong2 l4p[kL ? kMirrorL : 1], l6b[kL ? kMirrorL : 1], l6p[kL ? kMirrorL : 1];
    const MirrorImage& fi = img;
    const int lane = int(threadIdx.x & 63), w = int(threadIdx.x >> 6);
    SwTables tb = sw_tables(sw);
    if (kL) {
        const int t = int(threadIdx.x);
        if (t < sw.nb4) {
            l4b[t] = glb_ld(sw.b4 + t);
            l4p[t] = glb_ld(reinterpret_cast<const ulonglong2*>(sw.p4) + t);
        }
        if (t < sw.nb6) {
            l6b[t] = glb_ld(reinterpret_cast<const ulonglong2*>(sw.b6) + t);
            l6p[t] = glb_ld(reinterpret_cast<const ulonglong2*>(sw.p6) + t);
        }
        __syncthreads();
        tb = SwTables{l4b, reinterpret_cast<const uint64_t*>(l4p),
                      reinterpret_cast<const uint64_t*>(l6b), reinterpret_cast<const uint64_t*>(l6p),
                      sw.bp, sw.pp, sw.bm, sw.pm};
    }
    ChunksT<kPerTicket, kTailChunks, kTailRounds, 25> ch(ticket, (n + 63) / 64);   // chunks.h
    int64_t c = ch.first(w);
    LaneSpan cur = c < ch.nchunks ? lane_span(off, c * 64, n) : LaneSpan{0, 0};
    while (c < ch.nchunks) {
        const int64_t base = c * 64;
        const int64_t i = base + lane;
        uint32_t o0, o1, a0 = 0;
        span_of(cur, base, n, &o0, &o1);
        const uint32_t a = cur.a, e = cur.e;
        const int64_t nx = ch.next(c);
        if (nx < ch.nchunks) cur = lane_span(off, nx * 64, n);             // next chunk's
        const bool staged = kStage && stage_wave<kMirrorStage>(blob, o0, o1, stage[w], &a0);
        if (i < n) {
            const uint8_t* fp =
                staged ? reinterpret_cast<const uint8_t*>(stage[w]) + kApron + (a - a0) : blob + a;
            out[i] = kSw ? mirror_switch_sw<kL>(sw, tb, fp, int(e - a), layer)
                         : mirror_switch_one(fi, origin, fp, int(e - a), layer);
        }
        if (kStage) wave_done();
        c = nx;
    }
}

}  // namespace vcd

namespace vc {

namespace {
template <class K>
int mirror_grid(const LaunchCfg& c, K kernel, int64_t n) {
    return resident_grid(c, reinterpret_cast<const void*>(kernel), vcd::kMirrorBlock, 0,
                         (n + vcd::kMirrorBlock - 1) / vcd::kMirrorBlock);
}
}  // namespace

hipError_t launch_mirror_match(const LaunchCfg& c, const MirrorImage& img,
                               const MirrorSwImage* sw, int32_t origin, const vc_mirror_items& in,
                               int64_t n, uint64_t* out) {
    if (n <= 0) return hipSuccess;
    const MirrorSwImage none{};
    auto go = [&](auto kernel, const MirrorSwImage& s) {
        hipLaunchKernelGGL(kernel, dim3(mirror_grid(c, kernel, n)), dim3(vcd::kMirrorBlock), 0,
                           c.stream, img, s, origin, in, n, out);
    };
    if (sw && sw->lds && sw->nb4 <= vcd::kMatchL && sw->nb6 <= vcd::kMatchL &&
        sw->nbp <= vcd::kMatchL && sw->nbm <= vcd::kMatchL)
        go(vcd::mirror_match_kernel<true, true>, *sw);
    else if (sw) go(vcd::mirror_match_kernel<true, false>, *sw);
    else go(vcd::mirror_match_kernel<false, false>, none);
    return hipGetLastError();
}

namespace {
template <bool kStage, bool kSw, bool kL = false>
void mirror_switch_go(const LaunchCfg& c, const MirrorImage& img, const MirrorSwImage& sw,
                      int32_t origin, const uint8_t* blob, const uint32_t* off, int64_t n,
                      int layer, uint64_t* out) {
    const auto k = vcd::mirror_switch_kernel<kStage, kSw, kL>;
    hipLaunchKernelGGL(k, dim3(mirror_grid(c, k, n)), dim3(vcd::kMirrorBlock), 0, c.stream, img,
                       sw, origin, blob, off, n, layer, out, launch_ticket(c));
}
}  // namespace

// sw: the origin's bit-set image, or null for the per-filter kernel
hipError_t launch_mirror_switch(const LaunchCfg& c, const MirrorImage& img,
                                const MirrorSwImage* sw, int32_t origin, const uint8_t* blob,
                                const uint32_t* off, int64_t n, int layer, uint64_t* out) {
    if (n <= 0) return hipSuccess;
    const bool stage = (reinterpret_cast<uintptr_t>(blob) & 3) == 0;
    const MirrorSwImage none{};
    if (sw && stage && sw->lds && sw->nb4 <= vcd::kMirrorL && sw->nb6 <= vcd::kMirrorL)
        mirror_switch_go<true, true, true>(c, img, *sw, origin, blob, off, n, layer, out);
    else if (sw && stage) mirror_switch_go<true, true>(c, img, *sw, origin, blob, off, n, layer, out);
    else if (sw) mirror_switch_go<false, true>(c, img, *sw, origin, blob, off, n, layer, out);
    else if (stage) mirror_switch_go<true, false>(c, img, none, origin, blob, off, n, layer, out);
    else mirror_switch_go<false, false>(c, img, none, origin, blob, off, n, layer, out);
    return hipGetLastError();
}

}  // namespace vc

VC_DEVCHECK_READER(mirror)
