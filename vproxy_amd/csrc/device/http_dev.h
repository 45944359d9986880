// http_dev.h -- the upstream group of an HTTP/1 request: HttpContext.connectionHint
// over the request head, then Upstream.searchForGroup.
//
//   HttpSubContext states 0-8   base/.../processor/http1/HttpSubContext.java:394-534
//   HttpContext.connectionHint  base/.../processor/http1/HttpContext.java:55-71
//   Hint.ofHost / ofUri / ofHostUri, formatHost / formatUri   Hint.java:17-90
//   Upstream.searchForGroup     core/.../svrgroup/Upstream.java:187-198
//
// One lane per request head.  The parser's fields come out as spans of the
// head: theUri = the request target (state 2) with its CR bytes dropped;
// theHostHeader = the last "host" header's value (state 7: CR dropped) with
// String.trim() -- stored only when a byte follows its line feed (state 8
// stores a header on the next byte).  Parsing stops at the empty line that
// ends the headers (state 9); bytes after it are not read.
//
// A string with a CR or a byte >= 0x80 is written out for the search -- CR
// bytes dropped and every byte >= 0x80 as the UTF-8 of the Java char
// (char) b = U+FF00 | b (EF, BC | b >> 6, 80 | b & 3F), as the compiled
// annotations hold Java strings in UTF-8 (the DNS path does the same,
// hint_dev.h) -- into the launch's rewrite space, in the region three times
// the span's offset; plain strings (nearly all) are searched in place.  The
// space comes from the context's own arena ring (capi.cpp http_scratch),
// which keeps one arena of the largest batch's size instead of growing the
// counter passes' four.
// Included once, at the end of hint.hip (hint_dev.h's out-of-line
// functions belong to that translation unit).
#pragma once

namespace vcd {

constexpr int kHttpBlock = 128;
constexpr int kHttpWaves = kHttpBlock / 64;   // two waves: 7 workgroups (14 waves) per CU in
                                                 // LDS against 3 x 4 with four (4.86 -> 4.59 ms)
constexpr uint32_t kHttpStage = 10240;     // bytes of heads staged per wave (64 heads)

// Byte i of an item in global memory through 16-byte aligned loads, one
// block cached.  An aligned block holding a byte of the item lies inside
// that byte's page, so the bytes around the item it also reads cannot
// fault.  (Used for chunks the stage cannot hold and for unaligned blobs.)
struct HeadCur {
    uintptr_t base;
    uintptr_t blk = ~uintptr_t(0);
    uint4 v{0, 0, 0, 0};
    __device__ __forceinline__ const uint8_t* ptr() const {
        return reinterpret_cast<const uint8_t*>(base);
    }
    __device__ __forceinline__ uint32_t at(int i) {
        const uintptr_t a = base + uintptr_t(i);
        const uintptr_t b = a & ~uintptr_t(15);
        if (b != blk) {
            blk = b;
            v = *reinterpret_cast<const uint4*>(b);
        }
        const uint32_t k = uint32_t(a >> 2) & 3u;
        const uint32_t w = k == 0 ? v.x : k == 1 ? v.y : k == 2 ? v.z : v.w;
        return (w >> (8u * uint32_t(a & 3))) & 0xFFu;
    }
};

// A head staged in the wave's LDS copy.
struct StagedCur {
    const uint8_t* p;
    const uint32_t* stage;                // the wave's stage (for LdsSrc)
    __device__ __forceinline__ const uint8_t* ptr() const { return p; }
    __device__ __forceinline__ uint32_t at(int i) { return p[i]; }
};

// First i' in [i, n) whose byte is x or y (n if none).  The generic form
// goes byte by byte; a staged head is read a dword at a time from LDS (the
// aligned dwords around a staged head lie inside the stage and its apron).
template <class Cur>
__device__ __forceinline__ int find2(Cur& c, int i, int n, uint32_t x, uint32_t y) {
    uint32_t b;
    while (i < n && (b = c.at(i)) != x && b != y) ++i;
    return i;
}

__device__ __forceinline__ int find2(StagedCur& c, int i, int n, uint32_t x, uint32_t y) {
    const uintptr_t base = reinterpret_cast<uintptr_t>(c.p);
    const uint32_t mx = x * 0x01010101u, my = y * 0x01010101u;
    while (i < n) {
        const uintptr_t a = base + uintptr_t(i);
        const uint32_t sh = uint32_t(a & 3);
        const uint32_t w = *reinterpret_cast<const uint32_t*>(a - sh) >> (8 * sh);
        // bytes of w equal to x or y: a zero byte of (w ^ mx) or (w ^ my)
        const uint32_t zx = w ^ mx, zy = w ^ my;
        const uint32_t hx = (zx - 0x01010101u) & ~zx & 0x80808080u;
        const uint32_t hy = (zy - 0x01010101u) & ~zy & 0x80808080u;
        // the shift brought in zero bytes above the 4 - sh valid ones
        const uint32_t valid = sh ? ((1u << (8 * (4 - sh))) - 1u) : ~0u;
        const uint32_t hit = (hx | hy) & valid;
        if (hit) {
            const int k = __builtin_ctz(hit) >> 3;
            return i + k < n ? i + k : n;
        }
        i += int(4 - sh);
    }
    return n;
}

// No CR and no byte >= 0x80 in [s, e)?  Generic: byte by byte; staged: a
// dword at a time.
template <class Cur>
__device__ __forceinline__ bool plain_span(Cur& c, int s, int e) {
    bool plain = true;
    for (int j = s; j < e; ++j) {
        const uint32_t b = c.at(j);
        plain = plain && b != '\r' && b < 0x80u;
    }
    return plain;
}

__device__ __forceinline__ bool plain_span(StagedCur& c, int s, int e) {
    const uintptr_t base = reinterpret_cast<uintptr_t>(c.p);
    uint32_t bad = 0;
    for (int j = s; j < e;) {
        const uintptr_t a = base + uintptr_t(j);
        const uint32_t sh = uint32_t(a & 3);
        const uint32_t w = *reinterpret_cast<const uint32_t*>(a - sh) >> (8 * sh);
        const int take = e - j < int(4 - sh) ? e - j : int(4 - sh);
        const uint32_t keep = take >= 4 ? ~0u : ((1u << (8 * take)) - 1u);
        const uint32_t z = w ^ 0x0D0D0D0Du;
        // a CR byte (zero byte of z; the lowest flag is exact and any flag
        // means one exists) or a high bit, among the kept bytes
        bad |= (((z - 0x01010101u) & ~z & 0x80808080u) | (w & 0x80808080u)) & keep;
        j += take;
    }
    return bad == 0;
}

struct HttpFields {
    int us = 0, ue = 0;        // theUri: [us, ue) minus CR
    int hs = 0, he = 0;        // theHostHeader: [hs, he) minus CR (already trimmed)
    bool uri = false, host = false;
};

__device__ __forceinline__ bool ws(uint32_t b) { return b <= 0x20u; }   // String.trim

// The request line and headers of one head (HttpSubContext states 0-8).
template <class Cur>
__device__ HttpFields http_fields(Cur& c, int n) {
    HttpFields f;
    int i = 0;
    i = find2(c, i, n, ' ', ' ');                   // state 1: method
    if (i >= n) return f;
    const int us = ++i;
    uint32_t b = 0;
    i = find2(c, i, n, ' ', '\n');                  // state 2: uri
    if (i >= n) return f;
    b = c.at(i);
    f.uri = true;
    f.us = us;
    f.ue = i;
    if (b == ' ')
        i = find2(c, i, n, '\n', '\n');             // state 3: version
    if (i >= n) return f;
    ++i;
    for (;;) {
        // states 4 / 8: CR ignored, LF ends the headers, else a key starts
        while (i < n && (b = c.at(i)) == '\r') ++i;
        if (i >= n || b == '\n') return f;
        const int ks = i;
        i = find2(c, i, n, ':', ':');                // state 5: the key runs to ':'
        if (i >= n) return f;
        const int ke = i++;
        const int vs = i;
        i = find2(c, i, n, '\n', '\n');             // state 7: value to LF
        if (i + 1 >= n) return f;                    // stored on the next byte (state 8)
        const int ve = i++;
        int a = ks, e = ke;                          // key.trim().toLowerCase() == "host"
        while (a < e && ws(c.at(a))) ++a;
        while (e > a && ws(c.at(e - 1))) --e;
        if (e - a == 4 && (c.at(a) | 0x20u) == 'h' && (c.at(a + 1) | 0x20u) == 'o' &&
            (c.at(a + 2) | 0x20u) == 's' && (c.at(a + 3) | 0x20u) == 't') {
            // value.trim() after state 7 dropped CR (itself <= ' ')
            int x = vs, y = ve;
            while (x < y && ws(c.at(x))) ++x;
            while (y > x && ws(c.at(y - 1))) --y;
            f.host = true;
            f.hs = x;
            f.he = y;
        }
    }
}

// The Java string of head bytes [s, e) minus CR: in place when plain ASCII
// without CR; else written to out (3 * (e - s) bytes at most) -- CR dropped
// and every byte >= 0x80 as the UTF-8 of the Java char (char) b =
// U+FF00 | b (EF, BC | b >> 6, 80 | b & 3F), as the compiled annotations
// hold Java strings in UTF-8 (the DNS path does the same, hint_dev.h).
template <class Cur>
__device__ DStr http_str(Cur& c, int s, int e, uint8_t* out) {
    if (plain_span(c, s, e)) return DStr{c.ptr() + s, e - s};
    int k = 0;
    for (int j = s; j < e; ++j) {
        const uint32_t b = c.at(j);
        if (b == '\r') continue;
        if (b < 0x80u) {
            out[k++] = uint8_t(b);
        } else {
            out[k++] = 0xEF;
            out[k++] = uint8_t(0xBC | (b >> 6));
            out[k++] = uint8_t(0x80 | (b & 0x3F));
        }
    }
    return DStr{out, k};
}

// Upstream.searchForGroup(hint), port 0.  With a uri (and hint-uris in the
// image): by levels (hint_port0_levels, round 6) -- only the top host
// level's keys are scored, the uri keys probed only without a host level.
__device__ __forceinline__ int32_t http_search(const HintImage& img, HeadCur&, DStr host,
                                               DStr uri) {
    if (uri.n >= 0 && img.has_uri_keys) return hint_port0_levels(img, host, uri.p, uri.n);
    return search_for_group(img, host, 0, uri);
}

__device__ __forceinline__ int32_t http_search(const HintImage& img, StagedCur&, DStr host,
                                               DStr uri) {
    if (uri.n >= 0 && img.has_uri_keys) return hint_port0_levels(img, host, uri.p, uri.n);
    return search_for_group(img, host, 0, uri);
}

// One head: (group, kind).  Rewritten strings go to the launch's scratch,
// in the region three times the span's blob offset `a + s`.
template <class Cur>
__device__ __forceinline__ int32_t http_one(const HintImage& img, Cur& c, int n, uint32_t a,
                                            int64_t blob_bytes, uint8_t* scratch,
                                            uint8_t* kind_out, int abl) {
    if (int64_t(a) + n > blob_bytes) {         // the scratch covers 3 * blob_bytes only
        *kind_out = VC_HTTP_BAD_SPAN;
        return -1;
    }
    const HttpFields f = http_fields(c, n);
    const uint8_t kind = uint8_t((f.host ? 2 : 0) | (f.uri ? 1 : 0));
    *kind_out = kind;
    if (!kind || abl == 1) return -1;
    // HttpContext.connectionHint: ofUri / ofHost / ofHostUri, port 0
    DStr host{nullptr, -1}, uri{nullptr, -1};
    if (f.host) host = format_host(http_str(c, f.hs, f.he, scratch + 3 * (int64_t(a) + f.hs)));
    if (f.uri) uri = format_uri(http_str(c, f.us, f.ue, scratch + 3 * (int64_t(a) + f.us)));
    if (abl == 2) return host.n + uri.n;
    if (abl == 3) return search_for_group(img, host, 0, DStr{nullptr, -1});   // host only
    if (abl == 4) return search_for_group(img, DStr{nullptr, -1}, 0, uri);    // uri only
    return http_search(img, c, host, uri);
}

// kStage: each wave takes 64 consecutive heads at a time and copies their
// bytes into its LDS stage with coalesced loads (stage.h), so a lane walks
// its head in LDS: reading each head from global memory lane by lane made
// the wave wait on a load whenever any lane crossed into a new 16-byte
// block -- nearly every byte.  A chunk whose heads exceed the stage is read
// from global memory.  The blob must be dword aligned (launch_http_hint).
template <bool kStage>
__global__ __launch_bounds__(kHttpBlock) void http_hint_kernel(
    HintImage img, const uint8_t* __restrict__ blob, const uint32_t* __restrict__ off, int64_t n,
    int64_t blob_bytes, uint8_t* __restrict__ scratch, int32_t* __restrict__ out_group,
    uint8_t* __restrict__ out_kind, int abl) {
    __shared__ uint32_t stage[kStage ? kHttpWaves : 1][kStage ? (kHttpStage + 2 * kApron) / 4 : 1];
    const int lane = int(threadIdx.x & 63), w = int(threadIdx.x >> 6);
    const int64_t nchunks = (n + 63) / 64;
    const int64_t waves = int64_t(gridDim.x) * kHttpWaves;
    for (int64_t ch = int64_t(blockIdx.x) * kHttpWaves + w; ch < nchunks; ch += waves) {
        const int64_t base = ch * 64, i = base + lane;
        const LaneSpan sp = lane_span(off, base, n);
        uint32_t o0, o1, a0 = 0;
        span_of(sp, base, n, &o0, &o1);
        const bool staged = kStage && stage_wave<kHttpStage>(blob, o0, o1, stage[w], &a0);
        uint8_t kind = 0;
        int32_t g = -1;
        if (i < n) {
            if (staged) {
                StagedCur c{reinterpret_cast<const uint8_t*>(stage[w]) + kApron + (sp.a - a0),
                            stage[w]};
                g = http_one(img, c, int(sp.e - sp.a), sp.a, blob_bytes, scratch, &kind, abl);
            } else {
                HeadCur c{reinterpret_cast<uintptr_t>(blob + sp.a)};
                g = http_one(img, c, int(sp.e - sp.a), sp.a, blob_bytes, scratch, &kind, abl);
            }
            out_group[i] = g;
            if (out_kind) out_kind[i] = kind;
        }
        if (kStage) wave_done();
    }
}

}  // namespace vcd

namespace vc {

hipError_t launch_http_hint(const LaunchCfg& c, const HintImage& img, const uint8_t* blob,
                            int64_t blob_bytes, const uint32_t* off, int64_t n, int32_t* out_group,
                            uint8_t* out_kind) {
    if (n <= 0) return hipSuccess;
    int slot = -1;
    uint8_t* scratch = nullptr;
    ScratchRing* ring = c.http_scratch ? c.http_scratch : c.scratch;
    hipError_t e = ring ? ring->acquire(size_t(blob_bytes > 0 ? blob_bytes : 1) * 3, c.stream,
                                        &slot, &scratch)
                        : hipErrorInvalidValue;
    if (e != hipSuccess) return e;
    // timing-only ablations, in a build with -DVC_ABL_HTTP=k only: 1 parse
    // only, 2 parse + copies, no search, 3 search with the host alone, 4 with
    // the uri alone
#if defined(VC_ABL_HTTP)
    const int abl = VC_ABL_HTTP;
#else
    const int abl = 0;
#endif
    const int64_t want = (n + 64 * vcd::kHttpWaves - 1) / (64 * vcd::kHttpWaves);
    auto go = [&](auto kernel) {
        const int grid = resident_grid(c, reinterpret_cast<const void*>(kernel), vcd::kHttpBlock,
                                       0, want);
        hipLaunchKernelGGL(kernel, dim3(grid), dim3(vcd::kHttpBlock), 0, c.stream, img, blob, off,
                           n, blob_bytes, scratch, out_group, out_kind, abl);
    };
    // -DVC_HTTP_NOSTAGE (measurement builds only): every chunk through the
    // global-memory path
#if defined(VC_HTTP_NOSTAGE)
    const bool nostage = true;
#else
    const bool nostage = false;
#endif
    if ((reinterpret_cast<uintptr_t>(blob) & 3) == 0 && !nostage) go(vcd::http_hint_kernel<true>);
    else go(vcd::http_hint_kernel<false>);
    e = hipGetLastError();
    const hipError_t e2 = ring->release(slot, c.stream);
    return e != hipSuccess ? e : e2;
}

}  // namespace vc
