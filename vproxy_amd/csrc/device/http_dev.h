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
// A span that is plain ASCII with no CR inside is matched in place.  Any
// other is rewritten first into the launch's scratch, in the region three
// times the span's offset: CR bytes dropped and every byte >= 0x80 as the
// UTF-8 of the Java char (char) b = U+FF00 | b (EF, BC | b >> 6,
// 80 | b & 3F), as the compiled annotations hold Java strings in UTF-8
// (the DNS path does the same, hint_dev.h).
// Included once, at the end of hint.hip (hint_dev.h's out-of-line
// functions belong to that translation unit).
#pragma once

namespace vcd {

constexpr int kHttpBlock = 256;

// Byte i of an item through 16-byte aligned loads, one block cached.  An
// aligned block holding a byte of the item lies inside that byte's page, so
// the bytes around the item it also reads cannot fault.
struct HeadCur {
    uintptr_t base;
    uintptr_t blk = ~uintptr_t(0);
    uint4 v{0, 0, 0, 0};
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

struct HttpFields {
    int us = 0, ue = 0;        // theUri: [us, ue) minus CR
    int hs = 0, he = 0;        // theHostHeader: [hs, he) minus CR (already trimmed)
    bool uri = false, host = false;
};

__device__ __forceinline__ bool ws(uint32_t b) { return b <= 0x20u; }   // String.trim

// The request line and headers of one head (HttpSubContext states 0-8).
__device__ HttpFields http_fields(HeadCur& c, int n) {
    HttpFields f;
    int i = 0;
    while (i < n && c.at(i) != ' ') ++i;             // state 1: method
    if (i >= n) return f;
    const int us = ++i;
    uint32_t b = 0;
    while (i < n && (b = c.at(i)) != ' ' && b != '\n') ++i;   // state 2: uri
    if (i >= n) return f;
    f.uri = true;
    f.us = us;
    f.ue = i;
    if (b == ' ')
        while (i < n && c.at(i) != '\n') ++i;        // state 3: version
    if (i >= n) return f;
    ++i;
    for (;;) {
        // states 4 / 8: CR ignored, LF ends the headers, else a key starts
        while (i < n && (b = c.at(i)) == '\r') ++i;
        if (i >= n || b == '\n') return f;
        const int ks = i;
        while (i < n && c.at(i) != ':') ++i;         // state 5: the key runs to ':'
        if (i >= n) return f;
        const int ke = i++;
        const int vs = i;
        while (i < n && c.at(i) != '\n') ++i;        // state 7: value to LF
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
// without CR, else rewritten into out (3 * (e - s) bytes at most).
__device__ DStr http_str(HeadCur& c, const uint8_t* head, int s, int e, uint8_t* out) {
    bool plain = true;
    for (int j = s; j < e; ++j) {
        const uint32_t b = c.at(j);
        if (b == '\r' || b >= 0x80u) plain = false;
    }
    if (plain) return DStr{head + s, e - s};
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

__global__ __launch_bounds__(kHttpBlock) void http_hint_kernel(
    HintImage img, const uint8_t* __restrict__ blob, const uint32_t* __restrict__ off, int64_t n,
    uint8_t* __restrict__ scratch, int32_t* __restrict__ out_group, uint8_t* __restrict__ out_kind) {
    for (int64_t i = int64_t(blockIdx.x) * blockDim.x + threadIdx.x; i < n;
         i += int64_t(gridDim.x) * blockDim.x) {
        const uint32_t a = off[i], z = off[i + 1];
        const uint8_t* head = blob + a;
        HeadCur c{reinterpret_cast<uintptr_t>(head)};
        const HttpFields f = http_fields(c, int(z - a));
        const uint8_t kind = uint8_t((f.host ? 2 : 0) | (f.uri ? 1 : 0));
        int32_t g = -1;
        if (kind) {
            // HttpContext.connectionHint: ofUri / ofHost / ofHostUri, port 0
            DStr host{nullptr, -1}, uri{nullptr, -1};
            if (f.host)
                host = format_host(http_str(c, head, f.hs, f.he, scratch + 3 * (int64_t(a) + f.hs)));
            if (f.uri)
                uri = format_uri(http_str(c, head, f.us, f.ue, scratch + 3 * (int64_t(a) + f.us)));
            g = search_for_group(img, host, 0, uri);
        }
        out_group[i] = g;
        if (out_kind) out_kind[i] = kind;
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
    hipError_t e = c.scratch ? c.scratch->acquire(size_t(blob_bytes > 0 ? blob_bytes : 1) * 3,
                                                  c.stream, &slot, &scratch)
                             : hipErrorInvalidValue;
    if (e != hipSuccess) return e;
    const int64_t want = (n + vcd::kHttpBlock - 1) / vcd::kHttpBlock;
    const int grid = resident_grid(c, reinterpret_cast<const void*>(vcd::http_hint_kernel),
                                   vcd::kHttpBlock, 0, want);
    hipLaunchKernelGGL(vcd::http_hint_kernel, dim3(grid), dim3(vcd::kHttpBlock), 0, c.stream, img,
                       blob, off, n, scratch, out_group, out_kind);
    e = hipGetLastError();
    const hipError_t e2 = c.scratch->release(slot, c.stream);
    return e != hipSuccess ? e : e2;
}

}  // namespace vc
