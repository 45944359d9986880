// net.cpp -- see net.hpp.  Java semantics over ASCII bytes.
#include "net.hpp"

#include "../common/netmatch.h"

#include <cstring>
#include <vector>

namespace vc {
namespace {

// Utils.split (Utils.java:162-177): split on a literal, keep empty pieces.
std::vector<std::string_view> jsplit(std::string_view s, std::string_view sep) {
    std::vector<std::string_view> out;
    size_t last = 0;
    for (;;) {
        size_t idx = s.find(sep, last);
        if (idx == std::string_view::npos) {
            out.push_back(s.substr(last));
            return out;
        }
        out.push_back(s.substr(last, idx - last));
        last = idx + sep.size();
    }
}

bool is_hex(char c) {
    return (c >= '0' && c <= '9') || (c >= 'a' && c <= 'f') || (c >= 'A' && c <= 'F');
}
int hexv(char c) {
    if (c <= '9') return c - '0';
    if (c >= 'a') return c - 'a' + 10;
    return c - 'A' + 10;
}

// IP.parseIpv4String(String, byte[], int) (IP.java:129-155)
int v4_into(std::string_view s, uint8_t* bytes, int cap, int from) {
    auto parts = jsplit(s, ".");
    if (parts.size() != 4) return -1;
    for (size_t i = 0; i < parts.size(); ++i) {
        int idx = from + static_cast<int>(i);
        if (idx >= cap) return -1;
        std::string_view p = parts[i];
        if (p.size() > 3 || p.empty()) return -1;
        int num = 0;
        for (char c : p) {
            if (c < '0' || c > '9') return -1;
            num = num * 10 + (c - '0');
        }
        if (p[0] == '0' && p.size() > 1) return -1;
        if (num > 255) return -1;
        bytes[idx] = static_cast<uint8_t>(num);
    }
    return 4;
}

// IP.parseIpv6ColonPart (IP.java:200-248); `present` false == Java null
int v6_colon_part(bool present, std::string_view s, uint8_t* bytes, int from) {
    if (!present || s.empty()) return 0;
    if (from < 0) return -1;
    auto fields = jsplit(s, ":");
    for (size_t i = 0; i < fields.size(); ++i) {
        int base = from + 2 * static_cast<int>(i);
        if (base >= 16) return -1;
        std::string_view f = fields[i];
        if (f.size() > 4 || f.empty()) return -1;
        for (char c : f)
            if (!is_hex(c)) return -1;
        int v = 0;
        for (char c : f) v = v * 16 + hexv(c);
        if (f.size() >= 3) bytes[base] = static_cast<uint8_t>(v >> 8);
        bytes[base + 1] = static_cast<uint8_t>(v & 0xFF);
    }
    return static_cast<int>(fields.size()) * 2;
}

// IP.parseIpv6LastBits (IP.java:251-269), including the `4 + (-1)` quirk.
int v6_last_bits(std::string_view s, uint8_t* bytes) {
    size_t dot = s.find('.');
    if (dot != std::string_view::npos) {
        size_t colon = s.rfind(':', dot);
        if (colon == std::string_view::npos) return v4_into(s, bytes, 16, 12);
        std::string_view cpart = s.substr(0, colon);
        if (v4_into(s.substr(colon + 1), bytes, 16, 12) == -1) return -1;
        int pieces = static_cast<int>(jsplit(cpart, ":").size());
        return 4 + v6_colon_part(true, cpart, bytes, 16 - 4 - pieces * 2);
    }
    int pieces = static_cast<int>(jsplit(s, ":").size());
    return v6_colon_part(true, s, bytes, 16 - pieces * 2);
}

}  // namespace

std::optional<IpBytes> parse_ipv4(std::string_view s) {
    IpBytes r;
    if (v4_into(s, r.b.data(), 4, 0) == -1) return std::nullopt;
    r.len = 4;
    return r;
}

std::optional<IpBytes> parse_ipv6(std::string_view s) {
    if (s.size() >= 2 && s.front() == '[' && s.back() == ']') s = s.substr(1, s.size() - 2);
    if (jsplit(s, "::").size() - 1 > 1) return std::nullopt;
    size_t idx = s.find("::");
    bool dbl = idx != std::string_view::npos;
    std::string_view colon_only = dbl ? s.substr(0, idx) : std::string_view();
    std::string_view colon_dot = dbl ? s.substr(idx + 2) : s;
    IpBytes r;
    int c1 = v6_colon_part(dbl, colon_only, r.b.data(), 0);
    if (c1 == -1) return std::nullopt;
    int c2 = v6_last_bits(colon_dot, r.b.data());
    if (c2 == -1) return std::nullopt;
    if (dbl ? (c1 + c2 >= 16) : (c1 + c2 != 16)) return std::nullopt;
    r.len = 16;
    return r;
}

std::optional<IpBytes> parse_ip(std::string_view s) {
    if (s.find(':') != std::string_view::npos) return parse_ipv6(s);
    return parse_ipv4(s);
}

bool is_ipv6(std::string_view s) { return parse_ipv6(s).has_value(); }

bool is_ip_literal(std::string_view s) {
    // isIpv4 || isIpv6 (IP.java:271-300) reduces to: v6 parses || v4 parses
    return parse_ipv6(s).has_value() || parse_ipv4(s).has_value();
}

int parse_mask(int m, uint8_t out[16]) {
    if (m > 128) return -1;
    int len = m > 32 ? 16 : 4;
    for (int i = 0; i < len; ++i, m -= 8) {
        int ones = m > 8 ? 8 : m;                       // Utils.getByte: <=0 -> 0
        out[i] = ones <= 0 ? 0 : static_cast<uint8_t>(0xFF00u >> ones);
    }
    return len;
}

int mask_int(const uint8_t* mask, int mlen) {
    int zeros = 0;
    for (int i = mlen - 1; i >= 0; --i) {
        uint8_t b = mask[i];
        int tz = b == 0 ? 8 : __builtin_ctz(b);            // Utils.zeros
        if (tz == 0) break;
        zeros += tz;
    }
    return mlen * 8 - zeros;
}

bool valid_network(const uint8_t* a, int alen, const uint8_t* m, int mlen) {
    if (alen < mlen) return false;
    for (int i = 0; i < mlen; ++i)
        if ((a[i] & m[i]) != a[i]) return false;
    for (int i = mlen; i < alen; ++i)
        if (a[i] != 0) return false;
    return true;
}

bool mask_match(const uint8_t* in, int inlen, const uint8_t* rule, int rlen,
                const uint8_t* mask, int mlen) {
    // lengths other than 4 / 16 never occur in a Network or an IP
    if ((inlen != 4 && inlen != 16) || (rlen != 4 && rlen != 16) || (mlen != 4 && mlen != 16))
        return false;
    return vcn::mask_match(vcn::addr_of(in, inlen), vcn::addr_of(rule, rlen),
                           vcn::addr_of(mask, mlen));
}

bool net_equals(const vc_net& a, const vc_net& b) {
    return a.ip_len == b.ip_len && a.mask_len == b.mask_len &&
           std::memcmp(a.ip, b.ip, a.ip_len) == 0 && std::memcmp(a.mask, b.mask, a.mask_len) == 0;
}

std::optional<int32_t> java_parse_int(std::string_view s) {
    if (s.empty()) return std::nullopt;
    size_t k = 0;
    bool neg = false;
    if (s[0] == '-' || s[0] == '+') {
        neg = s[0] == '-';
        k = 1;
    }
    if (k >= s.size()) return std::nullopt;
    int64_t v = 0;
    for (; k < s.size(); ++k) {
        if (s[k] < '0' || s[k] > '9') return std::nullopt;
        v = v * 10 + (s[k] - '0');
        if (v > 2147483648LL) return std::nullopt;
    }
    if (neg) v = -v;
    if (v > 2147483647LL) return std::nullopt;
    return static_cast<int32_t>(v);
}

bool net_from_prefix(const uint8_t* ip, int iplen, int prefix, vc_net* out) {
    if (iplen != 4 && iplen != 16) return false;
    vc_net n{};
    int ml = parse_mask(prefix, n.mask);
    if (ml < 0) return false;
    std::memcpy(n.ip, ip, iplen);
    if (!valid_network(n.ip, iplen, n.mask, ml)) return false;
    n.ip_len = iplen;
    n.mask_len = ml;
    *out = n;
    return true;
}

bool net_parse(std::string_view s, vc_net* out) {
    // validNetworkStr: contains "/", split("/") has exactly 2 pieces
    size_t slash = s.find('/');
    if (slash == std::string_view::npos) return false;
    if (s.find('/', slash + 1) != std::string_view::npos) return false;
    if (slash == 0 || slash + 1 == s.size()) return false;   // String.split drops trailing empty
    auto m = java_parse_int(s.substr(slash + 1));
    if (!m) return false;
    auto ip = parse_ip(s.substr(0, slash));
    if (!ip) return false;
    return net_from_prefix(ip->b.data(), ip->len, *m, out);
}

}  // namespace vc
