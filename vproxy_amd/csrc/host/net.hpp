// net.hpp -- host-side IP / Network model (control plane of the classifier).
//
// Mirrors base/src/main/java/vfd/IP.java (literal parsers) and
// base/src/main/java/vproxybase/util/Network.java (mask bytes, validity,
// maskMatch, containment).  These run on the host only: rule parsing, the
// RouteTable insertion heuristic and the ACL projection compiler.
#pragma once

#include <array>
#include <cstdint>
#include <optional>
#include <string_view>

#include "vclassify.h"

namespace vc {

// A parsed IP literal: 4 or 16 bytes.
struct IpBytes {
    std::array<uint8_t, 16> b{};
    int len = 0;
};

// IP.parseIpv4String / parseIpv6String / parseIpString (IP.java:112-269).
std::optional<IpBytes> parse_ipv4(std::string_view s);
std::optional<IpBytes> parse_ipv6(std::string_view s);
std::optional<IpBytes> parse_ip(std::string_view s);
bool is_ipv6(std::string_view s);
bool is_ip_literal(std::string_view s);   // IP.isIpLiteral (IP.java:298-300)

// Network.parseMask (Network.java:101-133): 4 bytes if m <= 32 else 16.
// Returns mask length, or -1 when m > 128 (IllegalArgumentException).
int parse_mask(int m, uint8_t out[16]);
int mask_int(const uint8_t* mask, int mlen);                                // :135-145
bool valid_network(const uint8_t* a, int alen, const uint8_t* m, int mlen); // :163-181
bool mask_match(const uint8_t* in, int inlen, const uint8_t* rule, int rlen,
                const uint8_t* mask, int mlen);                             // :183-278

inline int net_prefix(const vc_net& n) { return mask_int(n.mask, n.mask_len); }
inline bool net_contains_ip(const vc_net& n, const uint8_t* ip, int iplen) {
    return mask_match(ip, iplen, n.ip, n.ip_len, n.mask, n.mask_len);
}
// Network.contains(Network) (Network.java:31-36)
inline bool net_contains_net(const vc_net& a, const vc_net& b) {
    return net_contains_ip(a, b.ip, b.ip_len) && net_prefix(a) < net_prefix(b);
}
bool net_equals(const vc_net& a, const vc_net& b);                          // :50-57
// Network(String) via validNetworkStr (Network.java:16-25,73-99)
bool net_parse(std::string_view s, vc_net* out);
bool net_from_prefix(const uint8_t* ip, int iplen, int prefix, vc_net* out);

// Java Integer.parseInt (decimal, optional sign, int32 range).
std::optional<int32_t> java_parse_int(std::string_view s);

}  // namespace vc
