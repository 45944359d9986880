// mirror.hpp -- host-side mirrors of the reference's rule containers.
//
// They keep rule lists in exactly the order the Java code would, because
// list order is the priority the GPU tables encode:
//   SecurityGroup  core/src/main/java/vproxy/component/secure/SecurityGroup.java
//   RouteTable     core/src/main/java/vswitch/RouteTable.java
//   hosts file     base/src/main/java/vproxybase/dns/Resolver.java:62-153
#pragma once

#include <cstdint>
#include <string>
#include <string_view>
#include <vector>

#include "vclassify.h"

namespace vc {

struct SecurityGroupRule {
    std::string alias;
    vc_net network;
    int protocol;      // VC_PROTO_TCP / VC_PROTO_UDP
    int32_t min_port, max_port;
    bool allow;
};

class SecurityGroup {
public:
    SecurityGroup(std::string alias, bool default_allow)
        : alias_(std::move(alias)), default_allow_(default_allow) {}
    const std::string& alias() const { return alias_; }
    bool default_allow() const { return default_allow_; }
    void set_default_allow(bool v) { default_allow_ = v; }
    int add_rule(SecurityGroupRule r);                 // SecurityGroup.java:56-83
    int remove_rule(std::string_view alias);           // SecurityGroup.java:85-103
    const std::vector<SecurityGroupRule>& tcp() const { return tcp_; }
    const std::vector<SecurityGroupRule>& udp() const { return udp_; }

private:
    std::string alias_;
    bool default_allow_;
    std::vector<SecurityGroupRule> tcp_, udp_;
};

struct RouteRule {
    std::string alias;
    vc_net rule;
    int to_vni = 0;
    bool has_ip = false;
    uint8_t ip[16] = {};
    int ip_len = 0;
};

class RouteTable {
public:
    RouteTable() = default;                                              // :25-28
    RouteTable(const vc_net& v4net, const vc_net* v6net, int vni);      // :30-42
    int add_rule(const RouteRule& r);                                   // :68-108
    int add_rules_bulk(std::vector<RouteRule> rules);                   // same result, fast path
    int del_rule(std::string_view alias);                               // :156-172
    const std::vector<RouteRule>& v4() const { return v4_; }
    const std::vector<RouteRule>& v6() const { return v6_; }
    int vni() const { return vni_; }                                     // Table.vni

private:
    int validate(const RouteRule& r) const;
    static void insert_ordered(const RouteRule& r, std::vector<RouteRule>& rules);  // :110-154
    bool has_default_v4_ = false, has_default_v6_ = false;
    RouteRule default_v4_, default_v6_;
    std::vector<RouteRule> v4_, v6_;
    int vni_ = 0;
};

// Resolver.getHosts over file text: map entries in insertion order.
struct HostsEntry {
    std::string key;
    int32_t value;  // index of the accepted host line
};
std::vector<HostsEntry> parse_hosts_text(std::string_view text);

}  // namespace vc
