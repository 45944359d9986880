// mirror.cpp -- see mirror.hpp.
#include "mirror.hpp"

#include <algorithm>
#include <cstring>
#include <unordered_map>
#include <unordered_set>

#include "net.hpp"

namespace vc {

// ---------------------------------------------------------------------------
// SecurityGroup
// ---------------------------------------------------------------------------
int SecurityGroup::add_rule(SecurityGroupRule r) {
    for (auto* lst : {&tcp_, &udp_})
        for (auto& x : *lst)
            if (x.alias == r.alias) return VC_EEXIST;               // :57-58
    auto& rules = r.protocol == VC_PROTO_TCP ? tcp_ : udp_;
    for (auto& x : rules)                                            // :67-74
        if (net_equals(x.network, r.network) && x.protocol == r.protocol &&
            x.min_port == r.min_port && x.max_port == r.max_port)
            return VC_EEXIST;
    rules.push_back(std::move(r));                                   // :75 (append)
    return VC_OK;
}

int SecurityGroup::remove_rule(std::string_view alias) {
    for (auto* lst : {&tcp_, &udp_}) {
        auto it = std::find_if(lst->begin(), lst->end(),
                               [&](const SecurityGroupRule& x) { return x.alias == alias; });
        if (it != lst->end()) {
            lst->erase(it);
            return VC_OK;
        }
    }
    return VC_ENOTFOUND;
}

// ---------------------------------------------------------------------------
// RouteTable
// ---------------------------------------------------------------------------
RouteTable::RouteTable(const vc_net& v4net, const vc_net* v6net, int vni) : vni_(vni) {
    has_default_v4_ = true;
    default_v4_.alias = "default";
    default_v4_.rule = v4net;
    default_v4_.to_vni = vni;
    v4_.push_back(default_v4_);
    if (v6net) {
        has_default_v6_ = true;
        default_v6_.alias = "default-v6";
        default_v6_.rule = *v6net;
        default_v6_.to_vni = vni;
        v6_.push_back(default_v6_);
    }
}

namespace {
bool rule_equals(const RouteRule& a, const RouteRule& b) {   // RouteRule.equals :209-218
    return a.to_vni == b.to_vni && a.alias == b.alias && net_equals(a.rule, b.rule) &&
           a.has_ip == b.has_ip &&
           (!a.has_ip || (a.ip_len == b.ip_len && std::memcmp(a.ip, b.ip, a.ip_len) == 0));
}
}  // namespace

int RouteTable::validate(const RouteRule& r) const {
    for (auto* lst : {&v4_, &v6_})
        for (auto& rr : *lst) {
            if (rr.alias == r.alias) return VC_EEXIST;               // :70-72
            if (net_equals(rr.rule, r.rule)) return VC_EEXIST;       // :73-75
        }
    if (r.alias == "default" && !(has_default_v4_ && rule_equals(r, default_v4_)))
        return VC_EXEXC;                                             // :86-89
    if (r.alias == "default-v6" && !(has_default_v6_ && rule_equals(r, default_v6_)))
        return VC_EXEXC;                                             // :90-93
    if (r.has_ip) {                                                  // :94-101
        if (!has_default_v6_ && r.ip_len == 16) return VC_EXEXC;
        // (a table built with RouteTable() has no default rule: Java would
        // NPE here; we report the validation failure instead)
        if (!has_default_v4_) return VC_EXEXC;
        if (!net_contains_ip(default_v4_.rule, r.ip, r.ip_len) &&
            (!has_default_v6_ || !net_contains_ip(default_v6_.rule, r.ip, r.ip_len)))
            return VC_EXEXC;
    }
    return VC_OK;
}

// RouteTable.addRule(RouteRule, List) -- the insertion-order heuristic, :110-154
void RouteTable::insert_ordered(const RouteRule& r, std::vector<RouteRule>& rules) {
    const int n = static_cast<int>(rules.size());
    int similar = -1;
    for (int i = 0; i < n; ++i)
        if (net_contains_net(rules[i].rule, r.rule) || net_contains_net(r.rule, rules[i].rule)) {
            similar = i;
            break;
        }
    if (similar == -1) {
        rules.push_back(r);
        return;
    }
    int at = 0;
    for (int i = similar; i < n; ++i) {
        const vc_net& curr = rules[i].rule;
        if (net_contains_net(curr, r.rule)) { at = i; break; }
        if (net_contains_net(r.rule, curr)) {
            if (i + 1 >= n) { at = i + 1; break; }
            const vc_net& next = rules[i + 1].rule;
            if (net_contains_net(r.rule, next)) continue;
            if (net_contains_net(next, r.rule)) { at = i + 1; break; }
        }
        at = i + 1;
        break;
    }
    rules.insert(rules.begin() + at, r);
}

int RouteTable::add_rule(const RouteRule& r) {
    int rc = validate(r);
    if (rc != VC_OK) return rc;
    insert_ordered(r, r.rule.ip_len == 4 ? v4_ : v6_);
    return VC_OK;
}

namespace {

struct PKey {
    uint64_t hi, lo;
    int len;
    int fam;   // 4 or 16: Network.equals compares the ip byte arrays, so families never collide
    bool operator==(const PKey& o) const {
        return hi == o.hi && lo == o.lo && len == o.len && fam == o.fam;
    }
};
struct PKeyHash {
    size_t operator()(const PKey& k) const {
        uint64_t h = k.hi * 0x9E3779B97F4A7C15ull ^
                     (k.lo + 0x632BE59BD9B4E019ull + (uint64_t)k.len + ((uint64_t)k.fam << 8));
        h ^= h >> 29;
        h *= 0xBF58476D1CE4E5B9ull;
        return static_cast<size_t>(h ^ (h >> 32));
    }
};

// Prefix key (network bits, length) of a rule as laid out in its family list.
PKey key_of(const vc_net& n) {
    uint8_t b[16] = {};
    std::memcpy(b, n.ip, n.ip_len);
    uint64_t hi = 0, lo = 0;
    for (int i = 0; i < 8; ++i) hi = (hi << 8) | b[i];
    for (int i = 8; i < 16; ++i) lo = (lo << 8) | b[i];
    if (n.ip_len == 4) hi = (hi >> 32) << 32;   // v4 keys live in the top 32 bits
    return PKey{hi, lo, mask_int(n.mask, n.mask_len), n.ip_len};
}

PKey truncate(const PKey& k, int len) {
    PKey r{0, 0, len, k.fam};
    if (len >= 64) {
        r.hi = k.hi;
        r.lo = len == 128 ? k.lo : (len == 64 ? 0 : (k.lo & ~(~0ull >> (len - 64))));
    } else {
        r.hi = len == 0 ? 0 : (k.hi & ~(~0ull >> len));
    }
    return r;
}

// Final list order for a shortest-first insertion sequence (SURVEY.md §8(a)
// R7): each rule lands immediately before its most specific container, so
// the list is the post-order of the containment forest with children in
// insertion order.  `seq` is in insertion order with non-decreasing length.
std::vector<RouteRule> postorder_build(std::vector<RouteRule> seq) {
    const int n = static_cast<int>(seq.size());
    std::unordered_map<PKey, int, PKeyHash> present;
    present.reserve(static_cast<size_t>(n) * 2);
    std::vector<int> parent(n, -1);
    uint64_t lens_present[3] = {0, 0, 0};   // bitset of present prefix lengths 0..128
    for (int i = 0; i < n; ++i) {
        PKey k = key_of(seq[i].rule);
        for (int l = k.len - 1; l >= 0; --l) {
            if (!((lens_present[l >> 6] >> (l & 63)) & 1)) continue;
            auto it = present.find(truncate(k, l));
            if (it != present.end()) {
                parent[i] = it->second;
                break;
            }
        }
        present.emplace(k, i);
        lens_present[k.len >> 6] |= 1ull << (k.len & 63);
    }
    // children lists in insertion order (CSR)
    std::vector<int> cnt(n + 1, 0), roots;
    for (int i = 0; i < n; ++i) {
        if (parent[i] < 0) roots.push_back(i);
        else cnt[parent[i] + 1]++;
    }
    for (int i = 0; i < n; ++i) cnt[i + 1] += cnt[i];
    std::vector<int> child(cnt[n]), fill(cnt.begin(), cnt.end() - 1);
    for (int i = 0; i < n; ++i)
        if (parent[i] >= 0) child[fill[parent[i]]++] = i;
    std::vector<RouteRule> out;
    out.reserve(n);
    std::vector<std::pair<int, int>> stack;   // (node, next child cursor)
    for (int root : roots) {
        stack.emplace_back(root, cnt[root]);
        while (!stack.empty()) {
            auto& top = stack.back();
            if (top.second < cnt[top.first + 1]) {
                int c = child[top.second++];
                stack.emplace_back(c, cnt[c]);
            } else {
                out.push_back(std::move(seq[top.first]));
                stack.pop_back();
            }
        }
    }
    return out;
}

}  // namespace

int RouteTable::add_rules_bulk(std::vector<RouteRule> rules) {
    // Fast path: per family, (existing list + new rules) must form a
    // shortest-first insertion sequence from an empty list, and no
    // validation may fail.  Otherwise insert one by one (exact heuristic).
    bool fast = true;
    std::unordered_set<std::string> aliases;
    std::unordered_set<PKey, PKeyHash> nets;
    for (auto* lst : {&v4_, &v6_})
        for (auto& r : *lst) {
            aliases.insert(r.alias);
            nets.insert(key_of(r.rule));
        }
    int last_len[2] = {-1, -1};
    for (auto* lst : {&v4_, &v6_}) {
        int f = lst == &v4_ ? 0 : 1;
        if (lst->size() > 1) fast = false;
        for (auto& r : *lst) last_len[f] = std::max(last_len[f], net_prefix(r.rule));
    }
    for (auto& r : rules) {
        if (!fast) break;
        int f = r.rule.ip_len == 4 ? 0 : 1;
        int len = net_prefix(r.rule);
        if (r.has_ip || r.alias == "default" || r.alias == "default-v6") fast = false;
        if (len < last_len[f]) fast = false;
        last_len[f] = len;
        if (!aliases.insert(r.alias).second) fast = false;
        if (!nets.insert(key_of(r.rule)).second) fast = false;
    }
    if (!fast) {
        for (auto& r : rules) {
            int rc = add_rule(r);
            if (rc != VC_OK) return rc;
        }
        return VC_OK;
    }
    // (the bulk path reports 1 so callers/tests can tell which path ran)
    std::vector<RouteRule> s4(v4_.begin(), v4_.end()), s6(v6_.begin(), v6_.end());
    for (auto& r : rules) (r.rule.ip_len == 4 ? s4 : s6).push_back(std::move(r));
    v4_ = postorder_build(std::move(s4));
    v6_ = postorder_build(std::move(s6));
    return 1;
}

int RouteTable::del_rule(std::string_view alias) {
    for (auto* lst : {&v4_, &v6_}) {
        for (size_t i = 0; i < lst->size(); ++i)
            if ((*lst)[i].alias == alias) {
                lst->erase(lst->begin() + static_cast<long>(i));
                return VC_OK;
            }
    }
    return VC_ENOTFOUND;
}

// ---------------------------------------------------------------------------
// Resolver.getHosts (Resolver.java:62-153)
// ---------------------------------------------------------------------------
namespace {
bool java_ws(char c) {
    return c == ' ' || c == '\t' || c == '\n' || c == 0x0B || c == '\f' || c == '\r' ||
           (c >= 0x1C && c <= 0x1F);
}
std::string_view jtrim(std::string_view s) {
    while (!s.empty() && static_cast<unsigned char>(s.front()) <= ' ') s.remove_prefix(1);
    while (!s.empty() && static_cast<unsigned char>(s.back()) <= ' ') s.remove_suffix(1);
    return s;
}
}  // namespace

std::vector<HostsEntry> parse_hosts_text(std::string_view text) {
    std::vector<HostsEntry> out;
    std::unordered_set<std::string> keys;
    int lines = 0;
    size_t pos = 0;
    while (pos < text.size()) {
        size_t end = pos;
        while (end < text.size() && text[end] != '\n' && text[end] != '\r') ++end;
        std::string_view line = text.substr(pos, end - pos);
        pos = end + 1;
        if (end < text.size() && text[end] == '\r' && pos < text.size() && text[pos] == '\n') ++pos;

        size_t hash = line.find('#');
        if (hash != std::string_view::npos) line = line.substr(0, hash);
        if (std::all_of(line.begin(), line.end(), java_ws)) continue;
        line = jtrim(line);
        std::vector<std::string_view> tok;
        size_t s = 0;
        for (size_t i = 0; i <= line.size(); ++i)
            if (i == line.size() || line[i] == ' ' || line[i] == '\t') {
                auto t = jtrim(line.substr(s, i - s));
                if (!t.empty()) tok.push_back(t);
                s = i + 1;
            }
        if (tok.size() < 2) continue;
        if (!parse_ip(tok[0])) continue;
        int entry = lines++;
        for (size_t i = 1; i < tok.size(); ++i) {
            std::string d1(tok[i]);
            std::string d2 = d1.back() == '.' ? d1.substr(0, d1.size() - 1) : d1 + ".";
            if (keys.count(d1) || keys.count(d2)) continue;
            keys.insert(d1);
            keys.insert(d2);
            out.push_back({d1, entry});
            out.push_back({d2, entry});
        }
    }
    return out;
}

}  // namespace vc
