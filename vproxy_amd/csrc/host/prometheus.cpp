// prometheus.cpp -- hit counters in vproxy's Prometheus text format
// (SURVEY.md §8(f) row 4), host only.
//
//   Metrics.toString        base/src/main/java/vproxybase/prometheus/Metrics.java:27-64
//   Metric (label quoting,  base/src/main/java/vproxybase/prometheus/Metric.java:15-25
//     sorted label keys)    quoting = vjson SimpleString.stringify (JSON string escape)
//   Counter.value()         base/src/main/java/vproxybase/prometheus/Counter.java:19-21
//   getExtraLabels          base/src/main/java/vproxybase/GlobalInspection.java:95-116
//   addMetric               base/src/main/java/vproxybase/GlobalInspection.java:118-125
#include "prometheus.hpp"

#include <algorithm>
#include <cstdio>
#include <cstring>

#include "vclassify.h"

namespace vc {

namespace {

// JSON string escape: printable ASCII as is except '"' and '\\'; the short
// escapes; every other char as \uXXXX (a byte >= 128 as the Latin-1 char).
std::string json_quote(const std::string& s) {
    std::string o = "\"";
    char buf[8];
    for (unsigned char c : s) {
        if (c > 31 && c < 127) {
            if (c == '"') o += "\\\"";
            else if (c == '\\') o += "\\\\";
            else o += char(c);
        } else if (c == '\b') o += "\\b";
        else if (c == '\f') o += "\\f";
        else if (c == '\n') o += "\\n";
        else if (c == '\r') o += "\\r";
        else if (c == '\t') o += "\\t";
        else {
            std::snprintf(buf, sizeof buf, "\\u%04x", unsigned(c));
            o += buf;
        }
    }
    return o + "\"";
}

// Character.isWhitespace over ASCII (String.isBlank)
bool java_ws(unsigned char c) {
    return c == ' ' || (c >= 0x09 && c <= 0x0D) || (c >= 0x1C && c <= 0x1F);
}

}  // namespace

std::string prometheus_text(const std::vector<PromMetric>& metrics,
                            const std::map<std::string, std::string>& help) {
    // sort by name; equal names keep creation (index) order
    std::vector<size_t> order(metrics.size());
    for (size_t i = 0; i < order.size(); ++i) order[i] = i;
    std::stable_sort(order.begin(), order.end(), [&](size_t a, size_t b) {
        return metrics[a].metric < metrics[b].metric;
    });
    std::string out;
    const std::string* last = nullptr;
    for (size_t k : order) {
        const PromMetric& m = metrics[k];
        if (!last || *last != m.metric) {
            auto h = help.find(m.metric);
            if (h != help.end()) out += "# HELP " + m.metric + " " + h->second + "\n";
            out += "# TYPE " + m.metric + " " + m.type + "\n";
        }
        last = &m.metric;
        out += m.metric + "{";
        bool first = true;
        for (const auto& kv : m.labels) {   // std::map: keys in String.compareTo order (ASCII)
            if (!first) out += ",";
            first = false;
            out += kv.first + "=" + json_quote(kv.second);
        }
        out += "} " + std::to_string(m.value) + "\n";
    }
    return out;
}

int parse_extra_labels(const char* spec, std::map<std::string, std::string>* out) {
    out->clear();
    if (!spec) return VC_OK;
    const std::string all(spec);
    size_t start = 0;
    while (start <= all.size()) {
        size_t comma = all.find(',', start);
        if (comma == std::string::npos) comma = all.size();
        const std::string piece = all.substr(start, comma - start);
        start = comma + 1;
        if (std::all_of(piece.begin(), piece.end(), [](char c) { return java_ws(c); })) continue;
        const size_t eq = piece.find('=');
        if (eq == std::string::npos) return VC_EINVAL;   // "invalid format, expecting k=v"
        (*out)[piece.substr(0, eq)] = piece.substr(eq + 1);
    }
    return VC_OK;
}

void hit_metrics(const uint64_t* acl, int n_tcp, int n_udp, const uint64_t* route, int n4, int n6,
                 const uint64_t* group, int n_groups,
                 const std::map<std::string, std::string>& extra, std::vector<PromMetric>* out,
                 std::map<std::string, std::string>* help) {
    auto add = [&](const char* metric, std::map<std::string, std::string> labels, uint64_t v) {
        for (const auto& kv : extra) labels[kv.first] = kv.second;   // putAll(extraLabels)
        out->push_back(PromMetric{metric, "counter", std::move(labels), int64_t(v)});
    };
    const char* acl_m = "security_group_rule_hit_count";
    const char* route_m = "route_table_rule_hit_count";
    const char* group_m = "upstream_server_group_hit_count";
    if (acl) {
        for (int i = 0; i < n_tcp; ++i)
            add(acl_m, {{"protocol", "TCP"}, {"rule", std::to_string(i)}}, acl[i]);
        for (int i = 0; i < n_udp; ++i)
            add(acl_m, {{"protocol", "UDP"}, {"rule", std::to_string(i)}}, acl[n_tcp + i]);
        add(acl_m, {{"protocol", "TCP"}, {"rule", "default"}}, acl[n_tcp + n_udp]);
        add(acl_m, {{"protocol", "UDP"}, {"rule", "default"}}, acl[n_tcp + n_udp + 1]);
        (*help)[acl_m] = "Packets matched per SecurityGroup rule (list index, or the default)";
    }
    if (route) {
        for (int i = 0; i < n4; ++i)
            add(route_m, {{"family", "v4"}, {"rule", std::to_string(i)}}, route[i]);
        for (int i = 0; i < n6; ++i)
            add(route_m, {{"family", "v6"}, {"rule", std::to_string(i)}}, route[n4 + i]);
        add(route_m, {{"family", "v4"}, {"rule", "none"}}, route[n4 + n6]);
        add(route_m, {{"family", "v6"}, {"rule", "none"}}, route[n4 + n6 + 1]);
        (*help)[route_m] = "Lookups matched per RouteTable rule (list index, or none)";
    }
    if (group) {
        for (int i = 0; i < n_groups; ++i)
            add(group_m, {{"group", std::to_string(i)}}, group[i]);
        add(group_m, {{"group", "none"}}, group[n_groups]);
        (*help)[group_m] = "Requests hinted to each Upstream server group (handle index, or none)";
    }
}

int copy_text(const std::string& text, char* buf, int64_t cap, int64_t* len) {
    if (len) *len = int64_t(text.size());
    if (!buf || cap <= int64_t(text.size())) return VC_ENOMEM;
    std::memcpy(buf, text.data(), text.size());
    buf[text.size()] = '\0';
    return VC_OK;
}

}  // namespace vc
