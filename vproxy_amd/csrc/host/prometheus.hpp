// prometheus.hpp -- Prometheus text exposition of the hit counters
// (SURVEY.md §8(f) row 4).  Host only; see prometheus.cpp.
#pragma once

#include <cstdint>
#include <map>
#include <string>
#include <vector>

namespace vc {

// One vproxybase.prometheus.Metric: name, type() string, labels (raw
// values, quoted at format time as Metric's constructor does) and value().
struct PromMetric {
    std::string metric;
    const char* type;
    std::map<std::string, std::string> labels;
    int64_t value;
};

// Metrics.toString: `metrics` in Metric.index (creation) order.
std::string prometheus_text(const std::vector<PromMetric>& metrics,
                            const std::map<std::string, std::string>& help);

// GlobalInspection.getExtraLabels over a "k1=v1,k2=v2" string.
int parse_extra_labels(const char* spec, std::map<std::string, std::string>* out);

// The hit counters laid out as vclassify.h's VC_COUNTERS_* arrays, each
// registered through GlobalInspection.addMetric (extra labels merged in);
// a null array is skipped.
void hit_metrics(const uint64_t* acl, int n_tcp, int n_udp, const uint64_t* route, int n4, int n6,
                 const uint64_t* group, int n_groups,
                 const std::map<std::string, std::string>& extra, std::vector<PromMetric>* out,
                 std::map<std::string, std::string>* help);

// Copy `text` to (buf, cap) NUL-terminated; *len = strlen(text).
// VC_ENOMEM (nothing written past cap) when cap <= strlen(text).
int copy_text(const std::string& text, char* buf, int64_t cap, int64_t* len);

}  // namespace vc
