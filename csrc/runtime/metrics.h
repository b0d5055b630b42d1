// Observability: a JSON-lines metrics sink and roctx trace ranges.
//
// The reference only prints per-token Eval/Pred/Sync lines and byte counters (dllama.cpp:57-113,
// nn-network.cpp:493-508). Here, in addition:
//   --metrics <file|->   one JSON object per forward (rows, wall/compute/sync ms, control-plane
//                        bytes, backend, nodes) appended to <file> (or stderr for "-");
//   DL_ROCTX=1           roctx ranges (forward / per kernel class in eager runs) for rocprofv3
//                        --marker-trace timelines; the roctx library is loaded lazily, so builds
//                        and runs without it are unaffected.
#pragma once

#include <cstdio>
#include <mutex>
#include <string>

namespace dl {

class MetricsSink {
  public:
    static MetricsSink &global();
    void open(const std::string &path);  // "" disables, "-" = stderr
    bool enabled() const { return f_ != nullptr; }
    void write(const std::string &jsonObject);  // one line
    ~MetricsSink();

  private:
    std::mutex mu_;
    FILE *f_ = nullptr;
    bool own_ = false;
};

// Milliseconds since the Unix epoch (metrics timestamps).
double epochMs();

// RAII roctx range; no-op unless DL_ROCTX=1 and the roctx library loads.
class TraceRange {
  public:
    explicit TraceRange(const char *name);
    ~TraceRange();
    TraceRange(const TraceRange &) = delete;
    TraceRange &operator=(const TraceRange &) = delete;
    static bool enabled();

  private:
    bool active_ = false;
};

}  // namespace dl
