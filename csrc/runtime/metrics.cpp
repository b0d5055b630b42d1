#include "metrics.h"

#include <dlfcn.h>

#include <chrono>
#include <cstdlib>

#include "../core/common.h"

namespace dl {

MetricsSink &MetricsSink::global() {
    static MetricsSink s;
    return s;
}

void MetricsSink::open(const std::string &path) {
    std::lock_guard<std::mutex> lk(mu_);
    if (f_ && own_) std::fclose(f_);
    f_ = nullptr;
    own_ = false;
    if (path.empty()) return;
    if (path == "-") {
        f_ = stderr;
        return;
    }
    f_ = std::fopen(path.c_str(), "a");
    if (!f_) throw Error("cannot open metrics file " + path);
    own_ = true;
}

void MetricsSink::write(const std::string &jsonObject) {
    std::lock_guard<std::mutex> lk(mu_);
    if (!f_) return;
    std::fputs(jsonObject.c_str(), f_);
    std::fputc('\n', f_);
    std::fflush(f_);
}

MetricsSink::~MetricsSink() {
    if (f_ && own_) std::fclose(f_);
}

double epochMs() {
    using namespace std::chrono;
    return (double)duration_cast<microseconds>(system_clock::now().time_since_epoch()).count() / 1000.0;
}

namespace {
struct Roctx {
    int (*push)(const char *) = nullptr;
    int (*pop)() = nullptr;
    Roctx() {
        const char *e = std::getenv("DL_ROCTX");
        if (!e || *e != '1') return;
        for (const char *lib : {"librocprofiler-sdk-roctx.so.1", "librocprofiler-sdk-roctx.so", "libroctx64.so"}) {
            void *h = dlopen(lib, RTLD_NOW | RTLD_GLOBAL);
            if (!h) continue;
            push = reinterpret_cast<int (*)(const char *)>(dlsym(h, "roctxRangePushA"));
            pop = reinterpret_cast<int (*)()>(dlsym(h, "roctxRangePop"));
            if (push && pop) return;
            push = nullptr;
            pop = nullptr;
        }
    }
};
const Roctx &roctx() {
    static Roctx r;
    return r;
}
}  // namespace

bool TraceRange::enabled() { return roctx().push != nullptr; }

TraceRange::TraceRange(const char *name) {
    if (roctx().push) {
        roctx().push(name);
        active_ = true;
    }
}

TraceRange::~TraceRange() {
    if (active_) roctx().pop();
}

}  // namespace dl
