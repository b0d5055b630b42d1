// Backend defaults: host-side sampling used by the CPU backend and as the reference for the
// device sampler (csrc/hip/kernels.hip sampleKernel).
#include "backend.h"

#include <algorithm>

#include <vector>

#include "../text/tokenizer.h"

namespace dl {

int sampleHost(float *logits, int vocab, const SampleSpec &s) {
    if (s.temperature < 0.f) return -1;
    Sampler smp(vocab, s.temperature, s.topp, 0);
    return smp.sampleWithCoin(logits, s.coin);
}

void Backend::forwardSample(int n, const int *tokens, const int *positions, const int *slots, const SampleSpec *specs,
                            int *out) {
    const int vocab = (int)header().vocabSize;
    if (plan().rank != 0) {  // workers take part in the forward; the root draws
        forward(n, tokens, positions, slots, nullptr);
        for (int i = 0; i < n; i++) out[i] = -1;
        return;
    }
    std::vector<float> logits((size_t)n * vocab);
    forward(n, tokens, positions, slots, logits.data());
    for (int i = 0; i < n; i++) out[i] = sampleHost(&logits[(size_t)i * vocab], vocab, specs[i]);
}

void Backend::launchIds(int n, const int *tokens, const int *positions, const int *slots, const SampleSpec *specs) {
    pendingIds_.assign(n, -1);
    if (specs)
        forwardSample(n, tokens, positions, slots, specs, pendingIds_.data());
    else
        forwardArgmax(n, tokens, positions, slots, pendingIds_.data());
}

void Backend::collectIds(int *out) {
    std::copy(pendingIds_.begin(), pendingIds_.end(), out);
    pendingIds_.clear();
}

void Backend::chainLaunch(int, int, int) { throw Error(name() + " backend: no chained decode"); }
int Backend::chainCollect() { throw Error(name() + " backend: no chained decode"); }

}  // namespace dl
