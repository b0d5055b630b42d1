// Native unit tests (the reference ships C++ test binaries: src/nn/nn-cpu-ops-test.cpp,
// nn-vulkan-test.cpp, src/tokenizer-test.cpp, built and run by its CI, .github/workflows/main.yml).
// Host-only: quantization codecs, the shard plan, RoPE table, CPU primitives, JSON, chat templates,
// the EOS detector and the TP fused-exchange plan helpers. Built by `make test-cpp`
// (build/unit_tests) and run by tests/test_cpp_units.py.
#include <unistd.h>

#include <cmath>
#include <cstdio>
#include <cstring>
#include <functional>
#include <string>
#include <vector>

#include "../../csrc/core/model_file.h"
#include "../../csrc/core/plan.h"
#include "../../csrc/core/quant.h"
#include "../../csrc/cpu/cpu_ops.h"
#include "../../csrc/net/json.h"
#include "../../csrc/text/tokenizer.h"

using namespace dl;

static int gFailed = 0, gRun = 0;

#define CHECK(cond)                                                                   \
    do {                                                                              \
        if (!(cond)) {                                                                \
            std::printf("  FAILED %s:%d: %s\n", __FILE__, __LINE__, #cond);           \
            ok = false;                                                               \
        }                                                                             \
    } while (0)
#define CHECK_NEAR(a, b, tol) CHECK(std::fabs((double)(a) - (double)(b)) <= (tol))

static void run(const char *name, const std::function<bool()> &fn) {
    gRun++;
    bool ok = false;
    try {
        ok = fn();
    } catch (const std::exception &e) {
        std::printf("  exception: %s\n", e.what());
    }
    std::printf("%s %s\n", ok ? "✅" : "❌", name);
    if (!ok) gFailed++;
}

int main() {
    run("q80 roundtrip within half a step", [] {
        bool ok = true;
        std::vector<float> x(256);
        for (size_t i = 0; i < x.size(); i++) x[i] = std::sin(0.37f * i) * (1.0f + i % 7);
        std::vector<BlockQ80> q(x.size() / 32);
        std::vector<float> y(x.size());
        quantizeQ80(x.data(), q.data(), x.size());
        dequantizeQ80(q.data(), y.data(), x.size());
        for (size_t b = 0; b < q.size(); b++) {
            const float d = f16ToF32(q[b].d);
            // half a step of the f32 scale used to round, plus 127 x the scale's f16 rounding
            for (int j = 0; j < 32; j++) CHECK(std::fabs(y[b * 32 + j] - x[b * 32 + j]) <= 0.57f * d + 1e-6f);
        }
        return ok;
    });
    run("q40 codes and scale (writer.py semantics: d = signed max / -8)", [] {
        bool ok = true;
        std::vector<float> x(32);
        for (int j = 0; j < 32; j++) x[j] = (float)j - 20.0f;  // max |.| = -20
        BlockQ40 b;
        quantizeQ40(x.data(), &b, 32);
        CHECK_NEAR(f16ToF32(b.d), 2.5f, 1e-6);  // -20 / -8
        std::vector<float> y(32);
        dequantizeQ40(&b, y.data(), 32);
        for (int j = 0; j < 32; j++) CHECK(std::fabs(y[j] - x[j]) <= 1.25f + 1e-5f);
        CHECK_NEAR(y[0], -20.0f, 1e-5);
        return ok;
    });
    run("f16 conversions round to nearest even", [] {
        bool ok = true;
        CHECK(f32ToF16(1.0f) == 0x3C00);
        CHECK(f32ToF16(-2.0f) == 0xC000);
        CHECK_NEAR(f16ToF32(0x3555), 0.333251953125, 1e-9);
        CHECK(f32ToF16(1.0f + 1.0f / 4096) == 0x3C00);  // halfway rounds to even
        return ok;
    });
    run("shard plan splits every tensor evenly (reference slicers)", [] {
        bool ok = true;
        ModelHeader h;
        h.dim = 4096;
        h.hiddenDim = 14336;
        h.nHeads = 32;
        h.nKvHeads = 8;
        h.vocabSize = 128256;
        h.nLayers = 32;
        h.seqLen = 128;
        for (u32 n : {1u, 2u, 4u, 8u}) {
            for (u32 r = 0; r < n; r++) {
                const ShardPlan p = ShardPlan::make(h, n, r);
                CHECK(p.q0 * n == h.dim && p.kv0 * n == h.kvDim() && p.hidden0 * n == h.hiddenDim);
                CHECK(p.vocab0 * n == h.vocabSize && p.kvMul == 4 && p.headSize == 128);
                CHECK(p.qStart() == r * p.q0 && p.vocabStart() == r * p.vocab0);
            }
        }
        bool threw = false;
        try {
            ShardPlan::make(h, 16, 0);  // more ranks than KV heads
        } catch (const std::exception &) {
            threw = true;
        }
        CHECK(threw);
        return ok;
    });
    run("rope table: Llama-3.1 golden at position 6 (nn-vulkan-test.cpp:468-474)", [] {
        bool ok = true;
        ModelHeader h;
        h.dim = 2048;
        h.nHeads = 32;
        h.seqLen = 64;
        h.ropeTheta = 500000.f;
        h.ropeScalingFactor = 32.f;
        h.ropeScalingLowFreqFactor = 1.f;
        h.ropeScalingHighFreqFactor = 4.f;
        h.ropeScalingOrigMaxSeqLen = 8192;
        const std::vector<float> t = buildRopeTable(h);
        std::vector<float> x(2048, 1.0f);
        cpu::ropeApply(x.data(), 2048, 6, 64, t.data());
        CHECK_NEAR(x[0], 1.239586f, 1e-5);
        CHECK_NEAR(x[3], -1.412105f, 1e-5);
        CHECK_NEAR(x[1988], -1.356766f, 1e-5);
        return ok;
    });
    run("cpu primitives: invRms / SiLU goldens (nn-cpu-ops-test.cpp)", [] {
        bool ok = true;
        const float x[8] = {0.1f, 0.3f, 0.2f, 0.4f, 0.6f, 0.5f, 0.0f, 0.8f};
        CHECK_NEAR(cpu::invRms(x, 8, 1e-5f), 1.0f / 0.4402f, 1e-3);
        CHECK_NEAR(cpu::silu(7.0f / 8.0f), 0.617802f, 1e-3);  // the reference's tolerance
        std::vector<float> s = {0.f, 0.125f, 0.25f, 0.375f, 0.5f, 0.625f, 0.75f, 0.875f};
        softmaxInPlace(s.data(), s.size());
        CHECK_NEAR(s[0], 0.077399f, 1e-3);
        CHECK_NEAR(s[7], 0.185917f, 1e-3);
        return ok;
    });
    run("json parse / dump roundtrip", [] {
        bool ok = true;
        using json::Value;
        const Value v = Value::parse(R"({"a":[1,2.5,"x\né"],"b":{"c":true,"d":null}})");
        CHECK(v["a"].items().size() == 3);
        CHECK_NEAR(v["a"].items()[1].asNumber(), 2.5, 0);
        CHECK(v["a"].items()[2].asString() == "x\n\xc3\xa9");
        CHECK(v["b"]["c"].asBool() && v["b"]["d"].isNull());
        const Value w = Value::parse(v.dump());
        CHECK(w.dump() == v.dump());
        return ok;
    });
    run("chat template llama3 and EOS detector with stop strings", [] {
        bool ok = true;
        ChatTemplateGenerator g(ChatTemplateType::LLAMA3, "", "<|eot_id|>", false);
        const GeneratedChat c = g.generate({ChatItem{"user", "hi"}}, true);
        CHECK(c.content.find("<|start_header_id|>user<|end_header_id|>\n\nhi<|eot_id|>") != std::string::npos);
        CHECK(c.content.find("<|start_header_id|>assistant<|end_header_id|>\n\n") != std::string::npos);
        EosDetector eos({7}, {"STOP"}, 4, 4);
        CHECK(eos.append(1, "hello ") == EosResult::NOT_EOS);
        eos.reset();  // the caller emits the delta and resets after NOT_EOS (scheduler.cpp)
        CHECK(eos.append(2, "ST") == EosResult::MAYBE_EOS);
        CHECK(eos.append(3, "OP") == EosResult::EOS);
        return ok;
    });
    run("parallel_reader", [] {
        // 3 MB file read back through 1 KB pieces on 8 threads, whole and as scattered ranges
        bool ok = true;
        char path[] = "/tmp/dl_unit_reader_XXXXXX";
        const int fd = mkstemp(path);
        CHECK(fd >= 0);
        std::vector<u8> data(3 << 20);
        for (size_t i = 0; i < data.size(); i++) data[i] = (u8)(i * 2654435761u >> 13);
        CHECK(::write(fd, data.data(), data.size()) == (ssize_t)data.size());
        ::close(fd);
        {
            ParallelReader r(path, 8, 1024);
            std::vector<u8> out(data.size());
            r.read(0, out.size(), out.data());
            CHECK(out == data);
            std::vector<u8> a(5000), b(77);
            r.readMany({{12345, a.size(), a.data()}, {data.size() - 77, b.size(), b.data()}});
            CHECK(std::memcmp(a.data(), data.data() + 12345, a.size()) == 0);
            CHECK(std::memcmp(b.data(), data.data() + data.size() - 77, b.size()) == 0);
            CHECK(r.bytesRead() == data.size() + 5077);
            bool threw = false;
            try {
                r.read(data.size() - 10, 100, a.data());
            } catch (const Error &) {
                threw = true;
            }
            CHECK(threw);  // short read past the end of the file
        }
        ::unlink(path);
        return ok;
    });
    std::printf("%d/%d native unit tests passed\n", gRun - gFailed, gRun);
    return gFailed ? 1 : 0;
}
