// Python bindings (pybind11) for tests, the torch oracle comparison and bench.py.
// The hot path never goes through Python: a forward call is one C++ call that replays a hipGraph.
#include <pybind11/numpy.h>
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include <cstring>

#include "../core/model_file.h"
#include "../core/plan.h"
#include "../core/quant.h"
#include "../cpu/cpu_ops.h"
#include "../hip/engine.h"
#include "../hip/ops.h"
#include "../runtime/backend.h"
#include "../runtime/weight_stream.h"
#include "../text/tokenizer.h"

namespace py = pybind11;
using namespace dl;

namespace {

py::dict headerToDict(const ModelHeader &h) {
    py::dict d;
    d["header_size"] = h.headerSize;
    d["file_size"] = h.fileSize;
    d["version"] = h.version;
    d["dim"] = h.dim;
    d["hidden_dim"] = h.hiddenDim;
    d["n_layers"] = h.nLayers;
    d["n_heads"] = h.nHeads;
    d["n_kv_heads"] = h.nKvHeads;
    d["n_experts"] = h.nExperts;
    d["vocab_size"] = h.vocabSize;
    d["seq_len"] = h.seqLen;
    d["orig_seq_len"] = h.origSeqLen;
    d["hidden_act"] = (int)h.hiddenAct;
    d["rope_theta"] = h.ropeTheta;
    d["rope_type"] = (int)h.ropeType;
    d["rope_scaling_factor"] = h.ropeScalingFactor;
    d["rope_scaling_low_freq_factor"] = h.ropeScalingLowFreqFactor;
    d["rope_scaling_high_freq_factor"] = h.ropeScalingHighFreqFactor;
    d["rope_scaling_orig_max_seq_len"] = h.ropeScalingOrigMaxSeqLen;
    d["norm_epsilon"] = h.normEpsilon;
    d["weight_type"] = (int)h.weightType;
    d["head_size"] = h.headSize();
    d["kv_dim"] = h.kvDim();
    return d;
}

ModelHeader dictToHeader(const py::dict &d) {
    ModelHeader h;
    h.dim = d["dim"].cast<u32>();
    h.hiddenDim = d["hidden_dim"].cast<u32>();
    h.nLayers = d["n_layers"].cast<u32>();
    h.nHeads = d["n_heads"].cast<u32>();
    h.nKvHeads = d["n_kv_heads"].cast<u32>();
    h.vocabSize = d["vocab_size"].cast<u32>();
    h.seqLen = d["seq_len"].cast<u32>();
    h.origSeqLen = h.seqLen;
    if (d.contains("rope_theta")) h.ropeTheta = d["rope_theta"].cast<float>();
    if (d.contains("hidden_act")) h.hiddenAct = (HiddenAct)d["hidden_act"].cast<int>();
    if (d.contains("rope_scaling_factor")) h.ropeScalingFactor = d["rope_scaling_factor"].cast<float>();
    if (d.contains("rope_scaling_low_freq_factor"))
        h.ropeScalingLowFreqFactor = d["rope_scaling_low_freq_factor"].cast<float>();
    if (d.contains("rope_scaling_high_freq_factor"))
        h.ropeScalingHighFreqFactor = d["rope_scaling_high_freq_factor"].cast<float>();
    if (d.contains("rope_scaling_orig_max_seq_len"))
        h.ropeScalingOrigMaxSeqLen = d["rope_scaling_orig_max_seq_len"].cast<u32>();
    if (d.contains("rope_type")) h.ropeType = (RopeType)d["rope_type"].cast<int>();
    h.weightType = d.contains("weight_type") ? (FloatType)d["weight_type"].cast<int>() : FloatType::Q40;
    return h;
}

EngineConfig makeConfig(const std::string &model, const std::string &bufferType, int nThreads, u32 maxSeqLen,
                        u32 maxBatch, u32 nSlots, int gpuIndex, bool useGraphs, bool kvBf16, py::object synthetic,
                        u64 seed) {
    EngineConfig c;
    c.modelPath = model;
    c.bufferType = parseFloatType(bufferType);
    c.nThreads = nThreads;
    c.maxSeqLen = maxSeqLen;
    c.maxBatch = maxBatch;
    c.nSlots = nSlots;
    c.gpuIndex = gpuIndex;
    c.useGraphs = useGraphs;
    c.kvBf16 = kvBf16;
    c.seed = seed;
    if (!synthetic.is_none()) {
        c.synthetic = true;
        c.syntheticHeader = dictToHeader(synthetic.cast<py::dict>());
    }
    return c;
}

template <typename T>
std::vector<int> toInts(const T &arr) {
    std::vector<int> v;
    for (auto x : arr) v.push_back(py::cast<int>(x));
    return v;
}

py::array_t<float> runForward(Backend &b, const std::vector<int> &tokens, const std::vector<int> &positions,
                              const std::vector<int> &slots) {
    const int n = (int)tokens.size();
    DL_CHECK(positions.size() == tokens.size() && slots.size() == tokens.size(), "input lengths");
    py::array_t<float> out({n, (int)b.header().vocabSize});
    {
        py::gil_scoped_release rel;
        b.forward(n, tokens.data(), positions.data(), slots.data(), out.mutable_data());
    }
    return out;
}

std::vector<int> runArgmax(Backend &b, const std::vector<int> &tokens, const std::vector<int> &positions,
                           const std::vector<int> &slots) {
    std::vector<int> out(tokens.size());
    py::gil_scoped_release rel;
    b.forwardArgmax((int)tokens.size(), tokens.data(), positions.data(), slots.data(), out.data());
    return out;
}

// Per-row draws: specs from (temperature, topp, coin) lists.
std::vector<int> runSample(Backend &b, const std::vector<int> &tokens, const std::vector<int> &positions,
                           const std::vector<int> &slots, const std::vector<float> &temps,
                           const std::vector<float> &topps, const std::vector<float> &coins) {
    const size_t n = tokens.size();
    DL_CHECK(temps.size() == n && topps.size() == n && coins.size() == n, "one (temperature, topp, coin) per row");
    std::vector<SampleSpec> specs(n);
    for (size_t i = 0; i < n; i++) specs[i] = SampleSpec{temps[i], topps[i], coins[i], 0.f};
    std::vector<int> out(n);
    py::gil_scoped_release rel;
    b.forwardSample((int)n, tokens.data(), positions.data(), slots.data(), specs.data(), out.data());
    return out;
}

// Device communicator owned from Python (xGMI one-shot collectives); shared with engines.
struct PyComm {
    std::shared_ptr<DeviceComm> comm;
};
struct PyRcclComm : PyComm {};
struct PyComputeOnlyComm : PyComm {};

// Keeps the device comm alive as long as the engine.
struct PyHipEngine {
    std::shared_ptr<DeviceComm> comm;
    std::unique_ptr<HipEngine> engine;
};


template <typename T>
std::vector<T> vec(const py::object &o) {  // None -> empty
    if (o.is_none()) return {};
    py::array_t<T, py::array::c_style | py::array::forcecast> a(o);
    return std::vector<T>(a.data(), a.data() + a.size());
}

template <typename T>
py::array_t<T> arr(const std::vector<T> &v, std::vector<py::ssize_t> shape) {
    py::array_t<T> a(shape);
    DL_CHECK((size_t)a.size() == v.size(), "result shape");
    std::memcpy(a.mutable_data(), v.data(), v.size() * sizeof(T));
    return a;
}

void bindOps(py::module_ &m) {
    // every py::object is converted to a std::vector while the GIL is held; only the device work
    // runs with it released
    py::module_ o = m.def_submodule("ops", "single-kernel entry points (csrc/hip/ops.h) for numerics tests");
    o.def("gemv_q40",
          [](py::object blocks, int rows, int n, py::object x, py::object residual, py::object normW, float eps, int epi) {
              const std::vector<uint8_t> w = vec<uint8_t>(blocks);
              const std::vector<float> in = vec<float>(x), res = vec<float>(residual), nw = vec<float>(normW);
              const int B = (int)(in.size() / n);
              std::vector<float> out, xn;
              {
                  py::gil_scoped_release rel;
                  out = ops::gemvQ40(w, rows, n, in, res, nw, eps, B, epi, &xn);
              }
              py::object xo = py::none();
              if (!xn.empty()) xo = arr(xn, {B, n});
              return py::make_tuple(arr(out, {B, (py::ssize_t)(out.size() / B)}), xo);
          },
          py::arg("blocks"), py::arg("rows"), py::arg("n"), py::arg("x"), py::arg("residual") = py::none(),
          py::arg("norm_w") = py::none(), py::arg("eps") = 1e-5f, py::arg("epi") = 0);
    o.def("gemv_q40_q80_in",
          [](py::object blocks, int rows, int n, py::object x) {
              const std::vector<uint8_t> w = vec<uint8_t>(blocks);
              const std::vector<float> in = vec<float>(x);
              const int B = (int)(in.size() / n);
              std::vector<float> out;
              {
                  py::gil_scoped_release rel;
                  out = ops::gemvQ40Q80In(w, rows, n, in, B);
              }
              return arr(out, {B, rows});
          },
          py::arg("blocks"), py::arg("rows"), py::arg("n"), py::arg("x"));
    o.def("gemm_q40",
          [](py::object blocks, int rows, int n, py::object x, py::object residual, py::object normW, float eps,
             int splits) {
              const std::vector<uint8_t> w = vec<uint8_t>(blocks);
              const std::vector<float> in = vec<float>(x), res = vec<float>(residual), nw = vec<float>(normW);
              const int M = (int)(in.size() / n);
              std::vector<float> out;
              {
                  py::gil_scoped_release rel;
                  out = ops::gemmQ40(w, rows, n, in, res, nw, eps, M, splits);
              }
              return arr(out, {M, rows});
          },
          py::arg("blocks"), py::arg("rows"), py::arg("n"), py::arg("x"), py::arg("residual") = py::none(),
          py::arg("norm_w") = py::none(), py::arg("eps") = 1e-5f, py::arg("splits") = 0);
    o.def("gemm_f32",
          [](py::object wts, int rows, int n, py::object x, py::object normW, float eps) {
              const std::vector<float> w = vec<float>(wts), in = vec<float>(x), nw = vec<float>(normW);
              const int M = (int)(in.size() / n);
              std::vector<float> out;
              {
                  py::gil_scoped_release rel;
                  out = ops::gemmF32(w, rows, n, in, nw, eps, M);
              }
              return arr(out, {M, rows});
          },
          py::arg("w"), py::arg("rows"), py::arg("n"), py::arg("x"), py::arg("norm_w") = py::none(),
          py::arg("eps") = 1e-5f);
    o.def("qkv_rope",
          [](py::object blocks, int q0, int kv0, int hs, int n, py::object x, py::object normW, float eps, py::object rope,
             int seqLen, std::vector<int> pos, bool kvBf16) {
              const std::vector<uint8_t> w = vec<uint8_t>(blocks);
              const std::vector<float> in = vec<float>(x), nw = vec<float>(normW), rp = vec<float>(rope);
              std::vector<float> k, v, q;
              {
                  py::gil_scoped_release rel;
                  q = ops::qkvRope(w, q0, kv0, hs, n, in, nw, eps, rp, seqLen, pos, kvBf16, &k, &v);
              }
              const py::ssize_t B = (py::ssize_t)pos.size();
              return py::make_tuple(arr(q, {B, q0}), arr(k, {B, kv0}), arr(v, {B, kv0}));
          },
          py::arg("blocks"), py::arg("q0"), py::arg("kv0"), py::arg("head_size"), py::arg("n"), py::arg("x"),
          py::arg("norm_w"), py::arg("eps"), py::arg("rope"), py::arg("seq_len"), py::arg("pos"), py::arg("kv_bf16") = true);
    o.def("attention",
          [](py::object q, py::object k, py::object v, int nSlots, int seqLen, int nHeads0, int kvMul, int hs,
             std::vector<int> pos, std::vector<int> slot, bool kvBf16, int impl) {
              const std::vector<float> qv = vec<float>(q), kv = vec<float>(k), vv = vec<float>(v);
              std::vector<float> out;
              {
                  py::gil_scoped_release rel;
                  out = ops::attention(qv, kv, vv, nSlots, seqLen, nHeads0, kvMul, hs, pos, slot, kvBf16, impl);
              }
              return arr(out, {(py::ssize_t)pos.size(), (py::ssize_t)nHeads0 * hs});
          },
          py::arg("q"), py::arg("k"), py::arg("v"), py::arg("n_slots"), py::arg("seq_len"), py::arg("n_heads0"),
          py::arg("kv_mul"), py::arg("head_size"), py::arg("pos"), py::arg("slot"), py::arg("kv_bf16") = true,
          py::arg("impl") = 0);
    o.def("sample",
          [](py::object logits, int B, py::object specs) {
              const std::vector<float> l = vec<float>(logits), sp = vec<float>(specs);
              std::vector<int> ids;
              {
                  py::gil_scoped_release rel;
                  ids = ops::sample(l, B, (int)(l.size() / B), sp);
              }
              return ids;
          });
    o.def("argmax",
          [](py::object logits, int B) {
              const std::vector<float> l = vec<float>(logits);
              std::vector<int> ids;
              {
                  py::gil_scoped_release rel;
                  ids = ops::argmax(l, B, (int)(l.size() / B));
              }
              return ids;
          },
          py::arg("logits"), py::arg("batch"));
    o.def("embedding",
          [](py::object table, int vocab, int dim, std::vector<int> tokens) {
              const std::vector<float> t = vec<float>(table);
              std::vector<float> out;
              {
                  py::gil_scoped_release rel;
                  out = ops::embedding(t, vocab, dim, tokens);
              }
              return arr(out, {(py::ssize_t)tokens.size(), dim});
          },
          py::arg("table"), py::arg("vocab"), py::arg("dim"), py::arg("tokens"));
}

}  // namespace

PYBIND11_MODULE(_C, m) {
    m.doc() = "MI355X-native distributed Llama engine (native core)";
    bindOps(m);
    m.def("set_log_level", &setLogLevel);
    m.def("hip_device_count", &hipDeviceCount);

    m.def("f32_to_f16", &f32ToF16);
    m.def("f16_to_f32", &f16ToF32);
    m.def("quantize_q80", [](py::array_t<float, py::array::c_style | py::array::forcecast> x) {
        const u64 n = (u64)x.size();
        py::array_t<uint8_t> out((py::ssize_t)(n / kQBlock * kQ80BlockBytes));
        quantizeQ80(x.data(), reinterpret_cast<BlockQ80 *>(out.mutable_data()), n);
        return out;
    });
    m.def("quantize_q40", [](py::array_t<float, py::array::c_style | py::array::forcecast> x) {
        const u64 n = (u64)x.size();
        py::array_t<uint8_t> out((py::ssize_t)(n / kQBlock * kQ40BlockBytes));
        quantizeQ40(x.data(), reinterpret_cast<BlockQ40 *>(out.mutable_data()), n);
        return out;
    });
    m.def("dequantize_q80", [](py::array_t<uint8_t, py::array::c_style> b) {
        const u64 n = (u64)b.size() / kQ80BlockBytes * kQBlock;
        py::array_t<float> out((py::ssize_t)n);
        dequantizeQ80(reinterpret_cast<const BlockQ80 *>(b.data()), out.mutable_data(), n);
        return out;
    });
    m.def("dequantize_q40", [](py::array_t<uint8_t, py::array::c_style> b) {
        const u64 n = (u64)b.size() / kQ40BlockBytes * kQBlock;
        py::array_t<float> out((py::ssize_t)n);
        dequantizeQ40(reinterpret_cast<const BlockQ40 *>(b.data()), out.mutable_data(), n);
        return out;
    });

    // CPU reference primitives (csrc/cpu/cpu_ops.h) for the reference-golden tests
    py::module_ co = m.def_submodule("cpu_ops", "CPU reference primitives (csrc/cpu/cpu_ops.h)");
    co.def("sample_host", [](py::array_t<float, py::array::c_style | py::array::forcecast> logits, float temp, float topp,
                             float coin) {
        std::vector<float> l(logits.data(), logits.data() + logits.size());
        return sampleHost(l.data(), (int)l.size(), SampleSpec{temp, topp, coin, 0.f});
    });
    co.def("inv_rms", [](py::array_t<float, py::array::c_style | py::array::forcecast> x, float eps) {
        return cpu::invRms(x.data(), (u32)x.size(), eps);
    });
    auto elementwise = [](float (*f)(float)) {
        return [f](py::array_t<float, py::array::c_style | py::array::forcecast> x) {
            py::array_t<float> out(x.size());
            for (py::ssize_t i = 0; i < x.size(); i++) out.mutable_data()[i] = f(x.data()[i]);
            return out;
        };
    };
    co.def("silu", elementwise(&cpu::silu));
    co.def("gelu", elementwise(&cpu::gelu));
    co.def("softmax", [](py::array_t<float, py::array::c_style | py::array::forcecast> x) {
        py::array_t<float> out(x.size());
        std::memcpy(out.mutable_data(), x.data(), x.size() * sizeof(float));
        softmaxInPlace(out.mutable_data(), (u64)x.size());
        return out;
    });
    // the engines' RoPE table ([seqLen][headSize/2] (cos, sin), Llama-3.1 scaling when the header
    // has rope_scaling_factor != 1) for a header dict
    co.def("rope_table", [](py::dict header) {
        const ModelHeader h = dictToHeader(header);
        std::vector<float> t = buildRopeTable(h);
        py::array_t<float> out({(py::ssize_t)h.seqLen, (py::ssize_t)(h.headSize() / 2), (py::ssize_t)2});
        std::memcpy(out.mutable_data(), t.data(), t.size() * sizeof(float));
        return out;
    });
    co.def("rope_apply", [](py::array_t<float, py::array::c_style | py::array::forcecast> x, int pos, int headSize,
                            py::array_t<float, py::array::c_style | py::array::forcecast> table) {
        py::array_t<float> out(x.size());
        std::memcpy(out.mutable_data(), x.data(), x.size() * sizeof(float));
        cpu::ropeApply(out.mutable_data(), (u32)x.size(), (u32)pos, (u32)headSize, table.data());
        return out;
    });
    // y[B][rows] = W . x[b] with W Q40 blocks [rows][cols/32] and x quantized to Q80 (the
    // reference's matmul_Q80_Q40_F32)
    co.def("matmul_q40_q80", [](py::array_t<uint8_t, py::array::c_style> blocks, int rows, int cols,
                                py::array_t<float, py::array::c_style | py::array::forcecast> x, int nThreads) {
        DL_CHECK(cols % kQBlock == 0 && (size_t)blocks.size() == (size_t)rows * cols / kQBlock * kQ40BlockBytes &&
                     x.size() % cols == 0, "matmul_q40_q80 shapes");
        const int B = (int)(x.size() / cols);
        std::vector<BlockQ80> xq((size_t)B * cols / kQBlock);
        quantizeQ80(x.data(), xq.data(), (u64)B * cols);
        std::vector<const BlockQ80 *> xs(B);
        py::array_t<float> out({(py::ssize_t)B, (py::ssize_t)rows});
        std::vector<float *> ys(B);
        for (int b = 0; b < B; b++) {
            xs[b] = xq.data() + (size_t)b * cols / kQBlock;
            ys[b] = out.mutable_data() + (size_t)b * rows;
        }
        ThreadPool pool(nThreads);
        py::gil_scoped_release rel;
        cpu::matmulQ40Q80(reinterpret_cast<const BlockQ40 *>(blocks.data()), rows, cols, xs.data(), B, ys.data(), pool);
        return out;
    }, py::arg("blocks"), py::arg("rows"), py::arg("cols"), py::arg("x"), py::arg("nthreads") = 4);

    m.def("load_header", [](const std::string &path, u32 maxSeqLen) { return headerToDict(loadModelHeader(path, maxSeqLen)); },
          py::arg("path"), py::arg("max_seq_len") = 0);
    m.def("tensor_table", [](const std::string &path) {
        ModelHeader h = loadModelHeader(path);
        py::list l;
        for (const auto &t : buildTensorTable(h)) {
            py::dict d;
            d["name"] = tensorKindName(t.kind);
            d["layer"] = t.layer;
            d["offset"] = t.offset;
            d["bytes"] = t.bytes;
            d["type"] = (int)t.type;
            d["rows"] = t.rows;
            d["cols"] = t.cols;
            l.append(d);
        }
        return l;
    });
    m.def("shard_plan", [](py::dict header, u32 nRanks, u32 rank) {
        ShardPlan p = ShardPlan::make(dictToHeader(header), nRanks, rank);
        py::dict d;
        d["q0"] = p.q0;
        d["kv0"] = p.kv0;
        d["hidden0"] = p.hidden0;
        d["vocab0"] = p.vocab0;
        d["n_heads0"] = p.nHeads0;
        d["n_kv_heads0"] = p.nKvHeads0;
        d["kv_mul"] = p.kvMul;
        return d;
    });
    m.def("rope_table", [](py::dict header) {
        std::vector<float> t = buildRopeTable(dictToHeader(header));
        return py::array_t<float>((py::ssize_t)t.size(), t.data());
    });

    py::class_<Tokenizer>(m, "Tokenizer")
        .def(py::init<const std::string &, bool>(), py::arg("path"), py::arg("verbose") = false)
        .def("encode",
             [](const Tokenizer &t, const std::string &text, bool addBos, bool addSpecial) {
                 return t.encode(text, addBos, addSpecial);
             },
             py::arg("text"), py::arg("add_bos") = true, py::arg("add_special_tokens") = false)
        .def("decode",
             [](Tokenizer &t, int token) -> py::object {
                 std::string out;
                 if (t.decode(token, out)) return py::bytes(out);
                 return py::none();
             })
        .def("reset_decoder", &Tokenizer::resetDecoder)
        .def("is_eos", &Tokenizer::isEos)
        .def("piece", [](const Tokenizer &t, int id) { return py::bytes(t.piece(id)); })
        .def_property_readonly("vocab_size", &Tokenizer::vocabSize)
        .def_property_readonly("bos_id", &Tokenizer::bosId)
        .def_property_readonly("eos_token_ids", &Tokenizer::eosTokenIds)
        .def_property_readonly("chat_template", [](const Tokenizer &t) { return py::bytes(t.chatTemplate()); });

    py::class_<Sampler>(m, "Sampler")
        .def(py::init<int, float, float, u64>())
        .def("sample",
             [](Sampler &s, py::array_t<float, py::array::c_style | py::array::forcecast> logits) {
                 std::vector<float> v(logits.data(), logits.data() + logits.size());
                 return s.sample(v.data());
             })
        .def("set_temp", &Sampler::setTemp)
        .def("set_seed", &Sampler::setSeed);

    py::enum_<EosResult>(m, "EosResult")
        .value("NOT_EOS", EosResult::NOT_EOS)
        .value("MAYBE_EOS", EosResult::MAYBE_EOS)
        .value("EOS", EosResult::EOS);
    py::class_<EosDetector>(m, "EosDetector")
        .def(py::init<std::vector<int>, std::vector<std::string>, int, int>())
        .def("append",
             [](EosDetector &d, int token, py::object piece) {
                 if (piece.is_none()) return d.append(token, nullptr);
                 std::string s = piece.cast<std::string>();
                 return d.append(token, s.c_str());
             })
        .def("get_delta",
             [](EosDetector &d) -> py::object {
                 std::string out;
                 if (d.getDelta(out)) return py::bytes(out);
                 return py::none();
             })
        .def("reset", &EosDetector::reset);

    py::class_<ChatTemplateGenerator>(m, "ChatTemplateGenerator")
        .def(py::init([](const std::string &type, const std::string &tmpl, const std::string &eos) {
                 return new ChatTemplateGenerator(type.empty() ? ChatTemplateType::UNKNOWN : parseChatTemplateType(type),
                                                  tmpl, eos, false);
             }),
             py::arg("type"), py::arg("template"), py::arg("eos"))
        .def_property_readonly("type", [](const ChatTemplateGenerator &g) { return chatTemplateTypeName(g.type()); })
        .def("generate", [](const ChatTemplateGenerator &g, const std::vector<std::pair<std::string, std::string>> &items,
                            bool appendGenerationPrompt) {
            std::vector<ChatItem> its;
            for (auto &p : items) its.push_back(ChatItem{p.first, p.second});
            GeneratedChat c = g.generate(its, appendGenerationPrompt);
            return py::make_tuple(py::bytes(c.content), py::bytes(c.publicPrompt));
        });

    py::class_<Backend>(m, "Backend")
        .def_property_readonly("header", [](const Backend &b) { return headerToDict(b.header()); })
        .def_property_readonly("name", &Backend::name)
        .def("forward", [](Backend &b, std::vector<int> t, std::vector<int> p, std::vector<int> s) { return runForward(b, t, p, s); },
             py::arg("tokens"), py::arg("positions"), py::arg("slots"))
        .def("forward_sample", &runSample, py::arg("tokens"), py::arg("positions"), py::arg("slots"),
             py::arg("temperatures"), py::arg("topps"), py::arg("coins"))
        .def("forward_argmax", [](Backend &b, std::vector<int> t, std::vector<int> p, std::vector<int> s) { return runArgmax(b, t, p, s); },
             py::arg("tokens"), py::arg("positions"), py::arg("slots"))
        .def("last_stats", [](const Backend &b) {
            ForwardStats s = b.lastStats();
            return py::make_tuple(s.computeMs, s.syncMs, s.sentBytes, s.recvBytes, s.xchgMs);
        });

    m.def("cpu_backend",
          [](const std::string &model, const std::string &bufferType, int nThreads, u32 maxSeqLen, u32 maxBatch,
             u32 nSlots) {
              EngineConfig c = makeConfig(model, bufferType, nThreads, maxSeqLen, maxBatch, nSlots, -1, false, false,
                                          py::none(), 1);
              return makeCpuBackend(c, nullptr);
          },
          py::arg("model"), py::arg("buffer_type") = "q80", py::arg("nthreads") = 1, py::arg("max_seq_len") = 0,
          py::arg("max_batch") = 32, py::arg("n_slots") = 1);

    // CPU tensor parallelism in one process (ThreadGroupComm): rank 0's logits of sequential
    // single-token forwards of `tokens` at positions 0.., [n][vocab], and the greedy continuation
    // of `steps` tokens after them (every rank agrees on it).
    m.def("cpu_simulate_tp",
          [](const std::string &model, const std::string &bufferType, int world, std::vector<int> tokens,
             const std::string &syncType, int steps, int nThreads) {
              EngineConfig c = makeConfig(model, bufferType, nThreads, 0, 8, 1, -1, false, false, py::none(), 1);
              c.syncType = parseFloatType(syncType);
              std::vector<float> logits;
              std::vector<int> greedy;
              u32 vocab = 0;
              {
                  py::gil_scoped_release rel;
                  auto comms = ThreadGroupComm::make(world);
                  std::vector<std::unique_ptr<Backend>> bes(world);
                  std::vector<std::string> errs(world);
                  std::vector<std::thread> th;
                  for (int r = 0; r < world; r++)
                      th.emplace_back([&, r] {
                          try {
                              bes[r] = makeCpuBackend(c, comms[r].get());
                              const u32 V = bes[r]->header().vocabSize;
                              std::vector<float> lg(V);
                              int pos = 0, slot0 = 0;
                              for (int t : tokens) {
                                  bes[r]->forward(1, &t, &pos, &slot0, r == 0 ? lg.data() : nullptr);
                                  if (r == 0) {
                                      vocab = V;
                                      logits.insert(logits.end(), lg.begin(), lg.end());
                                  }
                                  pos++;
                              }
                              if (steps > 0) {
                                  // first continuation token from the prompt's last logits (rank 0),
                                  // shared with the other ranks through the comm (exact for ids)
                                  float id = r == 0 ? (float)(std::max_element(lg.begin(), lg.end()) - lg.begin()) : 0.f;
                                  comms[r]->allReduceSum(&id, 1);
                                  int tok = (int)id;
                                  if (r == 0) greedy.push_back(tok);
                                  for (int s = 1; s < steps; s++) {
                                      int next = 0;
                                      bes[r]->forwardArgmax(1, &tok, &pos, &slot0, &next);
                                      pos++;
                                      tok = next;
                                      if (r == 0) greedy.push_back(tok);
                                  }
                              }
                          } catch (const std::exception &e) {
                              errs[r] = e.what();
                          }
                      });
                  for (auto &t : th) t.join();
                  for (auto &e : errs)
                      if (!e.empty()) throw Error("cpu_simulate_tp: " + e);
              }
              py::array_t<float> a({(py::ssize_t)tokens.size(), (py::ssize_t)vocab});
              std::memcpy(a.mutable_data(), logits.data(), logits.size() * 4);
              return py::make_tuple(a, greedy);
          },
          py::arg("model"), py::arg("buffer_type"), py::arg("world"), py::arg("tokens"), py::arg("sync_type") = "f32",
          py::arg("steps") = 0, py::arg("nthreads") = 1);

    m.def("bench_gemv_q40",
          [](int rows, int n, int pro, int epi, int B, int lanes, int passes, int copies, int iters) {
              return benchGemvQ40(rows, n, pro, epi, B, lanes, passes, copies, iters);
          },
          py::arg("rows"), py::arg("n"), py::arg("pro"), py::arg("epi"), py::arg("batch") = 1, py::arg("lanes") = 0,
          py::arg("passes") = 1, py::arg("copies") = 8, py::arg("iters") = 200, py::call_guard<py::gil_scoped_release>());
    m.def("trace_gemv_q40",
          [](int rows, int n, int pro, int epi, int B, int lanes, int passes, int copies, int iters) {
              std::vector<unsigned long long> t;
              double us;
              {
                  py::gil_scoped_release nogil;
                  us = benchGemvQ40(rows, n, pro, epi, B, lanes, passes, copies, iters, &t);
              }
              return py::make_tuple(us, py::array_t<unsigned long long>(t.size(), t.data()));
          },
          py::arg("rows"), py::arg("n"), py::arg("pro"), py::arg("epi"), py::arg("batch") = 1, py::arg("lanes") = 0,
          py::arg("passes") = 0, py::arg("copies") = 8, py::arg("iters") = 20,
          "bench_gemv_q40 with per-workgroup s_memrealtime stamps: (us, u64[iters*grid*4])");
    m.def("bench_gemm_q40", [](int rows, int n, int M, int epi, int copies, int iters) {
              return benchGemmQ40(rows, n, M, epi, copies, iters);
          }, py::arg("rows"), py::arg("n"), py::arg("tokens"), py::arg("epi") = 0,
          py::arg("copies") = 8, py::arg("iters") = 100, py::call_guard<py::gil_scoped_release>());
    m.def("bench_attention",
          [](int nh, int kvm, int hs, int seq, int pos, int B, int copies, int iters, bool kvBf16) {
              return benchAttention(nh, kvm, hs, seq, pos, B, copies, iters, nullptr, kvBf16);
          },
          py::arg("n_heads0"), py::arg("kv_mul"), py::arg("head_size"), py::arg("seq_len"), py::arg("pos"),
          py::arg("batch") = 1, py::arg("copies") = 32, py::arg("iters") = 200, py::arg("kv_bf16") = true,
          py::call_guard<py::gil_scoped_release>());
    m.def("trace_gemm_q40",
          [](int rows, int n, int M, int epi, int copies, int iters) {
              std::vector<unsigned long long> t;
              double us;
              {
                  py::gil_scoped_release rel;
                  us = benchGemmQ40(rows, n, M, epi, copies, iters, &t);
              }
              return py::make_tuple(us, t, (int)(t.size() / 8 / ((rows + 63) / 64)));
          },
          py::arg("rows"), py::arg("n"), py::arg("tokens"), py::arg("epi") = 0, py::arg("copies") = 8,
          py::arg("iters") = 50,
          "bench_gemm_q40, then one launch with per-workgroup stamps (gemm_dev.h gemmTrace): (us, u64[], splits)");
    m.def("trace_attention",
          [](int nh, int kvm, int hs, int seq, int pos, int B, int copies, int iters) {
              std::vector<unsigned long long> t;
              double us;
              {
                  py::gil_scoped_release rel;
                  us = benchAttention(nh, kvm, hs, seq, pos, B, copies, iters, &t);
              }
              return py::make_tuple(us, t);
          },
          py::arg("n_heads0"), py::arg("kv_mul"), py::arg("head_size"), py::arg("seq_len"), py::arg("pos"),
          py::arg("batch") = 1, py::arg("copies") = 32, py::arg("iters") = 50,
          "bench_attention, then one launch with per-workgroup stamps (kernels.h AttnArgs::trace): (us, u64[])");

    m.def("simulate_tp",
          [](const std::string &model, const std::string &bufferType, int world, std::vector<int> tokens, bool kvBf16,
             int gpuIndex, bool withFlags) -> py::object {
              EngineConfig c = makeConfig(model, bufferType, 1, 0, 8, 1, gpuIndex, false, kvBf16, py::none(), 1);
              std::vector<float> out;
              std::vector<int> blocks;
              {
                  py::gil_scoped_release rel;
                  out = simulateTensorParallel(c, world, tokens, &blocks);
              }
              const size_t vocab = out.size() / tokens.size();
              py::array_t<float> a({(py::ssize_t)tokens.size(), (py::ssize_t)vocab});
              std::memcpy(a.mutable_data(), out.data(), out.size() * 4);
              if (withFlags) return py::make_tuple(a, blocks);
              return a;
          },
          py::arg("model"), py::arg("buffer_type"), py::arg("world"), py::arg("tokens"), py::arg("kv_bf16") = false,
          py::arg("gpu_index") = 0, py::arg("attn_block_flags") = false);

    m.def("shard_bytes",
          [](const std::string &model, u32 world, u32 rank) {
              ModelFile f(model);
              const auto ranges = shardByteRanges(f.header(), f.tensors(), ShardPlan::make(f.header(), world, rank));
              u64 t = 0;
              for (auto &r : ranges) t += r.length;
              return t;
          },
          py::arg("model"), py::arg("world"), py::arg("rank"));

    m.def("rccl_unique_id", []() {
        auto v = rcclGetUniqueId();
        return py::bytes(std::string(v.begin(), v.end()));
    });

    py::class_<PyComm>(m, "XgmiComm")
        .def(py::init([](int rank, int world, size_t maxFloats, int gpuIndex) {
                 auto *c = new PyComm();
                 py::gil_scoped_release rel;
                 (void)hipSetDevice(gpuIndex);
                 c->comm = std::shared_ptr<DeviceComm>(makeXgmiComm(rank, world, maxFloats).release());
                 return c;
             }),
             py::arg("rank"), py::arg("world"), py::arg("max_floats"), py::arg("gpu_index") = 0)
        .def("handle", [](PyComm &c) { return py::bytes(xgmiHandle(c.comm.get())); })
        .def("connect",
             [](PyComm &c, const std::vector<py::bytes> &handles) {
                 std::vector<std::string> hs;
                 for (auto &h : handles) hs.push_back(std::string(h));
                 py::gil_scoped_release rel;
                 xgmiConnect(c.comm.get(), hs);
             })
        .def("timed_out", [](PyComm &c) { return xgmiTimedOut(c.comm.get()); })
        .def("set_low_latency", [](PyComm &c, bool on) { xgmiSetLowLatency(c.comm.get(), on); })
        .def("reset_error", [](PyComm &c) { xgmiResetError(c.comm.get()); })
        .def_property_readonly("cross_device", [](PyComm &c) { return xgmiCrossDevice(c.comm.get()); })
        .def_property_readonly("fenced", [](PyComm &c) { return xgmiFenced(c.comm.get()); })
        // µs per in-graph all-reduce of n floats (iters back-to-back collectives in one hipGraph)
        .def("bench_all_reduce",
             [](PyComm &c, size_t n, int iters) {
                 py::gil_scoped_release rel;
                 float *d;
                 hipStream_t s;
                 DL_HIP(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
                 DL_HIP(hipMalloc(&d, n * 4));
                 DL_HIP(hipMemset(d, 0, n * 4));
                 hipGraph_t g;
                 hipGraphExec_t ge;
                 DL_HIP(hipStreamBeginCapture(s, hipStreamCaptureModeThreadLocal));
                 for (int i = 0; i < iters; i++) c.comm->allReduceSum(d, n, s);
                 DL_HIP(hipStreamEndCapture(s, &g));
                 DL_HIP(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
                 DL_HIP(hipGraphLaunch(ge, s));
                 DL_HIP(hipStreamSynchronize(s));
                 hipEvent_t e0, e1;
                 DL_HIP(hipEventCreate(&e0));
                 DL_HIP(hipEventCreate(&e1));
                 DL_HIP(hipEventRecord(e0, s));
                 DL_HIP(hipGraphLaunch(ge, s));
                 DL_HIP(hipEventRecord(e1, s));
                 DL_HIP(hipEventSynchronize(e1));
                 float ms = 0;
                 DL_HIP(hipEventElapsedTime(&ms, e0, e1));
                 (void)hipGraphExecDestroy(ge);
                 (void)hipGraphDestroy(g);
                 (void)hipFree(d);
                 (void)hipStreamDestroy(s);
                 return (double)ms * 1000.0 / iters;
             },
             py::arg("n"), py::arg("iters") = 200)
        .def_property_readonly("rank", [](PyComm &c) { return c.comm->rank(); })
        .def_property_readonly("world", [](PyComm &c) { return c.comm->size(); })
        // test helpers: host vector in, collective result out (device round trip on the null stream)
        .def("all_reduce",
             [](PyComm &c, py::array_t<float, py::array::c_style | py::array::forcecast> x) {
                 const size_t n = (size_t)x.size();
                 py::array_t<float> out((py::ssize_t)n);
                 std::vector<float> h(x.data(), x.data() + n);
                 {
                     py::gil_scoped_release rel;
                     float *d;
                     DL_HIP(hipMalloc(&d, n * 4));
                     DL_HIP(hipMemcpy(d, h.data(), n * 4, hipMemcpyHostToDevice));
                     c.comm->allReduceSum(d, n, nullptr);
                     DL_HIP(hipMemcpy(h.data(), d, n * 4, hipMemcpyDeviceToHost));
                     DL_HIP(hipFree(d));
                 }
                 std::memcpy(out.mutable_data(), h.data(), n * 4);
                 return out;
             })
        .def("all_gather", [](PyComm &c, py::array_t<float, py::array::c_style | py::array::forcecast> x) {
            const size_t n = (size_t)x.size();
            const int w = c.comm->size();
            py::array_t<float> out((py::ssize_t)(n * w));
            std::vector<float> h(x.data(), x.data() + n), r(n * w);
            {
                py::gil_scoped_release rel;
                float *d, *o;
                DL_HIP(hipMalloc(&d, n * 4));
                DL_HIP(hipMalloc(&o, n * w * 4));
                DL_HIP(hipMemcpy(d, h.data(), n * 4, hipMemcpyHostToDevice));
                c.comm->allGather(d, o, n, nullptr);
                DL_HIP(hipMemcpy(r.data(), o, n * w * 4, hipMemcpyDeviceToHost));
                DL_HIP(hipFree(d));
                DL_HIP(hipFree(o));
            }
            std::memcpy(out.mutable_data(), r.data(), n * w * 4);
            return out;
        })
        // rank 0 gets every rank's x in rank order (other ranks: zeros)
        .def("gather_to_root", [](PyComm &c, py::array_t<float, py::array::c_style | py::array::forcecast> x) {
            const size_t n = (size_t)x.size();
            const int w = c.comm->size();
            py::array_t<float> out((py::ssize_t)(n * w));
            std::vector<float> h(x.data(), x.data() + n), r(n * w);
            {
                py::gil_scoped_release rel;
                float *d, *o;
                DL_HIP(hipMalloc(&d, n * 4));
                DL_HIP(hipMalloc(&o, n * w * 4));
                DL_HIP(hipMemset(o, 0, n * w * 4));
                DL_HIP(hipMemcpy(d, h.data(), n * 4, hipMemcpyHostToDevice));
                c.comm->gatherToRoot(d, o, n, nullptr);
                DL_HIP(hipMemcpy(r.data(), o, n * w * 4, hipMemcpyDeviceToHost));
                DL_HIP(hipFree(d));
                DL_HIP(hipFree(o));
            }
            std::memcpy(out.mutable_data(), r.data(), n * w * 4);
            return out;
        })
        .def("broadcast_ints", [](PyComm &c, std::vector<int> v, int root) {
            py::gil_scoped_release rel;
            int *d;
            DL_HIP(hipMalloc(&d, v.size() * 4));
            DL_HIP(hipMemcpy(d, v.data(), v.size() * 4, hipMemcpyHostToDevice));
            c.comm->broadcastInts(d, v.size(), root, nullptr);
            DL_HIP(hipMemcpy(v.data(), d, v.size() * 4, hipMemcpyDeviceToHost));
            DL_HIP(hipFree(d));
            return v;
        }, py::arg("values"), py::arg("root") = 0)
        // the engine's separate-collective schedule, eager or captured + replayed (engine.h)
        .def("schedule_check",
             [](PyComm &c, int layers, int rows, int dim, int vocab0, int runs, bool graph) {
                 py::gil_scoped_release rel;
                 return commScheduleCheck(*c.comm, layers, rows, dim, vocab0, runs, graph);
             },
             py::arg("layers") = 4, py::arg("rows") = 4, py::arg("dim") = 4096, py::arg("vocab0") = 1000,
             py::arg("runs") = 3, py::arg("graph") = true);

    // RCCL data plane (the fallback of the xGMI one): same helpers, created from an RCCL unique id
    py::class_<PyRcclComm, PyComm>(m, "RcclComm")
        .def(py::init([](py::bytes uid, int rank, int world, int gpuIndex) {
                 const std::string s = uid;
                 auto *c = new PyRcclComm();
                 py::gil_scoped_release rel;
                 DL_HIP(hipSetDevice(gpuIndex));
                 c->comm = std::shared_ptr<DeviceComm>(
                     makeRcclComm(std::vector<unsigned char>(s.begin(), s.end()), rank, world).release());
                 return c;
             }),
             py::arg("uid"), py::arg("rank") = 0, py::arg("world") = 1, py::arg("gpu_index") = 0);

    // compute-only TP rank (no peers, nothing exchanged): times a TP-N rank's shard on one GPU
    py::class_<PyComputeOnlyComm, PyComm>(m, "ComputeOnlyComm")
        .def(py::init([](int rank, int world, int gpuIndex) {
                 auto *c = new PyComputeOnlyComm();
                 DL_HIP(hipSetDevice(gpuIndex));
                 c->comm = std::shared_ptr<DeviceComm>(makeComputeOnlyComm(rank, world).release());
                 return c;
             }),
             py::arg("rank") = 0, py::arg("world") = 2, py::arg("gpu_index") = 0);

    py::class_<PyHipEngine>(m, "HipEngine")
        .def(py::init([](const std::string &model, const std::string &bufferType, u32 maxSeqLen, u32 maxBatch,
                         u32 nSlots, int gpuIndex, bool useGraphs, bool kvBf16, py::object synthetic, u64 seed,
                         int rank, int world, py::object uid, py::object comm, const std::string &syncType,
                         u32 kvPages, u32 kvPageSize, bool batchInvariant) {
                 EngineConfig c = makeConfig(model, bufferType, 1, maxSeqLen, maxBatch, nSlots, gpuIndex, useGraphs,
                                             kvBf16, synthetic, seed);
                 c.syncType = parseFloatType(syncType);
                 c.kvPages = kvPages;
                 c.kvPageSize = kvPageSize;
                 c.batchInvariant = batchInvariant;
                 auto *e = new PyHipEngine();
                 if (!comm.is_none()) e->comm = comm.cast<PyComm &>().comm;
                 py::gil_scoped_release rel;
                 if (world > 1 && !e->comm) {
                     std::string s;
                     {
                         py::gil_scoped_acquire acq;
                         s = uid.cast<std::string>();
                     }
                     (void)hipSetDevice(gpuIndex >= 0 ? gpuIndex : 0);
                     e->comm = std::shared_ptr<DeviceComm>(
                         makeRcclComm(std::vector<unsigned char>(s.begin(), s.end()), rank, world).release());
                 }
                 e->engine = makeHipEngine(c, e->comm.get());
                 return e;
             }),
             py::arg("model") = "", py::arg("buffer_type") = "q80", py::arg("max_seq_len") = 0,
             py::arg("max_batch") = 32, py::arg("n_slots") = 1, py::arg("gpu_index") = 0, py::arg("use_graphs") = true,
             py::arg("kv_bf16") = true, py::arg("synthetic") = py::none(), py::arg("seed") = 1234, py::arg("rank") = 0,
             py::arg("world") = 1, py::arg("uid") = py::none(), py::arg("comm") = py::none(),
             py::arg("sync_type") = "f32", py::arg("kv_pages") = 0, py::arg("kv_page_size") = 256,
             py::arg("batch_invariant") = false)
        .def_property_readonly("header", [](const PyHipEngine &e) { return headerToDict(e.engine->header()); })
        .def_property_readonly("device_bytes", [](const PyHipEngine &e) { return e.engine->deviceBytes(); })
        .def_property_readonly("tp_fused", [](const PyHipEngine &e) { return e.engine->tpFused(); })
        .def_property_readonly("attn_block", [](const PyHipEngine &e) { return e.engine->attnBlock(); })
        .def_property_readonly("wo_attn", [](const PyHipEngine &e) { return e.engine->woAttn(); })
        .def_property_readonly("prenorm", [](const PyHipEngine &e) { return e.engine->prenorm(); })
        .def_property_readonly("ffn_block", [](const PyHipEngine &e) { return e.engine->ffnBlock(); })
        .def("trace_attn_block",
             [](PyHipEngine &e, int token, int pos, int slot, int layer) {
                 py::gil_scoped_release rel;
                 return e.engine->traceAttnBlock(token, pos, slot, layer);
             },
             py::arg("token"), py::arg("pos"), py::arg("slot") = 0, py::arg("layer") = 1)
        .def_property_readonly("fused_grid_max", [](const PyHipEngine &e) { return e.engine->fusedGridMax(); })
        .def_property_readonly("kv_pages_free", [](const PyHipEngine &e) { return e.engine->kvPagesFree(); })
        .def("tp_batched_fused", [](const PyHipEngine &e, int n) { return e.engine->tpBatchedFused(n); }, py::arg("n"))
        .def_property_readonly("load_stats",
                               [](const PyHipEngine &e) {
                                   const Backend::LoadStats l = e.engine->loadStats();
                                   py::dict d;
                                   d["ms"] = l.ms;
                                   d["file_bytes"] = l.fileBytes;
                                   d["device_bytes"] = l.deviceBytes;
                                   return d;
                               })
        .def("forward", [](PyHipEngine &e, std::vector<int> t, std::vector<int> p, std::vector<int> s) { return runForward(*e.engine, t, p, s); },
             py::arg("tokens"), py::arg("positions"), py::arg("slots"))
        .def("forward_sample",
             [](PyHipEngine &e, std::vector<int> t, std::vector<int> p, std::vector<int> s, std::vector<float> temps,
                std::vector<float> topps, std::vector<float> coins) { return runSample(*e.engine, t, p, s, temps, topps, coins); },
             py::arg("tokens"), py::arg("positions"), py::arg("slots"), py::arg("temperatures"), py::arg("topps"),
             py::arg("coins"))
        .def("forward_argmax", [](PyHipEngine &e, std::vector<int> t, std::vector<int> p, std::vector<int> s) { return runArgmax(*e.engine, t, p, s); },
             py::arg("tokens"), py::arg("positions"), py::arg("slots"))
        .def("last_stats",
             [](const PyHipEngine &e) {  // (compute ms, sync ms, sent B, recv B, xchg ms) of the last call
                 ForwardStats s = e.engine->lastStats();
                 return py::make_tuple(s.computeMs, s.syncMs, s.sentBytes, s.recvBytes, s.xchgMs);
             })
        .def("decode_greedy",
             [](PyHipEngine &e, int steps, std::vector<int> tokens, std::vector<int> pos, std::vector<int> slots) {
                 const int nSeq = (int)tokens.size();
                 std::vector<int> out((size_t)steps * nSeq);
                 double ms;
                 {
                     py::gil_scoped_release rel;
                     ms = e.engine->decodeGreedyBatch(steps, nSeq, tokens.data(), pos.data(), slots.data(), out.data());
                 }
                 return py::make_tuple(ms, out);
             },
             py::arg("steps"), py::arg("tokens"), py::arg("positions"), py::arg("slots"))
        .def("profile_forward", [](PyHipEngine &e, std::vector<int> t, std::vector<int> p, std::vector<int> s) {
            e.engine->profileForward((int)t.size(), t.data(), p.data(), s.data());
        })
        .def("synchronize", [](PyHipEngine &e) { e.engine->synchronize(); });

}
