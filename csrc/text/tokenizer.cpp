#include "tokenizer.h"

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <fstream>

namespace dl {

namespace {
enum TokKey {
    T_VERSION = 0,
    T_VOCAB_SIZE = 1,
    T_MAX_TOKEN_LENGTH = 2,
    T_BOS_ID = 3,
    T_EOS_ID = 4,
    T_PAD_ID = 5,
    T_CHAT_EOS_ID = 6,
    T_CHAT_TEMPLATE = 7,
    T_CHAT_STOP = 8,
    T_N_EOS_TOKENS = 9,
};

struct Reader {
    const u8 *p;
    u64 n, off = 0;
    template <typename T>
    T get() {
        if (off + sizeof(T) > n) throw Error("tokenizer file truncated");
        T v;
        std::memcpy(&v, p + off, sizeof(T));
        off += sizeof(T);
        return v;
    }
    std::string bytes(u64 len) {
        if (off + len > n) throw Error("tokenizer file truncated");
        std::string s((const char *)p + off, len);
        off += len;
        return s;
    }
    void skip(u64 len) {
        if (off + len > n) throw Error("tokenizer file truncated");
        off += len;
    }
};
}  // namespace

Tokenizer::Tokenizer(const std::string &path, bool verbose) {
    std::ifstream f(path, std::ios::binary);
    if (!f) throw Error("Failed to open tokenizer file: " + path);
    std::vector<u8> data((std::istreambuf_iterator<char>(f)), std::istreambuf_iterator<char>());
    parse(data.data(), data.size(), verbose);
}

Tokenizer Tokenizer::fromBytes(const std::vector<u8> &bytes, bool verbose) {
    Tokenizer t;
    t.parse(bytes.data(), bytes.size(), verbose);
    return t;
}

void Tokenizer::parse(const u8 *data, u64 size, bool verbose) {
    Reader r{data, size};
    const i32 magic = r.get<i32>();
    int vocabSize = 0;
    if (magic == 0x567123) {
        vocabSize = (int)r.get<u32>();
        maxTokenLength_ = r.get<u32>();
        bosId_ = r.get<i32>();
        eos_.push_back(r.get<i32>());
        (void)r.get<i32>();  // pad
    } else if (magic == 0x567124) {
        const i32 headerSize = r.get<i32>();
        const int nKv = (headerSize - 8) / 4;
        int version = -1, chatTemplateLength = -1, nEos = 0;
        u64 skipBytes = 0;
        for (int i = 0; i < nKv; i += 2) {
            const i32 key = r.get<i32>(), value = r.get<i32>();
            switch (key) {
                case T_VERSION: version = value; break;
                case T_VOCAB_SIZE: vocabSize = value; break;
                case T_MAX_TOKEN_LENGTH: maxTokenLength_ = (u32)value; break;
                case T_BOS_ID: bosId_ = value; break;
                case T_EOS_ID: eos_.push_back(value); break;
                case T_CHAT_EOS_ID: eos_.push_back(value); break;
                case T_CHAT_TEMPLATE: chatTemplateLength = value; break;
                case T_CHAT_STOP: skipBytes += (u64)value; break;  // ignored, skipped
                case T_PAD_ID: break;
                case T_N_EOS_TOKENS: nEos = value; break;
                default: throw Error("Invalid tokenizer header key:" + std::to_string(key));
            }
        }
        if (version != 1) throw Error("Old tokenizer version, please regenerate your tokenizer");
        r.skip(skipBytes);
        if (chatTemplateLength > 0) {
            chatTemplate_ = r.bytes((u64)chatTemplateLength);
            hasChatTemplate_ = true;
        }
        for (int i = 0; i < nEos; i++) eos_.push_back(r.get<i32>());
    } else {
        throw Error("Invalid tokenizer file");
    }
    if (maxTokenLength_ < 1) throw Error("Invalid tokenizer max token length");
    DL_CHECK(vocabSize > 0, "tokenizer vocab size");
    vocab_.resize(vocabSize);
    scores_.resize(vocabSize);
    for (int i = 0; i < vocabSize; i++) {
        scores_[i] = r.get<float>();
        const i32 len = r.get<i32>();
        DL_CHECK(len >= 0, "negative token length");
        vocab_[i] = r.bytes((u64)len);
    }
    // The reference assumes bosId splits regular and special tokens (tokenizer.cpp:137-138): that
    // holds for Llama-3-style vocabularies whose specials are appended at the end. Tokenizers that
    // put their control tokens first (HF-trained BPE, sentencepiece <unk>/<s>/</s>) get the leading
    // run of bos/eos/"<...>" marker tokens as the special set instead.
    std::vector<bool> special(vocabSize, false);
    if (bosId_ < 0 || bosId_ >= vocabSize / 2) {
        for (int i = std::max(bosId_, 0); bosId_ >= 0 && i < vocabSize; i++) special[i] = true;
    } else {
        auto isMarker = [&](int i) {
            const std::string &v = vocab_[i];
            if (i == bosId_ || std::find(eos_.begin(), eos_.end(), i) != eos_.end()) return true;
            return v.size() >= 3 && v.front() == '<' && v.back() == '>';
        };
        for (int i = 0; i < vocabSize && isMarker(i); i++) special[i] = true;
        for (int e : eos_)
            if (e >= 0 && e < vocabSize) special[e] = true;
        special[bosId_] = true;
    }
    regular_.reserve(vocabSize * 2);
    for (int i = 0; i < vocabSize; i++) {
        if (special[i])
            specialIds_.push_back(i);
        else
            regular_.emplace(vocab_[i], i);  // first id wins
    }
    regularVocabSize_ = vocabSize - (int)specialIds_.size();
    if (verbose && logLevel() >= 1) {
        if (bosId_ >= 0 && bosId_ < vocabSize) std::printf("📄 BosId: %d (%s)\n", bosId_, vocab_[bosId_].c_str());
        if (!eos_.empty()) {
            std::printf("📄 EosId: ");
            for (int e : eos_)
                if (e >= 0 && e < vocabSize) std::printf("%d (%s) ", e, vocab_[e].c_str());
            std::printf("\n");
        }
        std::printf("📄 RegularVocabSize: %d\n", regularVocabSize_);
        std::printf("📄 SpecialVocabSize: %d\n", (int)specialIds_.size());
    }
}

int Tokenizer::findRegular(const std::string &s) const {
    auto it = regular_.find(s);
    return it == regular_.end() ? -1 : it->second;
}

int Tokenizer::findSpecialPrefix(const char *text, size_t remaining) const {
    for (int id : specialIds_) {
        const std::string &v = vocab_[id];
        if (v.size() <= remaining && std::memcmp(v.data(), text, v.size()) == 0) return id;
    }
    return -1;
}

std::vector<int> Tokenizer::encode(const std::string &text, bool addBos, bool addSpecialTokens) const {
    std::vector<int> tokens;
    tokens.reserve(text.size() + 2);
    if (addBos) tokens.push_back(bosId_);
    std::string acc;
    const char *c = text.c_str();
    const size_t n = text.size();
    for (size_t i = 0; i < n; i++) {
        if (addSpecialTokens) {
            const int sid = findSpecialPrefix(c + i, n - i);
            if (sid >= 0) {
                tokens.push_back(sid);
                i += vocab_[sid].size() - 1;
                continue;
            }
        }
        acc.push_back(c[i]);
        const int id = findRegular(acc);
        if (id != -1) {
            tokens.push_back(id);
            acc.clear();
        }
    }
    // Bytes that never formed a regular token are dropped (the reference asserts here).
    // Greedy merges of the best-scoring adjacent pair.
    std::string buf;
    while (true) {
        float bestScore = -1e10f;
        int bestId = -1, bestIdx = -1;
        for (size_t i = 0; i + 1 < tokens.size(); i++) {  // every pair, BOS included (reference order)
            buf.assign(vocab_[tokens[i]]);
            buf.append(vocab_[tokens[i + 1]]);
            const int id = findRegular(buf);
            if (id != -1 && scores_[id] > bestScore) {
                bestScore = scores_[id];
                bestId = id;
                bestIdx = (int)i;
            }
        }
        if (bestIdx == -1) break;
        tokens[bestIdx] = bestId;
        tokens.erase(tokens.begin() + bestIdx + 1);
    }
    return tokens;
}

bool Tokenizer::isEos(int token) const {
    for (int e : eos_)
        if (e == token) return true;
    return false;
}

// Emits all complete UTF-8 characters of the pending byte stream, keeps an incomplete tail,
// and replaces invalid sequences by U+FFFD (same recovery policy as tokenizer.cpp:214-279).
static bool flushUtf8(std::string &pending, std::string &out) {
    out.clear();
    size_t i = 0, checkpointSrc = 0;
    size_t checkpointDst = 0;
    unsigned expect = 0;
    const size_t n = pending.size();
    while (i < n) {
        const unsigned char c = (unsigned char)pending[i];
        bool recover = false;
        if (expect) {
            if ((c & 0xc0) == 0x80) {
                out.push_back((char)c);
                i++;
                expect--;
            } else {
                recover = true;
            }
        } else if (c <= 0x7f) {
            out.push_back((char)c);
            i++;
        } else if (c >= 0xc0 && c <= 0xdf) {
            out.push_back((char)c);
            i++;
            expect = 1;
        } else if (c >= 0xe0 && c <= 0xef) {
            out.push_back((char)c);
            i++;
            expect = 2;
        } else if (c >= 0xf0 && c <= 0xf7) {
            out.push_back((char)c);
            i++;
            expect = 3;
        } else {
            recover = true;
        }
        if (!recover) {
            if (!expect) {
                checkpointDst = out.size();
                checkpointSrc = i;
            }
        } else {
            if (expect)
                expect = 0;
            else
                i++;
            out.resize(checkpointDst);
            out.append("\xef\xbf\xbd");
            checkpointDst = out.size();
            checkpointSrc = i;
            std::fprintf(stderr, "Tokenizer: decoded invalid utf8 -- attempting stream recover\n");
        }
    }
    pending.erase(0, checkpointSrc);
    out.resize(checkpointDst);
    return !out.empty();
}

bool Tokenizer::decode(int token, std::string &out) {
    out.clear();
    if (token == bosId_) return false;
    if (isEos(token)) {
        if (!pending_.empty()) {
            out = pending_;
            pending_.clear();
            return true;
        }
        return false;
    }
    DL_CHECK(token >= 0 && token < (int)vocab_.size(), "token id out of range");
    pending_.append(vocab_[token]);
    return flushUtf8(pending_, out);
}

bool TokenDecoder::decode(int token, std::string &out) {
    out.clear();
    if (token == t_.bosId()) return false;
    if (t_.isEos(token)) {
        if (!pending_.empty()) {
            out = pending_;
            pending_.clear();
            return true;
        }
        return false;
    }
    DL_CHECK(token >= 0 && token < t_.vocabSize(), "token id out of range");
    pending_.append(t_.piece(token));
    return flushUtf8(pending_, out);
}

// ---------------------------------------------------------------- sampler

u32 randomU32(u64 *state) {
    // xorshift* (same generator as the reference so seeded runs reproduce)
    *state ^= *state >> 12;
    *state ^= *state << 25;
    *state ^= *state >> 27;
    return (u32)((*state * 0x2545F4914F6CDD1Dull) >> 32);
}

float randomF32(u64 *state) { return (float)(randomU32(state) >> 8) / 16777216.0f; }

void softmaxInPlace(float *x, u64 n) {
    if (n == 0) return;
    float mx = x[0];
    for (u64 i = 1; i < n; i++) mx = std::max(mx, x[i]);
    float sum = 0.f;
    for (u64 i = 0; i < n; i++) {
        x[i] = std::exp(x[i] - mx);
        sum += x[i];
    }
    const float inv = 1.0f / sum;
    for (u64 i = 0; i < n; i++) x[i] *= inv;
}

int argmax(const float *x, u64 n) {
    int best = 0;
    float bv = x[0];
    for (u64 i = 1; i < n; i++)
        if (x[i] > bv) {
            bv = x[i];
            best = (int)i;
        }
    return best;
}

Sampler::Sampler(int vocabSize, float temperature, float topp, u64 seed)
    : vocab_(vocabSize), temperature_(temperature), topp_(topp), rng_(seed) {
    probIndex_.reserve(vocabSize);
}

float Sampler::randomF32Impl() { return randomF32(&rng_); }

int Sampler::sample(float *logits) {
    if (temperature_ == 0.0f) return argmax(logits, vocab_);
    return sampleWithCoin(logits, randomF32(&rng_));
}

int Sampler::sampleWithCoin(float *logits, float coin) {
    if (temperature_ == 0.0f) return argmax(logits, vocab_);
    for (int i = 0; i < vocab_; i++) logits[i] /= temperature_;
    softmaxInPlace(logits, vocab_);
    if (topp_ <= 0.f || topp_ >= 1.f) {
        float cdf = 0.f;
        for (int i = 0; i < vocab_; i++) {
            cdf += logits[i];
            if (coin < cdf) return i;
        }
        return vocab_ - 1;
    }
    // nucleus sampling: candidates above the cutoff, sorted by probability (descending)
    const float cutoff = (1.0f - topp_) / (float)(vocab_ - 1);
    probIndex_.clear();
    for (int i = 0; i < vocab_; i++)
        if (logits[i] >= cutoff) probIndex_.emplace_back(logits[i], i);
    std::sort(probIndex_.begin(), probIndex_.end(),
              [](const std::pair<float, int> &a, const std::pair<float, int> &b) { return a.first > b.first; });
    float cum = 0.f;
    int last = (int)probIndex_.size() - 1;
    for (int i = 0; i < (int)probIndex_.size(); i++) {
        cum += probIndex_[i].first;
        if (cum > topp_) {
            last = i;
            break;
        }
    }
    const float r = coin * cum;
    float cdf = 0.f;
    for (int i = 0; i <= last; i++) {
        cdf += probIndex_[i].first;
        if (r < cdf) return probIndex_[i].second;
    }
    return probIndex_[last].second;
}

// ---------------------------------------------------------------- chat templates

ChatTemplateType parseChatTemplateType(const std::string &s) {
    if (s == "llama2") return ChatTemplateType::LLAMA2;
    if (s == "llama3") return ChatTemplateType::LLAMA3;
    if (s == "deepSeek3") return ChatTemplateType::DEEP_SEEK3;
    throw Error("Invalid chat template type: " + s);
}

const char *chatTemplateTypeName(ChatTemplateType t) {
    switch (t) {
        case ChatTemplateType::LLAMA2: return "llama2";
        case ChatTemplateType::LLAMA3: return "llama3";
        case ChatTemplateType::DEEP_SEEK3: return "deepSeek3";
        default: return "unknown";
    }
}

ChatTemplateGenerator::ChatTemplateGenerator(ChatTemplateType type, const std::string &chatTemplate,
                                             const std::string &eos, bool verbose)
    : type_(type), eos_(eos) {
    if (type_ == ChatTemplateType::UNKNOWN) {
        if (chatTemplate.empty()) throw Error("The tokenizer does not include chat template");
        if (chatTemplate.find("[INST]") != std::string::npos)
            type_ = ChatTemplateType::LLAMA2;
        else if (chatTemplate.find("<|start_header_id|>") != std::string::npos)
            type_ = ChatTemplateType::LLAMA3;
        else if (chatTemplate.find("<\xef\xbd\x9c" "Assistant\xef\xbd\x9c>") != std::string::npos)
            type_ = ChatTemplateType::DEEP_SEEK3;
        else
            throw Error("Not supported chat template");
    }
    if (verbose && logLevel() >= 1) std::printf("⭐ Chat template: %s\n", chatTemplateTypeName(type_));
}

GeneratedChat ChatTemplateGenerator::generate(const std::vector<ChatItem> &items, bool appendGenerationPrompt) const {
    GeneratedChat g;
    std::string &b = g.content;
    const std::string fwUser = "<\xef\xbd\x9cUser\xef\xbd\x9c>";
    const std::string fwAssistant = "<\xef\xbd\x9c" "Assistant\xef\xbd\x9c>";
    if (type_ == ChatTemplateType::LLAMA2) {
        size_t i = 0;
        if (items.size() >= 2 && items[0].role == "system" && items[1].role == "user") {
            b += "[INST] <<SYS>>\n" + items[0].message + "\n<</SYS>>\n\n" + items[1].message + " [/INST]" + eos_;
            i = 2;
        }
        for (; i < items.size(); i++) {
            if (items[i].role == "assistant")
                b += items[i].message + eos_;
            else if (items[i].role == "user")
                b += "[INST] " + items[i].message + " [/INST]" + eos_;
        }
    } else if (type_ == ChatTemplateType::LLAMA3) {
        for (const auto &it : items)
            b += "<|start_header_id|>" + it.role + "<|end_header_id|>\n\n" + it.message + eos_;
        if (appendGenerationPrompt) b += "<|start_header_id|>assistant<|end_header_id|>\n\n";
    } else if (type_ == ChatTemplateType::DEEP_SEEK3) {
        size_t i = 0;
        if (!items.empty() && items[0].role == "system") {
            b += items[0].message;
            i = 1;
        }
        for (; i < items.size(); i++) {
            if (items[i].role == "user")
                b += fwUser + items[i].message;
            else if (items[i].role == "assistant")
                b += fwAssistant + items[i].message;
        }
        if (appendGenerationPrompt) {
            b += fwAssistant + "<think>\n";
            g.publicPrompt = "<think>\n";
        }
    }
    return g;
}

// ---------------------------------------------------------------- EOS detector

EosDetector::EosDetector(std::vector<int> tokens, std::vector<std::string> pieces, int paddingLeft, int paddingRight)
    : tokens_(std::move(tokens)), pieces_(std::move(pieces)), paddingLeft_(paddingLeft), paddingRight_(paddingRight) {}

bool EosDetector::isEos(int token) const {
    for (int t : tokens_)
        if (t == token) return true;
    return false;
}

EosResult EosDetector::append(int tokenId, const char *piece) {
    if (piece != nullptr) buffer_.append(piece);
    if (isEos(tokenId)) {
        eosPos_ = (long)buffer_.size();
        return EosResult::EOS;
    }
    eosPos_ = -1;
    const long bufferPos = (long)buffer_.size();
    for (size_t s = 0; s < pieces_.size(); s++) {
        const long pieceSize = (long)pieces_[s].size();
        if (bufferPos > pieceSize + paddingLeft_ + paddingRight_) continue;
        for (int lo = 0; lo <= paddingLeft_; lo++) {
            long n = bufferPos - lo;
            if (n <= 0 || n > pieceSize + paddingRight_) continue;
            if (n > pieceSize) n = pieceSize;
            if (std::strncmp(buffer_.c_str() + lo, pieces_[s].c_str(), (size_t)n) == 0) {
                if (n == pieceSize) {
                    eosPos_ = lo;
                    buffer_.resize((size_t)lo);
                    return EosResult::EOS;
                }
                return EosResult::MAYBE_EOS;
            }
        }
    }
    return EosResult::NOT_EOS;
}

bool EosDetector::getDelta(std::string &out) const {
    if (buffer_.empty()) return false;
    if (eosPos_ == 0) return false;
    out = buffer_;
    return true;
}

ChatStops::ChatStops(const Tokenizer &t) {
    for (int id : t.eosTokenIds()) {
        stops.push_back(t.piece(id));
        maxStopLength = std::max(maxStopLength, t.piece(id).size());
    }
}

}  // namespace dl
