// Tokenizer (.t format), sampler, chat templates and stop-string detector.
//
// Behaviour parity with the reference (src/tokenizer.hpp, src/tokenizer.cpp):
//   .t parsing incl. legacy magic              tokenizer.cpp:42-170
//   regular/special vocab split at bosId       tokenizer.cpp:137-152
//   encode: special-prefix match, byte accumulation until a regular hit, greedy score merges
//                                              tokenizer.cpp:301-380
//   streaming UTF-8 safe decode               tokenizer.cpp:214-299
//   sampler (xorshift, temperature, top-p)     tokenizer.cpp:25-36, 382-502
//   chat templates llama2/llama3/deepSeek3     tokenizer.cpp:538-612
//   EosDetector with left/right padding        tokenizer.cpp:614-699
#pragma once

#include <string>
#include <unordered_map>
#include <vector>

#include "../core/common.h"

namespace dl {

class Tokenizer {
  public:
    explicit Tokenizer(const std::string &path, bool verbose = true);
    static Tokenizer fromBytes(const std::vector<u8> &bytes, bool verbose = false);

    std::vector<int> encode(const std::string &text, bool addBos, bool addSpecialTokens) const;
    // Streaming decode: returns true and sets `out` when printable text is available.
    bool decode(int token, std::string &out);
    void resetDecoder() { pending_.clear(); }
    bool isEos(int token) const;

    int vocabSize() const { return (int)vocab_.size(); }
    int bosId() const { return bosId_; }
    const std::vector<int> &eosTokenIds() const { return eos_; }
    const std::string &piece(int id) const { return vocab_.at(id); }
    float score(int id) const { return scores_.at(id); }
    const std::string &chatTemplate() const { return chatTemplate_; }
    bool hasChatTemplate() const { return hasChatTemplate_; }
    u32 maxTokenLength() const { return maxTokenLength_; }

  private:
    Tokenizer() = default;
    void parse(const u8 *data, u64 size, bool verbose);
    int findRegular(const std::string &s) const;
    int findSpecialPrefix(const char *text, size_t remaining) const;

    std::vector<std::string> vocab_;
    std::vector<float> scores_;
    std::vector<int> eos_;
    std::string chatTemplate_;
    bool hasChatTemplate_ = false;
    int bosId_ = -1;
    u32 maxTokenLength_ = 0;
    int regularVocabSize_ = 0;
    std::vector<int> specialIds_;
    std::unordered_map<std::string, int> regular_;
    std::string pending_;
};

// Per-sequence streaming decoder (the Tokenizer's own decode() keeps one shared buffer, like the
// reference; concurrent requests each need their own UTF-8 carry-over).
class TokenDecoder {
  public:
    explicit TokenDecoder(const Tokenizer &t) : t_(t) {}
    bool decode(int token, std::string &out);
    void reset() { pending_.clear(); }

  private:
    const Tokenizer &t_;
    std::string pending_;
};

class Sampler {
  public:
    Sampler(int vocabSize, float temperature, float topp, u64 seed);
    // NOTE: modifies `logits` in place when temperature > 0 (as the reference does).
    int sample(float *logits);
    // The random draw sample() makes (advances the generator identically); 0 when greedy. A
    // device sampler given this coin reproduces sample() (Backend::forwardSample).
    float drawCoin() { return temperature_ == 0.0f ? 0.0f : randomF32Impl(); }
    // sample() with an explicit coin (logits modified in place when temperature > 0)
    int sampleWithCoin(float *logits, float coin);
    float topp() const { return topp_; }
    void setTemp(float t) { temperature_ = t; }
    void setTopp(float p) { topp_ = p; }
    void setSeed(u64 s) { rng_ = s; }
    float temperature() const { return temperature_; }

  private:
    float randomF32Impl();
    int vocab_;
    float temperature_;
    float topp_;
    u64 rng_;
    std::vector<std::pair<float, int>> probIndex_;
};

u32 randomU32(u64 *state);
float randomF32(u64 *state);
void softmaxInPlace(float *x, u64 n);
int argmax(const float *x, u64 n);

enum class ChatTemplateType { UNKNOWN, LLAMA2, LLAMA3, DEEP_SEEK3 };
ChatTemplateType parseChatTemplateType(const std::string &s);
const char *chatTemplateTypeName(ChatTemplateType t);

struct ChatItem {
    std::string role;
    std::string message;
};

struct GeneratedChat {
    std::string content;
    std::string publicPrompt;  // text the model is "already saying" (e.g. "<think>\n")
};

class ChatTemplateGenerator {
  public:
    ChatTemplateGenerator(ChatTemplateType type, const std::string &chatTemplate, const std::string &eos,
                          bool verbose = true);
    GeneratedChat generate(const std::vector<ChatItem> &items, bool appendGenerationPrompt) const;
    ChatTemplateType type() const { return type_; }

  private:
    ChatTemplateType type_;
    std::string eos_;
};

enum class EosResult { NOT_EOS = 0, MAYBE_EOS = 1, EOS = 2 };

class EosDetector {
  public:
    EosDetector(std::vector<int> tokens, std::vector<std::string> pieces, int paddingLeft, int paddingRight);
    // piece may be null (nothing to append)
    EosResult append(int tokenId, const char *piece);
    // Returns false when there is no delta to emit.
    bool getDelta(std::string &out) const;
    void reset() {
        buffer_.clear();
        eosPos_ = -1;
    }

  private:
    bool isEos(int token) const;
    std::vector<int> tokens_;
    std::vector<std::string> pieces_;
    int paddingLeft_, paddingRight_;
    std::string buffer_;
    long eosPos_ = -1;
};

// Stop pieces derived from the tokenizer's EOS tokens (tokenizer.cpp:512-529).
struct ChatStops {
    std::vector<std::string> stops;
    size_t maxStopLength = 0;
    explicit ChatStops(const Tokenizer &t);
};

}  // namespace dl
