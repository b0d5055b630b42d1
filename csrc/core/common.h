// Core shared definitions for the MI355X-native distributed Llama engine.
//
// Float-type codes are the on-disk codes of the `.m` format
// (reference: src/nn/nn-quants.hpp:56-62, converter/writer.py:6-10).
#pragma once

#include <chrono>
#include <cstddef>
#include <cstdint>
#include <stdexcept>
#include <string>

namespace dl {

using u8 = std::uint8_t;
using i8 = std::int8_t;
using u16 = std::uint16_t;
using u32 = std::uint32_t;
using i32 = std::int32_t;
using u64 = std::uint64_t;
using i64 = std::int64_t;

enum class FloatType : int {
    UNK = -1,
    F32 = 0,
    F16 = 1,
    Q40 = 2,
    Q80 = 3,
};

constexpr int kQBlock = 32;          // Q40/Q80 block size (nn-quants.hpp:53-54)
constexpr int kQ40BlockBytes = 18;   // f16 d + 16 bytes of nibbles
constexpr int kQ80BlockBytes = 34;   // f16 d + 32 int8

const char *floatTypeName(FloatType t);
FloatType parseFloatType(const std::string &s);

// Bytes needed to store `n` consecutive elements of type `t` (n must be block aligned for quants).
u64 floatTypeBytes(FloatType t, u64 n);

class Error : public std::runtime_error {
  public:
    using std::runtime_error::runtime_error;
};

#define DL_CHECK(cond, msg)                                                                        \
    do {                                                                                           \
        if (!(cond)) throw ::dl::Error(std::string("check failed: ") + (msg) + " [" #cond "] at " + \
                                       __FILE__ + ":" + std::to_string(__LINE__));                 \
    } while (0)

class Timer {
  public:
    Timer() { reset(); }
    void reset() { t0_ = std::chrono::steady_clock::now(); }
    double elapsedMs() const {
        return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0_).count();
    }
    u64 elapsedUs() const {
        return (u64)std::chrono::duration_cast<std::chrono::microseconds>(std::chrono::steady_clock::now() - t0_)
            .count();
    }

  private:
    std::chrono::steady_clock::time_point t0_;
};

// Log verbosity: 0 = quiet (errors only), 1 = normal (reference-style emoji lines), 2 = debug.
int logLevel();
void setLogLevel(int level);

}  // namespace dl
