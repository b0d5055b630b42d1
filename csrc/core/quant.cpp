#include "quant.h"

#include <immintrin.h>

#include <atomic>
#include <cmath>
#include <cstring>

namespace dl {

static std::atomic<int> gLogLevel{1};
int logLevel() { return gLogLevel.load(); }
void setLogLevel(int level) { gLogLevel.store(level); }

const char *floatTypeName(FloatType t) {
    switch (t) {
        case FloatType::UNK: return "F_UNK";
        case FloatType::F32: return "F_32";
        case FloatType::F16: return "F_16";
        case FloatType::Q40: return "F_Q40";
        case FloatType::Q80: return "F_Q80";
    }
    throw Error("unknown float type");
}

FloatType parseFloatType(const std::string &s) {
    if (s == "f32") return FloatType::F32;
    if (s == "f16") return FloatType::F16;
    if (s == "q40") return FloatType::Q40;
    if (s == "q80") return FloatType::Q80;
    throw Error("Invalid float type: " + s);
}

u64 floatTypeBytes(FloatType t, u64 n) {
    switch (t) {
        case FloatType::F32: return n * 4;
        case FloatType::F16: return n * 2;
        case FloatType::Q40: DL_CHECK(n % kQBlock == 0, "Q40 size must be block aligned"); return n / kQBlock * kQ40BlockBytes;
        case FloatType::Q80: DL_CHECK(n % kQBlock == 0, "Q80 size must be block aligned"); return n / kQBlock * kQ80BlockBytes;
        default: throw Error("floatTypeBytes: unsupported type");
    }
}

// F16C gives IEEE round-to-nearest-even conversions in hardware (x86-64-v3 baseline).
float f16ToF32(u16 h) { return _cvtsh_ss(h); }
u16 f32ToF16(float f) { return (u16)_cvtss_sh(f, _MM_FROUND_TO_NEAREST_INT); }

void quantizeQ80(const float *x, BlockQ80 *out, u64 n) {
    DL_CHECK(n % kQBlock == 0, "quantizeQ80: n % 32");
    const u64 nb = n / kQBlock;
    for (u64 b = 0; b < nb; b++) {
        const float *v = x + b * kQBlock;
        float amax = 0.f;
        for (int j = 0; j < kQBlock; j++) amax = std::fmax(amax, std::fabs(v[j]));
        const float d = amax / 127.0f;
        const float id = d != 0.f ? 1.0f / d : 0.f;
        out[b].d = f32ToF16(d);
        for (int j = 0; j < kQBlock; j++) {
            float q = std::nearbyint(v[j] * id);
            q = q > 127.f ? 127.f : (q < -127.f ? -127.f : q);
            out[b].qs[j] = (i8)q;
        }
    }
}

void dequantizeQ80(const BlockQ80 *in, float *out, u64 n) {
    const u64 nb = n / kQBlock;
    for (u64 b = 0; b < nb; b++) {
        const float d = f16ToF32(in[b].d);
        for (int j = 0; j < kQBlock; j++) out[b * kQBlock + j] = in[b].qs[j] * d;
    }
}

void quantizeQ40(const float *x, BlockQ40 *out, u64 n) {
    DL_CHECK(n % kQBlock == 0, "quantizeQ40: n % 32");
    const u64 nb = n / kQBlock;
    for (u64 b = 0; b < nb; b++) {
        const float *v = x + b * kQBlock;
        // signed value with the largest magnitude; d = max / -8 (writer.py:35-37)
        float amax = 0.f, mx = 0.f;
        for (int j = 0; j < kQBlock; j++) {
            if (amax < std::fabs(v[j])) {
                amax = std::fabs(v[j]);
                mx = v[j];
            }
        }
        const float d = mx / -8.0f;
        const float id = d != 0.f ? 1.0f / d : 0.f;
        out[b].d = f32ToF16(d);
        for (int j = 0; j < kQBlock / 2; j++) {
            float a = v[j] * id + 8.5f, c = v[j + 16] * id + 8.5f;
            int qa = (int)std::floor(std::fmin(std::fmax(a, 0.f), 15.f));
            int qc = (int)std::floor(std::fmin(std::fmax(c, 0.f), 15.f));
            out[b].qs[j] = (u8)(qa | (qc << 4));
        }
    }
}

void dequantizeQ40(const BlockQ40 *in, float *out, u64 n) {
    const u64 nb = n / kQBlock;
    for (u64 b = 0; b < nb; b++) {
        const float d = f16ToF32(in[b].d);
        for (int j = 0; j < kQBlock / 2; j++) {
            out[b * kQBlock + j] = (float)((in[b].qs[j] & 0x0F) - 8) * d;
            out[b * kQBlock + j + 16] = (float)((in[b].qs[j] >> 4) - 8) * d;
        }
    }
}

}  // namespace dl
