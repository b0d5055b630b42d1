// Standalone check of the MFMA decode attention kernel (attn_mfma.hip) against a host fp32
// reference: one row, 8 KV heads x kvMul 4, head size 128, bf16 cache; prints per-head errors and
// the first outputs of head 0. Build: hipcc --offload-arch=gfx950 -O2 -I csrc probe_attn.hip
#define DL_AM_DEBUG 1
#include "../csrc/hip/attn_mfma.hip"
#include <cmath>
#include <cstring>
#include <cstdio>
#include <vector>
using namespace dl::hipk;
static uint16_t toBf(float f) { uint32_t u; std::memcpy(&u, &f, 4); return (uint16_t)((u + 0x7FFF + ((u >> 16) & 1)) >> 16); }
static float fromBf(uint16_t b) { uint32_t u = (uint32_t)b << 16; float f; std::memcpy(&f, &u, 4); return f; }
int main(int argc, char **argv) {
    const int pos = argc > 1 ? atoi(argv[1]) : 150, seq = 256, nH = 32, km = 4, hs = 128, kv0 = nH / km * hs;
    std::vector<float> q(nH * hs), k((size_t)seq * kv0), v((size_t)seq * kv0);
    unsigned s = 1;
    auto rnd = [&]() { s = s * 1664525u + 1013904223u; return ((s >> 8) & 0xFFFF) / 32768.0f - 1.0f; };
    for (auto &x : q) x = rnd();
    std::vector<uint16_t> kb(k.size()), vb(v.size());
    for (size_t i = 0; i < k.size(); i++) { kb[i] = toBf(rnd()); k[i] = fromBf(kb[i]); }
    for (size_t i = 0; i < v.size(); i++) { vb[i] = toBf(rnd()); v[i] = fromBf(vb[i]); }
    float *dq, *dout, *pO, *pML; uint16_t *dk, *dv; int *dpos, *dslot, *cnt;
    (void)hipMalloc(&dq, q.size() * 4); (void)hipMalloc(&dout, q.size() * 4);
    (void)hipMalloc(&dk, kb.size() * 2); (void)hipMalloc(&dv, vb.size() * 2);
    (void)hipMalloc(&pO, nH * 8 * hs * 4); (void)hipMalloc(&pML, nH * 8 * 2 * 4);
    (void)hipMalloc(&dpos, 4); (void)hipMalloc(&dslot, 4); (void)hipMalloc(&cnt, 4 * nH);
    int zero = 0;
    (void)hipMemcpy(dq, q.data(), q.size() * 4, hipMemcpyHostToDevice);
    (void)hipMemcpy(dk, kb.data(), kb.size() * 2, hipMemcpyHostToDevice);
    (void)hipMemcpy(dv, vb.data(), vb.size() * 2, hipMemcpyHostToDevice);
    (void)hipMemcpy(dpos, &pos, 4, hipMemcpyHostToDevice);
    (void)hipMemcpy(dslot, &zero, 4, hipMemcpyHostToDevice);
    (void)hipMemset(cnt, 0, 4 * nH);
    (void)hipMemset(dout, 0, q.size() * 4);
    AttnArgs a;
    a.q = dq; a.ldq = nH * hs; a.kcache = dk; a.vcache = dv; a.pos = dpos; a.slot = dslot;
    a.nHeads0 = nH; a.kvMul = km; a.hs = hs; a.kv0 = kv0; a.seqLen = seq; a.splitGrid = 1;
    a.partO = pO; a.partML = pML; a.out = dout; a.ldOut = nH * hs; a.kvBf16 = 1; a.counters = cnt;
    launchAttentionMfma(a, 1, 0);
    printf("launch: %s\n", hipGetErrorString(hipDeviceSynchronize()));
    std::vector<float> out(q.size()), dbg(nH * 8 * hs);
    (void)hipMemcpy(out.data(), dout, out.size() * 4, hipMemcpyDeviceToHost);
    (void)hipMemcpy(dbg.data(), pO, dbg.size() * 4, hipMemcpyDeviceToHost);
    // wave 0's first tile scores (keys 0..31 x columns 0..3 = heads 0..3 of KV head 0)
    for (int t = 0; t < 6; t++) {
        printf("key %d:", t);
        for (int cc = 0; cc < 4; cc++) {
            double d = 0;
            for (int i = 0; i < hs; i++) d += (double)q[cc * hs + i] * k[(size_t)t * kv0 + i];
            printf("  [%d] ref %.4f got %.4f", cc, d / std::sqrt((double)hs), dbg[t * 16 + cc]);
        }
        printf("\n");
    }
    // V^T fragment of lane (col, h), element j = V[key pi(h, j)][dim col] for n = 0
    int bad = 0;
    for (int l = 0; l < 64; l++)
        for (int j = 0; j < 8; j++) {
            const int cc = l & 15, hh = l >> 4, key = amKey(j < 4 ? 0 : 1, 4 * hh + (j & 3));
            const float want = v[(size_t)key * kv0 + cc], got = dbg[8192 + l * 8 + j];
            if (want != got && bad++ < 6) printf("vf lane %d el %d: want V[%d][%d]=%.4f got %.4f\n", l, j, key, cc, want, got);
        }
    printf("vf mismatches: %d\n", bad);
    for (int r = 0; r < 2; r++) {  // raw LDS rows (swizzled chunks): chunk position 0..3 first element
        printf("V LDS row %d:", r);
        for (int p = 0; p < 16; p++) printf(" %.3f", dbg[16384 + r * 128 + p * 8]);
        printf("\n   want chunk0..: ");
        for (int p = 0; p < 16; p++) printf(" %.3f", v[(size_t)r * kv0 + p * 8]);
        printf("\n");
    }
    printf("wave0 m/l col0: %.4f %.4f  col1: %.4f %.4f\n", dbg[4096], dbg[4097], dbg[4098], dbg[4099]);
    // unnormalised O of wave 0 (all its keys = the whole context when pos < 32) vs exp(s - m) V
    if (pos < 32) {
        for (int cc = 0; cc < 2; cc++) {
            std::vector<double> sc(pos + 1);
            for (int t = 0; t <= pos; t++) {
                double d = 0;
                for (int i = 0; i < hs; i++) d += (double)q[cc * hs + i] * k[(size_t)t * kv0 + i];
                sc[t] = std::exp(d / std::sqrt((double)hs) - dbg[4096 + 2 * cc]);
            }
            for (int dd = 0; dd < 4; dd++) {
                double o = 0;
                for (int t = 0; t <= pos; t++) o += sc[t] * v[(size_t)t * kv0 + dd];
                printf("O col %d dim %d: ref %.4f got %.4f\n", cc, dd, o, dbg[1024 + dd * 16 + cc]);
            }
        }
    }
    for (int hd = 0; hd < nH; hd++) {
        const int g = hd / km;
        std::vector<double> sc(pos + 1);
        double mx = -1e30;
        for (int t = 0; t <= pos; t++) {
            double d = 0;
            for (int i = 0; i < hs; i++) d += (double)q[hd * hs + i] * k[(size_t)t * kv0 + g * hs + i];
            sc[t] = d / std::sqrt((double)hs);
            mx = std::max(mx, sc[t]);
        }
        double l = 0;
        for (int t = 0; t <= pos; t++) l += (sc[t] = std::exp(sc[t] - mx));
        double err = 0, nrm = 0;
        for (int i = 0; i < hs; i++) {
            double o = 0;
            for (int t = 0; t <= pos; t++) o += sc[t] * v[(size_t)t * kv0 + g * hs + i];
            o /= l;
            err = std::max(err, std::fabs(o - out[hd * hs + i]));
            nrm = std::max(nrm, std::fabs(o));
            if (hd == 0 && i < 6) printf("  head0 dim %d: ref %.5f got %.5f\n", i, o, out[i]);
        }
        if (hd < 8 || err / nrm > 0.02) printf("head %2d: max err %.4f (max |ref| %.4f)\n", hd, err, nrm);
    }
    return 0;
}
