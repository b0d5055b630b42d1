// Decode attention on MFMA for bf16 KV caches (separate-kernel decode rows: serving batches, long
// contexts; reference: the per-row attention of src/nn/nn-cpu-ops.cpp:749-784 / :1135-1161).
//
// The VALU kernel (attnTask) spends 16 lanes and a cross-lane reduction per key and a serial
// online-softmax chain per 16-lane group: at long context it is latency-bound (21.9 us at pos 8000,
// profiles/r1_attention.md) while the KV stream alone takes ~6 us. Here one workgroup owns one
// (row, KV head, key chunk) and its 4 waves split the chunk's 32-key tiles (wave w: tiles w, w+4,
// ...). Per tile a wave
//   * copies K and V (32 keys x HS bf16 each) HBM -> its own LDS buffers with global_load_lds
//     (double-buffered, the next tile in flight; no barrier: only the issuing wave reads them),
//   * S^T = K . Q^T on v_mfma_f32_16x16x32_bf16 (A = 16 keys x 32 dims read row-wise from LDS,
//     B = the row's kvMul query heads as the MFMA columns, pre-scaled, in registers),
//   * one online-softmax step per column over the 32 keys (max / sum over the lane's 8 scores
//     and 2 cross-lane shuffles, instead of per key),
//   * O^T += V^T . P^T (B = P^T straight from the S^T accumulators; A = V^T read from the
//     row-major V tile with ds_read_b64_tr_b16, the hardware transpose read: no transposed cache).
// The LDS tile image is the 256-B-row layout (b) of cdna_hip_programming.md T10 (chunk ch of row r
// at 16 * (ch ^ (((r & 3) << 2) | ((r >> 2) & 3)))), written by the DMA as a permutation of each
// 1-KB wave-instruction image. The 4 waves' (max, sum, O) merge in LDS; chunks of one head group
// combine through attnFinish (fence-free last arriver, decode_dev.h) like the VALU kernel, with
// the same split plan (attnSplit), so both kernels share the engine's partial buffers.
#include "decode_dev.h"

#include <cstdlib>

namespace dl {
namespace hipk {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef short s16x4 __attribute__((ext_vector_type(4)));

static constexpr int kAmThreads = 256, kAmWaves = 4, kAmTile = 32, kAmHS = 128;
static constexpr int kAmTileBytes = kAmTile * kAmHS * 2;     // one K or V tile: 8 KB
static constexpr int kAmWaveBytes = 2 * 2 * kAmTileBytes;    // double-buffered K + V per wave
static constexpr size_t kAmLds = (size_t)kAmWaves * kAmWaveBytes + 64;

__device__ __forceinline__ int amSwz(int r) { return ((r & 3) << 2) | ((r >> 2) & 3); }
// Key (LDS row within a 32-key tile) of MFMA row m (0..15) of 16-key subtile u. MFMA row m = 4h + q
// lands on lane group h of the S^T output / P^T operand, and the V^T transposed read of group h
// fetches the 4 rows of its keys: with rows 8 apart for the two groups of a 32-lane half (h = 0 / 1
// -> rows 0..3 / 8..11, h = 2 / 3 -> 4..7 / 12..15) that read is bank-conflict free on the image
// (cdna_hip_programming.md T10), instead of 2-way for adjacent row blocks.
__host__ __device__ __forceinline__ int amKey(int u, int m) { return 16 * u + 8 * ((m >> 2) & 1) + 4 * (m >> 3) + (m & 3); }

template <int KM>
__global__ __launch_bounds__(kAmThreads) void attnDecodeMfmaKernel(AttnArgs a) {
    constexpr int HS = kAmHS, DS = HS / 32, NT = HS / 16;
    extern __shared__ __attribute__((aligned(16))) char smem[];
    const int g = blockIdx.x, c = blockIdx.y, b = blockIdx.z;
    const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63, col = lane & 15, h = lane >> 4;
    const int pos = a.pos[b], sl = a.slot[b], len = pos + 1;
    int nSplit, ch;
    attnSplit(len, a.splitGrid, nSplit, ch, a.chunkMin, a.shortLen);
    if (c >= nSplit) return;
    const int t0 = c * ch, t1 = min(t0 + ch, len);
    const int nTiles = (t1 - t0 + kAmTile - 1) / kAmTile;
    // stamps stay in SGPRs until the end (a store would join the vmcnt accounting of the DMA)
    unsigned long long tr[6] = {a.trace ? wall_clock64() : 0ull, 0ull, 0ull, 0ull, 0ull, 0ull};

    // this lane's column: query head g * KM + col (columns >= KM are zero and discarded); the q
    // loads are issued first, then the K / V DMA of the first two tiles, and only then are the q
    // values waited for (one memory round trip at entry instead of two)
    const float scale = 1.0f / sqrtf((float)HS);
    float4 qx[DS][2];
#pragma unroll
    for (int s = 0; s < DS; s++) {
        const float *qp = a.q + (size_t)b * a.ldq + (size_t)(g * KM + min(col, KM - 1)) * HS + 32 * s + 8 * h;
        qx[s][0] = ld4(qp);
        qx[s][1] = ld4(qp + 4);
    }

    char *wbuf = smem + wave * kAmWaveBytes;  // [2 buffers][K tile | V tile]
    const uint16_t *kc = reinterpret_cast<const uint16_t *>(a.kcache);
    const uint16_t *vc = reinterpret_cast<const uint16_t *>(a.vcache);
    const int nKv = a.kv0 / HS;
    // Paged cache: the chunk's page ids are loaded once, one per lane, before any DMA, and each
    // key's row comes from a lane shuffle. (A table load per key row made the compiler wait for
    // vmcnt(0) - every DMA already in flight - before each of the 16 wave-instructions of a tile.)
    const KvMap &km = a.kvMap;
    const int pg0 = km.table ? t0 >> km.pageShift : 0;
    // a chunk spans at most 64 pages (launchAttentionMfma checks): no per-key table load remains in
    // the issue loop, whose join would put a vmcnt(0) drain before every DMA pair
    const bool pgLanes = km.table != nullptr;
    int pgReg = 0;
    if (pgLanes) {
        // retired here, before any DMA: the waitcnt pass cannot track this load into the issue
        // loop's branches and would otherwise wait for vmcnt(0) at every shuffle
        int v = km.table[sl * km.pagesPerSlot + pg0 + min(lane, ((t1 - 1) >> km.pageShift) - pg0)];
        asm volatile("s_waitcnt vmcnt(0)" : "+v"(v));
        pgReg = v;
    }
    auto offOf = [&](int key) -> size_t {  // element offset of head g's vector at this key
        if (!pgLanes) return kvOffAt(km, a.seqLen, nKv, HS, (size_t)sl, key, g);
        const int pg = __shfl(pgReg, (key >> km.pageShift) - pg0);
        return kvOffAt(km, a.seqLen, nKv, HS, (size_t)pg, key, g);
    };
    // DMA of tile i (keys t0 + 32 i ...) into buffer bf: 8 + 8 wave-instructions of 4 rows x 256 B
    // (non-temporal: a decode row reads each layer's K / V once)
    auto issue = [&](int i, int bf) {
        char *kb = wbuf + bf * 2 * kAmTileBytes, *vb = kb + kAmTileBytes;
#pragma unroll
        for (int j = 0; j < kAmTile / 4; j++) {
            const int r = 4 * j + (lane >> 4), p = lane & 15;
            const int key = min(t0 + kAmTile * i + r, t1 - 1);  // past the chunk: masked below
            const size_t off = offOf(key) + (size_t)(p ^ amSwz(r)) * 8;
            __builtin_amdgcn_global_load_lds(const_cast<uint16_t *>(kc + off),
                                             reinterpret_cast<__attribute__((address_space(3))) void *>(
                                                 reinterpret_cast<uintptr_t>(kb + j * 1024)), 16, 0, 2);
            __builtin_amdgcn_global_load_lds(const_cast<uint16_t *>(vc + off),
                                             reinterpret_cast<__attribute__((address_space(3))) void *>(
                                                 reinterpret_cast<uintptr_t>(vb + j * 1024)), 16, 0, 2);
        }
    };

    f32x4 o[NT];
#pragma unroll
    for (int n = 0; n < NT; n++) o[n] = f32x4{0.f, 0.f, 0.f, 0.f};
    float m = -INFINITY, lsum = 0.f;
    // transposed-read address pieces of this lane (lane 4q + p of its 16-lane group h)
    const int tq = col >> 2, tp = col & 3;
    // Rounds of 4 tiles (wave w: tile 4 r + w), the same count on every wave: LDS-DMA data is ordered
    // for a ds_read only by the issuing wave's counted vmcnt FOLLOWED BY a workgroup barrier
    // (cdna_hip_programming.md, "Read a staged buffer one phase after the wait that retires it")
    const int nRounds = (nTiles + kAmWaves - 1) / kAmWaves;
    // both prologue tiles are issued unconditionally (a tile past the chunk re-reads its last key:
    // harmless, never consumed), so the vmcnt the q values wait for is the same on every wave
    issue(wave, 0);
    issue(wave + kAmWaves, 1);
    const float qs = col < KM ? scale : 0.f;
    bf16x8 qf[DS];
#pragma unroll
    for (int s = 0; s < DS; s++) {
        const float4 x0 = qx[s][0], x1 = qx[s][1];
        const float v[8] = {x0.x * qs, x0.y * qs, x0.z * qs, x0.w * qs, x1.x * qs, x1.y * qs, x1.z * qs, x1.w * qs};
#pragma unroll
        for (int j = 0; j < 8; j++) qf[s][j] = (__bf16)v[j];
    }
    if (a.trace) tr[1] = wall_clock64();
    for (int k = 0; k < nRounds; k++) {
        const int i = k * kAmWaves + wave;
        if (i + kAmWaves < nTiles)
            asm volatile("s_waitcnt vmcnt(16)" ::: "memory");  // tile i landed, tile i + 4 in flight
        else
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();
        if (a.trace && k == 0) tr[2] = wall_clock64();
        if (i >= nTiles) continue;  // wave-uniform; the barrier above is reached by every wave
        const char *kb = wbuf + (k & 1) * 2 * kAmTileBytes, *vb = kb + kAmTileBytes;
        const int tb = t0 + kAmTile * i;
        f32x4 st[2];
#pragma unroll
        for (int u = 0; u < 2; u++) {
            st[u] = f32x4{0.f, 0.f, 0.f, 0.f};
            const int r = amKey(u, col);
#pragma unroll
            for (int s = 0; s < DS; s++) {
                const bf16x8 kf = *reinterpret_cast<const bf16x8 *>(kb + r * 256 + 16 * ((4 * s + h) ^ amSwz(r)));
                st[u] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(kf, qf[s], st[u], 0, 0, 0);
            }
        }
#ifdef DL_AM_DEBUG
        if (g == 0 && c == 0 && b == 0 && i == 0)
            for (int u = 0; u < 2; u++)
                for (int e = 0; e < 4; e++) a.partO[amKey(u, 4 * h + e) * 16 + col] = st[u][e];
#endif
        float mx = -INFINITY;
#pragma unroll
        for (int u = 0; u < 2; u++)
#pragma unroll
            for (int e = 0; e < 4; e++) {
                if (tb + amKey(u, 4 * h + e) >= t1) st[u][e] = -INFINITY;
                mx = fmaxf(mx, st[u][e]);
            }
        mx = fmaxf(mx, __shfl_xor(mx, 16));
        mx = fmaxf(mx, __shfl_xor(mx, 32));
        const float mn = fmaxf(m, mx);
        const float corr = m == -INFINITY ? 0.f : __expf(m - mn);
        bf16x8 pf;
        float ps = 0.f;
#pragma unroll
        for (int u = 0; u < 2; u++)
#pragma unroll
            for (int e = 0; e < 4; e++) {
                const float p = st[u][e] == -INFINITY ? 0.f : __expf(st[u][e] - mn);
                ps += p;
                pf[4 * u + e] = (__bf16)p;
            }
        lsum = lsum * corr + ps;
        m = mn;
#pragma unroll
        for (int n = 0; n < NT; n++) {
            // A = V^T (16 dims x 32 keys): elements 0-3 keys 4h..4h+3, 4-7 keys 16+4h.., the
            // order of P^T's registers; lane 4q+p of group h addresses row r0 + q, dims 16n+4p..
            s16x4 vv[2];
#pragma unroll
            for (int u = 0; u < 2; u++) {
                const int r = amKey(u, 4 * h + tq);
                const char *ad = vb + r * 256 + 16 * ((2 * n + (tp >> 1)) ^ amSwz(r)) + 8 * (tp & 1);
                vv[u] = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
                    reinterpret_cast<__attribute__((address_space(3))) s16x4 *>(reinterpret_cast<uintptr_t>(ad)));
            }
            // whole-register bit casts (per-element short -> __bf16 inserts were miscompiled by
            // ROCm 7.2's hipcc into a broadcast of element 0: scripts/probe_attn.hip)
            const u32x2 lo = __builtin_bit_cast(u32x2, vv[0]), hi = __builtin_bit_cast(u32x2, vv[1]);
            const bf16x8 vf = __builtin_bit_cast(bf16x8, u32x4{lo.x, lo.y, hi.x, hi.y});
#ifdef DL_AM_DEBUG
            if (g == 0 && c == 0 && b == 0 && i == 0 && n == 0)
                for (int e = 0; e < 8; e++) {
                    a.partO[8192 + lane * 8 + e] = (float)vf[e];
                    a.partO[12288 + lane * 8 + e] = (float)pf[e];
                }
            if (g == 0 && c == 0 && b == 0 && i == 0 && n == 0)  // raw V tile rows 0..3, LDS order
                for (int e = lane; e < 4 * 128; e += 64)
                    a.partO[16384 + e] = __uint_as_float((uint32_t)reinterpret_cast<const uint16_t *>(vb)[e] << 16);
#endif
            o[n] *= corr;
            o[n] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(vf, pf, o[n], 0, 0, 0);
        }
        // this buffer's reads retire before the DMA of tile i + 8 overwrites it
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        if (i + 2 * kAmWaves < nTiles) issue(i + 2 * kAmWaves, k & 1);
    }
    lsum += __shfl_xor(lsum, 16);
    lsum += __shfl_xor(lsum, 32);
    if (a.trace) tr[3] = wall_clock64();
#ifdef DL_AM_DEBUG
    if (g == 0 && c == 0 && b == 0 && wave == 0) {
        for (int n = 0; n < NT; n++)
            for (int e = 0; e < 4; e++) a.partO[1024 + (16 * n + 4 * h + e) * 16 + col] = o[n][e];
        a.partO[4096 + lane * 2] = m;
        a.partO[4096 + lane * 2 + 1] = lsum;
    }
#endif

    // merge the waves (LDS: the tile buffers are free once every wave is past its loop)
    __syncthreads();
    float *oW = reinterpret_cast<float *>(smem);  // [4 waves][KM][HS]
    float *mW = oW + kAmWaves * KM * HS;          // [4][KM]
    float *lW = mW + kAmWaves * KM;               // [4][KM]
    float *redL = lW + kAmWaves * KM;             // [KM][HS]
    float *mlL = redL + KM * HS;                  // [KM][2]
    int *flagL = reinterpret_cast<int *>(mlL + 2 * KM);
    float *scratch = reinterpret_cast<float *>(flagL + 4);  // attnFinish: 2 * KM * splitGrid
    if (col < KM) {
        if (h == 0) {
            mW[wave * KM + col] = wave < nTiles ? m : -INFINITY;
            lW[wave * KM + col] = wave < nTiles ? lsum : 0.f;
        }
#pragma unroll
        for (int n = 0; n < NT; n++)
#pragma unroll
            for (int e = 0; e < 4; e++) oW[(wave * KM + col) * HS + 16 * n + 4 * h + e] = o[n][e];
    }
    __syncthreads();
    for (int i = tid; i < KM * HS; i += kAmThreads) {
        const int hh = i / HS;
        float M = -INFINITY;
#pragma unroll
        for (int w = 0; w < kAmWaves; w++) M = fmaxf(M, mW[w * KM + hh]);
        float acc = 0.f, Ls = 0.f;
#pragma unroll
        for (int w = 0; w < kAmWaves; w++) {
            const float e = mW[w * KM + hh] == -INFINITY ? 0.f : __expf(mW[w * KM + hh] - M);
            acc += e * oW[(w * KM + hh) * HS + (i % HS)];
            Ls += e * lW[w * KM + hh];
        }
        redL[i] = acc;
        if (i % HS == 0) {
            mlL[hh * 2] = M;
            mlL[hh * 2 + 1] = Ls;
        }
    }
    __syncthreads();
    if (a.trace) tr[4] = wall_clock64();
    const bool fin = attnFinish<KM, HS, kAmThreads>(a, b, g, c, nSplit, redL, mlL, flagL, scratch);
    if (a.trace && tid == 0) {
        tr[5] = wall_clock64();
        unsigned long long *t = a.trace + 8 * (((size_t)b * gridDim.y + c) * gridDim.x + g);
        for (int i = 0; i < 6; i++) t[i] = tr[i];
        t[6] = fin ? 1ull : 0ull;
    }
}

// ------------------------------------------------------------------------------------------------
// Prefill attention with the same staging (the batched path's rows; reference: the per-row causal
// attention of nn-cpu-ops.cpp:1135-1161 for every prompt row). A workgroup owns one KV head and a
// block of 4 x 16 / kvMul rows of one slot: wave w's 16 MFMA columns are (row, query head) pairs, so
// every S^T / O^T MFMA is fully used, and all 4 waves read every K / V tile of the chunk from LDS.
// The chunk's tiles are DMA'd in rounds of 4 (wave w copies tile 4 r + w), two rounds in flight
// (128 KB of LDS); the previous kernel (kernels.hip attnPrefillKernel) staged one 32-key tile ahead
// through registers with a transposing LDS scatter for V. Causal mask per column (key <= the row's
// position); chunks of long contexts combine through the last arriver as before.
// ------------------------------------------------------------------------------------------------
static constexpr int kApRound = 4;  // tiles per round (one per wave)
static constexpr size_t kApLds = 2 * kApRound * 2 * kAmTileBytes + 64;

static constexpr int kApMaxTiles = 256;  // per-chunk page list of the prefill kernel (paged caches)

template <int KM>
__global__ __launch_bounds__(kAmThreads) void attnPrefillDmaKernel(AttnArgs a, int nRows) {
    constexpr int HS = kAmHS, DS = HS / 32, NT = HS / 16, RPW = 16 / KM, RPB = kAmWaves * RPW;
    extern __shared__ __attribute__((aligned(16))) char smem[];
    const int nKv = a.nHeads0 / KM;
    const int g = blockIdx.x % nKv, rb = blockIdx.x / nKv, c = blockIdx.y;
    const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63, col = lane & 15, h = lane >> 4;
    const int b0 = rb * RPB;
    const int maxLen = rowsMaxLen(a.pos, b0, RPB, nRows);
    int nSplit = (maxLen + 255) / 256;
    nSplit = max(1, min(min(nSplit, a.splitGrid), HS / 2));  // combine weights: 64 columns x nSplit in LDS
    const int ch = ((maxLen + nSplit - 1) / nSplit + kAmTile - 1) / kAmTile * kAmTile;
    if (c >= nSplit) return;
    const int k0 = c * ch, k1 = min(k0 + ch, maxLen);
    const int sl = a.slot[b0];  // every row of the block (host-checked)
    const int row = b0 + wave * RPW + col / KM, head = g * KM + col % KM;
    const bool rowOk = row < nRows;
    const int myLen = rowOk ? a.pos[row] + 1 : 0;
    const float scale = 1.0f / sqrtf((float)HS);
    bf16x8 qf[DS];
#pragma unroll
    for (int s = 0; s < DS; s++) {
        float v[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
        if (rowOk) {
            const float *qp = a.q + (size_t)row * a.ldq + (size_t)head * HS + 32 * s + 8 * h;
            const float4 x0 = ld4(qp), x1 = ld4(qp + 4);
            v[0] = x0.x * scale; v[1] = x0.y * scale; v[2] = x0.z * scale; v[3] = x0.w * scale;
            v[4] = x1.x * scale; v[5] = x1.y * scale; v[6] = x1.z * scale; v[7] = x1.w * scale;
        }
#pragma unroll
        for (int j = 0; j < 8; j++) qf[s][j] = (__bf16)v[j];
    }
    const uint16_t *kc = reinterpret_cast<const uint16_t *>(a.kcache);
    const uint16_t *vc = reinterpret_cast<const uint16_t *>(a.vcache);
    const int nTiles = (k1 - k0 + kAmTile - 1) / kAmTile, nRounds = (nTiles + kApRound - 1) / kApRound;
    // paged cache: the chunk's per-tile pages in LDS before any DMA (a tile never crosses a page; a
    // table load per key row put a vmcnt(0) drain before every DMA pair, contiguous caches included)
    __shared__ int pageL[kApMaxTiles];
    if (a.kvMap.table)
        for (int i = tid; i < nTiles; i += kAmThreads) pageL[i] = (int)kvPageOf(a.kvMap, sl, k0 + i * kAmTile);
    __syncthreads();
    auto tileBuf = [&](int bf, int tt) { return smem + (size_t)(bf * kApRound + tt) * 2 * kAmTileBytes; };
    // wave w copies tile kApRound * r + w of round r into buffer bf (16 wave-instructions, or none)
    auto issue = [&](int r, int bf) {
        const int t = kApRound * r + wave;
        if (t >= nTiles) return;
        char *kb = tileBuf(bf, wave), *vb = kb + kAmTileBytes;
#pragma unroll
        for (int j = 0; j < kAmTile / 4; j++) {
            const int rr = 4 * j + (lane >> 4), p = lane & 15;
            const int key = min(k0 + kAmTile * t + rr, k1 - 1);  // past the chunk: masked below
            const size_t blk = a.kvMap.table ? (size_t)pageL[t] : (size_t)sl;
            const size_t off = kvOffAt(a.kvMap, a.seqLen, nKv, HS, blk, key, g) + (size_t)(p ^ amSwz(rr)) * 8;
            __builtin_amdgcn_global_load_lds(const_cast<uint16_t *>(kc + off),
                                             reinterpret_cast<__attribute__((address_space(3))) void *>(
                                                 reinterpret_cast<uintptr_t>(kb + j * 1024)), 16, 0, 0);
            __builtin_amdgcn_global_load_lds(const_cast<uint16_t *>(vc + off),
                                             reinterpret_cast<__attribute__((address_space(3))) void *>(
                                                 reinterpret_cast<uintptr_t>(vb + j * 1024)), 16, 0, 0);
        }
    };
    f32x4 o[NT];
#pragma unroll
    for (int n = 0; n < NT; n++) o[n] = f32x4{0.f, 0.f, 0.f, 0.f};
    float m = -INFINITY, lsum = 0.f;
    const int tq = col >> 2, tp = col & 3;
    issue(0, 0);
    if (nRounds > 1) issue(1, 1);
    for (int r = 0; r < nRounds; r++) {
        // this wave's copy of round r landed (round r + 1's may stay in flight), then every wave's
        if (r + 1 < nRounds && kApRound * (r + 1) + wave < nTiles)
            asm volatile("s_waitcnt vmcnt(16)" ::: "memory");
        else
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();
        for (int tt = 0; tt < kApRound; tt++) {
            const int t = kApRound * r + tt;
            if (t >= nTiles) break;  // uniform over the workgroup
            const char *kb = tileBuf(r & 1, tt), *vb = kb + kAmTileBytes;
            const int tb = k0 + kAmTile * t;
            f32x4 st[2];
#pragma unroll
            for (int u = 0; u < 2; u++) {
                st[u] = f32x4{0.f, 0.f, 0.f, 0.f};
                const int rr = amKey(u, col);
#pragma unroll
                for (int s = 0; s < DS; s++) {
                    const bf16x8 kf = *reinterpret_cast<const bf16x8 *>(kb + rr * 256 + 16 * ((4 * s + h) ^ amSwz(rr)));
                    st[u] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(kf, qf[s], st[u], 0, 0, 0);
                }
            }
            float mx = -INFINITY;
#pragma unroll
            for (int u = 0; u < 2; u++)
#pragma unroll
                for (int e = 0; e < 4; e++) {
                    const int key = tb + amKey(u, 4 * h + e);
                    if (key >= k1 || key >= myLen) st[u][e] = -INFINITY;
                    mx = fmaxf(mx, st[u][e]);
                }
            mx = fmaxf(mx, __shfl_xor(mx, 16));
            mx = fmaxf(mx, __shfl_xor(mx, 32));
            const float mn = fmaxf(m, mx);
            const float corr = m == -INFINITY ? 0.f : __expf(m - mn);
            bf16x8 pf;
            float ps = 0.f;
#pragma unroll
            for (int u = 0; u < 2; u++)
#pragma unroll
                for (int e = 0; e < 4; e++) {
                    const float p = st[u][e] == -INFINITY ? 0.f : __expf(st[u][e] - mn);
                    ps += p;
                    pf[4 * u + e] = (__bf16)p;
                }
            lsum = lsum * corr + ps;
            m = mn;
#pragma unroll
            for (int n = 0; n < NT; n++) {
                s16x4 vv[2];
#pragma unroll
                for (int u = 0; u < 2; u++) {
                    const int rr = amKey(u, 4 * h + tq);
                    const char *ad = vb + rr * 256 + 16 * ((2 * n + (tp >> 1)) ^ amSwz(rr)) + 8 * (tp & 1);
                    vv[u] = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
                        reinterpret_cast<__attribute__((address_space(3))) s16x4 *>(reinterpret_cast<uintptr_t>(ad)));
                }
                const u32x2 lo = __builtin_bit_cast(u32x2, vv[0]), hi = __builtin_bit_cast(u32x2, vv[1]);
                const bf16x8 vf = __builtin_bit_cast(bf16x8, u32x4{lo.x, lo.y, hi.x, hi.y});
                o[n] *= corr;
                o[n] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(vf, pf, o[n], 0, 0, 0);
            }
        }
        // every wave's reads of buffer r & 1 retired before round r + 2 is copied into it
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();
        if (r + 2 < nRounds) issue(r + 2, r & 1);
    }
    lsum += __shfl_xor(lsum, 16);
    lsum += __shfl_xor(lsum, 32);
    // O^T accumulators: lane holds O[column][dim 16 n + 4 h + e]
    auto writeOut = [&](int rw, int hd, int d, const float (&v)[4]) {
        const size_t at = (size_t)rw * a.ldOut + (size_t)hd * HS + d;
        if (a.outH) {
            typedef _Float16 h4 __attribute__((ext_vector_type(4)));
            *reinterpret_cast<h4 *>(a.outH + at) = h4{(_Float16)v[0], (_Float16)v[1], (_Float16)v[2], (_Float16)v[3]};
        } else {
            *reinterpret_cast<float4 *>(a.out + at) = make_float4(v[0], v[1], v[2], v[3]);
        }
    };
    if (nSplit == 1) {
        if (rowOk) {
            const float il = lsum > 0.f ? 1.0f / lsum : 0.f;
#pragma unroll
            for (int n = 0; n < NT; n++) {
                const float v[4] = {o[n][0] * il, o[n][1] * il, o[n][2] * il, o[n][3] * il};
                writeOut(row, head, 16 * n + 4 * h, v);
            }
        }
        return;
    }
    // several chunks: publish (fence-free, gemm_dev.h pattern: write-through stores, drained, then
    // the arrival count), the last arriver combines in chunk order
    const int G = a.splitGrid;
    if (rowOk) {
        const size_t pb = ((size_t)row * a.nHeads0 + head) * G + c;
#pragma unroll
        for (int n = 0; n < NT; n++)
#pragma unroll
            for (int e = 0; e < 4; e++)
                __hip_atomic_store(a.partO + pb * HS + 16 * n + 4 * h + e, o[n][e], __ATOMIC_RELAXED,
                                   __HIP_MEMORY_SCOPE_AGENT);
        if (h == 0) {
            __hip_atomic_store(a.partML + pb * 2, m, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            __hip_atomic_store(a.partML + pb * 2 + 1, lsum, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    int *flagL = reinterpret_cast<int *>(smem + 2 * kApRound * 2 * kAmTileBytes);
    int *cnt = a.counters + (size_t)rb * nKv + g;
    if (tid == 0) flagL[0] = __hip_atomic_fetch_add(cnt, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == nSplit - 1;
    __syncthreads();
    if (!flagL[0]) return;
    if (tid == 0) __hip_atomic_store(cnt, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    auto ld = [](const float *q) { return __hip_atomic_load(q, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT); };
    constexpr int nCol = RPB * KM;  // 64 columns
    float *wts = reinterpret_cast<float *>(smem);  // [nCol][nSplit] (the tiles are free)
    float *tot = wts + nCol * (HS / 2);            // [nCol]
    if (tid < nCol) {
        const int rw = b0 + tid / KM, hd = g * KM + tid % KM;
        float M = -INFINITY, L = 0.f;
        if (rw < nRows) {
            const float *ml = a.partML + ((size_t)rw * a.nHeads0 + hd) * G * 2;
            for (int cc = 0; cc < nSplit; cc++) M = fmaxf(M, ld(ml + 2 * cc));
            for (int cc = 0; cc < nSplit; cc++) {
                const float mc = ld(ml + 2 * cc);
                const float w = (M == -INFINITY || mc == -INFINITY) ? 0.f : __expf(mc - M);
                wts[tid * nSplit + cc] = w;
                L += w * ld(ml + 2 * cc + 1);
            }
        }
        tot[tid] = L;
    }
    __syncthreads();
    for (int i = tid; i < nCol * (HS / 4); i += kAmThreads) {
        const int cl = i / (HS / 4), d = (i % (HS / 4)) * 4;
        const int rw = b0 + cl / KM, hd = g * KM + cl % KM;
        if (rw >= nRows) continue;
        const float *po = a.partO + ((size_t)rw * a.nHeads0 + hd) * G * HS + d;
        float acc[4] = {0.f, 0.f, 0.f, 0.f};
        for (int cc = 0; cc < nSplit; cc++) {
            const float w = wts[cl * nSplit + cc];
            const float *x = po + (size_t)cc * HS;
            acc[0] += w * ld(x); acc[1] += w * ld(x + 1); acc[2] += w * ld(x + 2); acc[3] += w * ld(x + 3);
        }
        const float il = tot[cl] > 0.f ? 1.0f / tot[cl] : 0.f;
        const float v[4] = {acc[0] * il, acc[1] * il, acc[2] * il, acc[3] * il};
        writeOut(rw, hd, d, v);
    }
}

bool attnPrefillDmaSupported(const AttnArgs &a) {
    return a.kvBf16 && a.hs == kAmHS && (a.kvMul == 1 || a.kvMul == 2 || a.kvMul == 4 || a.kvMul == 8 ||
                                                a.kvMul == 16);
}

void launchAttentionPrefillDma(const AttnArgs &a, int nRows, hipStream_t s) {
    const int nKv = a.nHeads0 / a.kvMul, rpb = kAmWaves * (16 / a.kvMul);
    {  // the longest chunk's tiles fit the kernel's LDS page list
        const int minSplits = std::max(1, std::min(a.splitGrid, kAmHS / 2));
        if (a.kvMap.table && ((a.seqLen + minSplits - 1) / minSplits + kAmTile - 1) / kAmTile + 1 > kApMaxTiles)
            throw Error("launchAttentionPrefillDma: paged context too long for the per-chunk page list");
    }
    const dim3 grid(nKv * ((nRows + rpb - 1) / rpb), a.splitGrid);
#define DL_AP_CASE(K)                                                                                 \
    if (a.kvMul == K) {                                                                               \
        allowLds((const void *)attnPrefillDmaKernel<K>, kApLds);                                      \
        hipLaunchKernelGGL((attnPrefillDmaKernel<K>), grid, dim3(kAmThreads), kApLds, s, a, nRows);   \
        return;                                                                                       \
    }
    DL_AP_CASE(1) DL_AP_CASE(2) DL_AP_CASE(4) DL_AP_CASE(8) DL_AP_CASE(16)
#undef DL_AP_CASE
    throw Error("launchAttentionPrefillDma: unsupported kvMul");
}

bool attnMfmaSupported(const AttnArgs &a) {
    return a.kvBf16 && a.hs == kAmHS && (a.kvMul == 1 || a.kvMul == 2 || a.kvMul == 4 || a.kvMul == 8) &&
           a.nHeads0 % a.kvMul == 0;
}

// DL_ATTN_MFMA: 0 = the VALU kernel everywhere, 1 = this kernel for every supported launch,
// default (-1) = this kernel when the cache is long enough for it to matter (seqLen >= 1024).
static int attnMfmaMode() {
    static const int v = [] {
        const char *e = std::getenv("DL_ATTN_MFMA");
        return e ? std::atoi(e) : -1;
    }();
    return v;
}

bool attnUsesMfma(const AttnArgs &a) {
    const int mode = attnMfmaMode();
    if (mode == 0 || !attnMfmaSupported(a)) return false;
    if (mode == 1) return true;
    return a.mfma >= 0 ? a.mfma == 1 : a.seqLen >= 1024;
}


// preloadModules(): one kernel of this translation unit's code object
const void *attnMfmaModuleKernel() { return (const void *)attnDecodeMfmaKernel<4>; }

void launchAttentionMfma(const AttnArgs &a, int B, hipStream_t s) {
    const dim3 grid(a.nHeads0 / a.kvMul, a.splitGrid, B);
    if (2 * a.kvMul * a.splitGrid * 4 + 4096 > (int)kAmLds) throw Error("attention split grid too large");
    if (a.kvMap.table && (a.chunkMax >> a.kvMap.pageShift) + 2 > 64)
        throw Error("launchAttentionMfma: a chunk spans more than 64 pages (one page id per lane)");
#define DL_AM_CASE(K)                                                                             \
    if (a.kvMul == K) {                                                                           \
        allowLds((const void *)attnDecodeMfmaKernel<K>, kAmLds);                                  \
        hipLaunchKernelGGL((attnDecodeMfmaKernel<K>), grid, dim3(kAmThreads), kAmLds, s, a);      \
        return;                                                                                   \
    }
    DL_AM_CASE(1) DL_AM_CASE(2) DL_AM_CASE(4) DL_AM_CASE(8)
#undef DL_AM_CASE
    throw Error("launchAttentionMfma: unsupported kvMul");
}

}  // namespace hipk
}  // namespace dl
