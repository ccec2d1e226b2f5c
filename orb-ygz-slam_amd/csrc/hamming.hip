// hamming.hip — ORBmatcher Hamming search on gfx950.
//
// DescriptorDistance (ORBmatcher.cc:1507-1523) = popcount(a XOR b) over 256 bits.
// Dense best/second-best: the inner candidate loops of SearchByProjection /
// SearchForInitialization / SearchByBoW (ORBmatcher.cc:43-126,375-478,1218-1350)
// keep `dist < bestDist` (first index wins on ties) and the second best.
// The dense search runs on the matrix cores (int8 MFMA, below); the
// candidate-list (CSR) distances are plain XOR + popcount per lane.
#include "common.hpp"

namespace ygzfe {

// ---------------------------------------------------------------------------
// Dense best / second best on the matrix cores.  For 256-bit descriptors
//   ham(q, t) = popc(t) - 2 popc(t & q) + popc(q) = sum_k t_k (1 - 2 q_k) + popc(q),
// so with the train bits as 0/1 bytes (A) and the query bits as +1/-1 bytes
// (B), one v_mfma_i32_32x32x32_i8 chain over K = 256 gives D[t][q] =
// ham(q, t) - popc(q) for a 32 x 32 tile, exactly (integer arithmetic).
// Lane l of a wave owns query column l & 31; its 16 accumulator registers are
// train rows (r & 3) + 8 (r >> 2) + 4 (l >> 5) of the tile.  The K order
// inside an operand is free as long as A and B agree: k-step s, lane half h
// carries descriptor bits [32 s + 16 h, 32 s + 16 h + 16).
//
// A workgroup serves kHamWaves x kHamGroups x 32 queries and streams the train set in
// 32-row tiles; each tile is expanded to bytes once into LDS (double buffered,
// by the first 256 threads) and read by all waves.  Per lane the running best /
// second best are keys
//   key = ((D + 256) << 22) | train_index
// so the smallest key is the smallest distance with the earliest index (the
// sequential loop's `dist < bestDist`), and second = min over the other keys.
// With k1 <= k2 that is  k2 = med3(k1, key, k2); k1 = min(k1, key)  (2 VALU,
// no branches), and the key itself is one v_lshl_add_u32 of the accumulator
// and a wave-uniform (SGPR) index base: inside the loop the index omits the
// lane half's row offset 4h, which is added once before the two halves merge
// (a constant per lane, so it keeps each lane's order).
// Each wave carries kHamGroups query groups of 32 (its B operands in registers), so
// every A operand read from LDS feeds kHamGroups MFMAs: with one group per wave the
// LDS reads of the train tiles (1 KB per wave per MFMA) matched the matrix cores'
// time per CU.  Two groups x 4 waves (121 VGPRs, 4 waves / SIMD): 1,023 pairs of 936
// rows 0.258 -> 0.245 ms, C5 stage 2.86 -> 2.69 ms (profiles/r05/hamming_groups/);
// 2 x 8 and 4 x 4 measured slower.  The kernel stays ~2.5x its MFMA floor: ~10 VALU
// per MFMA (keys + tile expansion) and 42 % of wave cycles waiting on LDS / loads.
//
// FP4 form (YGZ_HAM_FP4, the default): the same identity on the block-scaled
// v_mfma_scale_f32_32x32x64_f8f6f4 with both operands e2m1 (train bit -> 1.0 or 0.0,
// nibble 0x2 / 0x0; query bit -> -1.0 or +1.0, nibble 0xA / 0x2; unit E8M0 scales):
// K = 64 per instruction at the i8 instruction's cycles, so half the MFMAs, and half
// the LDS bytes per train row.  Every product is 0 or +-1 and every partial sum an
// integer below 2^24, so the f32 accumulation is exact; the accumulators start at
// 2^23 + 256, so their bit patterns are 0x4B000000 + (D + 256) and the key is
// (bits << 22) + index exactly as in the i8 form (the exponent bits shift out).
// Measured (tools/mb_hamming.py, 1,023 pairs of the bench's 936-row frames; C5 stage per
// step; profiles/r06/hamming_fp4*): i8 0.228 ms (2.56 ms), FP4 with per-element keys
// 0.197 ms (2.13 ms), FP4 with the accumulator keys below 0.162 ms (1.85 ms), bit-exact.
// Four query groups per wave or 8-wave workgroups measured the same or slower.
#ifndef YGZ_HAM_FP4
#define YGZ_HAM_FP4 1
#endif
#ifndef YGZ_HAM_WAVES
#define YGZ_HAM_WAVES 4
#endif
#ifndef YGZ_HAM_GROUPS
#define YGZ_HAM_GROUPS 2
#endif
constexpr int kHamWaves = YGZ_HAM_WAVES;     // query waves per workgroup
constexpr int kHamGroups = YGZ_HAM_GROUPS;   // 32-query groups per wave
constexpr int kHamQPB = 32 * kHamGroups * kHamWaves;  // queries per workgroup
static_assert(kHamWaves >= 4, "the 256 staging threads of a train tile");
// expanded train row (bytes, or nibbles in the FP4 form) + pad (conflict-free b128 reads)
constexpr int kHamRowBytes = (YGZ_HAM_FP4 ? 128 : 256) + 16;
constexpr int kHamTileBytes = 32 * kHamRowBytes;
constexpr uint32_t kHamNone = 0xFFFFFFFFu;
constexpr int kHamMaxTrain = 1 << 22;

typedef int ham_v4i __attribute__((ext_vector_type(4)));
typedef int ham_v16i __attribute__((ext_vector_type(16)));

// 4 bits -> 4 bytes of 0 / 1 (bit b -> byte b; the shifted copies of the
// nibble never overlap, so the product has no carries)
__device__ __forceinline__ uint32_t nib_bytes(uint32_t bits16, int m) {
    return (__umul24((bits16 >> (4 * m)) & 0xFu, 0x00204081u)) & 0x01010101u;
}

// (a << 22) + (u + c), u + c wave-uniform: one v_lshl_add_u32 with an SGPR
// operand (the SALU add is opaque, so the constant is not re-associated into a
// second VALU add; the shift-add stays plain C, so the MFMA -> VALU read
// hazard is still the compiler's to pad)
__device__ __forceinline__ uint32_t ham_key(int a, uint32_t u, uint32_t c) {
    uint32_t b;
    asm("s_add_u32 %0, %1, %2" : "=s"(b) : "s"(u), "s"(c) : "scc");
    return ((uint32_t)a << 22) + b;
}

__device__ __forceinline__ uint32_t ham_med3(uint32_t a, uint32_t b, uint32_t c) {
    uint32_t r;
    asm("v_med3_u32 %0, %1, %2, %3" : "=v"(r) : "v"(a), "v"(b), "v"(c));
    return r;
}

// 8 bits -> bit 0 of 8 nibbles (bit b -> nibble b)
__device__ __forceinline__ uint32_t spread8(uint32_t x) {
    x &= 0xFFu;
    x = (x | (x << 12)) & 0x000F000Fu;
    x = (x | (x << 6)) & 0x03030303u;
    x = (x | (x << 3)) & 0x11111111u;
    return x;
}
typedef int ham_v8i __attribute__((ext_vector_type(8)));
typedef float ham_v16f __attribute__((ext_vector_type(16)));
constexpr float kHamAccInit = 8388864.0f;  // 2^23 + 256

#if YGZ_HAM_FP4
__device__ __forceinline__ void ham_expand_store(uint8_t *s_tile, int row, int s, uint32_t w) {
    // dword s of train row `row` (bits 32 s .. 32 s + 31) -> 32 e2m1 nibbles 1.0 / 0.0: the
    // A operand of k-step s >> 1 for lane half s & 1 (16 bytes at s * 16 of the row)
    ham_v4i v;
#pragma unroll
    for (int m = 0; m < 4; m++) v[m] = (int)(spread8(w >> (8 * m)) << 1);
    *(ham_v4i *)(s_tile + row * kHamRowBytes + s * 16) = v;
}
#else
__device__ __forceinline__ void ham_expand_store(uint8_t *s_tile, int row, int s, uint32_t w) {
    // dword s of train row `row` -> A operands of k-step s for lane halves 0 and 1
    ham_v4i lo, hi;
#pragma unroll
    for (int m = 0; m < 4; m++) {
        lo[m] = (int)nib_bytes(w & 0xFFFFu, m);
        hi[m] = (int)nib_bytes(w >> 16, m);
    }
    ham_v4i *d = (ham_v4i *)(s_tile + row * kHamRowBytes + s * 32);
    d[0] = lo;
    d[1] = hi;
}
#endif

// Keys in the accumulators (FP4 form, train sets of <= kHamFusedRows rows): the train
// operand's block scale is 2^13 (E8M0 140), and the accumulators start at
//   2^23 + (256 << 13) + (tile << 5) + row      (row = the element's train row in the tile)
// so after the four MFMAs each holds 2^23 + ((D + 256) << 13) + index exactly (every
// partial sum an integer below 2^24), and its bit pattern IS the key: ordered by D, then
// by index, the exponent bits common to all.  The per-element key construction is gone;
// the tile term is added once per tile per wave (shared by the wave's query groups).
constexpr int kHamFusedRows = 8192;  // tile < 256: 8 bits between the row and D fields
#ifndef YGZ_HAM_FUSED
#define YGZ_HAM_FUSED 1
#endif
template <bool FUSED>
__device__ __forceinline__ void hamming_block_mfma(const uint8_t *__restrict__ q, int nq, const uint8_t *__restrict__ t, int nt,
                                   int32_t *__restrict__ bi_out, int32_t *__restrict__ bd_out,
                                   int32_t *__restrict__ sd_out, int qblock) {
    static_assert(!FUSED || YGZ_HAM_FP4, "accumulator keys need the FP4 form");
    constexpr int G = kHamGroups;
    __shared__ __attribute__((aligned(16))) uint8_t s_tile[2][kHamTileBytes];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, h = lane >> 5;
    // group g of this lane: query qi0 + 32 g
    const int qw = qblock * kHamQPB + wave * 32 * G, qi0 = qw + (lane & 31);
#if YGZ_HAM_FP4
    constexpr int KS = 4;  // k-steps of 64 bits
#else
    constexpr int KS = 8;  // k-steps of 32 bits
#endif
    // query operands: +1 / -1 of this lane's half of each k-step's bits
    ham_v4i bq[G][KS];
#pragma unroll
    for (int g = 0; g < G; g++) {
        const int qi = qi0 + 32 * g;
        uint32_t w[8] = {0, 0, 0, 0, 0, 0, 0, 0};
        if (qi < nq) {
            const uint4 *qp = reinterpret_cast<const uint4 *>(q + (size_t)qi * 32);
            const uint4 u0 = qp[0], u1 = qp[1];
            w[0] = u0.x; w[1] = u0.y; w[2] = u0.z; w[3] = u0.w;
            w[4] = u1.x; w[5] = u1.y; w[6] = u1.z; w[7] = u1.w;
        }
#if YGZ_HAM_FP4
#pragma unroll
        for (int s = 0; s < 4; s++) {
            // bits 64 s + 32 h .. + 31, selected arithmetically (a select on h compiled to an
            // indexed access of w through scratch)
            const uint32_t d = w[2 * s] ^ ((w[2 * s] ^ w[2 * s + 1]) & (0u - (uint32_t)h));
#pragma unroll
            for (int m = 0; m < 4; m++) bq[g][s][m] = (int)((spread8(d >> (8 * m)) << 3) | 0x22222222u);  // +1 / -1
        }
#else
#pragma unroll
        for (int s = 0; s < 8; s++) {
            const uint32_t half = (w[s] >> (16 * h)) & 0xFFFFu;
#pragma unroll
            for (int m = 0; m < 4; m++) {
                const uint32_t e = nib_bytes(half, m);            // 0 / 1 per byte
                bq[g][s][m] = (int)(((e << 8) - e) | 0x01010101u);  // 0 -> +1, 1 -> -1 (0xFF)
            }
        }
#endif
    }
    uint32_t k1[G], k2[G];
#pragma unroll
    for (int g = 0; g < G; g++) k1[g] = k2[g] = kHamNone;
    // FUSED: the accumulators' start values less the tile term (train row of element r
    // of lane half h: (r & 3) + 8 (r >> 2) + 4 h)
    uint32_t cbase[16];
#pragma unroll
    for (int r = 0; r < 16; r++) cbase[r] = 0x4B000000u + (256u << 13) + (uint32_t)((r & 3) + 8 * (r >> 2) + 4 * h);
    // waves whose queries all lie past nq only stage tiles
    const bool active = qw < nq;
    const int ntiles = (nt + 31) >> 5;
    // staging (threads < 256): thread -> (row tid >> 3, dword tid & 7) of a 32-row tile
    const int srow = tid >> 3, sdw = tid & 7;
    const bool stager = tid < 256;
    // branch-free buffer loads: rows past nt (and tiles past the last) read 0, and no
    // load sits under an exec branch, so the wait counts before each expansion stay exact
    const __amdgpu_buffer_rsrc_t rt = __builtin_amdgcn_make_buffer_rsrc((void *)t, 0, nt * 32, 0x00020000);
    auto fetch = [&](int tile) -> uint32_t {
        return __builtin_amdgcn_raw_buffer_load_b32(rt, (uint32_t)(tile * 32 + srow) * 32u + 4u * (uint32_t)sdw, 0, 0);
    };
    // tile t: MFMAs on buffer t & 1, then the next tile's dwords (fetched earlier)
    // expanded into the other buffer, then one barrier
    auto tile_step = [&](int tile, uint32_t nxt) {
        const uint8_t *L = s_tile[tile & 1];
        if (active) {
            const uint8_t *arow = L + (lane & 31) * kHamRowBytes + h * 16;
#if YGZ_HAM_FP4
            ham_v16f accf[G];
            if (FUSED) {
                ham_v16f c0;
                const uint32_t tterm = __builtin_amdgcn_readfirstlane((uint32_t)tile << 5);
#pragma unroll
                for (int r = 0; r < 16; r++) c0[r] = __uint_as_float(cbase[r] + tterm);
#pragma unroll
                for (int g = 0; g < G; g++) accf[g] = c0;
            } else {
#pragma unroll
                for (int g = 0; g < G; g++)
#pragma unroll
                    for (int r = 0; r < 16; r++) accf[g][r] = kHamAccInit;
            }
#pragma unroll
            for (int s = 0; s < 4; s++) {
                const ham_v4i a4 = *(const ham_v4i *)(arow + s * 32);
                const ham_v8i a = {a4[0], a4[1], a4[2], a4[3], 0, 0, 0, 0};
#pragma unroll
                for (int g = 0; g < G; g++) {
                    const ham_v8i b = {bq[g][s][0], bq[g][s][1], bq[g][s][2], bq[g][s][3], 0, 0, 0, 0};
                    accf[g] = __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(a, b, accf[g], 4, 4, 0, FUSED ? 140 : 127,
                                                                              0, 127);
                }
            }
            if (FUSED) {  // the accumulators are the keys
                if (tile * 32 + 32 <= nt) {
#pragma unroll
                    for (int g = 0; g < G; g++)
#pragma unroll
                        for (int r = 0; r < 16; r++) {
                            const uint32_t key = __float_as_uint(accf[g][r]);
                            k2[g] = ham_med3(k1[g], key, k2[g]);
                            k1[g] = min(k1[g], key);
                        }
                } else {  // partial last tile: rows past nt never win
#pragma unroll
                    for (int g = 0; g < G; g++)
#pragma unroll
                        for (int r = 0; r < 16; r++) {
                            const int row = tile * 32 + (r & 3) + 8 * (r >> 2) + 4 * h;
                            const uint32_t key = row < nt ? __float_as_uint(accf[g][r]) : kHamNone;
                            k2[g] = ham_med3(k1[g], key, k2[g]);
                            k1[g] = min(k1[g], key);
                        }
                }
            } else {
            ham_v16i acc[G];
#pragma unroll
            for (int g = 0; g < G; g++)
#pragma unroll
                for (int r = 0; r < 16; r++) acc[g][r] = __float_as_int(accf[g][r]);  // 0x4B000000 + D + 256
            const uint32_t tb = (uint32_t)tile * 32, tu = tb;
#else
            {
            ham_v16i acc[G];
#pragma unroll
            for (int g = 0; g < G; g++) acc[g] = (ham_v16i){};
#pragma unroll
            for (int s = 0; s < 8; s++) {
                const ham_v4i a = *(const ham_v4i *)(arow + s * 32);
#pragma unroll
                for (int g = 0; g < G; g++) acc[g] = __builtin_amdgcn_mfma_i32_32x32x32_i8(a, bq[g][s], acc[g], 0, 0, 0);
            }
            const uint32_t tb = (uint32_t)tile * 32, tu = (256u << 22) + tb;
#endif
            if (tb + 32 <= (uint32_t)nt) {
#pragma unroll
                for (int g = 0; g < G; g++)
#pragma unroll
                    for (int r = 0; r < 16; r++) {
                        const uint32_t key = ham_key(acc[g][r], tu, (uint32_t)((r & 3) + 8 * (r >> 2)));
                        k2[g] = ham_med3(k1[g], key, k2[g]);
                        k1[g] = min(k1[g], key);
                    }
            } else {  // partial last tile: rows past nt never win
#pragma unroll
                for (int g = 0; g < G; g++)
#pragma unroll
                    for (int r = 0; r < 16; r++) {
                        const uint32_t row = tb + (uint32_t)((r & 3) + 8 * (r >> 2) + 4 * h);
                        const uint32_t key =
                            row < (uint32_t)nt ? ham_key(acc[g][r], tu, (uint32_t)((r & 3) + 8 * (r >> 2))) : kHamNone;
                        k2[g] = ham_med3(k1[g], key, k2[g]);
                        k1[g] = min(k1[g], key);
                    }
            }
            }  // (FUSED else)
        }
        if (tile + 1 < ntiles && stager) ham_expand_store(s_tile[(tile + 1) & 1], srow, sdw, nxt);
        __syncthreads();  // tile + 1 staged; tile's buffer free for tile + 2
    };
    if (ntiles > 0 && stager) ham_expand_store(s_tile[0], srow, sdw, fetch(0));
    __syncthreads();
    // one tile ahead is enough: fetching two ahead (the loop unrolled by two, so the
    // fetch registers alternate without a copy) measured the same
    for (int tile = 0; tile < ntiles; tile++) tile_step(tile, fetch(tile + 1));
#pragma unroll
    for (int g = 0; g < G; g++) {
        // the lane half's row offset, then merge the two halves (same query, disjoint rows)
        uint32_t a1 = k1[g], a2 = k2[g];
        if (!FUSED) {  // (the accumulator keys carry it already)
            if (a1 != kHamNone) a1 += 4u * (uint32_t)h;
            if (a2 != kHamNone) a2 += 4u * (uint32_t)h;
        }
        const uint32_t o1 = (uint32_t)__shfl_xor((int)a1, 32, 64), o2 = (uint32_t)__shfl_xor((int)a2, 32, 64);
        const uint32_t K1 = min(a1, o1), K2 = min(max(a1, o1), min(a2, o2));
        const int qi = qi0 + 32 * g;
        if (h == 0 && qi < nq) {
            // popc(q) read again here: not held in registers through the tile loop
            const uint4 *qp = reinterpret_cast<const uint4 *>(q + (size_t)qi * 32);
            const uint4 u0 = qp[0], u1 = qp[1];
            const int pq = __popc(u0.x) + __popc(u0.y) + __popc(u0.z) + __popc(u0.w) + __popc(u1.x) + __popc(u1.y) +
                           __popc(u1.z) + __popc(u1.w);
            if (FUSED) {  // key bits 0x4B000000 + ((D + 256) << 13) + index
                bi_out[qi] = K1 == kHamNone ? -1 : (int)(K1 & 0x1FFFu);
                bd_out[qi] = K1 == kHamNone ? 257 : (int)((K1 >> 13) & 0x3FFu) - 256 + pq;
                sd_out[qi] = K2 == kHamNone ? 257 : (int)((K2 >> 13) & 0x3FFu) - 256 + pq;
            } else {
                bi_out[qi] = K1 == kHamNone ? -1 : (int)(K1 & (kHamMaxTrain - 1));
                bd_out[qi] = K1 == kHamNone ? 257 : (int)(K1 >> 22) - 256 + pq;
                sd_out[qi] = K2 == kHamNone ? 257 : (int)(K2 >> 22) - 256 + pq;
            }
        }
    }
}

__global__ __launch_bounds__(64 * kHamWaves) void k_hamming_best2(const uint8_t *__restrict__ q, int nq,
                                                       const uint8_t *__restrict__ t, int nt,
                                                       int32_t *__restrict__ bi, int32_t *__restrict__ bd,
                                                       int32_t *__restrict__ sd) {
    if (YGZ_HAM_FP4 && YGZ_HAM_FUSED && nt <= kHamFusedRows)
        hamming_block_mfma<(bool)YGZ_HAM_FP4>(q, nq, t, nt, bi, bd, sd, blockIdx.x);
    else
        hamming_block_mfma<false>(q, nq, t, nt, bi, bd, sd, blockIdx.x);
}

// batched: pair p matches the descriptors of frame qframe[p] against frame
// tframe[p] of a batch (rows [0, counts[f]) of a [F][row_cap][32] array);
// outputs at [p][row_cap].
__global__ __launch_bounds__(64 * kHamWaves) void k_hamming_best2_pairs(const uint8_t *__restrict__ desc,
                                                             const int32_t *__restrict__ counts, int row_cap,
                                                             const int32_t *__restrict__ qframe,
                                                             const int32_t *__restrict__ tframe,
                                                             int32_t *__restrict__ bi, int32_t *__restrict__ bd,
                                                             int32_t *__restrict__ sd) {
    const int p = blockIdx.y;
    const int qf = qframe[p], tf = tframe[p];
    const int nq = counts[qf], nt = counts[tf];
    if ((int)(blockIdx.x * kHamQPB) >= nq) return;
    if (YGZ_HAM_FP4 && YGZ_HAM_FUSED && nt <= kHamFusedRows)  // (wave-uniform: one pair per workgroup)
        hamming_block_mfma<(bool)YGZ_HAM_FP4>(desc + (size_t)qf * row_cap * 32, nq, desc + (size_t)tf * row_cap * 32,
                                              nt, bi + (size_t)p * row_cap, bd + (size_t)p * row_cap,
                                              sd + (size_t)p * row_cap, blockIdx.x);
    else
        hamming_block_mfma<false>(desc + (size_t)qf * row_cap * 32, nq, desc + (size_t)tf * row_cap * 32, nt,
                                  bi + (size_t)p * row_cap, bd + (size_t)p * row_cap, sd + (size_t)p * row_cap,
                                  blockIdx.x);
}

// CSR candidate distances: dist[k] for k in [row_ptr[i], row_ptr[i+1]) of query i.
__global__ __launch_bounds__(256) void k_hamming_csr(const uint8_t *__restrict__ q, int nq,
                                                     const uint8_t *__restrict__ t,
                                                     const int32_t *__restrict__ row_ptr,
                                                     const int32_t *__restrict__ cand, int32_t *__restrict__ dist) {
    const int i = blockIdx.x * (blockDim.x / 64) + (threadIdx.x >> 6);
    const int lane = threadIdx.x & 63;
    if (i >= nq) return;
    const uint4 *qp = reinterpret_cast<const uint4 *>(q + (size_t)i * 32);
    const uint4 u0 = qp[0], u1 = qp[1];
    for (int k = row_ptr[i] + lane; k < row_ptr[i + 1]; k += 64) {
        const uint4 *tp = reinterpret_cast<const uint4 *>(t + (size_t)cand[k] * 32);
        const uint4 v0 = tp[0], v1 = tp[1];
        dist[k] = __popc(u0.x ^ v0.x) + __popc(u0.y ^ v0.y) + __popc(u0.z ^ v0.z) + __popc(u0.w ^ v0.w) +
                  __popc(u1.x ^ v1.x) + __popc(u1.y ^ v1.y) + __popc(u1.z ^ v1.z) + __popc(u1.w ^ v1.w);
    }
}

hipError_t launch_hamming_best2(const uint8_t *q, int nq, const uint8_t *t, int nt, int32_t *bi, int32_t *bd,
                                int32_t *sd, hipStream_t st) {
    if (nq <= 0) return hipSuccess;
    if (nt > kHamMaxTrain) return hipErrorInvalidValue;  // train index must fit the key's 22 bits
    hipLaunchKernelGGL(k_hamming_best2, dim3((nq + kHamQPB - 1) / kHamQPB), dim3(64 * kHamWaves), 0, st, q, nq, t, nt, bi, bd,
                       sd);
    return hipGetLastError();
}

hipError_t launch_hamming_best2_pairs(const uint8_t *desc, const int32_t *counts, int row_cap, int npairs,
                                      const int32_t *qframe, const int32_t *tframe, int32_t *bi, int32_t *bd,
                                      int32_t *sd, hipStream_t st) {
    if (npairs <= 0) return hipSuccess;
    if (row_cap > kHamMaxTrain) return hipErrorInvalidValue;
    hipLaunchKernelGGL(k_hamming_best2_pairs, dim3((row_cap + kHamQPB - 1) / kHamQPB, npairs), dim3(64 * kHamWaves), 0, st,
                       desc, counts, row_cap, qframe, tframe, bi, bd, sd);
    return hipGetLastError();
}

hipError_t launch_hamming_csr(const uint8_t *q, int nq, const uint8_t *t, const int32_t *row_ptr,
                              const int32_t *cand, int32_t *dist, hipStream_t st) {
    if (nq <= 0) return hipSuccess;
    hipLaunchKernelGGL(k_hamming_csr, dim3((nq + 3) / 4), dim3(256), 0, st, q, nq, t, row_ptr, cand, dist);
    return hipGetLastError();
}

}  // namespace ygzfe
