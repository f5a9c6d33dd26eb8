// dsort_text.hip -- the reference's text codec on the GPU.
//
//   format: sorted keys -> output.txt bytes, one "%d\n" per key (reference server.c:518,
//           fprintf(output, "%d\n", ...) in merge_chunks);
//   parse:  input text -> keys: whitespace-separated %d tokens (server.c:179 and 213,
//           fscanf(file, "%d", ...)).  A token is [+-]?[0-9]+ ending at whitespace or the end of
//           the text; anything else is an error (the reference spins forever on it, SURVEY.md
//           §8a(4)).  Out-of-range values saturate at 2^32 and wrap to int32, the oracle's rule
//           (oracle.c oracle_parse_i32; %d overflow is undefined in the reference).
//
// Both run in three launches: a count pass (per tile: the text bytes of its keys, or the tokens
// of its text), an exclusive scan of the tile counts (one workgroup), and the pass that writes,
// every tile at its scanned offset.  Format builds each tile's bytes in LDS at the same 16-byte
// phase as their global position and stores whole 16-byte chunks (byte stores only at the two
// partial ends).  Parse stages its tile (+ halo) in LDS with 16-byte loads; token starts come from
// whitespace flags four bytes at a time, a token's digits from its 16 staged bytes.
// (Round 1 chained the tiles with a decoupled look-back instead, one pass: the inclusive prefix
// crossed about 64 tiles per status round trip, and that chain, not HBM, set the time -- 2^28 keys:
// format 1.74 ms, parse 2.5-2.8 ms, 36 % of a parse tile spent in the look-back.)
//
// Algorithmic HBM bytes: format 4 B/key read + the text written; parse the text read + 4 B/key
// written.  (The count passes read the keys, or the text, once more.)
#include <hip/hip_runtime.h>

#include <stdint.h>

#include "dsort_internal.h"

namespace dsort {
namespace tx {

constexpr int NT = 256;                  // threads per workgroup
constexpr int FK = 8;                    // keys per thread (format)
constexpr int FTILE = NT * FK;           // keys per format tile
constexpr int FBYTES = FTILE * 12;       // at most 12 bytes per key ("-2147483648\n")
constexpr int PB = 64;                   // text bytes per thread (parse)
constexpr int PTILE = NT * PB;           // text bytes per parse tile
constexpr int PHALO = 64;                // bytes staged past the tile (tokens that straddle it)
constexpr int PLDS = 16 + PTILE + PHALO; // staged bytes: 16 before the tile (the previous byte)

__device__ __forceinline__ int lane_id() { return threadIdx.x & 63; }

#ifdef DSORT_STAMPS
// Diagnostic build only: per-tile phase cycles of parse_kernel (thread 0's view), read back by
// dsort_debug_txstamps() (scripts/dev/txstamps.py).
__device__ unsigned long long g_txstamps[(1u << 18) * 8];
#define TXST(k)                                            \
    do {                                                   \
        const uint64_t t1_ = __builtin_amdgcn_s_memtime(); \
        tx_acc[k] = t1_ - tx_t0;                           \
        tx_t0 = t1_;                                       \
    } while (0)
#else
#define TXST(k) \
    do {        \
    } while (0)
#endif

__device__ __forceinline__ uint64_t wave_sum_u64(uint64_t v) {
    for (int o = 32; o >= 1; o >>= 1) v += __shfl_xor(v, o);
    return v;
}

// Exclusive scan of one value per thread over the 256-thread workgroup; `agg` = total.
__device__ __forceinline__ uint32_t block_scan(uint32_t v, uint32_t *wsum, uint32_t &agg) {
    const int lane = lane_id(), w = threadIdx.x >> 6;
    uint32_t incl = wave_incl_sum(v);
    if (lane == 63) wsum[w] = incl;
    __syncthreads();
    uint32_t woff = 0;
    agg = 0;
#pragma unroll
    for (int i = 0; i < NT / 64; ++i) {
        if (i < w) woff += wsum[i];
        agg += wsum[i];
    }
    return woff + incl - v;
}

__device__ __forceinline__ int dec_digits(uint32_t u) {
    return 1 + (u >= 10u) + (u >= 100u) + (u >= 1000u) + (u >= 10000u) + (u >= 100000u) +
           (u >= 1000000u) + (u >= 10000000u) + (u >= 100000000u) + (u >= 1000000000u);
}
__device__ __forceinline__ uint32_t mag(int32_t v) { return v < 0 ? 0u - (uint32_t)v : (uint32_t)v; }

// Sum of one value per thread over the workgroup (every thread gets it).
__device__ __forceinline__ uint32_t block_sum(uint32_t v, uint32_t *wsum) {
    uint32_t agg;
    (void)block_scan(v, wsum, agg);
    return agg;
}

// Per-tile totals -> exclusive prefixes (one workgroup of 1024 threads); *total = their sum.  A round
// takes SCAN_Q consecutive tiles per thread (16-byte loads), scans the thread sums, and stages the
// tiles' offsets from the round's start in LDS, so that the 8-byte prefixes go out coalesced.
// (Written straight from each thread's registers, every store instruction touched 64 lines: 105 us
// for the 180 000 tiles of 2^28 keys' text.)
constexpr int SCAN_T = 1024, SCAN_Q = 32, SCAN_ROUND = SCAN_T * SCAN_Q;
__global__ void __launch_bounds__(SCAN_T) tile_scan_kernel(const uint32_t *__restrict__ cnt, uint64_t *__restrict__ pref,
                                                           uint32_t ntiles, uint64_t *__restrict__ total) {
    __shared__ uint64_t wsum[SCAN_T / 64];
    __shared__ uint32_t rel[SCAN_ROUND + SCAN_ROUND / SCAN_Q];  // (one pad word per thread's run)
    const int lane = lane_id(), w = threadIdx.x >> 6;
    const auto slot = [](uint32_t j) { return j + j / SCAN_Q; };
    uint64_t carry = 0;
    for (uint32_t b0 = 0; b0 < ntiles; b0 += SCAN_ROUND) {
        const uint32_t i0 = b0 + SCAN_Q * threadIdx.x;
        uint32_t v[SCAN_Q];
        if (i0 + SCAN_Q <= ntiles) {
#pragma unroll
            for (int q = 0; q < SCAN_Q / 4; ++q) {
                const uint4 x = reinterpret_cast<const uint4 *>(cnt + i0)[q];
                v[4 * q] = x.x; v[4 * q + 1] = x.y; v[4 * q + 2] = x.z; v[4 * q + 3] = x.w;
            }
        } else {
#pragma unroll
            for (int q = 0; q < SCAN_Q; ++q) v[q] = i0 + q < ntiles ? cnt[i0 + q] : 0u;
        }
        uint32_t sum = 0;  // (a round's tiles hold < 2^32 bytes or tokens: 32768 tiles of <= 24 KiB)
#pragma unroll
        for (int q = 0; q < SCAN_Q; ++q) sum += v[q];
        uint32_t incl = wave_incl_sum(sum);
        if (lane == 63) wsum[w] = incl;
        __syncthreads();
        uint32_t ex = incl - sum, all = 0;
#pragma unroll
        for (int i = 0; i < SCAN_T / 64; ++i) {
            ex += i < w ? (uint32_t)wsum[i] : 0u;
            all += (uint32_t)wsum[i];
        }
#pragma unroll
        for (int q = 0; q < SCAN_Q; ++q) {
            rel[slot(SCAN_Q * threadIdx.x + q)] = ex;
            ex += v[q];
        }
        __syncthreads();
        const uint32_t nr = ntiles - b0 < (uint32_t)SCAN_ROUND ? ntiles - b0 : (uint32_t)SCAN_ROUND;
        for (uint32_t j = threadIdx.x; j < nr; j += SCAN_T) pref[b0 + j] = carry + rel[slot(j)];
        carry += all;
        __syncthreads();  // (wsum and rel are rewritten by the next round)
    }
    if (threadIdx.x == 0) *total = carry;
}

// ---------------------------------------------------------------------------- format ------
// The FK keys of thread t of tile `tile` and their %d\n lengths (0 past n).
__device__ __forceinline__ uint32_t format_keys(const int32_t *__restrict__ keys, uint64_t n, uint32_t tile,
                                                int32_t (&v)[FK], int (&len)[FK]) {
    const uint64_t k0 = (uint64_t)tile * FTILE + (uint64_t)FK * threadIdx.x;
    if (k0 + FK <= n && ((reinterpret_cast<uintptr_t>(keys + k0) & 15) == 0)) {
        const int4 a = *reinterpret_cast<const int4 *>(keys + k0);
        const int4 b = *reinterpret_cast<const int4 *>(keys + k0 + 4);
        v[0] = a.x; v[1] = a.y; v[2] = a.z; v[3] = a.w;
        v[4] = b.x; v[5] = b.y; v[6] = b.z; v[7] = b.w;
#pragma unroll
        for (int k = 0; k < FK; ++k) len[k] = dec_digits(mag(v[k])) + (v[k] < 0) + 1;
    } else {
#pragma unroll
        for (int k = 0; k < FK; ++k) {
            const bool ok = k0 + k < n;
            v[k] = ok ? keys[k0 + k] : 0;
            len[k] = ok ? dec_digits(mag(v[k])) + (v[k] < 0) + 1 : 0;
        }
    }
    uint32_t tot = 0;
#pragma unroll
    for (int k = 0; k < FK; ++k) tot += len[k];
    return tot;
}

// text bytes of every format tile
__global__ void __launch_bounds__(NT) format_count_kernel(const int32_t *__restrict__ keys, uint64_t n,
                                                          uint32_t *__restrict__ cnt) {
    __shared__ uint32_t wsum[NT / 64];
    int32_t v[FK];
    int len[FK];
    const uint32_t agg = block_sum(format_keys(keys, n, blockIdx.x, v, len), wsum);
    if (threadIdx.x == 0) cnt[blockIdx.x] = agg;
}

// (round 6) the formatted text's whole 16-byte chunks as non-temporal stores: format 1.27-1.30 ->
// 1.23-1.25 ms at 2^28 keys, 3 of 3 interleaved runs (profiles/r6_ab_text_format_nontemporal.log)
#ifndef DSORT_TEXT_NT
#define DSORT_TEXT_NT 1
#endif
__global__ void __launch_bounds__(NT) format_kernel(const int32_t *__restrict__ keys, uint64_t n,
                                                    char *__restrict__ text, uint64_t cap,
                                                    const uint64_t *__restrict__ pref) {
    __shared__ uint32_t wsum[NT / 64];
    __shared__ __attribute__((aligned(16))) char sb[FBYTES + 32];
    const uint32_t tile = blockIdx.x;
    const uint64_t O = pref[tile];
    int32_t v[FK];
    int len[FK];
    uint32_t agg;
    const uint32_t toff = block_scan(format_keys(keys, n, tile, v, len), wsum, agg);
    if (O + agg > cap) return;  // the host sizes `text` for 12 bytes per key; never taken then
    // bytes of the tile at LDS position sh + j, sh = the 16-byte phase of text + O
    const int sh = (int)(reinterpret_cast<uintptr_t>(text + O) & 15);
    int p = sh + (int)toff;
#pragma unroll
    for (int k = 0; k < FK; ++k) {
        if (!len[k]) continue;
        uint32_t u = mag(v[k]);
        if (v[k] < 0) sb[p] = '-';
        const int last = p + len[k] - 2;  // last digit
        int q = last;
        do {
            const uint32_t d = u / 10u;
            sb[q--] = (char)('0' + (u - d * 10u));
            u = d;
        } while (u);
        sb[last + 1] = '\n';
        p += len[k];
    }
    __syncthreads();
    char *ga = text + O - sh;  // 16-byte aligned
    const int hi = sh + (int)agg;
    const int nch = (hi + 15) >> 4;
    for (int c = threadIdx.x; c < nch; c += NT) {
        const int lo_b = c * 16, hi_b = lo_b + 16;
        if (lo_b >= sh && hi_b <= hi) {
#if DSORT_TEXT_NT
            typedef int text_v4i __attribute__((ext_vector_type(4)));
            __builtin_nontemporal_store(*reinterpret_cast<const text_v4i *>(sb + lo_b),
                                        reinterpret_cast<text_v4i *>(ga + lo_b));
#else
            *reinterpret_cast<int4 *>(ga + lo_b) = *reinterpret_cast<const int4 *>(sb + lo_b);
#endif
        } else {
            const int b0 = lo_b > sh ? lo_b : sh, b1 = hi_b < hi ? hi_b : hi;
            for (int b = b0; b < b1; ++b) ga[b] = sb[b];
        }
    }
}

// ----------------------------------------------------------------------------- parse ------
__device__ __forceinline__ bool is_ws(uint32_t c) { return c == 32u || (c - 9u) < 5u; }

// byte `pos` of the staged window, or of global memory past it (long tokens); ' ' outside the text
__device__ __forceinline__ uint32_t text_byte(const unsigned char *lb, int pos, const char *ga,
                                              const char *text, uint64_t len) {
    if (pos < PLDS) return lb[pos];
    const char *a = ga + pos;
    return (a >= text && a < text + len) ? (unsigned char)*a : 32u;
}

// Four bytes at once: bit 7 of byte k set iff byte k is whitespace (' ', 9..13) -- no carry
// crosses a byte: every subtraction is from a byte with bit 7 set.
__device__ __forceinline__ uint32_t ws_bits4(uint32_t x) {
    const uint32_t lo = x & 0x7F7F7F7Fu, t = x ^ 0x20202020u;
    const uint32_t nsp = (((t & 0x7F7F7F7Fu) + 0x7F7F7F7Fu) | t) & 0x80808080u;  // byte != ' '
    const uint32_t lt14 = ~((lo | 0x80808080u) - 0x0E0E0E0Eu);
    const uint32_t ge9 = (lo | 0x80808080u) - 0x09090909u;
    return ((~nsp & 0x80808080u) | (lt14 & ge9 & 0x80808080u)) & ~x;
}
// bit 7 of byte k set iff byte k is a decimal digit
__device__ __forceinline__ uint32_t dig_bits4(uint32_t x) {
    const uint32_t y = x ^ 0x30303030u;
    const uint32_t lt10 = ~(((y & 0x7F7F7F7Fu) | 0x80808080u) - 0x0A0A0A0Au);
    return lt10 & ~y & 0x80808080u;
}
// the four bit-7 flags of ws_bits4 / dig_bits4 -> bits 0..3
__device__ __forceinline__ uint32_t pack4(uint32_t m) {
    m >>= 7;
    return (m | (m >> 7) | (m >> 14) | (m >> 21)) & 15u;
}
// The byte loop of round 1, for the tokens the fast path leaves: the key of the token at LDS
// byte pos (text byte tpos); a token that is not [+-]?[0-9]+ followed by whitespace reports tpos.
__device__ uint32_t parse_slow(const unsigned char *lb, int pos, const char *ga, const char *text, uint64_t len,
                               uint64_t tpos, unsigned long long *err_pos) {
    uint32_t c = lb[pos];
    const bool neg = c == '-';
    if (c == '-' || c == '+') c = text_byte(lb, ++pos, ga, text, len);
    uint64_t val = 0;
    int nd = 0;
    while (c - '0' < 10u) {
        val = val * 10u + (c - '0');
        val = val > (1ull << 32) ? (1ull << 32) : val;
        ++nd;
        c = text_byte(lb, ++pos, ga, text, len);
    }
    if (nd == 0 || !is_ws(c)) atomicMin(err_pos, (unsigned long long)tpos);
    return (uint32_t)(neg ? 0ull - val : val);
}

// Token starts among a thread's 64 bytes (w16): a non-whitespace byte after whitespace (or after
// the start of the text).  Whitespace flags four bytes at a time, then one 64-bit mask.
__device__ __forceinline__ uint64_t token_starts(const uint32_t (&w16)[PB / 4], bool prev_ws) {
    uint64_t W = 0;
#pragma unroll
    for (int k = 0; k < PB / 4; ++k) W |= (uint64_t)pack4(ws_bits4(w16[k])) << (4 * k);
    return ~W & ((W << 1) | (prev_ws ? 1ull : 0ull));
}

// tokens of every parse tile, read straight from HBM (outside the text: ' ')
__global__ void __launch_bounds__(NT) parse_count_kernel(const char *__restrict__ text, uint64_t len,
                                                         uint32_t *__restrict__ cnt) {
    __shared__ uint32_t wsum[NT / 64];
    const uint64_t b0 = (uint64_t)blockIdx.x * PTILE + (uint64_t)PB * threadIdx.x;
    uint32_t w16[PB / 4];
    if (b0 + PB <= len) {
#pragma unroll
        for (int i = 0; i < PB / 16; ++i) {
            const uint4 q = reinterpret_cast<const uint4 *>(text + b0)[i];
            w16[4 * i] = q.x; w16[4 * i + 1] = q.y; w16[4 * i + 2] = q.z; w16[4 * i + 3] = q.w;
        }
    } else {
#pragma unroll
        for (int k = 0; k < PB / 4; ++k) {
            uint32_t x = 0;
#pragma unroll
            for (int b = 0; b < 4; ++b) {
                const uint64_t g = b0 + 4 * k + b;
                x |= (g < len ? (uint32_t)(unsigned char)text[g] : 32u) << (8 * b);
            }
            w16[k] = x;
        }
    }
    const bool prev_ws = b0 == 0 || b0 > len || is_ws((unsigned char)text[b0 - 1]);
    const uint32_t agg = block_sum((uint32_t)__popcll(token_starts(w16, prev_ws)), wsum);
    if (threadIdx.x == 0) cnt[blockIdx.x] = agg;
}

// The key of the token starting at LDS byte pos.  Fast path: the 16 staged bytes from the token's
// dword (pos + 15 < PLDS for every start of the tile); a sign, then L < 12 digits and a whitespace
// byte.  (Round 1 read every digit from LDS in a dependent chain of byte loads: 2.86 ms at 2^28
// keys, 0.18 of HBM.)  Longer tokens (leading zeros) and malformed ones take the byte loop.
__device__ __forceinline__ uint32_t parse_token(const uint32_t *lw, const unsigned char *lb, int pos, const char *ga,
                                                const char *text, uint64_t len, uint64_t tb,
                                                unsigned long long *err_pos) {
    const int a = pos >> 2;
    const uint64_t lo64 = (uint64_t)lw[a + 1] << 32 | lw[a], hi64 = (uint64_t)lw[a + 3] << 32 | lw[a + 2];
    const uint32_t c0 = (uint32_t)(lo64 >> (8 * (pos & 3))) & 255u;
    const bool neg = c0 == '-', sg = neg || c0 == '+';
    const uint32_t s8 = 8u * (uint32_t)((pos & 3) + (sg ? 1 : 0));  // 0..32
    const uint64_t r0 = s8 ? (lo64 >> s8) | (hi64 << (64u - s8)) : lo64, r1 = hi64 >> s8;
    const uint32_t e[3] = {(uint32_t)r0, (uint32_t)(r0 >> 32), (uint32_t)r1};  // bytes after the sign
    const uint32_t m12 = pack4(dig_bits4(e[0])) | pack4(dig_bits4(e[1])) << 4 | pack4(dig_bits4(e[2])) << 8;
    const int L = __ffs(~m12) - 1;  // leading digits, 0..12
    const uint32_t tw = L < 4 ? e[0] : (L < 8 ? e[1] : e[2]);
    const uint32_t term = (tw >> (8 * (L & 3))) & 255u;
    if (L > 0 && L < 12 && is_ws(term)) {
        uint32_t v = 0;
#pragma unroll
        for (int k = 0; k < 9; ++k) {
            const uint32_t d = ((e[k >> 2] >> (8 * (k & 3))) & 255u) - '0';
            v = k < L ? v * 10u + d : v;
        }
        uint64_t V = v;
#pragma unroll
        for (int k = 9; k < 11; ++k) {
            const uint32_t d = ((e[k >> 2] >> (8 * (k & 3))) & 255u) - '0';
            V = k < L ? V * 10u + d : V;
        }
        // the oracle's saturation at 2^32 (then the int32 wrap): a value >= 2^32 is key 0
        return V >= (1ull << 32) ? 0u : (neg ? 0u - (uint32_t)V : (uint32_t)V);
    }
    return parse_slow(lb, pos, ga, text, len, tb + pos - 16, err_pos);
}

__global__ void __launch_bounds__(NT) parse_kernel(const char *__restrict__ text, uint64_t len,
                                                   int32_t *__restrict__ keys, uint64_t cap,
                                                   const uint64_t *__restrict__ pref, unsigned long long *err_pos) {
    __shared__ uint32_t wsum[NT / 64];
    __shared__ __attribute__((aligned(16))) uint32_t lw[PLDS / 4];
#ifdef DSORT_STAMPS
    uint64_t tx_acc[8] = {}, tx_t0 = __builtin_amdgcn_s_memtime();
#endif
    const uint32_t tile = blockIdx.x;
    const uint64_t base = pref[tile];
    const uint64_t tb = (uint64_t)tile * PTILE;
    TXST(0);
    // LDS byte j <-> text byte tb - 16 + j (text is 16-byte aligned); outside the text: ' '
    const char *ga = text + tb - 16;
    for (int ci = threadIdx.x; ci < PLDS / 16; ci += NT) {
        const int64_t g0 = (int64_t)tb - 16 + 16 * ci;  // text index of the chunk's first byte
        uint4 q = make_uint4(0x20202020u, 0x20202020u, 0x20202020u, 0x20202020u);
        if (g0 >= 0 && g0 + 16 <= (int64_t)len) {
            q = *reinterpret_cast<const uint4 *>(text + g0);
        } else if (g0 + 16 > 0 && g0 < (int64_t)len) {
            uint32_t wv[4];
#pragma unroll
            for (int b = 0; b < 16; ++b) {
                const int64_t g = g0 + b;
                const uint32_t c = (g >= 0 && g < (int64_t)len) ? (unsigned char)text[g] : 32u;
                if ((b & 3) == 0) wv[b >> 2] = 0;
                wv[b >> 2] |= c << (8 * (b & 3));
            }
            q = make_uint4(wv[0], wv[1], wv[2], wv[3]);
        }
        *reinterpret_cast<uint4 *>(&lw[4 * ci]) = q;
    }
    __syncthreads();
    TXST(1);
    const unsigned char *lb = reinterpret_cast<const unsigned char *>(lw);
    const int my0 = 16 + PB * threadIdx.x;  // LDS index of this thread's first byte
    uint32_t w16[PB / 4];
#pragma unroll
    for (int i = 0; i < PB / 16; ++i) {
        const uint4 q = *reinterpret_cast<const uint4 *>(&lw[my0 / 4 + 4 * i]);
        w16[4 * i] = q.x; w16[4 * i + 1] = q.y; w16[4 * i + 2] = q.z; w16[4 * i + 3] = q.w;
    }
    uint64_t starts = token_starts(w16, is_ws(lb[my0 - 1]));
    uint32_t agg;
    uint64_t idx = base + block_scan((uint32_t)__popcll(starts), wsum, agg);
    TXST(2);
    while (starts) {
        const int i = __ffsll((long long)starts) - 1;
        starts &= starts - 1;
        const uint32_t key = parse_token(lw, lb, my0 + i, ga, text, len, tb, err_pos);
        if (idx < cap) keys[idx] = (int32_t)key;
        ++idx;
    }
    // (Measured and not kept: the tile's token starts listed in LDS and taken round-robin by the
    // threads -- balanced lanes, coalesced key stores -- 1.77-1.84 against 1.77 ms.)
#ifdef DSORT_STAMPS
    TXST(3);
    if (threadIdx.x == 0 && tile < (1u << 18))
        for (int k = 0; k < 4; ++k) g_txstamps[tile * 8 + k] = tx_acc[k];
#endif
}

}  // namespace tx

// The tile tables (per-tile counts, then their exclusive prefixes) and the reductions: red[1] =
// total bytes / tokens (the scan's), red[2] = first error position (~0: none).
static int text_prepare(dsort_ctx *ctx, uint64_t ntiles, hipStream_t s, uint32_t **cnt, uint64_t **pref) {
    const size_t cbytes = (ntiles * sizeof(uint32_t) + 255) & ~(size_t)255;
    int rc = ensure(ctx, &ctx->text_status, &ctx->text_status_bytes, cbytes + ntiles * sizeof(uint64_t),
                    "text tile tables");
    if (rc) return rc;
    *cnt = static_cast<uint32_t *>(ctx->text_status);
    *pref = reinterpret_cast<uint64_t *>(static_cast<char *>(ctx->text_status) + cbytes);
    DSORT_HIP(ctx, hipMemsetAsync(static_cast<char *>(ctx->red) + 16, 0xFF, 8, s));
    return DSORT_OK;
}

}  // namespace dsort

using namespace dsort;

extern "C" {

int dsort_format_text_dev_i32(dsort_ctx *ctx, const int32_t *d_keys, size_t n, char *d_text,
                              size_t cap, size_t *out_len, void *stream) {
    if (!ctx || !out_len || (n && (!d_keys || !d_text)))
        return set_err(ctx, DSORT_EINVAL, "null argument");
    if (cap / 12 < n) return set_err(ctx, DSORT_EINVAL, "text buffer smaller than 12 bytes per key");
    *out_len = 0;
    if (!n) return DSORT_OK;
    hipStream_t s = pick_stream(ctx, stream);
    const uint64_t ntiles = (n + tx::FTILE - 1) / tx::FTILE;
    if (ntiles > 0xFFFFFFFFull) return set_err(ctx, DSORT_EINVAL, "too many keys");
    uint32_t *cnt;
    uint64_t *pref;
    int rc = text_prepare(ctx, ntiles, s, &cnt, &pref);
    if (rc) return rc;
    uint64_t *red = static_cast<uint64_t *>(ctx->red);
    hipLaunchKernelGGL(tx::format_count_kernel, dim3((unsigned)ntiles), dim3(tx::NT), 0, s, d_keys, (uint64_t)n, cnt);
    hipLaunchKernelGGL(tx::tile_scan_kernel, dim3(1), dim3(tx::SCAN_T), 0, s, cnt, pref, (uint32_t)ntiles, red + 1);
    hipLaunchKernelGGL(tx::format_kernel, dim3((unsigned)ntiles), dim3(tx::NT), 0, s, d_keys,
                       (uint64_t)n, d_text, (uint64_t)cap, static_cast<const uint64_t *>(pref));
    DSORT_HIP(ctx, hipGetLastError());
    DSORT_HIP(ctx, hipMemcpyAsync(ctx->red_host, ctx->red, 24, hipMemcpyDeviceToHost, s));
    DSORT_HIP(ctx, hipStreamSynchronize(s));
    *out_len = ctx->red_host[1];
    return DSORT_OK;
}

int dsort_parse_text_dev_i32(dsort_ctx *ctx, const char *d_text, size_t len, int32_t *d_keys,
                             size_t cap, size_t *n_out, void *stream) {
    if (!ctx || !n_out || (len && !d_text) || (cap && !d_keys))
        return set_err(ctx, DSORT_EINVAL, "null argument");
    if (reinterpret_cast<uintptr_t>(d_text) & 15)
        return set_err(ctx, DSORT_EINVAL, "text buffer must be 16-byte aligned");
    *n_out = 0;
    if (!len) return DSORT_OK;
    hipStream_t s = pick_stream(ctx, stream);
    const uint64_t ntiles = (len + tx::PTILE - 1) / tx::PTILE;
    if (ntiles > 0xFFFFFFFFull) return set_err(ctx, DSORT_EINVAL, "text too long");
    uint32_t *cnt;
    uint64_t *pref;
    int rc = text_prepare(ctx, ntiles, s, &cnt, &pref);
    if (rc) return rc;
    uint64_t *red = static_cast<uint64_t *>(ctx->red);
    hipLaunchKernelGGL(tx::parse_count_kernel, dim3((unsigned)ntiles), dim3(tx::NT), 0, s, d_text, (uint64_t)len, cnt);
    hipLaunchKernelGGL(tx::tile_scan_kernel, dim3(1), dim3(tx::SCAN_T), 0, s, cnt, pref, (uint32_t)ntiles, red + 1);
    hipLaunchKernelGGL(tx::parse_kernel, dim3((unsigned)ntiles), dim3(tx::NT), 0, s, d_text,
                       (uint64_t)len, d_keys, (uint64_t)cap, static_cast<const uint64_t *>(pref),
                       reinterpret_cast<unsigned long long *>(red + 2));
    DSORT_HIP(ctx, hipGetLastError());
    DSORT_HIP(ctx, hipMemcpyAsync(ctx->red_host, ctx->red, 24, hipMemcpyDeviceToHost, s));
    DSORT_HIP(ctx, hipStreamSynchronize(s));
    *n_out = ctx->red_host[1];
    if (ctx->red_host[2] != ~0ull)
        return set_err(ctx, DSORT_EINVAL,
                       "not an integer token at byte " + std::to_string(ctx->red_host[2]));
    return DSORT_OK;
}

// Host-buffer forms for the C master (server.c's parse and output.txt write): stage through the
// context's device arenas.
int dsort_parse_text_i32(dsort_ctx *ctx, const char *text, size_t len, int32_t *keys, size_t cap,
                         size_t *n_out) {
    if (!ctx || !n_out || (len && !text) || (cap && !keys))
        return set_err(ctx, DSORT_EINVAL, "null argument");
    *n_out = 0;
    if (!len) return DSORT_OK;
    int rc = ensure(ctx, &ctx->io, &ctx->io_bytes, len, "text staging");
    if (!rc) rc = ensure(ctx, &ctx->io2, &ctx->io2_bytes, (cap ? cap : 1) * sizeof(int32_t), "key staging");
    if (rc) return rc;
    hipStream_t s = ctx->stream;
    DSORT_HIP(ctx, hipMemcpyAsync(ctx->io, text, len, hipMemcpyHostToDevice, s));
    size_t cnt = 0;
    rc = dsort_parse_text_dev_i32(ctx, static_cast<const char *>(ctx->io), len,
                                  static_cast<int32_t *>(ctx->io2), cap, &cnt, s);
    if (rc) return rc;
    const size_t got = cnt < cap ? cnt : cap;
    if (got) DSORT_HIP(ctx, hipMemcpyAsync(keys, ctx->io2, got * sizeof(int32_t), hipMemcpyDeviceToHost, s));
    DSORT_HIP(ctx, hipStreamSynchronize(s));
    *n_out = cnt;
    return DSORT_OK;
}

int dsort_format_text_i32(dsort_ctx *ctx, const int32_t *keys, size_t n, char *text, size_t cap,
                          size_t *len_out) {
    if (!ctx || !len_out || (n && (!keys || !text)))
        return set_err(ctx, DSORT_EINVAL, "null argument");
    *len_out = 0;
    if (!n) return DSORT_OK;
    int rc = ensure(ctx, &ctx->io, &ctx->io_bytes, n * sizeof(int32_t), "key staging");
    if (!rc) rc = ensure(ctx, &ctx->io2, &ctx->io2_bytes, 12 * n, "text staging");
    if (rc) return rc;
    hipStream_t s = ctx->stream;
    DSORT_HIP(ctx, hipMemcpyAsync(ctx->io, keys, n * sizeof(int32_t), hipMemcpyHostToDevice, s));
    size_t ln = 0;
    rc = dsort_format_text_dev_i32(ctx, static_cast<const int32_t *>(ctx->io), n,
                                   static_cast<char *>(ctx->io2), 12 * n, &ln, s);
    if (rc) return rc;
    if (ln > cap) return set_err(ctx, DSORT_EINVAL, "text buffer too small");
    DSORT_HIP(ctx, hipMemcpyAsync(text, ctx->io2, ln, hipMemcpyDeviceToHost, s));
    DSORT_HIP(ctx, hipStreamSynchronize(s));
    *len_out = ln;
    return DSORT_OK;
}

#ifdef DSORT_STAMPS
int dsort_debug_txstamps(void *host, size_t bytes) {
    return hipMemcpyFromSymbol(host, HIP_SYMBOL(tx::g_txstamps), bytes) == hipSuccess ? 0 : -1;
}
#endif

}  // extern "C"
