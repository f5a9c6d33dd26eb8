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
// Both are one pass over HBM: every workgroup takes the next tile (dynamic tile id), computes its
// byte (format) or token (parse) count, and gets its global offset from a decoupled look-back
// over the per-tile status words, then writes its output.  Format builds each tile's bytes in
// LDS at the same 16-byte phase as their global position and stores whole 16-byte chunks (byte
// stores only at the two partial ends).  Parse stages its tile (+ halo) in LDS with 16-byte
// loads and scans bytes from LDS.
//
// Algorithmic HBM bytes: format 4 B/key read + the text written; parse the text read + 4 B/key
// written.
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

constexpr uint64_t kAgg = 1ull << 62;    // status word: aggregate of this tile is published
constexpr uint64_t kIncl = 2ull << 62;   // status word: inclusive prefix is published
constexpr uint64_t kVal = kAgg - 1;

__device__ __forceinline__ int lane_id() { return threadIdx.x & 63; }

__device__ __forceinline__ uint64_t atomic_load_u64(const uint64_t *p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void atomic_store_u64(uint64_t *p, uint64_t v) {
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

__device__ __forceinline__ uint64_t wave_sum_u64(uint64_t v) {
    for (int o = 32; o >= 1; o >>= 1) v += __shfl_xor(v, o);
    return v;
}

// Decoupled look-back (wave 0 of a workgroup; all lanes return the same value): publishes the
// tile's aggregate, sums the predecessors' aggregates 64 tiles at a time back to the nearest
// published inclusive prefix, publishes its own inclusive prefix and returns the exclusive one.
// Termination: tile ids are handed out in workgroup start order, so every predecessor is running
// or done and publishes its aggregate without waiting on anyone.
__device__ uint64_t lookback(uint64_t *status, uint32_t id, uint64_t agg) {
    const int lane = lane_id();
    if (id == 0) {
        if (lane == 0) atomic_store_u64(&status[0], kIncl | agg);
        return 0;
    }
    if (lane == 0) atomic_store_u64(&status[id], kAgg | agg);
    uint64_t excl = 0;
    int64_t end = id;  // the window is tiles [end - 64, end), lane l at end - 1 - l
    while (true) {
        const int64_t j = end - 1 - lane;
        const uint64_t st = j >= 0 ? atomic_load_u64(&status[j]) : kIncl;  // before tile 0: 0
        const uint64_t flag = st >> 62;
        const unsigned long long incl = __ballot(flag == 2);
        const unsigned long long none = __ballot(flag == 0);
        const int fi = incl ? (int)__ffsll((long long)incl) - 1 : 64;  // nearest inclusive
        const unsigned long long need = fi == 64 ? ~0ull : ((2ull << fi) - 1);
        if (none & need) {
            __builtin_amdgcn_s_sleep(2);
            continue;
        }
        excl += wave_sum_u64(lane <= fi ? (st & kVal) : 0);
        if (fi < 64) break;
        end -= 64;
    }
    if (lane == 0) atomic_store_u64(&status[id], kIncl | (excl + agg));
    return excl;
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

// ---------------------------------------------------------------------------- format ------
__global__ void __launch_bounds__(NT) format_kernel(const int32_t *__restrict__ keys, uint64_t n,
                                                    char *__restrict__ text, uint64_t cap,
                                                    uint64_t *status, uint32_t *counter,
                                                    uint64_t *total, uint32_t ntiles) {
    __shared__ uint32_t sid;
    __shared__ uint32_t wsum[NT / 64];
    __shared__ uint64_t sbase;
    __shared__ __attribute__((aligned(16))) char sb[FBYTES + 32];
    if (threadIdx.x == 0) sid = atomicAdd(counter, 1u);
    __syncthreads();
    const uint32_t tile = sid;
    const uint64_t k0 = (uint64_t)tile * FTILE + (uint64_t)FK * threadIdx.x;
    int32_t v[FK];
    int len[FK];
    uint32_t tot = 0;
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
#pragma unroll
    for (int k = 0; k < FK; ++k) tot += len[k];
    uint32_t agg;
    const uint32_t toff = block_scan(tot, wsum, agg);
    if (threadIdx.x < 64) {
        const uint64_t ex = lookback(status, tile, agg);
        if (threadIdx.x == 0) sbase = ex;
    }
    __syncthreads();
    const uint64_t O = sbase;
    if (tile + 1 == ntiles && threadIdx.x == 0) *total = O + agg;
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
            *reinterpret_cast<int4 *>(ga + lo_b) = *reinterpret_cast<const int4 *>(sb + lo_b);
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

__global__ void __launch_bounds__(NT) parse_kernel(const char *__restrict__ text, uint64_t len,
                                                   int32_t *__restrict__ keys, uint64_t cap,
                                                   uint64_t *status, uint32_t *counter,
                                                   uint64_t *count, unsigned long long *err_pos,
                                                   uint32_t ntiles) {
    __shared__ uint32_t sid;
    __shared__ uint32_t wsum[NT / 64];
    __shared__ uint64_t sbase;
    __shared__ __attribute__((aligned(16))) uint32_t lw[PLDS / 4];
    if (threadIdx.x == 0) sid = atomicAdd(counter, 1u);
    __syncthreads();
    const uint32_t tile = sid;
    const uint64_t tb = (uint64_t)tile * PTILE;
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
    const unsigned char *lb = reinterpret_cast<const unsigned char *>(lw);
    const int my0 = 16 + PB * threadIdx.x;  // LDS index of this thread's first byte
    uint32_t w16[PB / 4];
#pragma unroll
    for (int i = 0; i < PB / 16; ++i) {
        const uint4 q = *reinterpret_cast<const uint4 *>(&lw[my0 / 4 + 4 * i]);
        w16[4 * i] = q.x; w16[4 * i + 1] = q.y; w16[4 * i + 2] = q.z; w16[4 * i + 3] = q.w;
    }
    // token starts: a non-whitespace byte after whitespace (or after the start of the text)
    uint64_t starts = 0;
    {
        bool prev_ws = is_ws(lb[my0 - 1]);
#pragma unroll
        for (int i = 0; i < PB; ++i) {
            const bool ws = is_ws((w16[i >> 2] >> (8 * (i & 3))) & 255u);
            if (!ws && prev_ws) starts |= 1ull << i;
            prev_ws = ws;
        }
    }
    uint32_t agg;
    const uint32_t toff = block_scan((uint32_t)__popcll(starts), wsum, agg);
    if (threadIdx.x < 64) {
        const uint64_t ex = lookback(status, tile, agg);
        if (threadIdx.x == 0) sbase = ex;
    }
    __syncthreads();
    uint64_t idx = sbase + toff;
    if (tile + 1 == ntiles && threadIdx.x == 0) *count = sbase + agg;
    while (starts) {
        const int i = __ffsll((long long)starts) - 1;
        starts &= starts - 1;
        int pos = my0 + i;
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
        if (nd == 0 || !is_ws(c)) atomicMin(err_pos, (unsigned long long)(tb + my0 - 16 + i));
        if (idx < cap) keys[idx] = (int32_t)(uint32_t)(neg ? 0ull - val : val);
        ++idx;
    }
}

}  // namespace tx

static int text_prepare(dsort_ctx *ctx, uint64_t ntiles, hipStream_t s) {
    int rc = ensure(ctx, &ctx->text_status, &ctx->text_status_bytes, ntiles * sizeof(uint64_t),
                    "text tile status");
    if (rc) return rc;
    DSORT_HIP(ctx, hipMemsetAsync(ctx->text_status, 0, ntiles * sizeof(uint64_t), s));
    // red[0]: tile counter (u32), red[1]: total bytes / tokens, red[2]: first error position
    DSORT_HIP(ctx, hipMemsetAsync(ctx->red, 0, 16, s));
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
    int rc = text_prepare(ctx, ntiles, s);
    if (rc) return rc;
    uint64_t *red = static_cast<uint64_t *>(ctx->red);
    hipLaunchKernelGGL(tx::format_kernel, dim3((unsigned)ntiles), dim3(tx::NT), 0, s, d_keys,
                       (uint64_t)n, d_text, (uint64_t)cap, static_cast<uint64_t *>(ctx->text_status),
                       reinterpret_cast<uint32_t *>(red), red + 1, (uint32_t)ntiles);
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
    int rc = text_prepare(ctx, ntiles, s);
    if (rc) return rc;
    uint64_t *red = static_cast<uint64_t *>(ctx->red);
    hipLaunchKernelGGL(tx::parse_kernel, dim3((unsigned)ntiles), dim3(tx::NT), 0, s, d_text,
                       (uint64_t)len, d_keys, (uint64_t)cap,
                       static_cast<uint64_t *>(ctx->text_status), reinterpret_cast<uint32_t *>(red),
                       red + 1, reinterpret_cast<unsigned long long *>(red + 2), (uint32_t)ntiles);
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

}  // extern "C"
