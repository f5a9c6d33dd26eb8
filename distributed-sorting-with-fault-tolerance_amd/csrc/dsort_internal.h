// dsort_internal.h -- private declarations shared by the libdsort translation units.
// gfx950 only (MI355X, CDNA4, wave64).  No CUDA shims, no dual platform paths.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stddef.h>

#include <string>

#include "dsort.h"

struct ncclComm;

namespace dsort {

// ----------------------------------------------------------------------------------------
// Geometry of the two hot kernels.  One workgroup owns one tile of TILE keys in LDS.
//   i32: 512 threads x 16 keys = 8192 keys = 32 KiB LDS per workgroup (4 workgroups / CU)
//   i64: 512 threads x  8 keys = 4096 keys = 32 KiB LDS per workgroup
// ----------------------------------------------------------------------------------------
template <typename T> struct Geom;
template <> struct Geom<int32_t> {
    static constexpr int THREADS = 512;
    static constexpr int K = 16;
    static constexpr int TILE = THREADS * K;
};
template <> struct Geom<int64_t> {
    static constexpr int THREADS = 512;
    static constexpr int K = 8;
    static constexpr int TILE = THREADS * K;
};

// One output tile of a 2-way merge pass: merge in[a_start, a_start+a_len) with
// in[b_start, b_start+b_len) into out[out_off, out_off + a_len + b_len).
struct Bucket2 {
    uint64_t out_off;
    uint64_t a_start;
    uint64_t b_start;
    uint32_t a_len;
    uint32_t b_len;
};

// A pair of adjacent runs to merge (irregular passes: user runs of arbitrary length).
struct Pair {
    uint64_t a_off;         // run A starts here; run B follows at a_off + a_len
    uint64_t a_len;
    uint64_t b_len;
    uint64_t first_bucket;  // global index of the pair's first output tile
};

}  // namespace dsort

// The context.  One per host thread, bound to one device.
struct dsort_ctx {
    int device = 0;
    hipStream_t stream = nullptr;
    std::string err;
    // grow-only device arenas
    void *scratch = nullptr;
    size_t scratch_bytes = 0;
    void *buckets = nullptr;
    size_t buckets_bytes = 0;
    void *pairs = nullptr;
    size_t pairs_bytes = 0;
    void *io = nullptr;        // staging for the host-buffer entry points
    size_t io_bytes = 0;
    void *io2 = nullptr;
    size_t io2_bytes = 0;
    void *red = nullptr;       // 64 B of reduction accumulators
    uint64_t *red_host = nullptr;  // pinned mirror
    // sample sort (multi-GPU)
    ncclComm *comm = nullptr;
    int nranks = 1;
    int rank = 0;
    void *local = nullptr;  // locally sorted chunk
    size_t local_bytes = 0;
    void *recv = nullptr;
    size_t recv_bytes = 0;
    void *recv2 = nullptr;
    size_t recv2_bytes = 0;
    void *small = nullptr;  // samples / splitters / counts on device
    size_t small_bytes = 0;
    void *small_host = nullptr;  // pinned
    size_t small_host_bytes = 0;
    // stage timing
    hipEvent_t ev[8] = {};
    unsigned ev_mask = 0;             // events recorded by the last call (bit i = ev[i])
    hipStream_t last_stream = nullptr;  // stream of the last asynchronous call
    static constexpr int kMaxKev = 128;  // per-launch events of the merge kernel (2 per pass)
    hipEvent_t kev[kMaxKev] = {};
    int kev_used = 0;
    bool ev_ok = false;
    dsort_stats stats = {};
};

namespace dsort {

int set_err(dsort_ctx *ctx, int code, const std::string &msg);
int hip_err(dsort_ctx *ctx, hipError_t e, const char *what);
int ensure(dsort_ctx *ctx, void **buf, size_t *have, size_t need, const char *what);

// Launchers (dsort_sort.hip).  All asynchronous on `s`.
// Sorts d_in[0..n) into d_keys (d_in may equal d_keys).
template <typename T>
int sort_device(dsort_ctx *ctx, const T *d_in, T *d_keys, size_t n, hipStream_t s, bool timed);
template <typename T>
int merge_device(dsort_ctx *ctx, const T *d_in, const size_t *lens, int k, T *d_out,
                 hipStream_t s);

}  // namespace dsort

#define DSORT_HIP(ctx, call)                                      \
    do {                                                          \
        hipError_t e_ = (call);                                   \
        if (e_ != hipSuccess) return dsort::hip_err((ctx), e_, #call); \
    } while (0)
