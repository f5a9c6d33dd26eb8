// dsort_api.hip -- the C ABI of libdsort (include/dsort.h): contexts, host-buffer entry points,
// device utilities (generators, parity checks), sample-sort planning and the multi-GPU sample
// sort over RCCL.
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <signal.h>
#include <stdint.h>
#include <stdio.h>
#include <string.h>
#include <time.h>
#include <unistd.h>

#include <algorithm>
#include <cmath>
#include <mutex>
#include <new>
#include <string>
#include <vector>

#include "dsort_internal.h"
#include "dsort_tx.h"

#define DSORT_VERSION_STRING "libdsort 0.1 (gfx950, HIP " DSORT_STR(HIP_VERSION_MAJOR) "." DSORT_STR(HIP_VERSION_MINOR) ")"
#define DSORT_STR2(x) #x
#define DSORT_STR(x) DSORT_STR2(x)

namespace dsort {

int set_err(dsort_ctx *ctx, int code, const std::string &msg) {
    if (ctx) ctx->err = msg;
    return code;
}

int hip_err(dsort_ctx *ctx, hipError_t e, const char *what) {
    std::string m = std::string(what) + ": " + hipGetErrorString(e);
    int code = (e == hipErrorOutOfMemory || e == hipErrorMemoryAllocation) ? DSORT_ENOMEM : DSORT_EHIP;
    return set_err(ctx, code, m);
}

int ensure(dsort_ctx *ctx, void **buf, size_t *have, size_t need, const char *what) {
    if (need <= *have && *buf) return DSORT_OK;
    if (*buf) {
        // the old arena may still be used by queued work on any stream of this device.  Inside the
        // bucket exchange's second level (ctx->poll_waits) the keys are still in flight on the comm
        // stream, which a dead peer never completes: a device-wide synchronize would hang there, so
        // wait for the streams that read the arenas (the sort's and the side stream) with polled
        // waits that see the abort flag and the deadline (the comm stream touches only the
        // partition and receive buffers, which never grow in that window)
        if (ctx->poll_waits) {
            int rc = sync_stream(ctx, ctx->poll_stream, "arena grow (sort stream)");
            if (!rc && ctx->side) rc = sync_stream(ctx, ctx->side, "arena grow (side stream)");
            if (rc) return rc;
        } else {
            hipError_t e = hipDeviceSynchronize();
            if (e != hipSuccess) return hip_err(ctx, e, "hipDeviceSynchronize (arena grow)");
        }
        release_dev(ctx, *buf);
        *buf = nullptr;
        *have = 0;
    }
    size_t sz = need < 256 ? 256 : need;
    hipError_t e = hipMalloc(buf, sz);
    if (e != hipSuccess) {
        *buf = nullptr;
        return set_err(ctx, DSORT_ENOMEM, std::string("hipMalloc failed for ") + what + " (" +
                                              std::to_string(sz) + " bytes): " + hipGetErrorString(e));
    }
    *have = sz;
    return DSORT_OK;
}

void release_dev(dsort_ctx *ctx, void *p) {
    if (!p) return;
    if (ctx->poll_waits) {
        ctx->dev_later.push_back(p);
        ++ctx->deferred_n;
    } else {
        (void)hipFree(p);
    }
}
void release_host(dsort_ctx *ctx, void *p) {
    if (!p) return;
    if (ctx->poll_waits) {
        ctx->host_later.push_back(p);
        ++ctx->deferred_n;
    } else {
        (void)hipHostFree(p);
    }
}
void flush_later(dsort_ctx *ctx) {
    for (void *p : ctx->dev_later) (void)hipFree(p);
    for (void *p : ctx->host_later) (void)hipHostFree(p);
    ctx->dev_later.clear();
    ctx->host_later.clear();
}

// grow-only pinned host buffer
static int ensure_host(dsort_ctx *ctx, void **buf, size_t *have, size_t need) {
    if (need <= *have && *buf) return DSORT_OK;
    if (*buf) release_host(ctx, *buf);
    *buf = nullptr;
    *have = 0;
    if (hipHostMalloc(buf, need, hipHostMallocDefault) != hipSuccess) {
        *buf = nullptr;
        return set_err(ctx, DSORT_ENOMEM, "hipHostMalloc failed (" + std::to_string(need) + " bytes)");
    }
    *have = need;
    return DSORT_OK;
}

hipStream_t pick_stream(dsort_ctx *ctx, void *stream) {
    if (stream == DSORT_NULL_STREAM) return static_cast<hipStream_t>(nullptr);
    return stream ? static_cast<hipStream_t>(stream) : ctx->stream;
}
static hipStream_t pick(dsort_ctx *ctx, void *stream) { return pick_stream(ctx, stream); }

// ------------------------------------------------------------------ utility kernels ------
__device__ __forceinline__ uint64_t splitmix64(uint64_t x) {
    x += 0x9E3779B97F4A7C15ull;
    x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
    x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
    return x ^ (x >> 31);
}

__global__ void gen_uniform_i32_kernel(int32_t *out, uint64_t n, uint64_t seed) {
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride)
        out[i] = (int32_t)(uint32_t)(splitmix64(seed + i) >> 32);
}

__global__ void gen_uniform_i64_kernel(int64_t *out, uint64_t n, uint64_t seed) {
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride)
        out[i] = (int64_t)splitmix64(seed + i);
}

// Truncated continuous power law over ranks [1, 2^24], exponent s = 1.2:
// rank = floor((1 + u*((2^24+1)^(1-s) - 1))^(1/(1-s))).  Heavy head (rank 1 ~ 13% of keys).
__global__ void gen_zipf_i64_kernel(int64_t *out, uint64_t n, uint64_t seed) {
    const double s = 1.2, nr = 16777216.0;
    const double e = 1.0 - s;
    const double top = pow(nr + 1.0, e) - 1.0;
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
        const double u = (double)(splitmix64(seed + i) >> 11) * 0x1.0p-53;
        double r = floor(pow(1.0 + u * top, 1.0 / e));
        if (r < 1.0) r = 1.0;
        if (r > nr) r = nr;
        out[i] = (int64_t)((uint64_t)r * 0x9E3779B97F4A7C15ull);
    }
}

template <typename T>
__global__ void __launch_bounds__(256) fingerprint_kernel(const T *keys, uint64_t n,
                                                          unsigned long long *acc) {
    uint64_t s = 0, x = 0;
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
        const uint64_t k = sizeof(T) == 4 ? (uint64_t)(uint32_t)keys[i] : (uint64_t)keys[i];
        s += splitmix64(k);
        x ^= splitmix64(k ^ 0xD1B54A32D192ED03ull);
    }
    __shared__ uint64_t ss[256], sx[256];
    ss[threadIdx.x] = s;
    sx[threadIdx.x] = x;
    __syncthreads();
    for (int w = 128; w > 0; w >>= 1) {
        if ((int)threadIdx.x < w) {
            ss[threadIdx.x] += ss[threadIdx.x + w];
            sx[threadIdx.x] ^= sx[threadIdx.x + w];
        }
        __syncthreads();
    }
    if (threadIdx.x == 0) {
        atomicAdd(&acc[0], (unsigned long long)ss[0]);
        atomicXor(&acc[1], (unsigned long long)sx[0]);
    }
}

template <typename T>
__global__ void __launch_bounds__(256) descents_kernel(const T *keys, uint64_t n,
                                                       unsigned long long *acc) {
    unsigned long long c = 0;
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x + 1; i < n; i += stride)
        c += keys[i - 1] > keys[i] ? 1 : 0;
    __shared__ unsigned long long sc[256];
    sc[threadIdx.x] = c;
    __syncthreads();
    for (int w = 128; w > 0; w >>= 1) {
        if ((int)threadIdx.x < w) sc[threadIdx.x] += sc[threadIdx.x + w];
        __syncthreads();
    }
    if (threadIdx.x == 0) atomicAdd(&acc[2], sc[0]);
}

// Regular samples of a sorted local run: sample j = keys[(j+1)*n/(s+1)].
template <typename T>
__global__ void sample_kernel(const T *keys, uint64_t n, int s, T *out) {
    const int j = blockIdx.x * blockDim.x + threadIdx.x;
    if (j >= s) return;
    if (n == 0) {
        out[j] = sizeof(T) == 4 ? (T)INT32_MAX : (T)INT64_MAX;
        return;
    }
    uint64_t idx = (uint64_t)(j + 1) * n / (uint64_t)(s + 1);
    if (idx >= n) idx = n - 1;
    out[j] = keys[idx];
}

// Composite-splitter cut positions in a sorted local run (same rule as dsort_plan_cuts_*):
// keys of this rank below splitter (v, r, i) in (value, rank, index) order.
template <typename T>
__global__ void cuts_kernel(const T *keys, uint64_t n, int my_rank, int nsplit, const T *sv,
                            const int32_t *sr, const uint64_t *si, uint64_t *cuts) {
    const int j = blockIdx.x * blockDim.x + threadIdx.x;
    if (j > nsplit) return;
    if (j == 0) {
        cuts[0] = 0;
        cuts[nsplit + 1] = n;
    }
    if (j == nsplit) return;
    const T v = sv[j];
    const int r = sr[j];
    uint64_t pos;
    if (r == my_rank) {
        pos = si[j] < n ? si[j] : n;
    } else {
        const bool upper = my_rank < r;  // equal keys of lower ranks go left
        uint64_t lo = 0, hi = n;
        while (lo < hi) {
            const uint64_t mid = (lo + hi) >> 1;
            const bool left = upper ? (keys[mid] <= v) : (keys[mid] < v);
            if (left) lo = mid + 1;
            else hi = mid;
        }
        pos = lo;
    }
    cuts[j + 1] = pos;
}

static unsigned grid_for(uint64_t n, int per_block) {
    uint64_t g = (n + per_block - 1) / per_block;
    if (g > 4096) g = 4096;
    if (g == 0) g = 1;
    return (unsigned)g;
}

template <typename T>
static int fingerprint_t(dsort_ctx *ctx, const T *d, size_t n, uint64_t *sum, uint64_t *xr,
                         uint64_t *desc, bool want_desc) {
    if (!ctx) return DSORT_EINVAL;
    hipStream_t s = ctx->stream;
    DSORT_HIP(ctx, hipMemsetAsync(ctx->red, 0, 64, s));
    if (n) {
        if (!want_desc)
            hipLaunchKernelGGL((fingerprint_kernel<T>), dim3(grid_for(n, 256 * 8)), dim3(256), 0, s,
                               d, (uint64_t)n, static_cast<unsigned long long *>(ctx->red));
        else
            hipLaunchKernelGGL((descents_kernel<T>), dim3(grid_for(n, 256 * 8)), dim3(256), 0, s, d,
                               (uint64_t)n, static_cast<unsigned long long *>(ctx->red));
        DSORT_HIP(ctx, hipGetLastError());
    }
    DSORT_HIP(ctx, hipMemcpyAsync(ctx->red_host, ctx->red, 64, hipMemcpyDeviceToHost, s));
    DSORT_HIP(ctx, hipStreamSynchronize(s));
    if (sum) *sum = ctx->red_host[0];
    if (xr) *xr = ctx->red_host[1];
    if (desc) *desc = ctx->red_host[2];
    return DSORT_OK;
}

// ------------------------------------------------------------------ host entry points ---
template <typename T>
static int sort_host(dsort_ctx *ctx, T *host, size_t n) {
    if (!ctx || (!host && n)) return set_err(ctx, DSORT_EINVAL, "null argument");
    if (n < 2) return DSORT_OK;
    int rc = ensure(ctx, &ctx->io, &ctx->io_bytes, n * sizeof(T), "staging");
    if (rc) return rc;
    hipStream_t s = ctx->stream;
    T *d = static_cast<T *>(ctx->io);
    DSORT_HIP(ctx, hipMemcpyAsync(d, host, n * sizeof(T), hipMemcpyHostToDevice, s));
    rc = sort_device<T>(ctx, d, d, n, s, true);
    if (rc) return rc;
    DSORT_HIP(ctx, hipMemcpyAsync(host, d, n * sizeof(T), hipMemcpyDeviceToHost, s));
    DSORT_HIP(ctx, hipStreamSynchronize(s));
    return DSORT_OK;
}

template <typename T>
static int merge_host(dsort_ctx *ctx, const T *const runs[], const size_t lens[], int k, T *out) {
    if (!ctx || k < 0 || (k > 0 && (!runs || !lens))) return set_err(ctx, DSORT_EINVAL, "bad argument");
    size_t n = 0;
    for (int j = 0; j < k; ++j) {
        if (lens[j] && !runs[j]) return set_err(ctx, DSORT_EINVAL, "null run");
        n += lens[j];
    }
    if (n == 0) return DSORT_OK;
    if (!out) return set_err(ctx, DSORT_EINVAL, "null output");
    int rc = ensure(ctx, &ctx->io, &ctx->io_bytes, n * sizeof(T), "staging");
    if (rc) return rc;
    rc = ensure(ctx, &ctx->io2, &ctx->io2_bytes, n * sizeof(T), "staging 2");
    if (rc) return rc;
    hipStream_t s = ctx->stream;
    T *din = static_cast<T *>(ctx->io), *dout = static_cast<T *>(ctx->io2);
    size_t off = 0;
    for (int j = 0; j < k; ++j) {
        if (lens[j])
            DSORT_HIP(ctx, hipMemcpyAsync(din + off, runs[j], lens[j] * sizeof(T),
                                          hipMemcpyHostToDevice, s));
        off += lens[j];
    }
    rc = merge_device<T>(ctx, din, lens, k, dout, s);
    if (rc) return rc;
    DSORT_HIP(ctx, hipMemcpyAsync(out, dout, n * sizeof(T), hipMemcpyDeviceToHost, s));
    DSORT_HIP(ctx, hipStreamSynchronize(s));
    return DSORT_OK;
}

// ------------------------------------------------------------------ planning (host) -----
template <typename T>
static int plan_splitters(int nranks, int s, const T *samples, const uint64_t *idx, T *sv,
                          int32_t *sr, uint64_t *si) {
    if (nranks < 1 || s < 1 || !samples || !idx) return DSORT_EINVAL;
    if (nranks == 1) return DSORT_OK;
    if (!sv || !sr || !si) return DSORT_EINVAL;
    struct S {
        T v;
        int32_t r;
        uint64_t i;
    };
    std::vector<S> all((size_t)nranks * s);
    for (int r = 0; r < nranks; ++r)
        for (int j = 0; j < s; ++j) all[(size_t)r * s + j] = S{samples[(size_t)r * s + j], r, idx[(size_t)r * s + j]};
    std::sort(all.begin(), all.end(), [](const S &a, const S &b) {
        if (a.v != b.v) return a.v < b.v;
        if (a.r != b.r) return a.r < b.r;
        return a.i < b.i;
    });
    // splitter q sits at the q-th P-quantile of the merged sample (PSRS with oversampling s)
    const size_t m = all.size();
    for (int q = 1; q < nranks; ++q) {
        size_t pos = (size_t)q * m / (size_t)nranks;
        if (pos >= m) pos = m - 1;
        sv[q - 1] = all[pos].v;
        sr[q - 1] = all[pos].r;
        si[q - 1] = all[pos].i;
    }
    return DSORT_OK;
}

template <typename T>
static int plan_cuts(const T *sorted, size_t n, int my_rank, int nranks, const T *sv,
                     const int32_t *sr, const uint64_t *si, uint64_t *cuts) {
    if (nranks < 1 || !cuts || (n && !sorted)) return DSORT_EINVAL;
    cuts[0] = 0;
    cuts[nranks] = n;
    for (int q = 0; q + 1 < nranks; ++q) {
        uint64_t pos;
        if (sr[q] == my_rank) {
            pos = si[q] < n ? si[q] : n;
        } else {
            const bool upper = my_rank < sr[q];
            const T *p = upper ? std::upper_bound(sorted, sorted + n, sv[q])
                               : std::lower_bound(sorted, sorted + n, sv[q]);
            pos = (uint64_t)(p - sorted);
        }
        cuts[q + 1] = pos;
    }
    return DSORT_OK;
}

// ------------------------------------------------------------------ sample sort ---------
static const int kSamplesPerRank = 512;

template <typename T> static ncclDataType_t nccl_type();
template <> ncclDataType_t nccl_type<int32_t>() { return ncclInt32; }
template <> ncclDataType_t nccl_type<int64_t>() { return ncclInt64; }


static double now_ms() {
    timespec ts;
    clock_gettime(CLOCK_MONOTONIC, &ts);
    return ts.tv_sec * 1e3 + ts.tv_nsec * 1e-6;
}

// The communicator mutex of a context: held by a running exchange or communicator set-up;
// dsort_comm_abort from another thread finds it taken and only raises ctx->abort_req (dsort.h).
static std::mutex &comm_mutex(dsort_ctx *ctx) { return ctx->comm_mu; }

static void abort_comm_locked(dsort_ctx *ctx) {
    if (ctx->comm) ncclCommAbort(ctx->comm);
    ctx->comm = nullptr;
    ctx->has_transport = false;
    ctx->nranks = 1;
    ctx->rank = 0;
}

// Every wait of an exchange: polls the stream, RCCL's asynchronous error (non-blocking
// communicator), the abort flag and the deadline, and aborts the communicator on a failure,
// instead of a hipStreamSynchronize that a dead peer would block forever.
// hold (DSORT_OPT_TEST_HOLD_EXCHANGE): the wait reports "not done" as if a peer never sent, until
// the abort flag or the deadline ends it.
static int exch_wait(dsort_ctx *ctx, hipStream_t s, bool with_stream, double deadline, const char *what,
                     bool hold = false) {
    PollPause pause;
    for (;;) {
        const hipError_t q0 = with_stream ? hipStreamQuery(s) : hipSuccess;
        const hipError_t q = hold && q0 == hipSuccess ? hipErrorNotReady : q0;
        ncclResult_t ae = ncclSuccess;
        if (ctx->comm) ncclCommGetAsyncError(ctx->comm, &ae);
        if (q == hipSuccess && ae != ncclInProgress && (ae == ncclSuccess || !ctx->comm)) return DSORT_OK;
        if (q != hipSuccess && q != hipErrorNotReady) return hip_err(ctx, q, what);
        if (ae != ncclSuccess && ae != ncclInProgress) {
            abort_comm_locked(ctx);
            return set_err(ctx, DSORT_ECOMM, std::string(what) + ": RCCL error " + ncclGetErrorString(ae) +
                                                 " (a peer failed); communicator aborted");
        }
        if (ctx->abort_req.load()) {
            abort_comm_locked(ctx);
            return set_err(ctx, DSORT_ECOMM, std::string(what) + ": aborted by dsort_comm_abort");
        }
        if (deadline > 0 && now_ms() > deadline) {
            abort_comm_locked(ctx);
            return set_err(ctx, DSORT_ETIMEOUT, std::string(what) + ": no progress before the deadline "
                                                    "(DSORT_OPT_COMM_TIMEOUT_MS); communicator aborted");
        }
        pause();  // (a wait on the critical path of every exchange step)
    }
}

// An RCCL call on the non-blocking communicator: ncclInProgress is success-so-far.
#define DSORT_NCCLNB(ctx, call)                                                           \
    do {                                                                                  \
        ncclResult_t r_ = (call);                                                         \
        if (r_ != ncclSuccess && r_ != ncclInProgress) {                                  \
            abort_comm_locked(ctx);                                                       \
            return dsort::set_err((ctx), DSORT_ECOMM,                                     \
                                  std::string(#call) + ": " + ncclGetErrorString(r_));    \
        }                                                                                 \
    } while (0)

static void exchange_fault_point(dsort_ctx *ctx, int stage) {
    if (ctx->opt.kill_in_exchange == stage) raise(SIGKILL);
}

// DSORT_OPT_TEST_FAIL_EXCHANGE = k (host transport): a local error of this rank right before its
// k-th collective (0 = the key-count all-gather), returned like any other local error -- the
// sequence's guard reports it to the peers at the next gate (dsort_tx.h)
static int tx_fault_point(dsort_ctx *ctx) {
    if (ctx->tx && ctx->opt.test_fail_exchange >= 0 && ctx->opt.test_fail_exchange == ctx->tx->collectives_done())
        return set_err(ctx, DSORT_EHIP, "injected local failure before collective " +
                                            std::to_string(ctx->opt.test_fail_exchange) +
                                            " of the exchange (DSORT_OPT_TEST_FAIL_EXCHANGE)");
    return DSORT_OK;
}

// All-gather of `count` uint64 per rank (RCCL through the context's small device buffer, or the
// host transport): out[r * count + i] = rank r's src[i].
static int allgather_u64(dsort_ctx *ctx, const uint64_t *src, size_t count, uint64_t *out, hipStream_t s,
                         double deadline, const char *what) {
    const int P = ctx->nranks;
    if (ctx->has_transport) {
        if (!ctx->tx) return set_err(ctx, DSORT_EINVAL, std::string(what) + ": no sample sort running");
        if (int rc_ = tx_fault_point(ctx)) return rc_;
        const int rc = ctx->tx->allgather(src, out, count * 8, what);
        return rc ? set_err(ctx, rc, ctx->tx->error()) : DSORT_OK;
    }
    const size_t bytes = count * 8 * (size_t)(P + 1);
    int rc = ensure(ctx, &ctx->small, &ctx->small_bytes, bytes, "sample-sort small buffers");
    if (rc) return rc;
    if (ctx->small_host_bytes < bytes) {
        if (ctx->small_host) (void)hipHostFree(ctx->small_host);
        ctx->small_host = nullptr;
        ctx->small_host_bytes = 0;
        DSORT_HIP(ctx, hipHostMalloc(&ctx->small_host, bytes, hipHostMallocDefault));
        ctx->small_host_bytes = bytes;
    }
    uint64_t *d = static_cast<uint64_t *>(ctx->small), *h = static_cast<uint64_t *>(ctx->small_host);
    memcpy(h, src, count * 8);
    DSORT_HIP(ctx, hipMemcpyAsync(d, h, count * 8, hipMemcpyHostToDevice, s));
    DSORT_NCCLNB(ctx, ncclAllGather(d, d + count, count, ncclUint64, ctx->comm, s));
    rc = exch_wait(ctx, s, false, deadline, what);
    if (rc) return rc;
    DSORT_HIP(ctx, hipMemcpyAsync(h + count, d + count, count * 8 * (size_t)P, hipMemcpyDeviceToHost, s));
    rc = exch_wait(ctx, s, true, deadline, what);
    if (rc) return rc;
    memcpy(out, h + count, count * 8 * (size_t)P);
    return DSORT_OK;
}

// The context's comm stream (the bucket exchange's sends and receives) and its events.
static int comm_stream(dsort_ctx *ctx) {
    // (the highest priority: a hardware queue of its own -- a stream created after the sort's may
    // share its queue, and then nothing on it runs beside the sort's kernels)
    int lo = 0, hi = 0;
    if (!ctx->xs && (hipDeviceGetStreamPriorityRange(&lo, &hi) != hipSuccess ||
                     hipStreamCreateWithPriority(&ctx->xs, hipStreamNonBlocking, hi) != hipSuccess))
        return set_err(ctx, DSORT_EHIP, "hipStreamCreate (comm stream)");
    for (auto &e : ctx->xev)
        if (!e && hipEventCreateWithFlags(&e, hipEventDisableTiming) != hipSuccess)
            return set_err(ctx, DSORT_EHIP, "hipEventCreate (comm stream)");
    return DSORT_OK;
}

// DSORT_OPT_TEST_WAVE_FENCE (test only): fingerprints (fingerprint_kernel: sum and xor of
// splitmix64, order independent) of device ranges taken on the sort stream before and after a step
// of the exchange; any range that changed fails the sort with DSORT_EHIP naming it.  Value 2 tests
// the fence itself: one key of the first range is flipped between the two prints.
template <typename T>
__global__ void fence_poke_kernel(T *p) {
    p[0] ^= (T)1;
}

template <typename T>
struct WaveFence {
    struct R {
        const T *p;
        uint64_t n;
        std::string what;
    };
    std::vector<R> r;
    bool on() const { return !r.empty(); }
    void add(const T *p, uint64_t n, std::string what) {
        if (n) r.push_back(R{p, n, std::move(what)});
    }
    int prepare(dsort_ctx *ctx) {
        if (r.empty()) return DSORT_OK;
        const size_t bytes = r.size() * 4 * sizeof(unsigned long long);
        int rc = ensure(ctx, &ctx->fence, &ctx->fence_bytes, bytes, "wave fence");
        return rc ? rc : ensure_host(ctx, &ctx->fence_host, &ctx->fence_host_bytes, bytes);
    }
    // which = 0: before, 1: after
    int print(dsort_ctx *ctx, hipStream_t s, int which) {
        auto *acc = static_cast<unsigned long long *>(ctx->fence) + (size_t)which * 2 * r.size();
        DSORT_HIP(ctx, hipMemsetAsync(acc, 0, r.size() * 2 * sizeof(unsigned long long), s));
        for (size_t i = 0; i < r.size(); ++i) {
            hipLaunchKernelGGL((fingerprint_kernel<T>), dim3(grid_for(r[i].n, 256 * 8)), dim3(256), 0, s, r[i].p,
                               r[i].n, acc + 2 * i);
            DSORT_HIP(ctx, hipGetLastError());
        }
        return DSORT_OK;
    }
    int check(dsort_ctx *ctx, hipStream_t s, double deadline) {
        if (ctx->opt.test_wave_fence == 2) {
            hipLaunchKernelGGL((fence_poke_kernel<T>), dim3(1), dim3(1), 0, s, const_cast<T *>(r[0].p));
            DSORT_HIP(ctx, hipGetLastError());
        }
        int rc = print(ctx, s, 1);
        if (rc) return rc;
        const size_t m = r.size() * 4;
        DSORT_HIP(ctx, hipMemcpyAsync(ctx->fence_host, ctx->fence, m * sizeof(unsigned long long),
                                      hipMemcpyDeviceToHost, s));
        if ((rc = exch_wait(ctx, s, true, deadline, "wave fence"))) return rc;
        const auto *h = static_cast<const unsigned long long *>(ctx->fence_host);
        const size_t R2 = 2 * r.size();
        for (size_t i = 0; i < r.size(); ++i)
            if (h[2 * i] != h[R2 + 2 * i] || h[2 * i + 1] != h[R2 + 2 * i + 1])
                return set_err(ctx, DSORT_EHIP, "DSORT_OPT_TEST_WAVE_FENCE: wave 0's second level / tile sort changed " +
                                                    r[i].what + " (" + std::to_string(r[i].n) + " keys)");
        ctx->stats.fence_ranges += (int)r.size();
        return DSORT_OK;
    }
};

// The bucket exchange (dsort_internal.h): samples of the unsorted keys from every
// rank -> the same Btot global splitters everywhere -> this rank's keys partitioned into the Btot
// buckets (the first level of the one-GPU sort) -> buckets [q Bl, (q+1) Bl) to rank q (RCCL
// grouped send/recv over xGMI) -> the received pieces of this rank's Bl buckets finished by the
// second level and the tile sort.  Replaces the gather + merge_chunks of server.c:414-415 and
// 500-515: nothing is merged.
template <typename T>
static int sample_sort_bx(dsort_ctx *ctx, const T *d_in, const BxPlan &pl, T **d_out, size_t *n_out, hipStream_t s,
                          double deadline) {
    const int P = pl.P, me = pl.me, Bl = pl.Bl, Bt = pl.Btot;
    const bool host_tx = ctx->has_transport;
    // The exchange in W waves of this rank's buckets (two or more buckets: W = 2), see step 4
    const int W = Bl >= 2 ? 2 : 1;
    if (host_tx) ctx->tx->plan(2 + W);  // samples, bucket starts, the waves (dsort_tx.h)
    const size_t rec = (size_t)pl.s_max * sizeof(BxSample);
    int rc = ensure(ctx, &ctx->bxs, &ctx->bxs_bytes, rec * (size_t)(P + 1), "bucket-exchange samples");
    if (rc) return rc;
    BxSample *mine = static_cast<BxSample *>(ctx->bxs), *all = mine + pl.s_max;
    // 1. samples, all-gathered
    if ((rc = bx_sample<T>(ctx, d_in, pl, mine, s))) return rc;
    if (!host_tx) {
        DSORT_NCCLNB(ctx, ncclAllGather(mine, all, (size_t)pl.s_max * 2, ncclInt64, ctx->comm, s));
        rc = exch_wait(ctx, s, false, deadline, "sample all-gather (enqueue)");
        if (rc) return rc;
    } else {
        rc = ensure_host(ctx, &ctx->xfer, &ctx->xfer_bytes, rec * (size_t)(P + 1));
        if (rc) return rc;
        char *hm = static_cast<char *>(ctx->xfer), *ha = hm + rec;
        DSORT_HIP(ctx, hipMemcpyAsync(hm, mine, rec, hipMemcpyDeviceToHost, s));
        rc = exch_wait(ctx, s, true, deadline, "samples");
        if (rc) return rc;
        if ((rc = tx_fault_point(ctx))) return rc;
        if ((rc = ctx->tx->allgather(hm, ha, rec, "samples all-gather"))) return set_err(ctx, rc, ctx->tx->error());
        DSORT_HIP(ctx, hipMemcpyAsync(all, ha, rec * (size_t)P, hipMemcpyHostToDevice, s));
    }
    exchange_fault_point(ctx, 1);
    // 2. global splitters and this rank's first partition level (the host waits for the bucket
    //    starts while the scatter runs); kill stage 0
    const uint64_t *hb;
    T *part;
    std::vector<uint8_t> pure;
    rc = bx_partition<T>(ctx, d_in, pl, all, s, true, &hb, &part, pure);
    if (rc) return rc;
    // 3. every rank's bucket starts, on the comm stream: they are on the host before the scatter
    //    ends, so the all-gather, the exchange's enqueue and the first wave's tables overlap it (on
    //    the sort stream they queued behind it: about 0.14 ms of idle GPU per 2^27-key rank)
    if (!host_tx && (rc = comm_stream(ctx))) return rc;
    std::vector<uint64_t> hb_all((size_t)P * (Bt + 1));
    {
        const std::vector<uint64_t> mine_hb(hb, hb + Bt + 1);
        rc = allgather_u64(ctx, mine_hb.data(), (size_t)Bt + 1, hb_all.data(), host_tx ? s : ctx->xs, deadline,
                           "bucket starts all-gather");
        if (rc) return rc;
    }
    // The exchange in W waves of this rank's buckets (two or more buckets: W = 2): wave w ships
    // buckets [jb[w], jb[w+1]) of every rank's range, and over RCCL the second level of wave 0 runs
    // while wave 1's keys are on the links (the sends and receives go on the comm stream; the sort
    // stream waits for each wave's event).  (The host transport and a single rank run the same waves
    // one after the other: the same layout and second-level calls as the 8-GPU run.)
    const int jb[3] = {0, W == 2 ? Bl / 2 : Bl, Bl};
    // Positions in `part` and in the receive buffer follow every rank's compacted starts (a pure
    // bucket -- its keys dropped by the scatter, bx_partition -- of size 0); the output sizes follow
    // the real starts.
    std::vector<uint64_t> hc_all(hb_all.size());
    for (int r = 0; r < P; ++r) {
        const uint64_t *h = hb_all.data() + (size_t)r * (Bt + 1);
        uint64_t *c = hc_all.data() + (size_t)r * (Bt + 1), run = 0;
        for (int g = 0; g <= Bt; ++g) {
            c[g] = run;
            if (g < Bt && !pure[(size_t)g]) run += h[g + 1] - h[g];
        }
    }
    const uint64_t *hme = hc_all.data() + (size_t)me * (Bt + 1);
    auto hof = [&](int r) { return hc_all.data() + (size_t)r * (Bt + 1); };
    std::vector<uint64_t> rlen(P, 0);
    uint64_t sent = 0, nout = 0;
    for (int q = 0; q < P; ++q) {
        rlen[q] = hof(q)[(size_t)(me + 1) * Bl] - hof(q)[(size_t)me * Bl];
        if (q != me) sent += hme[(size_t)(q + 1) * Bl] - hme[(size_t)q * Bl];
        const uint64_t *h = hb_all.data() + (size_t)q * (Bt + 1);
        nout += h[(size_t)(me + 1) * Bl] - h[(size_t)me * Bl];
    }
    uint64_t nrecv = 0;  // (keys received: the compacted sizes)
    for (int q = 0; q < P; ++q) nrecv += rlen[q];
    // The other ranks' pieces land behind this rank's partitioned keys when they fit (its own buckets
    // are then read in place: no copy); else everything goes to a receive buffer.
    const bool behind = nrecv - rlen[me] <= pl.recv_room;
    // per wave and source: where its pieces land (rpos) and the source position of its first key of
    // the wave's first bucket (base)
    std::vector<uint64_t> rpos((size_t)W * P), base((size_t)W * P), rcnt((size_t)W * P);
    {
        uint64_t o = behind ? pl.n_local : 0;
        for (int w = 0; w < W; ++w)
            for (int q = 0; q < P; ++q) {
                const size_t k = (size_t)w * P + q;
                rcnt[k] = hof(q)[(size_t)me * Bl + jb[w + 1]] - hof(q)[(size_t)me * Bl + jb[w]];
                if (behind && q == me) {
                    base[k] = hme[(size_t)me * Bl + jb[w]];
                    rpos[k] = 0;
                    continue;
                }
                base[k] = rpos[k] = o;
                o += rcnt[k];
            }
    }
    if (!behind) {
        rc = ensure(ctx, &ctx->recv, &ctx->recv_bytes, (nrecv ? nrecv : 1) * sizeof(T) + 16, "receive buffer");
        if (rc) return rc;
    }
    rc = ensure(ctx, &ctx->recv2, &ctx->recv2_bytes, (nout ? nout : 1) * sizeof(T), "sorted slice");
    if (rc) return rc;
    T *rb = behind ? part : static_cast<T *>(ctx->recv);  // (the second level's source)
    exchange_fault_point(ctx, 2);
    // DSORT_OPT_TEST_WAVE_FENCE: what wave 1 still needs while wave 0's second level and tile sort
    // run -- its sends (part, every q != me), this rank's own wave-1 buckets (read in place when
    // `behind`) and its landing zone -- fingerprinted before and after wave 0 (dsort.h).  Set up before anything is
    // enqueued on the comm stream (the arena may grow)
    WaveFence<T> fence;
    if (ctx->opt.test_wave_fence && W == 2) {
        const int w = 1;
        for (int q = 0; q < P; ++q) {
            const uint64_t so = hme[(size_t)q * Bl + jb[w]], sn = hme[(size_t)q * Bl + jb[w + 1]] - so;
            fence.add(part + so, sn, q != me ? "wave-1 send range of part to rank " + std::to_string(q)
                                             : std::string("this rank's own wave-1 buckets in part"));
            const size_t k = (size_t)w * P + q;
            // (over RCCL with peers the landing zone fills while wave 0 runs: not fenced there)
            if (!(behind && q == me) && (host_tx || P == 1))
                fence.add(rb + rpos[k], rcnt[k], "wave-1 landing zone of the keys from rank " + std::to_string(q));
        }
        if ((rc = fence.prepare(ctx))) return rc;
    }
    // 4. the buckets to their ranks: per wave one send and one receive per peer (all-to-all-v over
    //    xGMI), on the comm stream after the partition
    if (ctx->ev_ok) {
        DSORT_HIP(ctx, hipEventRecord(ctx->ev[5], s));
        ctx->ev_mask |= 32u;
    }
    hipStream_t cs = s;
    if (!host_tx) {
        cs = ctx->xs;
        DSORT_HIP(ctx, hipEventRecord(ctx->xev[2], s));
        DSORT_HIP(ctx, hipStreamWaitEvent(cs, ctx->xev[2], 0));
        for (int w = 0; w < W; ++w) {
            DSORT_NCCLNB(ctx, ncclGroupStart());
            for (int q = 0; q < P; ++q) {
                if (q == me) continue;
                const uint64_t so = hme[(size_t)q * Bl + jb[w]], sn = hme[(size_t)q * Bl + jb[w + 1]] - so;
                const size_t k = (size_t)w * P + q;
                if (sn) DSORT_NCCLNB(ctx, ncclSend(part + so, sn, nccl_type<T>(), q, ctx->comm, cs));
                if (rcnt[k]) DSORT_NCCLNB(ctx, ncclRecv(rb + rpos[k], rcnt[k], nccl_type<T>(), q, ctx->comm, cs));
            }
            DSORT_NCCLNB(ctx, ncclGroupEnd());
            // (a non-blocking communicator may still be enqueueing the group: the wave's event
            // goes on the stream behind its kernels)
            rc = exch_wait(ctx, cs, false, deadline, "key all-to-all (enqueue)");
            if (rc) return rc;
            const size_t km = (size_t)w * P + me;
            if (!behind && rcnt[km])
                DSORT_HIP(ctx, hipMemcpyAsync(rb + rpos[km], part + hme[(size_t)me * Bl + jb[w]], rcnt[km] * sizeof(T),
                                              hipMemcpyDeviceToDevice, cs));
            DSORT_HIP(ctx, hipEventRecord(ctx->xev[w], cs));
        }
    }
    if (host_tx) {
        // The same order as RCCL's: wave w's send ranges are staged from `part` right
        // before its all-to-all, and wave w's second level and tile sort are queued before wave
        // w+1 is staged -- so wave 1's sends are read from `part` after wave 0's kernels ran on it,
        // as the 8-GPU run reads them while those kernels run.  The host buffer mirrors `part`
        // (send displacements = positions in part); the receive layout is the device one minus
        // the partition (behind: the other sources from n_local on, this rank's own buckets not
        // shipped).
        rc = ensure_host(ctx, &ctx->xfer, &ctx->xfer_bytes, (pl.n_local ? pl.n_local : 1) * sizeof(T));
        if (rc) return rc;
        rc = ensure_host(ctx, &ctx->xfer2, &ctx->xfer2_bytes, (nrecv ? nrecv : 1) * sizeof(T));
        if (rc) return rc;
        const uint64_t shift = behind ? pl.n_local : 0;
        T *outp = static_cast<T *>(ctx->recv2);
        uint64_t out_off = 0;
        for (int w = 0; w < W; ++w) {
            std::vector<size_t> sc(P), sd(P), rcn(P), rd(P);
            uint64_t lo = ~0ull, hi = 0;
            for (int q = 0; q < P; ++q) {
                const size_t k = (size_t)w * P + q;
                const bool self = behind && q == me;
                const uint64_t so = hme[(size_t)q * Bl + jb[w]];
                sd[q] = so * sizeof(T);
                sc[q] = self ? 0 : (hme[(size_t)q * Bl + jb[w + 1]] - so) * sizeof(T);
                rcn[q] = self ? 0 : rcnt[k] * sizeof(T);
                rd[q] = self ? 0 : (rpos[k] - shift) * sizeof(T);
                if (sc[q])  // (stage this wave's range for q, and nothing else)
                    DSORT_HIP(ctx, hipMemcpyAsync(static_cast<char *>(ctx->xfer) + sd[q], part + so, sc[q],
                                                  hipMemcpyDeviceToHost, s));
                if (!self && rcnt[k]) {
                    lo = std::min<uint64_t>(lo, rpos[k]);
                    hi = std::max<uint64_t>(hi, rpos[k] + rcnt[k]);
                }
            }
            rc = exch_wait(ctx, s, true, deadline, w ? "key staging (wave 1)" : "key staging (wave 0)");
            if (rc) return rc;
            if ((rc = tx_fault_point(ctx))) return rc;
            if ((rc = ctx->tx->alltoallv(ctx->xfer, sc.data(), sd.data(), ctx->xfer2, rcn.data(), rd.data(),
                                         w ? "key all-to-all (wave 1)" : "key all-to-all (wave 0)")))
                return set_err(ctx, rc, ctx->tx->error());
            if (hi > lo)
                DSORT_HIP(ctx, hipMemcpyAsync(rb + lo, static_cast<char *>(ctx->xfer2) + (lo - shift) * sizeof(T),
                                              (hi - lo) * sizeof(T), hipMemcpyHostToDevice, s));
            if (w == 0 && ctx->ev_ok) {
                DSORT_HIP(ctx, hipEventRecord(ctx->ev[6], s));  // (the first wave's keys in)
                DSORT_HIP(ctx, hipEventRecord(ctx->ev[3], s));
                ctx->ev_mask |= 64u | 8u;
            }
            if (w == 0 && fence.on() && (rc = fence.print(ctx, s, 0))) return rc;
            uint64_t nw = 0;
            rc = bx_local_sort<T>(ctx, rb, outp, pl, hb_all.data(), hc_all.data(), base.data() + (size_t)w * P, jb[w], jb[w + 1],
                                  out_off, w, W, s, true, &nw);
            if (rc) return rc;
            out_off += nw;
            if (w == 0 && fence.on() && (rc = fence.check(ctx, s, deadline))) return rc;
        }
        flush_later(ctx);
        ctx->last_stream = s;
        ctx->stats.keys_in = pl.n_local;
        ctx->stats.keys_out = nout;
        ctx->stats.keys_sent = sent;
        ctx->stats.exchange_path = 1;
        *d_out = outp;
        *n_out = nout;
        return DSORT_OK;
    }
    // 5. the second level and the tile sort of this rank's buckets, wave by wave, each queued behind
    //    its receives while later waves are in flight (the host builds and uploads a wave's tables
    //    meanwhile); the host waits inside poll the abort flag and the deadline, as a dead peer never
    //    completes the stream.  Kill stages 1 and 2 (after the first wave's).
    T *outp = static_cast<T *>(ctx->recv2);
    ctx->poll_waits = true;
    ctx->poll_deadline = deadline;
    ctx->poll_stream = s;
    uint64_t out_off = 0;
    for (int w = 0; w < W && !rc; ++w) {
        DSORT_HIP(ctx, hipStreamWaitEvent(s, ctx->xev[w], 0));
        if (w == 0 && ctx->ev_ok) {
            DSORT_HIP(ctx, hipEventRecord(ctx->ev[6], s));  // (the first wave's keys in)
            DSORT_HIP(ctx, hipEventRecord(ctx->ev[3], s));
            ctx->ev_mask |= 64u | 8u;
        }
        if (w == 0 && fence.on()) rc = fence.print(ctx, s, 0);
        uint64_t nw = 0;
        if (!rc)
            rc = bx_local_sort<T>(ctx, rb, outp, pl, hb_all.data(), hc_all.data(), base.data() + (size_t)w * P, jb[w], jb[w + 1],
                                  out_off, w, W, s, true, &nw);
        out_off += nw;
        if (!rc && w == 0 && fence.on()) rc = fence.check(ctx, s, deadline);
    }
    ctx->poll_waits = false;
    if (rc) {
        // The arenas the second level replaced while the keys were in flight (release_dev) are
        // freed once no kernel can touch them (a faulted sort kept its multi-GB scratch
        // until the next good exchange, so the recovery ran at twice the footprint).  After a
        // communicator failure the abort ends the comm stream's kernels; after a local failure
        // every send and receive was enqueued and still completes: wait for it, bounded by the
        // deadline and the abort flag (a failing wait aborts the communicator).
        if (rc == DSORT_ECOMM || rc == DSORT_ETIMEOUT) {
            abort_comm_locked(ctx);
        } else {
            const std::string err = ctx->err;
            (void)exch_wait(ctx, cs, true, deadline, "key all-to-all (after a local failure)");
            ctx->err = err;
        }
        if (hipStreamSynchronize(s) == hipSuccess) flush_later(ctx);
        return rc;
    }
    // the receives have landed (and the test hold, DSORT_OPT_TEST_HOLD_EXCHANGE, is released)
    rc = exch_wait(ctx, cs, true, deadline, "key all-to-all", ctx->opt.test_hold_exchange != 0);
    if (rc) {
        // (a failed final wait has aborted the communicator, or met a HIP error: the arenas the
        // second level replaced go once the sort stream is idle, as on the failures above --
        // tests/test_gpu_faults.py::test_faulted_exchanges_release_replaced_arenas)
        if (hipStreamSynchronize(s) == hipSuccess) flush_later(ctx);
        return rc;
    }
    flush_later(ctx);  // (the buffers the second level replaced while the keys were in flight)
    ctx->last_stream = s;
    ctx->stats.keys_in = pl.n_local;
    ctx->stats.keys_out = nout;
    ctx->stats.keys_sent = sent;
    ctx->stats.exchange_path = 1;
    *d_out = outp;
    *n_out = nout;
    return DSORT_OK;
}

template <typename T>
static int sample_sort(dsort_ctx *ctx, const T *d_in, size_t n_local, T **d_out, size_t *n_out,
                       void *stream, bool presorted) {
    if (!ctx || !d_out || !n_out || (n_local && !d_in)) return set_err(ctx, DSORT_EINVAL, "null argument");
    std::unique_lock<std::mutex> lock(comm_mutex(ctx));
    if (ctx->abort_req.load()) {
        abort_comm_locked(ctx);
        return set_err(ctx, DSORT_ECOMM, "communicator aborted (dsort_comm_abort)");
    }
    if (!ctx->comm && !ctx->has_transport)
        return set_err(ctx, DSORT_ECOMM, "communicator not initialised (dsort_comm_init)");
    hipStream_t s = pick(ctx, stream);
    const double deadline = ctx->opt.comm_timeout_ms > 0 ? now_ms() + (double)ctx->opt.comm_timeout_ms : 0.0;
    const int P = ctx->nranks, me = ctx->rank, S = kSamplesPerRank;
    const bool host_tx = ctx->has_transport;
    int rc;
    // host transport: the sequence of collectives with its gates (dsort_tx.h); leaving this call
    // before the last collective on any error reports the failure to the peers at the next gate
    // (the guard), so none of them blocks in a collective this rank never joins.  The first
    // collective is the key-count all-gather (the presorted entry starts with the samples).
    TxSeq txs(ctx->transport, P, deadline, presorted ? 3 : 1);
    struct TxScope {
        dsort_ctx *c;
        ~TxScope() { c->tx = nullptr; }
    } tx_scope{ctx};
    TxGuard tx_guard;
    if (host_tx) {
        ctx->tx = &txs;
        tx_guard.seq = &txs;
    }
    if (!presorted) {
        // every rank's key count decides the path, the same on every rank: the bucket exchange, or
        // (small inputs, partition switched off) sort locally and merge the received runs
        std::vector<uint64_t> n_of(P);
        const uint64_t nl = n_local;
        rc = allgather_u64(ctx, &nl, 1, n_of.data(), s, deadline, "key count all-gather");
        if (rc) return rc;
        BxPlan pl;
        if (bx_make_plan(ctx->opt, P, me, n_of.data(), (int)sizeof(T), pl)) {
            ctx->stats = fresh_stats();
            return sample_sort_bx<T>(ctx, d_in, pl, d_out, n_out, s, deadline);
        }
        if (host_tx) txs.plan(3);  // samples, count matrix, keys
    }
    const T *d_keys;
    dsort_stats st = fresh_stats();
    if (presorted) {
        // the caller already holds a sorted local run (fault recovery: a survivor merged the
        // chunks it sorted)
        d_keys = d_in;
        ctx->ev_mask = 0;
        ctx->last_stream = s;
        if (ctx->ev_ok) {
            for (int e = 0; e < 3; ++e) DSORT_HIP(ctx, hipEventRecord(ctx->ev[e], s));
            ctx->ev_mask = 7u;
        }
        st.keys_in = n_local;
    } else {
        // 1. local sort (the worker's merge_sort) into the context's local arena
        rc = ensure(ctx, &ctx->local, &ctx->local_bytes, (n_local ? n_local : 1) * sizeof(T), "local run");
        if (rc) return rc;
        T *dk = static_cast<T *>(ctx->local);
        rc = sort_device<T>(ctx, d_in, dk, n_local, s, true);
        if (rc) return rc;
        d_keys = dk;
        st = ctx->stats;
    }
    // device small-area layout
    const size_t off_samp = 0;                                   // S keys
    const size_t off_all = off_samp + (size_t)S * sizeof(T);      // P*S keys
    const size_t off_n = off_all + (size_t)P * S * sizeof(T);     // P uint64 (n_local of all)
    const size_t off_sv = off_n + (size_t)P * 8;                  // P keys (splitter values)
    const size_t off_sr = off_sv + (size_t)P * sizeof(T);         // P int32
    const size_t off_si = off_sr + (size_t)P * 8;                 // P uint64
    const size_t off_cut = off_si + (size_t)P * 8;                // P+1 uint64
    const size_t off_cnt = off_cut + (size_t)(P + 1) * 8;         // P uint64 (send counts)
    const size_t off_mat = off_cnt + (size_t)P * 8;               // P*P uint64
    const size_t total_small = off_mat + (size_t)P * P * 8 + 64;
    rc = ensure(ctx, &ctx->small, &ctx->small_bytes, total_small, "sample-sort small buffers");
    if (rc) return rc;
    if (ctx->small_host_bytes < total_small) {
        if (ctx->small_host) (void)hipHostFree(ctx->small_host);
        ctx->small_host = nullptr;
        ctx->small_host_bytes = 0;
        DSORT_HIP(ctx, hipHostMalloc(&ctx->small_host, total_small, hipHostMallocDefault));
        ctx->small_host_bytes = total_small;
    }
    char *dsm = static_cast<char *>(ctx->small);
    char *hsm = static_cast<char *>(ctx->small_host);
    // 2. regular samples + local size
    hipLaunchKernelGGL((sample_kernel<T>), dim3((S + 255) / 256), dim3(256), 0, s, d_keys,
                       (uint64_t)n_local, S, reinterpret_cast<T *>(dsm + off_samp));
    DSORT_HIP(ctx, hipGetLastError());
    uint64_t nl = n_local;
    DSORT_HIP(ctx, hipMemcpyAsync(dsm + off_cnt, &nl, 8, hipMemcpyHostToDevice, s));
    // 3. all-gather samples and sizes
    if (!host_tx) {
        DSORT_NCCLNB(ctx, ncclGroupStart());
        DSORT_NCCLNB(ctx, ncclAllGather(dsm + off_samp, dsm + off_all, (size_t)S, nccl_type<T>(), ctx->comm, s));
        DSORT_NCCLNB(ctx, ncclAllGather(dsm + off_cnt, dsm + off_n, 1, ncclUint64, ctx->comm, s));
        DSORT_NCCLNB(ctx, ncclGroupEnd());
        rc = exch_wait(ctx, s, false, deadline, "sample all-gather (enqueue)");
        if (rc) return rc;
        DSORT_HIP(ctx, hipMemcpyAsync(hsm + off_all, dsm + off_all, (size_t)P * S * sizeof(T) + (size_t)P * 8,
                                      hipMemcpyDeviceToHost, s));
        rc = exch_wait(ctx, s, true, deadline, "sample all-gather");
        if (rc) return rc;
    } else {
        // [S samples | n_local] per rank through the caller's all-gather
        const size_t rec = (size_t)S * sizeof(T) + 8;
        rc = ensure_host(ctx, &ctx->xfer, &ctx->xfer_bytes, rec * (size_t)(P + 1));
        if (rc) return rc;
        char *mine = static_cast<char *>(ctx->xfer), *all = mine + rec;
        DSORT_HIP(ctx, hipMemcpyAsync(mine, dsm + off_samp, (size_t)S * sizeof(T), hipMemcpyDeviceToHost, s));
        rc = exch_wait(ctx, s, true, deadline, "local sort");
        if (rc) return rc;
        memcpy(mine + (size_t)S * sizeof(T), &nl, 8);
        if ((rc = tx_fault_point(ctx))) return rc;
        if ((rc = txs.allgather(mine, all, rec, "samples all-gather"))) return set_err(ctx, rc, txs.error());
        for (int r = 0; r < P; ++r) {
            memcpy(hsm + off_all + (size_t)r * S * sizeof(T), all + (size_t)r * rec, (size_t)S * sizeof(T));
            memcpy(hsm + off_n + (size_t)r * 8, all + (size_t)r * rec + (size_t)S * sizeof(T), 8);
        }
    }
    exchange_fault_point(ctx, 1);
    // 4. splitters on the host (tiny: P*S composites)
    {
        const T *hs = reinterpret_cast<const T *>(hsm + off_all);
        const uint64_t *hn = reinterpret_cast<const uint64_t *>(hsm + off_n);
        std::vector<uint64_t> idx((size_t)P * S);
        for (int r = 0; r < P; ++r) dsort_plan_sample_positions(hn[r], S, &idx[(size_t)r * S]);
        T *sv = reinterpret_cast<T *>(hsm + off_sv);
        int32_t *sr = reinterpret_cast<int32_t *>(hsm + off_sr);
        uint64_t *si = reinterpret_cast<uint64_t *>(hsm + off_si);
        rc = plan_splitters<T>(P, S, hs, idx.data(), sv, sr, si);
        if (rc) return set_err(ctx, rc, "splitter planning failed");
        DSORT_HIP(ctx, hipMemcpyAsync(dsm + off_sv, hsm + off_sv, off_cut - off_sv, hipMemcpyHostToDevice, s));
    }
    // 5. cuts and send counts
    hipLaunchKernelGGL((cuts_kernel<T>), dim3(1), dim3(((P + 63) / 64) * 64), 0, s, d_keys,
                       (uint64_t)n_local, me, P - 1, reinterpret_cast<const T *>(dsm + off_sv),
                       reinterpret_cast<const int32_t *>(dsm + off_sr),
                       reinterpret_cast<const uint64_t *>(dsm + off_si),
                       reinterpret_cast<uint64_t *>(dsm + off_cut));
    DSORT_HIP(ctx, hipGetLastError());
    DSORT_HIP(ctx, hipMemcpyAsync(hsm + off_cut, dsm + off_cut, (size_t)(P + 1) * 8, hipMemcpyDeviceToHost, s));
    rc = exch_wait(ctx, s, true, deadline, "cut search");
    if (rc) return rc;
    const uint64_t *hcut = reinterpret_cast<const uint64_t *>(hsm + off_cut);
    uint64_t *hcnt = reinterpret_cast<uint64_t *>(hsm + off_cnt);
    for (int r = 0; r < P; ++r) hcnt[r] = hcut[r + 1] - hcut[r];
    // 6. count matrix
    if (!host_tx) {
        DSORT_HIP(ctx, hipMemcpyAsync(dsm + off_cnt, hcnt, (size_t)P * 8, hipMemcpyHostToDevice, s));
        DSORT_NCCLNB(ctx, ncclAllGather(dsm + off_cnt, dsm + off_mat, (size_t)P, ncclUint64, ctx->comm, s));
        rc = exch_wait(ctx, s, false, deadline, "count all-gather (enqueue)");
        if (rc) return rc;
        DSORT_HIP(ctx, hipMemcpyAsync(hsm + off_mat, dsm + off_mat, (size_t)P * P * 8, hipMemcpyDeviceToHost, s));
        rc = exch_wait(ctx, s, true, deadline, "count all-gather");
        if (rc) return rc;
    } else {
        if ((rc = tx_fault_point(ctx))) return rc;
        if ((rc = txs.allgather(hcnt, hsm + off_mat, (size_t)P * 8, "count all-gather"))) return set_err(ctx, rc, txs.error());
    }
    const uint64_t *mat = reinterpret_cast<const uint64_t *>(hsm + off_mat);  // mat[src*P + dst]
    std::vector<size_t> rlen(P);
    std::vector<uint64_t> roff(P + 1, 0);
    for (int r = 0; r < P; ++r) {
        rlen[r] = mat[(size_t)r * P + me];
        roff[r + 1] = roff[r] + rlen[r];
    }
    const uint64_t nrecv = roff[P];
    rc = ensure(ctx, &ctx->recv, &ctx->recv_bytes, (nrecv ? nrecv : 1) * sizeof(T), "receive buffer");
    if (rc) return rc;
    rc = ensure(ctx, &ctx->recv2, &ctx->recv2_bytes, (nrecv ? nrecv : 1) * sizeof(T), "merge output");
    if (rc) return rc;
    T *rb = static_cast<T *>(ctx->recv);
    exchange_fault_point(ctx, 2);
    uint64_t sent = 0;
    for (int r = 0; r < P; ++r) sent += r == me ? 0 : hcnt[r];
    if (ctx->ev_ok) {
        DSORT_HIP(ctx, hipEventRecord(ctx->ev[5], s));
        ctx->ev_mask |= 32u;
    }
    // 7. key exchange: one send and one receive per peer link, grouped (RCCL all-to-all-v)
    if (!host_tx) {
        DSORT_NCCLNB(ctx, ncclGroupStart());
        for (int r = 0; r < P; ++r) {
            if (r == me) continue;
            if (hcnt[r]) DSORT_NCCLNB(ctx, ncclSend(d_keys + hcut[r], hcnt[r], nccl_type<T>(), r, ctx->comm, s));
            if (rlen[r]) DSORT_NCCLNB(ctx, ncclRecv(rb + roff[r], rlen[r], nccl_type<T>(), r, ctx->comm, s));
        }
        DSORT_NCCLNB(ctx, ncclGroupEnd());
        rc = exch_wait(ctx, s, false, deadline, "key all-to-all (enqueue)");
        if (rc) return rc;
        if (ctx->ev_ok) {
            DSORT_HIP(ctx, hipEventRecord(ctx->ev[6], s));
            ctx->ev_mask |= 64u;
        }
        if (hcnt[me])
            DSORT_HIP(ctx, hipMemcpyAsync(rb + roff[me], d_keys + hcut[me], hcnt[me] * sizeof(T),
                                          hipMemcpyDeviceToDevice, s));
    } else {
        // host-staged all-to-all-v: D2H the sorted run, exchange, H2D the received runs
        rc = ensure_host(ctx, &ctx->xfer, &ctx->xfer_bytes, (n_local ? n_local : 1) * sizeof(T));
        if (rc) return rc;
        rc = ensure_host(ctx, &ctx->xfer2, &ctx->xfer2_bytes, (nrecv ? nrecv : 1) * sizeof(T));
        if (rc) return rc;
        if (n_local)
            DSORT_HIP(ctx, hipMemcpyAsync(ctx->xfer, d_keys, n_local * sizeof(T), hipMemcpyDeviceToHost, s));
        rc = exch_wait(ctx, s, true, deadline, "key staging");
        if (rc) return rc;
        std::vector<size_t> sc(P), sd(P), rcn(P), rd(P);
        for (int r = 0; r < P; ++r) {
            sc[r] = hcnt[r] * sizeof(T);
            sd[r] = hcut[r] * sizeof(T);
            rcn[r] = rlen[r] * sizeof(T);
            rd[r] = roff[r] * sizeof(T);
        }
        if ((rc = tx_fault_point(ctx))) return rc;
        if ((rc = txs.alltoallv(ctx->xfer, sc.data(), sd.data(), ctx->xfer2, rcn.data(), rd.data(), "key all-to-all")))
            return set_err(ctx, rc, txs.error());
        if (nrecv) DSORT_HIP(ctx, hipMemcpyAsync(rb, ctx->xfer2, nrecv * sizeof(T), hipMemcpyHostToDevice, s));
        if (ctx->ev_ok) {
            DSORT_HIP(ctx, hipEventRecord(ctx->ev[6], s));
            ctx->ev_mask |= 64u;
        }
    }
    if (ctx->ev_ok) {
        DSORT_HIP(ctx, hipEventRecord(ctx->ev[3], s));
        ctx->ev_mask |= 8u;
    }
    // 8. merge the P received runs (source-rank order keeps the merge deterministic); the
    // local sort's statistics and per-launch events stay
    T *outp = static_cast<T *>(ctx->recv2);
    rc = merge_device<T>(ctx, rb, rlen.data(), P, outp, s, true);
    if (rc) return rc;
    if (!host_tx) {  // the receives must have landed before the caller reads the slice
        rc = exch_wait(ctx, s, true, deadline, "key all-to-all", ctx->opt.test_hold_exchange != 0);
        if (rc) return rc;
    }
    if (ctx->ev_ok) {
        DSORT_HIP(ctx, hipEventRecord(ctx->ev[4], s));
        ctx->ev_mask |= 16u;
    }
    ctx->last_stream = s;
    st.keys_out = nrecv;
    st.keys_sent = sent;
    st.exchange_path = 2;
    ctx->stats = st;
    *d_out = outp;
    *n_out = nrecv;
    return DSORT_OK;
}

}  // namespace dsort

using namespace dsort;

// ======================================================================== C ABI =========
// (stats.deferred_frees / pending_frees of the call, whatever it returns)
template <typename T>
static int sample_sort_entry(dsort_ctx *ctx, const T *d, size_t n, T **o, size_t *no, void *st, bool presorted) {
    if (!ctx) return DSORT_EINVAL;
    const uint64_t d0 = ctx->deferred_n;
    const int rc = sample_sort<T>(ctx, d, n, o, no, st, presorted);
    ctx->stats.deferred_frees = (int)(ctx->deferred_n - d0);
    ctx->stats.pending_frees = (int)(ctx->dev_later.size() + ctx->host_later.size());
    return rc;
}

extern "C" {

const char *dsort_version(void) { return DSORT_VERSION_STRING; }

int dsort_init(dsort_ctx **out, int device) {
    if (!out) return DSORT_EINVAL;
    *out = nullptr;
    int count = 0;
    if (hipGetDeviceCount(&count) != hipSuccess || count <= 0) return DSORT_ENODEV;
    if (device < 0 || device >= count) return DSORT_ENODEV;
    hipDeviceProp_t prop;
    if (hipGetDeviceProperties(&prop, device) != hipSuccess) return DSORT_ENODEV;
    if (strncmp(prop.gcnArchName, "gfx950", 6) != 0) return DSORT_ENODEV;
    dsort_ctx *ctx = new (std::nothrow) dsort_ctx();
    if (!ctx) return DSORT_ENOMEM;
    ctx->device = device;
    if (hipSetDevice(device) != hipSuccess ||
        hipStreamCreateWithFlags(&ctx->stream, hipStreamNonBlocking) != hipSuccess) {
        delete ctx;
        return DSORT_EHIP;
    }
    if (hipMalloc(&ctx->red, 64) != hipSuccess ||
        hipHostMalloc((void **)&ctx->red_host, 64, hipHostMallocDefault) != hipSuccess) {
        dsort_finalize(ctx);
        return DSORT_ENOMEM;
    }
    ctx->ev_ok = true;
    for (auto &e : ctx->ev)
        if (hipEventCreate(&e) != hipSuccess) ctx->ev_ok = false;
    for (auto &e : ctx->kev)
        if (hipEventCreate(&e) != hipSuccess) ctx->ev_ok = false;
    ctx->ev_created = ctx->ev_ok;
    *out = ctx;
    return DSORT_OK;
}

int dsort_finalize(dsort_ctx *ctx) {
    if (!ctx) return DSORT_EINVAL;
    (void)hipSetDevice(ctx->device);
    if (ctx->stream) (void)hipStreamSynchronize(ctx->stream);
    if (ctx->comm) {
        ncclCommAbort(ctx->comm);  // peers may be gone: never wait for them here
        ctx->comm = nullptr;
    }
    ctx->poll_waits = false;
    flush_later(ctx);
    void *bufs[] = {ctx->scratch, ctx->scratch2, ctx->splits, ctx->groups, ctx->io, ctx->io2, ctx->red,
                    ctx->local, ctx->recv, ctx->recv2, ctx->small, ctx->text_status,
                    ctx->bucket, ctx->sub, ctx->sub_alt, ctx->stmp, ctx->bxs, ctx->tfb, ctx->fence};
    for (void *b : bufs)
        if (b) (void)hipFree(b);
    if (ctx->red_host) (void)hipHostFree(ctx->red_host);
    if (ctx->small_host) (void)hipHostFree(ctx->small_host);
    if (ctx->xfer) (void)hipHostFree(ctx->xfer);
    if (ctx->xfer2) (void)hipHostFree(ctx->xfer2);
    if (ctx->fence_host) (void)hipHostFree(ctx->fence_host);
    if (ctx->groups_host) (void)hipHostFree(ctx->groups_host);
    if (ctx->groups_ev) (void)hipEventDestroy(ctx->groups_ev);
    if (ctx->bucket_host) (void)hipHostFree(ctx->bucket_host);
    if (ctx->bucket_ev) (void)hipEventDestroy(ctx->bucket_ev);
    if (ctx->sub_host) (void)hipHostFree(ctx->sub_host);
    if (ctx->sub_ev) (void)hipEventDestroy(ctx->sub_ev);
    if (ctx->side_ev) (void)hipEventDestroy(ctx->side_ev);
    if (ctx->ready_ev) (void)hipEventDestroy(ctx->ready_ev);
    if (ctx->side) (void)hipStreamDestroy(ctx->side);
    for (auto &e : ctx->xev)
        if (e) (void)hipEventDestroy(e);
    if (ctx->xs) (void)hipStreamDestroy(ctx->xs);
    if (ctx->done_ev) (void)hipEventDestroy(ctx->done_ev);
    for (auto &e : ctx->ev)
        if (e) (void)hipEventDestroy(e);
    for (auto &e : ctx->kev)
        if (e) (void)hipEventDestroy(e);
    if (ctx->stream) (void)hipStreamDestroy(ctx->stream);
    delete ctx;
    return DSORT_OK;
}

const char *dsort_last_error(const dsort_ctx *ctx) { return ctx ? ctx->err.c_str() : "null context"; }

int dsort_set_option(dsort_ctx *ctx, int option, int64_t v) {
    if (!ctx) return DSORT_EINVAL;
    dsort_opts &o = ctx->opt;
    switch (option) {
        case DSORT_OPT_BUCKETS:
            if (v < -1 || v == 1 || v > 1024) return set_err(ctx, DSORT_EINVAL, "DSORT_OPT_BUCKETS: -1, 0 or 2..1024");
            o.buckets = v;
            return DSORT_OK;
        case DSORT_OPT_BUCKET_KEYS:
            if (v < 1) return set_err(ctx, DSORT_EINVAL, "DSORT_OPT_BUCKET_KEYS: >= 1");
            o.bucket_keys = v;
            return DSORT_OK;
        case DSORT_OPT_BUCKET_OVERSAMPLE:
            if (v < 1 || v > 4096) return set_err(ctx, DSORT_EINVAL, "DSORT_OPT_BUCKET_OVERSAMPLE: 1..4096");
            o.bucket_os = v;
            return DSORT_OK;
        case DSORT_OPT_MAX_FANIN_LOG2:
            if (v != -1 && (v < 1 || v > kMaxLogF)) return set_err(ctx, DSORT_EINVAL, "DSORT_OPT_MAX_FANIN_LOG2: -1 or 1..5");
            o.max_logf = v;
            return DSORT_OK;
        case DSORT_OPT_KILL_AFTER_STAGE:
            if (v < -1) return set_err(ctx, DSORT_EINVAL, "DSORT_OPT_KILL_AFTER_STAGE: -1 or a stage index");
            o.kill_after_pass = v;
            return DSORT_OK;
        case DSORT_OPT_KILL_IN_EXCHANGE:
            if (v != -1 && v != 1 && v != 2) return set_err(ctx, DSORT_EINVAL, "DSORT_OPT_KILL_IN_EXCHANGE: -1, 1 or 2");
            o.kill_in_exchange = v;
            return DSORT_OK;
        case DSORT_OPT_SUB_KEYS:
            if (v < -1) return set_err(ctx, DSORT_EINVAL, "DSORT_OPT_SUB_KEYS: -1, 0 or >= 1");
            ctx->opt.sub_keys = v;
            return DSORT_OK;
        case DSORT_OPT_SUB_OVERSAMPLE:
            if (v != -1 && (v < 1 || v > 64)) return set_err(ctx, DSORT_EINVAL, "DSORT_OPT_SUB_OVERSAMPLE: -1 or 1..64");
            ctx->opt.sub_os = v;
            return DSORT_OK;
        case DSORT_OPT_SUB_GATHER:
            if (v != 0 && v != 1) return set_err(ctx, DSORT_EINVAL, "DSORT_OPT_SUB_GATHER: 0 or 1");
            ctx->opt.sub_gather = v;
            return DSORT_OK;
        case DSORT_OPT_COMM_TIMEOUT_MS:
            if (v < 0) return set_err(ctx, DSORT_EINVAL, "DSORT_OPT_COMM_TIMEOUT_MS: >= 0");
            o.comm_timeout_ms = v;
            return DSORT_OK;
        case DSORT_OPT_TEST_HOLD_EXCHANGE:
            if (v != 0 && v != 1) return set_err(ctx, DSORT_EINVAL, "DSORT_OPT_TEST_HOLD_EXCHANGE: 0 or 1");
            o.test_hold_exchange = v;
            return DSORT_OK;
        case DSORT_OPT_TEST_FAIL_EXCHANGE:
            if (v < -1) return set_err(ctx, DSORT_EINVAL, "DSORT_OPT_TEST_FAIL_EXCHANGE: -1 or a collective index");
            o.test_fail_exchange = v;
            return DSORT_OK;
        case DSORT_OPT_STAGE_TIMING:
            if (v != 0 && v != 1) return set_err(ctx, DSORT_EINVAL, "DSORT_OPT_STAGE_TIMING: 0 or 1");
            o.stage_timing = v;
            ctx->ev_ok = ctx->ev_created && v != 0;
            return DSORT_OK;
        case DSORT_OPT_TEST_TILE_CAP:
            if (v < 0) return set_err(ctx, DSORT_EINVAL, "DSORT_OPT_TEST_TILE_CAP: >= 0");
            o.test_tile_cap = v;
            return DSORT_OK;
        case DSORT_OPT_TEST_WAVE_FENCE:
            if (v < 0 || v > 2) return set_err(ctx, DSORT_EINVAL, "DSORT_OPT_TEST_WAVE_FENCE: 0, 1 or 2");
            o.test_wave_fence = v;
            return DSORT_OK;
        default:
            return set_err(ctx, DSORT_EINVAL, "unknown option " + std::to_string(option));
    }
}

int dsort_get_option(const dsort_ctx *ctx, int option, int64_t *v) {
    if (!ctx || !v) return DSORT_EINVAL;
    const dsort_opts &o = ctx->opt;
    switch (option) {
        case DSORT_OPT_BUCKETS: *v = o.buckets; return DSORT_OK;
        case DSORT_OPT_BUCKET_KEYS: *v = o.bucket_keys; return DSORT_OK;
        case DSORT_OPT_BUCKET_OVERSAMPLE: *v = o.bucket_os; return DSORT_OK;
        case DSORT_OPT_MAX_FANIN_LOG2: *v = o.max_logf; return DSORT_OK;
        case DSORT_OPT_KILL_AFTER_STAGE: *v = o.kill_after_pass; return DSORT_OK;
        case DSORT_OPT_KILL_IN_EXCHANGE: *v = o.kill_in_exchange; return DSORT_OK;
        case DSORT_OPT_COMM_TIMEOUT_MS: *v = o.comm_timeout_ms; return DSORT_OK;
        case DSORT_OPT_TEST_HOLD_EXCHANGE: *v = o.test_hold_exchange; return DSORT_OK;
        case DSORT_OPT_TEST_FAIL_EXCHANGE: *v = o.test_fail_exchange; return DSORT_OK;
        case DSORT_OPT_STAGE_TIMING: *v = o.stage_timing; return DSORT_OK;
        case DSORT_OPT_TEST_TILE_CAP: *v = o.test_tile_cap; return DSORT_OK;
        case DSORT_OPT_TEST_WAVE_FENCE: *v = o.test_wave_fence; return DSORT_OK;
        case DSORT_OPT_SUB_KEYS: *v = o.sub_keys; return DSORT_OK;
        case DSORT_OPT_SUB_OVERSAMPLE: *v = o.sub_os; return DSORT_OK;
        case DSORT_OPT_SUB_GATHER: *v = o.sub_gather; return DSORT_OK;
        default: return DSORT_EINVAL;
    }
}

int dsort_get_stats(const dsort_ctx *cctx, dsort_stats *out) {
    if (!cctx || !out) return DSORT_EINVAL;
    dsort_ctx *ctx = const_cast<dsort_ctx *>(cctx);
    *out = ctx->stats;
    if (!ctx->ev_ok) return DSORT_OK;
    if (hipStreamSynchronize(ctx->last_stream) != hipSuccess) return DSORT_EHIP;
    float ms = 0;
    auto el = [&](int a, int b) -> double {
        if (!(ctx->ev_mask & (1u << a)) || !(ctx->ev_mask & (1u << b))) return 0.0;
        return hipEventElapsedTime(&ms, ctx->ev[a], ctx->ev[b]) == hipSuccess ? (double)ms : 0.0;
    };
    out->merge_kernel_ms = 0;
    out->merge_kernel_launches = 0;
    for (int i = 0; i + 1 < ctx->kev_used; i += 2) {
        if (hipEventQuery(ctx->kev[i + 1]) != hipSuccess) break;
        if (hipEventElapsedTime(&ms, ctx->kev[i], ctx->kev[i + 1]) == hipSuccess) {
            out->merge_kernel_ms += ms;
            out->merge_kernel_launches += 1;
        }
    }
    out->block_sort_ms = el(0, 1);
    out->merge_ms = el(1, 2);
    // (the bucket exchange's first wave recorded its tile sort and second level at 22/23, 28/29)
    out->tile_sort_kernel_ms = el(7, 8) + el(22, 23);
    out->partition_ms = el(0, 7);
    out->bucket_hist_ms = el(9, 10);
    out->bucket_scatter_ms = el(11, 12);
    out->sub_partition_ms = el(13, 14) + el(28, 29);
    if (ctx->ev_mask & 16u) {
        out->exchange_ms = el(2, 3);
        out->final_merge_ms = el(3, 4);
        out->total_ms = el(0, 4);
        out->alltoall_ms = el(5, 6);
    } else {
        out->total_ms = el(0, 2);
    }
    return DSORT_OK;
}

int dsort_synchronize(dsort_ctx *ctx) {
    if (!ctx) return DSORT_EINVAL;
    DSORT_HIP(ctx, hipStreamSynchronize(ctx->last_stream));
    DSORT_HIP(ctx, hipStreamSynchronize(ctx->stream));
    return DSORT_OK;
}

int dsort_sort_stages(const dsort_ctx *ctx, size_t n, int key_bytes, int *stages) {
    if (!stages || (key_bytes != 4 && key_bytes != 8)) return DSORT_EINVAL;
    static const dsort_opts defaults{};
    *stages = sort_stages(ctx ? ctx->opt : defaults, n, key_bytes);
    return DSORT_OK;
}

int dsort_sample_sort_stages(const dsort_ctx *ctx, size_t n_total, int nranks, int rank, int key_bytes,
                             int *stages) {
    if (!stages || nranks < 1 || rank < 0 || rank >= nranks || (key_bytes != 4 && key_bytes != 8)) return DSORT_EINVAL;
    static const dsort_opts defaults{};
    const dsort_opts &o = ctx ? ctx->opt : defaults;
    std::vector<uint64_t> n_of(nranks);
    for (int r = 0; r < nranks; ++r) n_of[r] = n_total / nranks + ((uint64_t)r < n_total % nranks ? 1 : 0);
    BxPlan pl;
    *stages = bx_make_plan(o, nranks, rank, n_of.data(), key_bytes, pl) ? 3 : sort_stages(o, n_of[rank], key_bytes);
    return DSORT_OK;
}

int dsort_sort_i32(dsort_ctx *ctx, int32_t *keys, size_t n) { return sort_host<int32_t>(ctx, keys, n); }
int dsort_sort_i64(dsort_ctx *ctx, int64_t *keys, size_t n) { return sort_host<int64_t>(ctx, keys, n); }

int dsort_sort_dev_i32(dsort_ctx *ctx, int32_t *d, size_t n, void *stream) {
    if (!ctx || (n && !d)) return set_err(ctx, DSORT_EINVAL, "null argument");
    return sort_device<int32_t>(ctx, d, d, n, pick(ctx, stream), true);
}
int dsort_sort_dev_i64(dsort_ctx *ctx, int64_t *d, size_t n, void *stream) {
    if (!ctx || (n && !d)) return set_err(ctx, DSORT_EINVAL, "null argument");
    return sort_device<int64_t>(ctx, d, d, n, pick(ctx, stream), true);
}
int dsort_sort_dev_copy_i32(dsort_ctx *ctx, const int32_t *in, int32_t *out, size_t n, void *stream) {
    if (!ctx || (n && (!in || !out))) return set_err(ctx, DSORT_EINVAL, "null argument");
    return sort_device<int32_t>(ctx, in, out, n, pick(ctx, stream), true);
}
int dsort_sort_dev_copy_i64(dsort_ctx *ctx, const int64_t *in, int64_t *out, size_t n, void *stream) {
    if (!ctx || (n && (!in || !out))) return set_err(ctx, DSORT_EINVAL, "null argument");
    return sort_device<int64_t>(ctx, in, out, n, pick(ctx, stream), true);
}

int dsort_merge_i32(dsort_ctx *ctx, const int32_t *const runs[], const size_t lens[], int k, int32_t *out) {
    return merge_host<int32_t>(ctx, runs, lens, k, out);
}
int dsort_merge_i64(dsort_ctx *ctx, const int64_t *const runs[], const size_t lens[], int k, int64_t *out) {
    return merge_host<int64_t>(ctx, runs, lens, k, out);
}
int dsort_merge_dev_i32(dsort_ctx *ctx, const int32_t *d_in, const size_t lens[], int k, int32_t *d_out,
                        void *stream) {
    if (!ctx || k < 0 || (k && !lens)) return set_err(ctx, DSORT_EINVAL, "bad argument");
    return merge_device<int32_t>(ctx, d_in, lens, k, d_out, pick(ctx, stream));
}
int dsort_merge_dev_i64(dsort_ctx *ctx, const int64_t *d_in, const size_t lens[], int k, int64_t *d_out,
                        void *stream) {
    if (!ctx || k < 0 || (k && !lens)) return set_err(ctx, DSORT_EINVAL, "bad argument");
    return merge_device<int64_t>(ctx, d_in, lens, k, d_out, pick(ctx, stream));
}

int dsort_comm_unique_id(char id[DSORT_UNIQUE_ID_BYTES]) {
    static_assert(sizeof(ncclUniqueId) == DSORT_UNIQUE_ID_BYTES, "ncclUniqueId size");
    if (!id) return DSORT_EINVAL;
    ncclUniqueId u;
    if (ncclGetUniqueId(&u) != ncclSuccess) return DSORT_ECOMM;
    memcpy(id, &u, sizeof(u));
    return DSORT_OK;
}

int dsort_comm_init(dsort_ctx *ctx, int nranks, int rank, const char id[DSORT_UNIQUE_ID_BYTES]) {
    if (!ctx || !id || nranks < 1 || rank < 0 || rank >= nranks) return set_err(ctx, DSORT_EINVAL, "bad argument");
    if (ctx->comm || ctx->has_transport) return set_err(ctx, DSORT_EINVAL, "communicator already initialised");
    DSORT_HIP(ctx, hipSetDevice(ctx->device));
    std::unique_lock<std::mutex> lock(comm_mutex(ctx));
    ctx->abort_req.store(0);  // a flag left by the previous communicator's abort
    ncclUniqueId u;
    memcpy(&u, id, sizeof(u));
    ncclComm_t c = nullptr;
    // non-blocking communicator: no RCCL call may block on a dead peer (exch_wait polls instead)
    ncclConfig_t cfg = NCCL_CONFIG_INITIALIZER;
    cfg.blocking = 0;
    ncclResult_t r = ncclCommInitRankConfig(&c, nranks, u, rank, &cfg);
    const double deadline = ctx->opt.comm_timeout_ms > 0 ? now_ms() + (double)ctx->opt.comm_timeout_ms : 0.0;
    while (r == ncclInProgress && c) {
        ncclCommGetAsyncError(c, &r);
        if (r != ncclInProgress) break;
        if (deadline > 0 && now_ms() > deadline) {
            ncclCommAbort(c);
            return set_err(ctx, DSORT_ETIMEOUT, "ncclCommInitRankConfig: peers did not join before the deadline");
        }
        if (ctx->abort_req.load()) {
            ncclCommAbort(c);
            ctx->abort_req.store(0);
            return set_err(ctx, DSORT_ECOMM, "ncclCommInitRankConfig: aborted by dsort_comm_abort");
        }
        usleep(50);
    }
    if (r != ncclSuccess) {
        if (c) ncclCommAbort(c);
        return set_err(ctx, DSORT_ECOMM, std::string("ncclCommInitRankConfig: ") + ncclGetErrorString(r) +
                                             " (RCCL needs one GPU per rank; ranks sharing a GPU use "
                                             "dsort_comm_init_transport)");
    }
    ctx->comm = c;
    ctx->nranks = nranks;
    ctx->rank = rank;
    return DSORT_OK;
}

int dsort_comm_init_transport(dsort_ctx *ctx, int nranks, int rank, const dsort_transport *t) {
    if (!ctx || !t || !t->allgather || !t->alltoallv || nranks < 1 || rank < 0 || rank >= nranks)
        return set_err(ctx, DSORT_EINVAL, "bad argument");
    std::unique_lock<std::mutex> lock(comm_mutex(ctx));
    if (ctx->comm || ctx->has_transport) return set_err(ctx, DSORT_EINVAL, "communicator already initialised");
    ctx->abort_req.store(0);  // a flag left by the previous communicator's abort
    ctx->transport = *t;
    ctx->has_transport = true;
    ctx->nranks = nranks;
    ctx->rank = rank;
    return DSORT_OK;
}

int dsort_comm_deadline_ms(const dsort_ctx *ctx, int64_t *remaining_ms) {
    if (!ctx || !remaining_ms) return DSORT_EINVAL;
    *remaining_ms = ctx->tx ? ctx->tx->remaining_ms() : -1;
    return DSORT_OK;
}

int dsort_comm_abort(dsort_ctx *ctx) {
    if (!ctx) return DSORT_EINVAL;
    std::unique_lock<std::mutex> lock(comm_mutex(ctx), std::try_to_lock);
    if (!lock.owns_lock()) {  // an exchange is running on another thread: it aborts itself
        ctx->abort_req.store(1);
        return DSORT_OK;
    }
    abort_comm_locked(ctx);
    ctx->abort_req.store(0);
    return DSORT_OK;
}

int dsort_comm_destroy(dsort_ctx *ctx) {
    if (!ctx) return DSORT_EINVAL;
    std::unique_lock<std::mutex> lock(comm_mutex(ctx));
    ctx->has_transport = false;
    if (ctx->comm) {
        (void)hipStreamSynchronize(ctx->stream);
        // non-blocking communicator: finalize, wait for it (never longer than the exchange
        // deadline, 10 s without one, or an abort request: a peer that died after its last
        // collective must not hold this rank in shutdown), then destroy -- else abort
        const double limit = ctx->opt.comm_timeout_ms > 0 ? (double)ctx->opt.comm_timeout_ms : 10000.0;
        const double deadline = now_ms() + limit;
        ncclResult_t r = ncclCommFinalize(ctx->comm);
        while (r == ncclInProgress) {
            ncclCommGetAsyncError(ctx->comm, &r);
            if (r != ncclInProgress) break;
            if (ctx->abort_req.load() || now_ms() > deadline) break;
            usleep(50);
        }
        if (r == ncclSuccess) ncclCommDestroy(ctx->comm);
        else ncclCommAbort(ctx->comm);
    }
    ctx->comm = nullptr;
    ctx->nranks = 1;
    ctx->rank = 0;
    return DSORT_OK;
}

int dsort_sample_sort_dev_i32(dsort_ctx *ctx, const int32_t *d, size_t n, int32_t **o, size_t *no, void *st) {
    return sample_sort_entry<int32_t>(ctx, d, n, o, no, st, false);
}
int dsort_sample_sort_dev_i64(dsort_ctx *ctx, const int64_t *d, size_t n, int64_t **o, size_t *no, void *st) {
    return sample_sort_entry<int64_t>(ctx, d, n, o, no, st, false);
}
int dsort_sample_merge_dev_i32(dsort_ctx *ctx, const int32_t *d, size_t n, int32_t **o, size_t *no, void *st) {
    return sample_sort_entry<int32_t>(ctx, d, n, o, no, st, true);
}
int dsort_sample_merge_dev_i64(dsort_ctx *ctx, const int64_t *d, size_t n, int64_t **o, size_t *no, void *st) {
    return sample_sort_entry<int64_t>(ctx, d, n, o, no, st, true);
}

int dsort_plan_sample_positions(size_t n, int s, uint64_t *idx) {
    if (s < 1 || !idx) return DSORT_EINVAL;
    for (int j = 0; j < s; ++j) {
        uint64_t p = n ? (uint64_t)(j + 1) * (uint64_t)n / (uint64_t)(s + 1) : 0;
        if (n && p >= n) p = n - 1;
        idx[j] = p;
    }
    return DSORT_OK;
}

int dsort_plan_splitters_i32(int nranks, int s, const int32_t *samples, const uint64_t *idx,
                             int32_t *sv, int32_t *sr, uint64_t *si) {
    return plan_splitters<int32_t>(nranks, s, samples, idx, sv, sr, si);
}
int dsort_plan_splitters_i64(int nranks, int s, const int64_t *samples, const uint64_t *idx,
                             int64_t *sv, int32_t *sr, uint64_t *si) {
    return plan_splitters<int64_t>(nranks, s, samples, idx, sv, sr, si);
}
int dsort_plan_cuts_i32(const int32_t *sorted, size_t n, int my_rank, int nranks, const int32_t *sv,
                        const int32_t *sr, const uint64_t *si, uint64_t *cuts) {
    return plan_cuts<int32_t>(sorted, n, my_rank, nranks, sv, sr, si, cuts);
}
int dsort_plan_cuts_i64(const int64_t *sorted, size_t n, int my_rank, int nranks, const int64_t *sv,
                        const int32_t *sr, const uint64_t *si, uint64_t *cuts) {
    return plan_cuts<int64_t>(sorted, n, my_rank, nranks, sv, sr, si, cuts);
}

int dsort_gen_uniform_i32(dsort_ctx *ctx, int32_t *d, size_t n, uint64_t seed, uint64_t first, void *stream) {
    if (!ctx || (n && !d)) return set_err(ctx, DSORT_EINVAL, "null argument");
    if (!n) return DSORT_OK;
    hipLaunchKernelGGL(gen_uniform_i32_kernel, dim3(grid_for(n, 256 * 4)), dim3(256), 0, pick(ctx, stream), d,
                       (uint64_t)n, seed + first);
    DSORT_HIP(ctx, hipGetLastError());
    return DSORT_OK;
}
int dsort_gen_uniform_i64(dsort_ctx *ctx, int64_t *d, size_t n, uint64_t seed, uint64_t first, void *stream) {
    if (!ctx || (n && !d)) return set_err(ctx, DSORT_EINVAL, "null argument");
    if (!n) return DSORT_OK;
    hipLaunchKernelGGL(gen_uniform_i64_kernel, dim3(grid_for(n, 256 * 4)), dim3(256), 0, pick(ctx, stream), d,
                       (uint64_t)n, seed + first);
    DSORT_HIP(ctx, hipGetLastError());
    return DSORT_OK;
}
int dsort_gen_zipf_i64(dsort_ctx *ctx, int64_t *d, size_t n, uint64_t seed, uint64_t first, void *stream) {
    if (!ctx || (n && !d)) return set_err(ctx, DSORT_EINVAL, "null argument");
    if (!n) return DSORT_OK;
    hipLaunchKernelGGL(gen_zipf_i64_kernel, dim3(grid_for(n, 256 * 4)), dim3(256), 0, pick(ctx, stream), d,
                       (uint64_t)n, seed + first);
    DSORT_HIP(ctx, hipGetLastError());
    return DSORT_OK;
}

int dsort_fingerprint_i32(dsort_ctx *ctx, const int32_t *d, size_t n, uint64_t *sum, uint64_t *xr) {
    return fingerprint_t<int32_t>(ctx, d, n, sum, xr, nullptr, false);
}
int dsort_fingerprint_i64(dsort_ctx *ctx, const int64_t *d, size_t n, uint64_t *sum, uint64_t *xr) {
    return fingerprint_t<int64_t>(ctx, d, n, sum, xr, nullptr, false);
}
int dsort_count_descents_i32(dsort_ctx *ctx, const int32_t *d, size_t n, uint64_t *count) {
    return fingerprint_t<int32_t>(ctx, d, n, nullptr, nullptr, count, true);
}
int dsort_count_descents_i64(dsort_ctx *ctx, const int64_t *d, size_t n, uint64_t *count) {
    return fingerprint_t<int64_t>(ctx, d, n, nullptr, nullptr, count, true);
}

int dsort_dev_alloc(dsort_ctx *ctx, void **p, size_t bytes) {
    if (!ctx || !p) return DSORT_EINVAL;
    DSORT_HIP(ctx, hipMalloc(p, bytes ? bytes : 1));
    return DSORT_OK;
}
int dsort_dev_free(dsort_ctx *ctx, void *p) {
    if (!ctx) return DSORT_EINVAL;
    if (p) DSORT_HIP(ctx, hipFree(p));
    return DSORT_OK;
}
int dsort_copy_h2d(dsort_ctx *ctx, void *d, const void *h, size_t bytes) {
    if (!ctx) return DSORT_EINVAL;
    if (bytes) DSORT_HIP(ctx, hipMemcpy(d, h, bytes, hipMemcpyHostToDevice));
    return DSORT_OK;
}
int dsort_copy_d2h(dsort_ctx *ctx, void *h, const void *d, size_t bytes) {
    if (!ctx) return DSORT_EINVAL;
    if (bytes) DSORT_HIP(ctx, hipMemcpy(h, d, bytes, hipMemcpyDeviceToHost));
    return DSORT_OK;
}

int dsort_copy_d2d(dsort_ctx *ctx, void *d, const void *src, size_t bytes) {
    if (!ctx) return DSORT_EINVAL;
    if (bytes) {
        DSORT_HIP(ctx, hipMemcpyAsync(d, src, bytes, hipMemcpyDeviceToDevice, ctx->stream));
        DSORT_HIP(ctx, hipStreamSynchronize(ctx->stream));
    }
    return DSORT_OK;
}
int dsort_host_register(dsort_ctx *ctx, void *host, size_t bytes) {
    if (!ctx || (!host && bytes)) return DSORT_EINVAL;
    if (bytes) DSORT_HIP(ctx, hipHostRegister(host, bytes, hipHostRegisterDefault));
    return DSORT_OK;
}
int dsort_host_unregister(dsort_ctx *ctx, void *host) {
    if (!ctx) return DSORT_EINVAL;
    if (host) DSORT_HIP(ctx, hipHostUnregister(host));
    return DSORT_OK;
}

int dsort_write_text_i32(const char *path, const int32_t *keys, size_t n) {
    if (!path || (n && !keys)) return DSORT_EINVAL;
    FILE *f = fopen(path, "w");
    if (!f) return DSORT_EINVAL;
    std::vector<char> buf(1 << 20);
    size_t o = 0;
    char tmp[16];
    for (size_t i = 0; i < n; ++i) {
        if (o + 13 > buf.size()) {
            if (fwrite(buf.data(), 1, o, f) != o) { fclose(f); return DSORT_EINVAL; }
            o = 0;
        }
        int64_t v = keys[i];
        const bool neg = v < 0;
        uint64_t u = neg ? (uint64_t)(-v) : (uint64_t)v;
        int t = 0;
        do { tmp[t++] = (char)('0' + u % 10); u /= 10; } while (u);
        if (neg) buf[o++] = '-';
        while (t) buf[o++] = tmp[--t];
        buf[o++] = '\n';
    }
    if (o && fwrite(buf.data(), 1, o, f) != o) { fclose(f); return DSORT_EINVAL; }
    return fclose(f) == 0 ? DSORT_OK : DSORT_EINVAL;
}

}  // extern "C"
