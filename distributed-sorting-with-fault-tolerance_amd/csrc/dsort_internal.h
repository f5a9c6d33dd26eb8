// dsort_internal.h -- private declarations shared by the libdsort translation units.
// gfx950 only (MI355X, CDNA4, wave64).  No CUDA shims, no dual platform paths.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stddef.h>

#include <atomic>
#include <mutex>
#include <string>
#include <vector>

#include "dsort.h"

struct ncclComm;
namespace dsort {
class TxSeq;
}

namespace dsort {

// ----------------------------------------------------------------------------------------
// k-way merge passes.  A pass merges GROUPS of up to F sorted runs (F a power of two <= kMaxF)
// that lie back to back; every group's output is cut into TILE-key output tiles, one workgroup
// per tile.  Regular passes (the sort): runs of length R, groups of F runs, so every group is
// a multiple of TILE long and tile j covers output [j*TILE, (j+1)*TILE).  Irregular passes (the
// master merge, the multi-GPU receive merge): a table of groups with arbitrary run lengths.
// ----------------------------------------------------------------------------------------
constexpr int kMaxLogF = 5;
constexpr int kMaxF = 1 << kMaxLogF;

struct GroupK {
    uint64_t base;        // first key of the group (input and output index)
    uint64_t first_tile;  // global index of the group's first output tile
    uint64_t total;       // keys in the group
    uint32_t nruns;       // runs in the group (<= F of the pass)
    uint32_t pad;
    uint64_t roff[kMaxF + 1];  // run i = [base + roff[i], base + roff[i+1])
};

struct PassDesc {
    uint64_t n;              // keys in the whole array
    uint64_t R;              // regular: run length (a multiple of TILE)
    int F;                   // runs per group, power of two
    int ngroups;             // irregular: entries in `groups`
    const GroupK *groups;    // irregular: group table (device memory)
    const uint32_t *tile_group = nullptr;  // irregular, optional: group of every output tile
};

}  // namespace dsort

// Per-context options (dsort_set_option; defaults = the tuned values).
struct dsort_opts {
    int64_t buckets = -1;           // DSORT_OPT_BUCKETS: -1 auto, 0 off, B forced
    int64_t bucket_keys = 1 << 20;  // DSORT_OPT_BUCKET_KEYS
#ifndef DSORT_BUCKET_OS_DEFAULT
#define DSORT_BUCKET_OS_DEFAULT 128
#endif
    int64_t bucket_os = DSORT_BUCKET_OS_DEFAULT;  // DSORT_OPT_BUCKET_OVERSAMPLE
    int64_t max_logf = -1;          // DSORT_OPT_MAX_FANIN_LOG2: -1 = per key type default
    int64_t kill_after_pass = -1;   // DSORT_OPT_KILL_AFTER_STAGE
    int64_t stage_timing = 1;       // DSORT_OPT_STAGE_TIMING
    int64_t kill_in_exchange = -1;  // DSORT_OPT_KILL_IN_EXCHANGE
    int64_t comm_timeout_ms = 0;    // DSORT_OPT_COMM_TIMEOUT_MS
    int64_t test_hold_exchange = 0; // DSORT_OPT_TEST_HOLD_EXCHANGE
    int64_t test_fail_exchange = -1; // DSORT_OPT_TEST_FAIL_EXCHANGE
    int64_t test_tile_cap = 0;      // DSORT_OPT_TEST_TILE_CAP
    int64_t test_wave_fence = 0;    // DSORT_OPT_TEST_WAVE_FENCE
    int64_t sub_keys = -1;          // DSORT_OPT_SUB_KEYS: -1 = 3/16 of a tile, 0 = no second level
    int64_t sub_os = -1;            // DSORT_OPT_SUB_OVERSAMPLE: -1 = 8 (4 at sub-buckets <= TILE/8)
    int64_t sub_gather = 1;         // DSORT_OPT_SUB_GATHER
};

// The context.  One per host thread, bound to one device.
struct dsort_ctx {
    dsort_opts opt;
    int nested = 0;  // > 0 inside a sort the library runs for itself (the splitter-sample sort):
                     // such a sort never buckets and never fires the fault injection
    int stages_done = 0;            // kill points the running (outermost) sort has passed
    std::atomic<int> abort_req{0};  // dsort_comm_abort from another thread during an exchange
    std::mutex comm_mu;             // held by a running exchange / communicator set-up (dsort.h)
    int device = 0;
    hipStream_t stream = nullptr;
    std::string err;
    // grow-only device arenas
    void *scratch = nullptr;
    size_t scratch_bytes = 0;
    void *splits = nullptr;   // per-tile split vectors of a k-way pass (uint32 x F per tile)
    size_t splits_bytes = 0;
    void *groups = nullptr;   // irregular group tables (device)
    size_t groups_bytes = 0;
    void *groups_host = nullptr;  // pinned staging of the group tables
    size_t groups_host_bytes = 0;
    hipEvent_t groups_ev = nullptr;  // last H2D copy out of groups_host
    bool groups_ev_pending = false;
    void *scratch2 = nullptr; // second scratch for multi-level irregular merges
    size_t scratch2_bytes = 0;
    void *io = nullptr;        // staging for the host-buffer entry points
    size_t io_bytes = 0;
    void *io2 = nullptr;
    size_t io2_bytes = 0;
    void *bucket = nullptr;       // partition pass of the bucketed int32 sort (dsort_bucket.h)
    size_t bucket_bytes = 0;
    void *bucket_host = nullptr;  // pinned: bucket starts
    size_t bucket_host_bytes = 0;
    hipEvent_t bucket_ev = nullptr;
    void *sub = nullptr;          // second partition level (dsort_sub.h)
    size_t sub_bytes = 0;
    void *sub_alt = nullptr;      // the bucket exchange's second wave uses the other of the two
    size_t sub_alt_bytes = 0;     // (the first wave's kernels still read theirs)
    void *stmp = nullptr;         // merge output of a split sub-bucket (merge_split_subbuckets)
    size_t stmp_bytes = 0;
    void *sub_host = nullptr;     // pinned: bucket table, chunk table, tile / merge-record counts
    size_t sub_host_bytes = 0;
    hipEvent_t sub_ev = nullptr;
    hipStream_t side = nullptr;   // copies that overlap the first-level scatter (both directions)
    hipEvent_t side_ev = nullptr;  // side -> sort stream
    hipEvent_t ready_ev = nullptr; // sort stream -> side
    // End of the last sort / merge on its stream: a call on another stream waits for it, since
    // the arenas are shared and a call returns while its last kernels still run.
    hipEvent_t done_ev = nullptr;
    hipStream_t done_stream = nullptr;
    bool done_pending = false;
    void *tfb = nullptr;          // tiles the bin sort declined (+ their count, on the device)
    size_t tfb_bytes = 0;
    void *text_status = nullptr;  // per-tile counts and their prefixes of the text codec
    size_t text_status_bytes = 0;
    void *red = nullptr;       // 64 B of reduction accumulators
    uint64_t *red_host = nullptr;  // pinned mirror
    // sample sort (multi-GPU)
    ncclComm *comm = nullptr;
    bool has_transport = false;   // host transport instead of RCCL (dsort_comm_init_transport)
    dsort_transport transport = {};
    dsort::TxSeq *tx = nullptr;   // the running sample sort's host-transport sequence (dsort_tx.h)
    void *xfer = nullptr;         // pinned host staging of the host transport
    size_t xfer_bytes = 0;
    void *xfer2 = nullptr;
    size_t xfer2_bytes = 0;
    void *fence = nullptr;        // DSORT_OPT_TEST_WAVE_FENCE: fingerprints (device, pinned mirror)
    size_t fence_bytes = 0;
    void *fence_host = nullptr;
    size_t fence_host_bytes = 0;
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
    void *bxs = nullptr;    // bucket exchange: this rank's and every rank's splitter samples
    size_t bxs_bytes = 0;
    const uint32_t *bk_hot = nullptr;  // the last first level's runs flag (device, BkMap.hot)
    hipStream_t xs = nullptr;     // bucket exchange: the comm stream of its sends and receives
    hipEvent_t xev[3] = {};       // ... a wave's receives done (0, 1), the partition done (2)
    int ev_off = 0;               // stage events 1, 7, 8, 13, 14 of the bucket exchange's first
                                  // wave go to 16, 22, 23, 28, 29 (dsort_get_stats adds them up)
    int ev_done = 2;        // the stage event a sort's second level records at its end (the bucket
                            // exchange records its own end as event 4)
    // The bucket exchange runs its second level while the keys are still in flight: the sort's
    // host waits then poll (abort flag, deadline) instead of blocking on a stream a dead peer
    // would never complete (sync_event / sync_stream, dsort_wave.hip).
    bool poll_waits = false;
    double poll_deadline = 0.0;  // ms on the CLOCK_MONOTONIC scale, 0 = none
    hipStream_t poll_stream = nullptr;  // the sort stream of those waits (ensure() polls it, and the
                                        // side stream, instead of a device-wide synchronize)
    // buffers replaced while poll_waits is set: hipFree / hipHostFree synchronize the device, which
    // would wait for the comm stream, so they are released once the exchange is over (flush_later)
    std::vector<void *> dev_later, host_later;
    uint64_t deferred_n = 0;  // arenas whose release was deferred so far (stats.deferred_frees)
    // stage timing
    hipEvent_t ev[30] = {};  // 0 start, 1 tile sort done, 2 local sort done, 3 exchange done,
                             // 4 final merge done, 5/6 around the key all-to-all, 7/8 around the
                             // tile sort kernel, 9/10 around the first-level histogram, 11/12
                             // around the first-level scatter, 13/14 around the second-level
                             // partition
    unsigned ev_mask = 0;             // events recorded by the last call (bit i = ev[i])
    hipStream_t last_stream = nullptr;  // stream of the last asynchronous call
    static constexpr int kMaxKev = 128;  // per-launch events of the merge kernel (2 per pass)
    hipEvent_t kev[kMaxKev] = {};
    int kev_used = 0;
    bool ev_ok = false;       // stage events recorded: created, and DSORT_OPT_STAGE_TIMING on
    bool ev_created = false;
    dsort_stats stats = {};
};

namespace dsort {

// Inclusive sum over a wave (DPP row shifts, then the row broadcasts of lane 15 and 31).
__device__ __forceinline__ uint32_t wave_incl_sum(uint32_t v) {
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x111, 0xF, 0xF, false);  // row_shr:1
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x112, 0xF, 0xF, false);  // row_shr:2
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x114, 0xF, 0xF, false);  // row_shr:4
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x118, 0xF, 0xF, false);  // row_shr:8
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x142, 0xA, 0xF, false);  // row_bcast:15
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x143, 0xC, 0xF, false);  // row_bcast:31
    return v;
}

// The statistics of a call before it records anything (first_level_map -1: no bucketed sort ran).
inline dsort_stats fresh_stats() {
    dsort_stats s{};
    s.first_level_map = -1;
    return s;
}

int set_err(dsort_ctx *ctx, int code, const std::string &msg);
// the stream argument of the C-ABI: NULL = the context's stream, DSORT_NULL_STREAM = stream 0
hipStream_t pick_stream(dsort_ctx *ctx, void *stream);
int hip_err(dsort_ctx *ctx, hipError_t e, const char *what);
int ensure(dsort_ctx *ctx, void **buf, size_t *have, size_t need, const char *what);
// hipFree / hipHostFree of a replaced buffer, deferred while ctx->poll_waits (see dsort_ctx)
void release_dev(dsort_ctx *ctx, void *p);
void release_host(dsort_ctx *ctx, void *p);
void flush_later(dsort_ctx *ctx);

// The sort and the k-way merge (dsort_wave.hip), both key widths.  All asynchronous on `s`.
// sort_device sorts d_in[0..n) into d_keys (d_in may equal d_keys).  merge_device with
// keep_stats leaves the statistics and per-launch events of the preceding local sort alone (the
// sample sort's final merge).
template <typename T>
int sort_device(dsort_ctx *ctx, const T *d_in, T *d_keys, size_t n, hipStream_t s, bool timed);
template <typename T>
int merge_device(dsort_ctx *ctx, const T *d_in, const size_t *lens, int k, T *d_out,
                 hipStream_t s, bool keep_stats = false);
// Fault injection for the fault-tolerance tests and bench (BASELINE config C5): with
// DSORT_OPT_KILL_AFTER_STAGE = k the process SIGKILLs itself right after stage k of a local
// (non-nested) sort has finished on the GPU -- a worker dying mid-sort.  The stages of a sort, in
// order (sort_stages counts them):
//   bucketed sort (>= 2^25 keys)  0 first-level partition, 1 second-level partition, 2 tile sort
//     (with DSORT_OPT_SUB_KEYS = 0: 0 partition, 1 tile sort, 2 + p merge pass p)
//   merge path                    0 tile sort, 1 + p merge pass p
// A kill stage the sort never reaches makes the sort return DSORT_EINVAL (sort_device).
void fault_point(dsort_ctx *ctx, hipStream_t s, int stage);
// Kill points of a top-level sort of n keys of key_bytes bytes under `opt` (the bucketed path
// without the second level has data-dependent merge passes: the guaranteed minimum).
int sort_stages(const dsort_opts &opt, uint64_t n, int key_bytes);
// Host waits of the sort: blocking, or (ctx->poll_waits) polling with the abort flag and deadline
// (DSORT_ECOMM / DSORT_ETIMEOUT).
int sync_event(dsort_ctx *ctx, hipEvent_t e, const char *what);
int sync_stream(dsort_ctx *ctx, hipStream_t s, const char *what);
// The pause between two polls of a polled wait: yield for the first POLL_SPIN_MS of the wait,
// then sleep.  (A usleep of a few us sleeps about 60 us with the default timer slack: measured
// as 40-85 us of idle GPU after every polled tile-count and all-gather wait of the bucket
// exchange -- 0.2 ms of a 2^27-key rank's 1.7 ms.)
struct PollPause {
    static constexpr double POLL_SPIN_MS = 20.0;
    double t0 = -1.0;
    void operator()();
};
// Largest log2 fan-in of one merge pass: the option, else the key type's default.
int max_logf(const dsort_opts &opt, int type_default, int type_cap);

// ----------------------------------------------------------------------------------------
// Bucket exchange (the multi-GPU sample sort): every rank cuts its UNSORTED keys
// into Btot = P * Bl global buckets by splitters taken from every rank's samples (the first
// partition level of the one-GPU sort, with global splitters), ships buckets [q Bl, (q+1) Bl) to
// rank q, and finishes its own Bl buckets with the second level and the tile sort -- the received
// pieces of a bucket are its chunks.  No sorted runs are merged anywhere.
// ----------------------------------------------------------------------------------------
struct BxSample {  // a splitter sample: key (sign-extended) and position in its rank's keys
    int64_t k;
    uint64_t i;
};
struct BxPlan {
    int P, me, Bl, Btot;
    uint64_t n_local, n_total;
    uint32_t s_max;                 // sample records per rank (the all-gather's unit)
    uint64_t recv_room;             // keys the partition buffer holds past this rank's own: the
                                    // other ranks' pieces land there (no copy of its own buckets)
    std::vector<uint64_t> n_of;     // keys of every rank
    std::vector<uint64_t> ioff;     // composite index of every rank's first key (prefix of n_of)
    std::vector<uint32_t> s_of;     // real samples of every rank (the rest of its s_max: padding)
};
// The plan from every rank's key count; false when the bucket exchange does not apply (too few
// keys, the second level or the partition switched off): the caller takes the sort-then-merge path.
bool bx_make_plan(const dsort_opts &opt, int P, int me, const uint64_t *n_of, int key_bytes, BxPlan &plan);
// 1. this rank's s_of[me] regular samples of d_in into d_smp (s_max records, the rest padded)
template <typename T>
int bx_sample(dsort_ctx *ctx, const T *d_in, const BxPlan &pl, BxSample *d_smp, hipStream_t s);
// 2. the global splitters from every rank's records (d_all: P * s_max), then the first partition
//    level of d_in into ctx->scratch (bucket-major, Btot buckets; recv_room more keys fit behind
//    them).  *hb = this rank's bucket starts (host, Btot + 1), *part = the partitioned keys.  Kill
//    stage 0 fires here.
//    pure[g] (Btot): global bucket g lies between two splitters of one key.  Its keys are dropped
//    (DSORT_BX_DROP_PURE, round 6): part holds the others at the compacted starts -- every pure
//    bucket of size 0 -- and the owner fills a pure bucket with its key, so its keys never cross
//    the links.
template <typename T>
int bx_partition(dsort_ctx *ctx, const T *d_in, const BxPlan &pl, const BxSample *d_all, hipStream_t s, bool timed,
                 const uint64_t **hb, T **part, std::vector<uint8_t> &pure);
// 3. after the exchange: src holds the pieces of this rank's buckets from every source r, source
//    r's in bucket order from src[base[r]] on (base: of the wave's first bucket);
//    hb_all[r * (Btot + 1) + g] = source r's bucket starts, hc_all its compacted starts (the pieces'
//    positions: a pure bucket has none).  Sorts them into out (nrecv keys; src holds at least nrecv
//    keys: the second level's scratch).  Kill stages 1 and 2 fire here.
//    The buckets [j_lo, j_hi) of this rank (wave w of W) into out + out_off; *n_out = their keys.
template <typename T>
int bx_local_sort(dsort_ctx *ctx, T *src, T *out, const BxPlan &pl, const uint64_t *hb_all, const uint64_t *hc_all,
                  const uint64_t *base, int j_lo, int j_hi, uint64_t out_off, int w, int W, hipStream_t s,
                  bool timed, uint64_t *n_out);

}  // namespace dsort

#define DSORT_HIP(ctx, call)                                      \
    do {                                                          \
        hipError_t e_ = (call);                                   \
        if (e_ != hipSuccess) return dsort::hip_err((ctx), e_, #call); \
    } while (0)
