// dsort_sort.hip -- entry points of the worker sort and the master merge inside libdsort, and the
// pieces every driver shares (fault injection, fan-in cap).
//
// Replaces merge_sort()/merge() (reference client.c:140-173) and the merge loop of
// merge_chunks() (reference server.c:481-515).  Same result: the input multiset in ascending
// signed order; equal keys from different runs are emitted lower run first, like the reference's
// `<=` (client.c:152) and lowest-index-wins argmin (server.c:504) -- unobservable for keys-only
// data.  Both key widths run on the wave-register kernels of dsort_wave.hip.
#include <hip/hip_runtime.h>

#include <stdint.h>

#include <csignal>
#include <type_traits>

#include "dsort_internal.h"

namespace dsort {

int max_logf(const dsort_ctx *ctx, int type_default, int type_cap) {
    const int64_t o = ctx->opt.max_logf;
    const int x = o < 0 ? type_default : (int)o;
    return x < 1 ? 1 : (x > type_cap ? type_cap : x);
}

void fault_point(dsort_ctx *ctx, hipStream_t s, int pass_done) {
    if (ctx->nested == 0 && ctx->opt.kill_after_pass >= 0 && ctx->opt.kill_after_pass == pass_done) {
        (void)hipStreamSynchronize(s);
        raise(SIGKILL);
    }
}

template <typename T>
int sort_device(dsort_ctx *ctx, const T *d_in, T *d_keys, size_t n, hipStream_t s, bool timed) {
    if constexpr (std::is_same<T, int32_t>::value) return wave_sort_i32(ctx, d_in, d_keys, n, s, timed);
    else return wave_sort_i64(ctx, d_in, d_keys, n, s, timed);
}

// k-way merge of back-to-back runs of arbitrary lengths (the master merge, server.c:481-515,
// and the multi-GPU receive merge); lower runs win ties at every level.
template <typename T>
int merge_device(dsort_ctx *ctx, const T *d_in, const size_t *lens, int k, T *d_out, hipStream_t s,
                 bool keep_stats) {
    if constexpr (std::is_same<T, int32_t>::value) return wave_merge_i32(ctx, d_in, lens, k, d_out, s, keep_stats);
    else return wave_merge_i64(ctx, d_in, lens, k, d_out, s, keep_stats);
}

template int sort_device<int32_t>(dsort_ctx *, const int32_t *, int32_t *, size_t, hipStream_t, bool);
template int sort_device<int64_t>(dsort_ctx *, const int64_t *, int64_t *, size_t, hipStream_t, bool);
template int merge_device<int32_t>(dsort_ctx *, const int32_t *, const size_t *, int, int32_t *, hipStream_t,
                                   bool);
template int merge_device<int64_t>(dsort_ctx *, const int64_t *, const size_t *, int, int64_t *, hipStream_t,
                                   bool);

}  // namespace dsort
