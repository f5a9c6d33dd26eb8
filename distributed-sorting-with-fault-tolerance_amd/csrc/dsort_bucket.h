// dsort_bucket.h -- the int32 sort with a sample-splitter partition pass in front (included by
// dsort_wave.hip inside namespace dsort::wv; uses its tile sort and k-way pass kernels).
//
// The multi-GPU design cuts the keys into key ranges with sample-sort splitters and sorts every
// range on its own GPU.  The same idea inside one GPU's HBM: B buckets (about
// 2^21 keys each) by splitters taken from a regular sample, in (key, input index) order so that
// duplicates are spread over buckets like any other key; one partition pass writes every bucket
// contiguously; then the tile sort and the k-way merge passes run inside every bucket.  A
// partition pass resolves log2(B) bits of the order in about one read + one write of the keys
// (plus a read for the histogram), where a merge pass resolves log2(F) = 4: at 2^30 keys the
// 16 bits of merging above the 16384-key tiles become 9 bits of partition + 7 bits of merging,
// 2 merge passes instead of 4.
//
// Kernels (all keyed by the composite c = key * 2^32 + input index, unique per key):
//   bucket_sample_kernel   s regular samples -> composites (sorted by the int64 sort)
//   bucket_splitter_kernel splitter b = sample (b+1)*s/B - 1; padded with +inf to BP
//   bucket_hist_kernel     per 65536-key workgroup: keys per bucket (LDS atomics)
//   bucket_colsum_kernel   per 64 workgroups: column sums        } exclusive scan of the
//   bucket_scan_kernel     one workgroup: chunk prefixes, bucket   } histograms in (bucket,
//                          starts, tile table of the tile sort     }  workgroup) order
//   bucket_offsets_kernel  per-workgroup bucket offsets          }
//   bucket_scatter_kernel  per 16384-key sub-tile: keys grouped by bucket in LDS, then written
//                          to their buckets (consecutive lanes on consecutive keys of a bucket)
#pragma once

constexpr int BK_T = 1024;               // threads of the partition kernels
constexpr int BK_K = 16;                 // keys per thread per sub-tile
constexpr int BK_SUB = BK_T * BK_K;      // 16384 keys per sub-tile
constexpr int BK_SUBS = 4;               // sub-tiles per workgroup
constexpr int BK_WG = BK_SUB * BK_SUBS;  // 65536 keys per partition workgroup
constexpr int BK_MAXB = 1024;            // buckets at most (<= threads, one bucket per thread)
constexpr int BK_OS = 32;                // samples per bucket
constexpr int BK_CHUNK = 64;             // workgroups per column-sum chunk

struct TileRef {
    uint64_t base;   // first key of the tile
    uint32_t valid;  // keys in the tile (<= TILE)
    uint32_t pad;
};

__device__ __forceinline__ int64_t composite(int32_t key, uint64_t idx) {
    return (int64_t)((uint64_t)(int64_t)key << 32 | (uint32_t)idx);
}

// bucket of composite c: the number of splitters below c (spl holds BP entries, +inf padded)
__device__ __forceinline__ int bucket_of(const int64_t *spl, int BP, int64_t c) {
    int lo = 0;
    for (int st = BP >> 1; st >= 1; st >>= 1) lo += spl[lo + st - 1] < c ? st : 0;
    return lo;
}

// Radix-assisted lookup: slot = top BK_SLOTB bits of the (sign-flipped) key; rng[slot] packs
// the number of splitters whose key lies below the slot (low 16 bits) and below the next slot
// (high 16 bits).  Only splitters inside the key's slot need a comparison -- usually none or
// one -- instead of a log2(B)-step search with bank conflicts on every step.
constexpr int BK_SLOTB = 12;
constexpr int BK_SLOTS = 1 << BK_SLOTB;

__device__ __forceinline__ void build_slots(const int64_t *spl, int BP, uint32_t *rng) {
    for (int i = threadIdx.x; i < BK_SLOTS; i += blockDim.x) {
        uint32_t cnt[2];
#pragma unroll
        for (int e = 0; e < 2; ++e) {
            // splitters with key < (slot i + e) start, as a composite: key * 2^32 + 0
            const uint64_t su = (uint64_t)(i + e) << (32 - BK_SLOTB);  // biased key of the start
            const int64_t c = i + e == BK_SLOTS ? INT64_MAX
                                                : (int64_t)((uint64_t)((uint32_t)su ^ 0x80000000u) << 32);
            cnt[e] = (uint32_t)bucket_of(spl, BP, c);
        }
        rng[i] = cnt[0] | (cnt[1] << 16);
    }
}

__device__ __forceinline__ int bucket_fast(const int64_t *spl, const uint32_t *rng, int32_t key,
                                           int64_t c) {
    const uint32_t r = rng[((uint32_t)key ^ 0x80000000u) >> (32 - BK_SLOTB)];
    int lo = (int)(r & 0xFFFF), hi = (int)(r >> 16);
    while (lo < hi) {  // lower bound among the splitters of the slot
        const int mid = (lo + hi) >> 1;
        if (spl[mid] < c) lo = mid + 1;
        else hi = mid;
    }
    return lo;
}

__global__ void __launch_bounds__(256) bucket_sample_kernel(const int32_t *__restrict__ in,
                                                            uint64_t n, int64_t *__restrict__ smp,
                                                            uint32_t s) {
    const uint32_t k = blockIdx.x * 256 + threadIdx.x;
    if (k >= s) return;
    const uint64_t pos = ((2 * (uint64_t)k + 1) * n) / (2 * (uint64_t)s);
    smp[k] = composite(in[pos], pos);
}

__global__ void __launch_bounds__(BK_MAXB) bucket_splitter_kernel(const int64_t *__restrict__ smp,
                                                                 int B, int BP,
                                                                 int64_t *__restrict__ spl) {
    const int b = threadIdx.x;
    if (b < BP) spl[b] = b < B - 1 ? smp[(uint64_t)(b + 1) * BK_OS - 1] : INT64_MAX;
}

__device__ __forceinline__ void load_splitters(const int64_t *spl_g, int BP, int64_t *spl) {
    for (int b = threadIdx.x; b < BP; b += BK_T) spl[b] = spl_g[b];
}

// counts[g * B + b] = keys of workgroup g's 65536 keys in bucket b
__global__ void __launch_bounds__(BK_T) bucket_hist_kernel(const int32_t *__restrict__ in,
                                                           uint64_t n,
                                                           const int64_t *__restrict__ spl_g,
                                                           int B, int BP,
                                                           uint32_t *__restrict__ counts) {
    __shared__ int64_t spl[BK_MAXB];
    __shared__ uint32_t rng[BK_SLOTS];
    __shared__ uint32_t hist[BK_MAXB];
    load_splitters(spl_g, BP, spl);
    for (int b = threadIdx.x; b < B; b += BK_T) hist[b] = 0;
    __syncthreads();
    build_slots(spl, BP, rng);
    __syncthreads();
    const uint64_t g0 = (uint64_t)blockIdx.x * BK_WG;
#pragma unroll 1
    for (int sub = 0; sub < BK_SUBS; ++sub) {
        const uint64_t b0 = g0 + (uint64_t)sub * BK_SUB + threadIdx.x;
        int32_t key[BK_K];
#pragma unroll
        for (int k = 0; k < BK_K; ++k) {
            const uint64_t i = b0 + (uint64_t)k * BK_T;
            key[k] = i < n ? in[i] : 0;
        }
#pragma unroll
        for (int k = 0; k < BK_K; ++k) {
            const uint64_t i = b0 + (uint64_t)k * BK_T;
            if (i < n) atomicAdd(&hist[bucket_fast(spl, rng, key[k], composite(key[k], i))], 1u);
        }
    }
    __syncthreads();
    for (int b = threadIdx.x; b < B; b += BK_T) counts[(uint64_t)blockIdx.x * B + b] = hist[b];
}

// part[c * B + b] = sum of counts[g * B + b] over the BK_CHUNK workgroups g of chunk c
__global__ void __launch_bounds__(BK_MAXB) bucket_colsum_kernel(const uint32_t *__restrict__ counts,
                                                               uint32_t G, int B,
                                                               uint64_t *__restrict__ part) {
    const int b = threadIdx.x;
    if (b >= B) return;
    const uint32_t g0 = blockIdx.x * BK_CHUNK;
    const uint32_t g1 = g0 + BK_CHUNK < G ? g0 + BK_CHUNK : G;
    uint64_t sum = 0;
    for (uint32_t g = g0; g < g1; ++g) sum += counts[(uint64_t)g * B + b];
    part[(uint64_t)blockIdx.x * B + b] = sum;
}

// Tiles of a bucket [sk, sk + len): a head tile up to the next 4-key boundary (0..3 keys), then
// TILE-key tiles from there, so every other tile starts 16-byte aligned (the tile sort's
// 16-byte loads).  The host plans the merge passes with the same rule (bucket_tiles).
__host__ __device__ __forceinline__ uint64_t bucket_head(uint64_t sk, uint64_t len) {
    const uint64_t h = (4 - (sk & 3)) & 3;
    return h < len ? h : len;
}
__host__ __device__ __forceinline__ uint64_t bucket_tiles(uint64_t sk, uint64_t len) {
    const uint64_t h = bucket_head(sk, len);
    return (h ? 1 : 0) + (len - h + TILE - 1) / TILE;
}

// exclusive scan of one value per thread over a BK_MAXB-thread workgroup; `all` = total
__device__ __forceinline__ uint64_t scan_excl_u64(uint64_t v, uint64_t *wsum, uint64_t &all) {
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    uint64_t incl = v;
    for (int o = 1; o < 64; o <<= 1) {
        const uint64_t y = __shfl_up(incl, o);
        if (lane >= o) incl += y;
    }
    __syncthreads();
    if (lane == 63) wsum[w] = incl;
    __syncthreads();
    uint64_t off = 0;
    all = 0;
    for (int i = 0; i < BK_MAXB / 64; ++i) {
        if (i < w) off += wsum[i];
        all += wsum[i];
    }
    return off + incl - v;
}

// One workgroup: part -> exclusive prefix over chunks (in place); bucket starts bstart[0..B];
// the tile table of the tile sort (every bucket cut into tiles, bucket_tiles) and its size.
__global__ void __launch_bounds__(BK_MAXB) bucket_scan_kernel(uint64_t *__restrict__ part,
                                                             uint32_t nchunk, int B,
                                                             uint64_t *__restrict__ bstart,
                                                             uint32_t *__restrict__ tpre,
                                                             TileRef *__restrict__ tt,
                                                             uint32_t *__restrict__ ntiles) {
    __shared__ uint64_t wsum[BK_MAXB / 64];
    const int b = threadIdx.x;
    uint64_t tot = 0;
    if (b < B) {
        for (uint32_t c = 0; c < nchunk; ++c) {
            const uint64_t v = part[(uint64_t)c * B + b];
            part[(uint64_t)c * B + b] = tot;
            tot += v;
        }
    }
    uint64_t allk, allt;
    const uint64_t sk = scan_excl_u64(tot, wsum, allk);
    const uint64_t nt = b < B ? bucket_tiles(sk, tot) : 0;
    const uint64_t st = scan_excl_u64(nt, wsum, allt);
    if (b < B) {
        bstart[b] = sk;
        tpre[b] = (uint32_t)st;
        const uint64_t h = bucket_head(sk, tot);
        uint64_t k = st;
        if (h) tt[k++] = TileRef{sk, (uint32_t)h, 0};
        for (uint64_t base = sk + h; base < sk + tot; base += TILE) {
            const uint64_t rem = sk + tot - base;
            tt[k++] = TileRef{base, (uint32_t)(rem < (uint64_t)TILE ? rem : TILE), 0};
        }
    }
    if (b == 0) {
        bstart[B] = allk;
        tpre[B] = (uint32_t)allt;
        *ntiles = (uint32_t)allt;
    }
}

// offs[g * B + b] = global position of workgroup g's first key of bucket b
__global__ void __launch_bounds__(BK_MAXB) bucket_offsets_kernel(const uint32_t *__restrict__ counts,
                                                                const uint64_t *__restrict__ part,
                                                                const uint64_t *__restrict__ bstart,
                                                                uint32_t G, int B,
                                                                uint64_t *__restrict__ offs) {
    const int b = threadIdx.x;
    if (b >= B) return;
    const uint32_t g0 = blockIdx.x * BK_CHUNK;
    const uint32_t g1 = g0 + BK_CHUNK < G ? g0 + BK_CHUNK : G;
    uint64_t run = bstart[b] + part[(uint64_t)blockIdx.x * B + b];
    for (uint32_t g = g0; g < g1; ++g) {
        offs[(uint64_t)g * B + b] = run;
        run += counts[(uint64_t)g * B + b];
    }
}

// Per 16384-key sub-tile: every key takes a slot of its bucket in LDS (atomic on the sub-tile
// histogram), the sub-tile is laid out bucket by bucket, and consecutive threads write
// consecutive keys of a bucket to its global range.  The order of keys inside a bucket is not
// kept (the bucket is sorted afterwards; the keys carry no payload).
__global__ void __launch_bounds__(BK_T) bucket_scatter_kernel(const int32_t *__restrict__ in,
                                                              uint64_t n,
                                                              const int64_t *__restrict__ spl_g,
                                                              int B, int BP,
                                                              const uint64_t *__restrict__ offs,
                                                              int32_t *__restrict__ out) {
    __shared__ int64_t spl[BK_MAXB];
    __shared__ uint32_t rng[BK_SLOTS];
    __shared__ uint64_t goff[BK_MAXB];   // next global position of each bucket (this workgroup)
    __shared__ uint32_t hist[BK_MAXB];   // sub-tile histogram, then its exclusive scan
    __shared__ uint32_t wsum[BK_T / 64];
    __shared__ int32_t lk[BK_SUB];       // the sub-tile grouped by bucket
    __shared__ uint16_t lb[BK_SUB];      // bucket of every LDS slot
    load_splitters(spl_g, BP, spl);
    for (int b = threadIdx.x; b < B; b += BK_T) goff[b] = offs[(uint64_t)blockIdx.x * B + b];
    __syncthreads();
    build_slots(spl, BP, rng);
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const uint64_t g0 = (uint64_t)blockIdx.x * BK_WG;
    // keys of the next sub-tile are loaded while the current one is placed (software pipeline)
    int32_t nxt[BK_K];
#pragma unroll
    for (int k = 0; k < BK_K; ++k) {
        const uint64_t i = g0 + threadIdx.x + (uint64_t)k * BK_T;
        nxt[k] = i < n ? in[i] : 0;
    }
#pragma unroll 1
    for (int sub = 0; sub < BK_SUBS; ++sub) {
        const uint64_t s0 = g0 + (uint64_t)sub * BK_SUB;
        if (s0 >= n) break;  // workgroup-uniform
        for (int b = threadIdx.x; b < B; b += BK_T) hist[b] = 0;
        __syncthreads();
        int32_t key[BK_K];
        int bk[BK_K];
        uint32_t slot[BK_K];
#pragma unroll
        for (int k = 0; k < BK_K; ++k) key[k] = nxt[k];
        if (sub + 1 < BK_SUBS) {
#pragma unroll
            for (int k = 0; k < BK_K; ++k) {
                const uint64_t i = s0 + BK_SUB + threadIdx.x + (uint64_t)k * BK_T;
                nxt[k] = i < n ? in[i] : 0;
            }
        }
#pragma unroll
        for (int k = 0; k < BK_K; ++k) {
            const uint64_t i = s0 + threadIdx.x + (uint64_t)k * BK_T;
            bk[k] = -1;
            if (i < n) {
                bk[k] = bucket_fast(spl, rng, key[k], composite(key[k], i));
                slot[k] = atomicAdd(&hist[bk[k]], 1u);
            }
        }
        __syncthreads();
        // exclusive scan of the sub-tile histogram (one bucket per thread)
        const uint32_t hv = threadIdx.x < (unsigned)B ? hist[threadIdx.x] : 0;
        uint32_t incl = hv;
        for (int o = 1; o < 64; o <<= 1) {
            const uint32_t y = __shfl_up(incl, o);
            if (lane >= o) incl += y;
        }
        if (lane == 63) wsum[w] = incl;
        __syncthreads();
        uint32_t woff = 0;
        for (int i = 0; i < w; ++i) woff += wsum[i];
        if (threadIdx.x < (unsigned)B) hist[threadIdx.x] = woff + incl - hv;
        __syncthreads();
#pragma unroll
        for (int k = 0; k < BK_K; ++k) {
            if (bk[k] >= 0) {
                const uint32_t p = hist[bk[k]] + slot[k];
                lk[p] = key[k];
                lb[p] = (uint16_t)bk[k];
            }
        }
        __syncthreads();
        const uint32_t cnt = s0 + BK_SUB <= n ? BK_SUB : (uint32_t)(n - s0);
#pragma unroll
        for (int k = 0; k < BK_K; ++k) {
            const uint32_t p = threadIdx.x + k * BK_T;
            if (p < cnt) {
                const int b = lb[p];
                out[goff[b] + (p - hist[b])] = lk[p];
            }
        }
        __syncthreads();
        // advance every bucket's global position by this sub-tile's keys
        if (threadIdx.x < (unsigned)B) {
            const uint32_t nxt = threadIdx.x + 1 < (unsigned)B ? hist[threadIdx.x + 1] : cnt;
            goff[threadIdx.x] += nxt - hist[threadIdx.x];
        }
        __syncthreads();
    }
}
