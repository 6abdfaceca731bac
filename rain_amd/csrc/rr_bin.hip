// rr_bin.hip — binning without a per-frame depth sort.
//
// The reference sorts 64-bit (tile << 32 | depth bits) keys emitted in Gaussian index order
// (rasterizer_impl.cu:59-100, 292-300), so every tile's list is in (depth, index) order.  Rounds
// 1-3 of this build got that order from a global stable depth sort of the P Gaussians (3 radix
// passes = 9 launches per frame) followed by a stable bin sort of the pairs emitted in depth order.
// Here the pairs are emitted in INDEX order, stable-sorted by bin id only (rr_sort.hip, 2 passes),
// and every bin's run — index-ordered, ~10^3 pairs — is sorted by depth inside one workgroup
// (k_sortexpand: stable LSD radix sort in LDS on the Gaussian's depth key), which yields the same
// (depth, index) order per bin, and so per tile, at a fraction of the launches.
//
// Early-stop binning (rr_kernels.hpp BlendPhase) splits the pairs by DEPTH instead of by depth
// rank: phase A holds the pairs of the Gaussians nearer than a cut chosen per frame from a sampled,
// pair-weighted depth histogram (~1/den of the pairs), phase B the others.  Each tile's phase-A
// list is then a prefix of its full depth-ordered list and the B list the rest, which is all the
// two-phase blend needs (any cut gives the full lists' outputs).
//
//   k_split_scan_totals  per block of Gaussians: the frame totals from the preprocess block sums
//                        and the depth cut from sampled {depth key, pairs} (every workgroup, the
//                        same cut; workgroup 0 publishes the frame's total pairs to the host,
//                        rr_api.hip mailbox), then the block's {A pairs, B pairs} totals
//   k_split_scan         inclusive scan of {A pairs, B pairs} per Gaussian in index order; its last
//                        thread leaves the phases' counts in FrameTotals (device-side only)
//   k_sortexpand<K>    per bin: depth sort of its run + the split into its four tiles' lists
#include <algorithm>

#include "rr_common.hpp"
#include "rr_kernels.hpp"
#include "rr_sortexpand.hpp"

namespace rr {

// ---- the depth cut of early-stop binning ------------------------------------------------------
// Pair-weighted histogram of the sampled Gaussians' depth keys (key >> kCutShift, 4096 buckets over
// the 27-bit key range; deeper keys share the last bucket), then the first bucket whose inclusive
// prefix reaches 1/den of the sampled pairs: phase A takes the keys below that bucket's end.
// den <= 1, a frame below min_pairs pairs or no sampled pair: cut = all ones (one phase).
constexpr int kCutBuckets = 4096;
constexpr int kCutShift = kDepthKeyBits - 12;
// Per-bucket sums fit 32 bits: <= 4096 samples of at most 2^18 bins each.
constexpr int kCutSamples = 4096;

// Clears the image buffer's per-frame block (tile ranges, counters, open bits, bin runs and counts:
// rr_api.hip carve_img) in a grid-stride loop, 16 B per store (a carved array: 16-B aligned).
__device__ __forceinline__ void clear_words(uint32_t* __restrict__ zero, int nzero) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x, nth = gridDim.x * blockDim.x;
    const int nv = nzero >> 2;
    for (int j = i; j < nv; j += nth) reinterpret_cast<uint4*>(zero)[j] = make_uint4(0u, 0u, 0u, 0u);
    for (int j = 4 * nv + i; j < nzero; j += nth) zero[j] = 0u;
}

// The samples: NS / 64 evenly spaced runs of 64 consecutive Gaussians (every Gaussian up to
// NS): a wave's 64 lanes read one run's keys and pair counts as two contiguous 256-B and
// 512-B pieces, so the one workgroup gathers its 4096 samples from ~400 cache lines instead of ~8000
// scattered ones (which took a separate many-workgroup launch: 4.4 us).  Runs of consecutive
// indices are as good a sample as evenly spaced Gaussians here: the cut only steers the split's
// balance, any cut gives the same lists.

// The frame's totals (L, rect, wide: the preprocess block sums) and the depth cut, computed by one
// workgroup of NT threads — every workgroup of the split scan's first launch, each from the same
// inputs by the same steps: the same cut.
template <int NT>
struct CutShared {
    uint32_t hist[kCutBuckets];
    unsigned long long red[3][NT / 64];
    uint32_t wide, cut;
};
struct CutResult {
    unsigned long long L, rect;
    uint32_t wide, cut;  // cut: all ones for a one-phase frame
};
template <int NT, int NS = kCutSamples>
__device__ __forceinline__ CutResult depth_cut(CutShared<NT>& sh, int P, const uint32_t* __restrict__ keys,
                                               const uint2* __restrict__ tiles, const uint2* __restrict__ block_sums,
                                               const uint32_t* __restrict__ block_wide, int nb, uint32_t den,
                                               uint32_t min_pairs) {
    static_assert(NS % NT == 0 && NS % 64 == 0 && NS <= kCutSamples, "samples: runs of 64, whole rounds");
    constexpr int SPT = NS / NT;           // samples per thread
    constexpr int QB = kCutSamples / NT;   // block records per thread and round (all in flight)
    constexpr int NCH = NS / 64;           // runs of 64 consecutive Gaussians
    constexpr int NW = NT / 64;
    const int t = threadIdx.x, lane = t & 63, w = t >> 6;
    for (int i = t; i < kCutBuckets; i += NT) sh.hist[i] = 0u;
    if (t == 0) {
        sh.wide = 0u;
        sh.cut = 0xffffffffu;
    }
    // every sample load in flight before the first LDS atomic
    uint2 sm[SPT];
#pragma unroll
    for (int r = 0; r < SPT; r++) {
        const int s = t + r * NT;
        const int idx = P <= NS ? min(s, P - 1) : min((int)(((long long)(s >> 6) * P) / NCH) + (s & 63), P - 1);
        sm[r] = make_uint2(keys[idx], tiles[idx].x);
        if (P <= NS && s >= P) sm[r].y = 0u;
    }
    unsigned long long L = 0, rect = 0, S = 0;
    uint32_t wide = 0;
    for (int i0 = 0; i0 < nb; i0 += QB * NT) {
        uint2 v[QB];
        uint32_t wd[QB];
#pragma unroll
        for (int q = 0; q < QB; q++) {
            const int i = min(i0 + q * NT + t, nb - 1);
            v[q] = block_sums[i];
            wd[q] = block_wide[i];
        }
#pragma unroll
        for (int q = 0; q < QB; q++)
            if (i0 + q * NT + t < nb) {
                L += v[q].x;
                rect += v[q].y;
                wide |= wd[q];
            }
    }
    __syncthreads();
#pragma unroll
    for (int r = 0; r < SPT; r++)
        if (sm[r].y) {
            const uint32_t n = min(sm[r].y, 1u << 18);
            atomicAdd(&sh.hist[min(sm[r].x >> kCutShift, (uint32_t)kCutBuckets - 1u)], n);
            S += n;
        }
    if (wide) atomicOr(&sh.wide, 1u);
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        L += __shfl_xor(L, o);
        rect += __shfl_xor(rect, o);
        S += __shfl_xor(S, o);
    }
    if (lane == 0) {
        sh.red[0][w] = L;
        sh.red[1][w] = rect;
        sh.red[2][w] = S;
    }
    __syncthreads();
    L = rect = S = 0;
#pragma unroll
    for (int i = 0; i < NW; i++) {
        L += sh.red[0][i];
        rect += sh.red[1][i];
        S += sh.red[2][i];
    }
    const bool one_phase = den <= 1u || L < (unsigned long long)min_pairs || S == 0ull;
    if (!one_phase) {
        // BPT buckets per thread, block-wide inclusive scan of their sums
        constexpr int BPT = kCutBuckets / NT;
        unsigned long long v[BPT], sum = 0;
#pragma unroll
        for (int k = 0; k < BPT; k++) {
            v[k] = sh.hist[BPT * t + k];
            sum += v[k];
        }
        unsigned long long incl = sum;
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
            const unsigned long long y = __shfl_up(incl, o);
            if (lane >= o) incl += y;
        }
        __syncthreads();  // sh.red reads above are done
        if (lane == 63) sh.red[0][w] = incl;
        __syncthreads();
        unsigned long long run = incl - sum;
        for (int i = 0; i < w; i++) run += sh.red[0][i];
        // first bucket whose inclusive prefix reaches S / den (prefix * den >= S)
#pragma unroll
        for (int k = 0; k < BPT; k++) {
            run += v[k];
            if (run * den >= S) {
                const uint32_t b = (uint32_t)(BPT * t + k);
                atomicMin(&sh.cut, b + 1u >= (uint32_t)kCutBuckets ? 0xffffffffu : (b + 1u) << kCutShift);
                break;
            }
        }
    }
    __syncthreads();
    return CutResult{L, rect, sh.wide, one_phase ? 0xffffffffu : sh.cut};
}

// The frame's counts and cut into FrameTotals, and to the host (rr_api.hip pair_counts_wait) now,
// while the split scan runs: the host sizes the binning by the total and leaves the phases' split
// on the device.  One thread.
__device__ __forceinline__ void publish_cut(const CutResult& r, FrameTotals* ft, uint32_t* box, uint32_t seq) {
    ft->L = r.L;
    ft->rect = r.rect;
    ft->wide = r.wide;
    ft->cut = r.cut;
    if (box) {
        const uint32_t sat = 0xffffffffu;
        __hip_atomic_store(box + 0, r.L > sat ? sat : (uint32_t)r.L, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        __hip_atomic_store(box + 1, r.rect > sat ? sat : (uint32_t)r.rect, __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_SYSTEM);
        __hip_atomic_store(box + 3, r.wide, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        // The host reads only the mailbox words, which the system-scope stores above write
        // through to host memory (sc0 sc1): waiting for their completion orders them before the
        // sequence number.  A release store here would also write back every dirty line of this
        // XCD's L2 (buffer_wbl2: megabytes after the backward's streaming writes), which nothing
        // the host reads needs.
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __hip_atomic_store(box + 2, seq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    }
}

// ---- the phases' Gaussian lists: scan of {A pairs, B pairs, A rows, B rows} in index order ------
// Gaussian i has n_i bin pairs; it belongs to phase A if n_i > 0 and its depth key < cut, to phase B
// if n_i > 0 otherwise.  One inclusive scan of the four counts gives every phase's list in index
// order: list_X[r] = {Gaussian index, inclusive pair offset} of the phase's r-th Gaussian — what
// the duplicate walks (its windows cover consecutive pairs of one list, so a window visits only the
// Gaussians it emits for, as the depth-ordered lists of rounds 1-3 did).  Pair offsets saturate at
// 2^32 - 1 (the host rejects totals above 2^29).  Blocks of kPairScanItems; the block totals are
// summed by every later block (2 launches) or first scanned by one workgroup (large P).
struct Quad {
    unsigned long long pa, pb, ca, cb;
};
__device__ __forceinline__ Quad quad_add(Quad x, Quad y) { return Quad{x.pa + y.pa, x.pb + y.pb, x.ca + y.ca, x.cb + y.cb}; }
__device__ __forceinline__ Quad quad_shfl_up(Quad x, int o) {
    return Quad{__shfl_up(x.pa, o), __shfl_up(x.pb, o), __shfl_up(x.ca, o), __shfl_up(x.cb, o)};
}
__device__ __forceinline__ Quad quad_shfl_xor(Quad x, int o) {
    return Quad{__shfl_xor(x.pa, o), __shfl_xor(x.pb, o), __shfl_xor(x.ca, o), __shfl_xor(x.cb, o)};
}
__device__ __forceinline__ Quad split_item(const uint2* tiles, const uint32_t* keys, uint32_t cut, size_t i) {
    const uint32_t n = tiles[i].x;
    const bool a = keys[i] < cut;
    return Quad{a ? n : 0ull, a ? 0ull : n, (a && n) ? 1ull : 0ull, (!a && n) ? 1ull : 0ull};
}
// block-wide sum of one Quad per thread (256 threads); s: [4] Quads
__device__ __forceinline__ Quad quad_block_sum(Quad x, Quad* s) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) x = quad_add(x, quad_shfl_xor(x, o));
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    __syncthreads();
    if (lane == 0) s[w] = x;
    __syncthreads();
    return quad_add(quad_add(s[0], s[1]), quad_add(s[2], s[3]));
}

// The depth cut computed here by every workgroup (depth_cut<256>: the same cut in each) and
// published by workgroup 0 (no launch of its own).  Each workgroup samples kCutScanSamples
// Gaussians (16 runs of 64: the cut only steers the phases' balance, and the per-workgroup
// histogram is 4x cheaper than 4096 samples).
constexpr int kCutScanSamples = 1024;
__global__ __launch_bounds__(256) void k_split_scan_totals(const uint2* __restrict__ tiles,
                                                           const uint32_t* __restrict__ keys, int P,
                                                           FrameTotals* __restrict__ ft, Quad* __restrict__ tot,
                                                           uint32_t* __restrict__ zero, int nzero, CutArgs ca) {
    __shared__ Quad s[4];
    __shared__ CutShared<256> sh;
    // this block's items first: their loads overlap the cut's
    constexpr int IPT = kPairScanItems / 256;
    const size_t b0 = (size_t)blockIdx.x * kPairScanItems;
    uint32_t in[IPT], ik[IPT];
#pragma unroll
    for (int r = 0; r < IPT; r++) {
        const size_t i = b0 + (size_t)r * 256 + threadIdx.x;
        in[r] = i < (size_t)P ? tiles[i].x : 0u;
        ik[r] = i < (size_t)P ? keys[i] : 0u;
    }
    const CutResult r = depth_cut<256, kCutScanSamples>(sh, P, keys, tiles, ca.block_sums, ca.block_wide,
                                                        (P + 255) / 256, ca.den, ca.min_pairs);
    if (blockIdx.x == 0 && threadIdx.x == 0) publish_cut(r, ft, ca.box, ca.seq);
    const uint32_t cut = r.cut;
    if (zero) clear_words(zero, nzero);
    Quad x{0, 0, 0, 0};
#pragma unroll
    for (int r = 0; r < IPT; r++) {  // split_item's arithmetic on the prefetched values
        const bool a = ik[r] < cut;
        const uint32_t n = in[r];
        x = quad_add(x, Quad{a ? n : 0ull, a ? 0ull : n, (a && n) ? 1ull : 0ull, (!a && n) ? 1ull : 0ull});
    }
    x = quad_block_sum(x, s);
    if (threadIdx.x == 0) tot[blockIdx.x] = x;
}

// Exclusive scan, in place, of nb block totals (one workgroup; large P, where re-summing the earlier
// totals in every block would grow with nb^2).
__global__ __launch_bounds__(256) void k_split_scan_prefix(Quad* __restrict__ tot, int nb) {
    __shared__ Quad s_w[4];
    const int t = threadIdx.x, lane = t & 63, w = t >> 6;
    Quad carry{0, 0, 0, 0};
    for (int base = 0; base < nb; base += 256) {
        const int i = base + t;
        const Quad v = i < nb ? tot[i] : Quad{0, 0, 0, 0};
        Quad incl = v;
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
            const Quad y = quad_shfl_up(incl, o);
            if (lane >= o) incl = quad_add(incl, y);
        }
        __syncthreads();
        if (lane == 63) s_w[w] = incl;
        __syncthreads();
        Quad ex = quad_add(carry, Quad{incl.pa - v.pa, incl.pb - v.pb, incl.ca - v.ca, incl.cb - v.cb});
        for (int k = 0; k < w; k++) ex = quad_add(ex, s_w[k]);
        if (i < nb) tot[i] = ex;
        carry = quad_add(carry, quad_add(quad_add(s_w[0], s_w[1]), quad_add(s_w[2], s_w[3])));
    }
}

__device__ __forceinline__ uint32_t sat32(unsigned long long v) { return v > 0xffffffffull ? 0xffffffffu : (uint32_t)v; }

// The phases' counts stay on the device (the duplicate and sort launches read them from ft).
__device__ __forceinline__ void store_split(FrameTotals* ft, const Quad& q) {
    ft->LA = sat32(q.pa);
    ft->LB = sat32(q.pb);
    ft->GA = (uint32_t)q.ca;
    ft->GB = (uint32_t)q.cb;
}

// Entry r covers the pairs [a, b) of its phase: it is the first entry of every window of kSplitWin
// pairs that starts in that range (the duplicate's window starts, one launch less).
__device__ __forceinline__ void mark_windows(uint32_t* first, uint32_t nwin, unsigned long long a,
                                             unsigned long long b, uint32_t r) {
    for (unsigned long long k = (a + kSplitWin - 1) / kSplitWin; k * kSplitWin < b && k < nwin; k++)
        first[k] = r;
}

template <bool PREFIX>
__global__ __launch_bounds__(256) void k_split_scan(const uint2* __restrict__ tiles, const uint32_t* __restrict__ keys,
                                                    int P, const Quad* __restrict__ tot, PhaseLists lists,
                                                    FrameTotals* __restrict__ ft) {
    constexpr int IPT = kPairScanItems / 256;  // 8 consecutive items per thread
    __shared__ Quad s[4];
    __shared__ Quad s_w[4];
    const int t = threadIdx.x, lane = t & 63, w = t >> 6;
    const uint32_t cut = ft->cut;
    const size_t i0 = (size_t)blockIdx.x * kPairScanItems + (size_t)t * IPT;
    Quad v[IPT];
#pragma unroll
    for (int k = 0; k < IPT; k++) v[k] = i0 + k < (size_t)P ? split_item(tiles, keys, cut, i0 + k) : Quad{0, 0, 0, 0};
    Quad base{0, 0, 0, 0};
    if (PREFIX) {
        base = tot[blockIdx.x];
    } else {
        for (int j = t; j < (int)blockIdx.x; j += 256) base = quad_add(base, tot[j]);
        base = quad_block_sum(base, s);
    }
    Quad tsum{0, 0, 0, 0};
#pragma unroll
    for (int k = 0; k < IPT; k++) tsum = quad_add(tsum, v[k]);
    Quad incl = tsum;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const Quad y = quad_shfl_up(incl, o);
        if (lane >= o) incl = quad_add(incl, y);
    }
    if (lane == 63) s_w[w] = incl;
    __syncthreads();
    Quad ex = quad_add(base, Quad{incl.pa - tsum.pa, incl.pb - tsum.pb, incl.ca - tsum.ca, incl.cb - tsum.cb});
#pragma unroll
    for (int k = 0; k < 4; k++)
        if (k < w) ex = quad_add(ex, s_w[k]);
#pragma unroll
    for (int k = 0; k < IPT; k++) {
        const size_t i = i0 + k;
        const Quad e = ex;  // exclusive counts before item i
        ex = quad_add(ex, v[k]);
        if (v[k].ca) {
            lists.idx_a[e.ca] = (uint32_t)i;
            lists.off_a[e.ca] = sat32(ex.pa);
            mark_windows(lists.first_a, lists.nwin, e.pa, ex.pa, (uint32_t)e.ca);
        } else if (v[k].cb) {
            lists.idx_b[e.cb] = (uint32_t)i;
            lists.off_b[e.cb] = sat32(ex.pb);
            mark_windows(lists.first_b, lists.nwin, e.pb, ex.pb, (uint32_t)e.cb);
        }
    }
    // the last thread of the grid holds the frame's totals (items past P count as 0)
    if (blockIdx.x == gridDim.x - 1 && t == 255) store_split(ft, ex);
}

// the split scan's block totals
size_t split_scan_temp_bytes(int P) {
    return (size_t)std::max((P + kPairScanItems - 1) / kPairScanItems, 1) * sizeof(Quad);
}

void launch_split_scan(const uint2* tiles, const uint32_t* keys, int P, PhaseLists lists, FrameTotals* ft, void* temp,
                       int direct_blocks, uint32_t* zero, int nzero, const CutArgs& cut, hipStream_t st) {
    if (P <= 0) return;
    const int nb = (P + kPairScanItems - 1) / kPairScanItems;
    Quad* tot = static_cast<Quad*>(temp);
    k_split_scan_totals<<<nb, 256, 0, st>>>(tiles, keys, P, ft, tot, zero, nzero, cut);
    if (nb <= direct_blocks) {
        k_split_scan<false><<<nb, 256, 0, st>>>(tiles, keys, P, tot, lists, ft);
    } else {
        k_split_scan_prefix<<<1, 256, 0, st>>>(tot, nb);
        k_split_scan<true><<<nb, 256, 0, st>>>(tiles, keys, P, tot, lists, ft);
    }
}

// ---- per bin: depth order + the four tile lists (rr_sortexpand.hpp) ----------------------------
// per-bin runs longer than this go through the global path (Tuning::sx_lds_cap lowers it for tests)
uint32_t sx_lds_cap(int cap) {
    const int t = tuning().sx_lds_cap;
    return (uint32_t)(t >= 1 && t < cap ? t : cap);
}

// Phase B of the gather path (k_dup_gather emitted its pairs densely, [0, n), in no particular
// order): k_bin_count counts them per bin, k_bin_scatter turns the counts into every bin's run
// (bounds) and drops each pair's value into its bin's run (order inside a bin arbitrary:
// k_sortexpand restores (depth, index) order).  Two launches instead of the bin sort's five.  Count and
// scatter run kBinGroups workgroups over the same
// strided item sets; each aggregates its items per bin in LDS, so a global atomic is paid per
// (workgroup, bin) and not per pair (per-pair atomics on a few hot bins serialise: +40 us).
constexpr int kBinScanMax = 16384;  // bins one workgroup holds (4K frames: 8160)
constexpr int kBinGroups = 64;
__global__ __launch_bounds__(1024) void k_bin_count(const void* __restrict__ keys_v, int wide_keys,
                                                    const uint32_t* __restrict__ n_dev, int nb,
                                                    uint32_t* __restrict__ bin_cnt) {
    __shared__ uint32_t h[kBinScanMax];
    const int t = threadIdx.x;
    const uint32_t n = *n_dev;
    const uint32_t per = (n + kBinGroups - 1) / kBinGroups;
    const uint32_t i0 = blockIdx.x * per, i1 = min(n, i0 + per);
    if (i0 >= i1) return;
    for (int b = t; b < nb; b += 1024) h[b] = 0u;
    __syncthreads();
    for (uint32_t i = i0 + t; i < i1; i += 1024) {  // keys >= nb: the duplicate's unused reserved slots
        const uint32_t k = wide_keys ? static_cast<const uint32_t*>(keys_v)[i] : static_cast<const uint16_t*>(keys_v)[i];
        if (k < (uint32_t)nb) atomicAdd(&h[k], 1u);
    }
    __syncthreads();
    for (int b = t; b < nb; b += 1024)
        if (h[b]) atomicAdd(&bin_cnt[b], h[b]);
}

// The bins' runs and the scatter in one launch: every workgroup scans the final per-bin counts
// itself (bin_cnt[0, nb): k_bin_count's), workgroup 0 writes the runs (bounds), and each workgroup
// reserves its slots of each bin with an atomic on the zeroed fill counters bin_cnt[nb, 2 nb) —
// the one-workgroup scan launch between count and scatter is gone.
__global__ __launch_bounds__(1024) void k_bin_scatter(const void* __restrict__ keys_v, int wide_keys,
                                                      const uint32_t* __restrict__ vals,
                                                      const uint32_t* __restrict__ n_dev, int nb,
                                                      uint32_t* __restrict__ bin_cnt, uint2* __restrict__ bounds,
                                                      uint32_t* __restrict__ vals_out, uint32_t* __restrict__ kept) {
    __shared__ uint32_t h[kBinScanMax];
    __shared__ uint32_t s_start[kBinScanMax];
    __shared__ uint32_t wsum[16];
    const int t = threadIdx.x, lane = t & 63, w = t >> 6;
    const uint32_t n = *n_dev;
    const uint32_t per = (n + kBinGroups - 1) / kBinGroups;
    const uint32_t i0 = blockIdx.x * per, i1 = min(n, i0 + per);
    if (i0 >= i1) return;  // (n == 0: the zeroed bounds already say so)
    auto key = [&](uint32_t i) -> uint32_t {
        return wide_keys ? static_cast<const uint32_t*>(keys_v)[i] : static_cast<const uint16_t*>(keys_v)[i];
    };
    // exclusive scan of the counts: thread t owns bins [kPer t, kPer t + kPer)
    constexpr int kPer = kBinScanMax / 1024;
    const int b0 = t * kPer;
    uint32_t c[kPer], sum = 0;
#pragma unroll
    for (int k = 0; k < kPer; k++) {
        c[k] = b0 + k < nb ? bin_cnt[b0 + k] : 0u;
        sum += c[k];
    }
    for (int b = t; b < nb; b += 1024) h[b] = 0u;
    uint32_t incl = sum;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const uint32_t y = (uint32_t)__shfl_up((int)incl, o);
        if (lane >= o) incl += y;
    }
    if (lane == 63) wsum[w] = incl;
    __syncthreads();
    uint32_t run = incl - sum;
    for (int i = 0; i < w; i++) run += wsum[i];
#pragma unroll
    for (int k = 0; k < kPer; k++) {
        if (b0 + k < nb) {
            s_start[b0 + k] = run;
            if (blockIdx.x == 0) bounds[b0 + k] = make_uint2(~run, run + c[k]);  // {~start, end}
        }
        run += c[k];
    }
    if (kept && blockIdx.x == 0 && t == 1023) *kept = run;  // the pairs the bins hold (frame stats)
    for (uint32_t i = i0 + t; i < i1; i += 1024) {
        const uint32_t k = key(i);
        if (k < (uint32_t)nb) atomicAdd(&h[k], 1u);
    }
    __syncthreads();
    for (int b = t; b < nb; b += 1024)  // this workgroup's slots of each bin
        if (h[b]) h[b] = s_start[b] + atomicAdd(&bin_cnt[nb + b], h[b]);
    __syncthreads();
    for (uint32_t i = i0 + t; i < i1; i += 1024) {
        const uint32_t k = key(i);
        if (k < (uint32_t)nb) vals_out[atomicAdd(&h[k], 1u)] = vals[i];
    }
}

// per bin: open test (phase B), the bin's run (bounds: the bin sort's last scatter or k_bin_scatter),
// then sortexpand_run
template <typename K, int NT>
__global__ __launch_bounds__(NT) void k_sortexpand(const uint2* __restrict__ bounds,
                                                    const K* __restrict__ keys, const uint32_t* __restrict__ vals,
                                                    const uint32_t* __restrict__ depth_keys,
                                                    const FrameTotals* __restrict__ ft, int gx, int gy,
                                                    uint32_t out_base, uint32_t* __restrict__ point_list,
                                                    uint2* __restrict__ ranges, const uint32_t* __restrict__ open_bits,
                                                    uint32_t lds_cap, int ipasses, int bucket) {
    constexpr int CAP = NT == 1024 ? kSxCapB : kSxCap;
    __shared__ SxSharedT<NT / 64, CAP> sh;
    const int bgx = bins_x(gx);
    const int bin = blockIdx.x;
    const int X = bin % bgx, Y = bin / bgx;
    if (open_bits) {  // phase B: a bin whose tiles all closed in phase A holds no pair, and its
                      // tiles' ranges were cleared with the frame's: nothing to search or write
        bool any = false;
#pragma unroll
        for (int b = 0; b < 4; b++) {
            const int tx = 2 * X + (b & 1), ty = 2 * Y + (b >> 1);
            if (tx < gx && ty < gy) {
                const uint32_t tile = (uint32_t)(ty * gx + tx);
                any = any || ((open_bits[tile >> 5] >> (tile & 31)) & 1u);
            }
        }
        if (!any) return;  // block-uniform
    }
    const uint2 run = bounds[bin];  // the bin's run [lo, hi) of the bin-sorted pairs, {~lo, hi}
    const uint32_t lo = run.y ? ~run.x : 0u;
    sortexpand_run<NT, CAP>(sh, X, Y, gx, gy, lo, run.y - lo, vals, false, depth_keys, ft->wide != 0u, ipasses,
                            out_base, point_list, ranges, lds_cap, bucket != 0);
}

template <typename K>
void launch_sortexpand(const K* keys, const uint32_t* vals, const uint32_t* depth_keys, const FrameTotals* ft, int gx,
                       int gy, uint32_t out_base, uint32_t* point_list, uint2* ranges, const uint32_t* open_bits,
                       const uint2* bounds, hipStream_t st) {
    const int nb = bins_x(gx) * bins_y(gy);
    if (nb <= 0) return;
    k_sortexpand<K, 256><<<nb, 256, 0, st>>>(bounds, keys, vals, depth_keys, ft, gx, gy, out_base, point_list, ranges,
                                             open_bits, sx_lds_cap(kSxCap), 0, tuning().sx_bucket);
}
template void launch_sortexpand<uint16_t>(const uint16_t*, const uint32_t*, const uint32_t*, const FrameTotals*, int,
                                          int, uint32_t, uint32_t*, uint2*, const uint32_t*, const uint2*, hipStream_t);
template void launch_sortexpand<uint32_t>(const uint32_t*, const uint32_t*, const uint32_t*, const FrameTotals*, int,
                                          int, uint32_t, uint32_t*, uint2*, const uint32_t*, const uint2*, hipStream_t);

int index_passes(int P) {  // 9-bit passes covering the Gaussian indices [0, P)
    int b = 1;
    while (b < 28 && (1u << b) < (uint32_t)P) b++;
    return (b + 8) / 9;
}

template <typename K>
bool launch_sortexpand_small(int P, const K* keys, const uint32_t* vals, const uint32_t* n_dev, uint32_t* bin_cnt,
                             uint32_t* vals_sorted, const uint32_t* depth_keys, const FrameTotals* ft, int gx, int gy,
                             uint32_t out_base, uint32_t* point_list, uint2* ranges, const uint32_t* open_bits,
                             uint2* bounds, uint32_t* kept, hipStream_t st) {
    const int nb = bins_x(gx) * bins_y(gy);
    if (nb <= 0 || nb > kBinScanMax) return false;
    const int wk = sizeof(K) == 4;
    k_bin_count<<<kBinGroups, 1024, 0, st>>>(keys, wk, n_dev, nb, bin_cnt);
    k_bin_scatter<<<kBinGroups, 1024, 0, st>>>(keys, wk, vals, n_dev, nb, bin_cnt, bounds, vals_sorted, kept);
    // phase B: few bins hold pairs, so a bin's latency sets the launch's time — 1024 threads per bin
    // (its LDS runs hold kSxCapB pairs)
    k_sortexpand<K, 1024><<<nb, 1024, 0, st>>>(bounds, keys, vals_sorted, depth_keys, ft, gx, gy, out_base, point_list,
                                               ranges, open_bits, sx_lds_cap(kSxCapB), index_passes(P),
                                               tuning().sx_bucket);
    return true;
}
template bool launch_sortexpand_small<uint16_t>(int, const uint16_t*, const uint32_t*, const uint32_t*, uint32_t*,
                                                uint32_t*, const uint32_t*, const FrameTotals*, int, int, uint32_t,
                                                uint32_t*, uint2*, const uint32_t*, uint2*, uint32_t*, hipStream_t);
template bool launch_sortexpand_small<uint32_t>(int, const uint32_t*, const uint32_t*, const uint32_t*, uint32_t*,
                                                uint32_t*, const uint32_t*, const FrameTotals*, int, int, uint32_t,
                                                uint32_t*, uint2*, const uint32_t*, uint2*, uint32_t*, hipStream_t);

}  // namespace rr
