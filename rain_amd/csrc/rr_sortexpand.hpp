// rr_sortexpand.hpp — the per-bin depth sort and tile-list split of the binning (device code shared
// by rr_bin.hip's k_sortexpand and the phase-B forward blend that sorts its bin itself,
// rr_blend_fwd_s.hip).
#pragma once
#include "rr_common.hpp"
#include "rr_kernels.hpp"

namespace rr {

// ---- per bin: depth order + the four tile lists -----------------------------------------------
// A bin's run of the bin-sorted pairs holds one pair per Gaussian in index order (stable bin sort of
// index-ordered emission).  A stable LSD radix sort on the Gaussians' depth keys (3 passes of 9
// bits, or 4 of 8 when a visible key needs more than 27 bits) makes it (depth, index) order — the
// reference's per-tile order (rasterizer_impl.cu:292-300) — and the run is then split stably into
// its tiles' lists (one ballot per mask bit), written at out_base + 4 lo + b len with the tile's
// range (rasterizer_impl.cu:105-127).  Runs of up to CAP pairs are sorted in LDS, longer ones
// pass through the scratch arrays in chunks of CAP (same ranking, one global digit scan per
// pass).  Ranking (rr_sort.hip's): wave w owns the contiguous items [w 64 R, (w + 1) 64 R) in
// rounds of 64; lanes holding the same digit find each other with one ballot per digit bit.
#ifndef RR_SX_CAP
#define RR_SX_CAP 2048  // 4096: ranges stage 0.110 vs 0.095 ms/step (profiles/r04h_sortexpand_cap_ab.jsonl)
#endif
constexpr int kSxCap = RR_SX_CAP;
// Phase B's 1024-thread sort-expand holds runs of up to kSxCapB in LDS (66 KB, two workgroups per
// CU): its bins' runs are a few open tiles' whole tails, often over 2048 pairs, and the global path
// cost those frames ~30 us more (tools/phaseb_profile.py)
#ifndef RR_SX_CAP_B
#define RR_SX_CAP_B 4096
#endif
constexpr int kSxCapB = RR_SX_CAP_B;
#ifndef RR_SX_GLOBAL
#define RR_SX_GLOBAL 1  // 0: ISA inspection builds without the long-run path
#endif

// NW waves per workgroup (4: 256 threads; 16: the 1024-thread phase-B sort-expand), runs of up to
// CAP items in LDS
template <int NW, int CAP>
struct SxSharedT {
    uint32_t k[CAP];
    uint32_t v[CAP];
    uint32_t wcnt[NW][512];  // per-wave digit counts, then per-wave cursors (also the NW 512 buckets)
    uint32_t cursor[512];    // global path: next slot of each digit across the chunks
    uint32_t wsum[NW][4];
};

// One chunk's items (registers kr / vr, R rounds, `len` valid) ranked on digit (key >> shift) & mask
// and stored at base[d] + (rank among the chunk's digit-d items, in input order) — to LDS
// (dst_lds) or to a global scratch run (dst_g).  base: the digit's first slot (LDS path: the
// chunk's exclusive digit prefix; global path: cursor[d]).  Ends with the chunk's digit counts
// added to cursor (global path).
template <int NT, int CAP>
__device__ __forceinline__ void sx_rank_chunk(SxSharedT<NT / 64, CAP>& sh, const uint32_t (&kr)[CAP / NT],
                                              const uint32_t (&vr)[CAP / NT], int R, uint32_t len, int shift,
                                              int db, bool global, uint2* dst_g) {
    constexpr int MR = CAP / NT, NW = NT / 64;
    const int t = threadIdx.x, lane = t & 63, w = t >> 6;
    const int ndig = 1 << db;
    const uint32_t mask = (uint32_t)ndig - 1u;
    const uint32_t wl = (uint32_t)w * 64 * R;
    for (int d = lane; d < ndig; d += 64) sh.wcnt[w][d] = 0;
    __builtin_amdgcn_wave_barrier();
#pragma unroll
    for (int r = 0; r < MR; r++)
        if (r < R && wl + (uint32_t)r * 64 + lane < len) atomicAdd(&sh.wcnt[w][(kr[r] >> shift) & mask], 1u);
    __syncthreads();
    if (w == 0) {  // digits in order, waves in order inside a digit (DPL consecutive digits per lane)
        const int dpl = ndig / 64;
        uint32_t sum = 0;
        for (int i = 0; i < dpl; i++) {
            const int d = dpl * lane + i;
#pragma unroll
            for (int v = 0; v < NW; v++) sum += sh.wcnt[v][d];
        }
        uint32_t incl = sum;
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
            const uint32_t y = (uint32_t)__shfl_up((int)incl, o);
            if (lane >= o) incl += y;
        }
        uint32_t run = incl - sum;
        for (int i = 0; i < dpl; i++) {
            const int d = dpl * lane + i;
            uint32_t r2 = global ? sh.cursor[d] : run, tot = 0;
#pragma unroll
            for (int v = 0; v < NW; v++) {
                const uint32_t x = sh.wcnt[v][d];
                sh.wcnt[v][d] = r2;
                r2 += x;
                tot += x;
            }
            if (global) sh.cursor[d] += tot;
            run += tot;
        }
    }
    __syncthreads();
    const uint64_t lt = (1ull << lane) - 1ull;
#pragma unroll
    for (int r = 0; r < MR; r++) {
        if (r >= R || wl + (uint32_t)r * 64 >= len) continue;  // wave-uniform
        const bool valid = wl + (uint32_t)r * 64 + lane < len;
        const uint32_t d = (kr[r] >> shift) & mask;
        uint64_t m = __ballot(valid);
        for (int b = 0; b < db; b++) {
            const bool bit = (d >> b) & 1u;
            const uint64_t bb = __ballot(bit);
            m &= bit ? bb : ~bb;
        }
        const uint32_t rank = (uint32_t)__popcll(m & lt);
        const uint32_t pos = sh.wcnt[w][d] + rank;  // every lane reads before any leader writes
        __builtin_amdgcn_wave_barrier();
        if (valid && rank == 0) sh.wcnt[w][d] = pos + (uint32_t)__popcll(m);
        __builtin_amdgcn_wave_barrier();
        if (valid) {
            if (global) {
                dst_g[pos] = make_uint2(kr[r], vr[r]);
            } else {
                sh.k[pos] = kr[r];
                sh.v[pos] = vr[r];
            }
        }
    }
    __syncthreads();
}

// After a depth-only sort of a run in no particular order: every group of equal depth keys put in
// Gaussian-index order in place, one thread per group (groups are clones at one position: a few
// items).  Returns true when a group longer than kTieMax was left for a full index-pass sort.
constexpr uint32_t kTieMax = 32;
template <int NT, typename KeyAt, typename ValAt, typename SetVal>
__device__ __forceinline__ bool fix_ties(uint32_t len, KeyAt key_at, ValAt val_at, SetVal set_val) {
    bool big = false;
    for (uint32_t i = threadIdx.x; i + 1 < len; i += NT) {
        const uint32_t k = key_at(i);
        if (key_at(i + 1) != k || (i > 0 && key_at(i - 1) == k)) continue;  // not a group's first item
        uint32_t j = i + 2;
        while (j < len && j - i <= kTieMax && key_at(j) == k) j++;
        if (j - i > kTieMax) {
            big = true;
            continue;
        }
        for (uint32_t a = i + 1; a < j; a++) {  // insertion sort on the index
            const uint32_t v = val_at(a);
            uint32_t b = a;
            while (b > i && (val_at(b - 1) & BIN_ID_MASK) > (v & BIN_ID_MASK)) {
                set_val(b, val_at(b - 1));
                b--;
            }
            set_val(b, v);
        }
    }
    return __syncthreads_or(big);
}

// Bucket sort of a run of len <= CAP items (depth keys kr / values vr in registers, R rounds per
// wave as in sx_rank_chunk) into (depth key, Gaussian index) order — the reference's per-tile order —
// in sh.k / sh.v, whatever order the run arrived in: one counting pass over NW 512 buckets
// spanning the run's own key range [kmin, kmax], then each bucket (a few items) insertion-sorted by
// one thread on (key, index).  One histogram, one scan and one scatter instead of the three 9-bit
// LSD passes (each a histogram, a 512-digit scan and a ballot ranking), and equal depths need no
// extra index passes.  Returns false, with nothing written to sh.k / sh.v, when a bucket holds more
// than kSxBucketMax items (strongly clustered depths, many exact copies): the caller then sorts
// with the LSD passes.
#ifndef RR_SX_BUCKET_MAX
#define RR_SX_BUCKET_MAX 16
#endif
constexpr uint32_t kSxBucketMax = RR_SX_BUCKET_MAX;
template <int NT, int CAP>
__device__ __forceinline__ bool bucket_sort_run(SxSharedT<NT / 64, CAP>& sh, const uint32_t (&kr)[CAP / NT],
                                                const uint32_t (&vr)[CAP / NT], int R, uint32_t len) {
    constexpr int MR = CAP / NT, NW = NT / 64;
    constexpr int kSxBuckets = NW * 512;  // the per-wave digit counters of SxSharedT
    constexpr int kLg = 9 + (NW >= 2) + (NW >= 4) + (NW >= 8) + (NW >= 16);  // log2(kSxBuckets)
    static_assert((1 << kLg) == kSxBuckets, "bucket count");
    const int t = threadIdx.x, lane = t & 63, w = t >> 6;
    const uint32_t wl = (uint32_t)w * 64 * R;
    uint32_t* hist = &sh.wcnt[0][0];
    uint32_t kmin = 0xffffffffu, kmax = 0u;
#pragma unroll
    for (int r = 0; r < MR; r++)
        if (r < R && wl + (uint32_t)r * 64 + lane < len) {
            kmin = min(kmin, kr[r]);
            kmax = max(kmax, kr[r]);
        }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        kmin = min(kmin, (uint32_t)__shfl_xor((int)kmin, o));
        kmax = max(kmax, (uint32_t)__shfl_xor((int)kmax, o));
    }
    if (lane == 0) {
        sh.wsum[w][0] = kmin;
        sh.wsum[w][1] = kmax;
    }
    for (int i = t; i < kSxBuckets; i += NT) hist[i] = 0u;
    __syncthreads();
#pragma unroll
    for (int i = 0; i < NW; i++) {
        kmin = min(kmin, sh.wsum[i][0]);
        kmax = max(kmax, sh.wsum[i][1]);
    }
    const uint32_t span = kmax - kmin;
    // (span >> shift) < kSxBuckets
    const int shift = span < (uint32_t)kSxBuckets ? 0 : 32 - __clz((int)span) - kLg;
    uint32_t bk[MR];
#pragma unroll
    for (int r = 0; r < MR; r++) {
        bk[r] = (kr[r] - kmin) >> shift;
        if (r < R && wl + (uint32_t)r * 64 + lane < len) atomicAdd(&hist[bk[r]], 1u);
    }
    __syncthreads();
    // exclusive bucket starts: thread t owns buckets [BPT t, BPT t + BPT)
    constexpr int BPT = kSxBuckets / NT;
    uint32_t c[BPT], sum = 0, mx = 0;
#pragma unroll
    for (int k = 0; k < BPT; k++) {
        c[k] = hist[BPT * t + k];
        sum += c[k];
        mx = max(mx, c[k]);
    }
    uint32_t incl = sum;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const uint32_t y = (uint32_t)__shfl_up((int)incl, o);
        if (lane >= o) incl += y;
    }
    if (lane == 63) sh.wsum[w][2] = incl;
    if (__syncthreads_or(mx > kSxBucketMax)) return false;  // (the barrier also publishes wsum)
    uint32_t run = incl - sum;
    for (int i = 0; i < w; i++) run += sh.wsum[i][2];
#pragma unroll
    for (int k = 0; k < BPT; k++) {
        hist[BPT * t + k] = run;
        run += c[k];
    }
    __syncthreads();
#pragma unroll
    for (int r = 0; r < MR; r++)
        if (r < R && wl + (uint32_t)r * 64 + lane < len) {
            const uint32_t pos = atomicAdd(&hist[bk[r]], 1u);
            sh.k[pos] = kr[r];
            sh.v[pos] = vr[r];
        }
    __syncthreads();
    // hist[b] is now bucket b's end, hist[b - 1] its start.  Each item's place inside its bucket in
    // parallel: its rank among the bucket's items on (depth key, Gaussian index) — a strict order,
    // the indices of one bin being distinct — then every item written to its place.  (One thread
    // insertion-sorting each bucket cost 17.5 us of the 90 us ranges stage: the buckets' lengths
    // are skewed and the workgroup waits for the longest; profiles/r05_sortexpand_probe_ab.jsonl.)
    uint32_t pk[MR], pv[MR], pr[MR];
#pragma unroll
    for (int r = 0; r < MR; r++) {
        const uint32_t a = (uint32_t)t + (uint32_t)NT * (uint32_t)r;
        pr[r] = 0xffffffffu;
        if (r < R && a < len) {
            const uint32_t k = sh.k[a], v = sh.v[a], vi = v & BIN_ID_MASK;
            const uint32_t b = (k - kmin) >> shift;
            const uint32_t s0 = b ? hist[b - 1] : 0u, e = hist[b];
            uint32_t rank = s0;
            for (uint32_t j = s0; j < e; j++) {
                const uint32_t qk = sh.k[j];
                rank += (qk < k || (qk == k && (sh.v[j] & BIN_ID_MASK) < vi)) ? 1u : 0u;
            }
            pk[r] = k;
            pv[r] = v;
            pr[r] = rank;
        }
    }
    __syncthreads();  // every read of the bucket order before the first write
#pragma unroll
    for (int r = 0; r < MR; r++)
        if (pr[r] != 0xffffffffu) {
            sh.k[pr[r]] = pk[r];
            sh.v[pr[r]] = pv[r];
        }
    __syncthreads();
    return true;
}

// One bin's run of `len` (bin, Gaussian) pairs in index order -> depth order -> its four tiles'
// lists at out_base + 4 lo + b len, and the tiles' ranges.  The run is vals[lo, lo + len) or, with
// lds_vals (len <= CAP), already in sh.v.  Runs longer than lds_cap (<= CAP) are sorted
// through global scratch: the run's own output region of point_list (4 slots per pair = two uint2
// arrays of len), with the sorted values put back into vals[lo, lo + len) before the tile split
// overwrites that region — no scratch arrays in the binning buffer.
template <int NT, int CAP>
__device__ __forceinline__ void sortexpand_run(SxSharedT<NT / 64, CAP>& sh, int X, int Y, int gx, int gy, uint32_t lo,
                                               uint32_t len,
                                               const uint32_t* __restrict__ vals, bool lds_vals,
                                               const uint32_t* __restrict__ depth_keys, bool wide, int ipasses,
                                               uint32_t out_base, uint32_t* __restrict__ point_list,
                                               uint2* __restrict__ ranges, uint32_t lds_cap, bool bucket) {
    constexpr int MR = CAP / NT, NW = NT / 64;
    const int t = threadIdx.x, lane = t & 63, w = t >> 6;
    // The depth key: 27 bits in 3 passes of 9, wider frames in 4 of 8.  A run in no particular order
    // (ipasses > 0: the phase-B pairs of the gather path) needs index order among equal depth keys:
    // its LDS path sorts by depth alone and, only if two neighbours then share a key, sorts again
    // with ipasses 9-bit passes on the Gaussian index first; its global path always does.
    const int dbd = wide ? 8 : 9;
    int ip = 0;  // index passes of the current attempt
    auto shift_of = [&](int p) { return p < ip ? 9 * p : (p - ip) * dbd; };
    auto db_of = [&](int p) { return p < ip ? 9 : dbd; };
    auto key_of = [&](int p, uint32_t v) { return p < ip ? (v & BIN_ID_MASK) : depth_keys[v & BIN_ID_MASK]; };
    bool global = false;  // the sorted run is back in vals[lo, lo + len)
    if (len > 1 && len <= lds_cap) {
        const int R = (int)((len + NT - 1) / NT);
        const uint32_t wl = (uint32_t)w * 64 * R;
        uint32_t kr[MR], vr[MR];
        // every round's loads unconditional, the index clamped into the run: a condition (per lane or
        // on R) made the compiler branch and wait around each load; the clamped extra loads hit the
        // cache line of the run's last item and are never used (items past len are not ranked)
        if (lds_vals) {  // gathered into sh.v by the caller
#pragma unroll
            for (int r = 0; r < MR; r++) vr[r] = sh.v[min(wl + (uint32_t)r * 64 + lane, len - 1)];
            __syncthreads();  // every read of the gathered run before the first pass writes sh.v
        } else {
#pragma unroll
            for (int r = 0; r < MR; r++) vr[r] = vals[lo + min(wl + (uint32_t)r * 64 + lane, len - 1)];
        }
        bool sorted = false;
        if (bucket) {
#pragma unroll
            for (int r = 0; r < MR; r++) kr[r] = depth_keys[vr[r] & BIN_ID_MASK];  // all gathers in flight
            sorted = bucket_sort_run<NT, CAP>(sh, kr, vr, R, len);  // block-uniform
        }
        for (int attempt = 0; !sorted; attempt++) {
            const int passes = ip + (wide ? 4 : 3);
#pragma unroll
            for (int r = 0; r < MR; r++) kr[r] = key_of(0, vr[r]);  // all gathers in flight
            for (int p = 0; p < passes; p++) {
                sx_rank_chunk<NT, CAP>(sh, kr, vr, R, len, shift_of(p), db_of(p), false, nullptr);
                if (p + 1 < passes) {
                    const bool rekey = p + 1 == ip;  // index order done: the depth keys from here on
#pragma unroll
                    for (int r = 0; r < MR; r++) {
                        const uint32_t i = wl + (uint32_t)r * 64 + lane;
                        if (r < R && i < len) {
                            kr[r] = sh.k[i];
                            vr[r] = sh.v[i];
                        }
                    }
                    if (rekey)
#pragma unroll
                        for (int r = 0; r < MR; r++) kr[r] = depth_keys[vr[r] & BIN_ID_MASK];
                    __syncthreads();  // every read of this pass's order before the next pass's writes
                }
            }
            if (ipasses == 0 || attempt > 0) break;
            // unordered run sorted by depth alone: equal keys put in index order in place, or (a long
            // group) the full sort with the index passes first
            if (!fix_ties<NT>(
                    len, [&](uint32_t i) { return sh.k[i]; }, [&](uint32_t i) { return sh.v[i]; },
                    [&](uint32_t i, uint32_t v) { sh.v[i] = v; }))
                break;  // block-uniform
            ip = ipasses;
#pragma unroll
            for (int r = 0; r < MR; r++) vr[r] = sh.v[min(wl + (uint32_t)r * 64 + lane, len - 1)];
            __syncthreads();  // every read of the depth order before the index passes write sh.v
        }
    } else if (RR_SX_GLOBAL && len > lds_cap) {
        // chunks of CAP in order; pass p reads run p - 1 (pass 0: the run's values with their
        // keys) and writes scratch p % 2 (halves of the run's point_list region, 8-B aligned:
        // out_base is a multiple of 4 slots)
        uint2* const scr0 = reinterpret_cast<uint2*>(point_list + out_base + 4u * lo);
        uint2* const scr1 = scr0 + len;
        const uint2* sorted_g = nullptr;
      for (int attempt = 0;; attempt++) {
        const int passes = ip + (wide ? 4 : 3);
        for (int p = 0; p < passes; p++) {
            const int db = db_of(p), shift = shift_of(p);
            const int ndig = 1 << db;
            const uint32_t mask = (uint32_t)ndig - 1u;
            const uint2* src = p == 0 ? nullptr : ((p & 1) ? scr0 : scr1);
            uint2* dst = (p & 1) ? scr1 : scr0;
            const bool fresh = src == nullptr || p == ip;  // keys recomputed from the values
            // digit totals of the whole run -> each digit's first slot
            for (int d = t; d < ndig; d += NT) sh.cursor[d] = 0;
            __syncthreads();
            for (uint32_t i = t; i < len; i += NT) {
                const uint32_t k = fresh ? key_of(p, src ? src[i].y : vals[lo + i]) : src[i].x;
                atomicAdd(&sh.cursor[(k >> shift) & mask], 1u);
            }
            __syncthreads();
            if (w == 0) {
                const int dpl = ndig / 64;
                uint32_t sum = 0;
                for (int i = 0; i < dpl; i++) sum += sh.cursor[dpl * lane + i];
                uint32_t incl = sum;
#pragma unroll
                for (int o = 1; o < 64; o <<= 1) {
                    const uint32_t y = (uint32_t)__shfl_up((int)incl, o);
                    if (lane >= o) incl += y;
                }
                uint32_t run = incl - sum;
                for (int i = 0; i < dpl; i++) {
                    const uint32_t x = sh.cursor[dpl * lane + i];
                    sh.cursor[dpl * lane + i] = run;
                    run += x;
                }
            }
            __syncthreads();
            for (uint32_t c0 = 0; c0 < len; c0 += CAP) {
                const uint32_t clen = min((uint32_t)CAP, len - c0);
                const int R = (int)((clen + NT - 1) / NT);
                const uint32_t wl = (uint32_t)w * 64 * R;
                uint32_t kr[MR], vr[MR];
                if (src) {
#pragma unroll
                    for (int r = 0; r < MR; r++) {  // clamped, unconditional loads (see above)
                        const uint2 e = src[c0 + min(wl + (uint32_t)r * 64 + lane, clen - 1)];
                        kr[r] = e.x;
                        vr[r] = e.y;
                    }
                } else {
#pragma unroll
                    for (int r = 0; r < MR; r++) vr[r] = vals[lo + c0 + min(wl + (uint32_t)r * 64 + lane, clen - 1)];
                }
                if (fresh)
#pragma unroll
                    for (int r = 0; r < MR; r++) kr[r] = key_of(p, vr[r]);
                sx_rank_chunk<NT, CAP>(sh, kr, vr, R, clen, shift, db, true, dst);
            }
            __syncthreads();
        }
        sorted_g = ((passes - 1) & 1) ? scr1 : scr0;
        if (ipasses == 0 || attempt > 0) break;
        uint2* sg = const_cast<uint2*>(sorted_g);
        __threadfence_block();
        if (!fix_ties<NT>(
                len, [&](uint32_t i) { return sg[i].x; }, [&](uint32_t i) { return sg[i].y; },
                [&](uint32_t i, uint32_t v) { sg[i].y = v; }))
            break;
        // a long group: the full sort, index passes first, from the run's original values
        ip = ipasses;
      }
        // the sorted values back over the run's input (read only by pass 0), freeing the region
        uint32_t* const vw = const_cast<uint32_t*>(vals) + lo;
        for (uint32_t i = t; i < len; i += NT) vw[i] = sorted_g[i].y;
        __syncthreads();
        global = true;
    }
    // the four tile lists, stable, from the depth-ordered run (LDS, global scratch, or the single /
    // empty run straight from vals)
    const uint64_t lt = (1ull << lane) - 1ull;
    const uint32_t dst0 = out_base + 4u * lo;
    uint32_t carry[4] = {0u, 0u, 0u, 0u};
    for (uint32_t r0 = 0; r0 < len; r0 += NT) {
        const uint32_t j = r0 + (uint32_t)t;
        uint32_t v = 0u;
        if (j < len) v = (global || (len <= 1 && !lds_vals)) ? vals[lo + j] : sh.v[j];
        const uint32_t m = j < len ? v >> BIN_SHIFT : 0u;
        uint32_t rank[4];
#pragma unroll
        for (int b = 0; b < 4; b++) {
            const uint64_t bal = __ballot((m >> b) & 1u);
            rank[b] = (uint32_t)__popcll(bal & lt);
            if (lane == 0) sh.wsum[w][b] = (uint32_t)__popcll(bal);
        }
        __syncthreads();
#pragma unroll
        for (int b = 0; b < 4; b++) {
            uint32_t pre = carry[b], tot = 0;
#pragma unroll
            for (int i = 0; i < NW; i++) {
                pre += i < w ? sh.wsum[i][b] : 0u;
                tot += sh.wsum[i][b];
            }
            if ((m >> b) & 1u) point_list[dst0 + (uint32_t)b * len + pre + rank[b]] = v & BIN_ID_MASK;
            carry[b] += tot;
        }
        __syncthreads();
    }
    if (t < 4) {
        const int tx = 2 * X + (t & 1), ty = 2 * Y + (t >> 1);
        const uint32_t s = dst0 + (uint32_t)t * len;
        if (tx < gx && ty < gy) ranges[ty * gx + tx] = make_uint2(s, s + carry[t]);
    }
}


}  // namespace rr
