// rr_sort.hip — stable LSD radix sort of (key, u32 value) pairs, written for CDNA4.
//
// Used for the bin sorts of the binning (L pairs, <= 16-bit bin keys, or 32 beyond 65536 bins);
// replaces rocPRIM's device radix sort (Onesweep look-back latency bound here; merge path below
// 2^20 items).  (Rounds 1-3 also ran a per-frame depth sort of the P Gaussians on it; the bins'
// depth order now comes from k_sortexpand, rr_bin.hip.)
//
// Each pass sorts by one digit of <= 8 bits with a count / scan / scatter split over "units" of
// one workgroup (4 wave64s) x R rounds x 64 items (R chosen per call so that small inputs still
// spread over enough workgroups):
//   * k_rs_count: digit histogram of the unit in LDS -> counts[digit][unit] (digit-major);
//   * k_rs_scan_rows: per digit, exclusive scan of its counts over the units (+ digit totals);
//     the scatter adds the digit bases, so every (digit, unit) gets its first output slot;
//   * k_rs_scatter: (1) per-wave digit counts, (2) block-local digit starts in LDS, (3) each wave
//     walks its rounds in order; lanes holding the same digit find each other with one ballot per
//     digit bit (wave-wide match), rank = popcount of lower matching lanes, the group leader
//     advances the per-(wave, digit) cursor; the item is staged in LDS at its block-local sorted
//     position, (4) the staged unit is written out in order, so consecutive threads write
//     consecutive addresses of each digit's run (coalesced) instead of scattering single items.
// Order inside a unit is (wave, round, lane) = input order and units are scanned in order, so
// every pass is stable.  A producer that filters its output (the early-stop duplicate pass) may
// leave units sparse (unit_len[u] items each, positions kept) and only the device knows the total
// (n_dev): the first pass then compacts, and every later pass reads the count from the device.
// Digits are <= 8 bits, or <= 9 bits where that saves a pass (the 27-bit depth sort: 3 x 9 instead
// of 4 x 7); the bits are spread evenly over the passes (13 -> 7 + 6).
#include "rr_common.hpp"
#include "rr_kernels.hpp"

namespace rr {

namespace {

constexpr int kWaves = 4;       // waves per workgroup (unit) of the count kernel
#ifndef RR_SORT_SW
#define RR_SORT_SW 8
#endif
// waves per workgroup of the scatter (4 or 8): 8 halves each wave's serial rank rounds for the
// same unit (depth sort 0.0913 -> 0.0877 ms/step, profiles/r03_sort_scatter8_ab.jsonl)
constexpr int kScatterWaves = RR_SORT_SW;
constexpr int kMaxRounds = 16;  // rounds of 64 items per wave
constexpr int kMaxUnitItems = 64 * kWaves * kMaxRounds;  // 4096
static_assert(kMaxUnitItems == kSortMaxUnit, "rr_kernels.hpp kSortMaxUnit");

// passes of a sort of `bits` bits: 8-bit digits, or 9-bit ones for 25..27 bits (3 passes instead of
// 4; the tile sorts, whose first-pass counts come from the duplicate's 256-digit histogram, keep
// 8-bit digits)
__host__ __device__ constexpr int sort_passes(int bits) {
    return bits <= 0 ? 0 : (bits >= 25 && bits <= 27) ? 3 : (bits + 7) / 8;
}
__host__ __device__ constexpr int sort_max_dbits(int bits) {
    return bits <= 0 ? 0 : (bits + sort_passes(bits) - 1) / sort_passes(bits);
}

// Items of one unit: [unit * unit_items, unit * unit_items + len).  Contiguous input has
// len = min(unit_items, n - base) with n from the host or, when only the device knows it (a
// filtered producer), from *n_dev; a producer that leaves its units sparse passes every unit's
// length in unit_len.
__device__ __forceinline__ uint32_t unit_length(const uint32_t* unit_len, const uint32_t* n_dev, size_t n, int unit,
                                                uint32_t unit_items) {
    if (unit_len) return unit_len[unit];
    const size_t nn = n_dev ? (size_t)*n_dev : n;
    const size_t base = (size_t)unit * unit_items;
    return base >= nn ? 0u : (uint32_t)min((size_t)unit_items, nn - base);
}

template <typename K, int MAXR, int DB>
__global__ __launch_bounds__(64 * kWaves) void k_rs_count(const K* __restrict__ keys, size_t n, int shift, int dbits,
                                                          int rounds, uint32_t* __restrict__ counts, int units,
                                                          const uint32_t* __restrict__ n_dev) {
    __shared__ uint32_t hist[1 << DB];
    const int t = threadIdx.x;
    const int ndig = 1 << dbits;
    for (int d = t; d < ndig; d += 64 * kWaves) hist[d] = 0;
    const int unit = blockIdx.x;
    const uint32_t unit_items = (uint32_t)rounds * 64 * kWaves;
    const size_t base = (size_t)unit * unit_items;
    const uint32_t len = unit_length(nullptr, n_dev, n, unit, unit_items);
    const uint32_t mask = (uint32_t)ndig - 1u;
    uint32_t dr[MAXR];
#pragma unroll
    for (int r = 0; r < MAXR; r++) {  // all loads in flight before the first LDS atomic
        const uint32_t li = (uint32_t)r * 64 * kWaves + t;
        dr[r] = (r < rounds && li < len) ? (((uint32_t)keys[base + li] >> shift) & mask) : 0xffffffffu;
    }
    __syncthreads();
#pragma unroll
    for (int r = 0; r < MAXR; r++)
        if (dr[r] != 0xffffffffu) atomicAdd(&hist[dr[r]], 1u);
    __syncthreads();
    for (int d = t; d < ndig; d += 64 * kWaves) counts[(size_t)d * units + unit] = hist[d];
}

// Exclusive scan of each digit's row of counts over the units (one workgroup per digit) ->
// offsets[d][unit] relative to the digit, and the digit's total.  The scatter adds the digit bases
// (exclusive scan of the <= 256 totals) itself.  Replaces a device scan call and its host-side
// dispatch overhead.  Rows of up to 256 * kScanReg units are read into registers in one go (thread
// t owns a contiguous run of units), so the scan waits for one load latency instead of one per
// 256 units; longer rows are walked in tiles of 256.
constexpr int kScanReg = 16;
__device__ __forceinline__ uint32_t block_exclusive_scan256(uint32_t v, uint32_t* wsum, uint32_t& total) {
    const int t = threadIdx.x, lane = t & 63, w = t >> 6;
    uint32_t incl = v;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const uint32_t y = (uint32_t)__shfl_up((int)incl, o);
        if (lane >= o) incl += y;
    }
    if (lane == 63) wsum[w] = incl;
    __syncthreads();
    uint32_t wpre = 0;
    total = 0;
#pragma unroll
    for (int i = 0; i < 4; i++) {
        wpre += i < w ? wsum[i] : 0u;
        total += wsum[i];
    }
    return wpre + incl - v;
}

__global__ __launch_bounds__(256) void k_rs_scan_rows(const uint32_t* __restrict__ counts,
                                                      uint32_t* __restrict__ offsets, int units,
                                                      uint32_t* __restrict__ totals) {
    __shared__ uint32_t wsum[4];
    const int d = blockIdx.x, t = threadIdx.x;
    const uint32_t* row = counts + (size_t)d * units;
    uint32_t* out = offsets + (size_t)d * units;
    if (units <= 256 * kScanReg) {
        const int c = (units + 255) / 256;  // units per thread
        const int u0 = t * c;
        uint32_t v[kScanReg], sum = 0;
#pragma unroll
        for (int i = 0; i < kScanReg; i++) {
            v[i] = (i < c && u0 + i < units) ? row[u0 + i] : 0u;
            sum += v[i];
        }
        uint32_t total;
        uint32_t run = block_exclusive_scan256(sum, wsum, total);
#pragma unroll
        for (int i = 0; i < kScanReg; i++) {
            if (i < c && u0 + i < units) out[u0 + i] = run;
            run += v[i];
        }
        if (t == 0) totals[d] = total;
        return;
    }
    uint32_t carry = 0;
    for (int base = 0; base < units; base += 256) {
        const int u = base + t;
        const uint32_t v = u < units ? row[u] : 0u;
        uint32_t tile;
        const uint32_t ex = block_exclusive_scan256(v, wsum, tile);
        if (u < units) out[u] = carry + ex;
        carry += tile;
        __syncthreads();
    }
    if (t == 0) totals[d] = carry;
}

// MAXR: rounds the kernel is compiled for (>= the call's rounds).  Small units get a small
// instance: the LDS staging is sized by it, so e.g. the 512-item units of a 1M-key sort fit ~4x
// more workgroups per CU than a 4096-item staging area allows.
template <typename K, int MAXR, int DB, int SW>
__global__ __launch_bounds__(64 * SW) void k_rs_scatter(const K* __restrict__ keys_in,
                                                            const uint32_t* __restrict__ vals_in,
                                                            K* __restrict__ keys_out, uint32_t* __restrict__ vals_out,
                                                            size_t n, int shift, int dbits, int rounds,
                                                            const uint32_t* __restrict__ offsets, int units,
                                                            const uint32_t* __restrict__ totals,
                                                            const uint32_t* __restrict__ unit_len,
                                                            const uint32_t* __restrict__ n_dev,
                                                            uint2* __restrict__ bounds) {
    constexpr int ND = 1 << DB;  // digits the kernel is compiled for (>= 1 << dbits)
    constexpr int DPL = ND / 64;  // digits per lane in the digit scans
    __shared__ uint32_t dbase[ND];         // first output slot of each digit
    __shared__ uint32_t wcnt[SW][ND];  // per-wave digit counts, then per-wave cursors
    __shared__ uint32_t dstart[ND];        // block-local start of each digit's run
    __shared__ uint32_t goff[ND];          // global slot of block-local position 0 of each digit's run
    __shared__ uint32_t s_val[64 * SW * MAXR];
    __shared__ K s_key[64 * SW * MAXR];
    __shared__ uint32_t s_nu;  // items staged
    const int t = threadIdx.x, lane = t & 63, w = t >> 6;
    const int ndig = 1 << dbits;
    const uint32_t mask = (uint32_t)ndig - 1u;
    const int unit = blockIdx.x;
    const uint32_t unit_items = (uint32_t)rounds * 64 * SW;
    const size_t ubase = (size_t)unit * unit_items;
    const uint32_t len = unit_length(unit_len, n_dev, n, unit, unit_items);
    if (len == 0) return;  // empty unit (sparse producer / past the device-side count): no output
    // wave w owns the contiguous items [wl, wl + 64 * rounds) of the unit (local indices)
    const uint32_t wl = (uint32_t)w * 64 * rounds;
    const size_t wbase = ubase + wl;
    for (int d = lane; d < ndig; d += 64) wcnt[w][d] = 0;
    for (int d = t; d < ndig; d += 64 * SW) goff[d] = offsets[(size_t)d * units + unit];
    if (w == 1) {  // digit bases: exclusive scan of the digit totals (DPL per lane, then shuffles)
        uint32_t tv[DPL], sum = 0;
#pragma unroll
        for (int i = 0; i < DPL; i++) {
            const int d = DPL * lane + i;
            tv[i] = d < ndig ? totals[d] : 0u;
            sum += tv[i];
        }
        uint32_t incl = sum;
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
            const uint32_t y = (uint32_t)__shfl_up((int)incl, o);
            if (lane >= o) incl += y;
        }
        uint32_t run = incl - sum;
#pragma unroll
        for (int i = 0; i < DPL; i++) {
            dbase[DPL * lane + i] = run;
            run += tv[i];
        }
    }
    // the wave's items go to registers once (all loads in flight together); counting, ranking
    // and staging then run from registers
    K kr[MAXR];
    uint32_t vr[MAXR];
#pragma unroll
    for (int r = 0; r < MAXR; r++) {
        const size_t i = wbase + (size_t)r * 64 + lane;
        const bool valid = r < rounds && wl + (uint32_t)r * 64 + lane < len;
        kr[r] = valid ? keys_in[i] : (K)~(K)0;
        vr[r] = valid ? (vals_in ? vals_in[i] : (uint32_t)i) : 0u;
    }
    auto live = [&](int r) { return r < rounds && wl + (uint32_t)r * 64 + lane < len; };
    __syncthreads();
#pragma unroll
    for (int r = 0; r < MAXR; r++) {
        if (live(r)) atomicAdd(&wcnt[w][((uint32_t)kr[r] >> shift) & mask], 1u);
    }
    __syncthreads();
    // block-local starts: digits in order, then waves in order inside each digit.  Wave 0 scans the
    // <= ND digit totals: DPL consecutive digits per lane, then a 6-step shuffle scan of lane sums.
    if (w == 0) {
        uint32_t tot[DPL], sum = 0;
#pragma unroll
        for (int i = 0; i < DPL; i++) {
            const int d = DPL * lane + i;
            tot[i] = 0;
            if (d < ndig)
#pragma unroll
                for (int v = 0; v < SW; v++) tot[i] += wcnt[v][d];
            sum += tot[i];
        }
        uint32_t incl = sum;
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
            const uint32_t y = (uint32_t)__shfl_up((int)incl, o);
            if (lane >= o) incl += y;
        }
        uint32_t run = incl - sum;  // exclusive prefix of this lane's first digit
#pragma unroll
        for (int i = 0; i < DPL; i++) {
            const int d = DPL * lane + i;
            if (d < ndig) {
                dstart[d] = run;
                goff[d] += dbase[d] - run;
                uint32_t r2 = run;
#pragma unroll
                for (int v = 0; v < SW; v++) {
                    const uint32_t x = wcnt[v][d];
                    wcnt[v][d] = r2;
                    r2 += x;
                }
            }
            run += tot[i];
        }
        if (lane == 63) s_nu = run;
    }
    __syncthreads();
    const uint64_t lt = (1ull << lane) - 1ull;
#pragma unroll
    for (int r = 0; r < MAXR; r++) {
        if (r >= rounds || wl + (uint32_t)r * 64 >= len) continue;  // wave-uniform; keeps the loop unrollable
        const bool valid = live(r);
        const K k = kr[r];
        const uint32_t v = vr[r];
        const uint32_t d = ((uint32_t)k >> shift) & mask;
        uint64_t m = __ballot(valid);
        for (int b = 0; b < dbits; b++) {
            const bool bit = (d >> b) & 1u;
            const uint64_t bb = __ballot(bit);
            m &= bit ? bb : ~bb;
        }
        const uint32_t rank = (uint32_t)__popcll(m & lt);
        const uint32_t lpos = wcnt[w][d] + rank;  // every lane reads before any leader writes
        __builtin_amdgcn_wave_barrier();
        if (valid && rank == 0) wcnt[w][d] = lpos + (uint32_t)__popcll(m);
        __builtin_amdgcn_wave_barrier();
        if (valid) {
            s_key[lpos] = k;
            s_val[lpos] = v;
        }
    }
    __syncthreads();
    const int nu = (int)s_nu;
    for (int j = t; j < nu; j += 64 * SW) {
        const K k = s_key[j];
        const uint32_t d = ((uint32_t)k >> shift) & mask;
        const uint32_t pos = goff[d] + (uint32_t)j;
        if (keys_out) keys_out[pos] = k;
        vals_out[pos] = s_val[j];
        if (bounds) {
            // last pass (the unit's items in final key order): a key's first and last item of this
            // unit bound its run; the units' pieces of one run are adjacent, so the minimum start and
            // the maximum end over them are the run (rr_kernels.hpp bounds encoding: x = ~start,
            // y = end, atomic max on zeroed words).  A unit holds few distinct keys: ~2 atomics each.
            if (j == 0 || s_key[j - 1] != k) atomicMax(&bounds[(uint32_t)k].x, ~pos);
            if (j + 1 == nu || s_key[j + 1] != k) atomicMax(&bounds[(uint32_t)k].y, pos + 1u);
        }
    }
}

struct SortLayout {
    void* keys_alt;
    uint32_t* vals_alt;
    uint32_t* counts;
    uint32_t* offsets;
    uint32_t* totals;  // [512] per-digit totals of the current pass
    size_t total;
};

// rounds per wave: full 16 for large inputs, fewer for small ones so that there are >= ~min_units
// units (Tuning::sort_min_units, default 128; interleaved A/B on the bench step: with 8-bit digits
// 512 beat 1024 by 1.7%; with the 8-wave scatter (round 3) the 3-pass depth sort of 1M keys
// preferred its largest units: 128 (4096-item units) 0.086 vs 0.088 ms/step with 256 and 0.102
// with 512, profiles/r03_sort_units_ab.jsonl).  Sorts of <= 16-bit keys (the bin sorts) target
// more, smaller units (Tuning::sort_min_units_tile, default 1024): their first pass's units are the
// duplicate's windows, whose workgroups are latency-bound (duplicate 0.098 -> 0.092, bin sort 0.087
// -> 0.077 ms/step with 1024).  Tuning::sort_max_rounds caps the rounds (tests: 2048-item units).
int rounds_for(size_t n, int bits) {
    const Tuning& tu = tuning();
    const size_t mu = (size_t)(bits <= 16 ? tu.sort_min_units_tile : tu.sort_min_units);
    int r = std::min(tu.sort_max_rounds, kMaxRounds);
    while (r > 1 && (n + (size_t)64 * kWaves * r - 1) / ((size_t)64 * kWaves * r) < mu) r >>= 1;
    return r;
}

// n_hint (0: n): the size the unit length is chosen for, where n is only a capacity and the device
// holds the count (the binning's phases: sized by the frame's pair total, filled ~1/3 and ~2/3)
template <typename K>
SortLayout sort_layout(void* buf, size_t n, int bits, size_t n_hint) {
    auto al = [](size_t x) { return (x + 255) & ~size_t(255); };
    SortLayout s{};
    const int rounds = rounds_for(n_hint ? n_hint : n, bits);
    const size_t units = (n + (size_t)64 * kWaves * rounds - 1) / ((size_t)64 * kWaves * rounds);
    const int dmax = sort_max_dbits(bits);
    const size_t nc = std::max<size_t>(((size_t)1 << dmax) * units, 1);
    char* p = static_cast<char*>(buf);
    size_t off = 0;
    auto take = [&](size_t bytes) {
        void* r = p ? p + off : nullptr;
        off = al(off + std::max<size_t>(bytes, 1));
        return r;
    };
    s.keys_alt = take(n * sizeof(K));
    s.vals_alt = static_cast<uint32_t*>(take(n * 4));
    s.counts = static_cast<uint32_t*>(take(nc * 4));
    s.offsets = static_cast<uint32_t*>(take(nc * 4));
    s.totals = static_cast<uint32_t*>(take(512 * 4));
    s.total = off;
    return s;
}

}  // namespace

template <typename K>
size_t radix_sort_temp_bytes(size_t n, int bits, size_t n_hint) {
    return sort_layout<K>(nullptr, n, bits, n_hint).total;
}

template <typename K>
RadixPlan radix_sort_plan(void* temp, size_t n, int begin_bit, int end_bit, size_t n_hint) {
    RadixPlan p{};
    const int bits = end_bit - begin_bit;
    if (n == 0 || bits <= 0) return p;
    const SortLayout s = sort_layout<K>(temp, n, bits, n_hint);
    const int passes = sort_passes(bits);
    p.rounds = rounds_for(n_hint ? n_hint : n, bits);
    p.unit_items = 64 * kWaves * p.rounds;
    p.units = (int)((n + p.unit_items - 1) / p.unit_items);
    p.dbits0 = (bits + passes - 1) / passes;
    p.counts = s.counts;
    return p;
}

thread_local const char* g_why = "";
const char* radix_sort_last_error() { return g_why; }

template <typename K>
hipError_t radix_sort_pairs(void* temp, size_t temp_bytes, const K* keys_in, K* keys_out, const uint32_t* vals_in,
                            uint32_t* vals_out, size_t n, int begin_bit, int end_bit, hipStream_t st,
                            bool first_counts_ready, const uint32_t* unit_len, const uint32_t* n_dev, size_t n_hint,
                            uint2* bounds) {
    const int bits = end_bit - begin_bit;
    if (n == 0) return hipSuccess;
    g_why = "";
    if (n > 0xffffffffull || bits <= 0 || bits > (int)(8 * sizeof(K))) return g_why = "bad size/bits", hipErrorInvalidValue;
    if (unit_len && !n_dev) return g_why = "sparse units without n_dev", hipErrorInvalidValue;
    const SortLayout s = sort_layout<K>(temp, n, bits, n_hint);
    if (temp_bytes < s.total) return g_why = "temp too small", hipErrorInvalidValue;
    const int passes = sort_passes(bits);
    const int rounds = rounds_for(n_hint ? n_hint : n, bits);
    const int units = (int)((n + (size_t)64 * kWaves * rounds - 1) / ((size_t)64 * kWaves * rounds));
    const K* ksrc = keys_in;
    const uint32_t* vsrc = vals_in;
    int shift = begin_bit;
    for (int p = 0; p < passes; p++) {
        // spread the bits evenly over the passes (13 -> 7 + 6)
        const int dbits = (bits - (shift - begin_bit) + (passes - p) - 1) / (passes - p);
        const bool last = p == passes - 1;
        // destinations alternate so that the last pass lands in the caller's buffers
        const bool to_out = ((passes - 1 - p) % 2) == 0;
        K* kdst = to_out ? keys_out : static_cast<K*>(s.keys_alt);
        uint32_t* vdst = to_out ? vals_out : s.vals_alt;
        if (!last && kdst == nullptr) return g_why = "no key storage", hipErrorInvalidValue;
        if (!(p == 0 && first_counts_ready)) {
            if (p == 0 && unit_len) return g_why = "sparse units need producer counts", hipErrorInvalidValue;
            auto count = dbits > 8 ? (rounds <= 2   ? k_rs_count<K, 2, 9>
                                      : rounds <= 4 ? k_rs_count<K, 4, 9>
                                      : rounds <= 8 ? k_rs_count<K, 8, 9>
                                                    : k_rs_count<K, kMaxRounds, 9>)
                                   : (rounds <= 2   ? k_rs_count<K, 2, 8>
                                      : rounds <= 4 ? k_rs_count<K, 4, 8>
                                      : rounds <= 8 ? k_rs_count<K, 8, 8>
                                                    : k_rs_count<K, kMaxRounds, 8>);
            count<<<units, 64 * kWaves, 0, st>>>(ksrc, n, shift, dbits, rounds, s.counts, units, n_dev);
        }
        k_rs_scan_rows<<<1 << dbits, 256, 0, st>>>(s.counts, s.offsets, units, s.totals);
        // the scatter ranks a unit with kScatterWaves waves (the same unit_items: rounds_s rounds
        // per wave) where the unit has at least 2 count rounds
        const int sw = (rounds >= 2 && kScatterWaves == 8) ? 8 : 4;
        const int rs = rounds * kWaves / sw;
        auto scatter =
            sw == 8 ? (dbits > 8 ? (rs <= 2 ? k_rs_scatter<K, 2, 9, 8> : rs <= 4 ? k_rs_scatter<K, 4, 9, 8>
                                                                        : k_rs_scatter<K, 8, 9, 8>)
                                 : (rs <= 2 ? k_rs_scatter<K, 2, 8, 8> : rs <= 4 ? k_rs_scatter<K, 4, 8, 8>
                                                                        : k_rs_scatter<K, 8, 8, 8>))
                    : (dbits > 8 ? (rs <= 2   ? k_rs_scatter<K, 2, 9, 4>
                                    : rs <= 4 ? k_rs_scatter<K, 4, 9, 4>
                                    : rs <= 8 ? k_rs_scatter<K, 8, 9, 4>
                                              : k_rs_scatter<K, kMaxRounds, 9, 4>)
                                 : (rs <= 2   ? k_rs_scatter<K, 2, 8, 4>
                                    : rs <= 4 ? k_rs_scatter<K, 4, 8, 4>
                                    : rs <= 8 ? k_rs_scatter<K, 8, 8, 4>
                                              : k_rs_scatter<K, kMaxRounds, 8, 4>));
        scatter<<<units, 64 * sw, 0, st>>>(ksrc, vsrc, kdst, vdst, n, shift, dbits, rs, s.offsets, units,
                                               s.totals, p == 0 ? unit_len : nullptr, n_dev, last ? bounds : nullptr);
        ksrc = kdst;
        vsrc = vdst;
        shift += dbits;
    }
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) g_why = "kernel launch";
    return e;
}

template size_t radix_sort_temp_bytes<uint16_t>(size_t, int, size_t);
template size_t radix_sort_temp_bytes<uint32_t>(size_t, int, size_t);
template hipError_t radix_sort_pairs<uint16_t>(void*, size_t, const uint16_t*, uint16_t*, const uint32_t*, uint32_t*,
                                               size_t, int, int, hipStream_t, bool, const uint32_t*,
                                               const uint32_t*, size_t, uint2*);
template hipError_t radix_sort_pairs<uint32_t>(void*, size_t, const uint32_t*, uint32_t*, const uint32_t*, uint32_t*,
                                               size_t, int, int, hipStream_t, bool, const uint32_t*,
                                               const uint32_t*, size_t, uint2*);
template RadixPlan radix_sort_plan<uint16_t>(void*, size_t, int, int, size_t);
template RadixPlan radix_sort_plan<uint32_t>(void*, size_t, int, int, size_t);

}  // namespace rr
